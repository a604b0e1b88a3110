"""CPU: known-answer tests that pin the encoder restatement (oracle/lossy_rd.c)
and the tables the GPU encoder uploads, from values the reference holds or
that follow by hand from its Go source.

  VP8FixedCostsI4 rows     internal/lossy/debug_trellis_test.go:261-290 (reference KAT)
  RDScore                  encode_test.go:362-371 (reference KAT)
  QuantizeCoeffs           encode_test.go:148-197 (reference cases, exact values
                           worked out below from encode_quant.go:16-75)
  DequantCoeffs            encode_test.go:199-211 (reference KAT)
  qualityToQIndex          encode_test.go:63-81 (reference KAT)
  TokenCostForCoeffs       encode_quant.go:170-220, hand-derived from the tables
  TrellisQuantizeBlock     encode_trellis.go:23-301: all-zero pre-scan exit,
                           EOB after zigzag position 15, level choice bounds
"""
import ctypes

import numpy as np
import pytest

import oracle as O

SQ = O.SQUANT_DTYPE


def squant(quant, iquant, bias, dc_quant, dc_iquant, dc_bias, sharpen=None):
    sq = np.zeros(1, SQ)
    sq["quant"], sq["iquant"], sq["bias"] = quant, iquant, bias
    sq["dc_quant"], sq["dc_iquant"], sq["dc_bias"] = dc_quant, dc_iquant, dc_bias
    if sharpen is not None:
        sq["sharpen"][0] = sharpen
    return sq


def quantize(vals, sq, first=0):
    inp = np.zeros(16, np.int16)
    inp[:len(vals)] = vals
    out = np.zeros(16, np.int16)
    nz = O.lib.or_quantize_coeffs(inp.ctypes.data, out.ctypes.data, sq.ctypes.data, first)
    return nz, out


# the reference's test quantiser (encode_test.go:150-157): q 10, Y1 biases
REF_SQ = dict(quant=10, iquant=(1 << 17) // 10, bias=110 << 9, dc_quant=10, dc_iquant=(1 << 17) // 10, dc_bias=96 << 9)


def test_fixed_costs_i4_reference_rows():
    """debug_trellis_test.go:261-290: VP8FixedCostsI4[0][0], [0][1] and [9][9]."""
    want = {(0, 0): [40, 1151, 1723, 1874, 2103, 2019, 1628, 1777, 2226, 2137],
            (0, 1): [192, 469, 1296, 1308, 1849, 1794, 1781, 1703, 1713, 1522],
            (9, 9): [305, 1167, 1358, 899, 1587, 1587, 987, 1988, 1332, 501]}
    oracle = np.zeros(1000, np.uint16)
    O.lib.or_fixed_costs_i4(oracle.ctypes.data)
    oracle = oracle.reshape(10, 10, 10)
    from webp_amd import frames
    product = frames.fixed_costs_i4()  # the table wg_encode_mbs uploads (host copy)
    for (t, l), row in want.items():
        assert list(oracle[t, l]) == row, (t, l)
        assert list(product[t, l]) == row, (t, l)
    assert (oracle == product).all()


def test_rd_score():
    """encode_test.go:362-371: RDScore(100, 50, 10) = 50*10 + 256*100."""
    assert O.lib.or_rd_score(100, 50, 10) == 50 * 10 + 256 * 100


def test_quality_to_qindex():
    """encode_test.go:63-81 ({0: 127, 100: 0, 50: 38..39}); q75 is index 26."""
    assert O.lib.or_quality_to_qindex(0) == 127
    assert O.lib.or_quality_to_qindex(100) == 0
    assert 38 <= O.lib.or_quality_to_qindex(50) <= 39
    assert O.lib.or_quality_to_qindex(75) == 26


def test_quantize_reference_case():
    """encode_test.go:148-172 (in {100, -50, 25}); exact values from
    QUANTDIV (v*iQ + B) >> 17 with iQ = 13107:
      DC  (100*13107 + 96<<9) >> 17 = 1359852 >> 17 = 10
      AC  (50*13107 + 110<<9) >> 17 =  711670 >> 17 = 5  -> -5
      AC  (25*13107 + 110<<9) >> 17 =  383995 >> 17 = 2
    nz count: raster 2 is zigzag position 5 -> 6."""
    nz, out = quantize([100, -50, 25], squant(**REF_SQ))
    assert list(out[:4]) == [10, -5, 2, 0] and not out[4:].any()
    assert nz == 6


def test_quantize_all_zero_and_skip_dc():
    """encode_test.go:174-197."""
    nz, out = quantize([], squant(**REF_SQ))
    assert nz == 0 and not out.any()
    nz, out = quantize([999, 50], squant(**REF_SQ), first=1)
    assert out[0] == 0 and out[1] == 5 and nz == 2


def test_dequant_reference_case():
    """encode_test.go:199-211."""
    inp = np.zeros(16, np.int16)
    inp[:3] = [10, -5, 3]
    out = np.zeros(16, np.int16)
    O.lib.or_dequant_coeffs(inp.ctypes.data, out.ctypes.data, squant(10, 0, 0, 10, 0, 0).ctypes.data)
    assert list(out[:3]) == [100, -50, 30]


def test_quantize_clamp_wrap_and_sharpen():
    """Edge arithmetic of quantizeCoeffsGo (encode_quant.go:52-73):
      - clamp: quant 1 (iQ 131072), v = 32767: (32767*131072 + 56320) >> 17 = 32767 -> 2047
      - uint32 wrap: v = 32767 + sharpen 100 = 32867: 32867*131072 = 4307943424
        wraps to 12976128; (12976128 + 56320) >> 17 = 99 (Go and C both multiply in uint32)
      - sharpen lifts |v| before the sign is reapplied, negative results floor at 0.
    """
    sq = squant(1, 1 << 17, 110 << 9, 1, 1 << 17, 96 << 9)
    nz, out = quantize([0, 32767], sq)
    assert out[1] == 2047 and nz == 2
    sharp = np.zeros(16, np.int16)
    sharp[1] = 100
    nz, out = quantize([0, -32767], squant(1, 1 << 17, 110 << 9, 1, 1 << 17, 96 << 9, sharpen=sharp))
    assert out[1] == -99
    sharp[2] = -50
    nz, out = quantize([0, 0, 40], squant(**REF_SQ, sharpen=sharp))
    assert out[2] == 0 and nz == 2  # max(40 - 50, 0) = 0; raster 1 (sharpen 100 -> (100*13107+56320)>>17 = 10)
    assert out[1] == 10


def _tables():
    import re
    txt = open(O.os.path.join(O._HERE, "vp8_tables.h")).read()

    def tab(name):
        body = txt[txt.index(name + "["):]
        body = body[body.index("{") + 1:body.index("};")]
        return np.array([int(x) for x in re.findall(r"-?\d+", body)])
    return {k: tab(k) for k in ("vp8_entropy_cost", "vp8_level_fixed_costs", "vp8_zigzag", "vp8_bands")}


def test_token_cost_hand_derived():
    """TokenCostForCoeffs (encode_quant.go:170-220), expected values spelled
    out from its branches with the default probabilities:
      - empty block: one EOB at band(first) / ctx0;
      - a single level 1 at zigzag position 15: 15 zero tokens (ctx 0 after the
        first), then non-zero + level 1 and no trailing EOB (n never passes 15);
      - level 2 at position 0 then EOB at position 1 with ctx 2."""
    T = _tables()
    ec, fixed, zz, bands = T["vp8_entropy_cost"], T["vp8_level_fixed_costs"], T["vp8_zigzag"], T["vp8_bands"]
    proba = O.default_proba()
    P = proba.reshape(4, 8, 3, 11)
    for typ in (0, 1, 3):
        for ctx0 in (0, 1, 2):
            c = np.zeros(16, np.int16)
            assert O.lib.or_token_cost(c.ctypes.data, 0, typ, proba.ctypes.data, ctx0, 0) == ec[P[typ, 0, ctx0, 0]]
            # level 1 at zigzag position 15
            c[zz[15]] = -1
            want, ctx = 0, ctx0
            for n in range(15):
                p = P[typ, bands[n], ctx]
                want += ec[255 - p[0]] + ec[p[1]]
                ctx = 0
            p = P[typ, bands[15], ctx]
            want += ec[255 - p[0]] + ec[255 - p[1]] + fixed[1] + ec[p[2]]
            assert O.lib.or_token_cost(c.ctypes.data, 16, typ, proba.ctypes.data, ctx0, 0) == want
            # level 2 at position 0, EOB next
            c[:] = 0
            c[zz[0]] = 2
            p = P[typ, bands[0], ctx0]
            want = ec[255 - p[0]] + ec[255 - p[1]] + fixed[2] + ec[255 - p[2]] + ec[p[3]] + ec[p[4]]
            want += ec[P[typ, bands[1], 2, 0]]
            assert O.lib.or_token_cost(c.ctypes.data, 1, typ, proba.ctypes.data, ctx0, 0) == want


def trellis(vals_zigzag, sq, first=0, ctx_type=3, init_ctx=0, lam=100):
    zz = _tables()["vp8_zigzag"]
    inp = np.zeros(16, np.int16)
    for n, v in enumerate(vals_zigzag):
        inp[zz[n]] = v
    out = np.zeros(16, np.int16)
    proba = O.default_proba()
    nz = O.lib.or_trellis_quantize(inp.ctypes.data, out.ctypes.data, sq.ctypes.data, first, ctx_type, init_ctx,
                                   proba.ctypes.data, lam)
    return nz, out, inp


def test_trellis_zero_prescan_and_bounds():
    """encode_trellis.go: a block whose levels all quantise to 0 under the
    neutral rounding exits before the DP with an all-zero result; otherwise
    every output level is 0, L0 or L0 + 1 (L0 = (|c| + sharpen) * iQ >> 17)."""
    sq = squant(**REF_SQ)
    nz, out, _ = trellis([5, -9, 3], sq)  # 9 * 13107 >> 17 = 0
    assert nz == 0 and not out.any()
    rng = np.random.default_rng(5)
    for lam in (0, 50, 5000):
        for _ in range(200):
            vals = rng.integers(-400, 400, 16)
            nz, out, inp = trellis(vals, sq, lam=lam)
            for r in range(16):
                c = abs(int(inp[r]))
                iq = REF_SQ["dc_iquant"] if r == 0 else REF_SQ["iquant"]
                L0 = min((c * iq) >> 17, 2047)
                assert abs(int(out[r])) in (0, L0, L0 + 1)
                assert out[r] == 0 or np.sign(out[r]) == np.sign(inp[r])


def test_trellis_eob_at_position_15():
    """A lone large coefficient at zigzag position 15 survives and the
    returned nz count is 16 (no EOB token follows position 15)."""
    sq = squant(**REF_SQ)
    vals = [0] * 15 + [600]
    nz, out, _ = trellis(vals, sq, lam=10)
    zz = _tables()["vp8_zigzag"]
    L0 = (600 * REF_SQ["iquant"]) >> 17  # 7864200 >> 17 = 59
    assert L0 == 59
    assert nz == 16 and out[zz[15]] in (L0, L0 + 1) and not np.delete(out, zz[15]).any()
