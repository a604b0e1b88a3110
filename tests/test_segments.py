"""CPU: the encoder's segment analysis (analysis() after computeAlphas,
internal/lossy/encode_analysis.go:29-903) -- the restatement
(oracle/segments.c), the host-built quantiser table the GPU kernel uses
(wg_encoder_config), and why a libm pow may stand in for Go's math.Pow.

The GPU kernel (k_segments) is compared with the oracle in
tests/test_gpu_segments.py."""
import numpy as np
import pytest

import oracle as O


def test_pow_step_has_margin():
    """setSegmentParams computes q = int(127 * (1 - c_base ** (1 - amp*alpha)))
    (encode_analysis.go:128-142, math.Pow).  Go's Pow and libm's pow may differ
    in the last few ulps.  Over every input the encoder can see (quality
    0..100, SNS 0..100, segment alpha -127..127) the value 127*(1 - c) is
    either exact (c = 0 or 1, or the exponent is 1 so Pow returns c_base
    itself) or at least 1e-9 away from the next integer, far beyond any ulp
    error (127 * 4 ulp(1) ~ 1e-13), so the truncated quantiser is the same
    with either pow."""
    q = np.arange(101, dtype=np.float64)
    c = q / 100.0
    lin = np.where(c < 0.75, c * (2.0 / 3.0), 2.0 * c - 1.0)
    cbase = np.power(lin, 1.0 / 3.0)
    cbase[0], cbase[100] = 0.0, 1.0
    sns = np.arange(101, dtype=np.float64)
    amp = 0.9 * sns / 100.0 / 128.0
    alpha = np.arange(-127, 128, dtype=np.float64)
    expn = 1.0 - amp[:, None] * alpha[None, :]                       # (sns, alpha)
    cc = np.power(cbase[:, None, None], expn[None, :, :])             # (quality, sns, alpha)
    t = 127.0 * (1.0 - cc)
    exact = (cbase[:, None, None] == 0.0) | (cbase[:, None, None] == 1.0) | (expn[None, :, :] == 1.0)
    frac = np.abs(t - np.round(t))
    worst = frac[~exact].min()
    assert worst > 1e-9, worst
    # the quality -> compression step itself (qualityToCompression's cube root)
    tq = 127.0 * (1.0 - cbase[1:100])
    assert np.abs(tq - np.round(tq)).min() > 1e-9


def test_product_quant_table_matches_oracle():
    """wg_encoder_config's table (the GPU side) equals or_segment_quant."""
    from webp_amd import frames
    for quality, sns in [(75, 50), (0, 50), (100, 50), (30, 0), (50, 100), (90, 80), (75, -1), (1, 1)]:
        cfg = frames.encoder_config(quality=quality, sns_strength=sns)
        want = [O.lib.or_segment_quant(quality, sns, a) for a in range(-127, 128)]
        assert list(cfg["seg_quant"][0][:255]) == want, (quality, sns)


def analysis(alphas, mbw, mbh, uv_sum, **kw):
    return O.segment_analysis(np.asarray(alphas, np.int32), mbw, mbh, uv_sum, O.encoder_config(**kw))


def test_single_segment():
    """encode_test.go:373-386 (Segments = 1 -> every MB in segment 0), and the
    quantiser is qualityToQIndex when the segment alpha is 0."""
    rng = np.random.default_rng(1)
    ids, info, segs = analysis(rng.integers(0, 256, 64), 8, 8, 64 * 40, segments=1)
    assert not ids.any() and info["num_segments"] == 1
    assert (info["quant"] == O.lib.or_quality_to_qindex(75)).all()


def test_kmeans_hand_case():
    """assignSegments on two alpha clusters {10 x 20, 10 x 200}, 4 segments:
    centres start at 20 + (2k+1)*180/8 = 42, 87, 132, 177; the first pass maps
    alpha 20 -> centre 0 and 200 -> centre 3 and moves them onto the clusters
    (displacement 22 + 23 >= 5), the second pass moves nothing: centres
    20, 87, 132, 200, weighted average 110.  Segment alphas
    255*(c - 110)/180 = -127 (clamped), -32, 31, 127; betas 0, 95, 159, 255."""
    a = np.array([20] * 10 + [200] * 10)
    ids, info, _ = analysis(a, 5, 4, 0, sns_strength=0, filter_strength=0)
    # with SNS 0 every segment gets the base quantiser: simplifySegments merges all
    assert info["num_segments"] == 1 and not ids.any()
    ids, info, _ = analysis(a, 5, 4, 0, sns_strength=100, filter_strength=0)
    assert list(info["alpha"]) == [-127, -32, 31, 127]
    assert list(info["beta"]) == [0, 94, 158, 255]  # 255*67/180 = 94.9, 255*112/180 = 158.7
    assert info["num_segments"] == 4  # four distinct quantisers: nothing merges
    assert (ids[:10] == 0).all() and (ids[10:] == 3).all()


def test_segment_map_reset_when_probas_round_to_255():
    """setSegmentProbas (:874-903): with 3 segments, 8150 MBs in segment 0 and
    5 + 5 in segments 1 and 2 make every tree probability round to 255
    ((255*8155 + 4080)/8160, (255*8150 + 4077)/8155, (255*5 + 2)/5), so the map
    is dropped and all MBs use segment 0."""
    a = np.array([0] * 8150 + [100] * 5 + [255] * 5)
    ids, info, _ = analysis(a, 120, 68, 0, sns_strength=100, filter_strength=0, segments=3)
    assert info["num_segments"] == 3
    assert not ids.any() and info["update_map"] == 0
    assert list(info["seg_proba"][:3]) == [255, 255, 255]


def test_uv_deltas():
    """dq_uv_ac = clamp((uv - 64)*10/70 * sns/100, -4, 6), dq_uv_dc = -4*sns/100
    (Go integer division truncates toward zero)."""
    a = np.full(16, 50)
    for uv_avg, sns, ac, dc in [(64, 50, 0, -2), (19, 50, -3, -2), (200, 100, 6, -4), (0, 100, -4, -4), (57, 100, -1, -4),
                                (58, 100, 0, -4),
                                (127, 30, 2, -1)]:
        _, info, segs = analysis(a, 4, 4, uv_avg * 16, sns_strength=sns)
        assert (info["dq_uv_ac"], info["dq_uv_dc"]) == (ac, dc), (uv_avg, sns)
        assert info["global_uv_alpha"] == uv_avg


def test_smoothing_majority():
    """smoothSegmentMap (:76-119, preprocessing bit 0): an isolated MB inside a
    uniform 3x3 neighbourhood takes the majority segment."""
    a = np.full((6, 6), 30)
    a[:, 3:] = 220
    a[2, 1] = 220  # lone high-alpha MB in the low half
    ids0, _, _ = analysis(a, 6, 6, 0, sns_strength=100, filter_strength=0)
    ids1, _, _ = analysis(a, 6, 6, 0, sns_strength=100, filter_strength=0, preprocessing=1)
    ids0, ids1 = ids0.reshape(6, 6), ids1.reshape(6, 6)
    assert ids0[2, 1] != ids0[2, 0] and ids1[2, 1] == ids1[2, 0]
    assert (ids1[0] == ids0[0]).all()  # border rows are not smoothed


@pytest.mark.parametrize("seed", range(6))
def test_random_invariants(seed):
    rng = np.random.default_rng(seed)
    mbw, mbh = int(rng.integers(1, 40)), int(rng.integers(1, 30))
    a = np.clip(rng.normal(rng.integers(0, 255), rng.integers(1, 80), mbw * mbh), 0, 255).astype(np.int32)
    ids, info, segs = analysis(a, mbw, mbh, int(rng.integers(0, 255)) * mbw * mbh, segments=int(rng.integers(1, 5)),
                               preprocessing=int(rng.integers(0, 2)))
    assert ids.max(initial=0) < max(info["num_segments"], 1)
    assert 0 <= info["quant"].min() and info["quant"].max() <= 127
    for k in range(4):  # setupSegment with the frame's dq deltas
        ref = O.setup_segment(int(info["quant"][k]), (0, 0, 0, int(info["dq_uv_dc"]), int(info["dq_uv_ac"])))
        assert segs[k].tobytes() == ref.tobytes()
