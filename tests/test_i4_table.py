"""The table-driven I4 row predictor of k_decode_split (decode.hip
`pred4_row_tab` / `kI4Code`, round 6) restated on the CPU byte for byte --
E = L3 L2 L1 L0 X T0..T7 packed, A3 = lerp(lerp(left, right, floor), centre,
round), A2 = lerp(E, right, round), DC, TM, the pool layout -- with the code
words parsed from the kernel source, checked against the oracle's 4x4
predictor (oracle/dsp_pred.c or_pred_luma4, predict_lossy.go:185-424) on
random and saturated contexts for every mode and row.  The GPU side is
covered by the decoder suites (tests/test_c3_real.py, test_gpu_frames.py)."""
import os
import re

import numpy as np

import oracle as O

SRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "webp_amd", "csrc", "decode.hip")


def code_table():
    src = open(SRC).read()
    body = src[src.index("kI4Code[40] = {"):]
    body = body[:body.index("};")]
    words = [tuple(int(v) for v in m.split(",")) for m in re.findall(r"i4c\(([^)]*)\)", body)]
    assert len(words) == 40
    return np.array(words, dtype=np.int64).reshape(10, 4, 4)  # [mode][row][pixel] -> pool byte


def lerp(a, b, up):  # v_lerp_u8 per byte
    return (a + b + up) >> 1


def pool(X, T, L, y):
    E = np.array([L[3], L[2], L[1], L[0], X] + list(T), dtype=np.int64)
    ext = np.concatenate([[E[0]], E, [E[12]] * 4])  # ext[i + 1] = E[i]; E[-1] = E[0], E[13..] = E[12]
    a3 = [lerp(lerp(ext[i], ext[i + 2], 0), ext[i + 1], 1) for i in range(16)]
    a2 = [lerp(ext[i + 1], ext[i + 2], 1) for i in range(12)]
    dc = (int(np.sum(T[:4])) + int(np.sum(L)) + 4) >> 3
    tm = [min(max(int(L[y]) - int(X) + int(t), 0), 255) for t in T[:4]]
    return np.array(a3 + a2 + list(E[:4]) + [dc] * 4 + tm, dtype=np.int64)


def oracle_block(mode, X, T, L):
    buf = np.zeros(O.YUV_SIZE, dtype=np.uint8)
    off = O.YOFF + 4 * O.BPS + 8  # a block with room for its context
    buf[off - 1 - O.BPS] = X
    buf[off - O.BPS: off - O.BPS + 8] = T
    for j in range(4):
        buf[off - 1 + j * O.BPS] = L[j]
    O.lib.or_pred_luma4(mode, O.ptr(buf), off)
    return np.array([[buf[off + y * O.BPS + x] for x in range(4)] for y in range(4)])


def test_i4_code_table_matches_oracle():
    code = code_table()
    rng = np.random.default_rng(6)
    for it in range(400):
        if it % 4 == 0:  # saturated: the clamps and the rounding at 0 / 255
            X, T, L = int(rng.choice([0, 255])), rng.choice([0, 255], 8), rng.choice([0, 255], 4)
        else:
            X, T, L = int(rng.integers(256)), rng.integers(0, 256, 8), rng.integers(0, 256, 4)
        pools = [pool(X, T, L, y) for y in range(4)]
        for mode in range(10):
            want = oracle_block(mode, X, T, L)
            got = np.array([[pools[y][code[mode, y, x]] for x in range(4)] for y in range(4)])
            assert (got == want).all(), (mode, X, T, L, got, want)
