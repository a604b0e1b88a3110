"""Row rescaler (internal/dsp/rescale.go).

The reference has no tests and no callers for rescale.go, and its arithmetic
is not libwebp's (no x_add-1 adjustment, FYScale only when expanding), so no
third-party fixture applies: parity is pinned by properties of the C
restatement (oracle/rescale.c) -- equal sizes give the identity, integer-ratio
shrinks of a constant plane stay constant -- and by the restatement itself.

CPU: the properties; the host plan (wg_rescaler_plan_host, the size-only walk
of the Go state machine that the GPU kernel consumes) replayed in numpy
== the oracle's row-by-row import/export on every size class.
GPU (-m gpu): wg_rescale == oracle, bit-exact, batched, on shrink / expand /
mixed sizes, 1-pixel edges and 4096^2 -> 2048^2."""
import ctypes

import numpy as np
import pytest

import oracle as O

SIZES = [(16, 16, 16, 16), (37, 23, 37, 23), (64, 48, 32, 24), (100, 80, 33, 17), (13, 9, 40, 30),
         (20, 20, 7, 50), (7, 50, 20, 9), (1, 1, 5, 5), (1, 5, 1, 2), (300, 1, 3, 1), (5, 7, 1, 1),
         (257, 129, 256, 128), (640, 480, 320, 240), (99, 101, 101, 99), (3, 3, 1000, 2)]


def plane(h, w, seed):
    return np.random.default_rng(seed).integers(0, 256, (h, w), dtype=np.uint8)


def test_identity_size():
    for i, (w, h) in enumerate([(2, 1), (16, 16), (37, 23), (301, 7)]):
        p = plane(h, w, i)
        out, rows = O.rescale_plane(p, w, h)
        assert rows == h and (out == p).all()


def test_fxy_scale_overflow_gives_zero():
    # RescalerInit (rescale.go:94-101): dst_h << 32 / (src_w * src_h) overflows
    # uint32 when dst_h >= src_w * src_h (a 1-pixel-wide, non-shrinking
    # column); FXYScale becomes 0 and the Go export writes zeros.
    for h in (1, 5):
        out, rows = O.rescale_plane(plane(h, 1, h) | 1, 1, h)
        assert rows == h and (out == 0).all()


@pytest.mark.parametrize("fx,fy", [(2, 2), (4, 1), (1, 3), (8, 8)])
def test_integer_shrink_constant(fx, fy):
    for c in (0, 1, 77, 254, 255):
        p = np.full((24 * fy, 40 * fx), c, np.uint8)
        out, rows = O.rescale_plane(p, 40, 24)
        assert rows == 24 and (out == c).all(), (fx, fy, c)


def _plan(sw, sh, dw, dh):
    from webp_amd._lib import call, lib
    buf = np.zeros(lib.wg_rescaler_plan_bytes(dw, dh), np.uint8)
    rows = ctypes.c_int32(0)
    call("wg_rescaler_plan_host", sw, sh, dw, dh, buf.ctypes.data, ctypes.addressof(rows))
    hd = buf[:64].view(np.int32)
    xt = buf[64:64 + 32 * dw].view(np.int32).reshape(dw, 8)
    yt = buf[64 + 32 * dw:].view(np.int32).reshape(dh, 4)
    return hd, xt, yt, rows.value


def _mult_fix(x, y):
    return ((x.astype(np.uint64) * np.uint64(y) + np.uint64(1 << 31)) >> np.uint64(32)).astype(np.uint32)


def _replay(src, dw, dh):
    """numpy statement of k_rescale over the host plan."""
    sh, sw = src.shape
    hd, xt, yt, rows = _plan(sw, sh, dw, dh)
    x_expand, y_expand = hd[4], hd[5]
    x_add, x_sub = np.uint32(hd[6]), np.uint32(hd[7])
    fx, fy, fxy = (np.uint32(hd[8].view(np.uint32)), np.uint32(hd[9].view(np.uint32)),
                   np.uint32(hd[10].view(np.uint32)))

    def frow(r):
        row = src[r].astype(np.uint32)
        out = np.zeros(dw, np.uint32)
        with np.errstate(over="ignore"):
            for x in range(dw):
                a, b, c, neg, pidx, pneg = (int(v) for v in xt[x, :6])
                if x_expand:
                    left, right = row[a], row[b]
                    out[x] = right * x_add + (left - right) * np.uint32(c & 0xFFFFFFFF)
                    continue
                s = np.uint32(0)
                if pidx >= 0 and pneg != 0:
                    s = _mult_fix(np.array([row[pidx] * np.uint32(pneg & 0xFFFFFFFF)], np.uint32), fx)[0]
                base = np.uint32(0)
                for i in range(b):
                    base = row[a + i]
                    s += base
                s += base * np.uint32(c)
                out[x] = s * x_sub - base * np.uint32(neg & 0xFFFFFFFF)
        return out

    dst = np.zeros((dh, dw), np.uint8)
    with np.errstate(over="ignore"):
        for y in range(rows):
            s0, s1, b = int(yt[y, 0]), int(yt[y, 1]), int(yt[y, 2]) & 0xFFFFFFFF
            if y_expand:
                f = frow(s0)
                j = f
                if b:
                    ir = np.zeros(dw, np.uint32) if s1 < 0 else frow(s1)
                    i = np.uint64((1 << 32) - b) * f.astype(np.uint64) + np.uint64(b) * ir.astype(np.uint64)
                    j = ((i + np.uint64(1 << 31)) >> np.uint64(32)).astype(np.uint32)
                v = _mult_fix(j, fy)
            else:
                acc = np.zeros(dw, np.uint32)
                for s in range(s0, s1 + 1):
                    acc += frow(s)
                v = _mult_fix(acc, fxy)
            dst[y] = np.minimum(v, 255).astype(np.uint8)
    return dst, rows


@pytest.mark.parametrize("size", [s for s in SIZES if s[2] * max(s[0], s[2]) <= 200000])
def test_plan_replay_matches_oracle(size):
    sw, sh, dw, dh = size
    src = plane(sh, sw, sw * 7 + dh)
    exp, erows = O.rescale_plane(src, dw, dh)
    got, rows = _replay(src, dw, dh)
    assert rows == erows
    assert (got == exp).all()


@pytest.mark.gpu
@pytest.mark.parametrize("size", SIZES)
def test_gpu_rescale(cuda, size):
    import torch

    from webp_amd.rescale import Rescaler
    sw, sh, dw, dh = size
    n = 3
    src = np.stack([plane(sh, sw, 100 * k + sw) for k in range(n)])
    r = Rescaler(sw, sh, dw, dh)
    got = r.rescale(torch.from_numpy(src).to(cuda)).cpu().numpy()
    for k in range(n):
        exp, rows = O.rescale_plane(src[k], dw, dh)
        assert r.rows == rows
        assert (got[k] == exp).all(), (size, k)


@pytest.mark.gpu
def test_gpu_rescale_large(cuda):
    import torch

    from webp_amd.rescale import rescale_plane
    src = plane(4096, 4096, 5)
    got = rescale_plane(torch.from_numpy(src).to(cuda), 2048, 2048).cpu().numpy()
    exp, rows = O.rescale_plane(src, 2048, 2048)
    assert rows == 2048 and (got == exp).all()
    src = plane(1080, 1920, 6)
    got = rescale_plane(torch.from_numpy(src).to(cuda), 1280, 720).cpu().numpy()
    exp, rows = O.rescale_plane(src, 1280, 720)
    assert (got == exp).all()
