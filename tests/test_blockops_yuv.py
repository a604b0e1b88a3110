"""The block-level entry points of the functions the frame kernels run fused
(SURVEY 8(b) layer 1): UpsampleLinePair[NRGBA],
AccumulateRGBA, ConvertRGBA32ToUV[Dithered] + VP8Random, SSE / PSNRFromSSE,
DistoStats / SSIMFromStats[Clipped] / SSIMFromBlocks.

CPU: the oracle against the reference's own known answers for these
functions (testc/ssim/ssim_test.go:162-258: identical pixels -> 1.0,
hat-weighted identical 7x7 -> 1.0, zero stats -> 0; random_test.go's
sequence is pinned in tests/test_dither.py; the upsampler in
tests/test_oracle.py from upsample_test.go) and PSNRFromSSE's closed form.
GPU: every entry point, batched through the C ABI (webp_amd.dsp), bit-exact
against the oracle per instance; SSIM / PSNR doubles compared exactly (the
same integer inputs and the same float64 expression)."""
import math

import numpy as np
import pytest

import oracle as O


def rng(seed):
    return np.random.default_rng(seed)


# ---------------- CPU: the oracle's pins ----------------

def test_ssim_from_stats_reference_answers():
    g = np.random.Generator(np.random.PCG64(45))
    for _ in range(200):  # identical pixels (ssim_test.go:165-186)
        v = g.integers(0, 256, g.integers(10, 110)).astype(np.uint8)
        st = O.disto_stats(v[None], v[None])
        assert abs(O.ssim_from_stats(st, False) - 1.0) <= 1e-6
    hat = [1, 2, 3, 4, 3, 2, 1]
    for _ in range(50):  # hat-weighted identical 7x7 (:191-210): each pixel repeated w times
        vals = []
        for y in range(7):
            for x in range(7):
                vals += [int(g.integers(28, 228))] * (hat[x] * hat[y])
        v = np.array(vals, np.uint8)[None]
        st = O.disto_stats(v, v)
        assert st[0] == 256 and abs(O.ssim_from_stats(st, False) - 1.0) <= 1e-6
    assert O.ssim_from_stats(np.zeros(6, np.uint32), False) == 0.0  # zero_w (:251-256)


def test_psnr_from_sse_closed_form():
    assert O.psnr_from_sse(0, 10) == 99.0 and O.psnr_from_sse(5, 0) == 99.0
    for sse, count in [(1, 1), (1000, 100), (65025, 1), (123456789, 1 << 20), (3, 7)]:
        assert O.psnr_from_sse(sse, count) == pytest.approx(10 * math.log10(65025.0 / (sse / count)), rel=1e-15)


def test_disto_stats_wrap_like_go_uint32():
    a = np.full((300, 300), 255, np.uint8)
    st = O.disto_stats(a, a)
    assert st[3] == (300 * 300 * 255 * 255) % (1 << 32)  # Xxm wraps as Go's uint32 field


# ---------------- GPU: the batched entry points vs the oracle ----------------

def dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t):
    import torch
    torch.cuda.synchronize()
    return t.cpu().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("width", [1, 2, 3, 4, 17, 64, 1920, 1921])
@pytest.mark.parametrize("nrgba", [False, True])
@pytest.mark.parametrize("last_row", [False, True])
def test_gpu_upsample_line_pairs(cuda, width, nrgba, last_row):
    from webp_amd import dsp
    n, cw = 5, (width + 1) // 2
    r = rng(width * 4 + nrgba * 2 + last_row)
    ty, by = r.integers(0, 256, (2, n, width + 3), dtype=np.uint8)
    tu, tv, bu, bv = r.integers(0, 256, (4, n, cw + 2), dtype=np.uint8)
    at, ab = r.integers(0, 256, (2, n, width + 1), dtype=np.uint8)
    args = [dev(ty), None if last_row else dev(by), dev(tu), dev(tv), dev(bu), dev(bv), width]
    if nrgba:
        got_t, got_b = dsp.UpsampleLinePairNRGBA(*args, alpha_top=dev(at), alpha_bot=None if last_row else dev(ab))
    else:
        got_t, got_b = dsp.UpsampleLinePair(*args)
    got_t = host(got_t)
    got_b = None if got_b is None else host(got_b)
    for i in range(n):
        et, eb = O.upsample_line_pair(ty[i], None if last_row else by[i], tu[i], tv[i], bu[i], bv[i], width, nrgba,
                                      at[i] if nrgba else None, (None if last_row else ab[i]) if nrgba else None)
        assert (got_t[i] == et).all(), i
        if not last_row:
            assert (got_b[i] == eb).all(), i


@pytest.mark.gpu
def test_gpu_upsample_line_pairs_no_alpha(cuda):
    from webp_amd import dsp
    n, width = 3, 33
    r = rng(7)
    ty, by = r.integers(0, 256, (2, n, width), dtype=np.uint8)
    tu, tv, bu, bv = r.integers(0, 256, (4, n, 17), dtype=np.uint8)
    got_t, got_b = dsp.UpsampleLinePairNRGBA(dev(ty), dev(by), dev(tu), dev(tv), dev(bu), dev(bv), width)
    got_t, got_b = host(got_t), host(got_b)
    for i in range(n):
        et, eb = O.upsample_line_pair(ty[i], by[i], tu[i], tv[i], bu[i], bv[i], width, True)
        assert (got_t[i] == et).all() and (got_b[i] == eb).all()
        assert (got_t[i][3::4] == 255).all()


def alpha_rows(r, n, L, kind):
    if kind == "opaque":
        return np.full((n, L), 255, np.uint8)
    if kind == "clear":
        return np.zeros((n, L), np.uint8)
    a = r.integers(0, 256, (n, L), dtype=np.uint8)
    a[:, ::5] = 255
    a[:, 1::7] = 0
    return a


@pytest.mark.gpu
@pytest.mark.parametrize("width", [1, 2, 3, 7, 64, 1919])
@pytest.mark.parametrize("alpha", ["opaque", "clear", "mixed"])
def test_gpu_accumulate_rgba(cuda, width, alpha):
    import torch

    from webp_amd import dsp
    n, stride = 4, width + 5
    r = rng(width + len(alpha))
    L = 2 * stride
    ch = r.integers(0, 256, (3, n, L), dtype=np.uint8)
    a = alpha_rows(r, n, L, alpha)
    got = host(dsp.AccumulateRGBA(dev(ch[0]), dev(ch[1]), dev(ch[2]), dev(a), stride, width).view(torch.int16))
    for i in range(n):
        exp = O.accumulate_rgba(ch[0][i], ch[1][i], ch[2][i], a[i], stride, width)
        assert (got[i].view(np.uint16) == exp).all(), i


@pytest.mark.gpu
@pytest.mark.parametrize("width", [1, 5, 960, 961])
def test_gpu_convert_rgba32_to_uv(cuda, width):
    import torch

    from webp_amd import dsp
    n = 6
    r = rng(width)
    rgb = r.integers(0, 1021, (n, 4 * width + 8)).astype(np.uint16)
    u, v = dsp.ConvertRGBA32ToUV(dev(rgb.view(np.int16)).view(torch.uint16), width)
    u, v = host(u), host(v)
    for i in range(n):
        eu, ev = O.convert_rgba32_to_uv(rgb[i], width)
        assert (u[i] == eu).all() and (v[i] == ev).all()


@pytest.mark.gpu
@pytest.mark.parametrize("dithering", [0.0, 0.5, 1.0])
def test_gpu_convert_rgba32_to_uv_dithered(cuda, dithering):
    """Each row has its own VP8Random; two calls in a row continue the
    sequences, and the device states after them equal the oracle's."""
    import torch

    from webp_amd import dsp
    n, width = 70, 301  # more rows than one 64-lane block
    r = rng(int(dithering * 10))
    states = dsp.InitRandom(dithering, n)
    ost = [O.random_init(dithering) for _ in range(n)]
    # give the rows different histories: row i first draws i pixels' worth
    for i in range(n):
        pre = r.integers(0, 1021, (4 * i + 4,)).astype(np.uint16)
        O.convert_rgba32_to_uv(pre, i, ost[i])
    states = torch.from_numpy(np.stack([s.view(np.uint8).reshape(-1) for s in ost])).cuda()
    for rep in range(2):
        rgb = r.integers(0, 1021, (n, 4 * width)).astype(np.uint16)
        u, v = dsp.ConvertRGBA32ToUVDithered(dev(rgb.view(np.int16)).view(torch.uint16), width, states)
        u, v = host(u), host(v)
        for i in range(n):
            eu, ev = O.convert_rgba32_to_uv(rgb[i], width, ost[i])
            assert (u[i] == eu).all() and (v[i] == ev).all(), (rep, i)
    got_states = host(states)
    for i in range(n):
        assert (got_states[i] == ost[i].view(np.uint8).reshape(-1)).all()


@pytest.mark.gpu
@pytest.mark.parametrize("w,h", [(1, 1), (4, 4), (16, 16), (37, 23), (1920, 1080)])
def test_gpu_sse_psnr(cuda, w, h):
    import torch

    from webp_amd import dsp
    n, stride = 3, w + 3
    r = rng(w * h)
    pix = r.integers(0, 256, (n, stride * h), dtype=np.uint8)
    ref = np.clip(pix.astype(int) + r.integers(-9, 10, pix.shape), 0, 255).astype(np.uint8)
    ref[0] = pix[0]  # identical pair: SSE 0 -> PSNR 99
    sse = dsp.SSE(dev(pix), dev(ref), w, h, stride, stride)
    count = torch.full((n,), w * h, dtype=torch.int64, device="cuda")
    psnr = host(dsp.PSNRFromSSE(sse, count))
    sse = host(sse).view(np.uint64)
    for i in range(n):
        e = O.lib.or_sse_plane(O.u8(pix[i]), stride, O.u8(ref[i]), stride, w, h)
        assert sse[i] == e
        assert psnr[i] == O.psnr_from_sse(e, w * h)  # bit-exact double
    assert psnr[0] == 99.0


@pytest.mark.gpu
@pytest.mark.parametrize("w,h", [(1, 1), (7, 7), (16, 16), (45, 29), (4096, 4096)])
def test_gpu_disto_stats_and_ssim(cuda, w, h):
    from webp_amd import dsp
    n = 2 if w * h > 1e6 else 4
    r = rng(w + h)
    pix = r.integers(0, 256, (n, w * h), dtype=np.uint8)
    ref = np.clip(pix.astype(int) + r.integers(-20, 21, pix.shape), 0, 255).astype(np.uint8)
    ref[-1] = pix[-1]
    st = dsp.DistoStatsOfBlocks(dev(pix), dev(ref), w, h, w, w)
    s_f = host(dsp.SSIMFromStats(st))
    s_c = host(dsp.SSIMFromStats(st, clipped=True))
    blocks = host(dsp.SSIMFromBlocks(dev(pix), dev(ref), w, h, w, w))
    st = host(st).view(np.uint32)
    for i in range(n):
        e = O.disto_stats(pix[i].reshape(h, w), ref[i].reshape(h, w))
        assert (st[i] == e).all(), (i, st[i], e)
        assert s_f[i] == O.ssim_from_stats(e, False) and s_c[i] == O.ssim_from_stats(e, True)
        assert blocks[i] == s_c[i]
