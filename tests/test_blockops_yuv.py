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


# ---------------- PointSampleRow, ConvertARGBToY / ConvertARGBToUV (VERDICT r03 missing 1) ----------------
# The reference holds no test vectors for these three; the oracle is checked
# against a numpy restatement written from upsample.go:238-245 and
# yuv.go:138-171, 270-330 directly (parity pinned through RGBToY / RGBToU /
# RGBToV / YUVToRGB, whose import and upsample paths equal libwebp).

def _np_clip_uv(x, rnd):
    x = (x + rnd + (128 << 18)) >> 18
    return np.where((x & ~0xff) == 0, x, np.where(x < 0, 0, 255)).astype(np.uint8)


def _np_argb_to_y(argb):
    a = argb.astype(np.int64)
    r, g, b = (a >> 16) & 255, (a >> 8) & 255, a & 255
    return ((16839 * r + 33059 * g + 6420 * b + (1 << 15) + (16 << 16)) >> 16).astype(np.uint8)


def _np_argb_to_uv(argb, w, do_store, u0=None, v0=None):
    a = argb[:w].astype(np.int64)
    half = w >> 1
    p0, p1 = a[0:2 * half:2], a[1:2 * half:2]
    r = ((p0 >> 15) & 0x1fe) + ((p1 >> 15) & 0x1fe)
    g = ((p0 >> 7) & 0x1fe) + ((p1 >> 7) & 0x1fe)
    b = ((p0 << 1) & 0x1fe) + ((p1 << 1) & 0x1fe)
    if w & 1:
        q = a[w - 1]
        r = np.append(r, (q >> 14) & 0x3fc)
        g = np.append(g, (q >> 6) & 0x3fc)
        b = np.append(b, (q << 2) & 0x3fc)
    rnd = (1 << 15) << 2
    tu = _np_clip_uv(-9719 * r - 19081 * g + 28800 * b, rnd)
    tv = _np_clip_uv(28800 * r - 24116 * g - 4684 * b, rnd)
    if do_store:
        return tu, tv
    return ((u0.astype(int) + tu + 1) >> 1).astype(np.uint8), ((v0.astype(int) + tv + 1) >> 1).astype(np.uint8)


def _np_point_sample(y, u, v, w):
    out = np.zeros(3 * w, np.uint8)
    for x in range(w):
        O.lib.or_yuv_to_rgb(int(y[x]), int(u[x >> 1]), int(v[x >> 1]), O.u8(out, 3 * x))
    return out


@pytest.mark.parametrize("w", [1, 2, 3, 5, 64, 255])
def test_oracle_argb_rows_and_point_sample(w):
    r = rng(w + 100)
    argb = r.integers(0, 1 << 32, w + 3, dtype=np.uint64).astype(np.uint32)
    argb[:3] = [0xff000000, 0xffffffff, 0x00ff00ff][: min(3, w + 3)]
    assert (O.convert_argb_to_y(argb, w) == _np_argb_to_y(argb[:w])).all()
    eu, ev = _np_argb_to_uv(argb, w, True)
    gu, gv = O.convert_argb_to_uv(argb, w, True)
    assert (gu == eu).all() and (gv == ev).all()
    u0, v0 = r.integers(0, 256, (2, (w + 1) // 2), dtype=np.uint8)
    eu, ev = _np_argb_to_uv(argb, w, False, u0, v0)
    gu, gv = O.convert_argb_to_uv(argb, w, False, u0, v0)
    assert (gu == eu).all() and (gv == ev).all()
    y = r.integers(0, 256, w, dtype=np.uint8)
    u, v = r.integers(0, 256, (2, (w + 1) // 2), dtype=np.uint8)
    ps = O.point_sample_row(y, u, v, w)
    assert (ps == _np_point_sample(y, u, v, w)).all()
    # nearest sampling: pixels 2c and 2c + 1 share a chroma sample, so a flat
    # luma row gives equal RGB triples in pairs
    flat = O.point_sample_row(np.full(w, 77, np.uint8), u, v, w).reshape(w, 3)
    assert (flat[0:w - 1:2] == flat[1:w:2]).all()


@pytest.mark.gpu
@pytest.mark.parametrize("width", [1, 2, 3, 17, 1920, 1921])
@pytest.mark.parametrize("odd_dst", [False, True])
def test_gpu_point_sample_rows(cuda, width, odd_dst):
    from webp_amd import dsp
    n, cw = 5, (width + 1) // 2
    r = rng(width + 7 * odd_dst)
    y = r.integers(0, 256, (n, width + 3), dtype=np.uint8)
    u, v = r.integers(0, 256, (2, n, cw + 1), dtype=np.uint8)
    got = dsp.PointSampleRow(dev(y), dev(u), dev(v), width)
    if odd_dst:  # an odd destination pitch takes the byte-store path of the kernel
        import torch
        from webp_amd._lib import call
        buf = torch.zeros((n, 3 * width + 1), dtype=torch.uint8, device="cuda")
        yt, ut, vt = dev(y), dev(u), dev(v)
        call("wg_point_sample_rows", yt.data_ptr(), ut.data_ptr(), vt.data_ptr(), yt.stride(0), ut.stride(0),
             buf.data_ptr() + 1, buf.stride(0), width, n, torch.cuda.current_stream().cuda_stream)
        got = buf[:, 1:]
    got = host(got)
    for i in range(n):
        assert (got[i] == O.point_sample_row(y[i], u[i], v[i], width)).all(), i


@pytest.mark.gpu
@pytest.mark.parametrize("width", [1, 2, 3, 17, 1920, 1921])
def test_gpu_convert_argb_rows(cuda, width):
    import torch

    from webp_amd import dsp
    n, cw = 6, (width + 1) // 2
    r = rng(width + 11)
    argb = r.integers(0, 1 << 32, (n, width + 2), dtype=np.uint64).astype(np.uint32)
    ta = dev(argb.view(np.int32))
    y = host(dsp.ConvertARGBToY(ta, width))
    u, v = dsp.ConvertARGBToUV(ta, width, True)
    hu, hv = host(u), host(v)
    for i in range(n):
        assert (y[i] == O.convert_argb_to_y(argb[i], width)).all(), i
        eu, ev = O.convert_argb_to_uv(argb[i], width, True)
        assert (hu[i] == eu).all() and (hv[i] == ev).all(), i
    # the second row of a 2x2 block: doStore false averages into the first row's samples
    argb2 = r.integers(0, 1 << 32, (n, width), dtype=np.uint64).astype(np.uint32)
    u2, v2 = dsp.ConvertARGBToUV(dev(argb2.view(np.int32)), width, False, u, v)
    assert u2.data_ptr() == u.data_ptr()
    u2, v2 = host(u2), host(v2)
    for i in range(n):
        eu, ev = O.convert_argb_to_uv(argb2[i], width, False, hu[i], hv[i])
        assert (u2[i] == eu).all() and (v2[i] == ev).all(), i
    assert torch.cuda.is_available()


@pytest.mark.gpu
def test_gpu_block_wrappers_reject_short_rows(cuda):
    """undersized rows raise before anything reaches the GPU."""
    from webp_amd import dsp
    r = rng(3)
    pix = dev(r.integers(0, 256, (2, 16 * 16 - 1), dtype=np.uint8))
    with pytest.raises(ValueError):
        dsp.SSE(pix, pix, 16, 16, 16, 16)
    with pytest.raises(ValueError):
        dsp.DistoStatsOfBlocks(pix, pix, 16, 16, 16, 16)
    ch = dev(r.integers(0, 256, (2, 20), dtype=np.uint8))
    with pytest.raises(ValueError):
        dsp.AccumulateRGBA(ch, ch, ch, ch, 12, 10)  # needs stride + width = 22 per row
    y, c = dev(np.zeros((2, 9), np.uint8)), dev(np.zeros((2, 4), np.uint8))
    with pytest.raises(ValueError):
        dsp.UpsampleLinePair(y, y, c, c, c, c, 9)  # chroma rows need 5
    with pytest.raises(ValueError):
        dsp.PointSampleRow(y, c, c, 10)
    with pytest.raises(ValueError):
        dsp.ConvertARGBToY(dev(np.zeros((2, 3), np.int32)), 4)
