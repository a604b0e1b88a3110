"""Alpha-plane filters and alpha processing.

CPU: the C restatement (oracle/alpha.c) --
  * unfilter(filter(x)) == x for every filter and ragged shapes (1xN, Nx1);
  * estimateBestFilter + getNumColors pinned against libwebp 1.6.0 (Pillow's
    copy): encoded at method 3 with 16 < colours <= 192, libwebp tries only
    its estimated filter (alpha_enc.c GetFilterMap, mirrored by
    alpha.go:271-300), so the ALPH header's filter bits == the estimate;
  * premultiply / 4444 / dispatch / extract / the row helpers against
    independent numpy statements of alpha_proc.go.
The inverse premultiply follows the Go code (alphaGetScale, alpha_proc.go:19:
(255<<24)/a), which differs from libwebp's by design (testc/alpha says so),
so it is pinned by restatement only.
GPU (-m gpu): every wg_alpha_* / wg_* alpha entry point == oracle, bit-exact,
incl. gradient unfilter across many 64-row bands and odd widths."""
import numpy as np
import pytest

import oracle as O

SHAPES = [(1, 1), (1, 9), (9, 1), (2, 2), (37, 53), (65, 64), (66, 65), (130, 67), (200, 301)]


def plane(h, w, seed, kind="noise"):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    if kind == "noise":
        return rng.integers(0, 256, (h, w), dtype=np.uint8)
    if kind == "grad":
        return ((x * 3 + y * 2) % 256).astype(np.uint8)
    return (((x // 7) * 13 + (y // 5) * 11 + rng.integers(0, 3, (h, w))) % 256).astype(np.uint8)


@pytest.mark.parametrize("f", [0, 1, 2, 3])
def test_filter_round_trip(f):
    for i, (h, w) in enumerate(SHAPES):
        for kind in ("noise", "grad", "steps"):
            p = plane(h, w, i, kind)
            d = O.alpha_filter(f, p)
            assert (O.alpha_unfilter(f, d) == p).all(), (f, h, w, kind)


def test_filter_definitions():
    """Spot checks straight from alpha.go:387-454 on a 3x3 plane."""
    p = np.array([[10, 20, 5], [30, 25, 250], [0, 255, 7]], np.uint8)
    h = O.alpha_filter(1, p).astype(np.int64)
    assert h.tolist() == [[10, 10, 241], [20, 251, 225], [226, 255, 8]]
    v = O.alpha_filter(2, p).astype(np.int64)
    assert v.tolist() == [[10, 10, 241], [20, 5, 245], [226, 230, 13]]
    g = O.alpha_filter(3, p).astype(np.int64)
    # row 1: x=1 pred clip(30+20-10)=40 -> 25-40; x=2 pred clip(25+5-20)=10 -> 240
    assert g[1].tolist() == [20, (25 - 40) & 255, 240]
    assert (O.alpha_filter(0, p) == p).all()


def _alph_filter_bits(data):
    i = 12
    while i + 8 <= len(data):
        tag, n = data[i:i + 4], int.from_bytes(data[i + 4:i + 8], "little")
        if tag == b"ALPH":
            return (data[i + 8] >> 2) & 3
        i += 8 + n + (n & 1)
    return None


def test_estimate_best_filter_vs_libwebp():
    import libwebp_ref as L
    if not L.available:
        pytest.skip("Pillow's libwebp not present")
    rng = np.random.default_rng(1)
    seen = set()
    for w, h in [(64, 48), (101, 37)]:
        y, x = np.mgrid[0:h, 0:w]
        cases = [((x * 3) // 2 % 64 + 60 + rng.integers(0, 3, (h, w))), ((y * 2) % 100 + 20 + (x // 16)),
                 ((x + y) % 150 + rng.integers(0, 2, (h, w))), rng.integers(100, 150, (h, w)),
                 (((x // 7) * 13 + (y // 5) * 11) % 180), ((x * y) % 97 + 50)]
        for a in cases:
            a = a.astype(np.uint8)
            nc = O.alpha_num_colors(a)
            assert nc == len(np.unique(a))
            if not 16 < nc <= 192:
                continue
            rgba = rng.integers(0, 256, (h, w, 4), dtype=np.uint8)
            rgba[..., 3] = a
            got = _alph_filter_bits(L.encode_lossy_cfg(rgba, 75.0, method=3))
            est = O.alpha_estimate_best_filter(a)
            assert got == est, (w, h, nc, got, est)
            seen.add(est)
    assert seen >= {0, 1, 2, 3}, seen  # every filter id exercised


# ---- premultiply: independent numpy statements of alpha_proc.go:13-135 ----

def np_scale(a, inverse):
    a = a.astype(np.uint64)
    return np.where(a == 0, 0, (255 << 24) // np.maximum(a, 1)) if inverse else a * ((1 << 24) // 255)


def np_mult(x, s):
    return ((x.astype(np.uint64) * s + (1 << 23)) >> 24) & 0xff


def np_apply(px, ao, ro, inverse):
    """px (N, 4) uint8 pixels."""
    out = px.copy()
    a = px[:, ao].astype(np.uint64)
    s = np_scale(a, inverse)
    for c in range(3):
        v = np_mult(px[:, ro + c], s)
        out[:, ro + c] = np.where(a == 255, px[:, ro + c], np.where(a == 0, 0, v)).astype(np.uint8)
    return out


def pixels(n, seed):
    rng = np.random.default_rng(seed)
    px = rng.integers(0, 256, (n, 4), dtype=np.uint8)
    for ao in (0, 3):
        k = rng.integers(0, 4, n)
        px[k == 0, ao] = 0
        px[k == 1, ao] = 255
    return px


@pytest.mark.parametrize("alpha_first", [False, True])
@pytest.mark.parametrize("inverse", [False, True])
def test_apply_alpha_multiply(alpha_first, inverse):
    h, w, stride = 13, 21, 21 * 4 + 12
    buf = np.random.default_rng(3).integers(0, 256, (h, stride), dtype=np.uint8)
    buf[:, :w * 4] = pixels(h * w, 4).reshape(h, w * 4)
    got = O.apply_alpha_multiply(buf, alpha_first, inverse, width=w)
    ao, ro = (0, 1) if alpha_first else (3, 0)
    want = buf.copy()
    want[:, :w * 4] = np_apply(buf[:, :w * 4].reshape(-1, 4), ao, ro, inverse).reshape(h, w * 4)
    assert (got == want).all()


@pytest.mark.parametrize("inverse", [False, True])
def test_mult_argb(inverse):
    px = pixels(4096, 5)
    words = px.view("<u4").reshape(-1)  # little-endian: B G R A = 0xAARRGGBB
    got = O.mult_argb(words, inverse)
    want = np_apply(px, 3, 0, inverse).view("<u4").reshape(-1)
    a = words >> 24
    want = np.where(a == 0, 0, want)  # MultARGBRow zeroes the whole word (alpha is 0 anyway)
    assert (got == want).all()


def test_apply_alpha_multiply_4444():
    h, w, stride = 9, 17, 17 * 2 + 6
    buf = np.random.default_rng(6).integers(0, 256, (h, stride), dtype=np.uint8)
    buf[::3, 1:w * 2:2] |= 0x0f
    buf[1::3, 1:w * 2:2] &= 0xf0
    got = O.apply_alpha_multiply_4444(buf, width=w)
    rg, ba = buf[:, 0:w * 2:2].astype(np.int64), buf[:, 1:w * 2:2].astype(np.int64)
    a = ba & 15
    r, g, b = ((rg >> 4) * a + 7) // 15, ((rg & 15) * a + 7) // 15, ((ba >> 4) * a + 7) // 15
    want = buf.copy()
    keep = a == 15
    want[:, 0:w * 2:2] = np.where(keep, rg, (r << 4) | g)
    want[:, 1:w * 2:2] = np.where(keep, ba, (b << 4) | a)
    assert (got == want).all()


@pytest.mark.parametrize("alpha_off", [0, 3])
def test_dispatch_extract(alpha_off):
    rng = np.random.default_rng(7)
    h, w = 5, 17
    al = rng.integers(0, 256, (h, w + 3), dtype=np.uint8)
    dst = rng.integers(0, 256, (h, w * 4 + 8), dtype=np.uint8)
    d, any_t = O.dispatch_alpha(al, dst, alpha_off, width=w)
    want = dst.copy()
    want[:, alpha_off:w * 4:4] = al[:, :w]
    assert (d == want).all() and any_t
    opaque = np.full_like(al, 255)
    _, any_t = O.dispatch_alpha(opaque, dst, alpha_off, width=w)
    assert not any_t
    a2, all_op = O.extract_alpha(d, np.zeros((h, w + 1), np.uint8), alpha_off, width=w)
    assert (a2[:, :w] == al[:, :w]).all() and (a2[:, w:] == 0).all() and all_op == 0
    d2, _ = O.dispatch_alpha(opaque, dst, alpha_off, width=w)
    _, all_op = O.extract_alpha(d2, np.zeros((h, w), np.uint8), alpha_off, width=w)
    assert all_op == 1


def test_row_helpers():
    rng = np.random.default_rng(8)
    b = np.full(100, 255, np.uint8)
    assert not O.has_alpha(b, 1)
    b[77] = 3
    assert O.has_alpha(b, 1)
    assert not O.has_alpha(b, 4)  # 77 is not an alpha position at step 4
    b4 = np.full(64, 255, np.uint8)
    b4[5] = 0  # not an alpha position for step 4
    assert not O.has_alpha(b4, 4)
    b4[8] = 0
    assert O.has_alpha(b4, 4)
    argb = rng.integers(0, 2 ** 32, 500, dtype=np.uint64).astype(np.uint32)
    argb[::7] &= 0x00ffffff
    got = O.alpha_replace(argb, 0xdeadbeef)
    assert (got == np.where(argb >> 24 == 0, np.uint32(0xdeadbeef), argb)).all()
    al = rng.integers(0, 256, (6, 11), dtype=np.uint8)
    g = O.dispatch_alpha_to_green(al, 13)
    assert (g[:, :11] == al.astype(np.uint32) << 8).all() and (g[:, 11:] == 0).all()
    assert (O.extract_green(argb) == ((argb >> 8) & 0xff)).all()
    r, gg, bb = (rng.integers(0, 256, 90, dtype=np.uint8) for _ in range(3))
    p = O.pack_rgb(r, gg, bb, 30, 3)
    want = 0xff000000 | r[::3].astype(np.uint32) << 16 | gg[::3].astype(np.uint32) << 8 | bb[::3]
    assert (p == want).all()


# ------------------------------------------------------------------ GPU

def _t(a, dev):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _u32(a):
    return np.ascontiguousarray(a, np.uint32).view(np.int32)


@pytest.mark.gpu
def test_gpu_filter_unfilter(cuda):
    import torch
    from webp_amd import alpha as A
    shapes = SHAPES + [(700, 513), (1, 4096), (4096, 3)]
    for f in range(4):
        for i, (h, w) in enumerate(shapes):
            for kind in ("noise", "steps"):
                n = 3 if h * w < 100000 else 1
                p = np.stack([plane(h, w, 10 * i + k, kind) for k in range(n)])
                want_f = np.stack([O.alpha_filter(f, x) for x in p])
                got_f = A.alpha_filter(f, _t(p, cuda)).cpu().numpy()
                assert (got_f == want_f).all(), ("filter", f, h, w, kind)
                d = _t(want_f, cuda)
                A.alpha_unfilter(f, d, check=True)
                got = d.cpu().numpy()
                assert (got == p).all(), ("unfilter", f, h, w, kind, np.argwhere(got != p)[:4])
    torch.cuda.synchronize()


@pytest.mark.gpu
def test_gpu_unfilter_arbitrary_residuals(cuda):
    """Unfilter of random residual planes (not produced by the forward filter)."""
    from webp_amd import alpha as A
    for f in (1, 2, 3):
        for i, (h, w) in enumerate([(130, 67), (257, 129), (1000, 61), (64 * 9 + 2, 200)]):
            r = np.stack([plane(h, w, 100 + 5 * i + k) for k in range(2)])
            want = np.stack([O.alpha_unfilter(f, x) for x in r])
            d = _t(r, cuda)
            A.alpha_unfilter(f, d, check=True)
            assert (d.cpu().numpy() == want).all(), (f, h, w)


@pytest.mark.gpu
def test_gpu_estimate(cuda):
    from webp_amd import alpha as A
    planes = []
    for i, (h, w) in enumerate([(1, 1), (3, 3), (4, 5), (37, 53), (48, 64), (101, 37)]):
        for kind in ("noise", "grad", "steps"):
            planes.append(plane(h, w, i, kind))
    for p in planes:
        assert A.estimate_best_filter(_t(p, cuda)) == O.alpha_estimate_best_filter(p), p.shape
        assert A.get_num_colors(_t(p, cuda)) == O.alpha_num_colors(p), p.shape
    # batched: images straddling colour-count blocks
    b = np.stack([plane(37, 53, k, ("noise", "grad", "steps")[k % 3]) for k in range(7)])
    best, colors = A.estimate_best_filter_async(_t(b, cuda))
    assert best.tolist() == [O.alpha_estimate_best_filter(x) for x in b]
    assert colors.tolist() == [O.alpha_num_colors(x) for x in b]


@pytest.mark.gpu
def test_gpu_premultiply(cuda):
    from webp_amd import alpha as A
    h, w, stride = 33, 45, 45 * 4 + 8
    rng = np.random.default_rng(9)
    for alpha_first in (False, True):
        for inverse in (False, True):
            imgs = rng.integers(0, 256, (3, h * stride), dtype=np.uint8)
            for k in range(3):
                imgs[k].reshape(h, stride)[:, :w * 4] = pixels(h * w, k).reshape(h, w * 4)
            want = np.stack([O.apply_alpha_multiply(x.reshape(h, stride), alpha_first, inverse, width=w).reshape(-1)
                             for x in imgs])
            t = _t(imgs, cuda)
            A.ApplyAlphaMultiply(t, alpha_first, w, h, stride, inverse)
            assert (t.cpu().numpy() == want).all(), (alpha_first, inverse)
    for inverse in (False, True):
        words = pixels(10007, 11).view("<u4").reshape(-1)
        t = _t(_u32(words), cuda)
        A.MultARGBRow(t, inverse)
        assert (t.cpu().numpy().view(np.uint32) == O.mult_argb(words, inverse)).all()
    buf = rng.integers(0, 256, (2, 19 * 40), dtype=np.uint8)
    want = np.stack([O.apply_alpha_multiply_4444(x.reshape(19, 40), width=17).reshape(-1) for x in buf])
    t = _t(buf, cuda)
    A.ApplyAlphaMultiply4444(t, 17, 19, 40)
    assert (t.cpu().numpy() == want).all()


@pytest.mark.gpu
def test_gpu_dispatch_extract_helpers(cuda):
    import torch
    from webp_amd import alpha as A
    rng = np.random.default_rng(12)
    for (h, w) in [(5, 17), (300, 301)]:
        for alpha_off in (0, 3):
            for opaque in (False, True):
                al = rng.integers(0, 256, (h, w + 3), dtype=np.uint8)
                if opaque:
                    al[:] = 255
                dst = rng.integers(0, 256, (h, w * 4 + 8), dtype=np.uint8)
                want_d, want_any = O.dispatch_alpha(al, dst, alpha_off, width=w)
                td = _t(dst, cuda)
                got_any = A.DispatchAlpha(_t(al, cuda), w + 3, w, h, td, w * 4 + 8, alpha_off)
                assert got_any == want_any and (td.cpu().numpy() == want_d).all()
                want_a, want_op = O.extract_alpha(want_d, np.zeros((h, w + 1), np.uint8), alpha_off, width=w)
                ta = torch.zeros((h, w + 1), dtype=torch.uint8, device=cuda)
                got_op = A.ExtractAlpha(_t(want_d, cuda), w * 4 + 8, w, h, ta, w + 1, alpha_off)
                assert got_op == want_op and (ta.cpu().numpy() == want_a).all()
    b = np.full(100003, 255, np.uint8)
    assert not A.HasAlpha8b(_t(b, cuda), b.size) and not A.HasAlpha32b(_t(b, cuda), b.size // 4)
    b[99999] = 7
    assert A.HasAlpha8b(_t(b, cuda), b.size) == O.has_alpha(b, 1)
    assert A.HasAlpha32b(_t(b, cuda), b.size // 4) == O.has_alpha(b, 4)
    b[4 * 1000] = 0
    assert A.HasAlpha32b(_t(b, cuda), b.size // 4) == O.has_alpha(b, 4) is True
    argb = rng.integers(0, 2 ** 32, 70001, dtype=np.uint64).astype(np.uint32)
    argb[::5] &= 0x00ffffff
    t = _t(_u32(argb), cuda)
    A.AlphaReplace(t, argb.size, 0xdeadbeef)
    assert (t.cpu().numpy().view(np.uint32) == O.alpha_replace(argb, 0xdeadbeef)).all()
    al = rng.integers(0, 256, (41, 57), dtype=np.uint8)
    g = torch.zeros((41, 60), dtype=torch.int32, device=cuda)
    A.DispatchAlphaToGreen(_t(al, cuda), 57, 57, 41, g, 60)
    assert (g.cpu().numpy().view(np.uint32) == O.dispatch_alpha_to_green(al, 60)).all()
    out = torch.empty(argb.size, dtype=torch.uint8, device=cuda)
    A.ExtractGreen(_t(_u32(argb), cuda), out, argb.size)
    assert (out.cpu().numpy() == O.extract_green(argb)).all()
    r, gg, bb = (rng.integers(0, 256, 3 * 5000, dtype=np.uint8) for _ in range(3))
    po = torch.empty(5000, dtype=torch.int32, device=cuda)
    A.PackRGB(_t(r, cuda), _t(gg, cuda), _t(bb, cuda), 5000, 3, po)
    assert (po.cpu().numpy().view(np.uint32) == O.pack_rgb(r, gg, bb, 5000, 3)).all()


def _bins_np(p):
    """estimateBestFilter's 4 x 16 'seen' bins (alpha.go:321-375) as one 64-bit word."""
    h, w = p.shape
    a = p.astype(np.int64)
    seen = 0
    for j in range(2, h - 1, 2):
        mean = int(a[j, 0])
        for i in range(2, w - 1, 2):
            cur = int(a[j, i])
            seen |= 1 << (abs(cur - mean) >> 4)
            mean = (3 * mean + cur + 2) >> 2
    if h > 3 and w > 3:
        j = np.arange(2, h - 1, 2)[:, None]
        i = np.arange(2, w - 1, 2)[None, :]
        cur, left, top, tl = a[j, i], a[j, i - 1], a[j - 1, i], a[j - 1, i - 1]
        grad = np.clip(left + top - tl, 0, 255)
        for f, d in ((1, np.abs(cur - left) >> 4), (2, np.abs(cur - top) >> 4), (3, np.abs(cur - grad) >> 4)):
            for v in np.unique(d):
                seen |= 1 << (16 * f + int(v))
    return seen


@pytest.mark.gpu
def test_gpu_estimate_bins(cuda):
    """The raw bins (work buffer word per image) == a numpy statement, on planes
    whose bins are sparse, fast-path (w % 16 == 0) and byte-path widths."""
    import torch
    from webp_amd._lib import call, lib
    for i, (h, w) in enumerate([(64, 128), (130, 96), (33, 47), (200, 256), (5, 16), (71, 1000)]):
        y, x = np.mgrid[0:h, 0:w]
        rng = np.random.default_rng(i)
        kinds = [((x * 3 + y) % 256), ((x // 9) * 20 + (y // 7) * 5) % 256, rng.integers(0, 40, (h, w)),
                 (((x * y) >> 4) % 256)]
        b = np.stack([k.astype(np.uint8) for k in kinds])
        n = b.shape[0]
        t = torch.from_numpy(b).to(cuda).contiguous()
        best = torch.empty(n, dtype=torch.int32, device=cuda)
        colors = torch.empty(n, dtype=torch.int32, device=cuda)
        work = torch.empty(lib.wg_alpha_estimate_work_bytes(n), dtype=torch.uint8, device=cuda)
        call("wg_alpha_estimate_filter", t.data_ptr(), w, h, h * w, n, best.data_ptr(), colors.data_ptr(),
             work.data_ptr(), torch.cuda.current_stream().cuda_stream)
        bins = work[:8 * n].cpu().numpy().view(np.uint64)
        for k in range(n):
            assert int(bins[k]) == _bins_np(b[k]), (h, w, k, hex(int(bins[k])), hex(_bins_np(b[k])))
            assert int(best[k]) == O.alpha_estimate_best_filter(b[k])
            assert int(colors[k]) == O.alpha_num_colors(b[k])


@pytest.mark.gpu
def test_gpu_unfilter_fast_path_bands(cuda):
    """16-B-aligned widths through the LDS-staged gradient walk and the
    segmented vertical scan: several chunks and bands, ragged last band."""
    from webp_amd import alpha as A
    for f in (2, 3):
        for i, (h, w) in enumerate([(64 * 5 + 2, 320), (129, 256), (2, 64), (700, 4096 // 8), (18, 16), (66, 64),
                                    (64 * 3 + 1, 80), (1025, 1024), (2, 4096), (200, 4096 + 16)]):
            r = np.stack([plane(h, w, 300 + 5 * i + k) for k in range(3)])
            want = np.stack([O.alpha_unfilter(f, x) for x in r])
            d = _t(r, cuda)
            A.alpha_unfilter(f, d, check=True)
            assert (d.cpu().numpy() == want).all(), (f, h, w)


@pytest.mark.gpu
def test_gpu_gradient_unfilter_both_walks(cuda, monkeypatch):
    """The register-resident diagonal walk (k_alpha_gdiag, 16-B widths >= 64)
    and the LDS-staged one it replaced (k_alpha_gbands, forced by
    WG_ALPHA_GBANDS) give the oracle's planes; every 16-step chunk offset,
    ragged last bands, a 1-row last band, and 4096-wide rows."""
    from webp_amd import alpha as A
    shapes = [(66, 64), (130, 96), (64 * 4 + 1, 4096), (64 + 17, 2048 + 48)]
    for use_old in (False, True):
        if use_old:
            monkeypatch.setenv("WG_ALPHA_GBANDS", "1")
        else:
            monkeypatch.delenv("WG_ALPHA_GBANDS", raising=False)
        for i, (h, w) in enumerate(shapes):
            r = np.stack([plane(h, w, 700 + 3 * i + k) for k in range(2)])
            want = np.stack([O.alpha_unfilter(3, x) for x in r])
            d = _t(r, cuda)
            A.alpha_unfilter(3, d, check=True)
            assert (d.cpu().numpy() == want).all(), (use_old, h, w, np.argwhere(d.cpu().numpy() != want)[:4])
