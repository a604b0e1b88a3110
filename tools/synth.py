"""Seeded synthetic inputs shared by tests/ and bench.py.

Images:  gradient  R=x%256, G=y%256, B=(x+y)%256 (bench_test.go:97-111);
                   with a seed, the same pattern from origin (13 seed, 7 seed)
         noise     uniform bytes (seeded)
         photo     testdata/test_color.png (1536x1024, the reference's own test
                   image, committed as tests/golden/test_color_png.npz) tiled,
                   from a seed-dependent origin
         blobs     smooth low-frequency pattern (lets the loop filters fire)
Macroblocks: parsed VP8 macroblock data in the wire format of
include/webpgpu.h (wg_mb_info + int16[384] coefficients): a seeded mix of
I16 / I4 macroblocks with sparse dequantised coefficient blocks whose 2-bit
nz codes are consistent with what parseResiduals (decode_mb.go:313-430)
would emit; loop-filter strengths from precomputeFilterStrengths
(decode_frame.go:220-280).  numpy only.
"""
import numpy as np

ZIGZAG = np.array([0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15])  # constants.go:86

MB_INFO_DTYPE = np.dtype([
    ("non_zero_y", "<u4"), ("non_zero_uv", "<u4"), ("imodes", "u1", (16,)),
    ("is_i4x4", "u1"), ("uv_mode", "u1"), ("skip", "u1"), ("segment", "u1"),
    ("f_limit", "u1"), ("f_ilevel", "u1"), ("f_inner", "u1"), ("hev_thresh", "u1"),
])


def gradient_rgba(w, h, seed=0):
    y, x = np.mgrid[0:h, 0:w]
    x, y = x + 13 * seed, y + 7 * seed
    img = np.empty((h, w, 4), np.uint8)
    img[..., 0] = x % 256
    img[..., 1] = y % 256
    img[..., 2] = (x + y) % 256
    img[..., 3] = 255
    return img


def noise_rgba(w, h, seed=42, alpha=False):
    rng = np.random.default_rng(seed)
    img = rng.integers(0, 256, (h, w, 4), dtype=np.uint8)
    if not alpha:
        img[..., 3] = 255
    return img


_PHOTO = None


def test_color_rgba():
    """testdata/test_color.png as RGBA (1024 x 1536 x 4), decoded once from the
    committed PNG bytes."""
    global _PHOTO
    if _PHOTO is None:
        import io
        import os

        from PIL import Image
        path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                            "test_color_png.npz")
        png = np.load(path)["png"].tobytes()
        _PHOTO = np.ascontiguousarray(np.array(Image.open(io.BytesIO(png)).convert("RGBA")))
    return _PHOTO


def photo_rgba(w, h, seed=0):
    """SURVEY 8(d) "P": test_color.png tiled to w x h (seed 0: from its
    top-left corner, as tests/golden/make_golden.py's C3 image), other seeds
    from the origin (97 seed mod 1536, 61 seed mod 1024) of the tiling."""
    img = test_color_rgba()
    ih, iw = img.shape[:2]
    x0, y0 = (97 * seed) % iw, (61 * seed) % ih
    reps = (-(-(h + y0) // ih), -(-(w + x0) // iw), 1)
    return np.ascontiguousarray(np.tile(img, reps)[y0:y0 + h, x0:x0 + w])


def blobs_rgba(w, h, seed=7, alpha=False):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w].astype(np.float64)
    img = np.empty((h, w, 4), np.uint8)
    for c in range(4):
        acc = np.zeros((h, w))
        for _ in range(4):
            fx, fy = rng.uniform(0.002, 0.03, 2)
            ph = rng.uniform(0, 6.28, 2)
            acc += np.sin(x * fx + ph[0]) * np.cos(y * fy + ph[1])
        img[..., c] = np.clip(128 + 30 * acc, 0, 255).astype(np.uint8)
    if not alpha:
        img[..., 3] = 255
    else:
        img[..., 3] = ((x.astype(np.int64) * y.astype(np.int64)) % 256).astype(np.uint8)  # SURVEY 8(d) alpha variant
    return img


def filter_strength(level, sharpness=0, i4x4=False):
    """precomputeFilterStrengths for one (segment, i4x4) (decode_frame.go:220-280),
    without LF deltas.  Returns (f_limit, f_ilevel, f_inner_base, hev_thresh)."""
    level = min(max(level, 0), 63)
    if level == 0:
        return 0, 0, int(i4x4), 0
    ilevel = level
    if sharpness > 0:
        ilevel >>= 2 if sharpness > 4 else 1
        ilevel = min(ilevel, 9 - sharpness)
    ilevel = max(ilevel, 1)
    hev = 2 if level >= 40 else (1 if level >= 15 else 0)
    return 2 * level + ilevel, ilevel, int(i4x4), hev


def _nz_code(nz, dc_nz):
    return 3 if nz > 3 else (2 if nz > 1 else dc_nz)


def random_macroblocks(n_mb, seed=1, levels=(20,), sharpness=0, p_i4=0.5, max_coeff=None, dense=False):
    """Returns (mb_info structured array [n_mb], coeffs int16 [n_mb, 384]).

    Coefficient blocks: last zigzag position L drawn so ~40% of blocks are
    empty, and at most `4` non-zero levels (Laplacian, lambda 1.5) unless
    dense=True (full-range int16 stress: every coefficient random).
    """
    rng = np.random.default_rng(seed)
    mb = np.zeros(n_mb, MB_INFO_DTYPE)
    co = np.zeros((n_mb, 384), np.int16)
    is_i4 = rng.random(n_mb) < p_i4
    mb["is_i4x4"] = is_i4
    mb["imodes"] = np.where(is_i4[:, None], rng.integers(0, 10, (n_mb, 16)),
                            np.repeat(rng.integers(0, 4, (n_mb, 1)), 16, 1))
    mb["uv_mode"] = rng.integers(0, 4, n_mb)
    seg = rng.integers(0, len(levels), n_mb)
    mb["segment"] = seg
    qdc, qac = 33, 38  # q75-ish dequant factors (KDcTable/KAcTable, constants.go:91-132)
    nzy = np.zeros(n_mb, np.uint64)
    nzuv = np.zeros(n_mb, np.uint64)
    for b in range(24):
        luma = b < 16
        first = np.where(luma & ~is_i4, 1, 0)
        if dense:
            vals = rng.integers(-32768, 32768, (n_mb, 16))
            last = np.full(n_mb, 15)
        else:
            last = rng.choice(np.arange(-1, 16), n_mb,
                              p=np.array([0.4, 0.2, 0.12, 0.08, 0.06] + [0.14 / 12] * 12))
            lv = np.maximum(1, np.round(rng.exponential(1.5, (n_mb, 16)))).astype(np.int64)
            lv *= rng.choice([-1, 1], (n_mb, 16))
            keep = rng.random((n_mb, 16)) < 0.5
            pos = np.arange(16)[None, :]
            mask = (pos <= last[:, None]) & (keep | (pos == last[:, None])) & (pos >= first[:, None])
            q = np.where(pos == 0, qdc, qac)
            vals = np.where(mask, lv * q, 0)
            # cap to "at most 4 non-zeros" like the survey's synthetic decode input
            cnt = np.cumsum(vals != 0, axis=1)
            vals = np.where(cnt <= 4, vals, 0)
            nzpos = np.where(vals != 0, pos, -1).max(axis=1)
            last = np.maximum(nzpos, first - 1)
            if max_coeff is not None:
                vals = np.clip(vals, -max_coeff, max_coeff)
        raster = np.zeros((n_mb, 16), np.int64)
        raster[:, ZIGZAG] = vals
        if luma:
            # I16: the DC slot holds the (already inverse-WHT'd) DC
            dc = np.round(rng.normal(0, 120, n_mb)).astype(np.int64) * (rng.random(n_mb) < 0.7)
            raster[:, 0] = np.where(is_i4, raster[:, 0], dc)
        co[:, 16 * b:16 * b + 16] = raster.astype(np.int16)
        nz = last + 1
        nz = np.where(first == 1, np.maximum(nz, 1), nz)
        dc_nz = (raster[:, 0] != 0).astype(np.int64)
        code = np.array([_nz_code(a, d) for a, d in zip(nz, dc_nz)], np.uint64)
        if dense:
            code = np.full(n_mb, 3, np.uint64)
        if luma:
            nzy = nzy | (code << np.uint64(30 - 2 * b))
        else:
            c = b - 16
            pl, k = c // 4, c % 4
            # U codes in bits 0..7, V in 8..15; block k of a plane at bits 2*(3-k) (row-major shift order)
            nzuv = nzuv | (code << np.uint64(8 * pl + 2 * (3 - k)))
    mb["non_zero_y"] = nzy.astype(np.uint32)
    mb["non_zero_uv"] = nzuv.astype(np.uint32)
    skip = (mb["non_zero_y"] == 0) & (mb["non_zero_uv"] == 0) & ~is_i4
    mb["skip"] = skip
    for i, lev in enumerate(levels):
        for i4 in (0, 1):
            sel = (seg == i) & (is_i4 == bool(i4))
            fl, il, inner, hev = filter_strength(lev, sharpness, bool(i4))
            mb["f_limit"][sel] = fl
            mb["f_ilevel"][sel] = il
            mb["hev_thresh"][sel] = hev
            mb["f_inner"][sel] = np.where(inner | ~skip[sel], 1, 0)  # decodeMB: FInner || !skip
    return mb, co
