"""The reference's own test files (testdata/*.webp) and the known answers its
tests hold for them, run through the oracle (CPU) and the product (GPU).

- webp_test.go:190-221 (TestDecode_Lossless_SelectPredictor): eight ARGB
  pixels of testdata/lossless/bug-decode/input-vp8l.webp (320x320, subtract
  green + predictor transform with Select tiles), libwebp dwebp's values.
- webp_test.go:166-183 (TestDecode_Lossy_Blue16x16): the centre pixel of
  testdata/blue_16x16_lossy.webp, (1, 128, 255) per dwebp; :135-164 the red
  4x4 lossy / lossless files; :225-239 red_4x4_lossless.webp.
- Every file in full against libwebp 1.6.0's WebPDecodeRGBA
  (tests/golden/reference_testdata.npz, made by tests/golden/make_golden.py).

The VP8L files are entropy-decoded by oracle/vp8l_dec.c (test
infrastructure: the entropy coder is outside the hot path); the inverse
transforms, which are on it (A25), run on the restatement
(CPU tests) and on the GPU kernels through the C ABI (GPU tests).  The VP8
files go through the product's host parser (wg_vp8_parse), then the oracle
or the GPU reconstruct + loop filter + fancy upsample.
"""
import os

import numpy as np
import pytest

import oracle as O

REF = np.load(os.path.join(os.path.dirname(__file__), "golden", "reference_testdata.npz"))
VP8L_FILES = ["red_4x4_lossless", "gradient_8x8_lossless", "input_vp8l"]
VP8_FILES = ["blue_16x16_lossy", "red_4x4_lossy"]

# webp_test.go:207-216: (x, y, r, g, b, a)
SELECT_PREDICTOR_KAT = [(0, 0, 178, 176, 173, 255), (1, 1, 176, 174, 171, 255), (50, 50, 166, 164, 162, 255),
                        (160, 160, 5, 3, 3, 255), (319, 319, 180, 170, 157, 255), (0, 319, 163, 165, 162, 255),
                        (319, 0, 146, 146, 146, 255), (200, 100, 0, 0, 0, 255)]


def argb_to_rgba(a):
    a = np.asarray(a, np.uint32)
    return np.stack([(a >> 16) & 255, (a >> 8) & 255, a & 255, a >> 24], -1).astype(np.uint8)


def webp(name):
    return REF[name + "_webp"].tobytes()


# ---------------- CPU: oracle pinned by the reference's answers ----------------

def test_select_predictor_kat_oracle():
    dec = O.vp8l_decode_entropy(webp("input_vp8l"))
    assert (dec["width"], dec["height"]) == (320, 320)
    # the stream exercises the predictor transform (the Select regression of issue #2)
    assert O.VP8L_PREDICTOR in [t["type"] for t in dec["transforms"]]
    rgba = argb_to_rgba(O.vp8l_apply_inverse(dec))
    for x, y, *want in SELECT_PREDICTOR_KAT:
        assert tuple(rgba[y, x]) == tuple(want), (x, y)


@pytest.mark.parametrize("name", VP8L_FILES)
def test_vp8l_files_oracle_vs_libwebp(name):
    rgba = argb_to_rgba(O.vp8l_apply_inverse(O.vp8l_decode_entropy(webp(name))))
    assert (rgba == REF[name + "_rgba"]).all()


def test_vp8l_transform_kinds_covered():
    """Between them the files use all four transforms (colour indexing on the
    red 4x4, predictor + cross-colour on the gradient, subtract green +
    predictor on the regression image)."""
    kinds = set()
    for name in VP8L_FILES:
        kinds |= {t["type"] for t in O.vp8l_decode_entropy(webp(name))["transforms"]}
    assert kinds == {0, 1, 2, 3}


def oracle_decode_vp8(data):
    from test_oracle import libwebp_skip_rule
    from webp_amd import frames
    dims, mb, co = frames.vp8_parse(data)
    w, h = dims["width"], dims["height"]
    y, u, v = O.decode_frame(mb, co, dims["filter_type"], dims["mbw"], dims["mbh"])
    ly, lu, lv = O.decode_frame(libwebp_skip_rule(mb), co, dims["filter_type"], dims["mbw"], dims["mbh"])
    return dims, O.build_nrgba(y, u, v, w, h), O.build_nrgba(ly, lu, lv, w, h)


@pytest.mark.parametrize("name", VP8_FILES)
def test_vp8_files_oracle(name):
    dims, rgba, rgba_lw = oracle_decode_vp8(webp(name))
    assert (rgba_lw == REF[name + "_rgba"]).all()
    assert (rgba == rgba_lw).all()  # neither file has an all-zero non-skipped I16 macroblock


def test_blue16_centre_pixel():
    """webp_test.go:177-182: dwebp gives (1, 128, 255) at (8, 8); the test
    itself asserts B >= 200, R <= 50, A == 255."""
    _, rgba, _ = oracle_decode_vp8(webp("blue_16x16_lossy"))
    assert tuple(rgba[8, 8]) == (1, 128, 255, 255)


def test_red4_lossy_pixel():
    """webp_test.go:157-163: red-dominant pixel (0, 0)."""
    _, rgba, _ = oracle_decode_vp8(webp("red_4x4_lossy"))
    r, g, b, a = rgba[0, 0]
    assert r >= 200 and g <= 50 and b <= 50 and a == 255


# ---------------- GPU: the product's inverse transforms / decode path ----------------

def gpu_apply_inverse(dec):
    """applyInverseTransforms (decode_transform.go:134-156) on the GPU kernels."""
    import torch
    from webp_amd import lossless as L
    cur = L.to_argb_tensor(dec["pixels"][None])
    for t in reversed(dec["transforms"]):
        if t["type"] == O.VP8L_PREDICTOR:
            cur = L.predictor_inverse(L.to_argb_tensor(t["data"][None]), t["bits"], cur, check=True)
        elif t["type"] == O.VP8L_CROSS_COLOR:
            cur = L.color_space_inverse(L.to_argb_tensor(t["data"][None]), t["bits"], cur)
        elif t["type"] == O.VP8L_SUBTRACT_GREEN:
            cur = L.AddGreen(cur.clone())
        else:
            cur = L.color_index_inverse(L.to_argb_tensor(t["data"]), t["bits"], t["xsize"], cur)
    torch.cuda.synchronize()
    return L.from_argb_tensor(cur)[0]


@pytest.mark.gpu
def test_select_predictor_kat_gpu(cuda):
    rgba = argb_to_rgba(gpu_apply_inverse(O.vp8l_decode_entropy(webp("input_vp8l"))))
    for x, y, *want in SELECT_PREDICTOR_KAT:
        assert tuple(rgba[y, x]) == tuple(want), (x, y)


@pytest.mark.gpu
@pytest.mark.parametrize("name", VP8L_FILES)
def test_vp8l_files_gpu_vs_libwebp(cuda, name):
    dec = O.vp8l_decode_entropy(webp(name))
    got = gpu_apply_inverse(dec)
    assert (got == O.vp8l_apply_inverse(dec)).all()
    assert (argb_to_rgba(got) == REF[name + "_rgba"]).all()


@pytest.mark.gpu
@pytest.mark.parametrize("name", VP8_FILES)
def test_vp8_files_gpu(cuda, name):
    import torch
    from test_oracle import libwebp_skip_rule
    from webp_amd import frames
    dims, mb, co = frames.vp8_parse(webp(name))
    w, h, ft, mbw, mbh = (dims[k] for k in ("width", "height", "filter_type", "mbw", "mbh"))
    _, want, want_lw = oracle_decode_vp8(webp(name))
    for info, exp in ((mb, want), (libwebp_skip_rule(mb), REF[name + "_rgba"])):
        y, u, v = frames.decode_frames(frames.mb_info_tensor(info), torch.from_numpy(co).cuda(), ft, mbw, mbh, 1,
                                       check=True)
        rgba = frames.build_nrgba(y, u, v, w, h)
        torch.cuda.synchronize()
        assert (rgba.cpu().numpy()[0] == exp).all()
    if name == "blue_16x16_lossy":
        assert tuple(rgba.cpu().numpy()[0][8, 8]) == (1, 128, 255, 255)


# ---------------- select_predictor_test.go: the reference's Select grid ----------------

def select_grid_image():
    """TestSelectPredictorEncoderMatchesDecoder's grid (select_predictor_test.go:17-31):
    left / top / topLeft built from 9 values per channel pair, 531441 triples.
    Triple j sits in a 2 x 2 cell of a 2-wide image (rows 2j, 2j + 1): topLeft,
    top / left, target; every x > 0, y > 0 pixel uses the Select predictor
    (mode 11, 4 x 4 tiles), the target's residual is 0, and the other residuals
    are chosen so that the pixels reconstruct to the triple -- so the decoded
    target is Select(left, top, topLeft).  Select is restated here from
    selectPredictor (decode_transform.go:376-414): top if sum(|L - TL|) -
    sum(|T - TL|) <= 0, else left."""
    vals = np.array([0, 1, 7, 64, 127, 128, 200, 254, 255], np.uint32)
    g = np.stack(np.meshgrid(*([vals] * 6), indexing="ij"), -1).reshape(-1, 6)
    lr, lg, tr, tg, cr, cg = g.T
    left = 0xff000000 | lr << 16 | lg << 8 | lr
    top = 0xff000000 | tr << 16 | tg << 8 | tg
    tl = 0xff000000 | cr << 16 | cg << 8 | cr

    def chans(p):
        return np.stack([(p >> s) & 0xff for s in (0, 8, 16, 24)]).astype(np.int64)

    def select(L, T, TL):
        pa = (np.abs(chans(L) - chans(TL)) - np.abs(chans(T) - chans(TL))).sum(axis=0)
        return np.where(pa <= 0, T, L).astype(np.uint32)

    def sub(a, b):  # per-channel a - b mod 256
        return (((chans(a) - chans(b)) & 0xff) << np.array([0, 8, 16, 24])[:, None]).sum(axis=0).astype(np.uint32)

    n = len(g)
    target = select(left, top, tl)
    img = np.empty((2 * n, 2), np.uint32)
    img[0::2, 0], img[0::2, 1], img[1::2, 0], img[1::2, 1] = tl, top, left, target
    res = np.empty_like(img)
    res[0, 0] = sub(tl[:1], np.array([0xff000000], np.uint32))[0]    # black predictor
    res[0, 1] = sub(top[:1], tl[:1])[0]                              # row 0: L
    res[1:, 0] = sub(img[1:, 0], img[:-1, 0])                        # column 0: T
    res[1::2, 1] = 0                                                 # the targets
    res[2::2, 1] = sub(top[1:], select(tl[1:], target[:-1], left[:-1]))  # Select onto the next cell's top
    modes = np.full(((2 * n + 3) // 4, 1), 0xff000000 | 11 << 8, np.uint32)
    return img, res, modes


def test_select_grid_oracle():
    img, res, modes = select_grid_image()
    assert (O.vp8l_inverse_predictor(modes, 2, res) == img).all()


@pytest.mark.gpu
def test_select_grid_gpu(cuda):
    """The GPU inverse predictor's Select on the reference's test grid."""
    from webp_amd import lossless as L
    img, res, modes = select_grid_image()
    out = L.predictor_inverse(L.to_argb_tensor(modes[None]), 2, L.to_argb_tensor(res[None]), check=True)
    assert (L.from_argb_tensor(out)[0] == img).all()
