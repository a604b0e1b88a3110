"""TEST INFRASTRUCTURE ONLY -- ctypes bridge to the third-party libwebp that
ships with Pillow in this image (libwebp 1.6.0 / libsharpyuv 0.4.2).

Used as a *secondary* external oracle to pin the C restatement in oracle/
(SURVEY.md 8(c)): VP8 decoding is normative, so WebPDecodeYUV pins
reconstruct + loop filter; WebPDecodeRGBA pins fancy upsampling + YUV->RGB;
WebPPictureImportRGBA pins the RGBA->YUV420 import; WebPPlaneDistortion pins
plane SSIM.  Nothing here is part of the product.  Every entry point returns
None-able results so tests can skip when Pillow's libwebp is absent.
"""
import ctypes
import glob
import os

import numpy as np

_LIBS = glob.glob("/usr/local/lib/python3.10/dist-packages/pillow.libs/libwebp-*.so*")
_SHARP = glob.glob("/usr/local/lib/python3.10/dist-packages/pillow.libs/libsharpyuv-*.so*")

lib = None
if _LIBS:
    try:
        if _SHARP:
            ctypes.CDLL(_SHARP[0], mode=ctypes.RTLD_GLOBAL)
        lib = ctypes.CDLL(_LIBS[0])
    except OSError:
        lib = None

available = lib is not None

if available:
    _u8p = ctypes.POINTER(ctypes.c_uint8)
    _ip = ctypes.POINTER(ctypes.c_int)
    lib.WebPEncodeRGBA.restype = ctypes.c_size_t
    lib.WebPEncodeRGBA.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                   ctypes.POINTER(_u8p)]
    lib.WebPEncodeLosslessRGBA.restype = ctypes.c_size_t
    lib.WebPEncodeLosslessRGBA.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           ctypes.POINTER(_u8p)]
    lib.WebPDecodeYUV.restype = _u8p
    lib.WebPDecodeYUV.argtypes = [ctypes.c_void_p, ctypes.c_size_t, _ip, _ip, ctypes.POINTER(_u8p),
                                  ctypes.POINTER(_u8p), _ip, _ip]
    lib.WebPDecodeRGBA.restype = _u8p
    lib.WebPDecodeRGBA.argtypes = [ctypes.c_void_p, ctypes.c_size_t, _ip, _ip]
    lib.WebPFree.argtypes = [ctypes.c_void_p]
    lib.WebPPlaneDistortion.restype = ctypes.c_int
    lib.WebPPlaneDistortion.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                                        ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_int,
                                        ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]
    lib.WebPPictureInitInternal.restype = ctypes.c_int
    lib.WebPPictureInitInternal.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.WebPPictureImportRGBA.restype = ctypes.c_int
    lib.WebPPictureImportRGBA.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    lib.WebPPictureFree.argtypes = [ctypes.c_void_p]
    lib.WebPPictureSharpARGBToYUVA.restype = ctypes.c_int
    lib.WebPPictureSharpARGBToYUVA.argtypes = [ctypes.c_void_p]


def encode_lossy(rgba, quality=75.0):
    """libwebp WebPEncodeRGBA -> bytes."""
    h, w, _ = rgba.shape
    rgba = np.ascontiguousarray(rgba, np.uint8)
    out = ctypes.POINTER(ctypes.c_uint8)()
    n = lib.WebPEncodeRGBA(rgba.ctypes.data, w, h, w * 4, float(quality), ctypes.byref(out))
    data = ctypes.string_at(out, n)
    lib.WebPFree(out)
    return data


def decode_yuv(data):
    """WebPDecodeYUV -> (Y, U, V) cropped planes (h x w, (h+1)/2 x (w+1)/2)."""
    w, h = ctypes.c_int(), ctypes.c_int()
    u = ctypes.POINTER(ctypes.c_uint8)()
    v = ctypes.POINTER(ctypes.c_uint8)()
    ys, uvs = ctypes.c_int(), ctypes.c_int()
    y = lib.WebPDecodeYUV(data, len(data), ctypes.byref(w), ctypes.byref(h), ctypes.byref(u), ctypes.byref(v),
                          ctypes.byref(ys), ctypes.byref(uvs))
    W, H = w.value, h.value
    cw, ch = (W + 1) // 2, (H + 1) // 2
    Y = np.ctypeslib.as_array(y, shape=(H * ys.value,)).reshape(H, ys.value)[:, :W].copy()
    U = np.ctypeslib.as_array(u, shape=((ch - 1) * uvs.value + cw,))
    V = np.ctypeslib.as_array(v, shape=((ch - 1) * uvs.value + cw,))
    Uo = np.stack([U[r * uvs.value: r * uvs.value + cw] for r in range(ch)])
    Vo = np.stack([V[r * uvs.value: r * uvs.value + cw] for r in range(ch)])
    lib.WebPFree(y)
    return Y, Uo, Vo


def decode_rgba(data):
    w, h = ctypes.c_int(), ctypes.c_int()
    p = lib.WebPDecodeRGBA(data, len(data), ctypes.byref(w), ctypes.byref(h))
    out = np.ctypeslib.as_array(p, shape=(h.value, w.value, 4)).copy()
    lib.WebPFree(p)
    return out


def plane_ssim(a, b):
    """WebPPlaneDistortion(type=1): float32 sum of per-pixel SSIM (x_step=1)."""
    a = np.ascontiguousarray(a, np.uint8)
    b = np.ascontiguousarray(b, np.uint8)
    h, w = a.shape
    dist, res = ctypes.c_float(), ctypes.c_float()
    ok = lib.WebPPlaneDistortion(a.ctypes.data, w, b.ctypes.data, w, w, h, 1, 1, ctypes.byref(dist),
                                 ctypes.byref(res))
    assert ok
    return float(dist.value)


# WebPPicture field offsets (libwebp encode.h, LP64)
_PIC_SIZE = 512
_OFF_USE_ARGB, _OFF_W, _OFF_H, _OFF_Y, _OFF_U, _OFF_V, _OFF_YS, _OFF_UVS = 0, 8, 12, 16, 24, 32, 40, 44


def _pic_planes(buf, w, h):
    def rd(off, t):
        return t.from_buffer(buf, off).value
    y = rd(_OFF_Y, ctypes.c_void_p)
    u = rd(_OFF_U, ctypes.c_void_p)
    v = rd(_OFF_V, ctypes.c_void_p)
    ys = rd(_OFF_YS, ctypes.c_int)
    uvs = rd(_OFF_UVS, ctypes.c_int)
    cw, ch = (w + 1) // 2, (h + 1) // 2
    Y = np.ctypeslib.as_array(ctypes.cast(y, ctypes.POINTER(ctypes.c_uint8)), shape=(h, ys))[:, :w].copy()
    U = np.ctypeslib.as_array(ctypes.cast(u, ctypes.POINTER(ctypes.c_uint8)), shape=(ch, uvs))[:, :cw].copy()
    V = np.ctypeslib.as_array(ctypes.cast(v, ctypes.POINTER(ctypes.c_uint8)), shape=(ch, uvs))[:, :cw].copy()
    return Y, U, V


def import_rgba(rgba):
    """WebPPictureImportRGBA with use_argb=0 -> (Y, U, V) cropped planes."""
    h, w, _ = rgba.shape
    rgba = np.ascontiguousarray(rgba, np.uint8)
    buf = (ctypes.c_uint8 * _PIC_SIZE)()
    assert lib.WebPPictureInitInternal(buf, 0x0200 + 0x10)
    ctypes.c_int.from_buffer(buf, _OFF_USE_ARGB).value = 0
    ctypes.c_int.from_buffer(buf, _OFF_W).value = w
    ctypes.c_int.from_buffer(buf, _OFF_H).value = h
    assert lib.WebPPictureImportRGBA(buf, rgba.ctypes.data, w * 4)
    planes = _pic_planes(buf, w, h)
    lib.WebPPictureFree(buf)
    return planes


# WebPConfig field offsets (libwebp encode.h; all 4-byte fields)
_CFG_SIZE = 256
_CFG_FIELDS = {"quality": (4, ctypes.c_float), "method": (8, ctypes.c_int), "segments": (24, ctypes.c_int),
               "sns_strength": (28, ctypes.c_int), "filter_strength": (32, ctypes.c_int),
               "filter_sharpness": (36, ctypes.c_int), "filter_type": (40, ctypes.c_int),
               "autofilter": (44, ctypes.c_int), "partitions": (72, ctypes.c_int),
               "use_sharp_yuv": (104, ctypes.c_int)}
_OFF_WRITER, _OFF_CUSTOM = 96, 104

if available:
    lib.WebPConfigInitInternal.restype = ctypes.c_int
    lib.WebPConfigInitInternal.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_int]
    lib.WebPValidateConfig.restype = ctypes.c_int
    lib.WebPValidateConfig.argtypes = [ctypes.c_void_p]
    lib.WebPEncode.restype = ctypes.c_int
    lib.WebPEncode.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.WebPMemoryWriterInit.argtypes = [ctypes.c_void_p]
    lib.WebPMemoryWriterClear.argtypes = [ctypes.c_void_p]


def encode_lossy_cfg(rgba, quality=75.0, **fields):
    """WebPEncode with an advanced WebPConfig (filter_type 0 = simple / 1 = strong,
    filter_sharpness, filter_strength, partitions, segments, method, ...) -> bytes."""
    h, w, _ = rgba.shape
    rgba = np.ascontiguousarray(rgba, np.uint8)
    cfg = (ctypes.c_uint8 * _CFG_SIZE)()
    assert lib.WebPConfigInitInternal(cfg, 0, float(quality), 0x0210)
    for k, v in fields.items():
        off, t = _CFG_FIELDS[k]
        t.from_buffer(cfg, off).value = v
    assert lib.WebPValidateConfig(cfg), fields
    pic = (ctypes.c_uint8 * _PIC_SIZE)()
    assert lib.WebPPictureInitInternal(pic, 0x0210)
    ctypes.c_int.from_buffer(pic, _OFF_USE_ARGB).value = 0
    ctypes.c_int.from_buffer(pic, _OFF_W).value = w
    ctypes.c_int.from_buffer(pic, _OFF_H).value = h
    assert lib.WebPPictureImportRGBA(pic, rgba.ctypes.data, w * 4)
    mw = (ctypes.c_uint8 * 64)()
    lib.WebPMemoryWriterInit(mw)
    ctypes.c_void_p.from_buffer(pic, _OFF_WRITER).value = ctypes.cast(lib.WebPMemoryWrite, ctypes.c_void_p).value
    ctypes.c_void_p.from_buffer(pic, _OFF_CUSTOM).value = ctypes.addressof(mw)
    ok = lib.WebPEncode(cfg, pic)
    mem = ctypes.c_void_p.from_buffer(mw, 0).value
    size = ctypes.c_size_t.from_buffer(mw, 8).value
    data = ctypes.string_at(mem, size) if ok else None
    lib.WebPMemoryWriterClear(mw)
    lib.WebPPictureFree(pic)
    assert ok, "WebPEncode failed"
    return data


# libsharpyuv 0.4.2 (Pillow's copy): SharpYuvConvert, the C library the
# reference's testc/sharpyuv compares its Go SharpYUV against (tolerance +-1).
sharp = None
if _SHARP:
    try:
        sharp = ctypes.CDLL(_SHARP[0])
        sharp.SharpYuvInit.argtypes = [ctypes.c_void_p]
        sharp.SharpYuvConvert.restype = ctypes.c_int
        sharp.SharpYuvConvert.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] * 3 + [ctypes.c_void_p, ctypes.c_int] * 3 + \
            [ctypes.c_int] * 3 + [ctypes.c_void_p]
        sharp.SharpYuvInit(None)
    except (OSError, AttributeError):
        sharp = None


def sharpyuv_convert(rgb, matrix):
    """SharpYuvConvert on packed RGB (h, w, 3) -> (Y, U, V) 8-bit planes."""
    rgb = np.ascontiguousarray(rgb, np.uint8)
    h, w, _ = rgb.shape
    cw, ch = (w + 1) // 2, (h + 1) // 2
    Y = np.zeros((h, w), np.uint8)
    U = np.zeros((ch, cw), np.uint8)
    V = np.zeros((ch, cw), np.uint8)
    m = np.ascontiguousarray(matrix, np.int32)
    base = rgb.ctypes.data
    ok = sharp.SharpYuvConvert(base, base + 1, base + 2, 3, 3 * w, 8, Y.ctypes.data, w, U.ctypes.data, cw,
                               V.ctypes.data, cw, 8, w, h, m.ctypes.data)
    assert ok
    return Y, U, V
