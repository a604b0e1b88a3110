"""Dithered RGB->YUV import (ConvertRGBA32ToUVDithered +
VP8Random, importImage's dithered path internal/lossy/encode.go:690-940).

CPU: the product's dither plan (the VP8Random stream wg_dither_plan builds)
equals the oracle's generator (itself pinned by random_test.go in
tests/test_oracle.py), webp.Encode's amplitude matches for every quality, and
the kernel's per-pixel formula applied to the plan in numpy reproduces the
oracle's serial dithered import.  GPU: wg_import_rgba_dithered vs the oracle,
bit-exact."""
import ctypes

import numpy as np
import pytest

import oracle as O
from tools import synth


class Rng(ctypes.Structure):  # or_random
    _fields_ = [("index1", ctypes.c_int), ("index2", ctypes.c_int), ("tab", ctypes.c_uint32 * 55), ("amp", ctypes.c_int)]


def oracle_draws(n, num_bits):
    rg = Rng()
    O.lib.or_random_init.argtypes = [ctypes.c_void_p, ctypes.c_float]
    O.lib.or_random_bits2.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    O.lib.or_random_bits2.restype = ctypes.c_int
    O.lib.or_random_init(ctypes.byref(rg), ctypes.c_float(1.0))
    return rg, [O.lib.or_random_bits2(ctypes.byref(rg), num_bits, 256) - (1 << (num_bits - 1)) for _ in range(n)]


def plan_host(w, h):
    from webp_amd import _lib
    padw, padh = 16 * ((w + 15) >> 4), 16 * ((h + 15) >> 4)
    buf = np.zeros(_lib.lib.wg_dither_plan_bytes(w, h), np.uint8)
    _lib.call("wg_dither_plan_host", w, h, buf.ctypes.data)
    dy = buf[:padw * padh * 2].view(np.int16).reshape(padh, padw)
    duv = buf[padw * padh * 2:].view(np.int32).reshape(padh // 2, padw)
    return dy, duv


def test_amp_matches_float32_strength():
    from webp_amd import frames
    for q in range(101):
        s = O.lib.or_dithering_strength(float(q))
        x = np.float32(q) / np.float32(100.0)
        x2 = x * x
        assert np.float32(s) == np.float32(1.0) + np.float32(-0.5) * x2 * x2
        assert frames.dither_amp(q, 2) == int(np.float32(256.0) * np.float32(s))
        assert frames.dither_amp(q, 1) == 0  # no dithering without preprocessing bit 1
    assert frames.dither_amp(75, 2) == 215  # 256 * 431/512 = 215.5


def test_plan_is_the_vp8random_stream():
    w, h = 40, 20  # padded 48 x 32: 1536 Y draws, then 768 U/V draws
    dy, duv = plan_host(w, h)
    _, y16 = oracle_draws(dy.size + duv.size, 16)
    assert list(dy.reshape(-1)) == y16[:dy.size]
    # the U/V draws continue the same stream at 18 bits
    rg, _ = oracle_draws(dy.size, 16)
    uv = [O.lib.or_random_bits2(ctypes.byref(rg), 18, 256) - (1 << 17) for _ in range(duv.size)]
    assert list(duv.reshape(-1)) == uv


def numpy_dithered_y(rgba, amp):
    """The kernel's Y arithmetic (import.hip k_import<true>) in numpy over the plan."""
    h, w, _ = rgba.shape
    dy, duv = plan_host(w, h)
    padh, padw = dy.shape
    ys = np.minimum(np.arange(padh), h - 1)
    xs = np.minimum(np.arange(padw), w - 1)
    p = rgba[ys][:, xs].astype(np.int64)
    rnd = ((dy.astype(np.int64) * amp) >> 8) + (1 << 15)
    return ((16839 * p[..., 0] + 33059 * p[..., 1] + 6420 * p[..., 2] + rnd + (16 << 16)) >> 16).astype(np.uint8)


@pytest.mark.parametrize("w,h,alpha", [(33, 17, False), (64, 48, True), (17, 40, True)])
def test_numpy_y_plane_matches_oracle(w, h, alpha):
    rgba = synth.blobs_rgba(w, h, seed=w, alpha=alpha)
    amp = 215
    ey, eu, ev = O.import_rgba_dithered(rgba, has_alpha=alpha, dithering=amp / 256 + 1e-6)
    y = numpy_dithered_y(rgba, amp)
    assert (y == ey).all()
    ny, nu, nv = O.import_rgba(rgba, has_alpha=alpha)
    assert (ey != ny).any()  # dithering changes some pixels ...
    assert np.abs(ey.astype(int) - ny.astype(int)).max() <= 1  # ... by at most one step


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,alpha", [(33, 17, False), (64, 48, True), (17, 40, True), (1920, 1080, False),
                                       (7, 3, True)])
def test_gpu_dithered_import(cuda, w, h, alpha):
    import torch
    from webp_amd import frames
    imgs = [synth.blobs_rgba(w, h, seed=w, alpha=alpha), synth.noise_rgba(w, h, seed=h, alpha=alpha)]
    for q in (75, 20, 100):
        amp = frames.dither_amp(q, 2)
        Y, U, V = frames.import_rgba_dithered(torch.from_numpy(np.stack(imgs)).cuda(), amp, has_alpha=alpha)
        for i, img in enumerate(imgs):
            ey, eu, ev = O.import_rgba_dithered(img, has_alpha=alpha, quality=float(q))
            assert (Y[i].cpu().numpy() == ey).all(), (q, i, "Y")
            assert (U[i].cpu().numpy() == eu).all() and (V[i].cpu().numpy() == ev).all(), (q, i, "UV")
