"""C3 on real content: one 4096x4096
libwebp 1.6.0 q75 bitstream of the tiled testdata/test_color.png
(tests/golden/c3_4096_q75.npz, made by tests/golden/make_golden.py), decoded
through the reference's path -- the parse (decode.go:207-560), reconstructRow +
filterRowAt (decode.go:532-560) and buildNRGBA (webp.go:379-450):

  CPU  the oracle's decode + build_nrgba equals libwebp's WebPDecodeYUV /
       WebPDecodeRGBA at full size (SHA-256 of libwebp's pixels, kept in the
       fixture), under libwebp's skip rule (test_oracle.libwebp_skip_rule);
  GPU  wg_vp8_parse -> wg_decode_frames -> wg_upsample_nrgba equals the oracle
       bit for bit on every pixel at 4096x4096, and libwebp's hashes under
       libwebp's skip rule."""
import hashlib
import os

import numpy as np
import pytest

import oracle as O
from test_oracle import libwebp_skip_rule
from webp_amd import frames

Z = np.load(os.path.join(os.path.dirname(__file__), "golden", "c3_4096_q75.npz"))
W = H = 4096


def sha(a):
    return np.frombuffer(hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest(), np.uint8)


def parsed():
    dims, mb, co = frames.vp8_parse(Z["webp"].tobytes())
    assert (dims["width"], dims["height"], dims["mbw"], dims["mbh"]) == (W, H, 256, 256)
    return dims, mb, co


def test_c3_oracle_vs_libwebp():
    dims, mb, co = parsed()
    y, u, v = O.decode_frame(libwebp_skip_rule(mb), co, dims["filter_type"], 256, 256)
    assert (sha(y[:H, :W]) == Z["y_sha256"]).all()
    assert (sha(u[:H // 2, :W // 2]) == Z["u_sha256"]).all() and (sha(v[:H // 2, :W // 2]) == Z["v_sha256"]).all()
    assert (sha(O.build_nrgba(y, u, v, W, H)) == Z["rgba_sha256"]).all()


@pytest.mark.gpu
def test_c3_gpu_vs_oracle_and_libwebp(cuda):
    import torch
    dims, mb, co = parsed()
    ft = dims["filter_type"]
    d_co = torch.from_numpy(co).cuda()
    # the reference's rule: bit-exact against the oracle on every pixel
    Y, U, V = frames.decode_frames(frames.mb_info_tensor(mb), d_co, ft, 256, 256, 1, check=True)
    rgba = frames.build_nrgba(Y, U, V, W, H)
    torch.cuda.synchronize()
    ey, eu, ev = O.decode_frame(mb, co, ft, 256, 256)
    assert (Y[0].cpu().numpy() == ey).all() and (U[0].cpu().numpy() == eu).all() and (V[0].cpu().numpy() == ev).all()
    assert (rgba[0].cpu().numpy() == O.build_nrgba(ey, eu, ev, W, H)).all()
    # libwebp's rule: its WebPDecodeRGBA pixels (by hash)
    Y, U, V = frames.decode_frames(frames.mb_info_tensor(libwebp_skip_rule(mb)), d_co, ft, 256, 256, 1, check=True)
    rgba = frames.build_nrgba(Y, U, V, W, H)
    assert (sha(rgba[0].cpu().numpy()) == Z["rgba_sha256"]).all()
