"""C3 (BASELINE.json configs[2]) and single-frame latencies on one GPU.

  C3 real: one 4096x4096 lossy decode of a libwebp q75 bitstream of the tiled
      testdata/test_color.png (tests/golden/c3_4096_q75.npz): the host parse
      (wg_vp8_parse) timed apart, then reconstruct + loop filter
      (k_decode_split) + fancy upsample to NRGBA (k_upsample) on the GPU;
  C3 synthetic: the same decode from seeded synthetic parsed macroblocks
      (SURVEY.md 8(d) recipe, normal filter, half I4), also at batch 4 / 16;
  C2: one 1920x1080 q75 encode RD pass (k_encode_rows) on each content type;
  plus the same decode at batch 4 / 16 to show where a single image stops
  filling the chip.
Prints one line per case (ms, MPix/s).  Not the driver bench."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402
from tools import synth  # noqa: E402
from webp_amd import frames  # noqa: E402

REPS = int(os.environ.get("REPS", "5"))


def timed(fn):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(REPS):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


def decode_case(n_img, w, h):
    mbw, mbh = (w + 15) >> 4, (h + 15) >> 4
    mb, co = synth.random_macroblocks(mbw * mbh, seed=5, levels=(20, 32))
    mbt = frames.mb_info_tensor(np.tile(mb, n_img))
    cot = torch.from_numpy(np.tile(co, (n_img, 1))).cuda()
    Y, U, V = frames.decode_frames(mbt, cot, 2, mbw, mbh, n_img, check=True)
    out = frames.build_nrgba(Y, U, V, w, h)
    t_dec = timed(lambda: frames.decode_frames(mbt, cot, 2, mbw, mbh, n_img, out=(Y, U, V)))
    t_up = timed(lambda: frames.build_nrgba(Y, U, V, w, h, out=out))
    px = n_img * w * h
    print(f"decode {n_img}x{w}x{h}: reconstruct+filter {t_dec:.3f} ms, upsample {t_up:.3f} ms, "
          f"total {t_dec + t_up:.3f} ms = {px / (t_dec + t_up) / 1e3:.1f} MPix/s")


def decode_real():
    import time
    z = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                             "c3_4096_q75.npz"))
    data = z["webp"].tobytes()
    t0 = time.perf_counter()
    dims, mb, co = frames.vp8_parse(data)
    t_parse = (time.perf_counter() - t0) * 1e3
    w, h, mbw, mbh, ft = dims["width"], dims["height"], dims["mbw"], dims["mbh"], dims["filter_type"]
    mbt = frames.mb_info_tensor(mb)
    cot = torch.from_numpy(co).cuda()
    Y, U, V = frames.decode_frames(mbt, cot, ft, mbw, mbh, 1, check=True)
    out = frames.build_nrgba(Y, U, V, w, h)
    t_dec = timed(lambda: frames.decode_frames(mbt, cot, ft, mbw, mbh, 1, out=(Y, U, V)))
    t_up = timed(lambda: frames.build_nrgba(Y, U, V, w, h, out=out))
    i4 = float(mb["is_i4x4"].mean())
    print(f"decode C3 real q75 {w}x{h} (test_color tiled, {len(data)} B, {i4:.2f} I4, filter {ft}): host parse "
          f"{t_parse:.1f} ms; reconstruct+filter {t_dec:.3f} ms, upsample {t_up:.3f} ms, total {t_dec + t_up:.3f} ms "
          f"= {w * h / (t_dec + t_up) / 1e3:.1f} MPix/s")


def encode_case(kind, w=1920, h=1080):
    """C2: the encode DSP path of one frame at the reference's q75 defaults
    (import -> analysis -> segment analysis -> MB RD, frames.encode_frames),
    and its RD launch alone."""
    mbw, mbh = (w + 15) >> 4, (h + 15) >> 4
    gen = {"gradient": lambda: synth.gradient_rgba(w, h), "noise": lambda: synth.noise_rgba(w, h, seed=3),
           "blobs": lambda: synth.blobs_rgba(w, h, seed=3)}[kind]
    rgba = torch.from_numpy(gen()[None]).cuda()
    out, rec, seg_ids, segs, _ = frames.encode_frames(rgba)
    t_full = timed(lambda: frames.encode_frames(rgba, check=False))
    Y, U, V = frames.import_rgba(rgba, has_alpha=False)
    proba = O.default_proba()
    t = timed(lambda: frames.encode_mbs(Y, U, V, w, h, seg_ids, segs, proba, out=out, recon=rec))
    print(f"encode C2 1x{w}x{h} {kind}: import+analysis+segments+RD {t_full:.3f} ms = {w * h / t_full / 1e3:.1f} "
          f"MPix/s; RD alone {t:.3f} ms")


def main():
    decode_real()
    for n in (1, 4, 16):
        decode_case(n, 4096, 4096)
    if os.environ.get("C3_ONLY") != "1":
        for kind in ("gradient", "blobs", "noise"):
            encode_case(kind)


if __name__ == "__main__":
    main()
