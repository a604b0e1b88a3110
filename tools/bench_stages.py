"""Per-stage timing experiments (not the driver bench): each stage of the
pipeline alone on a batch of 1920x1080 frames, with decode variants
(filter type, I4 share) to locate the cost.  Prints one line per case."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from tools import synth  # noqa: E402
from webp_amd import _lib, frames  # noqa: E402

W, H = 1920, 1080
MBW, MBH = 120, 68
B = int(os.environ.get("BATCH", "64"))
REPS = int(os.environ.get("REPS", "5"))


def timeit(fn, reps=REPS):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


def main():
    dev = torch.device("cuda")
    img = torch.from_numpy(synth.blobs_rgba(W, H, seed=3)).to(dev)
    rgba = img.unsqueeze(0).repeat(B, 1, 1, 1).contiguous()
    Y, U, V = frames.import_rgba(rgba, has_alpha=False)
    px = B * W * H
    if os.environ.get("DECODE_ONLY"):
        return decode_cases(Y, U, V, px, dev)
    if os.environ.get("ENCODE_ONLY"):
        return encode_cases(Y, U, V, px, dev)
    t = timeit(lambda: frames.import_rgba(rgba, has_alpha=False, out=(Y, U, V)))
    print(f"import      {t:8.3f} ms  {px / t / 1e3:9.1f} MPix/s  {5.5 * px / t / 1e6:7.1f} GB/s")
    al = torch.empty((B, MBW * MBH), dtype=torch.int32, device=dev)
    us = torch.empty((B,), dtype=torch.int32, device=dev)
    t = timeit(lambda: frames.analysis_alphas(Y, U, V, W, H, out=(al, us, None, None)))
    print(f"analysis    {t:8.3f} ms  {px / t / 1e3:9.1f} MPix/s  {1.5 * px / t / 1e6:7.1f} GB/s")
    out = torch.empty((B, H, W, 4), dtype=torch.uint8, device=dev)
    t = timeit(lambda: frames.build_nrgba(Y, U, V, W, H, out=out))
    print(f"upsample    {t:8.3f} ms  {px / t / 1e3:9.1f} MPix/s  {5.5 * px / t / 1e6:7.1f} GB/s")
    if os.environ.get("STREAM_ONLY"):
        return
    decode_cases(Y, U, V, px, dev)
    encode_cases(Y, U, V, px, dev)


def encode_cases(Y, U, V, px, dev):
    segs = np.stack([frames.setup_segment(q) for q in (20, 24, 28, 32)])
    mbs = MBW * MBH
    seg_ids = torch.from_numpy((np.arange(B * mbs) % 4).astype(np.uint8)).to(dev)
    import oracle as O
    proba = O.default_proba()
    out, rec = frames.encode_mbs(Y, U, V, W, H, seg_ids, segs, proba)
    t = timeit(lambda: frames.encode_mbs(Y, U, V, W, H, seg_ids, segs, proba, out=out, recon=rec))
    print(f"encode_rd   {t:8.3f} ms  {px / t / 1e3:9.1f} MPix/s  ({B} frames)")


def decode_cases(Y, U, V, px, dev):
    work = torch.empty(_lib.lib.wg_decode_work_bytes(MBW, MBH, B), dtype=torch.uint8, device=dev)
    dY, dU, dV = torch.empty_like(Y), torch.empty_like(U), torch.empty_like(V)
    for ft, p_i4 in ((2, 0.5), (0, 0.5), (2, 0.0), (2, 1.0), (1, 0.5)):
        mb, co = synth.random_macroblocks(MBW * MBH * 4, seed=11, levels=(20, 32), p_i4=p_i4)
        mb_t = frames.mb_info_tensor(mb).view(4, -1, 32)
        co_t = torch.from_numpy(co).to(dev).view(4, -1, 384)
        mbs = mb_t.repeat(B // 4, 1, 1).reshape(-1, 32).contiguous()
        cos = co_t.repeat(B // 4, 1, 1).reshape(-1, 384).contiguous()
        t = timeit(lambda: frames.decode_frames(mbs, cos, ft, MBW, MBH, B, out=(dY, dU, dV), work=work))
        print(f"decode ft={ft} i4={p_i4:.1f} {t:8.3f} ms  {px / t / 1e3:9.1f} MPix/s")


if __name__ == "__main__":
    main()
