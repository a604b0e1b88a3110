"""Decode (reconstruct + filter) timing by shape, one image: 1 MB row, one
band (4 rows), two bands, ... up to 4096x4096 -- separates the per-MB time of
a row from the row-to-row and band-to-band lag.  Seeded synthetic
macroblocks (half I4, normal filter)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from tools import synth  # noqa: E402
from webp_amd import frames  # noqa: E402

REPS = int(os.environ.get("REPS", "10"))
P_I4 = float(os.environ.get("P_I4", "0.5"))


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


def main():
    mbw = 256
    for mbh in (1, 2, 4, 8, 16, 64, 256):
        mb, co = synth.random_macroblocks(mbw * mbh, seed=5, levels=(20, 32), p_i4=P_I4)
        mbt = frames.mb_info_tensor(mb)
        cot = torch.from_numpy(co).cuda()
        out = frames.decode_frames(mbt, cot, 2, mbw, mbh, 1, check=True)
        ms = timed(lambda: frames.decode_frames(mbt, cot, 2, mbw, mbh, 1, out=out))
        print(f"{mbw}x{mbh} MBs: {ms:.3f} ms = {ms * 1e3 / mbw:.2f} us per MB of a row")


if __name__ == "__main__":
    main()
