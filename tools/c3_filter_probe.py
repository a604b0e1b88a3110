"""C3's real stream decoded with its own loop filter (type 2), the simple one
(1, luma only) and none (0, F only copies and stores): how much of the
4096^2 decode's time the filter wave's chain and work add to the
reconstruction chain.  Timing only (types 0 / 1 are not this stream's
output).  Not the driver bench."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from tools.bench_c3 import timed  # noqa: E402
from webp_amd import frames  # noqa: E402


def main():
    z = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                             "c3_4096_q75.npz"))
    dims, mb, co = frames.vp8_parse(z["webp"].tobytes())
    mbw, mbh = dims["mbw"], dims["mbh"]
    mbt = frames.mb_info_tensor(mb)
    cot = torch.from_numpy(co).cuda()
    for ft in (2, 1, 0, 2):
        Y, U, V = frames.decode_frames(mbt, cot, ft, mbw, mbh, 1, check=True)
        t = timed(lambda: frames.decode_frames(mbt, cot, ft, mbw, mbh, 1, out=(Y, U, V)))
        print(f"C3 real, filter type {ft}: reconstruct+filter {t:.3f} ms")


if __name__ == "__main__":
    main()
