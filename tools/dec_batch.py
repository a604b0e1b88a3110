"""Diagnostic: decode (reconstruct + filter, k_decode_split) time of the
bench's libwebp q75 1080p bitstreams: one frame of each content alone, and
the bench's 64-frame mix -- how far the batch is above its slowest frame's
wavefront."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from webp_amd import frames  # noqa: E402

parsed = bench.parsed_bitstreams()
MBW, MBH = bench.MBW, bench.MBH


def timed(kinds):
    n = len(kinds)
    mb = frames.mb_info_tensor(np.concatenate([parsed[k][0] for k in kinds]))
    co = torch.from_numpy(np.concatenate([parsed[k][1] for k in kinds])).cuda()
    Y, U, V = frames.decode_frames(mb, co, 2, MBW, MBH, n, check=True)
    ts = []
    for _ in range(9):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        frames.decode_frames(mb, co, 2, MBW, MBH, n, out=(Y, U, V))
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


for k in bench.CONTENTS:
    print(f"1 x {k}: {timed([k]):.3f} ms", flush=True)
mix = [bench.CONTENTS[i % 3] for i in range(64)]
print(f"64 mixed: {timed(mix):.3f} ms", flush=True)
print(f"64 heavy-first order: {timed(sorted(mix, key=lambda k: k != 'noise')):.3f} ms", flush=True)
