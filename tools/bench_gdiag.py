"""Gradient alpha unfilter time vs image height (one 4096-wide plane): the
intercept is one band's walk (w + 63 steps), the slope the lag each further
band adds.  WG_ALPHA_GBANDS=1 times the LDS-staged walk instead."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from webp_amd import alpha as A  # noqa: E402

W = int(os.environ.get("W", "4096"))
for h in [int(v) for v in os.environ.get("HS", "65,129,257,513,1025,2049,4096").split(",")]:
    r = torch.randint(0, 256, (1, h, W), dtype=torch.uint8, device="cuda")
    work = r.clone()
    ts = []
    for _ in range(7):
        work.copy_(r)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        A.alpha_unfilter(3, work)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    bands = (h - 1 + 63) // 64
    t = float(np.median(ts))
    print(f"h={h:5d} bands={bands:3d}: {t:.4f} ms  ({t / (W + 63 + (bands - 1) * 64) * 1e6:.1f} ns per ideal step)",
          flush=True)
