"""Encoder (k_encode_rows) time vs batch size: where the row wavefront's
critical path (mbw + 2 (mbh - 1) macroblock latencies per image) stops
bounding the launch and wave slots start to.  The bench's frames
(bench.frame_rgba: G / N / P in turn, a distinct seed per frame) and the
reference's q75 segment setup, like bench.py.
Prints one line per batch size.  Diagnostic only (not the driver bench)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402
import bench  # noqa: E402
from webp_amd import frames  # noqa: E402

W, H = 1920, 1080
MBW, MBH = 120, 68
BATCHES = [int(b) for b in os.environ.get("BATCHES", "1,3,8,16,32,64").split(",")]
planes = [O.import_rgba(bench.frame_rgba(g), has_alpha=False) for g in range(max(BATCHES))]
for B in BATCHES:
    Y = torch.from_numpy(np.stack([planes[i][0] for i in range(B)])).cuda()
    U = torch.from_numpy(np.stack([planes[i][1] for i in range(B)])).cuda()
    V = torch.from_numpy(np.stack([planes[i][2] for i in range(B)])).cuda()
    alphas, uv_sum = frames.analysis_alphas(Y, U, V, W, H)
    seg_ids, segs, _ = frames.segment_analysis(frames.encoder_config(), alphas, uv_sum, MBW, MBH)
    proba = O.default_proba()
    work = frames.encode_row_order(alphas, MBW, MBH) if os.environ.get("ROW_ORDER", "1") == "1" else None
    out, rec = frames.encode_mbs(Y, U, V, W, H, seg_ids, segs, proba, work=work, check=True)
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        frames.encode_mbs(Y, U, V, W, H, seg_ids, segs, proba, out=out, recon=rec, work=work)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    t = float(np.median(ts))
    print(f"B={B:3d}: {t:7.3f} ms  {t / B:6.3f} ms/frame  {B * W * H / t / 1e3:8.1f} MPix/s  "
          f"per-MB-latency bound {t / (MBW + 2 * (MBH - 1)) * 1e3:6.1f} us", flush=True)
