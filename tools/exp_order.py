"""Diagnostic: k_encode_rows launch time for 64 mixed 1080p frames with the
(row, frame) dequeue order and with wg_encode_row_order's schedule (textured
frames' rows ahead), outputs compared; and the per-content mean alpha the
schedule ranks frames by.  (The head-start sweep quoted in DESIGN.md was
measured with a host-built order through a debug hook since removed.)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402
from tools import synth  # noqa: E402
from webp_amd import frames  # noqa: E402

W, H, MBW, MBH, B = 1920, 1080, 120, 68, 64
gens = [lambda: synth.gradient_rgba(W, H), lambda: synth.noise_rgba(W, H, seed=3), lambda: synth.blobs_rgba(W, H, seed=3)]
planes = [O.import_rgba(g(), has_alpha=False) for g in gens]
Y = torch.from_numpy(np.stack([planes[i % 3][0] for i in range(B)])).cuda()
U = torch.from_numpy(np.stack([planes[i % 3][1] for i in range(B)])).cuda()
V = torch.from_numpy(np.stack([planes[i % 3][2] for i in range(B)])).cuda()
alphas, uv_sum = frames.analysis_alphas(Y, U, V, W, H)
seg_ids, segs, info = frames.segment_analysis(frames.encoder_config(), alphas, uv_sum, MBW, MBH)
print("mean alpha by content (gradient, noise, blobs):", alphas.float().mean(dim=1).cpu().numpy()[:3])
proba = frames.default_proba()
ref, _ = frames.encode_mbs(Y, U, V, W, H, seg_ids, segs, proba, check=True)


def timed(work):
    out, rec = frames.encode_mbs(Y, U, V, W, H, seg_ids, segs, proba, work=work, check=True)
    assert torch.equal(out, ref), "outputs differ"
    ts = []
    for _ in range(7):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        frames.encode_mbs(Y, U, V, W, H, seg_ids, segs, proba, out=out, recon=rec, work=work)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    frames.encode_status(work, MBW, B)
    return float(np.median(ts))


plain = torch.zeros(frames.lib.wg_encode_work_bytes(MBW, MBH, B), dtype=torch.uint8, device="cuda")
print(f"(row, frame) order: {timed(plain):.3f} ms", flush=True)
print(f"wg_encode_row_order: {timed(frames.encode_row_order(alphas, MBW, MBH)):.3f} ms", flush=True)
