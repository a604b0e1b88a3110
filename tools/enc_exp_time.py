"""Encoder A/B timing (tools/gpu_enc_exp.sh): one-frame RD launches (noise,
gradient: the C2 critical path on a wave pair per row) and the bench's
64-frame mixed launch (one wave a row), median of 7 each."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402
from tools import synth  # noqa: E402
from webp_amd import frames  # noqa: E402

W, H, MBW, MBH = 1920, 1080, 120, 68
gens = {"gradient": lambda: synth.gradient_rgba(W, H), "noise": lambda: synth.noise_rgba(W, H, seed=3),
        "blobs": lambda: synth.blobs_rgba(W, H, seed=3)}
planes = {k: O.import_rgba(g(), has_alpha=False) for k, g in gens.items()}
proba = O.default_proba()


def run(kinds):
    B = len(kinds)
    Y = torch.from_numpy(np.stack([planes[k][0] for k in kinds])).cuda()
    U = torch.from_numpy(np.stack([planes[k][1] for k in kinds])).cuda()
    V = torch.from_numpy(np.stack([planes[k][2] for k in kinds])).cuda()
    alphas, uv_sum = frames.analysis_alphas(Y, U, V, W, H)
    seg_ids, segs, _ = frames.segment_analysis(frames.encoder_config(), alphas, uv_sum, MBW, MBH)
    work = frames.encode_row_order(alphas, MBW, MBH)
    out, rec = frames.encode_mbs(Y, U, V, W, H, seg_ids, segs, proba, work=work, check=True)
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


res = {"noise1": run(["noise"]), "grad1": run(["gradient"]), "blobs1": run(["blobs"]),
       "mix64": run([("gradient", "noise", "blobs")[i % 3] for i in range(64)])}
print(" ".join(f"{k}={v:.3f}ms" for k, v in res.items()), flush=True)
