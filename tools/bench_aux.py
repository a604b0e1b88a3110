"""SURVEY.md 8(f)#4 stages on one GPU: the ALPH filters / unfilters / filter
estimate, premultiply and the row rescaler, on a batch of 4096x4096 alpha
planes (N planes).  Per stage: median device time with HIP events on the
current stream (the stream every wg_* call here launches on) and the HBM
roofline fraction from the algorithmic bytes (read once + written once).
Prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from tools import synth  # noqa: E402
from webp_amd import alpha as A  # noqa: E402
from webp_amd.rescale import Rescaler  # noqa: E402

S = int(os.environ.get("S", "4096"))
N = int(os.environ.get("N", "4"))
REPS = int(os.environ.get("REPS", "10"))
PEAK = 8000.0


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


def stage(out, name, fn, bytes_):
    ms = timed(fn)
    out[name] = {"ms": round(ms, 4), "GB/s": round(bytes_ / ms / 1e6, 1), "frac": round(bytes_ / ms / 1e6 / PEAK, 4)}


def main():
    rgba = synth.blobs_rgba(S, S, seed=5, alpha=True)
    planes = torch.from_numpy(np.ascontiguousarray(rgba[..., 3])).cuda().unsqueeze(0).repeat(N, 1, 1).contiguous()
    px = N * S * S
    out = {}
    filt = torch.empty_like(planes)
    for f, name in ((1, "horizontal"), (2, "vertical"), (3, "gradient")):
        stage(out, f"filter_{name}", lambda f=f: A.alpha_filter(f, planes, out=filt), 2 * px)
        A.alpha_filter(f, planes, out=filt)
        work = filt.clone()
        # unfilter in place: restore the filtered copy first (the copy is timed apart and subtracted)
        t_copy = timed(lambda: work.copy_(filt))
        ms = timed(lambda: (work.copy_(filt), A.alpha_unfilter(f, work))) - t_copy
        out[f"unfilter_{name}"] = {"ms": round(ms, 4), "GB/s": round(2 * px / ms / 1e6, 1),
                                   "frac": round(2 * px / ms / 1e6 / PEAK, 4)}
    stage(out, "estimate_filter+colors", lambda: A.estimate_best_filter_async(planes), px)
    img = torch.from_numpy(rgba).cuda().view(torch.uint8).reshape(1, -1).repeat(N, 1).contiguous()
    stage(out, "apply_alpha_multiply", lambda: A.ApplyAlphaMultiply(img, False, S, S, 4 * S, False), 8 * px)
    for (dw, dh) in ((S // 2, S // 2), (1920, 1080), (S + S // 2, S + S // 2)):
        r = Rescaler(S, S, dw, dh)
        dst = torch.zeros((N, dh, dw), dtype=torch.uint8, device="cuda")
        stage(out, f"rescale_{S}to{dw}x{dh}", lambda r=r, dst=dst: r.rescale(planes, out=dst), px + N * dw * r.rows)
    print(json.dumps({"config": f"{N} x {S}x{S} alpha planes (blobs, alpha=(x*y)%256 mix), 1 GPU", "stages": out}))


if __name__ == "__main__":
    main()
