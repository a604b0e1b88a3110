"""C5 stages on one GPU (BASELINE.json configs[4]: 4096x4096 RGBA lossless
predictor + SharpYUV + SSIM; the 8-GPU run shards images): per-stage device
time with HIP events on the current stream and the HBM roofline fraction of
each kernel from its algorithmic bytes.  Prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from tools import synth  # noqa: E402
from webp_amd import frames, lossless as L  # noqa: E402

N = int(os.environ.get("N", "4096"))
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


def main():
    rgba = synth.blobs_rgba(N, N, seed=5, alpha=True).astype(np.uint32)
    argb = (rgba[..., 3] << 24) | (rgba[..., 0] << 16) | (rgba[..., 1] << 8) | rgba[..., 2]
    t = L.to_argb_tensor(argb[None])
    px = N * N
    out = {}
    ms = timed(lambda: L.SubtractGreen(t))
    out["subtract_green"] = {"ms": ms, "GB/s": 8 * px / ms / 1e6}
    modes, res = L.ResidualImage(t, 5, 75)
    ms = timed(lambda: L.ResidualImage(t, 5, 75, out=(modes, res)))
    out["residual_image"] = {"ms": ms, "MPix/s": px / ms / 1e3, "GB/s": 8 * px / ms / 1e6}
    inv = torch.empty_like(res)
    ms = timed(lambda: L.predictor_inverse(modes, 5, res, out=inv))
    out["inverse_predictor"] = {"ms": ms, "MPix/s": px / ms / 1e3, "GB/s": 8 * px / ms / 1e6}
    # cross-colour transform (in place; repeated on its own output) and its inverse
    cc = t.clone()
    data = L.ColorSpaceTransform(cc, 5)
    ms = timed(lambda: L.ColorSpaceTransform(cc, 5, data=data))
    out["cross_color"] = {"ms": ms, "MPix/s": px / ms / 1e3, "GB/s": 8 * px / ms / 1e6}
    cinv = torch.empty_like(cc)
    ms = timed(lambda: L.color_space_inverse(data, 5, cc, out=cinv))
    out["cross_color_inverse"] = {"ms": ms, "MPix/s": px / ms / 1e3, "GB/s": 8 * px / ms / 1e6}
    pal = L.to_argb_tensor(np.arange(16, dtype=np.uint32) * 0x01010101)
    packed = torch.randint(0, 2 ** 31 - 1, (1, N, N // 2), dtype=torch.int32, device="cuda")
    ci = torch.empty_like(t)
    ms = timed(lambda: L.color_index_inverse(pal, 1, N, packed, out=ci))
    out["color_index_inverse"] = {"ms": ms, "MPix/s": px / ms / 1e3, "GB/s": 6 * px / ms / 1e6}
    rgb = torch.from_numpy(np.ascontiguousarray(rgba[..., :3].astype(np.uint8))).cuda().unsqueeze(0)
    Ys, Us, Vs = frames.sharpyuv_convert(rgb)
    work = torch.empty(frames.lib.wg_sharpyuv_work_bytes(N, N, 1), dtype=torch.uint8, device="cuda")
    ms = timed(lambda: frames.sharpyuv_convert(rgb, out=(Ys, Us, Vs), work=work))
    out["sharpyuv"] = {"ms": ms, "MPix/s": px / ms / 1e3, "GB/s": 4.5 * px / ms / 1e6}
    y = torch.from_numpy(rgba[..., 1].astype(np.uint8)).cuda().unsqueeze(0)
    y2 = torch.clamp(y.int() + torch.randint(-8, 9, y.shape, device="cuda", dtype=torch.int32), 0, 255).to(torch.uint8)
    ms = timed(lambda: frames.plane_ssim(y, y2))
    out["plane_ssim"] = {"ms": ms, "MPix/s": px / ms / 1e3, "GB/s": 2 * px / ms / 1e6}
    for v in out.values():
        if "GB/s" in v:
            v["frac"] = v["GB/s"] / PEAK
        for k in list(v):
            v[k] = round(v[k], 4)
    print(json.dumps({"config": f"C5 {N}x{N} RGBA, bits 5, q75, 1 GPU", "stages": out}))


if __name__ == "__main__":
    main()
