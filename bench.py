"""Benchmark: MPixels/s of the VP8 encode+decode DSP path on 1920x1080 frames.

One step = one pass of the hot path over this rank's batch of synthetic
1920x1080 frames, all inputs resident in HBM before timing starts:
  encode side  import RGBA->YUV420 (k_import)  ->  analysis alphas (k_analysis)
               ->  macroblock RD loop, Phase A of encodeFrameParallel (k_encode_rows)
  decode side  reconstruct + loop filter of parsed macroblocks (k_decode_rows)
               ->  fancy upsample to NRGBA (k_upsample)
The decode side consumes seeded synthetic parsed-macroblock data (tools/synth.py,
SURVEY.md 8(d) C3 recipe).  Segment ids for the RD loop come from the analysis
alphas (quartiles, standing in for the CPU-side AssignSegments k-means) with
q75-range quantisers per segment.

Multi-GPU: one process per GPU (torch.distributed.run), frames sharded across
ranks with no data-path collective ("weak" scaling); value = all pixels / max
rank time.  Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

W, H = 1920, 1080
MBW, MBH = (W + 15) >> 4, (H + 15) >> 4
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec

# Algorithmic (compulsory) HBM bytes per source pixel, SURVEY.md 8(d)
BYTES_PER_PX = {
    "import": 4.0 + 1.5,              # RGBA in, Y + U/V out
    "analysis": 1.5,                  # Y/U/V planes in (alphas out ~0)
    "encode": 1.5 + 864 / 256.0 + 1.5,  # YUV in, MBEncInfo (800 B levels + info) + reconstruction out
    "decode": (384 * 2 + 32 + 384) / 256.0,  # coeffs + mb info in, YUV out (recon and filter fused)
    "upsample": 1.5 + 4.0,            # YUV in, NRGBA out
}


KERNELS = {"import": "k_import", "analysis": "k_analysis", "encode": "k_encode_rows", "decode": "k_decode_rows",
           "upsample": "k_upsample"}
SEG_Q = (22, 25, 28, 31)  # quantiser index per segment: q75 (index 26) +- SNS-style offsets
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_traffic.json")


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC pass
    (tools/profile.sh -> tools/pmc_summary.py --json; FETCH_SIZE doubled per
    MI355X_MICROARCH.md's gfx950 correction, + WRITE_SIZE), or None."""
    try:
        rec = json.load(open(PMC_FILE))[kernel]
        return int(rec["hbm_bytes_per_launch"]), os.path.relpath(PMC_FILE, ROOT)
    except (OSError, KeyError, ValueError):
        return None, None


def default_proba():
    """CoeffsProba0 (internal/lossy/proba.go:45): the token probabilities
    Phase A prices with after ResetProba; read from the generated table."""
    import re
    txt = open(os.path.join(ROOT, "webp_amd", "csrc", "vp8_tables.h")).read()
    body = txt[txt.index("vp8_coeffs_proba0["):]
    body = body[body.index("{") + 1:body.index("};")]
    return np.array([int(x) for x in re.findall(r"\d+", body)], np.uint8)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--batch", type=int, default=64, help="frames per GPU per step (C4: 512 frames / 8 GPUs)")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="budget for the CPU baseline sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    return p.parse_args()


def make_inputs(batch, rank, device):
    from tools import synth
    from webp_amd import frames
    gens = [lambda s: synth.gradient_rgba(W, H), lambda s: synth.noise_rgba(W, H, seed=s),
            lambda s: synth.blobs_rgba(W, H, seed=s)]
    base = [gens[k](rank * 3 + k) for k in range(3)]
    rgba = torch.empty((batch, H, W, 4), dtype=torch.uint8, device=device)
    for i in range(batch):
        rgba[i].copy_(torch.from_numpy(base[(i + rank) % 3]))
    mb, co = synth.random_macroblocks(MBW * MBH * 4, seed=100 + rank, levels=(20, 32))
    per = MBW * MBH
    mb_t = frames.mb_info_tensor(mb, device).view(4, per, 32)
    co_t = torch.from_numpy(co).to(device).view(4, per, 384)
    mb_all = torch.empty((batch, per, 32), dtype=torch.uint8, device=device)
    co_all = torch.empty((batch, per, 384), dtype=torch.int16, device=device)
    for i in range(batch):
        mb_all[i].copy_(mb_t[i % 4])
        co_all[i].copy_(co_t[i % 4])
    return rgba, mb_all.view(-1, 32), co_all.view(-1, 384), (mb, co)


class Pipeline:
    """Pre-allocated buffers + the 4 stages; optional per-stage HIP events."""

    def __init__(self, rgba, mb, co, batch, device):
        from webp_amd import _lib, frames
        self.frames = frames
        self.rgba, self.mb, self.co, self.batch = rgba, mb, co, batch
        self.Y = torch.empty((batch, 16 * MBH, 16 * MBW), dtype=torch.uint8, device=device)
        self.U = torch.empty((batch, 8 * MBH, 8 * MBW), dtype=torch.uint8, device=device)
        self.V = torch.empty_like(self.U)
        self.alphas = torch.empty((batch, MBW * MBH), dtype=torch.int32, device=device)
        self.uv_sum = torch.empty((batch,), dtype=torch.int32, device=device)
        self.segs = torch.from_numpy(np.stack([frames.setup_segment(q) for q in SEG_Q]).view(np.uint8).copy()).to(device)
        self.proba = torch.from_numpy(default_proba()).to(device)
        self.seg_ids = torch.empty((batch, MBW * MBH), dtype=torch.uint8, device=device)
        self.enc_out = torch.empty((batch * MBW * MBH, frames.MB_ENC_DTYPE.itemsize), dtype=torch.uint8, device=device)
        self.rY, self.rU, self.rV = torch.empty_like(self.Y), torch.empty_like(self.U), torch.empty_like(self.U)
        self.enc_work = torch.empty(_lib.lib.wg_encode_work_bytes(MBW, MBH, batch), dtype=torch.uint8, device=device)
        self.dY = torch.empty_like(self.Y)
        self.dU = torch.empty_like(self.U)
        self.dV = torch.empty_like(self.U)
        self.work = torch.empty(_lib.lib.wg_decode_work_bytes(MBW, MBH, batch), dtype=torch.uint8, device=device)
        self.out = torch.empty((batch, H, W, 4), dtype=torch.uint8, device=device)
        self.stage_ms = {k: 0.0 for k in BYTES_PER_PX}
        self.events = []

    def step(self, record=False):
        f = self.frames
        ev = []
        if record:
            ev.append(torch.cuda.Event(enable_timing=True))
            ev[-1].record()
        f.import_rgba(self.rgba, has_alpha=False, out=(self.Y, self.U, self.V))
        if record:
            ev.append(torch.cuda.Event(enable_timing=True)); ev[-1].record()
        f.analysis_alphas(self.Y, self.U, self.V, W, H, out=(self.alphas, self.uv_sum, None, None))
        if record:
            ev.append(torch.cuda.Event(enable_timing=True)); ev[-1].record()
        torch.clamp(self.alphas >> 6, max=3, out=self.alphas)
        self.seg_ids.copy_(self.alphas)
        f.encode_mbs(self.Y, self.U, self.V, W, H, self.seg_ids, self.segs, self.proba, out=self.enc_out,
                     recon=(self.rY, self.rU, self.rV), work=self.enc_work)
        if record:
            ev.append(torch.cuda.Event(enable_timing=True)); ev[-1].record()
        f.decode_frames(self.mb, self.co, 2, MBW, MBH, self.batch, out=(self.dY, self.dU, self.dV), work=self.work)
        if record:
            ev.append(torch.cuda.Event(enable_timing=True)); ev[-1].record()
        f.build_nrgba(self.dY, self.dU, self.dV, W, H, out=self.out)
        if record:
            ev.append(torch.cuda.Event(enable_timing=True)); ev[-1].record()
            self.events.append(ev)

    def collect(self):
        torch.cuda.synchronize()
        names = list(BYTES_PER_PX)
        for ev in self.events:
            for k, name in enumerate(names):
                self.stage_ms[name] += ev[k].elapsed_time(ev[k + 1])
        n = max(1, len(self.events))
        return {k: v / n for k, v in self.stage_ms.items()}


def cpu_baseline(seconds, mb_co):
    """C restatement of the reference Go CPU path (oracle/), 1 thread, on a
    bounded sample of the same per-frame workload."""
    import oracle as O
    from tools import synth
    img = synth.blobs_rgba(W, H, seed=1)
    mb, co = mb_co
    per = MBW * MBH
    mb1, co1 = mb[:per], co[:per]
    frames_done, t0 = 0, time.perf_counter()
    segs = np.stack([O.setup_segment(q) for q in SEG_Q])
    proba = default_proba()
    while True:
        Y, U, V = O.import_rgba(img, has_alpha=False)
        alphas, _, _, _ = O.compute_alphas(Y, U, V, W, H)
        seg_ids = np.minimum(np.asarray(alphas) >> 6, 3).astype(np.uint8)
        O.encode_frame_rd(Y, U, V, W, H, seg_ids, segs, proba, method=4, quality=75)
        dy, du, dv = O.decode_frame(mb1, co1, 2, MBW, MBH)
        O.build_nrgba(dy, du, dv, W, H)
        frames_done += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": round(frames_done * W * H / el / 1e6, 2), "unit": "MPixels/s", "cores": 1, "kind": "port",
            "sample": f"{frames_done} x 1920x1080 frames (import+analysis+MB RD+decode+upsample), C restatement of the "
                      "reference Go CPU path, single thread"}


def timed_region(step, steps, warmup, world, sync, device):
    """W untimed steps, then exactly K timed steps bracketed by a barrier and
    a device sync on both sides; returns the MAX over ranks of the elapsed
    seconds (all_reduce MAX on the process group: RCCL on the GPU box, gloo
    in tests/test_multi_rank.py)."""
    for _ in range(warmup):
        step()
    sync()
    if world > 1:
        torch.distributed.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step(record=True)
    sync()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def aggregate_mpix_s(world, batch, steps, elapsed):
    """Whole-job throughput: every rank's pixels over the slowest rank's time
    (weak scaling: each rank owns `batch` frames)."""
    return world * batch * W * H * steps / elapsed / 1e6


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    import webp_amd
    webp_amd.device_check()

    rgba, mb, co, mb_co = make_inputs(args.batch, rank, device)
    pipe = Pipeline(rgba, mb, co, args.batch, device)
    elapsed = timed_region(pipe.step, args.steps, args.warmup, world, torch.cuda.synchronize, device)
    stage = pipe.collect()

    if rank == 0:
        value = aggregate_mpix_s(world, args.batch, args.steps, elapsed)
        dominant = max(stage, key=stage.get)
        px_rank_step = args.batch * W * H
        kernel = KERNELS[dominant]
        achieved = BYTES_PER_PX[dominant] * px_rank_step / (stage[dominant] / 1e3) / 1e9
        traffic, traffic_src = pmc_traffic(kernel)
        rec = {
            "metric": "MPixels/s encode+decode DSP path (1920x1080 q75)",
            "value": round(value, 1),
            "unit": "MPixels/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (gradient/noise/blobs RGBA; seeded parsed-macroblock data for the decode side)",
            "config": {"workload": f"{args.batch} x 1920x1080 frames per GPU per step (C2 frame, C4 per-GPU share): "
                                   "import+analysis+MB RD loop (encode DSP, method 4) + reconstruct+loopfilter+upsample (decode DSP)",
                       "frames_per_gpu": args.batch, "width": W, "height": H, "parallelism": f"frames sharded x{world}"},
            "stage_ms": {k: round(v, 3) for k, v in stage.items()},
            "roofline": {"kernel": kernel, "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "traffic_source": traffic_src, "bytes_per_px": BYTES_PER_PX[dominant],
                         "algorithmic_bytes_per_launch": int(BYTES_PER_PX[dominant] * px_rank_step),
                         "avg_launch_ms": round(stage[dominant], 4), "launches_per_step": 1},
            "stage_roofline": {k: {"kernel": KERNELS[k], "GB/s": round(BYTES_PER_PX[k] * px_rank_step / (v / 1e3) / 1e9, 1),
                                   "frac": round(BYTES_PER_PX[k] * px_rank_step / (v / 1e3) / 1e9 / HBM_PEAK_GBS, 4)}
                               for k, v in stage.items()},
        }
        if not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline(args.cpu_seconds, mb_co)
        print(json.dumps(rec), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
