"""Benchmark: MPixels/s of the VP8 encode+decode DSP path on 1920x1080 frames.

One step = one pass of the hot path over this rank's batch of synthetic
1920x1080 frames, all inputs resident in HBM before timing starts:
  encode side  import RGBA->YUV420 (k_import)  ->  analysis alphas (k_analysis)
               ->  macroblock RD loop, Phase A of encodeFrameParallel (k_encode_rows)
  decode side  reconstruct + loop filter of parsed macroblocks (k_decode_bands)
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


KERNELS = {"import": "k_import", "analysis": "k_analysis", "encode": "k_encode_rows", "decode": "k_decode_bands",
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


VALU_FILE = os.path.join(ROOT, "profiles", "pmc_valu.json")
# VALU issue peak: 256 CUs x 4 SIMDs, one 64-lane VALU instruction per SIMD
# every 2 cycles (MI355X_MICROARCH.md), at the 2.4 GHz peak clock.
VALU_PEAK_WINST_S = 256 * 4 * 0.5 * 2.4e9


def pmc_valu(kernel, launch_ms, step_ms):
    """VALU issue rate of `kernel` from the committed SQ pass (tools/profile.sh:
    SQ_INSTS_VALU per launch) over this run's measured launch time, against
    the SIMD issue peak; None if the pass is absent."""
    try:
        rec = json.load(open(VALU_FILE))[kernel]
    except (OSError, KeyError, ValueError):
        return None
    insts = rec["SQ_INSTS_VALU"]
    rate = insts / (launch_ms / 1e3)
    out = {"kernel": kernel, "insts_valu_per_launch": int(insts), "achieved": round(rate / 1e12, 4),
           "peak": round(VALU_PEAK_WINST_S / 1e12, 4), "unit": "T wave-instr/s",
           "frac": round(rate / VALU_PEAK_WINST_S, 4), "source": os.path.relpath(VALU_FILE, ROOT),
           "frac_per_step": round(insts / (step_ms / 1e3) / VALU_PEAK_WINST_S, 4)}
    return out


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
    p.add_argument("--slots", type=int, default=3, help="batches in flight (one HIP stream each)")
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


class Slot:
    """One in-flight batch: its own HIP stream and every output / work buffer."""

    def __init__(self, batch, device, frames, lib):
        self.stream = torch.cuda.Stream(device)
        self.Y = torch.empty((batch, 16 * MBH, 16 * MBW), dtype=torch.uint8, device=device)
        self.U = torch.empty((batch, 8 * MBH, 8 * MBW), dtype=torch.uint8, device=device)
        self.V = torch.empty_like(self.U)
        self.alphas = torch.empty((batch, MBW * MBH), dtype=torch.int32, device=device)
        self.uv_sum = torch.empty((batch,), dtype=torch.int32, device=device)
        self.seg_ids = torch.empty((batch, MBW * MBH), dtype=torch.uint8, device=device)
        self.enc_out = torch.empty((batch * MBW * MBH, frames.MB_ENC_DTYPE.itemsize), dtype=torch.uint8, device=device)
        self.rY, self.rU, self.rV = torch.empty_like(self.Y), torch.empty_like(self.U), torch.empty_like(self.U)
        self.enc_work = torch.empty(lib.wg_encode_work_bytes(MBW, MBH, batch), dtype=torch.uint8, device=device)
        self.dY = torch.empty_like(self.Y)
        self.dU = torch.empty_like(self.U)
        self.dV = torch.empty_like(self.U)
        self.work = torch.empty(lib.wg_decode_work_bytes(MBW, MBH, batch), dtype=torch.uint8, device=device)
        self.out = torch.empty((batch, H, W, 4), dtype=torch.uint8, device=device)


class Pipeline:
    """The 5 stages over pre-allocated buffers, optional per-stage HIP events.

    With `slots` > 1, consecutive steps alternate between slots, each with its
    own HIP stream and buffers, so step k+1's kernels fill the CUs that step
    k's encoder RD wavefront leaves idle in its ramp-down.  Every
    step still runs every stage over its whole batch; the timed region ends
    with a device-wide synchronisation."""

    def __init__(self, rgba, mb, co, batch, device, slots=1):
        from webp_amd import _lib, frames
        self.frames = frames
        self.rgba, self.mb, self.co, self.batch = rgba, mb, co, batch
        self.segs = torch.from_numpy(np.stack([frames.setup_segment(q) for q in SEG_Q]).view(np.uint8).copy()).to(device)
        self.proba = torch.from_numpy(default_proba()).to(device)
        self.slots = [Slot(batch, device, frames, _lib.lib) for _ in range(slots)]
        self.k = 0
        self.stage_ms = {k: 0.0 for k in BYTES_PER_PX}
        self.events = []
        torch.cuda.synchronize(device)  # inputs made on the default stream are ready for every slot stream

    def step(self, record=False):
        sl = self.slots[self.k % len(self.slots)]
        self.k += 1
        with torch.cuda.stream(sl.stream):
            self._stages(sl, record)

    def _stages(self, sl, record):
        f = self.frames
        ev = []

        def mark():
            if record:
                ev.append(torch.cuda.Event(enable_timing=True))
                ev[-1].record()  # on the slot's stream (the current stream here)

        mark()
        f.import_rgba(self.rgba, has_alpha=False, out=(sl.Y, sl.U, sl.V))
        mark()
        f.analysis_alphas(sl.Y, sl.U, sl.V, W, H, out=(sl.alphas, sl.uv_sum, None, None))
        mark()
        torch.clamp(sl.alphas >> 6, max=3, out=sl.alphas)
        sl.seg_ids.copy_(sl.alphas)
        f.encode_mbs(sl.Y, sl.U, sl.V, W, H, sl.seg_ids, self.segs, self.proba, out=sl.enc_out,
                     recon=(sl.rY, sl.rU, sl.rV), work=sl.enc_work)
        mark()
        f.decode_frames(self.mb, self.co, 2, MBW, MBH, self.batch, out=(sl.dY, sl.dU, sl.dV), work=sl.work)
        mark()
        f.build_nrgba(sl.dY, sl.dU, sl.dV, W, H, out=sl.out)
        mark()
        if record:
            self.events.append(ev)

    def collect(self):
        torch.cuda.synchronize()
        names = list(BYTES_PER_PX)
        for ev in self.events:
            for k, name in enumerate(names):
                self.stage_ms[name] += ev[k].elapsed_time(ev[k + 1])
        n = max(1, len(self.events))
        return {k: v / n for k, v in self.stage_ms.items()}


def cpu_threads():
    """Host cores this run may use: the box's CPU share (OMP_NUM_THREADS is set
    to it on the GPU box) capped by the affinity mask."""
    n = len(os.sched_getaffinity(0))
    env = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(env))) if env and env.isdigit() else max(1, min(n, 16))


def cpu_baseline(seconds, mb_co):
    """C restatement of the reference Go CPU path (oracle/) on a bounded sample
    of the same per-frame workload: first one thread, then one frame per
    thread on every host core this run may use (ctypes releases the GIL for
    the C calls).  The reference parallelises inside a frame (row workers,
    encode_parallel.go:176); across independent frames is the same work with
    no synchronisation, so the threaded figure is an upper bound of what its
    CPU path reaches on these cores."""
    import concurrent.futures as cf

    import oracle as O
    from tools import synth
    img = synth.blobs_rgba(W, H, seed=1)
    mb, co = mb_co
    per = MBW * MBH
    mb1, co1 = mb[:per], co[:per]
    segs = np.stack([O.setup_segment(q) for q in SEG_Q])
    proba = default_proba()

    def one_frame():
        Y, U, V = O.import_rgba(img, has_alpha=False)
        alphas, _, _, _ = O.compute_alphas(Y, U, V, W, H)
        seg_ids = np.minimum(np.asarray(alphas) >> 6, 3).astype(np.uint8)
        O.encode_frame_rd(Y, U, V, W, H, seg_ids, segs, proba, method=4, quality=75)
        dy, du, dv = O.decode_frame(mb1, co1, 2, MBW, MBH)
        O.build_nrgba(dy, du, dv, W, H)

    def run(budget):
        done, t0 = 0, time.perf_counter()
        while True:
            one_frame()
            done += 1
            el = time.perf_counter() - t0
            if el >= budget:
                return done, el

    f1, e1 = run(seconds / 3)  # also initialises the oracle's lazily built tables before threading
    single = f1 * W * H / e1 / 1e6
    threads = cpu_threads()
    if threads > 1:
        t0 = time.perf_counter()
        with cf.ThreadPoolExecutor(threads) as ex:
            res = list(ex.map(lambda _: run(seconds * 2 / 3), range(threads)))
        el = time.perf_counter() - t0
        fn = sum(r[0] for r in res)
        value = fn * W * H / el / 1e6
    else:
        fn, value = f1, single
    return {"value": round(value, 2), "unit": "MPixels/s", "cores": threads, "kind": "port",
            "single_thread_value": round(single, 2),
            "sample": f"{fn} x 1920x1080 frames on {threads} threads (one frame per thread; {f1} frames on 1 thread "
                      "before it) of import+analysis+MB RD+decode+upsample, C restatement of the reference Go CPU path"}


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
    pipe = Pipeline(rgba, mb, co, args.batch, device, slots=args.slots)
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
                       "frames_per_gpu": args.batch, "width": W, "height": H, "parallelism": f"frames sharded x{world}", "batches_in_flight": args.slots},
            "stage_ms": {k: round(v, 3) for k, v in stage.items()},
            "roofline": {"kernel": kernel, "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "traffic_source": traffic_src, "bytes_per_px": BYTES_PER_PX[dominant],
                         "algorithmic_bytes_per_launch": int(BYTES_PER_PX[dominant] * px_rank_step),
                         "avg_launch_ms": round(stage[dominant], 4), "launches_per_step": 1,
                         # with batches in flight the launches overlap: bytes per step over the step time
                         "achieved_per_step": round(BYTES_PER_PX[dominant] * px_rank_step / (elapsed / args.steps) / 1e9, 1),
                         "launches_in_flight": args.slots},
            "stage_roofline": {k: {"kernel": KERNELS[k], "GB/s": round(BYTES_PER_PX[k] * px_rank_step / (v / 1e3) / 1e9, 1),
                                   "frac": round(BYTES_PER_PX[k] * px_rank_step / (v / 1e3) / 1e9 / HBM_PEAK_GBS, 4)}
                               for k, v in stage.items()},
        }
        valu = pmc_valu(kernel, stage[dominant], elapsed / args.steps * 1e3)
        if valu is not None:
            rec["valu"] = valu
        if not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline(args.cpu_seconds, mb_co)
        print(json.dumps(rec), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
