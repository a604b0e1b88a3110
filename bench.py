"""Benchmark: MPixels/s of the VP8 encode+decode DSP path on 1920x1080 frames.

One step = one pass of the hot path over this rank's batch of 1920x1080
frames, all inputs resident in HBM before timing starts:
  encode side  import RGBA->YUV420 (k_import) -> computeAlphas (k_analysis)
               -> segment analysis (k_segments: assignSegments k-means,
                  setSegmentParams, setupSegment at the reference's q75 defaults)
               -> macroblock RD loop, Phase A of encodeFrameParallel (k_encode_rows)
  decode side  reconstruct + loop filter (k_decode_bands at the bench batch;
               wg_decode_kernel names the one launched) of libwebp q75
               bitstreams of the same three contents, parsed once on the host by
               wg_vp8_parse (tests/golden/q75_1080p.npz), -> fancy upsample to
               NRGBA (k_upsample)
Contents: G gradient, N noise, P photo (the reference's
testdata/test_color.png tiled); frame i of rank r is content i % 3 with seed
r * batch + i, so every frame of the C4 job is distinct on the encode side
(the decode side replays the three contents' libwebp streams).
The encode configuration is webp.Encode's DefaultOptions (quality 75, method
4, SNS 50, filter strength 60, 4 segments; internal/lossy/encode.go:66-86).

After the timed region the in-kernel dependency waits are checked
(wg_encode_status / wg_decode_status: the last launch of each slot plus the
library's device-wide count of timed-out waits, which covers every timed
launch).  Then, untimed for `value`:
  - `runs`: the median of --runs repeats of a short timed region, for the
    whole path and for the encode side and the decode side alone;
  - an isolated one-batch pass for each kernel's launch time (the roofline);
  - one-frame encodes (C2), whose RD launch is the macroblock wavefront's
    critical path: the per-MB latency bench reports as the encoder's limiter;
  - the measured copy-kernel HBM ceiling (tools/libprobe.so);
  - `c3`: one real 4096x4096 q75 decode (tests/golden/c3_4096_q75.npz:
    libwebp's encode of test_color.png tiled), reconstruct + filter +
    upsample, and `c5`: SubtractGreen + ResidualImage (bits 5, q75), SharpYUV
    and plane SSIM on a 4096x4096 N + G blend (BASELINE.json configs 2 and 4,
    one GPU), each with ms, MPix/s and its HBM roofline fraction.

Multi-GPU: one process per GPU, frames sharded across ranks with no data-path
collective in the timed region ("weak" scaling); value = all pixels / max rank
time.  `python bench.py --gpus N` with N > 1 starts the N ranks itself
(torch.distributed.run in a child process, before anything touches the GPU);
under an external torch.distributed.run, WORLD_SIZE must equal --gpus.  With
N > 1, each rank then sends its last batch's outputs (wg_mb_enc records,
reconstruction, NRGBA) to rank 0 with grouped RCCL send/recv
(webp_amd/shard.py), timed and reported separately ("gather"), outside `value`.
Rank 0 prints one JSON line.
"""
import argparse
import contextlib
import json
import os
import socket
import subprocess
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
    "segments": 5.0 / 256,            # alphas in (4 B/MB), segment ids out (1 B/MB)
    "encode": 1.5 + 864 / 256.0 + 1.5,  # YUV in, MBEncInfo (800 B levels + info) + reconstruction out
    "decode": (384 * 2 + 32 + 384) / 256.0,  # coeffs + mb info in, YUV out (recon and filter fused)
    "upsample": 1.5 + 4.0,            # YUV in, NRGBA out
}
KERNELS = {"import": "k_import", "analysis": "k_analysis", "segments": "k_segments", "encode": "k_encode_rows",
           "decode": "k_decode_split", "upsample": "k_upsample"}  # decode: set from wg_decode_kernel at report time
CONTENTS = ("grad", "noise", "photo")
BITSTREAMS = os.path.join(ROOT, "tests", "golden", "q75_1080p.npz")
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_traffic.json")
VALU_FILE = os.path.join(ROOT, "profiles", "pmc_valu.json")
# SQ passes over one 64 x 1080p k_encode_rows launch (tools/gpu_enc_pmc.sh): wave
# cycles, instruction mix, waits, LDS array cycles
ENC_SQ_FILE = os.path.join(ROOT, "profiles", "enc_sq.json")
CLOCK_HZ = 2.4e9  # MI355X_MICROARCH.md: shader clock
SIMDS = 256 * 4
# VALU issue peak: 256 CUs x 4 SIMDs, one 64-lane VALU instruction per SIMD
# every 2 cycles (MI355X_MICROARCH.md), at the 2.4 GHz peak clock.
VALU_PEAK_WINST_S = 256 * 4 * 0.5 * 2.4e9
ENC_CFG = dict(quality=75, method=4, sns_strength=50, filter_strength=60, filter_sharpness=0, filter_type=1,
               segments=4, preprocessing=0)


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC pass
    (tools/profile.sh -> tools/pmc_summary.py --json; FETCH_SIZE doubled per
    MI355X_MICROARCH.md's gfx950 correction, + WRITE_SIZE), or None."""
    try:
        rec = json.load(open(PMC_FILE))[kernel]
        return int(rec["hbm_bytes_per_launch"]), os.path.relpath(PMC_FILE, ROOT)
    except (OSError, KeyError, ValueError):
        return None, None


def pmc_valu(kernel, launch_ms, step_ms):
    """VALU issue rate of `kernel` from the committed SQ pass (SQ_INSTS_VALU per
    launch) over its isolated launch time, against the SIMD issue peak; None
    if the pass is absent."""
    try:
        rec = json.load(open(VALU_FILE))[kernel]
    except (OSError, KeyError, ValueError):
        return None
    insts = rec["SQ_INSTS_VALU"]
    rate = insts / (launch_ms / 1e3)
    return {"kernel": kernel, "insts_valu_per_launch": int(insts), "achieved": round(rate / 1e12, 4),
            "peak": round(VALU_PEAK_WINST_S / 1e12, 4), "unit": "T wave-instr/s",
            "frac": round(rate / VALU_PEAK_WINST_S, 4), "source": os.path.relpath(VALU_FILE, ROOT),
            "frac_per_step": round(insts / (step_ms / 1e3) / VALU_PEAK_WINST_S, 4)}


def slot_model(launch_ms, batch, enc_waves_per_simd=2):
    """The encoder launch as wave-slot time: the wave cycles
    one launch spends per macroblock (SQ_WAVE_CYCLES of the committed SQ pass,
    quad-cycles x 4, waits included) x the macroblocks / the resident wave
    slots / the clock, beside the measured launch; plus where a wave's cycles
    go (issuing, waiting on LDS / memory, waiting for issue) and how busy the
    HBM, VALU and LDS are.  None without the pass."""
    try:
        rec = json.load(open(ENC_SQ_FILE))["k_encode_rows"]
    except (OSError, KeyError, ValueError):
        return None
    mbs = batch * MBW * MBH
    wave_cyc = rec["SQ_WAVE_CYCLES"] * 4
    slots = SIMDS * enc_waves_per_simd
    launch_cyc = launch_ms / 1e3 * CLOCK_HZ
    pred_ms = wave_cyc / slots / CLOCK_HZ * 1e3
    return {
        "source": os.path.relpath(ENC_SQ_FILE, ROOT),
        "wave_cycles_per_mb": int(wave_cyc / mbs), "mbs_per_launch": mbs, "resident_wave_slots": slots,
        "predicted_full_slots_ms": round(pred_ms, 3), "measured_launch_ms": round(launch_ms, 3),
        "slot_fill": round(pred_ms / launch_ms, 3),
        "wave_time": {"issuing": round(rec["SQ_ACTIVE_INST_ANY"] / rec["SQ_WAVE_CYCLES"], 3),
                      "waiting_on_results": round(rec["SQ_WAIT_ANY"] / rec["SQ_WAVE_CYCLES"], 3),
                      "waiting_for_issue": round(rec["SQ_WAIT_INST_ANY"] / rec["SQ_WAVE_CYCLES"], 3)},
        "valu_busy": round(rec["SQ_INSTS_VALU"] * 2 / (SIMDS * launch_cyc), 3),
        "lds_array_busy": round(rec["SQ_LDS_IDX_ACTIVE"] / (SIMDS / 4 * launch_cyc), 3),
        "lds_bank_conflict_share": round(rec["SQ_LDS_BANK_CONFLICT"] / rec["SQ_LDS_IDX_ACTIVE"], 3),
        "note": "slot_fill < 1 is the launch's ramp and tail (fewer rows than slots); per-wave time is issue + "
                "LDS round trips of an in-order wave: a third wave per SIMD (12-wave workgroups, round 4) did not "
                "raise throughput",
    }


def bound_of(hbm_frac, model):
    """roofline.bound from the measurements: 'hbm' when the kernel moves at
    least half of HBM peak, else what the slot model says a wave is doing."""
    if hbm_frac >= 0.5:
        return "hbm"
    if model is None:
        return "latency"
    return "issue+lds-latency (in-order waves; HBM %.3f, VALU %.2f, LDS array %.2f busy)" % (
        hbm_frac, model["valu_busy"], model["lds_array_busy"])


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--batch", type=int, default=64, help="frames per GPU per step (C4: 512 frames / 8 GPUs)")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="budget for the CPU baseline sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--slots", type=int, default=3, help="batches in flight (two HIP streams each)")
    p.add_argument("--no-split", dest="split", action="store_false",
                   help="run each batch's decode side after its encode side on the batch's one stream instead of "
                        "on a second stream beside it (round 4, tools/gpu_bench_cfg.sh, 3 alternations: split "
                        "6,470-6,697 mean / 6,387-6,446 median MPix/s, one stream 6,374-6,389 / 6,208-6,401: with one "
                        "stream a batch's next encode waits behind its own decode, which runs slowly beside the "
                        "other batches' encodes, and the GPU idles at the ends of the decodes)")
    p.add_argument("--iso-steps", type=int, default=2, help="untimed one-batch passes for the isolated kernel times")
    p.add_argument("--no-gather", action="store_true",
                   help="with N > 1, skip the gather of the last batch's outputs to rank 0 (timed apart from value)")
    p.add_argument("--runs", type=int, default=10, help="repeats of the short timed region for the medians")
    p.add_argument("--run-steps", type=int, default=6, help="steps per median run")
    p.add_argument("--no-c3c5", dest="c3c5", action="store_false",
                   help="skip the C3 / C5 single-GPU measurements (reported beside value, not in it)")
    p.add_argument("--launcher-check", action="store_true",
                   help="CPU/gloo: start the ranks, join them and time an empty step; no GPU work, no measurement "
                        "(tests/test_bench_launch.py)")
    return p.parse_args()


def content_rgba(kind, seed):
    from tools import synth
    return {"grad": lambda: synth.gradient_rgba(W, H, seed=seed), "noise": lambda: synth.noise_rgba(W, H, seed=seed),
            "photo": lambda: synth.photo_rgba(W, H, seed=seed)}[kind]()


def frame_rgba(g):
    """Global frame g of the job (rank r's frame i: g = r * batch + i): content g % 3, seed g."""
    return content_rgba(CONTENTS[g % 3], g)


def parsed_bitstreams():
    """(dims, mb_info, coeffs) of the three libwebp q75 1080p bitstreams, parsed by the product parser."""
    from webp_amd import frames
    z = np.load(BITSTREAMS)
    out = {}
    for k in CONTENTS:
        dims, mb, co = frames.vp8_parse(z[k].tobytes())
        assert (dims["width"], dims["height"], dims["filter_type"]) == (W, H, 2), dims
        out[k] = (mb, co)
    return out


def make_inputs(batch, rank, device):
    """Frame i of rank r is global frame g = r * batch + i: content g % 3 with
    seed g (frame_rgba), so every frame of every rank is distinct.  The decode
    side takes content g % 3's parsed libwebp bitstream."""
    from webp_amd import frames
    rgba = torch.empty((batch, H, W, 4), dtype=torch.uint8, device=device)
    for i in range(batch):
        rgba[i].copy_(torch.from_numpy(frame_rgba(rank * batch + i)))
    parsed = parsed_bitstreams()
    per = MBW * MBH
    mb_t = [frames.mb_info_tensor(parsed[k][0], device).view(per, 32) for k in CONTENTS]
    co_t = [torch.from_numpy(parsed[k][1]).to(device).view(per, 384) for k in CONTENTS]
    mb_all = torch.empty((batch, per, 32), dtype=torch.uint8, device=device)
    co_all = torch.empty((batch, per, 384), dtype=torch.int16, device=device)
    for i in range(batch):
        mb_all[i].copy_(mb_t[(rank * batch + i) % 3])
        co_all[i].copy_(co_t[(rank * batch + i) % 3])
    return rgba, mb_all.view(-1, 32), co_all.view(-1, 384), parsed


class Slot:
    """One in-flight batch: its own HIP stream and every output / work buffer."""

    def __init__(self, batch, device, frames, lib):
        self.stream = torch.cuda.Stream(device)
        self.dstream = torch.cuda.Stream(device)  # the decode side (independent of the encode side's data)
        self.Y = torch.empty((batch, 16 * MBH, 16 * MBW), dtype=torch.uint8, device=device)
        self.U = torch.empty((batch, 8 * MBH, 8 * MBW), dtype=torch.uint8, device=device)
        self.V = torch.empty_like(self.U)
        self.alphas = torch.empty((batch, MBW * MBH), dtype=torch.int32, device=device)
        self.uv_sum = torch.empty((batch,), dtype=torch.int32, device=device)
        self.seg_ids = torch.empty((batch, MBW * MBH), dtype=torch.uint8, device=device)
        self.segs = torch.empty((batch, 4 * frames.SEGMENT_DTYPE.itemsize), dtype=torch.uint8, device=device)
        self.seg_info = torch.empty((batch, frames.FRAME_SEGS_DTYPE.itemsize), dtype=torch.uint8, device=device)
        self.enc_out = torch.empty((batch * MBW * MBH, frames.MB_ENC_DTYPE.itemsize), dtype=torch.uint8, device=device)
        self.rY, self.rU, self.rV = torch.empty_like(self.Y), torch.empty_like(self.U), torch.empty_like(self.U)
        self.enc_work = torch.empty(lib.wg_encode_work_bytes(MBW, MBH, batch), dtype=torch.uint8, device=device)
        self.dY = torch.empty_like(self.Y)
        self.dU = torch.empty_like(self.U)
        self.dV = torch.empty_like(self.U)
        self.work = torch.empty(lib.wg_decode_work_bytes(MBW, MBH, batch), dtype=torch.uint8, device=device)
        self.out = torch.empty((batch, H, W, 4), dtype=torch.uint8, device=device)
        self.used = False


class Pipeline:
    """The 6 stages over pre-allocated buffers, optional per-stage HIP events.

    With `slots` > 1, consecutive steps alternate between slots, each with its
    own HIP stream and buffers, so step k+1's kernels fill the CUs that step
    k's encoder RD wavefront leaves idle in its ramp-down.  Every
    step still runs every stage over its whole batch; the timed region ends
    with a device-wide synchronisation."""

    def __init__(self, rgba, mb, co, batch, device, slots=1, split=False):
        from webp_amd import _lib, frames
        self.frames = frames
        self.rgba, self.mb, self.co, self.batch = rgba, mb, co, batch
        self.split = split  # decode side on the slot's second stream, beside its encode side
        self.cfg = frames.encoder_config(**ENC_CFG)
        self.proba = frames.default_proba(device)
        self.slots = [Slot(batch, device, frames, _lib.lib) for _ in range(slots)]
        self.k = 0
        self.events = []
        # Bind every slot stream to its hardware queue now: the first kernel on
        # a new stream makes the runtime create and map a queue, and doing that
        # while a persistent kernel runs on another queue stalled that kernel
        # past its 2 s dependency-wait bound (the first overlapped step timed
        # out; tools/debug_timeouts.py).
        for sl in self.slots:
            with torch.cuda.stream(sl.stream):
                sl.uv_sum.zero_()
            with torch.cuda.stream(sl.dstream):
                sl.dY[:1, :1].zero_()
        torch.cuda.synchronize(device)  # inputs made on the default stream are ready for every slot stream

    def step(self, record=False, side=None):
        """One pass over the batch; side "encode" / "decode" runs that half alone (the per-side medians)."""
        sl = self.slots[self.k % len(self.slots)]
        self.k += 1
        sl.used = True
        with torch.cuda.stream(sl.stream):
            self._stages(sl, record and side is None, side)

    def _stages(self, sl, record, side=None):
        """Encode side on the slot's stream; decode side on its second stream
        (split) or after the encode side on the same one.  The encode and
        decode sides share no data, so with `split` a slot's decode runs
        beside its encode; the step's region still covers both (the timed
        region ends with a device-wide synchronisation)."""
        f = self.frames
        ev = []

        def mark(stream=None):
            if record:
                ev.append(torch.cuda.Event(enable_timing=True))
                ev[-1].record(stream)  # the slot's stream (current) unless given

        # (the decode side needs no wait: its inputs were ready before the first
        # step, and a slot's decodes are ordered by its decode stream)
        dstream = sl.dstream if self.split else None
        mark()
        if side != "decode":
            f.import_rgba(self.rgba, has_alpha=False, out=(sl.Y, sl.U, sl.V))
            mark()
            f.analysis_alphas(sl.Y, sl.U, sl.V, W, H, out=(sl.alphas, sl.uv_sum, None, None))
            mark()
            f.segment_analysis(self.cfg, sl.alphas, sl.uv_sum, MBW, MBH, out=(sl.seg_ids, sl.segs, sl.seg_info))
            f.encode_row_order(sl.alphas, MBW, MBH, work=sl.enc_work)
            mark()
            f.encode_mbs(sl.Y, sl.U, sl.V, W, H, sl.seg_ids, sl.segs, self.proba, method=ENC_CFG["method"],
                         quality=ENC_CFG["quality"], out=sl.enc_out, recon=(sl.rY, sl.rU, sl.rV), work=sl.enc_work)
            mark()
        if side != "encode":
            ctx = torch.cuda.stream(dstream) if dstream is not None else contextlib.nullcontext()
            with ctx:
                if dstream is not None and record:  # decode's own start mark, on its stream
                    ev.append(torch.cuda.Event(enable_timing=True))
                    ev[-1].record(dstream)
                f.decode_frames(self.mb, self.co, 2, MBW, MBH, self.batch, out=(sl.dY, sl.dU, sl.dV), work=sl.work)
                mark(dstream)
                f.build_nrgba(sl.dY, sl.dU, sl.dV, W, H, out=sl.out)
                mark(dstream)
        if record:
            self.events.append(ev)

    def stage_ms(self):
        """Average per-stage event time over the recorded steps (synchronises)."""
        torch.cuda.synchronize()
        names = list(BYTES_PER_PX)
        acc = {k: 0.0 for k in names}
        for ev in self.events:
            # consecutive marks; split: the decode side's own start mark sits
            # between the encode side's last mark and the decode mark
            pairs = [(k, k + 1) for k in range(len(names))]
            if len(ev) == len(names) + 2:
                pairs = pairs[:4] + [(5, 6), (6, 7)]
            for (a, b), name in zip(pairs, names):
                acc[name] += ev[a].elapsed_time(ev[b])
        n = max(1, len(self.events))
        self.events = []
        return {k: v / n for k, v in acc.items()}

    def check_status(self):
        """Raises if an in-kernel dependency wait timed out: the slots' last
        launches (their work-buffer flags) or any earlier launch (the library's
        device-wide count of timed-out waits, never reset)."""
        for sl in self.slots:
            if sl.used:
                with torch.cuda.stream(sl.stream):
                    self.frames.encode_status(sl.enc_work, MBW, self.batch)
                with torch.cuda.stream(sl.dstream if self.split else sl.stream):
                    self.frames.decode_status(sl.work, MBW, self.batch)


def cpu_threads():
    """Host cores this run may use: the box's CPU share (OMP_NUM_THREADS is set
    to it on the GPU box) capped by the affinity mask."""
    n = len(os.sched_getaffinity(0))
    env = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(env))) if env and env.isdigit() else max(1, min(n, 16))


def cpu_baseline(seconds, parsed):
    """C restatement of the reference Go CPU path (oracle/) on a bounded sample
    of the same per-frame workload and the same content mix as the GPU batch
    (frame i: content i % 3 for both the encode and the decode side): import
    -> computeAlphas -> segment analysis -> Phase A RD -> decode of the parsed
    q75 bitstream -> upsample.  First one thread, then one frame per thread on
    every host core this run may use (ctypes releases the GIL for the C calls).
    The reference parallelises inside a frame (row workers,
    encode_parallel.go:176); across independent frames is the same work with
    no synchronisation, so the threaded figure is an upper bound of what its
    CPU path reaches on these cores."""
    import concurrent.futures as cf

    import oracle as O
    imgs = [frame_rgba(j) for j in range(3)]
    cfg = O.encoder_config(**ENC_CFG)
    proba = O.default_proba()

    def one_frame(i):
        k = i % 3
        Y, U, V = O.import_rgba(imgs[k], has_alpha=False)
        O.encode_frame(Y, U, V, W, H, cfg, proba)
        mb, co = parsed[CONTENTS[k]]
        dy, du, dv = O.decode_frame(mb, co, 2, MBW, MBH)
        O.build_nrgba(dy, du, dv, W, H)

    def run(budget, start):
        done, t0 = 0, time.perf_counter()
        while True:
            one_frame(start + done)
            done += 1
            el = time.perf_counter() - t0
            if el >= budget and done % 3 == 0:
                return done, el

    f1, e1 = run(seconds / 3, 0)  # also initialises the oracle's lazily built tables before threading
    single = f1 * W * H / e1 / 1e6
    threads = cpu_threads()
    if threads > 1:
        t0 = time.perf_counter()
        with cf.ThreadPoolExecutor(threads) as ex:
            res = list(ex.map(lambda t: run(seconds * 2 / 3, t), range(threads)))
        el = time.perf_counter() - t0
        fn = sum(r[0] for r in res)
        value = fn * W * H / el / 1e6
    else:
        fn, value = f1, single
    return {"value": round(value, 2), "unit": "MPixels/s", "cores": threads, "kind": "port",
            "single_thread_value": round(single, 2),
            "sample": f"{fn} x 1920x1080 frames on {threads} threads (one frame per thread, contents gradient/noise/"
                      f"photo in turn; {f1} frames on 1 thread before it) of import+analysis+segments+MB RD+q75 "
                      "decode+upsample, C restatement of the reference Go CPU path"}


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


def isolated_stage_ms(rgba, mb, co, batch, device, steps):
    """Per-kernel launch time with one batch in flight (no overlap with other
    slots' kernels): the roofline's launch duration."""
    pipe = Pipeline(rgba, mb, co, batch, device, slots=1, split=False)
    pipe.step()
    torch.cuda.synchronize()
    for _ in range(steps):
        pipe.step(record=True)
    ms = pipe.stage_ms()
    pipe.check_status()
    return ms


def median_runs(pipe, runs, steps, world, device):
    """BASELINE.md 2's statistic: the median over `runs` short timed regions
    (each bracketed like the main one, MAX over ranks) of MPix/s for the whole
    path and for each side alone.  One untimed step before each side."""
    out = {}
    for side in (None, "encode", "decode"):
        pipe.step(side=side)
        vals = []
        for _ in range(runs):
            el = timed_region(lambda record=False: pipe.step(side=side), steps, 0, world, torch.cuda.synchronize,
                              device)
            vals.append(aggregate_mpix_s(world, pipe.batch, steps, el))
        vals.sort()
        m = len(vals)
        med = vals[m // 2] if m % 2 else (vals[m // 2 - 1] + vals[m // 2]) / 2
        out[side or "encode+decode"] = {"median": round(med, 1), "min": round(vals[0], 1), "max": round(vals[-1], 1)}
    pipe.events = []
    return {"runs": runs, "steps_per_run": steps, "unit": "MPixels/s", **out}


def single_frame_encode(device, reps=3):
    """C2 (one 1920x1080 frame, q75 defaults) per content: the encode DSP path
    (import -> analysis -> segments -> RD) and the RD launch alone, best of
    `reps`, event-timed on the current stream.  A one-frame RD launch is the
    macroblock wavefront's critical path: (mbw + 2 (mbh - 1)) macroblock
    times of the row's wave pair, which gives the per-MB latency."""
    from webp_amd import frames
    cfg = frames.encoder_config(**ENC_CFG)
    proba = frames.default_proba(device)
    steps_cp = MBW + 2 * (MBH - 1)
    res = {}
    for j, kind in enumerate(CONTENTS):
        rgba = torch.from_numpy(frame_rgba(j)[None]).to(device)
        best_path = best_rd = None
        for rep in range(reps + 1):
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record()
            Y, U, V = frames.import_rgba(rgba, has_alpha=False)
            al, uvs = frames.analysis_alphas(Y, U, V, W, H)
            ids, segs, _ = frames.segment_analysis(cfg, al, uvs, MBW, MBH, info=False)
            work = frames.encode_row_order(al, MBW, MBH)
            e[1].record()
            frames.encode_mbs(Y, U, V, W, H, ids, segs, proba, method=ENC_CFG["method"], quality=ENC_CFG["quality"],
                              work=work)
            e[2].record()
            frames.encode_status(work, MBW, 1)
            rd, path = e[1].elapsed_time(e[2]), e[0].elapsed_time(e[2])
            if rep > 0:  # the first pass builds the per-device tables
                best_rd = rd if best_rd is None else min(best_rd, rd)
                best_path = path if best_path is None else min(best_path, path)
        res[kind] = {"path_ms": round(best_path, 3), "rd_ms": round(best_rd, 3),
                     "mpix_s": round(W * H / best_path / 1e3, 1),
                     "per_mb_us": round(best_rd * 1e3 / steps_cp, 2)}
    return {"frames": res, "critical_path_mb_steps": steps_cp}


C3_STREAM = os.path.join(ROOT, "tests", "golden", "c3_4096_q75.npz")
C5_N = 4096
# algorithmic HBM bytes per pixel of the C5 stages: ARGB in and
# out (8), packed RGB in + Y / U / V out (4.5, SharpYUV), two planes in (2, SSIM)
C5_BYTES_PER_PX = {"subtract_green": 8.0, "residual_image": 8.0, "sharpyuv": 4.5, "plane_ssim": 2.0}


def event_ms(fn, reps):
    """Median over `reps` of fn's device time, HIP events on the current stream
    (one untimed call first)."""
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2]


def stage_record(ms, px, bytes_per_px, kernel):
    gbs = bytes_per_px * px / (ms / 1e3) / 1e9
    return {"kernel": kernel, "ms": round(ms, 4), "MPix/s": round(px / ms / 1e3, 1), "bytes_per_px": bytes_per_px,
            "GB/s": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4)}


def c3_decode(device, reps=10):
    """BASELINE.json configs[2]: one 4096x4096 lossy decode -- a libwebp q75
    stream of test_color.png tiled, parsed on the host by
    wg_vp8_parse (timed apart), then reconstruct + loop filter and fancy
    upsample to NRGBA on the GPU; median device times over `reps`."""
    from webp_amd import _lib, frames
    data = np.load(C3_STREAM)["webp"].tobytes()
    t0 = time.perf_counter()
    dims, mb, co = frames.vp8_parse(data)
    parse_ms = (time.perf_counter() - t0) * 1e3
    w, h, mbw, mbh, ft = (dims[k] for k in ("width", "height", "mbw", "mbh", "filter_type"))
    mbt = frames.mb_info_tensor(mb, device)
    cot = torch.from_numpy(co).to(device)
    work = torch.empty(_lib.lib.wg_decode_work_bytes(mbw, mbh, 1), dtype=torch.uint8, device=device)
    Y, U, V = frames.decode_frames(mbt, cot, ft, mbw, mbh, 1, work=work)
    out = frames.build_nrgba(Y, U, V, w, h)
    dec_ms = event_ms(lambda: frames.decode_frames(mbt, cot, ft, mbw, mbh, 1, out=(Y, U, V), work=work), reps)
    up_ms = event_ms(lambda: frames.build_nrgba(Y, U, V, w, h, out=out), reps)
    frames.decode_status(work, mbw, 1)
    dk = {1: "k_decode_split", 2: "k_decode_bands"}.get(_lib.lib.wg_decode_kernel(mbh, 1), "k_decode_split")
    px = w * h
    return {"workload": f"one {w}x{h} q75 decode (libwebp stream of testdata/test_color.png tiled, {len(data)} B, "
                        f"{float(mb['is_i4x4'].mean()):.2f} I4, filter type {ft}), reconstruct + loop filter + fancy "
                        "upsample to NRGBA",
            "host_parse_ms": round(parse_ms, 2), "total_ms": round(dec_ms + up_ms, 4),
            "MPix/s": round(px / (dec_ms + up_ms) / 1e3, 1),
            "reconstruct_filter": stage_record(dec_ms, px, BYTES_PER_PX["decode"], dk),
            "upsample": stage_record(up_ms, px, BYTES_PER_PX["upsample"], "k_upsample"),
            "bound": "the macroblock wavefront of one image (latency), not HBM", "reps": reps}


def c5_stages(device, reps=10):
    """BASELINE.json configs[4] on one GPU: a 4096x4096 RGBA N + G blend
     through SubtractGreen + ResidualImage (bits 5, q75), SharpYUV
    (WebP matrix, sRGB) and plane SSIM (Y of the source vs Y + noise);
    median device times over `reps`."""
    from tools import synth
    from webp_amd import frames
    from webp_amd import lossless as L
    n = C5_N
    blend = ((synth.noise_rgba(n, n, seed=55).astype(np.uint16) + 3 * synth.gradient_rgba(n, n).astype(np.uint16))
             // 4).astype(np.uint8)
    blend[..., 3] = 255
    c = blend.astype(np.uint32)
    argb = (c[..., 3] << 24) | (c[..., 0] << 16) | (c[..., 1] << 8) | c[..., 2]
    t = L.to_argb_tensor(argb[None], device)
    px = n * n
    out = {}
    g = t.clone()
    out["subtract_green"] = stage_record(event_ms(lambda: L.SubtractGreen(g), reps), px,
                                         C5_BYTES_PER_PX["subtract_green"], "k_vp8l_green")
    L.SubtractGreen(t)
    modes, res = L.ResidualImage(t, 5, 75)
    out["residual_image"] = stage_record(event_ms(lambda: L.ResidualImage(t, 5, 75, out=(modes, res)), reps), px,
                                         C5_BYTES_PER_PX["residual_image"], "k_vp8l_select_q3 + k_vp8l_residual")
    rgb = torch.from_numpy(np.ascontiguousarray(blend[..., :3])).to(device).unsqueeze(0)
    Ys, Us, Vs = frames.sharpyuv_convert(rgb)
    work = torch.empty(frames.lib.wg_sharpyuv_work_bytes(n, n, 1), dtype=torch.uint8, device=device)
    out["sharpyuv"] = stage_record(event_ms(lambda: frames.sharpyuv_convert(rgb, out=(Ys, Us, Vs), work=work), reps),
                                   px, C5_BYTES_PER_PX["sharpyuv"], "k_sharp_*")
    y = torch.from_numpy(np.ascontiguousarray(blend[..., 1])).to(device).unsqueeze(0)
    y2 = torch.clamp(y.int() + torch.randint(-8, 9, y.shape, device=device, dtype=torch.int32, generator=None),
                     0, 255).to(torch.uint8)
    out["plane_ssim"] = stage_record(event_ms(lambda: frames.plane_ssim(y, y2), reps), px,
                                     C5_BYTES_PER_PX["plane_ssim"], "k_ssim")
    torch.cuda.synchronize()
    return {"workload": f"one {n}x{n} RGBA noise + gradient blend (SURVEY 8(d) C5), 1 GPU", "stages": out,
            "reps": reps}


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(argv, n):
    """`python bench.py --gpus N` (N > 1) without a launcher: run N ranks under
    torch.distributed.run in a child process and return its exit code.  This
    process never touches the GPU (importing torch does not initialise HIP),
    so nothing is re-executed after a device was opened; rank 0's JSON line
    reaches stdout through the child."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL on this pool
    return subprocess.run(cmd, env=env).returncode


def gather_check_tensors(rank, batch=2, w=64, h=48):
    """Stand-ins for a slot's outputs (wg_mb_enc records, reconstruction, NRGBA)
    in the bench's dtypes and layouts, filled with a rank-specific pattern."""
    mbw, mbh = (w + 15) // 16, (h + 15) // 16
    shapes = [((batch * mbw * mbh, 864), torch.uint8), ((batch, 16 * mbh, 16 * mbw), torch.uint8),
              ((batch, 8 * mbh, 8 * mbw), torch.uint8), ((batch, 8 * mbh, 8 * mbw), torch.uint8),
              ((batch, h, w, 4), torch.uint8)]
    out = []
    for j, (shape, dt) in enumerate(shapes):
        n = int(np.prod(shape))
        out.append(((torch.arange(n, dtype=torch.int64) * (7 + j) + 31 * rank + j) % 251).to(dt).reshape(shape))
    return out


def launcher_check(args, world, rank):
    """--launcher-check: the launch / join / timing path on gloo with an empty
    step (no GPU, nothing measured), then the N > 1 gather of main()
    (shard.timed_gather_to_root) over stand-in outputs; rank 0 prints the
    ranks that joined and whether it received every rank's tensors intact."""
    dev = torch.device("cpu")
    if world > 1:
        torch.distributed.init_process_group("gloo")
    joined = torch.ones(1)
    if world > 1:
        torch.distributed.all_reduce(joined)
    elapsed = timed_region(lambda record=False: None, args.steps, args.warmup, world, lambda: None, dev)
    gather = None
    if world > 1 and not args.no_gather:
        from webp_amd import shard
        gather, parts = shard.timed_gather_to_root(gather_check_tensors(rank), world, rank, dev, keep=True)
        if rank == 0:
            gather["ok"] = len(parts) == world and all(
                len(parts[r]) == 5 and all(torch.equal(a, b) for a, b in zip(parts[r], gather_check_tensors(r)))
                for r in range(world))
    if rank == 0:
        print(json.dumps({"metric": "launcher check (no GPU work; not a measurement)", "value": None,
                          "n_gpus": world, "ranks_joined": int(joined.item()), "steps": args.steps,
                          "warmup": args.warmup, "elapsed_s": elapsed, "gather": gather}), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(sys.argv[1:], args.gpus))
    world = int(env_world or "1")
    if world != args.gpus:
        print(f"bench.py: {world} ranks were launched (WORLD_SIZE) but --gpus is {args.gpus}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.launcher_check:
        return launcher_check(args, world, rank)
    if world > 1:
        torch.cuda.set_device(local)
        torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    import webp_amd
    webp_amd.device_check()
    joined = torch.ones(1, device=device)
    if world > 1:
        torch.distributed.all_reduce(joined)  # every rank that joined the process group (RCCL)
    joined = int(joined.item())
    if joined != args.gpus:
        print(f"bench.py: {joined} ranks joined, --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)

    rgba, mb, co, parsed = make_inputs(args.batch, rank, device)
    pipe = Pipeline(rgba, mb, co, args.batch, device, slots=args.slots, split=args.split)
    elapsed = timed_region(pipe.step, args.steps, args.warmup, world, torch.cuda.synchronize, device)
    overlapped = pipe.stage_ms()
    pipe.check_status()  # raises if any launch so far hit an in-kernel wait timeout
    runs = median_runs(pipe, args.runs, args.run_steps, world, device) if args.runs > 0 else None
    pipe.check_status()
    iso = isolated_stage_ms(rgba, mb, co, args.batch, device, args.iso_steps)
    gather = None
    if world > 1 and not args.no_gather:
        from webp_amd import shard
        sl = pipe.slots[(pipe.k - 1) % len(pipe.slots)]
        gather = shard.timed_gather_to_root([sl.enc_out, sl.rY, sl.rU, sl.rV, sl.out], world, rank, device)
    del pipe
    c2 = single_frame_encode(device) if rank == 0 else None
    copy = c3 = c5 = None
    if rank == 0:
        from tools import fetch_calib
        copy = fetch_calib.copy_peak(device)
        if args.c3c5:
            c3 = c3_decode(device)
            c5 = c5_stages(device)
    torch.cuda.synchronize()

    if rank == 0:
        value = aggregate_mpix_s(world, args.batch, args.steps, elapsed)
        step_ms = elapsed / args.steps * 1e3
        dominant = max(iso, key=iso.get)
        px_rank_step = args.batch * W * H
        from webp_amd import _lib
        dk = _lib.lib.wg_decode_kernel(MBH, args.batch)  # the decode kernel this batch launches
        KERNELS["decode"] = {1: "k_decode_split", 2: "k_decode_bands"}.get(dk, KERNELS["decode"])
        kernel = KERNELS[dominant]
        alg = BYTES_PER_PX[dominant] * px_rank_step
        achieved = alg / (iso[dominant] / 1e3) / 1e9
        traffic, traffic_src = pmc_traffic(kernel)
        model = slot_model(iso[dominant], args.batch) if kernel == "k_encode_rows" else None
        rec = {
            "metric": "MPixels/s encode+decode DSP path (1920x1080 q75)",
            "value": round(value, 1),
            "unit": "MPixels/s",
            "n_gpus": world,
            "ranks_joined": joined,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(step_ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic RGBA for the encode side, SURVEY 8(d) G / N / P (gradient, noise, the reference's "
                    "testdata/test_color.png tiled), a distinct seed per frame; libwebp q75 encodes of the three "
                    "contents, parsed by wg_vp8_parse, for the decode side",
            "config": {"workload": f"{args.batch} x 1920x1080 frames per GPU per step (C2 frame, C4 per-GPU share): "
                                   "import+analysis+segments+MB RD loop (encode DSP) + reconstruct+loopfilter+upsample "
                                   "of q75 bitstreams (decode DSP)",
                       "encoder": "webp.Encode DefaultOptions: q75 method 4 sns 50 filter 60 segments 4; segment "
                                  "ids and per-segment quantisers from assignSegments/setSegmentParams on the GPU "
                                  "(k_segments)",
                       "frames_per_gpu": args.batch, "width": W, "height": H, "parallelism": f"frames sharded x{world}",
                       "batches_in_flight": args.slots,
                       "streams_per_batch": 2 if args.split else 1},
            "value_stat": f"mean over the {args.steps} timed steps (the contract's K-step region); medians in `runs`",
            "runs": runs,
            "stage_ms_isolated": {k: round(v, 3) for k, v in iso.items()},
            "stage_ms_overlapped": {k: round(v, 3) for k, v in overlapped.items()},
            "roofline": {"kernel": kernel, "bound": bound_of(achieved / HBM_PEAK_GBS, model), "peak_kind": "hbm",
                         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "traffic_source": traffic_src, "bytes_per_px": BYTES_PER_PX[dominant],
                         "algorithmic_bytes_per_launch": int(alg),
                         "avg_launch_ms": round(iso[dominant], 4), "launch_ms_source": "isolated one-batch pass",
                         "launches_per_step": 1,
                         "measured_copy_peak": copy,
                         "frac_of_measured_copy_peak": round(achieved / copy["GB/s"], 4) if copy else None,
                         # with batches in flight the launches overlap: bytes per step over the step time
                         "achieved_per_step": round(alg / (step_ms / 1e3) / 1e9, 1),
                         "frac_per_step": round(alg / (step_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                         "launches_in_flight": args.slots,
                         "isolated_vs_step": "the isolated launch is longer than ms_per_step because consecutive "
                                             "batches' launches overlap on their own streams",
                         "limiter": "wave-slot time per macroblock (instruction issue + LDS round trips of in-order "
                                    "waves), not HBM: see slot_model, critical_path and valu",
                         "slot_model": model},
            "stage_roofline": {k: {"kernel": KERNELS[k],
                                   "GB/s": round(BYTES_PER_PX[k] * px_rank_step / (v / 1e3) / 1e9, 1),
                                   "frac": round(BYTES_PER_PX[k] * px_rank_step / (v / 1e3) / 1e9 / HBM_PEAK_GBS, 4)}
                               for k, v in iso.items()},
        }
        if c2 is not None:
            slow = max(c2["frames"].values(), key=lambda r: r["rd_ms"])
            rec["roofline"]["critical_path"] = {
                "model": "a one-frame RD launch = (mbw + 2 (mbh - 1)) macroblock latencies of the row's wave pair; "
                         "a batch launch ends on its slowest frame's path plus slot contention",
                "mb_steps": c2["critical_path_mb_steps"],
                "per_mb_us": {k: r["per_mb_us"] for k, r in c2["frames"].items()},
                "slowest_frame_rd_ms": slow["rd_ms"],
                "batch_launch_over_slowest_frame": round(iso[dominant] / slow["rd_ms"], 3)}
            rec["c2_single_frame"] = c2["frames"]
        valu = pmc_valu(kernel, iso[dominant], step_ms)
        if valu is not None:
            rec["valu"] = valu
        if gather is not None:
            rec["gather"] = gather
        if c3 is not None:
            rec["c3"] = c3
        if c5 is not None:
            rec["c5"] = c5
        if not args.no_cpu_baseline and world == 1:  # the CPU baseline is timed at N = 1 only, after the GPU phase
            rec["cpu_baseline"] = cpu_baseline(args.cpu_seconds, parsed)
        print(json.dumps(rec), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
