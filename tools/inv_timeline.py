"""Per-band timeline of k_vp8l_inverse on C5's 4096x4096 (bits 5) image.

  make -C webp_amd variant NAME=timelines DEFS=-DWG_TIMELINES
  WEBPGPU_LIB=webp_amd/libwebpgpu_timelines.so python tools/inv_timeline.py [out.json]

The stamps build records per band (32 rows) the s_memrealtime (100 MHz) at
its start and end and the ticks it spent re-polling the band above's
hand-off granules.  Printed: the launch span, each band's walk time and
per-step time (steps = width + 2 * 31; band 0, which waits on nothing, gives
the free-running step), the end-to-end lag between consecutive bands in
steps and beyond the 64 the diagonal needs, and the poll time -- what the
walk's (2 * height + width) x step-time chain and the hand-offs each cost.
`python tools/inv_timeline.py --from saved.json` recomputes from a record."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from tools import synth  # noqa: E402
from webp_amd import lossless as L  # noqa: E402
from webp_amd._lib import call, lib  # noqa: E402

N = int(os.environ.get("N", "4096"))
BITS = 5
TICK_NS = 10.0  # s_memrealtime: 100 MHz


def summarize(start, end, poll, polls):
    walk = end - start
    steps = N + 2 * 31
    step_ns = walk / steps * 1e3
    lag = np.diff(end)
    return {
        "span_us": round(float(end.max()), 1),
        "walk_us": {"median": round(float(np.median(walk)), 1), "min": round(float(walk.min()), 1)},
        "step_ns_free": round(float(step_ns.min()), 1),
        "lag_us": {"median": round(float(np.median(lag)), 2), "min": round(float(lag.min()), 2),
                   "max": round(float(lag.max()), 2)},
        "lag_steps_median": round(float(np.median(lag) * 1e3 / step_ns.min()), 1),
        "lag_steps_over_diagonal": round(float(np.median(lag) * 1e3 / step_ns.min() - 64), 1),
        "poll_us_per_band": {"median": round(float(np.median(poll)), 1), "max": round(float(poll.max()), 1)},
        "polls_per_band_median": int(np.median(polls)) if polls is not None else None,
        "chain_bound_us": round(float((2 * N + N) * step_ns.min() / 1e3), 1),
    }


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--from":
        rec = json.load(open(sys.argv[2]))
        b = np.array(rec["bands"], dtype=np.float64)
        rec.update(summarize(b[:, 0], b[:, 1], b[:, 2], None))
        for k in ("step_ns", "lag_steps_median_old"):
            rec.pop(k, None)
        print(json.dumps({k: v for k, v in rec.items() if k != "bands"}))
        if len(sys.argv) > 3:
            json.dump(rec, open(sys.argv[3], "w"), indent=1)
        return
    rgba = synth.blobs_rgba(N, N, seed=5, alpha=True).astype(np.uint32)
    argb = (rgba[..., 3] << 24) | (rgba[..., 0] << 16) | (rgba[..., 1] << 8) | rgba[..., 2]
    t = L.to_argb_tensor(argb[None])
    modes, res = L.ResidualImage(t, BITS, 75)
    out = torch.empty_like(res)
    bands = (N + 31) // 32
    wb = lib.wg_vp8l_inverse_work_bytes(N, N, 1)
    hand = 16 + 8 * bands * ((N + 1) & ~1)
    assert wb == hand + 32 * bands, "not a WG_TIMELINES build (work bytes %d)" % wb
    work = torch.empty(wb, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    for _ in range(3):  # warm-up, then the recorded launch
        call("wg_vp8l_inverse_predictor", modes.data_ptr(), BITS, N, N, N * N, 1, res.data_ptr(), out.data_ptr(),
             work.data_ptr(), stream)
        call("wg_vp8l_inverse_status", work.data_ptr(), stream)
    torch.cuda.synchronize()
    assert torch.equal(out, t), "inverse != source"
    st = work[hand:].cpu().numpy().view(np.uint64).reshape(bands, 4).astype(np.int64)
    t0 = st[:, 0].min()
    start, end = (st[:, 0] - t0) * TICK_NS / 1e3, (st[:, 1] - t0) * TICK_NS / 1e3  # us
    poll = (st[:, 2] & 0xFFFFFFFF) * TICK_NS / 1e3
    polls = st[:, 2] >> 32
    # every band starts at once (all resident) and waits: the lag shows in the ends
    rec = {"config": f"C5 {N}x{N} bits {BITS}: k_vp8l_inverse, one wave per 32-row band",
           **summarize(start, end, poll, polls),
           "bands": [[round(float(a), 2), round(float(b), 2), round(float(c), 2)] for a, b, c in zip(start, end, poll)]}
    line = json.dumps({k: v for k, v in rec.items() if k != "bands"})
    print(line)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()
