"""Per-wave timeline of k_sharp_wave on C5's 4096x4096 image (SharpYUV's four
refinement iterations as a pipeline of column-band waves).

  make -C webp_amd variant NAME=timelines DEFS=-DWG_TIMELINES
  WEBPGPU_LIB=webp_amd/libwebpgpu_timelines.so python tools/sharp_timeline.py [out.json]

The timelines build records per workgroup (image, iteration, band) and role
(wave A: the Gauss-Seidel chain and the chroma update; wave B: the second row
of each row pair) the s_memrealtime (100 MHz) at the walk's start and end and
the ticks spent waiting: on other workgroups' progress words in global
memory (the input state of iteration k - 1, the neighbour bands' halo rows)
and on the partner wave's LDS progress.  Printed: the span, each
iteration's finish, how far iteration k + 1 trails iteration k, and the
waits' shares of the walk."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from tools import synth  # noqa: E402
from webp_amd import frames  # noqa: E402
from webp_amd._lib import lib  # noqa: E402

N = int(os.environ.get("N", "4096"))
TICK_US = 0.01  # s_memrealtime: 100 MHz
WB_OWN = 32


def layout(width, height, n=1):
    """sharpyuv.hip sharp_layout / wg_sharpyuv_work_bytes: (offset of the timeline records, bands)."""
    w, h = (width + 1) & ~1, (height + 1) & ~1
    uv_rs = (3 * (w // 2) + 7) & ~7
    y_elems = (w * h + 7) & ~7
    uv_elems = uv_rs * (h // 2)
    bytes_img = 2 * (6 * y_elems + 6 * uv_elems)
    nb = (w // 2 + WB_OWN - 1) // WB_OWN
    tail = n * bytes_img
    return tail + ((n * (32 + 4 + 16 * nb) + 7) & ~7) + n * 4 * nb * 2 * WB_OWN * 8, nb  # (after the edge granules)


def main():
    rgba = synth.blobs_rgba(N, N, seed=5, alpha=True)
    rgb = torch.from_numpy(np.ascontiguousarray(rgba[..., :3])).cuda().unsqueeze(0)
    off, nb = layout(N, N)
    wb = lib.wg_sharpyuv_work_bytes(N, N, 1)
    assert wb >= off + 64 * 4 * nb, "not a WG_TIMELINES build (work bytes %d)" % wb
    work = torch.empty(wb, dtype=torch.uint8, device="cuda")
    Y, U, V = frames.sharpyuv_convert(rgb, work=work)
    for _ in range(2):  # warm-up, then the recorded launch
        Y, U, V, its = frames.sharpyuv_convert(rgb, out=(Y, U, V), work=work, iterations=True)
    torch.cuda.synchronize()
    st = work[off:off + 64 * 4 * nb].cpu().numpy().view(np.uint64).reshape(4, nb, 2, 4).astype(np.int64)
    t0 = st[..., 0].min()
    start = (st[..., 0] - t0) * TICK_US
    end = (st[..., 1] - t0) * TICK_US
    gwait = (st[..., 2] & 0xFFFFFFFF) * TICK_US
    lwait = (st[..., 3] & 0xFFFFFFFF) * TICK_US
    walk = end - start
    span = float(end.max())
    fin = [float(end[k].max()) for k in range(4)]
    # iteration k + 1 trails k: per band, the end of A (the chain) of k + 1 minus that of k
    trail = [float(np.median(end[k + 1, :, 0] - end[k, :, 0])) for k in range(3)]
    rec = {
        "config": f"C5 {N}x{N}: k_sharp_wave, 4 iterations x {nb} column bands, 2 waves a band",
        "iterations_run": int(its[0]),
        "span_us": round(span, 1),
        "iteration_end_us": [round(x, 1) for x in fin],
        "iteration_trail_us_median": [round(x, 1) for x in trail],
        "walk_us_median": {"A": round(float(np.median(walk[..., 0])), 1), "B": round(float(np.median(walk[..., 1])), 1)},
        "start_us_max": round(float(start.max()), 1),
        "global_wait_share": {"A": round(float(gwait[..., 0].sum() / walk[..., 0].sum()), 3),
                              "B": round(float(gwait[..., 1].sum() / walk[..., 1].sum()), 3)},
        "lds_wait_share": {"A": round(float(lwait[..., 0].sum() / walk[..., 0].sum()), 3),
                           "B": round(float(lwait[..., 1].sum() / walk[..., 1].sum()), 3)},
        "iteration0_walk_us": {"min": round(float(walk[0, :, 0].min()), 1), "max": round(float(walk[0, :, 0].max()), 1)},
        "waves": [[[round(float(start[k, b, r]), 1), round(float(end[k, b, r]), 1), round(float(gwait[k, b, r]), 1),
                    round(float(lwait[k, b, r]), 1)] for r in range(2) for b in range(nb)] for k in range(4)],
    }
    print(json.dumps({k: v for k, v in rec.items() if k != "waves"}))
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()
