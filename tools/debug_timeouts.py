"""GPU: where does a timed-out encoder row wait come from?  Runs bench
pipeline steps back to back (no sync between them) and reads each launch's own
flag (ctl[1], copied on its stream) and the library's sticky diagnostics."""
import ctypes
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from webp_amd import frames  # noqa: E402
from webp_amd._lib import lib  # noqa: E402

dev = torch.device("cuda", 0)
OFF = 64 * 120 * 64  # ctl = work + n * mbw * REC


def diag():
    try:
        frames.encode_status(WORK, 120, 1)
        return "ok"
    except Exception as e:  # noqa: BLE001
        return str(e)


WORK = torch.zeros(frames.lib.wg_encode_work_bytes(120, 68, 1), dtype=torch.uint8, device=dev)
print("start", diag(), flush=True)
rgba, mb, co, parsed = bench.make_inputs(64, 0, dev)
plan = [(3, 4, False), (3, 4, False), (1, 3, False), (3, 6, False)]
if len(sys.argv) > 1:
    plan = [tuple(int(x) for x in a.split(",")) for a in sys.argv[1:]]
import os  # noqa: E402
WARM = os.environ.get("WARM") == "1"
for slots, steps, sync in plan:
    pipe = bench.Pipeline(rgba, mb, co, 64, dev, slots=slots)
    if WARM:  # a trivial kernel on every slot stream first (binds each stream to its HW queue)
        for sl in pipe.slots:
            with torch.cuda.stream(sl.stream):
                sl.uv_sum.zero_()
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    flags = []
    for k in range(steps):
        pipe.step()
        if sync:
            torch.cuda.synchronize()
        sl = pipe.slots[k % slots]
        with torch.cuda.stream(sl.stream):
            flags.append(sl.enc_work[OFF:OFF + 16].clone())
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    f = [x.view(torch.int32).tolist() for x in flags]
    print(f"slots={slots} steps={steps} sync={sync}: {el * 1e3:.1f} ms, ctl per launch {f}, diag {diag()}", flush=True)
    del pipe
