"""Cycles per step of a dependent VALU chain through one cross-lane move
(tools/dpp_probe.hip), one wave alone on the chip."""
import ctypes
import os

import torch

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libdpp_probe.so"))
out = torch.zeros(64, dtype=torch.int32, device="cuda")
cyc = torch.zeros(1, dtype=torch.int64, device="cuda")
n = 4096
for kind, name in enumerate(["wave_shr:1", "row_shr:1", "none", "row_bcast15+row_shr1", "ds_bpermute", "wave_shr+ds_write_b8"]):
    best = None
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        lib.probe_chain(kind, n, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(cyc.data_ptr()))
        e1.record()
        torch.cuda.synchronize()
        c = int(cyc.item()) / (16 * n)
        ns = e0.elapsed_time(e1) * 1e6 / (16 * n)
        best = (c, ns) if best is None or c < best[0] else best
    print(f"{name:24s} {best[0]:7.1f} s_memtime ticks per step, {best[1]:6.1f} ns per step (event)", flush=True)
