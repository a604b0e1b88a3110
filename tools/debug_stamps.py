"""Diagnostic: per-phase cycle stamps of k_decode_diag (build with OPT='-O3 -DWG_STAMPS')."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from tools import synth
from webp_amd import _lib, frames
B = int(os.environ.get("BATCH", "64"))
MBW, MBH = 120, 68
for p_i4, ft in ((0.5, 2), (0.0, 0)):
    mb, co = synth.random_macroblocks(MBW * MBH * B, seed=11, levels=(20, 32), p_i4=p_i4)
    Y, U, V = frames.decode_frames(frames.mb_info_tensor(mb), torch.from_numpy(co).cuda(), ft, MBW, MBH, B)
    torch.cuda.synchronize()
    n = 8192 * 12
    buf = (ctypes.c_ulonglong * n)()
    _lib.lib.wg_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert _lib.lib.wg_debug_stamps(ctypes.addressof(buf), n) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(8192, 12).astype(np.int64)
    t = 160
    x_lo = max(t - 2 * (MBH - 1), t & 1)
    x_hi = min(t, MBW - 1)
    count = (x_hi - x_lo) // 2 + 1
    nwg = count * B
    st = st[:nwg]
    t0 = st[:, 0].min()
    print(f"p_i4={p_i4} ft={ft}: {nwg} WGs, launch span {(st[:, 8 if ft else 9].max() - t0)} cycles; start spread {st[:, 0].max() - t0}")
    names = ["start->args", "args->ctx", "ctx->luma", "luma->chroma", "chroma->ctxw", "ctxw->fload", "fH", "fV", "wb"]
    pairs = [(0, 1), (1, 2), (2, 3), (3, 4), (4, 5), (5, 6), (6, 7), (7, 8)] if ft else [(0, 1), (1, 2), (2, 3), (3, 4), (4, 9)]
    for a, b in pairs:
        d = st[:, b] - st[:, a]
        d = d[st[:, b] > 0]
        print(f"   {a}->{b}: median {np.median(d):8.0f}  p90 {np.percentile(d, 90):8.0f}  max {d.max():8.0f} cycles")
