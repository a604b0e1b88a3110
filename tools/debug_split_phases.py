"""Diagnostic: cycles per MB and phase of k_decode_split (stamped build: make -C
webp_amd libwebpgpu_stamps.so; WEBPGPU_LIB=webp_amd/libwebpgpu_stamps.so).
BATCH frames of SIZE (4096 default: the C3 frame; "1080" for 1080p).  R = the
reconstruction wave, F = the filter wave of each row.  REAL=1:
C3's real q75 4096x4096 stream (tests/golden/c3_4096_q75.npz) instead of the
synthetic macroblocks."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from tools import synth
from webp_amd import _lib, frames
B = int(os.environ.get("BATCH", "1"))
MBW, MBH = (120, 68) if os.environ.get("SIZE") == "1080" else (256, 256)
names = ["R:wait", "R:loads", "R:luma", "R:chroma", "R:handoff", "R:publish", "F:wait", "F:tiles", "F:filter",
         "F:stores"]
_lib.lib.wg_debug_phases.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = (ctypes.c_ulonglong * 16)()
REAL = os.environ.get("REAL") == "1"
cases = [("real", None)] if REAL else [(0.5, 2), (0.0, 2), (1.0, 2)]
for p_i4, ft in cases:
    if REAL:
        z = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                                 "c3_4096_q75.npz"))
        dims, mb, co = frames.vp8_parse(z["webp"].tobytes())
        ft, MBW, MBH, B = dims["filter_type"], dims["mbw"], dims["mbh"], 1
        mbt, cot = frames.mb_info_tensor(mb), torch.from_numpy(co).cuda()
    else:
        nv = min(B, 4)
        mb, co = synth.random_macroblocks(MBW * MBH * nv, seed=11, levels=(20, 32), p_i4=p_i4)
        mbt = frames.mb_info_tensor(mb).view(nv, -1, 32).repeat(B // nv, 1, 1).reshape(-1, 32).contiguous()
        cot = torch.from_numpy(co).cuda().view(nv, -1, 384).repeat(B // nv, 1, 1).reshape(-1, 384).contiguous()
    frames.decode_frames(mbt, cot, ft, MBW, MBH, B)
    torch.cuda.synchronize()
    _lib.lib.wg_debug_phases(ctypes.addressof(buf), 16)  # reset after warmup
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); frames.decode_frames(mbt, cot, ft, MBW, MBH, B); e1.record(); torch.cuda.synchronize()
    _lib.lib.wg_debug_phases(ctypes.addressof(buf), 16)
    v = np.frombuffer(buf, dtype=np.uint64)[:10].astype(np.float64) / (MBW * MBH * B)
    print(f"p_i4={p_i4} ft={ft}: {e0.elapsed_time(e1):.3f} ms; cycles per MB: " +
          ", ".join(f"{n}={x:.0f}" for n, x in zip(names, v)) + f"; R={v[:6].sum():.0f} F={v[6:].sum():.0f}")
