"""Diagnostic: cycles per phase of k_encode_rows.

Run against the stamped build: make -C webp_amd libwebpgpu_stamps.so, then
WEBPGPU_LIB=webp_amd/libwebpgpu_stamps.so CONTENT=noise python tools/debug_enc_phases.py
(CONTENT = blobs | noise | gradient | mix (gradient / noise / blobs in turn) |
bench: bench.py's frames, frame_rgba(g) for g < BATCH)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import oracle as O
from webp_amd import _lib, frames
from tools import synth
B, W, H = int(os.environ.get("BATCH", "64")), 1920, 1080
MBW, MBH = 120, 68
names = ["wait", "import+ctx", "i16rd", "i4rd", "uvrd", "final", "recon+export", "c:dp(in trellis)", "i4:prescreen", "i4:select", "i4:candidates", "i4:winner", "c:coef-store", "c:trellis-prep", "c:dp+recon+disto", "c:rate+score"]
STAMPED = hasattr(_lib.lib, "wg_debug_enc_phases")  # only the stamped build (-DWG_STAMPS) exports it
if STAMPED:
    _lib.lib.wg_debug_enc_phases.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = (ctypes.c_ulonglong * 16)()
content = os.environ.get("CONTENT", "blobs")
gens = {"blobs": lambda: synth.blobs_rgba(W, H, seed=3), "noise": lambda: synth.noise_rgba(W, H, seed=3),
        "gradient": lambda: synth.gradient_rgba(W, H)}
if content == "bench":
    import bench
    rgba = torch.from_numpy(np.stack([bench.frame_rgba(g) for g in range(B)])).cuda()
    Yt, Ut, Vt = frames.import_rgba(rgba, has_alpha=False)
else:
    kinds = ["gradient", "noise", "blobs"] if content == "mix" else [content]
    planes = [O.import_rgba(gens[k](), has_alpha=False) for k in kinds]
    Yt = torch.from_numpy(np.stack([planes[i % len(planes)][0] for i in range(B)])).cuda()
    Ut = torch.from_numpy(np.stack([planes[i % len(planes)][1] for i in range(B)])).cuda()
    Vt = torch.from_numpy(np.stack([planes[i % len(planes)][2] for i in range(B)])).cuda()
# the reference's q75 defaults: alphas -> segment analysis on the device (as bench.py)
alphas, uv_sum = frames.analysis_alphas(Yt, Ut, Vt, W, H)
seg_ids, segs, _ = frames.segment_analysis(frames.encoder_config(), alphas, uv_sum, MBW, MBH)
out, rec = frames.encode_mbs(Yt, Ut, Vt, W, H, seg_ids, segs, O.default_proba())
torch.cuda.synchronize()
if STAMPED:
    _lib.lib.wg_debug_enc_phases(ctypes.addressof(buf), 16)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(); frames.encode_mbs(Yt, Ut, Vt, W, H, seg_ids, segs, O.default_proba(), out=out, recon=rec); e1.record()
torch.cuda.synchronize()
mbt = out[:, 848].cpu().numpy()  # wg_mb_enc mb_type (0 = I16, 1 = I4)
print(f"[{content}] I16 share {float((mbt == 0).mean()):.3f}")
if not STAMPED:
    print(f"[{content}] {e0.elapsed_time(e1):.3f} ms")
    sys.exit(0)
_lib.lib.wg_debug_enc_phases(ctypes.addressof(buf), 16)
v = np.frombuffer(buf, dtype=np.uint64)[:16].astype(np.float64) / (MBW * MBH * B)
print(f"[{content}] {e0.elapsed_time(e1):.3f} ms; cycles per MB: " + ", ".join(f"{n}={x:.0f}" for n, x in zip(names, v)) + f"; total={v[:7].sum():.0f}")
# the I4 RD's cycles outside its four stamped sub-phases: the per-step top-right
# wait (step 3), the block's source load and indices, the trellis r0 rows and
# the loop (stamps are exact differences, so this is too)
i4_sub = v[8] + v[9] + v[10] + v[11]
print(f"[{content}] i4rd {v[3]:.0f} = prescreen {v[8]:.0f} + select {v[9]:.0f} + candidates {v[10]:.0f} "
      f"(coefficient store {v[12]:.0f}, trellis prep {v[13]:.0f}, dp {v[7]:.0f}, recon+disto {v[14] - v[7]:.0f}, "
      f"rate+score {v[15]:.0f}) "
      f"+ winner {v[11]:.0f} + outside the sub-phases {v[3] - i4_sub:.0f}")
