"""Diagnostic: cycles per phase of k_encode_rows.

Run against the stamped build: make -C webp_amd libwebpgpu_stamps.so, then
WEBPGPU_LIB=webp_amd/libwebpgpu_stamps.so CONTENT=noise python tools/debug_enc_phases.py
(CONTENT = blobs | noise | gradient | mix, the bench's 3-way frame mix)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import oracle as O
from webp_amd import _lib, frames
from tools import synth
B, W, H = int(os.environ.get("BATCH", "64")), 1920, 1080
MBW, MBH = 120, 68
names = ["wait", "import+ctx", "i16rd", "i4rd", "uvrd", "final", "recon+export", "c:dp(in trellis)", "i4:prescreen", "i4:select", "i4:candidates", "i4:winner", "c:pred+fdct", "c:trellis", "c:recon+disto", "c:rate"]
STAMPED = hasattr(_lib.lib, "wg_debug_enc_phases")  # only the stamped build (-DWG_STAMPS) exports it
if STAMPED:
    _lib.lib.wg_debug_enc_phases.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = (ctypes.c_ulonglong * 16)()
content = os.environ.get("CONTENT", "blobs")
gens = {"blobs": lambda: synth.blobs_rgba(W, H, seed=3), "noise": lambda: synth.noise_rgba(W, H, seed=3),
        "gradient": lambda: synth.gradient_rgba(W, H)}
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
