"""Diagnostic: the row timeline of one k_encode_rows launch over the bench's
batch (64 1080p frames: bench.py's frame_rgba contents -- gradient / noise /
photo in turn, a distinct seed each -- the q75 segment setup and the row
schedule, as bench.py).  Answers what bounds the
launch: when each content's frames finish, how many rows are in flight over
time (the tail), and how long a row takes by content.

  make -C webp_amd libwebpgpu_rowtimes.so
  WEBPGPU_LIB=webp_amd/libwebpgpu_rowtimes.so python tools/enc_timeline.py

Env: BATCH (64), PAIR (unset: the library's choice; 0 / 1 forced), JSON (path
to also write the summary)."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import oracle as O  # noqa: E402
from webp_amd import _lib, frames  # noqa: E402

B, W, H = int(os.environ.get("BATCH", "64")), 1920, 1080
MBW, MBH = 120, 68
KINDS = ["grad", "noise", "photo"]
if os.environ.get("PAIR") is not None:
    os.environ["WG_ENCODE_PAIR"] = os.environ["PAIR"]
lib = _lib.lib
if not hasattr(lib, "wg_debug_enc_rows"):
    sys.exit("needs WEBPGPU_LIB=webp_amd/libwebpgpu_rowtimes.so")
lib.wg_debug_enc_rows.argtypes = [ctypes.c_void_p, ctypes.c_int]

rgba = torch.from_numpy(np.stack([bench.frame_rgba(g) for g in range(B)])).cuda()
Y, U, V = frames.import_rgba(rgba, has_alpha=False)
alphas, uv_sum = frames.analysis_alphas(Y, U, V, W, H)
seg_ids, segs, _ = frames.segment_analysis(frames.encoder_config(), alphas, uv_sum, MBW, MBH)
proba = O.default_proba()
work = frames.encode_row_order(alphas, MBW, MBH)
out, rec = frames.encode_mbs(Y, U, V, W, H, seg_ids, segs, proba, work=work, check=True)
summ = {}
for rep in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    frames.encode_mbs(Y, U, V, W, H, seg_ids, segs, proba, out=out, recon=rec, work=work)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
rows = B * MBH
buf = np.zeros((rows, 4), np.uint64)
lib.wg_debug_enc_rows(buf.ctypes.data, rows)
ro, t0, t1 = buf[:, 0].astype(np.int64), buf[:, 1].astype(np.int64), buf[:, 2].astype(np.int64)
base = t0.min()
t0 = (t0 - base) / 100.0  # 100 MHz ticks -> us
t1 = (t1 - base) / 100.0
img = ro % B
y = ro // B
kind = img % 3
span = t1.max()
print(f"launch {ms:.3f} ms (event); row timeline span {span / 1e3:.3f} ms over {rows} rows")
for k, name in enumerate(KINDS):
    sel = kind == k
    fin = np.array([t1[(img == i)].max() for i in range(B) if i % 3 == k])
    dur = (t1 - t0)[sel]
    print(f"  {name:8s}: frames finish {fin.min() / 1e3:6.2f} .. {fin.max() / 1e3:6.2f} ms; "
          f"row time median {np.median(dur) / 1e3:6.2f} ms (per MB {np.median(dur) / MBW:6.1f} us), "
          f"max {dur.max() / 1e3:6.2f} ms")
    summ[name] = {"finish_ms": [round(fin.min() / 1e3, 3), round(fin.max() / 1e3, 3)],
                  "row_ms_median": round(float(np.median(dur)) / 1e3, 3)}
# rows in flight over time, 1 ms bins
edges = np.arange(0, span + 1000, 1000)
inflight = [int(((t0 <= e) & (t1 > e)).sum()) for e in edges]
print("  rows in flight at 0,1,2.. ms:", inflight)
# the last rows: which frames and how far the slowest frame's rows trail
last = np.argsort(t1)[-10:]
print("  last rows (img, y, kind, start ms, end ms):",
      [(int(img[i]), int(y[i]), KINDS[kind[i]], round(t0[i] / 1e3, 2), round(t1[i] / 1e3, 2)) for i in last])
# slot occupancy: wave-time inside rows (waits for the row above included)
# over the resident wave slots x the span, and the waits before a row's
# first macroblock are not separable here (start = dequeue)
slots = int(os.environ.get("SLOTS", "2048"))
busy = float((t1 - t0).sum()) / (slots * span)
print(f"  row-time / (slots {slots} x span): {busy:.3f}")
summ.update({"launch_ms": round(ms, 3), "span_ms": round(span / 1e3, 3), "inflight_per_ms": inflight,
             "row_time_fill": round(busy, 3)})
if os.environ.get("RAW"):  # the raw timeline: dequeue index -> (ro, start us, end us, block << 8 | wave)
    np.savez_compressed(os.environ["RAW"], ro=ro, t0=t0, t1=t1, who=buf[:, 3].astype(np.int64), launch_ms=ms)
if os.environ.get("JSON"):
    json.dump(summ, open(os.environ["JSON"], "w"), indent=1)
