"""Diagnostic: one small encode vs the oracle, per-field / per-block mismatch report
(WG_ENCODE_PAIR picks the row schedule)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402
from tools import synth  # noqa: E402
from webp_amd import frames  # noqa: E402

FIELDS = ("coeffs", "modes", "nz_y", "nz_uv", "non_zero_y", "non_zero_uv", "mb_type", "i16_mode", "uv_mode", "nz_dc",
          "skip", "segment", "score")
w, h = int(os.environ.get("W", 16)), int(os.environ.get("H", 64))
method = int(os.environ.get("METHOD", 4))
y, u, v = O.import_rgba(synth.noise_rgba(w, h, seed=w), has_alpha=False)
qs = (20, 30, 40, 50)
mbw, mbh = frames.mb_dims(w, h)
segs = np.stack([O.setup_segment(q, method=method, sns_strength=50) for q in qs])
seg_ids = ((np.arange(mbw * mbh) * 7) % 4).astype(np.uint8)[None]
proba = O.default_proba()
out, (RY, RU, RV) = frames.encode_mbs(torch.from_numpy(y[None]).cuda(), torch.from_numpy(u[None]).cuda(),
                                      torch.from_numpy(v[None]).cuda(), w, h, torch.from_numpy(seg_ids).cuda(),
                                      segs.view(frames.SEGMENT_DTYPE), proba, method=method, quality=75, check=True)
got = out.cpu().numpy().view(frames.MB_ENC_DTYPE).reshape(mbw * mbh)
enc, ry, ru, rv = O.encode_frame_rd(y, u, v, w, h, seg_ids[0], segs, proba, method=method, quality=75)
for f in FIELDS:
    bad = np.argwhere(np.asarray(got[f] != enc[f]).reshape(len(enc), -1).any(axis=1)).ravel()
    print(f, "bad MBs", bad[:8])
for mb in range(min(3, len(enc))):
    print("MB", mb, "type got/exp", got["mb_type"][mb], enc["mb_type"][mb], "i16", got["i16_mode"][mb], enc["i16_mode"][mb],
          "uv", got["uv_mode"][mb], enc["uv_mode"][mb], "score", got["score"][mb], enc["score"][mb])
    g, e = got["coeffs"][mb].reshape(25, 16), enc["coeffs"][mb].reshape(25, 16)
    print("  blocks differing:", [i for i in range(25) if (g[i] != e[i]).any()])
    for i in [i for i in range(25) if (g[i] != e[i]).any()][:3]:
        print("   blk", i, "got", g[i].tolist(), "\n          exp", e[i].tolist())
print("RY ok", (RY.cpu().numpy()[0][:h, :w] == ry[:h, :w]).all(), "RU ok", (RU.cpu().numpy()[0] == ru).all())
