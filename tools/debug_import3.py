import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import oracle as O
from webp_amd import frames
G = np.load("tests/golden/libwebp_fixtures.npz")
rgba = G["imp_b_rgba"]
ey, eu, ev = O.import_rgba(rgba, True)
d = torch.from_numpy(np.ascontiguousarray(rgba[None])).cuda()
for it in range(6):
    Y, U, V = frames.import_rgba(d, has_alpha=True)
    torch.cuda.synchronize()
    U = U[0].cpu().numpy()
    bad = np.argwhere(U != eu)
    print("run", it, "U mismatches", len(bad), "cols mod 4:", np.bincount(bad[:, 1] % 4, minlength=4).tolist() if len(bad) else [])
    if len(bad):
        r, c = bad[0]
        print("   first", r, c, "gpu", U[r, c], "ora", eu[r, c], " rows with errors", sorted(set(bad[:, 0].tolist()))[:12])
