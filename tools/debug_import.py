"""Debug helper: GPU vs oracle import on a golden crop and a synthetic case."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import oracle as O
from tools import synth
from webp_amd import frames

G = np.load("tests/golden/libwebp_fixtures.npz")
cases = [("imp_b", G["imp_b_rgba"], True), ("noise200x3", synth.noise_rgba(200, 3, seed=203, alpha=True), True)]
for name, rgba, alpha in cases:
    h, w, _ = rgba.shape
    Y, U, V = frames.import_rgba(torch.from_numpy(np.ascontiguousarray(rgba[None])).cuda(), has_alpha=alpha)
    torch.cuda.synchronize()
    Y, U, V = Y[0].cpu().numpy(), U[0].cpu().numpy(), V[0].cpu().numpy()
    ey, eu, ev = O.import_rgba(rgba, has_alpha=alpha)
    for pn, a, b in (("Y", Y, ey), ("U", U, eu), ("V", V, ev)):
        bad = np.argwhere(a != b)
        print(name, pn, "shape", a.shape, "mismatches", len(bad), bad[:8].tolist())
        if len(bad):
            r, c = bad[0]
            print("  gpu", a[r, max(0, c - 4):c + 4], "ora", b[r, max(0, c - 4):c + 4])
