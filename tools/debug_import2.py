import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import oracle as O
from webp_amd import frames
G = np.load("tests/golden/libwebp_fixtures.npz")
rgba = G["imp_b_rgba"]
Y, U, V = frames.import_rgba(torch.from_numpy(np.ascontiguousarray(rgba[None])).cuda(), has_alpha=True)
torch.cuda.synchronize()
print("gpu U row0", U[0, 0, :4].tolist(), "V", V[0, 0, :4].tolist())
ey, eu, ev = O.import_rgba(rgba, True)
print("ora U row0", eu[0, :4].tolist(), "V", ev[0, :4].tolist())
for q in range(4):
    blk = rgba[0:2, 2*q:2*q+2].reshape(4, 4)
    print("q", q, [hex(int.from_bytes(bytes(b), 'little')) for b in blk])
