import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import oracle as O
from tools import synth
from webp_amd import frames
mbw, mbh, n = 2, 2, 1
mb, co = synth.random_macroblocks(n * mbw * mbh, seed=5, levels=(0,))
mb["is_i4x4"] = 0
mb["imodes"] = 0
mb["uv_mode"] = 0
mb["non_zero_y"] = 0
mb["non_zero_uv"] = 0
# MB(0,0): DC-only codes with distinct values so rows/cols differ
mb["non_zero_y"][0] = 0x55555555
co[0, :256:16] = np.arange(16) * 40 - 300
mb["non_zero_y"][1] = 0x55555555
co[1, :256:16] = -(np.arange(16) * 30) + 200
mb["non_zero_y"][2] = 0x55555555
co[2, :256:16] = np.arange(16) * 25 - 100
import sys as _s
mb["imodes"][3] = int(_s.argv[1]) if len(_s.argv) > 1 else 0
Y, U, V = frames.decode_frames(frames.mb_info_tensor(mb), torch.from_numpy(co).cuda(), 0, mbw, mbh, n)
torch.cuda.synchronize()
Y = Y[0].cpu().numpy()
ey, eu, ev = O.decode_frame(mb, co, 0, mbw, mbh)
print("gpu MB11 value", Y[16, 16], "oracle", ey[16, 16])
print("gpu frame row15 cols16-31", Y[15, 16:32].tolist(), "sum", int(Y[15,16:32].sum()))
print("gpu frame col15 rows16-31", Y[16:32, 15].tolist(), "sum", int(Y[16:32,15].sum()))
print("gpu MB00 row15", Y[15, 0:16].tolist(), "sum", int(Y[15,0:16].sum()))
print("gpu MB01 col 15", Y[16:32, 15].tolist())
print("gpu MB10 col 15", Y[0:16, 31].tolist())
for name, s in (("top10+left01", int(Y[15,16:32].sum()) + int(Y[16:32,15].sum())),):
    print(name, (s + 16) >> 5)
print("gpu MB11 row0", Y[16,16:32].tolist()); print("ora MB11 row0", ey[16,16:32].tolist()); print("gpu MB11 col0", Y[16:32,16].tolist())
