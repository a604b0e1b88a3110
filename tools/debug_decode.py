"""Debug helper: GPU vs oracle decode for the exact data of a test case."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import oracle as O
from tools import synth
from webp_amd import frames

mbw, mbh, n, ft, seed = (int(x) for x in sys.argv[1:6])
mb, co = synth.random_macroblocks(n * mbw * mbh, seed=seed, levels=(0, 10, 20, 40, 63))
Y, U, V = frames.decode_frames(frames.mb_info_tensor(mb), torch.from_numpy(co).cuda(), ft, mbw, mbh, n)
torch.cuda.synchronize()
Y, U, V = Y.cpu().numpy(), U.cpu().numpy(), V.cpu().numpy()
per = mbw * mbh
for i in range(n):
    ey, eu, ev = O.decode_frame(mb[i * per:(i + 1) * per], co[i * per:(i + 1) * per], ft, mbw, mbh)
    for name, a, b, s in (("Y", Y[i], ey, 16), ("U", U[i], eu, 8), ("V", V[i], ev, 8)):
        bad = np.argwhere(a != b)
        print("img", i, name, "mismatches", len(bad))
        if len(bad):
            r, c = bad[0]
            my, mx = r // s, c // s
            print(" first at", r, c, "MB", mx, my, "info", mb[i * per + my * mbw + mx])
            print(" gpu\n", a[my*s:(my+1)*s, mx*s:(mx+1)*s])
            print(" oracle\n", b[my*s:(my+1)*s, mx*s:(mx+1)*s])
            if my:
                print(" gpu top row", a[my*s-1, max(0, mx*s-1):(mx+1)*s])
                print(" ora top row", b[my*s-1, max(0, mx*s-1):(mx+1)*s])
# independent DC check for MB(1,1) of each image from the GPU frame (valid for filter 0)
for i in range(n):
    ey, eu, ev = O.decode_frame(mb[i * per:(i + 1) * per], co[i * per:(i + 1) * per], ft, mbw, mbh)
    for src, F in (("gpu", Y[i]), ("ora", ey)):
        top = int(F[15, 16:32].sum()); left = int(F[16:32, 15].sum())
        print(src, "img", i, "topsum", top, "leftsum", left, "dc", (top + left + 16) >> 5, "pix00", F[16, 16])
    print("left col gpu", Y[i][16:32, 15].tolist())
    print("left col ora", ey[16:32, 15].tolist())
