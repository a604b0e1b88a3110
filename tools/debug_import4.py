import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import oracle as O
from tools import synth
from webp_amd import frames
for w, h, alpha in ((1, 1, False), (4, 2, True)):
    rgba = synth.noise_rgba(w, h, seed=w + h, alpha=alpha)
    Y, U, V = frames.import_rgba(torch.from_numpy(rgba[None]).cuda(), has_alpha=alpha)
    torch.cuda.synchronize()
    ey, eu, ev = O.import_rgba(rgba, alpha)
    print(w, h, "px", [hex(int.from_bytes(bytes(b), 'little')) for b in rgba.reshape(-1, 4)])
    print(" gpu Y", Y[0, 0, :4].tolist(), "U", U[0, 0, :4].tolist(), "V", V[0, 0, :4].tolist())
    print(" ora Y", ey[0, :4].tolist(), "U", eu[0, :4].tolist(), "V", ev[0, :4].tolist())
    r, g, b = (int(x) for x in rgba[0, 0, :3])
    lin = [O.lib.or_gamma_to_linear(x) for x in (r, g, b)]
    c3 = [O.lib.or_linear_to_gamma(4 * l, 0) for l in lin]
    print(" ora c3", c3, "u", O.lib.or_rgb_to_u(*c3, 1 << 17), "v", O.lib.or_rgb_to_v(*c3, 1 << 17))
