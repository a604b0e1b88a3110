"""VP8L inverse predictor (k_vp8l_inverse) timing by shape: one band (64 rows)
gives the per-step cost, more bands the band-to-band lag.  Random residuals
and random tile modes 0..13 (bits 5); prints ms and us per diagonal step."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from webp_amd import lossless as L  # noqa: E402

REPS = int(os.environ.get("REPS", "10"))
MODES = int(os.environ.get("MODES", "14"))


def timed(fn):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(REPS):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


def main():
    rng = np.random.default_rng(1)
    for w, h in ((4096, 64), (4096, 128), (4096, 512), (4096, 4096)):
        res = L.to_argb_tensor(rng.integers(0, 2 ** 32, (1, h, w), dtype=np.uint32))
        tiles = rng.integers(0, MODES, (1, (h + 31) // 32, (w + 31) // 32), dtype=np.uint32)
        modes = L.to_argb_tensor((tiles << 8) | 0xff000000)
        out = torch.empty_like(res)
        ms = timed(lambda: L.predictor_inverse(modes, 5, res, out=out))
        steps = w + 2 * 63
        print(f"{w}x{h}: {ms:.3f} ms; one band's walk {steps} steps -> {ms * 1e3 / steps:.3f} us/step if alone")


if __name__ == "__main__":
    main()
