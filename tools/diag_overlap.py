"""Diagnostic only (never a bench line): step time with some stages left
out, to see what each side costs when batches overlap.
  python tools/diag_overlap.py  -> one line per variant"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402


def run(skip, slots, steps=12, warmup=3):
    dev = torch.device("cuda", 0)
    rgba, mb, co, _ = bench.make_inputs(64, 0, dev)
    pipe = bench.Pipeline(rgba, mb, co, 64, dev, slots=slots)
    f = pipe.frames
    if "decode" in skip:
        f = type("F", (), {})()
        for k in dir(pipe.frames):
            if not k.startswith("__"):
                setattr(f, k, getattr(pipe.frames, k))
        f.decode_frames = lambda *a, **k: None
        f.build_nrgba = lambda *a, **k: None
    if "encode" in skip:
        f = f if f is not pipe.frames else type("F", (), {k: getattr(pipe.frames, k) for k in dir(pipe.frames)
                                                         if not k.startswith("__")})()
        f.encode_mbs = lambda *a, **k: None
    pipe.frames = f
    el = bench.timed_region(pipe.step, steps, warmup, 1, torch.cuda.synchronize, dev)
    return el / steps * 1e3


if __name__ == "__main__":
    for slots in (1, 3):
        for skip in ((), ("decode",), ("encode",)):
            ms = run(skip, slots)
            print(f"slots={slots} skip={','.join(skip) or '-'} ms/step={ms:.3f}", flush=True)
