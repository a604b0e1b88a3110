"""Runs the 64 x 1080p decode batch a few times (for rocprofv3 counter passes)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tools import synth  # noqa: E402
from webp_amd import _lib, frames  # noqa: E402

MBW, MBH, B = 120, 68, int(os.environ.get("BATCH", "64"))
FT, P_I4 = int(os.environ.get("FT", "2")), float(os.environ.get("P_I4", "0.5"))
dev = torch.device("cuda")
mb, co = synth.random_macroblocks(MBW * MBH * 4, seed=11, levels=(20, 32), p_i4=P_I4)
mbs = frames.mb_info_tensor(mb).view(4, -1, 32).repeat(B // 4, 1, 1).reshape(-1, 32).contiguous()
cos = torch.from_numpy(co).to(dev).view(4, -1, 384).repeat(B // 4, 1, 1).reshape(-1, 384).contiguous()
work = torch.empty(_lib.lib.wg_decode_work_bytes(MBW, MBH, B), dtype=torch.uint8, device=dev)
out = (torch.empty((B, 16 * MBH, 16 * MBW), dtype=torch.uint8, device=dev),
       torch.empty((B, 8 * MBH, 8 * MBW), dtype=torch.uint8, device=dev),
       torch.empty((B, 8 * MBH, 8 * MBW), dtype=torch.uint8, device=dev))
for _ in range(int(os.environ.get("REPS", "3"))):
    frames.decode_frames(mbs, cos, FT, MBW, MBH, B, out=out, work=work)
torch.cuda.synchronize()
print("ok")
