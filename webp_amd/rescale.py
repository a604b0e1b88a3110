"""The row rescaler of internal/dsp/rescale.go on the GPU.

The reference exposes a row state machine (``Rescaler``, ``RescalerInit``
:63, ``RescalerImportRow`` :110, ``RescalerExportRow`` :185,
``RescalerHasDstRow`` / ``RescalerNeedsSrcRow`` :260-267) and leaves the
plane loop to its caller.  Here the unit is a batch of whole planes:

  Rescaler(src_w, src_h, dst_w, dst_h)   RescalerInit; builds the size-only
                                          plan once and keeps it on the device
  Rescaler.rescale(planes)                the import/export loop over every row
  rescale_plane(planes, dst_w, dst_h)     one-shot form

Planes are (n, h, w) or (h, w) uint8 CUDA tensors.  Rows the Go driver never
exports (the Go arithmetic is kept as written; see include/webpgpu.h 3d) are
left as zeros; ``Rescaler.rows`` says how many are written.
"""
import ctypes

import torch

from ._lib import call, lib


class Rescaler:
    def __init__(self, src_width, src_height, dst_width, dst_height, device="cuda"):
        if min(src_width, src_height, dst_width, dst_height) <= 0:
            raise ValueError("Rescaler: sizes must be positive")
        self.src_width, self.src_height = src_width, src_height
        self.dst_width, self.dst_height = dst_width, dst_height
        self.plan = torch.empty(lib.wg_rescaler_plan_bytes(dst_width, dst_height), dtype=torch.uint8, device=device)
        rows = ctypes.c_int32(0)
        call("wg_rescaler_plan", src_width, src_height, dst_width, dst_height, self.plan.data_ptr(),
             ctypes.addressof(rows), torch.cuda.current_stream().cuda_stream)
        self.rows = rows.value

    def rescale(self, planes, out=None):
        assert planes.is_cuda and planes.dtype == torch.uint8 and planes.is_contiguous()
        p = planes if planes.dim() == 3 else planes.unsqueeze(0)
        n, h, w = p.shape
        if (w, h) != (self.src_width, self.src_height):
            raise ValueError(f"Rescaler planned for {self.src_width}x{self.src_height}, got {w}x{h}")
        shape = (n, self.dst_height, self.dst_width)
        if out is None:
            out = torch.zeros(shape, dtype=torch.uint8, device=p.device)
        assert out.shape == shape and out.is_contiguous() and out.dtype == torch.uint8
        call("wg_rescale", self.plan.data_ptr(), self.dst_width, self.rows, p.data_ptr(), w, h * w, out.data_ptr(),
             self.dst_width, self.dst_height * self.dst_width, n, torch.cuda.current_stream().cuda_stream)
        return out if planes.dim() == 3 else out[0]


def rescale_plane(planes, dst_width, dst_height):
    h, w = planes.shape[-2:]
    return Rescaler(w, h, dst_width, dst_height, planes.device).rescale(planes)
