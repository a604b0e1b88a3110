"""Multi-GPU data path of the DSP hot path.

One process per GPU (torch.distributed: RCCL over xGMI on the GPU box, gloo
in the CPU tests).  Nothing on the compute path is collective; the only
exchange is the final gather of outputs to the rank that owns the result
(rank 0), as grouped point-to-point send/recv (``batch_isend_irecv``, which
the NCCL/RCCL backend issues inside one ncclGroupStart/End), never a
reduction.

Independent frames (C4): frame i belongs to rank i % world
(``frames_of``); each rank runs the whole device path on its frames and
``gather_frames`` hands rank 0 every frame's outputs in global order -- the
reference's per-image outputs (wg_mb_enc records, reconstruction, NRGBA).

One large plane, streaming stages (C5): tile rows are split into contiguous
bands (``band_of``).  A rank computes its band from its rows plus a halo
(``*_rows`` entry points of libwebpgpu: the VP8L residual reads one row
above the band, the plane SSIM three rows each side) and rank 0 assembles the
bands: residual rows and tile modes for ResidualImage, the per-tile SSIM
partial sums (reduced on rank 0 in the single-GPU order, so the sharded sum
is bit-identical).  The dependency stages (decoder reconstruct, encoder RD,
SharpYUV, VP8L inverse) do not shard inside one image; across images they
shard like C4.

Every helper takes a ``compute`` callable so the same sharding and gather
logic runs with the GPU kernels (default) or with CPU stand-ins in the gloo
tests (tests/test_shard.py)."""
import time

import numpy as np
import torch
import torch.distributed as dist


def frames_of(n, world, rank):
    """Global indices of the frames rank `rank` owns (round robin)."""
    return list(range(rank, n, world))


def band_of(tiles, world, rank):
    """Contiguous tile-row band [begin, end) of rank `rank` (the first
    tiles % world ranks take one extra row)."""
    base, rem = divmod(tiles, world)
    begin = rank * base + min(rank, rem)
    return begin, begin + base + (1 if rank < rem else 0)


def gather_to_root(local, world, rank, specs):
    """Send this rank's tensors to rank 0.  specs(r) -> [(shape, dtype)] of
    what rank r sends (known from the partition, so no size exchange).
    Returns, on rank 0, a list over ranks of lists of tensors (rank 0's own
    entry is `local`); None elsewhere."""
    if world == 1:
        return [list(local)]
    ops, recv = [], None
    if rank == 0:
        dev = local[0].device if local else torch.device("cpu")
        recv = [list(local)] + [[torch.empty(s, dtype=d, device=dev) for s, d in specs(r)] for r in range(1, world)]
        for r in range(1, world):
            ops += [dist.P2POp(dist.irecv, t, r) for t in recv[r] if t.numel()]
    else:
        ops = [dist.P2POp(dist.isend, t.contiguous(), 0) for t in local if t.numel()]
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    return recv


def gather_frames(outputs, n, world, rank):
    """outputs: tensors whose leading dim is this rank's frames (frames_of
    order).  Rank 0 gets the tensors with all n frames in global order."""
    mine = frames_of(n, world, rank)
    assert all(t.shape[0] == len(mine) for t in outputs)

    def specs(r):
        k = len(frames_of(n, world, r))
        return [((k,) + tuple(t.shape[1:]), t.dtype) for t in outputs]

    parts = gather_to_root(outputs, world, rank, specs)
    if parts is None:
        return None
    full = []
    for j, t in enumerate(outputs):
        out = torch.empty((n,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        for r in range(world):
            idx = frames_of(n, world, r)
            if idx:
                out[idx[0]::world] = parts[r][j].to(t.device)
        full.append(out)
    return full


def encode_frames_sharded(rgba_of, n, world, rank, compute=None):
    """C4: rank-local encode of this rank's frames, then the gather.
    rgba_of(indices) -> (k, h, w, 4) uint8 tensor of those frames (each rank
    reads / decodes only its own).  compute(rgba) -> list of per-frame output
    tensors (default: the device encode path, frames.encode_frames: wg_mb_enc
    bytes, reconstructed Y, U, V)."""
    if compute is None:
        compute = _device_encode
    outs = compute(rgba_of(frames_of(n, world, rank)))
    return gather_frames(outs, n, world, rank)


def _device_encode(rgba):
    from . import frames
    n = rgba.shape[0]
    out, (ry, ru, rv), _, _, _ = frames.encode_frames(rgba)
    return [out.view(n, -1), ry, ru, rv]


# ---------------- one large plane, row bands ----------------

def residual_image_sharded(argb, bits, quality, world, rank, compute=None):
    """C5 VP8L ResidualImage of one (h, w) ARGB image by tile-row bands.
    argb must hold at least this rank's band rows and the row above it.
    compute(argb, bits, quality, ty0, ty1) -> (modes (ty1-ty0, tx), residual
    rows (rows, w)) (default: wg_vp8l_residual_image_rows).  Rank 0 gets
    (modes (ty, tx), residuals (h, w)), identical to the one-GPU result."""
    h, w = argb.shape[-2:]
    ts = 1 << bits
    ty = (h + ts - 1) >> bits
    tx = (w + ts - 1) >> bits
    t0, t1 = band_of(ty, world, rank)
    compute = compute or _device_residual_rows
    if t1 > t0:
        modes, res = compute(argb, bits, quality, t0, t1)
    else:
        modes = argb.new_empty((0, tx))
        res = argb.new_empty((0, w))

    def rows(r):
        b0, b1 = band_of(ty, world, r)
        return max(0, min(b1 * ts, h) - b0 * ts)

    def specs(r):
        b0, b1 = band_of(ty, world, r)
        return [((b1 - b0, tx), argb.dtype), ((rows(r), w), argb.dtype)]

    parts = gather_to_root([modes, res], world, rank, specs)
    if parts is None:
        return None
    return torch.cat([p[0] for p in parts]), torch.cat([p[1] for p in parts])


def _device_residual_rows(argb, bits, quality, t0, t1):
    from ._lib import call
    from .lossless import _stream
    a = argb.contiguous()
    h, w = a.shape[-2:]
    tx = (w + (1 << bits) - 1) >> bits
    ty = (h + (1 << bits) - 1) >> bits
    modes = torch.empty((ty, tx), dtype=torch.int32, device=a.device)
    res = torch.empty((h, w), dtype=torch.int32, device=a.device)
    call("wg_vp8l_residual_image_rows", a.data_ptr(), w, h, h * w, bits, quality, t0, t1, 1, modes.data_ptr(),
         res.data_ptr(), _stream())
    return modes[t0:t1], res[t0 << bits:min(t1 << bits, h)]


SSIM_TILE = 16   # rows per tile row of wg_plane_ssim_rows
SSIM_STRIP = 58  # columns per partial sum (wg_plane_ssim_row_partials)


def ssim_row_partials(w):
    return (w + SSIM_STRIP - 1) // SSIM_STRIP


def plane_ssim_sharded(a, b, world, rank, compute=None, reduce=None):
    """C5 plane SSIM of one (h, w) pair by 16-row tile bands: each rank
    computes the per-tile partial sums of its band (it needs its rows plus 3
    halo rows each side), rank 0 gathers them in tile order and reduces them
    in the single-GPU order.  Rank 0 gets the float64 sum."""
    h, w = a.shape[-2:]
    ty = (h + SSIM_TILE - 1) // SSIM_TILE
    tx = ssim_row_partials(w)
    t0, t1 = band_of(ty, world, rank)
    compute = compute or _device_ssim_rows
    reduce = reduce or _device_ssim_reduce
    part = compute(a, b, t0, t1) if t1 > t0 else torch.empty(0, dtype=torch.float64, device=a.device)
    parts = gather_to_root([part], world, rank,
                           lambda r: [((tx * (band_of(ty, world, r)[1] - band_of(ty, world, r)[0]),), torch.float64)])
    if parts is None:
        return None
    return reduce(torch.cat([p[0] for p in parts]))


def _device_ssim_rows(a, b, t0, t1):
    from ._lib import call
    from .frames import _stream
    h, w = a.shape[-2:]
    tx = ssim_row_partials(w)
    out = torch.empty(tx * (t1 - t0), dtype=torch.float64, device=a.device)
    call("wg_plane_ssim_rows", a.data_ptr(), a.shape[-1], a.numel(), b.data_ptr(), b.shape[-1], b.numel(), w, h, t0, t1,
         1, out.data_ptr(), _stream())
    return out


def _device_ssim_reduce(partials):
    from ._lib import call
    from .frames import _stream
    out = torch.empty(1, dtype=torch.float64, device=partials.device)
    call("wg_plane_ssim_reduce", partials.data_ptr(), partials.numel(), 1, out.data_ptr(), _stream())
    return float(out.item())


# ---------------- bench helper ----------------

def timed_gather_to_root(tensors, world, rank, device, keep=False):
    """Gather every rank's batch outputs (same shapes on every rank) to rank 0,
    bracketed by barriers and device syncs; returns the timing record rank 0
    reports (bytes all ranks sent, wall time, aggregate GB/s into rank 0), and
    with keep=True also what rank 0 received (None on the other ranks)."""
    sync = torch.cuda.synchronize if device.type == "cuda" else (lambda: None)
    sync()
    dist.barrier()
    t0 = time.perf_counter()
    parts = gather_to_root(tensors, world, rank, lambda r: [(tuple(t.shape), t.dtype) for t in tensors])
    sync()
    dist.barrier()
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    per_rank = int(sum(x.numel() * x.element_size() for x in tensors))
    moved = per_rank * (world - 1)
    rec = {"what": "per-rank wg_mb_enc records + reconstruction + NRGBA of the last batch -> rank 0",
           "collective": "grouped send/recv (batch_isend_irecv)", "bytes_per_rank": per_rank,
           "bytes_to_root": moved, "ms": round(el * 1e3, 3), "GB/s_into_root": round(moved / max(el, 1e-9) / 1e9, 2)}
    if keep:
        return rec, parts
    del parts
    return rec


def assemble_frames_numpy(parts, n, world):
    """Host-side mirror of gather_frames' interleave (tests / tools)."""
    out = [None] * n
    for r in range(world):
        for j, i in enumerate(frames_of(n, world, r)):
            out[i] = parts[r][j]
    return np.stack(out)
