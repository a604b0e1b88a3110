"""CPU, gloo: the multi-GPU data path of webp_amd/shard.py
with world sizes 2 and 3.  The sharding and the gather to rank 0 are the
product code; the per-rank compute is an oracle stand-in (the GPU kernels
need a device), and every sharded result is byte-compared with a one-rank run
of the same stand-in:

  - C4 independent frames: Phase A of small frames (wg_mb_enc records + the
    reconstruction) per rank, gathered to rank 0 in global frame order;
  - C5 one plane: VP8L ResidualImage by tile-row bands (modes + residual rows)
    and the plane SSIM by 16-row bands (per-tile partial sums, reduced on
    rank 0).

tests/test_gpu_shard.py checks on the GPU that the band kernels reproduce the
whole-image results for any partition."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle as O
from tools import synth
from webp_amd import shard

W, H, N = 64, 64, 5


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_partitions():
    for n in (1, 5, 64, 512):
        for world in (1, 2, 3, 8):
            got = sorted(i for r in range(world) for i in shard.frames_of(n, world, r))
            assert got == list(range(n))
    for tiles in (1, 7, 128, 256):
        for world in (1, 2, 3, 8):
            bands = [shard.band_of(tiles, world, r) for r in range(world)]
            assert bands[0][0] == 0 and bands[-1][1] == tiles
            assert all(bands[r][1] == bands[r + 1][0] for r in range(world - 1))
            sizes = [b - a for a, b in bands]
            assert max(sizes) - min(sizes) <= 1


def frame_rgba(i):
    return [synth.gradient_rgba, lambda w, h: synth.noise_rgba(w, h, seed=i), lambda w, h: synth.blobs_rgba(w, h, seed=i)][i % 3](W, H)


def oracle_encode(rgba):
    """Stand-in for frames.encode_frames on one rank: per frame the wg_mb_enc
    bytes and the reconstructed planes."""
    recs, ys, us, vs = [], [], [], []
    for img in rgba.numpy():
        y, u, v = O.import_rgba(img, has_alpha=False)
        enc, (ry, ru, rv), _, _ = O.encode_frame(y, u, v, W, H)
        recs.append(enc.view(np.uint8).reshape(-1))
        ys.append(ry)
        us.append(ru)
        vs.append(rv)
    return [torch.from_numpy(np.stack(a)) for a in (recs, ys, us, vs)]


def rgba_of(idx):
    return torch.from_numpy(np.stack([frame_rgba(i) for i in idx]))


def argb_image():
    rgba = synth.blobs_rgba(70, 83, seed=3)
    rgba[::7, ::5] = synth.noise_rgba(70, 83, seed=4)[::7, ::5]
    a = rgba.astype(np.uint32)
    return (a[..., 3] << 24 | a[..., 0] << 16 | a[..., 1] << 8 | a[..., 2]).astype(np.uint32)


def oracle_residual_rows(argb, bits, quality, t0, t1):
    """Stand-in for wg_vp8l_residual_image_rows: the whole-image restatement,
    cut to the band."""
    modes, res = O.vp8l_residual_image(argb.numpy().view(np.uint32), bits, quality)
    h = argb.shape[0]
    return (torch.from_numpy(modes.view(np.int32)[t0:t1].copy()),
            torch.from_numpy(res.view(np.int32)[t0 << bits:min(t1 << bits, h)].copy()))


def ssim_tile_partials(a, b, t0, t1):
    """Stand-in for wg_plane_ssim_rows: per 16-row x 58-column tile the sum
    of the clipped-window SSIM (SSIMGetClipped, ssim.go:132) of its pixels."""
    a, b = a.numpy(), b.numpy()
    h, w = a.shape
    sw = shard.SSIM_STRIP
    out = []
    for ty in range(t0, t1):
        for tx in range(shard.ssim_row_partials(w)):
            s = 0.0
            for y in range(ty * 16, min(ty * 16 + 16, h)):
                for x in range(tx * sw, min(tx * sw + sw, w)):
                    s += O.lib.or_ssim_get_clipped(O.u8(a), w, O.u8(b), w, x, y, w, h)
            out.append(s)
    return torch.tensor(out, dtype=torch.float64)


def ssim_reduce(p):
    return float(p.numpy().sum())


def _run(world, rank):
    res = {}
    res["frames"] = shard.encode_frames_sharded(rgba_of, N, world, rank, compute=oracle_encode)
    argb = torch.from_numpy(argb_image().view(np.int32))
    res["resid"] = shard.residual_image_sharded(argb, 3, 75, world, rank, compute=oracle_residual_rows)
    rng = np.random.default_rng(9)
    pa = torch.from_numpy(rng.integers(0, 256, (37, 45), dtype=np.uint8))
    pb = torch.from_numpy(np.clip(pa.numpy().astype(int) + rng.integers(-9, 10, (37, 45)), 0, 255).astype(np.uint8))
    res["ssim"] = shard.plane_ssim_sharded(pa, pb, world, rank, compute=ssim_tile_partials, reduce=ssim_reduce)
    return res


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = _run(world, rank)
        if rank == 0:
            out["frames"] = [t.numpy() for t in res["frames"]]
            out["resid"] = [t.numpy() for t in res["resid"]]
            out["ssim"] = res["ssim"]
        else:
            out[f"none{rank}"] = res["frames"] is None and res["resid"] is None and res["ssim"] is None
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def single():
    res = _run(1, 0)
    return {"frames": [t.numpy() for t in res["frames"]], "resid": [t.numpy() for t in res["resid"]],
            "ssim": res["ssim"]}


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [2, 3])
def test_sharded_equals_one_rank(world, single):
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
        res = dict(out)
    for r in range(1, world):
        assert res[f"none{r}"]  # only rank 0 receives
    for a, b in zip(res["frames"], single["frames"]):
        assert a.shape == b.shape and a.tobytes() == b.tobytes()
    for a, b in zip(res["resid"], single["resid"]):
        assert a.shape == b.shape and a.tobytes() == b.tobytes()
    assert res["ssim"] == single["ssim"]


def test_one_rank_matches_direct(single):
    """The one-rank run itself is the plain restatement (frames in order)."""
    f0 = oracle_encode(rgba_of(range(N)))
    for a, b in zip(single["frames"], f0):
        assert a.tobytes() == b.numpy().tobytes()
    modes, res = O.vp8l_residual_image(argb_image(), 3, 75)
    assert single["resid"][0].view(np.uint32).tobytes() == modes.tobytes()
    assert single["resid"][1].view(np.uint32).tobytes() == res.tobytes()
