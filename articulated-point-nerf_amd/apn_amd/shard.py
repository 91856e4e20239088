"""Ray-sharded rendering of one frame over the GPUs of a node.

Every rank replicates the cheap per-frame work (skeleton, LBS, kNN grid, the per-ray in-bbox
sample counts) and renders one contiguous ray range holding ~1/world of the frame's in-bbox
samples; the per-ray outputs are then exchanged with one all-gather (RCCL over xGMI on the GPU
box, gloo in the CPU tests). Rays are independent given the warped cloud, so the assembled
frame is bit-identical to a single-GPU render (chunk invariance, tests/test_hip_parity.py).

Tile layout: [rays, 12] float32 = rgb_marched (3), rgb_marched_direct (3), depth (1),
weights (3), alphainv_last (1), alphainv_last_direct (1).
"""
from __future__ import annotations

import torch

TILE_KEYS = (("rgb_marched", 3), ("rgb_marched_direct", 3), ("depth", 1), ("weights", 3),
             ("alphainv_last", 1), ("alphainv_last_direct", 1))
TILE_WIDTH = sum(w for _, w in TILE_KEYS)


def balanced_ray_split(offsets: torch.Tensor, world: int) -> list[int]:
    """Ray boundaries b[0]=0 <= ... <= b[world]=R such that rank k's rays [b[k], b[k+1]) hold
    ~total/world in-bbox samples. ``offsets`` is the exclusive prefix sum of per-ray sample
    counts ([R+1], offsets[R] = total), on any device; one small device->host copy."""
    R = offsets.numel() - 1
    total = offsets[R:R + 1].to(torch.int64)
    k = torch.arange(1, world, device=offsets.device, dtype=torch.int64)
    targets = (total * k + world // 2) // world
    inner = torch.searchsorted(offsets[:R + 1].to(torch.int64).contiguous(), targets.contiguous())
    b = [0] + [min(max(int(x), 0), R) for x in inner.cpu().tolist()] + [R]
    for i in range(1, len(b)):  # monotone even for degenerate inputs
        b[i] = max(b[i], b[i - 1])
    return b


def pack_tile(out: dict, n_rays: int, device) -> torch.Tensor:
    """Per-ray outputs of TemporalPoints.forward -> [n_rays, 12] float32."""
    cols = []
    get = getattr(out, "raw", out.get)   # RenderOutput.raw: the kernels' values, no survivor-count sync
    for key, w in TILE_KEYS:
        v = get(key)
        if v is None:
            v = torch.ones(n_rays, w, device=device)  # NoPoints fallback has no alphainv
        cols.append(v.reshape(n_rays, w).float())
    return torch.cat(cols, dim=1).contiguous()


def unpack_tile(tile: torch.Tensor) -> dict:
    out, c = {}, 0
    for key, w in TILE_KEYS:
        v = tile[:, c:c + w]
        out[key] = v.reshape(-1) if w == 1 else v
        c += w
    return out


def gather_tiles(tile: torch.Tensor, bounds: list[int], group=None) -> torch.Tensor:
    """All-gather variable-length ray tiles (padded to the longest range) and concatenate
    them in ray order -> [R, TILE_WIDTH] on every rank."""
    import torch.distributed as dist
    world = len(bounds) - 1
    lens = [bounds[i + 1] - bounds[i] for i in range(world)]
    m = max(max(lens), 1)
    padded = torch.zeros(m, tile.shape[1], device=tile.device, dtype=tile.dtype)
    padded[:tile.shape[0]] = tile
    full = torch.empty(world * m, tile.shape[1], device=tile.device, dtype=tile.dtype)
    if dist.get_backend(group) == "gloo":
        dist.all_gather(list(full.view(world, m, -1).unbind(0)), padded, group=group)
    else:
        dist.all_gather_into_tensor(full, padded, group=group)
    return torch.cat([full[i * m:i * m + lens[i]] for i in range(world)], dim=0)


@torch.no_grad()
def render_sharded(model, t, render_kwargs, rank: int, world: int, group=None, **forward_kwargs) -> dict:
    """One frame rendered by ``world`` ranks: this rank's ray range through
    TemporalPoints.forward(ray_shard=(rank, world)), then the tile all-gather. Returns the
    reference output keys for all rays on every rank."""
    out = model(t, render_kwargs=render_kwargs, ray_shard=(rank, world), render_depth=True,
                render_weights=True, **forward_kwargs)
    r0, r1 = model.last_ray_range
    tile = pack_tile(out, r1 - r0, render_kwargs["rays_o"].device)
    full = gather_tiles(tile, model.last_ray_bounds, group) if world > 1 else tile
    res = unpack_tile(full)
    for k in ("t_hat_pcd", "joints", "bones"):
        res[k] = out.get(k)
    return res
