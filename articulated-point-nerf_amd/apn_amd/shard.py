"""Ray-sharded rendering of one frame over the GPUs of a node.

Every rank replicates the cheap per-frame work (skeleton, LBS, kNN grid) and renders its share
of the rays -- by default the interleaved 4096-ray blocks k, k + world, ... (the "blocks" split
below) -- and the per-ray outputs are then exchanged with one all-gather (RCCL over xGMI on the
GPU box, gloo in the CPU tests). Rays are independent given the warped cloud, so the assembled
frame is bit-identical to a single-GPU render (chunk invariance, tests/test_hip_parity.py).

Tile layout: [rays, 12] float32 = rgb_marched (3), rgb_marched_direct (3), depth (1),
weights (3), alphainv_last (1), alphainv_last_direct (1); render_sharded appends one column, the
ray's kNN survivor count, for the next frame's split.

Two splits (``render_sharded(split=...)``, default ``DEFAULT_SPLIT``, env APN_SHARD_SPLIT):

* ``"blocks"`` (default): fixed blocks of RAY_BLOCK consecutive rays dealt round-robin, rank k
  taking blocks k, k + world, ... Every rank holds the same number of rays (to one block), so the
  all-gather is unpadded, and the image-space interleave balances the work statistically from
  the first frame: at C2 with 8 ranks the slowest shard is 1.02x the mean (2.14 ms, bound 5.12x
  of the 10.98 ms frame) against 1.12x (2.27 ms) for the cost-balanced ranges below, whose
  unequal ray counts also pad the gather to the longest range (tools/shard_balance.py --split).
* ``"ranges"``: one contiguous ray range per rank. A shard's time follows its kNN survivors (the
  MLP's rows) far more than its in-bbox samples -- at C2 with 8 ranks, equal in-bbox shards held
  0.13M to 0.60M survivors and took 1.5 to 3.5 ms. The first frame splits the in-bbox samples;
  every later frame splits the previous frame's per-ray cost KEPT_WEIGHT * survivors + in-bbox
  samples (the survivor counts ride in the tile all-gather, so every rank computes the same split).
"""
from __future__ import annotations

import os

import torch

TILE_KEYS = (("rgb_marched", 3), ("rgb_marched_direct", 3), ("depth", 1), ("weights", 3),
             ("alphainv_last", 1), ("alphainv_last_direct", 1))
TILE_WIDTH = sum(w for _, w in TILE_KEYS)
KEPT_WEIGHT = 10   # cost of a survivor (neighbour MLP + its kNN) in in-bbox-sample units: ~4.5 vs ~0.45 ns at C2
RAY_BLOCK = 4096   # rays per block of the "blocks" split (~5 image rows at 800 wide; 64 and 800 measured slower)
DEFAULT_SPLIT = os.environ.get("APN_SHARD_SPLIT", "blocks")


def block_rays(R: int, rank: int, world: int, block: int = RAY_BLOCK) -> torch.Tensor:
    """Ray indices (int64, ascending, CPU) of rank's blocks k, k + world, ... of ``block`` rays
    (the last block of the frame may be short)."""
    if rank * block >= R:
        return torch.zeros(0, dtype=torch.int64)
    starts = torch.arange(rank * block, R, world * block, dtype=torch.int64)
    idx = (starts[:, None] + torch.arange(block, dtype=torch.int64)[None]).reshape(-1)
    return idx[idx < R]


def block_slots(R: int, world: int, block: int = RAY_BLOCK) -> int:
    """Block slots per rank: ceil(ceil(R / block) / world)."""
    return -(-(-(-R // block)) // world)


def assemble_blocks(parts: torch.Tensor, R: int, world: int, block: int = RAY_BLOCK) -> torch.Tensor:
    """[world, slots * block, w] per-rank tiles (rank k's blocks in order, zero-padded) -> the
    frame's [R, w] in ray order: block j is slot j // world of rank j % world."""
    per = block_slots(R, world, block)
    w = parts.shape[-1]
    return parts[:, :per * block].reshape(world, per, block, w).transpose(0, 1).reshape(per * world * block, w)[:R]


def gather_blocks(tile: torch.Tensor, R: int, world: int, block: int = RAY_BLOCK, group=None,
                  info: torch.Tensor | None = None):
    """All-gather of the "blocks" split: every rank's tile is padded to the same slots * block rows
    (at most one block of padding), plus one row carrying its frame_info [4] when given ->
    ([R, w] in ray order, infos [world, 4] int32 or None)."""
    import torch.distributed as dist
    m = block_slots(R, world, block) * block
    rows = m + (1 if info is not None else 0)
    assert tile.shape[0] <= m, (tile.shape, m)
    padded = torch.zeros(rows, tile.shape[1], device=tile.device, dtype=tile.dtype)
    padded[:tile.shape[0]] = tile
    if info is not None:
        padded[m, :4] = info.to(torch.int32).view(torch.float32)
    full = torch.empty(world * rows, tile.shape[1], device=tile.device, dtype=tile.dtype)
    if dist.get_backend(group) == "gloo":
        dist.all_gather(list(full.view(world, rows, -1).unbind(0)), padded, group=group)
    else:
        dist.all_gather_into_tensor(full, padded, group=group)
    parts = full.view(world, rows, -1)
    tiles = assemble_blocks(parts[:, :m], R, world, block)
    if info is None:
        return tiles, None
    return tiles, parts[:, m, :4].contiguous().view(torch.int32)


def cost_offsets(offsets: torch.Tensor, kept: torch.Tensor) -> torch.Tensor:
    """Exclusive prefix [R+1] (int64) of the per-ray cost KEPT_WEIGHT * kept + in-bbox samples."""
    R = offsets.numel() - 1
    o = offsets[:R + 1].to(torch.int64)
    cost = (o[1:] - o[:-1]) + KEPT_WEIGHT * kept.reshape(-1).to(torch.int64)
    return torch.cat([o.new_zeros(1), torch.cumsum(cost, 0)])


def split_inner(offsets: torch.Tensor, world: int) -> torch.Tensor:
    """The world - 1 inner ray boundaries of the balanced split, on the offsets' device (no host
    read): rank k's rays [b[k], b[k+1]) hold ~total/world in-bbox samples."""
    R = offsets.numel() - 1
    total = offsets[R:R + 1].to(torch.int64)
    k = torch.arange(1, world, device=offsets.device, dtype=torch.int64)
    targets = (total * k + world // 2) // world
    return torch.searchsorted(offsets[:R + 1].to(torch.int64).contiguous(), targets.contiguous())


def bounds_from_inner(inner, R: int) -> list[int]:
    """[0, *inner, R] clamped to [0, R] and made monotone (degenerate inputs)."""
    b = [0] + [min(max(int(x), 0), R) for x in inner] + [R]
    for i in range(1, len(b)):
        b[i] = max(b[i], b[i - 1])
    return b


def balanced_ray_split(offsets: torch.Tensor, world: int) -> list[int]:
    """Ray boundaries b[0]=0 <= ... <= b[world]=R such that rank k's rays [b[k], b[k+1]) hold
    ~total/world in-bbox samples. ``offsets`` is the exclusive prefix sum of per-ray sample
    counts ([R+1], offsets[R] = total), on any device; one small device->host copy."""
    return bounds_from_inner(split_inner(offsets, world).cpu().tolist(), offsets.numel() - 1)


class SplitTracker:
    """Sync-free ray split for consecutive sharded frames of one (ray count, world): the first
    frame reads its balanced split on the host; every frame then computes a split on the device
    (of its in-bbox counts, or -- after submit_cost -- of its per-ray cost) and copies it to pinned
    host memory without waiting. A frame uses the split computed two frames before it (kept in a
    queue of pending copies): by then the device has finished that copy even when the host runs a
    whole frame ahead, so the wait costs neither host nor device time (waiting on the previous
    frame's copy would hold the host until the device drains, and the device would then idle
    while the next frame's first launches are issued). Stale splits only move the balance, never
    the result: any contiguous split assembles the same frame. Every rank makes the same calls, so
    every rank switches at the same frame, and identical inputs give identical splits."""

    DEPTH = 2

    def __init__(self):
        self.bounds = None
        self._pending = []   # [(pinned host split, event)] oldest first
        self._free = []      # pinned buffers to reuse
        self.cost_mode = False   # set by the first submit_cost: later splits follow the survivors

    def bounds_for(self, offsets: torch.Tensor, world: int, advance: bool = True) -> list[int]:
        """advance=False (a frame rendered again after an overflow) keeps the current split, so the
        re-rendered range is the one the frame was gathered with."""
        R = offsets.numel() - 1
        if self.bounds is None:
            self.bounds = balanced_ray_split(offsets, world)
        elif not advance:
            return self.bounds
        elif len(self._pending) >= self.DEPTH:
            host, ev = self._pending.pop(0)
            ev.synchronize()
            self.bounds = bounds_from_inner(host.tolist(), R)
            self._free.append(host)
        if world > 1 and offsets.is_cuda and not self.cost_mode:
            self._launch(offsets, world)
        return self.bounds

    def _launch(self, prefix: torch.Tensor, world: int):
        host = self._free.pop() if self._free else torch.empty(world - 1, dtype=torch.int64, pin_memory=True)
        host.copy_(split_inner(prefix, world), non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._pending.append((host, ev))

    def submit_cost(self, offsets: torch.Tensor, kept: torch.Tensor, world: int):
        """After a frame's all-gather: a split from this frame's per-ray cost (``offsets`` = the
        frame's in-bbox prefix over all rays, ``kept`` = survivors per ray), computed and copied to
        the host without waiting; from the first call on, frames queue these instead of in-bbox
        splits."""
        if world > 1 and offsets.is_cuda:
            if not self.cost_mode:
                self._pending.clear()   # in-bbox splits still queued: superseded
            self._launch(cost_offsets(offsets, kept), world)
            self.cost_mode = True


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


def gather_tiles(tile: torch.Tensor, bounds: list[int], group=None, info: torch.Tensor | None = None):
    """All-gather variable-length ray tiles (padded to the longest range) and concatenate
    them in ray order -> [R, TILE_WIDTH] on every rank. With ``info`` (this rank's int32 frame_info
    [4], see apn_inbbox_fill_capped) one more row per rank carries it through the same
    collective: returns (tiles, infos [world, 4] int32)."""
    import torch.distributed as dist
    world = len(bounds) - 1
    lens = [bounds[i + 1] - bounds[i] for i in range(world)]
    m = max(max(lens), 1)
    rows = m + (1 if info is not None else 0)
    padded = torch.zeros(rows, tile.shape[1], device=tile.device, dtype=tile.dtype)
    padded[:tile.shape[0]] = tile
    if info is not None:
        padded[m, :4] = info.to(torch.int32).view(torch.float32)
    full = torch.empty(world * rows, tile.shape[1], device=tile.device, dtype=tile.dtype)
    if dist.get_backend(group) == "gloo":
        dist.all_gather(list(full.view(world, rows, -1).unbind(0)), padded, group=group)
    else:
        dist.all_gather_into_tensor(full, padded, group=group)
    tiles = torch.cat([full[i * rows:i * rows + lens[i]] for i in range(world)], dim=0)
    if info is None:
        return tiles
    return tiles, full.view(world, rows, -1)[:, m, :4].contiguous().view(torch.int32)


class ShardedFrame(dict):
    """The assembled frame of render_sharded. Ranks on the sync-free path may have dropped samples
    past their capacity; every rank's frame_info rode along in the all-gather, and the first read
    of any key checks them (one device read): if a rank overflowed, the frame is rendered again
    on this rank alone, exactly (no collective, so it is safe whichever ranks read the frame)."""

    def __init__(self, *a, infos=None, rerender=None, on_infos=None, **kw):
        super().__init__(*a, **kw)
        self._infos = infos
        self._rerender = rerender
        self._on_infos = on_infos

    def _resolve(self):
        if self._infos is None:
            return
        infos, self._infos = self._infos, None
        if self._on_infos is not None:
            self._on_infos(infos)
        if bool((infos[:, 2] != 0).any()):
            fresh = self._rerender(infos)
            dict.update(self, fresh)

    def __getitem__(self, k):
        self._resolve()
        return super().__getitem__(k)

    def get(self, k, default=None):
        self._resolve()
        return super().get(k, default)

    def keys(self):
        self._resolve()
        return super().keys()

    def items(self):
        self._resolve()
        return super().items()

    def __contains__(self, k):
        self._resolve()
        return super().__contains__(k)

    # every other read of the dict validates too (dict(frame) / {**frame} take the slow path
    # through keys() + __getitem__ because __iter__ is overridden)
    def values(self):
        self._resolve()
        return super().values()

    def __iter__(self):
        self._resolve()
        return super().__iter__()

    def __len__(self):
        self._resolve()
        return super().__len__()

    def pop(self, k, *default):
        self._resolve()
        return super().pop(k, *default)

    def copy(self):
        self._resolve()
        return dict(super().items())

    def raw(self, k, default=None):
        return super().get(k, default)


@torch.no_grad()
def render_sharded(model, t, render_kwargs, rank: int, world: int, group=None, split: str | None = None,
                   block: int = RAY_BLOCK, **forward_kwargs) -> dict:
    """One frame rendered by ``world`` ranks: this rank's rays through
    TemporalPoints.forward(ray_shard=(rank, world, block)) ("blocks" split) or
    forward(ray_shard=(rank, world)) ("ranges"), then the tile all-gather. Returns the reference
    output keys for all rays on every rank (a ShardedFrame, validated on first read)."""
    split = split or DEFAULT_SPLIT
    if split not in ("blocks", "ranges"):
        raise ValueError(f"split must be 'blocks' or 'ranges', got {split!r}")
    blocks = split == "blocks"
    shard = (rank, world, block) if blocks else (rank, world)
    out = model(t, render_kwargs=render_kwargs, ray_shard=shard, render_depth=True,
                render_weights=True, **forward_kwargs)
    return _assemble(model, t, out, render_kwargs, rank, world, group, blocks, block, forward_kwargs)


def capture_sharded(model, t, render_kwargs, rank: int, world: int, group=None, block: int = RAY_BLOCK,
                    workspace=None, **forward_kwargs):
    """The "blocks" split with this rank's frame captured as one HIP graph
    (TemporalPoints.capture_frame(ray_shard=(rank, world, block))): returns ``step(t)``, which
    replays the graph and all-gathers the tiles (the collective stays outside the graph, so the
    same step runs over RCCL or gloo) -> a ShardedFrame like render_sharded's. Capture again after
    changing the model or the rays. ``workspace``: the graph's per-frame buffers (frames in
    flight on one model give each step its own, see replay_in_flight)."""
    local = model.capture_frame(t, render_kwargs, ray_shard=(rank, world, block), capture_error_mode="thread_local",
                                workspace=workspace, **forward_kwargs)

    def step(t):
        out = local(t)
        return _assemble(model, t, out, render_kwargs, rank, world, group, True, block, forward_kwargs,
                         invalidate=local.invalidate)
    # (no step.graph: a re-capture replaces local.graph, and a reference here would keep the old
    # graph -- and the buffers only it holds -- alive)
    def assemble(t, out):   # the tiles of a replayed frame (step.local(t)) -> the all-gathered frame
        return _assemble(model, t, out, render_kwargs, rank, world, group, True, block, forward_kwargs,
                         invalidate=local.invalidate)
    step.local, step.overflowed, step.capacity, step.assemble = local, local.overflowed, local.capacity, assemble
    return step


def replay_in_flight(steps, ts, streams, comm, keep: bool = False, views=None) -> list:
    """Ray-shard frames with len(steps) frames in flight (bench.py --in-flight): frame i (time
    ts[i]) replays steps[i % n]'s graph (capture_sharded steps of one model, each captured into a
    workspace of its own -- apn_amd.pipeline.capture_sharded_in_flight) on
    streams[i % n], and its tile all-gather (step.assemble) runs on the ONE collective stream
    ``comm`` in frame order, so every rank issues the same collectives in the same order. A
    stream's next replay waits (event) for the assembly of its previous frame, whose tile it
    overwrites. ``views[i]`` (objects with ``rays`` = (rays_o, rays_d, viewdirs), ``c2w``, ``K``;
    synthetic.View): frame i's rays and camera, copied into the step's own inputs (``step.inputs``)
    on its stream before the replay. Returns every assembled frame (``keep``) or the last one, in
    a list."""
    n = len(steps)
    cur = torch.cuda.current_stream()
    ev = torch.cuda.Event()
    ev.record(cur)
    for s in list(streams) + [comm]:
        s.wait_event(ev)
    done = [torch.cuda.Event() for _ in range(n)]
    frames = []
    for i, t in enumerate(ts):
        s = streams[i % n]
        if i >= n:
            s.wait_event(done[i % n])   # frame i - n's tile has been packed and gathered
        with torch.cuda.stream(s):
            if views is not None:
                set_inputs(steps[i % n], views[i])
            o = steps[i % n].local(t)
        comm.wait_stream(s)
        with torch.cuda.stream(comm):
            f = steps[i % n].assemble(t, o)
            done[i % n].record(comm)
        frames = frames + [f] if keep else [f]
    for s in list(streams) + [comm]:
        cur.wait_stream(s)
    return frames


def set_inputs(step, view):
    """Copy a view's rays (and camera pose / intrinsics, when the step projects the skeleton) into
    a capture_sharded_in_flight step's input buffers, on the current stream."""
    inp = getattr(step, "inputs", None)
    if inp is None:
        raise RuntimeError("replay_in_flight(views=...): the steps need their own inputs "
                           "(pipeline.capture_sharded_in_flight)")
    for dst, src in zip(inp["rays"], view.rays):
        dst.copy_(src.reshape(dst.shape), non_blocking=True)
    if inp.get("poses") is not None:
        inp["poses"].copy_(view.c2w.reshape(inp["poses"].shape), non_blocking=True)
        inp["Ks"].copy_(view.K.reshape(inp["Ks"].shape), non_blocking=True)


def _assemble(model, t, out, render_kwargs, rank, world, group, blocks, block, forward_kwargs, invalidate=None):
    dev = render_kwargs["rays_o"].device
    R = render_kwargs["rays_o"].shape[0]
    n = model.last_ray_count
    tile = pack_tile(out, n, dev)
    info = getattr(out, "_info", None)
    if world > 1 and info is None:   # exact path: nothing was dropped
        info = torch.zeros(4, dtype=torch.int32, device=dev)
    if world > 1 and blocks:
        full, infos = gather_blocks(tile, R, world, block, group, info=info)
    elif world > 1:
        kept = model.last_kept_per_ray(n)
        tile = torch.cat([tile, kept.float().reshape(-1, 1)], dim=1)   # survivors per ray (exact in f32)
        full, infos = gather_tiles(tile, model.last_ray_bounds, group, info=info)
        tracker = model.last_split_tracker
        if tracker is not None and not model._force_exact:
            tracker.submit_cost(model.last_full_offsets, full[:, TILE_WIDTH].to(torch.int64), world)
    else:
        full, infos = tile, (info.view(1, 4) if info is not None else None)
        if invalidate is not None and infos is not None:
            infos = infos.clone()   # a replayed graph's static frame_info: the next replay overwrites it
    res = unpack_tile(full)
    for k in ("t_hat_pcd", "joints", "bones"):
        v = out.raw(k) if hasattr(out, "raw") else out.get(k)
        if invalidate is not None and isinstance(v, torch.Tensor):
            # a replayed graph's static buffer: copied (on this stream, before the caller records
            # the frame's done event), so a kept frame keeps its own values after later replays
            v = v.clone()
        res[k] = v

    def rerender(infos):
        # grow this rank's capacity from its in-bbox total (frame_info[1]) for the frames to come
        from .temporalpoints import _grow_capacity
        key = (R, rank, world, block) if blocks else (R, rank, world)
        model._capacity[key] = max(model._capacity.get(key, 0), _grow_capacity(int(infos[rank, 1])))
        model.sharded_rerenders = getattr(model, "sharded_rerenders", 0) + 1
        if invalidate is not None and int(infos[rank, 2]) != 0:
            # this rank's captured graph (capture_sharded) holds the old capacity: capture again
            # before its next replay, or every later frame overflows (and re-renders) as well
            invalidate()
        model._force_exact = True
        try:
            # the frame may be read after render_sharded's no_grad scope has exited: the re-render
            # must stay on the fused render path, not the differentiable one
            with torch.no_grad():
                whole = model(t, render_kwargs=render_kwargs, render_depth=True, render_weights=True,
                              **forward_kwargs)
            return {k: whole.get(k) for k, _ in TILE_KEYS} | {k: whole.get(k) for k in ("t_hat_pcd", "joints", "bones")}
        finally:
            model._force_exact = False
    on_infos = None
    if not blocks and world > 1 and infos.is_cuda:
        # the capacity for the frames to come, sync-free: the largest in-bbox share any rank had,
        # copied to the host without waiting; the next frame of this shard applies it once the copy
        # has landed (TemporalPoints._render), whether or not this frame is ever read
        mx = infos[:, 1].max().to(torch.int64)
        host = torch.empty(1, dtype=torch.int64, pin_memory=True)
        host.copy_(mx.reshape(1), non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        model._cap_updates[(R, rank, world)] = (host, ev)

    if not blocks and world > 1:
        def on_infos(infos):
            # the ranges split follows the survivors once the cost split starts, so a rank's in-bbox
            # share moves between frames: size every rank for the largest share any rank had
            from .temporalpoints import _grow_capacity
            key = (R, rank, world)
            model._capacity[key] = max(model._capacity.get(key, 0), _grow_capacity(int(infos[:, 1].max())))
    return ShardedFrame(res, infos=infos, rerender=rerender, on_infos=on_infos)
