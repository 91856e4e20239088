"""Host logic of the ray-sharded multi-GPU path (apn_amd/shard.py) on the CPU: the balanced
ray split and the tile all-gather over a real 2-process gloo group (the GPU box uses RCCL)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from apn_amd.shard import TILE_WIDTH, balanced_ray_split, gather_tiles, pack_tile, unpack_tile


def _offsets(counts):
    return torch.cat([torch.zeros(1, dtype=torch.int32), torch.cumsum(torch.as_tensor(counts), 0).to(torch.int32)])


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_balanced_split_covers_and_balances(world):
    g = torch.Generator().manual_seed(world)
    counts = torch.randint(0, 40, (5000,), generator=g)
    counts[:1000] = 0  # empty rays (background) at the start, like the top image rows
    offs = _offsets(counts)
    b = balanced_ray_split(offs, world)
    assert len(b) == world + 1 and b[0] == 0 and b[-1] == 5000
    assert all(b[i] <= b[i + 1] for i in range(world))
    total = int(offs[-1])
    for k in range(world):
        part = int(offs[b[k + 1]] - offs[b[k]])
        assert abs(part - total / world) <= 40 + 1, (k, part, total / world)


def test_balanced_split_degenerate():
    assert balanced_ray_split(_offsets([0, 0, 0]), 2) == [0, 0, 3] or balanced_ray_split(_offsets([0, 0, 0]), 2)[-1] == 3
    b = balanced_ray_split(_offsets([100]), 4)
    assert b[0] == 0 and b[-1] == 1 and b == sorted(b)
    b = balanced_ray_split(_offsets([]), 2)
    assert b == [0, 0, 0]


def test_pack_unpack_roundtrip():
    n = 7
    out = {"rgb_marched": torch.rand(n, 3), "rgb_marched_direct": torch.rand(n, 3), "depth": torch.rand(n),
           "weights": torch.rand(n, 3), "alphainv_last": torch.rand(n), "alphainv_last_direct": torch.rand(n)}
    tile = pack_tile(out, n, "cpu")
    assert tile.shape == (n, TILE_WIDTH)
    back = unpack_tile(tile)
    for k, v in out.items():
        assert torch.equal(back[k], v), k


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, counts, result_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        offs = _offsets(counts)
        bounds = balanced_ray_split(offs, world)
        R = len(counts)
        full = torch.arange(R * TILE_WIDTH, dtype=torch.float32).reshape(R, TILE_WIDTH)
        r0, r1 = bounds[rank], bounds[rank + 1]
        got = gather_tiles(full[r0:r1].clone(), bounds)
        # elapsed-time reduction of bench.py: max over ranks
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        result_q.put((rank, bool(torch.equal(got, full)), float(t)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("counts", [[3, 0, 5, 9, 1, 0, 0, 7, 2, 4, 6], [0] * 6 + [50]])
def test_gather_tiles_gloo_world2(counts):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, counts, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok, tmax in res:
        assert ok, rank
        assert tmax == float(world)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_point_shards_partition_the_cloud(world):
    """C5 point sharding (bench.py --config C5 with N>1): the ranks' point ranges partition the
    cloud, and the per-point LBS parameters the constructor derives (bone-distance weights) of
    the shards concatenate to the full model's -- so the sharded sweep skins exactly the full
    cloud."""
    from apn_amd import harness, synthetic as S
    scene = S.make_scene(S.SceneConfig("shard test", 3001, 24, 0, 0))
    full = harness.build_model(scene, "cpu")
    parts, ranges = [], []
    for r in range(world):
        sc = harness.shard_scene_points(scene, r, world)
        ranges.append(sc.extra["point_range"])
        m = harness.build_model(sc, "cpu")
        parts.append((m.canonical_pcd, m.weights.detach(), m.canonical_feat.detach()))
    assert ranges[0][0] == 0 and ranges[-1][1] == 3001
    assert all(ranges[i][1] == ranges[i + 1][0] for i in range(world - 1))
    assert torch.equal(torch.cat([p[0] for p in parts]), full.canonical_pcd)
    assert torch.equal(torch.cat([p[1] for p in parts]), full.weights.detach())
    assert torch.equal(torch.cat([p[2] for p in parts]), full.canonical_feat.detach())


def _worker_info(rank, world, port, result_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        bounds = [0, 3, 7]
        full = torch.arange(7 * TILE_WIDTH, dtype=torch.float32).reshape(7, TILE_WIDTH)
        info = torch.tensor([10 + rank, 20 + rank, rank, 30 + rank], dtype=torch.int32)
        got, infos = gather_tiles(full[bounds[rank]:bounds[rank + 1]].clone(), bounds, info=info)
        want = torch.tensor([[10, 20, 0, 30], [11, 21, 1, 31]], dtype=torch.int32)
        result_q.put((rank, bool(torch.equal(got, full)), bool(torch.equal(infos, want))))
    finally:
        dist.destroy_process_group()


def test_gather_tiles_carries_frame_info_gloo_world2():
    """The per-rank frame_info row rides in the same all-gather (ShardedFrame's overflow check)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_info, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert res == [(0, True, True), (1, True, True)]


def test_split_tracker_cpu_keeps_first_split():
    """Off the GPU there is no async copy: the tracker keeps the first frame's balanced split."""
    from apn_amd.shard import SplitTracker
    tr = SplitTracker()
    a = tr.bounds_for(_offsets([5, 0, 3, 9, 1, 4]), 2)
    b = tr.bounds_for(_offsets([0, 0, 0, 0, 30, 1]), 2)
    assert a == b == balanced_ray_split(_offsets([5, 0, 3, 9, 1, 4]), 2)


def test_cost_offsets_weights_survivors():
    """shard.cost_offsets: exclusive prefix of KEPT_WEIGHT * survivors + in-bbox samples per ray;
    the split of it puts equal cost (not equal samples) on each rank."""
    from apn_amd.shard import KEPT_WEIGHT, cost_offsets, split_inner, bounds_from_inner
    inb = [4, 4, 4, 4, 4, 4, 4, 4]
    kept = torch.tensor([4, 4, 4, 4, 0, 0, 0, 0], dtype=torch.int32)
    offs = _offsets(inb)
    c = cost_offsets(offs, kept)
    per = torch.tensor(inb) + KEPT_WEIGHT * kept.long()
    assert c.dtype == torch.int64 and c.tolist() == [0] + torch.cumsum(per, 0).tolist()
    b = bounds_from_inner(split_inner(c, 2).tolist(), len(inb))
    # equal in-bbox halves would be [0, 4, 8]; equal cost puts the boundary inside the first half
    assert b[0] == 0 and b[-1] == len(inb) and b[1] < 4
    costs = [int(c[b[i + 1]] - c[b[i]]) for i in range(2)]
    assert abs(costs[0] - costs[1]) <= 2 * int(per.max())   # a boundary lands within one ray of the target


@pytest.mark.parametrize("R,world,block", [(10, 2, 3), (11, 3, 2), (64, 8, 4), (5, 4, 4), (4096 * 3 + 7, 2, 4096)])
def test_block_split_partitions_and_assembles(R, world, block):
    """The "blocks" split: the ranks' rays partition the frame, each rank holds at most
    block_slots * block rays, and the zero-padded per-rank tiles assemble into ray order."""
    from apn_amd.shard import assemble_blocks, block_rays, block_slots
    idx = [block_rays(R, r, world, block) for r in range(world)]
    allr = torch.cat(idx)
    assert torch.equal(allr.sort().values, torch.arange(R))
    assert all(bool((i[1:] > i[:-1]).all()) for i in idx if i.numel() > 1)
    m = block_slots(R, world, block) * block
    assert max(i.numel() for i in idx) <= m
    assert max(i.numel() for i in idx) - min(i.numel() for i in idx) <= block
    full = torch.arange(R * 5, dtype=torch.float32).reshape(R, 5)
    parts = torch.zeros(world, m, 5)
    for r in range(world):
        parts[r, :idx[r].numel()] = full[idx[r]]
    assert torch.equal(assemble_blocks(parts, R, world, block), full)


def _worker_blocks(rank, world, port, R, block, result_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from apn_amd.shard import block_rays, gather_blocks
        full = torch.arange(R * TILE_WIDTH, dtype=torch.float32).reshape(R, TILE_WIDTH)
        idx = block_rays(R, rank, world, block)
        info = torch.tensor([10 + rank, 20 + rank, rank, 30 + rank], dtype=torch.int32)
        got, infos = gather_blocks(full[idx].clone(), R, world, block, info=info)
        want = torch.tensor([[10 + r, 20 + r, r, 30 + r] for r in range(world)], dtype=torch.int32)
        result_q.put((rank, bool(torch.equal(got, full)), bool(torch.equal(infos, want))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("R,block", [(23, 4), (24, 4), (3, 8)])
def test_gather_blocks_gloo_world2(R, block):
    """The unpadded block all-gather (plus the frame_info row) over two gloo processes, with a
    short last block on either rank and a rank without rays."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_blocks, args=(r, 2, port, R, block, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert res == [(0, True, True), (1, True, True)]


@pytest.mark.parametrize("read", ["getitem", "dict", "splat", "values", "iter", "len", "copy", "pop", "items"])
def test_sharded_frame_every_read_validates(read):
    """An overflowed ShardedFrame re-renders on its first read through ANY dict access path
    (dict(frame), {**frame}, values(), iteration, len, copy, pop skipped the check)."""
    from apn_amd.shard import ShardedFrame
    calls = []

    def rerender(infos):
        calls.append(infos[:, 2].tolist())
        return {"rgb_marched": torch.ones(4, 3), "depth": torch.full((4,), 2.0)}
    f = ShardedFrame({"rgb_marched": torch.zeros(4, 3), "depth": torch.zeros(4)},
                     infos=torch.tensor([[10, 10, 0, 5], [10, 20, 1, 5]], dtype=torch.int32), rerender=rerender)
    with torch.enable_grad():   # read after render_sharded's no_grad scope
        got = {"getitem": lambda: {"rgb_marched": f["rgb_marched"]}, "dict": lambda: dict(f),
               "splat": lambda: {**f}, "values": lambda: dict(zip(("rgb_marched", "depth"), list(f.values()))),
               "iter": lambda: {k: dict.__getitem__(f, k) for k in iter(f)},
               "len": lambda: (len(f), dict(dict.items(f)))[1], "copy": lambda: f.copy(),
               "pop": lambda: {"rgb_marched": f.pop("rgb_marched")}, "items": lambda: dict(f.items())}[read]()
    assert calls == [[0, 1]]   # exactly one re-render, on the first read
    assert torch.equal(got["rgb_marched"], torch.ones(4, 3))


def test_sharded_frame_reports_every_ranks_info_once():
    """The ranges split sizes each rank's sample capacity from the largest in-bbox share any rank
    had (the cost split moves shares between frames): ShardedFrame hands the gathered
    frame_infos to on_infos exactly once, on the first read, whether or not a rank overflowed."""
    from apn_amd.shard import ShardedFrame
    seen = []
    f = ShardedFrame({"depth": torch.zeros(4)}, infos=torch.tensor([[10, 7, 0, 5], [10, 9, 0, 5]], dtype=torch.int32),
                     rerender=lambda infos: pytest.fail("no rank overflowed"),
                     on_infos=lambda infos: seen.append(int(infos[:, 1].max())))
    assert seen == []
    _ = f["depth"]
    _ = dict(f)
    assert seen == [9]
