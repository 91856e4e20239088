"""Ray-sharded rendering across real processes (apn_amd/shard.py).

Two fresh child processes (torch.multiprocessing ``spawn``) each render their rays of one
frame through ``render_sharded`` (both splits: interleaved ray blocks, contiguous ranges) and assemble the frame with the tile all-gather over ``gloo``
(RCCL needs one GPU per rank; this box has one). Rank 0 also renders the frame in one process.
The assembled frames of both ranks must equal the single-process frame bit for bit.

The file name sorts first so that pytest runs this test before any other GPU test touches the
device in the parent: the parent never initialises the GPU before the children are spawned (it
does not touch it at all here)."""
import os
import socket
import tempfile

import pytest
import torch

pytestmark = pytest.mark.gpu

WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _assembled(out, R, dev):
    from apn_amd.shard import TILE_KEYS
    return torch.cat([out[k].reshape(R, w).float() for k, w in TILE_KEYS], dim=1).cpu()   # validated reads


def _worker(rank, world, port, outdir, split):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    from apn_amd import harness, synthetic as S
    from apn_amd.shard import RAY_BLOCK, capture_sharded, pack_tile, render_sharded, replay_in_flight
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        scene = S.make_scene(S.SceneConfig("spawn shard 200x200 50k pts 24 bones", 50_000, 24, 200, 200))
        model = harness.build_model(scene, dev)
        rk = scene.render_kwargs(dev)
        R = rk["rays_o"].shape[0]
        t0 = torch.tensor([scene.cfg.t], device=dev)
        t1 = torch.tensor([scene.cfg.t + 0.1], device=dev)
        poses, Ks = scene.c2w[None].to(dev), scene.K[None].to(dev)
        kw = dict(poses=poses, Ks=Ks, get_skeleton=True)
        tiles = {}
        with torch.no_grad():
            # frame 0: exact path (split and sample count read on the host); frames 1-2: the
            # sync-free path (previous frame's split, per-rank capacity); frame 3: rank 1 overflows
            # its capacity, which every rank must detect through the gathered frame_info rows
            # ("graph": the blocks split with each rank's frame replayed from a HIP graph, bench's step)
            step = capture_sharded(model, t0, rk, rank, world, **kw) if split == "graph" else None
            in_flight = None
            seq = (0, 1, 0, 1)
            if split == "graph2":
                # two frames in flight on ONE model (its shard graph captured into two workspaces),
                # one collective stream. Times (t0, t0, t1, t1): each graph renders both times, so a
                # replay that overwrote a frame's tile before its all-gather read it would show
                # (with (t0, t1, t0, t1) each graph always rendered the same time)
                from apn_amd.pipeline import capture_sharded_in_flight
                steps = capture_sharded_in_flight(model, t0, rk, rank, world, n=2, **kw)
                step = steps[0]
                seq = (0, 0, 1, 1)
                streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
                in_flight = replay_in_flight(steps, [(t0, t1)[j] for j in seq], streams, torch.cuda.Stream(dev),
                                             keep=True)
            for i, t in enumerate([(t0, t1)[j] for j in seq]):
                tiles[f"tidx{i}"] = torch.tensor(seq[i])
                if i == 3 and rank == 1 and step is None:
                    model._capacity[(R, rank, world, RAY_BLOCK) if split == "blocks" else (R, rank, world)] = 64
                if in_flight is not None:
                    out = in_flight[i]
                elif step is not None:
                    out = step(t)
                else:
                    out = render_sharded(model, t, rk, rank, world, split=split, **kw)
                tiles[f"assembled{i}"] = _assembled(out, R, dev)
                tiles[f"count{i}"] = torch.tensor(model.last_ray_count)
                if split == "ranges":
                    tiles[f"range{i}"] = torch.tensor(model.last_ray_range)
                    tiles[f"bounds{i}"] = torch.tensor(model.last_ray_bounds)
            if rank == 0:
                for i, t in enumerate((t0, t1)):
                    single = model(t, render_depth=True, render_kwargs=rk, render_weights=True, **kw)
                    tiles[f"single{i}"] = pack_tile(single, R, dev).cpu()
        torch.cuda.synchronize()
        torch.save(tiles, os.path.join(outdir, f"rank{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("split", ["blocks", "ranges", "graph", "graph2"])
def test_render_sharded_two_processes_bit_identical(split):
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(WORLD, _free_port(), d, split), nprocs=WORLD, join=True)
        res = [torch.load(os.path.join(d, f"rank{r}.pt"), weights_only=True) for r in range(WORLD)]
    for i in range(4):
        single = res[0][f"single{int(res[0][f'tidx{i}'])}"]
        R = single.shape[0]
        if split == "ranges":
            bounds = res[0][f"bounds{i}"].tolist()
            assert bounds[0] == 0 and bounds[-1] == R
            assert torch.equal(res[1][f"bounds{i}"], res[0][f"bounds{i}"]), i   # every rank on the same split
            # both ranks did real work (the object is hit by rays of both halves of the split)
            assert 0 < bounds[1] < R
        else:
            bounds = None
            assert int(res[0][f"count{i}"]) + int(res[1][f"count{i}"]) == R
        for r in range(WORLD):
            if split == "ranges":
                assert tuple(res[r][f"range{i}"].tolist()) == (bounds[r], bounds[r + 1])
            a = res[r][f"assembled{i}"]
            if not torch.equal(a, single):
                bad = (a != single).any(1).nonzero().flatten()
                cols = (a != single).any(0).nonzero().flatten().tolist()
                raise AssertionError(f"{split} frame {i} rank {r}: {len(bad)} rays differ (first {bad[:8].tolist()}), "
                                     f"columns {cols}, max |d| {float((a - single).abs().max()):.3e}, "
                                     f"bounds {bounds}")


def _concurrent_worker(rank, frames, outdir):
    """One of several processes sharing the GPU: the full render frame of the spawn scene, again and
    again; every frame's skinned cloud, survivor list and tile must equal the process's first."""
    from apn_amd import harness, synthetic as S
    from apn_amd.shard import pack_tile
    dev = torch.device("cuda", 0)
    scene = S.make_scene(S.SceneConfig("spawn shard 200x200 50k pts 24 bones", 50_000, 24, 200, 200))
    model = harness.build_model(scene, dev)
    rk = scene.render_kwargs(dev)
    R = rk["rays_o"].shape[0]
    t0 = torch.tensor([scene.cfg.t], device=dev)
    ref, bad = None, {"xyz": 0, "s_nbr": 0, "tile": 0}
    with torch.no_grad():
        for f in range(frames):
            out = model(t0, render_depth=True, render_kwargs=rk, render_weights=True)
            ns = int(model.last_stats["kept_samples"])
            cur = {"xyz": out["t_hat_pcd"].clone(), "s_nbr": model._ws.bufs["s_nbr"][:8 * ns].clone(),
                   "tile": pack_tile(out, R, dev)}
            if ref is None:
                ref = cur
                continue
            for k in bad:
                bad[k] += int(not torch.equal(cur[k], ref[k]))
    torch.save(bad, os.path.join(outdir, f"conc{rank}.pt"))


def test_concurrent_processes_render_deterministically():
    """Three processes render the same frame 150 times each on one GPU. Round 3's root cause of the
    two-process mismatch: packed-FP32 VALU in k_lbs_skin gave a wrong y coordinate
    for one 16-lane pass in ~8 % of such frames (tools/determinism_probe3.py); the library is now
    built without packed-FP32 instructions (tests/test_build_isa.py) and every frame must repeat."""
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_concurrent_worker, args=(150, d), nprocs=3, join=True)
        res = [torch.load(os.path.join(d, f"conc{r}.pt"), weights_only=True) for r in range(3)]
    assert all(sum(r.values()) == 0 for r in res), res
