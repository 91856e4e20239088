"""The sync-free render frame and its HIP-graph capture.

* after a ray count's first frame (which reads the in-bbox sample count once and sizes a
  capacity), frames keep that count on the device (apn_inbbox_fill_capped): the result equals the
  exact path bit for bit, and the frame statistics resolve lazily from the device frame_info;
* a frame whose samples overflow the capacity is detected on first read and rendered again on
  the exact path (same values as an exact frame), growing the capacity;
* TemporalPoints.capture_frame replays the whole no-grad forward as one HIP graph: each replay
  equals the eager frame at that time bit for bit."""
import pytest
import torch

pytestmark = pytest.mark.gpu

KEYS = ("rgb_marched", "rgb_marched_direct", "depth", "weights", "alphainv_last")


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch.device("cuda")


def _scene_model(dev, name="G3"):
    from apn_amd import harness, synthetic as S
    scene = S.make_scene(name)
    return scene, harness.build_model(scene, dev)


def _frame(model, t, rk):
    with torch.no_grad():
        o = model(t, render_depth=True, render_kwargs=rk, render_weights=True)
    return {k: o[k].clone() for k in KEYS}


def test_sync_free_frame_equals_exact(dev):
    scene, model = _scene_model(dev)
    rk = scene.render_kwargs(dev)
    R = len(rk["rays_o"])
    t = torch.tensor([scene.cfg.t], device=dev)
    a = _frame(model, t, rk)
    stats_a = model.last_stats.resolved()
    assert R in model._capacity and model._capacity[R] >= stats_a["inbbox_samples"]
    b = _frame(model, t, rk)
    assert model._last_info is not None          # the second frame took the capacity path
    stats_b = model.last_stats.resolved()
    assert stats_a == stats_b
    for k in KEYS:
        assert torch.equal(a[k], b[k]), k


def test_overflowing_frame_is_rendered_again(dev):
    scene, model = _scene_model(dev)
    rk = scene.render_kwargs(dev)
    R = len(rk["rays_o"])
    t = torch.tensor([scene.cfg.t], device=dev)
    exact = _frame(model, t, rk)
    n = model.last_stats["inbbox_samples"]
    model._capacity[R] = 64                       # far below the frame's sample count
    with torch.no_grad():
        o = model(t, render_depth=True, render_kwargs=rk, render_weights=True)
    assert model._last_info is not None and int(model._last_info[2]) == 1   # overflow flagged on the device
    for k in KEYS:                                 # first read: validated, rendered again exactly
        assert torch.equal(o[k], exact[k]), k
    assert model._capacity[R] >= n


def test_captured_frame_equals_eager(dev):
    scene, model = _scene_model(dev)
    rk = scene.render_kwargs(dev)
    t0 = torch.tensor([scene.cfg.t], device=dev)
    t1 = torch.tensor([scene.cfg.t + 0.15], device=dev)
    step = model.capture_frame(t0, rk)
    for t in (t0, t1, t0):
        g = step(t)
        got = {k: g[k].clone() for k in KEYS}
        ref = _frame(model, t, rk)
        for k in KEYS:
            assert torch.equal(got[k], ref[k]), k


def test_captured_frame_back_to_back(dev):
    """Consecutive replays with no eager frame in between (bench --graph on). Round 2 saw these
    fault on the second replay while the captured frame still held memset / memcpy nodes and the
    full per-frame weight repack; the frame now captures kernel nodes only (apn_common.h fill_i32 /
    copy_i32) and repacks only the pose-folded b1."""
    scene, model = _scene_model(dev)
    rk = scene.render_kwargs(dev)
    ts = [torch.tensor([scene.cfg.t + 0.05 * i], device=dev) for i in range(4)]
    poses, Ks = scene.c2w[None].to(dev), scene.K[None].to(dev)
    step = model.capture_frame(ts[0], rk, poses=poses, Ks=Ks, get_skeleton=True)   # the bench's frame
    kept = []
    for i in range(12):
        g = step(ts[i % 4])
        torch.cuda.synchronize()
        if i >= 8:
            kept.append({k: g[k].clone() for k in KEYS + ("joints",)})
    for i, got in enumerate(kept):
        with torch.no_grad():
            ref = model(ts[(8 + i) % 4], render_depth=True, render_kwargs=rk, render_weights=True, poses=poses,
                        Ks=Ks, get_skeleton=True)
        for k in KEYS + ("joints",):
            assert torch.equal(got[k], ref[k]), (i, k)


@pytest.mark.parametrize("n", [2, 3])
def test_two_frames_in_flight_equal_eager(dev, n):
    """n models of one scene (own workspaces), their captured frames replayed on n streams, frame i
    on stream i % n, ALL frames issued before anything is read (a read validates the
    frame through a host sync, which had serialised the frames): each frame's outputs are cloned
    on its own stream with RenderOutput.raw (no validation, no sync) right after its replay, the
    overflow flags are checked once after the streams are joined, and every frame equals the
    eager frame at its time bit for bit."""
    from apn_amd import harness
    scene, a = _scene_model(dev)
    models = [a] + [harness.build_model(scene, dev) for _ in range(n - 1)]
    rk = scene.render_kwargs(dev)
    ts = [torch.tensor([scene.cfg.t + 0.05 * i], device=dev) for i in range(4)]
    steps = [m.capture_frame(ts[0], rk) for m in models]
    streams = [torch.cuda.Stream(dev) for _ in range(n)]
    cur = torch.cuda.current_stream(dev)
    for s in streams:
        s.wait_stream(cur)
    got = []
    for i in range(8):
        with torch.cuda.stream(streams[i % n]):
            g = steps[i % n](ts[i % 4])
            got.append({k: g.raw(k).clone() for k in KEYS})
    for s in streams:
        cur.wait_stream(s)
    torch.cuda.synchronize()
    assert not any(st.overflowed() for st in steps)
    for i, frame in enumerate(got):
        ref = _frame(a, ts[i % 4], rk)
        for k in KEYS:
            assert torch.equal(frame[k], ref[k]), (i, k)


def test_captured_frame_overflow_recaptures(dev, monkeypatch):
    """A replay whose samples overflow the captured capacity is flagged (step.overflowed(), the OR
    of every replay's frame_info[2] accumulated inside the graph), its read re-renders it exactly,
    and the next step captures again with the grown capacity instead of overflowing every frame."""
    import apn_amd.temporalpoints as TP
    scene, model = _scene_model(dev)
    rk = scene.render_kwargs(dev)
    R = len(rk["rays_o"])
    # two times whose in-bbox sample counts differ: capture at the smaller one with no headroom
    ts = [torch.tensor([scene.cfg.t + 0.1 * i], device=dev) for i in range(6)]
    counts = []
    for t in ts:
        model._force_exact = True
        _frame(model, t, rk)
        model._force_exact = False
        counts.append(model.last_stats["inbbox_samples"])
    lo, hi = min(range(6), key=lambda i: counts[i]), max(range(6), key=lambda i: counts[i])
    assert counts[hi] > counts[lo], counts
    model._capacity.pop(R, None)
    monkeypatch.setattr(TP, "_grow_capacity", lambda n: int(n))
    step = model.capture_frame(ts[lo], rk)
    monkeypatch.undo()
    assert step.capacity() == counts[lo]
    g = step(ts[lo])
    torch.cuda.synchronize()
    assert not step.overflowed()
    g = step(ts[hi])                                   # more samples than the graph holds
    assert step.overflowed()
    got = {k: g[k].clone() for k in KEYS}              # first read: rendered again exactly
    ref = _frame(model, ts[hi], rk)
    for k in KEYS:
        assert torch.equal(got[k], ref[k]), k
    g = step(ts[hi])                                   # captured again with the grown capacity
    assert step.capacity() >= counts[hi]
    got = {k: g[k].clone() for k in KEYS}
    assert not step.overflowed()
    for k in KEYS:
        assert torch.equal(got[k], ref[k]), k


def test_captured_ray_block_shards_equal_eager_and_assemble(dev):
    """capture_frame(ray_shard=(rank, world, block)) -- the per-rank graph of shard.capture_sharded
    (bench --gpus N) -- replays back to back equal to the eager shard frame, and the ranks' replays
    assemble into the single-GPU frame."""
    from apn_amd.shard import assemble_blocks, block_slots, pack_tile
    scene, model = _scene_model(dev)
    rk = scene.render_kwargs(dev)
    R = len(rk["rays_o"])
    ts = [torch.tensor([scene.cfg.t + 0.07 * i], device=dev) for i in range(3)]
    world, block = 2, 512
    steps = [model.capture_frame(ts[0], rk, ray_shard=(r, world, block)) for r in range(world)]
    counts = [model._block_index[(R, r, world, block)].numel() for r in range(world)]
    for i in range(6):
        t = ts[i % 3]
        parts = torch.zeros(world, block_slots(R, world, block) * block, 12, device=dev)
        for r in range(world):
            g = steps[r](t)
            parts[r, :counts[r]] = pack_tile(g, counts[r], dev)
        with torch.no_grad():
            for r in range(world):
                e = model(t, render_depth=True, render_kwargs=rk, render_weights=True, ray_shard=(r, world, block))
                assert torch.equal(parts[r, :counts[r]], pack_tile(e, counts[r], dev)), (i, r)
        with torch.no_grad():
            full = pack_tile(model(t, render_depth=True, render_kwargs=rk, render_weights=True), R, dev)
        assert torch.equal(assemble_blocks(parts, R, world, block), full), i


def test_captured_shard_overflow_recaptures_and_releases(dev, monkeypatch):
    """shard.capture_sharded (bench --gpus N, one graph per rank): a replay that overflows the
    captured capacity is read through the assembled frame, which renders it again exactly AND makes
    the rank's graph capture again (before, every later frame overflowed again). The
    re-capture drops the old graph, and the workspace buffers retired while it was alive are
    released with it (no growth of Workspace.retired per capacity step). world = 1: the same code
    path without a process group."""
    import gc
    import apn_amd.temporalpoints as TP
    from apn_amd.shard import RAY_BLOCK, capture_sharded
    scene, model = _scene_model(dev)
    rk = scene.render_kwargs(dev)
    R = len(rk["rays_o"])
    ts = [torch.tensor([scene.cfg.t + 0.1 * i], device=dev) for i in range(6)]
    counts = []
    for t in ts:
        model._force_exact = True
        _frame(model, t, rk)
        model._force_exact = False
        counts.append(model.last_stats["inbbox_samples"])
    lo, hi = min(range(6), key=lambda i: counts[i]), max(range(6), key=lambda i: counts[i])
    assert counts[hi] > counts[lo], counts
    key = (R, 0, 1, RAY_BLOCK)
    model._capacity.pop(key, None)
    monkeypatch.setattr(TP, "_grow_capacity", lambda n: int(n))
    step = capture_sharded(model, ts[lo], rk, 0, 1)
    monkeypatch.undo()
    assert step.capacity() == counts[lo]
    g = step(ts[lo])
    torch.cuda.synchronize()
    assert not step.overflowed()
    g = step(ts[hi])
    assert step.overflowed()
    got = {k: g[k].clone() for k in KEYS}              # first read: rendered again exactly, graph invalidated
    ref = _frame(model, ts[hi], rk)
    for k in KEYS:
        assert torch.equal(got[k], ref[k]), k
    g = step(ts[hi])                                   # captured again with the grown capacity
    assert step.capacity() >= counts[hi]
    got = {k: g[k].clone() for k in KEYS}
    assert not step.overflowed()
    for k in KEYS:
        assert torch.equal(got[k], ref[k]), k
    gc.collect()
    # only the live graph may still hold retired buffers
    live = model._ws._holders
    assert len(live) == 1, live
    assert all(toks <= live for _, toks in model._ws.retired)
    n_retired = len(model._ws.retired)
    for _ in range(2):                                  # more growth steps: retired stays bounded
        model._capacity[key] = int(model._capacity[key] * 1.5)
        step.local.invalidate()
        g = step(ts[hi])
        got = {k: g[k].clone() for k in KEYS}
        for k in KEYS:
            assert torch.equal(got[k], ref[k]), k
        gc.collect()
        assert len(model._ws._holders) == 1
        assert len(model._ws.retired) <= max(n_retired, 16), len(model._ws.retired)


def test_successive_captures_with_aggressive_gc(dev):
    """tools/shard_balance.py captured one graph per ray shard in a loop and aborted at world 8:
    the previous shard's step (a closure cycle holding its graph) was freed by the cyclic garbage
    collector in the middle of the next capture, and hipGraphExecDestroy is refused while a stream
    captures. capture_frame now collects unreachable graphs before it captures. With the collector
    set to run at almost every allocation, successive captures (each dropping the previous step)
    must all succeed and replay the eager shard frames."""
    import gc
    from apn_amd.shard import RAY_BLOCK
    scene, model = _scene_model(dev)
    rk = scene.render_kwargs(dev)
    t = torch.tensor([scene.cfg.t], device=dev)
    world = 4
    R = rk["rays_o"].shape[0]
    block = min(RAY_BLOCK, R // (2 * world))   # every rank holds rays (a rank without any cannot capture)
    old = gc.get_threshold()
    gc.set_threshold(1, 1, 1)
    try:
        step = None
        for k in range(world):
            step = model.capture_frame(t, rk, ray_shard=(k, world, block))   # drops the previous step
            got = {key: step(t)[key].clone() for key in KEYS}
            with torch.no_grad():
                ref = model(t, render_depth=True, render_kwargs=rk, render_weights=True,
                            ray_shard=(k, world, block))
            for key in KEYS:
                assert torch.equal(got[key], ref[key]), (k, key)
    finally:
        gc.set_threshold(*old)


def test_shard_steps_dropped_inside_in_flight_replays_with_aggressive_gc(dev):
    """with the collector at its most aggressive, capture_sharded steps of one
    model (frames in flight, each in its own workspace) are dropped and captured again while
    replay_in_flight loops run: captures keep the collector off (temporalpoints._capture_guard),
    so no freed graph is destroyed mid-capture, and every assembled frame equals the eager one."""
    import gc
    from apn_amd.pipeline import capture_sharded_in_flight
    from apn_amd.shard import replay_in_flight
    scene, model = _scene_model(dev)
    rk = scene.render_kwargs(dev)
    ts = [torch.tensor([scene.cfg.t + 0.05 * i], device=dev) for i in range(3)]
    refs = [_frame(model, t, rk) for t in ts]
    old = gc.get_threshold()
    gc.set_threshold(1, 1, 1)
    try:
        for rnd in range(3):
            steps = capture_sharded_in_flight(model, ts[0], rk, 0, 1, n=3)   # drops the previous round's
            streams = [torch.cuda.Stream(dev) for _ in steps]
            comm = torch.cuda.Stream(dev)
            seq = [0, 0, 1, 1, 2, 2, 0]   # period 2 does not divide n = 3: every slot sees every time
            frames = replay_in_flight(steps, [ts[j] for j in seq], streams, comm, keep=True)
            torch.cuda.synchronize()
            assert gc.isenabled()
            for i, f in enumerate(frames):
                for k in KEYS:
                    assert torch.equal(f[k], refs[seq[i]][k]), (rnd, i, k)
    finally:
        gc.set_threshold(*old)
