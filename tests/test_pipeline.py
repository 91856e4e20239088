"""Frames in flight on ONE TemporalPoints (apn_amd.pipeline.FramePipeline).

The frame is captured n times, each capture into a per-frame workspace of its own, and frame i
replays graph i % n on stream i % n. Every test issues all frames before anything is read (reads
go through RenderOutput.raw on each frame's own stream, or the pipeline's pinned readback), uses
time sequences whose period does not divide n (so a slot renders different times and a missing
ordering would show), and compares every frame with the model's eager frame at its time bit for
bit. Reference loop: run.py:108-173 (render, then read back, one view at a time)."""
import numpy as np
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


def _eager(model, t, rk, **kw):
    with torch.no_grad():
        o = model(t, render_depth=True, render_kwargs=rk, render_weights=True, **kw)
    return {k: o[k].clone() for k in KEYS + (("joints",) if kw.get("get_skeleton") else ())}


@pytest.mark.parametrize("n", [2, 3])
def test_pipeline_frames_equal_eager(dev, n):
    from apn_amd.pipeline import FramePipeline
    scene, model = _scene_model(dev)
    rk = scene.render_kwargs(dev)
    ts = [torch.tensor([scene.cfg.t + 0.05 * i], device=dev) for i in range(4)]
    seq = [0, 0, 1, 2, 3, 3, 1, 2, 0, 1]
    pipe = FramePipeline(model, ts[0], rk, n=n, readback=None)
    got = []
    for i, j in enumerate(seq):
        h = pipe.submit(ts[j])
        with torch.cuda.stream(pipe.streams[i % n]):   # the frame's own stream: ordered after its replay
            got.append({k: h.device().raw(k).clone() for k in KEYS})
    pipe.join()
    torch.cuda.synchronize()
    assert not pipe.overflowed()
    refs = [_eager(model, t, rk) for t in ts]
    for i, j in enumerate(seq):
        for k in KEYS:
            assert torch.equal(got[i][k], refs[j][k]), (i, k)


def test_pipeline_shares_tables_not_frames(dev):
    """One model plus n per-frame workspaces: the layer-1 projection P lives once (the model's
    shared workspace), every per-frame buffer once per slot, nothing aliased between slots."""
    from apn_amd.pipeline import FramePipeline
    scene, model = _scene_model(dev)
    rk = scene.render_kwargs(dev)
    t = torch.tensor([scene.cfg.t], device=dev)
    _eager(model, t, rk)   # the model's own workspace (eager frames, re-renders)
    pipe = FramePipeline(model, t, rk, n=3, readback=None)
    assert "feat_proj" in model._ws_shared.bufs
    wss = pipe.workspaces
    for ws in wss:
        assert "feat_proj" not in ws.bufs and "mlp_w" in ws.bufs and "s_nbr" in ws.bufs
    for k in ("mlp_w", "recA", "q_pos", "s_nbr", "out12"):
        ptrs = {ws.bufs[k].data_ptr() for ws in wss} | {model._ws_eager.bufs[k].data_ptr()}
        assert len(ptrs) == len(wss) + 1, k


def test_pipeline_pose_embedding_frames_in_flight(dev):
    """G2 (ZJU, pose embedding): b1 follows each frame's pose embedding, so each slot packs its own
    weight buffer; frames at different times in flight together must not share it."""
    from apn_amd.pipeline import FramePipeline
    scene, model = _scene_model(dev, "G2")
    assert model.pose_embedding_dim > 0
    rk = scene.render_kwargs(dev)
    ts = [torch.tensor([scene.cfg.t + 0.1 * i], device=dev) for i in range(3)]
    seq = [0, 1, 1, 2, 0, 2, 1]
    pipe = FramePipeline(model, ts[0], rk, n=3, readback=None)
    got = []
    for i, j in enumerate(seq):
        h = pipe.submit(ts[j])
        with torch.cuda.stream(pipe.streams[i % 3]):
            got.append({k: h.device().raw(k).clone() for k in KEYS})
    pipe.join()
    torch.cuda.synchronize()
    refs = [_eager(model, t, rk) for t in ts]
    for i, j in enumerate(seq):
        for k in KEYS:
            assert torch.equal(got[i][k], refs[j][k]), (i, k)


def _views(scene, n, dev):
    """n camera poses around the scene's (small translations) and the view's rays on the device."""
    from apn_amd.tineuvox import get_rays_of_a_view
    c2w = scene.c2w.float()
    K = scene.K.float()
    H, W = scene.cfg.H, scene.cfg.W
    out = []
    for i in range(n):
        p = c2w.clone()
        p[:3, 3] += torch.tensor([0.02 * i, -0.01 * (i % 3), 0.015 * (i % 2)])
        p, Kd = p.to(dev), K.to(dev)
        ro, rd, vd = get_rays_of_a_view(H, W, Kd, p, False, inverse_y=bool(scene.inverse_y))
        out.append(((ro.reshape(-1, 3), rd.reshape(-1, 3), vd.reshape(-1, 3)), p[None], Kd[None]))
    return out


def test_pipeline_readback_views_equal_eager(dev):
    """Per-view rays, pose and intrinsics copied into the slots' static inputs; the pinned readback
    (rgb, depth, weights, projected joints) equals each view's eager frame."""
    from apn_amd.pipeline import FramePipeline
    scene, model = _scene_model(dev)
    rk = scene.render_kwargs(dev)
    views = _views(scene, 5, dev)
    ts = [torch.tensor([scene.cfg.t + 0.03 * i], device=dev) for i in range(5)]
    rk0 = dict(rk, rays_o=views[0][0][0], rays_d=views[0][0][1], viewdirs=views[0][0][2])
    pipe = FramePipeline(model, ts[0], rk0, n=3, poses=views[0][1], Ks=views[0][2], get_skeleton=True)
    res = list(pipe.render(ts, views))
    for i, r in enumerate(res):
        (ro, rd, vd), p, K = views[i]
        ref = _eager(model, ts[i], dict(rk, rays_o=ro, rays_d=rd, viewdirs=vd), poses=p, Ks=K, get_skeleton=True)
        for k in ("rgb_marched", "depth", "weights", "joints"):
            assert torch.equal(r[k], ref[k].cpu().reshape(r[k].shape)), (i, k)
    assert pipe.rerenders == 0


def test_pipeline_overflow_rerenders_and_recaptures(dev, monkeypatch):
    """A frame whose samples overflow its slot's captured capacity is rendered again exactly when
    its result is fetched (the model's own workspace, not a slot in flight), and that slot captures
    again before its next replay."""
    import apn_amd.temporalpoints as TP
    from apn_amd.pipeline import FramePipeline
    scene, model = _scene_model(dev)
    rk = scene.render_kwargs(dev)
    R = len(rk["rays_o"])
    ts = [torch.tensor([scene.cfg.t + 0.1 * i], device=dev) for i in range(6)]
    counts = []
    for t in ts:
        model._force_exact = True
        _eager(model, t, rk)
        model._force_exact = False
        counts.append(model.last_stats["inbbox_samples"])
    lo, hi = min(range(6), key=lambda i: counts[i]), max(range(6), key=lambda i: counts[i])
    assert counts[hi] > counts[lo], counts
    model._capacity.pop(R, None)
    monkeypatch.setattr(TP, "_grow_capacity", lambda n: int(n))
    pipe = FramePipeline(model, ts[lo], rk, n=2)
    monkeypatch.undo()
    seq = [lo, hi, hi, lo, hi]
    res = list(pipe.render([ts[j] for j in seq]))
    assert pipe.rerenders >= 1
    refs = {j: _eager(model, ts[j], rk) for j in (lo, hi)}
    for i, j in enumerate(seq):
        for k in ("rgb_marched", "depth", "weights"):
            assert torch.equal(res[i][k], refs[j][k].cpu().reshape(res[i][k].shape)), (i, k)


def test_render_viewpoints_in_flight_equals_serial(dev, tmp_path):
    """harness.render_viewpoints over 8 views at distinct times: 3 frames in flight (one model, its
    cached pipeline) returns exactly the images of the one-view-at-a-time path, and the PNGs match."""
    from apn_amd import harness as Hn
    scene, model = _scene_model(dev)
    rk = {k: v for k, v in scene.render_kwargs(dev).items() if k not in ("rays_o", "rays_d", "viewdirs")}
    n = 8
    poses = torch.stack([scene.c2w.float()] * n)
    poses[:, 0, 3] += torch.linspace(0, 0.1, n)
    HW = np.array([[scene.cfg.H, scene.cfg.W]] * n)
    Ks = torch.stack([scene.K.float()] * n)
    times = [scene.cfg.t + 0.02 * i for i in range(n)]
    kw = dict(test_times=times, verbose=False, inverse_y=bool(rk.get("inverse_y", False)))
    d1, d3 = tmp_path / "serial", tmp_path / "flight"
    d1.mkdir(), d3.mkdir()
    a = Hn.render_viewpoints(model, poses, HW, Ks, False, dict(rk), savedir=str(d1), in_flight=1, **kw)
    b = Hn.render_viewpoints(model, poses, HW, Ks, False, dict(rk), savedir=str(d3), in_flight=3, **kw)
    for x, y in zip(a[:3], b[:3]):
        assert x.shape == y.shape and np.array_equal(x, y)
    for i in range(n):
        assert (d1 / f"img_{i:03d}.png").read_bytes() == (d3 / f"img_{i:03d}.png").read_bytes()
    # the pipeline is cached on the model while its parameters are unchanged ...
    from apn_amd.pipeline import cached_pipeline
    assert len(model._pipelines) == 1
    pipe = next(iter(model._pipelines.values()))[1]
    c = Hn.render_viewpoints(model, poses, HW, Ks, False, dict(rk), in_flight=3, **kw)
    assert next(iter(model._pipelines.values()))[1] is pipe and np.array_equal(c[0], b[0])
    # ... and captured again after a parameter update (in place: the version moves)
    with torch.no_grad():
        model.feat_net[2][0].weight.mul_(1.01)
    d = Hn.render_viewpoints(model, poses, HW, Ks, False, dict(rk), in_flight=3, **kw)
    e = Hn.render_viewpoints(model, poses, HW, Ks, False, dict(rk), in_flight=1, **kw)
    assert next(iter(model._pipelines.values()))[1] is not pipe
    assert np.array_equal(d[0], e[0]) and not np.array_equal(d[0], b[0])
    del cached_pipeline


def test_render_viewpoints_pageable_stacks_equal_pinned(dev, monkeypatch):
    """A sweep whose result stacks exceed harness.PINNED_STACK_BYTES gets pageable numpy stacks
    filled through the pipeline's pinned slots (no pinned allocation the size of the sweep): the
    images are the same as with the pinned stacks."""
    from apn_amd import harness as Hn
    scene, model = _scene_model(dev)
    rk = {k: v for k, v in scene.render_kwargs(dev).items() if k not in ("rays_o", "rays_d", "viewdirs")}
    n = 7
    poses = torch.stack([scene.c2w.float()] * n)
    poses[:, 1, 3] += torch.linspace(0, 0.1, n)
    HW = np.array([[scene.cfg.H, scene.cfg.W]] * n)
    Ks = torch.stack([scene.K.float()] * n)
    kw = dict(test_times=[scene.cfg.t + 0.03 * i for i in range(n)], verbose=False,
              inverse_y=bool(rk.get("inverse_y", False)), in_flight=3)
    a = Hn.render_viewpoints(model, poses, HW, Ks, False, dict(rk), **kw)
    monkeypatch.setattr(Hn, "PINNED_STACK_BYTES", 0)
    b = Hn.render_viewpoints(model, poses, HW, Ks, False, dict(rk), **kw)
    for x, y in zip(a[:3], b[:3]):
        assert x.shape == y.shape and np.array_equal(x, y)


def test_held_pipeline_recaptures_after_weight_update(dev):
    """A FramePipeline held across a weight update: an eager frame after the update
    re-projects the shared layer-1 projection P with the new weights while the pipeline's
    workspaces still hold the old packed weights; the next submit must capture again, not replay a
    mix of the two models -- every later frame equals the eager frame of the updated model."""
    from apn_amd.pipeline import FramePipeline
    scene, model = _scene_model(dev)
    rk = scene.render_kwargs(dev)
    t = torch.tensor([scene.cfg.t], device=dev)
    pipe = FramePipeline(model, t, rk, n=2, readback=("rgb_marched", "depth", "weights"))
    old = pipe.submit(t).result()
    with torch.no_grad():
        model.feat_net[2][0].weight.mul_(1.02)
        model.rgbnet.views_linears[0].bias.add_(0.05)
    ref = _eager(model, t, rk)
    got = [pipe.submit(t) for _ in range(3)]
    for h in got:
        r = h.result()
        for k in ("rgb_marched", "depth", "weights"):
            assert torch.equal(r[k], ref[k].cpu().reshape(r[k].shape)), k
    assert not torch.equal(old["rgb_marched"], got[0].result()["rgb_marched"])


def test_cached_pipeline_follows_render_settings(dev):
    """cached_pipeline keys on the model's plain render settings too: changing
    fast_color_thres between two sweeps captures a new pipeline instead of replaying the old one."""
    from apn_amd.pipeline import cached_pipeline
    scene, model = _scene_model(dev)
    rk = scene.render_kwargs(dev)
    t = torch.tensor([scene.cfg.t], device=dev)
    p1 = cached_pipeline(model, t, rk, n=2, readback=("rgb_marched",))
    assert cached_pipeline(model, t, rk, n=2, readback=("rgb_marched",)) is p1
    thr = model.fast_color_thres
    model.fast_color_thres = 0.2
    try:
        p2 = cached_pipeline(model, t, rk, n=2, readback=("rgb_marched",))
        assert p2 is not p1
        r = p2.submit(t).result()
        ref = _eager(model, t, rk)
        assert torch.equal(r["rgb_marched"], ref["rgb_marched"].cpu().reshape(r["rgb_marched"].shape))
    finally:
        model.fast_color_thres = thr
