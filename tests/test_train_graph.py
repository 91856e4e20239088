"""The captured warp stage of the training step (apn_amd.train.warp_stage: skeleton + fused LBS +
pose embedding replayed as a forward and a backward HIP graph) against the eager composition it
captures: the step's outputs and every parameter gradient agree, on the first replay (capture)
and on later replays after optimizer updates, and the regularisers that read the pose state
(transformation regulariser: prev_thetas / prev_global_t) still receive gradients."""
import pytest
import torch

# a parameter's AccumulateGrad node reached from another stream is an error (train.graph_callable)
pytestmark = [pytest.mark.gpu, pytest.mark.autograd, pytest.mark.filterwarnings("error:The AccumulateGrad node")]


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch.device("cuda")


def _step(model, t, sub, target):
    model.zero_grad(set_to_none=True)
    out = model(t, render_kwargs=sub)
    loss = torch.nn.functional.mse_loss(out["rgb_marched"], target)
    loss = loss + 0.1 * model.get_transformation_regularisation_loss()
    loss = loss + 10.0 * model.get_neighbour_weight_tv_loss() + 0.2 * model.get_weight_sparsity_loss()
    loss.backward()
    grads = {k: p.grad.detach().clone() for k, p in model.named_parameters() if p.grad is not None}
    return float(loss.detach()), out["t_hat_pcd"].detach().clone(), grads


@pytest.mark.parametrize("name", ["C1", "G2"])
def test_graphed_warp_stage_equals_eager(dev, name):
    from apn_amd import harness, synthetic as S, train as T
    scene = S.make_scene(name)
    model = harness.build_model(scene, dev)
    rk = scene.render_kwargs(dev)
    g = torch.Generator(device=dev).manual_seed(0)
    sel = torch.randint(0, len(rk["rays_o"]), (4096,), device=dev, generator=g)
    sub = dict(rk)
    for k in ("rays_o", "rays_d", "viewdirs"):
        sub[k] = rk[k][sel]
    t = torch.tensor([scene.cfg.t], device=dev)
    with torch.no_grad():
        target = model(t + 0.1, render_kwargs=sub)["rgb_marched"].clone()
    assert T.GRAPH_WARP
    for it in range(3):
        T.GRAPH_WARP = False
        try:
            le, xe, ge = _step(model, t, sub, target)
        finally:
            T.GRAPH_WARP = True
        lg, xg, gg = _step(model, t, sub, target)
        assert "_warp_graph" in model.__dict__
        assert torch.equal(xe, xg), it
        assert abs(le - lg) <= 1e-6 * max(1.0, abs(le)), (it, le, lg)
        assert set(ge) == set(gg), set(ge) ^ set(gg)
        for k in ge:
            scale = float(ge[k].detach().abs().max().clamp_min(1e-30))
            err = float((ge[k] - gg[k]).detach().abs().max()) / scale
            assert err < 1e-4, (it, k, err)
        assert "forward_warp.transform_net.net.0.weight" in gg
        with torch.no_grad():   # an optimizer-like in-place update: the graph reads the new values
            for p in model.parameters():
                if p.grad is not None:
                    p.add_(p.grad, alpha=-1e-3)


def _torch_aggregate(ray_pts, s_i, xyz, Rinv, feat, pose, sig, rgb_c, alpha_c, poc, eps):
    """The reference composition (temporalpoints.py:452-494) in torch ops."""
    from apn_amd.tineuvox import poc_fre
    K = 8
    rel_p = ray_pts[:, None, :] - xyz[s_i, :]
    to_nn = (rel_p ** 2).sum(-1)
    w_direct = torch.exp(-(to_nn ** 2) / (2 * sig[s_i] ** 2 + 1e-12))
    w_dd = ((1. / K) * w_direct).unsqueeze(-1)
    w_direct = (w_direct / (w_direct.sum(dim=-1) + 1e-12)[:, None]).unsqueeze(-1)
    rgbd = (w_direct * rgb_c[s_i, :]).sum(dim=1)
    alphad = (w_dd * alpha_c[s_i].unsqueeze(-1)).sum(dim=1).squeeze(-1)
    w = 1 / (to_nn + eps)
    w = w / w.sum(dim=-1)[:, None]
    rel_c = (Rinv[s_i] * rel_p[:, :, None, :]).sum(-1).reshape(-1, 3)
    parts = [poc_fre(rel_c, poc), feat[s_i].reshape(-1, feat.shape[-1])]
    if pose is not None:
        parts.append(pose.expand(len(rel_c), -1))
    return w, rgbd, alphad, torch.cat(parts, -1)


@pytest.mark.parametrize("with_pose", [False, True])
def test_nbr_aggregate_vs_float64_autograd(dev, with_pose):
    """NbrAggregate + IdwSum (apn_nbr_train.hip: the training forward's direct blend, IDW weights,
    rel_c posenc, feat_net input rows and the IDW sum, forward and backward) against the torch
    composition of temporalpoints.py:452-494 run in float64 under autograd, on random clouds with
    shared neighbours (every gradient is a sum over several rows per point)."""
    from apn_amd.train import NbrAggregate, IdwSum, feat_in_columns
    g = torch.Generator().manual_seed(5 + with_pose)
    N, S, F, P, C = 3000, 2500, 32, 7, 16
    xyz = torch.rand(N, 3, generator=g)
    ray_pts = xyz[torch.randint(0, N, (S,), generator=g)] + 0.01 * torch.randn(S, 3, generator=g)
    s_i = torch.randint(0, N, (S, 8), generator=g)
    Rinv = torch.eye(3) + 0.2 * torch.randn(N, 3, 3, generator=g)
    feat = torch.randn(N, F, generator=g)
    pose = torch.randn(1, P, generator=g) if with_pose else None
    sig = 0.01 + 0.02 * torch.rand(N, generator=g)
    rgb_c, alpha_c = torch.rand(N, 3, generator=g), torch.rand(N, generator=g)
    poc = torch.tensor([2.0 ** i for i in range(10)])
    eps = 1e-6
    mats = [xyz, Rinv, feat, pose, sig, rgb_c, alpha_c]
    K = 3 + 60 + F + (P if with_pose else 0)
    proj = torch.randn(K, C, generator=g)
    grads_out = [torch.randn(S, 8, generator=g), torch.randn(S, 3, generator=g), torch.randn(S, generator=g),
                 torch.randn(S, C, generator=g)]

    def run(fn, dtype, device):
        ts = [None if m is None else m.to(device, dtype).requires_grad_(True) for m in mats]
        w, rgbd, ad, fin = fn(ray_pts.to(device, dtype), s_i.to(device), ts[0], ts[1], ts[2], ts[3], ts[4], ts[5], ts[6],
                              poc.to(device, dtype), eps)
        if fn is not _torch_aggregate:   # the padded column layout -> the reference's
            fin = fin[:, feat_in_columns(len(poc), F, P if with_pose else 0, device)]
        out = fin @ proj.to(device, dtype)
        h = IdwSum.apply(w, out) if fn is not _torch_aggregate else (out.reshape(S, 8, -1) * w.unsqueeze(-1)).sum(1)
        loss = sum((a * b.to(device, dtype)).sum() for a, b in zip((w, rgbd, ad, h), grads_out))
        loss.backward()
        return [w, rgbd, ad, fin, h], [None if t is None else t.grad for t in ts]

    outs, grads = run(NbrAggregate.apply, torch.float32, dev)
    routs, rgrads = run(_torch_aggregate, torch.float64, dev)
    touts, tgrads = run(_torch_aggregate, torch.float32, dev)   # fp32 conditioning floor (2^9 posenc)
    rel = lambda a, r: float((a.detach().double() - r.detach()).abs().max() / r.detach().abs().max())
    for i, (a, t, r) in enumerate(zip(outs, touts, routs)):
        assert rel(a, r) <= max(1e-5, 3 * rel(t, r)), (i, rel(a, r), rel(t, r))
    for i, (a, t, r) in enumerate(zip(grads, tgrads, rgrads)):
        if r is None:
            assert a is None
            continue
        assert rel(a, r) <= max(1e-5, 3 * rel(t, r)), (i, rel(a, r), rel(t, r))


@pytest.mark.parametrize("N", [1, 1000, 300_001])
def test_cloud_bbox_equals_torch_min_max(dev, N):
    """apn_cloud_bbox (the training forward's sampling bbox and grid bbox, temporalpoints.py:423-427)
    equals torch's min / max exactly, and its ordered encoding equals ordered_bbox's."""
    from apn_amd.train import cloud_bbox, cloud_min_max, ordered_bbox
    g = torch.Generator().manual_seed(N)
    xyz = (torch.randn(N, 3, generator=g) * torch.tensor([1.0, 0.2, 3.0]) - 0.5).to(dev)
    mm, o = cloud_bbox(xyz)
    lo, hi = cloud_min_max(xyz)
    assert torch.equal(mm, torch.cat([lo, hi]))
    assert torch.equal(o, ordered_bbox(xyz))
