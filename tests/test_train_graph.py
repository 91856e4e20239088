"""The captured warp stage of the training step (apn_amd.train.warp_stage: skeleton + fused LBS +
pose embedding replayed as a forward and a backward HIP graph) against the eager composition it
captures: the step's outputs and every parameter gradient agree, on the first replay (capture)
and on later replays after optimizer updates, and the regularisers that read the pose state
(transformation regulariser: prev_thetas / prev_global_t) still receive gradients."""
import pytest
import torch

pytestmark = [pytest.mark.gpu, pytest.mark.autograd]


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
    return float(loss), out["t_hat_pcd"].detach().clone(), grads


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
            scale = float(ge[k].abs().max().clamp_min(1e-30))
            err = float((ge[k] - gg[k]).abs().max()) / scale
            assert err < 1e-4, (it, k, err)
        assert "forward_warp.transform_net.net.0.weight" in gg
        with torch.no_grad():   # an optimizer-like in-place update: the graph reads the new values
            for p in model.parameters():
                if p.grad is not None:
                    p.add_(p.grad, alpha=-1e-3)
