"""GPU parity of the LBS paths the golden render tests do not reach:

* ``get_weights`` with a non-trivial merge (temporalpoints.py:401-414; the state after
  ``simplify_skeleton``): the fused softmax + merge-by-rule of ``apn_lbs_skin`` on the render path
  and on the record-free repose path, against the reference's own ``get_weights_merged`` fixture
  and the oracle's merged LBS;
* the C5 configuration at full size (BASELINE configs[4]: 1M points, 48 bones, the repose sweep
  of run.py:1364-1377) through ``k_lbs_skin_mfma``'s persistent grid-stride loop: several trips
  per wave, the register ring's clamped prefetch ``min(16 g + n, N - 1)`` and the wave-uniform
  exit. The
  oracle (CPU) checks a strided 50k-point subset plus the last point -- LBS is per point, so a
  subset model is exact."""
import numpy as np
import pytest
import torch

from golden_io import CASES, Golden
from oracle import apn_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch.device("cuda")


def _merged_model(g, dev):
    from model_io import model_from_golden
    m = model_from_golden(g, dev)
    rules = g.t("merge_rules")
    J = m.weights.shape[1]
    assert not torch.equal(rules, torch.arange(J))
    m.flat_merging_rules.copy_(rules.to(dev))
    m.merging_mat = torch.zeros(J, J, J)   # simplify_skeleton's marker (temporalpoints.py:405-410)
    return m, rules


@pytest.mark.parametrize("name", CASES)
def test_merge_rules_render_path_vs_reference(dev, name):
    g = Golden(name)
    m, rules = _merged_model(g, dev)
    ref_w = g.t("get_weights_merged")
    with torch.no_grad():
        assert (m.get_weights().cpu() - ref_w).abs().max() < 1e-6
        out = m(g.t("in_t").to(dev), render_depth=True, render_kwargs=g.render_kwargs(dev), render_weights=True)
    torch.cuda.synchronize()
    # the fused kernel's merged softmax (written for the training losses' _last_weights)
    assert (m._last_weights.cpu() - ref_w).abs().max() < 1e-6
    orc = g.oracle(mean_min_distance_value=g.t("in_mean_min_distance"), merging_rules=rules)
    assert (orc.get_weights() - ref_w).abs().max() < 1e-6
    _, (xyz, *_rest) = orc.warp(g.t("in_t"))
    assert (out["t_hat_pcd"].cpu() - xyz).abs().max() < 2e-6
    assert torch.isfinite(out["rgb_marched"]).all()


@pytest.mark.parametrize("name", CASES)
def test_merge_rules_repose_vs_oracle(dev, name):
    """repose with merge rules takes k_lbs_skin's record-free branch (the quad kernel needs the
    identity rules)."""
    g = Golden(name)
    m, rules = _merged_model(g, dev)
    orc = g.oracle(mean_min_distance_value=0.0, merging_rules=rules)
    rp = g.t("repose_rot_params")
    with torch.no_grad():
        xyz, jr = m.repose(rp.to(dev))
    xo, jo = orc.repose(rp)
    assert (xyz.cpu() - xo).abs().max() < 2e-6
    assert (jr.cpu() - jo).abs().max() < 1e-6


def _subset_oracle(model, idx):
    st = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    for k in ("weights", "canonical_feat", "canonical_alpha", "canonical_rgbs", "direct_eps", "gammas"):
        st[k] = st[k][idx]
    return O.OracleModel(st, model.canonical_pcd.cpu()[idx], model.bones, mean_min_distance_value=0.0)


def test_c5_full_size_repose_vs_oracle_subset(dev):
    from apn_amd import harness, synthetic as S
    scene = S.make_scene("C5")
    N, J = scene.cfg.N, scene.cfg.J
    assert (N, J) == (1_000_000, 48)
    model = harness.build_model(scene, dev)
    idx = torch.cat([torch.arange(0, N, 20), torch.tensor([N - 1])])
    orc = _subset_oracle(model, idx)
    poses = S.repose_sweep(J)
    assert len(poses) == 60
    for k in (3, 29, 47):
        with torch.no_grad():
            xyz, jr = model.repose(poses[k].to(dev))
        xyz = xyz.cpu()
        assert xyz.shape == (N, 3) and torch.isfinite(xyz).all()
        xo, jo = orc.repose(poses[k])
        err = (xyz[idx] - xo).abs().max()
        print(f"C5 pose {k}: max|d xyz| on {len(idx)} points = {float(err):.2e}")
        assert err < 2e-6
        assert (jr.cpu() - jo).abs().max() < 1e-6


def test_c5_repose_is_order_independent(dev):
    """Every lane of the persistent loop writes only its own points: the full-size result does not
    depend on the grid (two launches with different pose histories agree bit for bit)."""
    from apn_amd import harness, synthetic as S
    scene = S.make_scene("C5")
    model = harness.build_model(scene, dev)
    poses = S.repose_sweep(scene.cfg.J)
    with torch.no_grad():
        a = model.repose(poses[10].to(dev))[0].clone()
        model.repose(poses[50].to(dev))
        b = model.repose(poses[10].to(dev))[0]
    assert torch.equal(a, b)
    assert np.isfinite(b.cpu().numpy()).all()


def test_captured_repose_graph_equals_eager(dev):
    """TemporalPoints.capture_repose (skeleton + LBS in one HIP graph, the C5 bench step) replays
    the eager repose bit for bit over several poses of the sweep."""
    from apn_amd import harness, synthetic as S
    scene = S.make_scene(S.SceneConfig("graph repose", 50_000, 48, 0, 0))
    model = harness.build_model(scene, dev)
    poses = S.repose_sweep(48).to(dev)
    step = model.capture_repose(rot_dim=4)
    for k in (0, 7, 31, 59):
        with torch.no_grad():
            xe, je = (v.clone() for v in model.repose(poses[k]))
        xg, jg = step(poses[k])
        torch.cuda.synchronize()
        assert torch.equal(xg, xe) and torch.equal(jg, je), k


def _capture(model, poses, mode):
    """capture_repose in a test mode; batchedN = batched with N poses in flight."""
    return model.capture_repose(sweep=poses, batched=mode.startswith("batched"), pipelined=mode == "pipelined",
                                in_flight=int(mode[7:]) if mode[7:].isdigit() else 1)


def _ready(step, k, res):
    """The step's outputs for pose k on the caller's stream (poses in flight: wait on pose k's stream)."""
    if getattr(step, "streams", None):
        torch.cuda.current_stream().wait_stream(step.streams[k % len(step.streams)])
    return res


@pytest.mark.parametrize("mode", ["batched", "batched2", "batched3", "pipelined", "per_pose"])
def test_captured_repose_sweep_graph(dev, mode):
    """capture_repose(sweep=poses) -- in-order steps, a jump, a wrap-around and rot_params that are
    not a row of the sweep (eager fallback) all equal the eager repose bit for bit. batched (the
    default): every pose's skeleton in one launch per pass over the sweep, one LBS graph per pose;
    pipelined: each step's graph runs the next pose's skeleton beside its LBS; per_pose: one graph
    reading its pose through a device index it advances itself; batched2: batched with two poses in
    flight (pose k on stream k % 2 into output slot k % 2)."""
    from apn_amd import harness, synthetic as S
    scene = S.make_scene(S.SceneConfig("graph repose sweep", 30_000, 48, 0, 0))
    model = harness.build_model(scene, dev)
    poses = S.repose_sweep(48).to(dev).contiguous()
    P = poses.shape[0]
    step = _capture(model, poses, mode)
    order = [0, 1, 2, 3, 17, 18, P - 1, 0, 1, 5]
    for k in order:
        with torch.no_grad():
            xe, je = (v.clone() for v in model.repose(poses[k]))
        xg, jg = step(poses[k])
        torch.cuda.synchronize()
        assert torch.equal(xg, xe) and torch.equal(jg, je), k
    other = poses[3].clone() * 0.5
    with torch.no_grad():
        xe, je = (v.clone() for v in model.repose(other))
    xo, jo = step(other)
    assert torch.equal(xo, xe) and torch.equal(jo, je)
    xg, jg = step(poses[6])   # after the fallback: back on the graph at a new position
    with torch.no_grad():
        xe, je = model.repose(poses[6])
    torch.cuda.synchronize()
    assert torch.equal(xg, xe) and torch.equal(jg, je)


@pytest.mark.parametrize("mode", ["batched", "batched2", "batched3", "pipelined"])
def test_repose_sweep_modified_in_place(dev, mode):
    """The batched sweep computes every pose's skeleton at the start of a pass, the pipelined one
    pose i + 1's during step i; a sweep row changed in place in between must not be skinned from
    the stale skeleton (the step runs the skeleton again)."""
    from apn_amd import harness, synthetic as S
    scene = S.make_scene(S.SceneConfig("graph repose sweep inplace", 20_000, 24, 0, 0))
    model = harness.build_model(scene, dev)
    poses = S.repose_sweep(24).to(dev).contiguous()
    step = _capture(model, poses, mode)
    for k in range(4):
        step(poses[k])
    with torch.no_grad():
        poses[4].mul_(0.5)
    xg, jg = (v.clone() for v in _ready(step, 4, step(poses[4])))
    with torch.no_grad():
        xe, je = model.repose(poses[4])
    torch.cuda.synchronize()
    assert torch.equal(xg, xe) and torch.equal(jg, je)
    for k in range(5, 9):   # and in order again afterwards
        xg, jg = (v.clone() for v in _ready(step, k, step(poses[k])))
        with torch.no_grad():
            xe, je = model.repose(poses[k])
        torch.cuda.synchronize()
        assert torch.equal(xg, xe) and torch.equal(jg, je), k
