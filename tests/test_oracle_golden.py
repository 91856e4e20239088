"""Pin the CPU oracle against golden vectors produced by the reference's own Python
(tests/golden/make_golden.py). Tolerances: the reference itself reproduces its own
PointWarper output only to ~3e-7 across processes (MKL summation order), so float outputs
are compared at 1e-5; indices are compared exactly on identical inputs."""
import numpy as np
import pytest
import torch

from golden_io import CASES, Golden
from oracle import apn_oracle as O


@pytest.fixture(scope="module", params=CASES)
def golden(request):
    return Golden(request.param)


@pytest.fixture(scope="module")
def oracle_run(golden):
    m = golden.oracle()
    out = m.forward(golden.t("in_t"), render_depth=True, render_kwargs=golden.render_kwargs(),
                    render_weights=True, poses=golden.t("in_c2w")[None], Ks=golden.t("in_K")[None],
                    get_skeleton=True)
    return m, out


def test_mean_min_distance(golden, oracle_run):
    m, _ = oracle_run
    assert abs(float(m.mmd) - float(golden.t("in_mean_min_distance"))) < 1e-8


def test_get_weights(golden):
    m = golden.oracle(mean_min_distance_value=golden.t("in_mean_min_distance"))
    assert torch.equal(m.get_weights(), golden.t("get_weights_identity"))
    merged = O.get_weights(m.W, m.theta_weight, golden.t("merge_rules"))
    assert torch.equal(merged, golden.t("get_weights_merged"))


def test_pointwarper_t_path(golden):
    m = golden.oracle(mean_min_distance_value=golden.t("in_mean_min_distance"))
    _, (xyz, jr, G, jw, _, _) = m.warp(golden.t("in_t"))
    assert (xyz - golden.t("pw_t_xyz")).abs().max() < 1e-6
    assert (G - golden.t("pw_t_G")).abs().max() < 1e-6
    assert (jr - golden.t("pw_t_joints_rel")).abs().max() < 1e-6
    assert (jw - golden.t("pw_t_joints_warped")).abs().max() < 1e-6


def test_repose_rot_params_path(golden):
    m = golden.oracle(mean_min_distance_value=golden.t("in_mean_min_distance"))
    xyz, jr = m.repose(golden.t("repose_rot_params"))
    assert (xyz - golden.t("repose_xyz")).abs().max() < 1e-6
    assert (jr - golden.t("repose_joints_rel")).abs().max() < 1e-6


@pytest.mark.parametrize("key,tol", [("rgb_marched", 1e-5), ("rgb_marched_direct", 1e-5),
                                     ("depth", 1e-4), ("weights", 1e-5), ("alphainv_last", 1e-5),
                                     ("alphainv_last_direct", 1e-5), ("t_hat_pcd", 1e-6),
                                     ("joints", 1e-4)])
def test_forward_outputs(golden, oracle_run, key, tol):
    _, out = oracle_run
    a, b = out[key], golden.t("out_" + key)
    assert a.shape == b.shape
    assert (a - b).abs().max() <= tol


def test_sampling_exact_on_reference_bbox(golden):
    """Same bbox as the reference run -> identical in-bbox sample count (index path)."""
    rk = golden.render_kwargs()
    pts, mo, rid, sid, *_ = O.sample_pts_on_rays(
        rk["rays_o"].numpy(), rk["rays_d"].numpy(), golden.z["trace_xyz_min"], golden.z["trace_xyz_max"],
        rk["near"], rk["far"], rk["stepsize"] * golden.cfg("voxel_size"))
    assert int((~mo).sum()) == len(golden.z["trace_kmin_d2"])


def test_knn_exact_on_reference_cloud(golden):
    """Same query points / cloud as the reference run -> bit-identical kNN for survivors."""
    rk = golden.render_kwargs()
    pts, mo, *_ = O.sample_pts_on_rays(
        rk["rays_o"].numpy(), rk["rays_d"].numpy(), golden.z["trace_xyz_min"], golden.z["trace_xyz_max"],
        rk["near"], rk["far"], rk["stepsize"] * golden.cfg("voxel_size"))
    q = pts[~mo]
    d2, idx = O.knn_kmin(q, golden.z["out_t_hat_pcd"], 8)
    ref_d2, ref_idx = golden.z["trace_kmin_d2"], golden.z["trace_kmin_idx"]
    surv = ref_d2[:, -1] <= np.float32(0.01)
    assert np.array_equal(d2[:, -1] <= np.float32(0.01), surv)
    assert np.array_equal(idx[surv], ref_idx[surv])
    assert np.array_equal(d2[surv], ref_d2[surv])


def test_alpha2weight_matches_reference_inputs(golden):
    a = golden.z["trace_a2w_alpha"]; rid = golden.z["trace_a2w_ray_id"]
    R = len(golden.z["in_rays_o"])
    w, T, last, _, _ = O.alpha2weight(a, rid, R)
    assert np.all(np.isfinite(w)) and np.all((last >= 0) & (last <= 1))
    assert np.allclose(last, golden.z["out_alphainv_last"], atol=1e-5)


def test_bbox_sensitivity_of_reference_sampling():
    """Documents a property of the reference path itself: with the sampling bbox fixed, a
    3e-7 perturbation of the warped cloud leaves every kNN survivor unchanged, while letting
    the bbox follow the perturbed cloud (calc_min_max=True) changes the in-bbox sample set."""
    g = Golden("G1")
    t = g.z["out_t_hat_pcd"].astype(np.float32)
    rk = g.render_kwargs()
    sd = rk["stepsize"] * g.cfg("voxel_size")

    def survivors(cloud, lo, hi):
        pts, mo, *_ = O.sample_pts_on_rays(rk["rays_o"].numpy(), rk["rays_d"].numpy(), lo, hi, rk["near"],
                                           rk["far"], sd)
        d2, _ = O.knn_kmin(pts[~mo], cloud, 8)
        return int((d2[:, -1] <= np.float32(0.01)).sum()), int((~mo).sum())

    lo, hi = g.z["trace_xyz_min"], g.z["trace_xyz_max"]
    tp = (t + np.random.default_rng(0).uniform(-3e-7, 3e-7, t.shape)).astype(np.float32)
    assert survivors(tp, lo, hi) == survivors(t, lo, hi)
    lo2 = (tp.min(0) - np.float32(0.01)).astype(np.float32); hi2 = (tp.max(0) + np.float32(0.01)).astype(np.float32)
    assert survivors(tp, lo2, hi2)[1] != survivors(t, lo, hi)[1]


def test_oracle_train_forward_matches_render_and_golden(golden):
    """The oracle's autograd twin (train_pcd path) renders the same image as the
    no-grad oracle, matches the reference's golden render, and its gradients are finite and reach
    every parameter group of the path."""
    m = golden.oracle(mean_min_distance_value=golden.t("in_mean_min_distance"))
    ref = m.forward(golden.t("in_t"), render_kwargs=golden.render_kwargs(), knn_tree=False)
    params = O.oracle_trainable(m)
    out = O.oracle_forward_train(m, golden.t("in_t"), golden.render_kwargs(), knn_tree=False)
    assert (out["rgb_marched"].detach() - ref["rgb_marched"]).abs().max() < 1e-6
    assert (out["rgb_marched_direct"].detach() - ref["rgb_marched_direct"]).abs().max() < 1e-6
    err = (out["rgb_marched"].detach() - golden.t("out_rgb_marched")).abs().max(-1)[0]
    assert float((err > 1e-4).float().mean()) <= 5e-3
    loss = (out["rgb_marched"] - 0.5).pow(2).mean() + (out["rgb_marched_direct"] - 0.5).pow(2).mean()
    loss.backward()
    for k in ("weights", "theta_weight", "joints", "canonical_feat", "canonical_alpha", "canonical_rgbs",
              "direct_eps", "feat_net.0.weight", "densitynet.weight", "rgbnet.views_linears.2.weight",
              "forward_warp.transform_net.net.0.weight"):
        gk = params[k].grad
        assert gk is not None and torch.isfinite(gk).all() and float(gk.abs().max()) > 0, k
