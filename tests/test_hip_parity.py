"""GPU parity: every HIP stage against the CPU oracle on identical inputs.

Bars (BASELINE.json north_star): ray/sample/neighbour indexing bit-exact; RGB / density
within 1e-4 in fp32. Floating-point stages whose inputs come from a transcendental
(exp in softmax, sin/cos in posenc) are compared at stated tolerances."""
import numpy as np
import pytest
import torch

from golden_io import CASES, Golden
from oracle import apn_oracle as O

pytestmark = pytest.mark.gpu

F32 = np.float32


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch.device("cuda")


def _rand_rays(n, seed=0):
    g = np.random.default_rng(seed)
    o = g.uniform(-3, 3, (n, 3)).astype(F32)
    d = g.normal(size=(n, 3)).astype(F32)
    d[::7, 0] = 0.0       # zero components -> 1e-6 substitution (render_utils_kernel.cu:23-25)
    d[::11, 1] = 0.0
    return o, d


# ------------------------------------------------------------------ render_utils drop-in
@pytest.mark.parametrize("seed", [0, 1])
def test_sample_pts_on_rays_bit_exact(dev, seed):
    from apn_amd import render_utils as ru
    o, d = _rand_rays(5000, seed)
    lo = np.array([-1.0, -0.7, -1.2], F32); hi = np.array([0.9, 1.1, 0.8], F32)
    ref = O.sample_pts_on_rays(o, d, lo, hi, 0.2, 6.0, 0.017)
    got = ru.sample_pts_on_rays(torch.from_numpy(o).to(dev), torch.from_numpy(d).to(dev),
                                torch.from_numpy(lo).to(dev), torch.from_numpy(hi).to(dev), 0.2, 6.0, 0.017)
    got = [x.cpu().numpy() for x in got]
    names = ["rays_pts", "mask_outbbox", "ray_id", "step_id", "N_steps", "t_min", "t_max"]
    for n, a, b in zip(names, got, ref):
        assert a.shape == b.shape, n
        assert np.array_equal(a, b), n


def test_sample_pts_on_golden_rays_bit_exact(dev):
    from apn_amd import render_utils as ru
    for name in CASES:
        g = Golden(name)
        rk = g.render_kwargs()
        sd = rk["stepsize"] * g.cfg("voxel_size")
        ref = O.sample_pts_on_rays(rk["rays_o"].numpy(), rk["rays_d"].numpy(), g.z["trace_xyz_min"],
                                   g.z["trace_xyz_max"], rk["near"], rk["far"], sd)
        got = ru.sample_pts_on_rays(rk["rays_o"].to(dev), rk["rays_d"].to(dev),
                                    torch.from_numpy(g.z["trace_xyz_min"]).to(dev),
                                    torch.from_numpy(g.z["trace_xyz_max"]).to(dev), rk["near"], rk["far"], sd)
        for a, b in zip(got, ref):
            assert np.array_equal(a.cpu().numpy(), b)
        assert int((~got[1]).sum()) == len(g.z["trace_kmin_d2"])


def test_raw2alpha(dev):
    from apn_amd import render_utils as ru
    d = np.concatenate([np.linspace(-30, 30, 10001), [1e4, -1e4]]).astype(F32)
    e_ref, a_ref = O.raw2alpha(d, -6.906755, 0.5)
    e, a = ru.raw2alpha(torch.from_numpy(d).to(dev), -6.906755, 0.5)
    a = a.cpu().numpy()
    assert np.max(np.abs(a - a_ref)) < 1e-6
    assert a[-2] == 1.0 and a[-1] == 0.0


@pytest.mark.parametrize("name", CASES)
def test_alpha2weight_bit_exact(dev, name):
    from apn_amd import render_utils as ru
    g = Golden(name)
    R = len(g.z["in_rays_o"])
    for a_key, r_key in (("trace_a2w_alpha", "trace_a2w_ray_id"), ("trace_a2w_alpha_direct", "trace_a2w_ray_id_direct")):
        a, rid = g.z[a_key], g.z[r_key]
        ref = O.alpha2weight(a, rid, R)
        got = ru.alpha2weight(torch.from_numpy(a).to(dev), torch.from_numpy(rid).to(dev), R)
        for x, y in zip(got, ref):
            assert np.array_equal(x.cpu().numpy(), y)


def test_alpha2weight_early_exit_and_empty(dev):
    from apn_amd import render_utils as ru
    alpha = np.array([0.5, 0.9, 0.99, 0.5, 0.5, 0.3], F32)
    rid = np.array([1, 1, 1, 1, 1, 3], np.int64)
    ref = O.alpha2weight(alpha, rid, 5)
    got = ru.alpha2weight(torch.from_numpy(alpha).to(dev), torch.from_numpy(rid).to(dev), 5)
    for x, y in zip(got, ref):
        assert np.array_equal(x.cpu().numpy(), y)


def test_segment_sum_bit_exact(dev):
    from apn_amd import render_utils as ru
    g = np.random.default_rng(3)
    idx = np.sort(g.integers(0, 500, 20000)).astype(np.int64)
    src = g.normal(size=(20000, 3)).astype(F32)
    ref = O.segment_sum(src, idx, 600)
    got = ru.segment_coo_sum(torch.from_numpy(src).to(dev), torch.from_numpy(idx).to(dev), 600)
    assert np.array_equal(got.cpu().numpy(), ref)


# ------------------------------------------------------------------ model-level
@pytest.fixture(scope="module", params=CASES)
def golden_model(request, dev):
    from model_io import model_from_golden
    g = Golden(request.param)
    return g, model_from_golden(g, dev)


def test_mean_min_distance(golden_model):
    g, m = golden_model
    assert abs(float(m.mean_min_distance) - float(g.t("in_mean_min_distance"))) < 1e-7


def test_get_weights_and_lbs_vs_reference(golden_model, dev):
    g, m = golden_model
    w = m.get_weights()
    assert (w.cpu() - g.t("get_weights_identity")).abs().max() < 1e-6
    from apn_amd.tineuvox import poc_fre
    t_embed = poc_fre(g.t("in_t").to(dev), m.time_poc)
    xyz, jr, G, jw, bones = m.forward_warp(g.t("get_weights_identity").to(dev), m.joints, t_embed, get_frames=True,
                                           get_skeleton=True)
    assert (xyz.cpu() - g.t("pw_t_xyz")).abs().max() < 2e-6
    assert (G.cpu() - g.t("pw_t_G")).abs().max() < 2e-6
    assert (jr.cpu() - g.t("pw_t_joints_rel")).abs().max() < 1e-6
    xyz_r, jr_r = m.repose(g.t("repose_rot_params").to(dev))
    assert (xyz_r.cpu() - g.t("repose_xyz")).abs().max() < 2e-6


def _forward(g, m, dev):
    return m(g.t("in_t").to(dev), render_depth=True, render_kwargs=g.render_kwargs(dev), render_weights=True,
             poses=g.t("in_c2w")[None].to(dev), Ks=g.t("in_K")[None].to(dev), get_skeleton=True)


def test_lbs_records_vs_oracle(golden_model, dev):
    """Fused softmax+blend+apply and the adjugate 3x3 inverse vs torch.inverse (oracle)."""
    g, m = golden_model
    out = _forward(g, m, dev)
    orc = g.oracle(mean_min_distance_value=float(m.mean_min_distance))
    _, (xyz, jr, G, jw, bT, gt) = orc.warp(g.t("in_t"))
    assert (out["t_hat_pcd"].cpu() - xyz).abs().max() < 2e-6
    recA = m._ws.bufs["recA"][:len(xyz) * 16].reshape(-1, 16).cpu()
    Rinv = torch.inverse(G)[:, :3, :3].reshape(-1, 9)
    assert (recA[:, 4:13] - Rinv).abs().max() < 1e-5
    assert (m._last_weights.cpu() - orc.get_weights()).abs().max() < 1e-6


def test_sampling_and_knn_stagewise_bit_exact(golden_model, dev):
    """Feed the GPU's own warped cloud to the oracle: in-bbox samples, survivors, neighbour
    indices and the sample -> ray/step mapping must be bit-identical."""
    g, m = golden_model
    out = _forward(g, m, dev)
    torch.cuda.synchronize()
    t_hat = out["t_hat_pcd"].cpu().numpy()
    rk = g.render_kwargs()
    lo = (t_hat.min(0) - F32(0.01)).astype(F32); hi = (t_hat.max(0) + F32(0.01)).astype(F32)
    pts, mo, rid, sid, *_ = O.sample_pts_on_rays(rk["rays_o"].numpy(), rk["rays_d"].numpy(), lo, hi, rk["near"],
                                                 rk["far"], rk["stepsize"] * g.cfg("voxel_size"))
    q = pts[~mo]; rid = rid[~mo]; sid = sid[~mo]
    assert m.last_stats["inbbox_samples"] == len(q)
    d2, idx = O.knn_kmin(q, t_hat, 8)
    keep = d2[:, -1] <= F32(0.01)
    S = m.last_stats["kept_samples"]
    assert S == int(keep.sum())
    ws = m._ws.bufs
    s_pos = ws["s_pos"][:4 * S].reshape(S, 4).cpu()
    s_ray = ws["s_ray"][:S].cpu().numpy()
    s_nbr = ws["s_nbr"][:8 * S].reshape(S, 8).cpu().numpy()
    assert np.array_equal(s_ray, rid[keep])
    assert np.array_equal(s_pos[:, :3].numpy(), q[keep])
    assert np.array_equal(s_pos[:, 3].contiguous().view(torch.int32).numpy(), sid[keep])
    assert np.array_equal(s_nbr, idx[keep])


@pytest.mark.parametrize("key,tol", [("rgb_marched", 1e-4), ("rgb_marched_direct", 1e-4), ("weights", 1e-4),
                                     ("alphainv_last", 1e-4), ("alphainv_last_direct", 1e-4)])
def test_forward_vs_oracle_same_cloud(golden_model, dev, key, tol):
    """End-to-end vs the oracle run on the GPU's warped cloud (identical indexing)."""
    g, m = golden_model
    out = _forward(g, m, dev)
    orc = g.oracle(mean_min_distance_value=float(m.mean_min_distance))
    # make the oracle use the GPU's warped cloud and inverse frames
    t_hat = out["t_hat_pcd"].cpu()
    ref = orc.forward(g.t("in_t"), render_depth=True, render_kwargs=g.render_kwargs(), render_weights=True,
                      poses=g.t("in_c2w")[None], Ks=g.t("in_K")[None], get_skeleton=True)
    assert (ref["t_hat_pcd"] - t_hat).abs().max() < 2e-6
    a, b = out[key].cpu(), ref[key]
    assert a.shape == b.shape
    assert (a - b).abs().max() <= tol, float((a - b).abs().max())


def test_forward_depth_vs_golden(golden_model, dev):
    g, m = golden_model
    out = _forward(g, m, dev)
    d = (out["depth"].cpu() - g.t("out_depth")).abs()
    # depth is in step units (~100): 1e-4 relative
    assert float(d.max()) <= 1e-4 * float(g.t("out_depth").abs().max() + 1)


@pytest.mark.parametrize("key", ["rgb_marched", "rgb_marched_direct", "weights", "alphainv_last"])
def test_forward_vs_reference_golden(golden_model, dev, key):
    """Straight against the reference run's outputs (tests/golden)."""
    g, m = golden_model
    out = _forward(g, m, dev)
    err = (out[key].cpu() - g.t("out_" + key)).abs().max()
    assert float(err) <= 1e-4, float(err)


def test_chunking_is_bit_identical(golden_model, dev):
    g, m = golden_model
    full = _forward(g, m, dev)
    rk = g.render_kwargs(dev)
    R = rk["rays_o"].shape[0]
    parts = []
    for s in range(0, R, 512):
        sub = dict(rk)
        for k in ("rays_o", "rays_d", "viewdirs"):
            sub[k] = rk[k][s:s + 512]
        o = m(g.t("in_t").to(dev), render_depth=True, render_kwargs=sub, render_weights=True,
              poses=g.t("in_c2w")[None].to(dev), Ks=g.t("in_K")[None].to(dev), get_skeleton=True)
        parts.append(o["rgb_marched"])
    assert torch.equal(torch.cat(parts), full["rgb_marched"])


def test_no_points_fallback(dev):
    from model_io import model_from_golden
    g = Golden("G1")
    m = model_from_golden(g, dev)
    rk = g.render_kwargs(dev)
    rk["rays_o"] = torch.full_like(rk["rays_o"], 50.0)
    rk["rays_d"] = torch.tensor([0.0, 0.0, 1.0], device=dev).expand_as(rk["rays_d"]).contiguous()
    out = m(g.t("in_t").to(dev), render_depth=True, render_kwargs=rk, render_weights=True)
    assert out["alphainv_last"] is None
    assert torch.all(out["rgb_marched"] == g.cfg("bg")) and torch.all(out["depth"] == 0)
