"""Precision of the neighbour-MLP stage on weights and features that are
NOT fp16-representable, against the fp32 CPU oracle (temporalpoints.py:452-519; oracle
feat_net / rgbnet restate the reference's torch expressions).

The golden scenes (G1-G3) round every weight and feature to fp16 for compact fixtures, which
zeroes the lo(w) halves of the default 3-term fp16-split kernel (hi*hi + hi*lo + lo*hi). These
cases use PyTorch's default-init weights and N(0, 0.5^2) features as they come, then:

* ``w1e-2`` / ``w10``: every feat_net weight and bias scaled by 1e-2 / 10 (lo halves of the
  1e-2 weights are fp16 subnormals; x10 grows the layer-4 activations to ~1e3);
* ``act8192``: feat_net.0 and every feat_net bias x 8192, densitynet and rgbnet.feature_linears
  weights / 8192 -- the same function (LeakyReLU is positively homogeneous) with activations
  pushed to ~1e4;
* ``overflow``: the same with 2^17 -- layer-1 activations ~1.7e5 exceed fp16: the kernel's
  range guard must route the launch to the FP32 MFMA kernel (apn_point_mlp), still within the
  bar, and report it through the range flag.

Bar (north_star: RGB/density within 1e-4 fp32): alpha and rgb within 1e-5, the direct blend
within 1e-6, the weight-vis colour within 1e-5 -- the same bar as the golden stage test."""
import numpy as np
import pytest
import torch

from oracle import apn_oracle as O

pytestmark = pytest.mark.gpu

F32 = np.float32

FEAT_NET = ("feat_net.0", "feat_net.2.0", "feat_net.3.0", "feat_net.4")
MODES = {"plain": None, "w1e-2": 1e-2, "w10": 10.0, "act8192": 8192.0, "overflow": 2.0 ** 17}


def rescale(params, mode):
    st = {k: v.clone() for k, v in params.items()}
    c = MODES[mode]
    if mode in ("w1e-2", "w10"):
        for k in st:
            if k.split(".weight")[0].split(".bias")[0] in FEAT_NET:
                st[k] = st[k] * c
    elif mode in ("act8192", "overflow"):
        for k in ("feat_net.0.weight", "feat_net.0.bias", "feat_net.2.0.bias", "feat_net.3.0.bias", "feat_net.4.bias"):
            st[k] = st[k] * c
        st["densitynet.weight"] = st["densitynet.weight"] / c
        st["rgbnet.feature_linears.weight"] = st["rgbnet.feature_linears.weight"] / c
    return st


def scene_for(camera):
    from apn_amd import synthetic as S
    if camera == "dnerf":
        cfg = S.SceneConfig("prec dnerf 48x48 4k pts 8 bones", 4000, 8, 48, 48)
    else:
        cfg = S.SceneConfig("prec zju 40x40 3k pts 24 bones pose-emb 64", 3000, 24, 40, 40, camera="zju",
                            pose_embedding_dim=64)
    assert not cfg.fp16_exact
    return S.make_scene(cfg)


def run_mlp_stage(dev, m, orc, variant, render_kwargs, t):
    """apn_point_mlp (through the C-ABI) on the oracle's own kept samples, neighbour lists and
    records -> (out12 [S,12] on the CPU, oracle trace, range-flag)."""
    from apn_amd import _lib as L
    from apn_amd.ops import feat_project, mlp_range_fallback, pack_mlp_weights
    from test_hip_parity import _records
    colors = m._joint_colors(dev).cpu()
    orc.forward(t, render_depth=True, render_kwargs=render_kwargs, render_weights=True, perm=m.last_palette_perm)
    tr = orc.trace
    t_hat = tr["t_hat_pcd"]
    recA, recB = _records(orc, t_hat, colors)
    S = len(tr["s_i"])
    assert S > 100, S
    s_pos = np.concatenate([tr["pts"], tr["step_id"].astype(np.int32).view(F32)[:, None]], 1).astype(F32)
    args = [torch.from_numpy(s_pos).to(dev), torch.from_numpy(tr["ray_id"].astype(np.int32)).to(dev),
            torch.from_numpy(tr["s_i"].astype(np.int32)).to(dev)]
    ns = torch.tensor([S], dtype=torch.int32, device=dev)
    pe = tr["pose_embedding"].to(dev) if tr["pose_embedding"] is not None else None
    layers = [m.feat_net[0], m.feat_net[2][0], m.feat_net[3][0], m.feat_net[4]]
    wbuf = pack_mlp_weights(layers, m.densitynet, m.rgbnet, pe)
    feat = feat_project(m.canonical_feat, wbuf)
    vd = render_kwargs["viewdirs"].to(dev)
    recA_d, recB_d = recA.to(dev), recB.to(dev)
    out12 = torch.full((S, 12), float("nan"), device=dev)
    prev = L.load().apn_set_mlp_variant(variant)
    try:
        L.call("apn_point_mlp", L.ptr(args[0]), L.ptr(args[1]), L.ptr(args[2]), S, L.ptr(ns), L.ptr(recA_d),
               L.ptr(recB_d), L.ptr(feat), 128, L.ptr(vd), None, L.ptr(wbuf), 1e-6, float(orc.act_shift), 0.5, 0,
               L.ptr(out12), L.stream_ptr(dev))
        o = out12.cpu()
    finally:
        L.load().apn_set_mlp_variant(prev)
    return o, tr, mlp_range_fallback(wbuf)


def mlp_stage_f64(orc, tr, viewdirs):
    """alpha / rgb of the kept samples in float64 from the reference's own fp32 inputs: rel_p,
    to_nn and rel_c = Rinv[s_i] rel_p exactly as the (fp32) reference forms them
    (temporalpoints.py:446-447, 478-480), then the posenc, feat_net, IDW sum, densitynet,
    raw2alpha and rgbnet (temporalpoints.py:481-515) in float64."""
    d = torch.float64
    s_i = torch.from_numpy(tr["s_i"])
    K = s_i.shape[1]
    rel_p = torch.from_numpy(tr["pts"])[:, None, :] - tr["t_hat_pcd"][s_i, :]
    to_nn = (rel_p ** 2).sum(-1)
    Rk = tr["Rinv"][s_i, :, :][..., :3, :3]
    rel_c = torch.bmm(Rk.reshape(-1, 3, 3), rel_p.reshape(-1, 3).unsqueeze(-1)).squeeze(-1)
    st = {k: v.to(d) for k, v in orc.nets.items()}
    w = 1 / (to_nn.to(d) + 1e-6)
    w = (w / w.sum(-1, keepdim=True)).unsqueeze(-1)
    x = [O.poc_fre(rel_c.to(d), orc.pos_poc.to(d)), orc.feat[s_i].reshape(-1, orc.feat.shape[-1]).to(d)]
    if tr["pose_embedding"] is not None:
        x.append(tr["pose_embedding"].to(d).expand(len(x[0]), -1))
    h = (O.feat_net(torch.cat(x, -1), st).reshape(len(s_i), K, -1) * w).sum(1)
    dens = O._lin(h, st, "densitynet").squeeze(-1)
    alpha = 1 - (1 + torch.exp(dens + orc.act_shift)) ** (-0.5)
    views = O.poc_fre(viewdirs.to(d), orc.view_poc.to(d))[torch.from_numpy(tr["ray_id"])]
    rgb = torch.sigmoid(O.rgbnet(h, views, st))
    return alpha, rgb


def check_stage(o, tr, tag, f64=None):
    """alpha/rgb: within 1e-5 of the fp32 oracle -- or, when the fp32 oracle itself is further
    than 5e-6 from the float64 evaluation (ill-conditioned scaled networks), within
    max(1e-5, 2x the fp32 oracle's own error) of float64: as accurate as the reference's own fp32
    torch arithmetic. Direct blend (no MLP) 1e-6, weight-vis colour 1e-5 vs the fp32 oracle."""
    da = float((o[:, 3] - tr["alpha"]).abs().max())
    dr = float((o[:, 0:3] - tr["rgbs"]).abs().max())
    dad = float((o[:, 7] - tr["alpha_direct"]).abs().max())
    drd = float((o[:, 4:7] - tr["rgbs_direct"]).abs().max())
    dc = float((o[:, 8:11] - torch.from_numpy(tr["col"])).abs().max())
    worst = int((o[:, 0:3] - tr["rgbs"]).abs().max(-1)[0].argmax())
    tag += (f" [worst rgb sample {worst}: gpu {o[worst, 0:3].tolist()} oracle {tr['rgbs'][worst].tolist()} "
            f"ray {int(tr['ray_id'][worst])}]")
    msg = (f"{tag}: vs fp32 oracle max|d alpha| {da:.2e} max|d rgb| {dr:.2e} direct {dad:.1e}/{drd:.1e} "
           f"col {dc:.1e} (alpha range {float(tr['alpha'].min()):.3g}..{float(tr['alpha'].max()):.3g})")
    assert torch.isfinite(o).all()
    if f64 is not None:
        a64, r64 = f64
        ga = float((o[:, 3].double() - a64).abs().max()); oa = float((tr["alpha"].double() - a64).abs().max())
        gr = float((o[:, 0:3].double() - r64).abs().max()); orr = float((tr["rgbs"].double() - r64).abs().max())
        msg += f"; vs float64: gpu alpha {ga:.2e} rgb {gr:.2e}, fp32 oracle alpha {oa:.2e} rgb {orr:.2e}"
        print(msg)
        if max(oa, orr) > 5e-6:
            assert ga <= max(1e-5, 2 * oa) and gr <= max(1e-5, 2 * orr), msg
        else:
            assert da < 1e-5 and dr < 1e-5, msg
    else:
        print(msg)
        assert da < 1e-5 and dr < 1e-5, msg
    assert dad < 1e-6 and drd < 1e-6, msg
    assert dc < 1e-5, msg


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch.device("cuda")


@pytest.mark.parametrize("variant", [0, 1, 4], ids=["split3xfp16", "fp32", "split3xfp16_64rows"])
@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("camera", ["dnerf", "zju"])
def test_mlp_stage_non_fp16_exact(dev, camera, mode, variant):
    from apn_amd import harness, synthetic as S
    scene = scene_for(camera)
    scene.params = rescale(scene.params, mode)
    m = harness.build_model(scene, dev)
    m.palette_perm_device = "cpu"
    # the weights really are not fp16-representable (lo halves non-zero)
    w2 = m.feat_net[2][0].weight.detach()
    assert float((w2 - w2.half().float()).abs().max()) > 0
    st = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    orc = O.OracleModel(st, m.canonical_pcd.cpu(), m.bones, stepsize=S.STEPSIZE, voxel_size=S.VOXEL_SIZE,
                        fast_color_thres=S.FAST_COLOR_THRES, pose_embedding_dim=m.pose_embedding_dim,
                        act_shift=float(m.tineuvox.act_shift), voxel_size_ratio=float(m.tineuvox.voxel_size_ratio),
                        mean_min_distance_value=float(m.mean_min_distance))
    t = torch.tensor([scene.cfg.t])
    rk = scene.render_kwargs("cpu")
    with torch.no_grad():
        o, tr, fallback = run_mlp_stage(dev, m, orc, variant, rk, t)
        f64 = mlp_stage_f64(orc, tr, rk["viewdirs"])
    check_stage(o, tr, f"{camera}/{mode}/v{variant} fallback={fallback}", f64)
    if variant in (0, 4):
        # the guard fires exactly when a split value leaves the fp16 range
        assert fallback == (mode == "overflow"), fallback


def test_range_flag_is_sticky_until_resplit(dev):
    """After an overflowing launch the flag stays set (later launches with the same weights go
    straight to FP32: the split kernel's workgroups exit at once); re-packing the weights clears it."""
    from apn_amd import harness, synthetic as S
    from apn_amd.ops import mlp_range_fallback
    scene = scene_for("dnerf")
    scene.params = rescale(scene.params, "overflow")
    m = harness.build_model(scene, dev)
    rk = scene.render_kwargs(dev)
    t = torch.tensor([scene.cfg.t], device=dev)
    with torch.no_grad():
        a = m(t, render_kwargs=rk)["rgb_marched"].clone()
        wbuf = m._ws.bufs["mlp_w"]
        assert mlp_range_fallback(wbuf)
        b = m(t, render_kwargs=rk)["rgb_marched"].clone()
        assert torch.equal(a, b)
        assert mlp_range_fallback(wbuf)
        # weights back in range -> repacked (parameter versions change) -> flag cleared
        for nm in ("feat_net.0.weight", "feat_net.0.bias", "feat_net.2.0.bias", "feat_net.3.0.bias",
                   "feat_net.4.bias"):
            p = dict(m.named_parameters())[nm]
            p.mul_(2.0 ** -17)
        m.densitynet.weight.mul_(2.0 ** 17)
        m.rgbnet.feature_linears.weight.mul_(2.0 ** 17)
        c = m(t, render_kwargs=rk)["rgb_marched"]
        assert not mlp_range_fallback(wbuf)
        assert float((c - a).abs().max()) < 1e-4
