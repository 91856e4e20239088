"""Diagnostics for the stage-wise parity tests (run on the GPU box by hand)."""
import sys

import numpy as np
import torch

sys.path.insert(0, "tests"); sys.path.insert(0, "articulated-point-nerf_amd"); sys.path.insert(0, ".")
import test_hip_parity as T  # noqa: E402
from golden_io import Golden  # noqa: E402
from apn_amd import _lib as L  # noqa: E402
from apn_amd.ops import pack_mlp_weights  # noqa: E402
from model_io import model_from_golden  # noqa: E402

dev = torch.device("cuda")
g = Golden(sys.argv[1] if len(sys.argv) > 1 else "G1")
m = model_from_golden(g, dev)
m.palette_perm_device = "cpu"
t_hat = g.t("out_t_hat_pcd")
colors = m._joint_colors(dev).cpu()
orc, ref = T._oracle_on_cloud(g, t_hat, perm=m.last_palette_perm)
tr = orc.trace
recA, recB = T._records(orc, t_hat, colors)
S = len(tr["s_i"])
s_pos = np.concatenate([tr["pts"], tr["step_id"].astype(np.int32).view(np.float32)[:, None]], 1).astype(np.float32)
a0 = torch.from_numpy(s_pos).to(dev); a1 = torch.from_numpy(tr["ray_id"].astype(np.int32)).to(dev)
a2 = torch.from_numpy(tr["s_i"].astype(np.int32)).to(dev)
ns = torch.tensor([S], dtype=torch.int32, device=dev)
pe = tr["pose_embedding"].to(dev) if tr["pose_embedding"] is not None else None
layers = [m.feat_net[0], m.feat_net[2][0], m.feat_net[3][0], m.feat_net[4]]
wbuf = pack_mlp_weights(layers, m.densitynet, m.rgbnet, pe)
recA_d, recB_d = recA.to(dev), recB.to(dev)
for gb in (0,):
    out12 = torch.zeros(S, 12, device=dev)
    L.call("apn_point_mlp", L.ptr(a0), L.ptr(a1), L.ptr(a2), S, L.ptr(ns), L.ptr(recA_d), L.ptr(recB_d),
           L.ptr(m.canonical_feat.detach().contiguous()), 128, L.ptr(g.t("in_viewdirs").to(dev)), None, L.ptr(wbuf),
           1e-6, float(orc.act_shift), 0.5, gb, L.ptr(out12), L.stream_ptr(dev))
    o = out12.cpu()
    da = (o[:, 3] - tr["alpha"]).abs()
    dr = (o[:, 0:3] - tr["rgbs"]).abs().max(1)[0]
    bad = torch.nonzero(da > 1e-5).flatten()
    print(f"grid_blocks={gb} S={S} alpha maxdiff {float(da.max()):.3e} n_bad={len(bad)} rgb maxdiff {float(dr.max()):.3e}")
    print("  bad idx (first 20):", bad[:20].tolist(), " idx%8:", sorted(set((bad % 8).tolist())))
    dens_ref = tr["density"]
    print("  density range", float(dens_ref.min()), float(dens_ref.max()))
    for i in bad[:5].tolist():
        print("   i", i, "alpha gpu", float(o[i, 3]), "ref", float(tr["alpha"][i]), "dens", float(dens_ref[i]))
    print("  direct a", float((o[:, 7] - tr["alpha_direct"]).abs().max()), "col", float((o[:, 8:11] - torch.from_numpy(tr["col"])).abs().max()))

# composite
R = len(g.z["in_rays_o"])
smp = torch.zeros(S, 12)
smp[:, 0:3] = tr["rgbs"]; smp[:, 3] = tr["alpha"]; smp[:, 4:7] = tr["rgbs_direct"]; smp[:, 7] = tr["alpha_direct"]
smp[:, 8:11] = torch.from_numpy(tr["col"])
sp = np.zeros((S, 4), np.float32); sp[:, 3] = tr["step_id"].astype(np.int32).view(np.float32)
outs = [torch.empty(R, 3, device=dev), torch.empty(R, 3, device=dev), torch.empty(R, device=dev),
        torch.empty(R, 3, device=dev), torch.empty(R, device=dev), torch.empty(R, device=dev)]
rws = torch.empty(2 * R, dtype=torch.int32, device=dev)
smp_d, sp_d = smp.to(dev), torch.from_numpy(sp).to(dev)
L.call("apn_composite", L.ptr(smp_d), L.ptr(sp_d), L.ptr(a1), S, L.ptr(ns), R, 1e-4,
       g.cfg("bg"), *[L.ptr(x) for x in outs], L.ptr(rws), L.stream_ptr(dev))
for o, k in zip(outs, ["rgb_marched", "rgb_marched_direct", "depth", "weights", "alphainv_last", "alphainv_last_direct"]):
    d = (o.cpu() - ref[k]).abs().reshape(R, -1).max(1)[0]
    nb = int((d > 0).sum())
    print(f"composite {k}: n_diff={nb} max={float(d.max()):.3e}")
    if nb:
        r = int(torch.nonzero(d > 0)[0])
        sel = np.nonzero(tr["ray_id"] == r)[0]
        print("   ray", r, "gpu", o.cpu()[r].tolist(), "ref", ref[k][r].tolist(), "samples", len(sel),
              "alphas", [round(float(tr["alpha"][i]), 6) for i in sel[:8]])

# end-to-end: GPU forward vs golden reference and vs oracle on the GPU cloud
out = m(g.t("in_t").to(dev), render_depth=True, render_kwargs=g.render_kwargs(dev), render_weights=True,
        poses=g.t("in_c2w")[None].to(dev), Ks=g.t("in_K")[None].to(dev), get_skeleton=True)
th = out["t_hat_pcd"].cpu()
print("t_hat gpu-golden max", float((th - g.t("out_t_hat_pcd")).abs().max()))
orc2, ref2 = T._oracle_on_cloud(g, th, perm=m.last_palette_perm)
orc3, ref3 = T._oracle_on_cloud(g, g.t("out_t_hat_pcd"), perm=m.last_palette_perm)
print("survivors gpu-cloud", len(orc2.trace["s_i"]), "golden-cloud", len(orc3.trace["s_i"]))
for k in ["rgb_marched", "depth", "weights", "alphainv_last"]:
    a = out[k].cpu().reshape(R, -1); b = g.t("out_" + k).reshape(R, -1); c = ref2[k].reshape(R, -1); d3 = ref3[k].reshape(R, -1)
    e_gold = (a - b).abs().max(1)[0]; e_orc = (a - c).abs().max(1)[0]; e_oo = (c - d3).abs().max(1)[0]; e_og = (d3 - b).abs().max(1)[0]
    print(f"{k}: gpu-golden n>1e-4 {int((e_gold>1e-4).sum())} max {float(e_gold.max()):.2e} | gpu-oracle(gpu cloud) n {int((e_orc>1e-4).sum())} max {float(e_orc.max()):.2e} | oracle(gpu)-oracle(gold) n {int((e_oo>1e-4).sum())} | oracle(gold)-golden n {int((e_og>1e-4).sum())}")
    if int((e_gold > 1e-4).sum()):
        r = int(torch.argmax(e_gold))
        print("   worst ray", r, "gpu", a[r].tolist(), "golden", b[r].tolist(), "oracle(gpu)", c[r].tolist())
