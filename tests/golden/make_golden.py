"""Generate golden fixtures by running the REFERENCE's own Python on synthetic inputs.

Run in the build container only (needs /root/reference; never on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

What it does:
* imports ``lib/temporalpoints.py``, ``lib/pointwarper.py``, ``lib/tineuvox.py`` from
  /root/reference with the absent third-party modules stubbed in ``sys.modules``:
  pykeops (exact brute-force Kmin_argKmin), torch_scatter (segment_coo), roma, seaborn
  (hls palette), tkinter; ``torch.utils.cpp_extension.load`` is patched to return the
  oracle's restatement of ``render_utils_cuda`` (the CUDA sources do not build here);
* builds the synthetic scenes G1 (D-NeRF-like, J=8) and G2 (ZJU-like, J=24, pose
  embedding 64) with ``apn_amd.synthetic``;
* runs ``TemporalPoints.forward`` (the ``run.py --render_pcd`` call, run.py:149-151),
  ``repose`` (run.py:287 / temporalpoints.py:370), ``get_weights`` with a non-trivial
  merge, and ``PointWarper.forward`` on the t-path and the rot_params path;
* stores inputs + outputs as compressed .npz next to this script;
* T1: the stage-1 TiNeuVox model itself (lib/tineuvox.py:91-625) -- forward,
  mult_dist_interp, get_grid_as_point_cloud -- and get_rays_of_a_view (a-22).

* G4: a G1-sized D-NeRF scene with 24 bones whose features and network weights are NOT
  fp16-representable (``fp16_exact=False``), so the reference pins the lo halves of the split-MFMA
  MLP contraction too.

Usage: ``python tests/golden/make_golden.py [G1 G2 G3 G4 T1]`` (default: all).

The reference never travels: only the .npz data files are committed.
"""
from __future__ import annotations

import os
import sys
import types

sys.dont_write_bytecode = True
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = os.environ.get("APN_REFERENCE", "/root/reference")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "articulated-point-nerf_amd"))

import numpy as np
import torch

from oracle import apn_oracle as O
from apn_amd import synthetic as S

CAPTURE = {}


# ------------------------------------------------------------------ stubs
class _Lazy:
    """Minimal pykeops LazyTensor: supports ((x_i - y_j)**2).sum(-1).{Kmin_argKmin,argKmin}."""

    def __init__(self, x=None, y=None, stage="leaf"):
        self.x, self.y, self.stage = x, y, stage

    def __sub__(self, other):
        a, b = self.x, other.x
        return _Lazy(a, b, "diff")

    def __pow__(self, p):
        assert p == 2
        return _Lazy(self.x, self.y, "sq")

    def sum(self, dim):
        return _Lazy(self.x, self.y, "d2")

    def _knn(self, dim, K):
        assert dim == 1
        q = self.x.reshape(-1, 3).detach().numpy()
        p = self.y.reshape(-1, 3).detach().numpy()
        d2, idx = O.knn_kmin(q, p, K, use_tree=False)
        return torch.from_numpy(d2), torch.from_numpy(idx)

    def Kmin_argKmin(self, dim, K):
        d2, idx = self._knn(dim, K)
        CAPTURE.setdefault("kmin", []).append((d2.clone(), idx.clone()))
        return d2, idx

    def argKmin(self, dim, K):
        return self._knn(dim, K)[1]


def _segment_coo(src, index, out, reduce="sum"):
    assert reduce == "sum"
    res = O.segment_sum(src.detach().numpy(), index.numpy(), out.shape[0])
    return torch.from_numpy(res).to(src.dtype)


class _RenderUtils:
    @staticmethod
    def sample_pts_on_rays(rays_o, rays_d, xyz_min, xyz_max, near, far, stepdist):
        out = O.sample_pts_on_rays(rays_o.numpy(), rays_d.numpy(), xyz_min.detach().numpy(),
                                   xyz_max.detach().numpy(), float(near), float(far), float(stepdist))
        CAPTURE["sample"] = dict(xyz_min=xyz_min.detach().clone(), xyz_max=xyz_max.detach().clone(),
                                 near=near, far=far, stepdist=stepdist)
        return [torch.from_numpy(np.ascontiguousarray(x)) for x in out]

    @staticmethod
    def raw2alpha(density, shift, interval):
        e, a = O.raw2alpha(density.detach().numpy(), float(shift), float(interval))
        CAPTURE["raw2alpha"] = dict(density=density.detach().clone(), shift=float(shift), interval=float(interval))
        return torch.from_numpy(e), torch.from_numpy(a)

    @staticmethod
    def alpha2weight(alpha, ray_id, n_rays):
        out = O.alpha2weight(alpha.detach().numpy(), ray_id.numpy(), int(n_rays))
        CAPTURE.setdefault("alpha2weight", []).append((alpha.detach().clone(), ray_id.clone()))
        return [torch.from_numpy(x) for x in out]


def install_stubs():
    pk = types.ModuleType("pykeops"); pkt = types.ModuleType("pykeops.torch")
    pkt.LazyTensor = lambda t: _Lazy(t)
    pk.torch = pkt
    ts = types.ModuleType("torch_scatter"); ts.segment_coo = _segment_coo
    roma = types.ModuleType("roma")
    sb = types.ModuleType("seaborn"); sb.color_palette = lambda name, n: O.hls_palette(n)
    tk = types.ModuleType("tkinter"); tk.W = "w"
    sys.modules.update({"pykeops": pk, "pykeops.torch": pkt, "torch_scatter": ts, "roma": roma,
                        "seaborn": sb, "tkinter": tk})
    import torch.utils.cpp_extension as ce
    ce.load = lambda name, sources, verbose=False, **kw: _RenderUtils()


# ------------------------------------------------------------------ generation
def build_reference_model(scene):
    from lib import tineuvox as rtn
    from lib import temporalpoints as rtp
    c = scene.ctor
    tnv = rtn.TiNeuVox(xyz_min=list(map(float, c["xyz_min"])), xyz_max=list(map(float, c["xyz_max"])),
                       num_voxels=12 ** 3, num_voxels_base=12 ** 3, voxel_dim=12, defor_depth=3,
                       net_width=128, alpha_init=1e-3, fast_color_thres=1e-4, no_view_dir=False,
                       posbase_pe=10, viewbase_pe=4, timebase_pe=8, gridbase_pe=2)
    kw = dict(c)
    kw["tineuvox"] = tnv
    model = rtp.TemporalPoints(**kw)
    missing, unexpected = model.load_state_dict(scene.params, strict=False)
    assert not unexpected, unexpected
    return model, tnv


def dump_state(model):
    return {k: v.detach().clone() for k, v in model.state_dict().items()
            if not k.startswith("tineuvox.") and not k.startswith("timenet.")}


def gen_case(name, t=0.3):
    CAPTURE.clear()
    scene = S.make_scene(name)
    torch.manual_seed(1234)
    model, tnv = build_reference_model(scene)
    state = dump_state(model)
    mmd = model.mean_min_distance.detach().clone()
    rk = scene.render_kwargs("cpu")
    gen = {}
    with torch.no_grad():
        out = model(torch.tensor([t]), render_depth=True, render_kwargs=dict(rk), render_weights=True,
                    render_pcd_direct=True, poses=scene.c2w[None], Ks=scene.K[None],
                    cam_per_ray=torch.zeros(len(rk["rays_o"]))[:, None], get_skeleton=True)
        kmin_d2, kmin_idx = CAPTURE["kmin"][-1]
        a2w = CAPTURE["alpha2weight"]
        gen.update({
            "out_rgb_marched": out["rgb_marched"], "out_rgb_marched_direct": out["rgb_marched_direct"],
            "out_depth": out["depth"], "out_weights": out["weights"],
            "out_alphainv_last": out["alphainv_last"], "out_alphainv_last_direct": out["alphainv_last_direct"],
            "out_t_hat_pcd": out["t_hat_pcd"], "out_joints": out["joints"],
            "trace_xyz_min": CAPTURE["sample"]["xyz_min"], "trace_xyz_max": CAPTURE["sample"]["xyz_max"],
            "trace_kmin_d2": kmin_d2, "trace_kmin_idx": kmin_idx,
            "trace_density": CAPTURE["raw2alpha"]["density"],
            "trace_a2w_alpha": a2w[0][0], "trace_a2w_ray_id": a2w[0][1],
            "trace_a2w_alpha_direct": a2w[1][0], "trace_a2w_ray_id_direct": a2w[1][1],
        })
        w_id = model.get_weights()
        gen["get_weights_identity"] = w_id
        # PointWarper.forward, t-path and rot_params path (pointwarper.py:213-279)
        t_embed = rtn_poc(torch.tensor([t]), model.time_poc)
        xyz, jr, G, jw, _ = model.forward_warp(w_id, model.joints, t_embed, get_frames=True, get_skeleton=True)
        gen.update({"pw_t_xyz": xyz, "pw_t_joints_rel": jr, "pw_t_G": G, "pw_t_joints_warped": jw})
        J = len(scene.ctor["joints"])
        sweep = S.repose_sweep(J, steps=4, seed=0)
        rp = sweep[3]
        gen["repose_rot_params"] = rp
        xyz_r, jr_r = model.repose(rp)
        gen.update({"repose_xyz": xyz_r, "repose_joints_rel": jr_r})
        # non-trivial merge (temporalpoints.py:326-333)
        rules = torch.arange(J)
        rules[J - 1] = J - 2
        rules[2] = 0
        model.flat_merging_rules = rules
        model.merging_mat = torch.zeros(J, J, J)
        for i in range(J):
            model.merging_mat[i] = torch.eye(J) * (rules == i)
        gen["merge_rules"] = rules
        gen["get_weights_merged"] = model.get_weights()
    data = {"in_" + k: v for k, v in state.items()}
    data["in_canonical_pcd"] = scene.ctor["canonical_pcd"]
    data["in_bones"] = torch.tensor(scene.ctor["bones"])
    data["in_mean_min_distance"] = mmd
    data["in_t"] = torch.tensor([t])
    data["in_c2w"] = scene.c2w; data["in_K"] = scene.K
    data["in_rays_o"] = rk["rays_o"]; data["in_rays_d"] = rk["rays_d"]; data["in_viewdirs"] = rk["viewdirs"]
    data["cfg_near"] = torch.tensor(rk["near"]); data["cfg_far"] = torch.tensor(rk["far"])
    data["cfg_bg"] = torch.tensor(float(rk["bg"])); data["cfg_stepsize"] = torch.tensor(rk["stepsize"])
    data["cfg_voxel_size"] = torch.tensor(scene.ctor["voxel_size"])
    data["cfg_pose_embedding_dim"] = torch.tensor(scene.ctor["pose_embedding_dim"])
    data["cfg_act_shift"] = torch.tensor(float(tnv.act_shift), dtype=torch.float64)
    data["cfg_voxel_size_ratio"] = torch.tensor(float(tnv.voxel_size_ratio))
    data["cfg_inverse_y"] = torch.tensor(scene.inverse_y)
    data.update(gen)
    arrs = {}
    for k, v in data.items():
        if torch.is_tensor(v):
            v = v.detach().cpu()
            if k.startswith("in_") and v.dtype == torch.float32 and v.numel() > 1024 \
                    and torch.equal(v.half().float(), v):
                v = v.half()          # fp16-exact by construction (features, network weights)
            arrs[k] = v.numpy()
        else:
            arrs[k] = np.asarray(v)
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), f"golden_{name}.npz")
    np.savez_compressed(path, **arrs)
    surv = int((kmin_d2[:, -1] <= 0.01).sum())
    print(f"{name}: wrote {path} ({os.path.getsize(path) / 1e6:.2f} MB); "
          f"in-bbox samples {len(kmin_d2)}, survivors {surv}, hit rays "
          f"{int((out['alphainv_last'] < 1).sum())}")


def gen_checkpoint_case(name="G3"):
    """A TemporalPoints checkpoint in the reference layout -- {'model_kwargs': get_kwargs() (with
    the reference TiNeuVox *module*), 'model_state_dict'} as run.py saves it -- converted by
    apn_amd.checkpoint.to_weights_only into the weights-only file the loader reads
    (ckpt_<name>.pt). Float tensors that are fp16-exact by construction are stored as fp16
    (lossless; load_state_dict casts them back)."""
    sys.path.insert(0, os.path.join(ROOT, "articulated-point-nerf_amd"))
    from apn_amd import checkpoint as C
    scene = S.make_scene(name)
    torch.manual_seed(1234)
    model, tnv = build_reference_model(scene)
    ck = C.to_weights_only({"model_kwargs": model.get_kwargs(), "model_state_dict": model.state_dict()})
    assert ck["tineuvox_class"] == "TiNeuVox" and type(tnv).__module__ == "lib.tineuvox"

    def small(v):
        if torch.is_tensor(v) and v.dtype == torch.float32 and v.numel() > 1024 and torch.equal(v.half().float(), v):
            return v.half()
        if isinstance(v, dict):
            return {k: small(x) for k, x in v.items()}
        return v
    ck = {k: small(v) for k, v in ck.items()}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), f"ckpt_{name}.pt")
    torch.save(ck, path)
    print(f"ckpt {name}: wrote {path} ({os.path.getsize(path) / 1e6:.2f} MB); "
          f"{len(ck['model_state_dict'])} state keys, tineuvox kwargs {sorted(ck['tineuvox_kwargs'])}")


def rtn_poc(x, f):
    from lib.tineuvox import poc_fre
    return poc_fre(x, f)


# ------------------------------------------------------------------ TiNeuVox stage 1 + get_rays
T1 = dict(xyz_min=[-0.8, -0.9, -1.0], xyz_max=[0.8, 0.9, 1.0], num_voxels=16000, voxel_dim=12, defor_depth=5,
          net_width=128, alpha_init=1e-3, fast_color_thres=1e-4, no_view_dir=False, posbase_pe=10, viewbase_pe=4,
          timebase_pe=8, gridbase_pe=2, H=32, W=32, near=1.0, far=6.0, stepsize=0.5, bg=1.0)


def gen_tineuvox_case(name="T1"):
    """The reference's TiNeuVox (stage 1, lib/tineuvox.py:91-625) on a small random model: forward
    (tineuvox.py:458-564) with per-ray times, mult_dist_interp on random points inside and outside
    the grid (379-419), get_grid_as_point_cloud on the full grid and on a point subset (253-363,
    the run.py:1152-1194 export query); plus get_rays_of_a_view (675-738) for both camera
    conventions, both pixel modes and the flips."""
    from lib import tineuvox as rtn
    c = T1
    torch.manual_seed(7)
    model = rtn.TiNeuVox(xyz_min=c["xyz_min"], xyz_max=c["xyz_max"], num_voxels=c["num_voxels"],
                         num_voxels_base=c["num_voxels"], voxel_dim=c["voxel_dim"], defor_depth=c["defor_depth"],
                         net_width=c["net_width"], alpha_init=c["alpha_init"], fast_color_thres=c["fast_color_thres"],
                         no_view_dir=c["no_view_dir"], posbase_pe=c["posbase_pe"], viewbase_pe=c["viewbase_pe"],
                         timebase_pe=c["timebase_pe"], gridbase_pe=c["gridbase_pe"])
    g = torch.Generator().manual_seed(11)
    with torch.no_grad():
        model.feature.copy_(torch.randn(model.feature.shape, generator=g) * 0.5)
        model.densitynet.weight.mul_(40.0)     # densities over a wide range: both fast_color_thres
        model.densitynet.bias.fill_(1.0)       # masks and the T < 1e-3 early exit are exercised
    c2w = S.pose_spherical(30.0, -30.0, 3.5)
    H, W = c["H"], c["W"]
    focal = 0.5 * W / np.tan(0.5 * 0.6911112)
    K = S.intrinsics(H, W, focal)
    data = {}
    # get_rays_of_a_view (tineuvox.py:733-738), every option combination used by the loaders
    for inv_y in (False, True):
        for mode in ("center", "lefttop"):
            for fx, fy in ((False, False), (True, False), (False, True)):
                ro, rd, vd = rtn.get_rays_of_a_view(H, W, K, c2w, False, inverse_y=inv_y, flip_x=fx, flip_y=fy,
                                                    mode=mode)
                tag = f"rays_{int(inv_y)}{mode[0]}{int(fx)}{int(fy)}"
                data[tag + "_o"], data[tag + "_d"], data[tag + "_v"] = ro, rd, vd
    ro, rd, vd = rtn.get_rays_of_a_view(H, W, K, c2w, False, inverse_y=False, mode="center")
    ro, rd, vd = ro.reshape(-1, 3), rd.reshape(-1, 3), vd.reshape(-1, 3)
    N = len(ro)
    times = torch.where(torch.arange(N) < N // 2, torch.tensor(0.2), torch.tensor(0.7))[:, None]
    rk = dict(near=c["near"], far=c["far"], stepsize=c["stepsize"], bg=c["bg"])
    with torch.no_grad():
        out = model(ro, rd, vd, times, **rk)
        pts = torch.rand(3000, 3, generator=g) * 2.2 - 1.1      # inside and outside the grid
        vox = model.mult_dist_interp(pts)
        gp = model.get_grid_as_point_cloud(stepsize=c["stepsize"], time_sel=torch.tensor([[0.0]]),
                                           viewdir=vd.mean(0, keepdim=True), sampling_freq=1,
                                           alpha_xyz_only=False)
        sub = (torch.rand(700, 3, generator=g) * 2 - 1) * torch.tensor(c["xyz_max"])
        gs = model.get_grid_as_point_cloud(stepsize=c["stepsize"], time_sel=torch.tensor([[0.4]]),
                                           viewdir=vd.mean(0, keepdim=True), alpha_xyz_only=False, grid_xyz=sub)
    state = {k: v.detach().clone() for k, v in model.state_dict().items()}
    for k, v in state.items():
        data["in_" + k] = v
    data.update({"in_c2w": c2w, "in_K": K, "in_rays_o": ro, "in_rays_d": rd, "in_viewdirs": vd, "in_times": times,
                 "in_pts": pts, "in_sub_xyz": sub})
    for k, v in c.items():
        data["cfg_" + k] = torch.tensor(v)
    data["cfg_act_shift"] = torch.tensor(float(model.act_shift), dtype=torch.float64)
    data["cfg_voxel_size"] = model.voxel_size.detach().clone()
    data["cfg_voxel_size_ratio"] = torch.as_tensor(model.voxel_size_ratio).detach().clone()
    data["cfg_world_size"] = model.world_size.detach().clone()
    for k in ("alphainv_last", "weights", "rgb_marched", "raw_alpha", "raw_rgb", "ray_id", "s", "ray_pts_delta",
              "depth"):
        data["out_" + k] = out[k]
    data["out_n_max"] = torch.tensor(out["n_max"])
    data["out_vox"] = vox
    names = ["points", "alphas", "rgbs", "h_feature", "vox_feature", "binary_volume", "grid_xyz", "alpha_volume"]
    for nm, v in zip(names, gp):
        if nm in ("alphas", "rgbs", "grid_xyz", "alpha_volume"):
            data["grid_" + nm] = v
    for nm, v in zip(names, gs):
        if nm in ("alphas", "rgbs", "h_feature", "vox_feature"):
            data["sub_" + nm] = v
    arrs = {k: (v.detach().cpu().numpy() if torch.is_tensor(v) else np.asarray(v)) for k, v in data.items()}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), f"golden_{name}.npz")
    np.savez_compressed(path, **arrs)
    print(f"{name}: wrote {path} ({os.path.getsize(path) / 1e6:.2f} MB); world_size {model.world_size.tolist()}, "
          f"in-bbox samples {len(out['ray_pts_delta'])}, kept {len(out['ray_id'])}, "
          f"hit rays {int((out['alphainv_last'] < 1).sum())}")


def main():
    install_stubs()
    sys.path.insert(0, REF)
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    which = sys.argv[1:] or ["G1", "G2", "G3", "G4", "T1"]
    for name in which:
        if name.startswith("ckpt_"):
            gen_checkpoint_case(name[5:])
        elif name.startswith("T"):
            gen_tineuvox_case(name)
        else:
            gen_case(name)


if __name__ == "__main__":
    main()
