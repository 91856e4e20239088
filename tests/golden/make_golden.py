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
* stores inputs + outputs as compressed .npz next to this script.

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


def rtn_poc(x, f):
    from lib.tineuvox import poc_fre
    return poc_fre(x, f)


def main():
    install_stubs()
    sys.path.insert(0, REF)
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    for name in ("G1", "G2", "G3"):
        gen_case(name)


if __name__ == "__main__":
    main()
