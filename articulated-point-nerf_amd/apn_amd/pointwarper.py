"""PointWarper / TransformNet with the reference's API and state-dict names
(lib/pointwarper.py). The skeleton stage -- TransformNet (1x17 -> (J+1)x4), Rodrigues, the
rotation/sibling masks, the recursive-halving kinematic chain -- runs as ONE HIP launch
(``apn_skeleton_pose``, csrc/apn_skeleton.hip); ``pose_torch`` keeps the torch restatement the
tests compare it with. The per-point LBS blend + apply (the hot part, pointwarper.py:241-266)
runs in the HIP kernels ``apn_lbs_skin`` / ``k_lbs_skin_quad``.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib as L
from ._lib import call, ptr, stream_ptr


class TransformNet(torch.nn.Module):
    """pointwarper.py:5-37."""

    def __init__(self, input_dim, num_components, num_params_per_component, num_layers=3, hidden_dim=256):
        super().__init__()
        self.hidden_dim = hidden_dim
        self.num_components = num_components
        self.num_params_per_component = num_params_per_component
        self.out_dim = num_components * num_params_per_component
        self.register_buffer("rotation_switch_mask", torch.arange(0, num_components).long())
        layers = []
        for i in range(num_layers - 1):
            layers.append(torch.nn.Linear(input_dim if i == 0 else hidden_dim, hidden_dim))
            layers.append(torch.nn.ReLU())
        layers.append(torch.nn.Linear(hidden_dim, self.out_dim, bias=False))
        self.net = torch.nn.Sequential(*layers)

    def forward(self, x):
        from .linear import sequential
        b = x.shape[0]
        out = sequential(self.net, x)
        if b > 1:
            return out.reshape(b, self.num_components, self.num_params_per_component)
        return out.reshape(self.num_components, self.num_params_per_component)


def small_mm(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a @ b for the skeleton's 3x3 / 4x4 / 4x1 batches as a broadcast product and sum: elementwise
    kernels only (no library GEMM, whose argument uploads cannot sit inside the training step's
    captured warp graph, train.py)."""
    return (a.unsqueeze(-1) * b.unsqueeze(-3)).sum(-2)


def rodrigues(rvec: torch.Tensor):
    """pointwarper.py:118-143 (Neural Volumes form; 3- or 4-vector)."""
    if rvec.shape[-1] == 3:
        theta = torch.sqrt(1e-5 + torch.sum(rvec ** 2, dim=1))
        r = rvec / theta[:, None]
    elif rvec.shape[-1] == 4:
        theta = rvec[:, -1]
        r = rvec[:, :3]
        r = r / torch.sqrt(1e-5 + torch.sum(r ** 2, dim=1))[:, None]
    else:
        raise ValueError(rvec.shape)
    c, s = torch.cos(theta), torch.sin(theta)
    x, y, z = r[:, 0], r[:, 1], r[:, 2]
    R = torch.stack((x ** 2 + (1. - x ** 2) * c, x * y * (1. - c) - z * s, x * z * (1. - c) + y * s,
                     x * y * (1. - c) + z * s, y ** 2 + (1. - y ** 2) * c, y * z * (1. - c) - x * s,
                     x * z * (1. - c) - y * s, y * z * (1. - c) + x * s, z ** 2 + (1. - z ** 2) * c), dim=1)
    return R.view(-1, 3, 3), theta


class PointWarper(torch.nn.Module):
    """pointwarper.py:39-279. ``forward`` keeps the reference signature and return list."""

    def __init__(self, t_dim, canonical_pcd, joints, bones, num_layers=5, over_parameterized_rot=True):
        super().__init__()
        self.t_dim = t_dim
        self.params_per_compoent = 4
        self.register_buffer("canonical_pcd", torch.as_tensor(canonical_pcd).float(), persistent=False)
        self.num_layers = num_layers
        self.over_parameterized_rot = over_parameterized_rot
        self.init_tree(joints, bones)
        self.register_buffer("hom_row", torch.tensor([0, 0, 0, 1], dtype=torch.float32), persistent=False)
        self.transform_net = TransformNet(t_dim, len(joints) + 1, self.params_per_compoent, num_layers=num_layers)
        self.register_buffer("rot_mask", torch.zeros(len(joints), dtype=torch.bool))
        self.register_buffer("sibling_mask", torch.arange(0, len(joints)).long())

    def init_tree(self, joints, bones, old=False):
        """pointwarper.py:94-116 (the ``old=False`` tree used at construction)."""
        self.bones = bones
        self.parent_joint = {b[1]: b[0] for b in bones}
        self.child_joints = {k: [] for k in range(len(joints))}
        for k, p in self.parent_joint.items():
            self.child_joints[p].append(k)
        paths = [[0]]
        for i in range(len(bones)):
            j, inds = i + 1, []
            while j >= 0:
                inds.append(j)
                j = self.parent_joint.get(j, -1)
            paths.append(inds[::-1])
        depth = int(np.max([len(x) for x in paths]))
        pi = torch.full((len(paths), depth), -1, dtype=torch.long)
        for i, inds in enumerate(paths):
            pi[i, :len(inds)] = torch.tensor(inds)
        self.register_buffer("parent_indices", pi, persistent=False)
        self.register_buffer("parent_joint_ex", torch.tensor([self.parent_joint.get(i, 0) for i in range(len(paths))],
                                                             dtype=torch.long), persistent=False)

    Rodrigues = staticmethod(rodrigues)

    @classmethod
    def matrix_chain_product(cls, m):
        """pointwarper.py:145-153: recursive halving (binary-tree) product over dim 1."""
        L_ = m.shape[1]
        if L_ == 1:
            return m
        return small_mm(cls.matrix_chain_product(m[:, :L_ // 2]), cls.matrix_chain_product(m[:, L_ // 2:]))

    def calc_rec_abs_T_fast(self, R_t, joints):
        """pointwarper.py:156-193: M_j = [R_j | p - R_j p] about the parent joint p, chained
        root->joint; returns bone_Ts [J,4,4]."""
        J = R_t.shape[0]
        dev = R_t.device
        joints_old = torch.cat((self.hom_row[None, :3].to(dev), joints), 0)[self.parent_joint_ex + 1]
        M = torch.cat((torch.cat((R_t, joints_old[..., None] + small_mm(R_t, -joints_old[..., None])), -1),
                       self.hom_row[None, None].to(dev).repeat(J, 1, 1)), -2)
        M = torch.cat((torch.eye(4, device=dev)[None], M), 0)
        return self.matrix_chain_product(M[self.parent_indices + 1])[:, 0]

    def get_thetas(self, ts_embed):
        params = self.transform_net(ts_embed)
        rot = params[:, :-1, :3]
        shape = rot.shape[:2]
        _, thetas = self.Rodrigues(rot.reshape(shape[0] * shape[1], 3))
        return thetas.reshape(shape)

    def set_rotation_mask(self, rotations_to_keep):
        mask = ~rotations_to_keep
        if self.rot_mask is not None:
            mask = torch.logical_or(mask, self.rot_mask)
        self.rot_mask = mask

    def set_sibling_mask(self, sibling_mask):
        self.sibling_mask = sibling_mask.long()

    def _tn_packed(self, dev):
        """TransformNet weights packed for apn_skeleton_pose ([W0^T, b0, W1^T, b1, ..., W_last^T]),
        cached on the parameters' versions."""
        lins = [m for m in self.transform_net.net if isinstance(m, torch.nn.Linear)]
        key = (str(dev),) + tuple((p.data_ptr(), p._version) for m in lins for p in m.parameters())
        if getattr(self, "_tn_key", None) != key:
            parts = []
            for m in lins:   # W^T [in][out] per layer: coalesced GEMV loads (apn_skeleton.hip)
                parts.append(m.weight.detach().float().t().contiguous().reshape(-1))
                if m.bias is not None:
                    parts.append(m.bias.detach().float().reshape(-1))
            self._tn_buf = torch.cat(parts).to(dev).contiguous()
            self._tn_key = key
        return self._tn_buf, lins[0].in_features, lins[0].out_features, len(lins)

    def _tree_buffers(self, dev):
        key = (str(dev), self.sibling_mask.data_ptr(), self.sibling_mask._version,
               None if self.rot_mask is None else (self.rot_mask.data_ptr(), self.rot_mask._version))
        if getattr(self, "_tree_key", None) != key:
            self._tree = (self.parent_indices.to(dev, torch.int32).contiguous(),
                          self.parent_joint_ex.to(dev, torch.int32).contiguous(),
                          self.sibling_mask.to(dev, torch.int32).contiguous(),
                          None if self.rot_mask is None else self.rot_mask.to(dev, torch.int32).contiguous(),
                          torch.tensor(chain_program(self.parent_indices.shape[1]), dtype=torch.int32, device=dev))
            self._tree_key = key
        return self._tree

    def pose_buffers(self, J, dev):
        """Output buffers of one skeleton launch (``pose(out=...)``)."""
        return {"thetas": torch.empty(J, device=dev), "bone_Ts": torch.empty(J, 4, 4, device=dev),
                "T34": torch.empty(J, 12, device=dev), "gt": torch.empty(3, device=dev),
                "joints_rel": torch.empty(J, 3, device=dev)}

    def pose(self, joints, t=None, rot_params=None, global_t=None, time_poc=None, proj=None, sweep_index=None,
             out=None):
        """Skeleton stage of forward (pointwarper.py:216-239) as one HIP launch
        (apn_skeleton_frame): returns bone_Ts [J,4,4], global_t [3] and joints_rel [J,3]; the
        bone rows [J,12] for apn_lbs_skin are kept in ``last_T34``. Sets prev_params /
        prev_thetas / prev_global_t.

        ``time_poc`` given: ``t`` is the raw time [1] and its embedding poc_fre(t, time_poc)
        (tineuvox.py:872-878) is computed in the same launch. ``proj=(c2w [P,4,4], K [P,3,3])``:
        the skeleton projection project_point_to_image_plane(joints_rel + global_t, c2w, K)
        (temporalpoints.py:578-583) runs in the launch too, left in ``last_joints2d`` [P,J,2]
        (None when not requested or beyond the kernel's limits: the caller projects in torch).
        ``sweep_index`` (device int32 [1]): rot_params is a pose sweep [P, J, rot_dim]; the launch
        takes pose sweep_index % P and advances the index (TemporalPoints.capture_repose).
        ``out`` (``pose_buffers``): write thetas / bone_Ts / T34 / global_t / joints_rel there
        instead of fresh tensors (the pipelined repose sweep's double buffers)."""
        assert (t is None) ^ (rot_params is None)
        dev = joints.device
        L.require_cuda(joints, what="PointWarper.pose")
        J = joints.shape[0]
        pi, pjx, sib, rmask, prog = self._tree_buffers(dev)
        jts = joints.detach().float().contiguous()
        o = out if out is not None else self.pose_buffers(J, dev)
        thetas, bone_Ts, T34, gt, joints_rel = o["thetas"], o["bone_Ts"], o["T34"], o["gt"], o["joints_rel"]
        s = stream_ptr(dev)
        c2w = Km = j2d = None
        n_views = 0
        if proj is not None:
            c2w, Km = proj
            n_views = c2w.shape[0]
            if 0 < n_views <= 16 and n_views * J <= 1024 and tuple(c2w.shape[1:]) == (4, 4) and \
                    tuple(Km.shape) == (n_views, 3, 3):
                c2w = c2w.to(dev, torch.float32).contiguous()
                Km = Km.to(dev, torch.float32).contiguous()
                j2d = torch.empty(n_views, J, 2, device=dev)
            else:
                c2w = Km = None
                n_views = 0
        params = None
        if rot_params is None:
            tn, t_dim, hidden, n_layers = self._tn_packed(dev)
            params = torch.empty(J + 1, 4, device=dev)
            if time_poc is not None:
                tr = torch.as_tensor(t, dtype=torch.float32, device=dev).reshape(-1)
                if tr.numel() != 1 or 1 + 2 * time_poc.numel() != t_dim:
                    raise ValueError("PointWarper.pose: raw t must be one time and match the TransformNet input")
                poc = time_poc.detach().to(dev, torch.float32).contiguous()
                call("apn_skeleton_frame", ptr(tr), ptr(poc), poc.numel(), None, 4, J, ptr(tn), hidden, n_layers,
                     ptr(jts), ptr(pi), pi.shape[1], ptr(pjx), ptr(sib), ptr(rmask), ptr(params), ptr(thetas),
                     ptr(bone_Ts), ptr(T34), ptr(gt), ptr(joints_rel), ptr(prog), ptr(c2w), ptr(Km), n_views, ptr(j2d),
                     None, 0, s)
            else:
                te = t.detach().float().reshape(-1).contiguous()   # t is already the time embedding
                call("apn_skeleton_pose", ptr(te), te.numel(), None, 4, J, ptr(tn), hidden, n_layers, ptr(jts),
                     ptr(pi), pi.shape[1], ptr(pjx), ptr(sib), ptr(rmask), ptr(params), ptr(thetas), ptr(bone_Ts),
                     ptr(T34), ptr(gt), ptr(joints_rel), ptr(prog), s)
                j2d = None
            self.prev_params = params
            self.prev_global_t = gt
        else:
            rp = rot_params.detach().float().contiguous()
            n_sweep = rp.shape[0] if sweep_index is not None else 0
            if sweep_index is not None and (rp.dim() != 3 or rp.shape[1] != J):
                raise ValueError("PointWarper.pose: a sweep is [P, J, rot_dim]")
            call("apn_skeleton_frame", None, None, 0, ptr(rp), rp.shape[-1], J, None, 0, 0, ptr(jts), ptr(pi),
                 pi.shape[1], ptr(pjx), ptr(sib), ptr(rmask), None, ptr(thetas), ptr(bone_Ts), ptr(T34), ptr(gt),
                 ptr(joints_rel), ptr(prog), ptr(c2w), ptr(Km), n_views, ptr(j2d), ptr(sweep_index), n_sweep, s)
            if global_t is not None:
                gt = global_t
                j2d = None   # projected with the kernel's zero global_t: the caller projects in torch
        self.prev_thetas = thetas
        self.last_T34 = T34
        self.last_joints2d = j2d
        return bone_Ts, gt, joints_rel

    def pose_sweep(self, joints, sweep, out):
        """Every pose of a repose sweep [P, J, rot_dim] in one launch (apn_skeleton_sweep: one
        workgroup per pose, each exactly as ``pose(rot_params=sweep[p])``) into ``out`` =
        pose_buffers-shaped tensors with a leading P dimension."""
        dev = joints.device
        J = joints.shape[0]
        P, rot_dim = sweep.shape[0], sweep.shape[2]
        pi, pjx, sib, rmask, prog = self._tree_buffers(dev)
        jts = joints.detach().float().contiguous()
        call("apn_skeleton_sweep", ptr(sweep), P, rot_dim, J, ptr(jts), ptr(pi), pi.shape[1], ptr(pjx), ptr(sib),
             ptr(rmask), ptr(out["thetas"]), ptr(out["bone_Ts"]), ptr(out["T34"]), ptr(out["gt"]),
             ptr(out["joints_rel"]), ptr(prog), stream_ptr(dev))

    def pose_torch(self, joints, t=None, rot_params=None, global_t=None):
        """The skeleton stage as device torch ops (restatement of pointwarper.py:216-239 used to
        cross-check apn_skeleton_pose in the tests)."""
        assert (t is None) ^ (rot_params is None)
        if rot_params is None:
            params = self.transform_net(t.unsqueeze(0))
            self.prev_params = params
            global_t = params[-1, :3]
            R_t, self.prev_thetas = self.Rodrigues(params[:len(joints), :])
            self.prev_global_t = global_t
        else:
            R_t, self.prev_thetas = self.Rodrigues(rot_params)
        R_t = R_t[self.sibling_mask]
        if self.rot_mask is not None:
            # R_t[rot_mask] = I (pointwarper.py:230-231) without the boolean index's host sync
            R_t = torch.where(self.rot_mask.to(R_t.device)[:, None, None], torch.eye(3, device=R_t.device), R_t)
        bone_Ts = self.calc_rec_abs_T_fast(R_t, joints)
        if global_t is None:
            global_t = torch.zeros(3, dtype=torch.float32, device=bone_Ts.device)
        jh = torch.cat([joints, torch.ones((len(joints), 1), device=joints.device)], -1)
        joints_rel = small_mm(bone_Ts, jh.unsqueeze(-1)).squeeze(-1)[:, :3]
        return bone_Ts, global_t, joints_rel

    def forward(self, weights, joints, t=None, rot_params=None, global_t=None, get_frames=False,
                avg_procrustes=False, get_skeleton=False):
        """pointwarper.py:213-279 -> [xyz, joints_warped_rel, (weighted_G_tw), (joints_warped, bones)].
        The per-point blend and transform run in ``apn_lbs_skin`` (weights taken as given)."""
        if avg_procrustes:
            raise NotImplementedError("avg_procrustes needs roma.special_procrustes (out of scope)")
        bone_Ts, global_t, joints_rel = self.pose(joints, t, rot_params, global_t)
        xyz, G = lbs_apply(self.canonical_pcd, weights, bone_Ts, global_t, get_frames=get_frames)
        out = [xyz, joints_rel]
        if get_frames:
            out.append(G)
        if get_skeleton:
            out.append(joints_rel + global_t)
            out.append(self.bones)
        return out


def chain_program(n):
    """matrix_chain_product (pointwarper.py:145-153: prod(left floor(n/2)) @ prod(rest),
    recursively) as a postfix program over factor indices 0..n-1: d = push factor d, -1 =
    multiply the top two (left below right). Consumed by apn_skeleton_pose."""
    prog = []

    def rec(lo, hi):
        if hi - lo == 1:
            prog.append(lo)
            return
        mid = lo + (hi - lo) // 2
        rec(lo, mid)
        rec(mid, hi)
        prog.append(-1)
    rec(0, n)
    return prog


def lbs_apply(pcd, weights, bone_Ts, global_t, get_frames=False):
    """Blend + apply with given per-point weights (HIP); returns (xyz [N,3], G [N,4,4] or None)."""
    L.require_cuda(pcd, weights, bone_Ts, what="PointWarper.forward")
    N, J = weights.shape
    dev = pcd.device
    xyz = torch.empty(N, 3, device=dev)
    G = torch.empty(N, 4, 4, device=dev) if get_frames else None
    T34 = bone_Ts[:, :3, :].detach().float().reshape(J, 12).contiguous()
    gt = global_t.detach().float().reshape(3).contiguous()
    w = weights.detach().float().contiguous()
    call("apn_lbs_skin", ptr(pcd.contiguous()), ptr(w), N, J, None, 0.0, None, ptr(T34), ptr(gt), None, None, None,
         None, 0.0, 1, ptr(xyz), None, ptr(G), None, None, None, None, stream_ptr(dev))
    return xyz, G
