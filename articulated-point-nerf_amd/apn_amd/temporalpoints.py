"""TemporalPoints with the reference's constructor, ``forward()``, ``repose()``,
``get_weights()``, ``sample_ray()`` signatures and return dicts (lib/temporalpoints.py),
rendering through the fused HIP pipeline of libapn_hip.so:

    skeleton stage (torch, J-sized) -> apn_lbs_skin -> apn_grid_build -> apn_inbbox_count/fill
    -> apn_knn_radius -> apn_point_mlp -> apn_composite

One forward renders any number of rays in a single pass (the reference's 8192-ray chunking
is bit-identical to a single pass), so LBS, the 4x4 inverse and the kNN grid
are built once per call instead of once per chunk.
"""
from __future__ import annotations

import colorsys
import contextlib
import gc
import os
import ctypes as C

import numpy as np
import torch

from . import _lib as L
from . import roctx
from ._lib import call, ptr, stream_ptr
from .ops import Workspace, pack_mlp_weights
from .pointwarper import PointWarper
from .shard import SplitTracker
from .tineuvox import poc_fre

CELL_CAP = int(os.environ.get("APN_CELL_CAP", 1 << 20))
# the kNN's second grid on the grid's side stream (A/B: APN_AGRID_SIDE=0 builds it inside the kNN call)
AGRID_SIDE = os.environ.get("APN_AGRID_SIDE", "1") != "0"
# exact early ray termination of the neighbour MLP (apn_point_mlp_ert; APN_ERT=0: every kept sample)
ERT = os.environ.get("APN_ERT", "1") != "0"
ERT_PASSES = 9   # apn_mlp_layout.h ERT_PASSES


class NoPointsException(Exception):
    """temporalpoints.py:26-28."""


class FrameStats(dict):
    """Per-frame counts. 'kept_samples' (kNN survivors) -- and on the capacity-bounded path
    'inbbox_samples' too -- stay on the device until asked for, so rendering a frame needs no
    device->host sync."""

    def __init__(self, *args, nsurv=None, info=None, **kw):
        super().__init__(*args, **kw)
        self._nsurv = nsurv
        self._info = info   # apn_inbbox_fill_capped frame_info {queries, in-bbox total, overflow, survivors}

    def __missing__(self, key):
        if self._info is not None and key in ("inbbox_samples", "kept_samples"):
            v = self._info.tolist()
            self["inbbox_samples"], self["kept_samples"] = v[1], v[3]
            return self[key]
        if key == "kept_samples" and self._nsurv is not None:
            v = int(self._nsurv.item())
            self[key] = v
            return v
        raise KeyError(key)

    def get(self, key, default=None):
        try:
            return self[key]
        except KeyError:
            return default

    def resolved(self):
        self.get("kept_samples")
        self.get("inbbox_samples")
        return dict(self)


class RenderOutput(dict):
    """The dict ``TemporalPoints.forward`` returns on the render path.

    The fused pipeline keeps the kNN survivor count on the device (no host sync after the kNN
    stage). When no sample survives, the reference raises NoPointsException inside
    ``aggregate_pts`` and returns a different dict (temporalpoints.py:598-609): ``alphainv_last``
    is None, there is no ``alphainv_last_direct``, and ``depth`` / ``weights`` are present
    whatever ``render_depth`` / ``render_weights`` asked for. The colour values already agree
    (the kernels composite nothing: rgb = bg, depth = 0, weights = bg), so only the key set and
    ``alphainv_last`` differ -- they are resolved on the first access that can observe them,
    with one read of the device count. Reading rgb_marched / depth / weights, as the
    reference's render loops do (run.py:126-173), never syncs.

    On the capacity-bounded path (no host read of the in-bbox sample count, see
    TemporalPoints._render) the frame is validated on the first access of any key: one read of
    the device frame_info; a frame whose samples overflowed the capacity is rendered again on the
    exact path (``rerender``) and its values replace these."""

    _SENSITIVE = ("alphainv_last", "alphainv_last_direct", "depth", "weights")

    def __init__(self, *a, nsurv=None, n_rays=0, bg=0.0, info=None, rerender=None, **kw):
        super().__init__(*a, **kw)
        self._nsurv = nsurv
        self._n_rays = n_rays
        self._bg = bg
        self._info = info
        self._rerender = rerender

    def _resolve(self):
        if self._info is not None:
            info, self._info = self._info, None
            v = info.tolist()   # {queries, in-bbox total, overflow, survivors}
            if v[2]:
                fresh = self._rerender()
                dict.clear(self)
                dict.update(self, {k: dict.__getitem__(fresh, k) for k in dict.keys(fresh)})
                self._nsurv, self._n_rays, self._bg = fresh._nsurv, fresh._n_rays, fresh._bg
                self._rerender = None
                return self._resolve()
            self._nsurv = None
            n_surv, dev = v[3], info.device
        elif self._nsurv is not None:
            nsurv, self._nsurv = self._nsurv, None
            n_surv, dev = int(nsurv.item()), nsurv.device
        else:
            return
        if n_surv > 0:
            return
        R, bg = self._n_rays, self._bg
        super().pop("alphainv_last_direct", None)
        super().__setitem__("alphainv_last", None)
        if not dict.__contains__(self, "depth"):
            super().__setitem__("depth", torch.zeros(R, device=dev))
        if not dict.__contains__(self, "weights"):
            super().__setitem__("weights", torch.ones(R, 3, device=dev) * bg)

    def __getitem__(self, k):
        if self._info is not None or k in self._SENSITIVE:
            self._resolve()
        return super().__getitem__(k)

    def get(self, k, default=None):
        if self._info is not None or k in self._SENSITIVE:
            self._resolve()
        return super().get(k, default)

    def __contains__(self, k):
        if self._info is not None or k in self._SENSITIVE:
            self._resolve()
        return super().__contains__(k)

    def keys(self):
        self._resolve()
        return super().keys()

    def items(self):
        self._resolve()
        return super().items()

    def values(self):
        self._resolve()
        return super().values()

    def __iter__(self):
        self._resolve()
        return super().__iter__()

    def __len__(self):
        self._resolve()
        return super().__len__()

    def pop(self, k, *default):
        self._resolve()
        return super().pop(k, *default)

    def copy(self):
        self._resolve()
        return dict(super().items())

    def raw(self, k, default=None):
        """The fused pipeline's own value (no resolution, no sync)."""
        return super().get(k, default)


def hls_palette(n, h=0.01, l=0.6, s=0.65):
    """seaborn.color_palette('hls', n) (temporalpoints.py:692)."""
    hues = np.linspace(0, 1, n + 1)[:-1]
    hues += h
    hues %= 1
    hues -= hues.astype(int)
    return [colorsys.hls_to_rgb(x, l, s) for x in hues]


def project_point_to_image_plane(points, pose, intrinsic):
    """utils.py:435-450."""
    pose = torch.linalg.inv_ex(pose).inverse   # == pose.inverse() without its host-side singularity check (a sync)
    # the two bmm's as broadcast products over the 3-vectors (elementwise kernels, no library GEMM)
    points = (pose[:, None, :3, :3] * points[None, :, None, :]).sum(-1) + pose[:, None, :3, 3]
    points = (intrinsic[:, None, :, :] * points[:, :, None, :]).sum(-1)
    return points[:, :, :2] / points[:, :, 2:]


def _bone_distances(p, a, b):
    """Point-to-segment distances [B, N] (temporalpoints.py:206-233)."""
    s = b - a
    w = p[None, :, :] - a[:, None, :]
    ps = (w * s[:, None, :]).sum(-1)
    l2 = (s * s).sum(-1)
    d_lo = torch.norm(w, dim=-1)
    d_hi = torch.norm(p[None, :, :] - b[:, None, :], dim=-1)
    proj = a[:, None, :] + (ps / l2[:, None]).unsqueeze(-1) * s[:, None, :]
    d_in = torch.norm(p[None, :, :] - proj, dim=-1)
    lower = ps <= 0
    upper = (~lower) & (ps >= l2[:, None])
    return torch.where(lower, d_lo, torch.where(upper, d_hi, d_in))


def weights_from_bones(joints, bones, pcd, eps):
    """Initial raw LBS weights (temporalpoints.py:235-254 with add_noise=True, noise_var=0,
    add_zero_weight=True): [N, J] = [0 | 1 / (0.5 e^d + eps)] over the bone distances d."""
    a = torch.stack([joints[b[0]] for b in bones])
    b = torch.stack([joints[b[1]] for b in bones])
    d = _bone_distances(pcd, a, b)
    w = (1 / (0.5 * torch.e ** d + eps)).T.contiguous()
    return torch.cat([torch.zeros((len(w), 1)), w], dim=-1)


@contextlib.contextmanager
def _capture_guard():
    """Around a HIP-graph capture: destroy unreachable graphs first, then keep the cyclic garbage
    collector off until the capture has ended. A graph freed by the collector in the middle of a
    capture (an earlier step's closure cycle; allocations inside the capture can trigger a
    collection) would call hipGraphExecDestroy while the stream is capturing, which HIP refuses
    (the process aborts). Re-enabled in ``finally`` only if it was enabled on entry."""
    was = gc.isenabled()
    gc.collect()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


def _grow_capacity(n):
    """In-bbox sample capacity for a frame of n samples: 25 % headroom, 64k granules."""
    return max(65536, (int(n * 1.25) + 65535) // 65536 * 65536)


class TemporalPoints(torch.nn.Module):
    def __init__(self, canonical_pcd, canonical_alpha, canonical_feat, canonical_rgbs, skeleton_pcd, joints, bones,
                 xyz_min, xyz_max, tineuvox, neighbours=8, timebase_pe=8, eps=1e-6, stepsize=None, voxel_size=None,
                 fast_color_thres=0, embedding='full', frozen_view_dir=None, over_parameterized_rot=True,
                 re_init_feat=False, re_init_mlps=False, feat_depth=4, pose_embedding_dim=0, **kwargs):
        super().__init__()
        canonical_pcd = torch.as_tensor(canonical_pcd).float()
        joints = torch.as_tensor(joints)
        self.register_buffer("canonical_pcd", canonical_pcd, persistent=False)
        self.skeleton_pcd = skeleton_pcd
        self.bones = bones
        self.bone_arap_mask = torch.tensor(bones).reshape(-1)
        self.register_buffer("xyz_min", torch.Tensor(np.asarray(xyz_min, dtype=np.float32)))
        self.register_buffer("xyz_max", torch.Tensor(np.asarray(xyz_max, dtype=np.float32)))
        self.eps = torch.as_tensor(eps, dtype=torch.float32).clone()
        self._eps = float(eps)
        self.feat_depth = feat_depth
        self.timebase_pe = timebase_pe
        self.t_dim = 1 + timebase_pe * 2
        self.stepsize = stepsize
        self.voxel_size = voxel_size
        self.fast_color_thres = fast_color_thres
        self.embedding = embedding
        self.over_parameterized_rot = over_parameterized_rot
        self.joints_to_keep = None
        self.forward_warp_t_dim = self.t_dim
        self.weights = torch.nn.Parameter(self._weights_from_bones(joints.float(), bones, canonical_pcd))
        self.forward_warp = PointWarper(canonical_pcd=canonical_pcd, t_dim=self.forward_warp_t_dim, joints=joints,
                                        bones=bones, over_parameterized_rot=over_parameterized_rot)
        self.original_joints = torch.nn.Parameter(joints.to(torch.float32), requires_grad=False)
        self.joints = torch.nn.Parameter(joints.to(torch.float32))
        self.canonical_feat = torch.nn.Parameter(torch.as_tensor(canonical_feat).float())
        if re_init_feat:
            self.canonical_feat.data = torch.randn_like(self.canonical_feat)
        self.theta_weight = torch.nn.Parameter(torch.tensor([0.1]))
        self.merging_dict = None
        self.merging_mat = None
        gammas = torch.ones(len(canonical_pcd))
        self.gammas = torch.nn.Parameter(gammas + torch.randn_like(gammas) * 1e-2)
        self.pruned_joints = torch.zeros(len(joints), dtype=bool)
        self.register_buffer("flat_merging_rules", torch.arange(0, len(joints)))
        self.register_buffer("sibling_merging_rules", torch.zeros(len(joints), dtype=bool))
        self.canonical_rgbs = torch.nn.Parameter(torch.as_tensor(canonical_rgbs).float())
        self.canonical_alpha = torch.nn.Parameter(torch.as_tensor(canonical_alpha).float())
        self.direct_eps = torch.nn.Parameter(torch.tensor([0.05] * len(canonical_alpha)))
        self.register_buffer("time_poc", torch.FloatTensor([(2 ** i) for i in range(timebase_pe)]))
        self.neighbours = neighbours
        if neighbours != 8:
            raise NotImplementedError("the HIP kNN / MLP kernels are specialised for K=8 neighbours")
        self._mmd = None  # mean_min_distance, computed on the device on first use (temporalpoints.py:104-111)
        self.og_joint_distance = (self.original_joints[self.bone_arap_mask][0::2, :]
                                  - self.original_joints[self.bone_arap_mask][1::2, :])
        feat_in = self.canonical_feat.shape[-1] + 3 + 3 * tineuvox.posbase_pe * 2 + pose_embedding_dim
        width = self.canonical_feat.shape[-1]
        self.feat_net = torch.nn.Sequential(
            torch.nn.Linear(feat_in, width), torch.nn.LeakyReLU(inplace=True),
            *[torch.nn.Sequential(torch.nn.Linear(width, width), torch.nn.LeakyReLU(inplace=True))
              for _ in range(feat_depth - 2)],
            torch.nn.Linear(width, width), torch.nn.LeakyReLU(inplace=True))
        self.rgbnet = tineuvox.rgbnet
        self.densitynet = tineuvox.densitynet
        self.timenet = tineuvox.timenet
        if re_init_mlps:
            for m in (self.rgbnet, self.densitynet, self.timenet):
                m.apply(lambda x: x.reset_parameters() if hasattr(x, "reset_parameters") else None)
        self.time_poc = tineuvox.time_poc          # buffer (same values as the TiNeuVox one)
        self.no_view_dir = tineuvox.no_view_dir
        self.tineuvox = tineuvox
        self.register_buffer("xyz_max_canonical", canonical_pcd.max(dim=0)[0])
        self.register_buffer("xyz_min_canonical", canonical_pcd.min(dim=0)[0])
        self.frozen_view_dir = frozen_view_dir
        if frozen_view_dir is not None:
            vemb = poc_fre(torch.as_tensor(frozen_view_dir).float(), self.view_poc)
            self.viewdirs_emb = torch.nn.Parameter(vemb[None], requires_grad=False)
        self.pose_embedding_dim = pose_embedding_dim
        if pose_embedding_dim > 0:
            pin = len(self.joints) * (3 * len(self.pos_poc) * 2 + 3)
            self.pose_embedding_net = torch.nn.Sequential(
                torch.nn.Linear(pin, pin // 2), torch.nn.LeakyReLU(inplace=True),
                *[torch.nn.Sequential(torch.nn.Linear(pin // 2, pin // 2), torch.nn.LeakyReLU(inplace=True))
                  for _ in range(feat_depth - 2)],
                torch.nn.Linear(pin // 2, pose_embedding_dim), torch.nn.LeakyReLU(inplace=True))
        self.beta = torch.nn.Parameter(torch.tensor([0.5]))
        self.beta_min = torch.nn.Parameter(torch.tensor([0.0001]), requires_grad=False)
        self._ws = self._ws_eager = Workspace()   # per-frame buffers (use_workspace swaps them)
        self._ws_shared = Workspace()              # the layer-1 projection P, shared by every workspace
        self._palette_cache = {}
        self.palette_perm_device = None   # None: the weights' device (reference behaviour)
        self.timing = None          # set to {} to record HIP-event timings of the MLP launch
        self.last_stats = FrameStats()
        self._cap_updates = {}      # ranges-split shard -> (pinned max in-bbox share, event) (shard._assemble)
        self._capacity = {}         # ray count (or shard) -> in-bbox sample capacity of the sync-free render path
        # kNN grid build on a side stream, concurrent with the sampling (APN_CONCURRENT_GRID=0: serial)
        self.concurrent_grid = os.environ.get("APN_CONCURRENT_GRID", "1") != "0"
        self._side_streams = {}
        self._splits = {}           # (ray count, world) -> SplitTracker of the ray-sharded frames
        self.last_split_tracker = self.last_full_offsets = self._last_ray_ws = None
        self._block_index = {}      # (ray count, rank, world, block) -> ray indices of the "blocks" split
        self._force_exact = False
        self._last_info = None
        # the neighbour MLP only on the kept samples the compositing reads (apn_point_mlp_ert: every
        # ray's samples up to its T < 1e-3 break, in passes); the frame is bit-identical either way
        self.early_termination = ERT
        self.last_mlp_rows = None   # device int32 [ERT_PASSES]: samples per early-termination pass of the last frame

    # view_poc / pos_poc alias the TiNeuVox buffers (temporalpoints.py:148-150); as properties
    # they follow .to(device) (the reference relies on a CUDA default tensor type instead).
    @property
    def view_poc(self):
        return self.tineuvox.view_poc

    @property
    def pos_poc(self):
        return self.tineuvox.pos_poc

    # ------------------------------------------------------------------ construction helpers
    def _weights_from_bones(self, joints, bones, pcd, soft_weights=True):
        return weights_from_bones(joints, bones, pcd, self.eps)

    def get_kwargs(self):
        """temporalpoints.py:176-200."""
        return {'canonical_pcd': self.canonical_pcd, 'skeleton_pcd': self.skeleton_pcd,
                'canonical_alpha': self.canonical_alpha, 'canonical_feat': self.canonical_feat,
                'canonical_rgbs': self.canonical_rgbs, 'joints': self.joints, 'bones': self.bones,
                'neighbours': self.neighbours, 'timebase_pe': self.timebase_pe, 'eps': self.eps,
                'stepsize': self.stepsize, 'weights': self.weights, 'xyz_min': self.xyz_min.cpu().numpy(),
                'xyz_max': self.xyz_max.cpu().numpy(), 'tineuvox': self.tineuvox, 'voxel_size': self.voxel_size,
                'fast_color_thres': self.fast_color_thres, 'embedding': self.embedding,
                'frozen_view_dir': self.frozen_view_dir, 'over_parameterized_rot': self.over_parameterized_rot,
                'feat_depth': self.feat_depth, 'pose_embedding_dim': self.pose_embedding_dim}

    @property
    def mean_min_distance(self):
        """temporalpoints.py:104-111, computed with the HIP grid search (apn_nn1_distance)."""
        if self._mmd is None or self._mmd.device != self.canonical_pcd.device:
            pcd = self.canonical_pcd.contiguous()
            L.require_cuda(pcd, what="mean_min_distance")
            N, dev = pcd.shape[0], pcd.device
            nn = torch.empty(N, device=dev)
            sorted4 = torch.empty(N, 4, device=dev)
            bbox = torch.empty(8, dtype=torch.int32, device=dev)
            gws = torch.empty(int(L.load().apn_grid_workspace_bytes(N, CELL_CAP)), dtype=torch.uint8, device=dev)
            call("apn_nn1_distance", ptr(pcd), N, self._eps, CELL_CAP, ptr(nn), ptr(sorted4), ptr(bbox), ptr(gws),
                 stream_ptr(dev))
            self._mmd = nn.double().mean().float()
            self._mmd_f = float(self._mmd)
        return self._mmd

    # ------------------------------------------------------------------ training losses
    # (temporalpoints.py:714-800): torch expressions around neighbour indices from the HIP
    # kNN (apn_knn_points) in place of pykeops' argKmin, so autograd flows as in the reference.
    def _canonical_knn(self):
        """nn_i [N, neighbours] (self first) and nn_distance (temporalpoints.py:104-110)."""
        if getattr(self, "_nn_cache", None) is None or self._nn_cache[0].device != self.canonical_pcd.device:
            from .ops import knn_points
            pcd = self.canonical_pcd.detach().contiguous()
            _, nn_i = knn_points(pcd, pcd, self.neighbours)
            nn_distance = torch.sqrt(((pcd[:, None, :] - pcd[nn_i, :]) ** 2).sum(-1) + self.eps.to(pcd.device))
            from .train import reverse_csr
            self._nn_cache = (nn_i, nn_distance) + reverse_csr(nn_i)
        return self._nn_cache

    @property
    def nn_i(self):
        return self._canonical_knn()[0]

    @property
    def nn_distance(self):
        return self._canonical_knn()[1]

    def get_neighbour_weight_tv_loss(self):
        """temporalpoints.py:714-716 as the fused HIP NbrTVLoss (no [N,K,J] gather, no scatter-add
        backward)."""
        from .train import NbrTVLoss
        nn_i, _, rev_ptr, rev_edge = self._canonical_knn()
        return NbrTVLoss.apply(self._last_weights, nn_i, rev_ptr, rev_edge)

    def get_weight_sparsity_loss(self):
        """temporalpoints.py:718-721 as the fused HIP SparsityLoss."""
        from .train import SparsityLoss
        return SparsityLoss.apply(self._last_weights, float(self.eps))

    def get_arap_loss(self, warped_pcd, c=0.03):
        """temporalpoints.py:723-725 as the fused HIP ArapLoss (gather-only backward)."""
        from .train import ArapLoss
        nn_i, nn_distance, rev_ptr, rev_edge = self._canonical_knn()
        return ArapLoss.apply(warped_pcd, nn_i, nn_distance, float(self.eps), rev_ptr, rev_edge)

    def get_joint_arap_loss(self):
        joint_distance = (self.joints[self.bone_arap_mask][0::2, :] - self.joints[self.bone_arap_mask][1::2, :])
        return ((self.og_joint_distance.to(joint_distance.device) - joint_distance) ** 2).sum()

    def get_joint_chamfer_loss(self):
        dev = self.joints.device
        sk = self.skeleton_pcd
        if sk.device != dev:   # a device copy kept beside the (CPU) skeleton cloud: no per-step host copy
            key = (str(dev), sk.data_ptr(), sk._version)
            hit = self.__dict__.get("_skeleton_pcd_dev")
            if hit is None or hit[0] != key:
                hit = (key, sk.to(dev))
                self.__dict__["_skeleton_pcd_dev"] = hit
            sk = hit[1]
        _, c2 = self.get_chamfer_loss(sk, self.joints, c=None, get_raw=True)
        return c2.sum()

    def _rho(self, x, c):
        return (2 * (x / c) ** 2) / ((x / c) ** 2 + 4)

    def get_chamfer_loss(self, pcd1, pcd2, N=None, M=None, c=0.03, get_raw=False):
        from .ops import knn_points
        if N is not None:
            pcd1 = pcd1[torch.randint(0, pcd1.shape[0], (N,)).long().to(pcd1.device)]
        if M is not None:
            pcd2 = pcd2[torch.randint(0, pcd2.shape[0], (M,)).long().to(pcd2.device)]
        _, nn_i1 = knn_points(pcd1.detach(), pcd2.detach(), 1)   # D_ij.argKmin(dim=1, K=1)
        _, nn_i2 = knn_points(pcd2.detach(), pcd1.detach(), 1)   # D_ij.argKmin(dim=0, K=1)
        nn_distance1 = ((pcd1[:, None, :] - pcd2[nn_i1, :]) ** 2).sum(-1)
        nn_distance2 = ((pcd2[:, None, :] - pcd1[nn_i2, :]) ** 2).sum(-1)
        if get_raw:
            return nn_distance1, nn_distance2
        if c is None:
            return nn_distance1.mean() + nn_distance2.mean()
        return self._rho(nn_distance1, c).mean() + self._rho(nn_distance2, c).mean()

    def get_batch_chamfer_loss(self, pcd1, pcd2, N=None, M=None):
        """temporalpoints.py:765-795 (run.py:690 uses it on 2D projections): per batch element
        argKmin(K=1) both ways; 2D points are padded with a zero coordinate, which leaves every
        squared distance unchanged."""
        from .ops import knn_points
        assert len(pcd1) == len(pcd2)
        if N is not None:
            pcd1 = pcd1[:, torch.randint(0, pcd1.shape[1], (N,), device=pcd1.device).long()]
        if M is not None:
            pcd2 = pcd2[:, torch.randint(0, pcd2.shape[1], (M,), device=pcd1.device).long()]

        def pad3(x):
            x = x.detach().float()
            return torch.cat([x, x.new_zeros(x.shape[:-1] + (3 - x.shape[-1],))], -1) if x.shape[-1] < 3 else x
        nn_i1 = torch.stack([knn_points(pad3(a), pad3(b), 1)[1] for a, b in zip(pcd1, pcd2)])   # (B, N, 1)
        nn_i2 = torch.stack([knn_points(pad3(b), pad3(a), 1)[1] for a, b in zip(pcd1, pcd2)])   # (B, M, 1)
        idx = nn_i1.unsqueeze(-1).expand(-1, -1, -1, pcd2.shape[-1])
        nn_distance1 = (pcd1[:, :, None, :] - torch.gather(pcd2[:, :, None, :], 1, idx)).pow(2)
        idx = nn_i2.unsqueeze(-1).expand(-1, -1, -1, pcd1.shape[-1])
        nn_distance2 = (pcd2[:, :, None, :] - torch.gather(pcd1[:, :, None, :], 1, idx)).pow(2)
        return nn_distance1.sum(-1).mean() + nn_distance2.sum(-1).mean()

    def get_transformation_regularisation_loss(self, d=0.0873):
        t = self.forward_warp.prev_global_t.abs()
        thetas = self.forward_warp.prev_thetas.abs()
        return (torch.abs(t).sum() + thetas.sum()) / len(thetas + 1)

    # ------------------------------------------------------------------ reference API
    def _merge_rules(self):
        J = self.weights.shape[1]
        if self.merging_mat is None:
            return None
        rules = self.flat_merging_rules.to(torch.int64)
        if torch.equal(rules.cpu(), torch.arange(J)):
            return None
        return rules

    def get_weights(self):
        """temporalpoints.py:401-414: softmax(W / max(eps, theta)), columns merged by rule."""
        th = torch.max(self.eps.to(self.theta_weight.device), self.theta_weight)
        sm = torch.softmax(self.weights / th, dim=-1)
        rules = self._merge_rules()
        if rules is None:
            return sm
        out = torch.zeros_like(sm)
        out.index_add_(1, rules.to(sm.device), sm)
        return out

    def repose(self, rot_params, sweep_index=None):
        """temporalpoints.py:370-371 -> [xyz (N,3), joints_rel (J,3)] via the fused LBS kernel.
        (``sweep_index``: rot_params is a pose sweep, see capture_repose.)"""
        bone_Ts, global_t, joints_rel = self.forward_warp.pose(self.joints, rot_params=rot_params,
                                                               sweep_index=sweep_index)
        self._mark("frame")
        xyz, _, _ = self._lbs(bone_Ts, global_t, records=False, T34=self.forward_warp.last_T34)
        self._mark("lbs")
        return [xyz, joints_rel]

    def capture_repose(self, rot_dim=4, sweep=None, batched=True, pipelined=False, in_flight=1):
        """The repose step (skeleton launch + fused LBS launch, run.py:1355-1396 sweeps it per pose)
        captured once in a HIP graph: returns ``step(rot_params) -> (xyz, joints_rel)``, which
        copies rot_params [J, rot_dim] into the graph's input and replays it -- no per-pose host
        work besides one copy and one graph launch. The outputs are the graph's static buffers
        (overwritten by the next step). Capture again after changing the model.

        ``sweep`` = the poses of the sweep [P, J, rot_dim] (device): the graph reads pose
        ``index % P`` from the sweep itself and advances a device index, so a step that is given
        the next row of the sweep (the sweep's order, as run.py walks it) is one graph launch with
        no input copy; another row sets the index first (one small fill), and rot_params that are
        not a row of the sweep take the eager path.

        ``batched`` (with a sweep): the skeleton stage of every pose of the sweep runs as ONE launch
        (apn_skeleton_sweep, one workgroup per pose, each pose computed exactly as the per-pose
        launch computes it) at the start of every pass over the sweep -- a step asking for pose 0 --
        and whenever the sweep tensor was modified in place; each step is then one graph launch of
        the LBS kernel reading its pose's bone transforms (one captured graph per pose), so the
        one-workgroup skeleton launch (~10 us of latency plus a dependent launch) leaves the per-pose
        critical path. Every step still skins its pose in full; within a pass each pose's skeleton
        is computed once, as in the per-pose path.
        ``in_flight`` (batched only) = n > 1: poses in flight, pose i on ``step.streams[i % n]``
        into its own output slot ``step.outputs[i % n]`` (so the next pose's LBS starts while this
        one drains, instead of after a graph-launch gap); the returned xyz is then ready on that
        stream only: a consumer waits on it (``torch.cuda.current_stream().wait_stream(...)``) and
        has it until step i + n.
        ``pipelined`` (with a sweep, measured and not kept: 0.066 vs 0.052 ms per pose at C5):
        step i's graph runs pose i's LBS beside pose i + 1's skeleton on a forked side stream."""
        if sweep is not None and batched:
            return self._capture_repose_batched(sweep, in_flight=in_flight)
        if sweep is not None and pipelined:
            return self._capture_repose_pipelined(sweep)
        dev = self.canonical_pcd.device
        J = self.weights.shape[1]
        if sweep is not None:
            sweep = sweep.detach().to(dev, torch.float32).contiguous()
            if sweep.dim() != 3 or sweep.shape[1] != J:
                raise ValueError("capture_repose: sweep must be [P, J, rot_dim]")
            rot_dim = sweep.shape[2]
        rp = torch.zeros(J, rot_dim, device=dev)
        idx = torch.zeros(1, dtype=torch.int32, device=dev)
        with torch.no_grad():
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):   # warm-up: caches, workspaces, packed buffers
                self.repose(rp)
            torch.cuda.current_stream(dev).wait_stream(side)
            with _capture_guard():
                graph = torch.cuda.CUDAGraph()
                self._ws.hold(graph)   # the graph holds workspace addresses from here on
                with torch.cuda.graph(graph):
                    if sweep is None:
                        xyz, joints_rel = self.repose(rp)
                    else:
                        xyz, joints_rel = self.repose(sweep, sweep_index=idx)
        if sweep is None:
            def step(rot_params):
                rp.copy_(rot_params.reshape(J, rot_dim))
                graph.replay()
                return xyz, joints_rel
        else:
            P, row = sweep.shape[0], J * rot_dim * 4
            base = sweep.data_ptr()
            state = {"next": 0}
            idx.zero_()

            def step(rot_params):
                off = rot_params.data_ptr() - base
                if (rot_params.device != sweep.device or not rot_params.is_contiguous() or off < 0 or off % row
                        or off // row >= P or rot_params.numel() != J * rot_dim):
                    with torch.no_grad():
                        return self.repose(rot_params)
                i = off // row
                if i != state["next"]:
                    idx.fill_(i)
                state["next"] = (i + 1) % P
                graph.replay()
                return xyz, joints_rel

        step.graph, step.inputs = graph, (rp if sweep is None else (sweep, idx))
        return step

    def _capture_repose_batched(self, sweep, in_flight=1):
        dev = self.canonical_pcd.device
        N, J = self.weights.shape
        sweep = sweep.detach().to(dev, torch.float32).contiguous()
        if sweep.dim() != 3 or sweep.shape[1] != J:
            raise ValueError("capture_repose: sweep must be [P, J, rot_dim]")
        P, rot_dim = sweep.shape[0], sweep.shape[2]
        fw = self.forward_warp
        bufs = {"thetas": torch.empty(P, J, device=dev), "bone_Ts": torch.empty(P, J, 4, 4, device=dev),
                "T34": torch.empty(P, J, 12, device=dev), "gt": torch.empty(P, 3, device=dev),
                "joints_rel": torch.empty(P, J, 3, device=dev)}
        n_fl = max(1, int(in_flight))
        outs = [torch.empty(N, 3, device=dev) for _ in range(n_fl)]   # pose i -> outs[i % n_fl]

        def lbs(i):
            self._lbs(bufs["bone_Ts"][i], bufs["gt"][i], records=False, T34=bufs["T34"][i], out=outs[i % n_fl])

        with torch.no_grad():
            cur = torch.cuda.current_stream(dev)
            side = torch.cuda.Stream(dev)
            side.wait_stream(cur)
            with torch.cuda.stream(side):   # warm-up: caches, workspaces, packed buffers
                fw.pose_sweep(self.joints, sweep, bufs)
                lbs(0)
            cur.wait_stream(side)
            graphs = []
            with _capture_guard():
                g_skel = torch.cuda.CUDAGraph()
                self._ws.hold(g_skel)
                with torch.cuda.graph(g_skel):
                    fw.pose_sweep(self.joints, sweep, bufs)
                for i in range(P):
                    g = torch.cuda.CUDAGraph()
                    self._ws.hold(g)
                    with torch.cuda.graph(g):
                        lbs(i)
                    graphs.append(g)
        row = J * rot_dim * 4
        base = sweep.data_ptr()
        state = {"ver": None}   # the sweep version the skeleton batch was computed from
        streams = [torch.cuda.Stream(dev) for _ in range(n_fl)] if n_fl > 1 else None

        def step(rot_params):
            off = rot_params.data_ptr() - base
            if (rot_params.device != sweep.device or not rot_params.is_contiguous() or off < 0 or off % row
                    or off // row >= P or rot_params.numel() != J * rot_dim):
                if streams:   # the eager path runs on the caller's stream, after the poses in flight
                    for t in streams:
                        torch.cuda.current_stream(dev).wait_stream(t)
                with torch.no_grad():
                    return self.repose(rot_params)
            i = off // row
            if streams is None:
                if i == 0 or state["ver"] != sweep._version:
                    g_skel.replay()   # every pose's skeleton (a new pass over the sweep, or the sweep changed)
                    state["ver"] = sweep._version
                graphs[i].replay()
                return outs[0], bufs["joints_rel"][i]
            cur = torch.cuda.current_stream(dev)
            if i == 0 or state["ver"] != sweep._version:
                # the skeleton batch is rewritten: after every pose in flight has read it, and after
                # the caller's writes to the sweep; every slot's next pose after it
                for t in streams:
                    cur.wait_stream(t)
                g_skel.replay()
                state["ver"] = sweep._version
                for t in streams:
                    t.wait_stream(cur)
            with torch.cuda.stream(streams[i % n_fl]):
                graphs[i].replay()
            return outs[i % n_fl], bufs["joints_rel"][i]

        step.graph, step.inputs = graphs, (sweep,)
        step.streams, step.outputs = streams, outs
        return step

    def _capture_repose_pipelined(self, sweep):
        dev = self.canonical_pcd.device
        J = self.weights.shape[1]
        sweep = sweep.detach().to(dev, torch.float32).contiguous()
        if sweep.dim() != 3 or sweep.shape[1] != J:
            raise ValueError("capture_repose: sweep must be [P, J, rot_dim]")
        P, rot_dim = sweep.shape[0], sweep.shape[2]
        fw = self.forward_warp
        idx = torch.zeros(1, dtype=torch.int32, device=dev)
        bufs = [fw.pose_buffers(J, dev) for _ in range(2)]

        def skel(k):
            fw.pose(self.joints, rot_params=sweep, sweep_index=idx, out=bufs[k])

        def lbs(k):
            return self._lbs(bufs[k]["bone_Ts"], bufs[k]["gt"], records=False, T34=bufs[k]["T34"])[0]

        with torch.no_grad():
            cur = torch.cuda.current_stream(dev)
            side = torch.cuda.Stream(dev)
            side.wait_stream(cur)
            with torch.cuda.stream(side):   # warm-up: caches, workspaces, packed buffers
                for k in (0, 1):
                    skel(k)
                    lbs(k)
            cur.wait_stream(side)
            prologue, pair, xyz = [], [], []
            with _capture_guard():
                for k in (0, 1):
                    g = torch.cuda.CUDAGraph()
                    self._ws.hold(g)
                    with torch.cuda.graph(g):
                        skel(k)
                    prologue.append(g)
                for k in (0, 1):
                    g = torch.cuda.CUDAGraph()
                    self._ws.hold(g)
                    with torch.cuda.graph(g):
                        cap = torch.cuda.current_stream(dev)
                        fork = torch.cuda.Stream(dev)
                        fork.wait_stream(cap)
                        with torch.cuda.stream(fork):   # the next pose's skeleton, beside this pose's LBS
                            skel(1 - k)
                        xyz.append(lbs(k))
                        cap.wait_stream(fork)
                    pair.append(g)
        row = J * rot_dim * 4
        base = sweep.data_ptr()
        # k: the buffer holding the skeleton of pose `next` (None: nothing prefetched)
        state = {"next": 0, "k": None, "ver": sweep._version}

        def step(rot_params):
            off = rot_params.data_ptr() - base
            if (rot_params.device != sweep.device or not rot_params.is_contiguous() or off < 0 or off % row
                    or off // row >= P or rot_params.numel() != J * rot_dim):
                with torch.no_grad():
                    return self.repose(rot_params)
            i = off // row
            k = state["k"]
            if k is None or i != state["next"] or sweep._version != state["ver"]:
                idx.fill_(i)
                k = 0
                prologue[0].replay()   # pose i's skeleton into buffer 0 (the index moves to i + 1)
                state["ver"] = sweep._version
            pair[k].replay()           # LBS of pose i from buffer k | skeleton of pose i + 1 into 1 - k
            state["next"], state["k"] = (i + 1) % P, 1 - k
            return xyz[k], bufs[k]["joints_rel"]

        step.graph, step.inputs = pair, (sweep, idx)
        return step

    def capture_frame(self, t, render_kwargs, render_depth=True, render_weights=True, query_radius=0.01, poses=None,
                      Ks=None, get_skeleton=False, ray_shard=None, capture_error_mode="global", workspace=None):
        """The render frame for a fixed ray set (skeleton, LBS, grid, sampling, kNN, MLP,
        compositing: the whole no-grad forward) captured once in a HIP graph: returns
        ``step(t) -> RenderOutput``, which copies the time into the graph's input and replays it.
        The outputs are the graph's static buffers (overwritten by the next step); like an eager
        frame they are validated on first read (one read of the device frame_info) and a frame
        whose samples overflowed the capacity is rendered again eagerly. Needs no host sync inside
        the frame: the capacity is set by the warm-up frames. Capture again after changing the
        model or the rays. ``get_skeleton`` (with fixed ``poses`` / ``Ks``) captures the joint
        projection too, as the eager forward runs it. ``ray_shard=(rank, world, block)`` captures
        this rank's frame of the "blocks" ray split (apn_amd.shard.capture_sharded); the
        contiguous-range split is not capturable (its split moves from frame to frame).
        ``capture_error_mode`` goes to torch.cuda.graph ("thread_local" where other threads of the
        process -- a process group's watchdog -- may make HIP calls during the capture).
        ``workspace`` (an ops.Workspace): the per-frame buffers the graph captures (default: the
        model's own); frames in flight give each graph its own (apn_amd.pipeline). A frame that
        overflowed is rendered again in the model's own workspace."""
        if ray_shard is not None and len(ray_shard) != 3:
            raise ValueError("capture_frame: ray_shard must be (rank, world, block) (the blocks split)")
        dev = self.canonical_feat.device
        t_in = torch.as_tensor(t, dtype=torch.float32, device=dev).reshape(-1).clone()
        rk = dict(render_kwargs)
        R = len(rk['rays_o'])
        if get_skeleton:
            poses, Ks = poses.to(dev), Ks.to(dev, torch.float32)   # device-resident before the capture
        args = (render_depth, rk, query_radius, render_weights, None, poses, Ks, True, get_skeleton, ray_shard)
        cap_key = R if ray_shard is None else (R, *ray_shard)
        # sticky overflow flag of every replay since the last step.overflowed() (the OR of the
        # frames' frame_info[2], accumulated inside the graph): a caller that never reads its
        # frames (bench's timed loop) still learns whether any of them dropped samples
        ovf = torch.zeros(1, dtype=torch.int32, device=dev)
        st = {}

        def capture():
            with torch.no_grad(), self.use_workspace(workspace):
                side = torch.cuda.Stream(dev)
                side.wait_stream(torch.cuda.current_stream(dev))
                with torch.cuda.stream(side):   # warm-up: capacity (first frame), caches, workspaces
                    self._forward_render(t_in, *args)
                    warm = self._forward_render(t_in, *args)
                    # validate: an overflow renders again (the model's own workspace) and grows the
                    # capacity; read on the warm-up stream, which is the one that wrote the frame
                    warm.keys()
                torch.cuda.current_stream(dev).wait_stream(side)
                if self._capacity.get(cap_key) is None:
                    raise RuntimeError("capture_frame: no sample capacity for this ray set (empty frame?)")
                st.pop("graph", None)   # a re-capture: drop the old graph first (its retired buffers go with it)
                step.graph = None
                # the captured frame is one chain: the kNN grid build stays on the frame's own stream
                # (its side-stream branch made graphs of frames in flight land on shared hardware
                # queues -- GPU_MAX_HW_QUEUES = 4 -- and serialise: shards of 8 in flight 1.08 or
                # 1.28 ms per frame by capture, 1.01-1.04 ms as one chain; whole frames equal)
                grid_branch, self.concurrent_grid = self.concurrent_grid, False
                try:
                    with _capture_guard():
                        graph = torch.cuda.CUDAGraph()
                        self._ws.hold(graph)          # the graph holds workspace addresses from here on
                        self._ws_shared.hold(graph)   # (and the shared projection's)
                        with torch.cuda.graph(graph, capture_error_mode=capture_error_mode):
                            out = self._forward_render(t_in, *args)
                            if out._info is not None:
                                torch.bitwise_or(ovf, out._info[2:3], out=ovf)
                finally:
                    self.concurrent_grid = grid_branch
            st.update(graph=graph, static={k: dict.__getitem__(out, k) for k in dict.keys(out)}, info=out._info,
                      n_rays=out._n_rays, bg=out._bg, cap=self._capacity.get(cap_key), stale=False)
            step.graph = graph

        cap_ws = workspace if workspace is not None else self._ws_eager

        def step(t):
            if len(self.feat_net) == 6 and cap_ws.meta.get("pack_key") != self._mlp_weights_key():
                # the MLP weights changed since this graph packed them: the shared projection P may
                # already hold the new weights (an eager frame re-projected it), so replaying would
                # mix two models -- capture again (the capture's warm-up repacks this workspace)
                st["stale"] = True
            if st["stale"]:
                # a replay overflowed the captured capacity; its re-render grew the capacity, so
                # capture again (the old graph would overflow -- and re-render -- on every frame)
                t0 = t_in.clone()
                capture()
                t_in.copy_(t0)
            t_in.copy_(torch.as_tensor(t, dtype=torch.float32, device=dev).reshape(-1))
            st["graph"].replay()
            tt = t_in.clone()

            def rerender():
                st["stale"] = True
                self._force_exact = True
                try:
                    with torch.no_grad(), self.use_workspace(None):
                        return self._forward_render(tt, *args)
                finally:
                    self._force_exact = False
            return RenderOutput(dict(st["static"]), n_rays=st["n_rays"], bg=st["bg"], info=st["info"],
                                rerender=rerender)

        def overflowed():
            """True if any replay since the last call dropped samples past the captured capacity
            (one device read; clears the flag)."""
            v = bool(ovf.item())
            ovf.zero_()
            return v

        def invalidate():
            """Capture again before the next replay (the capacity grew: a frame read elsewhere,
            e.g. an assembled ray-shard frame, overflowed and was rendered again)."""
            st["stale"] = True

        capture()
        step.inputs, step.overflowed, step.invalidate = t_in, overflowed, invalidate
        step.capacity = lambda: st["cap"]
        return step

    def sample_ray(self, rays_o, rays_d, near, far, stepsize, xyz_min=None, xyz_max=None, **render_kwargs):
        """temporalpoints.py:373-399 through the render_utils drop-in."""
        from .ops import sample_pts_on_rays
        xyz_min = self.xyz_min if xyz_min is None else xyz_min
        xyz_max = self.xyz_max if xyz_max is None else xyz_max
        pts, mask_out, ray_id, step_id, *_ = sample_pts_on_rays(rays_o.contiguous(), rays_d.contiguous(), xyz_min,
                                                                xyz_max, near, far, stepsize * self.voxel_size)
        m = ~mask_out
        return pts[m], ray_id[m], step_id[m], m

    # ------------------------------------------------------------------ fused pipeline
    def _joint_colors(self, dev):
        """Weight-visualisation colours per LBS column (temporalpoints.py:690-699): seaborn hls
        palette over the columns with non-zero total weight, permuted by randperm(seed 0) on
        the weights' device. Softmax weights are > 0, so those columns are the merge targets."""
        rules = self._merge_rules()
        J = self.weights.shape[1]
        # the reference draws the permutation from a generator on the weights' device; a CPU
        # reference run draws a different one, so the device is selectable for comparisons
        perm_dev = torch.device(self.palette_perm_device) if self.palette_perm_device else dev
        key = (str(dev), str(perm_dev), None if rules is None else tuple(rules.tolist()))
        if key not in self._palette_cache:
            wmask = torch.zeros(J, dtype=torch.bool)
            if rules is None:
                wmask[:] = True
            else:
                wmask[rules.cpu()] = True
            m = int(wmask.sum())
            cols = torch.tensor(hls_palette(m), dtype=torch.float64)
            gen = torch.Generator(device=perm_dev)
            gen.manual_seed(0)
            perm = torch.randperm(m, generator=gen, device=perm_dev).cpu()
            colors = torch.zeros(J, 3, dtype=torch.float64)
            colors[torch.where(wmask)[0]] = cols[perm]
            self._palette_cache[key] = (colors.float().to(dev), perm)
        self.last_palette_perm = self._palette_cache[key][1]
        return self._palette_cache[key][0]

    def _lbs(self, bone_Ts, global_t, records=True, colors=None, T34=None, out=None):
        pcd = self.canonical_pcd.contiguous()
        L.require_cuda(pcd, self.weights, what="TemporalPoints")
        N, J = self.weights.shape
        dev = pcd.device
        ws = self._ws
        xyz = out if out is not None else torch.empty(N, 3, device=dev)
        wout = torch.empty(N, J, device=dev) if records else None
        recA = ws.get("recA", N * 16, torch.float32, dev) if records else None
        recB = ws.get("recB", N * 8, torch.float32, dev) if records else None
        bbox = ws.get("bbox_ord", 8, torch.int32, dev)
        if T34 is None:
            T34 = bone_Ts[:, :3, :].detach().float().reshape(J, 12).contiguous()
        gt = global_t.detach().float().reshape(3).contiguous()
        rules = self._merge_rules()
        rules32 = rules.to(device=dev, dtype=torch.int32).contiguous() if rules is not None else None
        mmd = 0.0
        if records:
            self.mean_min_distance
            mmd = self._mmd_f
        if self.timing is not None:   # HIP events right around the LBS launch (bench: the C5 roofline)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        call("apn_lbs_skin", ptr(pcd), ptr(self.weights.detach().contiguous()), N, J, ptr(self.theta_weight.detach()),
             self._eps, ptr(rules32), ptr(T34), ptr(gt), ptr(colors),
             ptr(self.canonical_alpha.detach().contiguous()) if records else None,
             ptr(self.canonical_rgbs.detach().contiguous()) if records else None,
             ptr(self.direct_eps.detach().contiguous()) if records else None, mmd, 0, ptr(xyz), ptr(wout), None,
             ptr(recA), ptr(recB), ptr(bbox) if records else None,   # the bbox only feeds the render's sampling
             ptr(ws.bytes("lbs_ws", L.load().apn_lbs_workspace_bytes(N), dev)), stream_ptr(dev))
        if self.timing is not None:
            e1.record()
            self.timing.setdefault("lbs_events", []).append((e0, e1))
        return xyz, wout, (recA, recB, bbox)

    def _mlp_weights_key(self):
        """Storage and in-place version of every tensor the packed MLP weights and the layer-1
        projection P are derived from."""
        layers = [self.feat_net[0], self.feat_net[2][0], self.feat_net[3][0], self.feat_net[4]]
        params = [p for l in layers for p in (l.weight, l.bias)] + list(self.densitynet.parameters()) + \
            list(self.rgbnet.parameters()) + [self.canonical_feat]
        return tuple((p.data_ptr(), p._version) for p in params)

    def _packed_weights(self, pose_embedding, dev):
        """Packed MLP weights + the per-point layer-1 projection, cached on parameter versions
        (only the pose-embedding bias fold changes per frame)."""
        if len(self.feat_net) != 6:
            raise NotImplementedError("the fused MLP kernel implements feat_depth=4 (the reference default)")
        from .ops import feat_project, fold_pose_bias, mlp_layout
        layers = [self.feat_net[0], self.feat_net[2][0], self.feat_net[3][0], self.feat_net[4]]
        key = self._mlp_weights_key()
        # the packed buffer (0.5 MB) belongs to the frame's workspace: its b1 follows the frame's
        # pose embedding and its range flag the frame's MLP launch, so frames in flight each keep
        # their own; the projection P (N x 512 B) depends on the weights only and is shared
        buf = self._ws.get("mlp_w", mlp_layout()["TOTAL"], torch.float32, dev)
        if key != self._ws.meta.get("pack_key"):
            pack_mlp_weights(layers, self.densitynet, self.rgbnet, pose_embedding, out=buf)
            self._ws.meta["pack_key"] = key
        elif pose_embedding is not None:   # same weights: only b1 follows the pose embedding
            fold_pose_bias(layers[0], pose_embedding, buf)
        if key != self._ws_shared.meta.get("proj_key") or "feat_proj" not in self._ws_shared.bufs:
            proj = self._ws_shared.get("feat_proj", self.canonical_feat.shape[0] * 128, torch.float32, dev)
            feat_project(self.canonical_feat, buf, out=proj.view(-1, 128))
            self._ws_shared.meta["proj_key"] = key
        return buf, self._ws_shared.bufs["feat_proj"]

    @contextlib.contextmanager
    def use_workspace(self, ws):
        """Run the fused frame in workspace ``ws`` (None: the model's own, used by eager frames).
        Frames in flight (apn_amd.pipeline.FramePipeline) each capture into a workspace of their
        own, so their per-frame buffers never alias; the projection P is shared."""
        prev, self._ws = self._ws, (self._ws_eager if ws is None else ws)
        try:
            yield self._ws
        finally:
            self._ws = prev

    def forward(self, t, render_depth=False, render_kwargs=None, query_radius=0.01, render_weights=False,
                rot_params=None, render_pcd_direct=False, poses=None, Ks=None, cam_per_ray=None, calc_min_max=True,
                get_skeleton=False, ray_shard=None):
        """temporalpoints.py:540-712.

        With autograd enabled (the reference's train_pcd step, run.py:574-716) this is the
        differentiable path ``_forward_train``; under ``torch.no_grad()`` (the reference's render
        loops, run.py:80, 241) it is the fused HIP pipeline.

        ``ray_shard=(rank, world)`` (not in the reference signature) renders only this rank's
        contiguous ray range with ~1/world of the frame's in-bbox samples; the range is left in
        ``self.last_ray_range``. ``ray_shard=(rank, world, block)`` renders the rank's blocks
        k, k + world, ... of ``block`` consecutive rays (their indices in
        ``self.last_ray_index``). Either way ``self.last_ray_count`` is the rank's ray count (see
        apn_amd.shard for the tile all-gather)."""
        assert (t is None) ^ (rot_params is None)
        # feat_depth != 4 (temporalpoints.py:53, 117-130): the fused MLP kernel is built for the
        # reference default; other depths render through the generic GPU path (HIP skinning / kNN /
        # loss kernels, the layers as GEMMs), the same code as the differentiable step
        generic = len(self.feat_net) != 6
        if torch.is_grad_enabled() or generic:
            if ray_shard is not None:
                raise NotImplementedError("ray_shard is a render-path option of the fused pipeline "
                                          "(torch.no_grad(), feat_depth=4)")
            from .train import forward_train
            return forward_train(self, t, render_depth, render_kwargs, query_radius, render_weights, rot_params,
                                 poses, Ks, calc_min_max, get_skeleton)
        with torch.no_grad():
            return self._forward_render(t, render_depth, render_kwargs, query_radius, render_weights, rot_params,
                                        poses, Ks, calc_min_max, get_skeleton, ray_shard)

    def _forward_render(self, t, render_depth, render_kwargs, query_radius, render_weights, rot_params, poses, Ks,
                        calc_min_max, get_skeleton, ray_shard):
        dev = self.canonical_feat.device
        L.require_cuda(self.canonical_feat, what="TemporalPoints.forward")
        self._last_ray_ws = None
        # skeleton stage: time embedding, TransformNet, chain and (get_skeleton) the joint projection
        # in one launch (apn_skeleton_frame)
        proj = (poses, Ks) if get_skeleton else None
        tt = None if rot_params is not None else torch.as_tensor(t, dtype=torch.float32, device=dev).reshape(-1)
        with roctx.stage("skeleton"):
            if tt is not None and tt.numel() == 1:
                bone_Ts, global_t, joints_rel = self.forward_warp.pose(self.joints, tt, None, time_poc=self.time_poc,
                                                                       proj=proj)
            else:
                t_embed = poc_fre(t, self.time_poc) if rot_params is None else None
                bone_Ts, global_t, joints_rel = self.forward_warp.pose(self.joints, t_embed, rot_params, proj=proj)
        colors = self._joint_colors(dev) if render_weights else None
        self._mark("frame")
        with roctx.stage("lbs"):
            t_hat_pcd, weights, recs = self._lbs(bone_Ts, global_t, records=True, colors=colors,
                                                 T34=self.forward_warp.last_T34)
        self._mark("lbs")
        self._last_weights = weights
        pose_embedding = None
        if self.pose_embedding_dim > 0:
            delta_joint = (self.joints - joints_rel).clone().detach()
            pose_embedding = self.pose_embedding_net(poc_fre(delta_joint, self.pos_poc).view(1, -1))
        joints = bones = None
        if get_skeleton:
            joints = self.forward_warp.last_joints2d
            if joints is None:
                joints = project_point_to_image_plane(joints_rel + global_t, poses.to(dev), Ks.to(dev, torch.float32))
            bones = self.bones
            if self.joints_to_keep is not None:
                joints = joints[:, self.joints_to_keep]
                bones = self.new_bones
        R = len(render_kwargs['rays_o'])
        try:
            out = self._render(t_hat_pcd, recs, query_radius, render_kwargs, pose_embedding, calc_min_max,
                               shard=ray_shard)
        except NoPointsException:
            bg = render_kwargs['bg']
            if ray_shard is not None:
                R = self.last_ray_count
            return {'rgb_marched': torch.ones(R, 3, device=dev) * bg,
                    'rgb_marched_direct': torch.ones(R, 3, device=dev) * bg,
                    'depth': torch.zeros(R, device=dev), 'weights': torch.ones(R, 3, device=dev) * bg,
                    't_hat_pcd': t_hat_pcd, 'alphainv_last': None, 'grid': None, 'joints': joints, 'bones': bones}
        rgb, rgb_d, depth, wvis, last, last_d = out
        info = self._last_info

        def rerender():   # the exact path (the frame overflowed its sample capacity)
            self._force_exact = True
            try:
                with torch.no_grad():
                    return self._forward_render(t, render_depth, render_kwargs, query_radius, render_weights,
                                                rot_params, poses, Ks, calc_min_max, get_skeleton, ray_shard)
            finally:
                self._force_exact = False
        ret = RenderOutput({'t_hat_pcd': t_hat_pcd, 'rgb_marched': rgb, 'alphainv_last': last,
                            'alphainv_last_direct': last_d, 'grid': None, 'rgb_marched_direct': rgb_d,
                            'joints': joints, 'bones': bones},
                           nsurv=self.last_stats._nsurv, n_rays=len(rgb), bg=float(render_kwargs['bg']),
                           info=info, rerender=rerender if info is not None else None)
        if render_depth:
            ret['depth'] = depth
        if render_weights:
            ret['weights'] = wvis
        return ret

    def last_kept_per_ray(self, n_rays):
        """kNN survivors per ray of the last fused render (its ray range), from the compositing
        kernel's per-ray segment bounds [beg | end] (rays without survivors: 0, 0); int32 [n_rays]
        (zeros if that frame composited nothing: no in-bbox sample)."""
        if self._last_ray_ws is None or self._last_ray_ws[1] != n_rays:
            return torch.zeros(n_rays, dtype=torch.int32, device=self.canonical_feat.device)
        rws, R = self._last_ray_ws
        return rws[R:2 * R] - rws[:R]

    def _mark(self, name):
        """HIP-event stage marker (only while self.timing is a dict): the time between consecutive
        markers is charged to the stage named by the later one."""
        if self.timing is None:
            return
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        self.timing.setdefault("marks", []).append((name, e))

    def _render(self, xyz, recs, query_radius, rk, pose_embedding, calc_min_max, shard=None):
        # roctx ranges per stage; the Sequence closes an open one if a stage raises
        with roctx.Sequence() as rx:
            return self._render_stages(rx, xyz, recs, query_radius, rk, pose_embedding, calc_min_max, shard)

    def _render_stages(self, rx, xyz, recs, query_radius, rk, pose_embedding, calc_min_max, shard):
        recA, recB, bbox_ord = recs
        dev = xyz.device
        lib = L.load()
        ws = self._ws
        s = stream_ptr(dev)
        N = xyz.shape[0]
        ro = rk['rays_o'].detach().float().contiguous()
        rd = rk['rays_d'].detach().float().contiguous()
        vd = rk['viewdirs'].detach().float().contiguous()
        L.require_cuda(ro, rd, vd, what="render_kwargs")
        R = ro.shape[0]
        block_key = None
        if shard is not None and len(shard) == 3:
            # interleaved ray blocks (shard.py "blocks" split): this rank's rays, gathered
            rank, world, block = shard
            block_key = (R, rank, world, block)
            idx = self._block_index.get(block_key)
            if idx is None or idx.device != dev:
                from .shard import block_rays
                idx = self._block_index[block_key] = block_rays(R, rank, world, block).to(dev)
            R = idx.numel()
            self.last_ray_index, self.last_ray_range, self.last_ray_count = idx, None, R
            if R == 0:
                raise NoPointsException("No rays in this shard.")
            # the three ray arrays gathered in one launch (apn_gather_rays)
            g_o = ws.get("shard_rays_o", R * 3, torch.float32, dev).view(R, 3)
            g_d = ws.get("shard_rays_d", R * 3, torch.float32, dev).view(R, 3)
            g_v = ws.get("shard_viewdirs", R * 3, torch.float32, dev).view(R, 3)
            call("apn_gather_rays", ptr(ro), ptr(rd), ptr(vd), ptr(idx), R, ptr(g_o), ptr(g_d), ptr(g_v), s)
            ro, rd, vd = g_o, g_d, g_v
        qr = float(query_radius)
        stepdist = float(rk['stepsize']) * float(self.voxel_size)
        interval = float(rk['stepsize']) * float(self.tineuvox.voxel_size_ratio)
        bg = float(rk['bg'])
        near, far = float(rk['near']), float(rk['far'])
        # sampling bbox (temporalpoints.py:423-427)
        rx.switch("sampling")
        if calc_min_max:
            bbox6 = ws.get("bbox6", 6, torch.float32, dev)
            call("apn_bbox_unpack", ptr(bbox_ord), qr, ptr(bbox6), s)
        else:
            bbox6 = torch.cat([self.xyz_min, self.xyz_max]).float().contiguous()
        self._mark("bbox")
        # kNN grid over the warped cloud. Outside stage timing it runs on a side stream, concurrently
        # with the in-bbox sampling below (neither reads the other's output; joined before the kNN),
        # so the grid build's short launches overlap the sampling's (also inside a captured frame)
        gws = ws.bytes("grid_ws", lib.apn_grid_workspace_bytes(N, CELL_CAP), dev)
        sorted4 = ws.get("sorted4", N * 4, torch.float32, dev)
        side = None
        if self.timing is None and self.concurrent_grid:
            cur = torch.cuda.current_stream(dev)
            side = self._side_streams.get(dev)
            if side is None:
                side = self._side_streams[dev] = torch.cuda.Stream(dev)
            side.wait_stream(cur)
            xyz.record_stream(side)
            with torch.cuda.stream(side):
                call("apn_grid_build", ptr(xyz), N, ptr(bbox_ord), qr, CELL_CAP, ptr(sorted4), ptr(gws),
                     stream_ptr(dev))
                grid_ready = torch.cuda.Event()
                grid_ready.record(side)
        else:
            call("apn_grid_build", ptr(xyz), N, ptr(bbox_ord), qr, CELL_CAP, ptr(sorted4), ptr(gws), s)
        self._mark("grid")
        # in-bbox samples
        offs = ws.get("offs", R + 1, torch.int32, dev)
        sws = ws.bytes("samp_ws", lib.apn_sample_pts_on_rays_workspace_bytes(R), dev)
        call("apn_inbbox_count", ptr(ro), ptr(rd), ptr(bbox6), near, far, stepdist, R, ptr(offs), ptr(sws), s)
        cap_key = R if block_key is None else block_key
        if shard is not None and block_key is None:
            # contiguous ray range holding ~1/world of the in-bbox samples; after
            # the first frame, the split of the previous frame's counts (no host sync, shard.py)
            rank, world = shard
            tracker = self._splits.setdefault((R, world), SplitTracker())
            bounds = tracker.bounds_for(offs, world, advance=not self._force_exact)
            self.last_split_tracker, self.last_full_offsets = tracker, offs
            cap_key = (R, rank, world)
            pend = self._cap_updates.pop(cap_key, None)   # the max share of an assembled frame (shard.py)
            if pend is not None:
                if pend[1].query():
                    self._capacity[cap_key] = max(self._capacity.get(cap_key, 0), _grow_capacity(int(pend[0][0])))
                else:
                    self._cap_updates[cap_key] = pend
            r0, r1 = bounds[rank], bounds[rank + 1]
            self.last_ray_range = (r0, r1)
            self.last_ray_bounds = bounds
            self.last_ray_count = r1 - r0
            ro, rd, vd = ro[r0:r1], rd[r0:r1], vd[r0:r1]
            offs = (offs[r0:r1 + 1] - offs[r0]).contiguous()
            R = r1 - r0
        # In-bbox sample count: the first frame of a ray count reads it (one host sync) and sizes
        # a capacity from it; later frames keep the count on the device -- buffers and launch
        # bounds use the capacity, apn_inbbox_fill_capped drops samples past it and reports an
        # overflow, which RenderOutput checks when the frame is first read (and then renders the
        # frame again on this exact path); a ray shard's capacity is keyed by its rank.
        cap = None if self._force_exact else self._capacity.get(cap_key)
        info = None
        if cap is None:
            n_bbox = int(offs[R].item())
            self.last_stats = FrameStats({"rays": R, "inbbox_samples": n_bbox})
            if n_bbox == 0:
                raise NoPointsException("No points.")
            self._capacity[cap_key] = max(self._capacity.get(cap_key, 0), _grow_capacity(n_bbox))
            Q = n_bbox
            q_pos = ws.get("q_pos", Q * 4, torch.float32, dev)
            q_ray = ws.get("q_ray", Q, torch.int32, dev)
            call("apn_inbbox_fill", ptr(ro), ptr(rd), ptr(bbox6), near, far, stepdist, R, ptr(offs), ptr(q_pos),
                 ptr(q_ray), s)
            nq_dev = C.c_void_p(offs.data_ptr() + 4 * R)
            nsurv = torch.empty(1, dtype=torch.int32, device=dev)   # per frame: FrameStats may read it later
        else:
            Q = cap
            q_pos = ws.get("q_pos", Q * 4, torch.float32, dev)
            q_ray = ws.get("q_ray", Q, torch.int32, dev)
            info = torch.empty(4, dtype=torch.int32, device=dev)   # {queries, total, overflow, survivors}
            call("apn_inbbox_fill_capped", ptr(ro), ptr(rd), ptr(bbox6), near, far, stepdist, R, ptr(offs), Q,
                 ptr(q_pos), ptr(q_ray), ptr(info), s)
            nq_dev = ptr(info)
            nsurv = info[3:]
            self.last_stats = FrameStats({"rays": R}, info=info)
        self._mark("sampling")
        agrid_ready = None
        if side is not None:
            # the kNN's second grid (needed by launches of more than 2^18 queries) continues on the
            # side stream, beside the kNN's first passes; apn_knn_radius_ev waits for it before the
            # passes that read it. The kNN itself waits only for the fine grid.
            if AGRID_SIDE and lib.apn_knn_uses_agrid(Q):
                with torch.cuda.stream(side):
                    call("apn_knn_agrid_build", ptr(gws), N, CELL_CAP, ptr(sorted4), stream_ptr(dev))
                    agrid_ready = torch.cuda.Event()
                    agrid_ready.record(side)
            cur.wait_event(grid_ready)
        rx.switch("knn")
        # radius kNN + compaction of survivors
        s_pos = ws.get("s_pos", Q * 4, torch.float32, dev)
        s_ray = ws.get("s_ray", Q, torch.int32, dev)
        s_nbr = ws.get("s_nbr", Q * 8, torch.int32, dev)
        kws = ws.bytes("knn_ws", lib.apn_knn_workspace_bytes(Q), dev)
        if agrid_ready is not None:
            call("apn_knn_radius_ev", ptr(q_pos), ptr(q_ray), Q, nq_dev, ptr(gws), N, CELL_CAP, ptr(sorted4), qr,
                 ptr(s_pos), ptr(s_ray), ptr(s_nbr), ptr(nsurv), ptr(kws), C.c_void_p(agrid_ready.cuda_event), s)
            cur.wait_stream(side)   # the side stream's work is joined before the frame ends
        else:
            call("apn_knn_radius", ptr(q_pos), ptr(q_ray), Q, nq_dev, ptr(gws), N,
                 CELL_CAP, ptr(sorted4), qr, ptr(s_pos), ptr(s_ray), ptr(s_nbr), ptr(nsurv), ptr(kws), s)
        self._mark("knn")
        rx.switch("mlp")
        # The survivor count stays on the device: the MLP and compositing kernels read it there and
        # Q bounds it, so no sync here. (If no sample survives, the kernels produce the
        # reference's NoPointsException values -- bg colour, depth 0 -- and RenderOutput gives
        # the reference's key set and alphainv_last=None when they are read.)
        S = Q
        self.last_stats._nsurv = nsurv
        self._last_info = info
        # neighbour MLP + heads + direct blend
        wbuf, proj = self._packed_weights(pose_embedding, dev)
        out12 = ws.get("out12", S * 12, torch.float32, dev)
        feat = proj
        vemb = self.viewdirs_emb.detach().reshape(-1).float().contiguous() if self.frozen_view_dir is not None else None
        if self.no_view_dir:
            raise NotImplementedError("no_view_dir=True breaks the reference forward (viewdirs_emb_reshape undefined)")
        if self.timing is not None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            self.timing.setdefault("marks", []).append(("mlp_setup", e0))
        if self.early_termination:
            ews = ws.bytes("ert_ws", lib.apn_point_mlp_ert_workspace_bytes(S, R), dev)
            rows = ws.get("ert_rows", ERT_PASSES, torch.int32, dev)
            self.last_mlp_rows = rows[:ERT_PASSES]
            pass_ev = evs = None
            if self.timing is not None:   # HIP events around each pass's MLP launches (bench's roofline)
                pass_ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * ERT_PASSES)]
                for e in pass_ev:
                    e.record()   # creates the event (the library records it again at its place)
                evs = (C.c_void_p * (2 * ERT_PASSES))(*[e.cuda_event for e in pass_ev])
                self.timing.setdefault("mlp_pass_events", []).append(pass_ev)
            # the direct-blend kernel runs inside, on this stream: on the grid's side stream beside the
            # passes (apn_direct_blend + with_direct = 0) the captured frames in flight stopped
            # overlapping (C2, 3 in flight: 6.58-6.60 vs 5.91-5.95 ms/frame, tools/ab_direct_side.sh)
            call("apn_point_mlp_ert", ptr(s_pos), ptr(s_ray), ptr(s_nbr), S, ptr(nsurv), R, ptr(recA), ptr(recB),
                 ptr(feat), 128, ptr(vd), ptr(vemb), ptr(wbuf), self._eps, float(self.tineuvox.act_shift), interval,
                 float(self.fast_color_thres), 1, ptr(out12), ptr(ews), ptr(rows), evs, s)
        else:
            self.last_mlp_rows = None
            call("apn_point_mlp", ptr(s_pos), ptr(s_ray), ptr(s_nbr), S, ptr(nsurv), ptr(recA), ptr(recB), ptr(feat),
                 128, ptr(vd), ptr(vemb), ptr(wbuf), self._eps, float(self.tineuvox.act_shift), interval, 0,
                 ptr(out12), s)
        if self.timing is not None:
            e1.record()
            rows = self.last_mlp_rows.clone() if self.last_mlp_rows is not None else None
            self.timing.setdefault("mlp_events", []).append((e0, e1, nsurv.clone(), rows))
            self.timing["marks"].append(("mlp", e1))
        rx.switch("composite")
        # compositing
        rgb = torch.empty(R, 3, device=dev); rgb_d = torch.empty(R, 3, device=dev)
        depth = torch.empty(R, device=dev); wvis = torch.empty(R, 3, device=dev)
        last = torch.empty(R, device=dev); last_d = torch.empty(R, device=dev)
        rws = ws.get("ray_ws", 2 * R, torch.int32, dev)
        self._last_ray_ws = (rws, R)
        call("apn_composite", ptr(out12), ptr(s_pos), ptr(s_ray), S, ptr(nsurv), R, float(self.fast_color_thres), bg,
             ptr(rgb), ptr(rgb_d), ptr(depth), ptr(wvis), ptr(last), ptr(last_d), ptr(rws), s)
        self._mark("composite")
        rx.switch(None)
        return rgb, rgb_d, depth, wvis, last, last_d
