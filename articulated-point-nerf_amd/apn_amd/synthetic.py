"""Synthetic scenes for the articulated-point render path.

The reference's datasets (D-NeRF / WIM / ZJU-MoCap) are not available offline, so every
benchmark and parity case runs on a procedurally generated scene of the same *shape*:

* a skeleton whose bone list satisfies the reference invariant ``bones[k] == [parent, k+1]``
  (skeletonizer.py:110-113, temporalpoints.py:236-249) -- SMPL topology for J=24, a 3-arm
  star for J=8, and longest-bone splitting for J=32/48;
* N canonical points in capsules of radius 0.08 around the bones;
* per-point features ~ N(0, 0.5^2), alpha/rgb ~ U(0,1), direct_eps = 0.05;
* network weights from PyTorch's default ``nn.Linear`` init under seed 0, with the
  ``densitynet`` bias set to +8 so compositing saturates and early ray termination fires;
* a D-NeRF-like camera (``pose_spherical``, load_dnerf.py:62-67) or a ZJU-like OpenCV camera
  (``inverse_y=True``; tineuvox.py:690-693).

Everything is generated on the CPU from ``torch.Generator().manual_seed(seed)`` so the same
scene can be rebuilt bit-identically on the GPU box. Nothing here reads /root/reference.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import torch

# SMPL joint parents (public SMPL kinematic tree). bones[k] = [parent(k+1), k+1].
SMPL_PARENTS = [-1, 0, 0, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 9, 9, 12, 13, 14, 16, 17, 18, 19, 20, 21]

# Hand-placed jumping-jacks-like SMPL joint layout, z up (metres-ish before normalisation).
_SMPL_JOINTS_Z_UP = [
    (0.00, 0.00, 0.95),    # 0 pelvis
    (0.09, 0.00, 0.87),    # 1 L hip
    (-0.09, 0.00, 0.87),   # 2 R hip
    (0.00, -0.01, 1.05),   # 3 spine1
    (0.13, 0.01, 0.50),    # 4 L knee
    (-0.13, 0.01, 0.50),   # 5 R knee
    (0.00, -0.01, 1.18),   # 6 spine2
    (0.16, -0.02, 0.09),   # 7 L ankle
    (-0.16, -0.02, 0.09),  # 8 R ankle
    (0.00, 0.00, 1.24),    # 9 spine3
    (0.17, 0.10, 0.03),    # 10 L foot
    (-0.17, 0.10, 0.03),   # 11 R foot
    (0.00, 0.00, 1.46),    # 12 neck
    (0.08, 0.00, 1.38),    # 13 L collar
    (-0.08, 0.00, 1.38),   # 14 R collar
    (0.00, 0.03, 1.63),    # 15 head
    (0.19, 0.00, 1.41),    # 16 L shoulder
    (-0.19, 0.00, 1.41),   # 17 R shoulder
    (0.44, 0.00, 1.47),    # 18 L elbow
    (-0.44, 0.00, 1.47),   # 19 R elbow
    (0.68, 0.00, 1.55),    # 20 L wrist
    (-0.68, 0.00, 1.55),   # 21 R wrist
    (0.77, 0.00, 1.58),    # 22 L hand
    (-0.77, 0.00, 1.58),   # 23 R hand
]


def smpl24_skeleton(height: float = 2.0):
    """24-joint SMPL-topology skeleton, centred, scaled to ``height`` along z."""
    j = np.asarray(_SMPL_JOINTS_Z_UP, dtype=np.float64)
    lo, hi = j.min(0), j.max(0)
    j = (j - 0.5 * (lo + hi)) * (height / (hi[2] - lo[2]))
    bones = [[SMPL_PARENTS[k], k] for k in range(1, 24)]
    return torch.tensor(j, dtype=torch.float32), bones


def star8_skeleton():
    """8-joint three-armed star: bones {[0,1],[0,2],[0,3],[1,4],[2,5],[3,6],[4,7]}."""
    j = np.array([
        (0.0, 0.0, 0.0), (0.3, 0.0, 0.3), (-0.3, 0.0, 0.3), (0.0, 0.05, -0.4),
        (0.6, 0.0, 0.6), (-0.6, 0.0, 0.6), (0.0, 0.1, -0.8), (0.9, 0.0, 0.85)], dtype=np.float32)
    bones = [[0, 1], [0, 2], [0, 3], [1, 4], [2, 5], [3, 6], [4, 7]]
    return torch.from_numpy(j), bones


def split_to(joints: torch.Tensor, bones, J: int):
    """Grow a skeleton to J joints by splitting the longest bone at its midpoint.

    The new joint gets index len(joints); bones are re-sorted by child index so
    ``bones[k] == [parent, k+1]`` keeps holding.
    """
    joints = joints.clone()
    parent = {c: p for p, c in bones}
    while len(joints) < J:
        lens = {c: float((joints[c] - joints[p]).norm()) for c, p in parent.items()}
        c = max(lens, key=lambda k: (lens[k], -k))
        p = parent[c]
        m = len(joints)
        joints = torch.cat([joints, (0.5 * (joints[p] + joints[c]))[None]], 0)
        parent[m] = p
        parent[c] = m
    bones = [[parent[c], c] for c in range(1, len(joints))]
    return joints, bones


def skeleton_for(J: int):
    if J == 8:
        return star8_skeleton()
    base_j, base_b = smpl24_skeleton()
    if J == 24:
        return base_j, base_b
    if J > 24:
        return split_to(base_j, base_b, J)
    raise ValueError(f"no synthetic skeleton with J={J}")


def capsule_points(joints: torch.Tensor, bones, N: int, radius: float, gen: torch.Generator):
    """N points uniform along bones chosen proportional to (length + radius), with a radial
    offset uniform in a ball of ``radius``."""
    a = torch.stack([joints[p] for p, _ in bones]).double()
    b = torch.stack([joints[c] for _, c in bones]).double()
    prob = (b - a).norm(dim=1) + radius
    bone = torch.multinomial(prob / prob.sum(), N, replacement=True, generator=gen)
    t = torch.rand(N, generator=gen, dtype=torch.float64)
    d = torch.randn(N, 3, generator=gen, dtype=torch.float64)
    d = d / d.norm(dim=1, keepdim=True).clamp_min(1e-12)
    r = radius * torch.rand(N, generator=gen, dtype=torch.float64) ** (1.0 / 3.0)
    pts = a[bone] + t[:, None] * (b[bone] - a[bone]) + d * r[:, None]
    return pts.float()


# ----------------------------------------------------------------------------------------
# Cameras (restated from the reference conventions; see docstring)
# ----------------------------------------------------------------------------------------

def pose_spherical(theta_deg: float, phi_deg: float, radius: float) -> torch.Tensor:
    """D-NeRF spherical pose: swap @ Ry(theta) @ Rx(phi) @ T_z(radius) (load_dnerf.py:62-67)."""
    th, ph = math.radians(theta_deg), math.radians(phi_deg)
    trans = np.eye(4); trans[2, 3] = radius
    rphi = np.eye(4); rphi[1, 1] = math.cos(ph); rphi[1, 2] = -math.sin(ph); rphi[2, 1] = math.sin(ph); rphi[2, 2] = math.cos(ph)
    rth = np.eye(4); rth[0, 0] = math.cos(th); rth[0, 2] = -math.sin(th); rth[2, 0] = math.sin(th); rth[2, 2] = math.cos(th)
    swap = np.array([[-1, 0, 0, 0], [0, 0, 1, 0], [0, 1, 0, 0], [0, 0, 0, 1]], dtype=np.float64)
    c2w = swap @ (rth.astype(np.float32).astype(np.float64) @ (rphi.astype(np.float32).astype(np.float64) @ trans))
    return torch.tensor(c2w, dtype=torch.float32)


def look_at_opencv(eye, target=(0.0, 0.0, 0.0), up=(0.0, 0.0, 1.0)) -> torch.Tensor:
    """OpenCV-convention camera (x right, y down, z forward) used with ``inverse_y=True``."""
    eye = np.asarray(eye, np.float64); target = np.asarray(target, np.float64); up = np.asarray(up, np.float64)
    z = target - eye; z /= np.linalg.norm(z)
    x = np.cross(z, up); x /= np.linalg.norm(x)
    y = np.cross(z, x)
    c2w = np.eye(4)
    c2w[:3, 0], c2w[:3, 1], c2w[:3, 2], c2w[:3, 3] = x, y, z, eye
    return torch.tensor(c2w, dtype=torch.float32)


def intrinsics(H: int, W: int, focal: float) -> torch.Tensor:
    return torch.tensor([[focal, 0.0, 0.5 * W], [0.0, focal, 0.5 * H], [0.0, 0.0, 1.0]], dtype=torch.float32)


def get_rays(H: int, W: int, K: torch.Tensor, c2w: torch.Tensor, inverse_y: bool = False):
    """Pixel-centre rays, row-major (H, W) flatten (tineuvox.py:675-703, mode='center').

    Returns rays_o, rays_d (not normalised), viewdirs (normalised), each (H*W, 3) float32,
    on the device of ``c2w``.
    """
    dev = c2w.device
    i = torch.arange(W, device=dev, dtype=torch.float32)[None, :].expand(H, W) + 0.5
    j = torch.arange(H, device=dev, dtype=torch.float32)[:, None].expand(H, W) + 0.5
    K = K.to(dev)
    if inverse_y:
        dirs = torch.stack([(i - K[0][2]) / K[0][0], (j - K[1][2]) / K[1][1], torch.ones_like(i)], -1)
    else:
        dirs = torch.stack([(i - K[0][2]) / K[0][0], -(j - K[1][2]) / K[1][1], -torch.ones_like(i)], -1)
    rays_d = torch.sum(dirs[..., None, :] * c2w[:3, :3], -1)
    rays_o = c2w[:3, 3].expand(rays_d.shape)
    viewdirs = rays_d / rays_d.norm(dim=-1, keepdim=True)
    return (rays_o.reshape(-1, 3).contiguous(), rays_d.reshape(-1, 3).contiguous(),
            viewdirs.reshape(-1, 3).contiguous())


# ----------------------------------------------------------------------------------------
# Scenes
# ----------------------------------------------------------------------------------------

@dataclass
class SceneConfig:
    name: str
    N: int
    J: int
    H: int
    W: int
    camera: str = "dnerf"            # "dnerf" | "zju"
    pose_embedding_dim: int = 0
    t: float = 0.3
    seed: int = 0
    feat_dim: int = 128
    fp16_exact: bool = False         # round features to fp16-representable values (fixtures)


CONFIGS = {
    # BASELINE.json configs
    "C1": SceneConfig("dnerf/jumpingjacks 64x64 10k pts 8 bones", 10_000, 8, 64, 64),
    "C2": SceneConfig("dnerf/jumpingjacks 800x800 300k pts 24 bones", 300_000, 24, 800, 800),
    "C3": SceneConfig("wim/spot 800x800 500k pts 32 bones", 500_000, 32, 800, 800),
    "C4": SceneConfig("zju/313 1024x1024 400k pts 24 bones pose-emb 64", 400_000, 24, 1024, 1024,
                      camera="zju", pose_embedding_dim=64),
    "C5": SceneConfig("repose_pcd 1M pts 48 bones LBS-only", 1_000_000, 48, 0, 0),
    # small parity cases (golden fixtures)
    "G1": SceneConfig("golden dnerf 48x48 4k pts 8 bones", 4_000, 8, 48, 48, fp16_exact=True),
    "G2": SceneConfig("golden zju 40x40 3k pts 8 bones pose-emb 64", 3_000, 8, 40, 40,
                      camera="zju", pose_embedding_dim=64, fp16_exact=True),
    "G3": SceneConfig("golden dnerf 40x40 2.5k pts 24 bones", 2_500, 24, 40, 40, fp16_exact=True),
    # features and network weights NOT fp16-representable: the reference itself then pins the lo
    # halves of the fp16-split MLP contraction
    "G4": SceneConfig("golden dnerf 48x48 4k pts 24 bones non-fp16-exact", 4_000, 24, 48, 48, fp16_exact=False),
}

# Render settings shared by every config (configs/nerf/default.py:57-66, 117-126)
VOXEL_SIZE = 0.034
STEPSIZE = 0.5
FAST_COLOR_THRES = 1e-4
QUERY_RADIUS = 0.01
NEIGHBOURS = 8
POSBASE_PE, VIEWBASE_PE, TIMEBASE_PE = 10, 4, 8
ALPHA_INIT = 1e-3
NET_WIDTH = 128


def camera_for(cfg: SceneConfig):
    """Returns (c2w, K, near, far, bg, inverse_y)."""
    if cfg.camera == "dnerf":
        c2w = pose_spherical(30.0, -30.0, 4.0)
        focal = 0.5 * cfg.W / math.tan(0.5 * 0.6911112)
        return c2w, intrinsics(cfg.H, cfg.W, focal), 2.0, 6.0, 1.0, False
    if cfg.camera == "zju":
        eye = (2.6 * math.cos(math.radians(40)) * math.cos(math.radians(15)),
               2.6 * math.sin(math.radians(40)) * math.cos(math.radians(15)),
               2.6 * math.sin(math.radians(15)))
        c2w = look_at_opencv(eye)
        focal = 0.5 * cfg.W / math.tan(0.5 * 0.85)
        return c2w, intrinsics(cfg.H, cfg.W, focal), 1.0, 4.0, 0.0, True
    raise ValueError(cfg.camera)


def make_network_params(J: int, pose_embedding_dim: int, seed: int, feat_dim: int = NET_WIDTH):
    """Random-init weights for every network on the path, keyed by the reference state-dict
    names. PyTorch default nn.Linear init under ``torch.manual_seed(seed)``."""
    state = {}
    cpu_rng = torch.random.get_rng_state()
    torch.manual_seed(seed)
    try:
        t_dim = 1 + 2 * TIMEBASE_PE
        # TransformNet 17 -> 256 x4 -> (J+1)*4, no bias on the last layer (pointwarper.py:5-27)
        dims = [t_dim, 256, 256, 256, 256]
        for li in range(4):
            lin = torch.nn.Linear(dims[li], dims[li + 1])
            state[f"forward_warp.transform_net.net.{2 * li}.weight"] = lin.weight.detach().clone()
            state[f"forward_warp.transform_net.net.{2 * li}.bias"] = lin.bias.detach().clone()
        lin = torch.nn.Linear(256, (J + 1) * 4, bias=False)
        state["forward_warp.transform_net.net.8.weight"] = lin.weight.detach().clone()
        # feat_net (temporalpoints.py:117-130), feat_depth=4
        d_in = feat_dim + 3 + 3 * POSBASE_PE * 2 + pose_embedding_dim
        names = ["feat_net.0", "feat_net.2.0", "feat_net.3.0", "feat_net.4"]
        fins = [d_in, feat_dim, feat_dim, feat_dim]
        for nm, fi in zip(names, fins):
            lin = torch.nn.Linear(fi, feat_dim)
            state[nm + ".weight"] = lin.weight.detach().clone()
            state[nm + ".bias"] = lin.bias.detach().clone()
        # densitynet Linear(128 -> 1) with +8 bias
        lin = torch.nn.Linear(feat_dim, 1)
        state["densitynet.weight"] = lin.weight.detach().clone()
        state["densitynet.bias"] = torch.full((1,), 8.0)
        # RGBNet(W=128, h_ch=128, views_ch=27) (tineuvox.py:65-88)
        views_ch = 3 + 3 * VIEWBASE_PE * 2
        lin = torch.nn.Linear(feat_dim, NET_WIDTH)
        state["rgbnet.feature_linears.weight"] = lin.weight.detach().clone()
        state["rgbnet.feature_linears.bias"] = lin.bias.detach().clone()
        lin = torch.nn.Linear(NET_WIDTH + views_ch, NET_WIDTH // 2)
        state["rgbnet.views_linears.0.weight"] = lin.weight.detach().clone()
        state["rgbnet.views_linears.0.bias"] = lin.bias.detach().clone()
        lin = torch.nn.Linear(NET_WIDTH // 2, 3)
        state["rgbnet.views_linears.2.weight"] = lin.weight.detach().clone()
        state["rgbnet.views_linears.2.bias"] = lin.bias.detach().clone()
        # pose_embedding_net (temporalpoints.py:161-171)
        if pose_embedding_dim > 0:
            pin = J * (3 * POSBASE_PE * 2 + 3)
            dims = [pin, pin // 2, pin // 2, pin // 2, pose_embedding_dim]
            names = ["pose_embedding_net.0", "pose_embedding_net.2.0", "pose_embedding_net.3.0",
                     "pose_embedding_net.4"]
            for nm, a, b in zip(names, dims[:-1], dims[1:]):
                lin = torch.nn.Linear(a, b)
                state[nm + ".weight"] = lin.weight.detach().clone()
                state[nm + ".bias"] = lin.bias.detach().clone()
    finally:
        torch.random.set_rng_state(cpu_rng)
    return state


@dataclass
class Scene:
    cfg: SceneConfig
    ctor: dict            # TemporalPoints constructor kwargs (minus ``tineuvox``)
    params: dict          # state-dict-keyed tensors to load with strict=False
    c2w: torch.Tensor
    K: torch.Tensor
    near: float
    far: float
    bg: float
    inverse_y: bool
    extra: dict = field(default_factory=dict)

    def rays(self, device="cpu"):
        return get_rays(self.cfg.H, self.cfg.W, self.K, self.c2w.to(device), inverse_y=self.inverse_y)

    def render_kwargs(self, device="cpu"):
        ro, rd, vd = self.rays(device)
        return {"rays_o": ro, "rays_d": rd, "viewdirs": vd, "near": self.near, "far": self.far,
                "bg": self.bg, "stepsize": STEPSIZE, "render_depth": True, "inverse_y": self.inverse_y}


def make_scene(name_or_cfg) -> Scene:
    cfg = CONFIGS[name_or_cfg] if isinstance(name_or_cfg, str) else name_or_cfg
    gen = torch.Generator().manual_seed(cfg.seed)
    joints, bones = skeleton_for(cfg.J)
    pcd = capsule_points(joints, bones, cfg.N, 0.08, gen)
    feat = torch.randn(cfg.N, cfg.feat_dim, generator=gen) * 0.5
    alpha = torch.rand(cfg.N, generator=gen)
    rgbs = torch.rand(cfg.N, 3, generator=gen)
    if cfg.fp16_exact:
        feat = feat.half().float()
    skel = torch.cat([joints[p][None] + torch.linspace(0, 1, 10)[:, None] * (joints[c] - joints[p])[None]
                      for p, c in bones], 0)
    lo = pcd.min(0)[0] - 0.3
    hi = pcd.max(0)[0] + 0.3
    ctor = dict(canonical_pcd=pcd, canonical_alpha=alpha, canonical_feat=feat, canonical_rgbs=rgbs,
                skeleton_pcd=skel, joints=joints, bones=bones, xyz_min=lo.numpy(), xyz_max=hi.numpy(),
                neighbours=NEIGHBOURS, timebase_pe=TIMEBASE_PE, stepsize=STEPSIZE,
                voxel_size=VOXEL_SIZE, fast_color_thres=FAST_COLOR_THRES,
                pose_embedding_dim=cfg.pose_embedding_dim)
    params = make_network_params(cfg.J, cfg.pose_embedding_dim, cfg.seed, cfg.feat_dim)
    if cfg.fp16_exact:
        params = {k: v.half().float() for k, v in params.items()}
    if cfg.H > 0:
        c2w, K, near, far, bg, inv_y = camera_for(cfg)
    else:
        c2w, K, near, far, bg, inv_y = torch.eye(4), torch.eye(3), 2.0, 6.0, 1.0, False
    return Scene(cfg, ctor, params, c2w, K, near, far, bg, inv_y)


@dataclass
class View:
    """One frame of a render loop: its time (a [1] tensor on the device), camera-to-world pose,
    intrinsics and rays (rays_o, rays_d, viewdirs), all resident on the device."""
    t: torch.Tensor
    c2w: torch.Tensor
    K: torch.Tensor
    rays: tuple


def view_sweep(scene: Scene, n: int = 16, device="cpu") -> list:
    """n distinct frames of the scene's render loop, as run.py:108-151 renders them: every frame
    a new time and a new camera pose. View 0 is the scene's own frame (cfg.t, its camera); view i
    orbits the camera by 360 i / n degrees about the scene's vertical axis at the same elevation
    and distance (D-NeRF: pose_spherical(30 + 360 i / n, -30, 4); ZJU: the look-at eye at azimuth
    40 + 360 i / n) and advances the time by 0.6 i / n (t stays in [0, 1))."""
    cfg = scene.cfg
    views = []
    for i in range(n):
        t = (cfg.t + 0.6 * i / n) % 1.0
        if cfg.camera == "dnerf":
            c2w = pose_spherical(30.0 + 360.0 * i / n, -30.0, 4.0)
        elif cfg.camera == "zju":
            az, el = math.radians(40.0 + 360.0 * i / n), math.radians(15)
            c2w = look_at_opencv((2.6 * math.cos(az) * math.cos(el), 2.6 * math.sin(az) * math.cos(el),
                                  2.6 * math.sin(el)))
        else:
            raise ValueError(cfg.camera)
        if i == 0:
            c2w, t = scene.c2w.clone(), cfg.t
        c2w = c2w.to(device)
        rays = get_rays(cfg.H, cfg.W, scene.K, c2w, inverse_y=scene.inverse_y)
        views.append(View(torch.tensor([t], dtype=torch.float32, device=device), c2w, scene.K.to(device), rays))
    return views


def repose_sweep(J: int, steps: int = 30, seed: int = 0) -> torch.Tensor:
    """run.py:1364-1377: randn(J,4)*0.2 with row 0 zero, linear ramp of ``steps`` + reverse."""
    g = torch.Generator().manual_seed(seed)
    target = torch.randn((J, 4), generator=g) * 0.2
    target[0] = 0.0
    ramp = target[None] * torch.linspace(0, 1, steps)[:, None, None]
    return torch.cat([ramp, ramp.flip(0)], 0)
