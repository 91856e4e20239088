"""The pieces of the reference's ``lib/tineuvox.py`` that the point render path uses
(SURVEY.md §2 row 4): RGBNet, the density head holder, poc_fre, Raw2Alpha /
Alphas2Weights (re-exported from ``ops``: HIP forward and backward) and ray generation.

The TiNeuVox voxel model itself (stage 1) is out of scope; ``TiNeuVoxHeads`` is the
lightweight holder TemporalPoints takes as its ``tineuvox`` argument
(temporalpoints.py:133-152): rgbnet, densitynet, timenet, the positional-encoding
frequency buffers, ``no_view_dir``, ``voxel_size_ratio``, ``act_shift``, ``activate_density``.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn as nn

from . import ops
# tineuvox.py:627-670: the backward-capable autograd Functions over the HIP kernels (one
# definition, shared with the render_utils drop-in)
from .ops import Alphas2Weights, Raw2Alpha  # noqa: F401


def poc_fre(input_data: torch.Tensor, poc_buf: torch.Tensor) -> torch.Tensor:
    """tineuvox.py:872-878: [x, sin(x (x) f), cos(x (x) f)] with a dim-major flatten."""
    emb = (input_data.unsqueeze(-1) * poc_buf).flatten(-2)
    return torch.cat([input_data, emb.sin(), emb.cos()], -1)


class RGBNet(nn.Module):
    """tineuvox.py:65-88 (same parameter names: feature_linears, views_linears.{0,2})."""

    def __init__(self, D=3, W=256, h_ch=256, views_ch=33, pts_ch=27, times_ch=17, output_ch=3):
        super().__init__()
        self.D, self.W = D, W
        self.input_ch, self.input_ch_views = h_ch, views_ch
        self.input_ch_pts, self.input_ch_times, self.output_ch = pts_ch, times_ch, output_ch
        self.feature_linears = nn.Linear(self.input_ch, W)
        self.views_linears = nn.Sequential(nn.Linear(W + self.input_ch_views, W // 2), nn.ReLU(),
                                           nn.Linear(W // 2, self.output_ch))

    def forward(self, input_h, input_views=None):
        feature = self.feature_linears(input_h)
        if input_views is not None:
            feature = torch.cat([feature, input_views], dim=-1)
        else:
            assert self.input_ch_views == 0
        return self.views_linears(feature)


class TiNeuVoxHeads(nn.Module):
    """Holder for the TiNeuVox members TemporalPoints uses (tineuvox.py:91-160, 396-400)."""

    def __init__(self, xyz_min, xyz_max, num_voxels=160 ** 3, num_voxels_base=160 ** 3, voxel_dim=12,
                 net_width=128, alpha_init=1e-3, posbase_pe=10, viewbase_pe=4, timebase_pe=8,
                 gridbase_pe=2, no_view_dir=False, **kwargs):
        super().__init__()
        self.no_view_dir = no_view_dir
        self.posbase_pe, self.viewbase_pe, self.timebase_pe, self.gridbase_pe = posbase_pe, viewbase_pe, timebase_pe, gridbase_pe
        self.register_buffer("xyz_min", torch.tensor(np.asarray(xyz_min, dtype=np.float32)))
        self.register_buffer("xyz_max", torch.tensor(np.asarray(xyz_max, dtype=np.float32)))
        self.alpha_init = alpha_init
        self.act_shift = np.log(1 / (1 - alpha_init) - 1)
        vol = (self.xyz_max - self.xyz_min).prod()
        self.voxel_size_base = (vol / num_voxels_base).pow(1 / 3)
        self.voxel_size = (vol / num_voxels).pow(1 / 3)
        self.voxel_size_ratio = self.voxel_size / self.voxel_size_base
        times_ch = 2 * timebase_pe + 1
        views_ch = 0 if no_view_dir else 3 + 3 * viewbase_pe * 2
        timenet_output = voxel_dim + voxel_dim * 2 * gridbase_pe
        self.timenet = nn.Sequential(nn.Linear(times_ch, net_width), nn.ReLU(inplace=True),
                                     nn.Linear(net_width, timenet_output))
        self.densitynet = nn.Linear(net_width, 1)
        self.rgbnet = RGBNet(W=net_width, h_ch=net_width, views_ch=views_ch)
        self.register_buffer("time_poc", torch.FloatTensor([(2 ** i) for i in range(timebase_pe)]))
        self.register_buffer("grid_poc", torch.FloatTensor([(2 ** i) for i in range(gridbase_pe)]))
        self.register_buffer("pos_poc", torch.FloatTensor([(2 ** i) for i in range(posbase_pe)]))
        self.register_buffer("view_poc", torch.FloatTensor([(2 ** i) for i in range(viewbase_pe)]))

    def activate_density(self, density, interval=None, act_shift=None):
        """tineuvox.py:396-400 -> Raw2Alpha (HIP raw2alpha)."""
        act_shift = act_shift if act_shift is not None else self.act_shift
        interval = interval if interval is not None else self.voxel_size_ratio
        shape = density.shape
        return Raw2Alpha.apply(density.flatten(), float(act_shift), float(interval)).reshape(shape).squeeze(-1)


def get_rays(H, W, K, c2w, inverse_y=False, flip_x=False, flip_y=False, mode="center"):
    """tineuvox.py:675-703 (mode 'center' / 'lefttop')."""
    dev = c2w.device
    i, j = torch.meshgrid(torch.linspace(0, W - 1, W, device=dev), torch.linspace(0, H - 1, H, device=dev),
                          indexing="ij")
    i, j = i.t().float(), j.t().float()
    if mode == "center":
        i, j = i + 0.5, j + 0.5
    elif mode != "lefttop":
        raise NotImplementedError(mode)
    if flip_x:
        i = i.flip((1,))
    if flip_y:
        j = j.flip((0,))
    K = K.to(dev)
    if inverse_y:
        dirs = torch.stack([(i - K[0][2]) / K[0][0], (j - K[1][2]) / K[1][1], torch.ones_like(i)], -1)
    else:
        dirs = torch.stack([(i - K[0][2]) / K[0][0], -(j - K[1][2]) / K[1][1], -torch.ones_like(i)], -1)
    rays_d = torch.sum(dirs[..., None, :] * c2w[:3, :3], -1)
    rays_o = c2w[:3, 3].expand(rays_d.shape)
    return rays_o, rays_d


def get_rays_of_a_view(H, W, K, c2w, ndc=False, inverse_y=False, flip_x=False, flip_y=False, mode="center"):
    """tineuvox.py:733-738 (NDC is out of scope: never used by the point path)."""
    if ndc:
        raise NotImplementedError("NDC rays are not used by the articulated point path")
    rays_o, rays_d = get_rays(H, W, K, c2w, inverse_y=inverse_y, flip_x=flip_x, flip_y=flip_y, mode=mode)
    viewdirs = rays_d / rays_d.norm(dim=-1, keepdim=True)
    return rays_o, rays_d, viewdirs
