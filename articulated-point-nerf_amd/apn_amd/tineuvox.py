"""The reference's ``lib/tineuvox.py`` as the point render path and its stage-1 source use it
(SURVEY.md §2 row 4, §8 f-3): RGBNet, the density head holder, poc_fre, Raw2Alpha /
Alphas2Weights (re-exported from ``ops``: HIP forward and backward), ray generation, and the
stage-1 TiNeuVox voxel model (``TiNeuVox`` below: constructor, state dict, forward,
get_grid_as_point_cloud, mult_dist_interp over the HIP field ``apn_tnv_field``; default
configuration only).

``TiNeuVoxHeads`` is the lightweight holder TemporalPoints takes as its ``tineuvox`` argument
when no stage-1 model is at hand (temporalpoints.py:133-152): rgbnet, densitynet, timenet, the
positional-encoding frequency buffers, ``no_view_dir``, ``voxel_size_ratio``, ``act_shift``,
``activate_density``.
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
        from .linear import linear, sequential
        feature = linear(input_h, self.feature_linears)
        if input_views is not None:
            feature = torch.cat([feature, input_views], dim=-1)
        else:
            assert self.input_ch_views == 0
        return sequential(self.views_linears, feature)


class TiNeuVoxHeads(nn.Module):
    """Holder for the TiNeuVox members TemporalPoints uses (tineuvox.py:91-160, 396-400)."""

    def __init__(self, xyz_min, xyz_max, num_voxels=160 ** 3, num_voxels_base=160 ** 3, voxel_dim=12,
                 net_width=128, alpha_init=1e-3, posbase_pe=10, viewbase_pe=4, timebase_pe=8,
                 gridbase_pe=2, no_view_dir=False, **kwargs):
        super().__init__()
        self._kwargs = dict(xyz_min=np.asarray(xyz_min, dtype=np.float32), xyz_max=np.asarray(xyz_max, dtype=np.float32),
                            num_voxels=num_voxels, num_voxels_base=num_voxels_base, voxel_dim=voxel_dim,
                            net_width=net_width, alpha_init=alpha_init, posbase_pe=posbase_pe,
                            viewbase_pe=viewbase_pe, timebase_pe=timebase_pe, gridbase_pe=gridbase_pe,
                            no_view_dir=no_view_dir)
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

    def get_kwargs(self):
        """Constructor arguments (the TiNeuVox.get_kwargs subset this holder takes)."""
        return dict(self._kwargs)

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


# ----------------------------------------------------------------------------------------------
# TiNeuVox stage 1: the voxel model the articulated point cloud is exported
# from (lib/tineuvox.py:91-625), same constructor, parameter / buffer names and methods. The
# field (deformation MLP, 3-scale trilinear feature-grid lookup, featurenet, density and colour
# heads) runs in the HIP kernels of csrc/apn_tineuvox.hip; only J- and time-sized pieces
# (timenet, per-time projections, weight packing) are torch ops on the device.
# ----------------------------------------------------------------------------------------------

class Deformation(nn.Module):
    """tineuvox.py:28-62 (parameter names _time.{i}, _time_out)."""

    def __init__(self, D=8, W=256, input_ch=27, input_ch_views=3, input_ch_time=9, skips=[]):
        super().__init__()
        self.D, self.W = D, W
        self.input_ch, self.input_ch_views, self.input_ch_time = input_ch, input_ch_views, input_ch_time
        self.skips = list(skips)
        layers = [nn.Linear(input_ch + input_ch_time, W)]
        for i in range(D - 2):
            layers.append(nn.Linear(W + (input_ch if i in self.skips else 0), W))
        self._time, self._time_out = nn.ModuleList(layers), nn.Linear(W, 3)

    def query_time(self, new_pts, t, net, net_final):
        h = torch.cat([new_pts, t], dim=-1)
        for i, layer in enumerate(net):
            h = torch.relu(layer(h))
            if i in self.skips:
                h = torch.cat([new_pts, h], -1)
        return net_final(h)

    def forward(self, input_pts, ts):
        return input_pts[:, :3] + self.query_time(input_pts, ts, self._time, self._time_out)


_TNV_LAYOUT = {}


def tnv_layout(defor_depth):
    """Float offsets of the packed TiNeuVox network buffer (apn_tnv_weight_layout)."""
    if defor_depth not in _TNV_LAYOUT:
        import ctypes as C
        from . import _lib as L
        arr = (C.c_int32 * 16)()
        n = L.load().apn_tnv_weight_layout(int(defor_depth), arr)
        names = ["D0E", "DH", "DOUT", "FW", "WD", "BD", "WH", "BH", "WV2", "BV2", "TOTAL", "KE", "KF", "KV"]
        if n != len(names):
            raise RuntimeError(f"apn_tnv_weight_layout returned {n}")
        _TNV_LAYOUT[defor_depth] = dict(zip(names, list(arr)[:n]))
    return _TNV_LAYOUT[defor_depth]


class TiNeuVox(nn.Module):
    """lib/tineuvox.py:91-625 with the field on the HIP kernels (inference: forward under
    ``torch.no_grad()``, get_grid_as_point_cloud, get_alpha_mask, mult_dist_interp). Stage-1
    training (autograd through the field) is out of scope: forward raises with grad enabled."""

    def __init__(self, xyz_min, xyz_max, num_voxels=0, num_voxels_base=0, add_cam=False, alpha_init=None,
                 fast_color_thres=0, voxel_dim=0, defor_depth=3, net_width=128, posbase_pe=10, viewbase_pe=4,
                 timebase_pe=8, gridbase_pe=2, feat_only=False, no_view_dir=True, **kwargs):
        super().__init__()
        self.add_cam = add_cam
        self.voxel_dim = voxel_dim
        self.defor_depth = defor_depth
        self.net_width = net_width
        self.feat_only = feat_only
        self.no_view_dir = no_view_dir
        self.posbase_pe, self.viewbase_pe, self.timebase_pe, self.gridbase_pe = posbase_pe, viewbase_pe, timebase_pe, gridbase_pe
        times_ch = 2 * timebase_pe + 1
        views_ch = 0 if no_view_dir else 3 + 3 * viewbase_pe * 2
        self.register_buffer("xyz_min", torch.tensor(np.asarray(xyz_min, dtype=np.float32)).float())
        self.register_buffer("xyz_max", torch.tensor(np.asarray(xyz_max, dtype=np.float32)).float())
        self.fast_color_thres = fast_color_thres
        self.num_voxels_base = num_voxels_base
        self.voxel_size_base = ((self.xyz_max - self.xyz_min).prod() / self.num_voxels_base).pow(1 / 3)
        self.alpha_init = alpha_init
        self.act_shift = np.log(1 / (1 - alpha_init) - 1)
        timenet_output = voxel_dim + voxel_dim * 2 * gridbase_pe
        self.timenet = nn.Sequential(nn.Linear(times_ch, net_width), nn.ReLU(inplace=True),
                                     nn.Linear(net_width, timenet_output))
        if add_cam:
            views_ch = 3 + 3 * viewbase_pe * 2 + timenet_output
            self.camnet = nn.Sequential(nn.Linear(times_ch, net_width), nn.ReLU(inplace=True),
                                        nn.Linear(net_width, timenet_output))
        grid_dim = voxel_dim * 3 + voxel_dim * 3 * 2 * gridbase_pe
        input_dim = grid_dim if feat_only else grid_dim + timenet_output + 3 + 3 * posbase_pe * 2
        self.featurenet = nn.Sequential(nn.Linear(input_dim, net_width), nn.ReLU(inplace=True))
        self.featurenet_width = net_width
        self._set_grid_resolution(num_voxels)
        self.deformation_net = Deformation(W=net_width, D=defor_depth, input_ch=3 + 3 * posbase_pe * 2,
                                           input_ch_time=timenet_output)
        self.densitynet = nn.Linear(net_width, 1)
        self.register_buffer("time_poc", torch.FloatTensor([(2 ** i) for i in range(timebase_pe)]))
        self.register_buffer("grid_poc", torch.FloatTensor([(2 ** i) for i in range(gridbase_pe)]))
        self.register_buffer("pos_poc", torch.FloatTensor([(2 ** i) for i in range(posbase_pe)]))
        self.register_buffer("view_poc", torch.FloatTensor([(2 ** i) for i in range(viewbase_pe)]))
        self.feature = nn.Parameter(torch.zeros([1, voxel_dim, *self.world_size], dtype=torch.float32))
        self.rgbnet = RGBNet(W=net_width, h_ch=net_width, views_ch=views_ch, pts_ch=3 + 3 * posbase_pe * 2,
                             times_ch=times_ch)
        self._pack_cache = None

    def _set_grid_resolution(self, num_voxels):
        self.num_voxels = num_voxels
        self.voxel_size = ((self.xyz_max - self.xyz_min).prod() / num_voxels).pow(1 / 3)
        self.world_size = ((self.xyz_max - self.xyz_min) / self.voxel_size).long()
        self.voxel_size_ratio = self.voxel_size / self.voxel_size_base

    def get_kwargs(self):
        """tineuvox.py:180-199."""
        return {'xyz_min': self.xyz_min.cpu().numpy(), 'xyz_max': self.xyz_max.cpu().numpy(),
                'num_voxels': self.num_voxels, 'num_voxels_base': self.num_voxels_base,
                'alpha_init': self.alpha_init, 'act_shift': self.act_shift,
                'voxel_size_ratio': self.voxel_size_ratio, 'fast_color_thres': self.fast_color_thres,
                'voxel_dim': self.voxel_dim, 'defor_depth': self.defor_depth, 'net_width': self.net_width,
                'posbase_pe': self.posbase_pe, 'viewbase_pe': self.viewbase_pe, 'timebase_pe': self.timebase_pe,
                'gridbase_pe': self.gridbase_pe, 'add_cam': self.add_cam, 'no_view_dir': self.no_view_dir}

    # -------------------------------------------------------------- HIP plumbing
    def _check_supported(self):
        if (self.voxel_dim, self.net_width, self.posbase_pe, self.gridbase_pe, self.viewbase_pe) != (12, 128, 10, 2, 4):
            raise NotImplementedError("the HIP TiNeuVox field implements voxel_dim=12, net_width=128, posbase_pe=10, "
                                      "gridbase_pe=2, viewbase_pe=4 (configs/nerf/default.py)")
        if self.add_cam or self.feat_only or self.deformation_net.skips:
            raise NotImplementedError("add_cam / feat_only / deformation skips are not implemented")
        from . import _lib as L
        L.require_cuda(self.feature, what="TiNeuVox")

    def _packed(self):
        """(wbuf, grid) for the HIP field, rebuilt when a parameter changes (versions)."""
        from . import _lib as L
        from ._lib import call, ptr, stream_ptr
        self._check_supported()
        dev = self.feature.device
        params = [self.feature] + [p for m in (self.deformation_net, self.featurenet, self.densitynet, self.rgbnet)
                                   for p in m.parameters()]
        key = tuple((p.data_ptr(), p._version) for p in params)
        if self._pack_cache is not None and self._pack_cache[0] == key:
            return self._pack_cache[1], self._pack_cache[2]
        D = self.defor_depth
        lay = tnv_layout(D)
        W = self.net_width
        buf = torch.zeros(lay["TOTAL"], device=dev)

        def put(off, t):
            t = t.detach().float().reshape(-1)
            buf[off:off + t.numel()].copy_(t)

        d0 = self.deformation_net._time[0].weight.detach().float()
        w0e = torch.zeros(W, lay["KE"], device=dev)
        w0e[:, :63] = d0[:, :63]
        put(lay["D0E"], w0e)
        for i in range(D - 2):
            lyr = self.deformation_net._time[1 + i]
            off = lay["DH"] + i * (W * W + W)
            put(off, lyr.weight)
            put(off + W * W, lyr.bias)
        put(lay["DOUT"], self.deformation_net._time_out.weight)
        put(lay["DOUT"] + 3 * W, self.deformation_net._time_out.bias)
        fw = self.featurenet[0].weight.detach().float()
        fwp = torch.zeros(W, lay["KF"], device=dev)
        fwp[:, :243] = fw[:, :243]
        put(lay["FW"], fwp)
        put(lay["WD"], self.densitynet.weight)
        put(lay["BD"], self.densitynet.bias)
        wf = self.rgbnet.feature_linears.weight.detach().double()
        bf = self.rgbnet.feature_linears.bias.detach().double()
        v0 = self.rgbnet.views_linears[0]
        wv0 = v0.weight.detach().double()
        wh = torch.zeros(64, lay["KV"], dtype=torch.float64, device=dev)
        wh[:, :W] = wv0[:, :W] @ wf
        wh[:, W:wv0.shape[1]] = wv0[:, W:]
        put(lay["WH"], wh)
        put(lay["BH"], wv0[:, :W] @ bf + v0.bias.detach().double())
        put(lay["WV2"], self.rgbnet.views_linears[2].weight)
        put(lay["BV2"], self.rgbnet.views_linears[2].bias)
        X, Y, Z = (int(v) for v in self.feature.shape[2:])
        nbytes = int(L.load().apn_tnv_grid_bytes(12, X, Y, Z))
        grid = torch.empty(nbytes // 4, device=dev)
        call("apn_tnv_grid_pack", ptr(self.feature.detach().float().contiguous()), 12, X, Y, Z, ptr(grid),
             stream_ptr(dev))
        self._pack_cache = (key, buf, grid)
        return buf, grid

    def _tproj(self, times):
        """[U, 256]: timenet(poc_fre(t)) through the time columns of deformation layer 0 and of
        featurenet, plus their biases (the per-time part of those two layers)."""
        tf = self.timenet(poc_fre(times.reshape(-1, 1).float(), self.time_poc))
        d0 = self.deformation_net._time[0]
        p0 = torch.nn.functional.linear(tf, d0.weight[:, 63:], d0.bias)
        f0 = self.featurenet[0]
        p1 = torch.nn.functional.linear(tf, f0.weight[:, 243:], f0.bias)
        return torch.cat([p0, p1], -1).float().contiguous()

    def _field(self, pts, ray_idx, time_idx, tproj, viewdirs=None, vemb=None, deform=True, want_h=False,
               want_vox=False, interval=None):
        """The HIP field at pts [S,3] -> (alpha [S], rgb [S,3], deformed pts [S,3], h, vox)."""
        from ._lib import call, ptr, stream_ptr
        wbuf, grid = self._packed()
        dev = pts.device
        S = pts.shape[0]
        X, Y, Z = (int(v) for v in self.feature.shape[2:])
        pos4 = torch.zeros(S, 4, device=dev)
        pos4[:, :3] = pts
        ns = torch.tensor([S], dtype=torch.int32, device=dev)
        out12 = torch.empty(S, 12, device=dev)
        delta = torch.empty(S, 3, device=dev)
        h = torch.empty(S, self.net_width, device=dev) if want_h else None
        vox = torch.empty(S, 36, device=dev) if want_vox else None
        interval = float(self.voxel_size_ratio) if interval is None else float(interval)
        call("apn_tnv_field", ptr(pos4), ptr(ray_idx.to(torch.int32).contiguous()),
             ptr(time_idx.to(torch.int32).contiguous()), S, ptr(ns), ptr(grid), X, Y, Z, ptr(self.xyz_min),
             ptr(self.xyz_max), ptr(wbuf), int(self.defor_depth), ptr(tproj),
             ptr(viewdirs.float().contiguous()) if viewdirs is not None else None,
             ptr(vemb.float().contiguous()) if vemb is not None else None, int(bool(deform)),
             float(self.act_shift), interval, ptr(out12), ptr(delta), ptr(h), ptr(vox), stream_ptr(dev))
        return out12[:, 3], out12[:, :3], delta, h, vox

    # -------------------------------------------------------------- reference API
    def get_grid_xyz(self, sampling_freq, xyz_min=None, xyz_max=None, world_size=None):
        """tineuvox.py:238-250."""
        xyz_min = self.xyz_min if xyz_min is None else xyz_min
        xyz_max = self.xyz_max if xyz_max is None else xyz_max
        world_size = self.world_size if world_size is None else world_size
        return torch.stack(torch.meshgrid(
            torch.linspace(xyz_min[0], xyz_max[0], int(world_size[0] * sampling_freq)),
            torch.linspace(xyz_min[1], xyz_max[1], int(world_size[1] * sampling_freq)),
            torch.linspace(xyz_min[2], xyz_max[2], int(world_size[2] * sampling_freq)), indexing="ij"), -1)

    def grid_sampler(self, xyz, *grids, mode=None, align_corners=True):
        """tineuvox.py:379-394 for arbitrary grids (a utility; the feature lookup of the field is
        mult_dist_interp on the HIP kernel)."""
        shape = xyz.shape[:-1]
        xyz = xyz.reshape(1, 1, 1, -1, 3)
        ind_norm = ((xyz - self.xyz_min) / (self.xyz_max - self.xyz_min)).flip((-1,)) * 2 - 1
        ret = [torch.nn.functional.grid_sample(g, ind_norm, mode="bilinear", align_corners=align_corners)
               .reshape(g.shape[1], -1).T.reshape(*shape, g.shape[1]) for g in grids]
        ret = [r.squeeze(-1) if r.shape[-1] == 1 else r for r in ret]
        return ret[0] if len(ret) == 1 else ret

    def mult_dist_interp(self, ray_pts_delta):
        """tineuvox.py:402-419 on the HIP kernel: [scale 1 | 1/2 | 1/4] x 12 trilinear features."""
        from ._lib import call, ptr, stream_ptr
        _, grid = self._packed()
        pts = ray_pts_delta.detach().float().reshape(-1, 3).contiguous()
        X, Y, Z = (int(v) for v in self.feature.shape[2:])
        out = torch.empty(pts.shape[0], 36, device=pts.device)
        call("apn_tnv_mult_dist_interp", ptr(pts), pts.shape[0], ptr(grid), X, Y, Z, ptr(self.xyz_min),
             ptr(self.xyz_max), ptr(out), stream_ptr(pts.device))
        return out if out.shape[0] != 1 or ray_pts_delta.dim() > 1 else out

    def activate_density(self, density, interval=None, act_shift=None):
        """tineuvox.py:396-400."""
        act_shift = act_shift if act_shift is not None else self.act_shift
        interval = interval if interval is not None else self.voxel_size_ratio
        shape = density.shape
        return Raw2Alpha.apply(density.flatten(), float(act_shift), float(interval)).reshape(shape).squeeze(-1)

    def get_mask(self, rays_o, rays_d, near, far, stepsize, **render_kwargs):
        """tineuvox.py:422-433."""
        shape = rays_o.shape[:-1]
        rays_o = rays_o.reshape(-1, 3).contiguous()
        rays_d = rays_d.reshape(-1, 3).contiguous()
        stepdist = stepsize * self.voxel_size
        _, mask_outbbox, ray_id = ops.sample_pts_on_rays(rays_o, rays_d, self.xyz_min, self.xyz_max, near, far,
                                                         float(stepdist))[:3]
        hit = torch.zeros([len(rays_o)], dtype=torch.bool, device=rays_o.device)
        hit[ray_id[~mask_outbbox]] = 1
        return hit.reshape(shape)

    def sample_ray(self, rays_o, rays_d, near, far, stepsize, is_train=False, **render_kwargs):
        """tineuvox.py:435-456 through the render_utils drop-in."""
        stepdist = stepsize * self.voxel_size
        ray_pts, mask_outbbox, ray_id, step_id, *_ = ops.sample_pts_on_rays(
            rays_o.contiguous(), rays_d.contiguous(), self.xyz_min, self.xyz_max, near, far, float(stepdist))
        mask_inbbox = ~mask_outbbox
        return ray_pts[mask_inbbox], ray_id[mask_inbbox], step_id[mask_inbbox], mask_inbbox

    def forward(self, rays_o, rays_d, viewdirs, times_sel, cam_sel=None, bg_points_sel=None, global_step=None,
                render_until=None, canonical_t=0, threshold=0.05, **render_kwargs):
        """tineuvox.py:458-564 (inference). Samples -> HIP field (deformation, 3-scale feature
        lookup, featurenet, density, colour) -> the reference's masks, Alphas2Weights and
        segment sums on the HIP drop-ins; the same return dict."""
        if torch.is_grad_enabled():
            raise NotImplementedError("TiNeuVox stage-1 training is out of scope; render under torch.no_grad()")
        assert len(rays_o.shape) == 2 and rays_o.shape[-1] == 3, 'Only suuport point queries in [N, 3] format'
        ret = {}
        N = len(rays_o)
        ray_pts, ray_id, step_id, _ = self.sample_ray(rays_o=rays_o, rays_d=rays_d, is_train=global_step is not None,
                                                      **render_kwargs)
        times, tinv = torch.unique(times_sel.reshape(-1).float(), return_inverse=True)
        tproj = self._tproj(times)
        interval = render_kwargs['stepsize'] * self.voxel_size_ratio
        alpha, rgb, ray_pts_delta, _, _ = self._field(ray_pts, ray_id, tinv, tproj, viewdirs=viewdirs,
                                                      interval=interval)
        if bg_points_sel is not None:
            ret['bg_points_delta'] = self.deformation_net(poc_fre(bg_points_sel, self.pos_poc),
                                                          self.timenet(poc_fre(times_sel, self.time_poc))[
                                                              :bg_points_sel.shape[0]])
        if self.fast_color_thres > 0:
            mask = alpha > self.fast_color_thres
            ray_id, step_id, alpha, rgb = ray_id[mask], step_id[mask], alpha[mask], rgb[mask]
        weights, alphainv_last = Alphas2Weights.apply(alpha, ray_id, N)
        if self.fast_color_thres > 0:
            mask = weights > self.fast_color_thres
            weights, alpha, ray_id, step_id, rgb = weights[mask], alpha[mask], ray_id[mask], step_id[mask], rgb[mask]
        rgb_marched = ops.segment_coo_sum(weights.unsqueeze(-1) * rgb, ray_id, N)
        rgb_marched = rgb_marched + alphainv_last.unsqueeze(-1) * render_kwargs['bg']
        n_samples = int(np.linalg.norm(self.world_size.cpu().numpy() + 1) / render_kwargs["stepsize"]) + 1
        s = (step_id + 0.5) / n_samples
        ret.update({'alphainv_last': alphainv_last, 'weights': weights, 'rgb_marched': rgb_marched,
                    'raw_alpha': alpha, 'raw_rgb': rgb, 'ray_id': ray_id, 's': s, 'n_max': n_samples,
                    'ray_pts_delta': ray_pts_delta})
        ret['depth'] = ops.segment_coo_sum(weights * step_id, ray_id, N)
        return ret

    @torch.no_grad()
    def get_grid_as_point_cloud(self, stepsize, time_sel=torch.tensor([[0., ]]), viewdir=torch.tensor([[0., 0., 0.]]),
                                cam_sel=None, threshold=None, canonical=False, sampling_freq=1, N_batch=2 ** 20,
                                blob_mask=None, alpha_xyz_only=True, grid_xyz=None):
        """tineuvox.py:253-363 (the canonical export query of run.py:1152-1194) on the HIP field:
        one launch over all grid points (N_batch only bounds the reference's memory)."""
        dev = self.feature.device
        if grid_xyz is None:
            grid_xyz = self.get_grid_xyz(sampling_freq)
        og_shape = grid_xyz.shape[:-1]
        pts = grid_xyz.reshape(-1, 3).to(dev).float().contiguous()
        tproj = self._tproj(torch.as_tensor(time_sel, dtype=torch.float32).reshape(1).to(dev))
        vemb = poc_fre(torch.as_tensor(viewdir).to(dev).float().reshape(1, 3), self.view_poc).reshape(-1)
        zeros = torch.zeros(pts.shape[0], dtype=torch.int32, device=dev)
        alpha, rgb, _, h, vox = self._field(pts, zeros, torch.zeros(1, dtype=torch.int32, device=dev), tproj,
                                            vemb=vemb, deform=not canonical, want_h=not alpha_xyz_only,
                                            want_vox=not alpha_xyz_only, interval=stepsize * self.voxel_size_ratio)
        alpha_volume = alpha.reshape(*og_shape)
        if alpha_xyz_only:
            return None, None, None, None, None, None, grid_xyz.reshape(*og_shape, 3), alpha_volume
        binary_volume = torch.zeros_like(alpha).reshape(*og_shape)
        return pts, alpha, rgb, h, vox, binary_volume, grid_xyz.reshape(*og_shape, 3), alpha_volume

    @torch.no_grad()
    def get_alpha_mask(self, stepsize, time_sel=torch.tensor([[0., ]]), viewdir=torch.tensor([[0., 0., 0.]]),
                       threshold=None, sampling_freq=1):
        """tineuvox.py:201-236."""
        *_, grid_xyz, alpha = self.get_grid_as_point_cloud(stepsize, time_sel=time_sel, viewdir=viewdir,
                                                           sampling_freq=1)
        if threshold is None and self.fast_color_thres > 0:
            mask = alpha > self.fast_color_thres
        else:
            mask = alpha > threshold
        return grid_xyz.view(*self.world_size, 3), mask.view(*self.world_size)

    @torch.no_grad()
    def scale_volume_grid(self, num_voxels):
        """tineuvox.py:365-372 (training-time progressive growing; torch trilinear resize)."""
        self._set_grid_resolution(num_voxels)
        self.feature = nn.Parameter(torch.nn.functional.interpolate(self.feature.data, size=tuple(self.world_size),
                                                                    mode='trilinear', align_corners=True))

    def feature_total_variation_add_grad(self, weight, dense_mode):
        """tineuvox.py:374-377 through the HIP total_variation_add_grad."""
        from .optim import total_variation_add_grad
        weight = weight * float(self.world_size.max()) / 128
        total_variation_add_grad(self.feature.float(), self.feature.grad.float(), weight, weight, weight, dense_mode)
