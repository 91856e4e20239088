"""Render harness: the counterpart of the reference's ``render_viewpoints`` /
``render_repose`` (run.py:80-239, 241-356) for synthetic scenes, minus file I/O and metrics
that need ground-truth images.

A frame is rendered with a single ``TemporalPoints.forward`` over all H*W rays (chunking is
optional and bit-identical); ``render_pcd_direct`` substitutes ``rgb_marched_direct`` for
``rgb_marched`` as run.py:162-163 does.
"""
from __future__ import annotations

import math

import torch

from . import synthetic as S
from .temporalpoints import TemporalPoints
from .tineuvox import TiNeuVoxHeads


def build_model(scene: S.Scene, device="cuda") -> TemporalPoints:
    """TemporalPoints(**scene.ctor, tineuvox=heads) with the scene's network weights loaded."""
    c = scene.ctor
    heads = TiNeuVoxHeads(c["xyz_min"], c["xyz_max"], num_voxels=160 ** 3, num_voxels_base=160 ** 3,
                          net_width=S.NET_WIDTH, alpha_init=S.ALPHA_INIT, posbase_pe=S.POSBASE_PE,
                          viewbase_pe=S.VIEWBASE_PE, timebase_pe=S.TIMEBASE_PE, no_view_dir=False)
    model = TemporalPoints(**c, tineuvox=heads)
    missing, unexpected = model.load_state_dict(scene.params, strict=False)
    if unexpected:
        raise KeyError(f"unexpected state-dict keys: {unexpected}")
    return model.to(device)


PER_POINT_CTOR = ("canonical_pcd", "canonical_alpha", "canonical_feat", "canonical_rgbs")


def shard_scene_points(scene: S.Scene, rank: int, world: int) -> S.Scene:
    """The scene restricted to rank's contiguous point range [N*rank/world, N*(rank+1)/world)
    (LBS is per point, so the shards skin independently; the skeleton,
    joints and networks are replicated). Per-point parameters derived in the constructor (the
    bone-distance LBS weights, direct_eps, gammas) are per point as well."""
    import copy
    from .temporalpoints import weights_from_bones
    N = len(scene.ctor["canonical_pcd"])
    r0, r1 = N * rank // world, N * (rank + 1) // world
    ctor = dict(scene.ctor)
    for k in PER_POINT_CTOR:
        ctor[k] = scene.ctor[k][r0:r1]
    out = copy.copy(scene)
    out.ctor = ctor
    # the raw LBS weights of the full cloud, sliced (the vectorised bone-distance pass is not
    # bit-stable under a change of N); loaded over the constructor's own by build_model
    full_w = weights_from_bones(torch.as_tensor(scene.ctor["joints"]).float(), scene.ctor["bones"],
                                torch.as_tensor(scene.ctor["canonical_pcd"]).float(), torch.tensor(1e-6))
    out.params = dict(scene.params, weights=full_w[r0:r1].contiguous())
    out.extra = dict(scene.extra, point_range=(r0, r1))
    return out


def render_kwargs_for(scene: S.Scene, device="cuda"):
    return scene.render_kwargs(device)


@torch.no_grad()
def render_frame(model, scene: S.Scene, t=None, rot_params=None, render_kwargs=None, chunk=None,
                 render_pcd_direct=False, device="cuda"):
    """One frame -> dict of (H, W, C) images: rgb, depth, weights (+ joints)."""
    rk = render_kwargs if render_kwargs is not None else scene.render_kwargs(device)
    H, W = scene.cfg.H, scene.cfg.W
    R = rk["rays_o"].shape[0]
    chunk = chunk or R
    outs = []
    t_arg = None if rot_params is not None else torch.tensor([scene.cfg.t if t is None else t], device=device)
    for s in range(0, R, chunk):
        sub = dict(rk)
        for k in ("rays_o", "rays_d", "viewdirs"):
            sub[k] = rk[k][s:s + chunk]
        out = model(t_arg, render_depth=True, render_kwargs=sub, render_weights=True, rot_params=rot_params,
                    render_pcd_direct=render_pcd_direct, poses=scene.c2w[None].to(device),
                    Ks=scene.K[None].to(device), get_skeleton=True)
        if render_pcd_direct:
            out["rgb_marched"] = out["rgb_marched_direct"]
        outs.append(out)
    res = {k: torch.cat([o[k] for o in outs]).reshape(H, W, -1) for k in ("rgb_marched", "depth", "weights")}
    res["joints"] = outs[0]["joints"]
    return res


def psnr(a: torch.Tensor, b: torch.Tensor) -> float:
    """run.py:186: -10 log10(mean((a-b)^2))."""
    mse = float(((a.float() - b.float()) ** 2).mean())
    return float("inf") if mse == 0 else -10.0 * math.log10(mse)
