"""Where the train_pcd step (tools/train_bench.py) synchronises the host with the GPU: one step
under torch.cuda.set_sync_debug_mode("warn"), each synchronising call's Python call site counted.

    python tools/train_syncs.py [--config C2]
"""
import argparse
import collections
import os
import sys
import traceback
import warnings

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "articulated-point-nerf_amd"), os.path.join(ROOT, "tools")]
import torch  # noqa: E402

import train_bench as TB  # noqa: E402
from apn_amd import harness, synthetic as S  # noqa: E402
from apn_amd.temporalpoints import project_point_to_image_plane  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    args = ap.parse_args()
    dev = torch.device("cuda")
    scene = S.make_scene(args.config)
    model = harness.build_model(scene, dev)
    rk = scene.render_kwargs(dev)
    R_all = len(rk["rays_o"])
    t = torch.tensor([scene.cfg.t], device=dev)
    with torch.no_grad():
        tgt = model(torch.tensor([0.6], device=dev), render_kwargs=rk)
        target_rgb = tgt["rgb_marched"].clone()
        poses, Ks = scene.c2w[None].to(dev), scene.K[None].to(dev)
        mask_pts = project_point_to_image_plane(tgt["t_hat_pcd"], poses, Ks).flip(-1)
    opt = TB.make_optimizer(model)
    gen = torch.Generator(device=dev).manual_seed(0)

    def step():
        sel = torch.randint(0, R_all, (8192,), device=dev, generator=gen)
        sub = dict(rk)
        for k in ("rays_o", "rays_d", "viewdirs"):
            sub[k] = rk[k][sel]
        opt.zero_grad(set_to_none=True)
        res = model(t, False, sub, render_pcd_direct=False)
        pcd = res["t_hat_pcd"]
        W = TB.W
        loss = W["render"] * torch.nn.functional.mse_loss(res["rgb_marched"], target_rgb[sel])
        loss = loss + W["arap"] * model.get_arap_loss(pcd)
        loss = loss + W["tv"] * model.get_neighbour_weight_tv_loss()
        loss = loss + W["sparsity"] * model.get_weight_sparsity_loss()
        loss = loss + W["transformation_reg"] * model.get_transformation_regularisation_loss()
        loss = loss + W["joint_chamfer"] * model.get_joint_chamfer_loss()
        proj = project_point_to_image_plane(pcd, poses, Ks).flip(-1)
        mp = mask_pts[:, torch.randint(0, mask_pts.shape[1], (3000,), device=dev, generator=gen)]
        loss = loss + W["chamfer2D"] * model.get_batch_chamfer_loss(proj, mp, N=3000, M=None)
        loss.backward()
        opt.step()

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    sites = collections.Counter()

    def hook(message, category, filename, lineno, file=None, line=None):
        st = [f for f in traceback.extract_stack()[:-1] if "/apn_amd/" in f.filename or "tools/" in f.filename]
        key = " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in reversed(st[-3:]))
        sites[key] += 1

    old = warnings.showwarning
    warnings.showwarning = hook
    torch.cuda.set_sync_debug_mode("warn")
    try:
        with warnings.catch_warnings():
            warnings.simplefilter("always")
            warnings.showwarning = hook
            step()
    finally:
        torch.cuda.set_sync_debug_mode(0)
        warnings.showwarning = old
    print(f"{sum(sites.values())} synchronising calls in one step")
    for k, n in sites.most_common():
        print(f"{n:4d}  {k}")


if __name__ == "__main__":
    main()
