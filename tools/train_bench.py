"""Training-step benchmark: the reference's train_pcd iteration (run.py:574-716)
on a BASELINE config -- N_rand random rays (configs/nerf/default.py:114: 8192) of one view, the
forward with autograd, the default loss weights (default.py:95-103: render 200, arap 5e-3,
joint chamfer 1, transformation reg 0.1, TV 10, sparsity 0.2, 2D chamfer 5e-3 against a projected
target cloud), backward, and MaskedAdam over the reference's lrate_* groups (default.py:86-92).

Prints one JSON line: train iterations/s, rays/s, per-stage ms (HIP events), and the oracle's CPU
autograd step on the same rays (render loss only) as the CPU baseline.

    python tools/train_bench.py [--config C2] [--steps 10] [--warmup 3] [--no-cpu-baseline]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "articulated-point-nerf_amd")]
import torch  # noqa: E402

from apn_amd import harness, synthetic as S  # noqa: E402
from apn_amd.optim import MaskedAdam  # noqa: E402
from apn_amd.temporalpoints import project_point_to_image_plane  # noqa: E402

LRATES = dict(gammas=1e-3, weights=1e-4, theta_weight=1e-4, forward_warp=1e-4, joints=1e-5, feat_net=1e-3)
W = dict(render=2e2, chamfer2D=5e-3, arap=5e-3, joint_chamfer=1.0, transformation_reg=1e-1, tv=1e1, sparsity=2e-1)


def make_optimizer(model):
    """utils.py:480-516 with the pcd stage's lrate_* keys."""
    groups = []
    for k, lr in LRATES.items():
        p = getattr(model, k)
        groups.append({'params': list(p.parameters()) if isinstance(p, torch.nn.Module) else [p], 'name': k,
                       'lr': lr, 'skip_zero_grad': False})
    return MaskedAdam(groups)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n-rand", type=int, default=8192)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    print(json.dumps(run(ap.parse_args())))


def run(args):
    """The timed train_pcd loop (see the module docstring); returns the result dict."""
    dev = torch.device("cuda")
    scene = S.make_scene(args.config)
    model = harness.build_model(scene, dev)
    rk = scene.render_kwargs(dev)
    R_all = len(rk["rays_o"])
    t = torch.tensor([scene.cfg.t], device=dev)
    with torch.no_grad():   # targets: the fused render / projected cloud at another time
        tgt = model(torch.tensor([0.6], device=dev), render_kwargs=rk)
        target_rgb = tgt["rgb_marched"].clone()
        poses, Ks = scene.c2w[None].to(dev), scene.K[None].to(dev)
        mask_pts = project_point_to_image_plane(tgt["t_hat_pcd"], poses, Ks).flip(-1)
    opt = make_optimizer(model)
    gen = torch.Generator(device=dev).manual_seed(0)
    ev = {}

    def mark(name):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        ev.setdefault(name, []).append(e)

    def step():
        sel = torch.randint(0, R_all, (args.n_rand,), device=dev, generator=gen)
        sub = dict(rk)
        for k in ("rays_o", "rays_d", "viewdirs"):
            sub[k] = rk[k][sel]
        mark("start")
        opt.zero_grad(set_to_none=True)
        res = model(t, False, sub, render_pcd_direct=False)
        pcd = res["t_hat_pcd"]
        loss = W["render"] * torch.nn.functional.mse_loss(res["rgb_marched"], target_rgb[sel])
        loss = loss + W["arap"] * model.get_arap_loss(pcd)
        loss = loss + W["tv"] * model.get_neighbour_weight_tv_loss()
        loss = loss + W["sparsity"] * model.get_weight_sparsity_loss()
        loss = loss + W["transformation_reg"] * model.get_transformation_regularisation_loss()
        loss = loss + W["joint_chamfer"] * model.get_joint_chamfer_loss()
        proj = project_point_to_image_plane(pcd, poses, Ks).flip(-1)
        mp = mask_pts[:, torch.randint(0, mask_pts.shape[1], (3000,), device=dev, generator=gen)]
        loss = loss + W["chamfer2D"] * model.get_batch_chamfer_loss(proj, mp, N=3000, M=None)
        mark("forward")
        loss.backward()
        mark("backward")
        opt.step()
        mark("optimizer")
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ev.clear()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    stages = {}
    names = ["start", "forward", "backward", "optimizer"]
    for a, b in zip(names[:-1], names[1:]):
        stages[b] = sum(x.elapsed_time(y) for x, y in zip(ev[a], ev[b])) / args.steps
    ms = wall * 1e3 / args.steps
    out = {"metric": f"train_pcd iterations/s ({args.config}, N_rand={args.n_rand})", "value": 1e3 / ms,
           "unit": "it/s", "rays_per_s": args.n_rand * 1e3 / ms, "ms_per_step": ms, "stage_ms": stages,
           "steps": args.steps, "warmup": args.warmup, "loss": float(loss.detach()), "dtype": "f32",
           "data": "synthetic", "config": {"workload": scene.cfg.name, "n_rand": args.n_rand},
           "survivors_last_step": int(model.last_stats.get("survivors", -1))}
    if not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(model, scene, rk, target_rgb, args.n_rand, t)
    return out


def cpu_baseline(model, scene, rk, target_rgb, n_rand, t):
    """The oracle's CPU autograd train step (render loss + backward) on the same ray count."""
    from oracle import apn_oracle as O
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    st = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    orc = O.OracleModel(st, model.canonical_pcd.cpu(), model.bones, stepsize=S.STEPSIZE, voxel_size=S.VOXEL_SIZE,
                        fast_color_thres=S.FAST_COLOR_THRES, pose_embedding_dim=model.pose_embedding_dim,
                        act_shift=float(model.tineuvox.act_shift),
                        voxel_size_ratio=float(model.tineuvox.voxel_size_ratio),
                        mean_min_distance_value=float(model.mean_min_distance))
    O.oracle_trainable(orc)
    g = torch.Generator().manual_seed(1)
    sel = torch.randint(0, len(rk["rays_o"]), (n_rand,), generator=g)
    sub = {k: (v.cpu()[sel] if k in ("rays_o", "rays_d", "viewdirs") else v) for k, v in rk.items()}
    t0 = time.perf_counter()
    ro = O.oracle_forward_train(orc, t.cpu(), sub, knn_tree=True)
    loss = 2e2 * torch.nn.functional.mse_loss(ro["rgb_marched"], target_rgb.cpu()[sel])
    loss.backward()
    dt = time.perf_counter() - t0
    return {"value": 1.0 / dt, "unit": "it/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"1 oracle train step (render loss + backward, scipy cKDTree kNN) on {n_rand} rays"}


if __name__ == "__main__":
    main()
