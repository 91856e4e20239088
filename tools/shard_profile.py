"""One rank's frame of the blocks ray split rendered repeatedly (for rocprofv3 --kernel-trace
--stats): where the per-shard time goes against 1/world of the full frame. Diagnostic tool.

    rocprofv3 --kernel-trace --stats -d gpurun_out/sp -- python tools/shard_profile.py --world 8
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "articulated-point-nerf_amd"))
from apn_amd import harness, synthetic as S  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--frames", type=int, default=20)
    args = ap.parse_args()
    torch.set_grad_enabled(False)
    dev = torch.device("cuda", 0)
    scene = S.make_scene(args.config)
    model = harness.build_model(scene, dev)
    rk = scene.render_kwargs(dev)
    t = torch.tensor([scene.cfg.t], device=dev)
    poses, Ks = scene.c2w[None].to(dev), scene.K[None].to(dev)
    kw = dict(render_depth=True, render_kwargs=rk, render_weights=True, poses=poses, Ks=Ks, get_skeleton=True)
    shard = (args.rank, args.world, 4096) if args.world > 1 else None
    for _ in range(3):
        model(t, ray_shard=shard, **kw)
    torch.cuda.synchronize(dev)
    for _ in range(args.frames):
        model(t, ray_shard=shard, **kw)
    torch.cuda.synchronize(dev)
    print(model.last_stats.resolved())


if __name__ == "__main__":
    main()
