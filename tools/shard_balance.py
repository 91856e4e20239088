"""Load balance of the ray-sharded frame measured on ONE GPU: the C2 frame's
shards for world = 2, 4, 8 rendered one after another (ray_shard=(k, world)), each timed with HIP
events, next to its in-bbox samples and kNN survivors (the MLP's work). The max over shards is
what a strong-scaling step waits for. Diagnostic tool (not a test).

    python tools/shard_balance.py [--config C2] [--reps 5] [--split inbbox|cost]
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
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--worlds", default="2,4,8")
    args = ap.parse_args()
    torch.set_grad_enabled(False)
    dev = torch.device("cuda", 0)
    scene = S.make_scene(args.config)
    model = harness.build_model(scene, dev)
    rk = scene.render_kwargs(dev)
    t = torch.tensor([scene.cfg.t], device=dev)
    poses, Ks = scene.c2w[None].to(dev), scene.K[None].to(dev)
    kw = dict(render_depth=True, render_kwargs=rk, render_weights=True, poses=poses, Ks=Ks, get_skeleton=True)

    def timed(fn, reps):
        for _ in range(2):
            fn()
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            out = fn()
        e1.record()
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) / reps, out

    full_ms, out = timed(lambda: model(t, **kw), args.reps)
    st = model.last_stats.resolved()
    print(f"full frame {full_ms:.3f} ms, {st}")
    for world in [int(w) for w in args.worlds.split(",")]:
        rows = []
        for k in range(world):
            ms, o = timed(lambda: model(t, ray_shard=(k, world), **kw), args.reps)
            s = model.last_stats.resolved()
            r0, r1 = model.last_ray_range
            rows.append((ms, s.get("inbbox_samples", -1), s.get("kept_samples", -1), r1 - r0))
        mx = max(r[0] for r in rows)
        mean = sum(r[0] for r in rows) / world
        print(f"world {world}: shard ms " + " ".join(f"{r[0]:.3f}" for r in rows)
              + f" | max {mx:.3f} mean {mean:.3f} (max/mean {mx / mean:.3f}); ideal full/world {full_ms / world:.3f}; "
              f"speedup bound {full_ms / mx:.2f}x")
        print("   kept per shard: " + " ".join(str(r[2]) for r in rows)
              + " | inbbox per shard: " + " ".join(str(r[1]) for r in rows)
              + " | rays: " + " ".join(str(r[3]) for r in rows))


if __name__ == "__main__":
    main()
