"""Probe: harness.render_viewpoints on the C2 scene, frames in flight, host readback: wall time per
frame and where the host spends it (cProfile of the timed call), next to the pipeline's bare
submit loop (no readback) on the same model.

    python tools/viewpoints_probe.py [--views 16] [--in-flight 3]
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "articulated-point-nerf_amd"))
from apn_amd import harness, synthetic as S  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--views", type=int, default=16)
    ap.add_argument("--in-flight", type=int, default=3)
    args = ap.parse_args()
    torch.set_grad_enabled(False)
    dev = torch.device("cuda", 0)
    scene = S.make_scene("C2")
    model = harness.build_model(scene, dev)
    rk = {k: v for k, v in scene.render_kwargs(dev).items() if k not in ("rays_o", "rays_d", "viewdirs")}
    n = args.views
    poses = scene.c2w[None].repeat(n, 1, 1)
    HW = [[scene.cfg.H, scene.cfg.W]] * n
    Ks = scene.K[None].repeat(n, 1, 1)
    times = [scene.cfg.t + 0.01 * i for i in range(n)]
    kw = dict(test_times=times, verbose=False, inverse_y=bool(rk.get("inverse_y", False)), in_flight=args.in_flight)
    harness.render_viewpoints(model, poses, HW, Ks, False, dict(rk), **kw)
    torch.cuda.synchronize()
    for rep in range(2):
        for nf in sorted({args.in_flight, 4}):
            t0 = time.perf_counter()
            harness.render_viewpoints(model, poses, HW, Ks, False, dict(rk), **dict(kw, in_flight=nf))
            torch.cuda.synchronize()
            print(f"render_viewpoints ({nf} in flight): {(time.perf_counter() - t0) / n * 1e3:.3f} ms/frame")
    pr = cProfile.Profile()
    pr.enable()
    t0 = time.perf_counter()
    harness.render_viewpoints(model, poses, HW, Ks, False, dict(rk), **kw)
    el = time.perf_counter() - t0
    pr.disable()
    print(f"profiled: {el / n * 1e3:.3f} ms/frame")
    pstats.Stats(pr).sort_stats("tottime").print_stats(18)
    pipe = next(p for p in (v[1] for v in model._pipelines.values()) if p.n == args.in_flight)
    t_arg = torch.tensor([scene.cfg.t], device=dev)
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n):
            pipe.submit(t_arg)
        pipe.join()
        torch.cuda.synchronize()
        print(f"bare submit loop (readback of rgb/depth/weights into the slots, no fetch): "
              f"{(time.perf_counter() - t0) / n * 1e3:.3f} ms/frame")
    ro = pipe.readback
    pipe.readback = ()
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n):
            pipe.submit(t_arg)
        pipe.join()
        torch.cuda.synchronize()
        print(f"bare submit loop, no readback: {(time.perf_counter() - t0) / n * 1e3:.3f} ms/frame")
    pipe.readback = ro


if __name__ == "__main__":
    main()
