"""Probe: frame throughput with n frames in flight. ONE TemporalPoints, its frame captured as a HIP
graph into n per-frame workspaces (capture_frame(workspace=...), as apn_amd.pipeline does); K
frames replayed one after another on one stream vs over n streams (frame i on stream i % n, so one
frame's MLP runs beside the next frames' kNN / sampling). Checks every graph's frame against an
eager frame of the model.

    python tools/frames_in_flight.py [--config C2] [--frames 20] [--shard RANK,WORLD]
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
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--n", type=int, default=2, help="frames in flight")
    ap.add_argument("--shard", default="", help="rank,world: replay that ray shard's graph (blocks split) instead")
    args = ap.parse_args()
    torch.set_grad_enabled(False)
    dev = torch.device("cuda", 0)
    scene = S.make_scene(args.config)
    rk = scene.render_kwargs(dev)
    t = torch.tensor([scene.cfg.t], device=dev)
    poses, Ks = scene.c2w[None].to(dev), scene.K[None].to(dev)
    from apn_amd.ops import Workspace
    m = harness.build_model(scene, dev)
    _ = m.mean_min_distance
    for _ in range(2):
        m(t, render_depth=True, render_kwargs=rk, render_weights=True, poses=poses, Ks=Ks, get_skeleton=True)
    shard = None
    if args.shard:
        rank, world = (int(v) for v in args.shard.split(","))
        shard = (rank, world, 4096)
    steps = [m.capture_frame(t, rk, poses=poses, Ks=Ks, get_skeleton=True, ray_shard=shard, workspace=Workspace())
             for _ in range(args.n)]
    torch.cuda.synchronize(dev)
    cur = torch.cuda.current_stream(dev)
    streams = [torch.cuda.Stream(dev) for _ in range(args.n)]

    def serial(k):
        for _ in range(k):
            steps[0](t)

    def pipelined(k):
        ev = torch.cuda.Event()
        ev.record(cur)
        for s in streams:
            s.wait_event(ev)
        for i in range(k):
            with torch.cuda.stream(streams[i % args.n]):
                steps[i % args.n](t)
        for s in streams:
            cur.wait_stream(s)

    def timed(fn, k):
        fn(2)
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn(k)
        e1.record()
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) / k

    for rep in range(3):
        ts = timed(serial, args.frames)
        tp = timed(pipelined, args.frames)
        print(f"rep {rep}: serial {ts:.3f} ms/frame, {args.n} in flight {tp:.3f} ms/frame ({ts / tp:.3f}x)")
    # every graph's frame equals an eager frame of the model bit for bit
    keys = ("rgb_marched", "depth", "alphainv_last")
    eager = m(t, render_depth=True, render_kwargs=rk, render_weights=True, poses=poses, Ks=Ks, get_skeleton=True,
              ray_shard=shard)
    ref = {k: eager[k].clone() for k in keys}
    same = []
    for i in range(args.n):
        with torch.cuda.stream(streams[i]):
            o = steps[i](t)
        torch.cuda.synchronize(dev)
        same.append(all(torch.equal(o[k], ref[k]) for k in keys))
    print(f"frames of the {args.n} graphs identical to the eager frame: {same}")

if __name__ == "__main__":
    main()
