"""Load balance of the ray-sharded frame measured on ONE GPU: the C2 frame's
shards for world = 2, 4, 8 rendered one after another (ray_shard=(k, world)), each timed with HIP
events, next to its in-bbox samples and kNN survivors (the MLP's work). The max over shards is
what a strong-scaling step waits for. Diagnostic tool (not a test).

    python tools/shard_balance.py [--config C2] [--reps 5] [--split inbbox,cost]

--split cost: the split render_sharded uses from the second frame on (shard.cost_offsets of the
previous frame's survivors and in-bbox samples), preset in the model's SplitTracker.
--split ilv<B> / gilv<B> (graph replays): the "blocks" split of render_sharded with blocks of B rays (rank k takes blocks
k, k + W, ...; ray_shard=(k, W, B)): equal ray counts, an unpadded all-gather.
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
    ap.add_argument("--split", default="inbbox,cost")
    ap.add_argument("--kept-weights", default="", help="comma list of shard.KEPT_WEIGHT values to try (cost split)")
    ap.add_argument("--in-flight", type=int, default=1,
                    help="gilv splits: replay each shard's frames with this many in flight (the shard's graph "
                         "captured into as many workspaces of one model, on as many streams, bench.py --in-flight; "
                         "no all-gather)")
    args = ap.parse_args()
    torch.set_grad_enabled(False)
    dev = torch.device("cuda", 0)
    scene = S.make_scene(args.config)
    model = harness.build_model(scene, dev)
    rk = scene.render_kwargs(dev)
    t = torch.tensor([scene.cfg.t], device=dev)
    poses, Ks = scene.c2w[None].to(dev), scene.K[None].to(dev)
    kw = dict(render_depth=True, render_kwargs=rk, render_weights=True, poses=poses, Ks=Ks, get_skeleton=True)

    stages = {}

    def timed(fn, reps, warm=2):
        for _ in range(warm):
            fn()
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            out = fn()
        e1.record()
        torch.cuda.synchronize(dev)
        ms = e0.elapsed_time(e1) / reps
        model.timing = {}   # one more frame with HIP-event stage marks
        fn()
        torch.cuda.synchronize(dev)
        marks = model.timing.get("marks", [])
        model.timing = None
        stages.clear()
        for (_, a), (name, b) in zip(marks[:-1], marks[1:]):
            if name != "frame":
                stages[name] = stages.get(name, 0.0) + a.elapsed_time(b)
        return ms, out

    from apn_amd.ops import Workspace
    extra = [Workspace() for _ in range(args.in_flight - 1)]   # frames in flight: per-frame workspaces of one model
    fl_streams = [torch.cuda.Stream(dev) for _ in range(args.in_flight)]

    def in_flight(gsteps):
        cur = torch.cuda.current_stream(dev)
        for s in fl_streams:
            s.wait_stream(cur)
        for i in range(len(gsteps) * 4):
            with torch.cuda.stream(fl_streams[i % len(gsteps)]):
                gsteps[i % len(gsteps)](t)
        for s in fl_streams:
            cur.wait_stream(s)

    full_ms, out = timed(lambda: model(t, **kw), args.reps)
    st = model.last_stats.resolved()
    print(f"full frame {full_ms:.3f} ms, {st}")
    from apn_amd.shard import SplitTracker, bounds_from_inner, cost_offsets, split_inner
    R = rk["rays_o"].shape[0]
    kept = model.last_kept_per_ray(R).clone()
    offs = model._ws.get("offs", R + 1, torch.int32, dev).clone()
    import apn_amd.shard as SH
    splits = args.split.split(",")
    if args.kept_weights:
        splits = [s for s in splits if s != "cost"] + [f"cost{w}" for w in args.kept_weights.split(",")]
    for split, world in [(sp, int(w)) for sp in splits for w in args.worlds.split(",")]:
        if split.startswith("ilv") or split.startswith("gilv"):
            graph = split.startswith("g")
            B = int(split[4:] if graph else split[3:])
            rows, fl_all = [], []
            for k in range(world):
                if graph:   # the rank's frame as one graph replay (shard.capture_sharded, bench's step)
                    fk = {n: v for n, v in kw.items() if n not in ("render_kwargs", "render_depth", "render_weights")}
                    gstep = model.capture_frame(t, rk, ray_shard=(k, world, B), **fk)
                    fn = lambda: gstep(t)   # noqa: E731
                    if extra:   # frames in flight: timed per frame (4 rounds of len(gsteps) frames per call)
                        gsteps = [gstep] + [model.capture_frame(t, rk, ray_shard=(k, world, B), workspace=w, **fk)
                                            for w in extra]
                        fl_ms, _ = timed(lambda: in_flight(gsteps), args.reps, warm=4)
                        print(f"   shard {k}: {args.in_flight} in flight {fl_ms / (4 * len(gsteps)):.3f} ms/frame")
                        fl_all.append((k, gsteps))
                else:
                    fn = lambda: model(t, ray_shard=(k, world, B), **kw)   # noqa: E731
                ms, o = timed(fn, args.reps)
                s = model.last_stats.resolved()
                rows.append((ms, s.get("inbbox_samples", -1), s.get("kept_samples", -1), model.last_ray_count))
                print(f"   shard {k}: {ms:.3f} ms, stages " + " ".join(f"{n} {v:.3f}" for n, v in stages.items()))
            if fl_all:   # every shard's in-flight replay again, after all shards were captured (the first
                # shard's first timing runs right after the previous world's graphs were dropped)
                again = []
                for k2, gs in fl_all:
                    fl_ms, _ = timed(lambda: in_flight(gs), args.reps, warm=2)
                    again.append(fl_ms / (4 * len(gs)))
                print(f"   {args.in_flight} in flight, all shards re-timed: " + " ".join(f"{v:.3f}" for v in again)
                      + f" | max {max(again):.3f} ms/frame")
                fl_all.clear()
            mx = max(r[0] for r in rows)
            mean = sum(r[0] for r in rows) / world
            print(f"[{split}] world {world}: shard ms " + " ".join(f"{r[0]:.3f}" for r in rows)
                  + f" | max {mx:.3f} mean {mean:.3f} (max/mean {mx / mean:.3f}); ideal full/world {full_ms / world:.3f}; "
                  f"speedup bound {full_ms / mx:.2f}x")
            print("   kept per shard: " + " ".join(str(r[2]) for r in rows)
                  + " | inbbox per shard: " + " ".join(str(r[1]) for r in rows))
            continue
        model._splits.clear()
        model._capacity = {k: v for k, v in model._capacity.items() if not isinstance(k, tuple)}
        if split.startswith("cost"):
            if split != "cost":
                SH.KEPT_WEIGHT = int(split[4:])
            tr = SplitTracker()
            tr.bounds = bounds_from_inner(split_inner(cost_offsets(offs, kept), world).cpu().tolist(), R)
            tr.cost_mode = True
            model._splits[(R, world)] = tr
        rows = []
        for k in range(world):
            ms, o = timed(lambda: model(t, ray_shard=(k, world), **kw), args.reps)
            s = model.last_stats.resolved()
            r0, r1 = model.last_ray_range
            rows.append((ms, s.get("inbbox_samples", -1), s.get("kept_samples", -1), r1 - r0))
            print(f"   shard {k}: {ms:.3f} ms, stages " + " ".join(f"{n} {v:.3f}" for n, v in stages.items()))
        mx = max(r[0] for r in rows)
        mean = sum(r[0] for r in rows) / world
        print(f"[{split}] world {world}: shard ms " + " ".join(f"{r[0]:.3f}" for r in rows)
              + f" | max {mx:.3f} mean {mean:.3f} (max/mean {mx / mean:.3f}); ideal full/world {full_ms / world:.3f}; "
              f"speedup bound {full_ms / mx:.2f}x")
        print("   kept per shard: " + " ".join(str(r[2]) for r in rows)
              + " | inbbox per shard: " + " ".join(str(r[1]) for r in rows)
              + " | rays: " + " ".join(str(r[3]) for r in rows))


if __name__ == "__main__":
    main()
