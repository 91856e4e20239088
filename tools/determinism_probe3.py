"""Determinism probe 3 (round 3): several processes share the GPU, each rendering the same frame
over and over (the spawn test's 200x200 / 50k-point / 24-bone scene; workers 0 and 1 render the
two shards of the 2-way blocks split, worker 2 the full frame), and every frame's stage outputs
are compared with the process's reference frame:

    t_hat_pcd -> bbox_ord -> sorted4 (as a set) -> in-bbox samples -> kNN survivors + neighbours
    -> MLP out12 -> per-ray tile

The first stage that differs names the kernel to look at. Diagnostic tool (not a test); the
parent never touches the GPU. Usage: python tools/determinism_probe3.py [frames] [mode] [nproc]
(mode: exact = every frame on the host-synced path, default = the capacity path after frame 0).
"""
from __future__ import annotations

import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "articulated-point-nerf_amd"))

STAGES = ("xyz", "bbox", "sorted_set", "q_pos", "q_ray", "nsurv", "s_pos", "s_ray", "s_nbr", "out12", "tile")


def snapshot(model, out, R):
    from apn_amd.shard import pack_tile
    ws = model._ws.bufs
    xyz = out.raw("t_hat_pcd").detach().clone()
    N = xyz.shape[0]
    snap = {"xyz": xyz, "bbox": ws["bbox_ord"][:6].clone(), "recA_xyz": ws["recA"][:N * 16].view(N, 16)[:, :3].clone()}
    s4 = ws["sorted4"][:N * 4].view(N, 4)
    idx = s4[:, 3].contiguous().view(torch.int32).long()
    canon = torch.empty_like(s4)
    canon[idx] = s4
    snap["sorted_set"] = canon.clone()
    snap["sorted_order"] = idx.clone()
    info = model._last_info
    if info is not None:
        nq = int(info[0].item())
    else:
        nq = int(model.last_stats["inbbox_samples"])
    snap["q_pos"] = ws["q_pos"][:nq * 4].clone()
    snap["q_ray"] = ws["q_ray"][:nq].clone()
    ns = int(model.last_stats._nsurv.item())
    snap["nsurv"] = torch.tensor([ns, nq])
    snap["s_pos"] = ws["s_pos"][:ns * 4].clone()
    snap["s_ray"] = ws["s_ray"][:ns].clone()
    snap["s_nbr"] = ws["s_nbr"][:ns * 8].clone()
    snap["out12"] = ws["out12"][:ns * 12].clone()
    snap["tile"] = pack_tile(out, R, xyz.device).clone()
    return snap


def first_diff(a, b):
    for k in STAGES:
        x, y = a[k], b[k]
        if x.shape != y.shape:
            return k, f"shape {tuple(x.shape)} vs {tuple(y.shape)}"
        ne = x != y
        if x.dtype.is_floating_point:
            ne = ne & ~(torch.isnan(x) & torch.isnan(y))
        if bool(ne.any()):
            nz = ne.nonzero().flatten()
            return k, f"{int(ne.sum())} differ, first at {nz[:6].tolist()}"
    return None, ""


def worker(wid, nproc, frames, mode, outdir):
    from apn_amd import harness, synthetic as S
    torch.set_grad_enabled(False)
    dev = torch.device("cuda", 0)
    scene = S.make_scene(S.SceneConfig("probe3 200x200 50k pts 24 bones", 50_000, 24, 200, 200))
    model = harness.build_model(scene, dev)
    rk = scene.render_kwargs(dev)
    R_all = rk["rays_o"].shape[0]
    t0 = torch.tensor([scene.cfg.t], device=dev)
    kw = dict(poses=scene.c2w[None].to(dev), Ks=scene.K[None].to(dev), get_skeleton=True, render_depth=True,
              render_weights=True)
    shard = (wid % 2, 2, 4096) if wid < 2 else None
    ref = None
    order_changes = 0
    bad = {}
    log = []
    t_start = time.time()
    for f in range(frames):
        if mode == "exact":
            model._force_exact = True
        out = model(t0, render_kwargs=rk, ray_shard=shard, **kw)
        R = model.last_ray_count if shard is not None else R_all
        torch.cuda.synchronize()
        snap = snapshot(model, out, R)
        model._force_exact = False
        if ref is None or (mode != "exact" and f == 1):
            ref = snap
            continue
        if not torch.equal(snap["sorted_order"], ref["sorted_order"]):
            order_changes += 1
        st, msg = first_diff(snap, ref)
        if st is not None:
            bad[st] = bad.get(st, 0) + 1
            if len(log) < 20:
                detail = ""
                if st == "xyz":
                    rows = (snap["xyz"] != ref["xyz"]).any(1).nonzero().flatten()[:3].tolist()
                    detail = "; ".join(f"pt {r}: now {snap['xyz'][r].tolist()} ref {ref['xyz'][r].tolist()} "
                                       f"recA now {snap['recA_xyz'][r].tolist()} ref {ref['recA_xyz'][r].tolist()}"
                                       for r in rows)
                log.append(f"frame {f}: first differing stage {st}: {msg} {detail}")
            if os.environ.get("PROBE_DUMP") and len(log) <= 1:
                torch.save({k: v.cpu() for k, v in snap.items()} | {f"ref_{k}": v.cpu() for k, v in ref.items()},
                           os.path.join(outdir, f"probe3_w{wid}_f{f}.pt"))
        if f % 200 == 0:
            print(f"worker {wid}: frame {f} ({time.time() - t_start:.1f} s) bad {bad}", flush=True)
    print(f"worker {wid} ({'shard %d of 2' % shard[0] if shard else 'full frame'}, mode {mode}): {frames} frames, "
          f"in-cell order changed in {order_changes}, first differing stages {bad}", flush=True)
    for line in log:
        print(f"  worker {wid}: {line}", flush=True)


def main():
    frames = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    mode = sys.argv[2] if len(sys.argv) > 2 else "default"
    nproc = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    outdir = os.path.join(ROOT, "gpurun_out", "probe3")
    os.makedirs(outdir, exist_ok=True)
    import torch.multiprocessing as mp
    mp.spawn(worker, args=(nproc, frames, mode, outdir), nprocs=nproc, join=True)


if __name__ == "__main__":
    main()
