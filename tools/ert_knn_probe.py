"""How much of the frame's kNN work lies past early ray termination (diagnostic, not a test).

Renders the frame once with every kept sample through the MLP (early_termination off), then walks
each ray's kept samples on the host with the compositing's rules (pre-mask alpha > thr, T in double,
break once T < 1e-3; apn_composite.hip) for the Point-NeRF path and the direct path, and counts
the in-bbox queries and kNN survivors whose step lies past the LATER of the two breaks: the queries
a kNN interleaved with the MLP passes could skip.

    python tools/ert_knn_probe.py [--config C2]
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "articulated-point-nerf_amd"))
from apn_amd import harness, synthetic as S  # noqa: E402


def breaks(ray, alpha, n_rays, thr):
    """Per ray: index (into the survivor arrays) of the sample whose update took T below 1e-3, or
    -1. Survivors are in (ray, step) order."""
    out = np.full(n_rays, -1, dtype=np.int64)
    T = np.ones(n_rays, dtype=np.float64)
    alive = np.ones(n_rays, dtype=bool)
    for i in range(len(ray)):
        r = ray[i]
        if not alive[r]:
            continue
        a = alpha[i]
        if thr <= 0 or a > thr:
            T[r] = np.float32(T[r] * (1.0 - float(a)))
            if T[r] < 1e-3:
                alive[r] = False
                out[r] = i
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    args = ap.parse_args()
    torch.set_grad_enabled(False)
    dev = torch.device("cuda", 0)
    scene = S.make_scene(args.config)
    model = harness.build_model(scene, dev)
    model.early_termination = False
    rk = scene.render_kwargs(dev)
    t = torch.tensor([scene.cfg.t], device=dev)
    poses, Ks = scene.c2w[None].to(dev), scene.K[None].to(dev)
    kw = dict(render_depth=True, render_kwargs=rk, render_weights=True, poses=poses, Ks=Ks, get_skeleton=True)
    for _ in range(2):
        model(t, **kw)
    torch.cuda.synchronize(dev)
    b = model._ws.bufs
    R = int(model._last_ray_ws[1])
    n_q = int(b["offs"][R].item())
    S_ = int(model.last_stats._nsurv.item())
    q_pos = b["q_pos"][: 4 * n_q].view(n_q, 4)
    q_step = q_pos[:, 3].contiguous().view(torch.int32).cpu().numpy().astype(np.int64)
    q_ray = b["q_ray"][:n_q].cpu().numpy()
    s_pos = b["s_pos"][: 4 * S_].view(S_, 4)
    s_step = s_pos[:, 3].contiguous().view(torch.int32).cpu().numpy().astype(np.int64)
    s_ray = b["s_ray"][:S_].cpu().numpy()
    out12 = b["out12"][: 12 * S_].view(S_, 12).cpu().numpy()
    thr = float(model.fast_color_thres)
    bp = breaks(s_ray, out12[:, 3], R, thr)
    bd = breaks(s_ray, out12[:, 7], R, thr)
    big = np.int64(1) << 40
    last_pn = np.where(bp >= 0, s_step[np.maximum(bp, 0)], big)
    last_d = np.where(bd >= 0, s_step[np.maximum(bd, 0)], big)
    last_both = np.maximum(last_pn, last_d)
    past_q_pn = q_step > last_pn[q_ray]
    past_q = q_step > last_both[q_ray]
    past_s_pn = s_step > last_pn[s_ray]
    past_s = s_step > last_both[s_ray]
    print(f"{args.config}: rays {R}, in-bbox queries {n_q}, survivors {S_}, thr {thr}")
    print(f"  rays terminated: point-nerf {int((bp >= 0).sum())}, direct {int((bd >= 0).sum())}, "
          f"both {int(((bp >= 0) & (bd >= 0)).sum())}")
    print(f"  past the point-nerf break: queries {past_q_pn.mean():.3f}, survivors {past_s_pn.mean():.3f}")
    print(f"  past both breaks:          queries {past_q.mean():.3f}, survivors {past_s.mean():.3f}")
    # the kNN's candidates (apn_knn.hip knn_radius_impl workspace: cand_blk | cand | cblk_cnt | cblk_off)
    al = lambda x: (x + 255) // 256 * 256  # noqa: E731
    Qcap = b["q_ray"].numel()
    nb = (Qcap + 255) // 256
    slots = nb * 256
    kws = b["knn_ws"]
    o_cand = al(slots * 4)
    o_off = o_cand + al(slots * 4) + al((nb + 2) * 4)
    n_c = int(kws[o_off + 4 * nb: o_off + 4 * nb + 4].view(torch.int32).item())
    cand = kws[o_cand: o_cand + 4 * n_c].view(torch.int32).cpu().numpy().astype(np.int64)
    c_ray, c_step = q_ray[cand], q_step[cand]
    past_c = c_step > last_both[c_ray]
    print(f"  candidates {n_c} ({n_c / n_q:.3f} of the queries); past both breaks {past_c.mean():.3f}")
    # per dead ray: candidates up to (and including) the later break
    print("  candidate rays sorted:", bool(np.all(np.diff(c_ray) >= 0)))
    dead = np.nonzero(last_both < big)[0]
    need_all = np.bincount(c_ray, weights=(c_step <= last_both[c_ray]).astype(np.float64), minlength=R)
    tot_all = np.bincount(c_ray, minlength=R)
    need, tot = need_all[dead], tot_all[dead]
    print("  dead rays: candidates needed, percentiles 50/75/90/95/99:", np.percentile(need, [50, 75, 90, 95, 99]))
    print("  dead rays: candidates total,  percentiles 50/75/90/95/99:", np.percentile(tot, [50, 75, 90, 95, 99]))
    print("  all rays: candidates total,  percentiles 50/75/90/95/99/max:", np.percentile(tot_all, [50, 75, 90, 95, 99, 100]))
    for W in (8, 16, 24, 32, 48, 64):
        done = (need <= W).mean()
        work = np.minimum(tot, W).sum() + (c_ray.size - tot.sum())
        print(f"  W={W}: dead rays finished in pass 1 {done:.3f}; candidates through the kNN in pass 1 "
              f"{work / n_c:.3f}; after pass 2 (rest of the unfinished) "
              f"{(work + np.where(need > W, tot - W, 0).sum()) / n_c:.3f}")


if __name__ == "__main__":
    main()
