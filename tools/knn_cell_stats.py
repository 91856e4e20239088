"""CPU emulation of the radius kNN's work at a BASELINE config (default C2), per fine grid cell:
how many in-bbox samples fall in each cell, the cell bounds u_rho (points in cells whose box lies
within rho of the cell's box, rho = r/4, r/2, r -- apn_knn.hip k_cell_bound3) and which level a
cell's queries start at. Sizes the cell-cooperative kNN (one workgroup per query cell scanning the
cell's rho-dilated point set from LDS). Diagnostic tool, numpy only (no GPU)."""
from __future__ import annotations

import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "articulated-point-nerf_amd"))
sys.path.insert(0, ROOT)


def grid_params(lo, hi, r, cap=1 << 20, subdiv=8):
    """apn_knn.hip k_grid_params."""
    h = np.float32(r / subdiv)
    for _ in range(64):
        d = (np.floor((hi - lo) / h) + 1).astype(np.int64)
        if np.prod(d.astype(np.float64)) <= cap:
            break
        h = np.float32(h * np.cbrt(np.prod(d.astype(np.float64)) / cap) * 1.01)
    return float(h), d


def main():
    from apn_amd import harness, synthetic as S
    from oracle.apn_oracle import OracleModel, sample_pts_on_rays
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
    scene = S.make_scene(cfg)
    model = harness.build_model(scene, "cpu")
    st = {k: v.detach() for k, v in model.state_dict().items()}
    orc = OracleModel(st, model.canonical_pcd, model.bones, mean_min_distance_value=0.0)
    with torch.no_grad():
        _, (xyz, *_rest) = orc.warp(torch.tensor([scene.cfg.t]))
    xyz = xyz.numpy().astype(np.float32)
    r2 = np.float32(0.01)
    r = float(np.sqrt(r2))
    lo, hi = xyz.min(0), xyz.max(0)
    rk = scene.render_kwargs("cpu")
    pts, mask_out, ray_id, step_id, *_ = sample_pts_on_rays(
        rk["rays_o"].numpy(), rk["rays_d"].numpy(), lo - r2, hi + r2, rk["near"], rk["far"],
        rk["stepsize"] * S.VOXEL_SIZE)
    q = pts[~mask_out]
    print(f"{cfg}: {len(xyz)} points, {len(q)} in-bbox samples, bbox {hi - lo}")
    h, d = grid_params(lo, hi, r)
    print(f"fine cell h = {h:.5f} (r/{r / h:.2f}), dims {d.tolist()} = {int(np.prod(d))} cells")

    def cell_of(p):
        c = np.clip(np.floor((p - lo) / np.float32(h)).astype(np.int64), 0, d - 1)
        return (c[:, 2] * d[1] + c[:, 1]) * d[0] + c[:, 0], c

    pc, _ = cell_of(xyz)
    counts = np.bincount(pc, minlength=int(np.prod(d))).reshape(d[2], d[1], d[0])
    # prefix over x per (z, y) row -> row-chord sums
    cs = np.concatenate([np.zeros((d[2], d[1], 1), np.int64), np.cumsum(counts, axis=2)], axis=2)
    qc, qcc = cell_of(q)
    cells, qcount = np.unique(qc, return_counts=True)
    cz, cy, cx = cells // (d[0] * d[1]), (cells // d[0]) % d[1], cells % d[0]
    lim = (r / h) ** 2 * 1.0002
    K = int(math.ceil(math.sqrt(lim))) + 1
    u = {f: np.zeros(len(cells), np.int64) for f in (1, 2, 4, 8)}
    for dz in range(-K, K + 1):
        z = cz + dz
        okz = (z >= 0) & (z < d[2])
        gz = max(abs(dz) - 1, 0)
        for dy in range(-K, K + 1):
            y = cy + dy
            ok = okz & (y >= 0) & (y < d[1])
            gy = max(abs(dy) - 1, 0)
            for f, u_f in u.items():
                rem = lim / (f * f) - gz * gz - gy * gy
                if rem < 0:
                    continue
                kx = int(math.floor(math.sqrt(rem))) + 1
                x0 = np.clip(cx - kx, 0, d[0] - 1)
                x1 = np.clip(cx + kx, 0, d[0] - 1)
                zz, yy = np.clip(z, 0, d[2] - 1), np.clip(y, 0, d[1] - 1)
                u_f += np.where(ok, cs[zz, yy, x1 + 1] - cs[zz, yy, x0], 0)
    cand = u[1] >= 8
    first = np.where(u[4] >= 8, 4, np.where(u[2] >= 8, 2, 1))
    print(f"query cells {len(cells)}, queries/cell mean {qcount.mean():.1f}, max {qcount.max()}")
    print(f"rejected by u1 < 8: {qcount[~cand].sum()} queries in {(~cand).sum()} cells")
    for f in (4, 2, 1):
        m = cand & (first == f)
        if m.any():
            uu = u[f][m]
            print(f"first level r/{f}: {m.sum()} cells, {qcount[m].sum()} queries; staged points u_r/{f} "
                  f"per cell mean {uu.mean():.0f} p50 {np.median(uu):.0f} p90 {np.percentile(uu, 90):.0f} max {uu.max()}; "
                  f"sum over cells {uu.sum() / 1e6:.2f} M; query x point pairs {(uu * qcount[m]).sum() / 1e9:.3f} G")
    for f in (2, 1):
        m = cand & (first > f)
        uu = u[f][m]
        print(f"escalation to r/{f} (all cells starting above it): staged {uu.sum() / 1e6:.2f} M points, "
              f"pairs {(uu * qcount[m]).sum() / 1e9:.3f} G (upper bound: every query escalates)")
    # exact 8th-nearest distances of the candidate queries (scipy cKDTree), then the cooperative
    # schedule: a cell runs levels rho = r/8 (optional), r/4, r/2, r from the first with u >= 8;
    # a query is done at rho once its 8th-best squared distance < rho^2 (1 - 2e-4)
    from scipy.spatial import cKDTree
    qm = cand[np.searchsorted(cells, qc)]
    qi = np.nonzero(qm)[0]
    d8 = cKDTree(xyz.astype(np.float64)).query(q[qi].astype(np.float64), k=8)[0][:, -1] ** 2
    cell_idx = np.searchsorted(cells, qc[qi])
    print(f"candidates {len(qi)}; 8th-NN dist / r: p10 {np.sqrt(np.percentile(d8, 10)) / r:.3f} "
          f"p50 {np.sqrt(np.median(d8)) / r:.3f} p90 {np.sqrt(np.percentile(d8, 90)) / r:.3f}; "
          f"survivors {(d8 <= r2).sum()}")
    for levels in ((8, 4, 2, 1), (4, 2, 1)):
        pairs = staged = 0
        active = np.ones(len(qi), bool)
        started = np.zeros(len(qi), bool)
        per_level = []
        for f in levels:
            # a query participates from its cell's first level with u_f >= 8 (or f = 1)
            ucell = u[f][cell_idx]
            start_here = ~started & ((ucell >= 8) | (f == 1))
            started |= start_here
            part = active & started
            # staged once per cell that has a participating query
            cells_used = np.unique(cell_idx[part])
            staged += u[f][cells_used].sum()
            pairs += ucell[part].sum()
            rho2 = r2 / (f * f)
            done = part & ((d8 < rho2 * (1 - 2e-4)) if f > 1 else True)
            per_level.append((f, int(part.sum()), len(cells_used), int(ucell[part].sum())))
            active &= ~done
        print(f"levels {levels}: query x point pairs {pairs / 1e9:.3f} G, staged points {staged / 1e6:.1f} M; "
              + "; ".join(f"r/{f}: {n} queries in {c} cells, {p / 1e6:.0f} M pairs" for f, n, c, p in per_level))


if __name__ == "__main__" and len(sys.argv) <= 2:
    main()


def tile_model(T=2, cfg="C2", levels=(8, 4, 2, 1), lanes_per_query_max=1):
    """Cost model of the tile-cooperative kNN: query tiles of T^3 fine cells; per tile and level
    rho, the points of every fine row (z, y) whose yz gap to the tile box is <= rho, over the
    row's x chord (tile x-range dilated by rho), staged in order of that yz gap (ring = floor of
    gap / h); each query lane scans the staged points ring by ring and leaves once the ring's lower
    bound h * ring exceeds its 8th-best distance. Reports wave-iterations of the scan (max over the
    wave's lanes, 64 queries per wave) and points staged."""
    from apn_amd import harness, synthetic as S
    from oracle.apn_oracle import OracleModel, sample_pts_on_rays
    from scipy.spatial import cKDTree
    scene = S.make_scene(cfg)
    model = harness.build_model(scene, "cpu")
    st = {k: v.detach() for k, v in model.state_dict().items()}
    orc = OracleModel(st, model.canonical_pcd, model.bones, mean_min_distance_value=0.0)
    with torch.no_grad():
        _, (xyz, *_r) = orc.warp(torch.tensor([scene.cfg.t]))
    xyz = xyz.numpy().astype(np.float32)
    r2 = np.float32(0.01)
    r = float(np.sqrt(r2))
    lo, hi = xyz.min(0), xyz.max(0)
    rk = scene.render_kwargs("cpu")
    pts, mask_out, *_ = sample_pts_on_rays(rk["rays_o"].numpy(), rk["rays_d"].numpy(), lo - r2, hi + r2,
                                          rk["near"], rk["far"], rk["stepsize"] * S.VOXEL_SIZE)
    q = pts[~mask_out]
    tree = cKDTree(xyz.astype(np.float64))
    d8 = tree.query(q.astype(np.float64), k=8)[0][:, -1]
    cand = d8 <= r * 1.5          # stand-in for the u1 >= 8 filter (the rest are rejected cheaply)
    q, d8 = q[cand], d8[cand]
    h, d = grid_params(lo, hi, r)
    c = np.clip(np.floor((q - lo) / np.float32(h)).astype(np.int64), 0, d - 1)
    t = c // T
    tid = (t[:, 2] * 1000 + t[:, 1]) * 1000 + t[:, 0]
    order = np.argsort(tid, kind="stable")
    tid_s = tid[order]
    starts = np.flatnonzero(np.r_[True, tid_s[1:] != tid_s[:-1]])
    ends = np.r_[starts[1:], len(tid_s)]
    pc = np.clip(np.floor((xyz - lo) / np.float32(h)).astype(np.int64), 0, d - 1)
    scan_iters = staged = pairs = 0
    rng = np.random.default_rng(0)
    sample = rng.choice(len(starts), size=min(len(starts), 1500), replace=False)
    for s_i in sample:
        idx = order[starts[s_i]:ends[s_i]]
        t0 = t[idx[0]] * T
        box_lo = lo + t0 * np.float32(h)
        box_hi = box_lo + T * np.float32(h)
        active = np.ones(len(idx), bool)
        near = np.asarray(tree.query_ball_point((box_lo + box_hi) / 2, 1.8 * r + T * h), dtype=np.int64)
        pcn, xyzn = pc[near], xyz[near]
        for f in levels:
            rho = r / f
            # candidate points: yz gap of their cell row to the tile box <= rho, x within rho of the box
            gap = np.maximum(np.maximum(box_lo - (lo + pcn * h + h), (lo + pcn * h) - box_hi), 0)
            yz = np.sqrt(gap[:, 1] ** 2 + gap[:, 2] ** 2)
            sel = (yz <= rho * 1.0001) & (gap[:, 0] <= rho * 1.0001)
            n_st = int(sel.sum())
            if f != 1 and n_st < 8:
                continue
            staged += n_st
            ring = np.floor(yz[sel] / h).astype(np.int64)
            P = xyzn[sel]
            ring_sorted = np.sort(ring)
            # per query: points scanned until ring lower bound h*ring > its final 8th distance at this level
            dq = np.sqrt(((q[idx][:, None, :] - P[None]) ** 2).sum(-1))
            dq = np.where(dq <= r, dq, np.inf)
            k8 = np.sort(dq, axis=1)[:, 7] if dq.shape[1] >= 8 else np.full(len(idx), np.inf)
            exit_ring = np.floor(np.minimum(k8, rho) / h).astype(np.int64)
            scanned = np.searchsorted(ring_sorted, exit_ring, side="right")
            scanned = np.where(active, scanned, 0)
            pairs += scanned.sum()
            na = active.sum()
            # 64 query lanes per wave-batch; a batch iterates as long as its longest lane
            sc = np.sort(scanned[active])[::-1]
            for b in range(0, len(sc), 64):
                scan_iters += sc[b]
            done = (k8 < rho * (1 - 2e-4)) | (f == 1)
            active &= ~done
            if not active.any():
                break
    frac = len(starts) / len(sample)
    print(f"T={T}: {len(starts)} tiles, {len(q) / len(starts):.1f} queries/tile; scaled to all tiles: "
          f"scan wave-iterations {scan_iters * frac / 1e6:.1f} M, pairs {pairs * frac / 1e9:.3f} G, "
          f"staged {staged * frac / 1e6:.1f} M points")


if __name__ == "__main__" and len(sys.argv) > 2 and sys.argv[2] == "tiles":
    for T in (1, 2, 4):
        tile_model(T, sys.argv[1])


def seed_model(cfg="C2"):
    """How tight is the 8-NN bound a query inherits from its ray neighbours (the samples one step
    before / after it on the same ray, stepdist = 0.17 r at C2)? For every candidate query whose
    neighbour survived: tau = max distance from the query to the neighbour's 8 nearest points
    (an upper bound on its own 8th-NN distance d8), reported as tau / d8 and tau / r."""
    from apn_amd import harness, synthetic as S
    from oracle.apn_oracle import OracleModel, sample_pts_on_rays
    from scipy.spatial import cKDTree
    scene = S.make_scene(cfg)
    model = harness.build_model(scene, "cpu")
    st = {k: v.detach() for k, v in model.state_dict().items()}
    orc = OracleModel(st, model.canonical_pcd, model.bones, mean_min_distance_value=0.0)
    with torch.no_grad():
        _, (xyz, *_r) = orc.warp(torch.tensor([scene.cfg.t]))
    xyz = xyz.numpy().astype(np.float32)
    r2 = np.float32(0.01)
    r = float(np.sqrt(r2))
    lo, hi = xyz.min(0), xyz.max(0)
    rk = scene.render_kwargs("cpu")
    pts, mask_out, ray_id, step_id, *_ = sample_pts_on_rays(
        rk["rays_o"].numpy(), rk["rays_d"].numpy(), lo - r2, hi + r2, rk["near"], rk["far"],
        rk["stepsize"] * S.VOXEL_SIZE)
    m = ~mask_out
    q, ray_id, step_id = pts[m], ray_id[m], step_id[m]
    tree = cKDTree(xyz.astype(np.float64))
    d, nn = tree.query(q.astype(np.float64), k=8)
    d8 = d[:, -1]
    surv = d8 <= r
    hard = (d8 > r / 4) & (d8 <= 1.5 * r)    # pass-B-like queries (not finished inside r/4)
    for name, off in (("prev", -1), ("next", 1), ("both", 0)):
        taus = []
        idx = np.nonzero(hard)[0]
        tau = np.full(len(idx), np.inf)
        for o in ((-1,) if off == -1 else (1,) if off == 1 else (-1, 1)):
            j = idx + o
            ok = (j >= 0) & (j < len(q))
            jj = np.clip(j, 0, len(q) - 1)
            ok &= (ray_id[jj] == ray_id[idx]) & (step_id[jj] == step_id[idx] + o) & surv[jj]
            pn = xyz[nn[jj]]                                   # [n, 8, 3]
            t = np.sqrt(((q[idx][:, None, :] - pn) ** 2).sum(-1)).max(1)
            tau = np.where(ok, np.minimum(tau, t), tau)
        have = np.isfinite(tau)
        ratio = tau[have] / d8[idx][have]
        print(f"{name}: {have.mean():.3f} of {len(idx)} hard queries have a surviving ray neighbour; "
              f"tau/d8 p50 {np.median(ratio):.3f} p90 {np.percentile(ratio, 90):.3f}; "
              f"(tau/r)^2 mean {np.mean((tau[have] / r) ** 2):.3f} vs (d8/r)^2 {np.mean((d8[idx][have] / r) ** 2):.3f}")


if __name__ == "__main__" and len(sys.argv) > 2 and sys.argv[2] == "seeds":
    seed_model(sys.argv[1])
