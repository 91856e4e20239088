"""Algorithmic work of the frame's radius kNN: what a perfect exact search
must touch, computed after the fact from the frame's own survivors, to set beside the measured
kNN time and the executed instruction count of its kernels.

The reference's search is a brute-force pykeops Kmin_argKmin over every (sample, point) pair
(/root/reference/lib/temporalpoints.py:433-447): Q x N distance evaluations. Our search
(csrc/apn_knn.hip, mode 9) scans x-rows of a uniform grid. Its algorithmic work is defined here
as the work of a PERFECT scan on a grid of cell h = r / 8 (the kernel's KNN_SUBDIV), one that
knows every query's final answer in advance:

  * a survivor (8th-NN squared distance d8 <= r^2) must read every point of the cells on the
    x-chords of its final ball (radius sqrt(d8)) -- the rows (y, z) whose slab is within
    sqrt(d8) of the query, each over the x-cells the ball's chord crosses; ``chord_rows`` and
    ``chord_points`` sum those over the survivors;
  * the points inside the final ball are K = 8 per survivor (ties aside): ``ball_points``;
  * a rejected sample costs one lookup of a coarse cell count (the classify test): 0 points.

``valu_lane_ops`` prices that work at 7 VALU lane operations per point (3 subtracts, 1 multiply,
2 fma, 1 compare with the 8th best) and 4 per row (slab bound, two cell-start offsets, the
compare), so the VALU-issue time of the perfect scan is valu_lane_ops / 64 lanes x 2 cycles per
wave instruction / 1024 SIMDs / clock (MI355X_MICROARCH.md: a wave issues a VALU instruction
over 2 cycles). That figure is a floor, not a target: the search is bound by dependent load
latency and lane divergence, which the executed instruction count (PMC SQ_INSTS_VALU) shows.
"""
import torch

KNN_K = 8
SUBDIV = 8                 # fine cell = r / 8, as KNN_SUBDIV in csrc/apn_knn.hip
OPS_PER_POINT = 7
OPS_PER_ROW = 4
SIMDS = 1024
CYCLES_PER_WAVE_VALU = 2


def _grid_counts(pts, lo, h, dims):
    c = torch.floor((pts - lo) / h).long()
    c = torch.minimum(torch.clamp(c, min=0), torch.tensor(dims, device=pts.device) - 1)
    dx, dy, dz = dims
    lin = (c[:, 2] * dy + c[:, 1]) * dx + c[:, 0]
    cnt = torch.bincount(lin, minlength=dx * dy * dz)
    pre = torch.zeros(dx * dy * dz + 1, dtype=torch.int64, device=pts.device)
    pre[1:] = torch.cumsum(cnt, 0)
    return pre


@torch.no_grad()
def knn_work(cloud, s_pos, s_nbr, r2, chunk=1 << 15):
    """cloud [N,3] (the warped points the kNN searched), s_pos [S,3] survivors' sample
    positions, s_nbr [S,8] their neighbour indices (into cloud), r2 = query radius squared.
    Returns the perfect-scan counts described in the module docstring."""
    dev = cloud.device
    cloud = cloud.float()
    S = int(s_pos.shape[0])
    r = float(r2) ** 0.5
    h = r / SUBDIV
    lo = cloud.min(0).values - 1e-6
    hi = cloud.max(0).values + 1e-6
    dims = [int(v) for v in (torch.floor((hi - lo) / h).long() + 1).tolist()]
    dx, dy, dz = dims
    pre = _grid_counts(cloud, lo, h, dims)
    m = SUBDIV + 1                                            # rows within r of the query's cell
    off = torch.arange(-m, m + 1, device=dev)
    oz, oy = torch.meshgrid(off, off, indexing="ij")
    oz, oy = oz.reshape(-1), oy.reshape(-1)
    rows = pts = 0
    for a in range(0, S, chunk):
        q = s_pos[a:a + chunk].float()
        nb = s_nbr[a:a + chunk].long()
        d = cloud[nb[:, KNN_K - 1]] - q                       # 8th neighbour (the lists are sorted)
        rho2 = (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]
        rho = rho2.sqrt()
        cq = torch.floor((q - lo) / h).long()
        cy = cq[:, 1:2] + oy                                  # [n, rows]
        cz = cq[:, 2:3] + oz
        # squared distance from the query to the (y, z) slab of each row
        y0 = lo[1] + cy * h
        z0 = lo[2] + cz * h
        ty = torch.clamp(torch.maximum(y0 - q[:, 1:2], q[:, 1:2] - (y0 + h)), min=0)
        tz = torch.clamp(torch.maximum(z0 - q[:, 2:3], q[:, 2:3] - (z0 + h)), min=0)
        syz = ty * ty + tz * tz
        ok = (syz <= rho2[:, None]) & (cy >= 0) & (cy < dy) & (cz >= 0) & (cz < dz)
        half = torch.sqrt(torch.clamp(rho2[:, None] - syz, min=0))
        x0 = torch.floor((q[:, 0:1] - half - lo[0]) / h).long()
        x1 = torch.floor((q[:, 0:1] + half - lo[0]) / h).long()
        ok &= (x1 >= 0) & (x0 < dx)
        x0, x1 = torch.clamp(x0, 0, dx - 1), torch.clamp(x1, 0, dx - 1)
        base = (torch.clamp(cz, 0, dz - 1) * dy + torch.clamp(cy, 0, dy - 1)) * dx
        cnt = pre[base + x1 + 1] - pre[base + x0]
        rows += int(ok.sum())
        pts += int(torch.where(ok, cnt, torch.zeros_like(cnt)).sum())
        del rho
    lane_ops = OPS_PER_POINT * pts + OPS_PER_ROW * rows
    return {"survivors": S, "grid_cell": h, "ball_points": KNN_K * S, "chord_rows": rows,
            "chord_points": pts, "valu_lane_ops": lane_ops}


def valu_issue_ms(lane_ops, clock_ghz):
    """VALU-issue time of lane_ops lane operations spread over the whole chip."""
    return lane_ops / 64 * CYCLES_PER_WAVE_VALU / SIMDS / (clock_ghz * 1e9) * 1e3
