"""The kNN work model (apn_amd/knn_work.py, reported in bench.py's "knn" object): the perfect-scan
counts equal a per-point brute-force evaluation of the same definition, and bound the ball."""
import numpy as np
import torch

from apn_amd.knn_work import knn_work, valu_issue_ms


def _brute(cloud, q, nb8, r2):
    h = r2 ** 0.5 / 8
    lo = cloud.min(0).values - 1e-6
    cc = torch.floor((cloud - lo) / h).long()
    y0, z0 = lo[1] + cc[:, 1] * h, lo[2] + cc[:, 2] * h
    pts = inball = 0
    for i in range(q.shape[0]):
        qq = q[i]
        d = cloud[nb8[i]] - qq
        rho2 = float((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2])
        ty = torch.clamp(torch.maximum(y0 - qq[1], qq[1] - (y0 + h)), min=0)
        tz = torch.clamp(torch.maximum(z0 - qq[2], qq[2] - (z0 + h)), min=0)
        syz = ty * ty + tz * tz
        half = torch.sqrt(torch.clamp(rho2 - syz, min=0))
        xa = torch.floor((qq[0] - half - lo[0]) / h).long()
        xb = torch.floor((qq[0] + half - lo[0]) / h).long()
        pts += int(((syz <= rho2) & (cc[:, 0] >= xa) & (cc[:, 0] <= xb)).sum())
        inball += int((((cloud - qq) ** 2).sum(1) <= rho2 * (1 + 1e-6)).sum())
    return pts, inball


def test_perfect_scan_counts_match_brute_force():
    rng = np.random.default_rng(0)
    cloud = torch.tensor(rng.random((3000, 3)), dtype=torch.float32) * 0.5
    q = torch.tensor(rng.random((300, 3)), dtype=torch.float32) * 0.6 - 0.05   # some outside the cloud
    d = ((q[:, None, :] - cloud[None]) ** 2).sum(-1)
    dd, nb = torch.sort(d, 1)
    keep = dd[:, 7] <= 0.01
    assert 0 < int(keep.sum()) < 300
    w = knn_work(cloud, q[keep], nb[keep, :8].int(), 0.01, chunk=37)
    pts, inball = _brute(cloud, q[keep], nb[keep, 7], 0.01)
    assert w["chord_points"] == pts
    assert w["chord_points"] >= inball >= w["ball_points"]
    assert w["valu_lane_ops"] == 7 * w["chord_points"] + 4 * w["chord_rows"]
    # 64 lanes x 1024 SIMDs per 2 cycles = 32768 lane ops per cycle; at 2 GHz 65536 per ns
    assert abs(valu_issue_ms(65536 * 1e6, 2.0) - 1.0) < 1e-9
