"""TiNeuVox stage 1 on the MI355X: the realistic 12 x 160^3 feature grid
(configs/nerf/default.py: num_voxels 160^3, voxel_dim 12, defor_depth 3, net_width 128).

Two HIP launches over the canonical export's query set (run.py:1152-1194: every grid point,
4.1 M points in raster order) and over as many uniformly random points (no locality):
  * apn_tnv_mult_dist_interp -- the 3-scale trilinear lookup alone (tineuvox.py:402-419);
  * apn_tnv_field -- deformation MLP + lookup + featurenet + density + rgb head (458-564).
Prints one JSON line: kernel times (HIP events, average of --reps launches), the lookup's HBM
roofline (unique bytes: the packed 3-scale grid once + 12 B in + 144 B out per point, against
8 TB/s; also the corner-gather rate, 3 x 8 x 48 B per point) and the field's F_alg rate
(flops of the reference's layers per sample) against the FP32 matrix peak."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "articulated-point-nerf_amd"))

HBM_PEAK_GBS = 8000.0
FP32_MFMA_PEAK_TFLOPS = 157.3


def field_flop_per_sample(D=3, W=128, pe=63, t_out=60, grid=180, views=27):
    deform = 2 * ((pe + t_out) * W + (D - 1) * W * W + W * 3)
    feat = 2 * (grid + t_out + pe) * W
    dens = 2 * W
    rgb = 2 * (W * W + (W + views) * W + W * 3)
    return deform + feat + dens + rgb


def timed(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--voxels", type=int, default=160)
    args = ap.parse_args()
    from apn_amd.tineuvox import TiNeuVox, poc_fre
    dev = torch.device("cuda")
    torch.manual_seed(0)
    nv = args.voxels ** 3
    m = TiNeuVox(xyz_min=[-1.0, -1.0, -1.0], xyz_max=[1.0, 1.0, 1.0], num_voxels=nv, num_voxels_base=nv,
                 voxel_dim=12, defor_depth=3, net_width=128, alpha_init=1e-3, fast_color_thres=1e-4,
                 no_view_dir=False).to(dev)
    with torch.no_grad():
        m.feature.normal_(0.0, 0.5)
    X, Y, Z = (int(v) for v in m.feature.shape[2:])
    with torch.no_grad():
        grid_pts = m.get_grid_xyz(1).reshape(-1, 3).to(dev).float().contiguous()
        n = grid_pts.shape[0]
        rand_pts = (torch.rand(n, 3, device=dev) * 2 - 1).contiguous()
        _, packed = m._packed()
        grid_bytes = packed.numel() * packed.element_size()
        tproj = m._tproj(torch.tensor([0.3], device=dev))
        vemb = poc_fre(torch.tensor([[0.0, 0.0, 1.0]], device=dev), m.view_poc).reshape(-1)
        zeros = torch.zeros(n, dtype=torch.int32, device=dev)
        res = {}
        for name, pts in (("export_grid", grid_pts), ("random", rand_pts)):
            t_lookup = timed(lambda: m.mult_dist_interp(pts), args.reps)
            t_field = timed(lambda: m._field(pts, zeros, zeros, tproj, vemb=vemb), args.reps)
            uniq = grid_bytes + n * (12 + 144)
            res[name] = {
                "points": n, "lookup_ms": t_lookup, "field_ms": t_field,
                "lookup_hbm_unique_GBs": uniq / (t_lookup * 1e-3) / 1e9,
                "lookup_hbm_frac": uniq / (t_lookup * 1e-3) / 1e9 / HBM_PEAK_GBS,
                "lookup_corner_gather_GBs": n * 3 * 8 * 48 / (t_lookup * 1e-3) / 1e9,
                "field_falg_tflops": n * field_flop_per_sample() / (t_field * 1e-3) / 1e12,
                "field_falg_frac_fp32_mfma": n * field_flop_per_sample() / (t_field * 1e-3) / 1e12 / FP32_MFMA_PEAK_TFLOPS,
                "field_points_per_s": n / (t_field * 1e-3),
            }
    line = {"workload": f"TiNeuVox stage-1 field, 12 x {X}x{Y}x{Z} grid (packed 3-scale {grid_bytes / 1e6:.0f} MB)",
            "lookup_bytes_model": "unique: packed 3-scale grid once + 12 B in + 144 B out per point; gather: 3 scales x 8 corners x 48 B",
            "field_flop_per_sample": field_flop_per_sample(), "peaks": {"hbm_GBs": HBM_PEAK_GBS,
                                                                       "fp32_mfma_tflops": FP32_MFMA_PEAK_TFLOPS},
            **res}
    print(json.dumps(line))


if __name__ == "__main__":
    main()
