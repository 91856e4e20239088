"""Debug aid: per-sample comparison GPU vs oracle for the worst rays of a full-size band
(the test_full_size_band_vs_oracle setup). Usage: python tools/debug_band.py C3 [key]"""
import sys, os
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "articulated-point-nerf_amd"), os.path.join(ROOT, "tests")]
from apn_amd import harness, synthetic as S
from oracle import apn_oracle as O
from oracle.flips import ray_errors, near_discontinuity, PATH_OF_KEY

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
key = sys.argv[2] if len(sys.argv) > 2 else "rgb_marched_direct"
dev = torch.device("cuda")
scene = S.make_scene(cfg)
model = harness.build_model(scene, dev)
rk = scene.render_kwargs(dev)
t = torch.tensor([scene.cfg.t], device=dev)
with torch.no_grad():
    out = model(t, render_depth=True, render_kwargs=rk, render_weights=True)
torch.cuda.synchronize()
H, W = scene.cfg.H, scene.cfg.W
sel = torch.cat([torch.arange(r * W, (r + 1) * W) for r in (H // 2 - 40, H // 2 + 40)])
st = {k: v.detach().cpu() for k, v in model.state_dict().items()}
orc = O.OracleModel(st, model.canonical_pcd.cpu(), model.bones, stepsize=S.STEPSIZE, voxel_size=S.VOXEL_SIZE,
                    fast_color_thres=S.FAST_COLOR_THRES, pose_embedding_dim=model.pose_embedding_dim,
                    act_shift=float(model.tineuvox.act_shift), voxel_size_ratio=float(model.tineuvox.voxel_size_ratio),
                    mean_min_distance_value=float(model.mean_min_distance))
sub = dict(rk)
for k in ("rays_o", "rays_d", "viewdirs"):
    sub[k] = rk[k][sel].cpu().contiguous()
ref = orc.forward(torch.tensor([scene.cfg.t]), render_depth=True, render_kwargs=sub, render_weights=True,
                  t_hat_override=out["t_hat_pcd"].cpu(), knn_tree=True, perm=model.last_palette_perm)
a = out[key].cpu()[sel].numpy(); b = ref[key].numpy()
err = ray_errors(a, b)
near = near_discontinuity(orc.trace, len(b), PATH_OF_KEY[key])
worst = np.argsort(-err)[:5]
ns = int(model.last_stats["kept_samples"])
ws = model._ws.bufs
s_ray = ws["s_ray"][:ns].cpu().numpy()
o12 = ws["out12"][:ns * 12].reshape(ns, 12).cpu().numpy()
s_nbr = ws["s_nbr"][:ns * 8].reshape(ns, 8).cpu().numpy()
tr = orc.trace
np.set_printoptions(precision=9, suppress=False, linewidth=200)
for r in worst:
    g = int(sel[r])
    print(f"band ray {r} (global {g}): err {err[r]:.3e} near={near[r]} gpu {a[r]} oracle {b[r]}")
    oi = np.nonzero(tr["ray_id"] == r)[0]
    gi = np.nonzero(s_ray == g)[0]
    print(f"  oracle samples {len(oi)}, gpu samples {len(gi)}")
    print("  oracle alpha_d", tr["alpha_direct"].numpy()[oi])
    print("  gpu    alpha_d", o12[gi, 7])
    print("  oracle alpha  ", tr["alpha"].numpy()[oi])
    print("  gpu    alpha  ", o12[gi, 3])
    print("  oracle rgb_d  ", tr["rgbs_direct"].numpy()[oi])
    print("  gpu    rgb_d  ", o12[gi, 4:7])
    print("  nbr equal", np.array_equal(np.sort(tr["s_i"][oi], 1), np.sort(s_nbr[gi], 1)) if len(oi) == len(gi) else "n/a")

# exact brute force for the samples whose neighbour lists differ
t_hat = out["t_hat_pcd"].cpu().numpy()
s_pos = ws["s_pos"][:ns * 4].reshape(ns, 4).cpu().numpy()
for r in worst[:2]:
    g = int(sel[r])
    oi = np.nonzero(tr["ray_id"] == r)[0]
    gi = np.nonzero(s_ray == g)[0]
    for a_, b_ in zip(oi, gi):
        on, gn = np.sort(tr["s_i"][a_]), np.sort(s_nbr[b_])
        if not np.array_equal(on, gn):
            q = s_pos[b_, :3].astype(np.float32)
            d = ((q[0] - t_hat[:, 0]) * (q[0] - t_hat[:, 0]) + (q[1] - t_hat[:, 1]) * (q[1] - t_hat[:, 1])) \
                + (q[2] - t_hat[:, 2]) * (q[2] - t_hat[:, 2])
            order = np.lexsort((np.arange(len(d)), d))[:12]
            print(f"ray {r} sample: q {q} oracle-pts {tr['pts'][a_]}")
            print("  oracle nbr", tr["s_i"][a_], "\n  gpu nbr   ", s_nbr[b_])
            print("  brute top12", order, d[order])
