"""Parity at the BASELINE frame sizes -- C2 (the headline: 800x800 rays, 300k points, 24 bones),
C3 (500k points, 32 bones) and C4 (ZJU inverse-y camera, 1024x1024, pose embedding: the largest
launch, ~20M in-bbox samples) -- over the WHOLE frame rather than a band:

* in-bbox sampling, bit-exact: the GPU's in-bbox samples (apn_inbbox_*: positions, ray ids, step
  ids, in (ray, step) order) against the oracle's sample_pts_on_rays restatement
  (render_utils_kernel.cu:138-236) on the same rays and the GPU's sampling bbox;
* radius kNN, bit-exact: every kNN survivor of the frame -- its ray id, step id and 8 neighbour
  indices in (distance, index) order -- against the oracle's exact search (float64 cKDTree
  candidates re-ranked in float32, every full window certified or re-searched over its whole
  ball: oracle.apn_oracle.knn_radius_certified) over all in-bbox samples on the GPU's warped cloud
  (temporalpoints.py:433-447). The frame runs the shipped library's mode 9 (fine-grid pass A,
  anisotropic-grid pass B, cost-ranked lanes);
* ray shards of that frame (the "blocks" split at 4 and 8 ranks): every survivor of a shard
  equals the full frame's survivor of the same ray and step;
* end to end at C2, C3 and C4: EVERY ray of the frame -- all six
  output keys -- against the oracle's forward (temporalpoints.py:540-712) on the GPU's warped cloud
  and rays, within 1e-5 unless the ray's oracle compositing sits on a discontinuity
  (oracle/flips.py, the rule of the band tests in test_hip_parity.py). C4 is the only config with
  the ZJU inverse-y camera (tineuvox.py:675-703) and the pose embedding (temporalpoints.py:571-576),
  and the largest launch (~5.6 M kept samples)."""
import time

import numpy as np
import pytest
import torch

from oracle import apn_oracle as O

pytestmark = pytest.mark.gpu

F32 = np.float32
KEYS = ["rgb_marched", "rgb_marched_direct", "weights", "alphainv_last", "alphainv_last_direct", "depth"]


@pytest.fixture(scope="module", params=["C2", "C3", "C4"])
def frame(request):
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from apn_amd import harness, synthetic as S
    config = request.param
    dev = torch.device("cuda")
    scene = S.make_scene(config)
    model = harness.build_model(scene, dev)
    rk = scene.render_kwargs(dev)
    t = torch.tensor([scene.cfg.t], device=dev)
    model._force_exact = True    # exact in-bbox count: every buffer holds exactly the frame's samples
    try:
        with torch.no_grad():
            out = model(t, render_depth=True, render_kwargs=rk, render_weights=True)
        torch.cuda.synchronize()
    finally:
        model._force_exact = False
    st = model.last_stats.resolved()
    from apn_amd.ops import mlp_range_fallback
    assert not mlp_range_fallback(model._ws.bufs["mlp_w"])   # no FP32 re-run: the split kernel's own frame
    nq, ns = st["inbbox_samples"], st["kept_samples"]
    ws = model._ws.bufs
    fr = {
        "config": config, "scene": scene, "rk": {k: (v.cpu() if torch.is_tensor(v) else v) for k, v in rk.items()},
        "xyz": out["t_hat_pcd"].detach().cpu().numpy().astype(F32),
        "bbox6": ws["bbox6"][:6].cpu().numpy(),
        "q_pos": ws["q_pos"][:4 * nq].view(nq, 4).cpu().numpy(),
        "q_ray": ws["q_ray"][:nq].cpu().numpy(),
        "s_pos": ws["s_pos"][:4 * ns].view(ns, 4).cpu().numpy(),
        "s_ray": ws["s_ray"][:ns].cpu().numpy(),
        "s_nbr": ws["s_nbr"][:8 * ns].view(ns, 8).cpu().numpy(),
        "out": {k: out[k].detach().cpu().numpy() for k in KEYS},
        "nq": nq, "ns": ns, "model": model, "t": t, "rk_dev": rk,
    }
    return fr


def test_full_frame_inbbox_samples_bit_exact(frame):
    from apn_amd import synthetic as S
    fr = frame
    rk = fr["rk"]
    lo, hi = fr["bbox6"][:3], fr["bbox6"][3:]
    ro, rd = rk["rays_o"].numpy(), rk["rays_d"].numpy()
    R = len(ro)
    pts_l, rid_l, sid_l = [], [], []
    for s in range(0, R, 1 << 17):   # ray chunks (samples of a ray depend on that ray and the bbox only)
        pts, mo, rid, sid, *_ = O.sample_pts_on_rays(ro[s:s + (1 << 17)], rd[s:s + (1 << 17)], lo, hi, rk["near"],
                                                     rk["far"], float(rk["stepsize"]) * S.VOXEL_SIZE)
        keep = ~mo
        pts_l.append(pts[keep]); rid_l.append(rid[keep] + s); sid_l.append(sid[keep])
    pts, rid, sid = np.concatenate(pts_l), np.concatenate(rid_l), np.concatenate(sid_l)
    print(f"{fr['config']}: {R} rays, {len(pts)} in-bbox samples")
    assert fr["nq"] == len(pts) > 1_000_000
    q = fr["q_pos"]
    assert np.array_equal(q[:, :3], pts)
    assert np.array_equal(fr["q_ray"], rid.astype(np.int32))
    assert np.array_equal(q[:, 3].view(np.int32), sid.astype(np.int32))


def test_full_frame_knn_survivors_bit_exact(frame):
    fr = frame
    q = fr["q_pos"]
    t0 = time.perf_counter()
    keep, idx, stats = O.knn_radius_certified(q[:, :3], fr["xyz"], K=8, r2=0.01)
    print(f"{fr['config']} full-frame kNN: {stats} ({time.perf_counter() - t0:.1f} s)")
    assert stats["queries"] == fr["nq"]
    assert fr["ns"] == int(keep.sum()) > 500_000
    # survivors in query order: ray id, step id (bits of w), position and the 8 neighbours
    assert np.array_equal(fr["s_ray"], fr["q_ray"][keep])
    assert np.array_equal(fr["s_pos"], q[keep])
    assert np.array_equal(fr["s_nbr"], idx[keep].astype(np.int32))


@pytest.mark.parametrize("world", [4, 8])
def test_ray_block_shard_knn_matches_full_frame(frame, world):
    from apn_amd.shard import RAY_BLOCK
    fr = frame
    m = fr["model"]
    m._force_exact = True
    try:
        with torch.no_grad():
            m(fr["t"], render_depth=True, render_kwargs=fr["rk_dev"], render_weights=True,
              ray_shard=(world - 1, world, RAY_BLOCK))
        torch.cuda.synchronize()
    finally:
        m._force_exact = False
    st = m.last_stats.resolved()
    nq, ns = st["inbbox_samples"], st["kept_samples"]
    if fr["config"] == "C2":   # above the small-batch pass B, below the one-lane cell bounds
        assert (1 << 18) < nq <= (3 << 20)
    ws = m._ws.bufs
    rays = m.last_ray_index.cpu().numpy()      # global ray of each local ray (ascending)
    s_ray = rays[ws["s_ray"][:ns].cpu().numpy()]
    s_pos = ws["s_pos"][:4 * ns].view(ns, 4).cpu().numpy()
    s_nbr = ws["s_nbr"][:8 * ns].view(ns, 8).cpu().numpy()
    sel = np.isin(fr["s_ray"], rays)
    assert ns == int(sel.sum()) > 100_000
    assert np.array_equal(s_ray, fr["s_ray"][sel])
    assert np.array_equal(s_pos, fr["s_pos"][sel])
    assert np.array_equal(s_nbr, fr["s_nbr"][sel])


def test_every_ray_vs_oracle(frame):
    """The whole frame end to end: the oracle's forward over all of its rays (640k at C2 / C3, 1M at
    C4; in chunks of 50 image rows: chunk invariance is the reference's own, and the bbox comes
    from the whole warped cloud)
    against the GPU frame, all six output keys, every ray within 1e-5 unless explained by a
    discontinuity of the reference's compositing (oracle/flips.py)."""
    from apn_amd import synthetic as S
    from oracle.flips import assert_flips_explained
    fr = frame
    model, scene, rk = fr["model"], fr["scene"], fr["rk"]
    st = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    orc = O.OracleModel(st, model.canonical_pcd.cpu(), model.bones, stepsize=S.STEPSIZE, voxel_size=S.VOXEL_SIZE,
                        fast_color_thres=S.FAST_COLOR_THRES, pose_embedding_dim=model.pose_embedding_dim,
                        act_shift=float(model.tineuvox.act_shift),
                        voxel_size_ratio=float(model.tineuvox.voxel_size_ratio),
                        mean_min_distance_value=float(model.mean_min_distance))
    H, W = scene.cfg.H, scene.cfg.W
    R = H * W
    rows = 50
    xyz = torch.from_numpy(fr["xyz"])
    n_bad = {k: 0 for k in KEYS}
    worst = {k: 0.0 for k in KEYS}
    t0 = time.perf_counter()
    kept = 0
    for r0 in range(0, H, rows):
        sel = slice(r0 * W, min(H, r0 + rows) * W)
        sub = dict(rk)
        for k in ("rays_o", "rays_d", "viewdirs"):
            sub[k] = rk[k][sel].contiguous()
        ref = orc.forward(torch.tensor([scene.cfg.t]), render_depth=True, render_kwargs=sub, render_weights=True,
                          t_hat_override=xyz, knn_tree=True, perm=model.last_palette_perm)
        if "alpha" not in orc.trace:
            # no kNN survivor in these rows (the oracle's NoPointsException dict, an artefact of the
            # chunking: the whole frame has survivors, so the GPU composited empty rays): background
            # colour, depth 0, transmittance 1 on every ray of the chunk
            bg = np.float32(rk["bg"])
            for key in ("rgb_marched", "rgb_marched_direct", "weights"):
                assert (fr["out"][key][sel] == bg).all(), key
            assert (fr["out"]["depth"][sel] == 0).all()
            for key in ("alphainv_last", "alphainv_last_direct"):
                assert (fr["out"][key][sel] == 1).all(), key
            continue
        kept += len(orc.trace["ray_id"])
        for key in KEYS:
            nb, w = assert_flips_explained(key, fr["out"][key][sel], ref[key].numpy(), orc.trace)
            n_bad[key] += nb
            worst[key] = max(worst[key], w)
    print(f"{fr['config']} every ray: {R} rays, {kept} kept samples, oracle {time.perf_counter() - t0:.1f} s; rays over 1e-5 "
          f"(all explained) {n_bad}; max error on rays off any discontinuity {worst}")
    assert kept == fr["ns"]
