"""Parity at the headline size (BASELINE configs[1], C2: 800x800 rays, 300k points, 24 bones),
stage-wise and bit-exact, over the WHOLE frame rather than a band:

* in-bbox sampling: the GPU's in-bbox samples (apn_inbbox_*: positions, ray ids, step ids, in
  (ray, step) order) against the oracle's sample_pts_on_rays restatement
  (render_utils_kernel.cu:138-236) on the same rays and the GPU's sampling bbox;
* radius kNN: every kNN survivor of the frame -- its ray id, step id and 8 neighbour indices in
  (distance, index) order -- against the oracle's exact search (float64 cKDTree candidates
  re-ranked in float32, every full window certified or re-searched over its whole ball:
  oracle.apn_oracle.knn_radius_certified) over all ~8M in-bbox samples on the GPU's warped cloud
  (temporalpoints.py:433-447). The frame runs the shipped library's mode 9 (fine-grid pass A,
  anisotropic-grid pass B, cost-ranked lanes);
* ray shards of that frame (the "blocks" split at 4 and 8 ranks, ~2M and ~1M in-bbox samples: the
  launch sizes where the kNN orders its workgroups heavy-first and the cell bounds run 16 lanes
  per cell): every survivor of a shard equals the full frame's survivor of the same ray and step."""
import numpy as np
import pytest
import torch

from oracle import apn_oracle as O

pytestmark = pytest.mark.gpu

F32 = np.float32


@pytest.fixture(scope="module")
def c2_frame():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from apn_amd import harness, synthetic as S
    dev = torch.device("cuda")
    scene = S.make_scene("C2")
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
        "scene": scene, "rk": {k: (v.cpu() if torch.is_tensor(v) else v) for k, v in rk.items()},
        "xyz": out["t_hat_pcd"].detach().cpu().numpy().astype(F32),
        "bbox6": ws["bbox6"][:6].cpu().numpy(),
        "q_pos": ws["q_pos"][:4 * nq].view(nq, 4).cpu().numpy(),
        "q_ray": ws["q_ray"][:nq].cpu().numpy(),
        "s_pos": ws["s_pos"][:4 * ns].view(ns, 4).cpu().numpy(),
        "s_ray": ws["s_ray"][:ns].cpu().numpy(),
        "s_nbr": ws["s_nbr"][:8 * ns].view(ns, 8).cpu().numpy(),
        "nq": nq, "ns": ns, "model": model, "t": t, "rk_dev": rk,
    }
    return fr


def test_c2_full_frame_inbbox_samples_bit_exact(c2_frame):
    from apn_amd import synthetic as S
    fr = c2_frame
    rk = fr["rk"]
    lo, hi = fr["bbox6"][:3], fr["bbox6"][3:]
    pts, mo, rid, sid, *_ = O.sample_pts_on_rays(rk["rays_o"].numpy(), rk["rays_d"].numpy(), lo, hi, rk["near"],
                                                 rk["far"], float(rk["stepsize"]) * S.VOXEL_SIZE)
    keep = ~mo
    assert fr["nq"] == int(keep.sum()) > 7_000_000
    q = fr["q_pos"]
    assert np.array_equal(q[:, :3], pts[keep])
    assert np.array_equal(fr["q_ray"], rid[keep].astype(np.int32))
    assert np.array_equal(q[:, 3].view(np.int32), sid[keep].astype(np.int32))


def test_c2_full_frame_knn_survivors_bit_exact(c2_frame):
    fr = c2_frame
    q = fr["q_pos"]
    keep, idx, stats = O.knn_radius_certified(q[:, :3], fr["xyz"], K=8, r2=0.01)
    print(f"C2 full-frame kNN: {stats}")
    assert stats["queries"] == fr["nq"]
    assert fr["ns"] == int(keep.sum()) > 1_500_000
    # survivors in query order: ray id, step id (bits of w), position and the 8 neighbours
    assert np.array_equal(fr["s_ray"], fr["q_ray"][keep])
    assert np.array_equal(fr["s_pos"], q[keep])
    assert np.array_equal(fr["s_nbr"], idx[keep].astype(np.int32))


@pytest.mark.parametrize("world", [4, 8])
def test_c2_ray_block_shard_knn_matches_full_frame(c2_frame, world):
    from apn_amd.shard import RAY_BLOCK
    fr = c2_frame
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
    assert (1 << 18) < nq <= (3 << 20)          # above the small-batch pass B, below the one-lane cell bounds
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
