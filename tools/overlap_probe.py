"""Probe: can the kNN of one ray chunk overlap the neighbour MLP of another on the same GPU?

Renders one C2 frame, then re-runs the frame's kNN (into scratch outputs) and MLP from the
frame's own buffers: sequentially on one stream, and concurrently on two streams, with the MLP
grid limited to G workgroups (2 per CU leaves VGPRs for the kNN waves). Prints the times.
Usage: python tools/overlap_probe.py [G ...]
"""
import ctypes as C
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "articulated-point-nerf_amd"))
from apn_amd import harness, synthetic as S, _lib as L  # noqa: E402
from apn_amd.temporalpoints import CELL_CAP  # noqa: E402


def main():
    torch.set_grad_enabled(False)   # the render path (with grad, forward() takes the training path)
    dev = torch.device("cuda", 0)
    scene = S.make_scene("C2")
    model = harness.build_model(scene, dev)
    rk = scene.render_kwargs(dev)
    t = torch.tensor([scene.cfg.t], device=dev)
    for _ in range(2):
        model(t, render_depth=True, render_kwargs=rk, render_weights=True)
    torch.cuda.synchronize()
    ws = model._ws.bufs
    lib = L.load()
    st = model.last_stats.resolved()
    n_bbox, S_kept = st["inbbox_samples"], st["kept_samples"]
    N = model.canonical_feat.shape[0]
    R = rk["rays_o"].shape[0]
    nsurv = model.last_stats._nsurv
    offs = ws["offs"]
    wbuf, proj = model._packed_weights(None, dev)
    # scratch kNN outputs (the MLP keeps reading the frame's own s_pos/s_ray/s_nbr)
    s_pos2 = torch.empty(n_bbox * 4, device=dev)
    s_ray2 = torch.empty(n_bbox, dtype=torch.int32, device=dev)
    s_nbr2 = torch.empty(n_bbox * 8, dtype=torch.int32, device=dev)
    ns2 = torch.empty(1, dtype=torch.int32, device=dev)
    kws = torch.empty(int(lib.apn_knn_workspace_bytes(n_bbox)), dtype=torch.uint8, device=dev)
    vd = rk["viewdirs"].float().contiguous()
    P = L.ptr

    def knn(stream):
        L.call("apn_knn_radius", P(ws["q_pos"]), P(ws["q_ray"]), n_bbox, C.c_void_p(offs.data_ptr() + 4 * R),
               P(ws["grid_ws"]), N, CELL_CAP, P(ws["sorted4"]), 0.01, P(s_pos2), P(s_ray2), P(s_nbr2), P(ns2),
               P(kws), C.c_void_p(stream.cuda_stream))

    def mlp(stream, G):
        L.call("apn_point_mlp", P(ws["s_pos"]), P(ws["s_ray"]), P(ws["s_nbr"]), n_bbox, P(nsurv), P(ws["recA"]),
               P(ws["recB"]), P(proj), 128, P(vd), None, P(wbuf), model._eps, float(model.tineuvox.act_shift),
               float(rk["stepsize"]) * float(model.tineuvox.voxel_size_ratio), G, P(ws["out12"]),
               C.c_void_p(stream.cuda_stream))

    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    print(f"n_bbox {n_bbox} kept {S_kept}")

    def timed(fn, reps=5):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    cur = torch.cuda.current_stream(dev)
    print(f"knn alone {timed(lambda: knn(cur)):.3f} ms")
    for G in [int(x) for x in sys.argv[1:]] or [0, 512, 768]:
        t_mlp = timed(lambda: mlp(cur, G))

        def both():
            ev = torch.cuda.Event()
            ev.record(cur)
            s1.wait_event(ev)
            s2.wait_event(ev)
            mlp(s1, G)
            knn(s2)
            e1, e2 = torch.cuda.Event(), torch.cuda.Event()
            e1.record(s1)
            e2.record(s2)
            cur.wait_event(e1)
            cur.wait_event(e2)

        def seq():
            mlp(cur, G)
            knn(cur)
        print(f"G={G}: mlp alone {t_mlp:.3f} ms, sequential mlp+knn {timed(seq):.3f} ms, "
              f"concurrent {timed(both):.3f} ms")


if __name__ == "__main__":
    main()
