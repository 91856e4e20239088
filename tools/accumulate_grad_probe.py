"""Where the training step meets autograd's "AccumulateGrad node's stream does not match" warning
(VERDICT r5 item 5): every occurrence is recorded with the Python stack that triggered it while a
C1 model runs, in order, (1) eager no-grad frames, (2) train steps with the captured warp stage
(train.warp_stage: torch.cuda.make_graphed_callables), (3) a forced re-capture (mask change),
(4) eager-warp steps, (5) graphed steps again, (6) tools/graph_capture_probe-style raw captures.

    python tools/accumulate_grad_probe.py [--config C1]
"""
import argparse
import os
import sys
import traceback
import warnings

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "articulated-point-nerf_amd")]
import torch  # noqa: E402

from apn_amd import harness, synthetic as S, train as T  # noqa: E402

HITS = []
PHASE = ["start"]


def _show(message, category, filename, lineno, file=None, line=None):
    if "AccumulateGrad" in str(message):
        stack = "".join(traceback.format_stack(limit=14)[:-2])
        HITS.append((PHASE[0], stack))
        print(f"[WARN in phase {PHASE[0]}]\n{stack}", flush=True)
    else:
        print(f"[other warning] {category.__name__}: {str(message)[:120]}", flush=True)


def step(model, t, sub, target):
    model.zero_grad(set_to_none=True)
    out = model(t, render_kwargs=sub)
    loss = torch.nn.functional.mse_loss(out["rgb_marched"], target)
    loss = loss + 0.1 * model.get_transformation_regularisation_loss()
    loss = loss + 10.0 * model.get_neighbour_weight_tv_loss() + 0.2 * model.get_weight_sparsity_loss()
    loss.backward()
    v = float(loss.detach())
    del out, loss
    return v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C1")
    args = ap.parse_args()
    warnings.simplefilter("always")
    warnings.showwarning = _show
    dev = torch.device("cuda")
    scene = S.make_scene(args.config)
    model = harness.build_model(scene, dev)
    rk = scene.render_kwargs(dev)
    g = torch.Generator(device=dev).manual_seed(0)
    sel = torch.randint(0, len(rk["rays_o"]), (4096,), device=dev, generator=g)
    sub = dict(rk)
    for k in ("rays_o", "rays_d", "viewdirs"):
        sub[k] = rk[k][sel]
    t = torch.tensor([scene.cfg.t], device=dev)
    PHASE[0] = "no-grad frames"
    with torch.no_grad():
        target = model(t + 0.1, render_kwargs=sub)["rgb_marched"].clone()
        model(t, render_kwargs=rk)
    PHASE[0] = "grad-enabled get_weights / pose_torch (eager, default stream)"
    w = model.get_weights()
    model.forward_warp.pose_torch(model.joints, T.poc_fre(t, model.time_poc), None)
    del w
    for i in range(3):
        PHASE[0] = f"graphed step {i}"
        print(PHASE[0], step(model, t, sub, target), flush=True)
    PHASE[0] = "forced re-capture (rot mask changed)"
    with torch.no_grad():
        model.forward_warp.rot_mask.copy_(model.forward_warp.rot_mask.clone())
    print(PHASE[0], step(model, t, sub, target), flush=True)
    for i in range(2):
        PHASE[0] = f"eager-warp step {i}"
        T.GRAPH_WARP = False
        try:
            print(PHASE[0], step(model, t, sub, target), flush=True)
        finally:
            T.GRAPH_WARP = True
    for i in range(2):
        PHASE[0] = f"graphed step after eager {i}"
        print(PHASE[0], step(model, t, sub, target), flush=True)
    torch.cuda.synchronize()
    print(f"RESULT: {len(HITS)} AccumulateGrad stream-mismatch warnings; phases: {sorted({p for p, _ in HITS})}",
          flush=True)


if __name__ == "__main__":
    main()
