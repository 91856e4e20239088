"""Which piece of the training warp stage (train._WarpStage) fails under HIP graph capture: each
piece's forward + autograd.grad captured on its own (torch.cuda.graph), progress printed before
each capture. Round 5's version warmed up on one stream and captured on another while the
warm-up's outputs (and with them the parameters' AccumulateGrad nodes of the warm-up stream) were
still alive: the captured backward then had to wait on that stream and the process aborted. The
fixed discipline (here and in train.graph_callable) keeps everything on one stream.

    python tools/graph_capture_probe.py [--config C1] [--only transformnet]
"""
import argparse
import gc
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "articulated-point-nerf_amd")]
import warnings  # noqa: E402

import torch  # noqa: E402

from apn_amd import harness, synthetic as S, train as T, linear as LIN  # noqa: E402
from apn_amd.tineuvox import poc_fre  # noqa: E402


def capture(name, fn, inputs):
    """Eager pass on the current stream, then warm-up and both captures on ONE side stream with
    the earlier passes' autograd graphs dropped first (train.graph_callable's discipline: no
    parameter AccumulateGrad node of another stream is alive when the backward is captured)."""
    print(f"[{name}] eager", flush=True)
    outs = [o for o in fn() if o.requires_grad]
    torch.autograd.grad(outs, inputs, [torch.ones_like(o) for o in outs], allow_unused=True)
    del outs
    gc.collect()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            outs = [o for o in fn() if o.requires_grad]
            torch.autograd.grad(outs, inputs, [torch.ones_like(o) for o in outs], allow_unused=True)
            del outs
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    print(f"[{name}] capture forward", flush=True)
    gf = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gf, stream=s):
        outs = [o for o in fn() if o.requires_grad]
    print(f"[{name}] capture backward", flush=True)
    gb = torch.cuda.CUDAGraph()
    gos = [torch.ones_like(o) for o in outs]
    with torch.cuda.graph(gb, stream=s):
        torch.autograd.grad(outs, inputs, gos, allow_unused=True)
    del outs
    gf.replay(); gb.replay()
    torch.cuda.synchronize()
    print(f"[{name}] ok", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C1")
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    warnings.filterwarnings("error", message="The AccumulateGrad node")
    dev = torch.device("cuda")
    scene = S.make_scene(args.config)
    model = harness.build_model(scene, dev)
    fw = model.forward_warp
    t = torch.tensor([scene.cfg.t], device=dev)
    te = poc_fre(t, model.time_poc)
    tn = list(fw.transform_net.parameters())
    pieces = {
        "transformnet": (lambda: [fw.transform_net(te.unsqueeze(0))], tn),
        "pose_torch": (lambda: list(fw.pose_torch(model.joints, te, None)), tn + [model.joints]),
        "lbs_train": (lambda: list(T.lbs_train(model, *fw.pose_torch(model.joints, te, None)[:2], identity_rules=True)),
                      tn + [model.joints, model.weights, model.theta_weight]),
    }
    for name, (fn, inputs) in pieces.items():
        if args.only and name != args.only:
            continue
        capture(name, fn, inputs)


if __name__ == "__main__":
    main()
