"""C5 repose step A/B on one box: the copy-input graph step vs the sweep-index graph step,
HIP-event timed over N poses of the sweep each. Diagnostic tool."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "articulated-point-nerf_amd"))
from apn_amd import harness, synthetic as S  # noqa: E402

torch.set_grad_enabled(False)
dev = torch.device("cuda", 0)
scene = S.make_scene("C5")
model = harness.build_model(scene, dev)
poses = S.repose_sweep(scene.cfg.J).to(dev).contiguous()
n = 300
for name, step in (("copy", model.capture_repose(rot_dim=4)), ("sweep", model.capture_repose(sweep=poses)),
                   ("copy", model.capture_repose(rot_dim=4)), ("sweep", model.capture_repose(sweep=poses))):
    for i in range(5):
        step(poses[i])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        step(poses[i % len(poses)])
    torch.cuda.synchronize()
    print(f"{name}: {1e3 * (time.perf_counter() - t0) / n:.4f} ms/pose")
