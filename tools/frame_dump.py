"""Render one frame of a BASELINE config and save its per-ray tile (and the MLP rows) to a file:
A/B builds or environment settings that must not change results are compared with
tools/frame_compare.py. Usage: python tools/frame_dump.py <out.pt> [config]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "articulated-point-nerf_amd"))
from apn_amd import harness, synthetic as S  # noqa: E402
from apn_amd.shard import pack_tile  # noqa: E402


def main():
    cfg = sys.argv[2] if len(sys.argv) > 2 else "C2"
    dev = torch.device("cuda", 0)
    scene = S.make_scene(cfg)
    model = harness.build_model(scene, dev)
    rk = scene.render_kwargs(dev)
    t = torch.tensor([scene.cfg.t], device=dev)
    with torch.no_grad():
        out = model(t, render_depth=True, render_kwargs=rk, render_weights=True)
        tile = pack_tile(out, rk["rays_o"].shape[0], dev).cpu()
    ns = int(model.last_stats["kept_samples"])
    torch.save({"tile": tile, "out12": model._ws.bufs["out12"][:12 * ns].cpu(), "kept": ns}, sys.argv[1])
    print(f"{cfg}: kept {ns}, saved {sys.argv[1]}")


if __name__ == "__main__":
    main()
