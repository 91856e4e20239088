"""Determinism probe: in one process, alternate small frames (a ray subset: the small-batch kNN
path) with full frames (mode 9 with the second grid), and compare every full frame with the first
bit for bit. Prints the number of differing rays per repeat. Diagnostic tool (not a test)."""
from __future__ import annotations

import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "articulated-point-nerf_amd"))
from apn_amd import harness, synthetic as S  # noqa: E402
from apn_amd.shard import pack_tile  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    torch.set_grad_enabled(False)
    dev = torch.device("cuda", 0)
    scene = S.make_scene(S.SceneConfig("probe 200x200 50k pts 24 bones", 50_000, 24, 200, 200))
    model = harness.build_model(scene, dev)
    rk = scene.render_kwargs(dev)
    R = rk["rays_o"].shape[0]
    t = torch.tensor([scene.cfg.t], device=dev)
    kw = dict(poses=scene.c2w[None].to(dev), Ks=scene.K[None].to(dev), get_skeleton=True, render_depth=True,
              render_weights=True)
    sub = dict(rk)
    for k in ("rays_o", "rays_d", "viewdirs"):
        sub[k] = rk[k][: R // 3].contiguous()
    ref = None
    bad_total = 0
    for i in range(reps):
        model(t, render_kwargs=sub, **kw).keys()
        out = model(t, render_kwargs=rk, **kw)
        tile = pack_tile(out, R, dev)
        torch.cuda.synchronize()
        st = model.last_stats.resolved()
        if ref is None:
            ref = tile.clone()
            print("full frame stats", st, flush=True)
            continue
        nb = int((tile != ref).any(1).sum())
        bad_total += nb
        print(f"rep {i}: {nb} rays differ (survivors {st.get('kept_samples')})", flush=True)
    print("TOTAL differing", bad_total)


if __name__ == "__main__":
    main()
