"""Determinism probe 2: one process renders the spawn test's sequence for BOTH ranks of a
2-way ray split (ray_shard=(k, 2) frames on the sync-free capacity path, a forced overflow) and
the full frame, and compares every shard tile with the same rays of the full frame. Prints the
differing rays per frame. Diagnostic tool (not a test)."""
from __future__ import annotations

import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "articulated-point-nerf_amd"))
from apn_amd import harness, synthetic as S  # noqa: E402
from apn_amd.shard import pack_tile  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    torch.set_grad_enabled(False)
    dev = torch.device("cuda", 0)
    scene = S.make_scene(S.SceneConfig("probe2 200x200 50k pts 24 bones", 50_000, 24, 200, 200))
    models = [harness.build_model(scene, dev) for _ in range(2)]   # one model per emulated rank
    rk = scene.render_kwargs(dev)
    R = rk["rays_o"].shape[0]
    ts = [torch.tensor([scene.cfg.t], device=dev), torch.tensor([scene.cfg.t + 0.1], device=dev)]
    kw = dict(poses=scene.c2w[None].to(dev), Ks=scene.K[None].to(dev), get_skeleton=True, render_depth=True,
              render_weights=True)
    single = [pack_tile(models[0](t, render_kwargs=rk, **kw), R, dev).clone() for t in ts]
    total = 0
    for it in range(reps):
        for fi, t in enumerate(ts):
            for k, m in enumerate(models):
                out = m(t, render_kwargs=rk, ray_shard=(k, 2), **kw)
                r0, r1 = m.last_ray_range
                tile = pack_tile(out, r1 - r0, dev)   # validated read (re-renders on overflow)
                if getattr(out, "_n_rays", r1 - r0) != r1 - r0 or tile.shape[0] != r1 - r0:
                    tile = pack_tile(out, R, dev)[r0:r1]
                ref = single[fi][r0:r1]
                nb = int((tile != ref).any(1).sum()) if tile.shape == ref.shape else -1
                total += max(nb, 0)
                if nb:
                    print(f"iter {it} frame {fi} shard {k}: {nb} rays differ (range {r0}-{r1})", flush=True)
        full = pack_tile(models[1](ts[it % 2], render_kwargs=rk, **kw), R, dev)
        nb = int((full != single[it % 2]).any(1).sum())
        total += nb
        if nb:
            print(f"iter {it}: full frame on model 1: {nb} rays differ", flush=True)
    torch.cuda.synchronize()
    print("TOTAL differing", total)


if __name__ == "__main__":
    main()
