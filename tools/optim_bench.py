"""HBM roofline of the optimizer-side kernels on one GPU.

adam_upd moves 28 B per element (reads param, grad, exp_avg, exp_avg_sq; writes param, exp_avg,
exp_avg_sq); total_variation_add_grad (dense) 12 B per element (param read once if the neighbour
reads hit cache, grad read + write). Sizes: the TiNeuVox feature grid of the reference's D-NeRF
config, 12 x 160^3 (49 M elements). Prints one JSON line per kernel.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "articulated-point-nerf_amd"))
from apn_amd import optim  # noqa: E402

HBM_PEAK_GBS = 8000.0


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    dev = torch.device("cuda", 0)
    shape = (1, 12, 160, 160, 160)
    n = 12 * 160 ** 3
    g = torch.Generator(device=dev).manual_seed(0)
    p = torch.randn(shape, device=dev, generator=g)
    gr = torch.randn(shape, device=dev, generator=g)
    m = torch.zeros_like(p); v = torch.zeros_like(p)
    step = [0]

    def adam():
        step[0] += 1
        optim.adam_upd(p, gr, m, v, step[0], 0.9, 0.99, 1e-3, 1e-8)
    for name, fn, bpe in (("adam_upd", adam, 28),
                          ("total_variation_add_grad(dense)",
                           lambda: optim.total_variation_add_grad(p, gr, 1e-3, 1e-3, 1e-3, True), 12)):
        ms = timed(fn)
        gbs = n * bpe / (ms * 1e-3) / 1e9
        print(json.dumps({"kernel": name, "elements": n, "bytes_per_element": bpe, "ms": round(ms, 4),
                          "achieved_GBs": round(gbs, 1), "frac_of_hbm_peak": round(gbs / HBM_PEAK_GBS, 3)}))


if __name__ == "__main__":
    main()
