"""The training step's Linear layers on the hand-written fp32 GEMM (apn_gemm.hip): forward with the
bias and the LeakyReLU / ReLU fused into the product's epilogue, backward as two more products --
dX = (dY * act'(Y)) W and [dW | db] = (dY * act'(Y))^T [X | 1] (split over the rows, summed in a
fixed order) -- with the activation derivative applied while the gradient is loaded.

The reference trains these layers through torch.nn.Linear under autograd (temporalpoints.py:491
feat_net, 496-515 densitynet / rgbnet, 380-381 pose_embedding_net, pointwarper.py:5-37
TransformNet; run.py:574-716); ``sequential(net, x)`` runs such a Sequential with the same
parameters and the same per-element arithmetic (f32 products and sums, in the kernel's order).
CUDA tensors only: on CPU tensors (the oracle and the host tests) the modules run as torch does.
"""
from __future__ import annotations

import torch

from ._lib import call, load, ptr, stream_ptr

SPLIT_ROWS = 512     # rows per split of the weight-gradient product (at least)
SPLIT_TILES = 1024   # aim: output tiles x splits of about this many workgroups


class _GemmLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, slope):
        if x.dtype != torch.float32 or weight.dtype != torch.float32:
            raise TypeError("apn linear: float32 only")
        dev = x.device
        x2 = x.reshape(-1, x.shape[-1]).contiguous()
        w = weight.contiguous()
        M, K = x2.shape
        N = w.shape[0]
        if w.shape[1] != K:
            raise ValueError(f"apn linear: input width {K} vs weight {tuple(w.shape)}")
        b = bias.contiguous() if bias is not None else None
        y = torch.empty(M, N, device=dev, dtype=torch.float32)
        act = slope is not None
        call("apn_gemm_f32", ptr(x2), None, ptr(w), ptr(y), ptr(b), M, N, K, K, K, N, 0, 1, 0.0, int(act),
             float(slope) if act else 0.0, stream_ptr(dev))
        ctx.save_for_backward(x2, w, y if act else None)
        ctx.slope, ctx.has_bias, ctx.in_shape = slope, bias is not None, x.shape
        return y.reshape(*x.shape[:-1], N)

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dy):
        x, w, y = ctx.saved_tensors
        dev = x.device
        M, K = x.shape
        N = w.shape[0]
        dy = dy.reshape(M, N).contiguous()
        sm = float(ctx.slope) if ctx.slope is not None else 1.0
        s = stream_ptr(dev)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(M, K, device=dev, dtype=torch.float32)
            call("apn_gemm_f32", ptr(dy), ptr(y), ptr(w), ptr(dx), None, M, K, N, N, K, K, 0, 0, sm, 0, 0.0, s)
            dx = dx.reshape(ctx.in_shape)
        want_b = ctx.has_bias and ctx.needs_input_grad[2]
        if ctx.needs_input_grad[1] or want_b:
            dw = torch.empty(N, K, device=dev, dtype=torch.float32)
            db = torch.empty(N, device=dev, dtype=torch.float32) if want_b else None
            tiles = -(-N // 64) * -(-(K + 1) // 64)
            splits = max(1, min(M // SPLIT_ROWS, SPLIT_TILES // tiles))
            ws = torch.empty(int(load().apn_gemm_f32_splitk_workspace_bytes(N, K, splits)) // 4 + 1,
                             device=dev, dtype=torch.float32)
            call("apn_gemm_f32_splitk", ptr(dy), ptr(y), ptr(x), ptr(dw), ptr(db), N, K, M, N, K, 1, 0, sm, splits,
                 ptr(ws), s)
        return dx, (dw if ctx.needs_input_grad[1] else None), db, None


def linear(x: torch.Tensor, layer: torch.nn.Linear, slope=None) -> torch.Tensor:
    """act(x W^T + b) for a torch.nn.Linear ``layer``; ``slope``: None (no activation), 0 (ReLU)
    or the LeakyReLU negative slope. CPU tensors: torch's own ops."""
    if not x.is_cuda:
        y = torch.nn.functional.linear(x, layer.weight, layer.bias)
        if slope is None:
            return y
        return torch.relu(y) if slope == 0 else torch.nn.functional.leaky_relu(y, slope)
    return _GemmLinear.apply(x, layer.weight, layer.bias, slope)


def _flatten(net):
    for m in net:
        if isinstance(m, torch.nn.Sequential):
            yield from _flatten(m)
        else:
            yield m


def sequential(net: torch.nn.Module, x: torch.Tensor) -> torch.Tensor:
    """A Sequential of Linear / LeakyReLU / ReLU (nested Sequentials flattened): each Linear runs
    with the activation that follows it fused into its epilogue."""
    mods = list(_flatten(net))
    i = 0
    while i < len(mods):
        m = mods[i]
        if isinstance(m, torch.nn.Linear):
            nxt = mods[i + 1] if i + 1 < len(mods) else None
            if isinstance(nxt, torch.nn.LeakyReLU):
                x = linear(x, m, float(nxt.negative_slope))
                i += 2
                continue
            if isinstance(nxt, torch.nn.ReLU):
                x = linear(x, m, 0.0)
                i += 2
                continue
            x = linear(x, m)
        else:
            x = m(x)
        i += 1
    return x
