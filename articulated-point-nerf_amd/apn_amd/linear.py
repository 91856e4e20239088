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
SPLIT_TILES = 512    # aim: output tiles x splits of about this many workgroups (more measured slower)


def _padded_rows(w: torch.Tensor) -> torch.Tensor:
    """W [N, K] as a view of rows padded to a multiple of 4 floats (a copy only when K % 4 != 0):
    16-B aligned rows take the product's vector loads."""
    N, K = w.shape
    if K % 4 == 0:
        return w.contiguous()
    buf = torch.zeros(N, -(-K // 4) * 4, device=w.device, dtype=w.dtype)
    buf[:, :K] = w.detach()
    return buf[:, :K]


class _GemmLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, slope, col_pos=None):
        if x.dtype != torch.float32 or weight.dtype != torch.float32:
            raise TypeError("apn linear: float32 only")
        dev = x.device
        x2 = x.reshape(-1, x.shape[-1])
        if x2.stride(-1) != 1 or x2.stride(0) < x2.shape[1]:
            x2 = x2.contiguous()
        lda = x2.stride(0)   # rows may be padded (pad_cat): 16-B aligned rows take the vector loads
        M, K = x2.shape
        N = weight.shape[0]
        if col_pos is not None:   # x holds weight column j at column col_pos[j]; other columns meet zeros
            wx = torch.zeros(N, -(-K // 4) * 4, device=dev, dtype=torch.float32)
            wx[:, col_pos] = weight.detach()
            w = wx[:, :K]
        else:
            if weight.shape[1] != K:
                raise ValueError(f"apn linear: input width {K} vs weight {tuple(weight.shape)}")
            w = _padded_rows(weight)
        b = bias.contiguous() if bias is not None else None
        y = torch.empty(M, N, device=dev, dtype=torch.float32)
        act = slope is not None
        call("apn_gemm_f32", ptr(x2), None, ptr(w), ptr(y), ptr(b), M, N, K, lda, w.stride(0), N, 0, 1, 0.0, int(act),
             float(slope) if act else 0.0, stream_ptr(dev))
        ctx.save_for_backward(x2, w, y if act else None)
        ctx.slope, ctx.has_bias, ctx.in_shape, ctx.col_pos = slope, bias is not None, x.shape, col_pos
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
            Kp = -(-K // 4) * 4   # 16-B rows for the next product's vector loads
            dx = torch.empty(M, Kp, device=dev, dtype=torch.float32)
            call("apn_gemm_f32", ptr(dy), ptr(y), ptr(w), ptr(dx), None, M, K, N, N, w.stride(0), Kp, 0, 0, sm, 0, 0.0,
                 s)
            dx = dx[:, :K]
            if len(ctx.in_shape) != 2:
                dx = dx.reshape(ctx.in_shape)
        want_b = ctx.has_bias and ctx.needs_input_grad[2]
        if ctx.needs_input_grad[1] or want_b:
            dw = torch.empty(N, K, device=dev, dtype=torch.float32)
            db = torch.empty(N, device=dev, dtype=torch.float32) if want_b else None
            bn = 192 if -(-K // 192) < -(-K // 128) else 128   # the kernel's column tile (apn_gemm.hip run)
            tiles = -(-N // 64) * -(-K // bn)
            splits = max(1, min(M // SPLIT_ROWS, SPLIT_TILES // tiles))
            ws = torch.empty(int(load().apn_gemm_f32_splitk_workspace_bytes(N, K, splits)) // 4 + 1,
                             device=dev, dtype=torch.float32)
            call("apn_gemm_f32_splitk", ptr(dy), ptr(y), ptr(x), ptr(dw), ptr(db), N, K, M, N, x.stride(0), 1, 0, sm,
                 splits, ptr(ws), s)
            if ctx.col_pos is not None:
                dw = dw[:, ctx.col_pos]
        return dx, (dw if ctx.needs_input_grad[1] else None), db, None, None


def pad_cat(parts) -> torch.Tensor:
    """torch.cat(parts, -1) for [M, k_i] tensors, written into rows padded to a multiple of 4 floats
    (a view of width sum k_i): the first layer's product then reads 16-B aligned rows."""
    M = parts[0].shape[0]
    K = sum(p.shape[-1] for p in parts)
    Kp = -(-K // 4) * 4
    if Kp == K or not parts[0].is_cuda:
        return torch.cat(parts, dim=-1)
    buf = torch.empty(M, Kp, device=parts[0].device, dtype=parts[0].dtype)
    c = 0
    for p in parts:
        buf[:, c:c + p.shape[-1]].copy_(p)
        c += p.shape[-1]
    return buf[:, :K]


def linear(x: torch.Tensor, layer: torch.nn.Linear, slope=None, col_pos=None) -> torch.Tensor:
    """act(x W^T + b) for a torch.nn.Linear ``layer``; ``slope``: None (no activation), 0 (ReLU)
    or the LeakyReLU negative slope. ``col_pos`` (CUDA, int64 [in_features]): x is wider than the
    layer and holds input j at column col_pos[j] (zero weight on the others). CPU tensors: torch's
    own ops."""
    if not x.is_cuda:
        if col_pos is not None:
            x = x[..., col_pos]
        y = torch.nn.functional.linear(x, layer.weight, layer.bias)
        if slope is None:
            return y
        return torch.relu(y) if slope == 0 else torch.nn.functional.leaky_relu(y, slope)
    return _GemmLinear.apply(x, layer.weight, layer.bias, slope, col_pos)


def _flatten(net):
    for m in net:
        if isinstance(m, torch.nn.Sequential):
            yield from _flatten(m)
        else:
            yield m


def sequential(net: torch.nn.Module, x: torch.Tensor, col_pos=None) -> torch.Tensor:
    """A Sequential of Linear / LeakyReLU / ReLU (nested Sequentials flattened): each Linear runs
    with the activation that follows it fused into its epilogue (``col_pos``: the first layer's,
    see linear)."""
    mods = list(_flatten(net))
    i = 0
    while i < len(mods):
        m = mods[i]
        if isinstance(m, torch.nn.Linear):
            nxt = mods[i + 1] if i + 1 < len(mods) else None
            cp, col_pos = col_pos, None
            if isinstance(nxt, torch.nn.LeakyReLU):
                x = linear(x, m, float(nxt.negative_slope), cp)
                i += 2
                continue
            if isinstance(nxt, torch.nn.ReLU):
                x = linear(x, m, 0.0, cp)
                i += 2
                continue
            x = linear(x, m, None, cp)
        else:
            x = m(x)
        i += 1
    return x
