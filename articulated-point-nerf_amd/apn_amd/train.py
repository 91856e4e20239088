"""Differentiable forward of TemporalPoints -- the reference's train_pcd step.

run.py:574-716 calls ``model(time_sel, False, render_kwargs, ...)`` with autograd on, takes
``rgb_marched`` into an MSE loss plus the regularisers and steps the optimizer.
``TemporalPoints.forward`` routes here whenever ``torch.is_grad_enabled()``; under
``torch.no_grad()`` it stays on the fused render pipeline.

What runs where:
  * ray sampling in the cloud's bbox, the uniform grid and the radius-bounded exact 8-NN
    (the pykeops ``Kmin_argKmin`` + radius filter, temporalpoints.py:423-447) -- HIP kernels
    through the C-ABI (``apn_grid_build``, ``apn_inbbox_count/fill``, ``apn_knn_radius``); they
    produce integer indices only, so nothing there needs a gradient;
  * ``Raw2Alpha`` / ``Alphas2Weights`` (tineuvox.py:627-670) -- the HIP forward and backward
    kernels (``apn_raw2alpha{,_backward}``, ``apn_alpha2weight{,_backward}``);
  * everything differentiable in between -- get_weights, the skeleton chain, LBS blend, the 3x3
    inverse, the IDW weights, the gathers, feat_net / densitynet / rgbnet, the direct blend and
    the ray sums -- as the reference's own torch expressions, so autograd gives the reference's
    gradients (the GEMMs go to hipBLASLt).
"""
from __future__ import annotations

import ctypes as C
import gc

import torch

from . import _lib as L
from . import linear as LIN
from ._lib import call, ptr, stream_ptr
from .ops import Alphas2Weights, Raw2Alpha
from .tineuvox import poc_fre

__all__ = ["forward_train", "LBSTrain", "lbs_train", "lbs_blend", "inv3x3", "radius_knn", "ordered_bbox",
           "reverse_csr", "NbrTVLoss", "ArapLoss",
           "feat_net_forward", "SparsityLoss"]


def cloud_min_max(xyz: torch.Tensor):
    """(min [3], max [3]) of an [N,3] cloud, reduced along contiguous rows of its transpose (the
    strided dim-0 reductions took ~0.15 ms each at 300k points); min/max are exact, so the values
    equal xyz.min(0)/xyz.max(0)."""
    xt = xyz.t().contiguous()
    return xt.amin(dim=1), xt.amax(dim=1)


def cloud_bbox(xyz: torch.Tensor):
    """(min/max [6] float, bbox_ord [8] int32) of an [N,3] device cloud in two launches
    (apn_cloud_bbox: block partials, one final block); the values equal cloud_min_max's (min and
    max are exact) and bbox_ord equals ordered_bbox's."""
    xyz = xyz.detach().float().contiguous()
    mm = torch.empty(6, device=xyz.device)
    ordv = torch.empty(8, dtype=torch.int32, device=xyz.device)
    ws = torch.empty(1024 * 6, device=xyz.device)
    call("apn_cloud_bbox", ptr(xyz), xyz.shape[0], ptr(mm), ptr(ordv), ptr(ws), stream_ptr(xyz.device))
    return mm, ordv


def ordered_bbox(xyz: torch.Tensor) -> torch.Tensor:
    """Cloud min/max as the order-preserving int32 encoding the grid kernels read
    (``float_to_ordered`` in csrc/apn_common.h), 8 slots like the LBS kernel's bbox_ord."""
    mm = torch.cat(cloud_min_max(xyz)).float().contiguous()
    i = mm.view(torch.int32)
    out = torch.zeros(8, dtype=torch.int32, device=xyz.device)
    out[:6] = torch.where(i >= 0, i, i ^ 0x7fffffff)
    return out


def lbs_blend(pcd, weights, bone_Ts, global_t):
    """pointwarper.py:241-266 as differentiable torch: G_n = sum_j W_nj T_j, x' = G_n [x;1] + t.
    Only the 3x4 rows are formed (the bottom row is exactly [0,0,0,1]); the per-point 3x3 products
    are broadcast multiply-adds (batched 3x3 bmm / linalg.inv go to tiny-GEMM / LU library kernels
    that cost ~10x more here)."""
    J = bone_Ts.shape[0]
    G = (weights @ bone_Ts[:, :3, :].reshape(J, 12)).reshape(-1, 3, 4)
    xyz = (G[:, :, :3] * pcd[:, None, :]).sum(-1) + G[:, :, 3] + global_t
    return xyz, G


def inv3x3(A):
    """Adjugate inverse of [N,3,3] (differentiable elementwise ops); == torch.inverse(G)[:, :3, :3]
    for the affine G of temporalpoints.py:569 up to float32 rounding."""
    a, b, c = A[:, 0, 0], A[:, 0, 1], A[:, 0, 2]
    d, e, f = A[:, 1, 0], A[:, 1, 1], A[:, 1, 2]
    g, h, i = A[:, 2, 0], A[:, 2, 1], A[:, 2, 2]
    c00, c01, c02 = e * i - f * h, f * g - d * i, d * h - e * g
    det = a * c00 + b * c01 + c * c02
    adj = torch.stack([c00, c * h - b * i, b * f - c * e,
                       c01, a * i - c * g, c * d - a * f,
                       c02, b * g - a * h, a * e - b * d], dim=-1)
    return (adj / det[:, None]).reshape(-1, 3, 3)


class LBSTrain(torch.autograd.Function):
    """get_weights + LBS blend/apply + the 3x3 inverse as one HIP forward and one HIP backward
    (apn_lbs_train_fwd / _bwd): (W [N,J], theta [1], T34 [J,12], global_t [3]) ->
    (xyz [N,3], Rinv [N,3,3], sm [N,J]); canonical points and eps are constants."""

    @staticmethod
    def forward(ctx, W, theta, T34, global_t, pcd, eps):
        N, J = W.shape
        dev = W.device
        Wc, th, T, gt = (x.detach().float().contiguous() for x in (W, theta, T34, global_t))
        sm = torch.empty(N, J, device=dev)
        G12 = torch.empty(N, 12, device=dev)
        xyz = torch.empty(N, 3, device=dev)
        Rinv = torch.empty(N, 3, 3, device=dev)
        call("apn_lbs_train_fwd", ptr(pcd), ptr(Wc), N, J, ptr(th), float(eps), ptr(T), ptr(gt), ptr(sm), ptr(G12),
             ptr(xyz), ptr(Rinv), stream_ptr(dev))
        ctx.save_for_backward(Wc, th, T, sm, Rinv, pcd)
        ctx.eps = float(eps)
        return xyz, Rinv, sm

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, d_xyz, d_Rinv, d_sm):
        Wc, th, T, sm, Rinv, pcd = ctx.saved_tensors
        N, J = Wc.shape
        dev = Wc.device
        c = lambda x: None if x is None else x.float().contiguous()
        d_xyz, d_Rinv, d_sm = c(d_xyz), c(d_Rinv), c(d_sm)
        dW = torch.empty(N, J, device=dev)
        dT = torch.empty(J, 12, device=dev)
        dgt = torch.empty(3, device=dev)
        dth = torch.empty(1, device=dev)
        ws = torch.empty(int(L.load().apn_lbs_train_workspace_bytes(N, J)), dtype=torch.uint8, device=dev)
        call("apn_lbs_train_bwd", ptr(pcd), ptr(Wc), N, J, ptr(th), ctx.eps, ptr(T), ptr(sm), ptr(Rinv), ptr(d_xyz),
             ptr(d_Rinv), ptr(d_sm), ptr(dW), ptr(dT), ptr(dgt), ptr(dth), ptr(ws), stream_ptr(dev))
        return dW, dth, dT, dgt, None, None


def reverse_csr(nn_i: torch.Tensor):
    """Reverse adjacency of the kNN graph nn_i [N,K] (int64): rev_ptr [N+1], rev_edge [N*K] = edge
    ids i*K+k grouped by their target nn_i[i,k], ascending within a target (stable sort) -- the
    in-edges the HIP loss backward gathers instead of an atomic scatter-add."""
    N = nn_i.shape[0]
    flat = nn_i.reshape(-1)
    rev_edge = torch.argsort(flat, stable=True).contiguous()
    rev_ptr = torch.zeros(N + 1, dtype=torch.int64, device=nn_i.device)
    rev_ptr[1:] = torch.cumsum(torch.bincount(flat, minlength=N), 0)
    return rev_ptr, rev_edge


def reverse_index(idx: torch.Tensor, n_targets: int):
    """rev_ptr [n_targets+1], rev_edge: the positions of idx (flattened, int64) grouped by value,
    ascending within a value (stable sort) -- the gather order of the per-point gradient sums."""
    flat = idx.reshape(-1)
    rev_edge = torch.argsort(flat, stable=True).contiguous()
    rev_ptr = torch.zeros(n_targets + 1, dtype=torch.int64, device=idx.device)
    # counts by index_add (bincount reads its bound back to the host)
    counts = torch.zeros(n_targets, dtype=torch.int64, device=idx.device).index_add_(0, flat, torch.ones_like(flat))
    rev_ptr[1:] = torch.cumsum(counts, 0)
    return rev_ptr, rev_edge


class NbrAggregate(torch.autograd.Function):
    """temporalpoints.py:452-491 for the training forward as one HIP forward (apn_nbr_train_fwd) and
    one HIP backward (apn_nbr_train_bwd): (ray_pts [S,3], s_i [S,8], xyz [N,3], Rinv [N,3,3],
    canonical_feat [N,F], pose_emb [1,P] | None, sig [N], rgb_c [N,3], alpha_c [N] (clipped), poc,
    eps) -> (w [S,8] IDW weights, rgb_d [S,3], alpha_d [S], feat_in [8S, PE4+F+P] in 16-B rows:
    posenc (PE = 3+6L columns) zero-padded to PE4 = 4 ceil(PE/4), then the features -- feat_in_columns
    gives where each of feat_net's first-layer inputs sits). Per-point gradients are gathered over
    the reverse adjacency of s_i (no atomics)."""

    @staticmethod
    def forward(ctx, ray_pts, s_i, xyz, Rinv, feat, pose_emb, sig, rgb_c, alpha_c, poc, eps):
        dev = xyz.device
        S = s_i.shape[0]
        F = feat.shape[1]
        P = pose_emb.shape[-1] if pose_emb is not None else 0
        L = poc.numel()
        PE4 = -(-(3 + 6 * L) // 4) * 4
        K = PE4 + F + P
        Kp = -(-K // 4) * 4
        c = lambda x: x.detach().float().contiguous()
        args = [c(ray_pts), s_i.contiguous(), c(xyz), c(Rinv), c(sig), c(rgb_c), c(alpha_c), c(poc)]
        w = torch.empty(S, 8, device=dev)
        rgbd = torch.empty(S, 3, device=dev)
        alphad = torch.empty(S, device=dev)
        buf = torch.empty(S * 8, Kp, device=dev)
        pe = c(pose_emb) if pose_emb is not None else None
        call("apn_nbr_train_fwd", S, ptr(args[0]), ptr(args[1]), ptr(args[2]), ptr(args[3]), ptr(c(feat)), F, ptr(pe),
             P, ptr(args[4]), ptr(args[5]), ptr(args[6]), ptr(args[7]), L, float(eps), ptr(w), ptr(rgbd), ptr(alphad),
             ptr(buf), Kp, stream_ptr(dev))
        ctx.save_for_backward(*args)
        ctx.meta = (S, xyz.shape[0], F, P, L, float(eps), K)
        ctx.pose_shape = pose_emb.shape if pose_emb is not None else None
        return w, rgbd, alphad, buf[:, :K]

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, d_w, d_rgbd, d_alphad, d_feat):
        ray_pts, s_i, xyz, Rinv, sig, rgb_c, alpha_c, poc = ctx.saved_tensors
        S, N, F, P, L, eps, K = ctx.meta
        dev = xyz.device
        c = lambda x: None if x is None else x.float().contiguous()
        d_w, d_rgbd, d_alphad = c(d_w), c(d_rgbd), c(d_alphad)
        if d_feat is not None and (d_feat.stride(-1) != 1 or d_feat.stride(0) < K):
            d_feat = d_feat.contiguous()
        ldd = d_feat.stride(0) if d_feat is not None else K
        rev_ptr, rev_edge = reverse_index(s_i, N)
        contrib = torch.empty(S * 8, 17, device=dev)
        d_xyz = torch.empty(N, 3, device=dev)
        d_R = torch.empty(N, 3, 3, device=dev)
        d_sig = torch.empty(N, device=dev)
        d_c = torch.empty(N, 3, device=dev)
        d_a = torch.empty(N, device=dev)
        want_feat = ctx.needs_input_grad[4] and d_feat is not None
        d_featp = torch.empty(N, F, device=dev) if want_feat else None
        call("apn_nbr_train_bwd", S, N, ptr(ray_pts), ptr(s_i), ptr(xyz), ptr(Rinv), ptr(sig), ptr(rgb_c), ptr(alpha_c),
             ptr(poc), L, eps, ptr(d_w), ptr(d_rgbd), ptr(d_alphad), ptr(d_feat), ldd, F, ptr(rev_ptr), ptr(rev_edge),
             ptr(contrib), ptr(d_xyz), ptr(d_R), ptr(d_sig), ptr(d_c), ptr(d_a), ptr(d_featp), stream_ptr(dev))
        d_pose = None
        if P > 0 and ctx.needs_input_grad[5] and d_feat is not None:
            d_pose = d_feat[:, K - P:].sum(0).reshape(ctx.pose_shape)
        return None, None, d_xyz, d_R, d_featp, d_pose, d_sig, d_c, d_a, None, None


_FEAT_COLS = {}


def feat_in_columns(L, F, P, device):
    """Column of feat_in (NbrAggregate) holding each of the reference's feat_net inputs
    [posenc (3+6L) | canonical_feat (F) | pose embedding (P)] (cached on the device)."""
    key = (L, F, P, str(device))
    if key not in _FEAT_COLS:
        PE = 3 + 6 * L
        PE4 = -(-PE // 4) * 4
        _FEAT_COLS[key] = torch.cat([torch.arange(PE), torch.arange(PE4, PE4 + F + P)]).to(device)
    return _FEAT_COLS[key]


class IdwSum(torch.autograd.Function):
    """h = sum_k w[s,k] out[8s+k] (temporalpoints.py:493-494) as apn_idw_sum_fwd / _bwd."""

    @staticmethod
    def forward(ctx, w, out):
        S, C = w.shape[0], out.shape[-1]
        w, out = w.contiguous(), out.reshape(S * 8, C).contiguous()
        h = torch.empty(S, C, device=out.device)
        call("apn_idw_sum_fwd", S, C, ptr(w), ptr(out), ptr(h), stream_ptr(out.device))
        ctx.save_for_backward(w, out)
        return h

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dh):
        w, out = ctx.saved_tensors
        S, C = w.shape[0], out.shape[-1]
        d_out = torch.empty_like(out) if ctx.needs_input_grad[1] else None
        d_w = torch.empty_like(w) if ctx.needs_input_grad[0] else None
        call("apn_idw_sum_bwd", S, C, ptr(w), ptr(out), ptr(dh.contiguous()), ptr(d_out), ptr(d_w),
             stream_ptr(out.device))
        return d_w, d_out


class NbrTVLoss(torch.autograd.Function):
    """get_neighbour_weight_tv_loss (temporalpoints.py:714-716): mean |w_i - w_nn(i,k)| over
    [N,K,J] as one fused HIP edge reduction (apn_nbr_tv_loss); backward apn_nbr_tv_loss_backward
    (out-edges + reverse-CSR in-edges, no scatter). nn_i / rev_ptr / rev_edge are constants."""

    @staticmethod
    def forward(ctx, w, nn_i, rev_ptr, rev_edge):
        L.require_cuda(w, nn_i, what="NbrTVLoss")
        wc = w.detach().float().contiguous()
        N, J = wc.shape
        K = nn_i.shape[1]
        dev = wc.device
        loss = torch.empty((), device=dev)
        ws = torch.empty(int(L.load().apn_nbr_loss_workspace_bytes()), dtype=torch.uint8, device=dev)
        call("apn_nbr_tv_loss", ptr(wc), N, J, ptr(nn_i), K, ptr(loss), ptr(ws), stream_ptr(dev))
        ctx.save_for_backward(wc, nn_i, rev_ptr, rev_edge)
        return loss

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, d_loss):
        wc, nn_i, rev_ptr, rev_edge = ctx.saved_tensors
        N, J = wc.shape
        dw = torch.empty_like(wc)
        dl = d_loss.float().contiguous()
        call("apn_nbr_tv_loss_backward", ptr(wc), N, J, ptr(nn_i), nn_i.shape[1], ptr(rev_ptr), ptr(rev_edge),
             ptr(dl), ptr(dw), stream_ptr(wc.device))
        return dw, None, None, None


class ArapLoss(torch.autograd.Function):
    """get_arap_loss (temporalpoints.py:723-725): sum_ik |d0_ik - sqrt(|x_i - x_nn(i,k)|^2 + eps)| as
    one fused HIP edge reduction (apn_arap_loss); backward apn_arap_loss_backward (gathers only).
    nn_i, the canonical distances d0 [N,K] and the reverse CSR are constants."""

    @staticmethod
    def forward(ctx, x, nn_i, d0, eps, rev_ptr, rev_edge):
        L.require_cuda(x, nn_i, d0, what="ArapLoss")
        xc = x.detach().float().contiguous()
        N = xc.shape[0]
        K = nn_i.shape[1]
        dev = xc.device
        d0c = d0.detach().float().contiguous()
        loss = torch.empty((), device=dev)
        ws = torch.empty(int(L.load().apn_nbr_loss_workspace_bytes()), dtype=torch.uint8, device=dev)
        call("apn_arap_loss", ptr(xc), N, ptr(nn_i), K, ptr(d0c), float(eps), ptr(loss), ptr(ws), stream_ptr(dev))
        ctx.save_for_backward(xc, nn_i, d0c, rev_ptr, rev_edge)
        ctx.eps = float(eps)
        return loss

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, d_loss):
        xc, nn_i, d0c, rev_ptr, rev_edge = ctx.saved_tensors
        dx = torch.empty_like(xc)
        dl = d_loss.float().contiguous()
        call("apn_arap_loss_backward", ptr(xc), xc.shape[0], ptr(nn_i), nn_i.shape[1], ptr(d0c), ctx.eps,
             ptr(rev_ptr), ptr(rev_edge), ptr(dl), ptr(dx), stream_ptr(xc.device))
        return dx, None, None, None, None, None


class SparsityLoss(torch.autograd.Function):
    """get_weight_sparsity_loss (temporalpoints.py:718-721) as one HIP partial pass
    (apn_weight_sparsity_loss) and one elementwise backward (apn_weight_sparsity_loss_backward)."""

    @staticmethod
    def forward(ctx, w, eps):
        L.require_cuda(w, what="SparsityLoss")
        wc = w.detach().float().contiguous()
        dev = wc.device
        loss = torch.empty((), device=dev)
        ws = torch.empty(int(L.load().apn_nbr_loss_workspace_bytes()), dtype=torch.uint8, device=dev)
        call("apn_weight_sparsity_loss", ptr(wc), wc.numel(), float(eps), ptr(loss), ptr(ws), stream_ptr(dev))
        ctx.save_for_backward(wc)
        ctx.eps = float(eps)
        return loss

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, d_loss):
        (wc,) = ctx.saved_tensors
        dw = torch.empty_like(wc)
        dl = d_loss.float().contiguous()
        call("apn_weight_sparsity_loss_backward", ptr(wc), wc.numel(), ctx.eps, ptr(dl), ptr(dw),
             stream_ptr(wc.device))
        return dw, None


def feat_net_forward(net: torch.nn.Module, x: torch.Tensor) -> torch.Tensor:
    """Run a Sequential of Linear / LeakyReLU (nested) on the hand-written GEMM (linear.sequential):
    same parameters, f32 products and sums per output element, the activation in the epilogue."""
    return LIN.sequential(net, x)


def lbs_train(model, bone_Ts, global_t, identity_rules=None):
    """(t_hat_pcd, Rinv, weights) of the training forward: the fused HIP Function for identity
    merge rules and J <= 64, else the torch composition (get_weights + lbs_blend + inv3x3).
    ``identity_rules``: model._merge_rules() is None, when the caller already knows (inside a
    graph capture the check's host copy is not allowed)."""
    J = bone_Ts.shape[0]
    if identity_rules is None:
        identity_rules = model._merge_rules() is None
    if identity_rules and J <= 64:
        pcd = model.forward_warp.canonical_pcd.detach().float().contiguous()
        th = model.theta_weight.reshape(1)
        gt = global_t.reshape(3)
        xyz, Rinv, weights = LBSTrain.apply(model.weights, th, bone_Ts[:, :3, :].reshape(J, 12), gt, pcd,
                                            model._eps)
        return xyz, Rinv, weights
    weights = model.get_weights()
    xyz, G = lbs_blend(model.forward_warp.canonical_pcd, weights, bone_Ts, global_t)
    return xyz, inv3x3(G[:, :, :3]), weights


# The warp stage of a training step -- skeleton (TransformNet, Rodrigues, masks, the kinematic
# chain), fused LBS, pose embedding -- has the same shapes every step, so it runs as a captured
# HIP graph pair (graph_callable: one forward replay, one backward replay) instead of ~100 forward
# and ~250 backward launches from the host. Off: the eager composition.
GRAPH_WARP = True


def graph_callable(module, sample, num_warmup=2):
    """``module`` (forward(x) -> tuple of tensors) captured as a forward and a backward HIP graph
    and wrapped in an autograd Function over (x, *module.parameters()): the role of
    torch.cuda.make_graphed_callables, with the streams kept consistent for autograd.

    Every parameter's AccumulateGrad node carries the stream it was created on, and a backward
    that reaches it from another stream makes autograd synchronise -- and, inside a capture, ends
    the capture when that stream is the default one (the core dump of round 5's capture probe).
    make_graphed_callables warms up on one stream, captures on another, and keeps the captured
    forward's autograd graph alive (its static outputs), so the parameters' nodes of the capture
    stream stay alive and every later training backward on the default stream met them ("The
    AccumulateGrad node's stream does not match ..."). Here: (1) unreachable graphs are collected
    first and the caller has dropped its references to earlier steps' graphs, so no node of
    another stream is alive; (2) warm-up and both captures run on ONE stream; (3) only detached
    aliases of the static outputs are kept, so the captured forward's autograd graph -- and with
    it the capture stream's AccumulateGrad nodes -- is freed before the first replay, and the
    training step's own forward creates the nodes on its stream."""
    dev = sample.device
    params = tuple(module.parameters())
    surface = (sample,) + params
    req_in = [i for i, t in enumerate(surface) if t.requires_grad]
    gc.collect()
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        for _ in range(num_warmup):
            outs = tuple(module(sample))
            req = [o for o in outs if o.requires_grad]
            if req:
                torch.autograd.grad(req, [surface[i] for i in req_in], [torch.empty_like(o) for o in req],
                                    allow_unused=True)
            del outs, req
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize(dev)
    static_in = sample.detach().clone()
    pool = torch.cuda.graph_pool_handle()
    fwd, bwd = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    from .temporalpoints import _capture_guard
    with _capture_guard():
        with torch.cuda.graph(fwd, pool=pool, stream=s):
            outs = tuple(module(static_in))
        req_out = [i for i, o in enumerate(outs) if o.requires_grad]
        static_gout = [torch.empty_like(outs[i]) for i in req_out]
        with torch.cuda.graph(bwd, pool=pool, stream=s):
            gin = torch.autograd.grad([outs[i] for i in req_out], [surface[i] for i in req_in], static_gout,
                                      allow_unused=True)
        static_out = tuple(o.detach() for o in outs)
        static_gin = [None] * len(surface)
        for i, g in zip(req_in, gin):
            static_gin[i] = g.detach() if g is not None else None
        del outs, gin
    torch.cuda.current_stream(dev).wait_stream(s)

    class _Graphed(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, *ps):
            if x.data_ptr() != static_in.data_ptr():
                static_in.copy_(x)
            fwd.replay()
            return tuple(o.detach() for o in static_out)

        @staticmethod
        @torch.autograd.function.once_differentiable
        def backward(ctx, *grads):
            for j, i in enumerate(req_out):
                g = grads[i]
                if g is None:
                    static_gout[j].zero_()
                elif g.data_ptr() != static_gout[j].data_ptr():
                    static_gout[j].copy_(g)
            bwd.replay()
            return tuple(g.detach() if g is not None else None for g in static_gin)

    def run(x):
        return _Graphed.apply(x, *params)
    run.graphs = (fwd, bwd)
    return run


class _WarpStage(torch.nn.Module):
    """pointwarper.py:213-239 + temporalpoints.py:401-414, 569, 478 (+ the pose embedding
    380-381) as one module over the parameters they read; forward(t_embed) returns every tensor
    the rest of the step uses: (t_hat_pcd, Rinv, weights, bone_Ts, global_t, joints_rel, thetas,
    params[, pose_embedding])."""

    def __init__(self, model, identity_rules):
        super().__init__()
        self.fw = model.forward_warp
        self.joints = model.joints
        self.weights = model.weights
        self.theta_weight = model.theta_weight
        self.pe = model.pose_embedding_net if model.pose_embedding_dim > 0 else None
        self._model = (model,)   # not a submodule: only the stage's own parameters are graph inputs
        self._identity_rules = identity_rules

    def forward(self, t_embed):
        model = self._model[0]
        bone_Ts, global_t, joints_rel = self.fw.pose_torch(self.joints, t_embed, None)
        xyz, Rinv, weights = lbs_train(model, bone_Ts, global_t, identity_rules=self._identity_rules)
        out = [xyz, Rinv, weights, bone_Ts, global_t, joints_rel, self.fw.prev_thetas, self.fw.prev_params]
        # no reference to this pass's autograd graph may outlive it: a parameter's AccumulateGrad
        # node kept alive from a pass on another stream makes the captured backward wait on that
        # stream, which ends the capture (warp_stage sets the pose state from the replay's outputs)
        self.fw.prev_thetas = self.fw.prev_params = self.fw.prev_global_t = None
        if self.pe is not None:
            delta_joint = (self.joints - joints_rel).clone().detach()
            out.append(LIN.sequential(self.pe, poc_fre(delta_joint, model.pos_poc).view(1, -1)))
        return tuple(out)


def _graphed_warp(model, t_embed):
    """The model's captured warp stage for this input shape, captured again when a parameter
    tensor, its requires_grad, or the skeleton's masks change."""
    fw = model.forward_warp
    identity_rules = model._merge_rules() is None
    params = [model.joints, model.weights, model.theta_weight] + list(fw.parameters())
    if model.pose_embedding_dim > 0:
        params += list(model.pose_embedding_net.parameters())
    key = (tuple(t_embed.shape), identity_rules, tuple((p.data_ptr(), p.requires_grad) for p in params),
           (fw.rot_mask.data_ptr(), fw.rot_mask._version), (fw.sibling_mask.data_ptr(), fw.sibling_mask._version),
           model.training)
    hit = model.__dict__.get("_warp_graph")
    if hit is not None and hit[0] == key:
        return hit[1]
    model.__dict__.pop("_warp_graph", None)
    # drop the model's references to earlier steps' autograd graphs (pose state, LBS weights):
    # their parameter AccumulateGrad nodes carry the stream those steps ran on (see _WarpStage)
    fw.prev_thetas = fw.prev_params = fw.prev_global_t = None
    model._last_weights = None
    stage = _WarpStage(model, identity_rules)
    stage.train(model.training)
    sample = t_embed.detach().clone()
    graphed = graph_callable(stage, sample)
    model.__dict__["_warp_graph"] = (key, graphed)
    return graphed


def warp_stage(model, t_embed):
    """(t_hat_pcd, Rinv, weights, bone_Ts, global_t, joints_rel, pose_embedding) of the training
    forward; sets the pose state the regularisers read (prev_thetas / prev_params / prev_global_t)
    and model._last_weights, as the eager composition does."""
    fw = model.forward_warp
    if GRAPH_WARP and t_embed.is_cuda and torch.is_grad_enabled():
        out = _graphed_warp(model, t_embed)(t_embed)
        xyz, Rinv, weights, bone_Ts, global_t, joints_rel, thetas, params = out[:8]
        fw.prev_thetas, fw.prev_params, fw.prev_global_t = thetas, params, global_t
        pose_embedding = out[8] if len(out) > 8 else None
    else:
        bone_Ts, global_t, joints_rel = fw.pose_torch(model.joints, t_embed, None)
        xyz, Rinv, weights = lbs_train(model, bone_Ts, global_t)
        pose_embedding = None
        if model.pose_embedding_dim > 0:
            delta_joint = (model.joints - joints_rel).clone().detach()
            pose_embedding = LIN.sequential(model.pose_embedding_net, poc_fre(delta_joint, model.pos_poc).view(1, -1))
    model._last_weights = weights
    return xyz, Rinv, weights, bone_Ts, global_t, joints_rel, pose_embedding


def radius_knn(model, xyz, bbox6, rk, query_radius, bbox_ord=None):
    """Sampling in bbox6 + radius-bounded exact 8-NN on the HIP path (temporalpoints.py:423-447).
    Returns (ray_pts [S,3], ray_id [S] i64, step_id [S] i64, s_i [S,8] i64, n_inbbox); S may be 0.
    ``bbox_ord``: the cloud's ordered bbox when the caller has it (cloud_bbox)."""
    from .temporalpoints import CELL_CAP
    dev = xyz.device
    lib = L.load()
    s = stream_ptr(dev)
    N = xyz.shape[0]
    xyz = xyz.detach().float().contiguous()
    ro = rk['rays_o'].detach().float().contiguous()
    rd = rk['rays_d'].detach().float().contiguous()
    L.require_cuda(ro, rd, what="render_kwargs")
    R = ro.shape[0]
    qr = float(query_radius)
    stepdist = float(rk['stepsize']) * float(model.voxel_size)
    near, far = float(rk['near']), float(rk['far'])
    if bbox_ord is None:
        bbox_ord = ordered_bbox(xyz)
    gws = torch.empty(int(lib.apn_grid_workspace_bytes(N, CELL_CAP)), dtype=torch.uint8, device=dev)
    sorted4 = torch.empty(N, 4, device=dev)
    call("apn_grid_build", ptr(xyz), N, ptr(bbox_ord), qr, CELL_CAP, ptr(sorted4), ptr(gws), s)
    offs = torch.empty(R + 1, dtype=torch.int32, device=dev)
    sws = torch.empty(int(lib.apn_sample_pts_on_rays_workspace_bytes(R)), dtype=torch.uint8, device=dev)
    call("apn_inbbox_count", ptr(ro), ptr(rd), ptr(bbox6), near, far, stepdist, R, ptr(offs), ptr(sws), s)
    n_bbox = int(offs[R].item())
    empty = (xyz.new_zeros(0, 3), torch.zeros(0, dtype=torch.int64, device=dev),
             torch.zeros(0, dtype=torch.int64, device=dev), torch.zeros(0, 8, dtype=torch.int64, device=dev), n_bbox)
    if n_bbox == 0:
        return empty
    q_pos = torch.empty(n_bbox, 4, device=dev)
    q_ray = torch.empty(n_bbox, dtype=torch.int32, device=dev)
    call("apn_inbbox_fill", ptr(ro), ptr(rd), ptr(bbox6), near, far, stepdist, R, ptr(offs), ptr(q_pos),
         ptr(q_ray), s)
    s_pos = torch.empty(n_bbox, 4, device=dev)
    s_ray = torch.empty(n_bbox, dtype=torch.int32, device=dev)
    s_nbr = torch.empty(n_bbox, 8, dtype=torch.int32, device=dev)
    nsurv = torch.empty(1, dtype=torch.int32, device=dev)
    kws = torch.empty(int(lib.apn_knn_workspace_bytes(n_bbox)), dtype=torch.uint8, device=dev)
    call("apn_knn_radius", ptr(q_pos), ptr(q_ray), n_bbox, C.c_void_p(offs.data_ptr() + 4 * R), ptr(gws), N,
         CELL_CAP, ptr(sorted4), qr, ptr(s_pos), ptr(s_ray), ptr(s_nbr), ptr(nsurv), ptr(kws), s)
    S = int(nsurv.item())
    if S == 0:
        return empty
    pos = s_pos[:S]
    return (pos[:, :3].contiguous(), s_ray[:S].long(), pos[:, 3].contiguous().view(torch.int32).long(),
            s_nbr[:S].long(), n_bbox)


def _ray_sum(src, ray_id, R):
    """torch_scatter.segment_coo(..., reduce='sum') into zeros (differentiable index_add)."""
    out = src.new_zeros((R,) + tuple(src.shape[1:]))
    return out.index_add(0, ray_id, src)


def forward_train(model, t, render_depth=False, render_kwargs=None, query_radius=0.01, render_weights=False,
                  rot_params=None, poses=None, Ks=None, calc_min_max=True, get_skeleton=False):
    """temporalpoints.py:540-712 (+ aggregate_pts 416-521) with autograd; same return dict."""
    from .temporalpoints import NoPointsException, project_point_to_image_plane
    rk = render_kwargs
    dev = model.canonical_feat.device
    L.require_cuda(model.canonical_feat, what="TemporalPoints.forward")
    K = model.neighbours
    # skeleton + LBS (temporalpoints.py:547-569; pointwarper.py:213-279)
    fw = model.forward_warp
    if rot_params is None:
        # get_weights + blend/apply + torch.inverse(G)[:, :3, :3] (569, 478), captured stage
        t_hat_pcd, Rinv, weights, bone_Ts, global_t, joints_rel, pose_embedding = warp_stage(
            model, poc_fre(t, model.time_poc))
    else:
        bone_Ts, global_t, joints_rel = fw.pose_torch(model.joints, None, rot_params)
        t_hat_pcd, Rinv, weights = lbs_train(model, bone_Ts, global_t)
        model._last_weights = weights
        delta_joint = (model.joints - joints_rel).clone().detach()
        pose_embedding = (LIN.sequential(model.pose_embedding_net, poc_fre(delta_joint, model.pos_poc).view(1, -1))
                          if model.pose_embedding_dim > 0 else None)
    joints = bones = None
    if get_skeleton:
        joints = project_point_to_image_plane(joints_rel + global_t, poses.to(dev), Ks.to(dev, torch.float32))
        bones = model.bones
        if model.joints_to_keep is not None:
            joints = joints[:, model.joints_to_keep]
            bones = model.new_bones
    R = len(rk['rays_o'])
    bg = rk['bg']
    # sampling bbox (423-427) and kNN (433-447)
    qr = float(query_radius)
    mm, bbox_ord = cloud_bbox(t_hat_pcd)
    if calc_min_max:
        bbox6 = torch.cat([mm[:3] - qr, mm[3:] + qr]).float().contiguous()
    else:
        bbox6 = torch.cat([model.xyz_min, model.xyz_max]).float().contiguous()
    ray_pts, ray_id, step_id, s_i, n_bbox = radius_knn(model, t_hat_pcd, bbox6, rk, qr, bbox_ord=bbox_ord)
    model.last_stats = {"rays": R, "inbbox_samples": n_bbox, "survivors": len(s_i)}
    model.last_train_knn = (ray_id, s_i)
    if len(s_i) == 0:       # NoPointsException fallback (598-609)
        return {'rgb_marched': torch.ones(R, 3, device=dev) * bg,
                'rgb_marched_direct': torch.ones(R, 3, device=dev) * bg,
                'depth': torch.zeros(R, device=dev), 'weights': torch.ones(R, 3, device=dev) * bg,
                't_hat_pcd': t_hat_pcd, 'alphainv_last': None, 'grid': None, 'joints': joints, 'bones': bones}
    # direct render blend (459-470, forced on at 592), IDW weights (472-475), rel_c + posenc + the
    # feat_net input rows (476-491): one HIP forward / backward (NbrAggregate)
    sig = model.mean_min_distance * torch.clamp(model.direct_eps, min=0.)
    w, rgbs_direct, alpha_direct, feat_in = NbrAggregate.apply(
        ray_pts, s_i, t_hat_pcd, Rinv, model.canonical_feat, pose_embedding, sig, model.canonical_rgbs.clip(0, 1),
        model.canonical_alpha.clip(0, 1), model.pos_poc, model._eps)
    cols = feat_in_columns(model.pos_poc.numel(), model.canonical_feat.shape[1],
                           pose_embedding.shape[-1] if pose_embedding is not None else 0, dev)
    out = LIN.sequential(model.feat_net, feat_in, col_pos=cols)
    h = IdwSum.apply(w, out)   # 493-494
    w = w.unsqueeze(-1)
    # heads (496-515)
    density = LIN.linear(h, model.densitynet).squeeze(-1)
    interval = float(rk['stepsize']) * float(model.tineuvox.voxel_size_ratio)
    alpha = Raw2Alpha.apply(density.contiguous(), float(model.tineuvox.act_shift), interval)
    if model.no_view_dir:
        raise NotImplementedError("no_view_dir=True breaks the reference forward (viewdirs_emb_reshape undefined)")
    if model.frozen_view_dir is not None:
        views = model.viewdirs_emb.expand(len(ray_id), -1)
    else:
        views = poc_fre(rk['viewdirs'], model.view_poc)[ray_id]
    rgbs = torch.sigmoid(model.rgbnet(h, views))
    lbsw = (weights[s_i, :] * w).sum(dim=1) if render_weights else None
    ray_id_d = ray_id
    thr = model.fast_color_thres
    # pre-masks (611-627) as zeroed alphas instead of dropped samples (no host sync for the count):
    # a zero alpha leaves the ray's transmittance and every other weight bit-identical, gets weight
    # 0 and no gradient, as a dropped sample would
    zero = alpha.new_zeros(())
    if thr > 0:
        alpha = torch.where(alpha > thr, alpha, zero)
        alpha_direct = torch.where(alpha_direct > thr, alpha_direct, zero)

    def a2w(a, rid):
        if a.numel() == 0:
            return a, torch.ones(R, device=dev)
        return Alphas2Weights.apply(a.contiguous(), rid.contiguous(), R)
    weights_r, alphainv_last = a2w(alpha, ray_id)
    weights_d, alphainv_last_d = a2w(alpha_direct, ray_id_d)
    # post-masks (633-651), zeroed the same way: the ray sums add exact zeros
    if thr > 0:
        weights_r = torch.where(weights_r > thr, weights_r, zero)
        weights_d = torch.where(weights_d > thr, weights_d, zero)
    # ray sums (653-677)
    rgb_marched = _ray_sum(weights_r.unsqueeze(-1) * rgbs, ray_id, R) + alphainv_last.unsqueeze(-1) * bg
    rgb_marched_d = _ray_sum(weights_d.unsqueeze(-1) * rgbs_direct, ray_id_d, R) + alphainv_last_d.unsqueeze(-1) * bg
    ret = {'t_hat_pcd': t_hat_pcd, 'rgb_marched': rgb_marched, 'alphainv_last': alphainv_last,
           'alphainv_last_direct': alphainv_last_d, 'grid': None, 'rgb_marched_direct': rgb_marched_d,
           'joints': joints, 'bones': bones}
    if render_depth:
        ret['depth'] = _ray_sum(weights_r * step_id, ray_id, R)
    if render_weights:      # 690-710
        col = lbsw @ model._joint_colors(dev)
        ret['weights'] = _ray_sum(weights_r.unsqueeze(-1) * col, ray_id, R) + alphainv_last.unsqueeze(-1) * bg
    return ret
