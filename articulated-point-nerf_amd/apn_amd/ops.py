"""Torch-facing wrappers over the C-ABI: allocation, stream plumbing, shape checks.

Every function here launches HIP kernels from libapn_hip.so on the current stream; none
has a CPU path.
"""
from __future__ import annotations

import math
import weakref

import torch

from . import _lib as L
from ._lib import call, ptr, stream_ptr


def _f32c(t):
    return t.detach().to(torch.float32).contiguous()


class Workspace:
    """Grow-only device scratch buffers keyed by name (reused across forward calls). While a HIP
    graph that captured them is alive (``hold(graph)``, called by capture_frame / capture_repose
    right before each capture), a replaced buffer is kept alive, not freed: the graph holds its
    address, and a later larger frame (an overflow rendered again exactly, another ray shard's
    capture, a bigger ray set) must not hand that memory to anything else. A retired buffer is
    released once every graph alive at its retirement has been destroyed (a re-capture drops the
    old graph), so repeated capacity growth does not accumulate buffers."""

    def __init__(self):
        self.bufs = {}
        self.meta = {}         # host-side keys of what the buffers hold (e.g. the packed weights' version)
        self.retired = []      # [(buffer, tokens of the graphs that may hold its address)]
        self._holders = set()  # tokens of the live graphs
        self._n = 0

    @property
    def pinned(self):
        return bool(self._holders)

    def hold(self, graph):
        """Register a graph about to capture workspace addresses; its token is released when the
        graph object is garbage-collected."""
        self._n += 1
        tok = self._n
        self._holders.add(tok)
        weakref.finalize(graph, self._release, tok)
        return tok

    def _release(self, tok):
        self._holders.discard(tok)
        keep = []
        for b, toks in self.retired:
            toks.discard(tok)
            if toks:
                keep.append((b, toks))
        self.retired = keep

    def get(self, name, numel, dtype, device):
        b = self.bufs.get(name)
        if b is None or b.numel() < numel or b.dtype != dtype or b.device != torch.device(device):
            if b is not None and self._holders:
                self.retired.append((b, set(self._holders)))
            b = torch.empty(max(int(numel), 1), dtype=dtype, device=device)
            self.bufs[name] = b
        return b[:max(int(numel), 1)]

    def bytes(self, name, nbytes, device):
        return self.get(name, (int(nbytes) + 255) // 256 * 256, torch.uint8, device)


# ----------------------------------------------------------------------------------------
# render_utils_cuda drop-ins (render_utils.cpp:144-155)
# ----------------------------------------------------------------------------------------

def sample_pts_on_rays(rays_o, rays_d, xyz_min, xyz_max, near, far, stepdist):
    """Returns [rays_pts, mask_outbbox, ray_id, step_id, N_steps, t_min, t_max] like
    render_utils_cuda.sample_pts_on_rays (render_utils_kernel.cu:190-236)."""
    L.require_cuda(rays_o, rays_d, xyz_min, xyz_max, what="sample_pts_on_rays")
    if not (rays_o.is_contiguous() and rays_d.is_contiguous()):
        raise RuntimeError("rays_o / rays_d must be contiguous")
    dev = rays_o.device
    ro, rd = _f32c(rays_o), _f32c(rays_d)
    lo, hi = _f32c(xyz_min), _f32c(xyz_max)
    R = ro.shape[0]
    t_min = torch.empty(R, device=dev); t_max = torch.empty(R, device=dev)
    n_steps = torch.empty(R, dtype=torch.int64, device=dev)
    offs = torch.empty(R + 1, dtype=torch.int32, device=dev)
    ws = torch.empty(int(L.load().apn_sample_pts_on_rays_workspace_bytes(R)) + 256, dtype=torch.uint8, device=dev)
    s = stream_ptr(dev)
    call("apn_sample_pts_on_rays_count", ptr(ro), ptr(rd), ptr(lo), ptr(hi), float(near), float(far),
         float(stepdist), R, ptr(t_min), ptr(t_max), ptr(n_steps), ptr(offs), ptr(ws), s)
    total = int(offs[R].item())
    pts = torch.empty(total, 3, device=dev)
    mask = torch.empty(total, dtype=torch.bool, device=dev)
    ray_id = torch.empty(total, dtype=torch.int64, device=dev)
    step_id = torch.empty(total, dtype=torch.int64, device=dev)
    call("apn_sample_pts_on_rays_fill", ptr(ro), ptr(rd), ptr(lo), ptr(hi), float(near), float(far),
         float(stepdist), R, ptr(offs), ptr(pts), ptr(mask), ptr(ray_id), ptr(step_id), s)
    return [pts, mask, ray_id, step_id, n_steps, t_min, t_max]


def raw2alpha(density, shift, interval):
    """render_utils_kernel.cu:357-393 -> (exp_d, alpha)."""
    L.require_cuda(density, what="raw2alpha")
    d = _f32c(density)
    e = torch.empty_like(d); a = torch.empty_like(d)
    call("apn_raw2alpha", ptr(d), float(shift), float(interval), d.numel(), ptr(e), ptr(a), stream_ptr(d.device))
    return e, a


def alpha2weight(alpha, ray_id, n_rays):
    """render_utils_kernel.cu:430-505 -> (weight, T, alphainv_last, i_start, i_end)."""
    L.require_cuda(alpha, ray_id, what="alpha2weight")
    a = _f32c(alpha); rid = ray_id.to(torch.int64).contiguous()
    n = a.numel(); dev = a.device
    w = torch.empty(n, device=dev); T = torch.empty(n, device=dev)
    last = torch.empty(int(n_rays), device=dev)
    i_s = torch.empty(int(n_rays), dtype=torch.int64, device=dev)
    i_e = torch.empty(int(n_rays), dtype=torch.int64, device=dev)
    call("apn_alpha2weight", ptr(a), ptr(rid), n, int(n_rays), ptr(w), ptr(T), ptr(last), ptr(i_s), ptr(i_e),
         stream_ptr(dev))
    return w, T, last, i_s, i_e


def raw2alpha_backward(exp_d, grad_back, interval):
    """render_utils.cpp:110-114 / render_utils_kernel.cu:395-428 -> grad w.r.t. density."""
    L.require_cuda(exp_d, grad_back, what="raw2alpha_backward")
    e = _f32c(exp_d); gb = _f32c(grad_back)
    if gb.numel() != e.numel():
        raise RuntimeError("raw2alpha_backward: exp and grad_back sizes differ")
    g = torch.empty_like(e)
    call("apn_raw2alpha_backward", ptr(e), ptr(gb), float(interval), e.numel(), ptr(g), stream_ptr(e.device))
    return g


def alpha2weight_backward(alpha, weight, T, alphainv_last, i_start, i_end, n_rays, grad_weights, grad_last):
    """render_utils.cpp:125-141 / render_utils_kernel.cu:507-561 -> grad w.r.t. alpha."""
    L.require_cuda(alpha, weight, T, alphainv_last, i_start, i_end, grad_weights, grad_last,
                   what="alpha2weight_backward")
    a = _f32c(alpha); w = _f32c(weight); t = _f32c(T); last = _f32c(alphainv_last)
    gw = _f32c(grad_weights); gl = _f32c(grad_last)
    i_s = i_start.to(torch.int64).contiguous(); i_e = i_end.to(torch.int64).contiguous()
    n = a.numel(); R = int(n_rays)
    if not (w.numel() == t.numel() == gw.numel() == n) or not (last.numel() == i_s.numel() == i_e.numel()
                                                              == gl.numel() == R):
        raise RuntimeError("alpha2weight_backward: inconsistent sizes")
    g = torch.empty_like(a)
    call("apn_alpha2weight_backward", ptr(a), ptr(w), ptr(t), ptr(last), ptr(i_s), ptr(i_e), n, R, ptr(gw), ptr(gl),
         ptr(g), stream_ptr(a.device))
    return g


def knn_points(q, pts, k, cell_cap=1 << 20):
    """K nearest points of ``pts`` for every row of ``q`` (unbounded; the pykeops argKmin of
    temporalpoints.py:104-111, 737-748) -> (d2 [M,k] float32 ascending, idx [M,k] int64)."""
    L.require_cuda(q, pts, what="knn_points")
    qq = _f32c(q).reshape(-1, 3); pp = _f32c(pts).reshape(-1, 3)
    M, N = qq.shape[0], pp.shape[0]
    if not 1 <= int(k) <= min(16, N):
        raise RuntimeError(f"knn_points: k must be in [1, min(16, n_points)], got {k}")
    dev = pp.device
    lib = L.load()
    sorted4 = torch.empty(N, 4, device=dev)
    bbox = torch.empty(8, dtype=torch.int32, device=dev)
    gws = torch.empty(int(lib.apn_grid_workspace_bytes(N, cell_cap)), dtype=torch.uint8, device=dev)
    idx = torch.empty(M, int(k), dtype=torch.int64, device=dev)
    d2 = torch.empty(M, int(k), device=dev)
    call("apn_knn_points", ptr(qq), M, ptr(pp), N, int(k), int(cell_cap), ptr(sorted4), ptr(bbox), ptr(gws),
         ptr(idx), ptr(d2), stream_ptr(dev))
    return d2, idx


class Alphas2Weights(torch.autograd.Function):
    """tineuvox.py:627-643 over the HIP ops: forward -> (weights, alphainv_last)."""

    @staticmethod
    def forward(ctx, alpha, ray_id, N):
        weights, T, alphainv_last, i_start, i_end = alpha2weight(alpha, ray_id, N)
        if alpha.requires_grad:
            ctx.save_for_backward(alpha, weights, T, alphainv_last, i_start, i_end)
            ctx.n_rays = N
        return weights, alphainv_last

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, grad_weights, grad_last):
        alpha, weights, T, alphainv_last, i_start, i_end = ctx.saved_tensors
        grad = alpha2weight_backward(alpha, weights, T, alphainv_last, i_start, i_end, ctx.n_rays,
                                     grad_weights, grad_last)
        return grad, None, None


class Raw2Alpha(torch.autograd.Function):
    """tineuvox.py:646-670 over the HIP ops: alpha = 1 - (1 + exp(density + shift))^(-interval)."""

    @staticmethod
    def forward(ctx, density, shift, interval):
        exp, alpha = raw2alpha(density, shift, interval)
        if density.requires_grad:
            ctx.save_for_backward(exp)
            ctx.interval = interval
        return alpha

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, grad_back):
        exp = ctx.saved_tensors[0]
        return raw2alpha_backward(exp, grad_back.contiguous(), ctx.interval), None, None


def segment_coo_sum(src, index, n_out):
    """torch_scatter.segment_coo(src, index, out=zeros, reduce='sum') for sorted index."""
    L.require_cuda(src, index, what="segment_coo")
    s2 = _f32c(src)
    C = math.prod(s2.shape[1:]) if s2.dim() > 1 else 1
    idx = index.to(torch.int64).contiguous()
    out = torch.empty((int(n_out),) + tuple(s2.shape[1:]), device=s2.device)
    ws = torch.empty(2 * max(int(n_out), 1), dtype=torch.int64, device=s2.device)
    call("apn_segment_sum", ptr(s2), ptr(idx), s2.shape[0], C, int(n_out), ptr(out), ptr(ws), stream_ptr(s2.device))
    return out


# ----------------------------------------------------------------------------------------
# packed MLP weights
# ----------------------------------------------------------------------------------------

_LAYOUT = None
_LAYOUT_NAMES = ["W1E", "B1", "W2", "B2", "W3", "B3", "W4", "B4", "WD", "BD", "WH", "BH", "WV2", "BV2", "W1F",
                 "TOTAL", "KE", "KV", "H16", "FLAG"]


def mlp_layout():
    global _LAYOUT
    if _LAYOUT is None:
        import ctypes as C
        arr = (C.c_int32 * 32)()
        n = L.load().apn_mlp_weight_layout(arr)
        if n != len(_LAYOUT_NAMES):
            raise RuntimeError(f"apn_mlp_weight_layout returned {n} offsets, expected {len(_LAYOUT_NAMES)}")
        _LAYOUT = dict(zip(_LAYOUT_NAMES, list(arr)[:n]))
    return _LAYOUT


def pack_mlp_weights(feat_net_layers, densitynet, rgbnet, pose_embedding=None, out=None):
    """Pack feat_net / densitynet / rgbnet (nn.Linear (out,in) layout, zero-padded K) into the
    buffer apn_point_mlp / apn_feat_project read (layout: apn_mlp_weight_layout):
      * feat_net.0 split into its posenc columns (W1E) and feature columns (W1F);
      * the pose-embedding columns (temporalpoints.py:487-488) folded into b1: b1 + W1p @ pe;
      * rgbnet.feature_linears folded into views_linears.0 (no activation in between):
        WH = [Wv0[:, :128] @ Wf | Wv0[:, 128:]], BH = Wv0[:, :128] @ bf + bv0 (float64 fold)."""
    lay = mlp_layout()
    l1, l2, l3, l4 = feat_net_layers
    dev = l1.weight.device
    buf = out if out is not None else torch.zeros(lay["TOTAL"], device=dev)
    L.require_cuda(buf, what="pack_mlp_weights")
    KE, KV = lay["KE"], lay["KV"]

    def put(name, t):
        t = t.detach().float().reshape(-1)
        buf[lay[name]:lay[name] + t.numel()].copy_(t)

    w1 = l1.weight.detach().float()
    n_emb, n_feat = 63, 128
    if w1.shape[1] < n_emb + n_feat:
        raise ValueError(f"feat_net.0 has {w1.shape[1]} inputs; expected >= {n_emb + n_feat}")
    w1e = torch.zeros(128, KE, device=dev)
    w1e[:, :n_emb] = w1[:, :n_emb]
    put("W1E", w1e)
    put("W1F", w1[:, n_emb:n_emb + n_feat].contiguous())
    b1 = l1.bias.detach().float()
    if pose_embedding is not None:
        b1 = b1 + (w1[:, n_emb + n_feat:] @ pose_embedding.reshape(-1, 1).float()).reshape(-1)
    elif w1.shape[1] != n_emb + n_feat:
        raise ValueError(f"feat_net.0 expects {w1.shape[1]} inputs but no pose embedding was given")
    put("B1", b1)
    for nm, l in (("2", l2), ("3", l3), ("4", l4)):
        put("W" + nm, l.weight); put("B" + nm, l.bias)
    put("WD", densitynet.weight); put("BD", densitynet.bias)
    wf = rgbnet.feature_linears.weight.detach().double()
    bf = rgbnet.feature_linears.bias.detach().double()
    v0 = rgbnet.views_linears[0]
    wv0 = v0.weight.detach().double()
    nh = wf.shape[0]
    wh = torch.zeros(64, KV, dtype=torch.float64, device=dev)
    wh[:, :nh] = wv0[:, :nh] @ wf
    wh[:, nh:wv0.shape[1]] = wv0[:, nh:]
    put("WH", wh)
    put("BH", wv0[:, :nh] @ bf + v0.bias.detach().double())
    v2 = rgbnet.views_linears[2]
    put("WV2", v2.weight); put("BV2", v2.bias)
    # fp16 hi/lo MFMA fragments of W1E (posenc columns reordered), W2-W4 and WH for the default
    # (3-term split) apn_point_mlp kernel
    call("apn_mlp_split_weights", ptr(buf), stream_ptr(dev))
    return buf


def fold_pose_bias(l1, pose_embedding, buf):
    """Per-frame update of a packed buffer whose weights are unchanged: only b1 depends on the
    pose embedding (temporalpoints.py:487-488, folded as in pack_mlp_weights). Also clears the
    range flag, as the full pack's split does, so the guard is judged per frame."""
    lay = mlp_layout()
    n_emb, n_feat = 63, 128
    w1 = l1.weight.detach().float()
    b1 = l1.bias.detach().float() + (w1[:, n_emb + n_feat:] @ pose_embedding.reshape(-1, 1).float()).reshape(-1)
    buf[lay["B1"]:lay["B1"] + b1.numel()].copy_(b1)
    buf[lay["FLAG"]:lay["FLAG"] + 1].view(torch.int32).zero_()
    if hasattr(L.load(), "apn_mlp_split_bias"):   # (absent only from A/B builds of earlier revisions)
        call("apn_mlp_split_bias", ptr(buf), stream_ptr(buf.device))   # b1 is also the bias column's weights
    return buf


def mlp_range_fallback(wbuf) -> bool:
    """True if the fp16-split MLP kernel met a value outside the fp16 range with these packed
    weights (its range flag, apn_mlp_layout.h OFF_FLAG), so apn_point_mlp recomputed the launch on
    the FP32 MFMA kernel. Reads one int from the device (a sync): for tests and diagnostics."""
    off = mlp_layout()["FLAG"]
    return bool(int(wbuf[off:off + 1].view(torch.int32).item()))


def feat_project(canonical_feat, wbuf, out=None):
    """apn_feat_project: per-point layer-1 feature projection [N,128]."""
    L.require_cuda(canonical_feat, wbuf, what="feat_project")
    f = canonical_feat.detach().float().contiguous()
    N = f.shape[0]
    P = out if out is not None else torch.empty(N, 128, device=f.device)
    call("apn_feat_project", ptr(f), N, f.shape[1], ptr(wbuf), ptr(P), stream_ptr(f.device))
    return P
