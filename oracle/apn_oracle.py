"""TEST INFRASTRUCTURE ONLY -- CPU restatement of the articulated-point render/deform path.

Each function cites the reference file:line it restates (paths relative to the reference
repository root). Floating-point conventions are fixed so that the HIP kernels can be
checked bit-exactly where the path produces indices:

* float32 everywhere the reference kernel uses ``float``; no fused multiply-add (numpy and
  torch-CPU elementwise ops round every operation; the HIP kernels that produce indices are
  compiled with ``-ffp-contract=off``);
* squared distances are ``(dx*dx + dy*dy) + dz*dz`` in float32 -- the reference recomputes
  ``to_nn = (rel_p**2).sum(-1)`` with exactly this association (temporalpoints.py:446-447);
* the double-precision promotions of the CUDA source are reproduced
  (render_utils_kernel.cu:47 and 450-451);
* kNN ties are broken by point index (pykeops leaves tie order unspecified).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this module.
"""
from __future__ import annotations

import colorsys
import math

import re

import numpy as np
import torch

F32 = np.float32


# ----------------------------------------------------------------------------------------
# Positional encoding -- tineuvox.py:872-878
# ----------------------------------------------------------------------------------------

def poc_fre(x: torch.Tensor, freqs: torch.Tensor) -> torch.Tensor:
    """[x, sin(x (x) f), cos(x (x) f)], dim-major flatten (x0f0..x0f{F-1}, x1f0, ...)."""
    emb = (x.unsqueeze(-1) * freqs).flatten(-2)
    return torch.cat([x, emb.sin(), emb.cos()], -1)


# ----------------------------------------------------------------------------------------
# render_utils_cuda restatement -- lib/cuda/render_utils_kernel.cu
# ----------------------------------------------------------------------------------------

def infer_t_minmax(rays_o, rays_d, xyz_min, xyz_max, near, far):
    """render_utils_kernel.cu:11-35. Zero direction components become (float)1e-6."""
    o = np.asarray(rays_o, F32); d = np.asarray(rays_d, F32)
    lo = np.asarray(xyz_min, F32); hi = np.asarray(xyz_max, F32)
    v = np.where(d == 0, F32(1e-6), d).astype(F32)
    a = ((hi[None, :] - o) / v).astype(F32)
    b = ((lo[None, :] - o) / v).astype(F32)
    mn = np.minimum(a, b); mx = np.maximum(a, b)
    near = F32(near); far = F32(far)
    t_min = np.maximum(np.minimum(np.maximum(np.maximum(mn[:, 0], mn[:, 1]), mn[:, 2]), far), near)
    t_max = np.maximum(np.minimum(np.minimum(np.minimum(mx[:, 0], mx[:, 1]), mx[:, 2]), far), near)
    return t_min.astype(F32), t_max.astype(F32)


def infer_n_samples(t_min, t_max, stepdist):
    """render_utils_kernel.cu:37-49: max(ceil((t_max-t_min)/stepdist), 1.) -> int64."""
    q = ((t_max - t_min).astype(F32) / F32(stepdist)).astype(F32)
    return np.maximum(np.ceil(q).astype(np.float64), 1.0).astype(np.int64)


def infer_ray_start_dir(rays_o, rays_d, t_min):
    """render_utils_kernel.cu:51-73: start = o + d*t_min; dir = d / |d|."""
    o = np.asarray(rays_o, F32); d = np.asarray(rays_d, F32)
    rnorm = np.sqrt(((d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]).astype(F32)).astype(F32)
    start = (o + (d * t_min[:, None]).astype(F32)).astype(F32)
    direc = (d / rnorm[:, None]).astype(F32)
    return start, direc


def sample_pts_on_rays(rays_o, rays_d, xyz_min, xyz_max, near, far, stepdist):
    """render_utils_kernel.cu:190-236 (host) + 138-188 (kernels).

    Returns [rays_pts (M,3) f32, mask_outbbox (M,) bool, ray_id (M,) i64, step_id (M,) i64,
    N_steps (R,) i64, t_min (R,) f32, t_max (R,) f32], M = sum(N_steps).
    """
    t_min, t_max = infer_t_minmax(rays_o, rays_d, xyz_min, xyz_max, near, far)
    n_steps = infer_n_samples(t_min, t_max, stepdist)
    R = len(n_steps)
    ray_id = np.repeat(np.arange(R, dtype=np.int64), n_steps)
    starts = np.concatenate([[0], np.cumsum(n_steps)[:-1]]).astype(np.int64)
    step_id = np.arange(len(ray_id), dtype=np.int64) - starts[ray_id]
    start, direc = infer_ray_start_dir(rays_o, rays_d, t_min)
    dist = (F32(stepdist) * step_id.astype(F32)).astype(F32)
    pts = (start[ray_id] + (direc[ray_id] * dist[:, None]).astype(F32)).astype(F32)
    lo = np.asarray(xyz_min, F32); hi = np.asarray(xyz_max, F32)
    mask_out = np.any(lo[None, :] > pts, axis=1) | np.any(hi[None, :] < pts, axis=1)
    return [pts, mask_out, ray_id, step_id, n_steps, t_min, t_max]


def raw2alpha(density, shift, interval):
    """render_utils_kernel.cu:357-393: e = exp(d+shift); alpha = 1 - (1+e)^(-interval)."""
    d = np.asarray(density, F32)
    with np.errstate(over="ignore"):
        e = np.exp((d + F32(shift)).astype(F32)).astype(F32)
        alpha = (F32(1) - np.power((F32(1) + e).astype(F32), F32(-F32(interval)))).astype(F32)
    return e, alpha


def alpha2weight(alpha, ray_id, n_rays):
    """render_utils_kernel.cu:430-505.

    Per ray (segments of the sorted ``ray_id``): T[i] = T_cum; w[i] = T_cum*alpha[i] (float);
    T_cum = (float)((double)T_cum * (1. - (double)alpha[i])); break after the sample whose
    update drops T_cum below 1e-3 (double compare). alphainv_last = T_cum (1 for empty rays).
    Vectorised over rays, sequential over the step within a ray.
    Returns [weight, T, alphainv_last, i_start, i_end].
    """
    a = np.asarray(alpha, F32); rid = np.asarray(ray_id, np.int64)
    n = len(a)
    weight = np.zeros(n, F32); T = np.ones(n, F32)
    last = np.ones(n_rays, F32)
    i_start = np.zeros(n_rays, np.int64); i_end = np.zeros(n_rays, np.int64)
    if n == 0:
        return [weight, T, last, i_start, i_end]
    chg = np.nonzero(rid[1:] != rid[:-1])[0] + 1
    i_start[rid[chg]] = chg
    i_end[rid[chg - 1]] = chg
    i_end[rid[n - 1]] = n
    rays = np.unique(rid)
    s = i_start[rays].copy(); e = i_end[rays].copy()
    Tc = np.ones(len(rays), F32)
    active = s < e
    pos = s.copy()
    while active.any():
        idx = pos[active]
        al = a[idx]
        tc = Tc[active]
        T[idx] = tc
        weight[idx] = (tc * al).astype(F32)
        tc_new = (tc.astype(np.float64) * (1.0 - al.astype(np.float64))).astype(F32)
        Tc[active] = tc_new
        pos[active] = idx + 1
        stop = tc_new.astype(np.float64) < 1e-3
        act_idx = np.nonzero(active)[0]
        active[act_idx[stop]] = False
        active &= pos < e
    i_end[rays] = pos
    last[rays] = Tc
    return [weight, T, last, i_start, i_end]


def raw2alpha_backward(exp_d, grad_back, interval):
    """render_utils_kernel.cu:395-406 (float instantiation), the backward of Raw2Alpha
    (tineuvox.py:662-670). min(exp_d, 1e10) has a double operand, so the product
    ((min * powf(1 + e, -interval - 1)) * interval) * grad_back runs in double and rounds to float
    once; the power itself is float."""
    e = np.asarray(exp_d, F32); gb = np.asarray(grad_back, F32)
    with np.errstate(over="ignore"):
        pw = np.power((F32(1) + e).astype(F32), (F32(-F32(interval)) - F32(1)).astype(F32)).astype(F32)
    m = np.minimum(e.astype(np.float64), 1e10)
    return (((m * pw.astype(np.float64)) * np.float64(F32(interval))) * gb.astype(np.float64)).astype(F32)


def alpha2weight_backward(alpha, weight, T, alphainv_last, i_start, i_end, n_rays, grad_weights, grad_last):
    """render_utils_kernel.cu:507-528, the backward of Alphas2Weights (tineuvox.py:637-643).

    Per ray, samples i_end-1 down to i_start: grad[i] = gw[i]*T[i] - back_cum/(1 - alpha[i] + 1e-10)
    with gw*T and 1 - alpha in float, the division and subtraction in double (1e-10 is a double
    literal), rounded at the store; back_cum (float) starts at grad_last*alphainv_last and adds
    gw[i]*weight[i]. Samples outside [i_start, i_end) get 0. Vectorised over rays."""
    a = np.asarray(alpha, F32); w = np.asarray(weight, F32); t = np.asarray(T, F32)
    gw = np.asarray(grad_weights, F32)
    last = np.asarray(alphainv_last, F32); gl = np.asarray(grad_last, F32)
    s = np.asarray(i_start, np.int64); e = np.asarray(i_end, np.int64)
    grad = np.zeros(len(a), F32)
    back = (gl * last).astype(F32)
    pos = e - 1
    active = pos >= s
    while active.any():
        r = np.nonzero(active)[0]
        idx = pos[r]
        den = (F32(1) - a[idx]).astype(F32).astype(np.float64) + 1e-10
        grad[idx] = ((gw[idx] * t[idx]).astype(F32).astype(np.float64) - back[r].astype(np.float64) / den).astype(F32)
        back[r] = (back[r] + (gw[idx] * w[idx]).astype(F32)).astype(F32)
        pos[r] = idx - 1
        active = pos >= s
    return grad


def _powf():
    """The C library's powf, which the reference's host code calls (std::pow(float, float));
    numpy's float32 power can differ from it by an ulp."""
    import ctypes
    import ctypes.util
    try:
        libm = ctypes.CDLL(ctypes.util.find_library("m") or "libm.so.6")
        f = libm.powf
        f.restype = ctypes.c_float
        f.argtypes = [ctypes.c_float, ctypes.c_float]
        return lambda x, y: F32(f(float(x), float(y)))
    except (OSError, AttributeError):   # pragma: no cover
        return lambda x, y: F32(np.power(F32(x), F32(y)))


def adam_step_size(step, beta1, beta2, lr):
    """adam_upd_kernel.cu:70 (host, float): lr * sqrt(1 - b2^step) / (1 - b1^step) with the C
    library's powf."""
    powf = _powf()
    b1, b2, lr = F32(beta1), F32(beta2), F32(lr)
    return F32(lr * np.sqrt(F32(1) - powf(b2, F32(step))) / (F32(1) - powf(b1, F32(step))))


def adam_upd(param, grad, exp_avg, exp_avg_sq, step, beta1, beta2, lr, eps, masked=False, perlr=None):
    """adam_upd_kernel.cu:8-58 in float without contraction (in place on the given arrays):
    m = b1 m + (1-b1) g; v = b2 v + ((1-b2) g) g; p -= (ss [* perlr]) m / (sqrt(v) + eps);
    masked: elements with g == 0 are left untouched."""
    p, g, m, v = param, np.asarray(grad, F32), exp_avg, exp_avg_sq
    b1, b2, e = F32(beta1), F32(beta2), F32(eps)
    ss = adam_step_size(step, beta1, beta2, lr)
    sel = (g != 0) if masked else np.ones(g.shape, bool)
    m_new = (b1 * m + (F32(1) - b1) * g).astype(F32)
    v_new = (b2 * v + ((F32(1) - b2) * g).astype(F32) * g).astype(F32)
    scale = (ss * np.asarray(perlr, F32)).astype(F32) if perlr is not None else ss
    p_new = (p - ((scale * m_new).astype(F32) / (np.sqrt(v_new) + e).astype(F32)).astype(F32)).astype(F32)
    m[sel] = m_new[sel]; v[sel] = v_new[sel]; p[sel] = p_new[sel]


def total_variation_add_grad(param, grad, wx, wy, wz, dense_mode):
    """total_variation_kernel.cu:13-67 on a [1, C, I, J, K] float grid, in place on ``grad``:
    six clamped differences in source order, weights / 6, the I direction weighted by wz."""
    P = np.asarray(param, F32)
    C, I, J, K = P.shape[1:]
    wy6, wz6 = F32(F32(wy) / F32(6)), F32(F32(wz) / F32(6))
    p = P.reshape(C, I, J, K)
    gr = grad.reshape(C, I, J, K)
    cl = lambda x: np.clip(x, F32(-1), F32(1)).astype(F32)
    z = np.zeros_like(p)

    def nb(axis, sh):   # clamp(p - neighbour) where the neighbour along ``axis`` (-sh side) exists
        d = np.zeros_like(p)
        src = [slice(None)] * 4; dst = [slice(None)] * 4
        if sh > 0:
            dst[axis] = slice(1, None); src[axis] = slice(0, -1)
        else:
            dst[axis] = slice(0, -1); src[axis] = slice(1, None)
        d[tuple(dst)] = cl(p[tuple(dst)] - p[tuple(src)])
        return d
    acc = z.copy()
    terms = [(3, 1, wz6), (3, -1, wz6), (2, 1, wy6), (2, -1, wy6), (1, 1, wz6), (1, -1, wz6)]
    for axis, sh, w in terms:
        acc = (acc + (w * nb(axis, sh)).astype(F32)).astype(F32)
    sel = np.ones_like(gr, bool) if dense_mode else (gr != 0)
    gr[sel] = (gr[sel] + acc[sel]).astype(F32)


def segment_sum(src, index, n):
    """torch_scatter.segment_coo(reduce='sum') over sorted ``index``: sequential in-order
    float32 accumulation into a zero output (temporalpoints.py:653-677)."""
    src = np.asarray(src, F32); index = np.asarray(index, np.int64)
    out = np.zeros((n,) + src.shape[1:], F32)
    np.add.at(out, index, src)
    return out


# ----------------------------------------------------------------------------------------
# kNN -- pykeops LazyTensor.Kmin_argKmin semantics (temporalpoints.py:433-437, 106-111)
# ----------------------------------------------------------------------------------------

def sqdist(q: np.ndarray, p: np.ndarray) -> np.ndarray:
    """Float32 squared distance (dx*dx + dy*dy) + dz*dz, broadcasting q[...,3] vs p[...,3]."""
    dx = (q[..., 0] - p[..., 0]).astype(F32)
    dy = (q[..., 1] - p[..., 1]).astype(F32)
    dz = (q[..., 2] - p[..., 2]).astype(F32)
    return ((dx * dx + dy * dy).astype(F32) + dz * dz).astype(F32)


def _finalize_topk(q, pts, cand, K):
    """Exact (d2, idx) lexicographic top-K among candidate indices cand (Q, C)."""
    d2 = sqdist(q[:, None, :], pts[cand])
    order = np.lexsort((cand, d2), axis=1)[:, :K]
    idx = np.take_along_axis(cand, order, 1)
    return np.take_along_axis(d2, order, 1), idx


def knn_kmin(query, points, K, chunk=2048, use_tree=None):
    """K smallest float32 squared distances (ascending, ties by index) and their indices.

    Brute force for small problems; a scipy cKDTree candidate search (K+6 candidates in
    float64, re-ranked in float32) for large ones.
    """
    q = np.ascontiguousarray(query, F32); p = np.ascontiguousarray(points, F32)
    Q, N = len(q), len(p)
    Kc = min(N, K + 6)
    if use_tree is None:
        use_tree = Q * N > 4e8
    d_out = np.empty((Q, K), F32); i_out = np.empty((Q, K), np.int64)
    if Q == 0:
        return d_out, i_out
    if use_tree:
        from scipy.spatial import cKDTree
        tree = cKDTree(p.astype(np.float64))
        for s in range(0, Q, 1 << 18):
            qq = q[s:s + (1 << 18)]
            _, cand = tree.query(qq.astype(np.float64), k=Kc, workers=torch.get_num_threads())
            cand = np.asarray(cand, np.int64).reshape(len(qq), Kc)
            d_out[s:s + len(qq)], i_out[s:s + len(qq)] = _finalize_topk(qq, p, cand, K)
        return d_out, i_out
    pt = torch.from_numpy(p)
    for s in range(0, Q, chunk):
        qq = q[s:s + chunk]
        qt = torch.from_numpy(qq)
        dx = qt[:, None, 0] - pt[None, :, 0]
        dy = qt[:, None, 1] - pt[None, :, 1]
        dz = qt[:, None, 2] - pt[None, :, 2]
        d2 = (dx * dx + dy * dy) + dz * dz
        cand = torch.topk(d2, Kc, dim=1, largest=False).indices.numpy().astype(np.int64)
        d_out[s:s + len(qq)], i_out[s:s + len(qq)] = _finalize_topk(qq, p, cand, K)
    return d_out, i_out


def knn_radius_certified(query, points, K=8, r2=0.01, kc=16, chunk=1 << 19, workers=None):
    """The render path's kNN + radius filter (temporalpoints.py:433-447: Kmin_argKmin K=8, keep a
    sample iff its K-th float32 squared distance <= query_radius) at full-frame sizes, with a
    certificate instead of a candidate-window assumption.

    A float64 cKDTree gives each query its ``kc`` nearest points within sqrt(r2)(1 + 1e-4) (a point
    beyond that bound cannot reach float32 d2 <= r2); they are re-ranked by the float32 distance
    (dx^2 + dy^2) + dz^2, ties by index. A query whose window is full (kc points inside the bound)
    is certified only if its window's largest float32 distance exceeds its K-th by more than the
    float32 / float64 rounding gap; every other full-window query is re-ranked over ALL points of
    its ball (query_ball_point). Returns (keep [Q] bool, idx [Q, K] int64 (valid where keep),
    stats dict)."""
    from scipy.spatial import cKDTree
    q = np.ascontiguousarray(query, F32); p = np.ascontiguousarray(points, F32)
    Q, N = len(q), len(p)
    workers = workers or torch.get_num_threads()
    bound = float(np.sqrt(np.float64(r2))) * (1 + 1e-4)
    tree = cKDTree(p.astype(np.float64))
    keep = np.zeros(Q, bool)
    idx = np.full((Q, K), -1, np.int64)
    n_redo = 0
    for s in range(0, Q, chunk):
        qq = q[s:s + chunk]
        _, cand = tree.query(qq.astype(np.float64), k=kc, distance_upper_bound=bound, workers=workers)
        cand = np.asarray(cand, np.int64)
        valid = cand < N
        cc = np.where(valid, cand, 0)
        d2 = np.where(valid, sqdist(qq[:, None, :], p[cc]), np.float32(np.inf))
        order = np.lexsort((np.where(valid, cand, N), d2), axis=1)
        d2s = np.take_along_axis(d2, order, 1)
        cs = np.take_along_axis(cand, order, 1)
        kth = d2s[:, K - 1]
        full = valid.all(1)
        # a full window holds the true top-K if no point outside it can be closer than its K-th:
        # every outside point is at float64 distance >= the window's largest, whose float32 d2
        # is within ~2^-22 relative of the float64 value
        unsure = full & ~(d2s[:, -1] > kth * np.float32(1 + 1e-5))
        kk = (kth <= np.float32(r2)) & ~unsure
        keep[s:s + len(qq)] = kk
        idx[s:s + len(qq)] = cs[:, :K]
        for i in np.nonzero(unsure)[0]:
            n_redo += 1
            ball = np.asarray(tree.query_ball_point(qq[i].astype(np.float64), bound), np.int64)
            dd = sqdist(qq[i][None, :], p[ball])
            o = np.lexsort((ball, dd))[:K]
            keep[s + i] = len(ball) >= K and dd[o[K - 1]] <= np.float32(r2)
            idx[s + i, :min(K, len(o))] = ball[o]
    return keep, idx, {"queries": Q, "survivors": int(keep.sum()), "rechecked_on_full_ball": n_redo}


def mean_min_distance(canonical_pcd, K=8, eps=1e-6):
    """temporalpoints.py:104-111: argKmin over the cloud itself (self-inclusive);
    nn_distance = sqrt(sum(delta^2) + eps); mean of column 1."""
    p = np.asarray(canonical_pcd, F32)
    _, idx = knn_kmin(p, p, K)
    pt = torch.from_numpy(p)
    nn_d = torch.sqrt(((pt[:, None, :] - pt[torch.from_numpy(idx), :]) ** 2).sum(-1) + torch.tensor(eps))
    return nn_d[:, 1].mean()


# ----------------------------------------------------------------------------------------
# seaborn.color_palette("hls", n) restatement (temporalpoints.py:692) -- parity unpinned
# ----------------------------------------------------------------------------------------

def hls_palette(n, h=0.01, l=0.6, s=0.65):
    hues = np.linspace(0, 1, n + 1)[:-1]
    hues += h
    hues %= 1
    hues -= hues.astype(int)
    return [colorsys.hls_to_rgb(hh, l, s) for hh in hues]


# ----------------------------------------------------------------------------------------
# PointWarper -- lib/pointwarper.py
# ----------------------------------------------------------------------------------------

def rodrigues(rvec: torch.Tensor):
    """pointwarper.py:118-143 (3-vector and 4-vector branches)."""
    if rvec.shape[-1] == 3:
        theta = torch.sqrt(1e-5 + torch.sum(rvec ** 2, dim=1))
        r = rvec / theta[:, None]
    elif rvec.shape[-1] == 4:
        theta = rvec[:, -1]
        r = rvec[:, :3]
        r = r / torch.sqrt(1e-5 + torch.sum(r ** 2, dim=1))[:, None]
    else:
        raise ValueError(rvec.shape)
    c = torch.cos(theta); s = torch.sin(theta)
    x, y, z = r[:, 0], r[:, 1], r[:, 2]
    R = torch.stack((
        x ** 2 + (1. - x ** 2) * c, x * y * (1. - c) - z * s, x * z * (1. - c) + y * s,
        x * y * (1. - c) + z * s, y ** 2 + (1. - y ** 2) * c, y * z * (1. - c) - x * s,
        x * z * (1. - c) - y * s, y * z * (1. - c) + x * s, z ** 2 + (1. - z ** 2) * c), dim=1)
    return R.view(-1, 3, 3), theta


def chain_product(m: torch.Tensor) -> torch.Tensor:
    """pointwarper.py:145-153: recursive halving product over dim 1."""
    L = m.shape[1]
    if L == 1:
        return m
    return chain_product(m[:, :L // 2]) @ chain_product(m[:, L // 2:])


def skeleton_tree(bones, J):
    """pointwarper.py:94-116 (``old=False``): parent_indices (J, depth) padded with -1 at
    the end, and parent_joint_ex (root -> 0)."""
    parent = {b[1]: b[0] for b in bones}
    paths = [[0]]
    for i in range(len(bones)):
        j = i + 1
        inds = []
        while j >= 0:
            inds.append(j)
            j = parent.get(j, -1)
        paths.append(inds[::-1])
    depth = max(len(x) for x in paths)
    pi = torch.full((len(paths), depth), -1, dtype=torch.long)
    for i, inds in enumerate(paths):
        pi[i, :len(inds)] = torch.tensor(inds)
    pex = torch.tensor([parent.get(i, 0) for i in range(len(paths))], dtype=torch.long)
    return pi, pex


def bone_transforms(R_t: torch.Tensor, joints: torch.Tensor, parent_indices, parent_joint_ex):
    """pointwarper.py:156-193 (``calc_rec_abs_T_fast``, the ``old`` formulation it returns)."""
    J = R_t.shape[0]
    joints_old = torch.cat((torch.zeros(1, 3), joints), 0)[parent_joint_ex + 1]
    hom = torch.tensor([0., 0., 0., 1.])
    M = torch.cat((torch.cat((R_t, joints_old[..., None] + R_t @ -joints_old[..., None]), -1),
                   hom[None, None].repeat(J, 1, 1)), -2)
    M = torch.cat((torch.eye(4)[None], M), 0)
    return chain_product(M[parent_indices + 1])[:, 0]


def transform_net(t_embed: torch.Tensor, tn: dict, J: int) -> torch.Tensor:
    """pointwarper.py:5-37: Linear/ReLU x4, final Linear without bias -> (J+1, 4)."""
    h = t_embed
    for li in range(4):
        h = torch.relu(torch.nn.functional.linear(h, tn[f"net.{2 * li}.weight"], tn[f"net.{2 * li}.bias"]))
    out = torch.nn.functional.linear(h, tn["net.8.weight"])
    return out.reshape(J + 1, 4)


def pointwarper_forward(st: dict, weights, joints, t_embed=None, rot_params=None, blend="sum"):
    """pointwarper.py:213-279 with get_frames=True, get_skeleton=True, avg_procrustes=False.

    Returns (xyz (N,3), joints_rel (J,3), G (N,4,4), joints_warped (J,3)).
    """
    J = joints.shape[0]
    if rot_params is None:
        params = transform_net(t_embed.unsqueeze(0), st["transform_net"], J)
        global_t = params[-1, :3]
        R_t, _ = rodrigues(params[:J, :])
    else:
        R_t, _ = rodrigues(rot_params)
        global_t = torch.zeros(3)
    R_t = R_t[st["sibling_mask"]]
    R_t[st["rot_mask"]] = torch.eye(3)
    bone_Ts = bone_transforms(R_t, joints, st["parent_indices"], st["parent_joint_ex"])
    if blend == "sum":
        G = (bone_Ts * weights[:, :, None, None]).sum(dim=1)
    else:   # another summation order, to measure the gradient's own float32 noise floor (tests)
        G = (weights @ bone_Ts.reshape(J, 16)).reshape(-1, 4, 4)
    xyz = st["canonical_pcd"]
    xyzh = torch.cat([xyz, torch.ones((len(xyz), 1))], -1)
    xyz = torch.bmm(G, xyzh.unsqueeze(-1)).squeeze(-1)[:, :3]
    jh = torch.cat([joints, torch.ones((J, 1))], -1)
    joints_rel = torch.bmm(bone_Ts, jh.unsqueeze(-1)).squeeze(-1)[:, :3]
    return (xyz + global_t).contiguous(), joints_rel, G, joints_rel + global_t, bone_Ts, global_t


# ----------------------------------------------------------------------------------------
# TemporalPoints -- lib/temporalpoints.py
# ----------------------------------------------------------------------------------------

def get_weights(W: torch.Tensor, theta_weight: torch.Tensor, flat_merging_rules, eps=1e-6):
    """temporalpoints.py:401-414: softmax(W/max(eps,theta)) then column merge
    out[:, i] = sum_{k: rules[k]==i} sm[:, k] (sequential in k)."""
    th = torch.max(torch.tensor(eps), theta_weight)
    sm = torch.softmax(W / th, dim=-1)
    rules = torch.as_tensor(flat_merging_rules).long()
    J = sm.shape[1]
    if torch.equal(rules, torch.arange(J)):
        return sm
    out = torch.zeros_like(sm)
    for k in range(J):
        out[:, rules[k]] += sm[:, k]
    return out


def project_point_to_image_plane(points, pose, K):
    """utils.py:435-450."""
    pts = torch.repeat_interleave(points.unsqueeze(0), len(pose), 0)
    pose = pose.inverse()
    pts = torch.bmm(pose[:, :3, :3], pts.transpose(1, 2)).transpose(1, 2) + pose[:, :3, 3:].transpose(1, 2)
    pts = torch.bmm(K, pts.transpose(1, 2)).transpose(1, 2)
    return pts[:, :, :2] / pts[:, :, 2:]


def _lin(x, st, name):
    return torch.nn.functional.linear(x, st[name + ".weight"], st.get(name + ".bias"))


def feat_net_names(st):
    """The Linear layers of feat_net in order (temporalpoints.py:123-130): feat_net.0, then
    feat_net.{2..depth-1}.0 (the hidden Sequentials), then feat_net.{depth} -- for the default
    feat_depth=4: feat_net.0, .2.0, .3.0, .4."""
    idx = []
    for k in st:
        m = re.fullmatch(r"feat_net\.(\d+)(\.0)?\.weight", k)
        if m:
            idx.append((int(m.group(1)), k[:-len(".weight")]))
    return [nm for _, nm in sorted(idx)]


def feat_net(x, st):
    """temporalpoints.py:123-130: feat_depth x [Linear + LeakyReLU(0.01)]."""
    for nm in feat_net_names(st):
        x = torch.nn.functional.leaky_relu(_lin(x, st, nm), 0.01)
    return x


def rgbnet(h, views, st):
    """tineuvox.py:65-88: feature_linears (no activation) -> cat views -> Linear/ReLU/Linear."""
    f = _lin(h, st, "rgbnet.feature_linears")
    if views is not None:
        f = torch.cat([f, views], -1)
    f = torch.relu(_lin(f, st, "rgbnet.views_linears.0"))
    return _lin(f, st, "rgbnet.views_linears.2")


def pose_embedding_net(x, st):
    for nm in ["pose_embedding_net.0", "pose_embedding_net.2.0", "pose_embedding_net.3.0",
               "pose_embedding_net.4"]:
        x = torch.nn.functional.leaky_relu(_lin(x, st, nm), 0.01)
    return x


class OracleModel:
    """CPU restatement of ``TemporalPoints`` built from a state dict (keys as in the
    reference) plus the non-state constructor arguments."""

    def __init__(self, state: dict, canonical_pcd, bones, *, stepsize=0.5, voxel_size=0.034,
                 fast_color_thres=1e-4, pose_embedding_dim=0, neighbours=8, eps=1e-6,
                 act_shift=None, voxel_size_ratio=1.0, frozen_view_dir=None,
                 mean_min_distance_value=None, merging_rules=None, sibling_mask=None,
                 rot_mask=None):
        g = lambda k: state[k].detach().cpu().float() if torch.is_tensor(state[k]) else state[k]
        self.st = {k: (v.detach().cpu() if torch.is_tensor(v) else v) for k, v in state.items()}
        self.canonical_pcd = torch.as_tensor(canonical_pcd).float().cpu()
        self.bones = [list(map(int, b)) for b in bones]
        self.joints = g("joints")
        self.J = self.joints.shape[0]
        self.W = g("weights")
        self.theta_weight = g("theta_weight")
        self.feat = g("canonical_feat")
        self.alpha_c = g("canonical_alpha")
        self.rgb_c = g("canonical_rgbs")
        self.direct_eps = g("direct_eps")
        self.rules = merging_rules if merging_rules is not None else torch.arange(self.J)
        self.stepsize = stepsize
        self.voxel_size = voxel_size
        self.fast_color_thres = fast_color_thres
        self.pose_embedding_dim = pose_embedding_dim
        self.K = neighbours
        self.eps = torch.tensor(eps)
        self.act_shift = math.log(1 / (1 - 1e-3) - 1) if act_shift is None else act_shift
        self.voxel_size_ratio = voxel_size_ratio
        self.frozen_view_dir = frozen_view_dir
        self.time_poc = torch.tensor([2.0 ** i for i in range(8)])
        self.pos_poc = torch.tensor([2.0 ** i for i in range(10)])
        self.view_poc = torch.tensor([2.0 ** i for i in range(4)])
        pi, pex = skeleton_tree(self.bones, self.J)
        self.pw = {
            "transform_net": {k[len("forward_warp.transform_net."):]: g(k) for k in state
                              if k.startswith("forward_warp.transform_net.net")},
            "sibling_mask": sibling_mask if sibling_mask is not None else torch.arange(self.J),
            "rot_mask": rot_mask if rot_mask is not None else torch.zeros(self.J, dtype=torch.bool),
            "parent_indices": pi, "parent_joint_ex": pex, "canonical_pcd": self.canonical_pcd,
        }
        self.nets = {k: g(k) for k in state if k.split(".")[0] in
                     ("feat_net", "rgbnet", "densitynet", "pose_embedding_net")}
        self.mmd = (mean_min_distance(self.canonical_pcd, neighbours, eps)
                    if mean_min_distance_value is None else torch.as_tensor(mean_min_distance_value))
        self.trace = {}

    # temporalpoints.py:401-414
    def get_weights(self):
        return get_weights(self.W, self.theta_weight, self.rules, float(self.eps))

    # temporalpoints.py:370-371
    def repose(self, rot_params):
        xyz, joints_rel, *_ = pointwarper_forward(self.pw, self.get_weights(), self.joints, rot_params=rot_params)
        return xyz, joints_rel

    def warp(self, t=None, rot_params=None):
        t_embed = poc_fre(torch.as_tensor(t).reshape(1).float(), self.time_poc) if rot_params is None else None
        weights = self.get_weights()
        return weights, pointwarper_forward(self.pw, weights, self.joints, t_embed, rot_params)

    # temporalpoints.py:373-399
    def sample_ray(self, rays_o, rays_d, near, far, stepsize, xyz_min, xyz_max):
        stepdist = stepsize * self.voxel_size
        pts, mask_out, ray_id, step_id, *_ = sample_pts_on_rays(
            rays_o.numpy(), rays_d.numpy(), xyz_min.numpy(), xyz_max.numpy(), near, far, stepdist)
        m = ~mask_out
        return pts[m], ray_id[m], step_id[m], m

    # temporalpoints.py:416-521
    def aggregate_pts(self, t_hat_pcd, Rinv, query_radius, render_kwargs, pose_embedding,
                      calc_min_max=True, knn_tree=None, bbox=None):
        R = len(render_kwargs["rays_o"])
        K = self.K
        if bbox is not None:   # calc_min_max=False: the model's xyz_min / xyz_max (temporalpoints.py:425-426)
            xyz_min, xyz_max = (torch.as_tensor(b).float() for b in bbox)
        elif calc_min_max:
            xyz_min = torch.min(t_hat_pcd, dim=0)[0] - query_radius
            xyz_max = torch.max(t_hat_pcd, dim=0)[0] + query_radius
        else:
            raise NotImplementedError("calc_min_max=False needs the TiNeuVox bbox")
        pts, ray_id, step_id, _ = self.sample_ray(render_kwargs["rays_o"], render_kwargs["rays_d"],
                                                  render_kwargs["near"], render_kwargs["far"],
                                                  render_kwargs["stepsize"], xyz_min, xyz_max)
        self.trace.update(xyz_min=xyz_min, xyz_max=xyz_max, n_inbbox=len(pts))
        if len(pts) == 0:
            return None
        tp = t_hat_pcd.numpy()
        d2, s_i = knn_kmin(pts, tp, K, use_tree=knn_tree)
        keep = np.nonzero(d2[:, -1] <= F32(query_radius))[0]
        s_i = s_i[keep]; ray_id = ray_id[keep]; step_id = step_id[keep]; pts = pts[keep]
        self.trace.update(s_i=s_i, ray_id=ray_id, step_id=step_id, keep=keep, pts=pts)
        if len(s_i) == 0:
            return None
        s_i_t = torch.from_numpy(s_i)
        ray_pts = torch.from_numpy(pts)
        rel_p = ray_pts[:, None, :] - t_hat_pcd[s_i_t, :]
        to_nn = (rel_p ** 2).sum(-1)
        features_k = self.feat[s_i_t, :]
        Rk = Rinv[s_i_t, :, :]
        # direct render (459-470), forced on at 592
        sig = self.mmd * torch.max(self.direct_eps, torch.tensor(0.))
        w_direct = torch.exp(-(to_nn ** 2) / (2 * (sig[s_i_t]) ** 2 + 1e-12))
        w_dd = (torch.tensor(1. / K) * w_direct).unsqueeze(-1)
        w_direct = (w_direct / (w_direct.sum(dim=-1) + 1e-12)[:, None]).unsqueeze(-1)
        rgbs_direct = (w_direct * self.rgb_c.clip(0, 1)[s_i_t, :]).sum(dim=1)
        alpha_direct = (w_dd * self.alpha_c.clip(0, 1)[s_i_t].unsqueeze(-1)).sum(dim=1).squeeze(-1)
        # point-NeRF aggregation (472-494)
        w = 1 / (to_nn + self.eps)
        w = (w / w.sum(dim=-1)[:, None]).unsqueeze(-1)
        rel_c = torch.bmm(Rk[..., :3, :3].reshape(-1, 3, 3), rel_p.reshape(-1, 3).unsqueeze(-1)).squeeze(-1)
        x = [poc_fre(rel_c, self.pos_poc), features_k.reshape(-1, features_k.shape[-1])]
        if pose_embedding is not None:
            x.append(pose_embedding.expand(len(x[0]), -1))
        out = feat_net(torch.cat(x, -1), self.nets)
        h = (out.reshape(len(s_i), K, -1) * w).sum(dim=1)
        density = _lin(h, self.nets, "densitynet").squeeze(-1)
        interval = render_kwargs["stepsize"] * self.voxel_size_ratio
        _, alpha = raw2alpha(density.numpy(), self.act_shift, interval)
        alpha = torch.from_numpy(alpha)
        if self.frozen_view_dir is not None:
            views = poc_fre(torch.as_tensor(self.frozen_view_dir).float(), self.view_poc)[None].expand(len(ray_id), -1)
        else:
            views = poc_fre(render_kwargs["viewdirs"], self.view_poc)[torch.from_numpy(ray_id)]
        rgbs = torch.sigmoid(rgbnet(h, views, self.nets))
        lbsw = (self._last_weights[s_i_t, :] * w).sum(dim=1)
        self.trace.update(to_nn=to_nn, h=h, density=density, alpha=alpha, rgbs=rgbs,
                          alpha_direct=alpha_direct, rgbs_direct=rgbs_direct, lbsw=lbsw)
        return rgbs, alpha, rgbs_direct, alpha_direct, lbsw, ray_id, step_id, R

    # temporalpoints.py:540-712
    @torch.no_grad()
    def forward(self, t, render_depth=False, render_kwargs=None, query_radius=0.01,
                render_weights=False, rot_params=None, poses=None, Ks=None, get_skeleton=False,
                calc_min_max=True, perm=None, knn_tree=None, t_hat_override=None, bbox=None):
        """``t_hat_override``: render against a given warped cloud (e.g. the GPU's) so that a
        1-ulp difference in the warp cannot flip a borderline kNN-radius decision. ``bbox`` =
        (xyz_min, xyz_max): the sampling bbox of calc_min_max=False (the model's stored bbox)."""
        assert (t is None) ^ (rot_params is None)
        rk = {k: (v.detach().cpu() if torch.is_tensor(v) else v) for k, v in render_kwargs.items()}
        weights, (t_hat, joints_rel, G, joints_w, bone_Ts, global_t) = self.warp(t, rot_params)
        if t_hat_override is not None:
            t_hat = torch.as_tensor(t_hat_override).detach().cpu().float().contiguous()
        self._last_weights = weights
        Rinv = torch.inverse(G)
        self.trace = dict(t_hat_pcd=t_hat, G=G, Rinv=Rinv, bone_Ts=bone_Ts, weights=weights,
                          joints_rel=joints_rel, global_t=global_t)
        delta = (self.joints - joints_rel)
        pose_embedding = (pose_embedding_net(poc_fre(delta, self.pos_poc).view(1, -1), self.nets)
                          if self.pose_embedding_dim > 0 else None)
        self.trace["pose_embedding"] = pose_embedding
        joints = bones = None
        if get_skeleton:
            joints = project_point_to_image_plane(joints_w, poses.cpu(), Ks.cpu().float())
            bones = self.bones
        R = len(rk["rays_o"])
        bg = rk["bg"]
        res = self.aggregate_pts(t_hat, Rinv, query_radius, rk, pose_embedding, calc_min_max, knn_tree, bbox)
        if res is None:  # NoPointsException fallback (598-609)
            return {"rgb_marched": torch.ones(R, 3) * bg, "rgb_marched_direct": torch.ones(R, 3) * bg,
                    "depth": torch.zeros(R), "weights": torch.ones(R, 3) * bg, "t_hat_pcd": t_hat,
                    "alphainv_last": None, "grid": None, "joints": joints, "bones": bones}
        rgbs, alpha, rgbs_d, alpha_d, lbsw, ray_id, step_id, N = res
        col_all = None
        if render_weights:
            # weight-visualisation colour per kept sample (temporalpoints.py:690-701)
            wmask = weights.sum(dim=0) > 0
            cols = torch.tensor(hls_palette(int(wmask.sum())))
            if perm is None:
                gen = torch.Generator(); gen.manual_seed(0)
                perm = torch.randperm(cols.shape[0], generator=gen)
            cols = cols[perm]
            col = 0
            for ci, wi in enumerate(torch.where(wmask)[0]):
                col = col + cols[ci, None] * lbsw[:, wi, None]
            col_all = torch.as_tensor(col).float().numpy()
            self.trace.update(col=col_all, perm=perm)
        thr = F32(self.fast_color_thres)
        ray_id_d = ray_id.copy()
        a = alpha.numpy(); ad = alpha_d.numpy()
        rgbs = rgbs.numpy(); rgbs_d = rgbs_d.numpy()
        col = col_all if col_all is not None else np.zeros((len(a), 3), F32)
        if self.fast_color_thres > 0:
            m = a > thr
            ray_id, step_id, a, rgbs, col = ray_id[m], step_id[m], a[m], rgbs[m], col[m]
            md = ad > thr
            ray_id_d, ad, rgbs_d = ray_id_d[md], ad[md], rgbs_d[md]
        w, _, last, *_ = alpha2weight(a, ray_id, N)
        wd, _, last_d, *_ = alpha2weight(ad, ray_id_d, N)
        if self.fast_color_thres > 0:
            m = w > thr
            w, a, ray_id, step_id, rgbs, col = w[m], a[m], ray_id[m], step_id[m], rgbs[m], col[m]
            md = wd > thr
            ray_id_d, ad, rgbs_d, wd = ray_id_d[md], ad[md], rgbs_d[md], wd[md]
        rgb_marched = segment_sum((w[:, None] * rgbs).astype(F32), ray_id, N)
        rgb_marched = (rgb_marched + (last[:, None] * F32(bg)).astype(F32)).astype(F32)
        rgb_marched_d = segment_sum((wd[:, None] * rgbs_d).astype(F32), ray_id_d, N)
        rgb_marched_d = (rgb_marched_d + (last_d[:, None] * F32(bg)).astype(F32)).astype(F32)
        ret = {"t_hat_pcd": t_hat, "rgb_marched": torch.from_numpy(rgb_marched),
               "alphainv_last": torch.from_numpy(last), "alphainv_last_direct": torch.from_numpy(last_d),
               "grid": None, "rgb_marched_direct": torch.from_numpy(rgb_marched_d),
               "joints": joints, "bones": bones}
        if render_depth:
            ret["depth"] = torch.from_numpy(segment_sum((w * step_id.astype(F32)).astype(F32), ray_id, N))
        if render_weights:
            wm = segment_sum((w[:, None] * col).astype(F32), ray_id, N)
            ret["weights"] = torch.from_numpy((wm + (last[:, None] * F32(bg)).astype(F32)).astype(F32))
        return ret


# ----------------------------------------------------------------------------------------
# Training-mode forward -- run.py:574-716 renders with autograd on.
# The render_utils kernels enter autograd through their restated forward/backward pairs
# (tineuvox.py:627-670), everything else is the reference's torch expressions.
# ----------------------------------------------------------------------------------------

class _Raw2AlphaFn(torch.autograd.Function):
    """tineuvox.py:646-670 over raw2alpha / raw2alpha_backward above."""

    @staticmethod
    def forward(ctx, density, shift, interval):
        e, a = raw2alpha(density.detach().numpy(), shift, interval)
        ctx.save_for_backward(torch.from_numpy(np.ascontiguousarray(e)))
        ctx.interval = interval
        return torch.from_numpy(np.ascontiguousarray(a))

    @staticmethod
    def backward(ctx, g):
        e, = ctx.saved_tensors
        return torch.from_numpy(raw2alpha_backward(e.numpy(), g.contiguous().numpy(), ctx.interval)), None, None


class _Alphas2WeightsFn(torch.autograd.Function):
    """tineuvox.py:627-643 over alpha2weight / alpha2weight_backward above."""

    @staticmethod
    def forward(ctx, alpha, ray_id, n_rays):
        w, T, last, i_s, i_e = alpha2weight(alpha.detach().numpy(), ray_id.numpy(), n_rays)
        ctx.saved = (alpha.detach().numpy(), w, T, last, i_s, i_e)
        ctx.n_rays = n_rays
        return torch.from_numpy(w), torch.from_numpy(last)

    @staticmethod
    def backward(ctx, gw, gl):
        a, w, T, last, i_s, i_e = ctx.saved
        g = alpha2weight_backward(a, w, T, last, i_s, i_e, ctx.n_rays, gw.contiguous().numpy(),
                                  gl.contiguous().numpy())
        return torch.from_numpy(g), None, None


def oracle_trainable(om: "OracleModel") -> dict:
    """Make the OracleModel's parameters autograd leaves; returns them under the reference's
    state-dict names."""
    params = {"weights": om.W, "theta_weight": om.theta_weight, "canonical_feat": om.feat,
              "canonical_alpha": om.alpha_c, "canonical_rgbs": om.rgb_c, "direct_eps": om.direct_eps,
              "joints": om.joints}
    for k, v in om.nets.items():
        params[k] = v
    for k, v in om.pw["transform_net"].items():
        params["forward_warp.transform_net." + k] = v
    for v in params.values():
        v.requires_grad_(True)
    return params


def oracle_forward_train(om: "OracleModel", t, render_kwargs, query_radius=0.01, xyz_min=None, xyz_max=None,
                         knn_tree=None, blend="sum", jitter=0.0, jitter_seed=0, t_hat_snap=None):
    """temporalpoints.py:540-712 + aggregate_pts (416-521) with autograd on (render_pcd_direct
    forced, no depth / weights outputs). ``xyz_min/xyz_max`` fix the sampling bbox (else the
    cloud's, 423-427). ``t_hat_snap``: see below. Returns rgb_marched, rgb_marched_direct,
    t_hat_pcd, last_weights."""
    rk = {k: (v.detach().cpu() if torch.is_tensor(v) else v) for k, v in render_kwargs.items()}
    R = len(rk["rays_o"]); K = om.K; bg = rk["bg"]
    t_embed = poc_fre(torch.as_tensor(t).reshape(1).float(), om.time_poc)
    weights = om.get_weights()
    t_hat, joints_rel, G, _, _, _ = pointwarper_forward(om.pw, weights, om.joints, t_embed, None, blend=blend)
    Rinv = torch.inverse(G)
    gen = torch.Generator().manual_seed(jitter_seed)

    def jit(x):
        # relative ulp-scale perturbation of the float32 quantities another device computes with
        # another summation order (warped cloud, 3x3 inverses, joint offsets): tests use it to
        # measure the gradient's own float32 noise floor
        if not jitter:
            return x
        sgn = torch.randint(0, 3, x.shape, generator=gen).float() - 1.0
        return x + x.detach() * (jitter * sgn)
    if t_hat_snap is not None:
        # take another device's warped cloud as the value (straight-through: the gradient still
        # flows through this oracle's own LBS), so a 1-ulp difference cannot flip a kNN decision
        t_hat = t_hat + (torch.as_tensor(t_hat_snap).detach().cpu().float() - t_hat).detach()
    t_hat = jit(t_hat)
    Rinv = jit(Rinv)
    pose_embedding = None
    if om.pose_embedding_dim > 0:
        delta = jit((om.joints - joints_rel).clone().detach())
        pose_embedding = pose_embedding_net(poc_fre(delta, om.pos_poc).view(1, -1), om.nets)
    if xyz_min is None:
        xyz_min = torch.min(t_hat.detach(), dim=0)[0] - query_radius
        xyz_max = torch.max(t_hat.detach(), dim=0)[0] + query_radius
    pts, ray_id, step_id, _ = om.sample_ray(rk["rays_o"], rk["rays_d"], rk["near"], rk["far"], rk["stepsize"],
                                            torch.as_tensor(xyz_min).cpu().float(),
                                            torch.as_tensor(xyz_max).cpu().float())
    d2, s_i = knn_kmin(pts, t_hat.detach().numpy(), K, use_tree=knn_tree)
    keep = np.nonzero(d2[:, -1] <= F32(query_radius))[0]
    s_i = torch.from_numpy(s_i[keep]); ray_id = torch.from_numpy(ray_id[keep]); ray_pts = torch.from_numpy(pts[keep])
    om.trace = dict(s_i=s_i, ray_id=ray_id, n_inbbox=len(pts), t_hat_pcd=t_hat.detach())
    rel_p = ray_pts[:, None, :] - t_hat[s_i, :]
    to_nn = (rel_p ** 2).sum(-1)
    sig = om.mmd * torch.max(om.direct_eps, torch.tensor(0.))
    w_direct = torch.exp(-(to_nn ** 2) / (2 * (sig[s_i]) ** 2 + 1e-12))
    w_dd = (torch.tensor(1. / K) * w_direct).unsqueeze(-1)
    w_direct = (w_direct / (w_direct.sum(dim=-1) + 1e-12)[:, None]).unsqueeze(-1)
    rgbs_d = (w_direct * om.rgb_c.clip(0, 1)[s_i, :]).sum(dim=1)
    alpha_d = (w_dd * om.alpha_c.clip(0, 1)[s_i].unsqueeze(-1)).sum(dim=1).squeeze(-1)
    w = 1 / (to_nn + om.eps)
    w = (w / w.sum(dim=-1)[:, None]).unsqueeze(-1)
    rel_c = torch.bmm(Rinv[s_i][..., :3, :3].reshape(-1, 3, 3), rel_p.reshape(-1, 3).unsqueeze(-1)).squeeze(-1)
    x = [poc_fre(rel_c, om.pos_poc), om.feat[s_i].reshape(-1, om.feat.shape[-1])]
    if pose_embedding is not None:
        x.append(pose_embedding.expand(len(x[0]), -1))
    h = (feat_net(torch.cat(x, -1), om.nets).reshape(len(s_i), K, -1) * w).sum(dim=1)
    density = _lin(h, om.nets, "densitynet").squeeze(-1)
    alpha = _Raw2AlphaFn.apply(density.contiguous(), om.act_shift, rk["stepsize"] * om.voxel_size_ratio)
    views = poc_fre(rk["viewdirs"], om.view_poc)[ray_id]
    rgbs = torch.sigmoid(rgbnet(h, views, om.nets))
    thr = om.fast_color_thres
    ray_id_d = ray_id
    if thr > 0:
        m = torch.where(alpha > thr)[0]
        ray_id, alpha, rgbs = ray_id[m], alpha[m], rgbs[m]
        md = torch.where(alpha_d > thr)[0]
        ray_id_d, alpha_d, rgbs_d = ray_id_d[md], alpha_d[md], rgbs_d[md]
    wr, last = _Alphas2WeightsFn.apply(alpha.contiguous(), ray_id, R)
    wd, last_d = _Alphas2WeightsFn.apply(alpha_d.contiguous(), ray_id_d, R)
    if thr > 0:
        m = torch.where(wr > thr)[0]
        wr, ray_id, rgbs = wr[m], ray_id[m], rgbs[m]
        md = torch.where(wd > thr)[0]
        wd, ray_id_d, rgbs_d = wd[md], ray_id_d[md], rgbs_d[md]
    rgb = torch.zeros(R, 3).index_add(0, ray_id, wr.unsqueeze(-1) * rgbs) + last.unsqueeze(-1) * bg
    rgb_d = torch.zeros(R, 3).index_add(0, ray_id_d, wd.unsqueeze(-1) * rgbs_d) + last_d.unsqueeze(-1) * bg
    return {"rgb_marched": rgb, "rgb_marched_direct": rgb_d, "t_hat_pcd": t_hat, "last_weights": weights}
