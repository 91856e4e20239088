"""Known-answer tests for the oracle's restatement of render_utils_kernel.cu, derived by
hand from the kernel source; these pin the parts no reference run can."""
import numpy as np

from oracle import apn_oracle as O

F32 = np.float32
LO = np.array([-1, -1, -1], F32)
HI = np.array([1, 1, 1], F32)


def test_axis_parallel_ray_zero_components():
    # d = (1,0,0): y/z components replaced by 1e-6 (render_utils_kernel.cu:23-25)
    o = np.array([[-3, 0, 0]], F32); d = np.array([[1, 0, 0]], F32)
    t_min, t_max = O.infer_t_minmax(o, d, LO, HI, 0.0, 10.0)
    assert t_min[0] == F32(2) and t_max[0] == F32(4)
    n = O.infer_n_samples(t_min, t_max, 0.5)
    assert n[0] == 4          # exact multiple: ceil(2/0.5) = 4


def test_missing_ray_gets_one_masked_sample():
    o = np.array([[-3, 5, 0]], F32); d = np.array([[1, 0, 0]], F32)
    pts, mo, rid, sid, n, t_min, t_max = O.sample_pts_on_rays(o, d, LO, HI, 0.5, 10.0, 0.1)
    assert n[0] == 1 and len(pts) == 1 and mo[0]
    assert rid[0] == 0 and sid[0] == 0


def test_step_ids_and_positions():
    o = np.array([[-3, 0, 0], [0, -3, 0.5]], F32); d = np.array([[2, 0, 0], [0, 1, 0]], F32)
    pts, mo, rid, sid, n, t_min, t_max = O.sample_pts_on_rays(o, d, LO, HI, 0.0, 100.0, 0.25)
    assert list(n) == [4, 8]
    assert list(rid) == [0] * 4 + [1] * 8
    assert list(sid) == list(range(4)) + list(range(8))
    # start = o + d*t_min (unnormalised d), dir = d/|d|
    assert np.allclose(pts[:4, 0], [-1, -0.75, -0.5, -0.25])
    assert np.allclose(pts[4:, 1], np.arange(8) * 0.25 - 1)


def test_raw2alpha_overflow_gives_one():
    e, a = O.raw2alpha(np.array([1e4, -1e4, 0.0], F32), -6.9, 0.5)
    assert np.isinf(e[0]) and a[0] == F32(1)
    assert a[1] == F32(0)
    assert np.isclose(a[2], 1 - (1 + np.exp(np.float32(-6.9))) ** -0.5, rtol=1e-6)


def test_alpha2weight_early_exit_and_empty_rays():
    alpha = np.array([0.5, 0.9, 0.99, 0.5, 0.5, 0.3], F32)
    rid = np.array([1, 1, 1, 1, 1, 3], np.int64)
    w, T, last, i_s, i_e = O.alpha2weight(alpha, rid, 5)
    # ray 1: T = 1, .5, .05, 5e-4 (<1e-3 -> break after the 3rd sample, which is written)
    assert np.allclose(T[:3], [1, 0.5, 0.05], rtol=1e-6)
    assert np.allclose(w[:3], [0.5, 0.45, 0.0495], rtol=1e-6)
    assert w[3] == 0 and w[4] == 0 and T[3] == 1 and T[4] == 1
    assert i_s[1] == 0 and i_e[1] == 3
    assert np.isclose(last[1], np.float32(np.float64(np.float32(0.05)) * (1 - np.float64(np.float32(0.99)))))
    # empty rays keep alphainv_last = 1
    assert last[0] == 1 and last[2] == 1 and last[4] == 1
    assert np.isclose(last[3], 0.7)
    assert i_s[3] == 5 and i_e[3] == 6


def test_alpha2weight_double_precision_update():
    # T_cum is updated in double and narrowed (render_utils_kernel.cu:450)
    alpha = np.full(50, 0.1, F32)
    rid = np.zeros(50, np.int64)
    w, T, last, *_ = O.alpha2weight(alpha, rid, 1)
    tc = F32(1)
    for i in range(50):
        assert T[i] == tc
        tc = F32(np.float64(tc) * (1.0 - np.float64(F32(0.1))))
        if np.float64(tc) < 1e-3:
            break
    assert last[0] == tc


def test_segment_sum_sequential():
    src = np.array([1e8, 1, -1e8, 1], F32)
    out = O.segment_sum(src, np.array([0, 0, 0, 1]), 2)
    # sequential float32: (1e8 + 1) - 1e8 = 0
    assert out[0] == F32(0) and out[1] == F32(1)


def test_knn_ties_broken_by_index():
    pts = np.array([[1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, 0, 0.5]], F32)
    d2, idx = O.knn_kmin(np.zeros((1, 3), F32), pts, 3)
    assert list(idx[0]) == [3, 0, 1] and d2[0, 0] == F32(0.25)


def test_raw2alpha_backward_is_the_derivative():
    """raw2alpha_backward (render_utils_kernel.cu:395-406) against float64 autograd of the
    forward alpha = 1 - (1 + exp(d + shift))^(-interval); the clamp min(exp, 1e10) only bites
    past d + shift ~ 23 (where the true derivative is ~interval * e^(-interval*(d+shift)))."""
    import torch
    rng = np.random.default_rng(0)
    shift, interval = -6.906755, 0.5
    d = rng.uniform(-10, 15, 2000).astype(np.float32)
    gb = rng.normal(size=2000).astype(np.float32)
    e, _ = O.raw2alpha(d, shift, interval)
    g = O.raw2alpha_backward(e, gb, interval)
    dt = torch.tensor(d, dtype=torch.float64, requires_grad=True)
    alpha = 1 - (1 + torch.exp(dt + np.float64(np.float32(shift)))) ** (-interval)
    alpha.backward(torch.tensor(gb, dtype=torch.float64))
    ref = dt.grad.numpy()
    assert np.allclose(g, ref, rtol=2e-6, atol=1e-12)
    # clamp: exp_d beyond 1e10 is replaced by 1e10 in the product
    big = np.array([1e12], np.float32)
    gc = O.raw2alpha_backward(big, np.ones(1, np.float32), interval)
    expect = 1e10 * np.float64(np.power(np.float32(1) + big[0], np.float32(-interval - 1))) * interval
    assert np.isclose(gc[0], expect, rtol=1e-6)


def test_alpha2weight_backward_is_the_derivative():
    """alpha2weight_backward (render_utils_kernel.cu:507-528) against float64 autograd of
    sum(gw * w) + sum(gl * alphainv_last) for rays that never reach the T < 1e-3 break; a ray
    that does break gets zero gradient past its i_end; empty rays give nothing."""
    import torch
    rng = np.random.default_rng(1)
    counts = [5, 0, 9, 1, 7]
    rid = np.concatenate([np.full(c, r) for r, c in enumerate(counts)]).astype(np.int64)
    a = rng.uniform(0.0, 0.3, len(rid)).astype(np.float32)
    R = len(counts)
    w, T, last, i_s, i_e = O.alpha2weight(a, rid, R)
    gw = rng.normal(size=len(a)).astype(np.float32)
    gl = rng.normal(size=R).astype(np.float32)
    g = O.alpha2weight_backward(a, w, T, last, i_s, i_e, R, gw, gl)
    at = torch.tensor(a, dtype=torch.float64, requires_grad=True)
    loss = 0
    for r in range(R):
        seg = at[rid == r]
        if len(seg) == 0:
            continue
        trans = torch.cumprod(torch.cat([torch.ones(1, dtype=torch.float64), 1 - seg]), 0)
        loss = loss + (torch.tensor(gw[rid == r], dtype=torch.float64) * seg * trans[:-1]).sum() + gl[r] * trans[-1]
    loss.backward()
    assert np.allclose(g, at.grad.numpy(), rtol=1e-5, atol=1e-6)
    # early exit: a saturating ray stops at the sample that drops T below 1e-3
    a2 = np.array([0.5, 0.999, 0.5, 0.5], np.float32)
    rid2 = np.zeros(4, np.int64)
    w2, T2, l2, s2, e2 = O.alpha2weight(a2, rid2, 1)
    g2 = O.alpha2weight_backward(a2, w2, T2, l2, s2, e2, 1, np.ones(4, np.float32), np.ones(1, np.float32))
    assert e2[0] == 2 and g2[2] == 0 and g2[3] == 0 and g2[0] != 0


def test_adam_oracle_first_step_and_float64():
    """adam_upd (adam_upd_kernel.cu:8-82): from zero state the first step moves every
    coordinate by ~lr * sign(g); five steps track a float64 evaluation of the same recurrence."""
    rng = np.random.default_rng(2)
    n = 1000
    p = rng.normal(size=n).astype(np.float32); p0 = p.copy()
    m = np.zeros(n, np.float32); v = np.zeros(n, np.float32)
    g = rng.normal(size=n).astype(np.float32)
    O.adam_upd(p, g, m, v, 1, 0.9, 0.99, 1e-3, 1e-8)
    assert np.allclose(p0 - p, 1e-3 * np.sign(g), rtol=1e-4, atol=1e-6)   # p - 1e-3 rounds at ulp(p) <= 2.4e-7
    p64, m64, v64 = p0.astype(np.float64), np.zeros(n), np.zeros(n)
    p = p0.copy(); m[:] = 0; v[:] = 0
    for step in range(1, 6):
        g = rng.normal(size=n).astype(np.float32)
        O.adam_upd(p, g, m, v, step, 0.9, 0.99, 1e-3, 1e-8)
        m64 = 0.9 * m64 + 0.1 * g; v64 = 0.99 * v64 + 0.01 * g.astype(np.float64) ** 2
        ss = 1e-3 * np.sqrt(1 - 0.99 ** step) / (1 - 0.9 ** step)
        p64 = p64 - ss * m64 / (np.sqrt(v64) + 1e-8)
    assert np.allclose(p, p64, rtol=1e-5, atol=1e-6)
    # masked: zero gradients leave parameter and moments untouched
    p = p0.copy(); m = np.ones(n, np.float32); v = np.ones(n, np.float32)
    g = np.zeros(n, np.float32); g[::3] = 1.0
    O.adam_upd(p, g, m, v, 1, 0.9, 0.99, 1e-3, 1e-8, masked=True)
    keep = g == 0
    assert np.array_equal(p[keep], p0[keep]) and np.all(m[keep] == 1) and np.all(p[~keep] != p0[~keep])


def test_total_variation_oracle_direct():
    """total_variation_add_grad (total_variation_kernel.cu:13-35) against a per-element loop of
    the kernel's expression (float64 accumulate is exact here: the terms are small multiples)."""
    rng = np.random.default_rng(4)
    P = rng.normal(size=(1, 2, 3, 4, 5)).astype(np.float32)
    G = rng.normal(size=P.shape).astype(np.float32)
    G.reshape(-1)[::4] = 0
    for dense in (True, False):
        got = G.copy()
        O.total_variation_add_grad(P, got, 1.0, 2.0, 3.0, dense)
        ref = G.copy().reshape(-1)
        p = P.reshape(-1)
        C, I, J, K = P.shape[1:]
        wy, wz = np.float32(2.0) / np.float32(6), np.float32(3.0) / np.float32(6)
        cl = lambda x: min(max(x, -1.0), 1.0)
        for idx in range(p.size):
            if not dense and ref[idx] == 0:
                continue
            k = idx % K; j = idx // K % J; i = idx // K // J % I
            acc = 0.0
            acc += 0 if k == 0 else wz * cl(p[idx] - p[idx - 1])
            acc += 0 if k == K - 1 else wz * cl(p[idx] - p[idx + 1])
            acc += 0 if j == 0 else wy * cl(p[idx] - p[idx - K])
            acc += 0 if j == J - 1 else wy * cl(p[idx] - p[idx + K])
            acc += 0 if i == 0 else wz * cl(p[idx] - p[idx - K * J])
            acc += 0 if i == I - 1 else wz * cl(p[idx] - p[idx + K * J])
            ref[idx] += acc
        assert np.allclose(got.reshape(-1), ref, rtol=1e-6, atol=1e-6)
