"""Neighbour-graph losses of the training step (temporalpoints.py:714-716 weight TV, 723-725 ARAP)
as fused HIP kernels (apn_nbr_tv_loss / apn_arap_loss + their gather-only backward).

The reference's own torch expressions, run under float64 autograd on the CPU with the same
neighbour graph, are the checker. Bars: loss within 1e-6 relative (ARAP 1e-5: a 2.4M-term fp32
sum); TV gradients within 1e-6 relative (its sign terms are exact, ties included: only the
fp32 product dL/count * s rounds); ARAP gradients within 1e-5 of dL per component; bit-identical results across repeated runs (no atomics)."""
import pytest
import torch

from apn_amd.train import ArapLoss, NbrTVLoss, reverse_csr


def _graph(n, k, seed, device="cpu"):
    g = torch.Generator().manual_seed(seed)
    nn = torch.randint(0, n, (n, k), generator=g)
    nn[:, 0] = torch.arange(n)   # self first, as the kNN graph is
    return nn.to(device)


def test_reverse_csr_cpu():
    nn = _graph(500, 8, 0)
    rev_ptr, rev_edge = reverse_csr(nn)
    assert rev_ptr[0] == 0 and rev_ptr[-1] == nn.numel()
    flat = nn.reshape(-1)
    for i in (0, 1, 17, 499):
        e = rev_edge[rev_ptr[i]:rev_ptr[i + 1]]
        assert torch.all(flat[e] == i)
        assert torch.all(e[1:] > e[:-1])                 # ascending edge ids within a target
        assert len(e) == int((flat == i).sum())


def _tv_ref(w, nn):
    diff = w[:, None, :] - w[nn, :]
    return torch.abs(diff).mean()


def _arap_ref(x, nn, d0, eps):
    wd = torch.sqrt((x[:, None, :] - x[nn, :]).pow(2).sum(-1) + eps)
    return (d0 - wd).abs().sum()


@pytest.mark.gpu
@pytest.mark.autograd
@pytest.mark.parametrize("n,J", [(1, 8), (777, 24), (20000, 24), (5000, 48)])
def test_nbr_tv_loss_vs_torch(n, J):
    dev = torch.device("cuda")
    K = 8 if n >= 8 else 1
    nn = _graph(n, K, n + J)
    g = torch.Generator().manual_seed(J)
    w = torch.softmax(torch.randn(n, J, generator=g) * 3, -1)
    w[: n // 10] = w[0]      # exact ties: sign(0) = 0 on both sides
    w64 = w.double().requires_grad_(True)
    ref = _tv_ref(w64, nn)
    ref.backward(torch.tensor(10.0, dtype=torch.float64))
    rp, re = reverse_csr(nn.to(dev))
    wd = w.to(dev).requires_grad_(True)
    loss = NbrTVLoss.apply(wd, nn.to(dev), rp, re)
    (10.0 * loss).backward()
    assert abs(float(loss.detach()) - float(ref.detach())) <= 1e-6 * max(1.0, float(ref.detach()))
    scale = 10.0 / (n * K * J)
    assert torch.allclose(wd.grad.cpu().double(), w64.grad, rtol=1e-6, atol=1e-6 * scale)
    # deterministic: a second run is bit-identical
    wd2 = w.to(dev).requires_grad_(True)
    l2 = NbrTVLoss.apply(wd2, nn.to(dev), rp, re)
    (10.0 * l2).backward()
    assert float(l2.detach()) == float(loss.detach()) and torch.equal(wd2.grad, wd.grad)


@pytest.mark.gpu
@pytest.mark.autograd
@pytest.mark.parametrize("n", [1, 777, 20000, 300000])
def test_arap_loss_vs_torch(n):
    from apn_amd.ops import knn_points
    dev = torch.device("cuda")
    K = 8 if n >= 8 else 1
    g = torch.Generator().manual_seed(n)
    pcd = torch.rand(n, 3, generator=g)
    eps = float(torch.tensor(1e-6))
    _, nn = knn_points(pcd.to(dev), pcd.to(dev), K)
    nn = nn.cpu()
    d0 = torch.sqrt(((pcd[:, None, :] - pcd[nn, :]) ** 2).sum(-1) + torch.tensor(1e-6))
    warped = pcd + 0.01 * torch.randn(n, 3, generator=g)
    x64 = warped.double().requires_grad_(True)
    ref = _arap_ref(x64, nn, d0.double(), eps)
    ref.backward(torch.tensor(5e-3, dtype=torch.float64))
    rp, re = reverse_csr(nn.to(dev))
    xd = warped.to(dev).requires_grad_(True)
    loss = ArapLoss.apply(xd, nn.to(dev), d0.to(dev), eps, rp, re)
    (5e-3 * loss).backward()
    assert abs(float(loss.detach()) - float(ref.detach())) <= 1e-5 * max(1.0, abs(float(ref.detach())))
    gref = x64.grad
    # per-edge terms are +-dL * diff/s (|.| <= dL); fp32 rounding of diff/s ~1e-7 relative per
    # term, summed over <= K + in-degree terms
    tol = 5e-3 * 1e-5
    bad = ((xd.grad.cpu().double() - gref).abs() > tol).float().mean()
    assert float(bad) <= 1e-4, float(bad)   # sign flips where d0 == s within rounding
    xd2 = warped.to(dev).requires_grad_(True)
    l2 = ArapLoss.apply(xd2, nn.to(dev), d0.to(dev), eps, rp, re)
    (5e-3 * l2).backward()
    assert float(l2.detach()) == float(loss.detach()) and torch.equal(xd2.grad, xd.grad)


@pytest.mark.gpu
@pytest.mark.autograd
def test_temporalpoints_losses_route_to_hip():
    """The TemporalPoints methods take the fused path and agree with the reference expressions on
    the model's own kNN graph."""
    import sys
    from golden_io import Golden
    from model_io import model_from_golden
    g = Golden("G1")
    m = model_from_golden(g, "cuda")
    nn_i, nn_d = m.nn_i, m.nn_distance
    m._last_weights = torch.softmax(m.weights.detach(), -1).requires_grad_(True)
    tv = m.get_neighbour_weight_tv_loss()
    assert tv.grad_fn is not None and "NbrTVLoss" in type(tv.grad_fn).__name__
    lw = m._last_weights.detach()
    assert abs(float(tv.detach()) - float(_tv_ref(lw.double(), nn_i))) < 1e-6
    x = m.canonical_pcd.detach().clone().requires_grad_(True)
    arap = m.get_arap_loss(x)
    assert "ArapLoss" in type(arap.grad_fn).__name__
    assert abs(float(arap.detach()) - float(_arap_ref(x.detach().double(), nn_i, nn_d.double(), float(m.eps)))) < 1e-4
    assert "apn_amd" in sys.modules


@pytest.mark.gpu
@pytest.mark.autograd
@pytest.mark.parametrize("slope", [None, 0.01, 0.0])
@pytest.mark.parametrize("M,K,N", [(1, 155, 128), (300, 128, 128), (4096 * 2 + 5, 155, 128), (212736 + 7, 128, 128),
                                   (26001, 128, 1), (1, 160, 64), (777, 33, 256), (5, 256, 97)])
def test_gemm_linear_vs_float64(M, K, N, slope):
    """apn_amd.linear (the training step's Linear layers on apn_gemm_f32 / apn_gemm_f32_splitk:
    feat_net, densitynet (N = 1), rgbnet, TransformNet (M = 1), with LeakyReLU / ReLU / no
    activation fused): output and all three gradients within fp32 rounding of float64. The
    activation's kink is taken from the fp32 output on both sides (a pre-activation within an ulp
    of 0 may have either sign), so the check isolates the products and sums."""
    from apn_amd.linear import _GemmLinear
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(M * 7 + N)
    x = torch.randn(M, K, generator=g)
    w = torch.randn(N, K, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g)
    dy = torch.randn(M, N, generator=g)
    ps = [t.to(dev).requires_grad_(True) for t in (x, w, b)]
    y = _GemmLinear.apply(*ps, slope)
    y.backward(dy.to(dev))
    x64, w64, b64 = (t.double().to(dev) for t in (x, w, b))
    pre = x64 @ w64.t() + b64
    if slope is None:
        y64, m64 = pre, torch.ones_like(pre)
    else:
        pos = y.detach().double() > 0
        y64 = torch.where(pos, pre, pre * slope)
        m64 = torch.where(pos, torch.ones_like(pre), torch.full_like(pre, slope))
    gd = dy.double().to(dev) * m64
    refs = {"y": y64, "x": gd @ w64, "w": gd.t() @ x64, "b": gd.sum(0)}
    for name, a in (("y", y), ("x", ps[0].grad), ("w", ps[1].grad), ("b", ps[2].grad)):
        r = refs[name]
        err = float((a.detach().double() - r.detach()).abs().max() / r.detach().abs().max().clamp_min(1e-30))
        assert err < 2e-6, (name, err)


def test_gemm_linear_sequential_matches_torch_on_cpu():
    """linear.sequential pairs each Linear with the LeakyReLU / ReLU after it (nested Sequentials
    flattened, the feat_net layout of temporalpoints.py:299-303); on CPU tensors it is torch's own
    forward, so it must equal the module bit for bit."""
    from apn_amd.linear import sequential
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(20, 16), torch.nn.LeakyReLU(),
                              torch.nn.Sequential(torch.nn.Linear(16, 16), torch.nn.ReLU()),
                              torch.nn.Linear(16, 8))
    x = torch.randn(5, 20)
    assert torch.equal(sequential(net, x), net(x))


@pytest.mark.gpu
@pytest.mark.autograd
@pytest.mark.parametrize("n,J", [(1, 1), (777, 24), (300000, 24)])
def test_weight_sparsity_loss_vs_float64(n, J):
    """SparsityLoss (temporalpoints.py:718-721) vs the float64 autograd of the reference
    expression, with exact 0 / 1 weights (log(eps) terms) included."""
    from apn_amd.train import SparsityLoss
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(n)
    w = torch.softmax(torch.randn(n, J, generator=g) * 4, -1)
    w.view(-1)[:3] = torch.tensor([0.0, 1.0, 0.5])[: w.numel()]
    eps = float(torch.tensor(1e-6))
    w64 = w.double().requires_grad_(True)
    ref = -(w64 * torch.log(w64 + eps) + (1 - w64) * torch.log(1 - w64 + eps)).mean()
    ref.backward(torch.tensor(0.2, dtype=torch.float64))
    wd = w.to(dev).requires_grad_(True)
    loss = SparsityLoss.apply(wd, eps)
    (0.2 * loss).backward()
    assert abs(float(loss.detach()) - float(ref.detach())) <= 2e-6 * max(1.0, abs(float(ref.detach())))
    err = (wd.grad.cpu().double() - w64.grad).abs() / w64.grad.abs().clamp_min(0.2 / w.numel())
    assert float(err.max()) < 1e-5, float(err.max())


@pytest.mark.gpu
@pytest.mark.autograd
def test_gemm_linear_padded_rows_equal_contiguous():
    """linear.pad_cat (feat_net's first-layer input, temporalpoints.py:488-491: posenc 63 + feature
    128 = 191 columns, written into 192-float rows): the product read through the padded 16-B rows
    and the gradients it returns equal those of the contiguous torch.cat input bit for bit."""
    from apn_amd.linear import _GemmLinear, pad_cat
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(3)
    a, b = torch.randn(5000, 63, generator=g), torch.randn(5000, 128, generator=g)
    w, bias = torch.randn(128, 191, generator=g) / 14, torch.randn(128, generator=g)
    dy = torch.randn(5000, 128, generator=g).to(dev)
    res = []
    for padded in (False, True):
        ps = [t.to(dev).requires_grad_(True) for t in (a, b, w, bias)]
        x = pad_cat(ps[:2]) if padded else torch.cat(ps[:2], -1)
        if padded:
            assert x.stride(0) == 192 and x.shape[1] == 191
        y = _GemmLinear.apply(x, ps[2], ps[3], 0.01)
        y.backward(dy)
        res.append([y.detach()] + [p.grad for p in ps])
    for u, v in zip(*res):
        assert torch.equal(u, v)
