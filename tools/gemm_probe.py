"""Probe: fp32 GEMM shapes of the training feat_net (rows = survivors x 8 neighbours) under the
available BLAS back-ends, forward (addmm) and backward (dX, dW). Prints ms per call."""
import sys
import torch

M = int(sys.argv[1]) if len(sys.argv) > 1 else 212736


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


dev = torch.device("cuda")
for lib in ("hipblaslt",):
    try:
        torch.backends.cuda.preferred_blas_library(lib)
    except Exception as ex:  # noqa: BLE001
        print(lib, "unavailable", ex)
        continue
    for K in (155, 128):
        x = torch.randn(M, K, device=dev)
        w = torch.randn(128, K, device=dev)
        b = torch.randn(128, device=dev)
        dy = torch.randn(M, 128, device=dev)
        f = timeit(lambda: torch.nn.functional.linear(x, w, b))
        dx = timeit(lambda: dy @ w)
        dw = timeit(lambda: dy.t() @ x)
        fl = 2 * M * K * 128 / 1e9
        print(f"{lib:10s} M={M} K={K}: fwd {f:.3f} ms ({fl / f:.1f} TF/s)  dX {dx:.3f} ms  dW {dw:.3f} ms", flush=True)
torch.backends.cuda.preferred_blas_library("hipblaslt")
for K in (155, 128):
    x = torch.randn(M, K, device=dev)
    dy = torch.randn(M, 128, device=dev)
    ref = (dy.double().t() @ x.double())
    for S in (16, 32, 64, 128, 256):
        Mc = M // S * S

        def splitk():
            a = dy[:Mc].view(S, -1, 128).transpose(1, 2)
            b = x[:Mc].view(S, -1, K)
            out = torch.bmm(a, b).sum(0)
            return out.addmm_(dy[Mc:].t(), x[Mc:])
        t = timeit(splitk)
        err = float((splitk().double() - ref).abs().max() / ref.abs().max())
        print(f"split-K bmm S={S} K={K}: dW {t:.3f} ms  rel err {err:.2e}", flush=True)
    print(f"plain dW rel err {float(((dy.t() @ x).double() - ref).abs().max() / ref.abs().max()):.2e}")
x = torch.randn(M, 128, device=dev)
print(f"copy-equivalent M x 128 fp32 clone: {timeit(lambda: x.clone()):.3f} ms")
