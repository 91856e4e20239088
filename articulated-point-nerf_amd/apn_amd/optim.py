"""Drop-ins for the reference's JIT-built optimizer modules, over the C-ABI:

    import apn_amd.optim as adam_upd_cuda            # lib/cuda/adam_upd.cpp:36-85
    import apn_amd.optim as total_variation_cuda     # lib/cuda/total_variation.cpp:16-24

Same function names, argument order and in-place semantics; inputs must be contiguous fp32
device tensors (the reference's CHECK_INPUT), else RuntimeError. No CPU fallback.
"""
from __future__ import annotations

import torch

from . import _lib as L
from ._lib import call, ptr, stream_ptr


def _check(*ts, what):
    L.require_cuda(*ts, what=what)
    for t in ts:
        if t is None:
            continue
        if not t.is_contiguous():
            raise RuntimeError(f"{what}: tensors must be contiguous")
        if t.dtype != torch.float32:
            raise RuntimeError(f"{what}: expected float32 tensors, got {t.dtype}")
    n = ts[0].numel()
    if any(t is not None and t.numel() != n for t in ts):
        raise RuntimeError(f"{what}: tensors differ in size")
    return n


def _bump(*ts):
    """The kernels write through raw pointers, which torch cannot see: bump the version counters
    so every cache keyed on ``(data_ptr, _version)`` (TemporalPoints' packed MLP weights and
    feature projection, PointWarper's packed TransformNet) notices the in-place update, as it
    would after a torch in-place op."""
    for t in ts:
        torch.autograd.graph.increment_version(t)


def adam_upd(param, grad, exp_avg, exp_avg_sq, step, beta1, beta2, lr, eps):
    """adam_upd_kernel.cu:8-23, 62-82 (in place)."""
    n = _check(param, grad, exp_avg, exp_avg_sq, what="adam_upd")
    call("apn_adam_upd", ptr(param), ptr(grad), ptr(exp_avg), ptr(exp_avg_sq), n, int(step), float(beta1),
         float(beta2), float(lr), float(eps), stream_ptr(param.device))
    _bump(param, exp_avg, exp_avg_sq)


def masked_adam_upd(param, grad, exp_avg, exp_avg_sq, step, beta1, beta2, lr, eps):
    """adam_upd_kernel.cu:25-40, 84-104: elements with grad == 0 are left untouched (in place)."""
    n = _check(param, grad, exp_avg, exp_avg_sq, what="masked_adam_upd")
    call("apn_masked_adam_upd", ptr(param), ptr(grad), ptr(exp_avg), ptr(exp_avg_sq), n, int(step), float(beta1),
         float(beta2), float(lr), float(eps), stream_ptr(param.device))
    _bump(param, exp_avg, exp_avg_sq)


def adam_upd_with_perlr(param, grad, exp_avg, exp_avg_sq, perlr, step, beta1, beta2, lr, eps):
    """adam_upd_kernel.cu:42-58, 106-128: per-element learning-rate scale (in place)."""
    n = _check(param, grad, exp_avg, exp_avg_sq, perlr, what="adam_upd_with_perlr")
    call("apn_adam_upd_with_perlr", ptr(param), ptr(grad), ptr(exp_avg), ptr(exp_avg_sq), ptr(perlr), n, int(step),
         float(beta1), float(beta2), float(lr), float(eps), stream_ptr(param.device))
    _bump(param, exp_avg, exp_avg_sq)


MULTI_MAX = 24   # tensors per apn_adam_multi launch


def adam_multi(batch):
    """One apn_adam_multi launch over [(param, grad, exp_avg, exp_avg_sq, step, beta1, beta2, lr,
    eps, masked)] (<= MULTI_MAX, contiguous fp32 device tensors): each tensor updated exactly as by
    adam_upd / masked_adam_upd."""
    import ctypes as C
    n = len(batch)
    if n == 0:
        return
    if n > MULTI_MAX:
        raise ValueError(f"adam_multi: at most {MULTI_MAX} tensors per launch")
    col = list(zip(*batch))
    ptrs = lambda ts: (C.c_void_p * n)(*[t.data_ptr() for t in ts])
    for t in col[1]:
        L.require_cuda(t, what="adam_multi")
    call("apn_adam_multi", n, ptrs(col[0]), ptrs(col[1]), ptrs(col[2]), ptrs(col[3]),
         (C.c_int64 * n)(*[t.numel() for t in col[0]]), (C.c_int32 * n)(*[int(x) for x in col[4]]),
         (C.c_float * n)(*col[5]), (C.c_float * n)(*col[6]), (C.c_float * n)(*col[7]), (C.c_float * n)(*col[8]),
         (C.c_int32 * n)(*[int(x) for x in col[9]]), stream_ptr(col[0][0].device))
    _bump(*col[0], *col[2], *col[3])


def total_variation_add_grad(param, grad, wx, wy, wz, dense_mode):
    """total_variation_kernel.cu:13-67: grad += clamped neighbour differences of the 5-D grid
    param [1, C, I, J, K] (weights / 6; the reference weights the I direction with wz)."""
    n = _check(param, grad, what="total_variation_add_grad")
    if param.dim() != 5:
        raise RuntimeError("total_variation_add_grad: param must be [1, C, I, J, K]")
    call("apn_total_variation_add_grad", ptr(param), ptr(grad), float(wx), float(wy), float(wz), param.shape[2],
         param.shape[3], param.shape[4], n, int(bool(dense_mode)), stream_ptr(param.device))
    _bump(grad)


class MaskedAdam(torch.optim.Optimizer):
    """lib/masked_adam.py:15-72 over the HIP kernels: per-voxel learning rate (set_pervoxel_lr)
    and the zero-grad-skipping update (param group key 'skip_zero_grad', required as in the
    reference)."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.99), eps=1e-8):
        if not 0.0 <= lr:
            raise ValueError(f"Invalid learning rate: {lr}")
        if not 0.0 <= eps:
            raise ValueError(f"Invalid epsilon value: {eps}")
        if not 0.0 <= betas[0] < 1.0:
            raise ValueError(f"Invalid beta parameter at index 0: {betas[0]}")
        if not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"Invalid beta parameter at index 1: {betas[1]}")
        self.per_lr = None
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps))

    def set_pervoxel_lr(self, count):
        assert self.param_groups[0]['params'][0].shape == count.shape
        self.per_lr = count.float() / count.max()

    @torch.no_grad()
    def step(self):
        batch = []   # (param, grad, exp_avg, exp_avg_sq, step, beta1, beta2, lr, eps, masked): one launch
        for group in self.param_groups:
            lr = group['lr']
            beta1, beta2 = group['betas']
            eps = group['eps']
            skip_zero_grad = group['skip_zero_grad']
            for param in group['params']:
                if param.grad is None:
                    continue
                state = self.state[param]
                if len(state) == 0:
                    state['step'] = 0
                    state['exp_avg'] = torch.zeros_like(param, memory_format=torch.preserve_format)
                    state['exp_avg_sq'] = torch.zeros_like(param, memory_format=torch.preserve_format)
                state['step'] += 1
                if self.per_lr is not None and param.shape == self.per_lr.shape:
                    adam_upd_with_perlr(param, param.grad, state['exp_avg'], state['exp_avg_sq'], self.per_lr,
                                        state['step'], beta1, beta2, lr, eps)
                elif param.is_cuda and param.is_contiguous() and param.grad.is_contiguous() \
                        and param.dtype == torch.float32 and param.grad.dtype == torch.float32:
                    batch.append((param, param.grad, state['exp_avg'], state['exp_avg_sq'], state['step'], beta1,
                                  beta2, lr, eps, bool(skip_zero_grad)))
                elif skip_zero_grad:
                    masked_adam_upd(param, param.grad, state['exp_avg'], state['exp_avg_sq'], state['step'], beta1,
                                    beta2, lr, eps)
                else:
                    adam_upd(param, param.grad, state['exp_avg'], state['exp_avg_sq'], state['step'], beta1, beta2,
                             lr, eps)
        for i in range(0, len(batch), MULTI_MAX):
            adam_multi(batch[i:i + MULTI_MAX])
