// Optimizer-side kernels of the reference's training loop:
//   adam_upd / masked_adam_upd / adam_upd_with_perlr   lib/cuda/adam_upd_kernel.cu:8-133
//   total_variation_add_grad                           lib/cuda/total_variation_kernel.cu:13-67
// All are HBM-bound elementwise passes. Each thread updates four consecutive elements with
// 16-B loads/stores where the buffers allow it (the arithmetic per element is unchanged), with a
// scalar tail. fp32, no contraction (-ffp-contract=off); the reference's nvcc build contracts
// a*b + c*d into fma by default, in an order the source does not fix, so parity against it is at
// fp tolerance, and bit-exact against the oracle's unfused restatement.
#include "apn_common.h"

#include <cmath>

namespace apn {

// one Adam element update (adam_upd_kernel.cu:19-21): m = b1 m + (1-b1) g; v = b2 v + ((1-b2) g) g;
// p -= (lr_t [* perlr] * m) / (sqrt(v) + eps)
__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float step_size, float b1, float b2,
                                          float eps, float plr) {
  m = b1 * m + (1.f - b1) * g;
  v = b2 * v + (1.f - b2) * g * g;
  p -= (step_size * plr) * m / (sqrtf(v) + eps);
}

// MODE 0: adam_upd, 1: masked_adam_upd (grad == 0 leaves the element untouched), 2: with perlr
template <int MODE>
__global__ void k_adam(float* __restrict__ param, const float* __restrict__ grad, float* __restrict__ exp_avg,
                       float* __restrict__ exp_avg_sq, const float* __restrict__ perlr, int64_t n, float step_size,
                       float b1, float b2, float eps, bool vec4) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (vec4) {
    const int64_t i0 = 4 * t;
    if (i0 + 3 < n) {
      float4 p = ((float4*)param)[t], m = ((float4*)exp_avg)[t], v = ((float4*)exp_avg_sq)[t];
      const float4 g = ((const float4*)grad)[t];
      const float4 l = MODE == 2 ? ((const float4*)perlr)[t] : make_float4(1.f, 1.f, 1.f, 1.f);
      float* pp = &p.x; float* mm = &m.x; float* vv = &v.x;
      const float* gg = &g.x; const float* ll = &l.x;
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (MODE != 1 || gg[c] != 0.f)
          MODE == 2 ? adam_elem(pp[c], gg[c], mm[c], vv[c], step_size * ll[c], b1, b2, eps, 1.f)
                    : adam_elem(pp[c], gg[c], mm[c], vv[c], step_size, b1, b2, eps, 1.f);
      ((float4*)param)[t] = p; ((float4*)exp_avg)[t] = m; ((float4*)exp_avg_sq)[t] = v;
      return;
    }
    // tail: the last (n % 4) elements, one thread each
    for (int64_t i = i0; i < n; ++i) {
      if (MODE == 1 && grad[i] == 0.f) continue;
      adam_elem(param[i], grad[i], exp_avg[i], exp_avg_sq[i], MODE == 2 ? step_size * perlr[i] : step_size, b1, b2,
                eps, 1.f);
    }
    return;
  }
  if (t >= n) return;
  if (MODE == 1 && grad[t] == 0.f) return;
  adam_elem(param[t], grad[t], exp_avg[t], exp_avg_sq[t], MODE == 2 ? step_size * perlr[t] : step_size, b1, b2, eps,
            1.f);
}

// total_variation_kernel.cu:13-35: six clamped neighbour differences; the i-direction uses wz
// (as the reference does -- wx is never read), each term added to a float in source order.
// blockIdx.y = plane (c, i); a thread owns V consecutive k of one (j) row: V = 4 turns the
// 8 scalar accesses per element into 16-B loads of the element and its j / i neighbours plus
// two scalar k-edge loads per four elements.
template <bool DENSE, int V>
__global__ void k_tv_add_grad(const float* __restrict__ param, float* __restrict__ grad, float wy, float wz,
                              int si, int sj, int sk) {
  const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;   // vector slot in the (j, k) plane
  const unsigned plane_sz = (unsigned)sj * (unsigned)sk;
  if (t * V >= plane_sz) return;
  const int plane = blockIdx.y, i = plane % si;
  const unsigned tk = t * V;
  const int j = (int)(tk / (unsigned)sk), k0 = (int)(tk - (unsigned)j * (unsigned)sk);
  const int64_t idx0 = (int64_t)plane * plane_sz + tk;
  typedef float vf __attribute__((ext_vector_type(V)));
  const vf p = *(const vf*)(param + idx0);
  vf g = *(const vf*)(grad + idx0);
  const vf pjm = j > 0 ? *(const vf*)(param + idx0 - sk) : p;
  const vf pjp = j < sj - 1 ? *(const vf*)(param + idx0 + sk) : p;
  const vf pim = i > 0 ? *(const vf*)(param + idx0 - plane_sz) : p;
  const vf pip = i < si - 1 ? *(const vf*)(param + idx0 + plane_sz) : p;
  const float kl = k0 > 0 ? param[idx0 - 1] : 0.f;
  const float kr = k0 + V < sk ? param[idx0 + V] : 0.f;
  auto cl = [](float v) { return fminf(fmaxf(v, -1.f), 1.f); };
#pragma unroll
  for (int c = 0; c < V; ++c) {
    if (!DENSE && g[c] == 0.f) continue;
    const int k = k0 + c;
    const float pl = c > 0 ? p[c > 0 ? c - 1 : 0] : kl;
    const float pr = c < V - 1 ? p[c < V - 1 ? c + 1 : 0] : kr;
    float acc = 0.f;
    acc += k == 0 ? 0.f : wz * cl(p[c] - pl);
    acc += k == sk - 1 ? 0.f : wz * cl(p[c] - pr);
    acc += j == 0 ? 0.f : wy * cl(p[c] - pjm[c]);
    acc += j == sj - 1 ? 0.f : wy * cl(p[c] - pjp[c]);
    acc += i == 0 ? 0.f : wz * cl(p[c] - pim[c]);
    acc += i == si - 1 ? 0.f : wz * cl(p[c] - pip[c]);
    g[c] += acc;
  }
  *(vf*)(grad + idx0) = g;
}

// adam_upd_kernel.cu:70, evaluated on the host in float as the reference's host code does
static float adam_step_size(int step, float b1, float b2, float lr) {
  return lr * std::sqrt(1.f - std::pow(b2, (float)step)) / (1.f - std::pow(b1, (float)step));
}

template <int MODE>
static int launch_adam(float* param, const float* grad, float* m, float* v, const float* perlr, int64_t n, int step,
                       float b1, float b2, float lr, float eps, void* stream) {
  if (n < 0 || (n > 0 && (!param || !grad || !m || !v || (MODE == 2 && !perlr)))) return APN_ERR_ARG;
  if (n == 0) return APN_OK;
  const float ss = adam_step_size(step, b1, b2, lr);
  auto al = [](const void* p) { return p == nullptr || ((uintptr_t)p & 15) == 0; };
  const bool vec4 = al(param) && al(grad) && al(m) && al(v) && (MODE != 2 || al(perlr));
  const int64_t threads = vec4 ? (n + 3) / 4 : n;
  hipLaunchKernelGGL(k_adam<MODE>, dim3(ceil_div(threads, 256)), dim3(256), 0, (hipStream_t)stream, param, grad, m,
                     v, perlr, n, ss, b1, b2, eps, vec4);
  return launch_status();
}

}  // namespace apn

using namespace apn;

// Multi-tensor form (MaskedAdam.step over every parameter tensor of a step in ONE launch): the
// tensors' pointers, sizes and per-tensor step sizes travel as kernel arguments (up to
// ADAM_MULTI_MAX tensors per launch); block b works on the tensor whose block range holds b, with
// the same per-element update (adam_elem, the same step size) as apn_adam_upd /
// apn_masked_adam_upd -- bit-identical to one launch per tensor.
constexpr int ADAM_MULTI_MAX = 24;
struct AdamMulti {
  float* p[ADAM_MULTI_MAX];
  const float* g[ADAM_MULTI_MAX];
  float* m[ADAM_MULTI_MAX];
  float* v[ADAM_MULTI_MAX];
  int64_t n[ADAM_MULTI_MAX];
  int block0[ADAM_MULTI_MAX + 1];   // first block of tensor i (block0[count] = grid)
  float step_size[ADAM_MULTI_MAX], b1[ADAM_MULTI_MAX], b2[ADAM_MULTI_MAX], eps[ADAM_MULTI_MAX];
  int masked[ADAM_MULTI_MAX];
  int count;
};

__global__ __launch_bounds__(256) void k_adam_multi(AdamMulti a) {
  int i = 0;
  while (i + 1 < a.count && (int)blockIdx.x >= a.block0[i + 1]) ++i;   // wave-uniform
  const int64_t t = (int64_t)(blockIdx.x - a.block0[i]) * 256 + threadIdx.x;
  if (t >= a.n[i]) return;
  if (a.masked[i] && a.g[i][t] == 0.f) return;
  adam_elem(a.p[i][t], a.g[i][t], a.m[i][t], a.v[i][t], a.step_size[i], a.b1[i], a.b2[i], a.eps[i], 1.f);
}

extern "C" int apn_adam_multi(int32_t count, float* const* params, const float* const* grads, float* const* exp_avgs,
                              float* const* exp_avg_sqs, const int64_t* numels, const int32_t* steps,
                              const float* beta1, const float* beta2, const float* lrs, const float* eps,
                              const int32_t* masked, void* stream) {
  if (count < 0 || count > ADAM_MULTI_MAX) return APN_ERR_ARG;
  AdamMulti a;
  int blocks = 0;
  a.count = count;
  for (int i = 0; i < count; ++i) {
    if (numels[i] < 0 || (numels[i] > 0 && (!params[i] || !grads[i] || !exp_avgs[i] || !exp_avg_sqs[i])))
      return APN_ERR_ARG;
    a.p[i] = params[i]; a.g[i] = grads[i]; a.m[i] = exp_avgs[i]; a.v[i] = exp_avg_sqs[i];
    a.n[i] = numels[i];
    a.block0[i] = blocks;
    blocks += ceil_div(numels[i], 256);
    a.step_size[i] = adam_step_size(steps[i], beta1[i], beta2[i], lrs[i]);
    a.b1[i] = beta1[i]; a.b2[i] = beta2[i]; a.eps[i] = eps[i];
    a.masked[i] = masked[i];
  }
  a.block0[count] = blocks;
  if (blocks == 0) return APN_OK;
  hipLaunchKernelGGL(k_adam_multi, dim3(blocks), dim3(256), 0, (hipStream_t)stream, a);
  return launch_status();
}

extern "C" int apn_adam_upd(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                            int32_t step, float beta1, float beta2, float lr, float eps, void* stream) {
  return launch_adam<0>(param, grad, exp_avg, exp_avg_sq, nullptr, n, step, beta1, beta2, lr, eps, stream);
}

extern "C" int apn_masked_adam_upd(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                                   int32_t step, float beta1, float beta2, float lr, float eps, void* stream) {
  return launch_adam<1>(param, grad, exp_avg, exp_avg_sq, nullptr, n, step, beta1, beta2, lr, eps, stream);
}

extern "C" int apn_adam_upd_with_perlr(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                                       const float* perlr, int64_t n, int32_t step, float beta1, float beta2,
                                       float lr, float eps, void* stream) {
  return launch_adam<2>(param, grad, exp_avg, exp_avg_sq, perlr, n, step, beta1, beta2, lr, eps, stream);
}

extern "C" int apn_total_variation_add_grad(const float* param, float* grad, float wx, float wy, float wz,
                                            int64_t sz_i, int64_t sz_j, int64_t sz_k, int64_t n, int32_t dense_mode,
                                            void* stream) {
  if (n < 0 || sz_i <= 0 || sz_j <= 0 || sz_k <= 0 || (n > 0 && (!param || !grad))) return APN_ERR_ARG;
  if (n == 0) return APN_OK;
  const int64_t plane = sz_j * sz_k, planes = n / plane;
  if (n % (sz_i * plane) != 0 || plane > 0x7fffffff || planes > 65535 * 1024 || sz_i > 0x7fffffff)
    return APN_ERR_ARG;
  (void)wx;  // total_variation_kernel.cu:30-31 weight the i direction with wz
  wy /= 6; wz /= 6;
  const bool v4 = sz_k % 4 == 0 && ((uintptr_t)param & 15) == 0 && ((uintptr_t)grad & 15) == 0;
  const int V = v4 ? 4 : 1;
  const dim3 grid(ceil_div(plane / V, 256), (unsigned)planes);
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, (hipStream_t)stream, param, grad, wy, wz, (int)sz_i, (int)sz_j,
                       (int)sz_k);
  };
  if (dense_mode) {
    if (v4) go(k_tv_add_grad<true, 4>); else go(k_tv_add_grad<true, 1>);
  } else {
    if (v4) go(k_tv_add_grad<false, 4>); else go(k_tv_add_grad<false, 1>);
  }
  return launch_status();
}
