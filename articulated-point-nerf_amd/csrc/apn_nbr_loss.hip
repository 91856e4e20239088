// Neighbour-graph regularisers of the training step over the static
// canonical kNN graph nn_i [N,K] (self first, temporalpoints.py:104-110):
//   get_neighbour_weight_tv_loss  temporalpoints.py:714-716   mean |w_i - w_nn(i,k)|  over [N,K,J]
//   get_arap_loss                 temporalpoints.py:723-725   sum |d0_ik - sqrt(|x_i - x_nn(i,k)|^2 + eps)|
// The reference materialises the [N,K,J] / [N,K,3] gathers and lets autograd scatter-add them back
// (index_put with accumulate). Here the forward is a fused edge reduction (no [N,K,*] tensor) and
// the backward is a pure gather: each point sums its out-edges and, through the reverse CSR of the
// graph (rev_ptr [N+1], rev_edge [N*K] = edge ids i*K+k grouped by target, ascending), its
// in-edges -- no atomics, so gradients are deterministic. Losses are block partials reduced by one
// block in a fixed order. fp32, -ffp-contract=off, the reference's expression order per element.
#include "apn_common.h"

#include <cmath>

namespace apn {

constexpr int kLossBlocks = 1024;   // fixed grid of the partial pass: deterministic reduction order
constexpr int kLossThreads = 256;

__device__ __forceinline__ float sgnf(float x) { return (float)(x > 0.f) - (float)(x < 0.f); }

__device__ __forceinline__ float block_sum(float v) {
  __shared__ float red[kLossThreads / 64];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float s = 0.f;
  if (threadIdx.x == 0)
    for (int w = 0; w < kLossThreads / 64; ++w) s += red[w];
  return s;
}

// Indices are 32-bit (the C entry points require n * max(J, K) < 2^31): a 64-bit division per
// element is a long software sequence on CDNA. KT = compile-time neighbour count (8, the
// TemporalPoints default) or 0 = runtime Kr.
// one thread per (point, channel): sum_k |w_i[j] - w_nn[j]|
template <int KT>
__global__ void __launch_bounds__(kLossThreads) k_tv_partial(const float* __restrict__ w, const int64_t* __restrict__ nn,
                                                             int n, int J, int Kr, float* __restrict__ partials) {
  const int K = KT ? KT : Kr;
  float acc = 0.f;
  const unsigned total = (unsigned)n * (unsigned)J;
  for (unsigned t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const unsigned i = t / (unsigned)J;
    const unsigned j = t - i * (unsigned)J;
    const float wi = w[t];
#pragma unroll
    for (int k = 0; k < K; ++k) acc += fabsf(wi - w[(unsigned)nn[i * K + k] * J + j]);
  }
  const float s = block_sum(acc);
  if (threadIdx.x == 0) partials[blockIdx.x] = s;
}

// one thread per edge (i, k): |d0 - sqrt((dx^2 + dy^2 + dz^2) + eps)|
__device__ __forceinline__ float edge_dist(const float* __restrict__ x, int64_t a, int64_t b, float eps, float& dx,
                                           float& dy, float& dz) {
  dx = x[3 * a] - x[3 * b];
  dy = x[3 * a + 1] - x[3 * b + 1];
  dz = x[3 * a + 2] - x[3 * b + 2];
  float u = dx * dx + dy * dy;
  u = u + dz * dz;
  return sqrtf(u + eps);
}

template <int KT>
__global__ void __launch_bounds__(kLossThreads) k_arap_partial(const float* __restrict__ x, const int64_t* __restrict__ nn,
                                                               const float* __restrict__ d0, int n, int Kr, float eps,
                                                               float* __restrict__ partials) {
  const int K = KT ? KT : Kr;
  float acc = 0.f;
  const unsigned total = (unsigned)n * (unsigned)K;
  for (unsigned e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    float dx, dy, dz;
    const float s = edge_dist(x, e / (unsigned)K, nn[e], eps, dx, dy, dz);
    acc += fabsf(d0[e] - s);
  }
  const float s = block_sum(acc);
  if (threadIdx.x == 0) partials[blockIdx.x] = s;
}

// loss_out[0] = (sum of partials in index order) * scale  (scale = 1/count for a mean, 1 for a sum)
__global__ void __launch_bounds__(kLossThreads) k_reduce_partials(const float* __restrict__ partials, int np,
                                                                  float inv_count, bool mean, float* __restrict__ out) {
  float acc = 0.f;
  for (int b = threadIdx.x; b < np; b += blockDim.x) acc += partials[b];
  const float s = block_sum(acc);
  if (threadIdx.x == 0) out[0] = mean ? s * inv_count : s;
}

// d w[i,j] = dL/count * (sum_k sgn(w_i - w_nn(i,k)) - sum_{e in rev(i)} sgn(w_src(e) - w_i))
template <int KT>
__global__ void __launch_bounds__(kLossThreads) k_tv_bwd(const float* __restrict__ w, const int64_t* __restrict__ nn,
                                                         const int64_t* __restrict__ rev_ptr,
                                                         const int64_t* __restrict__ rev_edge, int n, int J, int Kr,
                                                         const float* __restrict__ d_loss, float inv_count,
                                                         float* __restrict__ dw) {
  const int K = KT ? KT : Kr;
  const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (unsigned)n * (unsigned)J) return;
  const unsigned i = t / (unsigned)J;
  const unsigned j = t - i * (unsigned)J;
  const float wi = w[t];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < K; ++k) s += sgnf(wi - w[(unsigned)nn[i * K + k] * J + j]);
  for (unsigned e = (unsigned)rev_ptr[i], e1 = (unsigned)rev_ptr[i + 1]; e < e1; ++e)
    s -= sgnf(w[((unsigned)rev_edge[e] / (unsigned)K) * J + j] - wi);
  dw[t] = (d_loss[0] * inv_count) * s;
}

// d x_i = sum_k c_ik * (2 diff_ik) - sum_{e=(src,k) in rev(i)} c_e * (2 diff_e),
// c = (-sgn(d0 - s) dL) / (2 s)   (abs, sqrt and pow(2) backward in torch's order)
__device__ __forceinline__ float arap_coef(float d0, float s, float g) { return (-sgnf(d0 - s) * g) / (2.f * s); }

template <int KT>
__global__ void __launch_bounds__(kLossThreads) k_arap_bwd(const float* __restrict__ x, const int64_t* __restrict__ nn,
                                                           const float* __restrict__ d0,
                                                           const int64_t* __restrict__ rev_ptr,
                                                           const int64_t* __restrict__ rev_edge, int n, int Kr,
                                                           float eps, const float* __restrict__ d_loss,
                                                           float* __restrict__ dx_out) {
  const int K = KT ? KT : Kr;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float g = d_loss[0];
  float gx = 0.f, gy = 0.f, gz = 0.f;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int e = i * K + k;
    float dx, dy, dz;
    const float s = edge_dist(x, i, nn[e], eps, dx, dy, dz);
    const float c = arap_coef(d0[e], s, g);
    gx += c * (2.f * dx); gy += c * (2.f * dy); gz += c * (2.f * dz);
  }
  for (unsigned r = (unsigned)rev_ptr[i], r1 = (unsigned)rev_ptr[i + 1]; r < r1; ++r) {
    const unsigned e = (unsigned)rev_edge[r];
    float dx, dy, dz;
    const float s = edge_dist(x, e / (unsigned)K, i, eps, dx, dy, dz);
    const float c = arap_coef(d0[e], s, g);
    gx -= c * (2.f * dx); gy -= c * (2.f * dy); gz -= c * (2.f * dz);
  }
  dx_out[3 * i] = gx; dx_out[3 * i + 1] = gy; dx_out[3 * i + 2] = gz;
}

// get_weight_sparsity_loss (temporalpoints.py:718-721): -mean(w log(w + eps) + (1 - w) log(1 - w + eps))
// over the [N,J] skinning weights -- one partial pass instead of ~10 elementwise torch launches
// forward and ~12 backward.
__device__ __forceinline__ float sparsity_term(float w, float eps) {
  const float a = w * logf(w + eps);
  const float b = (1.f - w) * logf((1.f - w) + eps);
  return a + b;
}

__global__ void __launch_bounds__(kLossThreads) k_sparsity_partial(const float* __restrict__ w, int64_t n, float eps,
                                                                   float* __restrict__ partials) {
  float acc = 0.f;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x)
    acc += sparsity_term(w[t], eps);
  const float s = block_sum(acc);
  if (threadIdx.x == 0) partials[blockIdx.x] = s;
}

// d w = -(dL / n) (log(w + eps) + w / (w + eps) - log(1 - w + eps) - (1 - w) / (1 - w + eps))
__global__ void __launch_bounds__(kLossThreads) k_sparsity_bwd(const float* __restrict__ w, int64_t n, float eps,
                                                               const float* __restrict__ d_loss, float inv_count,
                                                               float* __restrict__ dw) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const float x = w[t];
  const float a = x + eps, b = (1.f - x) + eps;
  const float d = (logf(a) + x / a) - (logf(b) + (1.f - x) / b);
  dw[t] = (-(d_loss[0] * inv_count)) * d;
}

}  // namespace apn

using namespace apn;

extern "C" size_t apn_nbr_loss_workspace_bytes(void) { return (size_t)kLossBlocks * sizeof(float); }

// 32-bit element / edge indexing in the kernels
static inline bool fits32(int64_t n, int64_t a, int64_t b) { return n * (a > b ? a : b) < ((int64_t)1 << 31); }

#define APN_LAUNCH_K(kern, K, grid, ...)                                                                   \
  do {                                                                                                     \
    if ((K) == 8) hipLaunchKernelGGL(kern<8>, grid, dim3(kLossThreads), 0, (hipStream_t)stream, __VA_ARGS__); \
    else hipLaunchKernelGGL(kern<0>, grid, dim3(kLossThreads), 0, (hipStream_t)stream, __VA_ARGS__);          \
  } while (0)

static inline int partial_blocks(int64_t work) {
  const int b = ceil_div(work, kLossThreads);
  return b < 1 ? 1 : (b > kLossBlocks ? kLossBlocks : b);
}

extern "C" int apn_nbr_tv_loss(const float* w, int64_t n_points, int32_t n_channels, const int64_t* nn_i,
                               int32_t k, float* loss_out, void* workspace, void* stream) {
  if (n_points <= 0 || n_channels <= 0 || k <= 0 || !w || !nn_i || !loss_out || !workspace) return APN_ERR_ARG;
  if (!fits32(n_points, n_channels, k)) return APN_ERR_ARG;
  const int nb = partial_blocks(n_points * n_channels);
  APN_LAUNCH_K(k_tv_partial, k, dim3(nb), w, nn_i, (int)n_points, (int)n_channels, (int)k, (float*)workspace);
  const float inv = (float)(1.0 / ((double)n_points * (double)k * (double)n_channels));
  hipLaunchKernelGGL(k_reduce_partials, dim3(1), dim3(kLossThreads), 0, (hipStream_t)stream,
                     (const float*)workspace, nb, inv, true, loss_out);
  return launch_status();
}

extern "C" int apn_nbr_tv_loss_backward(const float* w, int64_t n_points, int32_t n_channels, const int64_t* nn_i,
                                        int32_t k, const int64_t* rev_ptr, const int64_t* rev_edge,
                                        const float* d_loss, float* dw, void* stream) {
  if (n_points <= 0 || n_channels <= 0 || k <= 0 || !w || !nn_i || !rev_ptr || !rev_edge || !d_loss || !dw)
    return APN_ERR_ARG;
  if (!fits32(n_points, n_channels, k)) return APN_ERR_ARG;
  const float inv = (float)(1.0 / ((double)n_points * (double)k * (double)n_channels));
  APN_LAUNCH_K(k_tv_bwd, k, dim3(ceil_div(n_points * n_channels, kLossThreads)), w, nn_i, rev_ptr, rev_edge,
               (int)n_points, (int)n_channels, (int)k, d_loss, inv, dw);
  return launch_status();
}

extern "C" int apn_arap_loss(const float* x, int64_t n_points, const int64_t* nn_i, int32_t k, const float* nn_dist0,
                             float eps, float* loss_out, void* workspace, void* stream) {
  if (n_points <= 0 || k <= 0 || !x || !nn_i || !nn_dist0 || !loss_out || !workspace) return APN_ERR_ARG;
  if (!fits32(n_points, 3, k)) return APN_ERR_ARG;
  const int nb = partial_blocks(n_points * k);
  APN_LAUNCH_K(k_arap_partial, k, dim3(nb), x, nn_i, nn_dist0, (int)n_points, (int)k, eps, (float*)workspace);
  hipLaunchKernelGGL(k_reduce_partials, dim3(1), dim3(kLossThreads), 0, (hipStream_t)stream,
                     (const float*)workspace, nb, 1.f, false, loss_out);
  return launch_status();
}

extern "C" int apn_arap_loss_backward(const float* x, int64_t n_points, const int64_t* nn_i, int32_t k,
                                      const float* nn_dist0, float eps, const int64_t* rev_ptr,
                                      const int64_t* rev_edge, const float* d_loss, float* dx, void* stream) {
  if (n_points <= 0 || k <= 0 || !x || !nn_i || !nn_dist0 || !rev_ptr || !rev_edge || !d_loss || !dx)
    return APN_ERR_ARG;
  if (!fits32(n_points, 3, k)) return APN_ERR_ARG;
  APN_LAUNCH_K(k_arap_bwd, k, dim3(ceil_div(n_points, kLossThreads)), x, nn_i, nn_dist0, rev_ptr, rev_edge,
               (int)n_points, (int)k, eps, d_loss, dx);
  return launch_status();
}

extern "C" int apn_weight_sparsity_loss(const float* w, int64_t n, float eps, float* loss_out, void* workspace,
                                        void* stream) {
  if (n <= 0 || !w || !loss_out || !workspace) return APN_ERR_ARG;
  const int nb = partial_blocks(n);
  hipLaunchKernelGGL(k_sparsity_partial, dim3(nb), dim3(kLossThreads), 0, (hipStream_t)stream, w, n, eps,
                     (float*)workspace);
  // loss = -(sum / n): the reduce kernel scales by -1/n
  hipLaunchKernelGGL(k_reduce_partials, dim3(1), dim3(kLossThreads), 0, (hipStream_t)stream,
                     (const float*)workspace, nb, (float)(-1.0 / (double)n), true, loss_out);
  return launch_status();
}

extern "C" int apn_weight_sparsity_loss_backward(const float* w, int64_t n, float eps, const float* d_loss, float* dw,
                                                 void* stream) {
  if (n <= 0 || !w || !d_loss || !dw) return APN_ERR_ARG;
  hipLaunchKernelGGL(k_sparsity_bwd, dim3(ceil_div(n, kLossThreads)), dim3(kLossThreads), 0, (hipStream_t)stream, w, n,
                     eps, d_loss, (float)(1.0 / (double)n), dw);
  return launch_status();
}
