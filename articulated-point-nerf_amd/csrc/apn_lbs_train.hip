// Differentiable LBS of the training path: forward and backward of
//   sm   = softmax(W / max(eps, theta))                     temporalpoints.py:401-414
//   G_n  = sum_j sm_nj T_j   (3x4 rows; bottom row exact)    pointwarper.py:241-243
//   x'_n = G_n[:, :3] p_n + G_n[:, 3] + global_t             pointwarper.py:253-266
//   Rinv_n = inverse(G_n)[:3, :3] (adjugate of the 3x3)      temporalpoints.py:569, 478
// as two per-point kernels, replacing ~150 small torch launches (softmax, blend GEMM, broadcast
// products, the inverse and all their backward ops) of the autograd composition.
//
// Backward per point (inputs dx [3], dRinv [9], dsm [J], each optional):
//   dA = dx p^T - Rinv^T dRinv Rinv^T,  db = dx          (A = G[:, :3], b = G[:, 3])
//   dsm_tot_j = dsm_j + <dG, T_j>;  dz_j = sm_j (dsm_tot_j - sum_k sm_k dsm_tot_k)
//   dW_j = dz_j / th;  dtheta += -sum_j dz_j W_j / th^2 (only while theta > eps)
//   dT_j += sm_j dG;  dglobal_t += dx
// dT = sm^T dG is a [J x N] . [N x 12] product with a long N: each backward block stages its
// points' sm rows and dG rows in LDS and computes its [J x 12] partial there (thread per output,
// fixed point order); dglobal_t / dtheta are wave-reduced. The per-block partials are summed by
// one block per value in a fixed order: deterministic, no atomics.
#include "apn_common.h"

namespace apn {

constexpr int LT_THREADS = 256;
constexpr int LB_THREADS = 128;   // backward: points per block (LDS tile 3 (J+1) + 13 floats per point)
constexpr int LT_MAXJ = 64;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(LT_THREADS) void k_lbs_train_fwd(const float* __restrict__ pcd,
                                                              const float* __restrict__ W, int64_t n, int J,
                                                              const float* __restrict__ theta, float eps,
                                                              const float* __restrict__ T34,
                                                              const float* __restrict__ gt, float* __restrict__ sm,
                                                              float* __restrict__ G12, float* __restrict__ xyz,
                                                              float* __restrict__ Rinv) {
  __shared__ float sT[LT_MAXJ * 12];
  extern __shared__ float tile[];   // [LT_THREADS][J + 1]: the block's W rows, then its sm rows
  const int sstride = J + 1;
  for (int i = threadIdx.x; i < J * 12; i += LT_THREADS) sT[i] = T34[i];
  const int64_t p0 = (int64_t)blockIdx.x * LT_THREADS;
  const int rows = (int)(n - p0 < LT_THREADS ? n - p0 : LT_THREADS);
  const int cnt = rows * J;
  for (int i = threadIdx.x; i < cnt; i += LT_THREADS) {   // coalesced: the rows are contiguous
    const int r = i / J;
    tile[r * sstride + (i - r * J)] = W[p0 * J + i];
  }
  __syncthreads();
  const int64_t p = p0 + threadIdx.x;
  const bool live = p < n;
  const float th = fmaxf(eps, theta[0]);
  float* w = tile + threadIdx.x * sstride;
  float g[12];
#pragma unroll
  for (int k = 0; k < 12; ++k) g[k] = 0.f;
  if (live) {
    float mx = -INFINITY;
    for (int j = 0; j < J; ++j) mx = fmaxf(mx, w[j] / th);
    float s = 0.f;
    for (int j = 0; j < J; ++j) s += expf(w[j] / th - mx);
    const float inv_s = 1.f / s;
    for (int j = 0; j < J; ++j) {
      const float v = expf(w[j] / th - mx) * inv_s;
      w[j] = v;
#pragma unroll
      for (int k = 0; k < 12; ++k) g[k] += v * sT[12 * j + k];
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < cnt; i += LT_THREADS) {
    const int r = i / J;
    sm[p0 * J + i] = tile[r * sstride + (i - r * J)];
  }
  if (!live) return;
  const float px = pcd[3 * p], py = pcd[3 * p + 1], pz = pcd[3 * p + 2];
#pragma unroll
  for (int r = 0; r < 3; ++r)
    xyz[3 * p + r] = g[4 * r] * px + g[4 * r + 1] * py + g[4 * r + 2] * pz + g[4 * r + 3] + gt[r];
#pragma unroll
  for (int k = 0; k < 12; ++k) G12[12 * p + k] = g[k];
  const float a = g[0], b = g[1], c = g[2], d = g[4], e = g[5], f = g[6], h0 = g[8], h = g[9], i = g[10];
  const float c00 = e * i - f * h, c01 = f * h0 - d * i, c02 = d * h - e * h0;
  const float rdet = 1.f / (a * c00 + b * c01 + c * c02);
  float* R = Rinv + 9 * p;
  R[0] = c00 * rdet; R[1] = (c * h - b * i) * rdet; R[2] = (b * f - c * e) * rdet;
  R[3] = c01 * rdet; R[4] = (a * i - c * h0) * rdet; R[5] = (c * d - a * f) * rdet;
  R[6] = c02 * rdet; R[7] = (b * h0 - a * h) * rdet; R[8] = (a * e - b * d) * rdet;
}

// part layout per block: [J*12] dT, [3] dglobal_t, [1] dtheta
__global__ __launch_bounds__(LB_THREADS) void k_lbs_train_bwd(
    const float* __restrict__ pcd, const float* __restrict__ W, int64_t n, int J, const float* __restrict__ theta,
    float eps, const float* __restrict__ T34, const float* __restrict__ sm, const float* __restrict__ Rinv,
    const float* __restrict__ dxyz, const float* __restrict__ dRinv, const float* __restrict__ dsm,
    float* __restrict__ dW, float* __restrict__ part) {
  __shared__ float sT[LT_MAXJ * 12];
  __shared__ float sRed[LB_THREADS / 64][4];
  extern __shared__ float dyn[];
  const int sstride = J + 1;                 // odd strides: conflict-free per-row access
  float* sS = dyn;                            // [LB_THREADS][J + 1]  sm rows of the block's points
  float* sD = sS + LB_THREADS * sstride;      // [LB_THREADS][J + 1]  dsm rows, then the dW rows
  float* sW = sD + LB_THREADS * sstride;      // [LB_THREADS][J + 1]  W rows
  float* sG = sW + LB_THREADS * sstride;      // [LB_THREADS][13]     dG rows
  for (int i = threadIdx.x; i < J * 12; i += LB_THREADS) sT[i] = T34[i];
  // the block's rows of sm / dsm / W are contiguous: coalesced loads into the LDS tiles
  const int64_t p0 = (int64_t)blockIdx.x * LB_THREADS;
  const int rows = (int)(n - p0 < LB_THREADS ? n - p0 : LB_THREADS);
  const int cnt = rows * J;
  for (int i = threadIdx.x; i < cnt; i += LB_THREADS) {
    const int r = i / J, c = i - r * J;
    sS[r * sstride + c] = sm[p0 * J + i];
    sD[r * sstride + c] = dsm ? dsm[p0 * J + i] : 0.f;
    sW[r * sstride + c] = W[p0 * J + i];
  }
  __syncthreads();
  const int64_t p = p0 + threadIdx.x;
  const bool live = p < n;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const float th_raw = theta[0];
  const float th = fmaxf(eps, th_raw);
  const int64_t q = live ? p : 0;
  float dx[3] = {0.f, 0.f, 0.f};
  if (live && dxyz) { dx[0] = dxyz[3 * q]; dx[1] = dxyz[3 * q + 1]; dx[2] = dxyz[3 * q + 2]; }
  const float px = pcd[3 * q], py = pcd[3 * q + 1], pz = pcd[3 * q + 2];
  float dG[12];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    dG[4 * r] = dx[r] * px; dG[4 * r + 1] = dx[r] * py; dG[4 * r + 2] = dx[r] * pz; dG[4 * r + 3] = dx[r];
  }
  if (live && dRinv) {
    float Ri[9], dR[9], X[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) { Ri[k] = Rinv[9 * q + k]; dR[k] = dRinv[9 * q + k]; }
    // X = dR Ri^T; M = Ri^T X; dA -= M
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) X[3 * r + c] = dR[3 * r] * Ri[3 * c] + dR[3 * r + 1] * Ri[3 * c + 1] + dR[3 * r + 2] * Ri[3 * c + 2];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) dG[4 * r + c] -= Ri[r] * X[c] + Ri[3 + r] * X[3 + c] + Ri[6 + r] * X[6 + c];
  }
  if (!live) {
#pragma unroll
    for (int k = 0; k < 12; ++k) dG[k] = 0.f;
  }
#pragma unroll
  for (int k = 0; k < 12; ++k) sG[threadIdx.x * 13 + k] = dG[k];
  float* smr = sS + threadIdx.x * sstride;
  float* dsr = sD + threadIdx.x * sstride;
  const float* wr = sW + threadIdx.x * sstride;
  // pass 1: sum_k sm_k dsm_tot_k
  float ssd = 0.f;
  for (int j = 0; j < J; ++j) {
    float t = live ? dsr[j] : 0.f;
#pragma unroll
    for (int k = 0; k < 12; ++k) t += dG[k] * sT[12 * j + k];
    ssd += (live ? smr[j] : 0.f) * t;
  }
  // pass 2: dW (into the dsm row, stored coalesced below), dtheta; dead rows of the sm tile
  // are zeroed for the dT partial
  float dth = 0.f;
  for (int j = 0; j < J; ++j) {
    float t = live ? dsr[j] : 0.f;
#pragma unroll
    for (int k = 0; k < 12; ++k) t += dG[k] * sT[12 * j + k];
    const float s_j = live ? smr[j] : 0.f;
    const float dz = s_j * (t - ssd);
    dsr[j] = dz / th;
    dth -= dz * (live ? wr[j] : 0.f);
    smr[j] = s_j;
  }
  dth = th_raw > eps ? dth / (th * th) : 0.f;
  const float e0 = wave_sum(dx[0]), e1 = wave_sum(dx[1]), e2 = wave_sum(dx[2]), e3 = wave_sum(live ? dth : 0.f);
  if (lane == 0) { sRed[wid][0] = e0; sRed[wid][1] = e1; sRed[wid][2] = e2; sRed[wid][3] = e3; }
  __syncthreads();
  for (int i = threadIdx.x; i < cnt; i += LB_THREADS) {
    const int r = i / J, c = i - r * J;
    dW[p0 * J + i] = sD[r * sstride + c];
  }
  const int nv = 12 * J + 4;
  float* out = part + (int64_t)blockIdx.x * nv;
  // dT partial: thread per (j, k), the block's points in order
  for (int o = threadIdx.x; o < 12 * J; o += LB_THREADS) {
    const int j = o / 12, k = o - 12 * j;
    float acc = 0.f;
#pragma unroll 8
    for (int r = 0; r < LB_THREADS; ++r) acc += sS[r * sstride + j] * sG[r * 13 + k];
    out[o] = acc;
  }
  if (threadIdx.x < 4) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < LB_THREADS / 64; ++w) v += sRed[w][threadIdx.x];
    out[12 * J + threadIdx.x] = v;
  }
}

// one block per reduced value (12 J + 4 of them): the block's threads stride over the per-block
// partials, then a fixed shuffle tree + a fixed combine of the wave sums (deterministic)
__global__ __launch_bounds__(256) void k_lbs_train_reduce(const float* __restrict__ part, int nblocks, int J,
                                                          float* __restrict__ dT34, float* __restrict__ dgt,
                                                          float* __restrict__ dtheta) {
  __shared__ float sw[4];
  const int nv = 12 * J + 4;
  const int i = blockIdx.x;
  float v = 0.f;
  for (int b = threadIdx.x; b < nblocks; b += 256) v += part[(int64_t)b * nv + i];
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) sw[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x != 0) return;
  v = (sw[0] + sw[1]) + (sw[2] + sw[3]);
  if (i < 12 * J) dT34[i] = v;
  else if (i < 12 * J + 3) dgt[i - 12 * J] = v;
  else dtheta[0] = v;
}

}  // namespace apn

using namespace apn;

extern "C" size_t apn_lbs_train_workspace_bytes(int64_t n_points, int32_t n_joints) {
  return (size_t)ceil_div(n_points > 0 ? n_points : 1, LB_THREADS) * (12 * (size_t)n_joints + 4) * sizeof(float);
}

extern "C" int apn_lbs_train_fwd(const float* pcd, const float* W, int64_t n, int32_t J, const float* theta,
                                 float eps, const float* T34, const float* global_t, float* sm_out, float* G12_out,
                                 float* xyz_out, float* Rinv_out, void* stream) {
  if (n < 0 || J < 1 || J > LT_MAXJ) return APN_ERR_ARG;
  if (n == 0) return APN_OK;
  if (!pcd || !W || !theta || !T34 || !global_t || !sm_out || !G12_out || !xyz_out || !Rinv_out) return APN_ERR_ARG;
  hipLaunchKernelGGL(k_lbs_train_fwd, dim3(ceil_div(n, LT_THREADS)), dim3(LT_THREADS),
                     (size_t)LT_THREADS * (J + 1) * sizeof(float), (hipStream_t)stream, pcd,
                     W, n, (int)J, theta, eps, T34, global_t, sm_out, G12_out, xyz_out, Rinv_out);
  return launch_status();
}

extern "C" int apn_lbs_train_bwd(const float* pcd, const float* W, int64_t n, int32_t J, const float* theta,
                                 float eps, const float* T34, const float* sm, const float* Rinv,
                                 const float* d_xyz, const float* d_Rinv, const float* d_sm, float* dW,
                                 float* dT34, float* d_global_t, float* d_theta, void* workspace, void* stream) {
  if (n < 1 || J < 1 || J > LT_MAXJ) return APN_ERR_ARG;
  if (!pcd || !W || !theta || !T34 || !sm || !Rinv || !dW || !dT34 || !d_global_t || !d_theta || !workspace)
    return APN_ERR_ARG;
  const int nb = ceil_div(n, LB_THREADS);
  float* part = (float*)workspace;
  const size_t lds = (size_t)LB_THREADS * (3 * (J + 1) + 13) * sizeof(float);
  hipLaunchKernelGGL(k_lbs_train_bwd, dim3(nb), dim3(LB_THREADS), lds, (hipStream_t)stream, pcd, W, n, (int)J, theta,
                     eps, T34, sm, Rinv, d_xyz, d_Rinv, d_sm, dW, part);
  hipLaunchKernelGGL(k_lbs_train_reduce, dim3(12 * J + 4), dim3(256), 0, (hipStream_t)stream, part,
                     nb, (int)J, dT34, d_global_t, d_theta);
  return launch_status();
}
