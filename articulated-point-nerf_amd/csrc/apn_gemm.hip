// fp32 GEMMs of the training step (feat_net / heads / TransformNet Linear layers, forward and
// backward; run.py:574-716 trains them through temporalpoints.py:491-515 and pointwarper.py:5-37)
// on v_mfma_f32_16x16x4_f32 -- f32 operands, f32 accumulate, every product and sum an exact f32
// fma (MI355X_MICROARCH.md: the f32-input MFMA is the f32 fma chain bit for bit), so the results
// are those of a float32 GEMM in this kernel's summation order.
//
//   C[m][n] = epi( sum_k opA[m][k] * opB[k][n] )
//   opA = A (row-major M x K, lda) or A^T (A stored K x M);  opB = B (K x N) or B^T (B stored N x K)
//   A2 (optional): opA *= (A2 > 0 ? 1 : slope_mask) elementwise on load -- the LeakyReLU
//                  derivative of the layer's output applied to the incoming gradient;
//   ones_col:      column N - 1 of opB reads 1 (the bias gradient rides as one more output column);
//   epi:           + bias[n], then LeakyReLU(slope_act) when act.
// Split-K over blockIdx.z writes partial products to C + z * M * ldc (apn_gemm_f32_splitk sums
// them in a fixed order), so every result is deterministic.
//
// Tile: 64 x 64 outputs per 256-thread workgroup, K in steps of 16 staged through LDS ([k][m]
// and [k][n], rows padded to 80 floats so the MFMA operand reads of the two 16-lane k rows land
// on different banks); wave (wm, wn) owns a 32 x 32 quarter = 2 x 2 MFMA tiles; the next K step's
// operands are loaded into registers while the current one is multiplied.
#include "apn_common.h"

#include <algorithm>

namespace apn {

namespace gemm {

constexpr int BM = 64, BN = 64, BK = 16, PAD = 80, THREADS = 256;
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct Args {
  const float* A;
  const float* A2;
  const float* B;
  float* C;
  const float* bias;
  int64_t M, N, K, lda, ldb, ldc, k_split;
  float slope_mask, slope_act;
  int act, ones_col;
};

template <bool TA, bool TB>
__global__ __launch_bounds__(THREADS) void k_gemm_f32(Args p) {
  __shared__ float As[BK][PAD];
  __shared__ float Bs[BK][PAD];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w & 1, wn = w >> 1;
  const int64_t m0 = (int64_t)blockIdx.x * BM, n0 = (int64_t)blockIdx.y * BN;
  const int64_t kb = (int64_t)blockIdx.z * p.k_split, ke = min(p.K, kb + p.k_split);
  float* const C = p.C + (int64_t)blockIdx.z * p.M * p.ldc;
  float ra[4], rb[4];
  auto load = [&](int64_t k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + THREADS * i;
      int mm, kk;
      if (TA) { kk = e >> 6; mm = e & 63; } else { mm = e >> 4; kk = e & 15; }
      const int64_t gm = m0 + mm, gk = k0 + kk;
      float v = 0.f;
      if (gm < p.M && gk < ke) {
        const int64_t o = TA ? gk * p.lda + gm : gm * p.lda + gk;
        v = p.A[o];
        if (p.A2) v = p.A2[o] > 0.f ? v : (p.slope_mask == 0.f ? 0.f : v * p.slope_mask);
      }
      ra[i] = v;
      int nn;
      if (TB) { nn = e >> 4; kk = e & 15; } else { kk = e >> 6; nn = e & 63; }
      const int64_t gn = n0 + nn, gk2 = k0 + kk;
      float u = 0.f;
      if (gn < p.N && gk2 < ke) {
        if (p.ones_col && gn == p.N - 1)
          u = 1.f;
        else
          u = p.B[TB ? gn * p.ldb + gk2 : gk2 * p.ldb + gn];
      }
      rb[i] = u;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + THREADS * i;
      if (TA) As[e >> 6][e & 63] = ra[i]; else As[e & 15][e >> 4] = ra[i];
      if (TB) Bs[e & 15][e >> 4] = rb[i]; else Bs[e >> 6][e & 63] = rb[i];
    }
  };
  f32x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int li = lane & 15, kq = lane >> 4;
  if (kb < ke) load(kb);
  for (int64_t k0 = kb; k0 < ke; k0 += BK) {
    __syncthreads();   // the previous step's operand reads are done
    store();
    __syncthreads();
    if (k0 + BK < ke) load(k0 + BK);
#pragma unroll
    for (int s = 0; s < BK / 4; ++s) {
      float a[2], b[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        a[t] = As[4 * s + kq][wm * 32 + t * 16 + li];
        b[t] = Bs[4 * s + kq][wn * 32 + t * 16 + li];
      }
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[x], b[y], acc[x][y], 0, 0, 0);
    }
  }
  // lane (li, kq) of tile (x, y) holds rows 4 kq .. 4 kq + 3, column li
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) {
      const int64_t col = n0 + wn * 32 + y * 16 + li;
      if (col >= p.N) continue;
      const float bv = p.bias ? p.bias[col] : 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t row = m0 + wm * 32 + x * 16 + 4 * kq + i;
        if (row >= p.M) continue;
        float v = acc[x][y][i];
        if (p.bias) v = v + bv;
        if (p.act) v = v > 0.f ? v : (p.slope_act == 0.f ? 0.f : v * p.slope_act);   // ReLU: +0
        C[row * p.ldc + col] = v;
      }
    }
}

// out[i] = sum_z part[z * n + i] (z ascending), split into out_main (the first cols of each row
// of width cols + extra) and out_extra (the trailing extra column, the bias gradient).
__global__ __launch_bounds__(256) void k_splitk_reduce(const float* __restrict__ part, int splits, int64_t rows,
                                                       int64_t width, int64_t cols, float* __restrict__ out_main,
                                                       float* __restrict__ out_extra) {
  const int64_t n = rows * width;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float s = 0.f;
    for (int z = 0; z < splits; ++z) s += part[z * n + i];
    const int64_t r = i / width, c = i - r * width;
    if (c < cols)
      out_main[r * cols + c] = s;
    else if (out_extra)
      out_extra[r] = s;
  }
}

template <bool TA, bool TB>
void launch(const Args& a, int splits, hipStream_t s) {
  dim3 grid((unsigned)ceil_div(a.M, BM), (unsigned)ceil_div(a.N, BN), (unsigned)splits);
  hipLaunchKernelGGL((k_gemm_f32<TA, TB>), grid, dim3(THREADS), 0, s, a);
}

int run(const Args& a, int ta, int tb, int splits, hipStream_t s) {
  if (ta && tb) launch<true, true>(a, splits, s);
  else if (ta) launch<true, false>(a, splits, s);
  else if (tb) launch<false, true>(a, splits, s);
  else launch<false, false>(a, splits, s);
  return launch_status();
}

}  // namespace gemm
}  // namespace apn

using namespace apn;

extern "C" int apn_gemm_f32(const float* A, const float* A2, const float* B, float* C, const float* bias, int64_t M,
                            int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int32_t trans_a,
                            int32_t trans_b, float slope_mask, int32_t act, float slope_act, void* stream) {
  if (M < 0 || N < 0 || K < 0 || !A || !B || !C) return APN_ERR_ARG;
  if (M == 0 || N == 0) return APN_OK;
  gemm::Args a{A, A2, B, C, bias, M, N, K, lda, ldb, ldc, K > 0 ? K : 1, slope_mask, slope_act, act, 0};
  return gemm::run(a, trans_a, trans_b, 1, (hipStream_t)stream);
}

extern "C" size_t apn_gemm_f32_splitk_workspace_bytes(int64_t M, int64_t N, int32_t splits) {
  return (size_t)(splits > 0 ? splits : 1) * (size_t)M * (size_t)(N + 1) * sizeof(float);
}

extern "C" int apn_gemm_f32_splitk(const float* A, const float* A2, const float* B, float* C, float* bias_grad,
                                   int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int32_t trans_a,
                                   int32_t trans_b, float slope_mask, int32_t splits, void* workspace,
                                   void* stream) {
  if (M < 0 || N < 0 || K < 0 || !A || !B || !C || !workspace || splits < 1) return APN_ERR_ARG;
  if (M == 0 || N == 0) return APN_OK;
  hipStream_t s = (hipStream_t)stream;
  const int64_t width = N + (bias_grad ? 1 : 0);
  int64_t kc = (K + splits - 1) / splits;
  kc = (kc + gemm::BK - 1) / gemm::BK * gemm::BK;
  if (kc < gemm::BK) kc = gemm::BK;
  const int sp = (int)((K + kc - 1) / kc > 0 ? (K + kc - 1) / kc : 1);
  float* part = (float*)workspace;
  gemm::Args a{A, A2, B, part, nullptr, M, width, K, lda, ldb, width, kc, slope_mask, 0.f, 0, bias_grad ? 1 : 0};
  int rc = gemm::run(a, trans_a, trans_b, sp, s);
  if (rc != APN_OK) return rc;
  const int64_t n = M * width;
  const int blocks = (int)std::min<int64_t>(ceil_div(n, 256), 4096);
  hipLaunchKernelGGL(gemm::k_splitk_reduce, dim3(blocks), dim3(256), 0, s, part, sp, M, width, N, C, bias_grad);
  return launch_status();
}
