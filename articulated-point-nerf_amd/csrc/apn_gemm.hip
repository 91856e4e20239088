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
//   row_sum:       (trans_a only) the row sums of opA over the K range are written beside the
//                  product (the bias gradient: sum over the batch of the incoming gradient);
//   epi:           + bias[n], then LeakyReLU(slope_act) when act.
// Split-K over blockIdx.z writes partial products to C + z * M * ldc (apn_gemm_f32_splitk sums
// them in a fixed order), so every result is deterministic.
//
// Tile: 64 x 128 outputs per 256-thread workgroup (a feat_net layer's 128 outputs in one tile, so
// each activation row is read once), K in steps of 32 staged through LDS in the source's own
// orientation ([m][k] rows of 34 floats or [k][m] rows of 80 / 144: conflict-free MFMA operand
// reads either way) from 16-B loads; wave w owns columns 32 w .. 32 w + 31 of all 64 rows
// (4 x 2 MFMA tiles); the next K step's operands are loaded into registers while the current one
// is multiplied.
#include "apn_common.h"

#include <algorithm>

namespace apn {

namespace gemm {

constexpr int BM = 64, BK = 32, THREADS = 256;
// LDS row strides (floats): K-major tiles [m][k] use BK + 2 (operand reads 2m + kq: the 32 lanes
// of a ds_read_b32 group on 32 banks), M/N-major tiles [k][m] use BM + 16 / BN + 16 (the two
// k rows of a read group 16 banks apart). BN = 64 NT: NT = 2 (128 outputs: the 128-wide layers)
// or 3 (192: feat_net's 191-wide first-layer input gradient and weight).
constexpr int SKM = BK + 2, SAM = BM + 16;
constexpr int A_LDS = (BM * SKM > BK * SAM) ? BM * SKM : BK * SAM;
template <int NT> struct BTile {
  static constexpr int BN = 64 * NT, SBN = BN + 16;
  static constexpr int LDS = (BN * SKM > BK * SBN) ? BN * SKM : BK * SBN;
};
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct Args {
  const float* A;
  const float* A2;
  const float* B;
  float* C;
  float* row_sum;   // [splits][M] when non-null (trans_a)
  const float* bias;
  int64_t M, N, K, lda, ldb, ldc, k_split;
  float slope_mask, slope_act;
  int act, vec_a, vec_b;
};

__device__ __forceinline__ float act_mask(float v, float a2, float slope) {
  return a2 > 0.f ? v : (slope == 0.f ? 0.f : v * slope);
}

// One slot = 4 consecutive elements of a tile along the source's contiguous dimension: a 16-B load
// when the whole slot is in bounds and the operand is 16-B aligned, else 4 guarded loads.
// A tile: BM x BK (8 slots per thread), B tile: BK x BN (8 NT slots per thread).
template <bool TA, bool TB, int NT>
__global__ __launch_bounds__(THREADS) void k_gemm_f32(Args p) {
  constexpr int BN = BTile<NT>::BN, SBN = BTile<NT>::SBN;
  __shared__ __attribute__((aligned(16))) float As[A_LDS];
  __shared__ __attribute__((aligned(16))) float Bs[BTile<NT>::LDS];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int li = lane & 15, kq = lane >> 4;
  const int64_t n0 = (int64_t)blockIdx.y * BN;
  const int64_t kb = (int64_t)blockIdx.z * p.k_split, ke = min(p.K, kb + p.k_split);
  float* const C = p.C + (int64_t)blockIdx.z * p.M * p.ldc;
  const int64_t nreal = p.N;
  f32x4 ra[2], rb[2 * NT];
  f32x4 rs = {0.f, 0.f, 0.f, 0.f};   // trans_a row sums: this thread's 4 rows m0 + 4 (tid & 15) + j
  // Interior tiles (every slot whole and in bounds: a workgroup-uniform test) load their operands
  // with no branch around the loads, and the LeakyReLU-derivative mask and the row sums wait for
  // store(): a load under a per-lane branch, or a value used at once, makes the compiler wait for
  // it right there (the phi copy at the join reads it), which exposed every K step's load latency.
  f32x4 ra2_0 = {0.f, 0.f, 0.f, 0.f}, ra2_1 = {0.f, 0.f, 0.f, 0.f};   // A2 slots of the interior path
  bool a_late = false;
  auto load = [&](int64_t m0, int64_t k0) __attribute__((always_inline)) {
    a_late = p.vec_a && m0 + BM <= p.M && k0 + BK <= ke;
    if (a_late) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int f = tid + THREADS * i;
        const int64_t gk = TA ? k0 + (f >> 4) : k0 + 4 * (f & 7);
        const int64_t gm = TA ? m0 + 4 * (f & 15) : m0 + (f >> 3);
        const int64_t o = TA ? gk * p.lda + gm : gm * p.lda + gk;
        ra[i] = *(const f32x4*)(p.A + o);
        if (p.A2) (i ? ra2_1 : ra2_0) = *(const f32x4*)(p.A2 + o);
      }
    } else {
#pragma unroll
    for (int i = 0; i < 2; ++i) {   // A: 512 slots
      const int f = tid + THREADS * i;
      // TA: source [k][m] contiguous in m (16 slots per k row); else [m][k] contiguous in k (8 per m row)
      const int64_t gk = TA ? k0 + (f >> 4) : k0 + 4 * (f & 7);
      const int64_t gm = TA ? m0 + 4 * (f & 15) : m0 + (f >> 3);
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      const bool full = TA ? (gk < ke && gm + 3 < p.M) : (gm < p.M && gk + 3 < ke);
      if (full && p.vec_a) {
        const int64_t o = TA ? gk * p.lda + gm : gm * p.lda + gk;
        v = *(const f32x4*)(p.A + o);
        if (p.A2) {
          const f32x4 u = *(const f32x4*)(p.A2 + o);
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = act_mask(v[j], u[j], p.slope_mask);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t mm = TA ? gm + j : gm, kk = TA ? gk : gk + j;
          if (mm < p.M && kk < ke) {
            const int64_t o = TA ? kk * p.lda + mm : mm * p.lda + kk;
            v[j] = p.A2 ? act_mask(p.A[o], p.A2[o], p.slope_mask) : p.A[o];
          }
        }
      }
      ra[i] = v;
      if (TA && p.row_sum) rs += v;
    }
    }
    if (p.vec_b && n0 + BN <= nreal && k0 + BK <= ke) {
#pragma unroll
      for (int i = 0; i < 2 * NT; ++i) {
        const int f = tid + THREADS * i;
        const int64_t gk = TB ? k0 + 4 * (f & 7) : k0 + f / (BN / 4);
        const int64_t gn = TB ? n0 + (f >> 3) : n0 + 4 * (f % (BN / 4));
        rb[i] = *(const f32x4*)(p.B + (TB ? gn * p.ldb + gk : gk * p.ldb + gn));
      }
    } else {
#pragma unroll
    for (int i = 0; i < 2 * NT; ++i) {   // B: 512 NT slots
      const int f = tid + THREADS * i;
      // TB: source [n][k] contiguous in k (8 slots per n row); else [k][n] contiguous in n (BN / 4 per k row)
      const int64_t gk = TB ? k0 + 4 * (f & 7) : k0 + f / (BN / 4);
      const int64_t gn = TB ? n0 + (f >> 3) : n0 + 4 * (f % (BN / 4));
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      const bool full = TB ? (gn < nreal && gk + 3 < ke) : (gk < ke && gn + 3 < nreal);
      if (full && p.vec_b) {
        v = *(const f32x4*)(p.B + (TB ? gn * p.ldb + gk : gk * p.ldb + gn));
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t nn = TB ? gn : gn + j, kk = TB ? gk + j : gk;
          if (kk < ke && nn < nreal) v[j] = p.B[TB ? nn * p.ldb + kk : kk * p.ldb + nn];
        }
      }
      rb[i] = v;
    }
    }
  };
  auto store = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int f = tid + THREADS * i;
      f32x4 v = ra[i];
      if (a_late) {   // the interior path's deferred mask and row sums, in the order of the load path
        const f32x4 u = i ? ra2_1 : ra2_0;
        if (p.A2) v = f32x4{act_mask(v[0], u[0], p.slope_mask), act_mask(v[1], u[1], p.slope_mask),
                            act_mask(v[2], u[2], p.slope_mask), act_mask(v[3], u[3], p.slope_mask)};
        if (TA && p.row_sum) rs += v;
      }
      if (TA) {
        *(f32x4*)(As + (f >> 4) * SAM + 4 * (f & 15)) = v;
      } else {
        float* d = As + (f >> 3) * SKM + 4 * (f & 7);
        typedef float f32x2 __attribute__((ext_vector_type(2)));
        *(f32x2*)d = f32x2{v[0], v[1]};
        *(f32x2*)(d + 2) = f32x2{v[2], v[3]};
      }
    }
#pragma unroll
    for (int i = 0; i < 2 * NT; ++i) {
      const int f = tid + THREADS * i;
      if (TB) {
        float* d = Bs + (f >> 3) * SKM + 4 * (f & 7);
        typedef float f32x2 __attribute__((ext_vector_type(2)));
        *(f32x2*)d = f32x2{rb[i][0], rb[i][1]};
        *(f32x2*)(d + 2) = f32x2{rb[i][2], rb[i][3]};
      } else {
        *(f32x4*)(Bs + (f / (BN / 4)) * SBN + 4 * (f % (BN / 4))) = rb[i];
      }
    }
  };
  // wave w: all 64 rows x columns 16 NT w .. 16 NT (w + 1) - 1 (4 x NT MFMA tiles)
  f32x4 acc[4][NT];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  // Persistent over M tiles (grid.x may be smaller than the tile count): the (tile, K step)
  // iterations run as one sequence, so the next tile's first operands load during this tile's last
  // step (a 128-deep K is only 4 steps: per-tile load latency would otherwise stay exposed).
  const int64_t n_mt = (p.M + BM - 1) / BM;
  const int64_t nk = ke > kb ? (ke - kb + BK - 1) / BK : 0;
  const int64_t my = n_mt > (int64_t)blockIdx.x ? (n_mt - 1 - (int64_t)blockIdx.x) / gridDim.x + 1 : 0;
  auto tile_m0 = [&](int64_t j) { return ((int64_t)blockIdx.x + j * gridDim.x) * BM; };
  auto epilogue = [&](int64_t m0) {
    if (TA && p.row_sum && blockIdx.y == 0) {   // the 16 threads sharing rows (tid & 15), fixed order
      __syncthreads();
      *(f32x4*)(As + (tid >> 4) * 64 + 4 * (tid & 15)) = rs;
      __syncthreads();
      if (tid < BM && m0 + tid < p.M) {
        float t = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) t += As[r * 64 + tid];
        p.row_sum[(int64_t)blockIdx.z * p.M + m0 + tid] = t;
      }
    }
    // lane (li, kq) of tile (x, y) holds rows 4 kq .. 4 kq + 3, column li
#pragma unroll
    for (int y = 0; y < NT; ++y) {
      const int64_t col = n0 + w * 16 * NT + y * 16 + li;
      if (col >= p.N) continue;
      const float bv = p.bias ? p.bias[col] : 0.f;
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int64_t row = m0 + x * 16 + 4 * kq + i;
          if (row >= p.M) continue;
          float v = acc[x][y][i];
          if (p.bias) v = v + bv;
          if (p.act) v = v > 0.f ? v : (p.slope_act == 0.f ? 0.f : v * p.slope_act);   // ReLU: +0
          C[row * p.ldc + col] = v;
        }
    }
  };
  if (nk == 0) {   // empty K range: the epilogue of zero products
    for (int64_t j = 0; j < my; ++j) epilogue(tile_m0(j));
    return;
  }
  const int64_t total = my * nk;
  if (total > 0) load(tile_m0(0), kb);
  for (int64_t it = 0; it < total; ++it) {
    __syncthreads();   // the previous step's operand reads are done
    store();
    __syncthreads();
    if (it + 1 < total) load(tile_m0((it + 1) / nk), kb + ((it + 1) % nk) * BK);
#pragma unroll
    for (int s = 0; s < BK / 4; ++s) {
      const int k = 4 * s + kq;
      float a[4], b[NT];
#pragma unroll
      for (int t = 0; t < 4; ++t) a[t] = TA ? As[k * SAM + t * 16 + li] : As[(t * 16 + li) * SKM + k];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int n = w * 16 * NT + t * 16 + li;
        b[t] = TB ? Bs[n * SKM + k] : Bs[k * SBN + n];
      }
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < NT; ++y) acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[x], b[y], acc[x][y], 0, 0, 0);
    }
    if (it % nk == nk - 1) {
      epilogue(tile_m0(it / nk));
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < NT; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
}

// out[o] = sum_z part[z * n + o] for o < n: 8 lanes per output each sum every 8th split (z
// ascending), then a fixed xor tree -- deterministic.
__global__ __launch_bounds__(256) void k_splitk_reduce(const float* __restrict__ part, int splits, int64_t n,
                                                       float* __restrict__ out) {
  const int zl = threadIdx.x & 7;
  for (int64_t o = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 3; o < n; o += (int64_t)gridDim.x * 32) {
    float s = 0.f;
#pragma unroll 4
    for (int z = zl; z < splits; z += 8) s += part[(int64_t)z * n + o];
    s += __shfl_xor(s, 1, 8);
    s += __shfl_xor(s, 2, 8);
    s += __shfl_xor(s, 4, 8);
    if (zl == 0) out[o] = s;
  }
}

template <bool TA, bool TB, int NT>
void launch(const Args& a, int splits, hipStream_t s) {
  // one M tile per workgroup: a persistent grid of the resident workgroups (4 per CU), each
  // looping over its tiles with the next tile's operands loaded during the last K step, measured
  // slower at C2 (forward 93 -> 122 us, dX 115 -> 155 us): the hardware's own refill of finished
  // workgroups overlaps loads and MFMAs better than one register stage per workgroup
  dim3 grid((unsigned)ceil_div(a.M, BM), (unsigned)ceil_div(a.N, BTile<NT>::BN), (unsigned)splits);
  hipLaunchKernelGGL((k_gemm_f32<TA, TB, NT>), grid, dim3(THREADS), 0, s, a);
}

inline int vec_ok(const float* p, int64_t ld) { return ((uintptr_t)p % 16 == 0) && (ld % 4 == 0); }

template <int NT>
void run_nt(const Args& a, int ta, int tb, int splits, hipStream_t s) {
  if (ta && tb) launch<true, true, NT>(a, splits, s);
  else if (ta) launch<true, false, NT>(a, splits, s);
  else if (tb) launch<false, true, NT>(a, splits, s);
  else launch<false, false, NT>(a, splits, s);
}

// 192-wide tiles when they cover N in fewer column tiles than 128-wide ones (N in 129..192)
int run(const Args& a, int ta, int tb, int splits, hipStream_t s) {
  if (ceil_div(a.N, 192) < ceil_div(a.N, 128)) run_nt<3>(a, ta, tb, splits, s);
  else run_nt<2>(a, ta, tb, splits, s);
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
  gemm::Args a{A, A2, B, C, nullptr, bias, M, N, K, lda, ldb, ldc, K > 0 ? K : 1, slope_mask, slope_act, act,
               gemm::vec_ok(A, lda) && (!A2 || gemm::vec_ok(A2, lda)), gemm::vec_ok(B, ldb)};
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
  if (bias_grad && !trans_a) return APN_ERR_ARG;   // row sums are gathered by the trans_a loader
  if (M == 0 || N == 0) return APN_OK;
  hipStream_t s = (hipStream_t)stream;
  int64_t kc = (K + splits - 1) / splits;
  kc = (kc + gemm::BK - 1) / gemm::BK * gemm::BK;
  if (kc < gemm::BK) kc = gemm::BK;
  const int sp = (int)((K + kc - 1) / kc > 0 ? (K + kc - 1) / kc : 1);
  float* part = (float*)workspace;
  float* rsum = part + (int64_t)sp * M * N;
  gemm::Args a{A, A2, B, part, bias_grad ? rsum : nullptr, nullptr, M, N, K, lda, ldb, N, kc, slope_mask, 0.f, 0,
               gemm::vec_ok(A, lda) && (!A2 || gemm::vec_ok(A2, lda)), gemm::vec_ok(B, ldb)};
  int rc = gemm::run(a, trans_a, trans_b, sp, s);
  if (rc != APN_OK) return rc;
  const int64_t n = M * N;
  hipLaunchKernelGGL(gemm::k_splitk_reduce, dim3((unsigned)std::min<int64_t>(ceil_div(n, 32), 4096)), dim3(256), 0, s,
                     part, sp, n, C);
  if (bias_grad)
    hipLaunchKernelGGL(gemm::k_splitk_reduce, dim3((unsigned)std::min<int64_t>(ceil_div(M, 32), 4096)), dim3(256), 0,
                       s, rsum, sp, M, bias_grad);
  return launch_status();
}
