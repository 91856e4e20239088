// Forward LBS skinning of the canonical cloud, one point per thread.
//
// Fuses, per point n:
//   get_weights            temporalpoints.py:401-414   w = merge(softmax(W[n] / max(eps, theta)))
//   PointWarper blend      pointwarper.py:241-266      G = sum_j w_j T_j ; x' = G [x;1] + global_t
//   torch.inverse(G)[:3,:3] temporalpoints.py:569,478  Rinv = inverse(G[:3,:3]) (adjugate)
//   direct-render sigma    temporalpoints.py:460-461   den = 2 (mmd * max(eps_n,0))^2 + 1e-12
//   weight-vis colour      temporalpoints.py:690-701   pcol = sum_j col_j w_j (double, rounded)
//   bbox of x'             temporalpoints.py:424       atomic min/max on order-preserving ints
// and writes the per-point records the kNN / MLP stages gather:
//   recA[n] = {x', y', z', den, Rinv(9, row-major), clip(alpha,0,1), 0, 0}   (64 B)
//   recB[n] = {clip(rgb,0,1), clip(alpha,0,1), pcol, 0}                      (32 B)
// (alpha twice: the direct blend reads recA's first and recB's two float4s, not recA[3])
// HBM-bound: per point it reads 12 + 4J + 4 + 12 + 4 bytes and writes 12 + 4J + 96 bytes.
#include "apn_common.h"
#include "apn_mlp_split.h"   // split4 (the hi/lo fp16 split of the 3-term MFMA)

#include <algorithm>

namespace apn {

constexpr int LBS_THREADS = 256;
constexpr int LBS_MAX_J = 64;
#ifndef QUAD_WAVES_PER_EU
#define QUAD_WAVES_PER_EU 4
#endif
#ifndef LBS_PF
#define LBS_PF 1   // rows in flight ahead of the one being skinned (k_lbs_skin_quad)
#endif

// Per-point tail shared by the LBS kernels: x' = G [x;1] + global_t, optional G (get_frames),
// records (adjugate inverse of the blended 3x3, direct-render sigma, clipped colours); bbox seed.
__device__ __forceinline__ void lbs_finish(int64_t n, const float (&G)[12], float sw, double pc0, double pc1, double pc2,
                                           const float* __restrict__ pcd, const float* __restrict__ global_t, float mmd,
                                           const float* __restrict__ direct_eps, const float* __restrict__ alpha_c,
                                           const float* __restrict__ rgb_c, float* __restrict__ xyz_out,
                                           float* __restrict__ G_out, float4* __restrict__ recA,
                                           float4* __restrict__ recB, float (&bmin)[3], float (&bmax)[3]) {
  if (G_out) {  // weighted_G_tw (pointwarper.py:243): rows 0..2 blended, row 3 = sum_j w_j [0,0,0,1]
    float4* go = (float4*)(G_out + 16 * n);
    go[0] = make_float4(G[0], G[1], G[2], G[3]);
    go[1] = make_float4(G[4], G[5], G[6], G[7]);
    go[2] = make_float4(G[8], G[9], G[10], G[11]);
    go[3] = make_float4(0.f, 0.f, 0.f, sw);
  }
  const float px = pcd[3 * n], py = pcd[3 * n + 1], pz = pcd[3 * n + 2];
  float x = ((G[0] * px + G[1] * py) + G[2] * pz) + G[3];
  float y = ((G[4] * px + G[5] * py) + G[6] * pz) + G[7];
  float z = ((G[8] * px + G[9] * py) + G[10] * pz) + G[11];
  x = x + global_t[0]; y = y + global_t[1]; z = z + global_t[2];
  xyz_out[3 * n] = x; xyz_out[3 * n + 1] = y; xyz_out[3 * n + 2] = z;
  bmin[0] = bmax[0] = x; bmin[1] = bmax[1] = y; bmin[2] = bmax[2] = z;
  if (recA) {
    // inverse of the blended 3x3 (adjugate / det)
    const float a00 = G[0], a01 = G[1], a02 = G[2], a10 = G[4], a11 = G[5], a12 = G[6];
    const float a20 = G[8], a21 = G[9], a22 = G[10];
    const float c00 = a11 * a22 - a12 * a21, c01 = a02 * a21 - a01 * a22, c02 = a01 * a12 - a02 * a11;
    const float c10 = a12 * a20 - a10 * a22, c11 = a00 * a22 - a02 * a20, c12 = a02 * a10 - a00 * a12;
    const float c20 = a10 * a21 - a11 * a20, c21 = a01 * a20 - a00 * a21, c22 = a00 * a11 - a01 * a10;
    const float det = (a00 * c00 + a01 * c10) + a02 * c20;
    const float id = 1.f / det;
    const float sig = mmd * fmaxf(direct_eps[n], 0.f);
    const float den = 2.f * (sig * sig) + 1e-12f;
    const float ac = fminf(fmaxf(alpha_c[n], 0.f), 1.f);
    recA[4 * n + 0] = make_float4(x, y, z, den);
    recA[4 * n + 1] = make_float4(c00 * id, c01 * id, c02 * id, c10 * id);
    recA[4 * n + 2] = make_float4(c11 * id, c12 * id, c20 * id, c21 * id);
    recA[4 * n + 3] = make_float4(c22 * id, ac, 0.f, 0.f);
    const float r = fminf(fmaxf(rgb_c[3 * n], 0.f), 1.f);
    const float g = fminf(fmaxf(rgb_c[3 * n + 1], 0.f), 1.f);
    const float b = fminf(fmaxf(rgb_c[3 * n + 2], 0.f), 1.f);
    recB[2 * n + 0] = make_float4(r, g, b, ac);
    recB[2 * n + 1] = make_float4((float)pc0, (float)pc1, (float)pc2, 0.f);
  }  // recA
}

// bbox: wave reduce, then across the block's waves; one partial per block, reduced by
// k_bbox_reduce (all blocks hitting 6 global atomics serialised at one L2 channel and cost
// ~0.3 ms at 300k points)
__device__ __forceinline__ void lbs_bbox_partial(const float (&bmin)[3], const float (&bmax)[3],
                                                 int* __restrict__ bbox_part) {
  const int tid = threadIdx.x;
  __shared__ float sbb[LBS_THREADS / 64][6];
  const int lane = tid & 63, wid = tid >> 6;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    float lo = bmin[a], hi = bmax[a];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      lo = fminf(lo, __shfl_xor(lo, o, 64));
      hi = fmaxf(hi, __shfl_xor(hi, o, 64));
    }
    if (lane == 0) {
      sbb[wid][a] = lo;
      sbb[wid][3 + a] = hi;
    }
  }
  __syncthreads();
  if (tid < 6) {
    float v = sbb[0][tid];
    for (int w = 1; w < LBS_THREADS / 64; ++w) v = tid < 3 ? fminf(v, sbb[w][tid]) : fmaxf(v, sbb[w][tid]);
    bbox_part[6 * blockIdx.x + tid] = float_to_ordered(v);
  }
}

__global__ __launch_bounds__(LBS_THREADS) void k_lbs_skin(
    const float* __restrict__ pcd, const float* __restrict__ W, int64_t N, int J,
    const float* __restrict__ theta_weight, float eps, const int* __restrict__ rules,
    const float* __restrict__ boneT12, const float* __restrict__ global_t, const float* __restrict__ colors,
    const float* __restrict__ alpha_c, const float* __restrict__ rgb_c, const float* __restrict__ direct_eps,
    float mmd, int weights_final, float* __restrict__ xyz_out, float* __restrict__ w_out,
    float* __restrict__ G_out, float4* __restrict__ recA, float4* __restrict__ recB, int* __restrict__ bbox_part) {
  extern __shared__ float lds[];
  const int Jp = J + 1;                          // odd row stride: conflict-free row reads
  float* sW = lds;                               // [LBS_THREADS][Jp]
  float* sT = sW + LBS_THREADS * Jp;             // [J][12]
  float* sC = sT + J * 12;                       // [J][3]
  int* sR = (int*)(sC + J * 3);                  // [J]
  const int tid = threadIdx.x;
  const int64_t n0 = (int64_t)blockIdx.x * LBS_THREADS;
  const int nvalid = (int)min<int64_t>(LBS_THREADS, N - n0);

  for (int e = tid; e < J * 12; e += LBS_THREADS) sT[e] = boneT12[e];
  for (int e = tid; e < J * 3; e += LBS_THREADS) sC[e] = colors ? colors[e] : 0.f;
  for (int e = tid; e < J; e += LBS_THREADS) sR[e] = rules ? rules[e] : e;
  // coalesced staging of the raw weight tile
  const float* Wt = W + n0 * J;
  const int tile_elems = nvalid * J;
  for (int e = tid; e < tile_elems; e += LBS_THREADS) {
    const int r = e / J, c = e - r * J;
    sW[r * Jp + c] = Wt[e];
  }
  __syncthreads();

  const bool valid = tid < nvalid;
  float bmin[3] = {INFINITY, INFINITY, INFINITY}, bmax[3] = {-INFINITY, -INFINITY, -INFINITY};
  if (valid) {
    const int64_t n = n0 + tid;
    float* row = sW + tid * Jp;
    if (!weights_final) {
    const float th = fmaxf(eps, theta_weight[0]);
    // softmax(W / th) over J (temporalpoints.py:403)
    float m = -INFINITY;
    for (int j = 0; j < J; ++j) {
      const float x = row[j] / th;
      row[j] = x;
      m = fmaxf(m, x);
    }
    float s = 0.f;
    for (int j = 0; j < J; ++j) {
      const float e = expf(row[j] - m);
      row[j] = e;
      s += e;
    }
    const float inv = 1.f / s;
    bool ident = true;
    for (int j = 0; j < J; ++j) ident &= (sR[j] == j);
    if (ident) {
      for (int j = 0; j < J; ++j) row[j] = row[j] * inv;
    } else {
      // merge columns (sequential in k, temporalpoints.py:412)
      float tmp[LBS_MAX_J];
      for (int j = 0; j < J; ++j) tmp[j] = 0.f;
      for (int k = 0; k < J; ++k) tmp[sR[k]] += row[k] * inv;
      for (int j = 0; j < J; ++j) row[j] = tmp[j];
    }
    }  // !weights_final
    // blend bone transforms (pointwarper.py:243)
    float G[12];
#pragma unroll
    for (int e = 0; e < 12; ++e) G[e] = 0.f;
    double pc0 = 0.0, pc1 = 0.0, pc2 = 0.0;
    for (int j = 0; j < J; ++j) {
      const float w = row[j];
      const float* T = sT + 12 * j;
#pragma unroll
      for (int e = 0; e < 12; ++e) G[e] = G[e] + w * T[e];
      pc0 += (double)sC[3 * j] * (double)w;
      pc1 += (double)sC[3 * j + 1] * (double)w;
      pc2 += (double)sC[3 * j + 2] * (double)w;
    }
    float sw = 0.f;
    if (G_out)
      for (int j = 0; j < J; ++j) sw = sw + row[j];
    lbs_finish(n, G, sw, pc0, pc1, pc2, pcd, global_t, mmd, direct_eps, alpha_c, rgb_c, xyz_out, G_out, recA, recB,
               bmin, bmax);
  }
  __syncthreads();
  if (w_out) {
    float* Wo = w_out + n0 * J;
    for (int e = tid; e < tile_elems; e += LBS_THREADS) {
      const int r = e / J, c = e - r * J;
      Wo[e] = sW[r * Jp + c];
    }
  }
  if (bbox_part) lbs_bbox_partial(bmin, bmax, bbox_part);
}

// Per-block bbox partials -> bbox_ord[6] (one workgroup, deterministic).
__global__ __launch_bounds__(256) void k_bbox_reduce(const int* __restrict__ part, int nblocks,
                                                     int* __restrict__ bbox_ord) {
  __shared__ int s[256][6];
  const int tid = threadIdx.x;
  int v[6] = {0x7f800000, 0x7f800000, 0x7f800000, (int)0x807fffff, (int)0x807fffff, (int)0x807fffff};
  for (int b = tid; b < nblocks; b += 256)
    for (int a = 0; a < 6; ++a) v[a] = a < 3 ? min(v[a], part[6 * b + a]) : max(v[a], part[6 * b + a]);
  for (int a = 0; a < 6; ++a) s[tid][a] = v[a];
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (tid < st)
      for (int a = 0; a < 6; ++a) s[tid][a] = a < 3 ? min(s[tid][a], s[tid + st][a]) : max(s[tid][a], s[tid + st][a]);
    __syncthreads();
  }
  if (tid < 6) bbox_ord[tid] = s[0][tid];
}

}  // namespace apn

using namespace apn;

extern "C" size_t apn_lbs_workspace_bytes(int64_t n_points) {
  // one bbox partial per block; the quad kernel runs LBS_THREADS / 4 points per block
  return n_points > 0 ? (size_t)ceil_div(n_points, LBS_THREADS / 4) * 6 * sizeof(int) : 0;
}

// xor-1 / xor-2 lane exchange inside a quad as DPP quad_perm moves (no LDS crossbar)
template <int CTRL>
__device__ __forceinline__ float quad_swap(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
template <int CTRL>
__device__ __forceinline__ double quad_swap(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffff), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, true);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
constexpr int QX1 = 0xB1, QX2 = 0x4E;   // quad_perm [1,0,3,2] and [2,3,0,1]

template <int JL>
__device__ __forceinline__ void quad_load_row(const float* __restrict__ src, float (&row)[JL]) {
  if constexpr (JL % 4 == 0) {
#pragma unroll
    for (int q = 0; q < JL / 4; ++q) {
#ifdef APN_LBS_NT   // A/B: streamed once, non-temporal
      typedef float f4v __attribute__((ext_vector_type(4)));
      const f4v w = __builtin_nontemporal_load((const f4v*)src + q);
      const float4 v = make_float4(w[0], w[1], w[2], w[3]);
#else
      const float4 v = ((const float4*)src)[q];
#endif
      row[4 * q] = v.x; row[4 * q + 1] = v.y; row[4 * q + 2] = v.z; row[4 * q + 3] = v.w;
    }
  } else if constexpr (JL % 2 == 0) {
#pragma unroll
    for (int q = 0; q < JL / 2; ++q) {
      const float2 v = ((const float2*)src)[q];
      row[2 * q] = v.x; row[2 * q + 1] = v.y;
    }
  } else {
#pragma unroll
    for (int q = 0; q < JL; ++q) row[q] = src[q];
  }
}

// Quad variant (record-free calls, identity merge rules, J % 4 == 0): four lanes share a point,
// each holding JL = J/4 consecutive weights in registers -- a point's 4J-byte row is read by its
// quad as one contiguous run (16/8-B loads), there is no LDS weight tile (which capped the LDS
// kernel at 3 blocks per CU at J = 48) and no staging barrier. Softmax max / sum and the blended G
// are combined across the quad with DPP moves ((q0 + q1) + (q2 + q3): sums regrouped by quarter,
// ~1 ulp from the sequential order of k_lbs_skin); lane 0 of the quad runs the per-point tail.
template <int JL>
__global__ __launch_bounds__(LBS_THREADS) __attribute__((amdgpu_waves_per_eu(QUAD_WAVES_PER_EU)))
void k_lbs_skin_quad(
    const float* __restrict__ pcd, const float* __restrict__ W, int64_t N, const float* __restrict__ theta_weight,
    float eps, const float* __restrict__ boneT12, const float* __restrict__ global_t,
    const float* __restrict__ colors, const float* __restrict__ alpha_c, const float* __restrict__ rgb_c,
    const float* __restrict__ direct_eps, float mmd, int weights_final, float* __restrict__ xyz_out,
    float* __restrict__ w_out, float* __restrict__ G_out, float4* __restrict__ recA, float4* __restrict__ recB,
    int* __restrict__ bbox_part) {
  constexpr int J = 4 * JL;
  constexpr int PPB = LBS_THREADS / 4;   // points per block step
  __shared__ __attribute__((aligned(16))) float sT[J * 12];
  __shared__ float sC[J * 3];
  const int tid = threadIdx.x, sub = tid & 3;
  for (int e = tid; e < J * 12; e += LBS_THREADS) sT[e] = boneT12[e];
  for (int e = tid; e < J * 3; e += LBS_THREADS) sC[e] = colors ? colors[e] : 0.f;
  const float th = weights_final ? 1.f : fmaxf(eps, theta_weight[0]);
  const float rth = 1.f / th;   // IEEE reciprocal, once per thread
  const int64_t stride = (int64_t)gridDim.x * PPB;
  int64_t n = (int64_t)blockIdx.x * PPB + (tid >> 2);
  // the next LBS_PF rows are in flight while the current one is processed (grid-stride)
  float nrow[LBS_PF][JL];
#pragma unroll
  for (int d = 0; d < LBS_PF; ++d) quad_load_row<JL>(W + min(n + d * stride, N - 1) * J + sub * JL, nrow[d]);
  __syncthreads();
  float bmin[3] = {INFINITY, INFINITY, INFINITY}, bmax[3] = {-INFINITY, -INFINITY, -INFINITY};
  const int64_t n_end = (N + PPB - 1) / PPB * PPB;   // every lane of a quad runs the same trips
  for (; n < n_end; n += stride) {
    const bool valid = n < N;
    float row[JL];
#pragma unroll
    for (int j = 0; j < JL; ++j) row[j] = nrow[0][j];
#pragma unroll
    for (int d = 0; d + 1 < LBS_PF; ++d)
#pragma unroll
      for (int j = 0; j < JL; ++j) nrow[d][j] = nrow[d + 1][j];
    quad_load_row<JL>(W + min(n + LBS_PF * stride, N - 1) * J + sub * JL, nrow[LBS_PF - 1]);
    if (!weights_final) {   // softmax(W / th) over J (temporalpoints.py:403)
      // W / th as the reciprocal product plus one fma residual correction (3 VALU instead of the
      // ~10 of an IEEE division; the corrected quotient is the correctly rounded one)
      float m = -INFINITY;
#pragma unroll
      for (int j = 0; j < JL; ++j) {
        const float q = row[j] * rth;
        row[j] = fmaf(fmaf(-q, th, row[j]), rth, q);
        m = fmaxf(m, row[j]);
      }
      m = fmaxf(m, quad_swap<QX1>(m));
      m = fmaxf(m, quad_swap<QX2>(m));
      // exp(x - m) on the transcendental unit (v_exp_f32 = 2^x): x - m <= 0, so the argument
      // rounding costs w |x - m| 2^-24 log2(e) absolute per weight (<= 3e-8, as w e^-d d <= 1/e)
      float sum = 0.f;
#pragma unroll
      for (int j = 0; j < JL; ++j) {
        row[j] = __builtin_amdgcn_exp2f((row[j] - m) * 1.4426950408889634f);
        sum += row[j];
      }
      sum += quad_swap<QX1>(sum);
      sum += quad_swap<QX2>(sum);
      const float inv = 1.f / sum;
#pragma unroll
      for (int j = 0; j < JL; ++j) row[j] = row[j] * inv;
    }
    float G[12];
#pragma unroll
    for (int e = 0; e < 12; ++e) G[e] = 0.f;
#pragma unroll
    for (int j = 0; j < JL; ++j) {
      const float4* T4 = (const float4*)(sT + 12 * (sub * JL + j));
      const float4 t0 = T4[0], t1 = T4[1], t2 = T4[2];
      const float T[12] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w, t2.x, t2.y, t2.z, t2.w};
      // fused multiply-add (v_pk_fma_f32: two per instruction); the record-free kernel's bar is
      // fp32 reassociation, not the render path's bit-exact skinned cloud
#pragma unroll
      for (int e = 0; e < 12; ++e) G[e] = fmaf(row[j], T[e], G[e]);
      __builtin_amdgcn_sched_barrier(0);   // one joint's bone row live at a time
    }
#pragma unroll
    for (int e = 0; e < 12; ++e) {
      G[e] += quad_swap<QX1>(G[e]);
      G[e] += quad_swap<QX2>(G[e]);
    }
    double pc0 = 0.0, pc1 = 0.0, pc2 = 0.0;
    if (colors) {
#pragma unroll
      for (int j = 0; j < JL; ++j) {
        const float* c = sC + 3 * (sub * JL + j);
        pc0 += (double)c[0] * (double)row[j];
        pc1 += (double)c[1] * (double)row[j];
        pc2 += (double)c[2] * (double)row[j];
      }
      pc0 += quad_swap<QX1>(pc0); pc0 += quad_swap<QX2>(pc0);
      pc1 += quad_swap<QX1>(pc1); pc1 += quad_swap<QX2>(pc1);
      pc2 += quad_swap<QX1>(pc2); pc2 += quad_swap<QX2>(pc2);
    }
    float sw = 0.f;
    if (G_out) {
#pragma unroll
      for (int j = 0; j < JL; ++j) sw = sw + row[j];
      sw += quad_swap<QX1>(sw);
      sw += quad_swap<QX2>(sw);
    }
    if (w_out && valid) {
      float* dst = w_out + n * J + sub * JL;
#pragma unroll
      for (int j = 0; j < JL; ++j) dst[j] = row[j];
    }
    if (valid && sub == 0) {
      float lo[3], hi[3];
      lbs_finish(n, G, sw, pc0, pc1, pc2, pcd, global_t, mmd, direct_eps, alpha_c, rgb_c, xyz_out, G_out, nullptr,
                 nullptr, lo, hi);
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        bmin[a] = fminf(bmin[a], lo[a]);
        bmax[a] = fmaxf(bmax[a], hi[a]);
      }
    }
  }
  if (bbox_part) lbs_bbox_partial(bmin, bmax, bbox_part);
}

// MFMA variant of the record-free softmax blend (repose / LBS-only sweeps: x' only, no weights,
// G, colours, records or bbox written). A wave skins 16 points per step: lane (n, g) = (lane & 15,
// lane >> 4) holds joints g*JL .. g*JL + JL - 1 of point n -- the quad kernel's per-lane 48-B
// segment of the row, so the loads are the same -- and the blend G^T[12 x 16 points] =
// T^T[12 x J] W^T[J x 16] is one 16x16 product on v_mfma_f32_16x16x32_f16 with the 3-term fp16
// split (hi*hi + hi*lo + lo*hi, fp32 accumulate; apn_mlp_h3.hip), K = the lane's joints in one or
// two 8-wide chunks. In the product's B layout lane (n, g) holds exactly its own weights and in the
// A layout lane (m, g) bone element m of the same joints (registers, once per launch), so no
// operand moves between lanes; the result lane (n, g) holds row g of point n's G, i.e. x'[g]
// directly. Against the quad kernel this removes the 12 FMA per joint of the VALU blend and the
// bone-row LDS reads (36 ds_read_b128 per 16 points); the softmax stays on the VALU (max and sum
// across the point's four lanes by permlane swaps, grouped (g0 + g1) + (g2 + g3) as the quad's
// DPP sums), its normalisation applied to the 12 blended values instead of the J weights. The
// exponentials are split as e 2^12 (exact; e <= 1) so that no weight above 2^-36 meets an fp16
// subnormal. Bar: fp32 reassociation (~2^-22 relative per product, tests/test_hip_parity.py).
typedef _Float16 lbs_h8 __attribute__((ext_vector_type(8)));
typedef float lbs_f4 __attribute__((ext_vector_type(4)));
#ifndef MFMA_WAVES_PER_EU
#define MFMA_WAVES_PER_EU 5
#endif
#ifndef LBS_MFMA_PF
#define LBS_MFMA_PF 1   // 16-point groups in flight ahead of the one being skinned, per wave
#endif

__device__ __forceinline__ float xor16_max(float v) {
  const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(s[0]), __uint_as_float(s[1]));
}
__device__ __forceinline__ float xor32_max(float v) {
  const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(s[0]), __uint_as_float(s[1]));
}
// s[0] + s[1] is (lower row + upper row) on both lanes of the pair: all four lanes of a point end
// with the same bits
__device__ __forceinline__ float xor16_sum(float v) {
  const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(s[0]) + __uint_as_float(s[1]);
}
__device__ __forceinline__ float xor32_sum(float v) {
  const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(s[0]) + __uint_as_float(s[1]);
}

template <int JL>
__global__ __launch_bounds__(LBS_THREADS) __attribute__((amdgpu_waves_per_eu(MFMA_WAVES_PER_EU)))
void k_lbs_skin_mfma(const float* __restrict__ pcd, const float* __restrict__ W, int64_t N,
                     const float* __restrict__ theta_weight, float eps, const float* __restrict__ boneT12,
                     const float* __restrict__ global_t, float* __restrict__ xyz_out) {
  constexpr int J = 4 * JL, NC = (JL + 7) / 8;
  const int lane = threadIdx.x & 63, n16 = lane & 15, g = lane >> 4;
  // A fragments: lane (m, g) holds T[g*JL + 8c + i][m] (rows m >= 12 and joints past JL are 0)
  lbs_h8 ahi[NC], alo[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int jj = 8 * c + i;
      const float v = (jj < JL && n16 < 12) ? boneT12[(g * JL + jj) * 12 + n16] : 0.f;
      const _Float16 h = (_Float16)v;
      ahi[c][i] = h;
      alo[c][i] = (_Float16)(v - (float)h);
    }
  }
  const float th = fmaxf(eps, theta_weight[0]);
  const float rth = 1.f / th;
  const float gt = global_t[g < 3 ? g : 0];
  const int64_t groups = (N + 15) / 16;
  const int64_t step = (int64_t)gridDim.x * (LBS_THREADS / 64);
  int64_t gi = (int64_t)blockIdx.x * (LBS_THREADS / 64) + (threadIdx.x >> 6);
  auto fetch = [&](int64_t gg, float (&row)[JL], float (&pc)[3]) {
    const int64_t p = min(gg * 16 + n16, N - 1);
    quad_load_row<JL>(W + p * J + g * JL, row);
    pc[0] = pcd[3 * p]; pc[1] = pcd[3 * p + 1]; pc[2] = pcd[3 * p + 2];
  };
  auto skin = [&](int64_t gg, const float (&w)[JL], const float (&pc)[3]) {
    const int64_t p = gg * 16 + n16;
    float row[JL];
    // softmax(W / th) (temporalpoints.py:403): the quotient as in k_lbs_skin_quad
    float m = -INFINITY;
#pragma unroll
    for (int j = 0; j < JL; ++j) {
      const float q = w[j] * rth;
      row[j] = fmaf(fmaf(-q, th, w[j]), rth, q);
      m = fmaxf(m, row[j]);
    }
    m = xor32_max(xor16_max(m));
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < JL; ++j) {
      row[j] = __builtin_amdgcn_exp2f((row[j] - m) * 1.4426950408889634f);
      sum += row[j];
    }
    sum = xor32_sum(xor16_sum(sum));
    const float sc = (1.f / sum) * 0x1p-12f;
    lbs_f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      mlpx::h4 hq[2], lq[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int j0 = 8 * c + 4 * u;
        if (j0 < JL) {
          const mlpx::f32x4 v = {row[j0] * 4096.f, j0 + 1 < JL ? row[j0 + 1] * 4096.f : 0.f,
                                 j0 + 2 < JL ? row[j0 + 2] * 4096.f : 0.f, j0 + 3 < JL ? row[j0 + 3] * 4096.f : 0.f};
          mlpx::split4(v, hq[u], lq[u]);
        } else {
          hq[u] = lq[u] = mlpx::h4{0, 0, 0, 0};
        }
      }
      const lbs_h8 bhi = __builtin_shufflevector(hq[0], hq[1], 0, 1, 2, 3, 4, 5, 6, 7);
      const lbs_h8 blo = __builtin_shufflevector(lq[0], lq[1], 0, 1, 2, 3, 4, 5, 6, 7);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi[c], bhi, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi[c], blo, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(alo[c], bhi, acc, 0, 0, 0);
    }
    // lane (n, g): row g of point n's G (pointwarper.py:241-266), then x'[g] = G_g [x; 1] + t[g]
    const float x = ((acc[0] * sc * pc[0] + acc[1] * sc * pc[1]) + acc[2] * sc * pc[2]) + acc[3] * sc;
    if (g < 3 && p < N) xyz_out[3 * p + g] = x + gt;
  };
  // LBS_MFMA_PF + 1 register buffers, the loop unrolled over them: buffer b is refilled with the
  // group LBS_MFMA_PF + 1 steps ahead right after it is skinned (no register rotation)
  constexpr int NB = LBS_MFMA_PF + 1;
  float buf[NB][JL], pcb[NB][3];
#pragma unroll
  for (int b = 0; b < NB; ++b) fetch(gi + b * step, buf[b], pcb[b]);
  for (;;) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      if (gi >= groups) return;   // wave-uniform
      skin(gi, buf[b], pcb[b]);
      fetch(gi + NB * step, buf[b], pcb[b]);
      gi += step;
    }
  }
}

extern "C" int apn_lbs_skin(const float* canonical_pcd, const float* raw_weights, int64_t n_points, int32_t n_joints,
                            const float* theta_weight, float eps, const int32_t* merge_rules, const float* bone_T34,
                            const float* global_t, const float* joint_colors, const float* canonical_alpha,
                            const float* canonical_rgbs, const float* direct_eps, float mean_min_distance,
                            int32_t weights_final, float* xyz_out, float* weights_out, float* G_out, float* recA16,
                            float* recB8, int32_t* bbox_ord, void* workspace, void* stream) {
  if (n_points <= 0 || n_joints <= 0 || n_joints > LBS_MAX_J) return APN_ERR_ARG;
  if (!canonical_pcd || !raw_weights || (!weights_final && !theta_weight) || !bone_T34 || !global_t || !xyz_out)
    return APN_ERR_ARG;
  if (bbox_ord && !workspace) return APN_ERR_ARG;
  if ((recA16 != nullptr) != (recB8 != nullptr)) return APN_ERR_ARG;
  if (recA16 && (!canonical_alpha || !canonical_rgbs || !direct_eps)) return APN_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int J = n_joints;
  const int nblocks = ceil_div(n_points, LBS_THREADS);
  int* part = bbox_ord ? (int*)workspace : nullptr;
  // quad kernel for the record-free calls (repose, LBS-only sweeps) with identity merge rules and
  // J % 4 == 0 (APN_LBS_LDS selects the LDS-tile kernel). The render path keeps k_lbs_skin: its
  // sequential sums reproduce the oracle's skinned cloud bit for bit, and the sampling bbox --
  // hence every sample position -- follows that cloud (bbox sensitivity).
  static const bool quad_ok = apn_env("APN_LBS_LDS") == nullptr;
  static const bool mfma_ok = apn_env("APN_LBS_QUAD") == nullptr;   // debug A/B: the VALU quad blend
  if (mfma_ok && quad_ok && !recA16 && !merge_rules && !weights_final && !weights_out && !G_out && !joint_colors &&
      !bbox_ord && J % 4 == 0 && J <= 64 && ((uintptr_t)raw_weights % 16) == 0) {
    static const int per_cu = [] {
      const char* e = apn_env("APN_LBS_BLOCKS_PER_CU");
      return e ? atoi(e) : 8;
    }();
    const int mblocks = (int)std::min<int64_t>(ceil_div(ceil_div(n_points, 16), LBS_THREADS / 64), 256 * per_cu);
    auto mf = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(mblocks), dim3(LBS_THREADS), 0, s, canonical_pcd, raw_weights, n_points,
                         theta_weight, eps, bone_T34, global_t, xyz_out);
    };
    switch (J / 4) {
      case 1: mf(k_lbs_skin_mfma<1>); break;
      case 2: mf(k_lbs_skin_mfma<2>); break;
      case 3: mf(k_lbs_skin_mfma<3>); break;
      case 4: mf(k_lbs_skin_mfma<4>); break;
      case 5: mf(k_lbs_skin_mfma<5>); break;
      case 6: mf(k_lbs_skin_mfma<6>); break;
      case 7: mf(k_lbs_skin_mfma<7>); break;
      case 8: mf(k_lbs_skin_mfma<8>); break;
      case 9: mf(k_lbs_skin_mfma<9>); break;
      case 10: mf(k_lbs_skin_mfma<10>); break;
      case 11: mf(k_lbs_skin_mfma<11>); break;
      case 12: mf(k_lbs_skin_mfma<12>); break;
      case 13: mf(k_lbs_skin_mfma<13>); break;
      case 14: mf(k_lbs_skin_mfma<14>); break;
      case 15: mf(k_lbs_skin_mfma<15>); break;
      default: mf(k_lbs_skin_mfma<16>); break;
    }
    return launch_status();
  }
  if (quad_ok && !recA16 && !merge_rules && J % 4 == 0 && ((uintptr_t)raw_weights % 16) == 0) {
    // grid-stride blocks (one row ahead); <= 1 partial per block. 32 blocks per CU: the launch
    // then carries more rows in flight per CU than the 4-per-CU persistent grid (C5, 1M points,
    // J = 48: 0.0511 -> 0.0429 ms; 6: 0.048, 12: 0.044, 64: 0.044 -- tools/c5_lbs_ab.sh); a
    // second row in flight per lane (LBS_PF = 2, 3) measured slower
    static const int per_cu = [] {
      const char* e = apn_env("APN_LBS_BLOCKS_PER_CU");
      return e ? atoi(e) : 32;
    }();
    const int qblocks = (int)std::min<int64_t>(ceil_div(n_points, LBS_THREADS / 4), 256 * per_cu);
    auto quad = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(qblocks), dim3(LBS_THREADS), 0, s, canonical_pcd, raw_weights, n_points,
                         theta_weight, eps, bone_T34, global_t, joint_colors, canonical_alpha, canonical_rgbs,
                         direct_eps, mean_min_distance, weights_final, xyz_out, weights_out, G_out, (float4*)recA16,
                         (float4*)recB8, part);
    };
    switch (J / 4) {
      case 1: quad(k_lbs_skin_quad<1>); break;
      case 2: quad(k_lbs_skin_quad<2>); break;
      case 3: quad(k_lbs_skin_quad<3>); break;
      case 4: quad(k_lbs_skin_quad<4>); break;
      case 5: quad(k_lbs_skin_quad<5>); break;
      case 6: quad(k_lbs_skin_quad<6>); break;
      case 7: quad(k_lbs_skin_quad<7>); break;
      case 8: quad(k_lbs_skin_quad<8>); break;
      case 9: quad(k_lbs_skin_quad<9>); break;
      case 10: quad(k_lbs_skin_quad<10>); break;
      case 11: quad(k_lbs_skin_quad<11>); break;
      case 12: quad(k_lbs_skin_quad<12>); break;
      case 13: quad(k_lbs_skin_quad<13>); break;
      case 14: quad(k_lbs_skin_quad<14>); break;
      case 15: quad(k_lbs_skin_quad<15>); break;
      default: quad(k_lbs_skin_quad<16>); break;
    }
    if (bbox_ord) hipLaunchKernelGGL(k_bbox_reduce, dim3(1), dim3(256), 0, s, part, qblocks, bbox_ord);
    return launch_status();
  }
  size_t lds = (size_t)(LBS_THREADS * (J + 1) + J * 12 + J * 3) * sizeof(float) + J * sizeof(int);
  hipLaunchKernelGGL(k_lbs_skin, dim3(nblocks), dim3(LBS_THREADS), lds, s, canonical_pcd, raw_weights, n_points, J,
                     theta_weight, eps, merge_rules, bone_T34, global_t, joint_colors, canonical_alpha, canonical_rgbs,
                     direct_eps, mean_min_distance, weights_final, xyz_out, weights_out, G_out, (float4*)recA16,
                     (float4*)recB8, part);
  if (bbox_ord) hipLaunchKernelGGL(k_bbox_reduce, dim3(1), dim3(256), 0, s, part, nblocks, bbox_ord);
  return launch_status();
}
