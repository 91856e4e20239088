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
//   recB[n] = {clip(rgb,0,1), 0, pcol, 0}                                     (32 B)
// HBM-bound: per point it reads 12 + 4J + 4 + 12 + 4 bytes and writes 12 + 4J + 96 bytes.
#include "apn_common.h"

namespace apn {

constexpr int LBS_THREADS = 256;
constexpr int LBS_MAX_J = 64;

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
    if (G_out) {  // weighted_G_tw (pointwarper.py:243): rows 0..2 blended, row 3 = sum_j w_j [0,0,0,1]
      float sw = 0.f;
      for (int j = 0; j < J; ++j) sw = sw + row[j];
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
    recB[2 * n + 0] = make_float4(r, g, b, 0.f);
    recB[2 * n + 1] = make_float4((float)pc0, (float)pc1, (float)pc2, 0.f);
    }  // recA
  }
  __syncthreads();
  if (w_out) {
    float* Wo = w_out + n0 * J;
    for (int e = tid; e < tile_elems; e += LBS_THREADS) {
      const int r = e / J, c = e - r * J;
      Wo[e] = sW[r * Jp + c];
    }
  }
  // bbox: wave reduce, then across the block's waves; one partial per block, reduced by
  // k_bbox_reduce (all blocks hitting 6 global atomics serialised at one L2 channel and cost
  // ~0.3 ms at 300k points)
  if (bbox_part) {
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
  return n_points > 0 ? (size_t)ceil_div(n_points, LBS_THREADS) * 6 * sizeof(int) : 0;
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
  size_t lds = (size_t)(LBS_THREADS * (J + 1) + J * 12 + J * 3) * sizeof(float) + J * sizeof(int);
  hipLaunchKernelGGL(k_lbs_skin, dim3(nblocks), dim3(LBS_THREADS), lds, s, canonical_pcd, raw_weights, n_points, J,
                     theta_weight, eps, merge_rules, bone_T34, global_t, joint_colors, canonical_alpha, canonical_rgbs,
                     direct_eps, mean_min_distance, weights_final, xyz_out, weights_out, G_out, (float4*)recA16,
                     (float4*)recB8, part);
  if (bbox_ord) hipLaunchKernelGGL(k_bbox_reduce, dim3(1), dim3(256), 0, s, part, nblocks, bbox_ord);
  return launch_status();
}
