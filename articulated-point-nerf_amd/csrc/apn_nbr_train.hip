// The training forward's neighbour aggregation around feat_net, forward and backward as HIP
// kernels (the autograd restatement is train.py's NbrAggregate / IdwSum):
//
//   rel_p  = x_s - p_n,  to_nn = |rel_p|^2                       temporalpoints.py:454-457
//   direct: e = exp(-to_nn^2 / (2 sig_n^2 + 1e-12)), rgb_d = sum_k e_k / (sum e + 1e-12) c_n,
//           alpha_d = sum_k e_k / 8 a_n                             temporalpoints.py:459-470
//   IDW:    w = (1 / (to_nn + eps)) / sum_k (...)                   temporalpoints.py:473-475
//   rel_c  = Rinv_n rel_p, posenc [rel_c | sin(rel_c f) | cos(rel_c f)] (dim-major)  478-488
//   feat_in row = [posenc | canonical_feat_n | pose embedding]      488-491
//   h = sum_k w_k feat_net(feat_in)_k                               493-494
//
// feat_in row layout: [posenc (PE = 3 + 6L) | 0 pad to PE4 = 4 ceil(PE / 4) | canonical_feat (F) |
// pose embedding (P)], so the feature columns start 16-B aligned (the caller's weight map puts W1's
// columns at those positions and a zero column on the pad, train.py). The sin/cos come from
// sincos_pe (the render MLP's, ~1e-7 absolute).
// One MLP row (sample s, neighbour k) per thread, the 8 rows of a sample in 8 adjacent lanes
// (width-8 shuffles for the sums over k); 128-row blocks stage the posenc columns through LDS so
// that feat_in / d_feat are written and read row-contiguously (the backward recomputes the same
// sin / cos). The backward writes each row's gradient terms for its neighbour point (position 3, Rinv 9, sigma 1, colour 3, alpha 1) and the per-point sums are
// gathered over the reverse adjacency of s_i in a fixed order (rev_ptr / rev_edge, train.py
// reverse_csr) -- no atomics, deterministic.
#include "apn_common.h"
#include "apn_mlp_split.h"   // sincos_pe: the render MLP's posenc sin/cos

#include <algorithm>

namespace apn {
namespace nbrt {

constexpr int NCONTRIB = 17;   // d_p (3), d_Rinv (9), d_sig (1), d_c (3), d_a (1)

__device__ __forceinline__ float sum8(float v) {
  v += __shfl_xor(v, 1, 8);
  v += __shfl_xor(v, 2, 8);
  v += __shfl_xor(v, 4, 8);
  return v;
}

struct Geo {
  float rp[3], t, e, D, w0;
};

__device__ __forceinline__ Geo geometry(const float* __restrict__ ray_pts, const float* __restrict__ xyz,
                                        const float* __restrict__ sig, int64_t s, int64_t n, float eps) {
  Geo g;
  g.rp[0] = ray_pts[3 * s] - xyz[3 * n];
  g.rp[1] = ray_pts[3 * s + 1] - xyz[3 * n + 1];
  g.rp[2] = ray_pts[3 * s + 2] - xyz[3 * n + 2];
  g.t = (g.rp[0] * g.rp[0] + g.rp[1] * g.rp[1]) + g.rp[2] * g.rp[2];
  const float sg = sig[n];
  g.D = 2.f * (sg * sg) + 1e-12f;
  g.e = expf(-(g.t * g.t) / g.D);
  g.w0 = 1.f / (g.t + eps);
  return g;
}

constexpr int RB = 128;      // rows per block of the posenc kernels

__global__ __launch_bounds__(RB) void k_nbr_train_fwd(int64_t S, const float* __restrict__ ray_pts,
                                                      const int64_t* __restrict__ s_i, const float* __restrict__ xyz,
                                                      const float* __restrict__ Rinv, const float* __restrict__ sig,
                                                      const float* __restrict__ rgb_c, const float* __restrict__ alpha_c,
                                                      const float* __restrict__ poc, int L, float eps,
                                                      float* __restrict__ w_out, float* __restrict__ rgbd,
                                                      float* __restrict__ alphad, float* __restrict__ feat_in,
                                                      int64_t ldf) {
  extern __shared__ float sPE[];   // [RB][LD]
  const int PE = 3 + 6 * L, PE4 = (PE + 3) & ~3, LD = PE | 1;   // odd LDS row stride: own-row writes spread over banks
  const int64_t row0 = (int64_t)blockIdx.x * RB;
  const int64_t row = row0 + threadIdx.x;
  const int64_t s = row >> 3;
  const int k = (int)(row & 7);
  const bool valid = s < S;   // a sample's 8 lanes are valid together (S * 8 rows)
  const int64_t n = valid ? s_i[row] : 0;
  const Geo g = geometry(ray_pts, xyz, sig, valid ? s : 0, n, eps);
  const float E = sum8(valid ? g.e : 0.f), W0 = sum8(valid ? g.w0 : 0.f);
  const float wd = g.e / (E + 1e-12f);
  float c0 = sum8(wd * rgb_c[3 * n]), c1 = sum8(wd * rgb_c[3 * n + 1]), c2 = sum8(wd * rgb_c[3 * n + 2]);
  const float ad = sum8((0.125f * g.e) * alpha_c[n]);
  if (valid) {
    w_out[row] = g.w0 / W0;
    if (k == 0) {
      rgbd[3 * s] = c0; rgbd[3 * s + 1] = c1; rgbd[3 * s + 2] = c2;
      alphad[s] = ad;
    }
  }
  const float* R = Rinv + 9 * n;
  float rc[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) rc[i] = (R[3 * i] * g.rp[0] + R[3 * i + 1] * g.rp[1]) + R[3 * i + 2] * g.rp[2];
  float* f = sPE + threadIdx.x * LD;
#pragma unroll
  for (int d = 0; d < 3; ++d) f[d] = rc[d];
  for (int d = 0; d < 3; ++d)
    for (int l = 0; l < L; ++l) {
      float sn, cs;
      mlpx::sincos_pe(rc[d] * poc[l], sn, cs);
      f[3 + d * L + l] = sn;
      f[3 + 3 * L + d * L + l] = cs;
    }
  __syncthreads();
  const int64_t nrows = min((int64_t)RB, S * 8 - row0);
  for (int i = threadIdx.x; i < nrows * PE4; i += RB) {
    const int r = i / PE4, c = i - r * PE4;
    feat_in[(row0 + r) * ldf + c] = c < PE ? sPE[r * LD + c] : 0.f;
  }
}

// feat_in[row, col0 + c] = src[idx[row], c] (idx = s_i, or none: row 0 of src for every row -- the
// pose embedding): one thread per 16-B chunk when F, col0 and ldd are multiples of 4, else per float.
__global__ __launch_bounds__(256) void k_gather_rows(int64_t rows, const int64_t* __restrict__ idx,
                                                     const float* __restrict__ src, int F, float* __restrict__ dst,
                                                     int64_t ldd, int col0, int vec) {
  const int W = vec ? F / 4 : F;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < rows * W; t += (int64_t)gridDim.x * 256) {
    const int64_t r = t / W;
    const int c = (int)(t - r * W);
    const float* a = src + (idx ? idx[r] : 0) * (int64_t)F;
    float* b = dst + r * ldd + col0;
    if (vec)
      *(float4*)(b + 4 * c) = *(const float4*)(a + 4 * c);
    else
      b[c] = a[c];
  }
}

__global__ __launch_bounds__(RB) void k_nbr_train_bwd(int64_t S, const float* __restrict__ ray_pts,
                                                      const int64_t* __restrict__ s_i, const float* __restrict__ xyz,
                                                      const float* __restrict__ Rinv, const float* __restrict__ sig,
                                                      const float* __restrict__ rgb_c, const float* __restrict__ alpha_c,
                                                      const float* __restrict__ poc, int L, float eps,
                                                      const float* __restrict__ d_w, const float* __restrict__ d_rgbd,
                                                      const float* __restrict__ d_alphad,
                                                      const float* __restrict__ d_feat, int64_t ldd,
                                                      float* __restrict__ contrib) {
  extern __shared__ float sD[];   // [RB][LD]
  const int PE = 3 + 6 * L, LD = PE | 1;
  const int64_t row0 = (int64_t)blockIdx.x * RB;
  const int64_t nrows = min((int64_t)RB, S * 8 - row0);
  if (d_feat) {   // the block's posenc gradient and values, read row-contiguously
    for (int i = threadIdx.x; i < nrows * PE; i += RB) {
      const int r = i / PE, c = i - r * PE;
      sD[r * LD + c] = d_feat[(row0 + r) * ldd + c];
    }
    __syncthreads();
  }
  const int64_t row = row0 + threadIdx.x;
  const int64_t s = row >> 3;
  const bool valid = s < S;
  const int64_t n = valid ? s_i[row] : 0;
  const int64_t ss = valid ? s : 0;
  const Geo g = geometry(ray_pts, xyz, sig, ss, n, eps);
  const float E = sum8(valid ? g.e : 0.f), W0 = sum8(valid ? g.w0 : 0.f);
  const float Ee = E + 1e-12f;
  const float wd = g.e / Ee;
  const float c[3] = {rgb_c[3 * n], rgb_c[3 * n + 1], rgb_c[3 * n + 2]};
  const float a = alpha_c[n];
  // direct blend: rgb_d = sum wd_k c_k, alpha_d = sum e_k / 8 a_k
  const float g0 = d_rgbd ? d_rgbd[3 * ss] : 0.f, g1 = d_rgbd ? d_rgbd[3 * ss + 1] : 0.f,
              g2 = d_rgbd ? d_rgbd[3 * ss + 2] : 0.f;
  const float ga = d_alphad ? d_alphad[ss] : 0.f;
  const float dwd = (g0 * c[0] + g1 * c[1]) + g2 * c[2];
  const float sum_dwd_wd = sum8(valid ? dwd * wd : 0.f);
  const float de = (dwd - sum_dwd_wd) / Ee + ga * 0.125f * a;
  // e = exp(-t^2 / D): d t, d D (-> d sig = dD * 4 sig)
  const float dt_direct = de * g.e * (-2.f * g.t / g.D);
  const float dD = de * g.e * (g.t * g.t) / (g.D * g.D);
  // IDW: w = w0 / W0, w0 = 1 / (t + eps)
  const float w = g.w0 / W0;
  const float dwv = d_w ? d_w[valid ? row : 0] : 0.f;
  const float sum_dw_w = sum8(valid ? dwv * w : 0.f);
  const float dw0 = (dwv - sum_dw_w) / W0;
  const float dt = dt_direct - dw0 * g.w0 * g.w0;
  // posenc -> rel_c: d/dx [x, sin(x f), cos(x f)] = [1, f cos, -f sin] (the forward's sincos_pe)
  const float* R = Rinv + 9 * n;
  float rc[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) rc[i] = (R[3 * i] * g.rp[0] + R[3 * i + 1] * g.rp[1]) + R[3 * i + 2] * g.rp[2];
  float drc[3] = {0.f, 0.f, 0.f};
  if (d_feat && valid) {
    const float* df = sD + threadIdx.x * LD;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      float acc = df[d];
      for (int l = 0; l < L; ++l) {
        float sn, cs;
        mlpx::sincos_pe(rc[d] * poc[l], sn, cs);
        acc += poc[l] * (cs * df[3 + d * L + l] - sn * df[3 + 3 * L + d * L + l]);
      }
      drc[d] = acc;
    }
  }
  // rel_c = R rel_p: dR[i][j] = drc[i] rel_p[j]; d rel_p = R^T drc + 2 rel_p dt
  float drp[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) drp[j] = (R[j] * drc[0] + R[3 + j] * drc[1]) + R[6 + j] * drc[2] + 2.f * g.rp[j] * dt;
  if (!valid) return;
  float* o = contrib + row * NCONTRIB;
#pragma unroll
  for (int j = 0; j < 3; ++j) o[j] = -drp[j];   // rel_p = x - p
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) o[3 + 3 * i + j] = drc[i] * g.rp[j];
  o[12] = dD * 4.f * sig[n];
  o[13] = wd * g0; o[14] = wd * g1; o[15] = wd * g2;
  o[16] = ga * 0.125f * g.e;
}

// Per point n: the sums of its rows' terms over rev_edge[rev_ptr[n] .. rev_ptr[n+1]) in order.
__global__ __launch_bounds__(256) void k_nbr_train_gather(int64_t N, const int64_t* __restrict__ rev_ptr,
                                                          const int64_t* __restrict__ rev_edge,
                                                          const float* __restrict__ contrib, float* __restrict__ d_xyz,
                                                          float* __restrict__ d_R, float* __restrict__ d_sig,
                                                          float* __restrict__ d_c, float* __restrict__ d_a) {
  const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  float acc[NCONTRIB];
#pragma unroll
  for (int c = 0; c < NCONTRIB; ++c) acc[c] = 0.f;
  for (int64_t e = rev_ptr[n]; e < rev_ptr[n + 1]; ++e) {
    const float* o = contrib + rev_edge[e] * NCONTRIB;
#pragma unroll
    for (int c = 0; c < NCONTRIB; ++c) acc[c] += o[c];
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) d_xyz[3 * n + j] = acc[j];
#pragma unroll
  for (int j = 0; j < 9; ++j) d_R[9 * n + j] = acc[3 + j];
  d_sig[n] = acc[12];
#pragma unroll
  for (int j = 0; j < 3; ++j) d_c[3 * n + j] = acc[13 + j];
  d_a[n] = acc[16];
}

// d_feat_pt[n, c] = sum over n's rows of d_feat[row, col0 + c]: one thread per 16-B chunk of a
// point's F columns when vec (F, col0, ldd multiples of 4), else per float.
__global__ __launch_bounds__(256) void k_feat_gather(int64_t N, const int64_t* __restrict__ rev_ptr,
                                                     const int64_t* __restrict__ rev_edge, const float* __restrict__ d_feat,
                                                     int64_t ldd, int col0, int F, int vec, float* __restrict__ out) {
  const int W = vec ? F / 4 : F;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < N * W; t += (int64_t)gridDim.x * 256) {
    const int64_t n = t / W;
    const int c = (int)(t - n * W);
    const int64_t e0 = rev_ptr[n], e1 = rev_ptr[n + 1];
    if (vec) {
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int64_t e = e0; e < e1; ++e) {
        const float4 v = *(const float4*)(d_feat + rev_edge[e] * ldd + col0 + 4 * c);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
      *(float4*)(out + n * (int64_t)F + 4 * c) = acc;
    } else {
      float acc = 0.f;
      for (int64_t e = e0; e < e1; ++e) acc += d_feat[rev_edge[e] * ldd + col0 + c];
      out[n * (int64_t)F + c] = acc;
    }
  }
}

// Cloud bounding box: per-block min / max of xyz [N,3] (exact), then one block over the partials;
// out6 = {min x, y, z, max x, y, z}, ord8 = the order-preserving int32 encoding of out6 (the grid
// kernels' bbox_ord, apn_common.h float_to_ordered) or NULL.
__global__ __launch_bounds__(256) void k_bbox_part(int64_t N, const float* __restrict__ xyz, float* __restrict__ part) {
  float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < N; i += (int64_t)gridDim.x * 256)
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const float v = xyz[3 * i + a];
      lo[a] = fminf(lo[a], v);
      hi[a] = fmaxf(hi[a], v);
    }
  __shared__ float sl[3][256], sh[3][256];
#pragma unroll
  for (int a = 0; a < 3; ++a) { sl[a][threadIdx.x] = lo[a]; sh[a][threadIdx.x] = hi[a]; }
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o)
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        sl[a][threadIdx.x] = fminf(sl[a][threadIdx.x], sl[a][threadIdx.x + o]);
        sh[a][threadIdx.x] = fmaxf(sh[a][threadIdx.x], sh[a][threadIdx.x + o]);
      }
    __syncthreads();
  }
  if (threadIdx.x < 3) {
    part[6 * blockIdx.x + threadIdx.x] = sl[threadIdx.x][0];
    part[6 * blockIdx.x + 3 + threadIdx.x] = sh[threadIdx.x][0];
  }
}

__global__ __launch_bounds__(256) void k_bbox_final(int nb, const float* __restrict__ part, float* __restrict__ out6,
                                                    int* __restrict__ ord8) {
  __shared__ float sp[6][256];
  float v[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) v[j] = j < 3 ? INFINITY : -INFINITY;
  for (int b = threadIdx.x; b < nb; b += 256)
#pragma unroll
    for (int j = 0; j < 6; ++j) v[j] = j < 3 ? fminf(v[j], part[6 * b + j]) : fmaxf(v[j], part[6 * b + j]);
#pragma unroll
  for (int j = 0; j < 6; ++j) sp[j][threadIdx.x] = v[j];
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o)
#pragma unroll
      for (int j = 0; j < 6; ++j)
        sp[j][threadIdx.x] = j < 3 ? fminf(sp[j][threadIdx.x], sp[j][threadIdx.x + o])
                                   : fmaxf(sp[j][threadIdx.x], sp[j][threadIdx.x + o]);
    __syncthreads();
  }
  if (threadIdx.x < 6) {
    const int j = threadIdx.x;
    const float r = sp[j][0];
    out6[j] = r;
    if (ord8) {
      const int i = __float_as_int(r);
      ord8[j] = i >= 0 ? i : (i ^ 0x7fffffff);
      if (j < 2) ord8[6 + j] = 0;
    }
  }
}

// h[s, c] = sum_k w[s, k] out[8 s + k, c] (k ascending); 64 lanes per sample.
__global__ __launch_bounds__(256) void k_idw_sum_fwd(int64_t S, int C, const float* __restrict__ w,
                                                     const float* __restrict__ out, float* __restrict__ h) {
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= S) return;
  float wk[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) wk[k] = w[8 * s + k];
  for (int c = threadIdx.x & 63; c < C; c += 64) {
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += wk[k] * out[(8 * s + k) * (int64_t)C + c];
    h[s * C + c] = acc;
  }
}

// d_out[8 s + k, c] = w[s, k] d_h[s, c];  d_w[s, k] = sum_c out[8 s + k, c] d_h[s, c]. One wave per
// sample, the C columns over the lanes, the row sums by a wave reduction.
__global__ __launch_bounds__(256) void k_idw_sum_bwd(int64_t S, int C, const float* __restrict__ w,
                                                     const float* __restrict__ out, const float* __restrict__ dh,
                                                     float* __restrict__ d_out, float* __restrict__ d_w) {
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= S) return;
  const int lane = threadIdx.x & 63;
  for (int k = 0; k < 8; ++k) {
    const float wk = w[8 * s + k];
    float acc = 0.f;
    for (int c = lane; c < C; c += 64) {
      const float g = dh[s * C + c];
      const int64_t o = (8 * s + k) * (int64_t)C + c;
      if (d_out) d_out[o] = wk * g;
      acc += out[o] * g;
    }
    if (d_w) {
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
      if (lane == 0) d_w[8 * s + k] = acc;
    }
  }
}

}  // namespace nbrt
}  // namespace apn

using namespace apn;

extern "C" int apn_nbr_train_fwd(int64_t S, const float* ray_pts, const int64_t* s_i, const float* xyz,
                                 const float* Rinv, const float* canonical_feat, int32_t F, const float* pose_emb,
                                 int32_t P, const float* sig, const float* rgb_c, const float* alpha_c,
                                 const float* poc, int32_t L, float eps, float* w_out, float* rgbd, float* alphad,
                                 float* feat_in, int64_t ldf, void* stream) {
  if (S < 0 || L < 0 || L > 16 || F < 0 || P < 0 || ldf < ((3 + 6 * (int64_t)L + 3) & ~3) + F + P) return APN_ERR_ARG;
  if (S == 0) return APN_OK;
  hipStream_t st = (hipStream_t)stream;
  const int64_t rows = S * 8;
  const size_t lds = (size_t)nbrt::RB * ((3 + 6 * L) | 1) * sizeof(float);
  hipLaunchKernelGGL(nbrt::k_nbr_train_fwd, dim3((unsigned)ceil_div(rows, nbrt::RB)), dim3(nbrt::RB), lds, st, S,
                     ray_pts, s_i, xyz, Rinv, sig, rgb_c, alpha_c, poc, L, eps, w_out, rgbd, alphad, feat_in, ldf);
  const int pe4 = (3 + 6 * L + 3) & ~3;
  const bool al = ldf % 4 == 0 && ((uintptr_t)feat_in % 16) == 0;
  auto gather = [&](const int64_t* idx, const float* src, int W, int col0) {
    const int vec = al && W % 4 == 0 && col0 % 4 == 0 && ((uintptr_t)src % 16) == 0;
    const int64_t work = rows * (vec ? W / 4 : W);
    hipLaunchKernelGGL(nbrt::k_gather_rows, dim3((unsigned)std::min<int64_t>(ceil_div(work, 256), 65536)), dim3(256), 0,
                       st, rows, idx, src, W, feat_in, ldf, col0, vec);
  };
  if (F > 0) gather(s_i, canonical_feat, F, pe4);
  if (P > 0) gather(nullptr, pose_emb, P, pe4 + F);
  return launch_status();
}

extern "C" int apn_nbr_train_bwd(int64_t S, int64_t N, const float* ray_pts, const int64_t* s_i, const float* xyz,
                                 const float* Rinv, const float* sig, const float* rgb_c, const float* alpha_c,
                                 const float* poc, int32_t L, float eps, const float* d_w, const float* d_rgbd,
                                 const float* d_alphad, const float* d_feat, int64_t ldd, int32_t F,
                                 const int64_t* rev_ptr, const int64_t* rev_edge, float* contrib, float* d_xyz,
                                 float* d_R, float* d_sig, float* d_c, float* d_a, float* d_featp, void* stream) {
  if (S < 0 || N < 0 || L < 0 || L > 16 || !contrib) return APN_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  const int64_t rows = S * 8;
  if (rows > 0)
    hipLaunchKernelGGL(nbrt::k_nbr_train_bwd, dim3((unsigned)ceil_div(rows, nbrt::RB)), dim3(nbrt::RB),
                       (size_t)nbrt::RB * ((3 + 6 * L) | 1) * sizeof(float), st, S, ray_pts, s_i, xyz, Rinv, sig, rgb_c,
                       alpha_c, poc, L, eps, d_w, d_rgbd, d_alphad, d_feat, ldd, contrib);
  if (N > 0) {
    hipLaunchKernelGGL(nbrt::k_nbr_train_gather, dim3((unsigned)ceil_div(N, 256)), dim3(256), 0, st, N, rev_ptr,
                       rev_edge, contrib, d_xyz, d_R, d_sig, d_c, d_a);
    if (d_featp && d_feat && F > 0) {
      const int col0 = (3 + 6 * L + 3) & ~3;
      const int vec = F % 4 == 0 && ldd % 4 == 0 && ((uintptr_t)d_feat % 16) == 0 && ((uintptr_t)d_featp % 16) == 0;
      const int64_t work = N * (vec ? F / 4 : F);
      hipLaunchKernelGGL(nbrt::k_feat_gather, dim3((unsigned)std::min<int64_t>(ceil_div(work, 256), 65536)), dim3(256), 0,
                         st, N, rev_ptr, rev_edge, d_feat, ldd, col0, F, vec, d_featp);
    }
  }
  return launch_status();
}

extern "C" int apn_idw_sum_fwd(int64_t S, int32_t C, const float* w, const float* out, float* h, void* stream) {
  if (S < 0 || C <= 0) return APN_ERR_ARG;
  if (S == 0) return APN_OK;
  hipLaunchKernelGGL(nbrt::k_idw_sum_fwd, dim3((unsigned)ceil_div(S, 4)), dim3(256), 0, (hipStream_t)stream, S, C, w,
                     out, h);
  return launch_status();
}

extern "C" int apn_idw_sum_bwd(int64_t S, int32_t C, const float* w, const float* out, const float* dh, float* d_out,
                               float* d_w, void* stream) {
  if (S < 0 || C <= 0) return APN_ERR_ARG;
  if (S == 0) return APN_OK;
  hipLaunchKernelGGL(nbrt::k_idw_sum_bwd, dim3((unsigned)ceil_div(S, 4)), dim3(256), 0, (hipStream_t)stream, S, C, w,
                     out, dh, d_out, d_w);
  return launch_status();
}

extern "C" int apn_cloud_bbox(const float* xyz, int64_t N, float* out6, int32_t* ord8, void* workspace, void* stream) {
  if (N <= 0 || !xyz || !out6 || !workspace) return APN_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  const int nb = (int)std::min<int64_t>(ceil_div(N, 256), 1024);
  hipLaunchKernelGGL(nbrt::k_bbox_part, dim3(nb), dim3(256), 0, st, N, xyz, (float*)workspace);
  hipLaunchKernelGGL(nbrt::k_bbox_final, dim3(1), dim3(256), 0, st, nb, (const float*)workspace, out6, ord8);
  return launch_status();
}
