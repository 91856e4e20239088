// Fused Point-NeRF neighbour MLP for the kept samples (temporalpoints.py:452-519):
//
//   per (sample s, neighbour k):  rel_p = x_s - p_k ; to_nn = |rel_p|^2
//                                 rel_c = Rinv_k rel_p ; row = [poc_fre(rel_c,10) (63), feat_k (128)]
//   feat_net (4 x Linear+LeakyReLU, 191->128->128->128->128)  on FP32 MFMA (v_mfma_f32_16x16x4_f32)
//   h_s = sum_k w_k out_k, w = IDW normalised (473-475, 493-494)
//   density = densitynet(h) -> raw2alpha (496-499, render_utils_kernel.cu:357-369)
//   rgb = sigmoid(rgbnet(h, poc_fre(viewdir,4)))   (503-515, tineuvox.py:65-88)
//   direct blend alpha_d / rgb_d (459-470), weight-vis colour sum_k w_k pcol_k (517-519, 697-699)
//
// Algebraic reassociations (exact in real arithmetic, ~1e-7 relative in fp32):
//   * layer 1: W1 [emb; feat_k] + b1 = W1e emb + (P[k] + b1), with the per-point projection
//     P = canonical_feat W1f^T computed once per model by k_feat_project (apn_feat_project);
//   * rgbnet: views_linears.0([feature_linears(h); v]) has no activation in between, so it is
//     one layer [Wv0a Wf | Wv0b] [h; v] + (Wv0a bf + bv0) (folded on the host in float64).
// Roofline accounting keeps the reference's F_alg.
//
// Tile = 8 samples x 8 neighbours = 64 MLP rows per 256-thread workgroup. The activation tile
// lives in LDS (64 x 200 fp32, row stride == 8 mod 64 floats: conflict-free ds_read_b128 for
// the 16x16x4 A-operand pattern), so 3 workgroups fit per CU. Each wave owns 32 output columns
// (2 N-tiles x 4 M-tiles of 16x16); B-operand fragments stream from L2-resident weights.
// k-permutation: for a 16-wide k chunk q, lane group g = lane>>4 holds k = 16q + 4g + t in
// element t of its float4, for both A (activations) and B (nn.Linear weight rows), so one
// 16-byte load feeds 4 MFMAs.
#include "apn_common.h"

namespace apn {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int TS = 8;             // samples per tile
constexpr int TR = TS * 8;        // MLP rows per tile
constexpr int XS = 200;           // LDS row stride (floats)
constexpr int MLP_THREADS = 256;
constexpr int FEAT = 128;
constexpr int KE = 64;            // positional encoding 63, zero-padded
constexpr int PCOL = 64;          // LDS column where the gathered P row starts
constexpr int KV = 160;           // head input: h (128) + view embedding (27) + pad

// Packed weight buffer layout (floats); apn_amd/ops.py:pack_mlp_weights reads it through
// apn_mlp_weight_layout().
constexpr int OFF_W1E = 0;                        // [128][64]  feat_net.0 columns 0..62
constexpr int OFF_B1 = OFF_W1E + 128 * KE;        // [128]      (+ pose-embedding fold)
constexpr int OFF_W2 = OFF_B1 + 128;              // [128][128]
constexpr int OFF_B2 = OFF_W2 + 128 * 128;
constexpr int OFF_W3 = OFF_B2 + 128;
constexpr int OFF_B3 = OFF_W3 + 128 * 128;
constexpr int OFF_W4 = OFF_B3 + 128;
constexpr int OFF_B4 = OFF_W4 + 128 * 128;
constexpr int OFF_WD = OFF_B4 + 128;              // [128]      densitynet
constexpr int OFF_BD = OFF_WD + 128;              // [4]
constexpr int OFF_WH = OFF_BD + 4;                // [64][160]  folded rgb head layer
constexpr int OFF_BH = OFF_WH + 64 * KV;          // [64]
constexpr int OFF_WV2 = OFF_BH + 64;              // [3][64]    views_linears.2
constexpr int OFF_BV2 = OFF_WV2 + 3 * 64;         // [4]
constexpr int OFF_W1F = OFF_BV2 + 4;              // [128][128] feat_net.0 columns 63..190 (for P)
constexpr int W_TOTAL = OFF_W1F + 128 * 128;

__device__ __forceinline__ float lrelu(float x) { return x >= 0.f ? x : x * 0.01f; }

// acc[mt][nt] += X[rows of mt][k chunk] * W[cols of nt][k chunk]^T over K (multiple of 16),
// X with row stride LD (floats).
template <int K, int MT, int NT, int LD, int UNR = 1>
__device__ __forceinline__ void mfma_acc(const float* __restrict__ X, int row0, const float* __restrict__ Wt,
                                         int col0, f32x4 (&acc)[MT][NT]) {
  const int lane = threadIdx.x & 63;
  const int li = lane & 15, g = lane >> 4;
  const float* xa = X + (row0 + li) * LD + 4 * g;
  const float* wb = Wt + (size_t)(col0 + li) * K + 4 * g;
  // B fragments (weights, from L2) are prefetched one k-chunk ahead so their latency hides
  // behind the current chunk's MFMAs.
  f32x4 b[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) b[nt] = *(const f32x4*)(wb + (size_t)nt * 16 * K);
#pragma unroll UNR
  for (int q = 0; q < K / 16; ++q) {
    f32x4 a[MT], bn[NT];
    const int qn = q + 1 < K / 16 ? q + 1 : q;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) bn[nt] = *(const f32x4*)(wb + (size_t)nt * 16 * K + 16 * qn);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) a[mt] = *(const f32x4*)(xa + mt * 16 * LD + 16 * q);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[mt][t], b[nt][t], acc[mt][nt], 0, 0, 0);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) b[nt] = bn[nt];
  }
}

template <int MT, int NT>
__device__ __forceinline__ void zero_acc(f32x4 (&acc)[MT][NT]) {
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// write lrelu(acc + bias) to X (C layout: col = lane&15, row = 4*(lane>>4) + r)
template <int MT, int NT>
__device__ __forceinline__ void store_act(float* __restrict__ X, int col0, const float* __restrict__ bias,
                                          const f32x4 (&acc)[MT][NT]) {
  const int lane = threadIdx.x & 63;
  const int li = lane & 15, g = lane >> 4;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int col = col0 + 16 * nt + li;
    const float bb = bias[col];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) X[(16 * mt + 4 * g + r) * XS + col] = lrelu(acc[mt][nt][r] + bb);
  }
}

template <int OCC, int UNR>
__global__ __launch_bounds__(MLP_THREADS, OCC) void k_point_mlp(
    const float4* __restrict__ s_pos, const int* __restrict__ s_ray, const int* __restrict__ s_nbr,
    const int* __restrict__ n_samples_dev, const float4* __restrict__ recA, const float4* __restrict__ recB,
    const float4* __restrict__ pproj, const float* __restrict__ viewdirs, const float* __restrict__ vemb_const,
    const float* __restrict__ wbuf, float eps, float shift, float interval, float4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) float X[TR * XS];
  __shared__ float sTo[TR];
  __shared__ int sNbr[TR];
  __shared__ float sIdw[TR];
  __shared__ float sRow[TR * 8];     // direct blend per row: wdir, alpha_c, rgb_c(3), pcol(3)
  __shared__ int sRay[TS];
  __shared__ float sOut[TS * 12];

  const int nS = *n_samples_dev;
  const int ntiles = (nS + TS - 1) / TS;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int li = lane & 15, g = lane >> 4;
  int prev_s0 = -1;
  // XCD-aware tile order: workgroups are dealt round-robin to the 8 XCDs, so XCD x = block % 8
  // takes the contiguous tile range x*chunk ... (x+1)*chunk -- neighbouring samples share
  // neighbour points, and their gathers then hit the same L2.
  const int nx = (gridDim.x % 8 == 0) ? 8 : 1;
  const int xcd = blockIdx.x % nx, per_xcd = gridDim.x / nx;
  const int chunk = (ntiles + nx - 1) / nx;
  const int t_beg = xcd * chunk, t_end = min(ntiles, t_beg + chunk);

  for (int tile = t_beg + blockIdx.x / nx; tile < t_end; tile += per_xcd) {
    const int s0 = tile * TS;
    // ------------------------------------------------ outputs of the previous tile
    if (prev_s0 >= 0 && tid < TS * 3 && prev_s0 + tid / 3 < nS)
      out[(size_t)prev_s0 * 3 + tid] = *(const float4*)(sOut + 4 * tid);
    // ------------------------------------------------ gather + posenc + direct-blend terms
    {
      const int r = tid >> 2, p = tid & 3;
      const int s = r >> 3, k = r & 7;
      const int gs = s0 + s;
      float* xr = X + r * XS;
      if (gs < nS) {
        const int nb = s_nbr[(size_t)gs * 8 + k];
        const float4 q = s_pos[gs];
        const float4 a0 = recA[4 * (size_t)nb + 0];
        const float4 a1 = recA[4 * (size_t)nb + 1];
        const float4 a2 = recA[4 * (size_t)nb + 2];
        const float4 a3 = recA[4 * (size_t)nb + 3];
        const float dx = q.x - a0.x, dy = q.y - a0.y, dz = q.z - a0.z;
        const float rc0 = (a1.x * dx + a1.y * dy) + a1.z * dz;
        const float rc1 = (a1.w * dx + a2.x * dy) + a2.y * dz;
        const float rc2 = (a2.z * dx + a2.w * dy) + a3.x * dz;
        const float tn = (dx * dx + dy * dy) + dz * dz;
        if (p == 0) {
          sTo[r] = tn;
          sNbr[r] = nb;
          xr[0] = rc0; xr[1] = rc1; xr[2] = rc2;
          xr[KE - 1] = 0.f;
          if (k == 0) sRay[s] = s_ray[gs];
        } else if (p == 1) {
          const float4 b0 = recB[2 * (size_t)nb], b1 = recB[2 * (size_t)nb + 1];
          float* rw = sRow + 8 * r;
          rw[0] = expf(-(tn * tn) / a0.w);   // temporalpoints.py:461 (to_nn is already squared)
          rw[1] = a3.y;
          rw[2] = b0.x; rw[3] = b0.y; rw[4] = b0.z;
          rw[5] = b1.x; rw[6] = b1.y; rw[7] = b1.z;
        }
        // 30 arguments rc[i] * 2^f (index a = 10 i + f): sin -> col 3 + a, cos -> col 33 + a
#pragma unroll
        for (int m = 0; m < 8; ++m) {
          const int a = p + 4 * m;
          if (a < 30) {
            const int ci = a / 10;
            const float v = (ci == 0 ? rc0 : (ci == 1 ? rc1 : rc2)) * (float)(1 << (a - 10 * ci));
            float sv, cv;
            sincosf(v, &sv, &cv);
            xr[3 + a] = sv;
            xr[33 + a] = cv;
          }
        }
        const float4* pr = pproj + (size_t)nb * (FEAT / 4);
#pragma unroll
        for (int m = 0; m < 8; ++m) *(float4*)(xr + PCOL + 4 * (p + 4 * m)) = pr[p + 4 * m];
      } else {
        for (int c = p; c < PCOL + FEAT; c += 4) xr[c] = 0.f;
        if (p == 0) {
          sTo[r] = 1.f; sNbr[r] = -1;
          if (k == 0) sRay[s] = 0;   // padding sample: keep the view-embedding gather in bounds
        } else if (p == 1) {
          for (int c = 0; c < 8; ++c) sRow[8 * r + c] = 0.f;
        }
      }
    }
    __syncthreads();
    if (tid < TS) {  // IDW weights (temporalpoints.py:473-475)
      float w[8], sum = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        w[k] = 1.f / (sTo[tid * 8 + k] + eps);
        sum += w[k];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) sIdw[tid * 8 + k] = w[k] / sum;
    }
    // ------------------------------------------------ feat_net (FP32 MFMA)
    const int col0 = 32 * wid;
    f32x4 acc[4][2];
    // layer 1: acc = P[nbr] (C layout read of the gathered P rows) + W1e emb; + b1 at the store
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const int col = col0 + 16 * nt + li;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[mt][nt][r] = X[(16 * mt + 4 * g + r) * XS + PCOL + col];
    }
    mfma_acc<KE, 4, 2, XS, UNR>(X, 0, wbuf + OFF_W1E, col0, acc);
    __syncthreads();
    store_act<4, 2>(X, col0, wbuf + OFF_B1, acc);
    __syncthreads();
#pragma unroll 1
    for (int layer = 0; layer < 3; ++layer) {
      const int ow = layer == 0 ? OFF_W2 : (layer == 1 ? OFF_W3 : OFF_W4);
      zero_acc(acc);
      mfma_acc<128, 4, 2, XS, UNR>(X, 0, wbuf + ow, col0, acc);
      __syncthreads();
      if (layer < 2) {
        store_act<4, 2>(X, col0, wbuf + ow + 128 * 128, acc);
        __syncthreads();
      }
    }
    // ------------------------------------------------ IDW reduction in registers
    // rows of M-tile mt: 16mt + 4g + r -> sample 2mt + (g>>1), neighbour 4(g&1) + r
    float hv[4][2];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const int s = 2 * mt + (g >> 1);
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const float bb = wbuf[OFF_B4 + col0 + 16 * nt + li];
        float pr[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) pr[r] = sIdw[s * 8 + 4 * (g & 1) + r] * lrelu(acc[mt][nt][r] + bb);
        float o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = __shfl_xor(pr[r], 16, 64);
        float h = 0.f;
        h = ((h + pr[0]) + pr[1]) + pr[2];
        h = h + pr[3];
        h = (((h + o[0]) + o[1]) + o[2]) + o[3];
        hv[mt][nt] = h;   // valid in lanes with (g & 1) == 0
      }
    }
    // H -> X rows 0..7 cols 0..127; view embedding -> cols 128..154; rows 8..15 zero (the last
    // barrier of the layer loop guarantees every wave has finished reading X)
    if ((g & 1) == 0) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) X[(2 * mt + (g >> 1)) * XS + col0 + 16 * nt + li] = hv[mt][nt];
    }
    for (int e = tid; e < 8 * KV; e += MLP_THREADS) X[(8 + e / KV) * XS + (e % KV)] = 0.f;
    {
      const int s = tid >> 5, e = tid & 31;
      float v = 0.f;
      if (e < 27) {
        if (vemb_const) {
          v = vemb_const[e];
        } else {
          const int ray = sRay[s];
          // poc_fre(viewdirs, 2^0..2^3): [v (3), sin (12), cos (12)], dim-major
          const int ee = e < 3 ? 0 : (e < 15 ? e - 3 : e - 15);
          const int ci = e < 3 ? e : ee >> 2;
          const float vv = viewdirs[3 * ray + ci];
          const float arg = vv * (float)(1 << (ee & 3));
          v = e < 3 ? vv : (e < 15 ? sinf(arg) : cosf(arg));
        }
      }
      X[s * XS + 128 + e] = v;
    }
    // direct blend + weight-vis colour (temporalpoints.py:459-470, 517-519): wave 1, lane =
    // (sample, quantity); sums over the 8 neighbours in order
    if (wid == 1) {
      const int s = lane >> 3, qn = lane & 7;
      const float* rw = sRow + 64 * s;
      float sumd = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) sumd += rw[8 * k];
      const float dn = sumd + 1e-12f;
      float acc1 = 0.f;
      if (qn == 0) {
#pragma unroll
        for (int k = 0; k < 8; ++k) acc1 += (0.125f * rw[8 * k]) * rw[8 * k + 1];
      } else if (qn < 4) {
#pragma unroll
        for (int k = 0; k < 8; ++k) acc1 += (rw[8 * k] / dn) * rw[8 * k + 1 + qn];
      } else if (qn < 7) {
#pragma unroll
        for (int k = 0; k < 8; ++k) acc1 += sIdw[8 * s + k] * rw[8 * k + 1 + qn];
      }
      // sOut[s] = {r, g, b, alpha, r_d, g_d, b_d, alpha_d, wr, wg, wb, 0}
      const int slot = qn == 0 ? 7 : (qn < 4 ? 3 + qn : (qn < 7 ? 4 + qn : 11));
      sOut[12 * s + slot] = acc1;
    }
    __syncthreads();
    // ------------------------------------------------ heads
    if (wid == 0) {  // densitynet: Linear(128 -> 1), lane = (sample, 16-channel slice)
      const int s = lane >> 3, part = lane & 7;
      const float* hrow = X + s * XS + 16 * part;
      const float* wd = wbuf + OFF_WD + 16 * part;
      float a = 0.f;
#pragma unroll
      for (int c = 0; c < 16; ++c) a += hrow[c] * wd[c];
      a += __shfl_xor(a, 1, 64);
      a += __shfl_xor(a, 2, 64);
      a += __shfl_xor(a, 4, 64);
      if (part == 0) {
        const float e = expf((a + wbuf[OFF_BD]) + shift);
        sOut[12 * s + 3] = 1.f - powf(1.f + e, -interval);
      }
    }
    f32x4 accv[1][1];
    zero_acc(accv);
    mfma_acc<KV, 1, 1, XS>(X, 0, wbuf + OFF_WH, 16 * wid, accv);
    __syncthreads();
    if (g < 2) {
      const int col = 16 * wid + li;
      const float bb = wbuf[OFF_BH + col];
#pragma unroll
      for (int r = 0; r < 4; ++r) X[(4 * g + r) * XS + col] = fmaxf(accv[0][0][r] + bb, 0.f);
    }
    __syncthreads();
    if (wid == 0 && lane < 48) {  // views_linears.2: Linear(64 -> 3) + sigmoid, 2 lanes per output
      const int s = lane / 6, o = (lane % 6) >> 1, half = lane & 1;
      const float* vrow = X + s * XS + 32 * half;
      const float* w2 = wbuf + OFF_WV2 + o * 64 + 32 * half;
      float a = 0.f;
#pragma unroll
      for (int c = 0; c < 32; ++c) a += vrow[c] * w2[c];
      a += __shfl_xor(a, 1, 64);
      if (half == 0) sOut[12 * s + o] = 1.f / (1.f + expf(-(a + wbuf[OFF_BV2 + o])));
    }
    __syncthreads();
    prev_s0 = s0;
  }
  if (prev_s0 >= 0 && tid < TS * 3 && prev_s0 + tid / 3 < nS)
    out[(size_t)prev_s0 * 3 + tid] = *(const float4*)(sOut + 4 * tid);
}

// P = canonical_feat (N x 128) W1f^T (128 x 128): 64-row tiles, 4 waves x 32 columns.
__global__ __launch_bounds__(256) void k_feat_project(const float4* __restrict__ feat, int64_t N,
                                                      const float* __restrict__ w1f, float* __restrict__ P) {
  __shared__ __attribute__((aligned(16))) float T[64 * 136];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int li = lane & 15, g = lane >> 4;
  for (int64_t t0 = (int64_t)blockIdx.x * 64; t0 < N; t0 += (int64_t)gridDim.x * 64) {
    for (int e = tid; e < 64 * 32; e += 256) {
      const int r = e >> 5, c4 = e & 31;
      const float4 v = (t0 + r < N) ? feat[(t0 + r) * 32 + c4] : make_float4(0.f, 0.f, 0.f, 0.f);
      *(float4*)(T + r * 136 + 4 * c4) = v;
    }
    __syncthreads();
    f32x4 acc[4][2];
    zero_acc(acc);
    mfma_acc<128, 4, 2, 136>(T, 0, w1f, 32 * wid, acc);
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t row = t0 + 16 * mt + 4 * g + r;
          if (row < N) P[row * 128 + 32 * wid + 16 * nt + li] = acc[mt][nt][r];
        }
    __syncthreads();
  }
}

}  // namespace apn

using namespace apn;

extern "C" int apn_mlp_weight_layout(int32_t* offsets) {
  const int32_t v[] = {OFF_W1E, OFF_B1, OFF_W2, OFF_B2, OFF_W3, OFF_B3, OFF_W4, OFF_B4, OFF_WD, OFF_BD,
                       OFF_WH, OFF_BH, OFF_WV2, OFF_BV2, OFF_W1F, W_TOTAL, KE, KV};
  for (int i = 0; i < (int)(sizeof(v) / sizeof(v[0])); ++i) offsets[i] = v[i];
  return (int)(sizeof(v) / sizeof(v[0]));
}

// Per-point layer-1 feature projection P [N,128] = canonical_feat [N,128] x W1f^T, with W1f the
// feature columns of feat_net.0 as packed at OFF_W1F of wbuf.
extern "C" int apn_feat_project(const float* canonical_feat, int64_t n_points, int32_t feat_dim, const float* wbuf,
                                float* proj, void* stream) {
  if (feat_dim != FEAT || n_points <= 0 || !canonical_feat || !wbuf || !proj) return APN_ERR_ARG;
  int blocks = (int)((n_points + 63) / 64);
  if (blocks > 256 * 8) blocks = 256 * 8;
  hipLaunchKernelGGL(k_feat_project, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const float4*)canonical_feat,
                     n_points, wbuf + OFF_W1F, proj);
  return launch_status();
}

// out12[n_samples][12] = {r,g,b,alpha, r_d,g_d,b_d,alpha_d, wr,wg,wb,0} per kept sample.
extern "C" int apn_point_mlp(const float* s_pos4, const int32_t* s_ray, const int32_t* s_nbr, int64_t max_samples,
                             const int32_t* n_samples_dev, const float* recA16, const float* recB8,
                             const float* feat_proj, int32_t feat_dim, const float* viewdirs,
                             const float* vemb_const, const float* wbuf, float eps, float act_shift,
                             float interval, int32_t grid_blocks, float* out12, void* stream) {
  if (feat_dim != FEAT) return APN_ERR_ARG;
  if (max_samples <= 0) return APN_OK;
  if (!s_pos4 || !s_ray || !s_nbr || !n_samples_dev || !recA16 || !recB8 || !feat_proj || !wbuf || !out12 ||
      (!viewdirs && !vemb_const))
    return APN_ERR_ARG;
  const int64_t ntiles = (max_samples + TS - 1) / TS;
  // variant 1 (2 waves/SIMD, B prefetch, unroll 2) is the default: 21.4 ms vs 22.9 ms for
  // 3 waves/SIMD at C2; APN_MLP_VARIANT selects the others for A/B runs.
  static const int variant = [] {
    const char* e = getenv("APN_MLP_VARIANT");
    return e ? atoi(e) : 1;
  }();
  const int occ = variant == 0 ? 3 : 2;
  int blocks = grid_blocks > 0 ? grid_blocks : 256 * occ * 8;
  if (blocks > ntiles) blocks = (int)ntiles;
  auto launch = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(MLP_THREADS), 0, (hipStream_t)stream, (const float4*)s_pos4, s_ray,
                       s_nbr, n_samples_dev, (const float4*)recA16, (const float4*)recB8, (const float4*)feat_proj,
                       viewdirs, vemb_const, wbuf, eps, act_shift, interval, (float4*)out12);
  };
  if (variant == 0) launch(k_point_mlp<3, 1>);
  else if (variant == 1) launch(k_point_mlp<2, 2>);
  else launch(k_point_mlp<2, 1>);
  return launch_status();
}
