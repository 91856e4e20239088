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
constexpr int K1 = 192;           // 63 + 128 = 191, zero-padded

// Packed weight buffer layout (floats). Mirrored by apn_amd/ops.py:pack_mlp_weights via
// apn_mlp_weight_layout().
constexpr int OFF_W1 = 0;                         // [128][192]
constexpr int OFF_B1 = OFF_W1 + 128 * K1;         // [128]
constexpr int OFF_W2 = OFF_B1 + 128;              // [128][128]
constexpr int OFF_B2 = OFF_W2 + 128 * 128;
constexpr int OFF_W3 = OFF_B2 + 128;
constexpr int OFF_B3 = OFF_W3 + 128 * 128;
constexpr int OFF_W4 = OFF_B3 + 128;
constexpr int OFF_B4 = OFF_W4 + 128 * 128;
constexpr int OFF_WD = OFF_B4 + 128;              // [128]
constexpr int OFF_BD = OFF_WD + 128;              // [4] (1 used)
constexpr int OFF_WF = OFF_BD + 4;                // [128][128] rgbnet.feature_linears
constexpr int OFF_BF = OFF_WF + 128 * 128;
constexpr int KV = 160;                           // 128 + 27 = 155, zero-padded
constexpr int OFF_WV0 = OFF_BF + 128;             // [64][160] rgbnet.views_linears.0
constexpr int OFF_BV0 = OFF_WV0 + 64 * KV;
constexpr int OFF_WV2 = OFF_BV0 + 64;             // [3][64] rgbnet.views_linears.2
constexpr int OFF_BV2 = OFF_WV2 + 3 * 64;         // [4]
constexpr int W_TOTAL = OFF_BV2 + 4;

__device__ __forceinline__ float lrelu(float x) { return x >= 0.f ? x : x * 0.01f; }

// acc[mt][nt] += X[rows of mt][k chunk] * W[cols of nt][k chunk]^T over K (multiple of 16)
template <int K, int MT, int NT>
__device__ __forceinline__ void mfma_layer(const float* __restrict__ X, int row0, const float* __restrict__ Wt,
                                           int col0, f32x4 (&acc)[MT][NT]) {
  const int lane = threadIdx.x & 63;
  const int li = lane & 15, g = lane >> 4;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float* xa = X + (row0 + li) * XS + 4 * g;
  const float* wb = Wt + (size_t)(col0 + li) * K + 4 * g;
#pragma unroll 2
  for (int q = 0; q < K / 16; ++q) {
    f32x4 a[MT], b[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) b[nt] = *(const f32x4*)(wb + (size_t)nt * 16 * K + 16 * q);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) a[mt] = *(const f32x4*)(xa + mt * 16 * XS + 16 * q);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[mt][t], b[nt][t], acc[mt][nt], 0, 0, 0);
  }
}

// write lrelu(acc + bias) to X (C layout: col = lane&15, row = 4*(lane>>4) + r)
template <int MT, int NT>
__device__ __forceinline__ void store_act(float* __restrict__ X, int row0, int col0, const float* __restrict__ bias,
                                          const f32x4 (&acc)[MT][NT], bool leaky) {
  const int lane = threadIdx.x & 63;
  const int li = lane & 15, g = lane >> 4;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int col = col0 + 16 * nt + li;
    const float bb = bias[col];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc[mt][nt][r] + bb;
        X[(row0 + 16 * mt + 4 * g + r) * XS + col] = leaky ? lrelu(v) : v;
      }
  }
}

__global__ __launch_bounds__(MLP_THREADS, 3) void k_point_mlp(
    const float4* __restrict__ s_pos, const int* __restrict__ s_ray, const int* __restrict__ s_nbr,
    const int* __restrict__ n_samples_dev, const float4* __restrict__ recA, const float4* __restrict__ recB,
    const float4* __restrict__ feat, const float* __restrict__ viewdirs, const float* __restrict__ vemb_const,
    const float* __restrict__ wbuf, float eps, float shift, float interval, float4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) float X[TR * XS];
  __shared__ float sTo[TR];
  __shared__ int sNbr[TR];
  __shared__ float sIdw[TR];
  __shared__ int sRay[TS];
  __shared__ float sAlpha[TS];
  __shared__ float sRgb[TS * 3];

  const int nS = *n_samples_dev;
  const int ntiles = (nS + TS - 1) / TS;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int li = lane & 15, g = lane >> 4;

  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int s0 = tile * TS;
    // ------------------------------------------------------------ gather + posenc
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
        if (p == 0) {
          sTo[r] = (dx * dx + dy * dy) + dz * dz;
          sNbr[r] = nb;
          xr[0] = rc0; xr[1] = rc1; xr[2] = rc2;
          xr[K1 - 1] = 0.f;
          if (k == 0) sRay[s] = s_ray[gs];
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
        const float4* fr = feat + (size_t)nb * (FEAT / 4);
#pragma unroll
        for (int m = 0; m < 8; ++m) {
          const float4 f = fr[p + 4 * m];
          float* d = xr + 63 + 4 * (p + 4 * m);
          d[0] = f.x; d[1] = f.y; d[2] = f.z; d[3] = f.w;
        }
      } else {
        for (int c = p; c < K1; c += 4) xr[c] = 0.f;
        if (p == 0) {
          sTo[r] = 1.f; sNbr[r] = -1;
          if (k == 0) sRay[s] = 0;   // padding sample: keep the view-embedding gather in bounds
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
    // ------------------------------------------------------------ feat_net (FP32 MFMA)
    f32x4 acc[4][2];
    const int col0 = 32 * wid;
    mfma_layer<K1, 4, 2>(X, 0, wbuf + OFF_W1, col0, acc);
    __syncthreads();
    store_act<4, 2>(X, 0, col0, wbuf + OFF_B1, acc, true);
    __syncthreads();
    mfma_layer<128, 4, 2>(X, 0, wbuf + OFF_W2, col0, acc);
    __syncthreads();
    store_act<4, 2>(X, 0, col0, wbuf + OFF_B2, acc, true);
    __syncthreads();
    mfma_layer<128, 4, 2>(X, 0, wbuf + OFF_W3, col0, acc);
    __syncthreads();
    store_act<4, 2>(X, 0, col0, wbuf + OFF_B3, acc, true);
    __syncthreads();
    mfma_layer<128, 4, 2>(X, 0, wbuf + OFF_W4, col0, acc);
    // ------------------------------------------------------------ IDW reduction in registers
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
    __syncthreads();   // all waves done reading X (layer-3 activations)
    // H -> X rows 0..7 (rows 8..15 zero, cols 0..159)
    if ((g & 1) == 0) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) X[(2 * mt + (g >> 1)) * XS + col0 + 16 * nt + li] = hv[mt][nt];
    }
    for (int e = tid; e < 8 * KV; e += MLP_THREADS) X[(8 + e / KV) * XS + (e % KV)] = 0.f;
    __syncthreads();
    // ------------------------------------------------------------ heads
    float dens = 0.f;
    if (tid < TS) {  // densitynet: Linear(128 -> 1)
      const float* wd = wbuf + OFF_WD;
      float a = 0.f;
      for (int c = 0; c < FEAT; ++c) a += X[tid * XS + c] * wd[c];
      dens = a + wbuf[OFF_BD];
    }
    f32x4 accf[1][2];
    mfma_layer<128, 1, 2>(X, 0, wbuf + OFF_WF, col0, accf);
    __syncthreads();
    // f = feature_linears(h) (no activation) -> X rows 0..7 cols 0..127 ; view embedding 128..154
    if (g < 2) {
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const int col = col0 + 16 * nt + li;
        const float bb = wbuf[OFF_BF + col];
#pragma unroll
        for (int r = 0; r < 4; ++r) X[(4 * g + r) * XS + col] = accf[0][nt][r] + bb;
      }
    }
    if (tid < TS * 32) {
      const int s = tid >> 5, e = tid & 31;
      if (e < 27) {
        float v;
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
        X[s * XS + 128 + e] = v;
      } else if (e < 32) {
        X[s * XS + 128 + e] = 0.f;   // cols 155..159
      }
    }
    __syncthreads();
    f32x4 accv[1][1];
    mfma_layer<KV, 1, 1>(X, 0, wbuf + OFF_WV0, 16 * wid, accv);
    __syncthreads();
    if (g < 2) {
      const int col = 16 * wid + li;
      const float bb = wbuf[OFF_BV0 + col];
#pragma unroll
      for (int r = 0; r < 4; ++r) X[(4 * g + r) * XS + col] = fmaxf(accv[0][0][r] + bb, 0.f);
    }
    if (tid < TS) {
      const float e = expf(dens + shift);
      sAlpha[tid] = 1.f - powf(1.f + e, -interval);
    }
    __syncthreads();
    if (tid < TS * 3) {
      const int s = tid / 3, o = tid % 3;
      const float* w2 = wbuf + OFF_WV2 + o * 64;
      float a = 0.f;
      for (int c = 0; c < 64; ++c) a += X[s * XS + c] * w2[c];
      a = a + wbuf[OFF_BV2 + o];
      sRgb[tid] = 1.f / (1.f + expf(-a));
    }
    __syncthreads();
    // ------------------------------------------------------------ direct blend + outputs
    if (tid < TS && s0 + tid < nS) {
      const int s = tid;
      float wdir[8], sumd = 0.f, ad = 0.f;
      float4 rgbc[8];
      float pc0 = 0.f, pc1 = 0.f, pc2 = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int nb = sNbr[s * 8 + k];
        const float tn = sTo[s * 8 + k];
        const float4 a0 = recA[4 * (size_t)nb];
        const float ac = recA[4 * (size_t)nb + 3].y;
        rgbc[k] = recB[2 * (size_t)nb];
        const float4 pcol = recB[2 * (size_t)nb + 1];
        wdir[k] = expf(-(tn * tn) / a0.w);
        sumd += wdir[k];
        ad += (0.125f * wdir[k]) * ac;
        const float wi = sIdw[s * 8 + k];
        pc0 += wi * pcol.x; pc1 += wi * pcol.y; pc2 += wi * pcol.z;
      }
      const float dn = sumd + 1e-12f;
      float rd = 0.f, gd = 0.f, bd = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float wn = wdir[k] / dn;
        rd += wn * rgbc[k].x; gd += wn * rgbc[k].y; bd += wn * rgbc[k].z;
      }
      const size_t o = (size_t)(s0 + s) * 3;
      out[o + 0] = make_float4(sRgb[3 * s], sRgb[3 * s + 1], sRgb[3 * s + 2], sAlpha[s]);
      out[o + 1] = make_float4(rd, gd, bd, ad);
      out[o + 2] = make_float4(pc0, pc1, pc2, 0.f);
    }
    __syncthreads();
  }
}

}  // namespace apn

using namespace apn;

extern "C" int apn_mlp_weight_layout(int32_t* offsets) {
  const int32_t v[] = {OFF_W1, OFF_B1, OFF_W2, OFF_B2, OFF_W3, OFF_B3, OFF_W4, OFF_B4, OFF_WD, OFF_BD,
                       OFF_WF, OFF_BF, OFF_WV0, OFF_BV0, OFF_WV2, OFF_BV2, W_TOTAL, K1, KV};
  for (int i = 0; i < (int)(sizeof(v) / sizeof(v[0])); ++i) offsets[i] = v[i];
  return (int)(sizeof(v) / sizeof(v[0]));
}

// out12[n_samples][12] = {r,g,b,alpha, r_d,g_d,b_d,alpha_d, wr,wg,wb,0} per kept sample.
extern "C" int apn_point_mlp(const float* s_pos4, const int32_t* s_ray, const int32_t* s_nbr, int64_t max_samples,
                             const int32_t* n_samples_dev, const float* recA16, const float* recB8,
                             const float* canonical_feat, int32_t feat_dim, const float* viewdirs,
                             const float* vemb_const, const float* wbuf, float eps, float act_shift,
                             float interval, int32_t grid_blocks, float* out12, void* stream) {
  if (feat_dim != FEAT) return APN_ERR_ARG;
  if (max_samples <= 0) return APN_OK;
  if (!s_pos4 || !s_ray || !s_nbr || !n_samples_dev || !recA16 || !recB8 || !canonical_feat || !wbuf || !out12 ||
      (!viewdirs && !vemb_const))
    return APN_ERR_ARG;
  const int64_t ntiles = (max_samples + TS - 1) / TS;
  int blocks = grid_blocks > 0 ? grid_blocks : 256 * 3 * 8;
  if (blocks > ntiles) blocks = (int)ntiles;
  hipLaunchKernelGGL(k_point_mlp, dim3(blocks), dim3(MLP_THREADS), 0, (hipStream_t)stream, (const float4*)s_pos4,
                     s_ray, s_nbr, n_samples_dev, (const float4*)recA16, (const float4*)recB8,
                     (const float4*)canonical_feat, viewdirs, vemb_const, wbuf, eps, act_shift, interval,
                     (float4*)out12);
  return launch_status();
}
