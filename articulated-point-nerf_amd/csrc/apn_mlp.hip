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
// the 16x16x4 A-operand pattern), 2 workgroups per CU. Each wave owns 32 output columns
// (2 N-tiles x 4 M-tiles of 16x16); B-operand fragments stream from L2-resident weights.
// k-permutation: for a 16-wide k chunk q, lane group g = lane>>4 holds k = 16q + 4g + t in
// element t of its float4, for both A (activations) and B (nn.Linear weight rows), so one
// 16-byte load feeds 4 MFMAs.
#include "apn_mlp_layout.h"

#include <algorithm>

namespace apn {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int XS = 200;           // LDS row stride (floats)
constexpr int PCOL = 64;          // LDS column where the gathered P row starts

// Small weights staged in LDS once per workgroup (biases, densitynet, views_linears.2).
constexpr int SW_B1 = 0, SW_B2 = 128, SW_B3 = 256, SW_B4 = 384, SW_WD = 512, SW_BD = 640, SW_BH = 644,
              SW_WV2 = 708, SW_BV2 = 900, SW_TOTAL = 904;

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

// Same contraction with the B chunk-0 fragments carried in `b` (loaded by the previous call) and
// chunk 0 of the next weight matrix Wn (row length KN) prefetched into `b` on exit, so the L2
// latency of a layer's first chunk hides behind the previous layer / tile.
template <int K, int MT, int NT, int LD, int UNR, int KN>
__device__ __forceinline__ void mfma_acc_pf(const float* __restrict__ X, const float* __restrict__ Wt, int col0,
                                            const float* __restrict__ Wn, f32x4 (&acc)[MT][NT], f32x4 (&b)[NT]) {
  const int lane = threadIdx.x & 63;
  const int li = lane & 15, g = lane >> 4;
  const float* xa = X + li * LD + 4 * g;
  const float* wb = Wt + (size_t)(col0 + li) * K + 4 * g;
  const float* wn = Wn + (size_t)(col0 + li) * KN + 4 * g;
  // software pipeline: the A (LDS) and B (L2) fragments of chunk q+1 are issued before the
  // MFMAs of chunk q; sched_barrier pins the issue point so the scheduler cannot sink the
  // loads next to their use (which exposed the L2 latency once per chunk).
  f32x4 a[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) a[mt] = *(const f32x4*)(xa + mt * 16 * LD);
#pragma unroll 2
  for (int q = 0; q < K / 16; ++q) {
    f32x4 an[MT], bn[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
      bn[nt] = *(const f32x4*)(q + 1 < K / 16 ? wb + (size_t)nt * 16 * K + 16 * (q + 1) : wn + (size_t)nt * 16 * KN);
    if (q + 1 < K / 16) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) an[mt] = *(const f32x4*)(xa + mt * 16 * LD + 16 * (q + 1));
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[mt][t], b[nt][t], acc[mt][nt], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) b[nt] = bn[nt];
    if (q + 1 < K / 16) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) a[mt] = an[mt];
    }
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

// Per-phase cycle sums of the TIMED variant (wave 0 of every workgroup): gather, layer 1,
// layers 2-4, epilogue, tiles, whole-kernel cycles. Read by apn_debug_mlp_phase_cycles.
__device__ unsigned long long g_mlp_phase[6];

template <int OCC, int UNR, bool TIMED = false>
__global__ __launch_bounds__(MLP_THREADS, OCC) void k_point_mlp(
    const float4* __restrict__ s_pos, const int* __restrict__ s_ray, const int* __restrict__ s_nbr,
    const int* __restrict__ n_samples_dev, const float4* __restrict__ recA, const float4* __restrict__ recB,
    const float4* __restrict__ pproj, const float* __restrict__ viewdirs, const float* __restrict__ vemb_const,
    const float* __restrict__ wbuf, float eps, float shift, float interval, float4* __restrict__ out,
    const int* __restrict__ run_if) {
  if (run_if) {  // range fallback of the fp16-split kernel: run only if it flagged this launch
    __shared__ int s_run;
    if (threadIdx.x == 0) s_run = __builtin_nontemporal_load(run_if);
    __syncthreads();
    if (!s_run) return;
  }
  __shared__ __attribute__((aligned(16))) float X[TR * XS];
  __shared__ float sTo[TR];
  __shared__ int sNbr[TR];
  __shared__ float sIdw[TR];
  __shared__ float sRow[TR * 8];     // direct blend per row: wdir, alpha_c, rgb_c(3), pcol(3)
  __shared__ float sOut[TS * 12];
  __shared__ float sV[TS * 32];      // view embedding per sample (27 + zero pad)
  __shared__ float sW[SW_TOTAL];

  const int nS = *n_samples_dev;
  const int ntiles = (nS + TS - 1) / TS;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int li = lane & 15, g = lane >> 4;
  int prev_s0 = -1;
  for (int i = tid; i < 128; i += MLP_THREADS) {
    sW[SW_B1 + i] = wbuf[OFF_B1 + i];
    sW[SW_B2 + i] = wbuf[OFF_B2 + i];
    sW[SW_B3 + i] = wbuf[OFF_B3 + i];
    sW[SW_B4 + i] = wbuf[OFF_B4 + i];
    sW[SW_WD + i] = wbuf[OFF_WD + i];
  }
  if (tid < 64) sW[SW_BH + tid] = wbuf[OFF_BH + tid];
  if (tid < 192) sW[SW_WV2 + tid] = wbuf[OFF_WV2 + tid];
  if (tid < 3) sW[SW_BV2 + tid] = wbuf[OFF_BV2 + tid];
  if (tid == 0) sW[SW_BD] = wbuf[OFF_BD];
  // XCD-aware tile order: workgroups are dealt round-robin to the 8 XCDs, so XCD x = block % 8
  // takes the contiguous tile range x*chunk ... (x+1)*chunk -- neighbouring samples share
  // neighbour points, and their gathers then hit the same L2.
  const int nx = (gridDim.x % 8 == 0) ? 8 : 1;
  const int xcd = blockIdx.x % nx, per_xcd = gridDim.x / nx;
  const int chunk = (ntiles + nx - 1) / nx;
  const int t_beg = xcd * chunk, t_end = min(ntiles, t_beg + chunk);

  unsigned long long ph[6] = {0, 0, 0, 0, 0, 0}, tk = 0, tk0 = 0;
  if (TIMED) tk0 = clock64();
#define APN_PHASE(i)                         \
  if (TIMED) {                               \
    const unsigned long long now = clock64(); \
    ph[i] += now - tk;                       \
    tk = now;                                \
  }
  // per-thread gather coordinates: row r = (sample s, neighbour k), quarter p of the row
  const int gr = tid >> 2, gp = tid & 3, gsm = gr >> 3, gk = gr & 7;
  // next-tile prefetch of the sample's neighbour index / position / ray (consumed one tile later)
  int pf_nb = -1, pf_ray = 0;
  float4 pf_q = make_float4(0.f, 0.f, 0.f, 0.f);
  auto fetch = [&](int tl) {
    const int gs = tl * TS + gsm;
    pf_nb = -1;
    if (tl < t_end && gs < nS) {
      pf_nb = s_nbr[(size_t)gs * 8 + gk];
      pf_q = s_pos[gs];
      pf_ray = s_ray[gs];
    }
  };
  int tile = t_beg + blockIdx.x / nx;
  fetch(tile);
  f32x4 bpf[2];   // carried B prefetch (chunk 0 of the next weight matrix)
  {
    const float* w0 = wbuf + OFF_W1E + (size_t)(32 * wid + li) * KE + 4 * g;
    bpf[0] = *(const f32x4*)w0;
    bpf[1] = *(const f32x4*)(w0 + 16 * KE);
  }
  for (; tile < t_end; tile += per_xcd) {
    const int s0 = tile * TS;
    if (TIMED) { tk = clock64(); ph[4] += 1; }
    // ------------------------------------------------ outputs of the previous tile
    if (prev_s0 >= 0 && tid < TS * 3 && prev_s0 + tid / 3 < nS)
      out[(size_t)prev_s0 * 3 + tid] = *(const float4*)(sOut + 4 * tid);
    // ------------------------------------------------ gather + posenc + direct-blend terms
    {
      const int r = gr, p = gp, s = gsm, k = gk;
      float* xr = X + r * XS;
      const int nb = pf_nb;
      const float4 q = pf_q;
      const int ray = pf_ray;
      if (nb >= 0) {
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
        {  // view embedding element e of this sample: poc_fre(viewdirs, 2^0..2^3) = [v, sin (12), cos (12)]
          const int e = 4 * k + p;
          float v = 0.f;
          if (e < 27) {
            if (vemb_const) {
              v = vemb_const[e];
            } else {
              const int ee = e < 3 ? 0 : (e < 15 ? e - 3 : e - 15);
              const int ci = e < 3 ? e : ee >> 2;
              const float vv = viewdirs[3 * ray + ci];
              const float arg = vv * (float)(1 << (ee & 3));
              v = e < 3 ? vv : (e < 15 ? sinf(arg) : cosf(arg));
            }
          }
          sV[s * 32 + e] = v;
        }
      } else {
        sV[s * 32 + 4 * k + p] = 0.f;
        for (int c = p; c < PCOL + FEAT; c += 4) xr[c] = 0.f;
        if (p == 0) {
          sTo[r] = 1.f; sNbr[r] = -1;
        } else if (p == 1) {
          for (int c = 0; c < 8; ++c) sRow[8 * r + c] = 0.f;
        }
      }
    }
    fetch(tile + per_xcd);
    __syncthreads();
    APN_PHASE(0)
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
    mfma_acc_pf<KE, 4, 2, XS, UNR, 128>(X, wbuf + OFF_W1E, col0, wbuf + OFF_W2, acc, bpf);
    __syncthreads();
    store_act<4, 2>(X, col0, sW + SW_B1, acc);
    __syncthreads();
    APN_PHASE(1)
#pragma unroll 1
    for (int layer = 0; layer < 3; ++layer) {
      const int ow = layer == 0 ? OFF_W2 : (layer == 1 ? OFF_W3 : OFF_W4);
      zero_acc(acc);
      if (layer < 2)
        mfma_acc_pf<128, 4, 2, XS, UNR, 128>(X, wbuf + ow, col0, wbuf + ow + 128 * 128 + 128, acc, bpf);
      else
        mfma_acc_pf<128, 4, 2, XS, UNR, KE>(X, wbuf + ow, col0, wbuf + OFF_W1E, acc, bpf);
      __syncthreads();
      if (layer < 2) {
        store_act<4, 2>(X, col0, sW + SW_B2 + 128 * layer, acc);
        __syncthreads();
      }
    }
    APN_PHASE(2)
    // head weights (folded rgb layer, this wave's 16 columns) -> registers; their latency hides
    // behind the IDW reduction and the direct blend
    f32x4 whr[KV / 16];
#pragma unroll
    for (int q = 0; q < KV / 16; ++q) whr[q] = *(const f32x4*)(wbuf + OFF_WH + (16 * wid + li) * KV + 16 * q + 4 * g);
    // ------------------------------------------------ IDW reduction in registers
    // rows of M-tile mt: 16mt + 4g + r -> sample 2mt + (g>>1), neighbour 4(g&1) + r
    float hv[4][2];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const int s = 2 * mt + (g >> 1);
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const float bb = sW[SW_B4 + col0 + 16 * nt + li];
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
    X[(tid >> 5) * XS + 128 + (tid & 31)] = sV[tid];
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
      const float* wd = sW + SW_WD + 16 * part;
      float a = 0.f;
#pragma unroll
      for (int c = 0; c < 16; ++c) a += hrow[c] * wd[c];
      a += __shfl_xor(a, 1, 64);
      a += __shfl_xor(a, 2, 64);
      a += __shfl_xor(a, 4, 64);
      if (part == 0) {
        const float e = expf((a + sW[SW_BD]) + shift);
        sOut[12 * s + 3] = 1.f - powf(1.f + e, -interval);
      }
    }
    f32x4 accv = {0.f, 0.f, 0.f, 0.f};
    {
      const float* xa = X + li * XS + 4 * g;
#pragma unroll
      for (int q = 0; q < KV / 16; ++q) {
        const f32x4 a = *(const f32x4*)(xa + 16 * q);
#pragma unroll
        for (int t = 0; t < 4; ++t) accv = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t], whr[q][t], accv, 0, 0, 0);
      }
    }
    __syncthreads();
    if (g < 2) {
      const int col = 16 * wid + li;
      const float bb = sW[SW_BH + col];
#pragma unroll
      for (int r = 0; r < 4; ++r) X[(4 * g + r) * XS + col] = fmaxf(accv[r] + bb, 0.f);
    }
    __syncthreads();
    if (wid == 0 && lane < 48) {  // views_linears.2: Linear(64 -> 3) + sigmoid, 2 lanes per output
      const int s = lane / 6, o = (lane % 6) >> 1, half = lane & 1;
      const float* vrow = X + s * XS + 32 * half;
      const float* w2 = sW + SW_WV2 + o * 64 + 32 * half;
      float a = 0.f;
#pragma unroll
      for (int c = 0; c < 32; ++c) a += vrow[c] * w2[c];
      a += __shfl_xor(a, 1, 64);
      if (half == 0) sOut[12 * s + o] = 1.f / (1.f + expf(-(a + sW[SW_BV2 + o])));
    }
    __syncthreads();
    APN_PHASE(3)
    prev_s0 = s0;
  }
#undef APN_PHASE
  if (TIMED && tid == 0) {
    ph[5] = clock64() - tk0;
    for (int i = 0; i < 6; ++i) atomicAdd(&g_mlp_phase[i], ph[i]);
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
                       OFF_WH, OFF_BH, OFF_WV2, OFF_BV2, OFF_W1F, W_TOTAL, KE, KV, OFF_H16, OFF_FLAG};
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

// Kernel selection: initialised from APN_MLP_VARIANT, changed by apn_set_mlp_variant.
static int& mlp_variant() {
  static int v = [] {
    const char* e = apn_env("APN_MLP_VARIANT");
    return e ? atoi(e) : 0;
  }();
  return v;
}

// 0 = fp16-split kernel (default), 1 = FP32 MFMA kernel; the debug build also has 2 / 3, the
// phase-timed builds of each (profiling aid).
// 4 = the 64-row fp16-split kernel (apn_mlp_h3.hip), the default before the 128-row tiles.
#ifdef APN_DEBUG_BUILD
static bool mlp_variant_ok(int v) { return v >= 0 && v <= 5; }
#else
static bool mlp_variant_ok(int v) { return v == 0 || v == 1 || v == 4; }
#endif
extern "C" int apn_set_mlp_variant(int32_t variant) {
  const int prev = mlp_variant();
  if (mlp_variant_ok(variant)) mlp_variant() = variant;
  return prev;
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
  // 0 (default) = 3-term fp16-split MFMA kernel on 128-row tiles (apn_mlp_h4.hip; wbuf prepared by
  // apn_mlp_split_weights), 1 = FP32 MFMA kernel (this file), 4 = the fp16-split kernel on 64-row
  // tiles (apn_mlp_h3.hip); debug build: 2 / 3 / 5 = phase-timed builds of 1 / 4 / 0.
  const int variant = mlp_variant();
  const bool t128 = variant == 0 || variant == 5;
  const int64_t ntiles = (max_samples + (t128 ? 16 : TS) - 1) / (t128 ? 16 : TS);
  static const int env_blocks = [] {
    const char* e = apn_env("APN_MLP_BLOCKS");
    return e ? atoi(e) : 0;
  }();
  if (grid_blocks <= 0) grid_blocks = env_blocks;
  // 64 workgroups per CU over the whole launch (3 resident at a time for the default kernel): the
  // grid-stride loop gives each ~17 tiles, which balances the tail better than 8 per CU (-1.5 %)
  // while keeping the cross-tile index prefetch; one workgroup per tile is 12 % slower.
  int blocks = grid_blocks > 0 ? grid_blocks : 256 * 64;
  if (blocks > ntiles) blocks = (int)ntiles;
  auto launch = [&](auto kern, int nblocks, const int* run_if) {
    hipLaunchKernelGGL(kern, dim3(nblocks), dim3(MLP_THREADS), 0, (hipStream_t)stream, (const float4*)s_pos4, s_ray,
                       s_nbr, n_samples_dev, (const float4*)recA16, (const float4*)recB8, (const float4*)feat_proj,
                       viewdirs, vemb_const, wbuf, eps, act_shift, interval, (float4*)out12, run_if);
  };
  if (variant == 1) {
    launch(k_point_mlp<2, 2>, blocks, nullptr);
#ifdef APN_DEBUG_BUILD
  } else if (variant == 2) {
    launch(k_point_mlp<2, 2, true>, blocks, nullptr);
#endif
  } else {
    if (t128)
      launch_point_mlp_h4(blocks, variant == 5, (hipStream_t)stream, (const float4*)s_pos4, s_ray, s_nbr, n_samples_dev,
                          (const float4*)recA16, (const float4*)recB8, (const float4*)feat_proj, viewdirs, vemb_const,
                          wbuf, eps, act_shift, interval, (float4*)out12);
    else
      launch_point_mlp_h3(blocks, variant == 3, (hipStream_t)stream, (const float4*)s_pos4, s_ray, s_nbr,
                          n_samples_dev, (const float4*)recA16, (const float4*)recB8, (const float4*)feat_proj,
                          viewdirs, vemb_const, wbuf, eps, act_shift, interval, (float4*)out12);
    // range fallback (apn_mlp_layout.h OFF_FLAG): the FP32 MFMA kernel redoes the launch iff the
    // split kernel flagged an out-of-fp16-range value; otherwise its workgroups exit at once
    // (8 per CU: a few microseconds). Stream order makes the flag visible; no host sync.
    int fb = 256 * 8;
    if (fb > blocks) fb = blocks;
    launch(k_point_mlp<2, 2>, fb, (const int*)(wbuf + OFF_FLAG));
  }
  return launch_status();
}

// The direct-path and weight-colour columns (4..11) of out12 for every kept sample
// (temporalpoints.py:459-470, 517-519), the fused MLP kernel's arithmetic; apn_point_mlp_ert
// runs it itself unless with_direct = 0.
extern "C" int apn_direct_blend(const float* s_pos4, const int32_t* s_nbr, int64_t max_samples,
                                const int32_t* n_samples_dev, const float* recA16, const float* recB8, float eps,
                                float* out12, void* stream) {
  if (max_samples <= 0) return APN_OK;
  if (!s_pos4 || !s_nbr || !n_samples_dev || !recA16 || !recB8 || !out12) return APN_ERR_ARG;
  return direct_blend((const float4*)s_pos4, s_nbr, max_samples, n_samples_dev, (const float4*)recA16,
                      (const float4*)recB8, eps, (float4*)out12, (hipStream_t)stream);
}

extern "C" size_t apn_point_mlp_ert_workspace_bytes(int64_t max_samples, int64_t n_rays) {
  return ert_workspace_bytes(max_samples > 0 ? max_samples : 1, n_rays > 0 ? n_rays : 1);
}

// apn_point_mlp with early ray termination (apn_ert.hip): the MLP's {rgb, alpha} columns for the
// kept samples the compositing reads (every ray's samples up to its T < 1e-3 break), in ERT_PASSES
// passes over the live rays; the direct-path and weight-colour columns for every kept sample. With
// apn_composite on the same samples the frame is bit-identical to apn_point_mlp's.
extern "C" int apn_point_mlp_ert(const float* s_pos4, const int32_t* s_ray, const int32_t* s_nbr, int64_t max_samples,
                                 const int32_t* n_samples_dev, int64_t n_rays, const float* recA16, const float* recB8,
                                 const float* feat_proj, int32_t feat_dim, const float* viewdirs,
                                 const float* vemb_const, const float* wbuf, float eps, float act_shift,
                                 float interval, float fast_color_thres, int32_t with_direct, float* out12,
                                 void* workspace, int32_t* pass_rows, void* const* pass_events, void* stream) {
  if (feat_dim != FEAT || n_rays <= 0) return APN_ERR_ARG;
  if (max_samples <= 0) return APN_OK;
  if (!s_pos4 || !s_ray || !s_nbr || !n_samples_dev || !recA16 || !recB8 || !feat_proj || !wbuf || !out12 ||
      !workspace || (!viewdirs && !vemb_const))
    return APN_ERR_ARG;
  if (mlp_variant() != 0)   // the pass lists exist for the default (128-row split) kernel only
    return apn_point_mlp(s_pos4, s_ray, s_nbr, max_samples, n_samples_dev, recA16, recB8, feat_proj, feat_dim,
                         viewdirs, vemb_const, wbuf, eps, act_shift, interval, 0, out12, stream);
  hipStream_t s = (hipStream_t)stream;
  const int64_t ntiles = (max_samples + 15) / 16;
  // a pass's size is known on the device only: a grid of ERT_MLP_BLOCKS workgroups (grid-stride
  // over the pass's tiles) instead of one per tile, so the passes that find few or no live rays
  // cost a few microseconds, not the dispatch of 16k workgroups that exit at once
  // sized by the launch's capacity: ~1/64 of its tiles, between 512 (2 per CU) and ERT_MLP_BLOCKS,
  // a multiple of 8 (the XCD-aware tile order): a ray shard's passes hold ~2k tiles, and at 2048
  // workgroups most of them staged the weights for one tile (shard of 8, same box, 4 in flight:
  // 0.909 / 0.925 ms at 512 vs 0.928 / 0.928 at 2048; the full frame keeps 2048)
  const int64_t want = std::max<int64_t>(512, std::min<int64_t>(ERT_MLP_BLOCKS, ntiles / 64)) & ~int64_t(7);
  const int blocks = (int)(ntiles < want ? ntiles : want);
  MlpPass pass = [&](const int* list, const int* n_list) {
    launch_point_mlp_h4(blocks, false, s, (const float4*)s_pos4, s_ray, s_nbr, n_list, (const float4*)recA16,
                        (const float4*)recB8, (const float4*)feat_proj, viewdirs, vemb_const, wbuf, eps, act_shift,
                        interval, (float4*)out12, list);
    return launch_status();
  };
  APN_TRY(ert_run((const float4*)s_pos4, s_ray, s_nbr, max_samples, n_samples_dev, n_rays, (const float4*)recA16,
                  (const float4*)recB8, eps, fast_color_thres, (float4*)out12, workspace, with_direct, pass_rows,
                  pass_events, s, pass));
  // range fallback (apn_mlp_layout.h OFF_FLAG): if any pass flagged an out-of-fp16-range value, the
  // FP32 MFMA kernel redoes every kept sample (all 12 columns, a superset of the passes); otherwise
  // its workgroups exit at once
  const int fb = blocks < 256 * 8 ? blocks : 256 * 8;
  auto fp32_kernel = k_point_mlp<2, 2>;
  hipLaunchKernelGGL(fp32_kernel, dim3(fb), dim3(MLP_THREADS), 0, s, (const float4*)s_pos4, s_ray, s_nbr,
                     n_samples_dev, (const float4*)recA16, (const float4*)recB8, (const float4*)feat_proj, viewdirs,
                     vemb_const, wbuf, eps, act_shift, interval, (float4*)out12, (const int*)(wbuf + OFF_FLAG));
  return launch_status();
}

#ifdef APN_DEBUG_BUILD
// Profiling aid: copy (and reset) the per-phase cycle sums of the timed MLP variants
// (APN_MLP_VARIANT=2, 3): {gather, layer 1, layers 2-4, epilogue, tiles, kernel} summed over
// workgroups. Synchronous.
extern "C" int apn_debug_mlp_phase_cycles(uint64_t* out6) {
  if (!out6) return APN_ERR_ARG;
  APN_HIP_TRY(hipDeviceSynchronize());
  APN_HIP_TRY(hipMemcpyFromSymbol(out6, HIP_SYMBOL(g_mlp_phase), sizeof(uint64_t) * 6));
  static const unsigned long long zero[6] = {0, 0, 0, 0, 0, 0};
  APN_HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_mlp_phase), zero, sizeof(zero)));
  APN_TRY(debug_phase_cycles_h3(out6));
  return debug_phase_cycles_h4(out6);
}
#endif  // APN_DEBUG_BUILD
