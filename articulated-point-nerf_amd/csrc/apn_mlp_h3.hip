// Fused Point-NeRF neighbour MLP (temporalpoints.py:452-519) on fp16 MFMA with a 3-term split:
// every fp32 operand x is carried as hi = fp16(x) (RNE) and lo = fp16(x - hi), and
//
//     a . b  ~=  hi(a) hi(b) + hi(a) lo(b) + lo(a) hi(b)        (fp32 accumulate)
//
// drops only lo(a) lo(b) (<= 2^-22 |a b|) and the fp16 rounding of the residual (<= 2^-22 |x|):
// ~2e-7 relative per product, the size of fp32's own rounding. v_mfma_f32_16x16x32_f16 runs
// 16x the FLOP rate of v_mfma_f32_16x16x4_f32, so the three terms cost 3/16 of the fp32 MFMA time.
// Range: |activations|, |weights| < 65504 (fp16 max). Guarded on the device: an activation or
// weight beyond it becomes inf/NaN in its hi half, and inf/NaN propagates through every later
// MFMA, ReLU and the IDW sum, so checking the IDW sums h (the last values split) catches all of
// them; the kernel then sets the range flag in wbuf and apn_point_mlp's FP32 MFMA launch redoes
// the samples (no host sync). The tests compare against the fp32 oracle.
//
// Same algebra as apn_mlp.hip (layer-1 projection P = canonical_feat W1f^T added to the
// accumulator, rgbnet feature_linears folded into views_linears.0); differences in structure:
//   * transposed product D^T[o][m] = W[o][k] X^T[k][m]: the weights are the MFMA A operand
//     (fragments pre-arranged by apn_mlp_split_weights, one coalesced 1 KB load per wave), the
//     activations the B operand, so a lane's accumulator holds 4 consecutive output features of
//     one MLP row -- the epilogue writes them as one 8-byte hi + one 8-byte lo LDS store;
//   * activations ping-pong between two LDS buffers (64 rows x [hi 128 | lo 128] halves, 16-B
//     chunks XOR-swizzled by row: conflict-free ds_read_b128 operand reads), one barrier per layer;
//   * the P rows are gathered straight into the layer-1 accumulators (global -> VGPR).
//
// Tile = 8 samples x 8 neighbours = 64 MLP rows per 256-thread workgroup (4 waves, wave w owns
// output features 32w..32w+31 of every layer), 3 workgroups per CU (APN_MLP_OCC=2: the ping-pong
// build at 2 per CU).
#include "apn_mlp_split.h"

namespace apn {
namespace h3 {

using namespace mlpx;

constexpr int XBUF = TR * XB;      // one activation buffer (32 KB)
constexpr int HB = 800;            // bytes per head-input row: hi 160 | lo 160 | pad (800/4 = 8 mod 64)
constexpr int HLO = 320;           // lo offset inside a head-input row

#ifndef APN_H3_ROWSTRIDE
#define APN_H3_ROWSTRIDE 9
#endif
// floats per MLP row of sRow (direct-blend terms: 8 used); 9 = odd stride, conflict-free columns
constexpr int RS = APN_H3_ROWSTRIDE;
#ifdef APN_H3_NO_HEADPF   // A/B: the head's fragments one chunk ahead inside the head loop
constexpr bool kHeadPF = false;
#else
constexpr bool kHeadPF = true;
#endif
#ifdef APN_H3_BPF   // A/B: B-operand activation fragments read one M-tile ahead in the OCC = 3 build
constexpr bool kBPF3 = true;
#else
constexpr bool kBPF3 = false;
#endif

constexpr int SW_B1 = 0, SW_B2 = 128, SW_B3 = 256, SW_B4 = 384, SW_WD = 512, SW_BD = 640, SW_BH = 644,
              SW_WV2 = 708, SW_BV2 = 900, SW_SC = 904, SW_DS = 912, SW_HSC = 921,
              SW_TOTAL = 924;

// acc[mt][j] += W[o-tile 2w+j] X^T over NQ chunks of 32. `a` carries chunk 0 of this matrix's
// fragments (block FB) in and chunk 0 of the next matrix (block FBN, NQN chunks, NTN o-tiles) out.
template <int NQ, int NQN, int NTN, int FB, int FBN, bool BPF = true>
__device__ __forceinline__ void layer_mfma(const char* __restrict__ X, rsrc_t rs, int vb, f32x4 (&acc)[4][2],
                                           h8 (&a)[2][2]) {
  const int lane = threadIdx.x & 63;
  const int li = lane & 15, g = lane >> 4;
#ifdef APN_H3_MT1
  if constexpr (!BPF) {
    // A/B: the activation fragments of the next M-tile (or of the next chunk's first M-tile) are
    // read before this M-tile's six MFMAs, so their LDS latency overlaps them (+8 VGPRs)
    h8 bh = *(const h8*)(X + act_off(li, g)), bl = *(const h8*)(X + act_off(li, g) + 256);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      h8 an[2][2];
      if (q + 1 < NQ) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int pt = 0; pt < 2; ++pt) an[j][pt] = frag(rs, vb, FB + (j * NQ + q + 1) * 2 + pt);
      } else {
#pragma unroll
        for (int j = 0; j < NTN; ++j)
#pragma unroll
          for (int pt = 0; pt < 2; ++pt) an[j][pt] = frag(rs, vb, FBN + j * NQN * 2 + pt);
      }
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        h8 nbh = bh, nbl = bl;
        if (mt + 1 < 4 || q + 1 < NQ) {
          const char* p = X + act_off(16 * ((mt + 1) & 3) + li, 4 * (mt + 1 < 4 ? q : q + 1) + g);
          nbh = *(const h8*)p;
          nbl = *(const h8*)(p + 256);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[mt][j] = mfma3(a[j][0], a[j][1], bh, bl, acc[mt][j]);
        bh = nbh;
        bl = nbl;
      }
      if (q + 1 < NQ) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          a[j][0] = an[j][0];
          a[j][1] = an[j][1];
        }
      } else {
#pragma unroll
        for (int j = 0; j < NTN; ++j) {
          a[j][0] = an[j][0];
          a[j][1] = an[j][1];
        }
      }
    }
    return;
  }
#endif
  if constexpr (!BPF) {
    // no B double-buffering (fewer VGPRs): the chunk's activation fragments are read per M-tile
    // right before its MFMAs
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      h8 an[2][2];
      if (q + 1 < NQ) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int pt = 0; pt < 2; ++pt) an[j][pt] = frag(rs, vb, FB + (j * NQ + q + 1) * 2 + pt);
      } else {
#pragma unroll
        for (int j = 0; j < NTN; ++j)
#pragma unroll
          for (int pt = 0; pt < 2; ++pt) an[j][pt] = frag(rs, vb, FBN + j * NQN * 2 + pt);
      }
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const char* p = X + act_off(16 * mt + li, 4 * q + g);
        const h8 bh = *(const h8*)p, bl = *(const h8*)(p + 256);
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[mt][j] = mfma3(a[j][0], a[j][1], bh, bl, acc[mt][j]);
      }
      if (q + 1 < NQ) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          a[j][0] = an[j][0];
          a[j][1] = an[j][1];
        }
      } else {
#pragma unroll
        for (int j = 0; j < NTN; ++j) {
          a[j][0] = an[j][0];
          a[j][1] = an[j][1];
        }
      }
    }
    return;
  }
  h8 b[4][2];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    const char* p = X + act_off(16 * mt + li, g);
    b[mt][0] = *(const h8*)p;
    b[mt][1] = *(const h8*)(p + 256);
  }
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    h8 an[2][2], bn[4][2];
    if (q + 1 < NQ) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int pt = 0; pt < 2; ++pt) an[j][pt] = frag(rs, vb, FB + (j * NQ + q + 1) * 2 + pt);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const char* p = X + act_off(16 * mt + li, 4 * (q + 1) + g);
        bn[mt][0] = *(const h8*)p;
        bn[mt][1] = *(const h8*)(p + 256);
      }
    } else {
#pragma unroll
      for (int j = 0; j < NTN; ++j)
#pragma unroll
        for (int pt = 0; pt < 2; ++pt) an[j][pt] = frag(rs, vb, FBN + j * NQN * 2 + pt);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) acc[mt][j] = mfma3(a[j][0], a[j][1], b[mt][0], b[mt][1], acc[mt][j]);
    __builtin_amdgcn_sched_barrier(0);
    if (q + 1 < NQ) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        a[j][0] = an[j][0];
        a[j][1] = an[j][1];
      }
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        b[mt][0] = bn[mt][0];
        b[mt][1] = bn[mt][1];
      }
    } else {
#pragma unroll
      for (int j = 0; j < NTN; ++j) {
        a[j][0] = an[j][0];
        a[j][1] = an[j][1];
      }
    }
  }
}

// Two-deep weight prefetch (the single-buffer OCC = 3 build): chunk q + 2's fragments are in flight
// while chunk q's MFMAs run -- the L2 latency of the 1-KB fragment loads is the MFMA phases' main
// wait (a probe with L1-resident weights ran 12 % faster), and the MFMA phases sit below the
// kernel's register peak (the gather), so the extra 16 VGPRs cost no occupancy. a0 / a1 carry
// chunks 0 / 1 of this matrix in (IN2 = false: chunk 1 is loaded here) and chunks 0 / 1 of the
// next matrix (block FBN, NQN chunks, NTN o-tiles) out (OUT2 = false: chunk 0 only).
#ifdef APN_H3_D2
constexpr bool kD2 = true;
#else
constexpr bool kD2 = false;   // measured: no gain over the one-deep prefetch (A/B builds only)
#endif
template <int NQ, int NQN, int NTN, int FB, int FBN, bool IN2, bool OUT2>
__device__ __forceinline__ void layer_mfma_d2(const char* __restrict__ X, rsrc_t rs, int vb, f32x4 (&acc)[4][2],
                                              h8 (&a0)[2][2], h8 (&a1)[2][2]) {
  static_assert(NQ >= 2, "two-deep prefetch needs two chunks");
  const int lane = threadIdx.x & 63;
  const int li = lane & 15, g = lane >> 4;
  if constexpr (!IN2) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int pt = 0; pt < 2; ++pt) a1[j][pt] = frag(rs, vb, FB + (j * NQ + 1) * 2 + pt);
  }
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    h8 an[2][2];
    if (q + 2 < NQ) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int pt = 0; pt < 2; ++pt) an[j][pt] = frag(rs, vb, FB + (j * NQ + q + 2) * 2 + pt);
    } else if (q + 2 == NQ || OUT2) {
      const int qn = q + 2 - NQ;   // chunk of the next matrix
#pragma unroll
      for (int j = 0; j < NTN; ++j)
#pragma unroll
        for (int pt = 0; pt < 2; ++pt) an[j][pt] = frag(rs, vb, FBN + (j * NQN + qn) * 2 + pt);
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const char* p = X + act_off(16 * mt + li, 4 * q + g);
      const h8 bh = *(const h8*)p, bl = *(const h8*)(p + 256);
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[mt][j] = mfma3(a0[j][0], a0[j][1], bh, bl, acc[mt][j]);
    }
    // rotate (only the o-tiles each chunk holds)
    const int nt1 = q + 1 < NQ ? 2 : NTN;   // a1 holds chunk q + 1 of this matrix or chunk 0 of the next
#pragma unroll
    for (int j = 0; j < 2; ++j)
      if (j < nt1) { a0[j][0] = a1[j][0]; a0[j][1] = a1[j][1]; }
    const int nt2 = q + 2 < NQ ? 2 : NTN;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      if (j < nt2 && (q + 2 <= NQ || OUT2)) { a1[j][0] = an[j][0]; a1[j][1] = an[j][1]; }
  }
}

// lrelu(acc [+ bias]) -> hi/lo halves of the next layer's input rows (transposed C layout: lane
// (li, g) of (mt, j) holds features 16(2w+j) + 4g + r of row 16 mt + li). Layers 2-4 start their
// accumulators from the bias (bias == nullptr here).

// Scaled weights (apn_mlp_layout.h OFF_SCALE): the accumulators hold 2^s (W x + b); `dsc` = 2^-s.
// Layer 1 adds its (unscaled) bias with one fma(acc, 2^-s, b) -- fma(a, 1, b) == a + b, so the
// unscaled mode is the plain sum; layers 2-4 (bias in the accumulator) multiply only when scaled
// (a wave-uniform branch).
__device__ __forceinline__ void store_act(char* __restrict__ X, int ot0, const float* __restrict__ bias,
                                          const f32x4 (&acc)[4][2], bool scaled, float dsc) {
  const int lane = threadIdx.x & 63;
  const int li = lane & 15, g = lane >> 4;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int o0 = 16 * (ot0 + j) + 4 * g;
    const f32x4 bb = bias ? *(const f32x4*)(bias + o0) : f32x4{0.f, 0.f, 0.f, 0.f};
    // chunk 4w + g holds o-tile 2w's features 4g..4g+3 then o-tile 2w+1's (apn_mlp_layout.h act_k_of)
    const int c = 2 * ot0 + g, sub = j * 8;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const f32x4 a = acc[mt][j];
      const f32x4 v = lrelu4(bias ? f32x4{fmaf(a[0], dsc, bb[0]), fmaf(a[1], dsc, bb[1]), fmaf(a[2], dsc, bb[2]),
                                          fmaf(a[3], dsc, bb[3])}
                                  : (scaled ? f32x4{a[0] * dsc, a[1] * dsc, a[2] * dsc, a[3] * dsc} : a));
      h4 hi, lo;
      split4(v, hi, lo);
      char* p = X + act_off(16 * mt + li, c) + sub;
      *(h4*)p = hi;
      *(h4*)(p + 256) = lo;
    }
  }
}

// Accumulators of a layer start from its bias (broadcast over the M-tiles): the bias add of the
// reference's x W^T + b costs no VALU (the first MFMA reads it as its C operand).
__device__ __forceinline__ void init_bias(f32x4 (&acc)[4][2], int ot0, const float* __restrict__ bias) {
  const int g = (threadIdx.x & 63) >> 4;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const f32x4 bb = *(const f32x4*)(bias + 16 * (ot0 + j) + 4 * g);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) acc[mt][j] = bb;
  }
}

__device__ unsigned long long g_phase[6];

// Gather of one tile: lane r of every wave owns MLP row r (sample r >> 3, neighbour r & 7), and
// wave p computes quarter p of the row's posenc columns -- the quarter is wave-uniform, so the
// argument indices, frequency scales and which-coordinate choices below are compile-time
// constants (one instantiation per wave) instead of per-lane selects. Split in two:
// ws_gather_load issues the neighbour-record and view-direction loads (a segment ahead),
// ws_gather writes the posenc hi/lo into PE (X layout, chunks 0..7) and the row records into
// sTo/sRow/sV.
struct GatherRegs {
  float4 a0, a1, a2, a3, b0, b1;
  float vv;
};

// Loads are unconditional (clamped indices; invalid rows read row 0 and are discarded later):
// a load under a divergent branch makes the compiler drain vmcnt(0) at the join, which would
// expose the latency of every load in flight.
__device__ __forceinline__ void ws_gather_load(int p, int nb, int ray, GatherRegs& G,
                                               const float4* __restrict__ recA, const float4* __restrict__ recB,
                                               const float* __restrict__ viewdirs,
                                               const float* __restrict__ vemb_const) {
  const int k = threadIdx.x & 7;
  const size_t n = (size_t)max(nb, 0);
#ifdef APN_H3_PROBE_NOREC   // timing probe only (wrong results): no neighbour-record loads
  G.a0 = make_float4(0.f, 0.f, 0.f, 1.f + (float)n);
  G.a1 = G.a2 = G.a3 = G.b0 = G.b1 = make_float4(0.01f, 0.f, 0.f, 0.f);
  G.vv = 0.f;
  return;
#endif
  G.a0 = recA[4 * n + 0];
  G.a1 = recA[4 * n + 1];
  G.a2 = recA[4 * n + 2];
  G.a3 = recA[4 * n + 3];
  G.b0 = recB[2 * n];
  G.b1 = recB[2 * n + 1];
  const int e = min(4 * k + p, 26);
  const int ee = e < 3 ? 0 : (e < 15 ? e - 3 : e - 15);
  G.vv = vemb_const ? 0.f : viewdirs[3 * (size_t)ray + (e < 3 ? e : ee >> 2)];
}

template <int P>
__device__ __forceinline__ void ws_gather_q(int nb, float4 q, const GatherRegs& G, char* __restrict__ PE,
                                            float* __restrict__ sTo, float* __restrict__ sRow,
                                            float* __restrict__ sV, const float* __restrict__ vemb_const) {
  // the lane index through an opaque asm: the per-lane LDS addresses below are then recomputed
  // in each tile (a few VALU) instead of hoisted out of the loop for all four quarter cases and
  // spilled to scratch (reloads that wait in vmcnt order behind the gather's loads)
  int r_ = threadIdx.x & 63;
  asm volatile("" : "+v"(r_));
  const int r = r_, s = r >> 3, k = r & 7;
  char* xr = PE + r * XB;
  const int c_sin = (2 * P) ^ (r & 15), c_cos = (2 * P + 1) ^ (r & 15);
  if (nb >= 0) {
    const float4 a0 = G.a0, a1 = G.a1, a2 = G.a2, a3 = G.a3;
    const float dx = q.x - a0.x, dy = q.y - a0.y, dz = q.z - a0.z;
    const float rc[3] = {(a1.x * dx + a1.y * dy) + a1.z * dz, (a1.w * dx + a2.x * dy) + a2.y * dz,
                         (a2.z * dx + a2.w * dy) + a3.x * dz};
    if constexpr (P == 0) {
      sTo[r] = (dx * dx + dy * dy) + dz * dz;
    } else if constexpr (P == 1) {
      const float tn = (dx * dx + dy * dy) + dz * dz;
      float* rw = sRow + RS * r;
      rw[0] = expf(-(tn * tn) / a0.w);   // temporalpoints.py:461 (to_nn is already squared)
      rw[1] = a3.y;
      rw[2] = G.b0.x; rw[3] = G.b0.y; rw[4] = G.b0.z;
      rw[5] = G.b1.x; rw[6] = G.b1.y; rw[7] = G.b1.z;
    }
    f32x4 sv0, sv1, cv0, cv1;   // arguments 8P .. 8P + 7 (apn_mlp_layout.h pe_col_to_ref)
    pe_chunk<8 * P>(rc, sv0, sv1, cv0, cv1);
    h4 hs0, ls0, hs1, ls1, hc0, lc0, hc1, lc1;
    split4(sv0, hs0, ls0); split4(sv1, hs1, ls1);
    split4(cv0, hc0, lc0); split4(cv1, hc1, lc1);
    *(h8*)(xr + (c_sin << 4)) = __builtin_shufflevector(hs0, hs1, 0, 1, 2, 3, 4, 5, 6, 7);
    *(h8*)(xr + (c_sin << 4) + 256) = __builtin_shufflevector(ls0, ls1, 0, 1, 2, 3, 4, 5, 6, 7);
    *(h8*)(xr + (c_cos << 4)) = __builtin_shufflevector(hc0, hc1, 0, 1, 2, 3, 4, 5, 6, 7);
    *(h8*)(xr + (c_cos << 4) + 256) = __builtin_shufflevector(lc0, lc1, 0, 1, 2, 3, 4, 5, 6, 7);
    const int e = 4 * k + P;   // view embedding element e of this sample
    float v = 0.f;
    if (e < 27) {
      if (vemb_const) {
        v = vemb_const[e];
      } else {
        const int ee = e < 3 ? 0 : (e < 15 ? e - 3 : e - 15);
        float sn_, cs_;
        sincos_pe(G.vv * (float)(1 << (ee & 3)), sn_, cs_);
        v = e < 3 ? G.vv : (e < 15 ? sn_ : cs_);
      }
    }
    sV[s * 32 + e] = v;
  } else {
    const h8 z = {0, 0, 0, 0, 0, 0, 0, 0};
    *(h8*)(xr + (c_sin << 4)) = z;
    *(h8*)(xr + (c_sin << 4) + 256) = z;
    *(h8*)(xr + (c_cos << 4)) = z;
    *(h8*)(xr + (c_cos << 4) + 256) = z;
    sV[s * 32 + 4 * k + P] = 0.f;
    if constexpr (P == 0) {
      sTo[r] = 1.f;
    } else if constexpr (P == 1) {
      for (int c = 0; c < 8; ++c) sRow[RS * r + c] = 0.f;
    }
  }
}

// Wave-uniform dispatch (p = the SGPR wave index).
__device__ __forceinline__ void ws_gather(int p, int nb, float4 q, const GatherRegs& G, char* __restrict__ PE,
                                          float* __restrict__ sTo, float* __restrict__ sRow, float* __restrict__ sV,
                                          const float* __restrict__ vemb_const) {
#ifdef APN_COUNT_ONE_QUARTER
  p = 0;
#endif
  switch (p) {
    case 0: ws_gather_q<0>(nb, q, G, PE, sTo, sRow, sV, vemb_const); break;
    case 1: ws_gather_q<1>(nb, q, G, PE, sTo, sRow, sV, vemb_const); break;
    case 2: ws_gather_q<2>(nb, q, G, PE, sTo, sRow, sV, vemb_const); break;
    default: ws_gather_q<3>(nb, q, G, PE, sTo, sRow, sV, vemb_const); break;
  }
}

// OCC = workgroups per CU: 2 = activations ping-pong between two LDS buffers (one barrier per
// layer); 3 = one activation buffer + a separate head-input buffer (45 KB of LDS, an extra barrier
// per layer, 12 waves per CU to hide the phases' latencies).
//
// SCALED: the weight-scale mode of wbuf (apn_mlp_layout.h OFF_SCALE), a block-uniform choice
// between two instantiations of the tile loop (the unscaled one carries no scale arithmetic).
template <bool TIMED, int OCC, bool SCALED>
__device__ __forceinline__ void mlp_tiles(
    const float4* __restrict__ s_pos, const int* __restrict__ s_ray, const int* __restrict__ s_nbr,
    const int* __restrict__ n_samples_dev, const float4* __restrict__ recA, const float4* __restrict__ recB,
    const float4* __restrict__ pproj, const float* __restrict__ viewdirs, const float* __restrict__ vemb_const,
    const float* __restrict__ wbuf, float eps, float shift, float interval, float4* __restrict__ out,
    char* const Xs, char* const Hs, float* const sTo, float* const sIdw, float* const sRow, float* const sOut,
    float* const sV, float* const sW, float* const sPart) {
  constexpr bool PP = OCC == 2;
  char* const X0 = Xs;
  char* const X1 = PP ? Xs + XBUF : Xs;
  char* const HX = PP ? X1 : Hs;     // head input rows

  const int nS = *n_samples_dev;
  const int ntiles = (nS + TS - 1) / TS;
  const int tid = threadIdx.x;
  // wave index as a wave-uniform (SGPR) value: the fragment offsets derived from it must be
  // scalar, or every buffer load becomes a readfirstlane waterfall loop
  const int lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, g = lane >> 4;
  // buffer resource over the fp16 fragments and the range flag right after them (written with a
  // buffer store: no extra 64-bit pointer live across the tile loop)
  const rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(wbuf + OFF_H16), 0, H_TOTAL * 2 + 4, 0x00020000);
  const int ot0 = 2 * wid;
  const int vb = (wid * FR_WAVE * FRAG_HALVES + lane * 8) * 2;   // this wave's fragment block + lane
  // per-matrix weight scales 2^s (W1E, W2, W3, W4, WH), kept in LDS with their inverses (exact:
  // powers of two) and read where used, so they hold no registers across the tile loop
  const float* const scp = wbuf + OFF_SCALE;
  for (int i = tid; i < 128; i += MLP_THREADS) {
    sW[SW_B1 + i] = wbuf[OFF_B1 + i];
    sW[SW_B2 + i] = SCALED ? wbuf[OFF_B2 + i] * scp[1] : wbuf[OFF_B2 + i];   // accumulator initial values: 2^s b
    sW[SW_B3 + i] = SCALED ? wbuf[OFF_B3 + i] * scp[2] : wbuf[OFF_B3 + i];
    sW[SW_B4 + i] = SCALED ? wbuf[OFF_B4 + i] * scp[3] : wbuf[OFF_B4 + i];
    sW[SW_WD + i] = wbuf[OFF_WD + i];
  }
  if (SCALED && tid < 6) {   // 0-3: W1E, W2, W3, W4; 4: WH h-columns (2^a); 5: WH view columns (2^b)
    sW[SW_SC + tid] = scp[tid];
    sW[SW_DS + tid] = 1.f / scp[tid];
  }
  if (SCALED && tid == 7) sW[SW_HSC] = scp[5] / scp[4];   // h' = h 2^(b-a): WH_h' h' = 2^b WH_h h
  if (tid < 64) sW[SW_BH + tid] = SCALED ? wbuf[OFF_BH + tid] * scp[5] : wbuf[OFF_BH + tid];
  if (tid < 192) sW[SW_WV2 + tid] = wbuf[OFF_WV2 + tid];
  if (tid < 3) sW[SW_BV2 + tid] = wbuf[OFF_BV2 + tid];
  if (tid == 0) sW[SW_BD] = wbuf[OFF_BD];
  if (SCALED) __syncthreads();   // the first tile reads the layer-1 scale before its first barrier
  // XCD-aware tile order (as apn_mlp.hip): XCD x = block % 8 walks a contiguous tile range, so
  // neighbouring samples (which share neighbour points) gather through the same L2.
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
  // next-tile prefetch (unconditional clamped loads, validity apart -- see ws_gather_load):
  // this thread's gather row (neighbour, sample position, ray) and the 4 rows whose P it loads
  int pf_nb = 0, pf_ray = 0, pf_pn[4];
  bool pf_ok = false, pf_pok[4];
  float4 pf_q = make_float4(0.f, 0.f, 0.f, 0.f);
  auto fetch = [&](int tl) {
    const int tc = min(tl, t_end - 1);
    const int gs = tc * TS + (lane >> 3);   // this lane's gather row: sample lane >> 3, neighbour lane & 7
    const int gc = min(gs, nS - 1);
    pf_ok = tl < t_end && gs < nS;
    pf_nb = s_nbr[(size_t)gc * 8 + (lane & 7)];
    pf_q = s_pos[gc];
    pf_ray = s_ray[gc];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const int m = 16 * mt + li;
      pf_pok[mt] = tl < t_end && tc * TS + (m >> 3) < nS;
      pf_pn[mt] = s_nbr[min((size_t)tc * TR + m, (size_t)nS * 8 - 1)];
    }
  };
  int tile = t_beg + blockIdx.x / nx;
  if (tile < t_end) fetch(tile);
  h8 a[2][2];    // carried A-fragment prefetch (chunk 0 of the next weight matrix)
  h8 a1[2][2];   // and chunk 1 (two-deep prefetch of the OCC = 3 build)
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int pt = 0; pt < 2; ++pt) a[j][pt] = frag(rs, vb, FR_W1E + j * 4 + pt);
  // layer-1 accumulators = P[nbr] (global -> VGPR; validity pok: rows past the last sample read
  // row 0, zeroed before layer 1)
  f32x4 acc[4][2];
  bool pok[4];
  auto load_p = [&](const int (&pn)[4], const bool (&pk)[4]) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      pok[mt] = pk[mt];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
#ifdef APN_H3_PROBE_NOP   // timing probe only (wrong results): no P-row gather
        const float4 v = make_float4(0.f, 0.f, 0.f, pn[mt] < 0 ? 1.f : 0.f);
#else
        const float4 v = pproj[(size_t)max(pn[mt], 0) * (FEAT / 4) + 4 * (ot0 + j) + g];
#endif
        acc[mt][j] = f32x4{v.x, v.y, v.z, v.w};
      }
    }
  };
  GatherRegs gregs;
  int prev_s0 = -1;
  bool range_bad = false;
  for (; tile < t_end; tile += per_xcd) {
    const int s0 = tile * TS;
    if (TIMED) { tk = clock64(); ph[4] += 1; }
    // ------------------------------------------------ loads: gather records first (consumed first),
    // then the layer-1 accumulators = P[nbr] (global -> VGPR), then the next tile's indices
    const int nb = pf_ok ? pf_nb : -1;
    const float4 q = pf_q;
    // loads in consumption order -- the gather's records, then the layer-1 accumulators = P[nbr],
    // then the next tile's indices. vmcnt is an in-order counter: a wait for a load also waits for
    // every load issued before it, so loads issued earlier (e.g. the next tile's P after layer 4,
    // measured +1.6 %) hold up the weight-fragment waits in between.
    ws_gather_load(wid, nb, pf_ray, gregs, recA, recB, viewdirs, vemb_const);
    int pn_tile[4];   // this tile's P-row indices (fetch below overwrites pf_pn with the next tile's)
    bool pok_tile[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) { pn_tile[mt] = pf_pn[mt]; pok_tile[mt] = pf_pok[mt]; }
    fetch(tile + per_xcd);
    // ------------------------------------------------ gather + posenc + direct-blend terms
    ws_gather(wid, nb, q, gregs, X0, sTo, sRow, sV, vemb_const);
    // layer-1 accumulators = P[nbr] (global -> VGPR), loaded after the gather's register peak:
    // held across it they pushed the kernel past its 168-VGPR budget (20 VGPRs spilled, their
    // reloads waiting in vmcnt order behind the gather's loads); measured 7.28 -> 6.92 ms
    load_p(pn_tile, pok_tile);
    if (SCALED) {   // layer-1 accumulators in the W1E scale: 2^s1 P
      const float sc1 = sW[SW_SC];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[mt][j] = acc[mt][j] * sc1;
    }
    __syncthreads();
    APN_PHASE(0)
    // ------------------------------------------------ outputs of the previous tile
    if (prev_s0 >= 0 && tid < TS * 3 && prev_s0 + tid / 3 < nS)
      out[(size_t)prev_s0 * 3 + tid] = *(const float4*)(sOut + 4 * tid);
    if (tid < TS) {  // IDW weights (temporalpoints.py:473-475)
      float w[8], sum = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        w[k] = __builtin_amdgcn_rcpf(sTo[tid * 8 + k] + eps);   // v_rcp_f32 (1 ulp)
        sum += w[k];
      }
      const float inv = __builtin_amdgcn_rcpf(sum);
#pragma unroll
      for (int k = 0; k < 8; ++k) sIdw[tid * 8 + k] = w[k] * inv;
    }
    if (s0 + TS > nS) {   // the last tile only (block-uniform): rows past the last sample loaded P rows of point 0
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          if (!pok[mt]) acc[mt][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    // ------------------------------------------------ feat_net: 4 x (Linear + LeakyReLU)
    if constexpr (PP || !kD2) layer_mfma<2, 4, 2, FR_W1E, FR_W2, PP || kBPF3>(X0, rs, vb, acc, a);
    else layer_mfma_d2<2, 4, 2, FR_W1E, FR_W2, false, true>(X0, rs, vb, acc, a, a1);
    if (!PP) __syncthreads();
    store_act(X1, ot0, nullptr, acc, SCALED, SCALED ? sW[SW_DS + 0] : 1.f);   // b1: the bias column
    __syncthreads();
    APN_PHASE(1)
    init_bias(acc, ot0, sW + SW_B2);
    if constexpr (PP || !kD2) layer_mfma<4, 4, 2, FR_W2, FR_W3, PP || kBPF3>(X1, rs, vb, acc, a);
    else layer_mfma_d2<4, 4, 2, FR_W2, FR_W3, true, true>(X1, rs, vb, acc, a, a1);
    if (!PP) __syncthreads();
    store_act(X0, ot0, nullptr, acc, SCALED, SCALED ? sW[SW_DS + 1] : 1.f);
    __syncthreads();
    init_bias(acc, ot0, sW + SW_B3);
    if constexpr (PP || !kD2) layer_mfma<4, 4, 2, FR_W3, FR_W4, PP || kBPF3>(X0, rs, vb, acc, a);
    else layer_mfma_d2<4, 4, 2, FR_W3, FR_W4, true, true>(X0, rs, vb, acc, a, a1);
    if (!PP) __syncthreads();
    store_act(X1, ot0, nullptr, acc, SCALED, SCALED ? sW[SW_DS + 2] : 1.f);
    __syncthreads();
    init_bias(acc, ot0, sW + SW_B4);
    if constexpr (PP || !kD2) layer_mfma<4, 5, 1, FR_W4, FR_WH, PP || kBPF3>(X1, rs, vb, acc, a);
    else layer_mfma_d2<4, 5, 1, FR_W4, FR_WH, true, true>(X1, rs, vb, acc, a, a1);
    if (!PP) __syncthreads();
    // layer-4 output lrelu(acc) (bias in the accumulator) as fp32 rows (for the IDW sum)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int o0 = 16 * (ot0 + j) + 4 * g;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
        *(f32x4*)(X0 + out32_off(16 * mt + li, o0 >> 2)) =
            lrelu4(SCALED ? acc[mt][j] * sW[SW_DS + 3] : acc[mt][j]);
    }
    // the head's remaining fragment chunks (1..4; chunk 0 came with layer 4) are issued here, a
    // whole IDW phase ahead of their MFMAs: in the head loop each chunk has only 3 MFMAs, so a
    // one-deep prefetch there waits out one L2 latency per chunk (the accumulators are dead now)
    constexpr bool kHeadEarly = !PP && !kD2 && kHeadPF;
    h8 hfr[KV / 32 - 1][2];
    if constexpr (kHeadEarly) {
#pragma unroll
      for (int q = 1; q < KV / 32; ++q)
#pragma unroll
        for (int pt = 0; pt < 2; ++pt) hfr[q - 1][pt] = frag(rs, vb, FR_WH + q * 2 + pt);
    }

    __syncthreads();
    APN_PHASE(2)
    // ------------------------------------------------ IDW sum (temporalpoints.py:493-494), density head
    {
      const int s = tid >> 5, oq = tid & 31;
      f32x4 h = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const f32x4 v = *(const f32x4*)(X0 + out32_off(8 * s + k, oq));
        const float w = sIdw[8 * s + k];
#pragma unroll
        for (int r = 0; r < 4; ++r) h[r] = fmaf(w, v[r], h[r]);
      }
      // densitynet Linear(128 -> 1) (tineuvox.py:158) over this thread's 4 features, then the half-wave
      const f32x4 wd = *(const f32x4*)(sW + SW_WD + 4 * oq);
      float d = ((h[0] * wd[0] + h[1] * wd[1]) + h[2] * wd[2]) + h[3] * wd[3];
      // the head's h input in the head's column scale (scaled mode): h' = h 2^(b-a), exact
      if (SCALED) h = h * sW[SW_HSC];
      // range guard (see the header comment) on the last values split: false for NaN too. The
      // flag store waits for the end of the tile loop (a store under a divergent branch inside the
      // loop makes every later vmcnt wait conservative)
#ifndef APN_H3_AB_NO_GUARD   // A/B builds only (tools/ab_build.sh): the guard's cost
      range_bad |= !(fmaxf(fmaxf(fabsf(h[0]), fabsf(h[1])), fmaxf(fabsf(h[2]), fabsf(h[3]))) <= H3_RANGE);
#endif
      d += __shfl_xor(d, 16, 64);
      d += __shfl_xor(d, 8, 64);
      d += __shfl_xor(d, 4, 64);
      d += __shfl_xor(d, 2, 64);
      d += __shfl_xor(d, 1, 64);
      if (oq == 0) {  // Raw2Alpha (render_utils_kernel.cu:357-369)
        // (1 + e)^-interval as exp2(-interval log2(1 + e)) on v_log_f32 / v_exp_f32 (1 ulp each; the
        // alpha error stays below 1e-7 absolute: |y| 2^-|y| <= 0.53 scales the exponent's error)
        const float e = expf((d + sW[SW_BD]) + shift);
        sOut[12 * s + 3] = 1.f - __builtin_amdgcn_exp2f(-interval * __builtin_amdgcn_logf(1.f + e));
      }
      // head input row s: [h (128) | view embedding (27) | 0] as hi/lo halves
      char* hr = HX + s * HB;
      h4 hi, lo;
      split4(h, hi, lo);
      *(h4*)(hr + 8 * oq) = hi;
      *(h4*)(hr + HLO + 8 * oq) = lo;
      const float ve = sV[s * 32 + oq];
      const _Float16 vh = (_Float16)ve;
      *(_Float16*)(hr + 2 * (128 + oq)) = vh;
      *(_Float16*)(hr + HLO + 2 * (128 + oq)) = (_Float16)(ve - (float)vh);
    }
    // direct blend + weight-vis colour (temporalpoints.py:459-470, 517-519): wave 1, lane =
    // (sample, quantity); sums over the 8 neighbours in order
    if (wid == 1) {
      const int s = lane >> 3, qn = lane & 7;
      const float* rw = sRow + 8 * RS * s;
      float sumd = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) sumd += rw[RS * k];
      const float idn = __builtin_amdgcn_rcpf(sumd + 1e-12f);
      float acc1 = 0.f;
      if (qn == 0) {
#pragma unroll
        for (int k = 0; k < 8; ++k) acc1 += (0.125f * rw[RS * k]) * rw[RS * k + 1];
      } else if (qn < 4) {
#pragma unroll
        for (int k = 0; k < 8; ++k) acc1 += (rw[RS * k] * idn) * rw[RS * k + 1 + qn];
      } else if (qn < 7) {
#pragma unroll
        for (int k = 0; k < 8; ++k) acc1 += sIdw[8 * s + k] * rw[RS * k + 1 + qn];
      }
      // sOut[s] = {r, g, b, alpha, r_d, g_d, b_d, alpha_d, wr, wg, wb, 0}
      const int slot = qn == 0 ? 7 : (qn < 4 ? 3 + qn : (qn < 7 ? 4 + qn : 11));
      sOut[12 * s + slot] = acc1;
    }
    __syncthreads();
    // ------------------------------------------------ rgb head: folded [h; v] -> 64, ReLU, -> 3, sigmoid
    {
      const int o0 = 16 * wid + 4 * g;
      f32x4 ah = *(const f32x4*)(sW + SW_BH + o0);   // views_linears.0 (folded) bias
      // B columns 8..15 of the 16-wide MFMA tile repeat rows 0..7: their outputs are never read
      // (each output column depends on its own B column only), so no zero fill or select
      const char* hr = HX + (li & (TS - 1)) * HB;
      if constexpr (kHeadEarly) {
        // the next tile's W1E chunk 0 first (it is carried across the gather), then 5 chunks of
        // MFMAs on fragments already in registers
        h8 an[2][2];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int pt = 0; pt < 2; ++pt) an[j][pt] = frag(rs, vb, FR_W1E + j * 4 + pt);
#pragma unroll
        for (int q = 0; q < KV / 32; ++q) {
          const h8 bh = *(const h8*)(hr + 16 * (4 * q + g));
          const h8 bl = *(const h8*)(hr + HLO + 16 * (4 * q + g));
          ah = q == 0 ? mfma3(a[0][0], a[0][1], bh, bl, ah) : mfma3(hfr[q - 1][0], hfr[q - 1][1], bh, bl, ah);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          a[j][0] = an[j][0];
          a[j][1] = an[j][1];
        }
      } else if constexpr (PP || !kD2) {
#pragma unroll
        for (int q = 0; q < KV / 32; ++q) {
          h8 an[2][2];
          if (q + 1 < KV / 32) {
#pragma unroll
            for (int pt = 0; pt < 2; ++pt) an[0][pt] = frag(rs, vb, FR_WH + (q + 1) * 2 + pt);
          } else {  // chunk 0 of the next tile's layer 1
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
              for (int pt = 0; pt < 2; ++pt) an[j][pt] = frag(rs, vb, FR_W1E + j * 4 + pt);
          }
          const h8 bh = *(const h8*)(hr + 16 * (4 * q + g));
          const h8 bl = *(const h8*)(hr + HLO + 16 * (4 * q + g));
          ah = mfma3(a[0][0], a[0][1], bh, bl, ah);
          if (q + 1 < KV / 32) {
            a[0][0] = an[0][0];
            a[0][1] = an[0][1];
          } else {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              a[j][0] = an[j][0];
              a[j][1] = an[j][1];
            }
          }
        }
      } else {
        // two-deep: a / a1 hold head chunks 0 / 1 (layer 4 carried them); chunk q + 2 in flight; the
        // next tile's W1E chunk 0 is the last prefetch (one deep across the gather, the register peak)
        constexpr int NQH = KV / 32;
#pragma unroll
        for (int q = 0; q < NQH; ++q) {
          h8 an[2][2];
          if (q + 2 < NQH) {
#pragma unroll
            for (int pt = 0; pt < 2; ++pt) an[0][pt] = frag(rs, vb, FR_WH + (q + 2) * 2 + pt);
          } else if (q + 2 == NQH) {
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
              for (int pt = 0; pt < 2; ++pt) an[j][pt] = frag(rs, vb, FR_W1E + j * 4 + pt);
          }
          const h8 bh = *(const h8*)(hr + 16 * (4 * q + g));
          const h8 bl = *(const h8*)(hr + HLO + 16 * (4 * q + g));
          ah = mfma3(a[0][0], a[0][1], bh, bl, ah);
          // rotate: a <- a1 (chunk q + 1, or the W1E chunk 0 with both o-tiles), a1 <- an
          if (q + 2 <= NQH) {
            const int nt1 = q + 1 < NQH ? 1 : 2;
#pragma unroll
            for (int j = 0; j < 2; ++j)
              if (j < nt1) { a[j][0] = a1[j][0]; a[j][1] = a1[j][1]; }
            const int nt2 = q + 2 < NQH ? 1 : 2;
#pragma unroll
            for (int j = 0; j < 2; ++j)
              if (j < nt2) { a1[j][0] = an[j][0]; a1[j][1] = an[j][1]; }
          } else {   // q = NQH - 1: a1 holds the W1E chunk 0
#pragma unroll
            for (int j = 0; j < 2; ++j) { a[j][0] = a1[j][0]; a[j][1] = a1[j][1]; }
          }
        }
      }
      // lane (li = sample, g): head features o = 16 wid + 4 g + r
      float pc[3] = {0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = fmaxf(SCALED ? ah[r] * sW[SW_DS + 5] : ah[r], 0.f);
#pragma unroll
        for (int c = 0; c < 3; ++c) pc[c] += v * sW[SW_WV2 + 64 * c + o0 + r];
      }
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        pc[c] += __shfl_xor(pc[c], 16, 64);
        pc[c] += __shfl_xor(pc[c], 32, 64);
      }
      if (g == 0 && li < TS) {
#pragma unroll
        for (int c = 0; c < 3; ++c) sPart[(wid * TS + li) * 4 + c] = pc[c];
      }
    }
    __syncthreads();
    if (tid < TS * 3) {  // views_linears.2 bias + sigmoid (temporalpoints.py:513-515)
      const int s = tid / 3, c = tid % 3;
      const float v = ((sPart[(0 * TS + s) * 4 + c] + sPart[(1 * TS + s) * 4 + c]) + sPart[(2 * TS + s) * 4 + c]) +
                      sPart[(3 * TS + s) * 4 + c];
      sOut[12 * s + c] = 1.f / (1.f + expf(-(v + sW[SW_BV2 + c])));
    }
    APN_PHASE(3)
    prev_s0 = s0;
  }
#undef APN_PHASE
  if (TIMED && tid == 0) {
    ph[5] = clock64() - tk0;
    for (int i = 0; i < 6; ++i) atomicAdd(&g_phase[i], ph[i]);
  }
  __syncthreads();
  if (prev_s0 >= 0 && tid < TS * 3 && prev_s0 + tid / 3 < nS)
    out[(size_t)prev_s0 * 3 + tid] = *(const float4*)(sOut + 4 * tid);
  if (range_bad) __builtin_amdgcn_raw_buffer_store_b32(1, rs, 0, H_TOTAL * 2, 0);   // the range flag (OFF_FLAG)
}

// One instantiation per weight-scale mode (separate register allocation); apn_point_mlp launches
// both and the one that does not match wbuf's mode exits at once (a launch with the range flag
// already set -- these weights overflowed before -- leaves every sample to the FP32 kernel).
// Block-uniform decisions: one read each, broadcast through LDS.
template <bool TIMED, int OCC, bool SCALED>
__global__ __launch_bounds__(MLP_THREADS, OCC) void k_point_mlp_h3(
    const float4* __restrict__ s_pos, const int* __restrict__ s_ray, const int* __restrict__ s_nbr,
    const int* __restrict__ n_samples_dev, const float4* __restrict__ recA, const float4* __restrict__ recB,
    const float4* __restrict__ pproj, const float* __restrict__ viewdirs, const float* __restrict__ vemb_const,
    const float* __restrict__ wbuf, float eps, float shift, float interval, float4* __restrict__ out) {
  constexpr bool PP = OCC == 2;
  __shared__ __attribute__((aligned(16))) char Xs[PP ? 2 * XBUF : XBUF];
  __shared__ __attribute__((aligned(16))) char Hs[PP ? 16 : TS * HB];
  __shared__ float sTo[TR];
  __shared__ float sIdw[TR];
  __shared__ float sRow[TR * RS];    // direct blend per row: wdir, alpha_c, rgb_c(3), pcol(3)
  __shared__ __attribute__((aligned(16))) float sOut[TS * 12];
  __shared__ float sV[TS * 32];      // view embedding per sample (27 + zero pad)
  __shared__ __attribute__((aligned(16))) float sW[SW_TOTAL];
  __shared__ float sPart[4 * TS * 4];
#ifndef APN_H3_AB_NO_GUARD
  __shared__ int s_skip;
  if (threadIdx.x == 0)
    s_skip = __builtin_nontemporal_load((const int*)(wbuf + OFF_FLAG)) != 0 ||
             (wbuf[OFF_SCALE + 6] != 0.f) != SCALED;
  __syncthreads();
  if (s_skip) return;
#else
  if (SCALED) return;
#endif
  mlp_tiles<TIMED, OCC, SCALED>(s_pos, s_ray, s_nbr, n_samples_dev, recA, recB, pproj, viewdirs, vemb_const, wbuf,
                                eps, shift, interval, out, Xs, Hs, sTo, sIdw, sRow, sOut, sV, sW, sPart);
}

// Per-group scales (apn_mlp_layout.h OFF_SCALE) from max|w| of W1E, W2, W3, W4 and the two
// column groups of the folded head WH (h columns 0..127, view columns 128..159 -- their
// magnitudes are unrelated: feature_linears is folded into the first group only): one
// workgroup, one pass over the fp32 region (67 584 weights).
__global__ __launch_bounds__(256) void k_weight_scales(float* __restrict__ wbuf) {
  constexpr int NG = 6;
  __shared__ float red[NG][256];
  const int tid = threadIdx.x;
#pragma unroll
  for (int m = 0; m < NG; ++m) red[m][tid] = 0.f;
  for (int i = tid; i < 128 * KE; i += 256) red[0][tid] = fmaxf(red[0][tid], fabsf(wbuf[OFF_W1E + i]));
  if (tid < 128) red[0][tid] = fmaxf(red[0][tid], fabsf(wbuf[OFF_B1 + tid]));   // the bias column
  for (int i = tid; i < 128 * 128; i += 256) {
    red[1][tid] = fmaxf(red[1][tid], fabsf(wbuf[OFF_W2 + i]));
    red[2][tid] = fmaxf(red[2][tid], fabsf(wbuf[OFF_W3 + i]));
    red[3][tid] = fmaxf(red[3][tid], fabsf(wbuf[OFF_W4 + i]));
  }
  for (int i = tid; i < 64 * KV; i += 256) {
    const int g = (i % KV) < 128 ? 4 : 5;
    red[g][tid] = fmaxf(red[g][tid], fabsf(wbuf[OFF_WH + i]));
  }
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (tid < w)
#pragma unroll
      for (int m = 0; m < NG; ++m) red[m][tid] = fmaxf(red[m][tid], red[m][tid + w]);
    __syncthreads();
  }
  if (tid == 0) {
    bool scaled = false;
    float mx[NG];
#pragma unroll
    for (int m = 0; m < NG; ++m) {
      mx[m] = red[m][0];
      // all-zero (or non-finite: left to the range guard) groups keep scale 1
      if (mx[m] > 0.f && mx[m] <= 3.0e38f && (mx[m] < SCALE_LO || mx[m] > SCALE_HI)) scaled = true;
    }
    // the folded head is scaled as one matrix (both column groups share the accumulator): its
    // max over both groups; the groups only decide whether scaling is needed at all
    mx[4] = mx[5] = fmaxf(mx[4], mx[5]);
#pragma unroll
    for (int m = 0; m < NG; ++m) {
      float sc = 1.f;
      if (scaled && mx[m] > 0.f && mx[m] <= 3.0e38f) {
        int e;
        frexpf(mx[m], &e);                        // mx = f 2^e, f in [0.5, 1)
        sc = ldexpf(1.f, SCALE_TARGET_EXP - e);   // mx * sc in [2^12, 2^13)
      }
      wbuf[OFF_SCALE + m] = sc;
    }
    wbuf[OFF_SCALE + 6] = scaled ? 1.f : 0.f;
    wbuf[OFF_SCALE + 7] = 0.f;
  }
}

// fp32 region of wbuf -> fp16 hi/lo fragments of w * 2^s (layout: apn_mlp_layout.h). One thread
// per (matrix, o-tile, chunk, lane).
__global__ void k_split_weights(float* __restrict__ wbuf) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t == 0) *(int*)(wbuf + OFF_FLAG) = 0;   // new weights: clear the range flag
  // fragment-lanes per matrix: W1E 8x2x64, W2..W4 8x4x64, WH 4x5x64
  constexpr int n1 = 8 * 2 * 64, n2 = 8 * 4 * 64, nh = 4 * 5 * 64;
  int mat, i;
  if (t < n1) { mat = 0; i = t; }
  else if (t < n1 + 3 * n2) { mat = 1 + (t - n1) / n2; i = (t - n1) % n2; }
  else if (t < n1 + 3 * n2 + nh) { mat = 4; i = t - n1 - 3 * n2; }
  else return;
  const int nq = mat == 0 ? 2 : (mat == 4 ? 5 : 4);
  const int lane = i & 63, q = (i >> 6) % nq, ot = (i >> 6) / nq;
  const int o = 16 * ot + (lane & 15), k0 = 32 * q + 8 * (lane >> 4);
  // wave-major block (apn_mlp_layout.h): W1E..W4 o-tile ot -> wave ot / 2, j = ot & 1; head -> wave ot
  const int fb = mat == 0 ? FR_W1E : (mat == 1 ? FR_W2 : (mat == 2 ? FR_W3 : (mat == 3 ? FR_W4 : FR_WH)));
  const int wave = mat == 4 ? ot : ot >> 1, j16 = mat == 4 ? 0 : ot & 1;
  const int fidx = wave * FR_WAVE + fb + (j16 * nq + q) * 2;
  _Float16* dst = (_Float16*)(wbuf + OFF_H16) + (size_t)fidx * FRAG_HALVES + lane * 8;
  const float sc_mat = wbuf[OFF_SCALE + mat], sc_view = wbuf[OFF_SCALE + 5];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = k0 + j;
    float w;
    if (mat == 0) {
      const int ref = pe_col_to_ref(k);
      w = ref == PE_BIAS ? wbuf[OFF_B1 + o] : (ref < 0 ? 0.f : wbuf[OFF_W1E + o * KE + ref]);
    } else if (mat == 4) {
      w = wbuf[OFF_WH + o * KV + k];
    } else {   // hidden activations in the kernels' K order (apn_mlp_layout.h act_k_of)
      const int off = mat == 1 ? OFF_W2 : (mat == 2 ? OFF_W3 : OFF_W4);
      w = wbuf[off + o * 128 + act_k_of(k)];
    }
    w *= (mat == 4 && k >= 128) ? sc_view : sc_mat;   // exact (powers of two)
    const _Float16 hi = (_Float16)w;
    dst[j] = hi;
    dst[FRAG_HALVES + j] = (_Float16)(w - (float)hi);
  }
}

// The bias column of W1E (apn_mlp_layout.h PE_BIAS, column 63 = k-chunk 1, lane group 3, half 7)
// from the fp32 b1 -- after a per-frame pose-embedding fold of b1 (ops.fold_pose_bias). A value
// beyond the fp16 range sets the range flag (the frame's MLP then runs on FP32 MFMA).
__global__ void k_split_bias(float* __restrict__ wbuf) {
  const int o = threadIdx.x;
  if (o >= 128) return;
  const float w = wbuf[OFF_B1 + o] * wbuf[OFF_SCALE + 0];
  const int ot = o >> 4, lane = (o & 15) + 48;
  const int fidx = (ot >> 1) * FR_WAVE + FR_W1E + ((ot & 1) * 2 + 1) * 2;
  _Float16* dst = (_Float16*)(wbuf + OFF_H16) + (size_t)fidx * FRAG_HALVES + lane * 8 + 7;
  const _Float16 hi = (_Float16)w;
  dst[0] = hi;
  dst[FRAG_HALVES] = (_Float16)(w - (float)hi);
  if (!(fabsf(w) <= H3_RANGE)) *(int*)(wbuf + OFF_FLAG) = 1;
}

}  // namespace h3

void launch_point_mlp_h3(int blocks, bool timed, hipStream_t stream, const float4* s_pos, const int* s_ray,
                         const int* s_nbr, const int* n_samples_dev, const float4* recA, const float4* recB,
                         const float4* pproj, const float* viewdirs, const float* vemb_const, const float* wbuf,
                         float eps, float shift, float interval, float4* out) {
  auto go = [&](auto kern, int nb) {
    hipLaunchKernelGGL(kern, dim3(nb), dim3(MLP_THREADS), 0, stream, s_pos, s_ray, s_nbr, n_samples_dev, recA, recB,
                       pproj, viewdirs, vemb_const, wbuf, eps, shift, interval, out);
  };
  // the scaled-weights instantiation runs on a smaller grid (a rare mode: weight magnitudes outside
  // [2^-5, 2^12]); when it does not match, its 8 workgroups per CU exit at once
  const int nb_scaled = blocks < 256 * 8 ? blocks : 256 * 8;
#ifdef APN_DEBUG_BUILD
  // debug build: the phase-timed kernels (APN_MLP_VARIANT=3) and the ping-pong build at 2
  // workgroups per CU (APN_MLP_OCC=2)
  static const int occ = [] {
    const char* e = apn_env("APN_MLP_OCC");
    return e ? atoi(e) : 3;
  }();
  if (occ == 3) {
    if (timed) { go(h3::k_point_mlp_h3<true, 3, false>, blocks); go(h3::k_point_mlp_h3<true, 3, true>, nb_scaled); }
    else { go(h3::k_point_mlp_h3<false, 3, false>, blocks); go(h3::k_point_mlp_h3<false, 3, true>, nb_scaled); }
  } else {
    if (timed) { go(h3::k_point_mlp_h3<true, 2, false>, blocks); go(h3::k_point_mlp_h3<true, 2, true>, nb_scaled); }
    else { go(h3::k_point_mlp_h3<false, 2, false>, blocks); go(h3::k_point_mlp_h3<false, 2, true>, nb_scaled); }
  }
#else
  (void)timed;
  go(h3::k_point_mlp_h3<false, 3, false>, blocks);
  go(h3::k_point_mlp_h3<false, 3, true>, nb_scaled);
#endif
}

int debug_phase_cycles_h3(uint64_t* out6) {
  uint64_t v[6];
  APN_HIP_TRY(hipMemcpyFromSymbol(v, HIP_SYMBOL(h3::g_phase), sizeof(v)));
  static const unsigned long long zero[6] = {0, 0, 0, 0, 0, 0};
  APN_HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(h3::g_phase), zero, sizeof(zero)));
  for (int i = 0; i < 6; ++i) out6[i] += v[i];
  return APN_OK;
}

}  // namespace apn

using namespace apn;

// fp32 packed weights -> the fp16 hi/lo fragment region read by the default apn_point_mlp kernel.
extern "C" int apn_mlp_split_weights(float* wbuf, void* stream) {
  if (!wbuf) return APN_ERR_ARG;
  constexpr int n = 8 * 2 * 64 + 3 * 8 * 4 * 64 + 4 * 5 * 64;
  hipLaunchKernelGGL(h3::k_weight_scales, dim3(1), dim3(256), 0, (hipStream_t)stream, wbuf);
  hipLaunchKernelGGL(h3::k_split_weights, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, wbuf);
  return launch_status();
}

extern "C" int apn_mlp_split_bias(float* wbuf, void* stream) {
  if (!wbuf) return APN_ERR_ARG;
  hipLaunchKernelGGL(h3::k_split_bias, dim3(1), dim3(128), 0, (hipStream_t)stream, wbuf);
  return launch_status();
}
