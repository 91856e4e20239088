// Fused Point-NeRF neighbour MLP (temporalpoints.py:452-519) on fp16 MFMA with the 3-term split
// (hi*hi + hi*lo + lo*hi, fp32 accumulate; apn_mlp_h3.hip's header explains the arithmetic and the
// range guard), on 128-row tiles: 16 samples x 8 neighbours per 256-thread workgroup, 2 workgroups
// per CU.
//
// Why 128 rows (apn_mlp_h3.hip runs 64): every wave streams its 66 weight fragments (66 KB: o-tiles
// 2w, 2w+1 of layers 1-4, o-tile w of the head) from L2 once per tile, so the L2 -> L1 weight
// stream per MLP row halves (~68 GB per C2 frame at 64 rows), and each fragment load now feeds 48
// MFMAs instead of 24 -- its L2 latency hides behind one chunk of MFMAs. The head's 16-wide MFMA
// B tile holds 16 real samples (no padding). Cost: 2 workgroups (8 waves) per CU instead of 3.
//
// Layout per workgroup (LDS, 74.6 KB): one activation buffer X of 128 rows x [hi 128 | lo 128] fp16
// (512 B rows, 16-B chunks XOR-swizzled by row: conflict-free ds_read_b128 operand reads), reused
// in place by every layer (a barrier between the last read and the first write), then for the
// layer-4 output as fp32 rows, then -- after the IDW sums are in registers -- for the 16 head-input
// rows. Activations are written as whole 16-B chunks with no cross-lane exchange: a lane holds 4
// features of each of its wave's two o-tiles for one row (the transposed product's C layout) and
// writes those 8 values as one hi and one lo chunk; W2-W4's fragments take their K columns in that
// order (apn_mlp_layout.h act_k_of). (Rounds 4-5 paired lanes with v_permlane16_swap for the same
// conflict-free ds_write_b128s.)
#include "apn_mlp_split.h"

// The layers' operand reads are pinned ahead of the MFMAs that do not need them (sched_barrier):
// left to the scheduler, each M-tile's activation reads sank below the previous M-tile's MFMAs into
// the registers those had just read, so every 6-MFMA step waited on its LDS read behind an s_nop
// hazard pad (685 pad states per wave-tile, 450 pinned): MLP 4.22 -> 3.94 ms per C2 frame.
#ifndef APN_H4_MERGED   // A/B builds: 0 launches the two weight-scale instantiations per pass
#define APN_H4_MERGED 1
#endif
#ifndef APN_H4_PIN   // A/B builds: 0 leaves the activation / fragment reads to the scheduler
#define APN_H4_PIN 1
#endif
// A/B builds: 1 requests the next tile's neighbour records in this tile's epilogue (after the
// head's weight fragments, which the head waits for first: vmcnt is in order), so the gather at the
// top of the next tile finds them in registers. Measured slower (round 6, same box, interleaved:
// MLP kernel 3.156-3.169 vs 3.084-3.092 ms per C2 frame; 227 vs 221 VGPRs): off.
#ifndef APN_H4_RECPF
#define APN_H4_RECPF 0
#endif
// A/B builds: workgroups of the second dispatch round (blockIdx 256..511: the second workgroup on
// each CU) start APN_H4_STAGGER x 127 x 64 cycles late, so the two workgroups of a CU -- whose
// waves share each SIMD -- do not run their gather / epilogue phases at the same time. Measured
// slower (round 6, same box: MLP kernel 3.08-3.11 -> 3.23-3.27 ms at 3, 3.40 ms at 6): off.
#ifndef APN_H4_STAGGER
#define APN_H4_STAGGER 0
#endif
// 1: the layer-1 P-row indices of the next tile come from LDS -- its gather rows' neighbour
// indices, which the gather threads fetch anyway (row m's P row is row m's neighbour) -- instead of
// 16 global loads (list + s_nbr per M-tile) and their address arithmetic per lane and tile.
#ifndef APN_H4_LDSPN
#define APN_H4_LDSPN 1
#endif
// 1: weight fragments two K-chunks ahead of their MFMAs (a second carried register set, across the
// layer boundaries and the head) instead of one: 194 -> 210 VGPRs (still 2 waves per SIMD). Same box,
// interleaved (round 6): MLP kernel 3.048 / 3.009 -> 3.003 / 2.984 ms per C2 frame, parity green.
#ifndef APN_H4_PF2
#define APN_H4_PF2 1
#endif
// 1: wave priority 1 while a wave runs a layer's MFMAs, 0 elsewhere (s_setprio): of the two waves of
// a SIMD (one per workgroup), the one in its MFMA phase issues first and the other's gather /
// epilogue VALU fills the cycles an MFMA leaves free. Same box, against two-deep fragments alone:
// 2.946 / 2.931 -> 2.902 / 2.928 ms (frame in flight equal, one at a time 5.85 -> 5.81 ms).
#ifndef APN_H4_PRIO
#define APN_H4_PRIO 1
#endif
// 1: layer 1's P rows requested before the gather instead of after it (their latency under the
// gather's VALU, the accumulators live through it; 210 -> 215 VGPRs, no spill). Same box, against
// PF2 + PRIO: MLP kernel 2.907 / 2.877 -> 2.859 / 2.856 ms per C2 frame (frac 0.57); phase split
// (debug build, full MLP) layer 1 14.9 -> 13.7 %, gather 17.6 -> 18.5 %, tile 41.8k -> 41.5k cycles.
#ifndef APN_H4_PEARLY
#define APN_H4_PEARLY 1
#endif
// APN_H4_IDWG (apn_mlp_layout.h): the IDW weights made in the gather.
// 1: head-input row s written inside the X rows that its own wave's IDW sum read (wave w sums
// samples 4w .. 4w + 3 over rows 32w .. 32w + 31, 16 KB), so no barrier between the IDW reads and
// the head-row writes (a wave's LDS accesses stay in program order); rows 832 B apart and shifted
// 16 B per wave so the head's 16 B-column reads (one row per lane) hit 16 distinct bank groups.
// Measured equal to slightly slower (round 6, same box, parity green: 2.981 / 2.948 -> 2.985 /
// 3.003 ms per C2 frame): the barrier's cost is the waves' skew there, which is small. Off.
#ifndef APN_H4_HEADW
#define APN_H4_HEADW 0
#endif
// 1 (early-termination passes' kernel): the next tile's posenc -- rel_c, the 16 sin / cos
// arguments, their hi / lo split -- computed inside this tile's layer-4 MFMA stream (its VALU
// scheduled into the MFMAs' issue gaps by sched_group_barrier instead of the phase-pinning fences)
// and held in 33 VGPRs until the next tile's gather stores them; the next tile's records are
// requested at the start of layer 3. Needs two-deep fragments off (255 VGPRs). Measured slower
// (round 6, same box, parity green: MLP kernel 2.883 / 2.888 -> 2.967 / 2.979 ms per C2 frame; the
// interleave itself compiled as asked, one VALU per MFMA gap): off.
#ifndef APN_H4_PEFILL
#define APN_H4_PEFILL 0
#endif

namespace apn {
namespace t128 {

using namespace mlpx;

constexpr int TS4 = 16;            // samples per tile
constexpr int TR4 = TS4 * 8;       // MLP rows per tile
constexpr int MT = TR4 / 16;       // 16-row M-tiles
constexpr int HB = 800;            // bytes per head-input row: hi 160 | lo 160 | pad (800/4 = 8 mod 64)
constexpr int HLO = 320;           // lo offset inside a head-input row
// byte offset of head-input row s (APN_H4_HEADW: inside wave s / 4's IDW rows)
__device__ __forceinline__ int head_row(int s) {
  return APN_H4_HEADW ? (s >> 2) * (32 * XB) + (s & 3) * 832 + (s >> 2) * 16 : s * HB;
}
constexpr int RS = 9;              // floats per row of sRow (8 used; odd stride: conflict-free columns)
static_assert(TS4 * HB <= TR4 * XB, "head rows alias the activation buffer");
static_assert(3 * 832 + 3 * 16 + HB <= 32 * XB, "a wave's head rows stay inside its IDW rows");

constexpr int SW_B1 = 0, SW_B2 = 128, SW_B3 = 256, SW_B4 = 384, SW_WD = 512, SW_BD = 640, SW_BH = 644,
              SW_WV2 = 708, SW_BV2 = 900, SW_SC = 904, SW_DS = 912, SW_HSC = 921, SW_TOTAL = 924;

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Neighbour records of this thread's gather row. The posenc work of a tile is split by rows and
// argument halves: thread t owns row r = t & 127 (sample r >> 3, neighbour r & 7) and half
// h = t >> 7 (wave-uniform) of its arguments -- chunk pairs 2h, 2h + 1, i.e. arguments 16h ..
// 16h + 15 (apn_mlp_layout.h pe_col_to_ref) -- so each row's records are read by two threads and
// its rel_c computed twice (the 4-way quarter split before this read and computed them four times),
// and consecutive frequencies of one coordinate meet in one thread (pe_chunk's double-angle steps).
struct GatherRegs {
  float4 a0, a1, a2, a3, b0, b1;
  float v0;   // the viewdir component of this thread's view-embedding job (vemb_job)
};

// The view embedding poc_fre(viewdirs, 2^0..3) of a sample (tineuvox.py:872-878: [v (3),
// sin(v_c 2^f) at 3 + 4c + f (12), cos(v_c 2^f) at 15 + 4c + f (12)]) is made by the sample's 16
// gather threads, thread ts = 2k + h: ts < 12 computes one sincos (c = ts / 4, f = ts % 4) and
// writes both its sine and its cosine slot; ts 12-14 copy the raw component ts - 12 and clear slot
// 15 + ts; ts 15 clears slots 30, 31 (the head's K padding).
__device__ __forceinline__ int vemb_comp(int ts) { return ts < 12 ? ts >> 2 : (ts < 15 ? ts - 12 : 0); }

// Loads are unconditional (clamped indices; invalid rows read row 0 and are discarded later): a
// load under a divergent branch makes the compiler drain vmcnt(0) at the join. recB (direct-blend
// colours) only where the direct blend is computed here (not in the early-termination passes).
template <bool DIRECT>
__device__ __forceinline__ void gather_load(int h, int k, int nb, int ray, GatherRegs& G,
                                            const float4* __restrict__ recA, const float4* __restrict__ recB,
                                            const float* __restrict__ viewdirs, const float* __restrict__ vemb_const) {
  const size_t n = (size_t)max(nb, 0);
  G.a0 = recA[4 * n + 0];
  G.a1 = recA[4 * n + 1];
  G.a2 = recA[4 * n + 2];
  G.a3 = recA[4 * n + 3];
  if (DIRECT) {
    G.b0 = recB[2 * n];
    G.b1 = recB[2 * n + 1];
  }
  G.v0 = vemb_const ? 0.f : viewdirs[3 * (size_t)ray + vemb_comp(2 * k + h)];
}

// A row's posenc chunks 4H .. 4H + 3 (chunk pairs 2H, 2H + 1: sin, cos) as hi / lo halves, and its
// squared distance, made ahead of the gather that stores them (APN_H4_PEFILL).
struct PeRegs {
  h8 hi[4], lo[4];
  float tn;
};

__device__ __forceinline__ void rel_c_of(float4 q, const GatherRegs& G, float (&rc)[3], float& tn) {
  const float4 a0 = G.a0, a1 = G.a1, a2 = G.a2, a3 = G.a3;
  const float dx = q.x - a0.x, dy = q.y - a0.y, dz = q.z - a0.z;
  // rel_c = Rinv (x - p) (temporalpoints.py:454-458)
  rc[0] = (a1.x * dx + a1.y * dy) + a1.z * dz;
  rc[1] = (a1.w * dx + a2.x * dy) + a2.y * dz;
  rc[2] = (a2.z * dx + a2.w * dy) + a3.x * dz;
  tn = (dx * dx + dy * dy) + dz * dz;
}

template <int H>
__device__ __forceinline__ void pe_compute(float4 q, const GatherRegs& G, PeRegs& P) {
  float rc[3];
  rel_c_of(q, G, rc, P.tn);
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    f32x4 sv0, sv1, cv0, cv1;
    if (u == 0)
      pe_chunk<16 * H>(rc, sv0, sv1, cv0, cv1);
    else
      pe_chunk<16 * H + 8>(rc, sv0, sv1, cv0, cv1);
    h4 hs0, ls0, hs1, ls1, hc0, lc0, hc1, lc1;
    split4(sv0, hs0, ls0); split4(sv1, hs1, ls1);
    split4(cv0, hc0, lc0); split4(cv1, hc1, lc1);
    P.hi[2 * u] = __builtin_shufflevector(hs0, hs1, 0, 1, 2, 3, 4, 5, 6, 7);
    P.lo[2 * u] = __builtin_shufflevector(ls0, ls1, 0, 1, 2, 3, 4, 5, 6, 7);
    P.hi[2 * u + 1] = __builtin_shufflevector(hc0, hc1, 0, 1, 2, 3, 4, 5, 6, 7);
    P.lo[2 * u + 1] = __builtin_shufflevector(lc0, lc1, 0, 1, 2, 3, 4, 5, 6, 7);
  }
}

// One chunk pair (arguments 8p .. 8p + 7) of row r: sines and cosines split into hi / lo halves and
// stored as whole 16-B chunks at their swizzled positions.
template <int PAIR>
__device__ __forceinline__ void pe_store(char* __restrict__ xr, int r, const float (&rc)[3]) {
  f32x4 sv0, sv1, cv0, cv1;
  pe_chunk<8 * PAIR>(rc, sv0, sv1, cv0, cv1);
  h4 hs0, ls0, hs1, ls1, hc0, lc0, hc1, lc1;
  split4(sv0, hs0, ls0); split4(sv1, hs1, ls1);
  split4(cv0, hc0, lc0); split4(cv1, hc1, lc1);
  const int c_sin = (2 * PAIR) ^ (r & 15), c_cos = (2 * PAIR + 1) ^ (r & 15);
  *(h8*)(xr + (c_sin << 4)) = __builtin_shufflevector(hs0, hs1, 0, 1, 2, 3, 4, 5, 6, 7);
  *(h8*)(xr + (c_sin << 4) + 256) = __builtin_shufflevector(ls0, ls1, 0, 1, 2, 3, 4, 5, 6, 7);
  *(h8*)(xr + (c_cos << 4)) = __builtin_shufflevector(hc0, hc1, 0, 1, 2, 3, 4, 5, 6, 7);
  *(h8*)(xr + (c_cos << 4) + 256) = __builtin_shufflevector(lc0, lc1, 0, 1, 2, 3, 4, 5, 6, 7);
}

// Row r = t & 127 of the tile, argument half H (= wave >> 1, a compile-time constant): the posenc
// chunk pairs 2H, 2H + 1, and -- half 0 -- the row's squared distance (sTo) or -- half 1 -- the
// direct-blend terms (sRow); the sample's view-embedding job ts = 2k + H (sV).
template <int H, bool DIRECT, bool FILL>
__device__ __forceinline__ void gather_q(int nb, float4 q, const GatherRegs& G, char* __restrict__ PE,
                                         float* __restrict__ sTo, float* __restrict__ sRow, float* __restrict__ sV,
                                         const float* __restrict__ vemb_const, float* __restrict__ sIdw, float eps,
                                         const PeRegs& P) {
  int r_ = threadIdx.x & 127;
  asm volatile("" : "+v"(r_));   // per-lane LDS addresses recomputed per tile, not hoisted and spilled
  const int r = r_, s = r >> 3, k = r & 7;
  char* xr = PE + r * XB;
  const int ts = 2 * k + H;
  float* const sv = sV + s * 32;
  float tn0 = 1.f;   // the row's squared distance (rows past the launch's end: 1)
  if (nb >= 0) {
    if constexpr (FILL) {   // the posenc made during the previous tile's layer 4
      static_assert(!DIRECT, "the fill path serves the early-termination passes");
      if constexpr (H == 0) {
        tn0 = P.tn;
        if (!APN_H4_IDWG) sTo[r] = tn0;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int c = (4 * H + u) ^ (r & 15);
        *(h8*)(xr + (c << 4)) = P.hi[u];
        *(h8*)(xr + (c << 4) + 256) = P.lo[u];
      }
    } else {
      float rc[3], tn;
      rel_c_of(q, G, rc, tn);
      if constexpr (H == 0) {
        tn0 = tn;
        if (!APN_H4_IDWG) sTo[r] = tn0;
      } else if constexpr (DIRECT) {
        float* rw = sRow + RS * r;
        rw[0] = expf(-(tn * tn) / G.a0.w);   // temporalpoints.py:461 (to_nn is already squared)
        rw[1] = G.a3.y;
        rw[2] = G.b0.x; rw[3] = G.b0.y; rw[4] = G.b0.z;
        rw[5] = G.b1.x; rw[6] = G.b1.y; rw[7] = G.b1.z;
      }
      pe_store<2 * H>(xr, r, rc);
      pe_store<2 * H + 1>(xr, r, rc);
    }
    if (ts < 12) {
      const int c = ts >> 2, f = ts & 3;
      float sn_, cs_;
      if (vemb_const) {
        sn_ = vemb_const[3 + 4 * c + f];
        cs_ = vemb_const[15 + 4 * c + f];
      } else {
        sincos_pe(G.v0 * (float)(1 << f), sn_, cs_);
      }
      sv[3 + 4 * c + f] = sn_;
      sv[15 + 4 * c + f] = cs_;
    } else if (ts < 15) {
      sv[ts - 12] = vemb_const ? vemb_const[ts - 12] : G.v0;
      sv[15 + ts] = 0.f;
    } else {
      sv[30] = 0.f;
      sv[31] = 0.f;
    }
  } else {
    const h8 z = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int c = 4 * H; c < 4 * H + 4; ++c) {
      *(h8*)(xr + ((c ^ (r & 15)) << 4)) = z;
      *(h8*)(xr + ((c ^ (r & 15)) << 4) + 256) = z;
    }
    sv[ts] = 0.f;        // the sample is past the launch's end: its 32 slots, two per thread
    sv[ts + 16] = 0.f;
    if constexpr (H == 0) {
      if (!APN_H4_IDWG) sTo[r] = 1.f;
    } else if constexpr (DIRECT) {
      for (int c = 0; c < 8; ++c) sRow[RS * r + c] = 0.f;
    }
  }
  if constexpr (H == 0 && APN_H4_IDWG) {   // outside the branch: every lane takes part in the shuffles
    const float w = __builtin_amdgcn_rcpf(tn0 + eps);   // v_rcp_f32 (1 ulp)
    float sum = w + __shfl_xor(w, 1, 64);
    sum += __shfl_xor(sum, 2, 64);
    sum += __shfl_xor(sum, 4, 64);
    sIdw[r] = w * __builtin_amdgcn_rcpf(sum);
  }
}

template <bool DIRECT, bool FILL>
__device__ __forceinline__ void gather(int h, int nb, float4 q, const GatherRegs& G, char* __restrict__ PE,
                                       float* __restrict__ sTo, float* __restrict__ sRow, float* __restrict__ sV,
                                       const float* __restrict__ vemb_const, float* __restrict__ sIdw, float eps,
                                       const PeRegs& P) {
  if (h == 0)
    gather_q<0, DIRECT, FILL>(nb, q, G, PE, sTo, sRow, sV, vemb_const, sIdw, eps, P);
  else
    gather_q<1, DIRECT, FILL>(nb, q, G, PE, sTo, sRow, sV, vemb_const, sIdw, eps, P);
}

// acc[mt][j] += W[o-tile 2w+j] X^T over NQ chunks of 32 and the tile's 8 M-tiles. `a` carries chunk
// 0 of this matrix's fragments (block FB) in and chunk 0 of the next matrix (block FBN, NQN chunks,
// NTN o-tiles) out: each chunk's fragments are requested a whole chunk (48 MFMAs) before use. The
// activation (B) fragments roll one M-tile ahead of their 6 MFMAs.
struct NoFill {
  __device__ void operator()() const {}
};

// FILL: `fill` (VALU work of its own) runs inside the layer's scheduling region and is spread over
// the MFMA issue gaps (sched_group_barrier) in place of the phase-pinning fences.
template <int NQ, int NQN, int NTN, int FB, int FBN, bool FILL = false, class F = NoFill>
__device__ __forceinline__ void layer_mfma(const char* __restrict__ X, rsrc_t rs, int vb, f32x4 (&acc)[MT][2],
                                           h8 (&a)[2][2], h8 (&a1)[2][2], F fill = F()) {
  const int lane = threadIdx.x & 63;
  const int li = lane & 15, g = lane >> 4;
  constexpr int NS = NQ * MT;   // (chunk, M-tile) steps
  constexpr int AHEAD = APN_H4_PF2 ? 2 : 1;   // K-chunks between a fragment load and its MFMAs
  // activation fragments of step t: (chunk t / MT, M-tile t % MT)
  auto act = [&](int t) { return X + act_off(16 * (t % MT) + li, 4 * (t / MT) + g); };
  h8 bh = *(const h8*)act(0), bl = *(const h8*)(act(0) + 256);
  if (APN_H4_PRIO) __builtin_amdgcn_s_setprio(1);
  fill();
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    h8 an[2][2];
    const int qn = q + AHEAD;   // the chunk whose fragments are requested now
    if (qn < NQ) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int pt = 0; pt < 2; ++pt) an[j][pt] = frag(rs, vb, FB + (j * NQ + qn) * 2 + pt);
    } else {   // the next matrix's chunk qn - NQ
#pragma unroll
      for (int j = 0; j < NTN; ++j)
#pragma unroll
        for (int pt = 0; pt < 2; ++pt) an[j][pt] = frag(rs, vb, FBN + (j * NQN + qn - NQ) * 2 + pt);
    }
#if APN_H4_PIN
    if (!FILL)
    __builtin_amdgcn_sched_barrier(0);   // the fragment loads issue here, before the MFMAs
#endif
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int t = q * MT + mt;
      h8 nbh = bh, nbl = bl;
      if (t + 1 < NS) {
        nbh = *(const h8*)act(t + 1);
        nbl = *(const h8*)(act(t + 1) + 256);
      }
#if APN_H4_PIN
      // the next M-tile's activation reads issue before this M-tile's MFMAs, into registers of their
      // own: no MFMA-read -> LDS-write hazard pad (s_nop) and the LDS latency under 6 MFMAs
      if (!FILL) __builtin_amdgcn_sched_barrier(0);
#endif
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[mt][j] = mfma3(a[j][0], a[j][1], bh, bl, acc[mt][j]);
#if APN_H4_PIN
      if (!FILL) __builtin_amdgcn_sched_barrier(0);
#endif
      bh = nbh;
      bl = nbl;
    }
    // rotate the carried sets: a <- a1 <- an (AHEAD 1: a <- an)
    const int nt_next = (q + 1 < NQ) ? 2 : NTN;   // o-tiles of the chunk a now receives
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (j < nt_next) {
        if (APN_H4_PF2) { a[j][0] = a1[j][0]; a[j][1] = a1[j][1]; }
        else { a[j][0] = an[j][0]; a[j][1] = an[j][1]; }
      }
      if (APN_H4_PF2 && j < (qn < NQ ? 2 : NTN)) { a1[j][0] = an[j][0]; a1[j][1] = an[j][1]; }
    }
  }
  if (FILL) {
    // the region's other VALU (the next tile's posenc, pe_compute) one instruction per MFMA issue
    // gap, each step's two activation reads ahead of its MFMAs
#pragma unroll
    for (int t = 0; t < NS; ++t) {
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);   // DS read
#pragma unroll
      for (int m = 0; m < 6; ++m) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);   // VALU
      }
    }
  }
  if (APN_H4_PRIO) __builtin_amdgcn_s_setprio(0);
}

// lrelu(acc [+ bias]) -> the next layer's input rows. Lane (li, g) of M-tile mt holds features
// 16 (2w + j) + 4g + r (j = 0, 1; r = 0..3) of row 16 mt + li: its 8 values are stored as one 16-B
// chunk of hi halves and one of lo halves, chunk 4w + g (the K order of apn_mlp_layout.h act_k_of,
// which W2..W4's fragments follow) -- no cross-lane exchange. `bias` (layer 1: the unscaled b1
// added as fma(acc, 2^-s, b)) or nullptr (layers 2-4: bias in the accumulator; scaled: times 2^-s).
__device__ __forceinline__ void store_act(char* __restrict__ X, int ot0, const float* __restrict__ bias,
                                          const f32x4 (&acc)[MT][2], bool scaled, float dsc) {
  const int lane = threadIdx.x & 63;
  const int li = lane & 15, g = lane >> 4;
  const int c = 2 * ot0 + g;
  f32x4 bb[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
    bb[j] = bias ? *(const f32x4*)(bias + 16 * (ot0 + j) + 4 * g) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    h4 hi[2], lo[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const f32x4 a = acc[mt][j];
      const f32x4 v = lrelu4(bias ? f32x4{fmaf(a[0], dsc, bb[j][0]), fmaf(a[1], dsc, bb[j][1]),
                                          fmaf(a[2], dsc, bb[j][2]), fmaf(a[3], dsc, bb[j][3])}
                                  : (scaled ? f32x4{a[0] * dsc, a[1] * dsc, a[2] * dsc, a[3] * dsc} : a));
      split4(v, hi[j], lo[j]);
    }
    char* p = X + act_off(16 * mt + li, c);
    *(h8*)p = __builtin_shufflevector(hi[0], hi[1], 0, 1, 2, 3, 4, 5, 6, 7);
    *(h8*)(p + 256) = __builtin_shufflevector(lo[0], lo[1], 0, 1, 2, 3, 4, 5, 6, 7);
  }
}

__device__ __forceinline__ void init_bias(f32x4 (&acc)[MT][2], int ot0, const float* __restrict__ bias) {
  const int g = (threadIdx.x & 63) >> 4;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const f32x4 bb = *(const f32x4*)(bias + 16 * (ot0 + j) + 4 * g);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[mt][j] = bb;
  }
}

// Phase cycle sums of the timed build (debug library, APN_MLP_VARIANT=5): {gather + loads,
// layer 1, layers 2-4, epilogue, tiles, whole kernel} over workgroups (wave 0's clock).
__device__ unsigned long long g_phase4[6];

// LISTED: the tile slots are the entries of ``list`` (sample indices, n_samples_dev entries) -- an
// early-ray-termination pass (apn_ert.hip) -- and only the Point-NeRF columns {rgb, alpha} of each
// sample are written (the direct-blend and weight-colour columns come from k_direct_blend).
template <bool SCALED, bool TIMED, bool LISTED>
__device__ __forceinline__ void mlp_tiles(
    const float4* __restrict__ s_pos, const int* __restrict__ s_ray, const int* __restrict__ s_nbr,
    const int* __restrict__ list, const int* __restrict__ n_samples_dev, const float4* __restrict__ recA, const float4* __restrict__ recB,
    const float4* __restrict__ pproj, const float* __restrict__ viewdirs, const float* __restrict__ vemb_const,
    const float* __restrict__ wbuf, float eps, float shift, float interval, float4* __restrict__ out,
    char* const X, float* const sTo, float* const sIdw, float* const sRow, float* const sOut, float* const sV,
    float* const sW, float* const sPart, int* const sNb) {
  const int nS = *n_samples_dev;
  const int ntiles = (nS + TS4 - 1) / TS4;
  // XCD-aware tile order: XCD x = block % 8 walks a contiguous tile range, so neighbouring samples
  // (which share neighbour points) gather through the same L2
  const int nx = (gridDim.x % 8 == 0) ? 8 : 1;
  const int xcd = blockIdx.x % nx, per_xcd = gridDim.x / nx;
  const int chunk = (ntiles + nx - 1) / nx;
  const int t_beg = xcd * chunk, t_end = min(ntiles, t_beg + chunk);
  // a workgroup without tiles (an early-termination pass that found no live rays, or more
  // workgroups than tiles) leaves before staging the weights (workgroup-uniform: no barrier yet)
  if (t_beg + (int)blockIdx.x / nx >= t_end) return;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, g = lane >> 4;
  const rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(wbuf + OFF_H16), 0, H_TOTAL * 2 + 4, 0x00020000);
  const int ot0 = 2 * wid;
  const int vb = (wid * FR_WAVE * FRAG_HALVES + lane * 8) * 2;
  const float* const scp = wbuf + OFF_SCALE;
  for (int i = tid; i < 128; i += MLP_THREADS) {
    sW[SW_B1 + i] = wbuf[OFF_B1 + i];
    sW[SW_B2 + i] = SCALED ? wbuf[OFF_B2 + i] * scp[1] : wbuf[OFF_B2 + i];
    sW[SW_B3 + i] = SCALED ? wbuf[OFF_B3 + i] * scp[2] : wbuf[OFF_B3 + i];
    sW[SW_B4 + i] = SCALED ? wbuf[OFF_B4 + i] * scp[3] : wbuf[OFF_B4 + i];
    sW[SW_WD + i] = wbuf[OFF_WD + i];
  }
  if (SCALED && tid < 6) {
    sW[SW_SC + tid] = scp[tid];
    sW[SW_DS + tid] = 1.f / scp[tid];
  }
  if (SCALED && tid == 7) sW[SW_HSC] = scp[5] / scp[4];
  if (tid < 64) sW[SW_BH + tid] = SCALED ? wbuf[OFF_BH + tid] * scp[5] : wbuf[OFF_BH + tid];
  if (tid < 192) sW[SW_WV2 + tid] = wbuf[OFF_WV2 + tid];
  if (tid < 3) sW[SW_BV2 + tid] = wbuf[OFF_BV2 + tid];
  if (tid == 0) sW[SW_BD] = wbuf[OFF_BD];
  if (SCALED) __syncthreads();

  // next-tile prefetch (unconditional clamped loads): this thread's gather row (tid & 127:
  // neighbour lane & 7 of sample (tid & 127) >> 3) and its 8 P rows
  const int gh = wid >> 1;   // the thread's posenc argument half (wave-uniform)
  int pf_nb, pf_ray, pf_pn[MT];
  bool pf_ok, pf_pok[MT];
  float4 pf_q;
  auto fetch = [&](int tl) {
    const int tc = min(tl, t_end - 1);
    {
      const int gs = tc * TS4 + ((tid & 127) >> 3);
      const int gc = min(gs, nS - 1);
      const int si = LISTED ? list[gc] : gc;
      pf_ok = tl < t_end && gs < nS;
      pf_nb = s_nbr[(size_t)si * 8 + (lane & 7)];
      pf_q = s_pos[si];
      pf_ray = s_ray[si];
    }
    if (!APN_H4_LDSPN) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int m = 16 * mt + li;
        pf_pok[mt] = tl < t_end && tc * TS4 + (m >> 3) < nS;
        if (LISTED)
          pf_pn[mt] = s_nbr[(size_t)list[min(tc * TS4 + (m >> 3), nS - 1)] * 8 + (m & 7)];
        else
          pf_pn[mt] = s_nbr[min((size_t)tc * TR4 + m, (size_t)nS * 8 - 1)];
      }
    }
  };
  int tile = t_beg + blockIdx.x / nx;
  if (APN_H4_STAGGER > 0 && ((blockIdx.x >> 8) & 1))
    for (int i = 0; i < APN_H4_STAGGER; ++i) __builtin_amdgcn_s_sleep(127);
  if (tile < t_end) fetch(tile);
  if (APN_H4_LDSPN) {   // the first tile's rows' neighbours (invalid rows: -1)
    if (tid < TR4) sNb[tid] = pf_ok ? pf_nb : -1;
    __syncthreads();
  }
  GatherRegs gn;   // the records of the tile about to be gathered (APN_H4_RECPF)
  if (APN_H4_RECPF && tile < t_end)
    gather_load<!LISTED>(gh, lane & 7, pf_ok ? pf_nb : -1, pf_ray, gn, recA, recB, viewdirs, vemb_const);
  constexpr bool FILL = APN_H4_PEFILL && LISTED;
  GatherRegs gx;   // FILL: the next tile's records, then its posenc (made during layer 4)
  PeRegs pe;
  if (FILL && tile < t_end) {   // the first tile's posenc
    gather_load<false>(gh, lane & 7, pf_ok ? pf_nb : -1, pf_ray, gx, recA, recB, viewdirs, vemb_const);
    if (gh == 0)
      pe_compute<0>(pf_q, gx, pe);
    else
      pe_compute<1>(pf_q, gx, pe);
  }
  h8 a[2][2], a1[2][2];   // carried A-fragment prefetch (chunks 0 [, 1] of the next weight matrix)
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int pt = 0; pt < 2; ++pt) {
      a[j][pt] = frag(rs, vb, FR_W1E + j * 4 + pt);
      a1[j][pt] = APN_H4_PF2 ? frag(rs, vb, FR_W1E + j * 4 + 2 + pt) : a[j][pt];
    }
  f32x4 acc[MT][2];
  bool pok[MT];
  int prev_s0 = -1;
  bool range_bad = false;
  unsigned long long ph[6] = {0, 0, 0, 0, 0, 0}, tk = 0, tk0 = 0;
  if (TIMED) tk0 = clock64();
#define APN_PHASE(i)                          \
  if (TIMED) {                                \
    const unsigned long long now = clock64(); \
    ph[i] += now - tk;                        \
    tk = now;                                 \
  }
  for (; tile < t_end; tile += per_xcd) {
    const int s0 = tile * TS4;
    if (TIMED) { tk = clock64(); ph[4] += 1; }
    // ------------------------------------------------ loads: the gather's records, then the next
    // tile's indices (vmcnt is in order: what is consumed first is issued first)
    const int nb0 = pf_ok ? pf_nb : -1;
    const float4 q0 = pf_q;
    GatherRegs g0;
    if (FILL)
      g0 = gx;   // its view component (the posenc is in pe)
    else if (APN_H4_RECPF)
      g0 = gn;
    else
      gather_load<!LISTED>(gh, lane & 7, nb0, pf_ray, g0, recA, recB, viewdirs, vemb_const);
    int pn_tile[MT];
    bool pok_tile[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      if (APN_H4_LDSPN) {   // row 16 mt + li's neighbour = its P row (written last tile, barriers since)
        pn_tile[mt] = sNb[16 * mt + li];
        pok_tile[mt] = pn_tile[mt] >= 0;
      } else {
        pn_tile[mt] = pf_pn[mt];
        pok_tile[mt] = pf_pok[mt];
      }
    }
    fetch(tile + per_xcd);
    // layer-1 accumulators = P[nbr] (global -> VGPR): before the gather (PEARLY), or after the
    // gather's register peak
    auto load_p = [&]() {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        pok[mt] = pok_tile[mt];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const float4 v = pproj[(size_t)max(pn_tile[mt], 0) * (FEAT / 4) + 4 * (ot0 + j) + g];
          acc[mt][j] = f32x4{v.x, v.y, v.z, v.w};
        }
      }
    };
    if (APN_H4_PEARLY) {
      load_p();
      __builtin_amdgcn_sched_barrier(0);   // issued here, not sunk into the gather
    }
    // ------------------------------------------------ gather + posenc + direct-blend terms
    gather<!LISTED, FILL>(gh, nb0, q0, g0, X, sTo, sRow, sV, vemb_const, sIdw, eps, pe);
    if (!APN_H4_PEARLY) load_p();
    if (SCALED) {
      const float sc1 = sW[SW_SC];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[mt][j] = acc[mt][j] * sc1;
    }
    __syncthreads();
    APN_PHASE(0)
    // ------------------------------------------------ outputs of the previous tile, IDW weights
    if (LISTED) {
      if (prev_s0 >= 0 && tid < TS4 && prev_s0 + tid < nS)
        out[(size_t)list[prev_s0 + tid] * 3] = *(const float4*)(sOut + 12 * tid);
    } else if (prev_s0 >= 0 && tid < TS4 * 3 && prev_s0 + tid / 3 < nS) {
      out[(size_t)prev_s0 * 3 + tid] = *(const float4*)(sOut + 4 * tid);
    }
    if (!APN_H4_IDWG && tid < TS4) {  // IDW weights (temporalpoints.py:473-475)
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
    if (s0 + TS4 > nS) {   // the last tile only: rows past the last sample loaded P rows of point 0
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          if (!pok[mt]) acc[mt][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    // ------------------------------------------------ feat_net: 4 x (Linear + LeakyReLU)
    layer_mfma<2, 4, 2, FR_W1E, FR_W2>(X, rs, vb, acc, a, a1);
    __syncthreads();
    store_act(X, ot0, nullptr, acc, SCALED, SCALED ? sW[SW_DS + 0] : 1.f);   // b1: the bias column
    __syncthreads();
    APN_PHASE(1)
    init_bias(acc, ot0, sW + SW_B2);
    layer_mfma<4, 4, 2, FR_W2, FR_W3>(X, rs, vb, acc, a, a1);
    __syncthreads();
    store_act(X, ot0, nullptr, acc, SCALED, SCALED ? sW[SW_DS + 1] : 1.f);
    __syncthreads();
    init_bias(acc, ot0, sW + SW_B3);
    if (FILL)   // the next tile's records (its indices came with this tile's fetch) for layer 4's fill
      gather_load<false>(gh, lane & 7, pf_ok ? pf_nb : -1, pf_ray, gx, recA, recB, viewdirs, vemb_const);
    layer_mfma<4, 4, 2, FR_W3, FR_W4>(X, rs, vb, acc, a, a1);
    __syncthreads();
    store_act(X, ot0, nullptr, acc, SCALED, SCALED ? sW[SW_DS + 2] : 1.f);
    __syncthreads();
    init_bias(acc, ot0, sW + SW_B4);
    if (FILL) {   // layer 4 with the next tile's posenc in its MFMA gaps (one copy per argument half)
      if (gh == 0)
        layer_mfma<4, 5, 1, FR_W4, FR_WH, true>(X, rs, vb, acc, a, a1, [&]() { pe_compute<0>(pf_q, gx, pe); });
      else
        layer_mfma<4, 5, 1, FR_W4, FR_WH, true>(X, rs, vb, acc, a, a1, [&]() { pe_compute<1>(pf_q, gx, pe); });
    } else {
      layer_mfma<4, 5, 1, FR_W4, FR_WH>(X, rs, vb, acc, a, a1);
    }
    // the next tile's gather rows' neighbours (fetched at this tile's top) for its P rows
    if (APN_H4_LDSPN && tid < TR4) sNb[tid] = pf_ok ? pf_nb : -1;
    __syncthreads();
    // layer-4 output lrelu(acc) as fp32 rows (the IDW sum reads them)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int o0 = 16 * (ot0 + j) + 4 * g;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        *(f32x4*)(X + out32_off(16 * mt + li, o0 >> 2)) = lrelu4(SCALED ? acc[mt][j] * sW[SW_DS + 3] : acc[mt][j]);
    }
    // the head's fragment chunks 1..4 (chunk 0 came with layer 4), a whole IDW phase ahead
    h8 hfr[KV / 32 - 1][2];
#pragma unroll
    for (int q = 1; q < KV / 32; ++q)
#pragma unroll
      for (int pt = 0; pt < 2; ++pt)   // (chunk 1 came with layer 4 too when two-deep: not reloaded)
        hfr[q - 1][pt] = (APN_H4_PF2 && q == 1) ? a1[0][pt] : frag(rs, vb, FR_WH + q * 2 + pt);
    // the next tile's records (its indices came with this tile's fetch)
    if (APN_H4_RECPF && tile + per_xcd < t_end)
      gather_load<!LISTED>(gh, lane & 7, pf_ok ? pf_nb : -1, pf_ray, gn, recA, recB, viewdirs, vemb_const);
    __syncthreads();
    APN_PHASE(2)
    // ------------------------------------------------ IDW sum (temporalpoints.py:493-494) into
    // registers: thread (sample s, oq) sums features 4 oq .. 4 oq + 3 and 64 + 4 oq .. (chunks oq,
    // oq + 16: conflict-free ds_read_b128), then the density head
    const int s_ = tid >> 4, oq = tid & 15;
    f32x4 h0 = {0.f, 0.f, 0.f, 0.f}, h1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int m = 8 * s_ + k;
      const f32x4 v0 = *(const f32x4*)(X + out32_off(m, oq));
      const f32x4 v1 = *(const f32x4*)(X + out32_off(m, oq + 16));
      const float w = sIdw[m];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        h0[r] = fmaf(w, v0[r], h0[r]);
        h1[r] = fmaf(w, v1[r], h1[r]);
      }
    }
    {
      // densitynet Linear(128 -> 1) (tineuvox.py:158) over this thread's 8 features, then the 16 lanes
      const f32x4 wd0 = *(const f32x4*)(sW + SW_WD + 4 * oq), wd1 = *(const f32x4*)(sW + SW_WD + 64 + 4 * oq);
      float d = (((h0[0] * wd0[0] + h0[1] * wd0[1]) + h0[2] * wd0[2]) + h0[3] * wd0[3]) +
                (((h1[0] * wd1[0] + h1[1] * wd1[1]) + h1[2] * wd1[2]) + h1[3] * wd1[3]);
      d += __shfl_xor(d, 8, 64);
      d += __shfl_xor(d, 4, 64);
      d += __shfl_xor(d, 2, 64);
      d += __shfl_xor(d, 1, 64);
      if (oq == 0) {  // Raw2Alpha (render_utils_kernel.cu:357-369): (1 + e)^-interval on v_log / v_exp
        const float e = expf((d + sW[SW_BD]) + shift);
        sOut[12 * s_ + 3] = 1.f - __builtin_amdgcn_exp2f(-interval * __builtin_amdgcn_logf(1.f + e));
      }
      if (SCALED) { h0 = h0 * sW[SW_HSC]; h1 = h1 * sW[SW_HSC]; }
      // range guard on the last values split (false for NaN too); the flag store waits for the end
      range_bad |= !(fmaxf(fmaxf(fmaxf(fabsf(h0[0]), fabsf(h0[1])), fmaxf(fabsf(h0[2]), fabsf(h0[3]))),
                           fmaxf(fmaxf(fabsf(h1[0]), fabsf(h1[1])), fmaxf(fabsf(h1[2]), fabsf(h1[3])))) <= H3_RANGE);
    }
    // direct blend + weight-vis colour (temporalpoints.py:459-470, 517-519): waves 1-2, lane =
    // (sample, quantity); sums over the 8 neighbours in order
    if (!LISTED && (wid == 1 || wid == 2)) {
      const int sl = (wid - 1) * 64 + lane;
      const int s = sl >> 3, qn = sl & 7;
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
    if (!APN_H4_HEADW) __syncthreads();   // every IDW read of X is done: the head rows may overwrite it
    {
      // head input row s: [h (128) | view embedding (27) | 0] as hi/lo halves (rows alias X)
      char* hr = X + head_row(s_);
      h4 hi0, lo0, hi1, lo1;
      split4(h0, hi0, lo0);
      split4(h1, hi1, lo1);
      *(h4*)(hr + 8 * oq) = hi0;
      *(h4*)(hr + 128 + 8 * oq) = hi1;
      *(h4*)(hr + HLO + 8 * oq) = lo0;
      *(h4*)(hr + HLO + 128 + 8 * oq) = lo1;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int e = 2 * oq + u;
        const float ve = sV[s_ * 32 + e];
        const _Float16 vh = (_Float16)ve;
        *(_Float16*)(hr + 2 * (128 + e)) = vh;
        *(_Float16*)(hr + HLO + 2 * (128 + e)) = (_Float16)(ve - (float)vh);
      }
    }
    __syncthreads();
    // ------------------------------------------------ rgb head: folded [h; v] -> 64, ReLU, -> 3, sigmoid
    {
      const int o0 = 16 * wid + 4 * g;
      f32x4 ah = *(const f32x4*)(sW + SW_BH + o0);   // views_linears.0 (folded) bias
      const char* hr = X + head_row(li);              // B column li = sample li (16 real columns)
      h8 an[2][2];   // the next tile's W1E chunk 0 (carried across the gather)
      h8 an1[2][2];   // and chunk 1 (two-deep)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int pt = 0; pt < 2; ++pt) {
          an[j][pt] = frag(rs, vb, FR_W1E + j * 4 + pt);
          an1[j][pt] = APN_H4_PF2 ? frag(rs, vb, FR_W1E + j * 4 + 2 + pt) : an[j][pt];
        }
#pragma unroll
      for (int q = 0; q < KV / 32; ++q) {
        const h8 bh = *(const h8*)(hr + 16 * (4 * q + g));
        const h8 bl = *(const h8*)(hr + HLO + 16 * (4 * q + g));
        ah = q == 0 ? mfma3(a[0][0], a[0][1], bh, bl, ah) : mfma3(hfr[q - 1][0], hfr[q - 1][1], bh, bl, ah);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        a[j][0] = an[j][0]; a[j][1] = an[j][1];
        a1[j][0] = an1[j][0]; a1[j][1] = an1[j][1];
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
      if (g == 0) {
#pragma unroll
        for (int c = 0; c < 3; ++c) sPart[(wid * TS4 + li) * 4 + c] = pc[c];
      }
    }
    __syncthreads();
    if (tid < TS4 * 3) {  // views_linears.2 bias + sigmoid (temporalpoints.py:513-515)
      const int s = tid / 3, c = tid % 3;
      const float v = ((sPart[(0 * TS4 + s) * 4 + c] + sPart[(1 * TS4 + s) * 4 + c]) + sPart[(2 * TS4 + s) * 4 + c]) +
                      sPart[(3 * TS4 + s) * 4 + c];
      sOut[12 * s + c] = 1.f / (1.f + expf(-(v + sW[SW_BV2 + c])));
    }
    APN_PHASE(3)
    prev_s0 = s0;
  }
#undef APN_PHASE
  if (TIMED && tid == 0) {
    ph[5] = clock64() - tk0;
    for (int i = 0; i < 6; ++i) atomicAdd(&g_phase4[i], ph[i]);
  }
  __syncthreads();
  if (LISTED) {
    if (prev_s0 >= 0 && tid < TS4 && prev_s0 + tid < nS)
      out[(size_t)list[prev_s0 + tid] * 3] = *(const float4*)(sOut + 12 * tid);
  } else if (prev_s0 >= 0 && tid < TS4 * 3 && prev_s0 + tid / 3 < nS) {
    out[(size_t)prev_s0 * 3 + tid] = *(const float4*)(sOut + 4 * tid);
  }
  if (range_bad) __builtin_amdgcn_raw_buffer_store_b32(1, rs, 0, H_TOTAL * 2, 0);   // the range flag (OFF_FLAG)
}

// One instantiation per weight-scale mode; apn_point_mlp launches both and the one that does not
// match wbuf's mode exits at once (as does every workgroup once the range flag is set).
template <bool SCALED, bool TIMED, bool LISTED>
__global__ __launch_bounds__(MLP_THREADS, 2) void k_point_mlp_h4(
    const float4* __restrict__ s_pos, const int* __restrict__ s_ray, const int* __restrict__ s_nbr,
    const int* __restrict__ list, const int* __restrict__ n_samples_dev, const float4* __restrict__ recA, const float4* __restrict__ recB,
    const float4* __restrict__ pproj, const float* __restrict__ viewdirs, const float* __restrict__ vemb_const,
    const float* __restrict__ wbuf, float eps, float shift, float interval, float4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) char X[TR4 * XB];
  __shared__ float sTo[TR4];
  __shared__ float sIdw[TR4];
  __shared__ float sRow[TR4 * RS];
  __shared__ __attribute__((aligned(16))) float sOut[TS4 * 12];
  __shared__ float sV[TS4 * 32];
  __shared__ __attribute__((aligned(16))) float sW[SW_TOTAL];
  __shared__ float sPart[4 * TS4 * 4];
  __shared__ int sNb[TR4];
  __shared__ int s_skip;
  if (threadIdx.x == 0)
    s_skip = __builtin_nontemporal_load((const int*)(wbuf + OFF_FLAG)) != 0 || (wbuf[OFF_SCALE + 6] != 0.f) != SCALED;
  __syncthreads();
  if (s_skip) return;
  mlp_tiles<SCALED, TIMED, LISTED>(s_pos, s_ray, s_nbr, list, n_samples_dev, recA, recB, pproj, viewdirs, vemb_const, wbuf, eps, shift,
                    interval, out, X, sTo, sIdw, sRow, sOut, sV, sW, sPart, sNb);
}

// The early-ray-termination passes' kernel: both weight-scale modes in one launch, the mode read
// from wbuf by each workgroup (one launch per pass instead of two; the registers are the larger
// mode's, below the 256 of two waves per SIMD either way).
__global__ __launch_bounds__(MLP_THREADS, 2) void k_point_mlp_h4_listed(
    const float4* __restrict__ s_pos, const int* __restrict__ s_ray, const int* __restrict__ s_nbr,
    const int* __restrict__ list, const int* __restrict__ n_samples_dev, const float4* __restrict__ recA, const float4* __restrict__ recB,
    const float4* __restrict__ pproj, const float* __restrict__ viewdirs, const float* __restrict__ vemb_const,
    const float* __restrict__ wbuf, float eps, float shift, float interval, float4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) char X[TR4 * XB];
  __shared__ float sTo[TR4];
  __shared__ float sIdw[TR4];
  __shared__ float sRow[TR4 * RS];
  __shared__ __attribute__((aligned(16))) float sOut[TS4 * 12];
  __shared__ float sV[TS4 * 32];
  __shared__ __attribute__((aligned(16))) float sW[SW_TOTAL];
  __shared__ float sPart[4 * TS4 * 4];
  __shared__ int sNb[TR4];
  __shared__ int s_mode;   // 0: unscaled weights, 1: scaled, 2: the range flag is set (skip)
  if (threadIdx.x == 0)
    s_mode = __builtin_nontemporal_load((const int*)(wbuf + OFF_FLAG)) != 0 ? 2 : (wbuf[OFF_SCALE + 6] != 0.f ? 1 : 0);
  __syncthreads();
  const int mode = s_mode;
  if (mode == 2) return;
  if (mode == 1)
    mlp_tiles<true, false, true>(s_pos, s_ray, s_nbr, list, n_samples_dev, recA, recB, pproj, viewdirs, vemb_const, wbuf, eps,
                                 shift, interval, out, X, sTo, sIdw, sRow, sOut, sV, sW, sPart, sNb);
  else
    mlp_tiles<false, false, true>(s_pos, s_ray, s_nbr, list, n_samples_dev, recA, recB, pproj, viewdirs, vemb_const, wbuf, eps,
                                  shift, interval, out, X, sTo, sIdw, sRow, sOut, sV, sW, sPart, sNb);
}

}  // namespace t128

void launch_point_mlp_h4(int blocks, bool timed, hipStream_t stream, const float4* s_pos, const int* s_ray, const int* s_nbr,
                         const int* n_samples_dev, const float4* recA, const float4* recB, const float4* pproj,
                         const float* viewdirs, const float* vemb_const, const float* wbuf, float eps, float shift,
                         float interval, float4* out, const int* list) {
  auto go = [&](auto kern, int nb) {
    hipLaunchKernelGGL(kern, dim3(nb), dim3(MLP_THREADS), 0, stream, s_pos, s_ray, s_nbr, list, n_samples_dev, recA,
                       recB, pproj, viewdirs, vemb_const, wbuf, eps, shift, interval, out);
  };
  const int nb_scaled = blocks < 256 * 8 ? blocks : 256 * 8;
  if (list) {   // early-ray-termination passes (9 per frame): one launch, either weight-scale mode
#if APN_H4_MERGED
    go(t128::k_point_mlp_h4_listed, blocks);
#else
    go(t128::k_point_mlp_h4<false, false, true>, blocks);
    go(t128::k_point_mlp_h4<true, false, true>, blocks < 256 ? blocks : 256);
#endif
    return;
  }
#ifdef APN_DEBUG_BUILD
  if (timed) {
    go(t128::k_point_mlp_h4<false, true, false>, blocks);
    go(t128::k_point_mlp_h4<true, true, false>, nb_scaled);
    return;
  }
#else
  (void)timed;
#endif
  go(t128::k_point_mlp_h4<false, false, false>, blocks);
  go(t128::k_point_mlp_h4<true, false, false>, nb_scaled);
}

int debug_phase_cycles_h4(uint64_t* out6) {
  uint64_t v[6];
  APN_HIP_TRY(hipMemcpyFromSymbol(v, HIP_SYMBOL(t128::g_phase4), sizeof(v)));
  static const unsigned long long zero[6] = {0, 0, 0, 0, 0, 0};
  APN_HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(t128::g_phase4), zero, sizeof(zero)));
  for (int i = 0; i < 6; ++i) out6[i] += v[i];
  return APN_OK;
}

}  // namespace apn
