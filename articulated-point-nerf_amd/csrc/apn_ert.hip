// Early ray termination for the neighbour MLP (exact): the reference's compositing
// (temporalpoints.py:611-651 -> Alphas2Weights, render_utils_kernel.cu:430-459) walks each ray's
// kept samples front to back and stops after the sample whose update takes T below 1e-3; the
// Point-NeRF columns {rgb, alpha} of every later sample of that ray are never read. The reference
// still runs feat_net / densitynet / rgbnet on them (temporalpoints.py:452-519). Here the MLP runs
// in passes over each ray's kept samples in step order -- two samples at a time up to local index
// 12, then [12, 16), [16, 24), [24, ...) -- and after each pass a per-ray walk with the compositing's own
// arithmetic (pre-mask alpha > thr, T in double, the same break test) retires the rays that
// terminated; the next pass lists only the live rays' next samples. Every sample the compositing
// reads has exactly the values a full MLP launch would give it (a sample's MLP rows do not depend
// on the other rows of its tile), so apn_composite's output is bit-identical (tests/test_ert.py) --
// unless the split kernel's fp16 range guard fires. Here only the samples the passes run can set
// it; the all-samples launch also checks the samples past each ray's break. When the only
// out-of-range value lies past a break, the all-samples frame is recomputed on FP32 MFMA and this
// one keeps its fp16-split values: the two then differ in bits (both within the precision bar).
//
// The direct path (alpha_d, rgb_d, temporalpoints.py:459-470) and the weight-visualisation colour
// (517-519) are cheap record blends; k_direct_blend computes them for every kept sample (the direct
// path has its own termination point), with the MLP kernel's arithmetic and order.
#include "apn_mlp_layout.h"

namespace apn {

// 1: the XCD-aware sample order below. Measured no better (round 6, same box, parity green: MLP
// stage minus the pass kernels 0.402 / 0.402 -> 0.417 / 0.413 ms per C2 frame): off.
#ifndef APN_DIRECT_XCD
#define APN_DIRECT_XCD 0
#endif

// out12 columns 4..11 = {r_d, g_d, b_d, alpha_d, wr, wg, wb, 0} of sample i, the arithmetic of the
// fused MLP kernel's gather (apn_mlp_h4.hip gather_q: squared distance, direct weight) and its
// epilogue (IDW weights, sequential sums over the 8 neighbours in order).
__global__ __launch_bounds__(256) void k_direct_blend(const float4* __restrict__ s_pos, const int* __restrict__ s_nbr,
                                                      const int* __restrict__ n_dev, const float4* __restrict__ recA,
                                                      const float4* __restrict__ recB, float eps,
                                                      float4* __restrict__ out) {
  const int n = *n_dev;
  // XCD-aware sample order: workgroup b runs on XCD b % 8, so each XCD walks one contiguous eighth
  // of the samples -- neighbouring samples share neighbour points, and their records then meet in
  // that XCD's L2 instead of being fetched by all eight (PMC: L2 hit 0.79, 0.63 GB of HBM per
  // launch against ~0.25 GB of samples and records, round 6)
  const int nx = APN_DIRECT_XCD && (gridDim.x % 8 == 0) ? 8 : 1;
  const int xcd = blockIdx.x % nx, per_xcd = gridDim.x / nx;
  const int chunk = (n + nx - 1) / nx;
  const int i_end = min(n, (xcd + 1) * chunk);
  for (int i = xcd * chunk + (int)(blockIdx.x / nx) * (int)blockDim.x + (int)threadIdx.x; i < i_end;
       i += per_xcd * (int)blockDim.x) {
    const float4 q = s_pos[i];
    const int4 nb0 = ((const int4*)s_nbr)[2 * (size_t)i], nb1 = ((const int4*)s_nbr)[2 * (size_t)i + 1];
    const int nbs[8] = {nb0.x, nb0.y, nb0.z, nb0.w, nb1.x, nb1.y, nb1.z, nb1.w};
    float to[8], dw[8], al[8];
    float3 cd[8], cw[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int nb = nbs[k];
      const size_t m = (size_t)max(nb, 0);
      // 3 of the point's 6 float4s: b0.w carries alpha (apn_lbs.hip record layout), so recA's
      // last float4 is not read
      const float4 a0 = recA[4 * m], b0 = recB[2 * m], b1 = recB[2 * m + 1];
      if (nb >= 0) {
        const float dx = q.x - a0.x, dy = q.y - a0.y, dz = q.z - a0.z;
        const float tn = (dx * dx + dy * dy) + dz * dz;
        to[k] = tn;
        dw[k] = expf(-(tn * tn) / a0.w);   // temporalpoints.py:461 (to_nn is already squared)
        al[k] = b0.w;
        cd[k] = make_float3(b0.x, b0.y, b0.z);
        cw[k] = make_float3(b1.x, b1.y, b1.z);
      } else {
        to[k] = 1.f;
        dw[k] = 0.f;
        al[k] = 0.f;
        cd[k] = make_float3(0.f, 0.f, 0.f);
        cw[k] = make_float3(0.f, 0.f, 0.f);
      }
    }
    float w[8], sum = 0.f, sumd = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      w[k] = __builtin_amdgcn_rcpf(to[k] + eps);   // v_rcp_f32, as the MLP kernel's IDW weights
      sum += w[k];
    }
    if (APN_H4_IDWG)   // the MLP kernel's shuffle-tree order (apn_mlp_layout.h)
      sum = ((w[0] + w[1]) + (w[2] + w[3])) + ((w[4] + w[5]) + (w[6] + w[7]));
    const float inv = __builtin_amdgcn_rcpf(sum);
#pragma unroll
    for (int k = 0; k < 8; ++k) sumd += dw[k];
    const float idn = __builtin_amdgcn_rcpf(sumd + 1e-12f);
    float ad = 0.f, rd = 0.f, gd = 0.f, bd = 0.f, wr = 0.f, wg = 0.f, wb = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      ad += (0.125f * dw[k]) * al[k];
      rd += (dw[k] * idn) * cd[k].x;
      gd += (dw[k] * idn) * cd[k].y;
      bd += (dw[k] * idn) * cd[k].z;
      const float iw = w[k] * inv;
      wr += iw * cw[k].x;
      wg += iw * cw[k].y;
      wb += iw * cw[k].z;
    }
    out[3 * (size_t)i + 1] = make_float4(rd, gd, bd, ad);
    out[3 * (size_t)i + 2] = make_float4(wr, wg, wb, 0.f);
  }
}

// One launch per pass. Pass 0 starts every ray at its first kept sample with T = 1; every later
// pass first walks ray r's samples of the previous pass with the compositing's arithmetic
// (apn_composite.hip k_composite_lds, Point-NeRF path: pre-mask, T in double, the break test) and
// retires the ray if its T fell below 1e-3. Then the ray's next min(B, left) samples go to the
// pass's list: a block scan of the counts, one atomic per block for the block's place in the list
// (the list's order between blocks varies from run to run; a sample's MLP result does not depend
// on its tile-mates, so the frame does not), and the pass size accumulates in *count -- the MLP
// launch's device count.
// APN_ERT_RAYLIST: pass 0 walks every ray and lists the rays it gave samples to (rl_out, *n_rl_out);
// every later pass walks only the previous pass's listed rays (rl_in) -- the rays still live --
// instead of all n_rays, and lists its own (the same block scan: one atomic per block for each).
#ifndef APN_ERT_RAYLIST
#define APN_ERT_RAYLIST 1
#endif
__global__ __launch_bounds__(256) void k_ert_pass(int64_t n_rays, int first, const int* __restrict__ beg,
                                                  const int* __restrict__ end, const float4* __restrict__ out,
                                                  float thr, int use_mask, int* __restrict__ pos,
                                                  float* __restrict__ T, int* __restrict__ cnt, int B,
                                                  int* __restrict__ list, int* __restrict__ count,
                                                  const int* __restrict__ prev_count, const int* __restrict__ rl_in,
                                                  const int* __restrict__ n_rl_in, int* __restrict__ rl_out,
                                                  int* __restrict__ n_rl_out) {
  __shared__ int s_wave[4];
  __shared__ int s_base, s_rbase;
  // an empty previous pass leaves every ray with nothing listed, so this pass and every later one
  // are empty too (their counts stay at the 0 they were filled with): the whole grid returns
  if (prev_count && *prev_count == 0) return;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  int64_t r = i;
  if (APN_ERT_RAYLIST && !first) {   // the rays the previous pass listed
    const int n_live = *n_rl_in;
    if ((int64_t)blockIdx.x * 256 >= n_live) return;   // workgroup-uniform
    r = i < n_live ? rl_in[i] : n_rays;
  }
  int c = 0, p = 0;
  if (r < n_rays) {
    const int e = end[r];
    if (first) {
      p = beg[r];
      T[r] = 1.f;
      c = min(e - p, B);
    } else {
      const int cp = cnt[r];
      p = pos[r];
      if (cp > 0) {
        float t = T[r];
        bool dead = false;
        for (int i = p; i < p + cp; ++i) {
          const float a = out[3 * (size_t)i].w;
          if (!use_mask || a > thr) {
            t = (float)((double)t * (1.0 - (double)a));
            if ((double)t < 1e-3) {
              dead = true;
              break;
            }
          }
        }
        p += cp;
        T[r] = t;
        c = dead ? 0 : min(e - p, B);
      }
    }
    pos[r] = p;
    cnt[r] = c;
  }
  // block-wide exclusive scans of c and (APN_ERT_RAYLIST, by ballot) of the live flag c > 0
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int inc = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(inc, o, 64);
    if (lane >= o) inc += v;
  }
  const unsigned long long live = APN_ERT_RAYLIST ? __ballot(c > 0) : 0ull;
  __shared__ int s_live[4];
  if (lane == 63) {
    s_wave[wid] = inc;
    s_live[wid] = __popcll(live);
  }
  __syncthreads();
  int wbase = 0, tot = 0, lbase = 0, ltot = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    wbase += w < wid ? s_wave[w] : 0;
    tot += s_wave[w];
    lbase += w < wid ? s_live[w] : 0;
    ltot += s_live[w];
  }
  if (threadIdx.x == 0) {
    s_base = tot > 0 ? atomicAdd(count, tot) : 0;
    if (APN_ERT_RAYLIST) s_rbase = ltot > 0 ? atomicAdd(n_rl_out, ltot) : 0;
  }
  __syncthreads();
  const int o = s_base + wbase + inc - c;
  for (int j = 0; j < c; ++j) list[o + j] = p + j;
  if (APN_ERT_RAYLIST && c > 0)
    rl_out[s_rbase + lbase + __popcll(live & ((1ull << lane) - 1ull))] = (int)r;
}

__global__ void k_ray_bounds_ert(const int* __restrict__ s_ray, const int* __restrict__ n_dev, int* __restrict__ beg,
                                 int* __restrict__ end) {
  const int n = *n_dev;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int r = s_ray[i];
  if (i == 0 || s_ray[i - 1] != r) beg[r] = i;
  if (i == n - 1 || s_ray[i + 1] != r) end[r] = i + 1;
}

int direct_blend(const float4* s_pos, const int* s_nbr, int64_t max_samples, const int* n_samples_dev,
                 const float4* recA, const float4* recB, float eps, float4* out, hipStream_t s) {
  const int blocks = ceil_div(max_samples, 256) < 256 * 16 ? ceil_div(max_samples, 256) : 256 * 16;
  hipLaunchKernelGGL(k_direct_blend, dim3(blocks), dim3(256), 0, s, s_pos, s_nbr, n_samples_dev, recA, recB, eps, out);
  return launch_status();
}

// workspace: beg, end, pos, cnt [n_rays] i32, T [n_rays] f32, the passes' list sizes
// [ERT_PASSES] i32, list [max_samples] i32, two live-ray lists [n_rays] i32 and their sizes
// [ERT_PASSES] i32
static size_t ert_ws_layout(int64_t max_samples, int64_t n_rays, size_t* off) {
  size_t o = 0;
  auto take = [&](size_t bytes) {
    size_t at = o;
    o += (bytes + 255) / 256 * 256;
    return at;
  };
  off[0] = take(4 * (size_t)n_rays);        // beg
  off[1] = take(4 * (size_t)n_rays);        // end
  off[2] = take(4 * (size_t)n_rays);        // pos
  off[3] = take(4 * (size_t)n_rays);        // cnt
  off[4] = take(4 * (size_t)n_rays);        // T
  off[5] = take(4 * (size_t)ERT_PASSES);    // pass sizes
  off[6] = take(4 * (size_t)max_samples);   // list
  off[7] = take(4 * (size_t)n_rays);        // live rays, even passes' output
  off[8] = take(4 * (size_t)n_rays);        // live rays, odd passes' output
  off[9] = take(4 * (size_t)ERT_PASSES);    // live-ray list sizes
  return o;
}

size_t ert_workspace_bytes(int64_t max_samples, int64_t n_rays) {
  size_t off[10];
  return ert_ws_layout(max_samples, n_rays, off);
}

// Per-ray local index ranges of the passes: two samples at a time for the first twelve (a ray's
// surplus over its break is at most one sample there), then 4, 8 and the rest.
static const int ERT_PASS[ERT_PASSES] = {2, 2, 2, 2, 2, 2, 4, 8, 1 << 30};

int ert_run(const float4* s_pos, const int* s_ray, const int* s_nbr, int64_t max_samples, const int* n_samples_dev,
            int64_t n_rays, const float4* recA, const float4* recB, float eps, float thr, float4* out, void* ws,
            int with_direct, int* stats, void* const* events, hipStream_t s, const MlpPass& mlp) {
  size_t off[10];
  ert_ws_layout(max_samples, n_rays, off);
  char* w = (char*)ws;
  int* beg = (int*)(w + off[0]);
  int* end = (int*)(w + off[1]);
  int* pos = (int*)(w + off[2]);
  int* cnt = (int*)(w + off[3]);
  float* T = (float*)(w + off[4]);
  int* sizes = (int*)(w + off[5]);
  int* list = (int*)(w + off[6]);
  int* rl[2] = {(int*)(w + off[7]), (int*)(w + off[8])};
  int* rl_n = (int*)(w + off[9]);
  const int rb = ceil_div(n_rays, 256);
  const int use_mask = thr > 0.f ? 1 : 0;
  APN_TRY(fill_i32(beg, 0, n_rays, s));   // rays without kept samples: beg = end = 0
  APN_TRY(fill_i32(end, 0, n_rays, s));
  APN_TRY(fill_i32(sizes, 0, ERT_PASSES, s));
  if (APN_ERT_RAYLIST) APN_TRY(fill_i32(rl_n, 0, ERT_PASSES, s));
  hipLaunchKernelGGL(k_ray_bounds_ert, dim3(ceil_div(max_samples, 256)), dim3(256), 0, s, s_ray, n_samples_dev, beg,
                     end);
  // direct path + weight colour of every kept sample (read up to the direct path's own break);
  // with_direct = 0: the caller runs apn_direct_blend itself (e.g. on a second stream beside the passes)
  if (with_direct) APN_TRY(direct_blend(s_pos, s_nbr, max_samples, n_samples_dev, recA, recB, eps, out, s));
  for (int p = 0; p < ERT_PASSES; ++p) {
    hipLaunchKernelGGL(k_ert_pass, dim3(rb), dim3(256), 0, s, n_rays, p == 0 ? 1 : 0, beg, end, (const float4*)out,
                       thr, use_mask, pos, T, cnt, ERT_PASS[p], list, sizes + p, p == 0 ? nullptr : sizes + p - 1,
                       (const int*)rl[(p + 1) & 1], p == 0 ? nullptr : rl_n + p - 1, rl[p & 1], rl_n + p);
    if (events) APN_HIP_TRY(hipEventRecord((hipEvent_t)events[2 * p], s));
    APN_TRY(mlp(list, sizes + p));
    if (events) APN_HIP_TRY(hipEventRecord((hipEvent_t)events[2 * p + 1], s));
  }
  if (stats) APN_TRY(copy_i32(sizes, stats, ERT_PASSES, s));
  return launch_status();
}

}  // namespace apn
