// Per-ray compositing of the kept samples, one ray per thread (temporalpoints.py:611-710):
//   pre-mask  alpha > fast_color_thres                         (611-626)
//   Alphas2Weights: T_i = prod_{j<i}(1 - a_j), w_i = T_i a_i,    (629-632 -> render_utils_kernel.cu:430-459)
//                   T updated in double, break once T < 1e-3 (the crossing sample is kept)
//   post-mask w > fast_color_thres                             (634-651)
//   segment sums: rgb (+ alphainv_last*bg), depth = sum w*step_id, weight-vis colour (+bg)
// for the Point-NeRF path and, independently masked, the direct path (alpha_d, rgb_d).
// Sequential per-ray accumulation in sample order reproduces segment_coo's sum order.
#include "apn_common.h"

#include <climits>

namespace apn {

__global__ void k_ray_bounds(const int* __restrict__ s_ray, const int* __restrict__ n_dev, int* __restrict__ beg,
                             int* __restrict__ end) {
  const int n = *n_dev;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int r = s_ray[i];
  if (i == 0 || s_ray[i - 1] != r) beg[r] = i;
  if (i == n - 1 || s_ray[i + 1] != r) end[r] = i + 1;
}

#ifdef APN_DEBUG_BUILD   // the one-ray-per-thread walk from global memory: debug build only (A/B)
// Both paths walk the ray's samples in one loop (each keeps its own T, mask and break -- the same
// arithmetic as two separate walks), and sample i + 1's records are loaded before sample i is
// accumulated: the per-ray chain of dependent loads is what a compositing thread waits on.
__global__ void k_composite(const float4* __restrict__ smp, const float4* __restrict__ s_pos,
                            const int* __restrict__ beg, const int* __restrict__ end, int64_t n_rays, float thr,
                            int use_mask, float bg, float* __restrict__ rgb_out, float* __restrict__ rgb_d_out,
                            float* __restrict__ depth_out, float* __restrict__ wvis_out, float* __restrict__ last_out,
                            float* __restrict__ last_d_out) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rays) return;
  const int b = beg[r], e = end[r];
  // Point-NeRF path (a) and direct path (d)
  float T = 1.f, cr = 0.f, cg = 0.f, cb = 0.f, dep = 0.f, wr = 0.f, wg = 0.f, wb = 0.f;
  float Td = 1.f, dr = 0.f, dg = 0.f, db = 0.f;
  bool run_a = true, run_d = true;
  float4 va, vd, vc, vp;
  if (b < e) {
    va = smp[3 * (size_t)b]; vd = smp[3 * (size_t)b + 1]; vc = smp[3 * (size_t)b + 2]; vp = s_pos[b];
  }
  for (int i = b; i < e && (run_a || run_d); ++i) {
    const float4 a4 = va, d4 = vd, c4 = vc, p4 = vp;
    if (i + 1 < e) {   // next sample's records in flight while this one is accumulated
      va = smp[3 * (size_t)(i + 1)]; vd = smp[3 * (size_t)(i + 1) + 1]; vc = smp[3 * (size_t)(i + 1) + 2];
      vp = s_pos[i + 1];
    }
    if (run_a) {
      const float a = a4.w;
      if (!use_mask || a > thr) {
        const float w = T * a;
        if (!use_mask || w > thr) {
          cr += w * a4.x; cg += w * a4.y; cb += w * a4.z;
          dep += w * (float)__float_as_int(p4.w);
          wr += w * c4.x; wg += w * c4.y; wb += w * c4.z;
        }
        T = (float)((double)T * (1.0 - (double)a));
        if ((double)T < 1e-3) run_a = false;
      }
    }
    if (run_d) {
      const float a = d4.w;
      if (!use_mask || a > thr) {
        const float w = Td * a;
        if (!use_mask || w > thr) { dr += w * d4.x; dg += w * d4.y; db += w * d4.z; }
        Td = (float)((double)Td * (1.0 - (double)a));
        if ((double)Td < 1e-3) run_d = false;
      }
    }
  }
  rgb_out[3 * r] = cr + T * bg; rgb_out[3 * r + 1] = cg + T * bg; rgb_out[3 * r + 2] = cb + T * bg;
  depth_out[r] = dep;
  wvis_out[3 * r] = wr + T * bg; wvis_out[3 * r + 1] = wg + T * bg; wvis_out[3 * r + 2] = wb + T * bg;
  last_out[r] = T;
  rgb_d_out[3 * r] = dr + Td * bg; rgb_d_out[3 * r + 1] = dg + Td * bg; rgb_d_out[3 * r + 2] = db + Td * bg;
  last_d_out[r] = Td;
}
#endif  // APN_DEBUG_BUILD

// The same per-ray walks with each wave's samples staged through LDS: a wave's 64 rays own one
// contiguous sample range (survivors are sorted by ray), which it loads in chunks of CMP_CH
// samples with coalesced stores into LDS; each lane then walks its ray from LDS. The walks are
// the sequential T products above (bit-identical); only the loads move, from a chain of
// dependent global reads per ray (long rays set the wave's time) to one coalesced stage per chunk.
constexpr int CMP_CH = 256;
__global__ __launch_bounds__(64) void k_composite_lds(const float4* __restrict__ smp, const float4* __restrict__ s_pos,
                                                      const int* __restrict__ beg, const int* __restrict__ end,
                                                      int64_t n_rays, float thr, int use_mask, float bg,
                                                      float* __restrict__ rgb_out, float* __restrict__ rgb_d_out,
                                                      float* __restrict__ depth_out, float* __restrict__ wvis_out,
                                                      float* __restrict__ last_out, float* __restrict__ last_d_out) {
  __shared__ float4 sA[CMP_CH], sD[CMP_CH], sC[CMP_CH];
  __shared__ float sStep[CMP_CH];
  const int lane = threadIdx.x;
  const int64_t r = (int64_t)blockIdx.x * 64 + lane;
  const bool valid = r < n_rays;
  const int b = valid ? beg[r] : 0, e = valid ? end[r] : 0;
  int lo = e > b ? b : INT_MAX, hi = e > b ? e : 0;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    lo = min(lo, __shfl_xor(lo, o, 64));
    hi = max(hi, __shfl_xor(hi, o, 64));
  }
  float T = 1.f, cr = 0.f, cg = 0.f, cb = 0.f, dep = 0.f, wr = 0.f, wg = 0.f, wb = 0.f;
  float Td = 1.f, dr = 0.f, dg = 0.f, db = 0.f;
  bool run_a = true, run_d = true;
  int i = b;
  for (int cs = lo; cs < hi; cs += CMP_CH) {
    const int ce = min(cs + CMP_CH, hi);
    __syncthreads();   // the previous chunk is consumed
    for (int j = lane; j < ce - cs; j += 64) {
      const size_t k = (size_t)(cs + j);
      sA[j] = smp[3 * k];
      sD[j] = smp[3 * k + 1];
      sC[j] = smp[3 * k + 2];
      sStep[j] = (float)__float_as_int(s_pos[k].w);
    }
    __syncthreads();
    for (; i < e && i < ce && (run_a || run_d); ++i) {
      const int j = i - cs;
      if (run_a) {
        const float4 a4 = sA[j];
        const float a = a4.w;
        if (!use_mask || a > thr) {
          const float w = T * a;
          if (!use_mask || w > thr) {
            cr += w * a4.x; cg += w * a4.y; cb += w * a4.z;
            dep += w * sStep[j];
            const float4 c4 = sC[j];
            wr += w * c4.x; wg += w * c4.y; wb += w * c4.z;
          }
          T = (float)((double)T * (1.0 - (double)a));
          if ((double)T < 1e-3) run_a = false;
        }
      }
      if (run_d) {
        const float4 d4 = sD[j];
        const float a = d4.w;
        if (!use_mask || a > thr) {
          const float w = Td * a;
          if (!use_mask || w > thr) { dr += w * d4.x; dg += w * d4.y; db += w * d4.z; }
          Td = (float)((double)Td * (1.0 - (double)a));
          if ((double)Td < 1e-3) run_d = false;
        }
      }
    }
  }
  if (!valid) return;
  rgb_out[3 * r] = cr + T * bg; rgb_out[3 * r + 1] = cg + T * bg; rgb_out[3 * r + 2] = cb + T * bg;
  depth_out[r] = dep;
  wvis_out[3 * r] = wr + T * bg; wvis_out[3 * r + 1] = wg + T * bg; wvis_out[3 * r + 2] = wb + T * bg;
  last_out[r] = T;
  rgb_d_out[3 * r] = dr + Td * bg; rgb_d_out[3 * r + 1] = dg + Td * bg; rgb_d_out[3 * r + 2] = db + Td * bg;
  last_d_out[r] = Td;
}

}  // namespace apn

using namespace apn;

// ray_ws: 2 * n_rays int32 scratch (segment bounds).
extern "C" int apn_composite(const float* smp12, const float* s_pos4, const int32_t* s_ray, int64_t max_samples,
                             const int32_t* n_samples_dev, int64_t n_rays, float fast_color_thres, float bg,
                             float* rgb_marched, float* rgb_marched_direct, float* depth, float* weights_vis,
                             float* alphainv_last, float* alphainv_last_direct, int32_t* ray_ws, void* stream) {
  if (n_rays <= 0 || !ray_ws || !rgb_marched || !rgb_marched_direct || !depth || !weights_vis || !alphainv_last ||
      !alphainv_last_direct)
    return APN_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  int* beg = ray_ws;
  int* end = ray_ws + n_rays;
  APN_TRY(fill_i32(ray_ws, 0, n_rays * 2, s));
  if (max_samples > 0)
    hipLaunchKernelGGL(k_ray_bounds, dim3(ceil_div(max_samples, 256)), dim3(256), 0, s, s_ray, n_samples_dev, beg,
                       end);
#ifdef APN_DEBUG_BUILD
  static const bool per_ray = [] {   // A/B: APN_COMPOSITE=seq runs the one-ray-per-thread walk from global
    const char* e = apn_env("APN_COMPOSITE");
    return e && e[0] == 's';
  }();
  if (per_ray)
    hipLaunchKernelGGL(k_composite, dim3(ceil_div(n_rays, 256)), dim3(256), 0, s, (const float4*)smp12,
                       (const float4*)s_pos4, beg, end, n_rays, fast_color_thres, fast_color_thres > 0.f ? 1 : 0, bg,
                       rgb_marched, rgb_marched_direct, depth, weights_vis, alphainv_last, alphainv_last_direct);
  else
#endif
    hipLaunchKernelGGL(k_composite_lds, dim3(ceil_div(n_rays, 64)), dim3(64), 0, s, (const float4*)smp12,
                       (const float4*)s_pos4, beg, end, n_rays, fast_color_thres, fast_color_thres > 0.f ? 1 : 0, bg,
                       rgb_marched, rgb_marched_direct, depth, weights_vis, alphainv_last, alphainv_last_direct);
  return launch_status();
}
