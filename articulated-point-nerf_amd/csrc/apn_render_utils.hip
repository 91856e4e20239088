// Ray sampling and compositing ops: the drop-in for the reference's `render_utils_cuda`
// module (lib/cuda/render_utils.cpp:144-155) plus the fused-pipeline sampling stage.
//
// Index-producing arithmetic follows render_utils_kernel.cu op-for-op and this file is
// compiled with -ffp-contract=off, so ray_id / step_id / in-bbox masks / sample positions
// are bit-identical to the CPU oracle (oracle/apn_oracle.py).
#include "apn_common.h"

#include <climits>

namespace apn {

struct RayGeom {
  float sx, sy, sz;   // start = o + d * t_min
  float dx, dy, dz;   // normalised direction
  int n;              // number of steps (>= 1)
};

// render_utils_kernel.cu:11-73 for one ray.
__device__ __forceinline__ RayGeom ray_geom(const float* __restrict__ o3, const float* __restrict__ d3,
                                            const float lo[3], const float hi[3], float near, float far,
                                            float stepdist, float* tmin_out = nullptr,
                                            float* tmax_out = nullptr) {
  const float ox = o3[0], oy = o3[1], oz = o3[2];
  const float rdx = d3[0], rdy = d3[1], rdz = d3[2];
  const float vx = (rdx == 0.f) ? 1e-6f : rdx;
  const float vy = (rdy == 0.f) ? 1e-6f : rdy;
  const float vz = (rdz == 0.f) ? 1e-6f : rdz;
  const float ax = (hi[0] - ox) / vx, ay = (hi[1] - oy) / vy, az = (hi[2] - oz) / vz;
  const float bx = (lo[0] - ox) / vx, by = (lo[1] - oy) / vy, bz = (lo[2] - oz) / vz;
  const float tmin = fmaxf(fminf(fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz)), far), near);
  const float tmax = fmaxf(fminf(fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz)), far), near);
  if (tmin_out) *tmin_out = tmin;
  if (tmax_out) *tmax_out = tmax;
  const float q = ceilf((tmax - tmin) / stepdist);
  RayGeom g;
  g.n = q > 1.f ? (int)q : 1;
  const float rn = sqrtf((rdx * rdx + rdy * rdy) + rdz * rdz);
  g.sx = ox + rdx * tmin; g.sy = oy + rdy * tmin; g.sz = oz + rdz * tmin;
  g.dx = rdx / rn; g.dy = rdy / rn; g.dz = rdz / rn;
  return g;
}

__device__ __forceinline__ bool sample_at(const RayGeom& g, int k, float stepdist, const float lo[3],
                                          const float hi[3], float& px, float& py, float& pz) {
  const float dist = stepdist * (float)k;
  px = g.sx + g.dx * dist; py = g.sy + g.dy * dist; pz = g.sz + g.dz * dist;
  const bool out = (lo[0] > px) | (lo[1] > py) | (lo[2] > pz) | (hi[0] < px) | (hi[1] < py) | (hi[2] < pz);
  return !out;
}

// ---------------------------------------------------------------- reference-mirror ops
__global__ void k_sample_count(const float* __restrict__ ro, const float* __restrict__ rd,
                               const float* __restrict__ xyz_min, const float* __restrict__ xyz_max,
                               float near, float far, float stepdist, int64_t n_rays,
                               float* __restrict__ t_min, float* __restrict__ t_max,
                               int64_t* __restrict__ n_steps, int* __restrict__ cnt) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rays) return;
  const float lo[3] = {xyz_min[0], xyz_min[1], xyz_min[2]};
  const float hi[3] = {xyz_max[0], xyz_max[1], xyz_max[2]};
  float a, b;
  RayGeom g = ray_geom(ro + 3 * r, rd + 3 * r, lo, hi, near, far, stepdist, &a, &b);
  t_min[r] = a; t_max[r] = b;
  n_steps[r] = g.n;
  cnt[r] = g.n;
}

__global__ void k_sample_fill(const float* __restrict__ ro, const float* __restrict__ rd,
                              const float* __restrict__ xyz_min, const float* __restrict__ xyz_max,
                              float near, float far, float stepdist, int64_t n_rays,
                              const int* __restrict__ off, float* __restrict__ pts,
                              uint8_t* __restrict__ mask_out, int64_t* __restrict__ ray_id,
                              int64_t* __restrict__ step_id) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rays) return;
  const float lo[3] = {xyz_min[0], xyz_min[1], xyz_min[2]};
  const float hi[3] = {xyz_max[0], xyz_max[1], xyz_max[2]};
  RayGeom g = ray_geom(ro + 3 * r, rd + 3 * r, lo, hi, near, far, stepdist);
  const int64_t base = off[r];
  for (int k = 0; k < g.n; ++k) {
    float px, py, pz;
    bool in = sample_at(g, k, stepdist, lo, hi, px, py, pz);
    const int64_t i = base + k;
    pts[3 * i] = px; pts[3 * i + 1] = py; pts[3 * i + 2] = pz;
    mask_out[i] = in ? 0 : 1;
    ray_id[i] = r;
    step_id[i] = k;
  }
}

// render_utils_kernel.cu:357-393
__global__ void k_raw2alpha(const float* __restrict__ density, float shift, float interval, int64_t n,
                            float* __restrict__ exp_d, float* __restrict__ alpha) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float e = expf(density[i] + shift);
  exp_d[i] = e;
  alpha[i] = 1.f - powf(1.f + e, -interval);
}

// render_utils_kernel.cu:461-471 + host fix at 489 (i_end of the last ray = n_pts)
__global__ void k_segment_bounds(const int64_t* __restrict__ ray_id, int64_t n, int64_t* __restrict__ i_start,
                                 int64_t* __restrict__ i_end) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (i > 0 && ray_id[i] != ray_id[i - 1]) {
    i_start[ray_id[i]] = i;
    i_end[ray_id[i - 1]] = i;
  }
  if (i == n - 1) i_end[ray_id[i]] = n;
}

// render_utils_kernel.cu:430-459: one ray per thread, T_cum update in double.
__global__ void k_alpha2weight(const float* __restrict__ alpha, int64_t n_rays, float* __restrict__ weight,
                               float* __restrict__ T, float* __restrict__ last,
                               const int64_t* __restrict__ i_start, int64_t* __restrict__ i_end) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rays) return;
  const int64_t s = i_start[r], e = i_end[r];
  float tc = 1.f;
  int64_t i;
  for (i = s; i < e; ++i) {
    const float a = alpha[i];
    T[i] = tc;
    weight[i] = tc * a;
    tc = (float)((double)tc * (1.0 - (double)a));
    if ((double)tc < 1e-3) { ++i; break; }
  }
  i_end[r] = i;
  last[r] = tc;
}

// render_utils_kernel.cu:395-406 (float instantiation). The clamp constant 1e10 is a double, so
// min() returns double and the whole product runs in double, rounded once at the store:
// ((min(e, 1e10) * powf(1 + e, -interval - 1)) * interval) * grad_back.
__global__ void k_raw2alpha_backward(const float* __restrict__ exp_d, const float* __restrict__ grad_back,
                                     float interval, int64_t n, float* __restrict__ grad) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float e = exp_d[i];
  const double m = fmin((double)e, 1e10);
  const float pw = powf(1.f + e, -interval - 1.f);
  grad[i] = (float)(((m * (double)pw) * (double)interval) * (double)grad_back[i]);
}

// render_utils_kernel.cu:507-528: one ray per thread, walking its samples backwards. back_cum
// accumulates in float; 1 - alpha is float, + 1e-10 (double) promotes the division and the
// subtraction to double, rounded at the store. Samples outside [i_start, i_end) keep grad = 0.
__global__ void k_alpha2weight_backward(const float* __restrict__ alpha, const float* __restrict__ weight,
                                        const float* __restrict__ T, const float* __restrict__ last,
                                        const int64_t* __restrict__ i_start, const int64_t* __restrict__ i_end,
                                        int64_t n_rays, const float* __restrict__ grad_weights,
                                        const float* __restrict__ grad_last, float* __restrict__ grad) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rays) return;
  const int64_t s = i_start[r], e = i_end[r];
  float back_cum = grad_last[r] * last[r];
  for (int64_t i = e - 1; i >= s; --i) {
    const float gw = grad_weights[i];
    grad[i] = (float)((double)(gw * T[i]) - (double)back_cum / ((double)(1.f - alpha[i]) + 1e-10));
    back_cum += gw * weight[i];
  }
}

__global__ void k_zero_f32(float* __restrict__ p, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = 0.f;
}

__global__ void k_a2w_init(int64_t n, int64_t n_rays, float* __restrict__ weight, float* __restrict__ T,
                           float* __restrict__ last, int64_t* __restrict__ i_start, int64_t* __restrict__ i_end) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { weight[i] = 0.f; T[i] = 1.f; }
  if (i < n_rays) { last[i] = 1.f; i_start[i] = 0; i_end[i] = 0; }
}

// torch_scatter.segment_coo(reduce='sum') into a zero output, sequential per segment.
__global__ void k_segment_sum(const float* __restrict__ src, int64_t C, int64_t n_out,
                              const int64_t* __restrict__ i_start, const int64_t* __restrict__ i_end,
                              float* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_out * C) return;
  const int64_t r = t / C, c = t % C;
  float acc = 0.f;
  for (int64_t i = i_start[r]; i < i_end[r]; ++i) acc += src[i * C + c];
  out[t] = acc;
}

__global__ void k_zero_i64(int64_t* p, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = 0;
}

// ---------------------------------------------------------------- fused pipeline sampling
// bbox6 = {lo x,y,z, hi x,y,z} of the sampling box (apn_bbox_unpack or the model bbox).
__global__ void k_inbbox_count(const float* __restrict__ ro, const float* __restrict__ rd,
                               const float* __restrict__ bbox6, float near, float far,
                               float stepdist, int64_t n_rays, int* __restrict__ cnt) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rays) return;
  const float lo[3] = {bbox6[0], bbox6[1], bbox6[2]}, hi[3] = {bbox6[3], bbox6[4], bbox6[5]};
  RayGeom g = ray_geom(ro + 3 * r, rd + 3 * r, lo, hi, near, far, stepdist);
  int c = 0;
  for (int k = 0; k < g.n; ++k) {
    float px, py, pz;
    c += sample_at(g, k, stepdist, lo, hi, px, py, pz) ? 1 : 0;
  }
  cnt[r] = c;
}

// frame_info = {min(total, cap), total, total > cap} from the exclusive scan's last entry (written
// by the fill's first thread: the capped fill's own launch)
__device__ __forceinline__ void frame_info_store(int n, int cap, int* __restrict__ info) {
  info[0] = n < cap ? n : cap;
  info[1] = n;
  info[2] = n > cap ? 1 : 0;
}

#ifdef APN_DEBUG_BUILD   // one ray per thread: debug build only (A/B against the block-cooperative fill)
// q_pos[i] = (x, y, z, bits(step_id)); q_ray[i] = ray id. Sorted by ray, then step.
// cap: samples at positions >= cap are not written (the capacity-bounded, sync-free render path:
// apn_inbbox_fill_capped); INT_MAX = every sample.

__global__ void k_inbbox_fill(const float* __restrict__ ro, const float* __restrict__ rd,
                              const float* __restrict__ bbox6, float near, float far,
                              float stepdist, int64_t n_rays, const int* __restrict__ off,
                              float4* __restrict__ q_pos, int* __restrict__ q_ray, int cap, int* __restrict__ info) {
  if (info && blockIdx.x == 0 && threadIdx.x == 0) frame_info_store(off[n_rays], cap, info);
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rays) return;
  int o = off[r];
  if (off[r + 1] == o || o >= cap) return;
  const float lo[3] = {bbox6[0], bbox6[1], bbox6[2]}, hi[3] = {bbox6[3], bbox6[4], bbox6[5]};
  RayGeom g = ray_geom(ro + 3 * r, rd + 3 * r, lo, hi, near, far, stepdist);
  for (int k = 0; k < g.n && o < cap; ++k) {
    float px, py, pz;
    if (sample_at(g, k, stepdist, lo, hi, px, py, pz)) {
      q_pos[o] = make_float4(px, py, pz, __int_as_float(k));
      q_ray[o] = (int)r;
      ++o;
    }
  }
}
#endif  // APN_DEBUG_BUILD

// The same samples, written block-cooperatively (k_inbbox_fill walks one ray per thread, so a
// wave's stores scatter over 64 rays' output ranges: 1.6 TB/s). The block's 256 rays own the
// contiguous output range [off[r0], off[r0 + 256]); thread t puts ray r0 + t's geometry and first
// in-bbox step into LDS, then the block walks the output range with coalesced stores, each slot
// finding its ray by binary search over the block's offsets. A ray's in-bbox steps are contiguous
// (every coordinate of start + dir * (stepdist * k) is monotone in k under rounding), so slot o of
// ray r is step k0[r] + (o - off[r]); positions come from the same ray_geom / sample_at arithmetic.
constexpr int FILL_RAYS = 256;
__global__ __launch_bounds__(FILL_RAYS) void k_inbbox_fill_blk(const float* __restrict__ ro,
                                                             const float* __restrict__ rd,
                                                             const float* __restrict__ bbox6, float near,
                                                             float far, float stepdist, int64_t n_rays,
                                                             const int* __restrict__ off, float4* __restrict__ q_pos,
                                                             int* __restrict__ q_ray, int cap, int* __restrict__ info) {
  __shared__ int sOff[FILL_RAYS + 1];
  __shared__ int sK0[FILL_RAYS];
  __shared__ float sG[6][FILL_RAYS];
  const int64_t r0 = (int64_t)blockIdx.x * FILL_RAYS;
  const int nr = (int)min((int64_t)FILL_RAYS, n_rays - r0);
  const int t = threadIdx.x;
  const float lo[3] = {bbox6[0], bbox6[1], bbox6[2]}, hi[3] = {bbox6[3], bbox6[4], bbox6[5]};
  if (info && blockIdx.x == 0 && t == 0) frame_info_store(off[n_rays], cap, info);   // no launch of its own
  if (t < nr) sOff[t] = off[r0 + t];
  if (t == 0 && nr > 0) sOff[nr] = off[r0 + nr];
  if (t < nr) {
    const int64_t r = r0 + t;
    const RayGeom g = ray_geom(ro + 3 * r, rd + 3 * r, lo, hi, near, far, stepdist);
    int k0 = 0;
    if (off[r + 1] > off[r]) {   // first in-bbox step (0 or 1 in practice: step 0 is on the entry face)
      float px, py, pz;
      while (k0 < g.n && !sample_at(g, k0, stepdist, lo, hi, px, py, pz)) ++k0;
    }
    sK0[t] = k0;
    sG[0][t] = g.sx; sG[1][t] = g.sy; sG[2][t] = g.sz;
    sG[3][t] = g.dx; sG[4][t] = g.dy; sG[5][t] = g.dz;
  }
  __syncthreads();
  if (nr <= 0) return;
  const int ob = sOff[0], oe = min(sOff[nr], cap);
  for (int o = ob + t; o < oe; o += FILL_RAYS) {
    int a = 0, b = nr - 1;   // the largest j with sOff[j] <= o (rays without samples share offsets)
    while (a < b) {
      const int m = (a + b + 1) >> 1;
      if (sOff[m] <= o) a = m; else b = m - 1;
    }
    RayGeom g;
    g.sx = sG[0][a]; g.sy = sG[1][a]; g.sz = sG[2][a];
    g.dx = sG[3][a]; g.dy = sG[4][a]; g.dz = sG[5][a];
    g.n = 0;
    const int k = sK0[a] + (o - sOff[a]);
    float px, py, pz;
    sample_at(g, k, stepdist, lo, hi, px, py, pz);
    q_pos[o] = make_float4(px, py, pz, __int_as_float(k));
    q_ray[o] = (int)(r0 + a);
  }
}

#ifdef APN_DEBUG_BUILD
static bool inbbox_fill_per_ray() {   // A/B: APN_INBBOX_FILL=ray selects the one-ray-per-thread fill
  static const bool v = [] {
    const char* e = apn_env("APN_INBBOX_FILL");
    return e && e[0] == 'r';
  }();
  return v;
}
#define APN_INBBOX_FILL_KERNEL (inbbox_fill_per_ray() ? k_inbbox_fill : k_inbbox_fill_blk)
#else
#define APN_INBBOX_FILL_KERNEL k_inbbox_fill_blk
#endif

// bbox_ord: ordered-int encoded [min x,y,z, max x,y,z] of the warped cloud (apn_lbs.hip);
// padded by query_radius exactly as temporalpoints.py:424 (float32 subtract / add).
__global__ void k_bbox_unpack(const int* __restrict__ bbox_ord, float qr, float* __restrict__ out6) {
  if (threadIdx.x < 3) out6[threadIdx.x] = ordered_to_float(bbox_ord[threadIdx.x]) - qr;
  else if (threadIdx.x < 6) out6[threadIdx.x] = ordered_to_float(bbox_ord[threadIdx.x]) + qr;
}

}  // namespace apn

using namespace apn;

// ---------------------------------------------------------------- C-ABI
extern "C" int apn_sample_pts_on_rays_count(const float* rays_o, const float* rays_d, const float* xyz_min,
                                            const float* xyz_max, float near, float far, float stepdist,
                                            int64_t n_rays, float* t_min, float* t_max, int64_t* n_steps,
                                            int32_t* offsets, void* workspace, void* stream) {
  if (n_rays < 0 || !offsets || (n_rays > 0 && (!rays_o || !rays_d || !xyz_min || !xyz_max))) return APN_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (n_rays == 0) return scan_exclusive_i32(nullptr, offsets, 0, workspace, s);
  // counts are staged in offsets[] itself? no: scan needs a separate input -> use the tail of workspace
  int* cnt = (int*)((char*)workspace + scan_workspace_bytes(n_rays));
  hipLaunchKernelGGL(k_sample_count, dim3(ceil_div(n_rays, 256)), dim3(256), 0, s, rays_o, rays_d, xyz_min,
                     xyz_max, near, far, stepdist, n_rays, t_min, t_max, n_steps, cnt);
  if (launch_status()) return APN_ERR_HIP;
  return scan_exclusive_i32(cnt, offsets, n_rays, workspace, s);
}

extern "C" size_t apn_sample_pts_on_rays_workspace_bytes(int64_t n_rays) {
  return scan_workspace_bytes(n_rays) + (size_t)(n_rays + 1) * sizeof(int);
}

extern "C" int apn_sample_pts_on_rays_fill(const float* rays_o, const float* rays_d, const float* xyz_min,
                                           const float* xyz_max, float near, float far, float stepdist,
                                           int64_t n_rays, const int32_t* offsets, float* rays_pts,
                                           uint8_t* mask_outbbox, int64_t* ray_id, int64_t* step_id,
                                           void* stream) {
  if (n_rays <= 0) return APN_OK;
  hipLaunchKernelGGL(k_sample_fill, dim3(ceil_div(n_rays, 256)), dim3(256), 0, (hipStream_t)stream, rays_o,
                     rays_d, xyz_min, xyz_max, near, far, stepdist, n_rays, offsets, rays_pts, mask_outbbox,
                     ray_id, step_id);
  return launch_status();
}

extern "C" int apn_raw2alpha(const float* density, float shift, float interval, int64_t n_pts, float* exp_d,
                             float* alpha, void* stream) {
  if (n_pts < 0) return APN_ERR_ARG;
  if (n_pts == 0) return APN_OK;
  hipLaunchKernelGGL(k_raw2alpha, dim3(ceil_div(n_pts, 256)), dim3(256), 0, (hipStream_t)stream, density, shift,
                     interval, n_pts, exp_d, alpha);
  return launch_status();
}

extern "C" int apn_alpha2weight(const float* alpha, const int64_t* ray_id, int64_t n_pts, int64_t n_rays,
                                float* weight, float* T, float* alphainv_last, int64_t* i_start, int64_t* i_end,
                                void* stream) {
  if (n_pts < 0 || n_rays < 0) return APN_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  int64_t m = n_pts > n_rays ? n_pts : n_rays;
  if (m == 0) return APN_OK;
  hipLaunchKernelGGL(k_a2w_init, dim3(ceil_div(m, 256)), dim3(256), 0, s, n_pts, n_rays, weight, T,
                     alphainv_last, i_start, i_end);
  if (n_pts == 0) return launch_status();
  hipLaunchKernelGGL(k_segment_bounds, dim3(ceil_div(n_pts, 256)), dim3(256), 0, s, ray_id, n_pts, i_start, i_end);
  hipLaunchKernelGGL(k_alpha2weight, dim3(ceil_div(n_rays, 256)), dim3(256), 0, s, alpha, n_rays, weight, T,
                     alphainv_last, i_start, i_end);
  return launch_status();
}

extern "C" int apn_raw2alpha_backward(const float* exp_d, const float* grad_back, float interval, int64_t n_pts,
                                      float* grad, void* stream) {
  if (n_pts < 0 || (n_pts > 0 && (!exp_d || !grad_back || !grad))) return APN_ERR_ARG;
  if (n_pts == 0) return APN_OK;
  hipLaunchKernelGGL(k_raw2alpha_backward, dim3(ceil_div(n_pts, 256)), dim3(256), 0, (hipStream_t)stream, exp_d,
                     grad_back, interval, n_pts, grad);
  return launch_status();
}

extern "C" int apn_alpha2weight_backward(const float* alpha, const float* weight, const float* T,
                                         const float* alphainv_last, const int64_t* i_start, const int64_t* i_end,
                                         int64_t n_pts, int64_t n_rays, const float* grad_weights,
                                         const float* grad_last, float* grad, void* stream) {
  if (n_pts < 0 || n_rays < 0) return APN_ERR_ARG;
  if (n_pts > 0 && (!alpha || !weight || !T || !grad_weights || !grad)) return APN_ERR_ARG;
  if (n_rays > 0 && (!alphainv_last || !i_start || !i_end || !grad_last)) return APN_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (n_pts == 0) return APN_OK;
  hipLaunchKernelGGL(k_zero_f32, dim3(ceil_div(n_pts, 256)), dim3(256), 0, s, grad, n_pts);
  if (n_rays > 0)
    hipLaunchKernelGGL(k_alpha2weight_backward, dim3(ceil_div(n_rays, 256)), dim3(256), 0, s, alpha, weight, T,
                       alphainv_last, i_start, i_end, n_rays, grad_weights, grad_last, grad);
  return launch_status();
}

extern "C" int apn_segment_sum(const float* src, const int64_t* index, int64_t n_pts, int64_t channels,
                               int64_t n_out, float* out, int64_t* seg_workspace, void* stream) {
  if (n_pts < 0 || channels <= 0 || n_out < 0) return APN_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (n_out == 0) return APN_OK;
  int64_t* i_start = seg_workspace;
  int64_t* i_end = seg_workspace + n_out;
  hipLaunchKernelGGL(k_zero_i64, dim3(ceil_div(2 * n_out, 256)), dim3(256), 0, s, seg_workspace, 2 * n_out);
  if (n_pts > 0)
    hipLaunchKernelGGL(k_segment_bounds, dim3(ceil_div(n_pts, 256)), dim3(256), 0, s, index, n_pts, i_start, i_end);
  hipLaunchKernelGGL(k_segment_sum, dim3(ceil_div(n_out * channels, 256)), dim3(256), 0, s, src, channels, n_out,
                     i_start, i_end, out);
  return launch_status();
}

extern "C" int apn_inbbox_count(const float* rays_o, const float* rays_d, const float* bbox6, float near, float far,
                                float stepdist, int64_t n_rays, int32_t* offsets, void* workspace, void* stream) {
  if (n_rays <= 0) return APN_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  int* cnt = (int*)((char*)workspace + scan_workspace_bytes(n_rays));
  hipLaunchKernelGGL(k_inbbox_count, dim3(ceil_div(n_rays, 256)), dim3(256), 0, s, rays_o, rays_d, bbox6, near,
                     far, stepdist, n_rays, cnt);
  if (launch_status()) return APN_ERR_HIP;
  return scan_exclusive_i32(cnt, offsets, n_rays, workspace, s);
}

extern "C" int apn_inbbox_fill(const float* rays_o, const float* rays_d, const float* bbox6, float near, float far,
                               float stepdist, int64_t n_rays, const int32_t* offsets, float* q_pos4, int32_t* q_ray,
                               void* stream) {
  if (n_rays <= 0) return APN_ERR_ARG;
  hipLaunchKernelGGL(APN_INBBOX_FILL_KERNEL, dim3(ceil_div(n_rays, 256)), dim3(256),
                     0, (hipStream_t)stream, rays_o, rays_d, bbox6, near, far, stepdist, n_rays, offsets,
                     (float4*)q_pos4, q_ray, INT_MAX, nullptr);
  return launch_status();
}

extern "C" int apn_inbbox_fill_capped(const float* rays_o, const float* rays_d, const float* bbox6, float near,
                                      float far, float stepdist, int64_t n_rays, const int32_t* offsets,
                                      int64_t capacity, float* q_pos4, int32_t* q_ray, int32_t* frame_info,
                                      void* stream) {
  if (n_rays <= 0 || capacity < 0 || capacity > INT_MAX || !frame_info) return APN_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(APN_INBBOX_FILL_KERNEL, dim3(ceil_div(n_rays, 256)), dim3(256),
                     0, s, rays_o, rays_d, bbox6, near, far, stepdist, n_rays, offsets, (float4*)q_pos4, q_ray,
                     (int)capacity, frame_info);
  return launch_status();
}

namespace apn {
// One thread per gathered ray: 3 x 12 B in, 3 x 12 B out.
__global__ void k_gather_rays(const float* __restrict__ a, const float* __restrict__ b, const float* __restrict__ c,
                              const int64_t* __restrict__ idx, int64_t n, float* __restrict__ oa,
                              float* __restrict__ ob, float* __restrict__ oc) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t r = idx[i];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    oa[3 * i + k] = a[3 * r + k];
    ob[3 * i + k] = b[3 * r + k];
    oc[3 * i + k] = c[3 * r + k];
  }
}
}  // namespace apn

extern "C" int apn_gather_rays(const float* rays_o, const float* rays_d, const float* viewdirs, const int64_t* index,
                               int64_t n, float* out_o, float* out_d, float* out_v, void* stream) {
  if (n < 0 || (n > 0 && (!rays_o || !rays_d || !viewdirs || !index || !out_o || !out_d || !out_v)))
    return APN_ERR_ARG;
  if (n == 0) return APN_OK;
  hipLaunchKernelGGL(k_gather_rays, dim3(ceil_div(n, 256)), dim3(256), 0, (hipStream_t)stream, rays_o, rays_d,
                     viewdirs, index, n, out_o, out_d, out_v);
  return launch_status();
}

extern "C" int apn_bbox_unpack(const int32_t* bbox_ord, float query_radius, float* out6, void* stream) {
  hipLaunchKernelGGL(k_bbox_unpack, dim3(1), dim3(64), 0, (hipStream_t)stream, bbox_ord, query_radius, out6);
  return launch_status();
}
