// Radius-bounded exact kNN over the warped cloud: the replacement for the reference's
// pykeops brute-force `Kmin_argKmin(K=8)` + radius filter (temporalpoints.py:433-447).
//
// Exactness: a sample survives the reference filter iff its 8th-nearest squared distance
// is <= query_radius. Every neighbour of a survivor therefore lies within r = sqrt(qr).
// The uniform grid has cells of side >= r * (1 + 2^-10), so all points within r of a query
// lie in the 27 cells around it, and the top-8 (by float32 (dx*dx+dy*dy)+dz*dz, ties by
// index) over those cells equals the global top-8 for every survivor. Non-survivors are
// discarded by the reference anyway. Distances use -ffp-contract=off arithmetic, so they
// equal the reference's recomputed `to_nn` bit-for-bit.
//
// Grid build: counting sort (count -> scan -> scatter) of float4 {x,y,z,bits(idx)}; the
// cells of one x-row are contiguous, so a query scans 9 contiguous ranges.
#include "apn_common.h"

namespace apn {

struct GridParams {
  float ox, oy, oz, h;        // fine grid origin and cell side
  float inv_h, r, r2, pad0;   // search radius r = sqrt(query_radius), r2 = query_radius
  int dx, dy, dz, nf;         // fine grid dims and cell count
  int cf, cdx, cdy, cdz;      // fine cells per coarse cell (coarse side >= r), coarse dims
  int nc, kmax, pad1, pad2;   // coarse cell count, ring limit (kmax * h >= r)
};

constexpr int KNN_K = 8;
constexpr int KNN_THREADS = 256;
constexpr int KNN_SUBDIV = 8;   // fine cell side = r / KNN_SUBDIV (before the cell cap)

__device__ __forceinline__ int floor_div(int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

__global__ void k_grid_params(const int* __restrict__ bbox_ord, float qr, int cap, int subdiv,
                              GridParams* __restrict__ gp) {
  if (threadIdx.x != 0) return;
  float lo[3], hi[3];
  for (int a = 0; a < 3; ++a) {
    lo[a] = ordered_to_float(bbox_ord[a]);
    hi[a] = ordered_to_float(bbox_ord[3 + a]);
  }
  const float r = sqrtf(qr);
  float h = r / (float)subdiv;
  int d[3];
  for (int it = 0; it < 64; ++it) {
    double prod = 1.0;
    for (int a = 0; a < 3; ++a) {
      d[a] = (int)floorf((hi[a] - lo[a]) / h) + 1;
      prod *= (double)d[a];
    }
    if (prod <= (double)cap) break;
    h *= (float)(cbrt(prod / (double)cap) * 1.01);
  }
  GridParams g;
  g.ox = lo[0]; g.oy = lo[1]; g.oz = lo[2];
  g.h = h; g.inv_h = 1.f / h; g.r = r; g.r2 = qr; g.pad0 = 0.f;
  g.dx = d[0]; g.dy = d[1]; g.dz = d[2];
  g.nf = d[0] * d[1] * d[2];
  g.cf = max(1, (int)ceilf(r * 1.0002f / h));
  g.cdx = (d[0] + g.cf - 1) / g.cf; g.cdy = (d[1] + g.cf - 1) / g.cf; g.cdz = (d[2] + g.cf - 1) / g.cf;
  g.nc = g.cdx * g.cdy * g.cdz;
  g.kmax = g.cf;
  g.pad1 = g.pad2 = 0;
  *gp = g;
}

__device__ __forceinline__ int cell_coord(float v, float o, float inv_h, int dim) {
  int i = (int)floorf((v - o) * inv_h);
  return min(max(i, 0), dim - 1);
}

__global__ void k_grid_count(const float* __restrict__ xyz, int64_t N, const GridParams* __restrict__ gp,
                             int* __restrict__ counts, int* __restrict__ ccount, int* __restrict__ pcell) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const GridParams g = *gp;
  const int cx = cell_coord(xyz[3 * n], g.ox, g.inv_h, g.dx);
  const int cy = cell_coord(xyz[3 * n + 1], g.oy, g.inv_h, g.dy);
  const int cz = cell_coord(xyz[3 * n + 2], g.oz, g.inv_h, g.dz);
  const int cell = (cz * g.dy + cy) * g.dx + cx;
  pcell[n] = cell;
  atomicAdd(counts + cell, 1);
  atomicAdd(ccount + ((cz / g.cf) * g.cdy + cy / g.cf) * g.cdx + cx / g.cf, 1);
}

__global__ void k_grid_scatter(const float* __restrict__ xyz, int64_t N, const int* __restrict__ pcell,
                               const int* __restrict__ cell_start, int* __restrict__ cursor,
                               float4* __restrict__ sorted) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const int cell = pcell[n];
  const int pos = cell_start[cell] + atomicAdd(cursor + cell, 1);
  sorted[pos] = make_float4(xyz[3 * n], xyz[3 * n + 1], xyz[3 * n + 2], __int_as_float((int)n));
}

__device__ __forceinline__ bool knn_less(float d, int i, float bd, int bi) {
  return d < bd || (d == bd && i < bi);
}

template <int K>
__device__ __forceinline__ void knn_insert(float d, int id, float (&bd)[K], int (&bi)[K]) {
  if (!knn_less(d, id, bd[K - 1], bi[K - 1])) return;
  bd[K - 1] = d; bi[K - 1] = id;
#pragma unroll
  for (int k = K - 1; k > 0; --k) {
    if (knn_less(bd[k], bi[k], bd[k - 1], bi[k - 1])) {
      float td = bd[k]; bd[k] = bd[k - 1]; bd[k - 1] = td;
      int ti = bi[k]; bi[k] = bi[k - 1]; bi[k - 1] = ti;
    }
  }
}

// Scan fine cells [x0,x1] of row (y,z) (contiguous in the sorted array) into the top-K.
template <int K, bool EXCL>
__device__ __forceinline__ void scan_cells(const int* __restrict__ cell_start, const float4* __restrict__ sorted,
                                           int c0, int c1, float qx, float qy, float qz, float dmax2, int excl,
                                           float (&bd)[K], int (&bi)[K]) {
  const int b = cell_start[c0], e = cell_start[c1 + 1];
  for (int p = b; p < e; ++p) {
    const float4 P = sorted[p];
    const float ddx = qx - P.x, ddy = qy - P.y, ddz = qz - P.z;
    const float d = (ddx * ddx + ddy * ddy) + ddz * ddz;
    const int id = __float_as_int(P.w);
    if (d <= dmax2 && (!EXCL || id != excl)) knn_insert<K>(d, id, bd, bi);
  }
}

// Cells at Chebyshev ring distance exactly k around fine cell (fx,fy,fz), clamped to the grid.
template <int K, bool EXCL>
__device__ __forceinline__ void scan_ring(const GridParams& g, const int* __restrict__ cell_start,
                                          const float4* __restrict__ sorted, int fx, int fy, int fz, int k,
                                          float qx, float qy, float qz, float dmax2, int excl, float (&bd)[K],
                                          int (&bi)[K]) {
  const int z0 = max(fz - k, 0), z1 = min(fz + k, g.dz - 1);
  const int y0 = max(fy - k, 0), y1 = min(fy + k, g.dy - 1);
  const int xa = fx - k, xb = fx + k;
  const int x0 = max(xa, 0), x1 = min(xb, g.dx - 1);
  if (x0 > x1) return;
  for (int z = z0; z <= z1; ++z) {
    const bool zs = (z == fz - k) || (z == fz + k);
    for (int y = y0; y <= y1; ++y) {
      const int row = (z * g.dy + y) * g.dx;
      if (zs || y == fy - k || y == fy + k) {
        scan_cells<K, EXCL>(cell_start, sorted, row + x0, row + x1, qx, qy, qz, dmax2, excl, bd, bi);
      } else {
        if (xa >= 0) scan_cells<K, EXCL>(cell_start, sorted, row + xa, row + xa, qx, qy, qz, dmax2, excl, bd, bi);
        if (xb < g.dx && k > 0)
          scan_cells<K, EXCL>(cell_start, sorted, row + xb, row + xb, qx, qy, qz, dmax2, excl, bd, bi);
      }
    }
  }
}

// One in-bbox sample per thread.
//  1. coarse rejection: fewer than K points in the 27 coarse cells (side >= r) around the
//     sample => fewer than K points within r => not a survivor;
//  2. ring search over fine cells, k = 0..kmax: after ring k every point closer than k*h is
//     found, so the search stops exactly once the K-th best is closer than k*h(1-1e-4), and at
//     kmax (kmax*h >= r) every point within r has been seen.
// Survivors are compacted per block (order preserved) into the block's slot range
// [blockIdx*256, ...); blk_cnt[blockIdx] = survivors in the block.
__global__ __launch_bounds__(KNN_THREADS) void k_knn_radius(
    const float4* __restrict__ q_pos, const int* __restrict__ q_ray, const int* __restrict__ n_q_dev,
    const GridParams* __restrict__ gp, const int* __restrict__ cell_start, const int* __restrict__ ccount,
    const float4* __restrict__ sorted, float4* __restrict__ t_pos, int* __restrict__ t_ray,
    int* __restrict__ t_nbr, int* __restrict__ blk_cnt) {
  __shared__ int wave_cnt[KNN_THREADS / 64];
  const int nq = *n_q_dev;
  const int i = blockIdx.x * KNN_THREADS + threadIdx.x;
  float bd[KNN_K];
  int bi[KNN_K];
#pragma unroll
  for (int k = 0; k < KNN_K; ++k) { bd[k] = INFINITY; bi[k] = 0x7fffffff; }
  float4 q = make_float4(0.f, 0.f, 0.f, 0.f);
  const GridParams g = *gp;
  if (i < nq) {
    q = q_pos[i];
    const int fx = (int)floorf((q.x - g.ox) * g.inv_h);
    const int fy = (int)floorf((q.y - g.oy) * g.inv_h);
    const int fz = (int)floorf((q.z - g.oz) * g.inv_h);
    const int cx = floor_div(fx, g.cf), cy = floor_div(fy, g.cf), cz = floor_div(fz, g.cf);
    int cnt = 0;
    for (int z = max(cz - 1, 0); z <= min(cz + 1, g.cdz - 1); ++z)
      for (int y = max(cy - 1, 0); y <= min(cy + 1, g.cdy - 1); ++y)
        for (int x = max(cx - 1, 0); x <= min(cx + 1, g.cdx - 1); ++x) cnt += ccount[(z * g.cdy + y) * g.cdx + x];
    if (cnt >= KNN_K) {
      for (int k = 0; k <= g.kmax; ++k) {
        scan_ring<KNN_K, false>(g, cell_start, sorted, fx, fy, fz, k, q.x, q.y, q.z, g.r2, -1, bd, bi);
        const float gk = (float)k * g.h * (1.f - 1e-4f);
        if (bd[KNN_K - 1] < gk * gk) break;
      }
    }
  }
  const bool surv = (i < nq) && (bd[KNN_K - 1] <= g.r2);
  // block-level order-preserving compaction
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const unsigned long long bal = __ballot(surv);
  const int before = __popcll(bal & ((1ull << lane) - 1ull));
  if (lane == 0) wave_cnt[wid] = __popcll(bal);
  __syncthreads();
  int base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < KNN_THREADS / 64; ++w) {
    base += (w < wid) ? wave_cnt[w] : 0;
    tot += wave_cnt[w];
  }
  if (surv) {
    const int slot = blockIdx.x * KNN_THREADS + base + before;
    t_pos[slot] = q;
    t_ray[slot] = q_ray[i];
    int4* nb = (int4*)(t_nbr + (int64_t)slot * KNN_K);
    nb[0] = make_int4(bi[0], bi[1], bi[2], bi[3]);
    nb[1] = make_int4(bi[4], bi[5], bi[6], bi[7]);
  }
  if (threadIdx.x == 0) blk_cnt[blockIdx.x] = tot;
}

__global__ __launch_bounds__(KNN_THREADS) void k_knn_compact(
    const float4* __restrict__ t_pos, const int* __restrict__ t_ray, const int* __restrict__ t_nbr,
    const int* __restrict__ blk_cnt, const int* __restrict__ blk_off, float4* __restrict__ s_pos,
    int* __restrict__ s_ray, int* __restrict__ s_nbr) {
  const int t = threadIdx.x;
  if (t >= blk_cnt[blockIdx.x]) return;
  const int src = blockIdx.x * KNN_THREADS + t;
  const int dst = blk_off[blockIdx.x] + t;
  s_pos[dst] = t_pos[src];
  s_ray[dst] = t_ray[src];
  const int4* a = (const int4*)(t_nbr + (int64_t)src * KNN_K);
  int4* b = (int4*)(s_nbr + (int64_t)dst * KNN_K);
  b[0] = a[0];
  b[1] = a[1];
}

// Nearest *other* point for every canonical point (temporalpoints.py:104-111: column 1 of the
// self-inclusive argKmin is the nearest other point, or a duplicate at distance 0). Ring
// search over the whole grid with the same exact stopping rule; brute force if the grid runs
// out. Output: sqrt(d2 + eps) per point.
__global__ void k_nn1(const float* __restrict__ xyz, int64_t N, const GridParams* __restrict__ gp,
                      const int* __restrict__ cell_start, const float4* __restrict__ sorted, float eps,
                      float* __restrict__ nn_dist) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const GridParams g = *gp;
  const float qx = xyz[3 * n], qy = xyz[3 * n + 1], qz = xyz[3 * n + 2];
  const int fx = cell_coord(qx, g.ox, g.inv_h, g.dx), fy = cell_coord(qy, g.oy, g.inv_h, g.dy);
  const int fz = cell_coord(qz, g.oz, g.inv_h, g.dz);
  float bd[1] = {INFINITY};
  int bi[1] = {0x7fffffff};
  const int kend = max(g.dx, max(g.dy, g.dz));
  bool done = false;
  for (int k = 0; k <= kend && k <= 64; ++k) {
    scan_ring<1, true>(g, cell_start, sorted, fx, fy, fz, k, qx, qy, qz, INFINITY, (int)n, bd, bi);
    const float gk = (float)k * g.h * (1.f - 1e-4f);
    if (bd[0] < gk * gk) { done = true; break; }
  }
  float best = bd[0];
  if (!done) {
    best = INFINITY;
    for (int64_t m = 0; m < N; ++m) {
      if (m == n) continue;
      const float ddx = qx - xyz[3 * m], ddy = qy - xyz[3 * m + 1], ddz = qz - xyz[3 * m + 2];
      best = fminf(best, (ddx * ddx + ddy * ddy) + ddz * ddz);
    }
  }
  nn_dist[n] = sqrtf(best + eps);
}

__global__ void k_bbox_from_points(const float* __restrict__ xyz, int64_t N, int* __restrict__ bbox_ord) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  if (n < N)
    for (int a = 0; a < 3; ++a) lo[a] = hi[a] = xyz[3 * n + a];
  for (int a = 0; a < 3; ++a) {
    float l = lo[a], h = hi[a];
    for (int o = 32; o > 0; o >>= 1) {
      l = fminf(l, __shfl_xor(l, o, 64));
      h = fmaxf(h, __shfl_xor(h, o, 64));
    }
    if ((threadIdx.x & 63) == 0 && l <= h) {
      atomicMin(bbox_ord + a, float_to_ordered(l));
      atomicMax(bbox_ord + 3 + a, float_to_ordered(h));
    }
  }
}

__global__ void k_bbox_init2(int* bbox_ord) {
  if (threadIdx.x < 3) bbox_ord[threadIdx.x] = 0x7f800000;
  else if (threadIdx.x < 6) bbox_ord[threadIdx.x] = (int)0x807fffff;
}

}  // namespace apn

using namespace apn;

// Workspace layout for apn_grid_build (bytes, each region 256-B aligned):
//   GridParams | counts[cap] | cell_start[cap+1] | cursor[cap] | pcell[N] | ccount[cap] | scan ws
static size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

extern "C" size_t apn_grid_workspace_bytes(int64_t n_points, int32_t cell_cap) {
  return al256(sizeof(GridParams)) + al256((size_t)cell_cap * 4) + al256((size_t)(cell_cap + 1) * 4) +
         al256((size_t)cell_cap * 4) + al256((size_t)n_points * 4) + al256((size_t)cell_cap * 4) +
         al256(scan_workspace_bytes(cell_cap));
}

struct GridWs {
  GridParams* gp; int* counts; int* cell_start; int* cursor; int* pcell; int* ccount; void* scan;
};
static GridWs grid_ws(void* ws, int64_t N, int cap) {
  char* p = (char*)ws;
  GridWs w;
  w.gp = (GridParams*)p; p += al256(sizeof(GridParams));
  w.counts = (int*)p; p += al256((size_t)cap * 4);
  w.cell_start = (int*)p; p += al256((size_t)(cap + 1) * 4);
  w.cursor = (int*)p; p += al256((size_t)cap * 4);
  w.pcell = (int*)p; p += al256((size_t)N * 4);
  w.ccount = (int*)p; p += al256((size_t)cap * 4);
  w.scan = p;
  return w;
}

extern "C" int apn_grid_build(const float* xyz, int64_t n_points, const int32_t* bbox_ord, float query_radius,
                              int32_t cell_cap, float* sorted_pts4, void* workspace, void* stream) {
  if (n_points <= 0 || cell_cap <= 0 || !xyz || !bbox_ord || !sorted_pts4 || !workspace) return APN_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  GridWs w = grid_ws(workspace, n_points, cell_cap);
  APN_HIP_TRY(hipMemsetAsync(w.counts, 0, (size_t)cell_cap * 4, s));
  APN_HIP_TRY(hipMemsetAsync(w.cursor, 0, (size_t)cell_cap * 4, s));
  APN_HIP_TRY(hipMemsetAsync(w.ccount, 0, (size_t)cell_cap * 4, s));
  hipLaunchKernelGGL(k_grid_params, dim3(1), dim3(64), 0, s, bbox_ord, query_radius, cell_cap, KNN_SUBDIV, w.gp);
  hipLaunchKernelGGL(k_grid_count, dim3(ceil_div(n_points, 256)), dim3(256), 0, s, xyz, n_points, w.gp, w.counts,
                     w.ccount, w.pcell);
  int st = scan_exclusive_i32(w.counts, w.cell_start, cell_cap, w.scan, s);
  if (st) return st;
  hipLaunchKernelGGL(k_grid_scatter, dim3(ceil_div(n_points, 256)), dim3(256), 0, s, xyz, n_points, w.pcell,
                     w.cell_start, w.cursor, (float4*)sorted_pts4);
  return launch_status();
}

extern "C" size_t apn_knn_workspace_bytes(int64_t n_queries) {
  int64_t nb = (n_queries + KNN_THREADS - 1) / KNN_THREADS;
  size_t slots = (size_t)nb * KNN_THREADS;
  return al256(slots * 16) + al256(slots * 4) + al256(slots * 4 * KNN_K) + al256((size_t)(nb + 1) * 4) +
         al256((size_t)(nb + 1) * 4) + al256(scan_workspace_bytes(nb));
}

// Queries: q_pos4[n_queries] {x,y,z,bits(step)} and q_ray. n_queries is an upper bound used for
// the launch; the live count is read on device from *n_queries_dev. Survivors (sorted by query
// order) go to s_pos4/s_ray/s_nbr and their count to *n_survivors_dev.
extern "C" int apn_knn_radius(const float* q_pos4, const int32_t* q_ray, int64_t n_queries,
                              const int32_t* n_queries_dev, const void* grid_workspace, int64_t n_points,
                              int32_t cell_cap, const float* sorted_pts4, float query_radius, float* s_pos4,
                              int32_t* s_ray, int32_t* s_nbr, int32_t* n_survivors_dev, void* workspace,
                              void* stream) {
  if (n_queries < 0 || !grid_workspace || !workspace) return APN_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (n_queries == 0) {
    APN_HIP_TRY(hipMemsetAsync(n_survivors_dev, 0, 4, s));
    return launch_status();
  }
  GridWs g = grid_ws((void*)grid_workspace, n_points, cell_cap);
  const int nb = ceil_div(n_queries, KNN_THREADS);
  const size_t slots = (size_t)nb * KNN_THREADS;
  char* p = (char*)workspace;
  float4* t_pos = (float4*)p; p += al256(slots * 16);
  int* t_ray = (int*)p; p += al256(slots * 4);
  int* t_nbr = (int*)p; p += al256(slots * 4 * KNN_K);
  int* blk_cnt = (int*)p; p += al256((size_t)(nb + 1) * 4);
  int* blk_off = (int*)p; p += al256((size_t)(nb + 1) * 4);
  void* sws = p;
  hipLaunchKernelGGL(k_knn_radius, dim3(nb), dim3(KNN_THREADS), 0, s, (const float4*)q_pos4, q_ray, n_queries_dev,
                     g.gp, g.cell_start, g.ccount, (const float4*)sorted_pts4, t_pos, t_ray, t_nbr, blk_cnt);
  int st = scan_exclusive_i32(blk_cnt, blk_off, nb, sws, s);
  if (st) return st;
  hipLaunchKernelGGL(k_knn_compact, dim3(nb), dim3(KNN_THREADS), 0, s, t_pos, t_ray, t_nbr, blk_cnt, blk_off,
                     (float4*)s_pos4, s_ray, s_nbr);
  APN_HIP_TRY(hipMemcpyAsync(n_survivors_dev, blk_off + nb, 4, hipMemcpyDeviceToDevice, s));
  return launch_status();
}

// Construction-time: per-point nearest-other distance sqrt(d2 + eps) over the canonical cloud.
extern "C" int apn_nn1_distance(const float* xyz, int64_t n_points, float eps, int32_t cell_cap, float* nn_dist,
                                float* sorted_pts4, int32_t* bbox_ord, void* grid_workspace, void* stream) {
  if (n_points <= 0) return APN_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_bbox_init2, dim3(1), dim3(64), 0, s, bbox_ord);
  hipLaunchKernelGGL(k_bbox_from_points, dim3(ceil_div(n_points, 256)), dim3(256), 0, s, xyz, n_points, bbox_ord);
  // cell side sqrt(0.01) unless the cap forces it larger
  int st = apn_grid_build(xyz, n_points, bbox_ord, 0.01f, cell_cap, sorted_pts4, grid_workspace, stream);
  if (st) return st;
  GridWs g = grid_ws(grid_workspace, n_points, cell_cap);
  hipLaunchKernelGGL(k_nn1, dim3(ceil_div(n_points, 256)), dim3(256), 0, s, xyz, n_points, g.gp, g.cell_start,
                     (const float4*)sorted_pts4, eps, nn_dist);
  return launch_status();
}
