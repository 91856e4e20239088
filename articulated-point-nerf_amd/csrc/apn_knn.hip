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
  float ox, oy, oz, inv_c;
  int dx, dy, dz, ncells;
  float c, pad0, pad1, pad2;
};

constexpr int KNN_K = 8;
constexpr int KNN_THREADS = 256;

__global__ void k_grid_params(const int* __restrict__ bbox_ord, float qr, int cap, GridParams* __restrict__ gp) {
  if (threadIdx.x != 0) return;
  float lo[3], hi[3];
  for (int a = 0; a < 3; ++a) {
    lo[a] = ordered_to_float(bbox_ord[a]);
    hi[a] = ordered_to_float(bbox_ord[3 + a]);
  }
  float c = sqrtf(qr) * 1.0009765625f;
  int d[3];
  for (int it = 0; it < 64; ++it) {
    double prod = 1.0;
    for (int a = 0; a < 3; ++a) {
      d[a] = (int)floorf((hi[a] - lo[a]) / c) + 1;
      prod *= (double)d[a];
    }
    if (prod <= (double)cap) break;
    c *= (float)(cbrt(prod / (double)cap) * 1.01);
  }
  GridParams g;
  g.ox = lo[0]; g.oy = lo[1]; g.oz = lo[2];
  g.c = c; g.inv_c = 1.f / c;
  g.dx = d[0]; g.dy = d[1]; g.dz = d[2];
  g.ncells = d[0] * d[1] * d[2];
  g.pad0 = g.pad1 = g.pad2 = 0.f;
  *gp = g;
}

__device__ __forceinline__ int cell_coord(float v, float o, float inv_c, int dim) {
  int i = (int)floorf((v - o) * inv_c);
  return min(max(i, 0), dim - 1);
}

__global__ void k_grid_count(const float* __restrict__ xyz, int64_t N, const GridParams* __restrict__ gp,
                             int* __restrict__ counts, int* __restrict__ pcell) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const GridParams g = *gp;
  const int cx = cell_coord(xyz[3 * n], g.ox, g.inv_c, g.dx);
  const int cy = cell_coord(xyz[3 * n + 1], g.oy, g.inv_c, g.dy);
  const int cz = cell_coord(xyz[3 * n + 2], g.oz, g.inv_c, g.dz);
  const int cell = (cz * g.dy + cy) * g.dx + cx;
  pcell[n] = cell;
  atomicAdd(counts + cell, 1);
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

// One in-bbox sample per thread. Survivors are compacted per block (order preserved) into
// the block's slot range [blockIdx*256, ...); blk_cnt[blockIdx] = survivors in the block.
__global__ __launch_bounds__(KNN_THREADS) void k_knn_radius(
    const float4* __restrict__ q_pos, const int* __restrict__ q_ray, const int* __restrict__ n_q_dev,
    const GridParams* __restrict__ gp, const int* __restrict__ cell_start, const float4* __restrict__ sorted,
    float qr, float4* __restrict__ t_pos, int* __restrict__ t_ray, int* __restrict__ t_nbr,
    int* __restrict__ blk_cnt) {
  __shared__ int wave_cnt[KNN_THREADS / 64];
  const int nq = *n_q_dev;
  const int i = blockIdx.x * KNN_THREADS + threadIdx.x;
  float bd[KNN_K];
  int bi[KNN_K];
#pragma unroll
  for (int k = 0; k < KNN_K; ++k) { bd[k] = INFINITY; bi[k] = 0x7fffffff; }
  float4 q = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < nq) {
    q = q_pos[i];
    const GridParams g = *gp;
    const int cx = (int)floorf((q.x - g.ox) * g.inv_c);
    const int cy = (int)floorf((q.y - g.oy) * g.inv_c);
    const int cz = (int)floorf((q.z - g.oz) * g.inv_c);
    const int x0 = max(cx - 1, 0), x1 = min(cx + 1, g.dx - 1);
    const int y0 = max(cy - 1, 0), y1 = min(cy + 1, g.dy - 1);
    const int z0 = max(cz - 1, 0), z1 = min(cz + 1, g.dz - 1);
    if (x0 <= x1) {
      for (int z = z0; z <= z1; ++z) {
        for (int y = y0; y <= y1; ++y) {
          const int rowc = (z * g.dy + y) * g.dx;
          const int b = cell_start[rowc + x0], e = cell_start[rowc + x1 + 1];
          for (int p = b; p < e; ++p) {
            const float4 P = sorted[p];
            const float ddx = q.x - P.x, ddy = q.y - P.y, ddz = q.z - P.z;
            const float d = (ddx * ddx + ddy * ddy) + ddz * ddz;
            if (d <= qr) knn_insert<KNN_K>(d, __float_as_int(P.w), bd, bi);
          }
        }
      }
    }
  }
  const bool surv = (i < nq) && (bd[KNN_K - 1] <= qr);
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

// Nearest *other* point for every canonical point (temporalpoints.py:104-111, column 1 of
// the self-inclusive argKmin). Grid search when the nearest neighbour is within one cell,
// brute force otherwise. Output: sqrt(d2 + eps) per point.
__global__ void k_nn1(const float* __restrict__ xyz, int64_t N, const GridParams* __restrict__ gp,
                      const int* __restrict__ cell_start, const float4* __restrict__ sorted, float eps,
                      float* __restrict__ nn_dist) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const GridParams g = *gp;
  const float qx = xyz[3 * n], qy = xyz[3 * n + 1], qz = xyz[3 * n + 2];
  const int cx = cell_coord(qx, g.ox, g.inv_c, g.dx), cy = cell_coord(qy, g.oy, g.inv_c, g.dy);
  const int cz = cell_coord(qz, g.oz, g.inv_c, g.dz);
  float best = INFINITY;
  for (int z = max(cz - 1, 0); z <= min(cz + 1, g.dz - 1); ++z)
    for (int y = max(cy - 1, 0); y <= min(cy + 1, g.dy - 1); ++y) {
      const int rowc = (z * g.dy + y) * g.dx;
      const int b = cell_start[rowc + max(cx - 1, 0)], e = cell_start[rowc + min(cx + 1, g.dx - 1) + 1];
      for (int p = b; p < e; ++p) {
        const float4 P = sorted[p];
        if (__float_as_int(P.w) == (int)n) continue;
        const float ddx = qx - P.x, ddy = qy - P.y, ddz = qz - P.z;
        best = fminf(best, (ddx * ddx + ddy * ddy) + ddz * ddz);
      }
    }
  if (!(best <= g.c * g.c * 0.999f)) {  // not provably the global minimum: brute force
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
//   GridParams | counts[cap] | cell_start[cap+1] | cursor[cap] | pcell[N] | scan ws
static size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

extern "C" size_t apn_grid_workspace_bytes(int64_t n_points, int32_t cell_cap) {
  return al256(sizeof(GridParams)) + al256((size_t)cell_cap * 4) + al256((size_t)(cell_cap + 1) * 4) +
         al256((size_t)cell_cap * 4) + al256((size_t)n_points * 4) + al256(scan_workspace_bytes(cell_cap));
}

struct GridWs {
  GridParams* gp; int* counts; int* cell_start; int* cursor; int* pcell; void* scan;
};
static GridWs grid_ws(void* ws, int64_t N, int cap) {
  char* p = (char*)ws;
  GridWs w;
  w.gp = (GridParams*)p; p += al256(sizeof(GridParams));
  w.counts = (int*)p; p += al256((size_t)cap * 4);
  w.cell_start = (int*)p; p += al256((size_t)(cap + 1) * 4);
  w.cursor = (int*)p; p += al256((size_t)cap * 4);
  w.pcell = (int*)p; p += al256((size_t)N * 4);
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
  hipLaunchKernelGGL(k_grid_params, dim3(1), dim3(64), 0, s, bbox_ord, query_radius, cell_cap, w.gp);
  hipLaunchKernelGGL(k_grid_count, dim3(ceil_div(n_points, 256)), dim3(256), 0, s, xyz, n_points, w.gp, w.counts,
                     w.pcell);
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
                     g.gp, g.cell_start, (const float4*)sorted_pts4, query_radius, t_pos, t_ray, t_nbr, blk_cnt);
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
