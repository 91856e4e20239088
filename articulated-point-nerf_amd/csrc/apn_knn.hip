// Radius-bounded exact kNN over the warped cloud: the replacement for the reference's
// pykeops brute-force `Kmin_argKmin(K=8)` + radius filter (temporalpoints.py:433-447).
//
// Exactness: a sample survives the reference filter iff its 8th-nearest squared distance
// is <= query_radius = r^2. Every neighbour of a survivor lies within r, so a search that has
// seen every point within r returns the reference's top-8 (by float32 (dx*dx+dy*dy)+dz*dz,
// ties by index; pykeops leaves tie order unspecified). Non-survivors are discarded by the
// reference anyway. Distances use -ffp-contract=off arithmetic, so they equal the reference's
// recomputed `to_nn` bit-for-bit.
//
// Data structure: a fine uniform grid (cell h = r / KNN_SUBDIV, bounded by a cell cap) built by
// counting sort into float4 {x,y,z,bits(idx)} -- the cells of one x-row are contiguous -- plus
// a coarse count grid (cell side cf*h >= r).
// Query (two passes):
//   classify: < 8 points in the 27 coarse cells around the sample => < 8 within r => reject
//             (55% of the in-bbox samples at C2); the rest are compacted in query order;
//   search:   cubes of Chebyshev radius k in {1, 2, 4, kmax} (kmax*h >= r), each scanned as
//             (2k+1)^2 contiguous x-rows; after cube k every point closer than k*h has been
//             seen, so the search stops exactly when the 8th best is closer than k*h(1-1e-4).
#include "apn_common.h"

namespace apn {

struct GridParams {
  float ox, oy, oz, h;        // fine grid origin and cell side
  float inv_h, r, r2, pad0;   // search radius r = sqrt(query_radius), r2 = query_radius
  int dx, dy, dz, nf;         // fine grid dims and cell count
  int cf, cdx, cdy, cdz;      // fine cells per coarse cell (coarse side >= r), coarse dims
  int nc, kmax, pad1, pad2;   // coarse cell count, search limit (kmax * h >= r)
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

template <int K, bool EXCL>
__device__ __forceinline__ void consider(const float4& P, float qx, float qy, float qz, float dmax2, int excl,
                                         float (&bd)[K], int (&bi)[K]) {
  const float ddx = qx - P.x, ddy = qy - P.y, ddz = qz - P.z;
  const float d = (ddx * ddx + ddy * ddy) + ddz * ddz;
  const int id = __float_as_int(P.w);
  if (d <= dmax2 && (!EXCL || id != excl)) knn_insert<K>(d, id, bd, bi);
}

// Scan points [b, e) of the sorted array into the top-K, 4 independent loads per step.
template <int K, bool EXCL>
__device__ __forceinline__ void scan_range(const float4* __restrict__ sorted, int b, int e, float qx, float qy,
                                           float qz, float dmax2, int excl, float (&bd)[K], int (&bi)[K]) {
  int p = b;
  for (; p + 4 <= e; p += 4) {
    const float4 P0 = sorted[p], P1 = sorted[p + 1], P2 = sorted[p + 2], P3 = sorted[p + 3];
    consider<K, EXCL>(P0, qx, qy, qz, dmax2, excl, bd, bi);
    consider<K, EXCL>(P1, qx, qy, qz, dmax2, excl, bd, bi);
    consider<K, EXCL>(P2, qx, qy, qz, dmax2, excl, bd, bi);
    consider<K, EXCL>(P3, qx, qy, qz, dmax2, excl, bd, bi);
  }
  for (; p < e; ++p) consider<K, EXCL>(sorted[p], qx, qy, qz, dmax2, excl, bd, bi);
}

// All points in the cube of Chebyshev radius k (fine cells) around (fx,fy,fz), clamped to the
// grid, as (2k+1)^2 contiguous x-rows. The next row's bounds are fetched before the current
// row is scanned.
template <int K, bool EXCL>
__device__ __forceinline__ void scan_cube(const GridParams& g, const int* __restrict__ cell_start,
                                          const float4* __restrict__ sorted, int fx, int fy, int fz, int k,
                                          float qx, float qy, float qz, float dmax2, int excl, float (&bd)[K],
                                          int (&bi)[K]) {
  const int x0 = max(fx - k, 0), x1 = min(fx + k, g.dx - 1);
  const int y0 = max(fy - k, 0), y1 = min(fy + k, g.dy - 1);
  const int z0 = max(fz - k, 0), z1 = min(fz + k, g.dz - 1);
  if (x0 > x1 || y0 > y1 || z0 > z1) return;
  const int ny = y1 - y0 + 1, nrows = ny * (z1 - z0 + 1);
  int row = (z0 * g.dy + y0) * g.dx;
  int b = cell_start[row + x0], e = cell_start[row + x1 + 1];
  for (int j = 0; j < nrows; ++j) {
    int nb = 0, ne = 0;
    if (j + 1 < nrows) {
      const int jj = j + 1;
      const int nrow = ((z0 + jj / ny) * g.dy + (y0 + jj % ny)) * g.dx;
      nb = cell_start[nrow + x0];
      ne = cell_start[nrow + x1 + 1];
    }
    scan_range<K, EXCL>(sorted, b, e, qx, qy, qz, dmax2, excl, bd, bi);
    b = nb; e = ne;
  }
}

__device__ __forceinline__ int next_level(int k, int kmax) { return k >= kmax ? kmax + 1 : min(2 * k, kmax); }

// Squared distance from coordinate v to the slab of cells [c0, c1] along one axis.
__device__ __forceinline__ float slab_d2(float v, float o, float h, int c0, int c1) {
  const float lo = o + (float)c0 * h, hi = o + (float)(c1 + 1) * h;
  const float d = v < lo ? lo - v : (v > hi ? v - hi : 0.f);
  return d * d;
}

// Ring k (Chebyshev distance exactly k) around (fx,fy,fz) as row segments; a segment is
// skipped when its box is farther than the current K-th best (or r), which only removes
// points that could not enter the top-K (box distance is a lower bound, with 1e-4 slack).
template <int K, bool EXCL>
__device__ __forceinline__ void scan_ring_culled(const GridParams& g, const int* __restrict__ cell_start,
                                                 const float4* __restrict__ sorted, int fx, int fy, int fz, int k,
                                                 float qx, float qy, float qz, float dmax2, int excl,
                                                 float (&bd)[K], int (&bi)[K]) {
  const int z0 = max(fz - k, 0), z1 = min(fz + k, g.dz - 1);
  const int y0 = max(fy - k, 0), y1 = min(fy + k, g.dy - 1);
  const int xa = fx - k, xb = fx + k;
  const int x0 = max(xa, 0), x1 = min(xb, g.dx - 1);
  if (x0 > x1) return;
  for (int z = z0; z <= z1; ++z) {
    const bool zs = (z == fz - k) || (z == fz + k);
    const float dz2 = slab_d2(qz, g.oz, g.h, z, z);
    for (int y = y0; y <= y1; ++y) {
      const float tau = fminf(bd[K - 1], dmax2) * 1.0001f;
      const float dyz2 = dz2 + slab_d2(qy, g.oy, g.h, y, y);
      if (dyz2 > tau) continue;
      const int row = (z * g.dy + y) * g.dx;
      if (zs || y == fy - k || y == fy + k) {
        if (dyz2 + slab_d2(qx, g.ox, g.h, x0, x1) <= tau)
          scan_range<K, EXCL>(sorted, cell_start[row + x0], cell_start[row + x1 + 1], qx, qy, qz, dmax2, excl, bd, bi);
      } else {
        if (xa >= 0 && dyz2 + slab_d2(qx, g.ox, g.h, xa, xa) <= tau)
          scan_range<K, EXCL>(sorted, cell_start[row + xa], cell_start[row + xa + 1], qx, qy, qz, dmax2, excl, bd, bi);
        if (xb < g.dx && k > 0 && dyz2 + slab_d2(qx, g.ox, g.h, xb, xb) <= tau)
          scan_range<K, EXCL>(sorted, cell_start[row + xb], cell_start[row + xb + 1], qx, qy, qz, dmax2, excl, bd, bi);
      }
    }
  }
}

// Insert with duplicate check (a ball scan of a larger radius revisits the points of the
// previous one; a revisited point has the same distance, so it is found in the list).
template <int K>
__device__ __forceinline__ void knn_insert_unique(float d, int id, float (&bd)[K], int (&bi)[K]) {
  if (!knn_less(d, id, bd[K - 1], bi[K - 1])) return;
#pragma unroll
  for (int k = 0; k < K; ++k)
    if (bi[k] == id) return;
  bd[K - 1] = d; bi[K - 1] = id;
#pragma unroll
  for (int k = K - 1; k > 0; --k) {
    if (knn_less(bd[k], bi[k], bd[k - 1], bi[k - 1])) {
      float td = bd[k]; bd[k] = bd[k - 1]; bd[k - 1] = td;
      int ti = bi[k]; bi[k] = bi[k - 1]; bi[k - 1] = ti;
    }
  }
}

template <int K>
__device__ __forceinline__ void scan_range_u(const float4* __restrict__ sorted, int b, int e, float qx, float qy,
                                             float qz, float dmax2, float (&bd)[K], int (&bi)[K]) {
  int p = b;
  for (; p + 4 <= e; p += 4) {
    float4 P[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) P[u] = sorted[p + u];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float ddx = qx - P[u].x, ddy = qy - P[u].y, ddz = qz - P[u].z;
      const float d = (ddx * ddx + ddy * ddy) + ddz * ddz;
      if (d <= dmax2) knn_insert_unique<K>(d, __float_as_int(P[u].w), bd, bi);
    }
  }
  for (; p < e; ++p) {
    const float4 P = sorted[p];
    const float ddx = qx - P.x, ddy = qy - P.y, ddz = qz - P.z;
    const float d = (ddx * ddx + ddy * ddy) + ddz * ddz;
    if (d <= dmax2) knn_insert_unique<K>(d, __float_as_int(P.w), bd, bi);
  }
}

// Every point whose cell intersects the ball of squared radius R2 around q, shrunk on the fly to
// the current K-th best: (z, y) rows outside the bound are skipped and each remaining row is
// scanned over the x-chord of the ball (cells [x0, x1] are contiguous in the sorted array).
// Bounds carry a 1e-4 relative slack, far above float rounding of the cell arithmetic.
template <int K>
__device__ __forceinline__ void scan_ball(const GridParams& g, const int* __restrict__ cell_start,
                                          const float4* __restrict__ sorted, float qx, float qy, float qz, float R2,
                                          float (&bd)[K], int (&bi)[K]) {
  const float R = sqrtf(R2) * 1.0001f;
  const int z0 = max((int)floorf((qz - R - g.oz) * g.inv_h), 0), z1 = min((int)floorf((qz + R - g.oz) * g.inv_h), g.dz - 1);
  const int y0 = max((int)floorf((qy - R - g.oy) * g.inv_h), 0), y1 = min((int)floorf((qy + R - g.oy) * g.inv_h), g.dy - 1);
  for (int z = z0; z <= z1; ++z) {
    const float dz2 = slab_d2(qz, g.oz, g.h, z, z);
    for (int y = y0; y <= y1; ++y) {
      const float tau = fminf(bd[K - 1], R2) * 1.0001f;
      const float dyz2 = dz2 + slab_d2(qy, g.oy, g.h, y, y);
      if (dyz2 > tau) continue;
      const float w = sqrtf(tau - dyz2) * 1.0001f;
      const int x0 = max((int)floorf((qx - w - g.ox) * g.inv_h), 0);
      const int x1 = min((int)floorf((qx + w - g.ox) * g.inv_h), g.dx - 1);
      if (x0 > x1) continue;
      const int row = (z * g.dy + y) * g.dx;
      scan_range_u<K>(sorted, cell_start[row + x0], cell_start[row + x1 + 1], qx, qy, qz, g.r2, bd, bi);
    }
  }
}

// Pass 1: coarse rejection. Queries with >= 8 points in the 27 coarse cells around them are
// compacted (in query order) per block into cand[blockIdx*256 ...]; blk_cnt[block] = count.
__global__ __launch_bounds__(KNN_THREADS) void k_knn_classify(const float4* __restrict__ q_pos,
                                                              const int* __restrict__ n_q_dev,
                                                              const GridParams* __restrict__ gp,
                                                              const int* __restrict__ ccount,
                                                              int* __restrict__ cand, int* __restrict__ blk_cnt) {
  __shared__ int wave_cnt[KNN_THREADS / 64];
  const int nq = *n_q_dev;
  const int i = blockIdx.x * KNN_THREADS + threadIdx.x;
  const GridParams g = *gp;
  bool keep = false;
  if (i < nq) {
    const float4 q = q_pos[i];
    const int cx = floor_div((int)floorf((q.x - g.ox) * g.inv_h), g.cf);
    const int cy = floor_div((int)floorf((q.y - g.oy) * g.inv_h), g.cf);
    const int cz = floor_div((int)floorf((q.z - g.oz) * g.inv_h), g.cf);
    int cnt = 0;
    for (int z = max(cz - 1, 0); z <= min(cz + 1, g.cdz - 1); ++z)
      for (int y = max(cy - 1, 0); y <= min(cy + 1, g.cdy - 1); ++y)
        for (int x = max(cx - 1, 0); x <= min(cx + 1, g.cdx - 1); ++x) cnt += ccount[(z * g.cdy + y) * g.cdx + x];
    keep = cnt >= KNN_K;
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const unsigned long long bal = __ballot(keep);
  const int before = __popcll(bal & ((1ull << lane) - 1ull));
  if (lane == 0) wave_cnt[wid] = __popcll(bal);
  __syncthreads();
  int base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < KNN_THREADS / 64; ++w) {
    base += (w < wid) ? wave_cnt[w] : 0;
    tot += wave_cnt[w];
  }
  if (keep) cand[blockIdx.x * KNN_THREADS + base + before] = i;
  if (threadIdx.x == 0) blk_cnt[blockIdx.x] = tot;
}

// Compact per-block int lists into a dense list (order preserved).
__global__ __launch_bounds__(KNN_THREADS) void k_compact_i32(const int* __restrict__ src,
                                                             const int* __restrict__ blk_cnt,
                                                             const int* __restrict__ blk_off,
                                                             int* __restrict__ dst) {
  const int t = threadIdx.x;
  if (t < blk_cnt[blockIdx.x]) dst[blk_off[blockIdx.x] + t] = src[blockIdx.x * KNN_THREADS + t];
}

// Pass 2: exact search for the compacted candidates. Survivors are compacted per block (order
// preserved) into slots [blockIdx*256, ...) of t_*; blk_cnt[block] = survivors.
__global__ __launch_bounds__(KNN_THREADS) void k_knn_search(
    const float4* __restrict__ q_pos, const int* __restrict__ q_ray, const int* __restrict__ cand,
    const int* __restrict__ n_cand_dev, const GridParams* __restrict__ gp, const int* __restrict__ cell_start,
    const float4* __restrict__ sorted, float4* __restrict__ t_pos, int* __restrict__ t_ray,
    int* __restrict__ t_nbr, int* __restrict__ blk_cnt, int mode) {
  __shared__ int wave_cnt[KNN_THREADS / 64];
  const int nc = *n_cand_dev;
  const int c = blockIdx.x * KNN_THREADS + threadIdx.x;
  float bd[KNN_K];
  int bi[KNN_K];
#pragma unroll
  for (int k = 0; k < KNN_K; ++k) { bd[k] = INFINITY; bi[k] = 0x7fffffff; }
  float4 q = make_float4(0.f, 0.f, 0.f, 0.f);
  int qi = 0;
  const GridParams g = *gp;
  if (c < nc) {
    qi = cand[c];
    q = q_pos[qi];
    if (mode == 0) {
      // expanding balls R = 2h, 4h, ..., r: after a ball every point within R has been seen, so
      // a K-th best strictly inside R is final
      float R = 2.f * g.h;
      for (;;) {
        const float Rl = fminf(R, g.r);
        const float R2 = Rl >= g.r ? g.r2 : Rl * Rl;
        scan_ball<KNN_K>(g, cell_start, sorted, q.x, q.y, q.z, R2, bd, bi);
        if (Rl >= g.r || bd[KNN_K - 1] < R2 * (1.f - 2e-4f)) break;
        R *= 2.f;
      }
    } else {
      const int fx = (int)floorf((q.x - g.ox) * g.inv_h);
      const int fy = (int)floorf((q.y - g.oy) * g.inv_h);
      const int fz = (int)floorf((q.z - g.oz) * g.inv_h);
      for (int k = 0; k <= g.kmax; ++k) {
        scan_ring_culled<KNN_K, false>(g, cell_start, sorted, fx, fy, fz, k, q.x, q.y, q.z, g.r2, -1, bd, bi);
        const float gk = (float)k * g.h * (1.f - 1e-4f);
        if (bd[KNN_K - 1] < gk * gk) break;
      }
    }
  }
  const bool surv = (c < nc) && (bd[KNN_K - 1] <= g.r2);
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
    t_ray[slot] = q_ray[qi];
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
// self-inclusive argKmin is the nearest other point, or a duplicate at distance 0). Cube search
// with the same exact stopping rule, radius doubling over the whole grid; brute force if the
// grid runs out. Output: sqrt(d2 + eps) per point.
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
  const int kend = min(max(g.dx, max(g.dy, g.dz)), 64);
  bool done = false;
  for (int k = 1; k <= kend; k *= 2) {
    bd[0] = INFINITY; bi[0] = 0x7fffffff;
    scan_cube<1, true>(g, cell_start, sorted, fx, fy, fz, k, qx, qy, qz, INFINITY, (int)n, bd, bi);
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

// Search strategy: 0 = expanding ball scans (default), 1 = culled Chebyshev rings.
// APN_KNN_MODE selects one for A/B measurements; both are exact.
static int knn_mode() {
  static int m = [] {
    const char* e = getenv("APN_KNN_MODE");
    return e ? atoi(e) : 0;
  }();
  return m;
}

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
  static const int subdiv = [] {
    const char* e = getenv("APN_KNN_SUBDIV");
    return e ? atoi(e) : KNN_SUBDIV;
  }();
  hipLaunchKernelGGL(k_grid_params, dim3(1), dim3(64), 0, s, bbox_ord, query_radius, cell_cap, subdiv, w.gp);
  hipLaunchKernelGGL(k_grid_count, dim3(ceil_div(n_points, 256)), dim3(256), 0, s, xyz, n_points, w.gp, w.counts,
                     w.ccount, w.pcell);
  int st = scan_exclusive_i32(w.counts, w.cell_start, cell_cap, w.scan, s);
  if (st) return st;
  hipLaunchKernelGGL(k_grid_scatter, dim3(ceil_div(n_points, 256)), dim3(256), 0, s, xyz, n_points, w.pcell,
                     w.cell_start, w.cursor, (float4*)sorted_pts4);
  return launch_status();
}

// kNN workspace: per-slot candidate / survivor staging + block counts/offsets + scan scratch.
extern "C" size_t apn_knn_workspace_bytes(int64_t n_queries) {
  int64_t nb = (n_queries + KNN_THREADS - 1) / KNN_THREADS;
  size_t slots = (size_t)nb * KNN_THREADS;
  return al256(slots * 4) * 2 + al256((size_t)(nb + 2) * 4) * 2 + al256(slots * 16) + al256(slots * 4) +
         al256(slots * 4 * KNN_K) + al256((size_t)(nb + 1) * 4) * 2 + al256(scan_workspace_bytes(nb));
}

// Queries: q_pos4[n_queries] {x,y,z,bits(step)} and q_ray. n_queries is an upper bound used for
// the launch; the live count is read on device from *n_queries_dev. Survivors (sorted by query
// order) go to s_pos4/s_ray/s_nbr and their count to *n_survivors_dev.
extern "C" int apn_knn_radius(const float* q_pos4, const int32_t* q_ray, int64_t n_queries,
                              const int32_t* n_queries_dev, const void* grid_workspace, int64_t n_points,
                              int32_t cell_cap, const float* sorted_pts4, float query_radius, float* s_pos4,
                              int32_t* s_ray, int32_t* s_nbr, int32_t* n_survivors_dev, void* workspace,
                              void* stream) {
  (void)query_radius;  // the grid was built for it (GridParams.r2)
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
  int* cand_blk = (int*)p; p += al256(slots * 4);
  int* cand = (int*)p; p += al256(slots * 4);
  int* cblk_cnt = (int*)p; p += al256((size_t)(nb + 2) * 4);
  int* cblk_off = (int*)p; p += al256((size_t)(nb + 2) * 4);
  float4* t_pos = (float4*)p; p += al256(slots * 16);
  int* t_ray = (int*)p; p += al256(slots * 4);
  int* t_nbr = (int*)p; p += al256(slots * 4 * KNN_K);
  int* blk_cnt = (int*)p; p += al256((size_t)(nb + 1) * 4);
  int* blk_off = (int*)p; p += al256((size_t)(nb + 1) * 4);
  void* sws = p;
  hipLaunchKernelGGL(k_knn_classify, dim3(nb), dim3(KNN_THREADS), 0, s, (const float4*)q_pos4, n_queries_dev, g.gp,
                     g.ccount, cand_blk, cblk_cnt);
  int st = scan_exclusive_i32(cblk_cnt, cblk_off, nb, sws, s);
  if (st) return st;
  hipLaunchKernelGGL(k_compact_i32, dim3(nb), dim3(KNN_THREADS), 0, s, cand_blk, cblk_cnt, cblk_off, cand);
  // candidates: count at cblk_off[nb]; launch over the upper bound nb blocks
  hipLaunchKernelGGL(k_knn_search, dim3(nb), dim3(KNN_THREADS), 0, s, (const float4*)q_pos4, q_ray, cand,
                     cblk_off + nb, g.gp, g.cell_start, (const float4*)sorted_pts4, t_pos, t_ray, t_nbr, blk_cnt,
                     knn_mode());
  st = scan_exclusive_i32(blk_cnt, blk_off, nb, sws, s);
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
  int st = apn_grid_build(xyz, n_points, bbox_ord, 0.01f, cell_cap, sorted_pts4, grid_workspace, stream);
  if (st) return st;
  GridWs g = grid_ws(grid_workspace, n_points, cell_cap);
  hipLaunchKernelGGL(k_nn1, dim3(ceil_div(n_points, 256)), dim3(256), 0, s, xyz, n_points, g.gp, g.cell_start,
                     (const float4*)sorted_pts4, eps, nn_dist);
  return launch_status();
}
