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

#include <algorithm>

namespace apn {

struct GridParams {
  float ox, oy, oz, h;        // fine grid origin and cell side
  float inv_h, r, r2, pad0;   // search radius r = sqrt(query_radius), r2 = query_radius
  int dx, dy, dz, nf;         // fine grid dims and cell count
  int cf, cdx, cdy, cdz;      // fine cells per coarse cell (coarse side >= r), coarse dims
  int nc, kmax, np, pad2;     // coarse cell count, search limit (kmax * h >= r), points in sorted
};

constexpr int KNN_K = 8;
constexpr int KNN_THREADS = 256;
// launch bound (in-bbox samples) up to which pass B runs 8 lanes per hard query
constexpr int64_t KNN_SPLIT_MAX_QUERIES = (int64_t)1 << 18;
constexpr int KNN_SUBDIV = 8;   // fine cell side = r / KNN_SUBDIV (before the cell cap)

__device__ __forceinline__ int floor_div(int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

__global__ void k_grid_params(const int* __restrict__ bbox_ord, float qr, int cap, int subdiv, int np,
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
  g.np = np;
  g.pad2 = 0;
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
  (void)ccount;
}

// Coarse-cell counts (the classify pass's 27-cell test) from the fine prefix: one thread per coarse
// cell sums its cf x cf fine rows (cell_start differences) -- no per-point atomics on the ~10^3
// coarse counters, which serialised at the L2.
__global__ void k_coarse_counts(const GridParams* __restrict__ gp, const int* __restrict__ cell_start,
                                int* __restrict__ ccount) {
  const GridParams g = *gp;
  // one wave per coarse cell, lane = one of its cf x cf fine (z, y) rows (a thread walking the
  // 64 rows waited on each row's two loads in turn: ~34 us), integer sum by shuffles (exact)
  const int lane = threadIdx.x & 63;
  const int wpb = blockDim.x >> 6;
  for (int c = blockIdx.x * wpb + (threadIdx.x >> 6); c < g.nc; c += gridDim.x * wpb) {
    const int ccx = c % g.cdx, ccy = (c / g.cdx) % g.cdy, ccz = c / (g.cdx * g.cdy);
    const int x0 = ccx * g.cf, x1 = min(x0 + g.cf, g.dx) - 1;
    int n = 0;
    for (int p = lane; p < g.cf * g.cf; p += 64) {
      const int z = ccz * g.cf + p / g.cf, y = ccy * g.cf + p % g.cf;
      if (z < g.dz && y < g.dy) {
        const int row = (z * g.dy + y) * g.dx;
        n += cell_start[row + x1 + 1] - cell_start[row + x0];
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o, 64);
    if (lane == 0) ccount[c] = n;
  }
}

// Points in the 3x3x3 coarse block around each coarse cell (clamped at the grid's faces): the
// classify test of k_knn_classify as one load per query instead of 27.
__global__ void k_coarse_sum27(const GridParams* __restrict__ gp, const int* __restrict__ ccount,
                               int* __restrict__ csum27) {
  const GridParams g = *gp;
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < g.nc; c += gridDim.x * blockDim.x) {
    const int cx = c % g.cdx, cy = (c / g.cdx) % g.cdy, cz = c / (g.cdx * g.cdy);
    int cnt = 0;
    for (int z = max(cz - 1, 0); z <= min(cz + 1, g.cdz - 1); ++z)
      for (int y = max(cy - 1, 0); y <= min(cy + 1, g.cdy - 1); ++y)
        for (int x = max(cx - 1, 0); x <= min(cx + 1, g.cdx - 1); ++x) cnt += ccount[(z * g.cdy + y) * g.cdx + x];
    csum27[c] = cnt;
  }
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

// Culling radii of the ball scans: v_sqrt_f32 (about 1 ulp) instead of the correctly rounded
// sqrtf sequence (~14 instructions: denormal scaling, two correction fmas). Every use is a bound
// with 1e-4 relative slack (plus 1e-12 absolute for denormal arguments), so the rows and cells a
// scan visits still cover the ball exactly as before. (APN_KNN_IEEE_SQRT: the library sqrtf.)
__device__ __forceinline__ float bound_sqrt(float x) {
#ifdef APN_KNN_IEEE_SQRT
  return sqrtf(x) * 1.0001f;
#else
  return __builtin_amdgcn_sqrtf(x) * 1.0001f + 1e-12f;
#endif
}
#ifdef APN_KNN_GLOBAL_POINTS   // A/B: pass B's point loads as clamped 64-bit global loads
constexpr bool kBufferPoints = false;
#else
constexpr bool kBufferPoints = true;
#endif
// Buffer-descriptor loads for the ball scans: 32-bit byte offsets (no 64-bit address arithmetic per
// load); reads past num_records return zeros. num_records and offsets are int32 byte counts, so a
// cloud of more than KNN_MAX_POINTS points (16 B each) would wrap and read zeros: apn_grid_build
// and apn_knn_radius refuse such clouds (APN_ERR_ARG) rather than return a wrong kNN.
constexpr int64_t KNN_MAX_POINTS = 0x7fffffffLL / 16;
typedef float knn_f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t knn_rsrc(const void* p, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, bytes, 0x00020000);
}
__device__ __forceinline__ float4 knn_ld_pt(__amdgpu_buffer_rsrc_t rs, int i) {
  const knn_f4v v = __builtin_bit_cast(knn_f4v, __builtin_amdgcn_raw_buffer_load_b128(rs, i * 16, 0, 0));
  return make_float4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ int knn_ld_i32(__amdgpu_buffer_rsrc_t rs, int i) {
  return (int)__builtin_amdgcn_raw_buffer_load_b32(rs, i * 4, 0, 0);
}
#ifdef APN_KNN_DUPCHECK_ALL   // A/B: the duplicate check on every insert (the round-2 kernels)
constexpr bool kFirstScanNoDup = false;
#else
constexpr bool kFirstScanNoDup = true;
#endif

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

// Top-K lists for the ball scans. ArrList: the (distance, index) arrays, pairwise compares.
// KeyList: one 64-bit key per entry, bits(d) << 32 | index -- for d >= 0 the unsigned key order is
// exactly knn_less (distance, then index), so each compare is one 64-bit integer compare; an insert
// computes every position flag from the old list (independent compares) and shifts with selects.
template <int K>
struct ArrList {
  float (&bd)[K];
  int (&bi)[K];
  __device__ __forceinline__ float worst() const { return bd[K - 1]; }
  __device__ __forceinline__ int index(int k) const { return bi[k]; }
  template <bool DUP>
  __device__ __forceinline__ void insert(float d, int id) {
    if constexpr (DUP) knn_insert_unique<K>(d, id, bd, bi);
    else knn_insert<K>(d, id, bd, bi);
  }
};

typedef unsigned long long knn_key_t;
__device__ __forceinline__ knn_key_t knn_key(float d, int i) {
  return ((knn_key_t)__float_as_uint(d) << 32) | (unsigned)i;
}

template <int K>
struct KeyList {
  knn_key_t kk[K];
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int k = 0; k < K; ++k) kk[k] = knn_key(INFINITY, 0x7fffffff);
  }
  __device__ __forceinline__ float worst() const { return __uint_as_float((unsigned)(kk[K - 1] >> 32)); }
  __device__ __forceinline__ float dist(int k) const { return __uint_as_float((unsigned)(kk[k] >> 32)); }
  __device__ __forceinline__ int index(int k) const { return (int)(unsigned)kk[k]; }
  template <bool DUP>
  __device__ __forceinline__ void insert(float d, int id) {
    const knn_key_t x = knn_key(d, id);
    if (!(x < kk[K - 1])) return;
    if constexpr (DUP) {
#pragma unroll
      for (int k = 0; k < K - 1; ++k)
        if (kk[k] == x) return;
    }
    bool m[K];
#pragma unroll
    for (int k = 0; k < K; ++k) m[k] = x < kk[k];   // monotone: false..false true..true
#ifndef APN_KNN_INTERLEAVED_INSERT
    // all compares first, each into its own SGPR pair, then the selects: interleaved, every select
    // pair waited out the VALU-SGPR-write -> mask-read hazard of the compare just before it (s_nop)
    __builtin_amdgcn_sched_barrier(0);
#endif
#pragma unroll
    for (int k = K - 1; k > 0; --k) kk[k] = m[k - 1] ? kk[k - 1] : (m[k] ? x : kk[k]);   // (m[k-1] implies m[k])
    kk[0] = m[0] ? x : kk[0];
  }
};

// pass A / pass B lists (mode 9): 64-bit keys, or (APN_KNN_PAIRLIST, A/B) the (distance, index) pairs
template <int K>
struct PairList {
  float bd[K];
  int bi[K];
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int k = 0; k < K; ++k) { bd[k] = INFINITY; bi[k] = 0x7fffffff; }
  }
  __device__ __forceinline__ float worst() const { return bd[K - 1]; }
  __device__ __forceinline__ float dist(int k) const { return bd[k]; }
  __device__ __forceinline__ int index(int k) const { return bi[k]; }
  template <bool DUP>
  __device__ __forceinline__ void insert(float d, int id) {
    if constexpr (DUP) knn_insert_unique<K>(d, id, bd, bi);
    else knn_insert<K>(d, id, bd, bi);
  }
};
#ifdef APN_KNN_PAIRLIST
typedef PairList<KNN_K> KnnList;
#else
typedef KeyList<KNN_K> KnnList;
#endif

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

// Signed offset sequence 0, -1, +1, -2, +2, ... (nearest-first order around a cell index).
__device__ __forceinline__ int nf_offset(int i) { return (i & 1) ? -((i + 1) >> 1) : (i >> 1); }

// scan_ball with the (z, y) rows visited nearest-first (offsets 0, -1, +1, ... around the query's
// cell), so the running K-th best -- and with it the row culling bound -- shrinks as early as
// possible. Same point set as scan_ball for the final result (culling is exact).
template <int K>
__device__ __forceinline__ void scan_ball_nf(const GridParams& g, const int* __restrict__ cell_start,
                                             const float4* __restrict__ sorted, float qx, float qy, float qz,
                                             float R2, float (&bd)[K], int (&bi)[K], int* ctr = nullptr) {
  const float R = sqrtf(R2) * 1.0001f;
  const int z0 = max((int)floorf((qz - R - g.oz) * g.inv_h), 0), z1 = min((int)floorf((qz + R - g.oz) * g.inv_h), g.dz - 1);
  const int y0 = max((int)floorf((qy - R - g.oy) * g.inv_h), 0), y1 = min((int)floorf((qy + R - g.oy) * g.inv_h), g.dy - 1);
  const int fz = min(max((int)floorf((qz - g.oz) * g.inv_h), z0), z1);
  const int fy = min(max((int)floorf((qy - g.oy) * g.inv_h), y0), y1);
  const int nz = 2 * max(fz - z0, z1 - fz) + 1, ny = 2 * max(fy - y0, y1 - fy) + 1;
  for (int iz = 0; iz < nz; ++iz) {
    const int z = fz + nf_offset(iz);
    if (z < z0 || z > z1) continue;
    const float dz2 = slab_d2(qz, g.oz, g.h, z, z);
    if (dz2 > fminf(bd[K - 1], R2) * 1.0001f) continue;
    for (int iy = 0; iy < ny; ++iy) {
      const int y = fy + nf_offset(iy);
      if (y < y0 || y > y1) continue;
      const float tau = fminf(bd[K - 1], R2) * 1.0001f;
      const float dyz2 = dz2 + slab_d2(qy, g.oy, g.h, y, y);
      if (dyz2 > tau) continue;
      const float w = sqrtf(tau - dyz2) * 1.0001f;
      const int x0 = max((int)floorf((qx - w - g.ox) * g.inv_h), 0);
      const int x1 = min((int)floorf((qx + w - g.ox) * g.inv_h), g.dx - 1);
      if (x0 > x1) continue;
      const int row = (z * g.dy + y) * g.dx;
      const int b = cell_start[row + x0], e = cell_start[row + x1 + 1];
      if (ctr) { ctr[0] += 1; ctr[1] += e - b; }
      scan_range_u<K>(sorted, b, e, qx, qy, qz, g.r2, bd, bi);
    }
  }
}

// Upper bound on the number of points within sqrt(R2) of q: the points of every cell on the
// ball's row chords (a superset of the ball). Loads only cell_start pairs (independent across
// rows, no point reads); stops as soon as the bound reaches `need`.
__device__ __forceinline__ int chord_count(const GridParams& g, const int* __restrict__ cell_start, float qx,
                                           float qy, float qz, float R2, int need, int* ctr = nullptr) {
  const float R = sqrtf(R2) * 1.0001f;
  const int z0 = max((int)floorf((qz - R - g.oz) * g.inv_h), 0), z1 = min((int)floorf((qz + R - g.oz) * g.inv_h), g.dz - 1);
  const int y0 = max((int)floorf((qy - R - g.oy) * g.inv_h), 0), y1 = min((int)floorf((qy + R - g.oy) * g.inv_h), g.dy - 1);
  const int fz = min(max((int)floorf((qz - g.oz) * g.inv_h), z0), z1);
  const int nz = 2 * max(fz - z0, z1 - fz) + 1;
  const float tau = R2 * 1.0001f;
  int c = 0;
  for (int iz = 0; iz < nz && c < need; ++iz) {
    const int z = fz + nf_offset(iz);
    if (z < z0 || z > z1) continue;
    const float dz2 = slab_d2(qz, g.oz, g.h, z, z);
    if (dz2 > tau) continue;
#pragma unroll 4
    for (int y = y0; y <= y1; ++y) {
      const float dyz2 = dz2 + slab_d2(qy, g.oy, g.h, y, y);
      const float w = sqrtf(fmaxf(tau - dyz2, 0.f)) * 1.0001f;
      const int x0 = max((int)floorf((qx - w - g.ox) * g.inv_h), 0);
      const int x1 = min((int)floorf((qx + w - g.ox) * g.inv_h), g.dx - 1);
      const int row = (z * g.dy + y) * g.dx;
      if (dyz2 <= tau && x0 <= x1) {
        c += cell_start[row + x1 + 1] - cell_start[row + x0];
        if (ctr) ctr[0] += 1;
      }
    }
  }
  return c;
}

// ---- accessor-templated variants: CS(z, y, x) returns cell_start[(z*dy + y)*dx + x] (from LDS
// when the tile kernel has staged that row, else from global memory).
template <int K, class CS>
__device__ __forceinline__ void scan_ball_cs(const GridParams& g, const CS& cs, const float4* __restrict__ sorted,
                                             float qx, float qy, float qz, float R2, float (&bd)[K], int (&bi)[K]) {
  const float R = sqrtf(R2) * 1.0001f;
  const int z0 = max((int)floorf((qz - R - g.oz) * g.inv_h), 0), z1 = min((int)floorf((qz + R - g.oz) * g.inv_h), g.dz - 1);
  const int y0 = max((int)floorf((qy - R - g.oy) * g.inv_h), 0), y1 = min((int)floorf((qy + R - g.oy) * g.inv_h), g.dy - 1);
  const int fz = min(max((int)floorf((qz - g.oz) * g.inv_h), z0), z1);
  const int fy = min(max((int)floorf((qy - g.oy) * g.inv_h), y0), y1);
  const int nz = 2 * max(fz - z0, z1 - fz) + 1, ny = 2 * max(fy - y0, y1 - fy) + 1;
  for (int iz = 0; iz < nz; ++iz) {
    const int z = fz + nf_offset(iz);
    if (z < z0 || z > z1) continue;
    const float dz2 = slab_d2(qz, g.oz, g.h, z, z);
    if (dz2 > fminf(bd[K - 1], R2) * 1.0001f) continue;
    for (int iy = 0; iy < ny; ++iy) {
      const int y = fy + nf_offset(iy);
      if (y < y0 || y > y1) continue;
      const float tau = fminf(bd[K - 1], R2) * 1.0001f;
      const float dyz2 = dz2 + slab_d2(qy, g.oy, g.h, y, y);
      if (dyz2 > tau) continue;
      const float w = sqrtf(tau - dyz2) * 1.0001f;
      const int x0 = max((int)floorf((qx - w - g.ox) * g.inv_h), 0);
      const int x1 = min((int)floorf((qx + w - g.ox) * g.inv_h), g.dx - 1);
      if (x0 > x1) continue;
      scan_range_u<K>(sorted, cs(z, y, x0), cs(z, y, x1 + 1), qx, qy, qz, g.r2, bd, bi);
    }
  }
}

template <class CS>
__device__ __forceinline__ int chord_count_cs(const GridParams& g, const CS& cs, float qx, float qy, float qz,
                                              float R2, int need) {
  const float R = sqrtf(R2) * 1.0001f;
  const int z0 = max((int)floorf((qz - R - g.oz) * g.inv_h), 0), z1 = min((int)floorf((qz + R - g.oz) * g.inv_h), g.dz - 1);
  const int y0 = max((int)floorf((qy - R - g.oy) * g.inv_h), 0), y1 = min((int)floorf((qy + R - g.oy) * g.inv_h), g.dy - 1);
  const int fz = min(max((int)floorf((qz - g.oz) * g.inv_h), z0), z1);
  const int nz = 2 * max(fz - z0, z1 - fz) + 1;
  const float tau = R2 * 1.0001f;
  int c = 0;
  for (int iz = 0; iz < nz && c < need; ++iz) {
    const int z = fz + nf_offset(iz);
    if (z < z0 || z > z1) continue;
    const float dz2 = slab_d2(qz, g.oz, g.h, z, z);
    if (dz2 > tau) continue;
    for (int y = y0; y <= y1; ++y) {
      const float dyz2 = dz2 + slab_d2(qy, g.oy, g.h, y, y);
      const float w = sqrtf(fmaxf(tau - dyz2, 0.f)) * 1.0001f;
      const int x0 = max((int)floorf((qx - w - g.ox) * g.inv_h), 0);
      const int x1 = min((int)floorf((qx + w - g.ox) * g.inv_h), g.dx - 1);
      if (dyz2 <= tau && x0 <= x1) c += cs(z, y, x1 + 1) - cs(z, y, x0);
    }
  }
  return c;
}

// ---- mode 5: tile-grouped search. Candidates are bucketed by tile (KT^3 fine cells); one
// workgroup per tile stages the cell_start row segments of the tile's r-dilated region in LDS,
// so the per-row bound lookups of every query in the tile are LDS reads, and the lanes of a
// workgroup are spatial neighbours (similar search depth, little divergence).
#ifdef APN_DEBUG_BUILD   // earlier search strategy: debug build only (cross-checks, A/B tools)
constexpr int KT = 4;
constexpr int KT_LDS = 12288;   // ints of staged row bounds per workgroup (48 KB)

__device__ __forceinline__ int tile_of(const GridParams& g, float4 q, int tdx, int tdy) {
  const int fx = cell_coord(q.x, g.ox, g.inv_h, g.dx), fy = cell_coord(q.y, g.oy, g.inv_h, g.dy);
  const int fz = cell_coord(q.z, g.oz, g.inv_h, g.dz);
  return ((fz / KT) * tdy + fy / KT) * tdx + fx / KT;
}

__global__ __launch_bounds__(KNN_THREADS) void k_tile_count(const float4* __restrict__ q_pos,
                                                           const int* __restrict__ cand,
                                                           const int* __restrict__ n_cand_dev,
                                                           const GridParams* __restrict__ gp, int* __restrict__ ctile,
                                                           int* __restrict__ tile_cnt) {
  const int c = blockIdx.x * KNN_THREADS + threadIdx.x;
  if (c >= *n_cand_dev) return;
  const GridParams g = *gp;
  const int tdx = (g.dx + KT - 1) / KT, tdy = (g.dy + KT - 1) / KT;
  const int t = tile_of(g, q_pos[cand[c]], tdx, tdy);
  ctile[c] = t;
  atomicAdd(tile_cnt + t, 1);
}

__global__ __launch_bounds__(KNN_THREADS) void k_tile_scatter(const int* __restrict__ n_cand_dev,
                                                             const int* __restrict__ ctile,
                                                             const int* __restrict__ tile_start,
                                                             int* __restrict__ tile_cursor, int* __restrict__ order) {
  const int c = blockIdx.x * KNN_THREADS + threadIdx.x;
  if (c >= *n_cand_dev) return;
  const int t = ctile[c];
  order[tile_start[t] + atomicAdd(tile_cursor + t, 1)] = c;
}
#endif  // APN_DEBUG_BUILD

// Non-zero entries -> list of their indices (any order); n_list[0] = count. One atomic per
// 1024-entry block (per-wave atomics on the single counter serialised at the L2).
constexpr int LIST_THREADS = 1024;
__global__ __launch_bounds__(LIST_THREADS) void k_tile_list(const int* __restrict__ tile_cnt, int n_tiles_max,
                                                           int* __restrict__ list, int* __restrict__ n_list) {
  __shared__ int wcnt[LIST_THREADS / 64];
  __shared__ int sbase;
  const int t = blockIdx.x * LIST_THREADS + threadIdx.x;
  const bool ne = t < n_tiles_max && tile_cnt[t] > 0;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const unsigned long long bal = __ballot(ne);
  if (lane == 0) wcnt[wid] = __popcll(bal);
  __syncthreads();
  if (threadIdx.x == 0) {
    int tot = 0;
    for (int w = 0; w < LIST_THREADS / 64; ++w) {
      const int c = wcnt[w];
      wcnt[w] = tot;
      tot += c;
    }
    sbase = tot ? atomicAdd(n_list, tot) : 0;
  }
  __syncthreads();
  if (ne) list[sbase + wcnt[wid] + __popcll(bal & ((1ull << lane) - 1ull))] = t;
}

#ifdef APN_DEBUG_BUILD   // earlier search strategy: debug build only (cross-checks, A/B tools)
__global__ __launch_bounds__(KNN_THREADS) void k_knn_tiles(
    const float4* __restrict__ q_pos, const int* __restrict__ cand, const GridParams* __restrict__ gp,
    const int* __restrict__ cell_start, const float4* __restrict__ sorted, const int* __restrict__ tile_list,
    const int* __restrict__ n_list_dev, const int* __restrict__ tile_start, const int* __restrict__ tile_cnt,
    const int* __restrict__ order, int* __restrict__ flag, int* __restrict__ t_nbr) {
  __shared__ int sCS[KT_LDS];
  const GridParams g = *gp;
  const int n_list = *n_list_dev;
  const int tdx = (g.dx + KT - 1) / KT, tdy = (g.dy + KT - 1) / KT;
  const int D = g.kmax + 1;
  for (int li = blockIdx.x; li < n_list; li += gridDim.x) {
    const int t = tile_list[li];
    const int tx = t % tdx, ty = (t / tdx) % tdy, tz = t / (tdx * tdy);
    // staged region: rows z in [rz0, rz0+nz), y in [ry0, ry0+ny), bound entries x in [rx0, rx0+nx1)
    const int rz0 = max(tz * KT - D, 0), rz1 = min(tz * KT + KT - 1 + D, g.dz - 1);
    const int ry0 = max(ty * KT - D, 0), ry1 = min(ty * KT + KT - 1 + D, g.dy - 1);
    const int rx0 = max(tx * KT - D, 0), rx1 = min(tx * KT + KT + D, g.dx);
    int nz = rz1 - rz0 + 1, ny = ry1 - ry0 + 1;
    const int nx1 = rx1 - rx0 + 1;
    if (nz * ny * nx1 > KT_LDS) nz = 0;   // does not fit: every lookup goes to global memory
    const int tot = nz * ny * nx1;
    for (int e = threadIdx.x; e < tot; e += KNN_THREADS) {
      const int ix = e % nx1, r = e / nx1;
      const int iy = r % ny, iz = r / ny;
      sCS[e] = cell_start[((rz0 + iz) * g.dy + ry0 + iy) * g.dx + rx0 + ix];
    }
    __syncthreads();
    auto cs = [&](int z, int y, int x) -> int {
      const unsigned iz = z - rz0, iy = y - ry0, ix = x - rx0;
      if (iz < (unsigned)nz && iy < (unsigned)ny && ix < (unsigned)nx1) return sCS[(iz * ny + iy) * nx1 + ix];
      return cell_start[(z * g.dy + y) * g.dx + x];
    };
    const int n = tile_cnt[t], base = tile_start[t];
    for (int i = threadIdx.x; i < n; i += KNN_THREADS) {
      const int c = order[base + i];
      const float4 q = q_pos[cand[c]];
      float bd[KNN_K];
      int bi[KNN_K];
#pragma unroll
      for (int k = 0; k < KNN_K; ++k) { bd[k] = INFINITY; bi[k] = 0x7fffffff; }
      if (g.h > 0.25f * g.r) {
        scan_ball_cs<KNN_K>(g, cs, sorted, q.x, q.y, q.z, g.r2, bd, bi);
      } else {
        // balls r/4, (chord-count rejection at r), r/2, r -- as mode 4
        scan_ball_cs<KNN_K>(g, cs, sorted, q.x, q.y, q.z, 0.0625f * g.r2, bd, bi);
        if (!(bd[KNN_K - 1] < 0.0625f * g.r2 * (1.f - 2e-4f))) {
          if (chord_count_cs(g, cs, q.x, q.y, q.z, g.r2, KNN_K) < KNN_K) {
            bd[KNN_K - 1] = INFINITY;
          } else {
            scan_ball_cs<KNN_K>(g, cs, sorted, q.x, q.y, q.z, 0.25f * g.r2, bd, bi);
            if (!(bd[KNN_K - 1] < 0.25f * g.r2 * (1.f - 2e-4f)))
              scan_ball_cs<KNN_K>(g, cs, sorted, q.x, q.y, q.z, g.r2, bd, bi);
          }
        }
      }
      const bool surv = bd[KNN_K - 1] <= g.r2;
      flag[c] = surv;
      if (surv) {
        int4* nb = (int4*)(t_nbr + (int64_t)c * KNN_K);
        nb[0] = make_int4(bi[0], bi[1], bi[2], bi[3]);
        nb[1] = make_int4(bi[4], bi[5], bi[6], bi[7]);
      }
    }
    __syncthreads();
  }
}
#endif  // APN_DEBUG_BUILD

// Pass 1: coarse rejection. Queries with >= 8 points in the 27 coarse cells around them are
// compacted (in query order) per block into cand[blockIdx*256 ...]; blk_cnt[block] = count.
__global__ __launch_bounds__(KNN_THREADS) void k_knn_classify(const float4* __restrict__ q_pos,
                                                              const int* __restrict__ n_q_dev,
                                                              const GridParams* __restrict__ gp,
                                                              const int* __restrict__ ccount,
                                                              const int* __restrict__ csum27,
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
    if (cx >= 0 && cx < g.cdx && cy >= 0 && cy < g.cdy && cz >= 0 && cz < g.cdz) {
      cnt = csum27[(cz * g.cdy + cy) * g.cdx + cx];
    } else {   // a query outside the grid (the sampling bbox is padded by r): the clamped block
      for (int z = max(cz - 1, 0); z <= min(cz + 1, g.cdz - 1); ++z)
        for (int y = max(cy - 1, 0); y <= min(cy + 1, g.cdy - 1); ++y)
          for (int x = max(cx - 1, 0); x <= min(cx + 1, g.cdx - 1); ++x) cnt += ccount[(z * g.cdy + y) * g.cdx + x];
    }
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

// kNN counters of the debug build's instrumented kernels (apn_debug_knn_stats)
__device__ unsigned long long g_knn_stats[5 * 4];

#ifdef APN_DEBUG_BUILD   // earlier search strategy: debug build only (cross-checks, A/B tools)
// Pass 2: exact search for the compacted candidates. Survivors are compacted per block (order
// preserved) into slots [blockIdx*256, ...) of t_*; blk_cnt[block] = survivors.
// Profiling aid (mode 3 = mode 2 + counters): per query class {stop at 2h, rejected by the chord
// count, stop at 4h, stop at r, rejected at r}: {queries, cycles, rows, points} summed.

template <bool STATS>
__global__ __launch_bounds__(KNN_THREADS) void k_knn_search(
    const float4* __restrict__ q_pos, const int* __restrict__ q_ray, const int* __restrict__ cand,
    const int* __restrict__ n_cand_dev, const GridParams* __restrict__ gp, const int* __restrict__ cell_start,
    const float4* __restrict__ sorted, float4* __restrict__ t_pos, int* __restrict__ t_ray,
    int* __restrict__ t_nbr, int* __restrict__ blk_cnt, int mode) {
  int ctr[2] = {0, 0};
  int* const cp = STATS ? ctr : nullptr;
  int cls = 0;
  const unsigned long long t0 = STATS ? clock64() : 0;
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
    if (mode >= 2) {
      // ball 2h (most samples inside the cloud stop here); then an exact rejection bound from the
      // r-ball's chord counts (87% of the remaining non-survivors, no point reads); then balls
      // 4h and r, rows nearest-first
      scan_ball_nf<KNN_K>(g, cell_start, sorted, q.x, q.y, q.z, 4.f * g.h * g.h, bd, bi, cp);
      if (!(bd[KNN_K - 1] < 4.f * g.h * g.h * (1.f - 2e-4f)) && 2.f * g.h < g.r) {
        if (chord_count(g, cell_start, q.x, q.y, q.z, g.r2, KNN_K, cp) < KNN_K) {
          bd[KNN_K - 1] = INFINITY;   // < 8 points within r: not a survivor
          cls = 1;
        } else {
          float R = 4.f * g.h;
          cls = 2;
          for (;;) {
            const float Rl = fminf(R, g.r);
            const float R2 = Rl >= g.r ? g.r2 : Rl * Rl;
            scan_ball_nf<KNN_K>(g, cell_start, sorted, q.x, q.y, q.z, R2, bd, bi, cp);
            if (Rl >= g.r || bd[KNN_K - 1] < R2 * (1.f - 2e-4f)) break;
            R *= 2.f;
          }
          if (!(bd[KNN_K - 1] < 16.f * g.h * g.h * (1.f - 2e-4f))) cls = bd[KNN_K - 1] <= g.r2 ? 3 : 4;
        }
      }
    } else if (mode == 0) {
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
  if (STATS && c < nc) {
    const unsigned long long dt = clock64() - t0;
    atomicAdd(&g_knn_stats[4 * cls + 0], 1ull);
    atomicAdd(&g_knn_stats[4 * cls + 1], dt);
    atomicAdd(&g_knn_stats[4 * cls + 2], (unsigned long long)ctr[0]);
    atomicAdd(&g_knn_stats[4 * cls + 3], (unsigned long long)ctr[1]);
  }
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

// ---- mode 4: the search split into two passes so each wave runs a uniform loop structure
// (one lane per query, lanes of a wave in the same phase; the single-pass kernel's lanes run
// different phases side by side and the wave executes their union).
// Pass A, every candidate: ball r/4; if 8 neighbours lie inside it the sample is a survivor;
// else the r-ball chord count (exact upper bound) rejects it when < 8; the rest are appended to
// the hard list. Results per candidate slot: flag[c] (survivor) and t_nbr[c].
__global__ __launch_bounds__(KNN_THREADS) void k_knn_pass_a(
    const float4* __restrict__ q_pos, const int* __restrict__ cand, const int* __restrict__ n_cand_dev,
    const GridParams* __restrict__ gp, const int* __restrict__ cell_start, const float4* __restrict__ sorted,
    int* __restrict__ flag, int* __restrict__ t_nbr, int* __restrict__ hard, int* __restrict__ n_hard) {
  const int nc = *n_cand_dev;
  const int c = blockIdx.x * KNN_THREADS + threadIdx.x;
  const GridParams g = *gp;
  bool push = false;
  if (c < nc) {
    const float4 q = q_pos[cand[c]];
    float bd[KNN_K];
    int bi[KNN_K];
#pragma unroll
    for (int k = 0; k < KNN_K; ++k) { bd[k] = INFINITY; bi[k] = 0x7fffffff; }
    bool done = true;
    if (g.h > 0.25f * g.r) {  // coarse (cell-capped) grid: the whole search here
      scan_ball_nf<KNN_K>(g, cell_start, sorted, q.x, q.y, q.z, g.r2, bd, bi);
    } else {
      const float R2 = 0.0625f * g.r2;   // ball r/4
      scan_ball_nf<KNN_K>(g, cell_start, sorted, q.x, q.y, q.z, R2, bd, bi);
      if (!(bd[KNN_K - 1] < R2 * (1.f - 2e-4f))) {
        if (chord_count(g, cell_start, q.x, q.y, q.z, g.r2, KNN_K) < KNN_K)
          bd[KNN_K - 1] = INFINITY;   // < 8 points within r
        else
          done = false;
      }
    }
    if (done) {
      const bool surv = bd[KNN_K - 1] <= g.r2;
      flag[c] = surv;
      if (surv) {
        int4* nb = (int4*)(t_nbr + (int64_t)c * KNN_K);
        nb[0] = make_int4(bi[0], bi[1], bi[2], bi[3]);
        nb[1] = make_int4(bi[4], bi[5], bi[6], bi[7]);
      }
    } else {
      push = true;
    }
  }
  const int lane = threadIdx.x & 63;
  const unsigned long long bal = __ballot(push);
  if (bal) {
    int base = 0;
    if (lane == 0) base = atomicAdd(n_hard, __popcll(bal));
    base = __shfl(base, 0, 64);
    if (push) hard[base + __popcll(bal & ((1ull << lane) - 1ull))] = c;
  }
}

// Pass B, the hard list: balls r/2, r with nearest-first rows and running culling.
__global__ __launch_bounds__(KNN_THREADS) void k_knn_pass_b(
    const float4* __restrict__ q_pos, const int* __restrict__ cand, const int* __restrict__ hard,
    const int* __restrict__ n_hard, const GridParams* __restrict__ gp, const int* __restrict__ cell_start,
    const float4* __restrict__ sorted, int* __restrict__ flag, int* __restrict__ t_nbr) {
  const int i = blockIdx.x * KNN_THREADS + threadIdx.x;
  if (i >= *n_hard) return;
  const GridParams g = *gp;
  const int c = hard[i];
  const float4 q = q_pos[cand[c]];
  float bd[KNN_K];
  int bi[KNN_K];
#pragma unroll
  for (int k = 0; k < KNN_K; ++k) { bd[k] = INFINITY; bi[k] = 0x7fffffff; }
  // balls r/2, r
  scan_ball_nf<KNN_K>(g, cell_start, sorted, q.x, q.y, q.z, 0.25f * g.r2, bd, bi);
  if (!(bd[KNN_K - 1] < 0.25f * g.r2 * (1.f - 2e-4f)))
    scan_ball_nf<KNN_K>(g, cell_start, sorted, q.x, q.y, q.z, g.r2, bd, bi);
  const bool surv = bd[KNN_K - 1] <= g.r2;
  flag[c] = surv;
  if (surv) {
    int4* nb = (int4*)(t_nbr + (int64_t)c * KNN_K);
    nb[0] = make_int4(bi[0], bi[1], bi[2], bi[3]);
    nb[1] = make_int4(bi[4], bi[5], bi[6], bi[7]);
  }
}
#endif  // APN_DEBUG_BUILD

// Ball scan as a per-lane state machine ("flat" loop): every iteration a lane either consumes
// points of its current row range, or takes over the row range it loaded one step earlier and
// examines the next row (nearest-first order, culled by the running K-th best) to load its
// bounds. The wave therefore advances all lanes together whatever their row lengths (the nested
// row/point loops of scan_ball_nf run the union of every lane's trip counts), and each row's
// bounds load has a whole point-consuming phase to arrive. Same point set and result as
// scan_ball_nf.
template <int K>
__device__ __forceinline__ void scan_ball_flat(const GridParams& g, const int* __restrict__ cell_start,
                                               const float4* __restrict__ sorted, float qx, float qy, float qz,
                                               float R2, float (&bd)[K], int (&bi)[K]) {
  const float R = sqrtf(R2) * 1.0001f;
  const int z0 = max((int)floorf((qz - R - g.oz) * g.inv_h), 0), z1 = min((int)floorf((qz + R - g.oz) * g.inv_h), g.dz - 1);
  const int y0 = max((int)floorf((qy - R - g.oy) * g.inv_h), 0), y1 = min((int)floorf((qy + R - g.oy) * g.inv_h), g.dy - 1);
  const int fz = min(max((int)floorf((qz - g.oz) * g.inv_h), z0), z1);
  const int fy = min(max((int)floorf((qy - g.oy) * g.inv_h), y0), y1);
  const int nz = 2 * max(fz - z0, z1 - fz) + 1, ny = 2 * max(fy - y0, y1 - fy) + 1;
  const int nrows = (z1 < z0 || y1 < y0) ? 0 : nz * ny;
  int cur = 0;                     // next row slot (iz * ny + iy) to examine
  int b = 0, e = 0;                // range being consumed
  int pb = 0, pe = 0;              // range loaded for the next row
  bool pend = false;
  for (;;) {
    const bool has_pts = b < e;
    if (!has_pts && !pend && cur >= nrows) break;
    if (has_pts) {
      const int p1 = b + 1 < e ? b + 1 : b;
      const float4 P0 = sorted[b], P1 = sorted[p1];
      const float d0x = qx - P0.x, d0y = qy - P0.y, d0z = qz - P0.z;
      const float d0 = (d0x * d0x + d0y * d0y) + d0z * d0z;
      const float d1x = qx - P1.x, d1y = qy - P1.y, d1z = qz - P1.z;
      const float d1 = (d1x * d1x + d1y * d1y) + d1z * d1z;
      if (d0 <= g.r2) knn_insert_unique<K>(d0, __float_as_int(P0.w), bd, bi);
      if (p1 != b && d1 <= g.r2) knn_insert_unique<K>(d1, __float_as_int(P1.w), bd, bi);
      b += 2;
      if (b > e) b = e;
    } else {
      if (pend) { b = pb; e = pe; pend = false; }
      // examine one row slot
      if (cur < nrows) {
        const int iz = cur / ny, iy = cur - iz * ny;
        ++cur;
        const int z = fz + nf_offset(iz), y = fy + nf_offset(iy);
        if (z >= z0 && z <= z1 && y >= y0 && y <= y1) {
          const float tau = fminf(bd[K - 1], R2) * 1.0001f;
          const float dyz2 = slab_d2(qz, g.oz, g.h, z, z) + slab_d2(qy, g.oy, g.h, y, y);
          if (dyz2 <= tau) {
            const float w = sqrtf(tau - dyz2) * 1.0001f;
            const int x0 = max((int)floorf((qx - w - g.ox) * g.inv_h), 0);
            const int x1 = min((int)floorf((qx + w - g.ox) * g.inv_h), g.dx - 1);
            if (x0 <= x1) {
              const int row = (z * g.dy + y) * g.dx;
              pb = cell_start[row + x0];
              pe = cell_start[row + x1 + 1];
              pend = true;
            }
          }
        }
      }
    }
  }
}

// scan_ball_flat with incremental slot iteration: slabs advance in nearest-first order, and a
// slab only enumerates the y offsets whose rows can intersect the ball under the current bound
// (|dy| <= floor(sqrt(tau - dz^2)/h) + 1), so the square's corners and culled slabs cost no
// iterations; no integer division per row.
// S > 1: the caller is one of S lanes sharing the query; in every slab this lane walks only the
// nearest-first y slots iy = slice, slice + S, ... (the slot -> row map depends on the query
// alone, so the lanes partition each slab's rows whatever bound sizes the slab). Pruning with
// the lane-local K-th distance stays exact: K points of this lane already beat every point of a
// pruned row.
// DUP = false: the caller's list holds no point this scan can reach (a first scan): plain inserts,
// no duplicate check (every point of the ball is visited at most once within one scan).
template <int K, bool STATS, int S, bool DUP, class L>
__device__ __forceinline__ void scan_ball_flat2_l(const GridParams& g, const int* __restrict__ cell_start,
                                                  const float4* __restrict__ sorted, float qx, float qy, float qz,
                                                  float R2, L& lst, unsigned* ctr = nullptr, int slice = 0) {
  const float R = bound_sqrt(R2);
  const __amdgpu_buffer_rsrc_t prs = knn_rsrc(sorted, g.np * 16);
  const __amdgpu_buffer_rsrc_t crs = knn_rsrc(cell_start, (g.nf + 1) * 4);
  const int z0 = max((int)floorf((qz - R - g.oz) * g.inv_h), 0), z1 = min((int)floorf((qz + R - g.oz) * g.inv_h), g.dz - 1);
  const int y0 = max((int)floorf((qy - R - g.oy) * g.inv_h), 0), y1 = min((int)floorf((qy + R - g.oy) * g.inv_h), g.dy - 1);
  const int fz = min(max((int)floorf((qz - g.oz) * g.inv_h), z0), z1);
  const int fy = min(max((int)floorf((qy - g.oy) * g.inv_h), y0), y1);
  const int nz = (z1 < z0 || y1 < y0) ? 0 : 2 * max(fz - z0, z1 - fz) + 1;
  const int ny = 2 * max(fy - y0, y1 - fy) + 1;
  int iz = -1, iy = 0, nyz = 0;    // current slab (nf index), next y slot, y slots of the slab
  int z = 0;
  float dz2 = 0.f;
  int b = 0, e = 0;                // range being consumed
  int pb = 0, pe = 0;              // range loaded for the next row
  bool pend = false;
  for (;;) {
    const bool has_pts = b < e;
    const bool rows_left = iy < nyz || iz + 1 < nz;
    if (!has_pts && !pend && !rows_left) break;
    if (STATS) ctr[has_pts ? 1 : 0]++;
    if (has_pts) {
      const int p1 = b + 1 < e ? b + 1 : b;
      const float4 P0 = kBufferPoints ? knn_ld_pt(prs, b) : sorted[b];
      const float4 P1 = kBufferPoints ? knn_ld_pt(prs, b + 1) : sorted[p1];
      // the indices pass through an empty asm so they are loaded with the coordinates (one
      // 16-B load per point) instead of by a separate load inside the insert branch, whose
      // vmcnt(0) would also drain the row-bound loads in flight
      int i0 = __float_as_int(P0.w), i1 = __float_as_int(P1.w);
      asm("" : "+v"(i0), "+v"(i1));
      const float d0x = qx - P0.x, d0y = qy - P0.y, d0z = qz - P0.z;
      const float d0 = (d0x * d0x + d0y * d0y) + d0z * d0z;
      const float d1x = qx - P1.x, d1y = qy - P1.y, d1z = qz - P1.z;
      const float d1 = (d1x * d1x + d1y * d1y) + d1z * d1z;
      if (d0 <= g.r2) lst.template insert<DUP>(d0, i0);
      if (p1 != b && d1 <= g.r2) lst.template insert<DUP>(d1, i1);
      b += 2;
      if (b > e) b = e;
    } else {
      if (pend) { b = pb; e = pe; pend = false; }
      const float tau = fminf(lst.worst(), R2) * 1.0001f;
      if (iy >= nyz) {               // next slab
        ++iz;
        iy = S == 1 ? 0 : slice;
        nyz = 0;
        if (iz < nz) {
          z = fz + nf_offset(iz);
          if (z >= z0 && z <= z1) {
            dz2 = slab_d2(qz, g.oz, g.h, z, z);
            if (dz2 <= tau) {
              const int my = (int)floorf(bound_sqrt(tau - dz2) * g.inv_h) + 1;
              nyz = min(2 * my + 1, ny);
            }
          }
        }
      } else {                       // one row of the slab
        const int y = fy + nf_offset(iy);
        iy += S;
        if (y >= y0 && y <= y1) {
          const float dyz2 = dz2 + slab_d2(qy, g.oy, g.h, y, y);
          if (dyz2 <= tau) {
            const float w = bound_sqrt(tau - dyz2);
            const int x0 = max((int)floorf((qx - w - g.ox) * g.inv_h), 0);
            const int x1 = min((int)floorf((qx + w - g.ox) * g.inv_h), g.dx - 1);
            if (x0 <= x1) {
              const int row = (z * g.dy + y) * g.dx;
              pb = kBufferPoints ? knn_ld_i32(crs, row + x0) : cell_start[row + x0];
              pe = kBufferPoints ? knn_ld_i32(crs, row + x1 + 1) : cell_start[row + x1 + 1];
              pend = true;
            }
          }
        }
      }
    }
  }
}

template <int K, bool STATS = false, int S = 1, bool DUP = true>
__device__ __forceinline__ void scan_ball_flat2(const GridParams& g, const int* __restrict__ cell_start,
                                                const float4* __restrict__ sorted, float qx, float qy, float qz,
                                                float R2, float (&bd)[K], int (&bi)[K], unsigned* ctr = nullptr,
                                                int slice = 0) {
  ArrList<K> lst{bd, bi};
  scan_ball_flat2_l<K, STATS, S, DUP>(g, cell_start, sorted, qx, qy, qz, R2, lst, ctr, slice);
}

// ---- mode 9: pass B on a second, anisotropic grid. A hard query's r-ball scan on the fine grid
// (h = r/8) walks ~220 (z, y) rows but reads only ~80 points: rows dominate. The second grid keeps
// the fine x cells (row chords stay tight) and merges AG_F x AG_F fine cells in y and z, so the
// r-ball has ~AG_F^2 fewer rows, each covering AG_F^2 fine rows. Its cell boundaries coincide with
// fine ones (AG_F a power of two: the products below are exact), and each point's cell is derived
// from its fine cell, so the cell-box distance bounds of the scan hold exactly as on the fine grid.
// Built per frame from the fine grid's sorted points (atomic counting sort: the order inside a
// cell is arbitrary, the top-K is not -- distance then index).
struct AGrid {
  float ox, oy, oz, hx;
  float hy, hz, ihx, ihy;
  float ihz, r, r2;
  int np;   // points in sorted2 (the buffer bound of the scans' point loads)
  int dx, dy, dz, nf;
};

__global__ void k_agrid_params(const GridParams* __restrict__ gp, int f, int np, AGrid* __restrict__ ag) {
  if (threadIdx.x != 0) return;
  const GridParams g = *gp;
  AGrid a;
  a.ox = g.ox; a.oy = g.oy; a.oz = g.oz;
  a.hx = g.h; a.hy = a.hz = g.h * (float)f;
  a.ihx = g.inv_h; a.ihy = a.ihz = g.inv_h / (float)f;
  a.r = g.r; a.r2 = g.r2; a.np = np;
  a.dx = g.dx; a.dy = (g.dy + f - 1) / f; a.dz = (g.dz + f - 1) / f;
  a.nf = a.dx * a.dy * a.dz;
  *ag = a;
}

__global__ void k_agrid_count(const float4* __restrict__ sorted, int64_t N, const GridParams* __restrict__ gp, int f,
                              int* __restrict__ counts, int* __restrict__ pcell) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const GridParams g = *gp;
  const float4 P = sorted[i];
  const int cx = cell_coord(P.x, g.ox, g.inv_h, g.dx);
  const int cy = cell_coord(P.y, g.oy, g.inv_h, g.dy) / f;
  const int cz = cell_coord(P.z, g.oz, g.inv_h, g.dz) / f;
  const int dy2 = (g.dy + f - 1) / f;
  const int cell = (cz * dy2 + cy) * g.dx + cx;
  pcell[i] = cell;
  atomicAdd(counts + cell, 1);
}

__global__ void k_agrid_scatter(const float4* __restrict__ sorted, int64_t N, const int* __restrict__ pcell,
                                const int* __restrict__ cell_start, int* __restrict__ cursor,
                                float4* __restrict__ sorted2) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const int cell = pcell[i];
  sorted2[cell_start[cell] + atomicAdd(cursor + cell, 1)] = sorted[i];
}

// scan_ball_flat2 on the anisotropic grid (cell sides hx, hy, hz): the same lock-step row/point
// state machine, nearest-first slabs, running K-th-best culling with 1e-4 slack.
// PTS points per point step (2 or 4). S > 1: one of S lanes sharing the query, walking the y slots
// slice, slice + S, ... of every slab (as scan_ball_flat2_l).
template <int K, bool STATS, int PTS, bool DUP, class L, int S = 1>
__device__ __forceinline__ void scan_ball_aniso_l(const AGrid& g, const int* __restrict__ cell_start,
                                                  const float4* __restrict__ sorted, float qx, float qy, float qz,
                                                  float R2, L& lst, unsigned* ctr = nullptr, int slice = 0) {
  const float R = bound_sqrt(R2);
  const __amdgpu_buffer_rsrc_t prs = knn_rsrc(sorted, g.np * 16);
  const __amdgpu_buffer_rsrc_t crs = knn_rsrc(cell_start, (g.nf + 1) * 4);
  const int z0 = max((int)floorf((qz - R - g.oz) * g.ihz), 0), z1 = min((int)floorf((qz + R - g.oz) * g.ihz), g.dz - 1);
  const int y0 = max((int)floorf((qy - R - g.oy) * g.ihy), 0), y1 = min((int)floorf((qy + R - g.oy) * g.ihy), g.dy - 1);
  const int fz = min(max((int)floorf((qz - g.oz) * g.ihz), z0), z1);
  const int fy = min(max((int)floorf((qy - g.oy) * g.ihy), y0), y1);
  const int nz = (z1 < z0 || y1 < y0) ? 0 : 2 * max(fz - z0, z1 - fz) + 1;
  const int ny = 2 * max(fy - y0, y1 - fy) + 1;
  int iz = -1, iy = 0, nyz = 0;
  int z = 0;
  float dz2 = 0.f;
  int b = 0, e = 0, pb = 0, pe = 0;
  bool pend = false;
  for (;;) {
    const bool has_pts = b < e;
    const bool rows_left = iz < nz && (iy < nyz || iz + 1 < nz);
    if (!has_pts && !pend && !rows_left) break;
    if (STATS) ctr[has_pts ? 1 : 0]++;
    if (has_pts) {
      float4 P[PTS];
      int id[PTS];
#pragma unroll
      for (int u = 0; u < PTS; ++u) {
        if constexpr (kBufferPoints) {
          // slots past the row read the next cells' points or, past the array, zeros -- b + u < e masks them
          P[u] = knn_ld_pt(prs, b + u);
        } else {
          P[u] = sorted[min(b + u, e - 1)];
        }
        id[u] = __float_as_int(P[u].w);
      }
#pragma unroll
      for (int u = 0; u < PTS; ++u) asm("" : "+v"(id[u]));
#pragma unroll
      for (int u = 0; u < PTS; ++u) {
        const float dx = qx - P[u].x, dy = qy - P[u].y, dz = qz - P[u].z;
        const float d = (dx * dx + dy * dy) + dz * dz;
        if (b + u < e && d <= g.r2) lst.template insert<DUP>(d, id[u]);
      }
      b += PTS;
      if (b > e) b = e;
    } else {
      if (pend) { b = pb; e = pe; pend = false; }
      const float tau = fminf(lst.worst(), R2) * 1.0001f;
      if (iy >= nyz) {
        ++iz;
        iy = S == 1 ? 0 : slice;
        nyz = 0;
        if (iz < nz) {
          z = fz + nf_offset(iz);
          if (z >= z0 && z <= z1) {
            dz2 = slab_d2(qz, g.oz, g.hz, z, z);
            if (dz2 <= tau) {
              const int my = (int)floorf(bound_sqrt(tau - dz2) * g.ihy) + 1;
              nyz = min(2 * my + 1, ny);
            }
          }
        }
      } else {
        const int y = fy + nf_offset(iy);
        iy += S;
        if (y >= y0 && y <= y1) {
          const float dyz2 = dz2 + slab_d2(qy, g.oy, g.hy, y, y);
          if (dyz2 <= tau) {
            const float w = bound_sqrt(tau - dyz2);
            const int x0 = max((int)floorf((qx - w - g.ox) * g.ihx), 0);
            const int x1 = min((int)floorf((qx + w - g.ox) * g.ihx), g.dx - 1);
            if (x0 <= x1) {
              const int row = (z * g.dy + y) * g.dx;
              pb = kBufferPoints ? knn_ld_i32(crs, row + x0) : cell_start[row + x0];
              pe = kBufferPoints ? knn_ld_i32(crs, row + x1 + 1) : cell_start[row + x1 + 1];
              pend = true;
            }
          }
        }
      }
    }
  }
}

template <int K, bool STATS = false, int PTS = 2, bool DUP = true>
__device__ __forceinline__ void scan_ball_aniso(const AGrid& g, const int* __restrict__ cell_start,
                                                const float4* __restrict__ sorted, float qx, float qy, float qz,
                                                float R2, float (&bd)[K], int (&bi)[K], unsigned* ctr = nullptr) {
  ArrList<K> lst{bd, bi};
  scan_ball_aniso_l<K, STATS, PTS, DUP>(g, cell_start, sorted, qx, qy, qz, R2, lst, ctr);
}

// ---- mode 6: per-cell rejection bound. For every fine cell C holding a candidate, U(C) = number
// of points in cells whose box lies within r of C's box -- an upper bound on the points within r of
// ANY query in C (also of a query just outside the grid, clamped into C: its distance to a point
// exceeds the box-box distance). Candidates with U(C) < 8 are rejected without a search; the
// cell count is ~10x smaller than the candidate count, so the bound costs a tenth of a per-query
// chord count.
__global__ __launch_bounds__(KNN_THREADS) void k_mark_cells(const float4* __restrict__ q_pos,
                                                           const int* __restrict__ cand,
                                                           const int* __restrict__ n_cand_dev,
                                                           const GridParams* __restrict__ gp, int* __restrict__ ccell,
                                                           int* __restrict__ mark) {
  const int c = blockIdx.x * KNN_THREADS + threadIdx.x;
  if (c >= *n_cand_dev) return;
  const GridParams g = *gp;
  const float4 q = q_pos[cand[c]];
  const int cell = (cell_coord(q.z, g.oz, g.inv_h, g.dz) * g.dy + cell_coord(q.y, g.oy, g.inv_h, g.dy)) * g.dx +
                   cell_coord(q.x, g.ox, g.inv_h, g.dx);
  ccell[c] = cell;
  mark[cell] = 1;
}

#ifdef APN_DEBUG_BUILD   // earlier search strategy: debug build only (cross-checks, A/B tools)
__global__ __launch_bounds__(KNN_THREADS) void k_cell_bound(const GridParams* __restrict__ gp,
                                                           const int* __restrict__ cell_start,
                                                           const int* __restrict__ list, const int* __restrict__ n_list,
                                                           int* __restrict__ ubound) {
  const int i = blockIdx.x * KNN_THREADS + threadIdx.x;
  if (i >= *n_list) return;
  const GridParams g = *gp;
  const int cell = list[i];
  const int cx = cell % g.dx, cy = (cell / g.dx) % g.dy, cz = cell / (g.dx * g.dy);
  const float lim = g.r2 * 1.0002f * g.inv_h * g.inv_h;   // (r/h)^2 with slack
  const int K = (int)ceilf(sqrtf(lim)) + 1;
  int u = 0;
  for (int dz = -K; dz <= K; ++dz) {
    const int z = cz + dz;
    if (z < 0 || z >= g.dz) continue;
    const float gz = (float)max(abs(dz) - 1, 0);
    for (int dy = -K; dy <= K; ++dy) {
      const int y = cy + dy;
      const float gy = (float)max(abs(dy) - 1, 0);
      const float rem = lim - gz * gz - gy * gy;
      if (y < 0 || y >= g.dy || rem < 0.f) continue;
      const int kx = (int)floorf(__builtin_amdgcn_sqrtf(rem)) + 1;
      const int row = (z * g.dy + y) * g.dx;
      u += cell_start[row + min(cx + kx, g.dx - 1) + 1] - cell_start[row + max(cx - kx, 0)];
    }
  }
  ubound[cell] = u;
}
#endif  // APN_DEBUG_BUILD

// Mode 8: the cell bound at three radii (r/4, r/2, r) in one pass -- u4[cell], u2[cell], u1[cell] --
// so a query skips every ball level that cannot hold 8 points for any query of its cell.
__global__ __launch_bounds__(KNN_THREADS) void k_cell_bound3(const GridParams* __restrict__ gp,
                                                            const int* __restrict__ cell_start,
                                                            const int* __restrict__ list,
                                                            const int* __restrict__ n_list, int* __restrict__ u1,
                                                            int* __restrict__ u2, int* __restrict__ u4) {
  const int i = blockIdx.x * KNN_THREADS + threadIdx.x;
  if (i >= *n_list) return;
  const GridParams g = *gp;
  const int cell = list[i];
  const int cx = cell % g.dx, cy = (cell / g.dx) % g.dy, cz = cell / (g.dx * g.dy);
  // (r/h)^2 with slack. The row half-widths below take v_sqrt_f32 (~1 ulp): the 2e-4 slack on lim
  // moves sqrt(rem) by >= 8e-4 cells (rem <= 64), so floor(sqrt(rem)) never drops below the exact
  // bound's (as in the ball scans' bound_sqrt)
  const float lim = g.r2 * 1.0002f * g.inv_h * g.inv_h;
  const int K = (int)ceilf(sqrtf(lim)) + 1;
  const __amdgpu_buffer_rsrc_t crs = knn_rsrc(cell_start, (g.nf + 1) * 4);
#ifdef APN_KNN_CB_GLOBAL   // A/B: the row bounds as global loads
  auto CS = [&](int x) { return cell_start[x]; };
#else
  auto CS = [&](int x) { return kBufferPoints ? knn_ld_i32(crs, x) : cell_start[x]; };
#endif
  int a1 = 0, a2 = 0, a4 = 0;
  for (int dz = -K; dz <= K; ++dz) {
    const int z = cz + dz;
    if (z < 0 || z >= g.dz) continue;
    const float gz = (float)max(abs(dz) - 1, 0);
    for (int dy = -K; dy <= K; ++dy) {
      const int y = cy + dy;
      const float gy = (float)max(abs(dy) - 1, 0);
      const float rem = lim - gz * gz - gy * gy;
      if (y < 0 || y >= g.dy || rem < 0.f) continue;
      const int row = (z * g.dy + y) * g.dx;
      const int kx = (int)floorf(__builtin_amdgcn_sqrtf(rem)) + 1;
      a1 += CS(row + min(cx + kx, g.dx - 1) + 1) - CS(row + max(cx - kx, 0));
      const float rem2 = 0.25f * lim - gz * gz - gy * gy;
      if (rem2 >= 0.f) {
        const int k2 = (int)floorf(__builtin_amdgcn_sqrtf(rem2)) + 1;
        a2 += CS(row + min(cx + k2, g.dx - 1) + 1) - CS(row + max(cx - k2, 0));
        const float rem4 = 0.0625f * lim - gz * gz - gy * gy;
        if (rem4 >= 0.f) {
          const int k4 = (int)floorf(__builtin_amdgcn_sqrtf(rem4)) + 1;
          a4 += CS(row + min(cx + k4, g.dx - 1) + 1) - CS(row + max(cx - k4, 0));
        }
      }
    }
  }
  u1[cell] = a1;
  u2[cell] = a2;
  u4[cell] = a4;
}

// k_cell_bound3 with 16 lanes per cell, for short cell lists (ray shards): one thread per cell
// walks its ~650 row loads in sequence, and with few cells that walk sets the launch time (a
// shard of 1/8 of a C2 frame took 117 us against 190 for the whole frame). Lane l takes every
// 16th (z, y) row of the window; the integer sums are combined with shuffles (exact, any order).
// On a full frame the list is long and the plain kernel is load-throughput bound (the 16-lane
// form measured 2x slower there), so apn_knn_radius picks by query count.
constexpr int CB_LANES = 16;
template <int CB_LANES>
__global__ __launch_bounds__(KNN_THREADS) void k_cell_bound3w(const GridParams* __restrict__ gp,
                                                             const int* __restrict__ cell_start,
                                                             const int* __restrict__ list,
                                                             const int* __restrict__ n_list, int* __restrict__ u1,
                                                             int* __restrict__ u2, int* __restrict__ u4) {
  const int nl = *n_list;
  const GridParams g = *gp;
  const int sub = threadIdx.x % CB_LANES;
  const float lim = g.r2 * 1.0002f * g.inv_h * g.inv_h;   // (r/h)^2 with slack, as k_cell_bound3
  const int K = (int)ceilf(sqrtf(lim)) + 1;
  const int W = 2 * K + 1;
  for (int base = blockIdx.x * (KNN_THREADS / CB_LANES); base < nl; base += gridDim.x * (KNN_THREADS / CB_LANES)) {
    const int i = base + threadIdx.x / CB_LANES;
    const bool ok = i < nl;
    const int cell = ok ? list[i] : 0;
    const int cx = cell % g.dx, cy = (cell / g.dx) % g.dy, cz = cell / (g.dx * g.dy);
    int a1 = 0, a2 = 0, a4 = 0;
    if (ok) {
      for (int p = sub; p < W * W; p += CB_LANES) {
        const int dz = p / W - K, dy = p % W - K;
        const int z = cz + dz, y = cy + dy;
        if (z < 0 || z >= g.dz || y < 0 || y >= g.dy) continue;
        const float gz = (float)max(abs(dz) - 1, 0), gy = (float)max(abs(dy) - 1, 0);
        const float rem = lim - gz * gz - gy * gy;
        if (rem < 0.f) continue;
        const int row = (z * g.dy + y) * g.dx;
        const int kx = (int)floorf(__builtin_amdgcn_sqrtf(rem)) + 1;
        a1 += cell_start[row + min(cx + kx, g.dx - 1) + 1] - cell_start[row + max(cx - kx, 0)];
        const float rem2 = 0.25f * lim - gz * gz - gy * gy;
        if (rem2 >= 0.f) {
          const int k2 = (int)floorf(__builtin_amdgcn_sqrtf(rem2)) + 1;
          a2 += cell_start[row + min(cx + k2, g.dx - 1) + 1] - cell_start[row + max(cx - k2, 0)];
          const float rem4 = 0.0625f * lim - gz * gz - gy * gy;
          if (rem4 >= 0.f) {
            const int k4 = (int)floorf(__builtin_amdgcn_sqrtf(rem4)) + 1;
            a4 += cell_start[row + min(cx + k4, g.dx - 1) + 1] - cell_start[row + max(cx - k4, 0)];
          }
        }
      }
    }
#pragma unroll
    for (int o = CB_LANES / 2; o > 0; o >>= 1) {
      a1 += __shfl_xor(a1, o, 64);
      a2 += __shfl_xor(a2, o, 64);
      a4 += __shfl_xor(a4, o, 64);
    }
    if (ok && sub == 0) {
      u1[cell] = a1;
      u2[cell] = a2;
      u4[cell] = a4;
    }
  }
}

// Heavy-first block order for the kNN passes of short launches (ray shards). A launch of ~1M
// queries fills the chip for only a few rounds of waves, so it waits on its slowest workgroups:
// the ones whose queries sit in dense cells. k_block_cost sums a per-query work estimate over
// each workgroup's 256 queries (pass A: the point count of the ball it scans, u4 or u1 of its
// cell; pass B: u2 + u1 or u1 by its first level); k_order_blocks (one workgroup) deals the block
// ids into 33 buckets by the bit length of their cost, heaviest bucket first, and the pass reads
// its block id through that permutation. Query results do not depend on the order.
template <bool PASS_B>
__global__ __launch_bounds__(KNN_THREADS) void k_block_cost(
    const int* __restrict__ n_a, const int* __restrict__ list1, const int* __restrict__ n1_dev,
    const int* __restrict__ list2, const int* __restrict__ n2_dev, const GridParams* __restrict__ gp,
    const int* __restrict__ ccell, const int* __restrict__ u1, const int* __restrict__ u2,
    const int* __restrict__ u4, int* __restrict__ cost) {
  __shared__ int sw[KNN_THREADS / 64];
  const int i = blockIdx.x * KNN_THREADS + threadIdx.x;
  int w = 0;
  if (!PASS_B) {
    if (i < *n_a) {
      const int cell = ccell[i];
      const int a1 = u1[cell];
      w = a1 < KNN_K ? 1 : (gp->h > 0.25f * gp->r ? a1 : u4[cell] + 1);
    }
  } else {
    const int n1 = *n1_dev, n2 = *n2_dev;
    if (i < n1 + n2) {
      const int hc = i < n1 ? list1[i] : list2[i - n1];
      const int cell = ccell[hc >> 1];
      w = (hc & 1) ? u1[cell] : u2[cell] + u1[cell];
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) w += __shfl_xor(w, o, 64);
  if ((threadIdx.x & 63) == 0) sw[threadIdx.x >> 6] = w;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
#pragma unroll
    for (int k = 0; k < KNN_THREADS / 64; ++k) t += sw[k];
    cost[blockIdx.x] = t;
  }
}

constexpr int ORDER_THREADS = 1024;

__global__ __launch_bounds__(ORDER_THREADS) void k_order_blocks(const int* __restrict__ cost, int nb,
                                                                int* __restrict__ perm) {
  __shared__ int hist[33];
  __shared__ int off[33];
  const int t = threadIdx.x;
  if (t < 33) hist[t] = 0;
  __syncthreads();
  for (int b = t; b < nb; b += ORDER_THREADS) {
    const unsigned c = (unsigned)max(cost[b], 0);
    atomicAdd(&hist[c ? 32 - __clz(c) : 0], 1);
  }
  __syncthreads();
  if (t == 0) {   // heaviest bucket first
    int run = 0;
    for (int k = 32; k >= 0; --k) { off[k] = run; run += hist[k]; }
  }
  __syncthreads();
  for (int b = t; b < nb; b += ORDER_THREADS) {
    const unsigned c = (unsigned)max(cost[b], 0);
    perm[atomicAdd(&off[c ? 32 - __clz(c) : 0], 1)] = b;
  }
}

// Pass B held to 64 VGPRs, 8 waves per SIMD (68 -> 64, 5 VGPRs spilled outside the point loop):
// 1365 -> 1345 us at C2. Pass A the same way ran 566 -> 616 us, so it keeps its 70 (7 waves).
#ifdef APN_KNN_B_W7   // A/B: pass B at the compiler's 68 VGPRs
#define APN_KNN_PASS_B_ATTR
#else
#define APN_KNN_PASS_B_ATTR __attribute__((amdgpu_waves_per_eu(PTS > 4 ? 4 : 8, 8)))
#endif
// Wave priority of the scanning passes (A/B builds; 0 = the default). With frames in flight the
// passes share SIMDs with the neighbour MLP of other frames, whose waves hold priority 1 through
// their MFMA streams (apn_mlp_h4.hip APN_H4_PRIO); a kNN wave issues rarely, on its dependent
// loads' return. Priority 2 / 3 measured equal (round 6, C2, 4 frames in flight, same box:
// 4.978 / 4.958 and 5.017 / 4.943 vs 4.957 / 4.976 ms per frame): off.
#ifndef APN_KNN_PRIO
#define APN_KNN_PRIO 0
#endif
#ifndef APN_KNN_A_PTS
#define APN_KNN_A_PTS 4
#endif
// points per step of pass A's fine-grid r/4 scan: 0 = scan_ball_flat2_l (2 points), 2 / 4 = the
// fine grid seen as an isotropic AGrid through scan_ball_aniso_l<PTS>
constexpr int kAPts = APN_KNN_A_PTS;
__device__ __forceinline__ AGrid agrid_of(const GridParams& g) {
  AGrid a;
  a.ox = g.ox; a.oy = g.oy; a.oz = g.oz;
  a.hx = a.hy = a.hz = g.h;
  a.ihx = a.ihy = a.ihz = g.inv_h;
  a.r = g.r; a.r2 = g.r2; a.np = g.np;
  a.dx = g.dx; a.dy = g.dy; a.dz = g.dz; a.nf = g.nf;
  return a;
}
#ifdef APN_KNN_NO_ASORT   // A/B: pass A lanes in candidate order
constexpr bool kSortA = false;
#else
constexpr bool kSortA = true;
#endif
// Pass A of mode 8: reject on u1 < 8; the r/4 ball (flat scan) only where u4 >= 8; the rest go to
// the hard list tagged with their first useful level (r/2 if u2 >= 8, else r).
template <bool ANISO>
__global__ __launch_bounds__(KNN_THREADS) void k_knn_pass_a8(
    const float4* __restrict__ q_pos, const int* __restrict__ cand, const int* __restrict__ n_cand_dev,
    const GridParams* __restrict__ gp, const int* __restrict__ cell_start, const float4* __restrict__ sorted,
    const int* __restrict__ ccell, const int* __restrict__ u1, const int* __restrict__ u2,
    const int* __restrict__ u4, int* __restrict__ flag, int* __restrict__ t_nbr, int* __restrict__ hard,
    int* __restrict__ n_hard, int* __restrict__ hard_r, int* __restrict__ n_hard_r, const AGrid* __restrict__ agp,
    const int* __restrict__ cell_start2, const float4* __restrict__ sorted2, const int* __restrict__ perm) {
  if (APN_KNN_PRIO) __builtin_amdgcn_s_setprio(APN_KNN_PRIO);
  const int nc = *n_cand_dev;
  const int base = (perm ? perm[blockIdx.x] : (int)blockIdx.x) * KNN_THREADS;
  int c = base + threadIdx.x;
  const GridParams g = *gp;
  if (kSortA) {
    // rank the workgroup's candidates by their scan cost (0 for the ones rejected or passed on without
    // a search, u4 for an r/4 ball) so the scanning lanes share waves (see kSortB)
    if (base >= nc) return;   // workgroup-uniform
    __shared__ unsigned skey[KNN_THREADS];
    const int tid = threadIdx.x;
    unsigned w = 0;
    if (c < nc) {
      const int cell = ccell[c];
      const int a1 = u1[cell];
      if (a1 >= KNN_K) {
        const bool coarse = g.h > 0.25f * g.r;
        const int a4 = coarse ? a1 : u4[cell];
        w = a4 >= KNN_K ? (unsigned)a4 : 0u;
      }
    }
    skey[tid] = ((0xffffffu - min(w, 0xffffffu)) << 8) | (unsigned)tid;
    __syncthreads();
#pragma unroll
    for (int k = 2; k <= KNN_THREADS; k <<= 1) {
#pragma unroll
      for (int j = k >> 1; j > 0; j >>= 1) {
        const int p = tid ^ j;
        if (p > tid) {
          const unsigned a = skey[tid], b = skey[p];
          if ((a > b) == ((tid & k) == 0)) { skey[tid] = b; skey[p] = a; }
        }
        __syncthreads();
      }
    }
    c = base + (int)(skey[tid] & (KNN_THREADS - 1));
  }
  bool push = false;
  int tag = 0;
  if (c < nc) {
    bool surv = false;
    const int cell = ccell[c];
    if (u1[cell] >= KNN_K) {
      const bool coarse = g.h > 0.25f * g.r;
      if (coarse || u4[cell] >= KNN_K) {
        const float4 q = q_pos[cand[c]];
        KnnList lst;
        lst.init();
        const float R2 = coarse ? g.r2 : 0.0625f * g.r2;
        if (ANISO) scan_ball_aniso_l<KNN_K, false, 2, !kFirstScanNoDup>(*agp, cell_start2, sorted2, q.x, q.y, q.z, R2, lst);
        else if constexpr (kAPts > 0)
          scan_ball_aniso_l<KNN_K, false, kAPts, !kFirstScanNoDup>(agrid_of(g), cell_start, sorted, q.x, q.y, q.z, R2, lst);
        else scan_ball_flat2_l<KNN_K, false, 1, !kFirstScanNoDup>(g, cell_start, sorted, q.x, q.y, q.z, R2, lst);
        if (R2 == g.r2 || lst.worst() < R2 * (1.f - 2e-4f)) {
          surv = lst.worst() <= g.r2;
          if (surv) {
            int4* nb = (int4*)(t_nbr + (int64_t)c * KNN_K);
            nb[0] = make_int4(lst.index(0), lst.index(1), lst.index(2), lst.index(3));
            nb[1] = make_int4(lst.index(4), lst.index(5), lst.index(6), lst.index(7));
          }
        } else {
          push = true;
        }
      } else {
        push = true;
      }
      tag = u2[cell] >= KNN_K ? 0 : 1;
    }
    if (!push) flag[c] = surv;
  }
  // two hard lists by first level, so the waves of pass B run queries of similar depth
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int lst = 0; lst < 2; ++lst) {
    const bool mine = push && tag == lst;
    const unsigned long long bal = __ballot(mine);
    if (bal) {
      int base = 0;
      if (lane == 0) base = atomicAdd(lst ? n_hard_r : n_hard, __popcll(bal));
      base = __shfl(base, 0, 64);
      if (mine) (lst ? hard_r : hard)[base + __popcll(bal & ((1ull << lane) - 1ull))] = 2 * c + tag;
    }
  }
}

#ifdef APN_DEBUG_BUILD   // earlier search strategy: debug build only (cross-checks, A/B tools)
// Pass B of mode 8: flat ball scans from the tagged first level (r/2 or r).
template <bool STATS>
__global__ __launch_bounds__(KNN_THREADS) void k_knn_pass_b8(
    const float4* __restrict__ q_pos, const int* __restrict__ cand, const int* __restrict__ hard,
    const int* __restrict__ n_hard, const GridParams* __restrict__ gp, const int* __restrict__ cell_start,
    const float4* __restrict__ sorted, int* __restrict__ flag, int* __restrict__ t_nbr) {
  const int i = blockIdx.x * KNN_THREADS + threadIdx.x;
  if (i >= *n_hard) return;
  unsigned c2[2] = {0, 0}, cr[2] = {0, 0};
  const GridParams g = *gp;
  const int hc = hard[i];
  const int c = hc >> 1;
  const float4 q = q_pos[cand[c]];
  float bd[KNN_K];
  int bi[KNN_K];
#pragma unroll
  for (int k = 0; k < KNN_K; ++k) { bd[k] = INFINITY; bi[k] = 0x7fffffff; }
  bool done = false;
  if ((hc & 1) == 0) {
    scan_ball_flat2<KNN_K, STATS>(g, cell_start, sorted, q.x, q.y, q.z, 0.25f * g.r2, bd, bi, c2);
    done = bd[KNN_K - 1] < 0.25f * g.r2 * (1.f - 2e-4f);
  }
  if (!done) scan_ball_flat2<KNN_K, STATS>(g, cell_start, sorted, q.x, q.y, q.z, g.r2, bd, bi, cr);
  const bool surv = bd[KNN_K - 1] <= g.r2;
  if (STATS) {   // per list: queries, done at r/2, survivors, r/2 row/pt iterations, r row/pt iterations,
                 // rejected after the full r scan and their iterations
    unsigned long long* st = g_knn_stats + 10 * (hc & 1);
    atomicAdd(&st[0], 1ull);
    if (done) atomicAdd(&st[1], 1ull);
    if (surv) atomicAdd(&st[2], 1ull);
    atomicAdd(&st[3], (unsigned long long)c2[0]);
    atomicAdd(&st[4], (unsigned long long)c2[1]);
    atomicAdd(&st[5], (unsigned long long)cr[0]);
    atomicAdd(&st[6], (unsigned long long)cr[1]);
    if (!done && !surv) { atomicAdd(&st[7], 1ull); atomicAdd(&st[8], (unsigned long long)(cr[0] + cr[1])); }
  }
  flag[c] = surv;
  if (surv) {
    int4* nb = (int4*)(t_nbr + (int64_t)c * KNN_K);
    nb[0] = make_int4(bi[0], bi[1], bi[2], bi[3]);
    nb[1] = make_int4(bi[4], bi[5], bi[6], bi[7]);
  }
}
#endif  // APN_DEBUG_BUILD

// top-K lists of the S lanes of a query group merged in every lane (snapshot, then unique
// inserts in a fixed lane order): all lanes end with the same sorted list
template <int S>
__device__ __forceinline__ void group_merge(float (&bd)[KNN_K], int (&bi)[KNN_K]) {
  float sd[KNN_K];
  int si[KNN_K];
#pragma unroll
  for (int k = 0; k < KNN_K; ++k) { sd[k] = bd[k]; si[k] = bi[k]; }
  const int lane = threadIdx.x & 63, base = lane & ~(S - 1), me = lane & (S - 1);
#pragma unroll
  for (int o = 1; o < S; ++o) {
    const int src = base | ((me + o) & (S - 1));
#pragma unroll
    for (int k = 0; k < KNN_K; ++k) {
      const float d = __shfl(sd[k], src, 64);
      const int id = __shfl(si[k], src, 64);
      knn_insert_unique<KNN_K>(d, id, bd, bi);
    }
  }
}

// Pass B with S lanes per hard query (few hard queries, e.g. the 8192-ray training batches,
// leave most CUs idle with one lane each): each lane scans its share of the ball's rows, the
// lists are merged after each ball, lane 0 writes. Same survivors and neighbours as k_knn_pass_b8.
template <int S>
__global__ __launch_bounds__(KNN_THREADS) void k_knn_pass_b8s(
    const float4* __restrict__ q_pos, const int* __restrict__ cand, const int* __restrict__ hard,
    const int* __restrict__ n_hard, const GridParams* __restrict__ gp, const int* __restrict__ cell_start,
    const float4* __restrict__ sorted, int* __restrict__ flag, int* __restrict__ t_nbr) {
  const int t = blockIdx.x * KNN_THREADS + threadIdx.x;
  const int i = t / S, slice = t & (S - 1);
  if (i >= *n_hard) return;   // uniform over the S lanes of a group
  const GridParams g = *gp;
  const int hc = hard[i];
  const int c = hc >> 1;
  const float4 q = q_pos[cand[c]];
  float bd[KNN_K];
  int bi[KNN_K];
#pragma unroll
  for (int k = 0; k < KNN_K; ++k) { bd[k] = INFINITY; bi[k] = 0x7fffffff; }
  bool done = false;
  if ((hc & 1) == 0) {
    scan_ball_flat2<KNN_K, false, S>(g, cell_start, sorted, q.x, q.y, q.z, 0.25f * g.r2, bd, bi, nullptr, slice);
    group_merge<S>(bd, bi);
    done = bd[KNN_K - 1] < 0.25f * g.r2 * (1.f - 2e-4f);
  }
  if (!done) {
    scan_ball_flat2<KNN_K, false, S>(g, cell_start, sorted, q.x, q.y, q.z, g.r2, bd, bi, nullptr, slice);
    group_merge<S>(bd, bi);
  }
  if (slice != 0) return;
  const bool surv = bd[KNN_K - 1] <= g.r2;
  flag[c] = surv;
  if (surv) {
    int4* nb = (int4*)(t_nbr + (int64_t)c * KNN_K);
    nb[0] = make_int4(bi[0], bi[1], bi[2], bi[3]);
    nb[1] = make_int4(bi[4], bi[5], bi[6], bi[7]);
  }
}

#ifdef APN_DEBUG_BUILD   // earlier search strategy: debug build only (cross-checks, A/B tools)
// Pass A of mode 6: candidates whose cell bound is < 8 are rejected; the rest run the r/4 ball
// and, unless it already holds the 8 nearest, go to the hard list (pass B).
__global__ __launch_bounds__(KNN_THREADS) void k_knn_pass_a6(
    const float4* __restrict__ q_pos, const int* __restrict__ cand, const int* __restrict__ n_cand_dev,
    const GridParams* __restrict__ gp, const int* __restrict__ cell_start, const float4* __restrict__ sorted,
    const int* __restrict__ ccell, const int* __restrict__ ubound, int* __restrict__ flag, int* __restrict__ t_nbr,
    int* __restrict__ hard, int* __restrict__ n_hard) {
  const int nc = *n_cand_dev;
  const int c = blockIdx.x * KNN_THREADS + threadIdx.x;
  const GridParams g = *gp;
  bool push = false;
  if (c < nc) {
    bool surv = false;
    if (ubound[ccell[c]] >= KNN_K) {
      const float4 q = q_pos[cand[c]];
      float bd[KNN_K];
      int bi[KNN_K];
#pragma unroll
      for (int k = 0; k < KNN_K; ++k) { bd[k] = INFINITY; bi[k] = 0x7fffffff; }
      const float R2 = g.h > 0.25f * g.r ? g.r2 : 0.0625f * g.r2;
      scan_ball_nf<KNN_K>(g, cell_start, sorted, q.x, q.y, q.z, R2, bd, bi);
      if (R2 == g.r2 || bd[KNN_K - 1] < R2 * (1.f - 2e-4f)) {
        surv = bd[KNN_K - 1] <= g.r2;
        if (surv) {
          int4* nb = (int4*)(t_nbr + (int64_t)c * KNN_K);
          nb[0] = make_int4(bi[0], bi[1], bi[2], bi[3]);
          nb[1] = make_int4(bi[4], bi[5], bi[6], bi[7]);
        }
      } else {
        push = true;
      }
    }
    if (!push) flag[c] = surv;
  }
  const int lane = threadIdx.x & 63;
  const unsigned long long bal = __ballot(push);
  if (bal) {
    int base = 0;
    if (lane == 0) base = atomicAdd(n_hard, __popcll(bal));
    base = __shfl(base, 0, 64);
    if (push) hard[base + __popcll(bal & ((1ull << lane) - 1ull))] = c;
  }
}

// Pass B with the flat ball scan (mode 7).
__global__ __launch_bounds__(KNN_THREADS) void k_knn_pass_b_flat(
    const float4* __restrict__ q_pos, const int* __restrict__ cand, const int* __restrict__ hard,
    const int* __restrict__ n_hard, const GridParams* __restrict__ gp, const int* __restrict__ cell_start,
    const float4* __restrict__ sorted, int* __restrict__ flag, int* __restrict__ t_nbr) {
  const int i = blockIdx.x * KNN_THREADS + threadIdx.x;
  if (i >= *n_hard) return;
  const GridParams g = *gp;
  const int c = hard[i];
  const float4 q = q_pos[cand[c]];
  float bd[KNN_K];
  int bi[KNN_K];
#pragma unroll
  for (int k = 0; k < KNN_K; ++k) { bd[k] = INFINITY; bi[k] = 0x7fffffff; }
  scan_ball_flat<KNN_K>(g, cell_start, sorted, q.x, q.y, q.z, 0.25f * g.r2, bd, bi);
  if (!(bd[KNN_K - 1] < 0.25f * g.r2 * (1.f - 2e-4f)))
    scan_ball_flat<KNN_K>(g, cell_start, sorted, q.x, q.y, q.z, g.r2, bd, bi);
  const bool surv = bd[KNN_K - 1] <= g.r2;
  flag[c] = surv;
  if (surv) {
    int4* nb = (int4*)(t_nbr + (int64_t)c * KNN_K);
    nb[0] = make_int4(bi[0], bi[1], bi[2], bi[3]);
    nb[1] = make_int4(bi[4], bi[5], bi[6], bi[7]);
  }
}
#endif  // APN_DEBUG_BUILD

// Survivor counts per block of candidate slots (for the order-preserving compaction).
__global__ __launch_bounds__(KNN_THREADS) void k_knn_flag_count(const int* __restrict__ flag,
                                                                const int* __restrict__ n_cand_dev,
                                                                int* __restrict__ blk_cnt) {
  __shared__ int wave_cnt[KNN_THREADS / 64];
  const int c = blockIdx.x * KNN_THREADS + threadIdx.x;
  const bool f = c < *n_cand_dev && flag[c];
  const unsigned long long bal = __ballot(f);
  if ((threadIdx.x & 63) == 0) wave_cnt[threadIdx.x >> 6] = __popcll(bal);
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int w = 0; w < KNN_THREADS / 64; ++w) t += wave_cnt[w];
    blk_cnt[blockIdx.x] = t;
  }
}

__global__ __launch_bounds__(KNN_THREADS) void k_knn_flag_compact(
    const float4* __restrict__ q_pos, const int* __restrict__ q_ray, const int* __restrict__ cand,
    const int* __restrict__ n_cand_dev, const int* __restrict__ flag, const int* __restrict__ t_nbr,
    const int* __restrict__ blk_off, float4* __restrict__ s_pos, int* __restrict__ s_ray, int* __restrict__ s_nbr,
    int nb, int* __restrict__ n_surv) {
  __shared__ int wave_cnt[KNN_THREADS / 64];
  const int c = blockIdx.x * KNN_THREADS + threadIdx.x;
  if (c == 0) *n_surv = blk_off[nb];   // the survivor count (the scan's total), no copy launch
  const bool f = c < *n_cand_dev && flag[c];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const unsigned long long bal = __ballot(f);
  if (lane == 0) wave_cnt[wid] = __popcll(bal);
  __syncthreads();
  int base = blk_off[blockIdx.x];
  for (int w = 0; w < wid; ++w) base += wave_cnt[w];
  if (!f) return;
  const int dst = base + __popcll(bal & ((1ull << lane) - 1ull));
  const int qi = cand[c];
  s_pos[dst] = q_pos[qi];
  s_ray[dst] = q_ray[qi];
  const int4* a = (const int4*)(t_nbr + (int64_t)c * KNN_K);
  int4* b = (int4*)(s_nbr + (int64_t)dst * KNN_K);
  b[0] = a[0];
  b[1] = a[1];
}

#ifdef APN_DEBUG_BUILD   // earlier search strategy: debug build only (cross-checks, A/B tools)
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
#endif  // APN_DEBUG_BUILD

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

// Unbounded K nearest neighbours of arbitrary queries in a point set (the pykeops
// `D_ij.argKmin(dim=1, K)` of temporalpoints.py:104-111, 737-748): cubes of Chebyshev radius
// 1, 2, 4, ... fine cells around the query's (clamped) cell; after cube k every point closer than
// k*h has been seen (also for a query outside the grid), so the search stops once the K-th best
// is closer than k*h. Queries still open after 64 rings fall back to a scan of every point.
// Ties by point index; distances (dx^2 + dy^2) + dz^2 as the reference's recomputation.
template <int K>
__global__ void k_knn_points(const float* __restrict__ q, int64_t M, const GridParams* __restrict__ gp,
                             const int* __restrict__ cell_start, const float4* __restrict__ sorted,
                             const float* __restrict__ pts, int64_t N, int k_out, int64_t* __restrict__ idx_out,
                             float* __restrict__ d2_out) {
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  const GridParams g = *gp;
  const float qx = q[3 * m], qy = q[3 * m + 1], qz = q[3 * m + 2];
  const int fx = cell_coord(qx, g.ox, g.inv_h, g.dx), fy = cell_coord(qy, g.oy, g.inv_h, g.dy);
  const int fz = cell_coord(qz, g.oz, g.inv_h, g.dz);
  float bd[K];
  int bi[K];
  const int dmax = max(g.dx, max(g.dy, g.dz));
  bool done = false;
  for (int k = 1; k <= 64; k *= 2) {
#pragma unroll
    for (int j = 0; j < K; ++j) { bd[j] = INFINITY; bi[j] = 0x7fffffff; }
    scan_cube<K, false>(g, cell_start, sorted, fx, fy, fz, k, qx, qy, qz, INFINITY, -1, bd, bi);
    const float gk = (float)k * g.h * (1.f - 1e-4f);
    if (bd[K - 1] < gk * gk || k >= dmax) { done = true; break; }   // k >= dmax: the cube is the grid
  }
  if (!done) {
#pragma unroll
    for (int j = 0; j < K; ++j) { bd[j] = INFINITY; bi[j] = 0x7fffffff; }
    for (int64_t n = 0; n < N; ++n) {
      const float dx = qx - pts[3 * n], dy = qy - pts[3 * n + 1], dz = qz - pts[3 * n + 2];
      const float d = (dx * dx + dy * dy) + dz * dz;
      knn_insert<K>(d, (int)n, bd, bi);
    }
  }
  for (int j = 0; j < k_out; ++j) {
    idx_out[m * k_out + j] = bi[j];
    d2_out[m * k_out + j] = bd[j];
  }
}

// Pass B of mode 9: k_knn_pass_b8 with the r/2 and r balls on the anisotropic grid. One launch
// over both hard lists (first list first: the host passes the heavier r list there, so the
// longest waves start first and the two lists share one tail); hard2 == nullptr: one list.
#ifdef APN_KNN_NO_BSORT   // A/B: pass B lanes in list order
constexpr bool kSortB = false;
#else
constexpr bool kSortB = true;
#endif
// kSortB: a workgroup's queries are ranked by their cost estimate (k_block_cost's: u1, plus u2 for the
// r/2 list) with a bitonic sort in LDS before the scans, so each wave holds queries of similar cost
// and fewer lanes idle while the wave's longest scan runs (the lanes still cover the same 256
// consecutive list entries: the workgroup's spatial locality is kept).
template <bool STATS, int PTS>
__global__ __launch_bounds__(KNN_THREADS) APN_KNN_PASS_B_ATTR void k_knn_pass_b9(
    const float4* __restrict__ q_pos, const int* __restrict__ cand, const int* __restrict__ hard,
    const int* __restrict__ n_hard, const int* __restrict__ hard2, const int* __restrict__ n_hard2,
    const AGrid* __restrict__ agp, const int* __restrict__ cell_start2, const float4* __restrict__ sorted2,
    int* __restrict__ flag, int* __restrict__ t_nbr, const int* __restrict__ perm, const int* __restrict__ ccell,
    const int* __restrict__ u1, const int* __restrict__ u2) {
  if (APN_KNN_PRIO) __builtin_amdgcn_s_setprio(APN_KNN_PRIO);
  const int base = (perm ? perm[blockIdx.x] : (int)blockIdx.x) * KNN_THREADS;
  const int n1 = *n_hard, n2 = hard2 ? *n_hard2 : 0;
  int i = base + threadIdx.x;
  if (kSortB && ccell) {
    if (base >= n1 + n2) return;   // workgroup-uniform
    __shared__ unsigned skey[KNN_THREADS];
    const int tid = threadIdx.x;
    unsigned w = 0;
    if (i < n1 + n2) {
      const int hc = i < n1 ? hard[i] : hard2[i - n1];
      const int cell = ccell[hc >> 1];
      w = (hc & 1) ? (unsigned)u1[cell] : (unsigned)(u2[cell] + u1[cell]);
    }
    // ascending keys = descending cost (heaviest wave first), entries past the list last
    skey[tid] = ((0xffffffu - min(w, 0xffffffu)) << 8) | (unsigned)tid;
    __syncthreads();
#pragma unroll
    for (int k = 2; k <= KNN_THREADS; k <<= 1) {
#pragma unroll
      for (int j = k >> 1; j > 0; j >>= 1) {
        const int p = tid ^ j;
        if (p > tid) {
          const unsigned a = skey[tid], b = skey[p];
          if ((a > b) == ((tid & k) == 0)) { skey[tid] = b; skey[p] = a; }
        }
        __syncthreads();
      }
    }
    i = base + (int)(skey[tid] & (KNN_THREADS - 1));
  }
  if (i >= n1 + n2) return;
  const AGrid g = *agp;
  unsigned c2[2] = {0, 0}, cr[2] = {0, 0};
  const int hc = i < n1 ? hard[i] : hard2[i - n1];
  const int c = hc >> 1;
  const float4 q = q_pos[cand[c]];
  KnnList lst;
  lst.init();
  bool done = false;
  if constexpr (kFirstScanNoDup) {
    // only the r scan after an r/2 scan revisits points already in the list
    if ((hc & 1) == 0) {
      scan_ball_aniso_l<KNN_K, STATS, PTS, false>(g, cell_start2, sorted2, q.x, q.y, q.z, 0.25f * g.r2, lst, c2);
      done = lst.worst() < 0.25f * g.r2 * (1.f - 2e-4f);
      if (!done) scan_ball_aniso_l<KNN_K, STATS, PTS, true>(g, cell_start2, sorted2, q.x, q.y, q.z, g.r2, lst, cr);
    } else {
      scan_ball_aniso_l<KNN_K, STATS, PTS, false>(g, cell_start2, sorted2, q.x, q.y, q.z, g.r2, lst, cr);
    }
  } else {
    if ((hc & 1) == 0) {
      scan_ball_aniso_l<KNN_K, STATS, PTS, true>(g, cell_start2, sorted2, q.x, q.y, q.z, 0.25f * g.r2, lst, c2);
      done = lst.worst() < 0.25f * g.r2 * (1.f - 2e-4f);
    }
    if (!done) scan_ball_aniso_l<KNN_K, STATS, PTS, true>(g, cell_start2, sorted2, q.x, q.y, q.z, g.r2, lst, cr);
  }
  const bool surv = lst.worst() <= g.r2;
  if (STATS) {
    unsigned long long* st = g_knn_stats + 10 * (hc & 1);
    atomicAdd(&st[0], 1ull);
    if (done) atomicAdd(&st[1], 1ull);
    if (surv) atomicAdd(&st[2], 1ull);
    atomicAdd(&st[3], (unsigned long long)c2[0]);
    atomicAdd(&st[4], (unsigned long long)c2[1]);
    atomicAdd(&st[5], (unsigned long long)cr[0]);
    atomicAdd(&st[6], (unsigned long long)cr[1]);
    if (!done && !surv) { atomicAdd(&st[7], 1ull); atomicAdd(&st[8], (unsigned long long)(cr[0] + cr[1])); }
  }
  flag[c] = surv;
  if (surv) {
    int4* nb = (int4*)(t_nbr + (int64_t)c * KNN_K);
    nb[0] = make_int4(lst.index(0), lst.index(1), lst.index(2), lst.index(3));
    nb[1] = make_int4(lst.index(4), lst.index(5), lst.index(6), lst.index(7));
  }
}

#ifdef APN_DEBUG_BUILD   // measured and not kept: S lanes per hard query of pass B (APN_KNN_B_LANES)
template <int S, class L>
__device__ __forceinline__ void group_merge_list(L& lst) {
  const L snap = lst;
  const int lane = threadIdx.x & 63, base = lane & ~(S - 1), me = lane & (S - 1);
#pragma unroll
  for (int o = 1; o < S; ++o) {
    const int src = base | ((me + o) & (S - 1));
#pragma unroll
    for (int k = 0; k < KNN_K; ++k) {
      const float d = __shfl(snap.dist(k), src, 64);
      const int id = __shfl(snap.index(k), src, 64);
      lst.template insert<true>(d, id);
    }
  }
}

// k_knn_pass_b9 with S lanes per hard query: each lane walks its share of every slab's rows
// (scan_ball_aniso_l's slices), the lists are merged after each ball (pruning with the lane-local
// K-th best is exact), lane 0 writes. Workgroup b covers part b % S of list block perm[b / S].
template <int S, int PTS>
__global__ __launch_bounds__(KNN_THREADS) void k_knn_pass_b9s(
    const float4* __restrict__ q_pos, const int* __restrict__ cand, const int* __restrict__ hard,
    const int* __restrict__ n_hard, const int* __restrict__ hard2, const int* __restrict__ n_hard2,
    const AGrid* __restrict__ agp, const int* __restrict__ cell_start2, const float4* __restrict__ sorted2,
    int* __restrict__ flag, int* __restrict__ t_nbr, const int* __restrict__ perm, const int* __restrict__ ccell,
    const int* __restrict__ u1, const int* __restrict__ u2) {
  constexpr int NQ = KNN_THREADS / S;
  const int blk = blockIdx.x / S, part = blockIdx.x % S;
  const int base = (perm ? perm[blk] : blk) * KNN_THREADS + part * NQ;
  const int n1 = *n_hard, n2 = hard2 ? *n_hard2 : 0;
  if (base >= n1 + n2) return;
  const int tid = threadIdx.x, grp = tid / S, slice = tid & (S - 1);
  int i = base + grp;
  if (kSortB && ccell) {
    __shared__ unsigned skey[NQ];
    if (tid < NQ) {
      unsigned w = 0;
      const int e = base + tid;
      if (e < n1 + n2) {
        const int hc = e < n1 ? hard[e] : hard2[e - n1];
        const int cell = ccell[hc >> 1];
        w = (hc & 1) ? (unsigned)u1[cell] : (unsigned)(u2[cell] + u1[cell]);
      }
      skey[tid] = ((0xffffffu - min(w, 0xffffffu)) << 8) | (unsigned)tid;
    }
    __syncthreads();
#pragma unroll
    for (int k = 2; k <= NQ; k <<= 1) {
#pragma unroll
      for (int j = k >> 1; j > 0; j >>= 1) {
        const int p = tid ^ j;
        if (tid < NQ && p > tid) {
          const unsigned a = skey[tid], b = skey[p];
          if ((a > b) == ((tid & k) == 0)) { skey[tid] = b; skey[p] = a; }
        }
        __syncthreads();
      }
    }
    i = base + (int)(skey[grp] & 0xffu);
  }
  if (i >= n1 + n2) return;
  const AGrid g = *agp;
  const int hc = i < n1 ? hard[i] : hard2[i - n1];
  const int c = hc >> 1;
  const float4 q = q_pos[cand[c]];
  KnnList lst;
  lst.init();
  bool first = true;
  if ((hc & 1) == 0) {
    scan_ball_aniso_l<KNN_K, false, PTS, !kFirstScanNoDup, KnnList, S>(g, cell_start2, sorted2, q.x, q.y, q.z,
                                                                     0.25f * g.r2, lst, nullptr, slice);
    group_merge_list<S>(lst);
    first = false;
  }
  if (first || !(lst.worst() < 0.25f * g.r2 * (1.f - 2e-4f))) {
    if (first)
      scan_ball_aniso_l<KNN_K, false, PTS, !kFirstScanNoDup, KnnList, S>(g, cell_start2, sorted2, q.x, q.y, q.z,
                                                                       g.r2, lst, nullptr, slice);
    else
      scan_ball_aniso_l<KNN_K, false, PTS, true, KnnList, S>(g, cell_start2, sorted2, q.x, q.y, q.z, g.r2, lst,
                                                            nullptr, slice);
    group_merge_list<S>(lst);
  }
  if (slice != 0) return;
  const bool surv = lst.worst() <= g.r2;
  flag[c] = surv;
  if (surv) {
    int4* nb = (int4*)(t_nbr + (int64_t)c * KNN_K);
    nb[0] = make_int4(lst.index(0), lst.index(1), lst.index(2), lst.index(3));
    nb[1] = make_int4(lst.index(4), lst.index(5), lst.index(6), lst.index(7));
  }
}
#endif  // APN_DEBUG_BUILD

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

static size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

// Search strategy. The shipped library runs mode 9 only (fine grid pass A, anisotropic second
// grid pass B; the 8-lane pass B for small launches). The debug build (libapn_hip_debug.so,
// -DAPN_DEBUG_BUILD; include/apn_hip_debug.h) keeps the earlier exact strategies 0-8 behind
// apn_set_knn_mode / APN_KNN_MODE, for the bit-identity cross-checks and the A/B tools.
#ifdef APN_DEBUG_BUILD
static int& knn_mode() {
  static int m = [] {
    const char* e = apn_env("APN_KNN_MODE");
    return e ? atoi(e) : 9;
  }();
  return m;
}

extern "C" int apn_set_knn_mode(int32_t mode) {
  const int prev = knn_mode();
  if (mode >= 0 && mode <= 9) knn_mode() = mode;
  return prev;
}

// Profiling aid (synchronous): copies and resets the kNN counters (20 uint64, see g_knn_stats):
// mode 3 query classes, or the mode-8 pass-B counters when APN_KNN_STATS is set.
extern "C" int apn_debug_knn_stats(uint64_t* out20) {
  if (!out20) return APN_ERR_ARG;
  APN_HIP_TRY(hipDeviceSynchronize());
  APN_HIP_TRY(hipMemcpyFromSymbol(out20, HIP_SYMBOL(g_knn_stats), sizeof(uint64_t) * 20));
  static const unsigned long long zero[20] = {};
  APN_HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_knn_stats), zero, sizeof(zero)));
  return APN_OK;
}
static const bool kKnnStats = apn_env("APN_KNN_STATS") != nullptr;   // profiling aid: apn_debug_knn_stats
#else
static constexpr int knn_mode() { return 9; }
static constexpr bool kKnnStats = false;
#endif

// Grid workspace (bytes, each region 256-B aligned):
//   GridParams | counts[cap] | cell_start[cap+1] | cursor[cap] | pcell[N] | ccount[cap] | scan ws |
//   tile_cnt[cap] | tile_start[cap+1] | tile_cursor[cap] | tile_list[cap] | n_tile_list[1]
// (tiles of KT^3 cells never outnumber cells, so cap bounds the tile arrays).
//   | AGrid | counts2[cap] | cursor2[cap] | cell_start2[cap+1] | pcell2[N] | sorted2[N] float4
// (the anisotropic second grid of kNN mode 9; its cells never outnumber the fine ones).
extern "C" size_t apn_grid_workspace_bytes(int64_t n_points, int32_t cell_cap) {
  return al256(sizeof(GridParams)) + al256((size_t)cell_cap * 4) + al256((size_t)(cell_cap + 1) * 4) +
         al256((size_t)cell_cap * 4) + al256((size_t)n_points * 4) + al256((size_t)cell_cap * 4) +
         al256(scan_workspace_bytes(cell_cap)) + al256((size_t)cell_cap * 4) * 3 +
         al256((size_t)(cell_cap + 1) * 4) + al256(4) + al256(sizeof(AGrid)) + al256((size_t)cell_cap * 4) * 2 +
         al256((size_t)(cell_cap + 1) * 4) + al256((size_t)n_points * 4) + al256((size_t)n_points * 16) +
         al256((size_t)cell_cap * 4);
}

struct GridWs {
  GridParams* gp; int* counts; int* cell_start; int* cursor; int* pcell; int* ccount; void* scan;
  int* tile_cnt; int* tile_start; int* tile_cursor; int* tile_list; int* n_tile_list;
  AGrid* ag; int* counts2; int* cursor2; int* cell_start2; int* pcell2; float4* sorted2; int* csum27;
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
  w.scan = p; p += al256(scan_workspace_bytes(cap));
  w.tile_cnt = (int*)p; p += al256((size_t)cap * 4);
  w.tile_start = (int*)p; p += al256((size_t)(cap + 1) * 4);
  w.tile_cursor = (int*)p; p += al256((size_t)cap * 4);
  w.tile_list = (int*)p; p += al256((size_t)cap * 4);
  w.n_tile_list = (int*)p; p += al256(4);
  w.ag = (AGrid*)p; p += al256(sizeof(AGrid));
  w.counts2 = (int*)p; p += al256((size_t)cap * 4);
  w.cursor2 = (int*)p; p += al256((size_t)cap * 4);
  w.cell_start2 = (int*)p; p += al256((size_t)(cap + 1) * 4);
  w.pcell2 = (int*)p; p += al256((size_t)N * 4);
  w.sorted2 = (float4*)p; p += al256((size_t)N * 16);
  w.csum27 = (int*)p;
  return w;
}

extern "C" int apn_grid_build(const float* xyz, int64_t n_points, const int32_t* bbox_ord, float query_radius,
                              int32_t cell_cap, float* sorted_pts4, void* workspace, void* stream) {
  if (n_points <= 0 || cell_cap <= 0 || !xyz || !bbox_ord || !sorted_pts4 || !workspace) return APN_ERR_ARG;
  if (n_points > KNN_MAX_POINTS) return APN_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  GridWs w = grid_ws(workspace, n_points, cell_cap);
  APN_TRY(fill4_i32(w.counts, cell_cap, w.cursor, cell_cap, nullptr, 0, nullptr, 0, s));
  static const int subdiv = [] {
    const char* e = apn_env("APN_KNN_SUBDIV");
    return e ? atoi(e) : KNN_SUBDIV;
  }();
  hipLaunchKernelGGL(k_grid_params, dim3(1), dim3(64), 0, s, bbox_ord, query_radius, cell_cap, subdiv,
                     (int)n_points, w.gp);
  hipLaunchKernelGGL(k_grid_count, dim3(ceil_div(n_points, 256)), dim3(256), 0, s, xyz, n_points, w.gp, w.counts,
                     w.ccount, w.pcell);
  int st = scan_exclusive_i32(w.counts, w.cell_start, cell_cap, w.scan, s);
  if (st) return st;
  // coarse cells never outnumber fine cells (cap)
  const int cgrid = (int)std::min<int64_t>(ceil_div(cell_cap, 256), 128);   // grid-stride over the coarse cells
  hipLaunchKernelGGL(k_coarse_counts, dim3(1024), dim3(256), 0, s, w.gp, w.cell_start, w.ccount);
  hipLaunchKernelGGL(k_coarse_sum27, dim3(cgrid), dim3(256), 0, s, w.gp, w.ccount, w.csum27);
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
static int64_t knn_small_max() {
  static const int64_t v = [] {
    const char* e = apn_env("APN_KNN_SMALL_MAX");
    return e ? (int64_t)atoll(e) : KNN_SPLIT_MAX_QUERIES;
  }();
  return v;
}
// small batches (the 8192-ray training steps) take the 8-lane fine-grid pass B; larger launches of
// mode 9 read the anisotropic second grid. Up to 2^18 queries: a ray shard of a full frame (~0.5-1M
// in-bbox samples at C2 over 8 GPUs) ran its kNN 2.3x slower on the 8-lane pass than on mode 9's
// (tools/shard_balance.py); APN_KNN_SMALL_MAX overrides in the debug build.
static bool knn_uses_agrid(int64_t n_queries) {
  return knn_mode() == 9 && !(!kKnnStats && n_queries <= knn_small_max());
}

// The second grid (k_agrid_*): cells of AG_F x AG_F fine cells in y and z, counting-sorted from the
// fine grid's sorted points. Reads only the fine grid (gp, sorted points) and writes only its own
// buffers (counts2, cursor2, cell_start2, pcell2, sorted2, the grid scan scratch).
static int agrid_build(GridWs& g, int64_t n_points, int cell_cap, const float* sorted_pts4, hipStream_t s) {
  static const int f = [] {
    const char* e = apn_env("APN_KNN_ANISO");
    const int v = e ? atoi(e) : 2;
    return (v == 1 || v == 2 || v == 4) ? v : 2;
  }();
  APN_TRY(fill4_i32(g.counts2, cell_cap, g.cursor2, cell_cap, nullptr, 0, nullptr, 0, s));
  hipLaunchKernelGGL(k_agrid_params, dim3(1), dim3(64), 0, s, g.gp, f, (int)n_points, g.ag);
  hipLaunchKernelGGL(k_agrid_count, dim3(ceil_div(n_points, 256)), dim3(256), 0, s, (const float4*)sorted_pts4,
                     n_points, g.gp, f, g.counts2, g.pcell2);
  const int st = scan_exclusive_i32(g.counts2, g.cell_start2, cell_cap, g.scan, s);
  if (st) return st;
  hipLaunchKernelGGL(k_agrid_scatter, dim3(ceil_div(n_points, 256)), dim3(256), 0, s, (const float4*)sorted_pts4,
                     n_points, g.pcell2, g.cell_start2, g.cursor2, g.sorted2);
  return launch_status();
}

static int knn_radius_impl(const float* q_pos4, const int32_t* q_ray, int64_t n_queries,
                           const int32_t* n_queries_dev, const void* grid_workspace, int64_t n_points,
                           int32_t cell_cap, const float* sorted_pts4, float query_radius, float* s_pos4,
                           int32_t* s_ray, int32_t* s_nbr, int32_t* n_survivors_dev, void* workspace,
                           void* agrid_ready, void* stream) {
  (void)query_radius;  // the grid was built for it (GridParams.r2)
  if (n_queries < 0 || !grid_workspace || !workspace) return APN_ERR_ARG;
  if (n_points > KNN_MAX_POINTS) return APN_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (n_queries == 0) {
    APN_TRY(fill_i32(n_survivors_dev, 0, 1, s));
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
                     g.ccount, g.csum27, cand_blk, cblk_cnt);
  int st = scan_exclusive_i32(cblk_cnt, cblk_off, nb, sws, s);
  if (st) return st;
  hipLaunchKernelGGL(k_compact_i32, dim3(nb), dim3(KNN_THREADS), 0, s, cand_blk, cblk_cnt, cblk_off, cand);
  // candidates: count at cblk_off[nb]; launch over the upper bound nb blocks
  if (knn_mode() == 8 || knn_mode() == 9) {
    const bool stats = kKnnStats;
    // small batches (the 8192-ray training steps): 8 lanes per hard query. Up to 2^18 queries:
    // a ray shard of a full frame (~0.5-1M in-bbox samples at C2 over 8 GPUs) ran its kNN 2.3x
    // slower on the 8-lane pass than on mode 9's (tools/shard_balance.py); APN_KNN_SMALL_MAX overrides
    const bool aniso = knn_uses_agrid(n_queries);
    const bool small = !stats && n_queries <= knn_small_max();
    if (aniso && !agrid_ready) {   // the second grid, here on the kNN's stream
      st = agrid_build(g, n_points, cell_cap, sorted_pts4, s);
      if (st) return st;
    }
    int* flag = t_ray;
    int* hard = cand_blk;
    int* n_hard = cblk_cnt + nb + 1;
    int* ccell = (int*)t_pos;
    int* mark = g.cursor;        // free after the grid build
    int* u1 = g.counts;          // free after the grid build
    int* u2 = g.tile_cnt;
    int* u4 = g.tile_cursor;
    int* n_hard_r = cblk_off + nb + 1;    // cblk_off has nb + 2 entries
    APN_TRY(fill4_i32(mark, cell_cap, g.n_tile_list, 1, n_hard, 1, n_hard_r, 1, s));
    hipLaunchKernelGGL(k_mark_cells, dim3(nb), dim3(KNN_THREADS), 0, s, (const float4*)q_pos4, cand, cblk_off + nb,
                       g.gp, ccell, mark);
    hipLaunchKernelGGL(k_tile_list, dim3(ceil_div(cell_cap, LIST_THREADS)), dim3(LIST_THREADS), 0, s, mark, cell_cap,
                       g.tile_list, g.n_tile_list);
    static const int64_t cb16_max = [] {   // query count up to which the cell bounds run 16 lanes per cell
      const char* e = apn_env("APN_CELL_BOUND16_MAX");
      return e ? (int64_t)atoll(e) : (int64_t)3 << 20;
    }();
    if (n_queries <= cb16_max) {
#ifdef APN_DEBUG_BUILD
      static const int cbl = [] {   // A/B: lanes per cell of the short-list cell bounds (16, 32 or 64)
        const char* e = apn_env("APN_CB_LANES");
        const int v = e ? atoi(e) : CB_LANES;
        return (v == 32 || v == 64) ? v : CB_LANES;
      }();
#else
      constexpr int cbl = CB_LANES;
#endif
      auto cb = cbl == 64 ? k_cell_bound3w<64> : (cbl == 32 ? k_cell_bound3w<32> : k_cell_bound3w<CB_LANES>);
      hipLaunchKernelGGL(cb,
                         dim3(std::max<int64_t>(1, std::min<int64_t>(256 * 16, ceil_div(std::min<int64_t>(cell_cap, slots) * cbl, KNN_THREADS)))),
                         dim3(KNN_THREADS), 0, s, g.gp, g.cell_start, g.tile_list, g.n_tile_list, u1, u2, u4);
    }
    else
      hipLaunchKernelGGL(k_cell_bound3, dim3(ceil_div(std::min<int64_t>(cell_cap, slots), KNN_THREADS)),
                         dim3(KNN_THREADS), 0, s, g.gp, g.cell_start, g.tile_list, g.n_tile_list, u1, u2, u4);
    int* hard_r = ccell + slots;          // second quarter of the t_pos region
    static const int64_t lpt_max = [] {   // query count up to which the passes run heavy blocks first
      const char* e = apn_env("APN_KNN_LPT_MAX");   // 8 shards 2.17 -> 2.05 ms, 2 shards (forced) 6.05 -> 5.86
      return e ? (int64_t)atoll(e) : (int64_t)6 << 20;
    }();
    // blk_cnt / blk_off are free until the survivor count below: block costs and the permutation
    int* perm = (aniso && n_queries <= lpt_max && nb <= (1 << 24)) ? blk_off : nullptr;
    if (perm) {
      hipLaunchKernelGGL(k_block_cost<false>, dim3(nb), dim3(KNN_THREADS), 0, s, cblk_off + nb, nullptr, nullptr,
                         nullptr, nullptr, g.gp, ccell, u1, u2, u4, blk_cnt);
      hipLaunchKernelGGL(k_order_blocks, dim3(1), dim3(ORDER_THREADS), 0, s, blk_cnt, nb, perm);
    }
#ifdef APN_DEBUG_BUILD
    static const bool a_aniso = apn_env("APN_KNN_A_ANISO") != nullptr;   // A/B: pass A's r/4 ball on the second grid
    auto pass_a = (aniso && a_aniso) ? k_knn_pass_a8<true> : k_knn_pass_a8<false>;
#else
    auto pass_a = k_knn_pass_a8<false>;
#endif
    if (aniso && agrid_ready) APN_HIP_TRY(hipStreamWaitEvent(s, (hipEvent_t)agrid_ready, 0));   // built on another stream
    hipLaunchKernelGGL(pass_a, dim3(nb), dim3(KNN_THREADS), 0,
                       s, (const float4*)q_pos4, cand, cblk_off + nb, g.gp, g.cell_start, (const float4*)sorted_pts4,
                       ccell, u1, u2, u4, flag, t_nbr, hard, n_hard, hard_r, n_hard_r, g.ag, g.cell_start2, g.sorted2,
                       perm);
    if (small) {
      const dim3 nb4(ceil_div(n_queries * 8, KNN_THREADS));
      hipLaunchKernelGGL(k_knn_pass_b8s<8>, nb4, dim3(KNN_THREADS), 0, s, (const float4*)q_pos4, cand, hard, n_hard,
                         g.gp, g.cell_start, (const float4*)sorted_pts4, flag, t_nbr);
      hipLaunchKernelGGL(k_knn_pass_b8s<8>, nb4, dim3(KNN_THREADS), 0, s, (const float4*)q_pos4, cand, hard_r,
                         n_hard_r, g.gp, g.cell_start, (const float4*)sorted_pts4, flag, t_nbr);
    } else if (aniso) {
#ifdef APN_DEBUG_BUILD
      static const int pts = [] {   // points per step of the scan (A/B: APN_KNN_PTS=2 or 8)
        const char* e = apn_env("APN_KNN_PTS");
        const int v = e ? atoi(e) : 4;
        return (v == 2 || v == 8) ? v : 4;
      }();
      auto pass_b = stats ? (pts == 4 ? k_knn_pass_b9<true, 4> : k_knn_pass_b9<true, 2>)
                          : (pts == 4 ? k_knn_pass_b9<false, 4>
                                      : (pts == 8 ? k_knn_pass_b9<false, 8> : k_knn_pass_b9<false, 2>));
#else
      auto pass_b = k_knn_pass_b9<false, 4>;
#endif
      static const bool split = [] {   // A/B: APN_KNN_B_SPLIT=1 runs the two lists as two launches
        const char* e = apn_env("APN_KNN_B_SPLIT");
        return e && atoi(e) == 1;
      }();
      if (split) {
        hipLaunchKernelGGL(pass_b, dim3(nb), dim3(KNN_THREADS), 0, s, (const float4*)q_pos4, cand, hard, n_hard,
                           nullptr, nullptr, g.ag, g.cell_start2, g.sorted2, flag, t_nbr, nullptr, ccell, u1, u2);
        hipLaunchKernelGGL(pass_b, dim3(nb), dim3(KNN_THREADS), 0, s, (const float4*)q_pos4, cand, hard_r,
                           n_hard_r, nullptr, nullptr, g.ag, g.cell_start2, g.sorted2, flag, t_nbr, nullptr, ccell, u1,
                           u2);
      } else {   // n_hard + n_hard_r <= candidates <= nb * KNN_THREADS
        if (perm) {
          hipLaunchKernelGGL(k_block_cost<true>, dim3(nb), dim3(KNN_THREADS), 0, s, nullptr, hard_r, n_hard_r, hard,
                             n_hard, g.gp, ccell, u1, u2, u4, blk_cnt);
          hipLaunchKernelGGL(k_order_blocks, dim3(1), dim3(ORDER_THREADS), 0, s, blk_cnt, nb, perm);
        }
#ifdef APN_DEBUG_BUILD
        static const int lanes = [] {   // A/B: APN_KNN_B_LANES = 2 or 4 lanes per hard query
          const char* e = apn_env("APN_KNN_B_LANES");
          const int v = e ? atoi(e) : 1;
          return (v == 2 || v == 4) ? v : 1;
        }();
        if (lanes > 1) {
          auto pass_bs = lanes == 2 ? k_knn_pass_b9s<2, 4> : k_knn_pass_b9s<4, 4>;
          hipLaunchKernelGGL(pass_bs, dim3(nb * lanes), dim3(KNN_THREADS), 0, s, (const float4*)q_pos4, cand, hard_r,
                             n_hard_r, hard, n_hard, g.ag, g.cell_start2, g.sorted2, flag, t_nbr, perm, ccell, u1, u2);
        } else
#endif
        hipLaunchKernelGGL(pass_b, dim3(nb), dim3(KNN_THREADS), 0, s, (const float4*)q_pos4, cand, hard_r,
                           n_hard_r, hard, n_hard, g.ag, g.cell_start2, g.sorted2, flag, t_nbr, perm, ccell, u1, u2);
      }
    } else {
#ifdef APN_DEBUG_BUILD
      auto pass_b = stats ? k_knn_pass_b8<true> : k_knn_pass_b8<false>;
      hipLaunchKernelGGL(pass_b, dim3(nb), dim3(KNN_THREADS), 0, s, (const float4*)q_pos4, cand, hard, n_hard,
                         g.gp, g.cell_start, (const float4*)sorted_pts4, flag, t_nbr);
      hipLaunchKernelGGL(pass_b, dim3(nb), dim3(KNN_THREADS), 0, s, (const float4*)q_pos4, cand, hard_r,
                         n_hard_r, g.gp, g.cell_start, (const float4*)sorted_pts4, flag, t_nbr);
#else
      return APN_ERR_ARG;   // unreachable: mode 9 always takes the small or the anisotropic pass B
#endif
    }
    hipLaunchKernelGGL(k_knn_flag_count, dim3(nb), dim3(KNN_THREADS), 0, s, flag, cblk_off + nb, blk_cnt);
    st = scan_exclusive_i32(blk_cnt, blk_off, nb, sws, s);
    if (st) return st;
    hipLaunchKernelGGL(k_knn_flag_compact, dim3(nb), dim3(KNN_THREADS), 0, s, (const float4*)q_pos4, q_ray, cand,
                       cblk_off + nb, flag, t_nbr, blk_off, (float4*)s_pos4, s_ray, s_nbr, nb,
                       n_survivors_dev);
    return launch_status();
  }
#ifndef APN_DEBUG_BUILD
  return APN_ERR_ARG;   // unreachable (mode 9)
#else
  if (knn_mode() == 6 || knn_mode() == 7) {
    int* flag = t_ray;
    int* hard = cand_blk;
    int* n_hard = cblk_cnt + nb + 1;
    int* ccell = (int*)t_pos;
    int* mark = g.cursor;        // free after the grid build
    int* ubound = g.counts;      // free after the grid build
    APN_TRY(fill_i32(mark, 0, cell_cap, s));
    APN_TRY(fill_i32(g.n_tile_list, 0, 1, s));
    APN_TRY(fill_i32(n_hard, 0, 1, s));
    hipLaunchKernelGGL(k_mark_cells, dim3(nb), dim3(KNN_THREADS), 0, s, (const float4*)q_pos4, cand, cblk_off + nb,
                       g.gp, ccell, mark);
    hipLaunchKernelGGL(k_tile_list, dim3(ceil_div(cell_cap, LIST_THREADS)), dim3(LIST_THREADS), 0, s, mark, cell_cap,
                       g.tile_list, g.n_tile_list);
    hipLaunchKernelGGL(k_cell_bound, dim3(ceil_div(std::min<int64_t>(cell_cap, slots), KNN_THREADS)),
                       dim3(KNN_THREADS), 0, s, g.gp, g.cell_start, g.tile_list, g.n_tile_list, ubound);
    hipLaunchKernelGGL(k_knn_pass_a6, dim3(nb), dim3(KNN_THREADS), 0, s, (const float4*)q_pos4, cand, cblk_off + nb,
                       g.gp, g.cell_start, (const float4*)sorted_pts4, ccell, ubound, flag, t_nbr, hard, n_hard);
    if (knn_mode() == 7)
      hipLaunchKernelGGL(k_knn_pass_b_flat, dim3(nb), dim3(KNN_THREADS), 0, s, (const float4*)q_pos4, cand, hard,
                         n_hard, g.gp, g.cell_start, (const float4*)sorted_pts4, flag, t_nbr);
    else
      hipLaunchKernelGGL(k_knn_pass_b, dim3(nb), dim3(KNN_THREADS), 0, s, (const float4*)q_pos4, cand, hard, n_hard,
                         g.gp, g.cell_start, (const float4*)sorted_pts4, flag, t_nbr);
    hipLaunchKernelGGL(k_knn_flag_count, dim3(nb), dim3(KNN_THREADS), 0, s, flag, cblk_off + nb, blk_cnt);
    st = scan_exclusive_i32(blk_cnt, blk_off, nb, sws, s);
    if (st) return st;
    hipLaunchKernelGGL(k_knn_flag_compact, dim3(nb), dim3(KNN_THREADS), 0, s, (const float4*)q_pos4, q_ray, cand,
                       cblk_off + nb, flag, t_nbr, blk_off, (float4*)s_pos4, s_ray, s_nbr, nb,
                       n_survivors_dev);
    return launch_status();
  }
  if (knn_mode() == 5) {
    int* flag = t_ray;
    int* order = cand_blk;
    int* ctile = (int*)t_pos;
    APN_TRY(fill_i32(g.tile_cnt, 0, cell_cap, s));
    APN_TRY(fill_i32(g.tile_cursor, 0, cell_cap, s));
    APN_TRY(fill_i32(g.n_tile_list, 0, 1, s));
    hipLaunchKernelGGL(k_tile_count, dim3(nb), dim3(KNN_THREADS), 0, s, (const float4*)q_pos4, cand, cblk_off + nb,
                       g.gp, ctile, g.tile_cnt);
    st = scan_exclusive_i32(g.tile_cnt, g.tile_start, cell_cap, g.scan, s);
    if (st) return st;
    hipLaunchKernelGGL(k_tile_scatter, dim3(nb), dim3(KNN_THREADS), 0, s, cblk_off + nb, ctile, g.tile_start,
                       g.tile_cursor, order);
    hipLaunchKernelGGL(k_tile_list, dim3(ceil_div(cell_cap, LIST_THREADS)), dim3(LIST_THREADS), 0, s, g.tile_cnt,
                       cell_cap, g.tile_list, g.n_tile_list);
    hipLaunchKernelGGL(k_knn_tiles, dim3(256 * 3), dim3(KNN_THREADS), 0, s, (const float4*)q_pos4, cand, g.gp,
                       g.cell_start, (const float4*)sorted_pts4, g.tile_list, g.n_tile_list, g.tile_start,
                       g.tile_cnt, order, flag, t_nbr);
    hipLaunchKernelGGL(k_knn_flag_count, dim3(nb), dim3(KNN_THREADS), 0, s, flag, cblk_off + nb, blk_cnt);
    st = scan_exclusive_i32(blk_cnt, blk_off, nb, sws, s);
    if (st) return st;
    hipLaunchKernelGGL(k_knn_flag_compact, dim3(nb), dim3(KNN_THREADS), 0, s, (const float4*)q_pos4, q_ray, cand,
                       cblk_off + nb, flag, t_nbr, blk_off, (float4*)s_pos4, s_ray, s_nbr, nb,
                       n_survivors_dev);
    return launch_status();
  }
  if (knn_mode() == 4) {
    int* flag = t_ray;              // per candidate slot
    int* hard = cand_blk;           // free after the candidate compaction
    int* n_hard = cblk_cnt + nb + 1;
    APN_TRY(fill_i32(n_hard, 0, 1, s));
    hipLaunchKernelGGL(k_knn_pass_a, dim3(nb), dim3(KNN_THREADS), 0, s, (const float4*)q_pos4, cand, cblk_off + nb,
                       g.gp, g.cell_start, (const float4*)sorted_pts4, flag, t_nbr, hard, n_hard);
    hipLaunchKernelGGL(k_knn_pass_b, dim3(nb), dim3(KNN_THREADS), 0, s, (const float4*)q_pos4, cand, hard, n_hard,
                       g.gp, g.cell_start, (const float4*)sorted_pts4, flag, t_nbr);
    hipLaunchKernelGGL(k_knn_flag_count, dim3(nb), dim3(KNN_THREADS), 0, s, flag, cblk_off + nb, blk_cnt);
    st = scan_exclusive_i32(blk_cnt, blk_off, nb, sws, s);
    if (st) return st;
    hipLaunchKernelGGL(k_knn_flag_compact, dim3(nb), dim3(KNN_THREADS), 0, s, (const float4*)q_pos4, q_ray, cand,
                       cblk_off + nb, flag, t_nbr, blk_off, (float4*)s_pos4, s_ray, s_nbr, nb,
                       n_survivors_dev);
    return launch_status();
  }
  if (knn_mode() == 3)
    hipLaunchKernelGGL(k_knn_search<true>, dim3(nb), dim3(KNN_THREADS), 0, s, (const float4*)q_pos4, q_ray, cand,
                       cblk_off + nb, g.gp, g.cell_start, (const float4*)sorted_pts4, t_pos, t_ray, t_nbr, blk_cnt,
                       3);
  else
    hipLaunchKernelGGL(k_knn_search<false>, dim3(nb), dim3(KNN_THREADS), 0, s, (const float4*)q_pos4, q_ray, cand,
                       cblk_off + nb, g.gp, g.cell_start, (const float4*)sorted_pts4, t_pos, t_ray, t_nbr, blk_cnt,
                       knn_mode());
  st = scan_exclusive_i32(blk_cnt, blk_off, nb, sws, s);
  if (st) return st;
  hipLaunchKernelGGL(k_knn_compact, dim3(nb), dim3(KNN_THREADS), 0, s, t_pos, t_ray, t_nbr, blk_cnt, blk_off,
                     (float4*)s_pos4, s_ray, s_nbr);
  APN_TRY(copy_i32(blk_off + nb, n_survivors_dev, 1, s));
  return launch_status();
#endif  // APN_DEBUG_BUILD
}

extern "C" int apn_knn_radius(const float* q_pos4, const int32_t* q_ray, int64_t n_queries,
                              const int32_t* n_queries_dev, const void* grid_workspace, int64_t n_points,
                              int32_t cell_cap, const float* sorted_pts4, float query_radius, float* s_pos4,
                              int32_t* s_ray, int32_t* s_nbr, int32_t* n_survivors_dev, void* workspace,
                              void* stream) {
  return knn_radius_impl(q_pos4, q_ray, n_queries, n_queries_dev, grid_workspace, n_points, cell_cap, sorted_pts4,
                         query_radius, s_pos4, s_ray, s_nbr, n_survivors_dev, workspace, nullptr, stream);
}

extern "C" int32_t apn_knn_uses_agrid(int64_t n_queries) { return knn_uses_agrid(n_queries) ? 1 : 0; }

extern "C" int apn_knn_agrid_build(const void* grid_workspace, int64_t n_points, int32_t cell_cap,
                                   const float* sorted_pts4, void* stream) {
  if (n_points <= 0 || cell_cap <= 0 || !grid_workspace || !sorted_pts4) return APN_ERR_ARG;
  if (n_points > KNN_MAX_POINTS) return APN_ERR_ARG;
  GridWs g = grid_ws((void*)grid_workspace, n_points, cell_cap);
  return agrid_build(g, n_points, cell_cap, sorted_pts4, (hipStream_t)stream);
}

extern "C" int apn_knn_radius_ev(const float* q_pos4, const int32_t* q_ray, int64_t n_queries,
                                 const int32_t* n_queries_dev, const void* grid_workspace, int64_t n_points,
                                 int32_t cell_cap, const float* sorted_pts4, float query_radius, float* s_pos4,
                                 int32_t* s_ray, int32_t* s_nbr, int32_t* n_survivors_dev, void* workspace,
                                 void* agrid_ready, void* stream) {
  if (!agrid_ready) return APN_ERR_ARG;
  return knn_radius_impl(q_pos4, q_ray, n_queries, n_queries_dev, grid_workspace, n_points, cell_cap, sorted_pts4,
                         query_radius, s_pos4, s_ray, s_nbr, n_survivors_dev, workspace, agrid_ready, stream);
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

// Small sets (the chamfer losses: a few thousand points on each side, often 2D pixel sets with
// a zero z): every query scans every point through 512-point LDS tiles, split over 8 waves
// (lane = query, wave = point slice) and merged in LDS -- no bbox / grid build
// launches, no ring search over a degenerate grid. Same distance expression and tie rule
// (knn_insert) as k_knn_points, so the result is the same brute-force answer.
constexpr int KNN_BRUTE_Q = 64;      // queries per block (one per lane of a wave)
constexpr int KNN_BRUTE_S = 8;       // waves per block: each scans every 8th point of a tile
constexpr int KNN_BRUTE_TILE = 512;  // points per LDS tile
template <int K>
__global__ __launch_bounds__(KNN_BRUTE_Q * KNN_BRUTE_S) void k_knn_brute(const float* __restrict__ q, int64_t M,
                                                                         const float* __restrict__ pts, int64_t N,
                                                                         int k_out, int64_t* __restrict__ idx_out,
                                                                         float* __restrict__ d2_out) {
  __shared__ float4 tile[KNN_BRUTE_TILE];
  __shared__ float md[KNN_BRUTE_S - 1][K][KNN_BRUTE_Q];
  __shared__ int mi[KNN_BRUTE_S - 1][K][KNN_BRUTE_Q];
  const int lane = threadIdx.x & 63, slice = threadIdx.x >> 6;
  const int64_t m = (int64_t)blockIdx.x * KNN_BRUTE_Q + lane;
  const bool live = m < M;
  const float qx = live ? q[3 * m] : 0.f, qy = live ? q[3 * m + 1] : 0.f, qz = live ? q[3 * m + 2] : 0.f;
  float bd[K];
  int bi[K];
#pragma unroll
  for (int j = 0; j < K; ++j) { bd[j] = INFINITY; bi[j] = 0x7fffffff; }
  for (int64_t base = 0; base < N; base += KNN_BRUTE_TILE) {
    __syncthreads();
    for (int i = threadIdx.x; i < KNN_BRUTE_TILE; i += KNN_BRUTE_Q * KNN_BRUTE_S) {
      const int64_t n = base + i;
      tile[i] = n < N ? make_float4(pts[3 * n], pts[3 * n + 1], pts[3 * n + 2], 0.f) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    __syncthreads();
    const int cnt = (int)(N - base < KNN_BRUTE_TILE ? N - base : KNN_BRUTE_TILE);
    for (int i = slice; i < cnt; i += KNN_BRUTE_S) {
      const float4 P = tile[i];
      const float dx = qx - P.x, dy = qy - P.y, dz = qz - P.z;
      const float d = (dx * dx + dy * dy) + dz * dz;
      knn_insert<K>(d, (int)(base + i), bd, bi);
    }
  }
  // merge: each slice holds the exact top K of its points; (d, index) order makes the merged
  // list the global top K whatever the slice assignment
  if (slice > 0) {
#pragma unroll
    for (int j = 0; j < K; ++j) { md[slice - 1][j][lane] = bd[j]; mi[slice - 1][j][lane] = bi[j]; }
  }
  __syncthreads();
  if (slice > 0 || !live) return;
  for (int s2 = 0; s2 < KNN_BRUTE_S - 1; ++s2)
#pragma unroll
    for (int j = 0; j < K; ++j) knn_insert<K>(md[s2][j][lane], mi[s2][j][lane], bd, bi);
  for (int j = 0; j < k_out; ++j) {
    idx_out[m * k_out + j] = bi[j];
    d2_out[m * k_out + j] = bd[j];
  }
}

// brute force when the whole pair count is small (and the grid would cost more than the scan)
static inline bool knn_points_brute(int64_t M, int64_t N) { return N <= 16384 && M * N <= ((int64_t)1 << 27); }

extern "C" int apn_knn_points(const float* q, int64_t n_queries, const float* pts, int64_t n_points, int32_t k,
                              int32_t cell_cap, float* sorted_pts4, int32_t* bbox_ord, void* grid_workspace,
                              int64_t* idx_out, float* d2_out, void* stream) {
  if (n_queries < 0 || n_points <= 0 || k < 1 || k > 16 || k > n_points || !pts || !sorted_pts4 || !bbox_ord ||
      !grid_workspace || (n_queries > 0 && (!q || !idx_out || !d2_out)))
    return APN_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (n_queries > 0 && knn_points_brute(n_queries, n_points)) {
    auto brute = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(ceil_div(n_queries, KNN_BRUTE_Q)), dim3(KNN_BRUTE_Q * KNN_BRUTE_S), 0, s, q,
                         n_queries, pts,
                         n_points, k, idx_out, d2_out);
    };
    if (k == 1) brute(k_knn_brute<1>);
    else if (k <= 8) brute(k_knn_brute<8>);
    else brute(k_knn_brute<16>);
    return launch_status();
  }
  hipLaunchKernelGGL(k_bbox_init2, dim3(1), dim3(64), 0, s, bbox_ord);
  hipLaunchKernelGGL(k_bbox_from_points, dim3(ceil_div(n_points, 256)), dim3(256), 0, s, pts, n_points, bbox_ord);
  int st = apn_grid_build(pts, n_points, bbox_ord, 0.01f, cell_cap, sorted_pts4, grid_workspace, stream);
  if (st) return st;
  if (n_queries == 0) return launch_status();
  GridWs g = grid_ws(grid_workspace, n_points, cell_cap);
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(ceil_div(n_queries, 128)), dim3(128), 0, s, q, n_queries, g.gp, g.cell_start,
                       (const float4*)sorted_pts4, pts, n_points, k, idx_out, d2_out);
  };
  if (k == 1) go(k_knn_points<1>);
  else if (k <= 8) go(k_knn_points<8>);
  else go(k_knn_points<16>);
  return launch_status();
}
