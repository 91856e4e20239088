// Device-wide exclusive prefix sum of int32 counts (rays, grid cells, kNN blocks). Up to 8192
// entries: one workgroup, one launch (scan_single).
// Per-block totals, then per-block scans that add the sum of the preceding blocks' totals -- each
// block sums them itself (nb <= SCAN_DIRECT_MAX blocks: every scan of the render frame, up to 8M
// elements), so two launches instead of three (the one-workgroup scan of the totals was a
// launch of its own, ~5 us of latency per scan). Larger inputs keep the three-launch form.
// Deterministic (no atomics), so every consumer sees the same offsets run to run.
#include "apn_common.h"

namespace apn {

constexpr int SCAN_THREADS = 256;
constexpr int SCAN_ITEMS = 8;
constexpr int SCAN_TILE = SCAN_THREADS * SCAN_ITEMS;  // 2048 elements per block

__device__ __forceinline__ int wave_incl_scan(int v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

// Block-wide exclusive scan of one value per thread; returns exclusive prefix, *total set.
__device__ __forceinline__ int block_excl_scan(int v, int* lds_waves, int* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int inc = wave_incl_scan(v);
  if (lane == 63) lds_waves[wid] = inc;
  __syncthreads();
  int base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < SCAN_THREADS / 64; ++w) {
    int x = lds_waves[w];
    base += (w < wid) ? x : 0;
    tot += x;
  }
  __syncthreads();
  *total = tot;
  return base + inc - v;
}

__global__ __launch_bounds__(SCAN_THREADS) void scan_block_totals(const int* __restrict__ in, int64_t n,
                                                                  int* __restrict__ totals) {
  __shared__ int lw[SCAN_THREADS / 64];
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_ITEMS;
  int s = 0;
#pragma unroll
  for (int i = 0; i < SCAN_ITEMS; ++i) s += (base + i < n) ? in[base + i] : 0;
  int tot;
  block_excl_scan(s, lw, &tot);
  if (threadIdx.x == 0) totals[blockIdx.x] = tot;
}

__global__ __launch_bounds__(1024) void scan_totals_single(int* __restrict__ totals, int nb) {
  // exclusive scan in place over nb block totals, one workgroup, chunks of 1024
  __shared__ int lw[16];
  __shared__ int carry_s;
  if (threadIdx.x == 0) carry_s = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int c = 0; c < nb; c += 1024) {
    int i = c + threadIdx.x;
    int v = i < nb ? totals[i] : 0;
    int inc = wave_incl_scan(v);
    if (lane == 63) lw[wid] = inc;
    __syncthreads();
    int base = 0, tot = 0;
    for (int w = 0; w < 16; ++w) {
      base += (w < wid) ? lw[w] : 0;
      tot += lw[w];
    }
    int carry = carry_s;
    if (i < nb) totals[i] = carry + base + inc - v;
    __syncthreads();
    if (threadIdx.x == 0) carry_s = carry + tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) totals[nb] = carry_s;
}

__global__ __launch_bounds__(SCAN_THREADS) void scan_block_apply(const int* __restrict__ in, int64_t n,
                                                                 const int* __restrict__ totals,
                                                                 int* __restrict__ out, int nb) {
  __shared__ int lw[SCAN_THREADS / 64];
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_ITEMS;
  int v[SCAN_ITEMS];
  int s = 0;
#pragma unroll
  for (int i = 0; i < SCAN_ITEMS; ++i) {
    v[i] = (base + i < n) ? in[base + i] : 0;
    s += v[i];
  }
  int tot;
  int run = block_excl_scan(s, lw, &tot) + totals[blockIdx.x];
#pragma unroll
  for (int i = 0; i < SCAN_ITEMS; ++i) {
    if (base + i < n) out[base + i] = run;
    run += v[i];
  }
  if (blockIdx.x == nb - 1 && threadIdx.x == 0) out[n] = totals[nb];
}

// The per-block scan with the block's offset = sum of totals[0 .. b-1], reduced by the block itself.
constexpr int SCAN_DIRECT_MAX = 4096;
__global__ __launch_bounds__(SCAN_THREADS) void scan_block_apply_direct(const int* __restrict__ in, int64_t n,
                                                                        const int* __restrict__ totals,
                                                                        int* __restrict__ out, int nb) {
  __shared__ int lw[SCAN_THREADS / 64];
  __shared__ int red[SCAN_THREADS / 64];
  const int b = blockIdx.x;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  // offset of this block (and, in the last block, the grand total): integer sums, any order is exact
  const int lim = b == nb - 1 ? nb : b;
  int part = 0;
  for (int i = threadIdx.x; i < lim; i += SCAN_THREADS) part += totals[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
  if (lane == 0) red[wid] = part;
  const int64_t base = (int64_t)b * SCAN_TILE + threadIdx.x * SCAN_ITEMS;
  int v[SCAN_ITEMS];
  int s = 0;
#pragma unroll
  for (int i = 0; i < SCAN_ITEMS; ++i) {
    v[i] = (base + i < n) ? in[base + i] : 0;
    s += v[i];
  }
  int tot;
  const int excl = block_excl_scan(s, lw, &tot);   // its barriers also publish red[]
  int off = 0;
#pragma unroll
  for (int w = 0; w < SCAN_THREADS / 64; ++w) off += red[w];
  // the last block summed all nb totals: its own offset is that minus its own total
  if (b == nb - 1) {
    if (threadIdx.x == 0) out[n] = off;
    off -= tot;
  }
  int run = excl + off;
#pragma unroll
  for (int i = 0; i < SCAN_ITEMS; ++i) {
    if (base + i < n) out[base + i] = run;
    run += v[i];
  }
}

// Short inputs (<= SCAN_SINGLE_MAX: the kNN's per-block counts of a ray shard, ~4k entries) in one
// launch: one 1024-thread workgroup, 8 entries per thread (6.4 us against 10.3 for the two-launch
// form on a shard of 8). Each further chunk of 8192 costs the workgroup a dependent round trip:
// at 31k entries (a whole C2 frame) it was ~30 us slower than the two-launch form.
constexpr int SCAN_SINGLE_MAX = 1 << 13;
constexpr int SCAN_SINGLE_ITEMS = 8;
__global__ __launch_bounds__(1024) void scan_single(const int* __restrict__ in, int64_t n, int* __restrict__ out) {
  __shared__ int lw[16];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  int carry = 0;   // the same in every thread
  for (int64_t c = 0; c < n; c += 1024 * SCAN_SINGLE_ITEMS) {
    const int64_t base = c + (int64_t)tid * SCAN_SINGLE_ITEMS;
    int v[SCAN_SINGLE_ITEMS];
    int sum = 0;
#pragma unroll
    for (int i = 0; i < SCAN_SINGLE_ITEMS; ++i) {
      v[i] = base + i < n ? in[base + i] : 0;
      sum += v[i];
    }
    const int inc = wave_incl_scan(sum);
    if (lane == 63) lw[wid] = inc;
    __syncthreads();
    int wb = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < 16; ++w) {
      const int x = lw[w];
      wb += w < wid ? x : 0;
      tot += x;
    }
    __syncthreads();   // lw is rewritten by the next chunk
    int run = carry + wb + inc - sum;
#pragma unroll
    for (int i = 0; i < SCAN_SINGLE_ITEMS; ++i) {
      if (base + i < n) out[base + i] = run;
      run += v[i];
    }
    carry += tot;
  }
  if (tid == 0) out[n] = carry;
}

size_t scan_workspace_bytes(int64_t n) {
  int64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
  return (size_t)(nb + 1) * sizeof(int);
}

int scan_exclusive_i32(const int* in, int* out, int64_t n, void* ws, hipStream_t s) {
  if (n <= 0) {
    APN_TRY(fill_i32(out, 0, 1, s));
    return launch_status();
  }
  if (n <= SCAN_SINGLE_MAX) {
    hipLaunchKernelGGL(scan_single, dim3(1), dim3(1024), 0, s, in, n, out);
    return launch_status();
  }
  int nb = ceil_div(n, SCAN_TILE);
  int* totals = (int*)ws;
  hipLaunchKernelGGL(scan_block_totals, dim3(nb), dim3(SCAN_THREADS), 0, s, in, n, totals);
  if (nb <= SCAN_DIRECT_MAX) {
    hipLaunchKernelGGL(scan_block_apply_direct, dim3(nb), dim3(SCAN_THREADS), 0, s, in, n, totals, out, nb);
    return launch_status();
  }
  hipLaunchKernelGGL(scan_totals_single, dim3(1), dim3(1024), 0, s, totals, nb);
  hipLaunchKernelGGL(scan_block_apply, dim3(nb), dim3(SCAN_THREADS), 0, s, in, n, totals, out, nb);
  return launch_status();
}

}  // namespace apn

extern "C" size_t apn_scan_workspace_bytes(int64_t n) { return apn::scan_workspace_bytes(n); }

extern "C" int apn_scan_exclusive_i32(const int32_t* in, int32_t* out, int64_t n, void* workspace,
                                      void* stream) {
  return apn::scan_exclusive_i32(in, out, n, workspace, (hipStream_t)stream);
}
