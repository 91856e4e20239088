// Shared helpers for the apn HIP kernels (gfx950 / MI355X only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/apn_hip.h"

#define APN_WAVE 64

namespace apn {

inline int launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? APN_OK : APN_ERR_HIP;
}

#define APN_HIP_TRY(x)                      \
  do {                                      \
    if ((x) != hipSuccess) return APN_ERR_HIP; \
  } while (0)

inline int ceil_div(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// Runtime A/B switches (environment variables) exist in the debug build only
// (libapn_hip_debug.so, -DAPN_DEBUG_BUILD, used by tools/ and the cross-check tests): the shipped
// libapn_hip.so reads no environment variable and always runs the defaults.
#ifdef APN_DEBUG_BUILD
inline const char* apn_env(const char* name) { return ::getenv(name); }
#else
inline const char* apn_env(const char*) { return nullptr; }
#endif

// Stream-ordered int32 fill and copy as plain kernels rather than hipMemsetAsync /
// hipMemcpyAsync, so a captured render frame holds kernel nodes only (the same node kind as
// the repose graph, which replays back to back without fault).
__global__ static void __launch_bounds__(256) k_fill_i32(int* __restrict__ p, int v, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) p[i] = v;
}
__global__ static void __launch_bounds__(64) k_copy_i32(const int* __restrict__ src, int* __restrict__ dst, int n) {
  for (int i = threadIdx.x; i < n; i += 64) dst[i] = src[i];
}
inline int fill_i32(int* p, int v, int64_t n, hipStream_t s) {
  if (n <= 0) return APN_OK;
  const int64_t nb = (n + 255) / 256;
  hipLaunchKernelGGL(k_fill_i32, dim3((unsigned)(nb < 2048 ? nb : 2048)), dim3(256), 0, s, p, v, n);
  return hipPeekAtLastError() == hipSuccess ? APN_OK : APN_ERR_HIP;
}
// Up to four int32 fills in one launch (per-frame counters and count arrays: each separate
// fill is a launch of its own inside the frame).
struct Fill4 {
  int* p[4];
  int64_t n[4];
  int v[4];
};
__global__ static void __launch_bounds__(256) k_fill4_i32(Fill4 f) {
  const int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x, st = (int64_t)gridDim.x * 256;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    for (int64_t i = i0; i < f.n[k]; i += st) f.p[k][i] = f.v[k];
}
inline int fill4_i32(int* p0, int64_t n0, int* p1, int64_t n1, int* p2 = nullptr, int64_t n2 = 0, int* p3 = nullptr,
                     int64_t n3 = 0, hipStream_t s = nullptr) {
  Fill4 f{{p0, p1, p2, p3}, {p0 ? n0 : 0, p1 ? n1 : 0, p2 ? n2 : 0, p3 ? n3 : 0}, {0, 0, 0, 0}};
  int64_t m = 1;
  for (int k = 0; k < 4; ++k) m = f.n[k] > m ? f.n[k] : m;
  const int64_t nb = (m + 255) / 256;
  hipLaunchKernelGGL(k_fill4_i32, dim3((unsigned)(nb < 2048 ? nb : 2048)), dim3(256), 0, s, f);
  return hipPeekAtLastError() == hipSuccess ? APN_OK : APN_ERR_HIP;
}
inline int copy_i32(const int* src, int* dst, int n, hipStream_t s) {
  hipLaunchKernelGGL(k_copy_i32, dim3(1), dim3(64), 0, s, src, dst, n);
  return hipPeekAtLastError() == hipSuccess ? APN_OK : APN_ERR_HIP;
}
#define APN_TRY(x)              \
  do {                          \
    int st_ = (x);              \
    if (st_) return st_;        \
  } while (0)

// Order-preserving float <-> int mapping for atomicMin/atomicMax on floats.
__device__ __forceinline__ int float_to_ordered(float f) {
  int i = __float_as_int(f);
  return i >= 0 ? i : (i ^ 0x7fffffff);
}
__device__ __forceinline__ float ordered_to_float(int i) {
  return __int_as_float(i >= 0 ? i : (i ^ 0x7fffffff));
}

// Exclusive scan of int32 (see apn_scan.hip). Writes out[0..n-1] and out[n] = total.
int scan_exclusive_i32(const int* in, int* out, int64_t n, void* ws, hipStream_t s);
size_t scan_workspace_bytes(int64_t n);

}  // namespace apn
