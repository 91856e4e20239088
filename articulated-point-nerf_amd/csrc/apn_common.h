// Shared helpers for the apn HIP kernels (gfx950 / MI355X only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

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
