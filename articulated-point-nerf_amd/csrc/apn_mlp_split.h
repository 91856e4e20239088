// Shared pieces of the fp16-split neighbour-MLP kernels (apn_mlp_h3.hip: 64-row tiles,
// apn_mlp_h4.hip: 128-row tiles): operand types, the posenc sin/cos, the hi/lo split, LeakyReLU,
// the 3-term MFMA, the weight-fragment loads and the swizzled LDS row layouts.
#pragma once
#include "apn_mlp_layout.h"

namespace apn {
namespace mlpx {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));

// bytes per activation row: hi 128 halves | lo 128 halves
constexpr int XB = 512;

// sin and cos of x for the positional encoding, |x| < ~1e6 (arguments are rel_c * 2^f, f <= 9):
// quadrant reduction k = rint(2x/pi), r = x - k pi/2 with pi/2 in two floats (fma, so k C1 is
// exact), minimax polynomials on |r| <= pi/4 (Cephes sinf/cosf coefficients). Max error ~1e-7
// absolute (fp32 sinf: ~7e-8), about a third of the VALU work of the library sincosf and no
// large-argument branch (whose registers the library path keeps live).
// k comes from the 1.5 2^23 rounding trick (one fma + one subtract, |2x/pi| < 2^22), which also
// leaves k mod 4 in the low mantissa bits: the quadrant's swap and sign flips are bit operations.
__device__ __forceinline__ void sincos_pe(float x, float& sn, float& cs) {
  const float kf = fmaf(x, 0.636619772367581343f, 12582912.f);
  const float k = kf - 12582912.f;
  const uint32_t qb = __float_as_uint(kf);
  float r = fmaf(k, -0x1.921fb6p+0f, x);
  r = fmaf(k, 0x1.777a5cp-25f, r);
  const float z = r * r;
  const float sp = fmaf(r * z, fmaf(fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f), r);
  const float cp = fmaf(z * z, fmaf(fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f),
                        fmaf(-0.5f, z, 1.f));
  const bool odd = qb & 1u;
  const float ss = odd ? cp : sp, cc = odd ? sp : cp;
  sn = __uint_as_float(__float_as_uint(ss) ^ ((qb << 30) & 0x80000000u));          // q & 2: -sin
  cs = __uint_as_float(__float_as_uint(cc) ^ (((qb + 1u) << 30) & 0x80000000u));   // (q + 1) & 2: -cos
}

// sin / cos of the positional-encoding arguments a = A0 .. A0 + 7 of one MLP row (a = 10 i + f:
// rel_c[i] * 2^f, tineuvox.py:872-878; apn_mlp_layout.h pe_col_to_ref): even frequencies (and the
// chunk's first argument) by sincos_pe, each odd frequency from the one below it by one
// double-angle step (sin 2x = 2 sin x cos x, cos 2x = 1 - 2 sin^2 x: 4 VALU instead of ~18; the
// argument doubles exactly, 2^f being a power of two). Error budget (float64 over |rel_c| <= 0.3,
// 2M draws): sincos_pe 9.2e-8 absolute, after one step 2.9e-7 (fp32 libm: 7e-8); the stage stays
// within 1e-5 of the fp32 oracle and of float64 (tests/test_mlp_precision.py). Slots 30 / 31 carry
// rel_c and the bias input 1 (see pe_col_to_ref).
template <int A0>
__device__ __forceinline__ void pe_chunk(const float (&rc)[3], f32x4& s0, f32x4& s1, f32x4& c0, f32x4& c1) {
  float sv[8], cv[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int a = A0 + j, i = a / 10, f = a % 10;
    if (a < 30) {
      if (j == 0 || (f & 1) == 0) {
        sincos_pe(rc[i] * (float)(1 << f), sv[j], cv[j]);
      } else {
        const float s = sv[j - 1], c = cv[j - 1];
        sv[j] = 2.f * (s * c);
        cv[j] = fmaf(-2.f * s, s, 1.f);
      }
    } else if (a == 30) {
      sv[j] = rc[0];
      cv[j] = rc[1];
    } else {
      sv[j] = rc[2];
      cv[j] = 1.f;   // the layer-1 bias column (apn_mlp_layout.h PE_BIAS)
    }
  }
  s0 = f32x4{sv[0], sv[1], sv[2], sv[3]};
  s1 = f32x4{sv[4], sv[5], sv[6], sv[7]};
  c0 = f32x4{cv[0], cv[1], cv[2], cv[3]};
  c1 = f32x4{cv[4], cv[5], cv[6], cv[7]};
}

// Byte offset of logical 16-B chunk c (8 halves, 0..15) of the hi part of activation row m.
__device__ __forceinline__ int act_off(int m, int c) { return m * XB + ((c ^ (m & 15)) << 4); }
// Byte offset of fp32 chunk c (4 floats, 0..31) of row m of the layer-4 output.
__device__ __forceinline__ int out32_off(int m, int c) { return m * XB + ((c ^ (m & 7)) << 4); }

// hi = fp16(v) (RNE, v_cvt_pk_f16_f32); lo = fp16(v - hi) with one v_fma_mix{lo,hi}_f16 per value
// (fma(hi as f16, -1, v as f32) rounded once to f16: v - hi is exact in fp32, so the bits equal
// cvt(v - cvt(hi))) instead of a convert-back, a subtraction and a second convert.
__device__ __forceinline__ uint32_t split_lo2(uint32_t hi2, float a, float b) {
  uint32_t lo2;
  asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %0, %1, -1.0, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
      : "=&v"(lo2) : "v"(hi2), "v"(a), "v"(b));
  return lo2;
}
__device__ __forceinline__ void split4(const f32x4& v, h4& hi, h4& lo) {
  hi = __builtin_convertvector(v, h4);
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  const u32x2 hb = __builtin_bit_cast(u32x2, hi);
  lo = __builtin_bit_cast(h4, (u32x2){split_lo2(hb[0], v[0], v[1]), split_lo2(hb[1], v[2], v[3])});
}
// LeakyReLU(0.01) = max(x, 0.01x) with scalar multiplies (packed f32 VALU beside MFMAs costs
// more than two plain ops, MI355X_MICROARCH.md constants table). The max is written as asm: the
// compiler's fmaxf/fmed3f first canonicalise an MFMA result (an extra v_max_f32 x, x, x per
// value, IEEE mode), a third of the epilogue's VALU. A NaN x gives NaN either way (both operands).
__device__ __forceinline__ float lrelu_asm(float x) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(x * 0.01f));
  return r;
}
__device__ __forceinline__ f32x4 lrelu4(const f32x4& v) {
  return f32x4{lrelu_asm(v[0]), lrelu_asm(v[1]), lrelu_asm(v[2]), lrelu_asm(v[3])};
}

__device__ __forceinline__ f32x4 mfma3(const h8& ahi, const h8& alo, const h8& bhi, const h8& blo, f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi, bhi, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi, blo, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(alo, bhi, acc, 0, 0, 0);
  return acc;
}

// Weight fragments are read through a buffer descriptor: the per-lane offset (lane * 16 B) is
// the only VGPR, the fragment offset a wave-uniform SGPR -- plain 64-bit pointers per fragment
// would be hoisted out of the tile loop by the compiler (~80 live VGPR pairs).
typedef __amdgpu_buffer_rsrc_t rsrc_t;

// Fragment f of this wave's block (apn_mlp_layout.h, wave-major): the per-lane VGPR offset
// vb = wave block + lane * 16 B is the only register; f is a compile-time constant after
// unrolling, so the scalar offset is an immediate / rematerialised constant.
__device__ __forceinline__ h8 frag(rsrc_t rs, int vb, int f) {
#ifdef APN_H3_PROBE_L1W   // timing probe only (wrong results): 4 fragments shared by every wave, L1-resident
  return __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(rs, (threadIdx.x & 63) * 16, (f & 3) * (FRAG_HALVES * 2), 0));
#endif
  return __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(rs, vb, f * (FRAG_HALVES * 2), 0));
}


}  // namespace mlpx
}  // namespace apn
