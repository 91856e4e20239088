// TiNeuVox stage-1 field on MI355X (lib/tineuvox.py:91-625): the voxel model
// the articulated point cloud is exported from. Per query point p (a ray sample, or a grid point
// of the canonical export, run.py:1152-1194):
//
//   pe   = poc_fre(p, 2^0..2^9)                                   (63)   tineuvox.py:479
//   p'   = p + Deformation([pe, timenet(poc_fre(t))])                      :487, 28-62
//          (Linear(123->128) + ReLU, (D-2) x [Linear(128->128) + ReLU], Linear(128->3))
//   vox  = 3-scale trilinear grid_sample of the 12-channel feature grid at p'  :402-419, 379-394
//          (scales 1, 1/2, 1/4 of the zero-padded grid; align_corners=True, zeros outside)
//   h    = ReLU(featurenet([poc_fre(vox, 2^0..2^1) (180), pe (63), timenet (60)]))   :497-501
//   alpha = raw2alpha(densitynet(h) + shift, interval)                      :503-506
//   rgb  = sigmoid(rgbnet(h, poc_fre(viewdir, 2^0..2^3)))                   :525-532
//
// Layout / arithmetic choices (all reassociations exact in R, ~1e-7 relative in fp32):
//   * the feature grid is repacked channels-last per scale ([x][y][z][12] fp32, 48 B per corner:
//     three 16-B loads) so a corner gather is one contiguous 48-B run; the three scales are
//     separate arrays (the reference's strided views [::2], [::4] of the padded grid);
//   * the time-feature columns of the first deformation layer and of featurenet are the same for
//     every sample of a time value: their products with timenet(t) (+ the layer bias) are
//     precomputed per distinct time (tproj [U][256], apn_amd/tineuvox.py) and gathered into the
//     accumulators, so the in-kernel contractions are K = 64 (posenc) and K = 256 (180 + 63 + pad);
//   * rgbnet.feature_linears folds into views_linears.0 (no activation between them) as in the
//     point path: one 160-wide layer [h; view embedding];
//   * matrices run on FP32 MFMA (v_mfma_f32_16x16x4_f32): tile = 64 samples x 128 features per
//     256-thread workgroup, activations in LDS (row stride 264 floats = 8 mod 64: conflict-free
//     b128 operand reads), weights streamed from L2 (0.3 MB per model).
#include "apn_common.h"

namespace apn {
namespace tnv {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int NC = 12;          // voxel_dim (feature channels)
constexpr int NF = 3 * NC;      // multi-scale features
constexpr int KE = 64;          // posenc 63 + zero pad
constexpr int KF = 256;         // featurenet operand: vox emb 180 | posenc 63 | zero pad 13
constexpr int PE_COL = 180;     // posenc columns inside the featurenet operand (also layer-0 operand)
constexpr int KV = 160;         // head operand: h 128 | view embedding 27 | zero pad 5
constexpr int WD = 128;         // net_width
constexpr int TS = 64;          // samples per tile
constexpr int THREADS = 256;
constexpr int XS = 264;         // LDS row stride (floats)
constexpr int HOUT = 160;       // LDS column of the head's 64-wide hidden output

// Packed weight layout (floats), for defor_depth D (nn.Linear [out][in] rows, K zero-padded).
struct Layout {
  int d0e, dh, dout, fw, wd, bd, wh, bh, wv2, bv2, total;
};
__host__ __device__ inline Layout layout(int D) {
  Layout L;
  int o = 0;
  L.d0e = o; o += WD * KE;                      // deformation layer 0, posenc columns
  L.dh = o; o += (D - 2) * (WD * WD + WD);      // hidden layers: W then b
  L.dout = o; o += 3 * WD + 4;                  // _time_out W [3][128] then b [3] (+pad)
  L.fw = o; o += WD * KF;                       // featurenet columns 0..242 (+pad)
  L.wd = o; o += WD;                            // densitynet
  L.bd = o; o += 4;
  L.wh = o; o += 64 * KV;                       // folded rgb head
  L.bh = o; o += 64;
  L.wv2 = o; o += 3 * 64;                       // views_linears.2
  L.bv2 = o; o += 4;
  L.total = o;
  return L;
}

// Padded grid size along an axis (tineuvox.py:404-407: (size - 1) made a multiple of 4) and the
// size of scale k (the [::2^k] view).
__host__ __device__ inline int padded(int n) { return (n - 1 + 3) / 4 * 4 + 1; }
__host__ __device__ inline int scaled(int n, int k) { return (padded(n) - 1) / (1 << k) + 1; }
__host__ __device__ inline int64_t scale_voxels(int X, int Y, int Z, int k) {
  return (int64_t)scaled(X, k) * scaled(Y, k) * scaled(Z, k);
}
__host__ __device__ inline int64_t scale_offset(int X, int Y, int Z, int k) {   // floats
  int64_t o = 0;
  for (int j = 0; j < k; ++j) o += scale_voxels(X, Y, Z, j) * NC;
  return o;
}

// feature [C][X][Y][Z] -> channels-last padded scale grids. One thread per (scale, voxel).
__global__ void k_grid_pack(const float* __restrict__ feat, int X, int Y, int Z, float* __restrict__ grid) {
  const int64_t n0 = scale_voxels(X, Y, Z, 0), n1 = scale_voxels(X, Y, Z, 1), n2 = scale_voxels(X, Y, Z, 2);
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n0 + n1 + n2;
       t += (int64_t)gridDim.x * blockDim.x) {
    int k = 0;
    int64_t v = t;
    if (v >= n0) { v -= n0; k = 1; if (v >= n1) { v -= n1; k = 2; } }
    const int sy = scaled(Y, k), sz = scaled(Z, k);
    const int z = (int)(v % sz), y = (int)((v / sz) % sy), x = (int)(v / ((int64_t)sy * sz));
    const int fx = x << k, fy = y << k, fz = z << k;   // fine (padded) coordinates
    const bool in = fx < X && fy < Y && fz < Z;       // F.pad zeros past the original grid
    float* dst = grid + scale_offset(X, Y, Z, k) + v * NC;
#pragma unroll
    for (int c = 0; c < NC; ++c)
      dst[c] = in ? feat[(((int64_t)c * X + fx) * Y + fy) * Z + fz] : 0.f;
  }
}

// Grid-sample index of coordinate p along an axis of the bbox [mn, mx] for a scale of size S:
// (p - mn) / (mx - mn) -> *2 - 1 (grid_sampler, tineuvox.py:384) -> ((u + 1) / 2) * (S - 1)
// (PyTorch grid_sampler_compute_source_index, align_corners=True). Same IEEE operations.
__device__ __forceinline__ float src_index(float p, float mn, float mx, int S) {
  const float u = ((p - mn) / (mx - mn)) * 2.f - 1.f;
  const float ix = ((u + 1.f) / 2.f) * (float)(S - 1);
  // |ix| beyond the grid only selects out-of-bounds (zero) corners; keep the int conversion defined
  return fminf(fmaxf(ix, -2.f), (float)(S + 1));
}

// Trilinear sample of the 12-channel scale grid at (ix, iy, iz) = (X, Y, Z) indices, zeros
// outside: PyTorch's 3-D bilinear grid_sampler (CPU), corner order tnw, tne, tsw, tse, bnw, bne,
// bsw, bse and weights (W-term)(H-term)(D-term) with W = our z, H = y, D = x (the flip of
// tineuvox.py:384).
__device__ __forceinline__ void trilinear12(const float* __restrict__ g, int SX, int SY, int SZ, float ix, float iy,
                                            float iz, float (&v)[NC]) {
#pragma unroll
  for (int c = 0; c < NC; ++c) v[c] = 0.f;
  if (!(ix == ix && iy == iy && iz == iz)) return;   // NaN position: every corner out of bounds
  const int x0 = (int)floorf(ix), y0 = (int)floorf(iy), z0 = (int)floorf(iz);
  const float wx0 = (float)(x0 + 1) - ix, wx1 = ix - (float)x0;
  const float wy0 = (float)(y0 + 1) - iy, wy1 = iy - (float)y0;
  const float wz0 = (float)(z0 + 1) - iz, wz1 = iz - (float)z0;
#pragma unroll
  for (int corner = 0; corner < 8; ++corner) {
    const int dx = corner >> 2, dy = (corner >> 1) & 1, dz = corner & 1;
    const int x = x0 + dx, y = y0 + dy, z = z0 + dz;
    const float w = ((dz ? wz1 : wz0) * (dy ? wy1 : wy0)) * (dx ? wx1 : wx0);
    if (x >= 0 && x < SX && y >= 0 && y < SY && z >= 0 && z < SZ) {
      const f32x4* src = (const f32x4*)(g + (((int64_t)x * SY + y) * SZ + z) * NC);
      const f32x4 a = src[0], b = src[1], cc = src[2];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[j] = v[j] + a[j] * w;
        v[4 + j] = v[4 + j] + b[j] * w;
        v[8 + j] = v[8 + j] + cc[j] * w;
      }
    }
  }
}

__device__ __forceinline__ void sample_scale(const float* __restrict__ grid, int X, int Y, int Z, int k, float px,
                                             float py, float pz, const float* __restrict__ mn,
                                             const float* __restrict__ mx, float (&v)[NC]) {
  const int SX = scaled(X, k), SY = scaled(Y, k), SZ = scaled(Z, k);
  trilinear12(grid + scale_offset(X, Y, Z, k), SX, SY, SZ, src_index(px, mn[0], mx[0], SX),
              src_index(py, mn[1], mx[1], SY), src_index(pz, mn[2], mx[2], SZ), v);
}

// mult_dist_interp (tineuvox.py:402-419): out [M][36] = [scale 1 (12) | 1/2 (12) | 1/4 (12)].
// One thread per (point, scale).
__global__ void k_mult_dist_interp(const float* __restrict__ pts, int64_t M, const float* __restrict__ grid, int X,
                                   int Y, int Z, const float* __restrict__ mn, const float* __restrict__ mx,
                                   float* __restrict__ out) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < 3 * M; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = t / 3;
    const int k = (int)(t % 3);
    float v[NC];
    sample_scale(grid, X, Y, Z, k, pts[3 * m], pts[3 * m + 1], pts[3 * m + 2], mn, mx, v);
#pragma unroll
    for (int c = 0; c < NC; ++c) out[m * NF + NC * k + c] = v[c];
  }
}

// acc[mt][nt] += X[rows][xcol + k] * Wt[col0 + 16 nt + li][k] over K (C layout as apn_mlp.hip).
template <int K, int MT, int NT>
__device__ __forceinline__ void mma(const float* __restrict__ X, int xcol, const float* __restrict__ Wt, int col0,
                                    f32x4 (&acc)[MT][NT]) {
  const int lane = threadIdx.x & 63;
  const int li = lane & 15, g = lane >> 4;
  const float* xa = X + li * XS + xcol + 4 * g;
  const float* wb = Wt + (size_t)(col0 + li) * K + 4 * g;
  f32x4 b[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) b[nt] = *(const f32x4*)(wb + (size_t)nt * 16 * K);
#pragma unroll 2
  for (int q = 0; q < K / 16; ++q) {
    f32x4 a[MT], bn[NT];
    const int qn = q + 1 < K / 16 ? q + 1 : q;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) bn[nt] = *(const f32x4*)(wb + (size_t)nt * 16 * K + 16 * qn);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) a[mt] = *(const f32x4*)(xa + mt * 16 * XS + 16 * q);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[mt][t], b[nt][t], acc[mt][nt], 0, 0, 0);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) b[nt] = bn[nt];
  }
}

// X[row][xcol + col] = relu(acc + bias[col]) (bias may be null), C layout.
template <int MT, int NT>
__device__ __forceinline__ void store_relu(float* __restrict__ X, int xcol, int col0, const float* __restrict__ bias,
                                           const f32x4 (&acc)[MT][NT]) {
  const int lane = threadIdx.x & 63;
  const int li = lane & 15, g = lane >> 4;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int col = col0 + 16 * nt + li;
    const float bb = bias ? bias[col] : 0.f;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) X[(16 * mt + 4 * g + r) * XS + xcol + col] = fmaxf(acc[mt][nt][r] + bb, 0.f);
  }
}

// accumulators <- the per-time projection row of each tile row (C layout)
__device__ __forceinline__ void init_tproj(f32x4 (&acc)[4][2], const float* __restrict__ tproj, const int* sT,
                                           int off, int col0) {
  const int lane = threadIdx.x & 63;
  const int li = lane & 15, g = lane >> 4;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float* row = tproj + (size_t)sT[16 * mt + 4 * g + r] * 256 + off + col0 + li;
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) acc[mt][nt][r] = row[16 * nt];
    }
}

__global__ __launch_bounds__(THREADS, 2) void k_tnv_field(
    const float4* __restrict__ pos4, const int* __restrict__ s_ray, const int* __restrict__ time_idx,
    const int* __restrict__ n_samples_dev, const float* __restrict__ grid, int X, int Y, int Z,
    const float* __restrict__ mn, const float* __restrict__ mx, const float* __restrict__ wbuf, int D,
    const float* __restrict__ tproj, const float* __restrict__ viewdirs, const float* __restrict__ vemb_const,
    int deform, float shift, float interval, float4* __restrict__ out12, float* __restrict__ delta_out,
    float* __restrict__ h_out, float* __restrict__ vox_out) {
  __shared__ __attribute__((aligned(16))) float Xs[TS * XS];
  __shared__ float sP[TS * 4];
  __shared__ int sT[TS];
  __shared__ int sR[TS];
  __shared__ float sA[TS];
  const Layout L = layout(D);
  const int nS = *n_samples_dev;
  const int ntiles = (nS + TS - 1) / TS;
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col0 = 32 * wid;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int s0 = tile * TS;
    // ---------------------------------------------------------------- rows
    if (tid < TS) {
      const int s = s0 + tid;
      const bool ok = s < nS;
      const float4 p = ok ? pos4[s] : make_float4(0.f, 0.f, 0.f, 0.f);
      const int r = ok ? s_ray[s] : 0;
      sP[4 * tid] = p.x; sP[4 * tid + 1] = p.y; sP[4 * tid + 2] = p.z;
      sR[tid] = r;
      sT[tid] = time_idx ? time_idx[r] : 0;
    }
    __syncthreads();
    // ---------------------------------------------------------------- posenc (tineuvox.py:872-878)
    {
      const int row = tid >> 2, part = tid & 3;
      float* xr = Xs + row * XS;
      const float p3[3] = {sP[4 * row], sP[4 * row + 1], sP[4 * row + 2]};
      for (int e = part; e < KE; e += 4) {
        float v = 0.f;
        if (e < 3) {
          v = p3[e];
        } else if (e < 63) {
          const int a = (e - 3) % 30, ci = a / 10, f = a % 10;
          const float arg = p3[ci] * (float)(1 << f);
          v = e < 33 ? sinf(arg) : cosf(arg);
        }
        xr[PE_COL + e] = v;   // column 243 (e = 63) = 0
      }
      for (int c = PE_COL + KE + part; c < KF; c += 4) xr[c] = 0.f;
    }
    __syncthreads();
    // ---------------------------------------------------------------- deformation (tineuvox.py:28-62)
    if (deform) {
      f32x4 acc[4][2];
      init_tproj(acc, tproj, sT, 0, col0);   // time columns . timenet(t) + b0
      mma<KE, 4, 2>(Xs, PE_COL, wbuf + L.d0e, col0, acc);
      store_relu<4, 2>(Xs, 0, col0, nullptr, acc);   // writes columns 0..127, reads were 180..243
      __syncthreads();
      for (int l = 0; l < D - 2; ++l) {
        const float* Wl = wbuf + L.dh + (size_t)l * (WD * WD + WD);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
        mma<WD, 4, 2>(Xs, 0, Wl, col0, acc);
        __syncthreads();
        store_relu<4, 2>(Xs, 0, col0, Wl + WD * WD, acc);
        __syncthreads();
      }
      if (tid < 3 * TS) {   // _time_out Linear(128 -> 3), then pts + dx
        const int row = tid / 3, o = tid % 3;
        const float* xr = Xs + row * XS;
        const float* w = wbuf + L.dout + o * WD;
        float d = 0.f;
        for (int k = 0; k < WD; ++k) d = d + xr[k] * w[k];
        const float pn = sP[4 * row + o] + (d + wbuf[L.dout + 3 * WD + o]);
        sP[4 * row + o] = pn;
        if (delta_out && s0 + row < nS) delta_out[(size_t)(s0 + row) * 3 + o] = pn;
      }
    } else if (delta_out && tid < 3 * TS && s0 + tid / 3 < nS) {
      delta_out[(size_t)(s0 + tid / 3) * 3 + tid % 3] = sP[4 * (tid / 3) + tid % 3];
    }
    __syncthreads();
    // ---------------------------------------------------------------- 3-scale trilinear + its posenc
    if (tid < 3 * TS) {   // wave k = scale k (scale-uniform waves), lane = row
      const int row = tid & 63, k = tid >> 6;
      float v[NC];
      sample_scale(grid, X, Y, Z, k, sP[4 * row], sP[4 * row + 1], sP[4 * row + 2], mn, mx, v);
      float* xr = Xs + row * XS;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int ch = NC * k + c;
        float s1, c1, s2, c2;
        sincosf(v[c], &s1, &c1);
        sincosf(v[c] * 2.f, &s2, &c2);
        xr[ch] = v[c];
        xr[NF + 2 * ch] = s1;
        xr[NF + 2 * ch + 1] = s2;
        xr[NF + 2 * NF + 2 * ch] = c1;
        xr[NF + 2 * NF + 2 * ch + 1] = c2;
      }
      if (vox_out && s0 + row < nS) {
#pragma unroll
        for (int c = 0; c < NC; ++c) vox_out[(size_t)(s0 + row) * NF + NC * k + c] = v[c];
      }
    }
    __syncthreads();
    // ---------------------------------------------------------------- featurenet (tineuvox.py:497-501)
    {
      f32x4 acc[4][2];
      init_tproj(acc, tproj, sT, 128, col0);   // time columns . timenet(t) + bias
      mma<KF, 4, 2>(Xs, 0, wbuf + L.fw, col0, acc);
      __syncthreads();
      store_relu<4, 2>(Xs, 0, col0, nullptr, acc);
      if (h_out) {
        const int li = lane & 15, g = lane >> 4;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = 16 * mt + 4 * g + r;
            if (s0 + row < nS)
#pragma unroll
              for (int nt = 0; nt < 2; ++nt)
                h_out[(size_t)(s0 + row) * WD + col0 + 16 * nt + li] = fmaxf(acc[mt][nt][r], 0.f);
          }
      }
    }
    __syncthreads();
    // ---------------------------------------------------------------- density + view embedding
    {
      const int row = tid >> 2, part = tid & 3;
      float* xr = Xs + row * XS;
      const float* wdv = wbuf + L.wd + 32 * part;
      float d = 0.f;
      for (int k = 0; k < 32; ++k) d = d + xr[32 * part + k] * wdv[k];
      d += __shfl_xor(d, 1, 64);
      d += __shfl_xor(d, 2, 64);
      if (part == 0) {   // Raw2Alpha (render_utils_kernel.cu:357-369)
        const float e = expf((d + wbuf[L.bd]) + shift);
        sA[row] = 1.f - powf(1.f + e, -interval);
      }
      const int ray = sR[row];
      for (int e = part; e < KV - WD; e += 4) {   // poc_fre(viewdirs, 2^0..2^3) (27) + pad
        float v = 0.f;
        if (e < 27) {
          if (vemb_const) {
            v = vemb_const[e];
          } else {
            const int ee = e < 3 ? 0 : (e < 15 ? e - 3 : e - 15);
            const float vv = viewdirs[3 * (size_t)ray + (e < 3 ? e : ee >> 2)];
            const float arg = vv * (float)(1 << (ee & 3));
            v = e < 3 ? vv : (e < 15 ? sinf(arg) : cosf(arg));
          }
        }
        xr[WD + e] = v;
      }
    }
    __syncthreads();
    // ---------------------------------------------------------------- folded rgb head
    {
      f32x4 acc[4][1];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) acc[mt][0] = f32x4{0.f, 0.f, 0.f, 0.f};
      mma<KV, 4, 1>(Xs, 0, wbuf + L.wh, 16 * wid, acc);
      store_relu<4, 1>(Xs, HOUT, 16 * wid, wbuf + L.bh, acc);   // writes 160..223, reads were 0..159
    }
    __syncthreads();
    if (tid < 3 * TS) {   // views_linears.2 (64 -> 3) + sigmoid
      const int row = tid / 3, o = tid % 3;
      const float* xr = Xs + row * XS + HOUT;
      const float* w = wbuf + L.wv2 + 64 * o;
      float a = 0.f;
      for (int k = 0; k < 64; ++k) a = a + xr[k] * w[k];
      sP[4 * row + o] = 1.f / (1.f + expf(-(a + wbuf[L.bv2 + o])));   // rgb (positions no longer needed)
    }
    __syncthreads();
    if (tid < TS && s0 + tid < nS) {
      float4* o = out12 + (size_t)(s0 + tid) * 3;
      o[0] = make_float4(sP[4 * tid], sP[4 * tid + 1], sP[4 * tid + 2], sA[tid]);
      o[1] = make_float4(0.f, 0.f, 0.f, 0.f);
      o[2] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    __syncthreads();
  }
}

}  // namespace tnv
}  // namespace apn

using namespace apn;

extern "C" int64_t apn_tnv_grid_bytes(int32_t C, int32_t X, int32_t Y, int32_t Z) {
  if (C != tnv::NC || X < 2 || Y < 2 || Z < 2) return -1;
  return (int64_t)sizeof(float) * tnv::scale_offset(X, Y, Z, 3);
}

extern "C" int apn_tnv_grid_pack(const float* feature, int32_t C, int32_t X, int32_t Y, int32_t Z, float* grid,
                                 void* stream) {
  if (C != tnv::NC || X < 2 || Y < 2 || Z < 2 || !feature || !grid) return APN_ERR_ARG;
  const int64_t n = tnv::scale_voxels(X, Y, Z, 0) + tnv::scale_voxels(X, Y, Z, 1) + tnv::scale_voxels(X, Y, Z, 2);
  int blocks = ceil_div(n, 256);
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(tnv::k_grid_pack, dim3(blocks), dim3(256), 0, (hipStream_t)stream, feature, X, Y, Z, grid);
  return launch_status();
}

extern "C" int apn_tnv_mult_dist_interp(const float* pts, int64_t n_pts, const float* grid, int32_t X, int32_t Y,
                                        int32_t Z, const float* xyz_min, const float* xyz_max, float* out,
                                        void* stream) {
  if (n_pts < 0 || X < 2 || Y < 2 || Z < 2) return APN_ERR_ARG;
  if (n_pts == 0) return APN_OK;
  if (!pts || !grid || !xyz_min || !xyz_max || !out) return APN_ERR_ARG;
  int blocks = ceil_div(3 * n_pts, 256);
  if (blocks > 256 * 64) blocks = 256 * 64;
  hipLaunchKernelGGL(tnv::k_mult_dist_interp, dim3(blocks), dim3(256), 0, (hipStream_t)stream, pts, n_pts, grid, X, Y,
                     Z, xyz_min, xyz_max, out);
  return launch_status();
}

extern "C" int apn_tnv_weight_layout(int32_t defor_depth, int32_t* offsets) {
  if (defor_depth < 2 || !offsets) return APN_ERR_ARG;
  const tnv::Layout L = tnv::layout(defor_depth);
  const int32_t v[] = {L.d0e, L.dh, L.dout, L.fw, L.wd, L.bd, L.wh, L.bh, L.wv2, L.bv2, L.total,
                       tnv::KE, tnv::KF, tnv::KV};
  for (int i = 0; i < (int)(sizeof(v) / sizeof(v[0])); ++i) offsets[i] = v[i];
  return (int)(sizeof(v) / sizeof(v[0]));
}

extern "C" int apn_tnv_field(const float* pos4, const int32_t* s_ray, const int32_t* time_idx, int64_t max_samples,
                             const int32_t* n_samples_dev, const float* grid, int32_t X, int32_t Y, int32_t Z,
                             const float* xyz_min, const float* xyz_max, const float* wbuf, int32_t defor_depth,
                             const float* tproj, const float* viewdirs, const float* vemb_const, int32_t deform,
                             float act_shift, float interval, float* out12, float* delta_out, float* h_out,
                             float* vox_out, void* stream) {
  if (max_samples < 0 || X < 2 || Y < 2 || Z < 2 || defor_depth < 2) return APN_ERR_ARG;
  if (max_samples == 0) return APN_OK;
  if (!pos4 || !s_ray || !n_samples_dev || !grid || !xyz_min || !xyz_max || !wbuf || !tproj || !out12 ||
      (!viewdirs && !vemb_const))
    return APN_ERR_ARG;
  const int64_t ntiles = (max_samples + tnv::TS - 1) / tnv::TS;
  int blocks = 256 * 16;
  if (blocks > ntiles) blocks = (int)ntiles;
  hipLaunchKernelGGL(tnv::k_tnv_field, dim3(blocks), dim3(tnv::THREADS), 0, (hipStream_t)stream, (const float4*)pos4,
                     s_ray, time_idx, n_samples_dev, grid, X, Y, Z, xyz_min, xyz_max, wbuf, defor_depth, tproj,
                     viewdirs, vemb_const, deform, act_shift, interval, (float4*)out12, delta_out, h_out, vox_out);
  return launch_status();
}
