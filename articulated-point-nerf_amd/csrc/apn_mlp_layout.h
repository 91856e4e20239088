// Tile shape and packed-weight layout shared by the neighbour-MLP kernels (apn_mlp.hip: FP32
// MFMA; apn_mlp_h3.hip: 3-term fp16-split MFMA) and apn_amd/ops.py:pack_mlp_weights (through
// apn_mlp_weight_layout()).
#pragma once
#include <functional>

#include "apn_common.h"

namespace apn {

constexpr int TS = 8;             // samples per tile
constexpr int TR = TS * 8;        // MLP rows per tile (sample, neighbour)
constexpr int MLP_THREADS = 256;
constexpr int FEAT = 128;
constexpr int KE = 64;            // positional encoding 63, zero-padded
constexpr int KV = 160;           // head input: h (128) + view embedding (27) + pad

// Packed weight buffer layout (floats). fp32 region: nn.Linear [out][in] rows.
constexpr int OFF_W1E = 0;                        // [128][64]  feat_net.0 columns 0..62
constexpr int OFF_B1 = OFF_W1E + 128 * KE;        // [128]      (+ pose-embedding fold)
constexpr int OFF_W2 = OFF_B1 + 128;              // [128][128]
constexpr int OFF_B2 = OFF_W2 + 128 * 128;
constexpr int OFF_W3 = OFF_B2 + 128;
constexpr int OFF_B3 = OFF_W3 + 128 * 128;
constexpr int OFF_W4 = OFF_B3 + 128;
constexpr int OFF_B4 = OFF_W4 + 128 * 128;
constexpr int OFF_WD = OFF_B4 + 128;              // [128]      densitynet
constexpr int OFF_BD = OFF_WD + 128;              // [4]
constexpr int OFF_WH = OFF_BD + 4;                // [64][160]  folded rgb head layer
constexpr int OFF_BH = OFF_WH + 64 * KV;          // [64]
constexpr int OFF_WV2 = OFF_BH + 64;              // [3][64]    views_linears.2
constexpr int OFF_BV2 = OFF_WV2 + 3 * 64;         // [4]
constexpr int OFF_W1F = OFF_BV2 + 4;              // [128][128] feat_net.0 columns 63..190 (for P)
constexpr int W_F32_TOTAL = OFF_W1F + 128 * 128;

// fp16 hi/lo region (written by apn_mlp_split_weights from the fp32 region): every matrix
// W [O][K] in MFMA fragments -- for o-tile ot (16 rows), k-chunk q (32 columns), part
// (0 = hi = fp16(w), 1 = lo = fp16(w - hi)), lane l: 8 halves W[16 ot + (l & 15)][32 q + 8 (l >> 4) + j].
// One 16-byte load per lane fetches a whole 1 KB fragment, coalesced.
// Wave-major: wave w of the kernel's workgroup owns o-tiles 2w, 2w+1 of W1E..W4 (j = ot & 1) and
// o-tile w of the head, and its 66 fragments are one contiguous block, fragment index
// FR_<matrix> + (j nq + q) 2 + part inside it -- the kernel's load offsets are then a per-wave
// VGPR base plus compile-time constants (no wave-dependent scalar offsets to keep live).
constexpr int OFF_H16 = (W_F32_TOTAL + 3) & ~3;   // float offset (16-B aligned)
constexpr int FRAG_HALVES = 64 * 8;               // one fragment part
constexpr int FR_W1E = 0;                         // fragment index inside a wave's block
constexpr int FR_W2 = FR_W1E + 2 * 2 * 2;
constexpr int FR_W3 = FR_W2 + 2 * 4 * 2;
constexpr int FR_W4 = FR_W3 + 2 * 4 * 2;
constexpr int FR_WH = FR_W4 + 2 * 4 * 2;
constexpr int FR_WAVE = FR_WH + 5 * 2;            // 66 fragments per wave
constexpr int H_TOTAL = 4 * FR_WAVE * FRAG_HALVES;   // halves, relative to OFF_H16
// Range flag (one int32, 4 floats reserved): the fp16-split kernel sets it when a value it must
// split into fp16 hi/lo halves is out of the fp16 range (or not finite); the FP32 MFMA kernel
// then re-runs the launch (apn_point_mlp). Sticky until the weights are re-split
// (apn_mlp_split_weights clears it), so later launches with the same weights go straight to FP32.
constexpr int OFF_FLAG = OFF_H16 + H_TOTAL / 2;
// Power-of-two weight scales of the fp16 hi/lo region (written by apn_mlp_split_weights):
// [W1E, W2, W3, W4, WH h-columns, WH view-columns, mode, 0]. fp16 has 5 exponent bits: the lo
// halves of weights below ~2^-3 are subnormal and lose relative precision. If every group's
// max|w| lies in [2^-5, 2^12] (all reference-initialised or trained networks seen), mode = 0 and
// every scale is 1 (the kernel then runs exactly the unscaled arithmetic). Otherwise mode = 1
// and each group is stored as w * 2^s with max|w 2^s| in [2^12, 2^13) -- exact in fp32 -- and
// the kernel multiplies the layer's accumulators by 2^-s (biases / projections pre-scaled by
// 2^s). The head's two column groups are tested separately (their magnitudes are unrelated:
// rgbnet.feature_linears folds into the h columns only) but scaled together, by the head's max
// (slots 4 and 5 are equal; the kernel's h-input factor 2^(s5 - s4) is then 1).
constexpr int OFF_SCALE = OFF_FLAG + 4;
constexpr int W_TOTAL = OFF_SCALE + 8;
constexpr float SCALE_LO = 0.03125f, SCALE_HI = 4096.f;   // unscaled range of max|w|
constexpr int SCALE_TARGET_EXP = 13;                        // scaled: max|w 2^s| in [2^12, 2^13)

// Column order of the positional encoding inside the fp16 kernels' layer-1 operand (64 columns,
// 8 chunks of 8): chunk pair p (p = 0..3) holds the arguments a = 8p .. 8p+7 -- chunk 2p their
// sines, chunk 2p+1 their cosines -- with a = 10 i + f the reference argument index (rel_c[i] * 2^f,
// poc_fre's dim-major order). Consecutive frequencies of one coordinate are then neighbours, and
// the gather computes every odd frequency from the even one below it by one double-angle step
// (pe_chunk, apn_mlp_split.h). Slots a = 30, 31 carry rel_c: sin slot 30 = rel_c[0], cos slot 30 =
// rel_c[1], sin slot 31 = rel_c[2]; cos slot 31 (column 63) is the constant 1 and its weights are
// b1, so the MFMAs add layer 1's bias (no VALU add in the activation store).
// Returns the reference embedding index (poc_fre order: [x(3), sin(30), cos(30)]) or PE_BIAS.
constexpr int PE_BIAS = -2;
__host__ __device__ constexpr int pe_col_to_ref(int c) {
  const int p = c >> 4, is_cos = (c >> 3) & 1, j = c & 7;
  const int a = 8 * p + j;
  if (a < 30) return (is_cos ? 33 : 3) + a;
  if (a == 30) return is_cos ? 1 : 0;
  return is_cos ? PE_BIAS : 2;
}

// K order of the fp16 kernels' hidden activations (the input of W2, W3, W4): position k of a
// 32-wide K chunk q holds feature act_k_of(k). A lane of wave w holds, after its layer's MFMAs,
// features 32w + 4g + r of o-tile 2w and 32w + 16 + 4g + r of o-tile 2w + 1 (r = 0..3, the
// transposed product's C layout) of one row: stored together as chunk 4w + g -- a whole 16-B
// chunk of hi halves and one of lo halves per lane, no cross-lane exchange -- so the weight
// fragments of W2..W4 take their columns in that order (k_split_weights).
__host__ __device__ constexpr int act_k_of(int k) {
  const int q = k >> 5, g = (k >> 3) & 3, r = k & 7;
  return 32 * q + (r < 4 ? 4 * g + r : 16 + 4 * g + r - 4);
}

// LeakyReLU(0.01): x >= 0 ? x : 0.01x == max(x, 0.01x) (the same rounded product; 2 VALU ops)
__device__ __forceinline__ float lrelu(float x) { return fmaxf(x, x * 0.01f); }

// Launcher of the fp16-split kernel (apn_mlp_h3.hip).
void launch_point_mlp_h3(int blocks, bool timed, hipStream_t stream, const float4* s_pos, const int* s_ray,
                         const int* s_nbr, const int* n_samples_dev, const float4* recA, const float4* recB,
                         const float4* pproj, const float* viewdirs, const float* vemb_const, const float* wbuf,
                         float eps, float shift, float interval, float4* out);
// Launcher of the fp16-split kernel on 128-row tiles (apn_mlp_h4.hip).
// ``list`` (optional): the launch's tile slots are these sample indices (n_samples_dev of them) and
// only each sample's {rgb, alpha} columns are written (early-ray-termination passes, apn_ert.hip).
void launch_point_mlp_h4(int blocks, bool timed, hipStream_t stream, const float4* s_pos, const int* s_ray, const int* s_nbr,
                         const int* n_samples_dev, const float4* recA, const float4* recB, const float4* pproj,
                         const float* viewdirs, const float* vemb_const, const float* wbuf, float eps, float shift,
                         float interval, float4* out, const int* list = nullptr);
// Early ray termination (apn_ert.hip): the MLP in ERT_PASSES passes over the live rays' next
// kept samples; ``MlpPass(list, n_list_dev)`` launches the MLP on one pass's sample list.
constexpr int ERT_PASSES = 9;
// 1: the MLP kernel's IDW weights (temporalpoints.py:473-475) made in its gather by the 128 threads
// that compute the rows' squared distances (the sample's 8 rows are 8 consecutive lanes: a 3-step
// xor-shuffle sum) instead of by 16 threads of wave 0 at the top of layer 1 (8 dependent LDS reads
// and adds per thread while the other waves run layer 1). The 8-term sum becomes the pairwise tree
// ((w0 + w1) + (w2 + w3)) + ((w4 + w5) + (w6 + w7)), which k_direct_blend (apn_ert.hip) then
// follows too, so the early-termination frame stays bit-identical to the full one. Measured slower
// (round 6, same box, parity green: MLP kernel 2.960 / 2.969 -> 2.995 / 3.005 ms per C2 frame; the
// two gather waves of half 0 carry the shuffles alone): off.
#ifndef APN_H4_IDWG
#define APN_H4_IDWG 0
#endif

#ifndef APN_ERT_MLP_BLOCKS
#define APN_ERT_MLP_BLOCKS 2048
#endif
constexpr int ERT_MLP_BLOCKS = APN_ERT_MLP_BLOCKS;   // workgroups per pass launch (8 per CU)
typedef std::function<int(const int*, const int*)> MlpPass;
size_t ert_workspace_bytes(int64_t max_samples, int64_t n_rays);
int ert_run(const float4* s_pos, const int* s_ray, const int* s_nbr, int64_t max_samples, const int* n_samples_dev,
            int64_t n_rays, const float4* recA, const float4* recB, float eps, float thr, float4* out, void* ws,
            int with_direct, int* stats, void* const* events, hipStream_t s, const MlpPass& mlp);
int direct_blend(const float4* s_pos, const int* s_nbr, int64_t max_samples, const int* n_samples_dev,
                 const float4* recA, const float4* recB, float eps, float4* out, hipStream_t s);
// Largest magnitude the fp16-split kernel carries through its hi/lo halves (fp16 max finite).
constexpr float H3_RANGE = 65504.f;
// Adds (and resets) the phase-timed fp16-split kernel's cycle sums into out6.
int debug_phase_cycles_h3(uint64_t* out6);
int debug_phase_cycles_h4(uint64_t* out6);

}  // namespace apn
