// Skeleton stage of PointWarper.forward (pointwarper.py:213-239) in one workgroup:
//   TransformNet (pointwarper.py:5-37, 17 -> 256 x4 (ReLU) -> (J+1)*4, last layer without bias)
//   -> Rodrigues (118-143) -> sibling / rotation masks (230-236)
//   -> M_j = [R_j | p - R_j p] about the parent joint p (167-172)
//   -> kinematic chain as the reference's recursive-halving matrix product (145-153, 173-175)
//   -> joints_rel = T_j [joint_j; 1] (258-260).
// The reference runs this as ~100 tiny torch launches per frame; here it is one launch (GEMV
// layers read 0.9 MB of transposed, coalesced weights once; the chain products run from LDS).
#include "apn_common.h"

namespace apn {

constexpr int SK_THREADS = 256;
constexpr int SK_MAX_J = 64;
constexpr int SK_MAX_DEPTH = 32;
constexpr int SK_STACK = 8;   // recursion depth of the halving tree for chains <= 32 factors: ceil(log2 32) + 1

// C = A B for row-major 4x4, the sum in k order.
__device__ __forceinline__ void mm4(const float* A, const float* B, float* C) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k)
      C[4 * i + k] = ((A[4 * i] * B[k] + A[4 * i + 1] * B[4 + k]) + A[4 * i + 2] * B[8 + k]) + A[4 * i + 3] * B[12 + k];
}

// matrix_chain_product (pointwarper.py:145-153) = prod(left half) @ prod(right half), left =
// first floor(L/2) factors, recursively. The recursion tree depends only on the chain length, so
// it is flattened once per launch into a postfix program (SK_LEAF | d = push factor d, SK_MUL =
// pop two, push their product) that every joint's thread then runs with its stack in LDS.
constexpr int SK_MUL = -1;
__device__ int chain_program(int n, int* prog, int (*st)[3]) {
  int sp = 0, np = 0;
  st[0][0] = 0; st[0][1] = n; st[0][2] = 0;
  while (sp >= 0) {
    int* f = st[sp];
    const int L = f[1] - f[0];
    if (L == 1) { prog[np++] = f[0]; --sp; continue; }
    if (f[2] == 0) { f[2] = 1; st[sp + 1][0] = f[0]; st[sp + 1][1] = f[0] + L / 2; st[sp + 1][2] = 0; ++sp; }
    else if (f[2] == 1) { f[2] = 2; st[sp + 1][0] = f[0] + L / 2; st[sp + 1][1] = f[1]; st[sp + 1][2] = 0; ++sp; }
    else { prog[np++] = SK_MUL; --sp; }
  }
  return np;
}

// Packed TransformNet weights (floats), each layer transposed so that thread o's loads over k are
// coalesced across the block: W0^T [T][H], b0 [H], then for l = 1..NL-2: Wl^T [H][H], bl [H], then
// W_last^T [H][(J+1)*4] (no bias). NL = num_layers (5 in the reference).
__global__ __launch_bounds__(SK_THREADS) void k_skeleton_pose(
    const float* __restrict__ t_embed, int t_dim, const float* __restrict__ rot_params, int rot_dim, int J,
    const float* __restrict__ tnw, int hidden, int n_layers, const float* __restrict__ joints,
    const int* __restrict__ parent_indices, int depth, const int* __restrict__ parent_joint_ex,
    const int* __restrict__ sibling_mask, const int* __restrict__ rot_mask, float* __restrict__ params_out,
    float* __restrict__ thetas_out, float* __restrict__ bone_T16, float* __restrict__ bone_T34,
    float* __restrict__ global_t_out, float* __restrict__ joints_rel_out, const int* __restrict__ chain_prog) {
  __shared__ float h[2][SK_THREADS];
  __shared__ float sP[SK_MAX_J + 1][4];
  __shared__ float sR[SK_MAX_J][9];
  __shared__ float sM[SK_MAX_J + 1][16];
  __shared__ int sProg[2 * SK_MAX_DEPTH];
  __shared__ int sFrames[SK_MAX_DEPTH + 2][3];
  __shared__ int sNProg;
  __shared__ float sStk[SK_MAX_J][SK_STACK][16];
  const int tid = threadIdx.x;
  const bool tpath = rot_params == nullptr;
  if (chain_prog) {   // the host's program for this depth (2 depth - 1 ops)
    if (tid < 2 * depth - 1) sProg[tid] = chain_prog[tid];
    if (tid == 0) sNProg = 2 * depth - 1;
  } else if (tid == SK_THREADS - 1) {
    sNProg = chain_program(depth, sProg, sFrames);   // overlaps the GEMVs
  }
  if (tpath) {
    // TransformNet: one output feature per thread (hidden <= 256), k summed in order
    if (tid < t_dim) h[0][tid] = t_embed[tid];
    __syncthreads();
    const float* w = tnw;
    int in_dim = t_dim, cur = 0;
    for (int l = 0; l < n_layers; ++l) {
      const bool last = l == n_layers - 1;
      const int out_dim = last ? (J + 1) * 4 : hidden;
      if (tid < out_dim) {
        const float* wc = w + tid;
        float a = 0.f;
#pragma unroll 8
        for (int k = 0; k < in_dim; ++k) a += wc[(size_t)k * out_dim] * h[cur][k];
        if (!last) {
          a += w[(size_t)out_dim * in_dim + tid];
          h[cur ^ 1][tid] = fmaxf(a, 0.f);
        } else {
          sP[tid >> 2][tid & 3] = a;
          params_out[tid] = a;
        }
      }
      w += (size_t)out_dim * in_dim + (last ? 0 : out_dim);
      in_dim = out_dim;
      cur ^= 1;
      __syncthreads();
    }
  } else {
    if (tid < J * rot_dim) sP[tid / rot_dim][tid % rot_dim] = rot_params[tid];
    __syncthreads();
  }
  // Rodrigues (pointwarper.py:118-143), thetas = prev_thetas
  if (tid < J) {
    const float* p = sP[tid];
    float theta, x, y, z;
    if (rot_dim == 3 && !tpath) {
      theta = sqrtf(1e-5f + ((p[0] * p[0] + p[1] * p[1]) + p[2] * p[2]));
      x = p[0] / theta; y = p[1] / theta; z = p[2] / theta;
    } else {
      theta = p[3];
      const float nrm = sqrtf(1e-5f + ((p[0] * p[0] + p[1] * p[1]) + p[2] * p[2]));
      x = p[0] / nrm; y = p[1] / nrm; z = p[2] / nrm;
    }
    thetas_out[tid] = theta;
    const float c = cosf(theta), s = sinf(theta);
    float* R = sR[tid];
    R[0] = x * x + (1.f - x * x) * c; R[1] = x * y * (1.f - c) - z * s; R[2] = x * z * (1.f - c) + y * s;
    R[3] = x * y * (1.f - c) + z * s; R[4] = y * y + (1.f - y * y) * c; R[5] = y * z * (1.f - c) - x * s;
    R[6] = x * z * (1.f - c) - y * s; R[7] = y * z * (1.f - c) + x * s; R[8] = z * z + (1.f - z * z) * c;
  }
  __syncthreads();
  // masks, local transforms about the parent joint (pointwarper.py:165-172)
  if (tid <= J) {
    float* M = sM[tid];
    if (tid == 0) {
      for (int e = 0; e < 16; ++e) M[e] = (e % 5 == 0) ? 1.f : 0.f;
    } else {
      const int j = tid - 1;
      float R[9];
      if (rot_mask && rot_mask[j]) {
        for (int e = 0; e < 9; ++e) R[e] = (e % 4 == 0) ? 1.f : 0.f;
      } else {
        const int sj = sibling_mask ? sibling_mask[j] : j;
        for (int e = 0; e < 9; ++e) R[e] = sR[sj][e];
      }
      const int pj = parent_joint_ex[j];
      const float px = joints[3 * pj], py = joints[3 * pj + 1], pz = joints[3 * pj + 2];
      // joints_old + R @ (-joints_old)
      const float tx = px + ((R[0] * -px + R[1] * -py) + R[2] * -pz);
      const float ty = py + ((R[3] * -px + R[4] * -py) + R[5] * -pz);
      const float tz = pz + ((R[6] * -px + R[7] * -py) + R[8] * -pz);
      M[0] = R[0]; M[1] = R[1]; M[2] = R[2]; M[3] = tx;
      M[4] = R[3]; M[5] = R[4]; M[6] = R[5]; M[7] = ty;
      M[8] = R[6]; M[9] = R[7]; M[10] = R[8]; M[11] = tz;
      M[12] = 0.f; M[13] = 0.f; M[14] = 0.f; M[15] = 1.f;
    }
  }
  __syncthreads();
  // kinematic chain per joint (pointwarper.py:173-175): the postfix program over the joint's
  // factors (parent_indices, -1 -> identity), top of stack in registers, the rest in LDS
  if (tid < J) {
    const int np = sNProg;
    const int* pidx = parent_indices + (size_t)tid * depth;
    float cur[16];
    int sp = -1;   // LDS stack entries below the top: sStk[tid][0..sp]
    for (int i = 0; i < np; ++i) {
      const int op = sProg[i];
      if (op == SK_MUL) {
        float t[16];
        mm4(sStk[tid][sp], cur, t);   // (left) @ (right = top)
        --sp;
#pragma unroll
        for (int e = 0; e < 16; ++e) cur[e] = t[e];
      } else {
        if (i > 0) {
          ++sp;
#pragma unroll
          for (int e = 0; e < 16; ++e) sStk[tid][sp][e] = cur[e];
        }
        const float* f = sM[pidx[op] + 1];
#pragma unroll
        for (int e = 0; e < 16; ++e) cur[e] = f[e];
      }
    }
    const float* T = cur;
    for (int e = 0; e < 16; ++e) bone_T16[16 * tid + e] = T[e];
    for (int e = 0; e < 12; ++e) bone_T34[12 * tid + e] = T[e];
    const float jx = joints[3 * tid], jy = joints[3 * tid + 1], jz = joints[3 * tid + 2];
    joints_rel_out[3 * tid + 0] = ((T[0] * jx + T[1] * jy) + T[2] * jz) + T[3];
    joints_rel_out[3 * tid + 1] = ((T[4] * jx + T[5] * jy) + T[6] * jz) + T[7];
    joints_rel_out[3 * tid + 2] = ((T[8] * jx + T[9] * jy) + T[10] * jz) + T[11];
  }
  if (tid < 3) global_t_out[tid] = tpath ? sP[J][tid] : 0.f;
}

}  // namespace apn

using namespace apn;

extern "C" int apn_skeleton_pose(const float* t_embed, int32_t t_dim, const float* rot_params, int32_t rot_dim,
                                 int32_t n_joints, const float* tn_weights, int32_t hidden, int32_t n_layers,
                                 const float* joints, const int32_t* parent_indices, int32_t depth,
                                 const int32_t* parent_joint_ex, const int32_t* sibling_mask, const int32_t* rot_mask,
                                 float* params_out, float* thetas_out, float* bone_T16, float* bone_T34,
                                 float* global_t_out, float* joints_rel_out, const int32_t* chain_prog,
                                 void* stream) {
  const bool tpath = rot_params == nullptr;
  if (n_joints <= 0 || n_joints > SK_MAX_J || depth <= 0 || depth > SK_MAX_DEPTH || !joints || !parent_indices ||
      !parent_joint_ex || !thetas_out || !bone_T16 || !bone_T34 || !global_t_out || !joints_rel_out)
    return APN_ERR_ARG;
  if (tpath && (!t_embed || !tn_weights || !params_out || t_dim <= 0 || t_dim > SK_THREADS || hidden <= 0 ||
                hidden > SK_THREADS || n_layers < 2 || (n_joints + 1) * 4 > SK_THREADS))
    return APN_ERR_ARG;
  if (!tpath && rot_dim != 3 && rot_dim != 4) return APN_ERR_ARG;

  hipLaunchKernelGGL(k_skeleton_pose, dim3(1), dim3(SK_THREADS), 0, (hipStream_t)stream, t_embed, t_dim, rot_params,
                     rot_dim, n_joints, tn_weights, hidden, n_layers, joints, parent_indices, depth, parent_joint_ex,
                     sibling_mask, rot_mask, params_out, thetas_out, bone_T16, bone_T34, global_t_out,
                     joints_rel_out, chain_prog);
  return launch_status();
}
