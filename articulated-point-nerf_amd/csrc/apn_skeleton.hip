// Skeleton stage of PointWarper.forward (pointwarper.py:213-239) in one workgroup:
//   [time embedding poc_fre(t) (tineuvox.py:872-878), optional]
//   TransformNet (pointwarper.py:5-37, 17 -> 256 x4 (ReLU) -> (J+1)*4, last layer without bias)
//   -> Rodrigues (118-143) -> sibling / rotation masks (230-236)
//   -> M_j = [R_j | p - R_j p] about the parent joint p (167-172)
//   -> kinematic chain as the reference's recursive-halving matrix product (145-153, 173-175)
//   -> joints_rel = T_j [joint_j; 1] (258-260)
//   -> [skeleton projection of joints_rel + global_t into the views (temporalpoints.py:578-583,
//       utils.py:435-450), optional].
// The reference runs this as ~100 tiny torch launches per frame; here it is one launch. The GEMV
// layers read 0.9 MB of transposed, coalesced weights once, split over 4 K-slices (1024 threads:
// a quarter of the dependent load batches per thread -- the stage is load-latency bound); the chain
// products run from LDS.
#include "apn_common.h"

namespace apn {

constexpr int SK_THREADS = 1024;
constexpr int SK_OUT = 256;                      // max GEMV width (hidden, (J+1)*4, t_dim)
constexpr int SK_SLICES = SK_THREADS / SK_OUT;   // K-slices per output feature
constexpr int SK_KMAX = SK_OUT / SK_SLICES;      // inputs per K-slice (in_dim <= SK_OUT)
constexpr int SK_MAX_J = 64;
constexpr int SK_MAX_VIEWS = 16;
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
    float* __restrict__ global_t_out, float* __restrict__ joints_rel_out, const int* __restrict__ chain_prog,
    const float* __restrict__ time_poc, int n_freq, const float* __restrict__ c2w, const float* __restrict__ Kmat,
    int n_views, float* __restrict__ joints2d_out, int* __restrict__ sweep_idx, int sweep_len) {
  __shared__ float h[2][SK_OUT];
  __shared__ float sPart[SK_SLICES][SK_OUT];
  __shared__ float sInv[SK_MAX_VIEWS][12];
  __shared__ float sJw[SK_MAX_J][3];
  __shared__ float sP[SK_MAX_J + 1][4];
  __shared__ float sR[SK_MAX_J][9];
  __shared__ float sM[SK_MAX_J + 1][16];
  __shared__ int sProg[2 * SK_MAX_DEPTH];
  __shared__ int sFrames[SK_MAX_DEPTH + 2][3];
  __shared__ int sNProg;
  __shared__ float sStk[SK_MAX_J][SK_STACK][16];
  const int tid = threadIdx.x;
  const bool tpath = rot_params == nullptr;
  // batch mode (rot path, no index, sweep_len > 0): block b computes pose b of the sweep into
  // output slot b (apn_skeleton_sweep: every pose of a repose sweep in one launch)
  if (!tpath && !sweep_idx && sweep_len > 0) {
    const size_t b = blockIdx.x;
    rot_params += b * J * rot_dim;
    thetas_out += b * J;
    bone_T16 += b * J * 16;
    bone_T34 += b * J * 12;
    global_t_out += b * 3;
    joints_rel_out += b * J * 3;
  }
  // sweep mode (rot path): rot_params holds sweep_len poses; this launch takes pose *sweep_idx and
  // advances the index (a captured repose step then needs no per-pose input copy)
  const int sweep_i = sweep_idx ? *sweep_idx : 0;
  if (sweep_idx) rot_params += (size_t)(sweep_i % sweep_len) * J * rot_dim;
  if (chain_prog) {   // the host's program for this depth (2 depth - 1 ops)
    if (tid < 2 * depth - 1) sProg[tid] = chain_prog[tid];
    if (tid == 0) sNProg = 2 * depth - 1;
  } else if (tid == SK_THREADS - 1) {
    sNProg = chain_program(depth, sProg, sFrames);   // overlaps the GEMVs
  }
  if (tpath) {
    // time embedding (tineuvox.py:872-878): [t, sin(t f_0..f_F-1), cos(t f_0..f_F-1)]
    if (tid < t_dim) {
      if (time_poc) {
        const float t = t_embed[0];
        h[0][tid] = tid == 0 ? t : (tid <= n_freq ? sinf(t * time_poc[tid - 1]) : cosf(t * time_poc[tid - 1 - n_freq]));
      } else {
        h[0][tid] = t_embed[tid];
      }
    }
    __syncthreads();
    // TransformNet: output feature o = tid % 256 over K-slice tid / 256 (each slice summed in k
    // order), the slices added pairwise
    const float* w = tnw;
    const int o = tid % SK_OUT, sl = tid / SK_OUT;
    const int n_w = t_dim * hidden + hidden + (n_layers - 2) * (hidden * hidden + hidden) + hidden * (J + 1) * 4;
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void*)tnw, 0, n_w * 4, 0x00020000);
    int in_dim = t_dim, cur = 0;
    for (int l = 0; l < n_layers; ++l) {
      const bool last = l == n_layers - 1;
      const int out_dim = last ? (J + 1) * 4 : hidden;
      const int kper = (in_dim + SK_SLICES - 1) / SK_SLICES;
      const int k0 = sl * kper, k1 = min(in_dim, k0 + kper);
      float a = 0.f;
      if (k1 - k0 == SK_KMAX) {   // the hidden and last layers (in_dim = 256): the slice's 64 weights
        // as one batch of buffer loads (a running 32-bit VGPR offset): one load latency per layer
        // instead of one per 16-load batch. Threads past out_dim read column out_dim - 1, unused.
        float wr[SK_KMAX];
        int off = (int)((w - tnw) + (size_t)k0 * out_dim + min(o, out_dim - 1)) * 4;
        const int st4 = out_dim * 4;
#pragma unroll
        for (int u = 0; u < SK_KMAX; ++u) {
          wr[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(wrs, off, 0, 0));
          off += st4;
          asm volatile("" : "+v"(off));   // not 64 hoisted scalar products
        }
        if (o < out_dim) {
#pragma unroll
          for (int u = 0; u < SK_KMAX; ++u) a += wr[u] * h[cur][k0 + u];   // k order, as before
        }
      } else if (o < out_dim) {   // the time-embedding layer (in_dim = t_dim): short slices
        const float* wc = w + o;
        for (int k = k0; k < k1; ++k) a += wc[(size_t)k * out_dim] * h[cur][k];
      }
      sPart[sl][o] = a;
      __syncthreads();
      if (tid < out_dim) {
        float v = (sPart[0][tid] + sPart[1][tid]) + (sPart[2][tid] + sPart[3][tid]);
        if (!last) {
          v += w[(size_t)out_dim * in_dim + tid];
          h[cur ^ 1][tid] = fmaxf(v, 0.f);
        } else {
          sP[tid >> 2][tid & 3] = v;
          params_out[tid] = v;
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
  // inverse of each view's camera-to-world matrix (torch.inverse, utils.py:437), Gauss-Jordan with
  // partial pivoting in double on threads the Rodrigues step leaves idle; rows 0-2 kept
  if (tid >= SK_OUT && tid < SK_OUT + n_views) {
    const int v = tid - SK_OUT;
    double A[4][8];
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) {
        A[i][j] = c2w[16 * v + 4 * i + j];
        A[i][4 + j] = i == j ? 1.0 : 0.0;
      }
    for (int c = 0; c < 4; ++c) {
      int p = c;
      for (int i = c + 1; i < 4; ++i)
        if (fabs(A[i][c]) > fabs(A[p][c])) p = i;
      if (p != c)
        for (int j = 0; j < 8; ++j) { const double tt = A[c][j]; A[c][j] = A[p][j]; A[p][j] = tt; }
      const double inv = 1.0 / A[c][c];
      for (int j = 0; j < 8; ++j) A[c][j] *= inv;
      for (int i = 0; i < 4; ++i)
        if (i != c) {
          const double f = A[i][c];
          for (int j = 0; j < 8; ++j) A[i][j] -= f * A[c][j];
        }
    }
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 4; ++j) sInv[v][4 * i + j] = (float)A[i][4 + j];
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
    float jr[3];
    jr[0] = ((T[0] * jx + T[1] * jy) + T[2] * jz) + T[3];
    jr[1] = ((T[4] * jx + T[5] * jy) + T[6] * jz) + T[7];
    jr[2] = ((T[8] * jx + T[9] * jy) + T[10] * jz) + T[11];
    for (int e = 0; e < 3; ++e) {
      joints_rel_out[3 * tid + e] = jr[e];
      sJw[tid][e] = jr[e] + (tpath ? sP[J][e] : 0.f);   // joints_rel + global_t (temporalpoints.py:580)
    }
  }
  if (tid < 3) global_t_out[tid] = tpath ? sP[J][tid] : 0.f;
  if (n_views > 0) {
    // project_point_to_image_plane (utils.py:435-450): x_cam = inv(c2w)[:3,:3] x + inv(c2w)[:3,3],
    // x_img = K x_cam, (u, v) = x_img[:2] / x_img[2]
    __syncthreads();
    if (tid < J * n_views) {
      const int v = tid / J, j = tid % J;
      const float* I = sInv[v];
      const float* Kv = Kmat + 9 * v;
      const float wx = sJw[j][0], wy = sJw[j][1], wz = sJw[j][2];
      float pc[3], q[3];
      for (int i = 0; i < 3; ++i) pc[i] = ((I[4 * i] * wx + I[4 * i + 1] * wy) + I[4 * i + 2] * wz) + I[4 * i + 3];
      for (int i = 0; i < 3; ++i) q[i] = (Kv[3 * i] * pc[0] + Kv[3 * i + 1] * pc[1]) + Kv[3 * i + 2] * pc[2];
      joints2d_out[2 * tid + 0] = q[0] / q[2];
      joints2d_out[2 * tid + 1] = q[1] / q[2];
    }
  }
  if (sweep_idx && tid == 0) *sweep_idx = (sweep_i + 1) % sweep_len;   // every thread read it before the barriers above
}

}  // namespace apn

using namespace apn;

extern "C" int apn_skeleton_frame(const float* t, const float* time_poc, int32_t n_freq, const float* rot_params,
                                  int32_t rot_dim, int32_t n_joints, const float* tn_weights, int32_t hidden,
                                  int32_t n_layers, const float* joints, const int32_t* parent_indices, int32_t depth,
                                  const int32_t* parent_joint_ex, const int32_t* sibling_mask, const int32_t* rot_mask,
                                  float* params_out, float* thetas_out, float* bone_T16, float* bone_T34,
                                  float* global_t_out, float* joints_rel_out, const int32_t* chain_prog,
                                  const float* c2w, const float* K, int32_t n_views, float* joints2d_out,
                                  int32_t* sweep_index, int32_t sweep_len, void* stream) {
  const bool tpath = rot_params == nullptr;
  const int t_dim = 1 + 2 * n_freq;
  if (n_joints <= 0 || n_joints > SK_MAX_J || depth <= 0 || depth > SK_MAX_DEPTH || !joints || !parent_indices ||
      !parent_joint_ex || !thetas_out || !bone_T16 || !bone_T34 || !global_t_out || !joints_rel_out)
    return APN_ERR_ARG;
  if (tpath && (!t || !time_poc || !tn_weights || !params_out || n_freq < 0 || t_dim > SK_OUT || hidden <= 0 ||
                hidden > SK_OUT || n_layers < 2 || (n_joints + 1) * 4 > SK_OUT))
    return APN_ERR_ARG;
  if (!tpath && rot_dim != 3 && rot_dim != 4) return APN_ERR_ARG;
  if (n_views < 0 || n_views > SK_MAX_VIEWS || n_joints * n_views > SK_THREADS ||
      (n_views > 0 && (!c2w || !K || !joints2d_out)))
    return APN_ERR_ARG;
  if (sweep_index && (tpath || sweep_len <= 0)) return APN_ERR_ARG;
  hipLaunchKernelGGL(k_skeleton_pose, dim3(1), dim3(SK_THREADS), 0, (hipStream_t)stream, t, t_dim, rot_params,
                     rot_dim, n_joints, tn_weights, hidden, n_layers, joints, parent_indices, depth, parent_joint_ex,
                     sibling_mask, rot_mask, params_out, thetas_out, bone_T16, bone_T34, global_t_out,
                     joints_rel_out, chain_prog, time_poc, n_freq, c2w, K, n_views, joints2d_out, sweep_index,
                     sweep_len);
  return launch_status();
}

// Every pose of a repose sweep [n_poses, J, rot_dim] in one launch (one workgroup per pose, the
// rot-param path of k_skeleton_pose); outputs are per-pose slices.
extern "C" int apn_skeleton_sweep(const float* rot_params, int32_t n_poses, int32_t rot_dim, int32_t n_joints,
                                  const float* joints, const int32_t* parent_indices, int32_t depth,
                                  const int32_t* parent_joint_ex, const int32_t* sibling_mask, const int32_t* rot_mask,
                                  float* thetas_out, float* bone_T16, float* bone_T34, float* global_t_out,
                                  float* joints_rel_out, const int32_t* chain_prog, void* stream) {
  if (n_poses <= 0 || !rot_params || (rot_dim != 3 && rot_dim != 4) || n_joints <= 0 || n_joints > SK_MAX_J ||
      depth <= 0 || depth > SK_MAX_DEPTH || !joints || !parent_indices || !parent_joint_ex || !thetas_out ||
      !bone_T16 || !bone_T34 || !global_t_out || !joints_rel_out)
    return APN_ERR_ARG;
  hipLaunchKernelGGL(k_skeleton_pose, dim3(n_poses), dim3(SK_THREADS), 0, (hipStream_t)stream, nullptr, 0, rot_params,
                     rot_dim, n_joints, nullptr, 0, 0, joints, parent_indices, depth, parent_joint_ex, sibling_mask,
                     rot_mask, nullptr, thetas_out, bone_T16, bone_T34, global_t_out, joints_rel_out, chain_prog,
                     nullptr, 0, nullptr, nullptr, 0, nullptr, nullptr, n_poses);
  return launch_status();
}

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
  if (tpath && (!t_embed || !tn_weights || !params_out || t_dim <= 0 || t_dim > SK_OUT || hidden <= 0 ||
                hidden > SK_OUT || n_layers < 2 || (n_joints + 1) * 4 > SK_OUT))
    return APN_ERR_ARG;
  if (!tpath && rot_dim != 3 && rot_dim != 4) return APN_ERR_ARG;

  hipLaunchKernelGGL(k_skeleton_pose, dim3(1), dim3(SK_THREADS), 0, (hipStream_t)stream, t_embed, t_dim, rot_params,
                     rot_dim, n_joints, tn_weights, hidden, n_layers, joints, parent_indices, depth, parent_joint_ex,
                     sibling_mask, rot_mask, params_out, thetas_out, bone_T16, bone_T34, global_t_out,
                     joints_rel_out, chain_prog, nullptr, 0, nullptr, nullptr, 0, nullptr, nullptr, 0);
  return launch_status();
}
