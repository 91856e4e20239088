/*
 * apn_hip.h -- C-ABI of libapn_hip.so, the MI355X (gfx950) implementation of the
 * articulated-point render/deform hot path of Articulated-Point-NeRF.
 *
 * Conventions
 *   - every pointer is a device pointer unless noted; arrays are dense row-major;
 *   - `stream` is a hipStream_t passed as void* (the caller's current stream);
 *   - functions only enqueue work (no host synchronisation) and return APN_OK or an error
 *     code; APN_ERR_ARG = invalid shape/pointer (the reference raises RuntimeError via
 *     TORCH_CHECK / assert, render_utils.cpp:40-42), APN_ERR_HIP = launch failure;
 *   - scratch memory is caller-provided (`*_workspace_bytes` queries), outputs are
 *     caller-allocated: no allocation happens inside the library.
 * Reference locations are relative to the reference repository root.
 */
#ifndef APN_HIP_H
#define APN_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define APN_OK 0
#define APN_ERR_ARG 1
#define APN_ERR_HIP 2

/* ---------------------------------------------------------------------------------------
 * Drop-in for the `render_utils_cuda` pybind module (lib/cuda/render_utils.cpp:144-155).
 * ------------------------------------------------------------------------------------- */

/* sample_pts_on_rays (render_utils.cpp:67-78, render_utils_kernel.cu:190-236), phase 1:
 * per-ray t_min/t_max/N_steps and the exclusive prefix sum of N_steps in offsets[0..n_rays]
 * (offsets[n_rays] = total_len). The caller reads total_len, allocates, then calls _fill. */
size_t apn_sample_pts_on_rays_workspace_bytes(int64_t n_rays);
int apn_sample_pts_on_rays_count(const float* rays_o, const float* rays_d, const float* xyz_min,
                                 const float* xyz_max, float near, float far, float stepdist,
                                 int64_t n_rays, float* t_min, float* t_max, int64_t* n_steps,
                                 int32_t* offsets, void* workspace, void* stream);
/* phase 2: rays_pts [total_len,3], mask_outbbox [total_len] (1 = outside), ray_id, step_id. */
int apn_sample_pts_on_rays_fill(const float* rays_o, const float* rays_d, const float* xyz_min,
                                const float* xyz_max, float near, float far, float stepdist,
                                int64_t n_rays, const int32_t* offsets, float* rays_pts,
                                uint8_t* mask_outbbox, int64_t* ray_id, int64_t* step_id, void* stream);

/* raw2alpha (render_utils.cpp:80-85, render_utils_kernel.cu:357-393):
 * exp_d = exp(density + shift); alpha = 1 - (1 + exp_d)^(-interval). */
int apn_raw2alpha(const float* density, float shift, float interval, int64_t n_pts, float* exp_d,
                  float* alpha, void* stream);

/* alpha2weight (render_utils.cpp:95-102, render_utils_kernel.cu:430-505); ray_id sorted. */
int apn_alpha2weight(const float* alpha, const int64_t* ray_id, int64_t n_pts, int64_t n_rays,
                     float* weight, float* T, float* alphainv_last, int64_t* i_start, int64_t* i_end,
                     void* stream);

/* raw2alpha_backward (render_utils.cpp:110-114, render_utils_kernel.cu:395-428), the backward of
 * Raw2Alpha (tineuvox.py:646-670): grad = min(exp_d, 1e10) (1 + exp_d)^(-interval-1) interval
 * grad_back, the product in double as in the reference's float instantiation. */
int apn_raw2alpha_backward(const float* exp_d, const float* grad_back, float interval, int64_t n_pts,
                           float* grad, void* stream);

/* alpha2weight_backward (render_utils.cpp:125-141, render_utils_kernel.cu:507-561), the backward
 * of Alphas2Weights (tineuvox.py:627-643); alpha/weight/T/alphainv_last/i_start/i_end are the
 * apn_alpha2weight outputs. grad [n_pts] is zero outside each ray's [i_start, i_end). */
int apn_alpha2weight_backward(const float* alpha, const float* weight, const float* T,
                              const float* alphainv_last, const int64_t* i_start, const int64_t* i_end,
                              int64_t n_pts, int64_t n_rays, const float* grad_weights,
                              const float* grad_last, float* grad, void* stream);

/* torch_scatter.segment_coo(src, index, out=zeros(n_out, C), reduce='sum')
 * (temporalpoints.py:653-677); index sorted; seg_workspace: 2*n_out int64. */
int apn_segment_sum(const float* src, const int64_t* index, int64_t n_pts, int64_t channels,
                    int64_t n_out, float* out, int64_t* seg_workspace, void* stream);

/* ---------------------------------------------------------------------------------------
 * Optimizer-side kernels, in place on fp32 device buffers of n elements.
 * ------------------------------------------------------------------------------------- */

/* adam_upd (adam_upd.cpp:36-48, adam_upd_kernel.cu:8-23, 62-82); the bias-corrected step size
 * lr sqrt(1 - b2^step) / (1 - b1^step) is evaluated on the host in float, as the reference does. */
int apn_adam_upd(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                 int32_t step, float beta1, float beta2, float lr, float eps, void* stream);

/* masked_adam_upd (adam_upd.cpp:50-62, adam_upd_kernel.cu:25-40): grad == 0 leaves the element. */
int apn_masked_adam_upd(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                        int32_t step, float beta1, float beta2, float lr, float eps, void* stream);

/* adam_upd_with_perlr (adam_upd.cpp:64-77, adam_upd_kernel.cu:42-58): step size scaled by perlr. */
int apn_adam_upd_with_perlr(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                            const float* perlr, int64_t n, int32_t step, float beta1, float beta2,
                            float lr, float eps, void* stream);

/* total_variation_add_grad (total_variation.cpp:16-20, total_variation_kernel.cu:13-67) on a
 * [1, C, sz_i, sz_j, sz_k] grid: grad += six clamped neighbour differences (weights / 6; the
 * reference weights the i direction with wz, wx is unused); dense_mode = 0 skips grad == 0. */
/* adam_upd / masked_adam_upd over `count` (<= 24) tensors in one launch (MaskedAdam.step,
 * lib/masked_adam.py:50-72): host arrays of device pointers, element counts, per-tensor step,
 * betas, lr, eps and masked flag (1 = leave elements with grad == 0 untouched); each element
 * updated exactly as by the single-tensor entry points. */
int apn_adam_multi(int32_t count, float* const* params, const float* const* grads, float* const* exp_avgs,
                   float* const* exp_avg_sqs, const int64_t* numels, const int32_t* steps, const float* beta1,
                   const float* beta2, const float* lrs, const float* eps, const int32_t* masked, void* stream);
int apn_total_variation_add_grad(const float* param, float* grad, float wx, float wy, float wz,
                                 int64_t sz_i, int64_t sz_j, int64_t sz_k, int64_t n,
                                 int32_t dense_mode, void* stream);

/* Differentiable LBS of the training path (replaces the autograd composition of
 * TemporalPoints.get_weights temporalpoints.py:401-414, PointWarper.forward's blend/apply
 * pointwarper.py:241-266 and torch.inverse(G)[:3,:3] temporalpoints.py:569). Identity merge rules,
 * 1 <= n_joints <= 64. T34 [J,12] = bone_Ts[:, :3, :]; theta = theta_weight (device, 1 float).
 * fwd: sm_out [N,J] softmax(W/max(eps,theta)), G12_out [N,12] blended 3x4 rows, xyz_out [N,3],
 * Rinv_out [N,9] (adjugate inverse of G[:, :3]).
 * bwd: d_xyz [N,3], d_Rinv [N,9], d_sm [N,J] (each may be NULL = zero) -> dW [N,J], dT34 [J,12],
 * d_global_t [3], d_theta [1] (overwritten; block partials reduced in a fixed order in workspace of
 * apn_lbs_train_workspace_bytes). */
size_t apn_lbs_train_workspace_bytes(int64_t n_points, int32_t n_joints);
int apn_lbs_train_fwd(const float* pcd, const float* W, int64_t n_points, int32_t n_joints,
                      const float* theta, float eps, const float* T34, const float* global_t,
                      float* sm_out, float* G12_out, float* xyz_out, float* Rinv_out, void* stream);
int apn_lbs_train_bwd(const float* pcd, const float* W, int64_t n_points, int32_t n_joints,
                      const float* theta, float eps, const float* T34, const float* sm,
                      const float* Rinv, const float* d_xyz, const float* d_Rinv, const float* d_sm,
                      float* dW, float* dT34, float* d_global_t, float* d_theta, void* workspace,
                      void* stream);

/* Neighbour-graph losses of the training step over the static canonical kNN graph nn_i [N,K]
 * (int64, self first; temporalpoints.py:104-110). Replace the gather + autograd scatter-add of
 * get_neighbour_weight_tv_loss (temporalpoints.py:714-716: mean |w_i - w_nn| over [N,K,J]) and
 * get_arap_loss (temporalpoints.py:723-725: sum |d0_ik - sqrt(|x_i - x_nn|^2 + eps)|).
 * Forward: loss_out[0] (device), block partials in `workspace` (apn_nbr_loss_workspace_bytes)
 * reduced in a fixed order. Backward: d_loss is the device scalar dL/dloss; rev_ptr [N+1] /
 * rev_edge [N*K] is the reverse CSR of the graph (edge ids i*K+k grouped by target, ascending);
 * dw [N,J] / dx [N,3] are overwritten (gathers only, no atomics). Requires n_points * max(n_channels
 * or 3, k) < 2^31 (32-bit indexing in the kernels). */
size_t apn_nbr_loss_workspace_bytes(void);
int apn_nbr_tv_loss(const float* w, int64_t n_points, int32_t n_channels, const int64_t* nn_i, int32_t k,
                    float* loss_out, void* workspace, void* stream);
int apn_nbr_tv_loss_backward(const float* w, int64_t n_points, int32_t n_channels, const int64_t* nn_i,
                             int32_t k, const int64_t* rev_ptr, const int64_t* rev_edge, const float* d_loss,
                             float* dw, void* stream);
int apn_arap_loss(const float* x, int64_t n_points, const int64_t* nn_i, int32_t k, const float* nn_dist0,
                  float eps, float* loss_out, void* workspace, void* stream);
int apn_arap_loss_backward(const float* x, int64_t n_points, const int64_t* nn_i, int32_t k,
                           const float* nn_dist0, float eps, const int64_t* rev_ptr, const int64_t* rev_edge,
                           const float* d_loss, float* dx, void* stream);
/* get_weight_sparsity_loss (temporalpoints.py:718-721) over w [n] (the [N,J] weights, flat):
 * loss_out[0] = -mean(w log(w + eps) + (1 - w) log(1 - w + eps)); backward dw [n] (overwritten). */
int apn_weight_sparsity_loss(const float* w, int64_t n, float eps, float* loss_out, void* workspace, void* stream);
int apn_weight_sparsity_loss_backward(const float* w, int64_t n, float eps, const float* d_loss, float* dw,
                                      void* stream);

/* ---------------------------------------------------------------------------------------
 * Fused render pipeline stages (TemporalPoints.forward, temporalpoints.py:540-712).
 * ------------------------------------------------------------------------------------- */

/* LBS skinning: get_weights (temporalpoints.py:401-414) + PointWarper blend/apply
 * (pointwarper.py:241-266) + torch.inverse(G)[:3,:3] (temporalpoints.py:569) + per-point
 * records for the kNN/MLP stages + bbox of the warped cloud (temporalpoints.py:424).
 *   bone_T34 [J,12]: rows 0..2 of each bone 4x4; merge_rules [J] int32 or NULL (identity);
 *   joint_colors [J,3] or NULL; weights_out [N,J] or NULL;
 *   recA16 [N,16] = {x,y,z, 2*(mmd*max(eps_n,0))^2+1e-12, Rinv(9), clip(alpha), 0,0};
 *   recB8 [N,8] = {clip(rgb), clip(alpha), sum_j col_j w_j, 0}; bbox_ord [6] ordered-int min/max of the
 *   skinned cloud or NULL; workspace: apn_lbs_workspace_bytes(n_points) (needed with bbox_ord). */
size_t apn_lbs_workspace_bytes(int64_t n_points);
int apn_lbs_skin(const float* canonical_pcd, const float* raw_weights, int64_t n_points,
                 int32_t n_joints, const float* theta_weight, float eps, const int32_t* merge_rules,
                 const float* bone_T34, const float* global_t, const float* joint_colors,
                 const float* canonical_alpha, const float* canonical_rgbs, const float* direct_eps,
                 float mean_min_distance, int32_t weights_final, float* xyz_out, float* weights_out,
                 float* G_out, float* recA16, float* recB8, int32_t* bbox_ord, void* workspace,
                 void* stream);
/* weights_final = 1: raw_weights already are the per-point LBS weights (PointWarper.forward
 * input, pointwarper.py:213) -- softmax/merge skipped. G_out [N,16] (weighted_G_tw) or NULL. */

/* Skeleton stage of PointWarper.forward (pointwarper.py:213-239, 118-193) in one launch:
 * TransformNet (t path: t_embed [t_dim] through tn_weights = [W0^T [t_dim][hidden], b0, W1^T, b1,
 * ..., W_last^T [hidden][(J+1)*4]] -- nn.Linear weights transposed, for coalesced loads -- with
 * ReLU between, n_layers Linear layers) or rot_params [J, rot_dim]
 * (rot_dim 3 or 4; t_embed = NULL) -> Rodrigues -> sibling_mask [J] / rot_mask [J] (int32, NULL =
 * identity / none) -> local transforms about parent_joint_ex [J] -> recursive-halving chain
 * product over parent_indices [J, depth] (-1 = identity). Outputs: params_out [(J+1)*4] (t path),
 * thetas [J], bone_T16 [J,16], bone_T34 [J,12] (rows 0..2), global_t [3] (params[J][:3]; 0 for
 * rot_params), joints_rel [J,3]. J <= 64, depth <= 32, hidden <= 256. chain_prog: the
 * recursive-halving product over `depth` factors as a postfix program (2 depth - 1 int32: factor
 * index d = push factor d, -1 = multiply the top two), e.g. precomputed once by the host
 * (PointWarper._tree_buffers); NULL = the kernel derives it. */
int apn_skeleton_pose(const float* t_embed, int32_t t_dim, const float* rot_params, int32_t rot_dim,
                      int32_t n_joints, const float* tn_weights, int32_t hidden, int32_t n_layers,
                      const float* joints, const int32_t* parent_indices, int32_t depth,
                      const int32_t* parent_joint_ex, const int32_t* sibling_mask,
                      const int32_t* rot_mask, float* params_out, float* thetas_out, float* bone_T16,
                      float* bone_T34, float* global_t_out, float* joints_rel_out, const int32_t* chain_prog, void* stream);

/* The render frame's whole skeleton stage in one launch (replaces, per frame, poc_fre(t, time_poc)
 * (tineuvox.py:872-878), PointWarper.forward's pose part (pointwarper.py:213-239) and, with
 * n_views > 0, project_point_to_image_plane(joints_rel + global_t, c2w, K) (temporalpoints.py:578-583,
 * utils.py:435-450)). As apn_skeleton_pose, except: t path = t [1] (device) with the time
 * embedding [t, sin(t f), cos(t f)] of the n_freq frequencies time_poc computed in the kernel
 * (t_dim = 1 + 2 n_freq); c2w [n_views,4,4], K [n_views,3,3] -> joints2d_out [n_views,J,2]
 * (n_views <= 16, n_views * J <= 1024; 0 = no projection). sweep_index (rot path, optional, device
 * int32): rot_params holds sweep_len poses [sweep_len, J, rot_dim]; the launch takes pose
 * *sweep_index % sweep_len and advances *sweep_index (the repose sweep of run.py:1355-1396 as a
 * captured graph without a per-pose input copy); NULL = rot_params is one pose. */
int apn_skeleton_frame(const float* t, const float* time_poc, int32_t n_freq, const float* rot_params,
                       int32_t rot_dim, int32_t n_joints, const float* tn_weights, int32_t hidden, int32_t n_layers,
                       const float* joints, const int32_t* parent_indices, int32_t depth,
                       const int32_t* parent_joint_ex, const int32_t* sibling_mask, const int32_t* rot_mask,
                       float* params_out, float* thetas_out, float* bone_T16, float* bone_T34,
                       float* global_t_out, float* joints_rel_out, const int32_t* chain_prog,
                       const float* c2w, const float* K, int32_t n_views, float* joints2d_out,
                       int32_t* sweep_index, int32_t sweep_len, void* stream);

/* Every pose of a repose sweep (run.py:1355-1396) in one launch: rot_params [n_poses, J, rot_dim]
 * -> per-pose thetas [n_poses, J], bone_T16 [n_poses, J, 16], bone_T34 [n_poses, J, 12], global_t
 * [n_poses, 3] (zeros: the rot path), joints_rel [n_poses, J, 3]; each pose exactly as
 * apn_skeleton_pose computes it (pointwarper.py:213-239, one workgroup per pose). */
int apn_skeleton_sweep(const float* rot_params, int32_t n_poses, int32_t rot_dim, int32_t n_joints,
                       const float* joints, const int32_t* parent_indices, int32_t depth,
                       const int32_t* parent_joint_ex, const int32_t* sibling_mask, const int32_t* rot_mask,
                       float* thetas_out, float* bone_T16, float* bone_T34, float* global_t_out,
                       float* joints_rel_out, const int32_t* chain_prog, void* stream);

/* Padded sampling bbox = bbox_ord -/+ query_radius (temporalpoints.py:424) as 6 floats. */
int apn_bbox_unpack(const int32_t* bbox_ord, float query_radius, float* out6, void* stream);

/* The rays of a ray shard (shard.py "blocks" split): rows index[0..n) of rays_o, rays_d and
 * viewdirs [R,3] gathered into out_o, out_d, out_v [n,3] in one launch (replaces three
 * index_select calls of the render loop, run.py:136-151 slicing). index: int64, in [0, R). */
int apn_gather_rays(const float* rays_o, const float* rays_d, const float* viewdirs, const int64_t* index,
                    int64_t n, float* out_o, float* out_d, float* out_v, void* stream);

/* In-bbox ray samples (sample_ray, temporalpoints.py:373-399, with the boolean compaction
 * done on device): per-ray counts -> offsets [n_rays+1]; then q_pos4 {x,y,z,bits(step)},
 * q_ray, sorted by (ray, step). bbox6 = {lo xyz, hi xyz} (device).
 * Workspace: apn_sample_pts_on_rays_workspace_bytes. */
int apn_inbbox_count(const float* rays_o, const float* rays_d, const float* bbox6, float near,
                     float far, float stepdist, int64_t n_rays, int32_t* offsets, void* workspace,
                     void* stream);
int apn_inbbox_fill(const float* rays_o, const float* rays_d, const float* bbox6, float near,
                    float far, float stepdist, int64_t n_rays, const int32_t* offsets,
                    float* q_pos4, int32_t* q_ray, void* stream);
/* apn_inbbox_fill with buffers sized `capacity` on the host: samples at positions >= capacity are
 * dropped, and frame_info[3] (device) = {min(total, capacity), total, total > capacity}. Element
 * 0 is the live query count apn_knn_radius reads on the device (n_queries = capacity), so the
 * frame needs no device->host read of the sample count; an overflowed frame is recomputed by the
 * caller (TemporalPoints: RenderOutput validation). */
int apn_inbbox_fill_capped(const float* rays_o, const float* rays_d, const float* bbox6, float near,
                           float far, float stepdist, int64_t n_rays, const int32_t* offsets,
                           int64_t capacity, float* q_pos4, int32_t* q_ray, int32_t* frame_info,
                           void* stream);

/* Uniform grid over the warped cloud (cell >= sqrt(query_radius)): counting sort into
 * sorted_pts4 [N,4] {x,y,z,bits(idx)}. cell_cap bounds the number of cells. The ball scans
 * address the cloud with 32-bit byte offsets: n_points > 2^27 - 1 is APN_ERR_ARG here and in
 * apn_knn_radius. */
size_t apn_grid_workspace_bytes(int64_t n_points, int32_t cell_cap);
int apn_grid_build(const float* xyz, int64_t n_points, const int32_t* bbox_ord, float query_radius,
                   int32_t cell_cap, float* sorted_pts4, void* workspace, void* stream);

/* Radius-bounded exact kNN (K=8), replacing pykeops Kmin_argKmin + the radius filter
 * (temporalpoints.py:433-447): survivors (8th-NN squared distance <= query_radius) in
 * query order -> s_pos4, s_ray, s_nbr [S,8]; S written to *n_survivors_dev. */
size_t apn_knn_workspace_bytes(int64_t n_queries);

/* The kNN's second (anisotropic) grid, built from the fine grid of apn_grid_build. Launches of more
 * than 2^18 queries read it (apn_knn_uses_agrid(n_queries) = 1); apn_knn_radius builds it itself.
 * apn_knn_agrid_build lets the host build it on another stream (beside the sampling and the kNN's
 * first passes) and apn_knn_radius_ev then waits on agrid_ready (a hipEvent_t recorded after that
 * build) right before the first pass that reads it. Same results as apn_knn_radius. */
int32_t apn_knn_uses_agrid(int64_t n_queries);
int apn_knn_agrid_build(const void* grid_workspace, int64_t n_points, int32_t cell_cap, const float* sorted_pts4,
                        void* stream);
int apn_knn_radius_ev(const float* q_pos4, const int32_t* q_ray, int64_t n_queries,
                      const int32_t* n_queries_dev, const void* grid_workspace, int64_t n_points,
                      int32_t cell_cap, const float* sorted_pts4, float query_radius, float* s_pos4,
                      int32_t* s_ray, int32_t* s_nbr, int32_t* n_survivors_dev, void* workspace,
                      void* agrid_ready, void* stream);
int apn_knn_radius(const float* q_pos4, const int32_t* q_ray, int64_t n_queries,
                   const int32_t* n_queries_dev, const void* grid_workspace, int64_t n_points,
                   int32_t cell_cap, const float* sorted_pts4, float query_radius, float* s_pos4,
                   int32_t* s_ray, int32_t* s_nbr, int32_t* n_survivors_dev, void* workspace,
                   void* stream);


/* mean_min_distance support (temporalpoints.py:104-111): per-point sqrt(d2_nn + eps) to the
 * nearest other point. Uses grid_workspace/sorted_pts4/bbox_ord as scratch. */
int apn_nn1_distance(const float* xyz, int64_t n_points, float eps, int32_t cell_cap, float* nn_dist,
                     float* sorted_pts4, int32_t* bbox_ord, void* grid_workspace, void* stream);

/* Unbounded K nearest neighbours (K <= 16) of queries q [n_queries,3] in pts [n_points,3] -- the
 * pykeops `LazyTensor` argKmin of the training losses (temporalpoints.py:104-111, 737-748, 777-780)
 * and of nn_i / nn_distance: grid over pts (scratch sorted_pts4 [n_points,4], bbox_ord [8],
 * grid_workspace of apn_grid_workspace_bytes(n_points, cell_cap)), ring search with an exact stop
 * rule, full scan for queries still open after 64 rings. Small sets (n_points <= 16384 and
 * n_queries * n_points <= 2^27: the chamfer losses) skip the grid and scan all points through LDS
 * tiles (the scratch buffers are then untouched). idx_out / d2_out [n_queries,k], ascending
 * squared distance, ties by index (pykeops leaves their order unspecified). */
int apn_knn_points(const float* q, int64_t n_queries, const float* pts, int64_t n_points, int32_t k,
                   int32_t cell_cap, float* sorted_pts4, int32_t* bbox_ord, void* grid_workspace,
                   int64_t* idx_out, float* d2_out, void* stream);

/* Packed MLP weight layout: writes 20 int32 offsets (W1E,B1,W2,B2,W3,B3,W4,B4,WD,BD,WH,BH,
 * WV2,BV2,W1F,TOTAL,KE,KV,H16,FLAG) and returns their count (float offsets; TOTAL = buffer
 * length). W1E = feat_net.0 columns 0..62 (posenc), W1F = feat_net.0 columns 63..190 (features),
 * WH/BH = rgbnet feature_linears folded into views_linears.0 (no activation between them),
 * see apn_mlp.hip; H16 = start of the fp16 hi/lo fragment region (apn_mlp_layout.h); FLAG = the
 * int32 range flag of the split kernel (non-zero: an out-of-fp16-range value was met and the
 * launch was recomputed on FP32 MFMA; cleared by apn_mlp_split_weights). */
int apn_mlp_weight_layout(int32_t* offsets);

/* Fill the fp16 hi/lo fragment region of a packed weight buffer from its fp32 region
 * (hi = fp16(w), lo = fp16(w - hi), MFMA fragment order) and clear its range flag. Call after
 * every change of the fp32 region and before apn_point_mlp with the default (split) kernel. */
int apn_mlp_split_weights(float* wbuf, void* stream);

/* Refresh only the layer-1 bias inside the fp16 fragment region (the split kernels take b1 as the
 * weights of a constant-1 input column) from the fp32 b1 of wbuf -- after a per-frame fold of the
 * pose embedding into b1 (temporalpoints.py:487-488). Sets the range flag if the scaled bias leaves
 * the fp16 range. */
int apn_mlp_split_bias(float* wbuf, void* stream);

/* Per-point layer-1 feature projection proj [N,128] = canonical_feat [N,128] x W1F^T
 * (temporalpoints.py:483-491 reassociated: W1 [emb; feat] = W1e emb + W1f feat). Computed once
 * per model; feat_dim must be 128. */
int apn_feat_project(const float* canonical_feat, int64_t n_points, int32_t feat_dim,
                     const float* wbuf, float* proj, void* stream);

/* Fused neighbour MLP + heads + direct blend (temporalpoints.py:452-519) for the kept
 * samples; out12 [S,12] = {r,g,b,alpha, r_d,g_d,b_d,alpha_d, wr,wg,wb,0}. feat_proj is the
 * apn_feat_project output (feat_dim 128). vemb_const [27] (frozen_view_dir) or NULL to embed
 * viewdirs[ray]. Default kernel: fp32 contraction as 3 fp16 MFMA terms (hi*hi + hi*lo + lo*hi,
 * fp32 accumulate; wbuf prepared by apn_mlp_split_weights), followed by an FP32-MFMA launch that
 * recomputes every sample only if the split kernel set the range flag (a weight or activation
 * beyond the fp16 range; see FLAG above) -- decided on the device, no host sync; variant 1 = the
 * FP32-MFMA kernel alone. */
int apn_point_mlp(const float* s_pos4, const int32_t* s_ray, const int32_t* s_nbr,
                  int64_t max_samples, const int32_t* n_samples_dev, const float* recA16,
                  const float* recB8, const float* feat_proj, int32_t feat_dim,
                  const float* viewdirs, const float* vemb_const, const float* wbuf, float eps,
                  float act_shift, float interval, int32_t grid_blocks, float* out12, void* stream);

/* apn_point_mlp with exact early ray termination (the render path's default; replaces the same
 * stage, temporalpoints.py:452-519, followed by the compositing's break at T < 1e-3,
 * render_utils_kernel.cu:445-451, as apn_composite applies it). The {rgb, alpha} columns are
 * computed only for the kept samples the compositing reads: the MLP runs in 9 passes over each
 * ray's kept samples in step order (two at a time up to local index 12, then [12,16) [16,24) [24,..)),
 * and after each pass a per-ray walk with apn_composite's arithmetic (fast_color_thres pre-mask,
 * T in double) retires the rays that terminated. The direct-path and weight-colour columns are
 * computed for every kept sample (with_direct = 1; 0: by the caller's apn_direct_blend). apn_composite
 * on the result gives exactly apn_point_mlp's frame.
 * Survivors must be sorted by ray (apn_knn_radius's order); n_rays bounds their ray ids.
 * workspace: apn_point_mlp_ert_workspace_bytes(max_samples, n_rays). pass_rows (optional, device
 * int32 [9]): the samples each pass ran the MLP on. pass_events (optional, eager calls only):
 * 18 hipEvent_t recorded on `stream` right before / after each pass's MLP launches. */
size_t apn_point_mlp_ert_workspace_bytes(int64_t max_samples, int64_t n_rays);
int apn_point_mlp_ert(const float* s_pos4, const int32_t* s_ray, const int32_t* s_nbr,
                      int64_t max_samples, const int32_t* n_samples_dev, int64_t n_rays,
                      const float* recA16, const float* recB8, const float* feat_proj, int32_t feat_dim,
                      const float* viewdirs, const float* vemb_const, const float* wbuf, float eps,
                      float act_shift, float interval, float fast_color_thres, int32_t with_direct,
                      float* out12, void* workspace, int32_t* pass_rows, void* const* pass_events,
                      void* stream);
/* The direct-path / weight-colour columns 4..11 of out12 (temporalpoints.py:459-470, 517-519) for
 * every kept sample, with the fused MLP kernel's arithmetic: what apn_point_mlp_ert computes first
 * when with_direct = 1; with 0 the caller runs this instead (TemporalPoints: on a second stream,
 * beside the MLP passes; both must finish before apn_composite). */
int apn_direct_blend(const float* s_pos4, const int32_t* s_nbr, int64_t max_samples,
                     const int32_t* n_samples_dev, const float* recA16, const float* recB8, float eps,
                     float* out12, void* stream);

/* Select the apn_point_mlp kernel (process-wide, default 0): 0 = 3-term fp16-split MFMA with the
 * FP32 range fallback, 1 = FP32 MFMA alone. (The debug build, include/apn_hip_debug.h, also takes
 * 2 / 3 = phase-timed builds of 1 / 0 and an initial value from env APN_MLP_VARIANT.) Returns the
 * previous selection; out-of-range values only query it. */
int apn_set_mlp_variant(int32_t variant);

/* Masks + Alphas2Weights + segment sums for both paths (temporalpoints.py:611-710).
 * ray_ws: 2*n_rays int32 scratch. */
int apn_composite(const float* smp12, const float* s_pos4, const int32_t* s_ray,
                  int64_t max_samples, const int32_t* n_samples_dev, int64_t n_rays,
                  float fast_color_thres, float bg, float* rgb_marched, float* rgb_marched_direct,
                  float* depth, float* weights_vis, float* alphainv_last,
                  float* alphainv_last_direct, int32_t* ray_ws, void* stream);


/* ---------------------------------------------------------------------------------------------
 * TiNeuVox stage 1: the voxel model the point cloud is exported from
 * (lib/tineuvox.py:91-625). voxel_dim must be 12, net_width 128, posbase_pe 10, viewbase_pe 4,
 * gridbase_pe 2 (the reference configuration); the deformation depth is a parameter.
 * ------------------------------------------------------------------------------------------- */

/* Bytes of the repacked 3-scale feature grid for a [1, C, X, Y, Z] feature (C must be 12), or -1. */
int64_t apn_tnv_grid_bytes(int32_t C, int32_t X, int32_t Y, int32_t Z);

/* feature [C][X][Y][Z] fp32 (TiNeuVox.feature) -> channels-last grids of the zero-padded feature
 * at scales 1, 1/2, 1/4 (tineuvox.py:402-411: F.pad to (size-1) % 4 == 0, views [::2], [::4]). */
int apn_tnv_grid_pack(const float* feature, int32_t C, int32_t X, int32_t Y, int32_t Z, float* grid,
                      void* stream);

/* TiNeuVox.mult_dist_interp (tineuvox.py:402-419, grid_sampler 379-394): trilinear
 * grid_sample (align_corners=True, zero padding) of the three scales at pts [n,3] ->
 * out [n,36] = [scale 1 | 1/2 | 1/4] x 12 channels. xyz_min/xyz_max: device [3]. */
int apn_tnv_mult_dist_interp(const float* pts, int64_t n_pts, const float* grid, int32_t X, int32_t Y,
                             int32_t Z, const float* xyz_min, const float* xyz_max, float* out, void* stream);

/* Packed TiNeuVox network layout for a deformation depth: writes 14 int32 (float offsets
 * D0E, DH, DOUT, FW, WD, BD, WH, BH, WV2, BV2, TOTAL, then KE, KF, KV) and returns the count. */
int apn_tnv_weight_layout(int32_t defor_depth, int32_t* offsets);

/* The TiNeuVox field at query points (tineuvox.py:479-532; get_grid_as_point_cloud 286-342):
 * posenc -> Deformation (if deform; tineuvox.py:28-62) -> 3-scale trilinear grid sample ->
 * posenc -> featurenet -> densitynet + raw2alpha, and rgbnet + sigmoid.
 * pos4 [S,4] {x,y,z,*}, s_ray [S] (index into time_idx / viewdirs), time_idx [R] (row of tproj
 * per ray; NULL = row 0), tproj [U,256] per-time projections (time columns of deformation
 * layer 0 and of featurenet applied to timenet(poc_fre(t)), plus their biases), viewdirs [R,3] or
 * vemb_const [27]. out12 [S,12] = {r,g,b,alpha, 0...} (the apn_composite layout); optional
 * delta_out [S,3] (deformed positions), h_out [S,128], vox_out [S,36]. The sample count is read
 * on the device (n_samples_dev <= max_samples). */
int apn_tnv_field(const float* pos4, const int32_t* s_ray, const int32_t* time_idx, int64_t max_samples,
                  const int32_t* n_samples_dev, const float* grid, int32_t X, int32_t Y, int32_t Z,
                  const float* xyz_min, const float* xyz_max, const float* wbuf, int32_t defor_depth,
                  const float* tproj, const float* viewdirs, const float* vemb_const, int32_t deform,
                  float act_shift, float interval, float* out12, float* delta_out, float* h_out,
                  float* vox_out, void* stream);

/* fp32 GEMMs of the training step (forward and backward of the Linear layers that the reference
 * trains through autograd: feat_net, densitynet, rgbnet, TransformNet, pose_embedding_net --
 * temporalpoints.py:491-515, pointwarper.py:5-37, run.py:574-716), on the f32-input MFMA (exact
 * f32 products and sums in the kernel's order):
 *   C[m][n] = epi( sum_k opA[m][k] opB[k][n] ),  opA = A (M x K, lda) or A^T (trans_a: A is K x M),
 *   opB = B (K x N, ldb) or B^T (trans_b: B is N x K);
 *   A2 (optional, same layout as A): opA *= (A2 > 0 ? 1 : slope_mask) -- a LeakyReLU derivative
 *   taken from the layer's output; epi: + bias[n] (optional), LeakyReLU(slope_act) when act. */
int apn_gemm_f32(const float* A, const float* A2, const float* B, float* C, const float* bias, int64_t M,
                 int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int32_t trans_a, int32_t trans_b,
                 float slope_mask, int32_t act, float slope_act, void* stream);
/* The same product with the reduction dimension K split over `splits` workgroup slices (weight
 * gradients: K = the rows of a batch), partial products summed in a fixed order: C [M, N]
 * (ldc = N); bias_grad (optional) [M] = sum_k opA[m][k] (the bias gradient, computed as one more
 * column of ones in opB). workspace: apn_gemm_f32_splitk_workspace_bytes(M, N, splits). */
size_t apn_gemm_f32_splitk_workspace_bytes(int64_t M, int64_t N, int32_t splits);
int apn_gemm_f32_splitk(const float* A, const float* A2, const float* B, float* C, float* bias_grad, int64_t M,
                        int64_t N, int64_t K, int64_t lda, int64_t ldb, int32_t trans_a, int32_t trans_b,
                        float slope_mask, int32_t splits, void* workspace, void* stream);

/* The training forward's neighbour aggregation (temporalpoints.py:452-494 under autograd,
 * run.py:574-716): per MLP row (sample s, neighbour k = s_i[s,k]) the IDW weight w [S,8], the
 * direct blend rgb_d [S,3] / alpha_d [S] (459-470), and the feat_net input row
 * feat_in[8s+k] = [rel_c | sin(rel_c f) | cos(rel_c f) | 0 pad to a multiple of 4 | canonical_feat[n]
 * | pose_emb] (L <= 16 pos frequencies poc[L], row stride ldf); sig = mean_min_distance *
 * max(direct_eps, 0), rgb_c / alpha_c the clipped canonical colours. */
int apn_nbr_train_fwd(int64_t S, const float* ray_pts, const int64_t* s_i, const float* xyz, const float* Rinv,
                      const float* canonical_feat, int32_t F, const float* pose_emb, int32_t P, const float* sig,
                      const float* rgb_c, const float* alpha_c, const float* poc, int32_t L, float eps, float* w_out,
                      float* rgbd, float* alphad, float* feat_in, int64_t ldf, void* stream);
/* Its backward: from d_w [S,8], d_rgbd [S,3], d_alphad [S], d_feat [8S, ldd] (any may be NULL)
 * the per-point gradients d_xyz [N,3], d_R [N,9], d_sig [N], d_c [N,3], d_a [N] and d_featp [N,F]
 * (canonical_feat), summed over each point's rows in the order of the reverse adjacency
 * rev_ptr [N+1] / rev_edge [8S] (deterministic); contrib: workspace [8S, 17]. */
int apn_nbr_train_bwd(int64_t S, int64_t N, const float* ray_pts, const int64_t* s_i, const float* xyz,
                      const float* Rinv, const float* sig, const float* rgb_c, const float* alpha_c, const float* poc,
                      int32_t L, float eps, const float* d_w, const float* d_rgbd, const float* d_alphad,
                      const float* d_feat, int64_t ldd, int32_t F, const int64_t* rev_ptr, const int64_t* rev_edge,
                      float* contrib, float* d_xyz, float* d_R, float* d_sig, float* d_c, float* d_a, float* d_featp,
                      void* stream);
/* h [S,C] = sum_k w[s,k] out[8s+k, :] (temporalpoints.py:493-494) and its backward
 * (d_out = w d_h, d_w[s,k] = <out[8s+k], d_h[s]>). */
int apn_idw_sum_fwd(int64_t S, int32_t C, const float* w, const float* out, float* h, void* stream);
int apn_idw_sum_bwd(int64_t S, int32_t C, const float* w, const float* out, const float* dh, float* d_out, float* d_w,
                    void* stream);
/* Bounding box of a cloud xyz [N,3]: out6 = {min, max} (exact), ord8 (optional) = its
 * order-preserving int32 encoding (the grid kernels' bbox_ord); workspace >= 1024 * 6 floats.
 * (temporalpoints.py:423-427 min/max of the warped cloud.) */
int apn_cloud_bbox(const float* xyz, int64_t N, float* out6, int32_t* ord8, void* workspace, void* stream);

/* Utilities */
size_t apn_scan_workspace_bytes(int64_t n);
int apn_scan_exclusive_i32(const int32_t* in, int32_t* out, int64_t n, void* workspace, void* stream);
const char* apn_version(void);

#ifdef __cplusplus
}
#endif
#endif /* APN_HIP_H */
