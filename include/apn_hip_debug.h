/* Debug-build-only entry points of the apn HIP library.
 *
 * The shipped library (articulated-point-nerf_amd/apn_amd/libapn_hip.so, include/apn_hip.h) runs
 * one search strategy and one kernel per stage and reads no environment variable. The debug
 * build (libapn_hip_debug.so: the same sources with -DAPN_DEBUG_BUILD, `make debug`) adds the
 * earlier exact kNN strategies 0-8 (bit-identity cross-checks in tests/test_hip_parity.py), the
 * environment A/B switches of tools/ (APN_KNN_*, APN_MLP_OCC, APN_COMPOSITE, APN_INBBOX_FILL,
 * APN_LBS_*) and the instrumented kernels behind the profiling aids below. It exports every
 * symbol of apn_hip.h plus these. */
#ifndef APN_HIP_DEBUG_H
#define APN_HIP_DEBUG_H

#include "apn_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Select the apn_knn_radius search strategy (process-wide; initial value from env APN_KNN_MODE,
 * default 9): 0 = expanding balls 2h, 4h, r; 1 = culled Chebyshev rings; 2 = ball 2h, then an
 * r-ball chord-count rejection bound, then balls 4h, r with nearest-first rows; 3 = 2 with
 * per-class counters (profiling aid); 4 = the mode-2 search split into two passes (2h ball +
 * chord count for all candidates, balls r/2, r for the rest); 5 = the mode-4 search with the
 * candidates bucketed by 4^3-cell tiles, one workgroup per tile staging the region's cell bounds
 * in LDS; 6 = per-cell rejection bound (points within r of the query's cell box, computed once per
 * occupied cell) + ball r/4, then balls r/2, r for the rest; 7 = 6 with the r/2, r balls as a
 * per-lane state machine (rows and points consumed in lock-step across the wave); 8 = 7 with the
 * cell bound also at r/4 and r/2, so each query starts at its first level that can hold 8 points,
 * and the r/4 ball as a state machine too; 9 = 8 with the r/2 and r balls scanned on a second,
 * anisotropic grid (fine x cells, 2x2 fine cells merged in y and z: ~4x fewer rows per ball; built
 * per call from sorted_pts4 into the grid workspace) and 4 points per scan step (env
 * APN_KNN_ANISO = 1/2/4 merge factor, APN_KNN_PTS = 2/4). All are exact. Returns the previous
 * selection; out-of-range values only query it. */
int apn_set_knn_mode(int32_t mode);

/* Profiling aid (synchronous): {queries, cycles, rows, points} for the mode-3 query classes
 * {stop at 2h, chord-count reject, stop at 4h, stop at r, reject at r}; with env APN_KNN_STATS
 * set, modes 8 and 9 fill [10*l .. 10*l+8] per hard list l instead: {queries, done at r/2, survivors,
 * r/2-scan row / point iterations, r-scan row / point iterations, rejected after the full r scan,
 * their iterations}. Resets them. */
int apn_debug_knn_stats(uint64_t* out20);

/* Profiling aid (synchronous): per-phase cycle sums of the timed k_point_mlp variant
 * (variants 2, 3) {gather, layer 1, layers 2-4, epilogue, tiles, kernel cycles}, summed over
 * workgroups since the last call; resets them. */
int apn_debug_mlp_phase_cycles(uint64_t* out6);

#ifdef __cplusplus
}
#endif

#endif /* APN_HIP_DEBUG_H */
