"""TEST INFRASTRUCTURE ONLY (tests/ and bench.py's cpu_baseline leg). Explained flips: the reference's compositing has three discontinuities, and a ray whose oracle
values sit on one of them may legitimately differ from the oracle by more than the fp tolerance
when an input moves by an ulp:

* the pre-mask ``alpha > fast_color_thres`` (temporalpoints.py:611-626);
* the post-mask ``weights > fast_color_thres`` (temporalpoints.py:634-651);
* the early exit ``T < 1e-3`` of alpha2weight (render_utils_kernel.cu:445-451), where the
  crossing sample is still written and every later one is dropped;
* (only when the two sides render different warped clouds) the kNN radius test
  ``to_nn[:, -1] <= query_radius`` (temporalpoints.py:439-447).

``assert_flips_explained`` requires every ray whose error exceeds ``cap`` to have an oracle
sample within ``tol`` of one of them, so no arithmetic error can hide behind a budget."""
from __future__ import annotations

import numpy as np

from oracle import apn_oracle as O

F32 = np.float32
PATH_OF_KEY = {"rgb_marched": "nerf", "depth": "nerf", "weights": "nerf", "alphainv_last": "nerf",
               "rgb_marched_direct": "direct", "alphainv_last_direct": "direct"}


def near_discontinuity(trace, n_rays, path, thr=1e-4, tol=1e-6, t_stop=1e-3):
    """bool [n_rays]: the oracle's compositing of the ray has an alpha or weight within ``tol`` of
    ``thr`` or a transmittance within ``tol`` of ``t_stop``. ``trace`` = OracleModel.trace after a
    forward (kept samples: 'alpha' / 'alpha_direct' and 'ray_id', sorted by ray)."""
    a = np.asarray(trace["alpha" if path == "nerf" else "alpha_direct"], dtype=F32).reshape(-1)
    rid = np.asarray(trace["ray_id"], dtype=np.int64).reshape(-1)
    near = np.zeros(n_rays, bool)
    np.logical_or.at(near, rid, np.abs(a.astype(np.float64) - thr) <= tol)
    m = a > F32(thr)
    a2, r2 = a[m], rid[m]
    if len(a2):
        w, T, last, i_s, i_e = O.alpha2weight(a2, r2, n_rays)
        written = np.zeros(len(a2), bool)   # samples alpha2weight processed (up to and incl. the break)
        for r in np.unique(r2):
            written[int(i_s[r]):int(i_e[r])] = True
        t_after = T.astype(np.float64) * (1.0 - a2.astype(np.float64))
        hit = written & ((np.abs(w.astype(np.float64) - thr) <= tol) | (np.abs(t_after - t_stop) <= tol))
        np.logical_or.at(near, r2, hit)
    return near


def ray_errors(a, b):
    a = np.asarray(a, np.float64).reshape(len(a), -1)
    b = np.asarray(b, np.float64).reshape(len(b), -1)
    return np.abs(a - b).max(1)


def assert_flips_explained(key, got, ref, trace, cap=1e-5, tol=1e-6, thr=1e-4, knn=None, query_radius=0.01):
    """Every ray with |got - ref| > cap must sit on a discontinuity (near_discontinuity).
    ``cap`` applies to colours/transmittances; depth (step units) uses cap x (max|ref| + 1).
    ``knn`` = (d8 [S_bbox] 8th-NN squared distance of every in-bbox sample, its ray id) adds the
    radius test as a discontinuity (for renders of two different warped clouds)."""
    got, ref = np.asarray(got), np.asarray(ref)
    R = len(ref)
    err = ray_errors(got, ref)
    if key == "depth":
        cap = cap * (float(np.abs(ref).max()) + 1.0)
    near = near_discontinuity(trace, R, PATH_OF_KEY[key], thr=thr, tol=tol)
    if knn is not None:
        d8, krid = (np.asarray(x) for x in knn)
        np.logical_or.at(near, krid.astype(np.int64), np.abs(d8.astype(np.float64) - query_radius) <= tol)
    bad = err > cap
    unexplained = np.nonzero(bad & ~near)[0]
    msg = (f"{key}: {int(bad.sum())} rays over {cap:.1e} ({int((bad & near).sum())} explained); "
           f"unexplained {unexplained[:10].tolist()} err {err[unexplained[:10]].tolist()}; "
           f"max err {float(err.max()):.2e}")
    print(msg)
    assert len(unexplained) == 0, msg
    return int(bad.sum()), float(err[~near].max()) if (~near).any() else 0.0
