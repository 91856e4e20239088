"""ctypes binding of libapn_hip.so (C-ABI declared in include/apn_hip.h).

The product path has no CPU fallback: importing an op that needs the library raises
``RuntimeError`` when libapn_hip.so is missing or cannot be loaded, and every C call that
returns a non-zero status raises as well.
"""
from __future__ import annotations

import contextlib
import ctypes as C
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("APN_HIP_LIB", os.path.join(_HERE, "libapn_hip.so"))

P = C.c_void_p
I64 = C.c_int64
I32 = C.c_int32
F32 = C.c_float
SZ = C.c_size_t

# name -> (restype, argtypes); must match include/apn_hip.h
SIGNATURES = {
    "apn_sample_pts_on_rays_workspace_bytes": (SZ, [I64]),
    "apn_sample_pts_on_rays_count": (C.c_int, [P, P, P, P, F32, F32, F32, I64, P, P, P, P, P, P]),
    "apn_sample_pts_on_rays_fill": (C.c_int, [P, P, P, P, F32, F32, F32, I64, P, P, P, P, P, P]),
    "apn_raw2alpha": (C.c_int, [P, F32, F32, I64, P, P, P]),
    "apn_alpha2weight": (C.c_int, [P, P, I64, I64, P, P, P, P, P, P]),
    "apn_raw2alpha_backward": (C.c_int, [P, P, F32, I64, P, P]),
    "apn_alpha2weight_backward": (C.c_int, [P, P, P, P, P, P, I64, I64, P, P, P, P]),
    "apn_segment_sum": (C.c_int, [P, P, I64, I64, I64, P, P, P]),
    "apn_lbs_workspace_bytes": (SZ, [I64]),
    "apn_lbs_skin": (C.c_int, [P, P, I64, I32, P, F32, P, P, P, P, P, P, P, F32, I32, P, P, P, P, P, P, P, P]),
    "apn_skeleton_pose": (C.c_int, [P, I32, P, I32, I32, P, I32, I32, P, P, I32, P, P, P, P, P, P, P, P, P, P, P]),
    "apn_skeleton_frame": (C.c_int, [P, P, I32, P, I32, I32, P, I32, I32, P, P, I32, P, P, P, P, P, P, P, P, P, P,
                                     P, P, I32, P, P, I32, P]),
    "apn_skeleton_sweep": (C.c_int, [P, I32, I32, I32, P, P, I32, P, P, P, P, P, P, P, P, P, P]),
    "apn_bbox_unpack": (C.c_int, [P, F32, P, P]),
    "apn_gather_rays": (C.c_int, [P, P, P, P, I64, P, P, P, P]),
    "apn_inbbox_count": (C.c_int, [P, P, P, F32, F32, F32, I64, P, P, P]),
    "apn_inbbox_fill": (C.c_int, [P, P, P, F32, F32, F32, I64, P, P, P, P]),
    "apn_inbbox_fill_capped": (C.c_int, [P, P, P, F32, F32, F32, I64, P, I64, P, P, P, P]),
    "apn_grid_workspace_bytes": (SZ, [I64, I32]),
    "apn_grid_build": (C.c_int, [P, I64, P, F32, I32, P, P, P]),
    "apn_knn_workspace_bytes": (SZ, [I64]),
    "apn_knn_radius": (C.c_int, [P, P, I64, P, P, I64, I32, P, F32, P, P, P, P, P, P]),
    "apn_knn_uses_agrid": (I32, [I64]),
    "apn_knn_agrid_build": (C.c_int, [P, I64, I32, P, P]),
    "apn_knn_radius_ev": (C.c_int, [P, P, I64, P, P, I64, I32, P, F32, P, P, P, P, P, P, P]),
    "apn_nn1_distance": (C.c_int, [P, I64, F32, I32, P, P, P, P, P]),
    "apn_knn_points": (C.c_int, [P, I64, P, I64, I32, I32, P, P, P, P, P, P]),
    "apn_mlp_weight_layout": (C.c_int, [P]),
    "apn_mlp_split_weights": (C.c_int, [P, P]),
    "apn_mlp_split_bias": (C.c_int, [P, P]),
    "apn_feat_project": (C.c_int, [P, I64, I32, P, P, P]),
    "apn_point_mlp": (C.c_int, [P, P, P, I64, P, P, P, P, I32, P, P, P, F32, F32, F32, I32, P, P]),
    "apn_point_mlp_ert_workspace_bytes": (SZ, [I64, I64]),
    "apn_point_mlp_ert": (C.c_int, [P, P, P, I64, P, I64, P, P, P, I32, P, P, P, F32, F32, F32, F32, I32, P, P, P, P,
                                    P]),
    "apn_direct_blend": (C.c_int, [P, P, I64, P, P, P, F32, P, P]),
    "apn_composite": (C.c_int, [P, P, P, I64, P, I64, F32, F32, P, P, P, P, P, P, P, P]),
    "apn_set_mlp_variant": (C.c_int, [I32]),
    "apn_adam_upd": (C.c_int, [P, P, P, P, I64, I32, F32, F32, F32, F32, P]),
    "apn_masked_adam_upd": (C.c_int, [P, P, P, P, I64, I32, F32, F32, F32, F32, P]),
    "apn_adam_upd_with_perlr": (C.c_int, [P, P, P, P, P, I64, I32, F32, F32, F32, F32, P]),
    "apn_total_variation_add_grad": (C.c_int, [P, P, F32, F32, F32, I64, I64, I64, I64, I32, P]),
    "apn_lbs_train_workspace_bytes": (SZ, [I64, I32]),
    "apn_lbs_train_fwd": (C.c_int, [P, P, I64, I32, P, F32, P, P, P, P, P, P, P]),
    "apn_lbs_train_bwd": (C.c_int, [P, P, I64, I32, P, F32, P, P, P, P, P, P, P, P, P, P, P, P]),
    "apn_nbr_loss_workspace_bytes": (SZ, []),
    "apn_nbr_tv_loss": (C.c_int, [P, I64, I32, P, I32, P, P, P]),
    "apn_nbr_tv_loss_backward": (C.c_int, [P, I64, I32, P, I32, P, P, P, P, P]),
    "apn_arap_loss": (C.c_int, [P, I64, P, I32, P, F32, P, P, P]),
    "apn_arap_loss_backward": (C.c_int, [P, I64, P, I32, P, F32, P, P, P, P, P]),
    "apn_weight_sparsity_loss": (C.c_int, [P, I64, F32, P, P, P]),
    "apn_weight_sparsity_loss_backward": (C.c_int, [P, I64, F32, P, P, P]),
    "apn_tnv_grid_bytes": (I64, [I32, I32, I32, I32]),
    "apn_tnv_grid_pack": (C.c_int, [P, I32, I32, I32, I32, P, P]),
    "apn_tnv_mult_dist_interp": (C.c_int, [P, I64, P, I32, I32, I32, P, P, P, P]),
    "apn_tnv_weight_layout": (C.c_int, [I32, P]),
    "apn_tnv_field": (C.c_int, [P, P, P, I64, P, P, I32, I32, I32, P, P, P, I32, P, P, P, I32, F32, F32, P, P, P,
                                P, P]),
    "apn_scan_workspace_bytes": (SZ, [I64]),
    "apn_scan_exclusive_i32": (C.c_int, [P, P, I64, P, P]),
    "apn_version": (C.c_char_p, []),
    "apn_adam_multi": (C.c_int, [I32, P, P, P, P, P, P, P, P, P, P, P, P]),
    "apn_gemm_f32": (C.c_int, [P, P, P, P, P, I64, I64, I64, I64, I64, I64, I32, I32, F32, I32, F32, P]),
    "apn_gemm_f32_splitk_workspace_bytes": (SZ, [I64, I64, I32]),
    "apn_nbr_train_fwd": (C.c_int, [I64, P, P, P, P, P, I32, P, I32, P, P, P, P, I32, F32, P, P, P, P, I64, P]),
    "apn_nbr_train_bwd": (C.c_int, [I64, I64, P, P, P, P, P, P, P, P, I32, F32, P, P, P, P, I64, I32, P, P, P, P, P,
                                    P, P, P, P, P]),
    "apn_cloud_bbox": (C.c_int, [P, I64, P, P, P, P]),
    "apn_idw_sum_fwd": (C.c_int, [I64, I32, P, P, P, P]),
    "apn_idw_sum_bwd": (C.c_int, [I64, I32, P, P, P, P, P, P]),
    "apn_gemm_f32_splitk": (C.c_int, [P, P, P, P, P, I64, I64, I64, I64, I64, I32, I32, F32, I32, P, P]),
}

# debug-build-only exports (include/apn_hip_debug.h; libapn_hip_debug.so)
DEBUG_SIGNATURES = {
    "apn_set_knn_mode": (C.c_int, [I32]),
    "apn_debug_knn_stats": (C.c_int, [P]),
    "apn_debug_mlp_phase_cycles": (C.c_int, [P]),
}
DEBUG_LIB_PATH = os.path.join(_HERE, "libapn_hip_debug.so")

_lib = None
_load_error = None
_debug_lib = None


def load():
    """Load libapn_hip.so once; raise RuntimeError (no fallback) if it is unavailable."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if _load_error is not None:
        raise RuntimeError(_load_error)
    if not os.path.exists(LIB_PATH):
        _load_error = (f"libapn_hip.so not found at {LIB_PATH}; build it with "
                       f"`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)")
        raise RuntimeError(_load_error)
    try:
        lib = C.CDLL(LIB_PATH)
    except OSError as e:  # pragma: no cover
        _load_error = f"failed to load {LIB_PATH}: {e}"
        raise RuntimeError(_load_error)
    ab_build = "APN_HIP_LIB" in os.environ   # an A/B build of an earlier revision (tools/)
    for name, (res, args) in SIGNATURES.items():
        if ab_build and not hasattr(lib, name):
            continue   # an entry point the earlier revision did not have (its callers skip it)
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    for name, (res, args) in DEBUG_SIGNATURES.items():   # APN_HIP_LIB = the debug build (tools/)
        if hasattr(lib, name):
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
    _lib = lib
    return lib


def load_debug():
    """The debug build (libapn_hip_debug.so: earlier kNN strategies, environment A/B switches,
    instrumented kernels; include/apn_hip_debug.h), for tools/ and the cross-check tests only. The
    product path never loads it."""
    global _debug_lib
    if _debug_lib is not None:
        return _debug_lib
    if not os.path.exists(DEBUG_LIB_PATH):
        raise RuntimeError(f"libapn_hip_debug.so not found at {DEBUG_LIB_PATH} (make -C csrc debug)")
    lib = C.CDLL(DEBUG_LIB_PATH)
    for name, (res, args) in {**SIGNATURES, **DEBUG_SIGNATURES}.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _debug_lib = lib
    return lib


@contextlib.contextmanager
def using(lib):
    """Route every call of this module through ``lib`` (e.g. load_debug()) inside the block: the
    cross-check tests run the same model code on the debug build's kernels."""
    global _lib
    load()
    prev, _lib = _lib, lib
    try:
        yield lib
    finally:
        _lib = prev


def exported_symbols():
    return list(SIGNATURES)


class APNError(RuntimeError):
    pass


_STATUS = {1: "invalid argument (shape/pointer)", 2: "HIP launch failure"}


def call(name, *args):
    rc = getattr(load(), name)(*args)
    if rc != 0:
        raise APNError(f"{name} failed: {_STATUS.get(rc, rc)}")
    return rc


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return C.c_void_p(t.data_ptr())


def stream_ptr(device=None):
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def require_cuda(*tensors, what="apn op"):
    for t in tensors:
        if t is not None and torch.is_tensor(t) and not t.is_cuda:
            raise RuntimeError(f"{what}: expected a device (HIP) tensor, got {t.device}")
