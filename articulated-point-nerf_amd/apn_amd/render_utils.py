"""Drop-in for the reference's JIT-built ``render_utils_cuda`` module
(lib/cuda/render_utils.cpp:144-155): same function names, arguments and tuple returns.

    import apn_amd.render_utils as render_utils_cuda
"""
from .ops import alpha2weight, raw2alpha, sample_pts_on_rays, segment_coo_sum  # noqa: F401

__all__ = ["sample_pts_on_rays", "raw2alpha", "alpha2weight", "segment_coo_sum"]
