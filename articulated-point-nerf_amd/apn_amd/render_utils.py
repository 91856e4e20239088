"""Drop-in for the reference's JIT-built ``render_utils_cuda`` module
(lib/cuda/render_utils.cpp:144-155): same function names, arguments and tuple returns.

    import apn_amd.render_utils as render_utils_cuda
"""
from .ops import (Alphas2Weights, Raw2Alpha, alpha2weight, alpha2weight_backward, raw2alpha,  # noqa: F401
                  raw2alpha_backward, sample_pts_on_rays, segment_coo_sum)

__all__ = ["sample_pts_on_rays", "raw2alpha", "raw2alpha_backward", "alpha2weight", "alpha2weight_backward",
           "segment_coo_sum", "Raw2Alpha", "Alphas2Weights"]
