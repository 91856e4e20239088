"""apn_amd -- MI355X-native articulated-point render/deform path.

Drop-in modules mirroring the reference (lukasuz/Articulated-Point-NeRF):
  * ``TemporalPoints``  (lib/temporalpoints.py)  -- forward / repose / get_weights / sample_ray
  * ``PointWarper``     (lib/pointwarper.py)     -- forward-LBS of the canonical cloud
  * ``render_utils``    (render_utils_cuda)      -- sample_pts_on_rays / raw2alpha / alpha2weight
  * ``tineuvox``        (lib/tineuvox.py)        -- TiNeuVox stage-1 field (HIP), RGBNet, heads
                                                    holder, poc_fre, rays
All compute goes through libapn_hip.so (HIP, gfx950); there is no CPU fallback.
"""
from . import render_utils, synthetic
from .pointwarper import PointWarper, TransformNet
from .temporalpoints import NoPointsException, TemporalPoints
from .tineuvox import Alphas2Weights, Raw2Alpha, RGBNet, TiNeuVox, TiNeuVoxHeads, get_rays_of_a_view, poc_fre

__all__ = ["TemporalPoints", "PointWarper", "TransformNet", "NoPointsException", "TiNeuVox", "TiNeuVoxHeads", "RGBNet",
           "Raw2Alpha", "Alphas2Weights", "poc_fre", "get_rays_of_a_view", "render_utils", "synthetic"]
