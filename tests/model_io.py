"""Build the product TemporalPoints from a golden fixture's constructor inputs + state."""
from __future__ import annotations

import torch

from apn_amd.temporalpoints import TemporalPoints
from apn_amd.tineuvox import TiNeuVoxHeads


def model_from_golden(g, device="cuda"):
    st = g.state()
    lo, hi = st["xyz_min"].numpy(), st["xyz_max"].numpy()
    heads = TiNeuVoxHeads(lo, hi, num_voxels=12 ** 3, num_voxels_base=12 ** 3, net_width=128, alpha_init=1e-3,
                          no_view_dir=False)
    model = TemporalPoints(g.t("in_canonical_pcd"), st["canonical_alpha"], st["canonical_feat"],
                           st["canonical_rgbs"], None, st["joints"], g.bones, lo, hi, heads,
                           stepsize=g.cfg("stepsize"), voxel_size=g.cfg("voxel_size"), fast_color_thres=1e-4,
                           pose_embedding_dim=int(g.cfg("pose_embedding_dim")))
    missing, unexpected = model.load_state_dict(st, strict=False)
    assert not unexpected, unexpected
    return model.to(device)
