"""Debug aid: LBSTrain (HIP) vs get_weights / torch LBS on a golden model."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "articulated-point-nerf_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402
from golden_io import Golden  # noqa: E402
from model_io import model_from_golden  # noqa: E402
from apn_amd.train import lbs_train, lbs_blend, inv3x3  # noqa: E402
from apn_amd.tineuvox import poc_fre  # noqa: E402

g = Golden(sys.argv[1] if len(sys.argv) > 1 else "G1")
m = model_from_golden(g, "cuda")
print("merge rules", m._merge_rules(), "J", m.weights.shape, "theta", m.theta_weight)
t = g.t("in_t").cuda()
bone_Ts, gt, jr = m.forward_warp.pose_torch(m.joints, poc_fre(t, m.time_poc), None)
xyz, Rinv, sm = lbs_train(m, bone_Ts, gt)
w = m.get_weights()
xyz2, G = lbs_blend(m.forward_warp.canonical_pcd, w, bone_Ts, gt)
R2 = inv3x3(G[:, :, :3])
print("sm", float((sm - w).abs().max()), "xyz", float((xyz - xyz2).abs().max()), "Rinv", float((Rinv - R2).abs().max()))
print("sm sum", float(sm.sum(1).min()), float(sm.sum(1).max()), sm.dtype, sm.is_contiguous(), sm.shape)
