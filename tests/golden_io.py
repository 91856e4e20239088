"""Load the golden fixtures written by tests/golden/make_golden.py."""
from __future__ import annotations

import os

import numpy as np
import torch

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = ("G1", "G2", "G3", "G4")


class Golden:
    def __init__(self, name: str):
        self.name = name
        z = np.load(os.path.join(GOLDEN_DIR, f"golden_{name}.npz"))  # allow_pickle=False
        self.z = {k: z[k] for k in z.files}

    def t(self, k, dtype=None):
        v = torch.from_numpy(np.array(self.z[k]))
        if v.dtype == torch.float16:
            v = v.float()
        return v if dtype is None else v.to(dtype)

    def state(self):
        return {k[3:]: self.t(k) for k in self.z if k.startswith("in_")
                and k not in ("in_canonical_pcd", "in_bones", "in_mean_min_distance", "in_t", "in_c2w",
                              "in_K", "in_rays_o", "in_rays_d", "in_viewdirs")}

    @property
    def bones(self):
        return self.z["in_bones"].tolist()

    def cfg(self, k):
        return self.z["cfg_" + k].item()

    def render_kwargs(self, device="cpu"):
        return {"rays_o": self.t("in_rays_o").to(device), "rays_d": self.t("in_rays_d").to(device),
                "viewdirs": self.t("in_viewdirs").to(device), "near": self.cfg("near"),
                "far": self.cfg("far"), "bg": self.cfg("bg"), "stepsize": self.cfg("stepsize"),
                "render_depth": True, "inverse_y": bool(self.cfg("inverse_y"))}

    def oracle(self, **kw):
        from oracle.apn_oracle import OracleModel
        return OracleModel(self.state(), self.t("in_canonical_pcd"), self.bones,
                           stepsize=self.cfg("stepsize"), voxel_size=self.cfg("voxel_size"),
                           fast_color_thres=1e-4, pose_embedding_dim=int(self.cfg("pose_embedding_dim")),
                           act_shift=float(self.cfg("act_shift")),
                           voxel_size_ratio=float(self.cfg("voxel_size_ratio")), **kw)
