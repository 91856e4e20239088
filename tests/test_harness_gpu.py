"""The render harness on the GPU (run.py:80-239 render_viewpoints, 241-356 render_repose, through
apn_amd.harness): per view the rays of tineuvox.get_rays_of_a_view, one fused forward per frame;
the returned images equal the model's own frame, the PNGs decode to to8b of them, the skeleton
is drawn on the weight images, PSNR / SSIM against ground truth are reported."""
import numpy as np
import pytest
import torch

from golden_io import Golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gm():
    from model_io import model_from_golden
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    g = Golden("G3")
    return g, model_from_golden(g, "cuda")


def _views(g, n=2, H=40, W=48):
    c2w = g.t("in_c2w").float()
    K = g.t("in_K").float().clone()
    K[0, 2], K[1, 2] = W / 2, H / 2
    poses = torch.stack([c2w] * n)
    poses[1:, :3, 3] += torch.tensor([0.05, 0.0, -0.03])
    return poses, np.array([[H, W]] * n), torch.stack([K] * n)


@torch.no_grad()
def test_render_viewpoints_matches_model_frames(gm, tmp_path):
    from apn_amd import harness as Hn
    from apn_amd.tineuvox import get_rays_of_a_view
    g, m = gm
    poses, HW, Ks = _views(g)
    rk = {k: v for k, v in g.render_kwargs("cuda").items() if k not in ("rays_o", "rays_d", "viewdirs")}
    times = [float(g.t("in_t")), float(g.t("in_t")) + 0.1]
    gt = [np.full((HW[i][0], HW[i][1], 3), 0.5, np.float32) for i in range(2)]
    rgbs, depths, weights, flows = Hn.render_viewpoints(m, poses, HW, Ks, False, dict(rk), gt_imgs=gt,
                                                        savedir=str(tmp_path), test_times=times, eval_psnr=True,
                                                        eval_ssim=True, verbose=False)
    assert rgbs.shape == (2, 40, 48, 3) and depths.shape == (2, 40, 48, 1) and weights.shape == (2, 40, 48, 3)
    for i in range(2):
        H, W = HW[i]
        # the harness makes each view's rays on the model's device (as the reference does on its poses')
        ro, rd, vd = get_rays_of_a_view(H, W, Ks[i].float().cuda(), poses[i].float().cuda(), False,
                                        inverse_y=rk["inverse_y"])
        sub = dict(rk, rays_o=ro.reshape(-1, 3), rays_d=rd.reshape(-1, 3), viewdirs=vd.reshape(-1, 3))
        out = m(torch.tensor([times[i]], device="cuda"), render_depth=True, render_kwargs=sub, render_weights=True)
        assert np.array_equal(rgbs[i], out["rgb_marched"].reshape(H, W, 3).cpu().numpy())
        assert np.array_equal(depths[i], out["depth"].reshape(H, W, 1).cpu().numpy())
        assert np.array_equal(Hn.read_png(tmp_path / f"img_{i:03d}.png"), Hn.to8b(rgbs[i]))
        w8 = Hn.read_png(tmp_path / f"weights_{i:03d}.png")   # written before the skeleton overlay
        assert np.array_equal(w8, Hn.to8b(out["weights"].reshape(H, W, 3).cpu().numpy()))
    assert (weights == 0).all(-1).any()   # the skeleton overlay drew black pixels
    res = open(tmp_path / "results.txt").read()
    assert res.startswith("psnr: ") and "ssim: " in res
    p = -10 * np.log10(np.mean((rgbs[0] - gt[0]) ** 2))
    assert abs(float(res.split()[1]) - np.mean([p, -10 * np.log10(np.mean((rgbs[1] - gt[1]) ** 2))])) < 1e-4


@torch.no_grad()
def test_render_repose(gm, tmp_path):
    from apn_amd import harness as Hn
    g, m = gm
    poses, HW, Ks = _views(g)
    rk = {k: v for k, v in g.render_kwargs("cuda").items() if k not in ("rays_o", "rays_d", "viewdirs")}
    rp = g.t("repose_rot_params")
    rot = torch.stack([rp, rp * 0.5])
    rgbs, depths, weights = Hn.render_repose(rot, poses, HW, Ks, False, m, dict(rk), savedir=str(tmp_path))
    assert rgbs.shape == (2, 40, 48, 3) and np.isfinite(rgbs).all()
    assert not np.array_equal(rgbs[0], rgbs[1])   # different poses
    assert (tmp_path / "img_001.png").exists() and (tmp_path / "weights_001.png").exists()
