"""Exact early ray termination of the neighbour MLP (apn_point_mlp_ert, apn_ert.hip).

The reference runs feat_net / densitynet / rgbnet on every kept sample (temporalpoints.py:452-519)
and its compositing then stops each ray at the sample whose update takes T below 1e-3
(render_utils_kernel.cu:445-451); the {rgb, alpha} of later samples are never read. The render
path runs the MLP only on the samples the compositing reads (passes over the live rays' next
samples) and the direct / weight-colour columns on every kept sample. The frame must be
bit-identical to the one that runs the MLP on every kept sample (while the fp16 range guard does
not fire: its FP32 re-run is decided per path, csrc/apn_ert.hip) -- on golden scenes, with and
without the fast_color_thres masks, on a scene whose rays never terminate, and on the whole C2,
C3 and C4 frames -- and the MLP must have skipped exactly the samples after each ray's break."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

KEYS = ("rgb_marched", "rgb_marched_direct", "depth", "weights", "alphainv_last", "alphainv_last_direct")


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch.device("cuda")


def _frame(model, t, rk, ert):
    model.early_termination = ert
    try:
        with torch.no_grad():
            o = model(t, render_depth=True, render_kwargs=rk, render_weights=True)
        out = {k: o[k].clone() for k in KEYS}
        ns = int(model.last_stats["kept_samples"])
        out12 = model._ws.bufs["out12"][:12 * ns].view(ns, 12).clone()
        s_ray = model._ws.bufs["s_ray"][:ns].clone()
        rows = model.last_mlp_rows.clone() if ert else None
    finally:
        model.early_termination = True
    return out, out12, s_ray, rows


def _breaks(alpha, s_ray, n_rays, thr):
    """Per kept sample: is it at or before its ray's break (the samples the compositing reads on the
    Point-NeRF path), by the compositing's own arithmetic (float T updated in double). Vectorised over
    rays (one numpy step per sample position along a ray), so the whole C4 frame takes seconds."""
    a = alpha.astype(np.float32)
    need = np.zeros(len(a), bool)
    starts = np.searchsorted(s_ray, np.arange(n_rays))
    ends = np.searchsorted(s_ray, np.arange(n_rays), side="right")
    rays = np.nonzero(ends > starts)[0]
    st, cnt = starts[rays], (ends - starts)[rays]
    T = np.ones(len(rays), np.float32)
    live = np.ones(len(rays), bool)
    for j in range(int(cnt.max()) if len(rays) else 0):
        act = live & (cnt > j)
        if not act.any():
            break
        i = st[act] + j
        need[i] = True
        ai = a[i]
        upd = (ai > np.float32(thr)) if thr > 0 else np.ones(len(i), bool)
        Ta = T[act]
        Tn = np.where(upd, (Ta.astype(np.float64) * (1.0 - ai.astype(np.float64))).astype(np.float32), Ta)
        T[act] = Tn
        brk = upd & (Tn.astype(np.float64) < 1e-3)
        idx = np.nonzero(act)[0]
        live[idx[brk]] = False
    return need


def _breaks_loop(alpha, s_ray, n_rays, thr):
    """The same walk ray by ray, sample by sample (the compositing's loop as written); pins the
    vectorised form above on the small scenes."""
    a = alpha.astype(np.float32)
    need = np.zeros(len(a), bool)
    starts = np.searchsorted(s_ray, np.arange(n_rays))
    ends = np.searchsorted(s_ray, np.arange(n_rays), side="right")
    for r in np.nonzero(ends > starts)[0]:
        T = np.float32(1)
        for i in range(starts[r], ends[r]):
            need[i] = True
            if thr <= 0 or a[i] > np.float32(thr):
                T = np.float32(np.float64(T) * (1.0 - np.float64(a[i])))
                if np.float64(T) < 1e-3:
                    break
    return need


def _check(model, t, rk, thr):
    full, f12, f_ray, _ = _frame(model, t, rk, False)
    ert, e12, e_ray, rows = _frame(model, t, rk, True)
    for k in KEYS:
        assert torch.equal(full[k], ert[k]), k
    assert torch.equal(f_ray, e_ray)
    f12, e12 = f12.cpu().numpy(), e12.cpu().numpy()
    # direct-path and weight-colour columns: every kept sample, bit-identical to the fused kernel's
    assert np.array_equal(f12[:, 4:], e12[:, 4:])
    # the MLP's columns: identical on every sample the compositing reads, and the passes ran on
    # exactly those plus at most the rest of the pass in which the ray broke
    need = _breaks(f12[:, 3], f_ray.cpu().numpy(), len(rk["rays_o"]), thr)
    if len(f12) < 200_000:
        assert np.array_equal(need, _breaks_loop(f12[:, 3], f_ray.cpu().numpy(), len(rk["rays_o"]), thr))
    assert np.array_equal(f12[need, :4], e12[need, :4])
    n_rows = int(rows.sum())
    assert need.sum() <= n_rows <= len(f12)
    return len(f12), int(need.sum()), n_rows, rows.tolist()


@pytest.mark.parametrize("name", ["G1", "G2", "G3", "G4", "C1"])
def test_ert_frame_bit_identical(dev, name):
    from apn_amd import harness, synthetic as S
    scene = S.make_scene(name)
    model = harness.build_model(scene, dev)
    rk = scene.render_kwargs(dev)
    for dt in (0.0, 0.13):
        t = torch.tensor([scene.cfg.t + dt], device=dev)
        kept, need, rows, per = _check(model, t, rk, model.fast_color_thres)
        print(f"{name} t+{dt}: kept {kept}, read by the compositing {need}, MLP rows {rows} {per}")


def test_ert_without_masks_and_without_termination(dev):
    """fast_color_thres = 0 (no pre/post masks: every sample enters the walk), and a scene whose
    densities are pushed down so that no ray terminates (every pass runs, the MLP sees every
    kept sample): both bit-identical."""
    from apn_amd import harness, synthetic as S
    scene = S.make_scene("G3")
    model = harness.build_model(scene, dev)
    rk = scene.render_kwargs(dev)
    t = torch.tensor([scene.cfg.t], device=dev)
    model.fast_color_thres = 0
    _check(model, t, rk, 0)
    model.fast_color_thres = S.FAST_COLOR_THRES
    with torch.no_grad():
        model.densitynet.bias.sub_(30.0)   # alpha ~ 0: T stays near 1 on every ray
    kept, need, rows, _ = _check(model, t, rk, model.fast_color_thres)
    assert rows == kept == need


@pytest.mark.parametrize("config", ["C2", "C3", "C4"])
def test_ert_full_frame_bit_identical(dev, config):
    """Whole BASELINE frames: C2, C3 and C4 (inverse-y camera, pose embedding, the largest launch
    and the only config with a sixth pass worth of rows past the fifth)."""
    from apn_amd import harness, synthetic as S
    scene = S.make_scene(config)
    model = harness.build_model(scene, dev)
    rk = scene.render_kwargs(dev)
    t = torch.tensor([scene.cfg.t], device=dev)
    kept, need, rows, per = _check(model, t, rk, model.fast_color_thres)
    print(f"{config}: kept {kept}, read by the compositing {need} ({need / kept:.3f}), MLP rows {rows} "
          f"({rows / kept:.3f}) per pass {per}")
    assert rows < kept


def test_direct_blend_entry_equals_inside(dev):
    """apn_direct_blend (the C-ABI form a caller runs itself with with_direct = 0) writes exactly the
    columns 4..11 apn_point_mlp_ert writes inside (and leaves the MLP's columns 0..3 alone)."""
    from apn_amd import harness, synthetic as S
    from apn_amd._lib import call, ptr, stream_ptr
    scene = S.make_scene("G4")
    model = harness.build_model(scene, dev)
    rk = scene.render_kwargs(dev)
    t = torch.tensor([scene.cfg.t], device=dev)
    _, f12, _, _ = _frame(model, t, rk, True)
    ws = model._ws.bufs
    ns = f12.shape[0]
    nsurv = torch.tensor([ns], dtype=torch.int32, device=dev)
    out = torch.full((ns, 12), -7.0, device=dev)
    call("apn_direct_blend", ptr(ws["s_pos"]), ptr(ws["s_nbr"]), ns, ptr(nsurv), ptr(ws["recA"]), ptr(ws["recB"]),
         model._eps, ptr(out), stream_ptr(dev))
    torch.cuda.synchronize()
    assert torch.equal(out[:, 4:], f12[:, 4:])
    assert (out[:, :4] == -7.0).all()
