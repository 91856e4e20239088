"""CPU-only checks of the product host side: the C-ABI library loads and exports every
symbol include/apn_hip.h declares, the ctypes table matches the header, and the
reference-shaped modules are state-dict compatible with the reference (golden fixtures)."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from golden_io import CASES, Golden

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "apn_hip.h")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(apn_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    from apn_amd import _lib
    lib = _lib.load()
    fns = header_functions()
    assert len(fns) >= 20
    for name in fns:
        assert hasattr(lib, name), name
    assert set(fns) == set(_lib.SIGNATURES), set(fns) ^ set(_lib.SIGNATURES)
    assert lib.apn_version().startswith(b"apn_hip")


def test_ctypes_arity_matches_header():
    from apn_amd import _lib
    txt = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    for name, (_, args) in _lib.SIGNATURES.items():
        m = re.search(name + r"\s*\(([^;]*)\)\s*;", txt)
        assert m, name
        params = [p for p in m.group(1).split(",") if p.strip() and p.strip() != "void"]
        assert len(params) == len(args), (name, len(params), len(args))


def test_workspace_queries_need_no_gpu():
    from apn_amd import _lib
    lib = _lib.load()
    assert lib.apn_scan_workspace_bytes(10_000) > 0
    assert lib.apn_grid_workspace_bytes(300_000, 1 << 20) > 4 * (1 << 20)
    assert lib.apn_knn_workspace_bytes(8_000_000) > 8_000_000 * 32
    arr = (ctypes.c_int32 * 32)()
    n = lib.apn_mlp_weight_layout(arr)
    assert n == 20 and arr[16] == 64 and arr[17] == 160 and arr[18] % 4 == 0 and arr[15] > arr[19] > arr[18]


def test_invalid_arguments_rejected_without_gpu():
    from apn_amd import _lib
    lib = _lib.load()
    assert lib.apn_point_mlp(*([None] * 3), 10, *([None] * 4), 64, *([None] * 3), 0.0, 0.0, 0.0, 0, None,
                             None) == 1  # feat_dim != 128
    assert lib.apn_lbs_skin(None, None, 0, 0, None, 0.0, None, None, None, None, None, None, None, 0.0, 0,
                            None, None, None, None, None, None, None, None) == 1
    assert lib.apn_lbs_workspace_bytes(300_000) == 6 * 4 * ((300_000 + 63) // 64)   # one partial per 64-point block
    # the kNN's second grid: launches of more than 2^18 queries; the event form needs its event
    assert lib.apn_knn_uses_agrid(1 << 18) == 0 and lib.apn_knn_uses_agrid((1 << 18) + 1) == 1
    # clouds past the 32-bit buffer-descriptor range are refused before any device work
    import ctypes
    buf = ctypes.create_string_buffer(64)
    p = ctypes.cast(buf, ctypes.c_void_p)
    big = 1 << 27
    assert lib.apn_grid_build(p, big, p, 0.01, 1024, p, p, None) == 1
    assert lib.apn_knn_radius(p, p, 16, p, p, big, 1024, p, 0.01, p, p, p, p, p, None) == 1
    assert lib.apn_knn_radius_ev(p, p, 16, p, p, 1000, 1024, p, 0.01, p, p, p, p, p, None, None) == 1
    assert lib.apn_knn_agrid_build(p, big, 1024, p, None) == 1


def test_missing_library_fails_loudly(monkeypatch):
    from apn_amd import _lib
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "_load_error", None)
    monkeypatch.setattr(_lib, "LIB_PATH", "/nonexistent/libapn_hip.so")
    with pytest.raises(RuntimeError):
        _lib.load()


def test_product_ops_refuse_cpu_tensors():
    from apn_amd import render_utils
    with pytest.raises(RuntimeError):
        render_utils.raw2alpha(torch.zeros(4), -6.9, 0.5)


@pytest.mark.parametrize("name", CASES)
def test_state_dict_compatible_with_reference(name):
    from model_io import model_from_golden
    g = Golden(name)
    model = model_from_golden(g, "cpu")
    ours = model.state_dict()
    for k, v in g.state().items():
        assert k in ours, k
        assert tuple(ours[k].shape) == tuple(v.shape), k
        assert torch.equal(ours[k].float(), v.float()), k


@pytest.mark.parametrize("name", CASES)
def test_constructor_lbs_weights_match_reference(name):
    """_weights_from_bones (temporalpoints.py:235-254) reproduces the reference's init."""
    from model_io import model_from_golden
    g = Golden(name)
    model = model_from_golden(g, "cpu")
    w = model._weights_from_bones(g.t("joints") if "joints" in g.z else g.state()["joints"], g.bones,
                                  g.t("in_canonical_pcd"))
    assert (w - g.state()["weights"]).abs().max() < 1e-6


def test_synthetic_scenes_satisfy_bone_invariant():
    from apn_amd import synthetic as S
    for J in (8, 24, 32, 48):
        joints, bones = S.skeleton_for(J)
        assert len(joints) == J and len(bones) == J - 1
        for k, (p, c) in enumerate(bones):
            assert c == k + 1 and 0 <= p < J and p != c
    sc = S.make_scene("C1")
    assert sc.ctor["canonical_pcd"].shape == (10_000, 3)
    ro, rd, vd = sc.rays()
    assert ro.shape == (64 * 64, 3) and torch.allclose(vd.norm(dim=-1), torch.ones(64 * 64))


def test_get_rays_matches_synthetic_rays():
    from apn_amd import synthetic as S
    from apn_amd.tineuvox import get_rays_of_a_view
    sc = S.make_scene("G2")
    ro, rd, vd = get_rays_of_a_view(sc.cfg.H, sc.cfg.W, sc.K, sc.c2w, inverse_y=True)
    ro2, rd2, vd2 = sc.rays()
    assert torch.equal(rd.reshape(-1, 3), rd2) and torch.equal(vd.reshape(-1, 3), vd2)


def test_bench_psnr_and_flop_accounting():
    """bench.py host logic: PSNR of identical renders is capped (not inf), a known MSE maps to
    its PSNR, and F_alg per kept sample is SURVEY.md 8(d)'s 1 230 848 / 1 361 920 flop."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    assert bench.flop_per_kept_sample(191) == 1_230_848
    assert bench.flop_per_kept_sample(255) == 1_361_920
    sel = torch.arange(4)
    a = {"rgb_marched": torch.full((6, 3), 0.5), "rgb_marched_direct": torch.full((6, 3), 0.5)}
    b = {"rgb_marched": torch.full((4, 3), 0.5), "rgb_marched_direct": torch.full((4, 3), 0.6)}
    r = bench.psnr_vs_oracle(a, b, sel)
    assert r["rgb_marched"] == 200.0 and r["rgb_marched_frac_rays_within_1e-4"] == 1.0
    assert abs(r["rgb_marched_direct"] - 20.0) < 1e-3 and r["rgb_marched_direct_frac_rays_within_1e-4"] == 0.0


def test_get_rays_of_a_view_pinned_to_reference():
    """tineuvox.get_rays_of_a_view (a-22; tineuvox.py:675-738) against the reference's own output
    for both camera conventions (inverse_y), both pixel modes and the flips (golden_T1.npz,
    written by tests/golden/make_golden.py from lib/tineuvox.py): bit-exact."""
    import numpy as np
    from apn_amd.tineuvox import get_rays_of_a_view
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden_T1.npz"))
    c2w, K = torch.from_numpy(z["in_c2w"]), torch.from_numpy(z["in_K"])
    H, W = int(z["cfg_H"]), int(z["cfg_W"])
    n = 0
    for inv_y in (False, True):
        for mode in ("center", "lefttop"):
            for fx, fy in ((False, False), (True, False), (False, True)):
                tag = f"rays_{int(inv_y)}{mode[0]}{int(fx)}{int(fy)}"
                ro, rd, vd = get_rays_of_a_view(H, W, K, c2w, False, inverse_y=inv_y, flip_x=fx, flip_y=fy, mode=mode)
                for got, key in ((ro, "_o"), (rd, "_d"), (vd, "_v")):
                    assert np.array_equal(got.numpy(), z[tag + key]), tag + key
                n += 1
    assert n == 12
    # the synthetic scenes' generator (apn_amd.synthetic.get_rays) is the same function flattened
    from apn_amd import synthetic as S
    ro, rd, vd = S.get_rays(H, W, K, c2w)
    assert np.array_equal(rd.numpy(), z["rays_0c00_d"].reshape(-1, 3))
    assert np.array_equal(vd.numpy(), z["rays_0c00_v"].reshape(-1, 3))


DEBUG_HEADER = os.path.join(ROOT, "include", "apn_hip_debug.h")


def test_product_library_has_no_debug_switches():
    """The shipped library runs one search strategy / kernel per stage: the debug entry points
    (include/apn_hip_debug.h) and the environment reads are in libapn_hip_debug.so only."""
    from apn_amd import _lib
    lib = _lib.load()
    txt = re.sub(r"/\*.*?\*/", "", open(DEBUG_HEADER).read(), flags=re.S)
    dbg_fns = sorted(set(re.findall(r"\b(apn_[a-z0-9_]+)\s*\(", txt)))
    assert set(dbg_fns) == set(_lib.DEBUG_SIGNATURES), set(dbg_fns) ^ set(_lib.DEBUG_SIGNATURES)
    for name in dbg_fns:
        assert not hasattr(lib, name), name
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"getenv" not in data                 # no environment-driven A/B switch in the product
    assert b"APN_KNN_MODE" not in data and b"APN_MLP_OCC" not in data


def test_debug_library_exports_product_and_debug_symbols():
    from apn_amd import _lib
    if not os.path.exists(_lib.DEBUG_LIB_PATH):
        pytest.skip("libapn_hip_debug.so not built")
    dbg = _lib.load_debug()
    for name in list(_lib.SIGNATURES) + list(_lib.DEBUG_SIGNATURES):
        assert hasattr(dbg, name), name
    assert dbg.apn_version() == b"apn_hip 0.1 gfx950 debug"
    assert _lib.load().apn_version() == b"apn_hip 0.1 gfx950"
