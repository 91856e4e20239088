"""Render harness: the counterpart of the reference's ``render_viewpoints`` /
``render_repose`` (run.py:80-239, 241-356) for synthetic scenes, minus file I/O and metrics
that need ground-truth images.

A frame is rendered with a single ``TemporalPoints.forward`` over all H*W rays (chunking is
optional and bit-identical); ``render_pcd_direct`` substitutes ``rgb_marched_direct`` for
``rgb_marched`` as run.py:162-163 does.
"""
from __future__ import annotations

import math

import torch

from . import synthetic as S
from .temporalpoints import TemporalPoints
from .tineuvox import TiNeuVoxHeads


def build_model(scene: S.Scene, device="cuda") -> TemporalPoints:
    """TemporalPoints(**scene.ctor, tineuvox=heads) with the scene's network weights loaded."""
    c = scene.ctor
    heads = TiNeuVoxHeads(c["xyz_min"], c["xyz_max"], num_voxels=160 ** 3, num_voxels_base=160 ** 3,
                          net_width=S.NET_WIDTH, alpha_init=S.ALPHA_INIT, posbase_pe=S.POSBASE_PE,
                          viewbase_pe=S.VIEWBASE_PE, timebase_pe=S.TIMEBASE_PE, no_view_dir=False)
    model = TemporalPoints(**c, tineuvox=heads)
    missing, unexpected = model.load_state_dict(scene.params, strict=False)
    if unexpected:
        raise KeyError(f"unexpected state-dict keys: {unexpected}")
    return model.to(device)


PER_POINT_CTOR = ("canonical_pcd", "canonical_alpha", "canonical_feat", "canonical_rgbs")


def shard_scene_points(scene: S.Scene, rank: int, world: int) -> S.Scene:
    """The scene restricted to rank's contiguous point range [N*rank/world, N*(rank+1)/world)
    (LBS is per point, so the shards skin independently; the skeleton,
    joints and networks are replicated). Per-point parameters derived in the constructor (the
    bone-distance LBS weights, direct_eps, gammas) are per point as well."""
    import copy
    from .temporalpoints import weights_from_bones
    N = len(scene.ctor["canonical_pcd"])
    r0, r1 = N * rank // world, N * (rank + 1) // world
    ctor = dict(scene.ctor)
    for k in PER_POINT_CTOR:
        ctor[k] = scene.ctor[k][r0:r1]
    out = copy.copy(scene)
    out.ctor = ctor
    # the raw LBS weights of the full cloud, sliced (the vectorised bone-distance pass is not
    # bit-stable under a change of N); loaded over the constructor's own by build_model
    full_w = weights_from_bones(torch.as_tensor(scene.ctor["joints"]).float(), scene.ctor["bones"],
                                torch.as_tensor(scene.ctor["canonical_pcd"]).float(), torch.tensor(1e-6))
    out.params = dict(scene.params, weights=full_w[r0:r1].contiguous())
    out.extra = dict(scene.extra, point_range=(r0, r1))
    return out


def render_kwargs_for(scene: S.Scene, device="cuda"):
    return scene.render_kwargs(device)


@torch.no_grad()
def render_frame(model, scene: S.Scene, t=None, rot_params=None, render_kwargs=None, chunk=None,
                 render_pcd_direct=False, device="cuda"):
    """One frame -> dict of (H, W, C) images: rgb, depth, weights (+ joints)."""
    rk = render_kwargs if render_kwargs is not None else scene.render_kwargs(device)
    H, W = scene.cfg.H, scene.cfg.W
    R = rk["rays_o"].shape[0]
    chunk = chunk or R
    outs = []
    t_arg = None if rot_params is not None else torch.tensor([scene.cfg.t if t is None else t], device=device)
    for s in range(0, R, chunk):
        sub = dict(rk)
        for k in ("rays_o", "rays_d", "viewdirs"):
            sub[k] = rk[k][s:s + chunk]
        out = model(t_arg, render_depth=True, render_kwargs=sub, render_weights=True, rot_params=rot_params,
                    render_pcd_direct=render_pcd_direct, poses=scene.c2w[None].to(device),
                    Ks=scene.K[None].to(device), get_skeleton=True)
        if render_pcd_direct:
            out["rgb_marched"] = out["rgb_marched_direct"]
        outs.append(out)
    res = {k: torch.cat([o[k] for o in outs]).reshape(H, W, -1) for k in ("rgb_marched", "depth", "weights")}
    res["joints"] = outs[0]["joints"]
    return res


def psnr(a: torch.Tensor, b: torch.Tensor) -> float:
    """run.py:186: -10 log10(mean((a-b)^2))."""
    mse = float(((a.float() - b.float()) ** 2).mean())
    return float("inf") if mse == 0 else -10.0 * math.log10(mse)


# ---------------------------------------------------------------------------------------------
# run.py --render_pcd / --render_test harness (f-2): render_viewpoints and render_repose with
# the reference's signatures and returns (run.py:80-239, 241-356), PNG output, PSNR / SSIM.
# A TemporalPoints frame runs as ONE forward over all H*W rays (the fused path is chunk-invariant,
# tests/test_hip_parity.py), so ``batch_size`` only chunks the stage-1 TiNeuVox model, as the
# reference does for it.

def to8b(x):
    """utils.to8b: uint8(255 * clip(x, 0, 1))."""
    import numpy as np
    return (255 * np.clip(x, 0, 1)).astype(np.uint8)


def write_png(path, img8):
    """8-bit greyscale / RGB / RGBA PNG writer (zlib, filter 0 per row) standing in for
    imageio.imwrite, which this image does not ship."""
    import struct
    import zlib
    import numpy as np
    a = np.ascontiguousarray(img8, dtype=np.uint8)
    if a.ndim == 2:
        a = a[:, :, None]
    h, w, c = a.shape
    ctype = {1: 0, 3: 2, 4: 6}[c]
    raw = np.concatenate([np.zeros((h, 1), np.uint8), a.reshape(h, w * c)], axis=1).tobytes()

    def chunk(tag, data):
        return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)
    png = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, ctype, 0, 0, 0)) + \
        chunk(b"IDAT", zlib.compress(raw, 6)) + chunk(b"IEND", b"")
    with open(path, "wb") as f:
        f.write(png)


def read_png(path):
    """The inverse of write_png (filter-0 images only): -> uint8 [H, W, C]."""
    import struct
    import zlib
    import numpy as np
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, hdr = 8, b"", None
    while pos < len(data):
        n = struct.unpack(">I", data[pos:pos + 4])[0]
        tag, body = data[pos + 4:pos + 8], data[pos + 8:pos + 8 + n]
        if tag == b"IHDR":
            hdr = struct.unpack(">IIBBBBB", body)
        elif tag == b"IDAT":
            idat += body
        pos += 12 + n
    w, h, _, ctype = hdr[:4]
    c = {0: 1, 2: 3, 6: 4}[ctype]
    rows = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 1 + w * c)
    assert (rows[:, 0] == 0).all(), "filter-0 rows only"
    return rows[:, 1:].reshape(h, w, c)


def _draw_line(img, p0, p1, color):
    """8-connected line (cv2.LINE_8 style) from p0 to p1 = (x, y), clipped to the image: the pixels
    of the integer error-term walk (x, y or both advance per step), in closed form -- along the
    major axis i = 0 .. d, the minor coordinate moves floor((2 i d_minor + d) / (2 d)) steps (the
    walk's own pixels, tests/test_harness_cpu.py::test_draw_line_closed_form_equals_walk)."""
    import numpy as np
    x0, y0 = int(p0[0]), int(p0[1])
    x1, y1 = int(p1[0]), int(p1[1])
    dx, dy = abs(x1 - x0), abs(y1 - y0)
    sx, sy = (1 if x0 < x1 else -1), (1 if y0 < y1 else -1)
    if dx >= dy:
        i = np.arange(dx + 1)
        k = (2 * i * dy + dx) // (2 * dx) if dx > 0 else np.zeros(1, np.int64)
        xs, ys = x0 + sx * i, y0 + sy * k
    else:
        i = np.arange(dy + 1)
        k = (2 * i * dx + dy) // (2 * dy)
        xs, ys = x0 + sx * k, y0 + sy * i
    H, W = img.shape[:2]
    m = (xs >= 0) & (xs < W) & (ys >= 0) & (ys < H)
    img[ys[m], xs[m]] = color


def _draw_line_walk(img, p0, p1, color):
    """The step-by-step error-term walk _draw_line restates in closed form (kept for the test)."""
    x0, y0 = int(p0[0]), int(p0[1])
    x1, y1 = int(p1[0]), int(p1[1])
    dx, dy = abs(x1 - x0), -abs(y1 - y0)
    sx, sy = (1 if x0 < x1 else -1), (1 if y0 < y1 else -1)
    err = dx + dy
    H, W = img.shape[:2]
    while True:
        if 0 <= x0 < W and 0 <= y0 < H:
            img[y0, x0] = color
        if x0 == x1 and y0 == y1:
            break
        e2 = 2 * err
        if e2 >= dy:
            err += dy
            x0 += sx
        if e2 <= dx:
            err += dx
            y0 += sy


def _draw_disc(img, c, radius, color):
    import numpy as np
    H, W = img.shape[:2]
    cx, cy = int(c[0]), int(c[1])
    y0, y1, x0, x1 = max(cy - radius, 0), min(cy + radius + 1, H), max(cx - radius, 0), min(cx + radius + 1, W)
    if y0 >= y1 or x0 >= x1:
        return
    ys, xs = np.mgrid[y0:y1, x0:x1]
    m = (xs - cx) ** 2 + (ys - cy) ** 2 <= radius * radius
    img[ys[m], xs[m]] = color


def draw_skeleton(img, joints, bones):
    """The skeleton overlay of run.py:225-233 (cv2.line thickness 1 per bone, cv2.circle radius 3
    filled per joint, black) on a float [H, W, 3] image, in place. joints: int32 [J, 2] (x, y).
    Pixel parity with OpenCV's rasteriser is unpinned (cv2 is absent here)."""
    for b in bones:
        _draw_line(img, joints[int(b[0])], joints[int(b[1])], 0.0)
    for j in range(len(joints)):
        _draw_disc(img, joints[j], 3, 0.0)
    return img


def rgb_ssim(img0, img1, max_val, filter_size=11, filter_sigma=1.5, k1=0.01, k2=0.03, return_map=False):
    """utils.rgb_ssim (the mip-NeRF SSIM): separable Gaussian blur ('valid' 2D convolutions),
    per-channel statistics, mean of the SSIM map."""
    import numpy as np
    from scipy.signal import convolve2d
    assert img0.ndim == 3 and img0.shape[-1] == 3 and img0.shape == img1.shape
    half = filter_size // 2
    offs = (np.arange(filter_size) - half + (2 * half - filter_size + 1) / 2) / filter_sigma
    g = np.exp(-0.5 * offs ** 2)
    g /= g.sum()

    def blur(z):
        return np.stack([convolve2d(convolve2d(z[..., c], g[:, None], mode="valid"), g[None, :], mode="valid")
                         for c in range(z.shape[-1])], -1)
    m0, m1 = blur(img0), blur(img1)
    s00 = np.maximum(0.0, blur(img0 ** 2) - m0 * m0)
    s11 = np.maximum(0.0, blur(img1 ** 2) - m1 * m1)
    s01 = blur(img0 * img1) - m0 * m1
    s01 = np.sign(s01) * np.minimum(np.sqrt(s00 * s11), np.abs(s01))
    c1, c2 = (k1 * max_val) ** 2, (k2 * max_val) ** 2
    smap = ((2 * m0 * m1 + c1) * (2 * s01 + c2)) / ((m0 * m0 + m1 * m1 + c1) * (s00 + s11 + c2))
    return smap if return_map else float(np.mean(smap))


def _scaled_views(HW, Ks, render_factor):
    import numpy as np
    if render_factor:
        HW = np.copy(HW) // render_factor
        Ks = torch.as_tensor(Ks).clone()
        Ks[:, :2, :3] = Ks[:, :2, :3] // render_factor
    return HW, torch.as_tensor(Ks)


def _finish(rgbs, depths, weights, joints, bones, savedir, psnrs, ssims, eval_psnr, eval_ssim):
    import os
    import numpy as np
    if psnrs or ssims:
        if savedir is not None:
            with open(os.path.join(savedir, "results.txt"), "w") as f:
                if eval_psnr:
                    f.write(f"psnr: {np.mean(psnrs)}\n")
                if eval_ssim:
                    f.write(f"ssim: {np.mean(ssims)}\n")
    if savedir is not None:
        for i, rgb in enumerate(rgbs):
            write_png(os.path.join(savedir, f"img_{i:03d}.png"), to8b(rgb))
        for i, w in enumerate(weights):
            write_png(os.path.join(savedir, f"weights_{i:03d}.png"), to8b(w))
    rgbs, depths, weights = np.asarray(rgbs), np.asarray(depths), np.asarray(weights)
    J = np.array([joints[i] for i in range(len(joints))]).astype(np.int32)
    if len(J) > 0 and bones is not None:
        for i in range(len(weights)):
            draw_skeleton(weights[i], J[i], bones)
    return rgbs, depths, weights


def _joint_record(out, joints, i, HW, render_kwargs):
    j = out.get("joints")
    if j is None:
        return None
    if not render_kwargs.get("inverse_y", False):   # run.py:151-152 (mirrors x by the first view's height)
        j[:, :, 0] = (int(HW[0][0]) - 1) - j[:, :, 0]
    if i not in joints:
        joints[i] = j[0].cpu().numpy()
    return out.get("bones")


def _view_rays(i, HW, Ks, c2w, ndc, inverse_y, flip_x, flip_y, fixed_viewdirs, dev):
    """View i's rays, generated on ``dev`` (the reference generates them on the poses' device)."""
    from .tineuvox import get_rays_of_a_view
    H, W = int(HW[i][0]), int(HW[i][1])
    K = Ks[i].to(dev, torch.float32)
    c2w = torch.as_tensor(c2w).to(dev, torch.float32)
    ro, rd, vd = get_rays_of_a_view(H, W, K, c2w, ndc, inverse_y=inverse_y, flip_x=flip_x, flip_y=flip_y)
    if fixed_viewdirs is not None:
        vd = torch.as_tensor(fixed_viewdirs).to(dev)
    return H, W, K, c2w, ro.reshape(-1, 3), rd.reshape(-1, 3), vd.reshape(-1, 3)


# render_viewpoints' result stacks stay in pinned host memory up to this size (16 views at 800x800
# take 287 MB); a longer sweep returns pageable arrays filled through the pipeline's pinned slots
PINNED_STACK_BYTES = 1 << 30


@torch.no_grad()
def render_viewpoints(model, render_poses, HW, Ks, ndc, render_kwargs, gt_imgs=None, savedir=None, test_times=None,
                      render_factor=0, eval_psnr=False, eval_ssim=False, eval_lpips_alex=False,
                      eval_lpips_vgg=False, inverse_y=False, flip_x=False, flip_y=False, batch_size=4096 * 2,
                      verbose=True, render_pcd_direct=False, render_flow=False, fixed_viewdirs=None, in_flight=4):
    """run.py:80-239: every view's rays (tineuvox.get_rays_of_a_view), the model at that view's
    time, rgb / depth / weight-visualisation images, optional PSNR / SSIM against gt_imgs, PNGs
    in savedir, the skeleton drawn on the weight images. Returns (rgbs, depths, weights, flows).

    A TemporalPoints model renders with ``in_flight`` frames in flight (apn_amd.pipeline): view
    i + 1 .. i + in_flight - 1 are queued on the GPU while view i is read back and scored, all
    from one model (its frame captured once per workspace, reused across calls while the model's
    parameters are unchanged). Every image equals the model's own frame for that view bit for bit
    (tests/test_pipeline.py). ``in_flight=1``: one eager forward per view, as the reference."""
    import os
    import numpy as np
    if eval_lpips_alex or eval_lpips_vgg:
        raise NotImplementedError("LPIPS needs the torchvision / lpips network weights, absent here")
    if render_flow:
        raise NotImplementedError("render_flow: the scene-flow output is not on the fused render path")
    assert len(render_poses) == len(HW) and len(HW) == len(Ks)
    HW, Ks = _scaled_views(HW, Ks, render_factor)
    is_tp = isinstance(model, TemporalPoints)
    rgbs, depths, weights, psnrs, ssims, joints, bones = [], [], [], [], [], {}, None

    def score(i, rgb):
        if gt_imgs is not None and render_factor == 0:
            if eval_psnr:
                psnrs.append(float(-10.0 * np.log10(np.mean(np.square(rgb - gt_imgs[i])))))
            if eval_ssim:
                ssims.append(rgb_ssim(rgb, gt_imgs[i], max_val=1))

    if is_tp and in_flight > 1 and len(render_poses) > 1 and len({(int(h), int(w)) for h, w in HW}) == 1:
        from .pipeline import cached_pipeline
        dev = model.canonical_feat.device
        rgb_key = "rgb_marched_direct" if render_pcd_direct else "rgb_marched"
        pipe, pending, stack, pinned = None, [], {}, {}
        n_views = len(render_poses)

        def fetch():
            # frame i is fetched while frames i + 1 .. i + n - 1 render: its images go straight from
            # the pinned readback into the result stacks, and its PNGs / skeleton overlay are made
            # here (in the order _finish would: PNGs first), overlapped with the GPU's next frames
            nonlocal bones
            i, H, W, h = pending.pop(0)
            if pinned:
                r = h.result()   # the frame's images are already in the pinned stacks (DMA at submit)
            else:   # pageable stacks: one host copy from the slot's pinned buffers
                r = h.result(into={rgb_key: stack["rgb"][i], "depth": stack["depth"][i],
                                   "weights": stack["weights"][i]})
            if "joints" in r:
                b = _joint_record({"joints": r["joints"], "bones": model.bones if model.joints_to_keep is None
                                   else model.new_bones}, joints, i, HW, render_kwargs)
                bones = b if b is not None else bones
            score(i, stack["rgb"][i])
            if savedir is not None:
                write_png(os.path.join(savedir, f"img_{i:03d}.png"), to8b(stack["rgb"][i]))
                write_png(os.path.join(savedir, f"weights_{i:03d}.png"), to8b(stack["weights"][i]))
            if i in joints and bones is not None:
                draw_skeleton(stack["weights"][i], np.asarray(joints[i]).astype(np.int32), bones)
        for i, c2w in enumerate(render_poses):
            H, W, K, c2w, ro, rd, vd = _view_rays(i, HW, Ks, c2w, ndc, inverse_y, flip_x, flip_y, fixed_viewdirs, dev)
            t = torch.as_tensor(test_times[i], dtype=torch.float32, device=dev).reshape(1)
            if pipe is None:
                rk = dict(render_kwargs, rays_o=ro, rays_d=rd, viewdirs=vd)
                pipe = cached_pipeline(model, t, rk, n=in_flight, render_depth=True, render_weights=True,
                                       poses=c2w[None], Ks=K[None], get_skeleton=True,
                                       readback=(rgb_key, "depth", "weights"))
                # the returned image stacks: up to PINNED_STACK_BYTES in pinned memory (torch's host
                # cache reuses it from call to call; each frame's readback is a DMA straight into its
                # slice, no host copy), a longer sweep in pageable numpy arrays (the frame goes
                # through its slot's pinned buffers, n_in_flight of them, and one host copy)
                use_pinned = n_views * H * W * 7 * 4 <= PINNED_STACK_BYTES
                for k, c in (("rgb", 3), ("depth", 1), ("weights", 3)):
                    if use_pinned:
                        pinned[k] = torch.empty((n_views, H, W, c), dtype=torch.float32, pin_memory=True)
                        stack[k] = pinned[k].numpy()
                    else:
                        stack[k] = np.empty((n_views, H, W, c), dtype=np.float32)
            dest = ({rgb_key: pinned["rgb"][i], "depth": pinned["depth"][i], "weights": pinned["weights"][i]}
                    if pinned else None)
            pending.append((i, H, W, pipe.submit(t, (ro, rd, vd), c2w[None], K[None], dest=dest)))
            if len(pending) >= in_flight:
                fetch()
        while pending:
            fetch()
        if verbose and psnrs:
            print("Testing psnr", np.mean(psnrs), "(avg)")
        if verbose and ssims:
            print("Testing ssim", np.mean(ssims), "(avg)")
        _finish([], [], [], {}, None, savedir, psnrs, ssims, eval_psnr, eval_ssim)   # results.txt
        return stack["rgb"], stack["depth"], stack["weights"], np.array([])

    for i, c2w in enumerate(render_poses):
        dev = model.canonical_feat.device if is_tp else torch.as_tensor(c2w).device
        H, W, K, c2w, ro, rd, vd = _view_rays(i, HW, Ks, c2w, ndc, inverse_y, flip_x, flip_y, fixed_viewdirs, dev)
        if is_tp:
            rk = dict(render_kwargs, rays_o=ro, rays_d=rd, viewdirs=vd)
            px = torch.stack(torch.meshgrid(torch.arange(0, W), torch.arange(0, H), indexing="ij"), -1)
            rk["pixel_coords"] = px.reshape(-1, 2).float().to(dev)
            t = torch.as_tensor(test_times[i], dtype=torch.float32, device=dev).reshape(1)
            out = model(t, render_depth=True, render_kwargs=rk, render_weights=True,
                        render_pcd_direct=render_pcd_direct, poses=c2w[None], Ks=K[None],
                        cam_per_ray=torch.zeros(len(ro))[:, None], get_skeleton=True)
            b = _joint_record(out, joints, i, HW, render_kwargs)
            bones = b if b is not None else bones
            rgb = (out["rgb_marched_direct"] if render_pcd_direct else out["rgb_marched"]).reshape(H, W, -1)
            res = {"rgb_marched": rgb, "depth": out["depth"].reshape(H, W, -1),
                   "weights": out["weights"].reshape(H, W, -1)}
        else:   # stage-1 TiNeuVox: the reference's chunked calls
            chunks = []
            ts = float(test_times[i]) * torch.ones_like(ro[:, :1])
            for a, b_, c, d in zip(ro.split(batch_size), rd.split(batch_size), vd.split(batch_size), ts.split(batch_size)):
                o = model(a, b_, c, d, **render_kwargs)
                chunks.append({k: o[k] for k in ("rgb_marched", "depth")})
            res = {k: torch.cat([c[k] for c in chunks]).reshape(H, W, -1) for k in ("rgb_marched", "depth")}
        rgb = res["rgb_marched"].cpu().numpy()
        rgbs.append(rgb)
        depths.append(res["depth"].cpu().numpy())
        if "weights" in res:
            weights.append(res["weights"].cpu().numpy())
        score(i, rgb)
    if verbose and psnrs:
        print("Testing psnr", np.mean(psnrs), "(avg)")
    if verbose and ssims:
        print("Testing ssim", np.mean(ssims), "(avg)")
    rgbs, depths, weights = _finish(rgbs, depths, weights, joints, bones, savedir, psnrs, ssims, eval_psnr, eval_ssim)
    return rgbs, depths, weights, np.array([])


@torch.no_grad()
def render_repose(rot_params, render_poses, HW, Ks, ndc, model, render_kwargs, gt_imgs=None, savedir=None,
                  render_factor=0, eval_psnr=False, eval_ssim=False, eval_lpips_alex=False, eval_lpips_vgg=False,
                  inverse_y=False, flip_x=False, flip_y=False):
    """run.py:241-356: view i rendered with the skeleton posed by rot_params[i] (the
    TemporalPoints rot_params path). Returns (rgbs, depths, weights)."""
    from .tineuvox import get_rays_of_a_view
    assert isinstance(model, TemporalPoints)
    assert len(render_poses) == len(HW) and len(HW) == len(Ks)
    HW, Ks = _scaled_views(HW, Ks, render_factor)
    dev = model.canonical_feat.device
    rgbs, depths, weights, joints, bones = [], [], [], {}, None
    for i, c2w in enumerate(render_poses):
        H, W = int(HW[i][0]), int(HW[i][1])
        ro, rd, vd = get_rays_of_a_view(H, W, Ks[i], c2w, ndc, inverse_y=inverse_y, flip_x=flip_x, flip_y=flip_y)
        rk = dict(render_kwargs, rays_o=ro.reshape(-1, 3).to(dev), rays_d=rd.reshape(-1, 3).to(dev),
                  viewdirs=vd.reshape(-1, 3).to(dev))
        out = model(None, render_depth=True, render_kwargs=rk, render_weights=True,
                    rot_params=torch.as_tensor(rot_params[i]).to(dev), calc_min_max=True, get_skeleton=True,
                    poses=torch.as_tensor(c2w)[None].to(dev), Ks=Ks[i][None].to(dev))
        b = _joint_record(out, joints, i, HW, render_kwargs)
        bones = b if b is not None else bones
        rgbs.append(out["rgb_marched"].reshape(H, W, -1).cpu().numpy())
        depths.append(out["depth"].reshape(H, W, -1).cpu().numpy())
        weights.append(out["weights"].reshape(H, W, -1).cpu().numpy())
    return _finish(rgbs, depths, weights, joints, bones, savedir, [], [], False, False)
