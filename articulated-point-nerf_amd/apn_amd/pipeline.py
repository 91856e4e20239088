"""Frames in flight on ONE TemporalPoints (the reference's render loop, run.py:108-173, renders a
view and reads it back before it starts the next).

A frame's stages depend on each other (the kNN needs the warped cloud, the MLP the kNN's
survivors), so inside one frame the latency-bound kNN passes, the small stages and the MLP run
one after another. ``FramePipeline`` keeps n frames in flight instead: the model's frame is
captured n times as a HIP graph, each capture into a per-frame workspace of its own
(``TemporalPoints.capture_frame(workspace=...)``), and frame i replays graph i % n on stream
i % n, so one frame's MLP runs beside the next frames' kNN and small stages. The model's
parameters, its canonical tables and the layer-1 projection P are shared: resident memory is one
model plus n per-frame workspaces (each also holds its own 0.5 MB packed-weight buffer, whose b1
follows the frame's pose embedding and whose range flag follows the frame's MLP launch).

Per frame, ``submit`` copies the frame's inputs (time; rays, camera pose and intrinsics when they
change per view) into the slot's static buffers on the slot's stream, replays the graph and --
with ``readback`` -- queues the device-to-host copies of the requested outputs into the slot's
pinned buffers. ``FrameHandle.result()`` waits for that frame only, validates it (its frame_info
rode along: a frame whose samples overflowed the captured capacity is rendered again exactly and
the slot is captured again before its next replay) and returns CPU tensors. A slot is reused only
after its previous frame has been fetched, so its static outputs and pinned buffers are never
overwritten under a reader. ``harness.render_viewpoints`` and bench.py's timed loop run on this.
"""
from __future__ import annotations

import numpy as np
import torch

from .ops import Workspace

READBACK = ("rgb_marched", "depth", "weights")


class FrameHandle:
    """One submitted frame. ``result()`` (readback pipelines): CPU tensors of the requested keys
    (+ ``joints`` with get_skeleton); ``device()``: the frame's RenderOutput on the device, valid
    until its slot is reused n frames later."""

    def __init__(self, pipe, slot, out, t, dest=None):
        self._pipe, self._slot, self._out, self._t = pipe, slot, out, t
        self._dest = dest   # submit(dest=...): the readback went straight into these pinned tensors
        self._res = None

    def done(self) -> bool:
        return self._res is not None or self._slot["done"].query()

    def device(self):
        if self._slot["handle"] is not self:
            raise RuntimeError("FrameHandle.device(): the slot has been reused by a later frame")
        return self._out

    def result(self, into=None) -> dict:
        """Wait for this frame, validate it, return its outputs as CPU tensors -- or, with ``into``
        ({key: numpy array}), copy them straight from the pinned buffers into those arrays (one host
        copy; harness.render_viewpoints fills its result stacks this way) and return ``into``."""
        if self._res is not None:
            if into is not None:
                for k, a in into.items():
                    np.copyto(a, self._res[k].numpy().reshape(a.shape))
                return into
            return self._res
        slot = self._slot
        if slot["handle"] is not self:
            raise RuntimeError("FrameHandle.result(): the slot has been reused by a later frame")
        if not self._pipe.readback:
            raise RuntimeError("FrameHandle.result(): the pipeline has no readback keys")
        slot["done"].synchronize()
        host = slot["host"]
        info = host["_info"].tolist()   # {queries, in-bbox total, overflow, survivors}
        if self._dest is not None:
            # the frame's outputs are already in the caller's pinned tensors (no host copy)
            if info[2]:
                fresh = self._out._rerender()
                for k, v in self._dest.items():
                    v.copy_(fresh[k].detach().reshape(v.shape))
                self._pipe.rerenders += 1
            res = dict(self._dest)
            if "joints" in host:
                res["joints"] = (fresh["joints"].detach().cpu().clone() if info[2] and self._pipe.get_skeleton
                                 else host["joints"].clone())
            res["kept_samples"], res["inbbox_samples"] = info[3], info[1]
            self._res = res
            return res
        if info[2]:
            # overflowed the captured capacity: the exact render (the model's own workspace; its
            # rerender also marks the slot's graph for a capture before its next replay)
            fresh = self._out._rerender()
            res = {k: fresh[k].detach().cpu().clone() for k in self._pipe.readback}
            if self._pipe.get_skeleton:
                res["joints"] = fresh["joints"].detach().cpu().clone()
            self._pipe.rerenders += 1
        elif into is not None:
            for k, a in into.items():
                np.copyto(a, host[k].numpy().reshape(a.shape))
            res = dict(into)
            if "joints" in host and "joints" not in into:
                res["joints"] = host["joints"].clone()
            res["kept_samples"], res["inbbox_samples"] = info[3], info[1]
            self._res = {k: (torch.from_numpy(v) if isinstance(v, np.ndarray) else v) for k, v in res.items()}
            return res
        else:
            res = {k: host[k].clone() for k in host if k != "_info"}
        res["kept_samples"], res["inbbox_samples"] = info[3], info[1]
        self._res = res
        if into is not None:
            for k, a in into.items():
                np.copyto(a, res[k].numpy().reshape(a.shape))
            return dict(into, **{k: v for k, v in res.items() if k not in into})
        return res


class FramePipeline:
    """n frames of ``model`` in flight on n streams (see the module docstring).

    ``render_kwargs`` / ``poses`` / ``Ks`` / ``t`` describe the frame used for the captures (its
    ray count is fixed; later frames pass their own rays, poses and Ks of the same shapes to
    ``submit``). ``readback``: output keys copied to pinned host memory per frame (None: none,
    frames are read on the device through ``FrameHandle.device()`` or not at all, as bench.py's
    timed loop does)."""

    def __init__(self, model, t, render_kwargs, n=4, render_depth=True, render_weights=True, query_radius=0.01,
                 poses=None, Ks=None, get_skeleton=False, readback=READBACK):
        if n < 1:
            raise ValueError("FramePipeline: n >= 1")
        self.model, self.n = model, n
        self.dev = dev = model.canonical_feat.device
        self.get_skeleton = get_skeleton
        self.readback = tuple(readback) if readback else ()
        self.R = len(render_kwargs["rays_o"])
        self.rerenders = 0
        self._count = 0
        t = torch.as_tensor(t, dtype=torch.float32, device=dev).reshape(-1)
        self._slots = []
        for _ in range(n):
            ws = Workspace()
            rk = dict(render_kwargs)
            for k in ("rays_o", "rays_d", "viewdirs"):
                rk[k] = render_kwargs[k].detach().to(dev, torch.float32).contiguous().clone()
            ps = poses.detach().to(dev, torch.float32).clone() if get_skeleton else None
            ks = Ks.detach().to(dev, torch.float32).clone() if get_skeleton else None
            step = model.capture_frame(t, rk, render_depth=render_depth, render_weights=render_weights,
                                       query_radius=query_radius, poses=ps, Ks=ks, get_skeleton=get_skeleton,
                                       workspace=ws)
            slot = {"ws": ws, "rk": rk, "poses": ps, "Ks": ks, "step": step, "stream": torch.cuda.Stream(dev),
                    "done": torch.cuda.Event(), "handle": None, "host": None}
            if self.readback:
                widths = {"rgb_marched": 3, "rgb_marched_direct": 3, "depth": 1, "weights": 3,
                          "alphainv_last": 1, "alphainv_last_direct": 1}
                host = {}
                for k in self.readback:
                    if k not in widths:
                        raise ValueError(f"FramePipeline: readback key {k!r} is not a per-ray output")
                    shape = (self.R, widths[k]) if widths[k] > 1 else (self.R,)
                    host[k] = torch.empty(shape, dtype=torch.float32, pin_memory=True)
                if get_skeleton:
                    host["joints"] = None   # shaped on the first frame
                host["_info"] = torch.empty(4, dtype=torch.int32, pin_memory=True)
                slot["host"] = host
            self._slots.append(slot)

    # ------------------------------------------------------------------------------------------
    @property
    def workspaces(self):
        return [s["ws"] for s in self._slots]

    @property
    def steps(self):
        return [s["step"] for s in self._slots]

    @property
    def streams(self):
        return [s["stream"] for s in self._slots]

    def overflowed(self) -> bool:
        """True if any replay since the last call dropped samples past its captured capacity."""
        return any([bool(s["step"].overflowed()) for s in self._slots])

    def join(self, stream=None):
        """Make ``stream`` (default: the current one) wait for every frame submitted so far."""
        cur = stream or torch.cuda.current_stream(self.dev)
        for s in self._slots:
            cur.wait_stream(s["stream"])

    def submit(self, t, rays=None, poses=None, Ks=None, dest=None) -> FrameHandle:
        """Queue the next frame: time ``t`` (and, when they change per view, ``rays`` =
        (rays_o, rays_d, viewdirs) [R, 3] each, ``poses`` [V, 4, 4], ``Ks`` [V, 3, 3]) on the next
        slot's stream. Inputs made on the caller's stream are ordered before the frame. ``dest``
        ({readback key: pinned CPU tensor}): the frame's outputs are copied by DMA straight into
        those tensors instead of the slot's pinned buffers (no host copy; harness.render_viewpoints
        hands in slices of its result stacks)."""
        slot = self._slots[self._count % self.n]
        self._count += 1
        prev = slot["handle"]
        if prev is not None and self.readback and prev._res is None:
            prev.result()   # the host takes its copy before the slot's pinned buffers are reused
        cur = torch.cuda.current_stream(self.dev)
        s = slot["stream"]
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            if rays is not None:
                for k, v in zip(("rays_o", "rays_d", "viewdirs"), rays):
                    if v.shape[0] != self.R:
                        raise ValueError(f"FramePipeline.submit: {self.R} rays expected, got {v.shape[0]}")
                    v = v.detach().reshape(self.R, 3)
                    if v.is_cuda:
                        v.record_stream(s)
                    slot["rk"][k].copy_(v, non_blocking=True)
            # the caller's device inputs are read on this stream: record the use, so the caching
            # allocator does not hand their blocks to the caller's next allocation before the copy
            # has run (harness.render_viewpoints drops each view's c2w / K right after submit)
            if poses is not None and slot["poses"] is not None:
                if poses.is_cuda:
                    poses.record_stream(s)
                slot["poses"].copy_(poses.reshape(slot["poses"].shape), non_blocking=True)
            if Ks is not None and slot["Ks"] is not None:
                if Ks.is_cuda:
                    Ks.record_stream(s)
                slot["Ks"].copy_(Ks.reshape(slot["Ks"].shape), non_blocking=True)
            if isinstance(t, torch.Tensor) and t.is_cuda:
                t.record_stream(s)
            tt = torch.as_tensor(t, dtype=torch.float32, device=self.dev).reshape(-1)
            out = slot["step"](tt)
            if self.readback:
                host = slot["host"]
                for k in self.readback:
                    if dest is not None and k in dest:
                        dest[k].copy_(out.raw(k).reshape(dest[k].shape), non_blocking=True)
                    else:
                        host[k].copy_(out.raw(k).reshape(host[k].shape), non_blocking=True)
                if self.get_skeleton:
                    j = out.raw("joints")
                    if host["joints"] is None or host["joints"].shape != j.shape:
                        host["joints"] = torch.empty(j.shape, dtype=j.dtype, pin_memory=True)
                    host["joints"].copy_(j, non_blocking=True)
                host["_info"].copy_(out._info if out._info is not None else torch.zeros(4, dtype=torch.int32,
                                                                                           device=self.dev),
                                    non_blocking=True)
            slot["done"].record(s)
        h = FrameHandle(self, slot, out, t, dest)
        slot["handle"] = h
        return h

    def render(self, ts, views=None):
        """Frames at times ``ts`` (views[i] = (rays, poses, Ks) or None), n in flight; yields each
        frame's result() in order, fetching frame i once frame i + n - 1 has been queued."""
        pending = []
        for i, t in enumerate(ts):
            v = views[i] if views is not None else None
            pending.append(self.submit(t, *(v or ())))
            if len(pending) >= self.n:
                yield pending.pop(0).result()
        for h in pending:
            yield h.result()


def capture_sharded_in_flight(model, t, render_kwargs, rank, world, group=None, n=4, **forward_kwargs):
    """n capture_sharded steps of one model, each captured into its own per-frame workspace and
    with its own input buffers (``step.inputs``: rays, and the camera pose / intrinsics when the
    skeleton is projected), for shard.replay_in_flight (the ray-shard frames in flight of bench.py
    --gpus N; a frame's view is copied into its step's inputs before the replay)."""
    from .shard import RAY_BLOCK, capture_sharded
    block = forward_kwargs.pop("block", RAY_BLOCK)
    dev = model.canonical_feat.device
    steps = []
    for _ in range(n):
        rk = dict(render_kwargs)
        for k in ("rays_o", "rays_d", "viewdirs"):
            rk[k] = render_kwargs[k].detach().to(dev, torch.float32).contiguous().clone()
        fk = dict(forward_kwargs)
        if fk.get("get_skeleton"):
            fk["poses"] = fk["poses"].detach().to(dev, torch.float32).clone()
            fk["Ks"] = fk["Ks"].detach().to(dev, torch.float32).clone()
        st = capture_sharded(model, t, rk, rank, world, group, block=block, workspace=Workspace(), **fk)
        st.inputs = {"rays": (rk["rays_o"], rk["rays_d"], rk["viewdirs"]), "poses": fk.get("poses"),
                     "Ks": fk.get("Ks")}
        steps.append(st)
    return steps


def _model_version(model):
    """What a captured frame bakes in besides its inputs: every parameter's and buffer's storage
    and in-place version (the packed MLP / TransformNet weights are derived from them on the host,
    so a graph captured before an update would replay the old ones)."""
    return tuple((p.data_ptr(), p._version) for p in list(model.parameters()) + list(model.buffers()))


def _render_settings(model):
    """The model's plain (non-tensor) attributes a captured frame bakes in: compositing masks,
    early ray termination, the kept joints, the density activation's shift and the IDW epsilon."""
    keep = model.joints_to_keep
    keep = tuple(keep.tolist()) if isinstance(keep, torch.Tensor) else (tuple(keep) if keep is not None else None)
    tnv = model.tineuvox
    return (float(model.fast_color_thres), bool(model.early_termination), keep,
            float(getattr(tnv, "act_shift", 0.0)), float(getattr(tnv, "voxel_size_ratio", 1.0)), float(model._eps))


def cached_pipeline(model, t, render_kwargs, n=4, **kw) -> FramePipeline:
    """The model's FramePipeline for this ray count and these render settings, captured on first
    use and reused while the model's parameters and plain render settings are unchanged
    (harness.render_viewpoints calls it once per viewpoint sweep). A pipeline whose model changed is
    dropped with its workspaces."""
    scal = tuple(sorted((k, v) for k, v in render_kwargs.items()
                        if isinstance(v, (int, float, bool, str)) or v is None))
    opts = tuple(sorted((k, v) for k, v in kw.items() if k not in ("poses", "Ks") and not isinstance(v, torch.Tensor)))
    key = (len(render_kwargs["rays_o"]), n, scal, opts, _render_settings(model))
    ver = _model_version(model)
    cache = model.__dict__.setdefault("_pipelines", {})
    hit = cache.get(key)
    if hit is not None and hit[0] == ver:
        return hit[1]
    cache.clear()   # one pipeline per model: n per-frame workspaces are ~2 GB each at C2
    torch.cuda.synchronize(model.canonical_feat.device)   # a dropped pipeline's frames may still run
    pipe = FramePipeline(model, t, render_kwargs, n=n, **kw)
    cache[key] = (_model_version(model), pipe)
    return pipe
