"""Benchmark: rendered rays/s of the articulated-point render path on MI355X.

Workload (BASELINE.json configs[1]): dnerf/jumpingjacks-like synthetic scene,
800x800 rays, 300k canonical points, 24 bones (SMPL topology), D-NeRF camera.
A step = one full frame: TemporalPoints.forward over all 640k rays (skeleton, LBS, grid,
sampling, radius kNN, neighbour MLP, compositing), inputs resident in HBM. As in the reference's
render loop (run.py:108-151) every timed frame is a NEW view: the timed loop cycles through
``--views`` (default 16) distinct frames, each its own time and camera pose (an orbit about the
subject, synthetic.view_sweep; view 0 = t 0.3 and the scene's camera), the view's rays, pose and
intrinsics copied into the frame's input buffers on the device per frame.
``config.same_view_ms_per_step`` is the same pipeline replaying view 0 only.

Multi-GPU (python -m torch.distributed.run ... bench.py --gpus N): one process per GPU. By
default (``--shard rays``) the N ranks render ONE frame together (BASELINE
configs C3/C4): every rank replicates the cheap per-frame stages, renders its interleaved
4096-ray blocks (apn_amd/shard.py "blocks" split), and the per-ray tiles are assembled with one
RCCL all-gather over xGMI -- strong scaling, ``value`` = frame rays / step time. ``--shard frames``
has every rank render its own frame instead (weak scaling, no data-path collective). C5
(LBS-only) shards the points N/W per rank with no collective (strong scaling). The timing is
barrier + synchronize bracketed and the max over ranks (all-reduce MAX of the elapsed time).

Frames in flight (``--in-flight``, default 4): a frame's stages run in sequence (the kNN needs the
warped cloud, the MLP the kNN's survivors), so one frame leaves the chip under-used while its kNN
and small stages run. With n frames in flight ONE TemporalPoints replays its frame, captured n
times into n per-frame workspaces (apn_amd.pipeline.FramePipeline; the canonical tables and the
layer-1 projection are shared), on n HIP streams, frame i on stream i % n: one frame's MLP runs
beside the next frames' kNN and sampling. Every frame is still rendered in full and is
bit-identical to a serial frame (tests/test_pipeline.py); ``config.serial_ms_per_step`` is the
same frames one at a time on one stream, ``render_viewpoints`` the drop-in render loop
(harness.render_viewpoints: 8 views at distinct times, host readback) on the same pipeline. Ray
shards keep their per-frame all-gathers on one collective stream in frame order
(apn_amd.shard.replay_in_flight).

Rank 0 prints ONE JSON line. Diagnostics go to stderr.

Launch: ``python bench.py --gpus N`` with N > 1 and no WORLD_SIZE in the environment starts the N
ranks itself (``spawn_ranks``: N child processes of this script, one per GPU, RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set) before anything touches the GPU -- the
replacement for the reference's sequential chunk loop (run.py:136-151) is then N processes, not
one. Under an outer launcher (torch.distributed.run) ``--gpus`` must equal WORLD_SIZE, or the run
aborts (``check_world``).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))


# ----------------------------------------------------------------------------- launcher (stdlib only;
# runs before torch is imported, so the parent never initialises the GPU)
def gpus_arg(argv):
    """The value of --gpus in argv (None when absent)."""
    for i, a in enumerate(argv):
        if a == "--gpus" and i + 1 < len(argv):
            return int(argv[i + 1])
        if a.startswith("--gpus="):
            return int(a.split("=", 1)[1])
    return None


def check_world(gpus, env):
    """World size of this process: WORLD_SIZE from an outer launcher, else 1. --gpus, when given,
    must match it (a mismatch would time fewer processes than the line claims)."""
    world = int(env.get("WORLD_SIZE", "1"))
    if gpus is not None and gpus != world:
        raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={world}; launch with --gpus {world} "
                         f"(or without an outer launcher, where bench.py starts the ranks itself)")
    return world


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_envs(n, port, base_env):
    """One environment per rank for a single-node launch of n ranks (one process per GPU)."""
    envs = []
    for r in range(n):
        e = dict(base_env)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0",
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        envs.append(e)
    return envs


def spawn_ranks(n, cmd, base_env=None, poll_s=0.2):
    """Start n child processes of ``cmd`` (rank environments from rank_envs), forward their output
    (only rank 0 prints the JSON line; the children inherit stdout / stderr), wait for all of them.
    If any child fails, the others are terminated (they would wait forever in a collective) and the
    first failing exit code is returned; 0 when every rank succeeded."""
    env = dict(os.environ if base_env is None else base_env)
    procs = [subprocess.Popen(cmd, env=e) for e in rank_envs(n, free_port(), env)]
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    if rc:
        print(f"bench.py: a rank failed with exit code {rc}; the other ranks were stopped", file=sys.stderr, flush=True)
    return rc


if __name__ == "__main__":
    _g = gpus_arg(sys.argv[1:])
    if _g is not None and _g > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(_g, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]))

import torch  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "articulated-point-nerf_amd"))
sys.path.insert(0, ROOT)

from apn_amd import harness, synthetic as S  # noqa: E402

FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: Peak FP32 (matrix), dense
FP16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16/F16 MFMA ~2.5 PF dense
# the default MLP kernel computes each fp32 product as 3 fp16 MFMA terms (hi*hi + hi*lo + lo*hi,
# fp32 accumulate), so fp32-accurate flops peak at a third of the fp16 dense rate
SPLIT3_PEAK_TFLOPS = FP16_MFMA_PEAK_TFLOPS / 3
HBM_PEAK_GBS = 8000.0


def flop_per_kept_sample(d_in=191, width=128):
    """K*2*(D_in*128 + 3*128^2) + 2*(128 + 128^2 + 155*64 + 64*3)."""
    return 8 * 2 * (d_in * width + 3 * width * width) + 2 * (128 + 128 * 128 + 155 * 64 + 64 * 3)


def mlp_pass_rows(ev, kept):
    """Samples the neighbour MLP ran on per early-termination pass (apn_point_mlp_ert's pass_rows),
    the mean over the timed eager frames (frames of distinct views differ), or [kept] when every
    kept sample went through it."""
    rows = [e[3] for e in ev if len(e) > 3 and e[3] is not None]
    if not rows:
        return [int(kept)]
    return [float(v) for v in torch.stack(rows).double().mean(0).tolist()]


def mean_kept(ev, kept):
    """Kept samples per timed eager frame, the mean over those frames."""
    return float(torch.stack([e[2].reshape(-1)[:1] for e in ev]).double().mean()) if ev else float(kept)


def mlp_pass_ms(timing):
    """Per-pass MLP kernel ms (mean over the timed eager frames) from the HIP events apn_point_mlp_ert
    records around each early-termination pass's MLP launches; None without early termination."""
    fr = timing.get("mlp_pass_events")
    if not fr:
        return None
    n = len(fr[0]) // 2
    return [sum(f[2 * p].elapsed_time(f[2 * p + 1]) for f in fr) / len(fr) for p in range(n)]


def mfma_executed_flop(n_samples, variant=0):
    """MFMA flops the MLP kernel issues per launch, 4 waves per tile.
    variant 1 (FP32 MFMA, 8-sample tiles): 16x16x4 f32 MFMAs for layer 1 (K=64), layers 2-4 (K=128)
    and the folded head (16 padded rows, K=160). Variants 0 / 4 (split, 16- / 8-sample tiles):
    16x16x32 f16 MFMAs, 3 per 32-wide k chunk and 16x16 output block: layer 1 (2 chunks), layers
    2-4 (4 chunks), 16 / 8 blocks per wave; head (5 chunks, 1 block)."""
    if variant in (0, 5):
        tiles = (n_samples + 15) // 16
        mfma_per_wave = 3 * (2 * 16 + 3 * 4 * 16 + 5 * 1)
        assert mfma_per_wave == 687
        return tiles * 4 * mfma_per_wave * (16 * 16 * 32 * 2)
    tiles = (n_samples + 7) // 8
    if variant in (1, 2):
        steps = lambda k: (k // 16) * 4          # 4 MFMA k-steps per 16-wide chunk
        mfma_per_wave = steps(64) * 8 + 3 * steps(128) * 8 + steps(160) * 1   # 8 = 4 M-tiles x 2 N-tiles
        assert mfma_per_wave == 936
        return tiles * 4 * mfma_per_wave * (16 * 16 * 4 * 2)
    mfma_per_wave = 3 * (2 * 8 + 3 * 4 * 8 + 5 * 1)
    assert mfma_per_wave == 351
    return tiles * 4 * mfma_per_wave * (16 * 16 * 32 * 2)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def emit(line, args):
    """The one JSON line on stdout (the driver's contract), optionally also to --out."""
    text = json.dumps(line)
    print(text, flush=True)
    if getattr(args, "out", None):
        with open(args.out, "w") as f:
            f.write(text + "\n")


def threads_note(threads):
    """Why the CPU baseline runs on this many threads: the GPU box gives one GPU's job a 16-core
    share of its host (OMP_NUM_THREADS / MAX_JOBS are set to 16 there; os.cpu_count() reports the
    whole machine), and torch's intra-op pool follows OMP_NUM_THREADS."""
    omp = os.environ.get("OMP_NUM_THREADS")
    return (f"{threads} threads = torch.get_num_threads() (OMP_NUM_THREADS={omp}: the box's CPU share for one GPU; "
            f"the host reports {os.cpu_count()} logical CPUs in total)")


def cpu_model_name():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(model, scene, rows, threads):
    """The oracle (CPU restatement, pure PyTorch + scipy cKDTree kNN) on a bounded sample:
    ``rows`` image rows spread evenly over the same frame (every H/rows-th row), so the
    object-hit fraction matches the full frame."""
    from oracle.apn_oracle import OracleModel
    torch.set_num_threads(threads)
    st = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    orc = OracleModel(st, model.canonical_pcd.cpu(), model.bones, stepsize=S.STEPSIZE, voxel_size=S.VOXEL_SIZE,
                      fast_color_thres=S.FAST_COLOR_THRES, pose_embedding_dim=model.pose_embedding_dim,
                      act_shift=float(model.tineuvox.act_shift),
                      voxel_size_ratio=float(model.tineuvox.voxel_size_ratio),
                      mean_min_distance_value=float(model.mean_min_distance))
    rk = scene.render_kwargs("cpu")
    H, W = scene.cfg.H, scene.cfg.W
    stride = max(1, H // rows)
    sel = torch.cat([torch.arange(r * W, (r + 1) * W) for r in range(stride // 2, H, stride)][:rows])
    sub = dict(rk)
    for k in ("rays_o", "rays_d", "viewdirs"):
        sub[k] = rk[k][sel].contiguous()
    t = torch.tensor([scene.cfg.t])
    ref = orc.forward(t, render_depth=True, render_kwargs=sub, render_weights=True, knn_tree=True)  # warm-up
    n_rep, t0 = 0, time.perf_counter()
    while n_rep < 2 or time.perf_counter() - t0 < 10.0:
        orc.forward(t, render_depth=True, render_kwargs=sub, render_weights=True, knn_tree=True)
        n_rep += 1
        if n_rep >= 6:
            break
    dt = (time.perf_counter() - t0) / n_rep
    nrays = rows * W
    return {"value": nrays / dt, "unit": "rays/s", "cores": threads, "cores_note": threads_note(threads),
            "cpu_model": cpu_model_name(), "kind": "port",
            "sample": f"{rows} evenly spaced rows x {W} = {nrays} rays of the same frame, {n_rep} timed repeats "
                      f"(oracle: torch-CPU MLP, scipy cKDTree kNN), {dt:.2f} s/band"}, ref, sel, (orc, sub, t)


def same_cloud_error(gpu_out, gpu_rk, perm, orc, sub, t, sel):
    """The oracle re-rendering the band against the GPU's own warped cloud (identical sample
    positions and neighbour lists): max |rgb - oracle| over all band rays, and over the rays whose
    oracle compositing is not within 1e-6 of a discontinuity (fast_color_thres on alpha/weight,
    T = 1e-3; oracle/flips.py) -- the arithmetic error of the GPU path at the bench size."""
    from oracle.flips import near_discontinuity, ray_errors, PATH_OF_KEY
    # the GPU's own rays (device and host torch may round a ray direction differently in the
    # last ulp, which moves that ray's samples)
    sub = dict(sub)
    for k in ("rays_o", "rays_d", "viewdirs"):
        sub[k] = gpu_rk[k][sel].detach().cpu().contiguous()
    ref = orc.forward(t, render_depth=True, render_kwargs=sub, render_weights=True, knn_tree=True,
                      t_hat_override=gpu_out["t_hat_pcd"].detach().cpu(), perm=perm)
    res = {"rays": int(sel.numel())}
    for key in ("rgb_marched", "rgb_marched_direct"):
        a = gpu_out[key].detach().float().cpu()[sel].numpy()
        b = ref[key].numpy()
        err = ray_errors(a, b)
        near = near_discontinuity(orc.trace, len(b), PATH_OF_KEY[key])
        res[key] = {"max_abs": float(err.max()), "max_abs_off_discontinuities": float(err[~near].max()),
                    "rays_over_1e-5": int((err > 1e-5).sum()),
                    "rays_over_1e-5_unexplained": int(((err > 1e-5) & ~near).sum())}
    return res


def psnr_vs_oracle(gpu_out, ref, sel):
    """PSNR of the GPU frame against the oracle's free-running render of the same rays (own LBS,
    own bbox; see DESIGN.md §5 for why free-running renders are compared by PSNR)."""
    res = {"rays": int(sel.numel())}
    for key in ("rgb_marched", "rgb_marched_direct"):
        a = gpu_out[key].detach().float().cpu()[sel]
        b = ref[key].detach().float().cpu()
        mse = float(((a - b) ** 2).mean())
        res[key] = round(-10.0 * math.log10(max(mse, 1e-20)), 2)
        res[key + "_frac_rays_within_1e-4"] = round(float(((a - b).abs().amax(-1) <= 1e-4).float().mean()), 5)
    return res


def lbs_sweep(args, rank, world, dev):
    """C5: LBS-only repose throughput (BASELINE.json configs[4]; run.py:1364-1377 sweep). One step
    = one pose of the sweep through TemporalPoints.repose (skeleton + fused LBS, 1M points, 48
    bones). With N>1 GPUs the points are sharded N/W per rank (LBS is per point;
    the skeleton stage is replicated, no collective) and every rank runs the same poses -- strong
    scaling. Roofline: k_lbs_skin_mfma against HBM with B_alg = N*(24 + 4J) bytes per pose
    (SURVEY.md 8(d)), per rank N_r points."""
    scene = S.make_scene(args.config)
    N_total = scene.cfg.N
    if world > 1:
        scene = harness.shard_scene_points(scene, rank, world)
    model = harness.build_model(scene, dev)
    N, J = len(scene.ctor["canonical_pcd"]), scene.cfg.J
    poses = S.repose_sweep(J).to(dev)
    # LBS kernel time for the roofline: 20 back-to-back LBS launches of one pose captured in a HIP
    # graph, HIP events around one replay (eager events around a single launch would also time
    # the host's launch latency whenever the device runs dry)
    with torch.no_grad():
        bone_Ts, gt, _ = model.forward_warp.pose(model.joints, rot_params=poses[0])
        T34 = model.forward_warp.last_T34
        for _ in range(2):
            model._lbs(bone_Ts, gt, records=False, T34=T34)
        torch.cuda.synchronize(dev)
        n_lbs = 20
        g_lbs = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g_lbs):
            for _ in range(n_lbs):
                model._lbs(bone_Ts, gt, records=False, T34=T34)
        g_lbs.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            g_lbs.replay()
        e1.record()
        torch.cuda.synchronize(dev)
        lbs_ms = e0.elapsed_time(e1) / (3 * n_lbs)
        del g_lbs
    # throughput: every pose of the sweep through the captured repose step, in the sweep's order:
    # each pass over the sweep starts with one launch computing every pose's skeleton, then one
    # LBS graph per pose (TemporalPoints.capture_repose(batched=True))
    mode = getattr(args, "repose_mode", "batched")
    n_fl = getattr(args, "repose_in_flight", 4) if mode == "batched" else 1
    step = model.capture_repose(sweep=poses, batched=mode == "batched", pipelined=mode == "pipelined",
                                in_flight=n_fl)
    for i in range(args.warmup):
        step(poses[i % len(poses)])
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(poses[i % len(poses)])
    torch.cuda.synchronize(dev)
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t)
    if rank != 0:
        return
    b_alg = N * (24 + 4 * J)
    lbs_traffic, lbs_src = latest_traffic("lbs_traffic_c5")
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        try:
            from oracle.apn_oracle import OracleModel
            torch.set_num_threads(torch.get_num_threads())
            st = {k: v.detach().cpu() for k, v in model.state_dict().items()}
            orc = OracleModel(st, model.canonical_pcd.cpu(), model.bones, mean_min_distance_value=0.0)
            pc = poses.cpu()
            orc.repose(pc[0])
            n_rep, c0 = 0, time.perf_counter()
            while n_rep < 2 or (time.perf_counter() - c0 < 10.0 and n_rep < 8):
                orc.repose(pc[n_rep % len(pc)])
                n_rep += 1
            dt = (time.perf_counter() - c0) / n_rep
            cpu = {"value": N / dt, "unit": "points/s", "cores": torch.get_num_threads(),
                   "cores_note": threads_note(torch.get_num_threads()),
                   "cpu_model": cpu_model_name(), "kind": "port",
                   "sample": f"{n_rep} poses of the same sweep, full 1M-point cloud (oracle: torch-CPU get_weights + "
                             f"LBS), {dt:.2f} s/pose"}
        except Exception as e:  # never lose the GPU line over the baseline leg
            log(f"cpu baseline failed: {e!r}")
    value = args.steps * N_total / elapsed
    line = {
        "metric": "LBS-only repose throughput, 1M pts, 48 bones (points/s)",
        "value": value, "unit": "points/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "strong" if world > 1 else "weak",
        "vs_baseline": None, "dtype": "fp32", "data": "synthetic (procedural 48-joint capsule cloud, repose sweep)",
        "config": {"workload": S.CONFIGS[args.config].name + f" ({args.config})", "points": N_total, "bones": J,
                   "points_per_rank": N, "poses_per_s": args.steps / elapsed,
                   "step": ("one captured graph per pose: the LBS launch reading its pose's bone transforms; the "
                            "skeleton stage of every pose of the sweep runs as ONE launch (one workgroup per pose) "
                            "at the start of every pass over the sweep -- inside the timed loop, 5 passes of 60 "
                            "poses here (TemporalPoints.capture_repose(sweep=..., batched=True, in_flight=n)); with "
                            "n = poses_in_flight > 1, pose i's graph runs on stream i % n into its own output slot "
                            "(every pose still skinned in full, each output kept until pose i + n)"),
                   "lbs_kernel_ms": lbs_ms, "poses_in_flight": n_fl,
                   "parallelism": f"points x{world} (no collective)" if world > 1 else "single"},
        "roofline": {"bound": "hbm", "kernel": "k_lbs_skin_mfma",
                     "achieved": b_alg / (lbs_ms * 1e-3) / 1e9 if lbs_ms > 0 else 0.0,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": b_alg / (lbs_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if lbs_ms > 0 else 0.0,
                     "traffic": (lbs_traffic or {}).get("bytes_per_launch"),
                     "traffic_source": (f"{lbs_src}: PMC passes on an earlier build; NOT measured in this run"
                                        if lbs_traffic else None),
                     "bytes_per_launch": b_alg, "avg_launch_ms": lbs_ms,
                     "note": "achieved = B_alg = N_r*(24+4J) bytes per pose (SURVEY.md 8(d) C5; N_r = this rank's "
                             "points) / avg LBS kernel time (HIP events around a graph of 20 back-to-back LBS "
                             "launches on the launch stream); the step also runs the skeleton kernel"},
        "cpu_baseline": cpu,
    }
    return line


def device_identity(dev):
    """This rank's GPU as the runtime names it: PCI domain / bus / device ids and UUID (a driver
    run with N ranks shows N distinct devices behind the all-gather), plus the host name."""
    import socket
    p = torch.cuda.get_device_properties(dev)
    ident = {"index": dev.index, "name": p.name, "hostname": socket.gethostname(),
             "visible_devices": os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES")}
    for a in ("pci_domain_id", "pci_bus_id", "pci_device_id", "gcnArchName"):
        v = getattr(p, a, None)
        if v is not None:
            ident[a] = v if isinstance(v, (int, str)) else str(v)
    u = getattr(p, "uuid", None)
    if u is not None:
        ident["uuid"] = str(u)
    return ident


def submit_view(pipe, views, i):
    """Frame i of the render loop: view i % len(views) -- its time, and (with more than one view)
    its rays, camera pose and intrinsics, copied into the slot's inputs on the slot's stream."""
    v = views[i % len(views)]
    if len(views) == 1:
        return pipe.submit(v.t)
    return pipe.submit(v.t, rays=v.rays, poses=v.c2w[None], Ks=v.K[None])


def replay_pipeline(pipe, views, k, serial=False):
    """k frames through one model's FramePipeline (apn_amd.pipeline: n captured frames, each in a
    workspace of its own, frame i on stream i % n), frame i = view i % len(views); the current
    stream joins them at the end. ``serial``: each frame waits for the previous one (one frame at a
    time on the GPU, no host sync). Returns the last frame's handle and the host seconds spent
    issuing."""
    h0 = time.perf_counter()
    h = None
    for i in range(k):
        h = submit_view(pipe, views, i)
        if serial:
            pipe.join()
    host = time.perf_counter() - h0
    pipe.join()
    return h, host


def view_rk(rk, v):
    return dict(rk, rays_o=v.rays[0], rays_d=v.rays[1], viewdirs=v.rays[2])


def presize_capacity(model, views, rk, ray_shard=None):
    """Every view rendered once on the exact path (the in-bbox count read back): the sample
    capacity the captured frames are sized with is then 1.25x the largest view's, so no timed frame
    of the sweep drops samples (``timed_frames_overflowed`` checks it)."""
    model._force_exact = True
    try:
        for v in views:
            model(v.t, render_depth=True, render_kwargs=view_rk(rk, v), render_weights=True,
                  **({"ray_shard": ray_shard} if ray_shard is not None else {}))
    finally:
        model._force_exact = False


def replay_sharded(steps_in_flight, views, k, streams, comm):
    """k ray-shard frames with len(steps_in_flight) in flight (apn_amd.shard.replay_in_flight),
    frame i = view i % len(views). Returns the last frame and the host seconds spent issuing."""
    from apn_amd.shard import replay_in_flight
    h0 = time.perf_counter()
    seq = [views[i % len(views)] for i in range(k)]
    out = replay_in_flight(steps_in_flight, [v.t for v in seq], streams, comm,
                           views=seq if len(views) > 1 else None)[-1]
    return out, time.perf_counter() - h0


def viewpoint_rate(model, scene, dev, n_views=16, in_flight=3):
    """harness.render_viewpoints (run.py:80-239) over n_views views (distinct times and camera poses,
    synthetic.view_sweep) -- rays made
    on the device per view, n frames in flight on the model's FramePipeline, rgb / depth / weights
    read back to host numpy per view -- timed after one untimed sweep (the captures). The drop-in
    render loop's rate next to the timed loop's."""
    from apn_amd.tineuvox import get_rays_of_a_view  # noqa: F401  (the harness's ray maker)
    H, W = scene.cfg.H, scene.cfg.W
    rk = {k: v for k, v in scene.render_kwargs(dev).items() if k not in ("rays_o", "rays_d", "viewdirs")}
    sweep = S.view_sweep(scene, n_views, "cpu")   # the timed loop's views: new time and camera pose each
    poses = torch.stack([v.c2w for v in sweep])
    HW = [[H, W]] * n_views
    Ks = scene.K[None].repeat(n_views, 1, 1)
    times = [float(v.t) for v in sweep]
    kw = dict(test_times=times, verbose=False, inverse_y=bool(rk.get("inverse_y", False)), in_flight=in_flight)
    for _ in range(2):   # the first call captures the pipeline, the second warms the pinned stacks
        harness.render_viewpoints(model, poses, HW, Ks, False, dict(rk), **kw)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    harness.render_viewpoints(model, poses, HW, Ks, False, dict(rk), **kw)
    el = time.perf_counter() - t0
    # the same pipeline's bare submit loop, every frame's rgb / depth / weights read back into the
    # slots' pinned buffers and nothing else: the PCIe readback's own cost (ROCm runs these
    # device-to-host copies as blit kernels on the CUs), without the harness
    pipe = next(iter(model._pipelines.values()))[1]
    t_arg = torch.tensor([scene.cfg.t], device=dev)
    for _ in range(2):
        pipe.submit(t_arg)
    pipe.join()
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    for _ in range(n_views):
        pipe.submit(t_arg)
    pipe.join()
    torch.cuda.synchronize(dev)
    bare = (time.perf_counter() - t1) / n_views * 1e3
    return {"views": n_views, "distinct_times": n_views, "frames_in_flight": in_flight,
            "ms_per_frame": el / n_views * 1e3, "rays_per_s": n_views * H * W / el,
            "pipeline_readback_ms_per_frame": bare,
            "note": "harness.render_viewpoints over views at distinct times and camera poses, one model (apn_amd.pipeline."
                    "FramePipeline: per-frame workspaces, shared canonical tables / projection), per view: rays "
                    "on the device, frame submitted, rgb / depth / weights read back to host numpy; second call "
                    "timed (the first captures)"}


def frame_rate(config, dev, steps=16, warmup=2, in_flight=3, n_views=16):
    """One GPU, one config (C3 / C4): whole frames replayed as HIP graphs over n_views distinct
    views (time and camera pose per frame), as the headline line, plus the MLP kernel's time from
    HIP events on eager frames of the same views and its F_alg roofline fraction. Rides along in
    the default line (`other_configs`), so every config has a driver-run number."""
    scene = S.make_scene(config)
    model = harness.build_model(scene, dev)
    rk = scene.render_kwargs(dev)
    R = rk["rays_o"].shape[0]
    t_arg = torch.tensor([scene.cfg.t], device=dev)
    poses, Ks = scene.c2w[None].to(dev), scene.K[None].to(dev)
    views = S.view_sweep(scene, n_views, dev)

    def kw(v):
        return dict(render_depth=True, render_kwargs=view_rk(rk, v), render_weights=True, poses=v.c2w[None],
                    Ks=v.K[None], get_skeleton=True)
    for i in range(warmup):
        model(views[i % n_views].t, **kw(views[i % n_views]))
    torch.cuda.synchronize(dev)
    stats = model.last_stats.resolved()
    presize_capacity(model, views, rk)
    model.timing = {}
    for i in range(5):
        model(views[i % n_views].t, **kw(views[i % n_views]))
    torch.cuda.synchronize(dev)
    timing, model.timing = model.timing, None
    ev = timing.get("mlp_events", [])
    mlp_ms = sum(e[0].elapsed_time(e[1]) for e in ev) / max(len(ev), 1)
    kept = mean_kept(ev, stats.get("kept_samples", 0))
    rows = mlp_pass_rows(ev, kept)
    pms = mlp_pass_ms(timing)
    if pms is not None:
        mlp_ms = sum(pms)
    from apn_amd.pipeline import FramePipeline
    pipe = FramePipeline(model, t_arg, rk, n=in_flight, poses=poses, Ks=Ks, get_skeleton=True, readback=None)
    replay_pipeline(pipe, views, n_views)
    pipe.overflowed()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    replay_pipeline(pipe, views, steps)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    overflowed = pipe.overflowed()
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    replay_pipeline(pipe, views[:1], steps)
    torch.cuda.synchronize(dev)
    same_view_ms = (time.perf_counter() - t1) / steps * 1e3
    d_in = 191 + model.pose_embedding_dim
    achieved = sum(rows) * flop_per_kept_sample(d_in) / (mlp_ms * 1e-3) / 1e12 if mlp_ms > 0 else 0.0
    return {"workload": S.CONFIGS[config].name + f" ({config})", "value": steps * R / elapsed, "unit": "rays/s",
            "ms_per_step": elapsed / steps * 1e3, "steps": steps, "rays_per_frame": R, "points": scene.cfg.N,
            "bones": scene.cfg.J, "inbbox_samples": stats.get("inbbox_samples"), "kept_samples": kept,
            "mlp_rows_per_pass": rows, "mlp_samples": sum(rows), "distinct_views": n_views,
            "same_view_ms_per_step": same_view_ms,
            "timed_frames_overflowed": overflowed, "frames_in_flight": pipe.n,
            "mlp_kernel_ms": mlp_ms, "mlp_roofline_frac": achieved / SPLIT3_PEAK_TFLOPS}


def other_configs(dev, in_flight=3):
    """C3, C4 (frames) and C5 (repose sweep) on this GPU, compact; a failure is reported, never fatal."""
    out = {}
    for cfg in ("C3", "C4"):
        try:
            out[cfg] = frame_rate(cfg, dev, in_flight=in_flight)
            log(f"[other configs] {cfg}: {out[cfg]['value'] / 1e6:.1f} M rays/s, {out[cfg]['ms_per_step']:.2f} ms/frame")
        except Exception as e:
            out[cfg] = {"error": repr(e)}
        torch.cuda.empty_cache()
    try:
        a = argparse.Namespace(config="C5", steps=300, warmup=3, no_cpu_baseline=True, repose_in_flight=4)
        c5 = lbs_sweep(a, 0, 1, dev)
        out["C5"] = {"workload": c5["config"]["workload"], "value": c5["value"], "unit": c5["unit"],
                     "ms_per_step": c5["ms_per_step"], "steps": a.steps, "lbs_kernel_ms": c5["config"]["lbs_kernel_ms"],
                     "lbs_roofline_frac": c5["roofline"]["frac"], "lbs_bytes_per_launch": c5["roofline"]["bytes_per_launch"]}
        log(f"[other configs] C5: {c5['value'] / 1e9:.2f} G points/s, LBS {c5['config']['lbs_kernel_ms']:.4f} ms")
    except Exception as e:
        out["C5"] = {"error": repr(e)}
    try:   # the train_pcd step (tools/train_bench.py) at C2, 8192 rays
        import importlib.util
        spec = importlib.util.spec_from_file_location("train_bench", os.path.join(ROOT, "tools", "train_bench.py"))
        tb = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(tb)
        with torch.enable_grad():
            tr = tb.run(argparse.Namespace(config="C2", steps=20, warmup=5, n_rand=8192, no_cpu_baseline=True))
        out["train_C2"] = {k: tr[k] for k in ("metric", "value", "unit", "ms_per_step", "stage_ms", "steps")}
        log(f"[other configs] train C2: {tr['ms_per_step']:.2f} ms/step")
    except Exception as e:
        out["train_C2"] = {"error": repr(e)}
    torch.cuda.empty_cache()
    out["note"] = ("one GPU each, after the headline run: C3/C4 = whole frames replayed as one HIP graph (10 timed), "
                   "MLP kernel ms from HIP events on 5 eager frames; C5 = 300 poses of the repose sweep graph, LBS "
                   "kernel from a graph of 20 launches (bench.py --config C5 gives the full line); train_C2 = 20 timed "
                   "train_pcd steps (forward with autograd, all default losses, backward, MaskedAdam)")
    return out


def frame_roofline(N, J, R, f_alg, ms_per_step, gpus=1):
    """SURVEY.md 8(d) binding fraction of the whole frame: t_roofline / t with t_roofline =
    max(B_alg / BW, F_alg / P) over the frame's GPUs. B_alg = N(60 + 4J) (LBS) + N(580 + 4J)
    (per-point tables once) + 36 R (rays) + 48 R (outputs); F_alg = the neighbour MLP's reference
    flops over all kept samples; P = the split-MFMA fp32-equivalent peak (fp16 dense / 3). The kNN's
    VALU work has no F_alg term: its time is part of the lost fraction."""
    b_alg = N * (60 + 4 * J) + N * (580 + 4 * J) + 36 * R + 48 * R
    t_hbm = b_alg / (HBM_PEAK_GBS * 1e9 * gpus) * 1e3
    t_mfma = f_alg / (SPLIT3_PEAK_TFLOPS * 1e12 * gpus) * 1e3
    t_fp32 = f_alg / (FP32_MFMA_PEAK_TFLOPS * 1e12 * gpus) * 1e3
    t_roof = max(t_hbm, t_mfma)
    return {"t_roofline_ms": t_roof, "bound": "mfma" if t_mfma >= t_hbm else "hbm", "frac": t_roof / ms_per_step,
            "b_alg_bytes": b_alg, "f_alg_flop": f_alg, "t_hbm_ms": t_hbm, "t_mfma_ms": t_mfma, "gpus": gpus,
            "frac_vs_fp32_matrix_peak": t_fp32 / ms_per_step,
            "note": "t_roofline = max(B_alg/8 TB/s, F_alg/833 TF) over the frame's GPUs (SURVEY.md 8(d)); "
                    "frac_vs_fp32_matrix_peak prices F_alg at the 157.3 TF FP32 matrix peak instead (> 1: the "
                    "kernel does not run on fp32 MFMA)"}


def latest_traffic(stem):
    """The newest committed PMC traffic summary profiles/rNN_<stem>.json -> (dict, relative path)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r[0-9][0-9]_{stem}.json")))
    for path in reversed(files):
        t = read_traffic(path)
        if t:
            return t, os.path.relpath(path, ROOT)
    return None, None


def knn_report(model, S_kept, inbbox, knn_ms):
    """The kNN next to its work (apn_amd/knn_work.py): the perfect-scan work of
    this frame's survivors and its VALU-issue floor, and the executed VALU instructions of the kNN
    kernels from the newest committed PMC summary (labelled with its file: not measured in this run)."""
    from apn_amd.knn_work import knn_work, valu_issue_ms
    import glob
    bufs = model._ws.bufs
    if not all(k in bufs for k in ("sorted4", "s_pos", "s_nbr")) or S_kept <= 0:
        return None
    s4 = bufs["sorted4"].view(-1, 4)
    idx = s4[:, 3].contiguous().view(torch.int32).long()
    cloud = torch.empty(s4.shape[0], 3, device=s4.device)
    cloud[idx] = s4[:, :3]
    w = knn_work(cloud, bufs["s_pos"].view(-1, 4)[:S_kept, :3], bufs["s_nbr"].view(-1, 8)[:S_kept],
                 0.01)   # the frame's query_radius (forward's default, which bench renders with)
    out = {"ms": round(knn_ms, 4), "queries": inbbox, "survivors": S_kept, "perfect_scan": w,
           "note": "perfect scan = survivors' final-ball x-chord rows/points on an r/8 grid (7 VALU lane ops per "
                   "point, 4 per row), rejected samples 0 points; floor_ms = its VALU issue time at the PMC clock"}
    # newest round first and, within a round, its final-state summary
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_pmc_summary_c2*.json")),
                   key=lambda f: (os.path.basename(f)[:3], "final" in os.path.basename(f), f))
    for path in reversed(files):
        pmc = read_traffic(path) or {}
        ks = {k: v for k, v in pmc.items() if ("knn" in k or "cell_bound" in k or "classify" in k)
              and "SQ_INSTS_VALU" in v}
        if not ks:
            continue
        clk = max(v.get("eff_clock_GHz", 2.4) for v in ks.values())
        insts = sum(v["SQ_INSTS_VALU"] for v in ks.values())
        out.update({"floor_ms": round(valu_issue_ms(w["valu_lane_ops"], clk), 4),
                    "executed_valu_insts": insts,
                    "executed_issue_ms": round(insts * 2 / 1024 / (clk * 1e9) * 1e3, 4),
                    "lane_efficiency": w["valu_lane_ops"] / (64 * insts),
                    "pmc_source": os.path.relpath(path, ROOT) + " (kNN kernels' SQ_INSTS_VALU per launch, "
                                                                 "earlier run, not this one)"})
        out["floor_frac"] = out["floor_ms"] / knn_ms if knn_ms > 0 else None
        break
    return out


def read_traffic(path):
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); N > 1 without an outer launcher starts the N ranks itself; "
                         "under one it must equal WORLD_SIZE")
    ap.add_argument("--steps", type=int, default=16)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--views", type=int, default=16,
                    help="distinct frames the timed loop cycles through, each a new time and camera pose as in "
                         "the reference's render loop (synthetic.view_sweep); 1 = replay the scene's own frame")
    ap.add_argument("--cpu-rows", type=int, default=48, help="image rows in the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-other-configs", action="store_true",
                    help="skip the compact C3 / C4 / C5 measurements the default one-GPU C2 line carries")
    ap.add_argument("--no-full-mlp-leg", action="store_true",
                    help="skip timing the same frames without early ray termination (full_mlp_ms_per_step)")
    ap.add_argument("--no-viewpoints", action="store_true",
                    help="skip the harness.render_viewpoints leg (8 views, frames in flight, host readback)")
    ap.add_argument("-o", "--out", default=None, help="also write the JSON line to this file")
    ap.add_argument("--repose-mode", choices=["batched", "per_pose", "pipelined"], default="batched",
                    help="C5: the captured repose step (TemporalPoints.capture_repose): batched = one skeleton "
                         "launch per pass over the sweep + one LBS graph per pose; per_pose = skeleton + LBS per "
                         "pose; pipelined = pose i's LBS beside pose i + 1's skeleton")
    ap.add_argument("--repose-in-flight", type=int, choices=[1, 2, 3, 4], default=4,
                    help="C5, batched: poses in flight (pose i on stream i %% n into output slot i %% n, "
                         "TemporalPoints.capture_repose(in_flight=n)); same box: 1: 0.0400-0.0403 ms per pose, "
                         "2: 0.0412-0.0414, 3: 0.0345-0.0363, 4: 0.0340 (profiles/r06_c5_inflight.log)")
    ap.add_argument("--shard", choices=["frames", "rays"], default="rays",
                    help="N>1: 'rays' (default) = the ranks split one frame's rays and all-gather the tiles "
                         "over RCCL (strong scaling, SURVEY.md 8(e)); 'frames' = every rank renders its own "
                         "frame (weak scaling, no data-path collective)")
    ap.add_argument("--in-flight", type=int, choices=[1, 2, 3, 4, 5, 6], default=None,
                    help="frames in flight: one model's frame captured into n workspaces, frame i on stream i %% n "
                         "(ray shards: the all-gathers in frame order on one collective stream); 1 = one "
                         "after another. Default 4 (C2, same box, 3 rounds: 4.96-5.07 vs 5.05-5.17 ms per frame at "
                         "3, profiles/r06_frame_inflight.log; a ray shard of 8: 0.945 vs 0.985 ms, shards of 2 / 4 "
                         "equal, 6 slower, profiles/r06_shard_inflight.log)")
    ap.add_argument("--graph", choices=["auto", "on", "off"], default="auto",
                    help="replay the frame as one HIP graph (TemporalPoints.capture_frame; with --shard rays "
                         "each rank's blocks, shard.capture_sharded); auto = on unless the ranks use the "
                         "'ranges' ray split (APN_SHARD_SPLIT=ranges: its split moves per frame)")
    args = ap.parse_args()
    torch.set_grad_enabled(False)   # a render benchmark: the reference renders under no_grad (run.py:80, 241)

    world = check_world(args.gpus, os.environ)
    if args.in_flight is None:
        args.in_flight = 4
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; APN_DIST_BACKEND=gloo rehearses N>1 with several ranks on one card
    local = local % max(torch.cuda.device_count(), 1)
    backend = os.environ.get("APN_DIST_BACKEND", "nccl")   # nccl = RCCL over xGMI
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group(backend)
    backend = "RCCL (xGMI)" if backend == "nccl" else backend
    dev = torch.device("cuda", local)

    if args.config == "C5":
        line = lbs_sweep(args, rank, world, dev)
        if line is not None:
            emit(line, args)
        if world > 1:
            torch.distributed.destroy_process_group()
        return
    scene = S.make_scene(args.config)
    shard_rays = args.shard == "rays" and world > 1
    if not shard_rays:  # weak scaling: every rank renders its own frame time
        scene.cfg.t = scene.cfg.t + 0.05 * rank
    t_setup = time.perf_counter()
    model = harness.build_model(scene, dev)
    rk = scene.render_kwargs(dev)
    R = rk["rays_o"].shape[0]
    t_arg = torch.tensor([scene.cfg.t], device=dev)
    _ = model.mean_min_distance
    torch.cuda.synchronize(dev)
    log(f"[rank {rank}] setup {time.perf_counter() - t_setup:.2f}s, rays/frame {R}")

    poses, Ks = scene.c2w[None].to(dev), scene.K[None].to(dev)
    from apn_amd import shard as SH
    # the blocks ray split captures each rank's frame as a graph; the ranges split moves per frame
    use_graph = args.graph == "on" or (args.graph == "auto" and not (shard_rays and SH.DEFAULT_SPLIT == "ranges"))
    # the render loop's frames: a new time and camera pose per frame (run.py:108-151), inputs on the device
    views = S.view_sweep(scene, max(1, args.views), dev)

    def eager_step(i=0):
        v = views[i % len(views)]
        if shard_rays:
            from apn_amd.shard import render_sharded
            return render_sharded(model, v.t, view_rk(rk, v), rank, world, poses=v.c2w[None], Ks=v.K[None],
                                  get_skeleton=True)
        return model(v.t, render_depth=True, render_kwargs=view_rk(rk, v), render_weights=True, poses=v.c2w[None],
                     Ks=v.K[None], get_skeleton=True)

    for i in range(args.warmup):
        eager_step(i)
    torch.cuda.synchronize(dev)
    stats = model.last_stats.resolved()
    if len(views) > 1 and use_graph:
        presize_capacity(model, views, rk, (rank, world, SH.RAY_BLOCK) if shard_rays else None)
        torch.cuda.synchronize(dev)
    log(f"[rank {rank}] scene: {stats}")
    shard_graphs, pipe, mem = [], None, {}
    mem["model_bytes"] = torch.cuda.memory_allocated(dev)
    if use_graph and shard_rays:   # this rank's blocks as one graph replay, then the tile all-gather
        try:
            # frames in flight: n shard graphs of this one model, each captured into its own
            # per-frame workspace (apn_amd.pipeline)
            from apn_amd.pipeline import capture_sharded_in_flight
            shard_graphs = capture_sharded_in_flight(model, t_arg, rk, rank, world, n=args.in_flight, poses=poses,
                                                     Ks=Ks, get_skeleton=True)
            graph_step = shard_graphs[0]
        except Exception as e:   # the eager shard frame runs the same kernels and the same collectives
            log(f"[rank {rank}] shard graph capture failed ({e!r}); timing eager shard frames")
            use_graph = False
            shard_graphs = []
            torch.cuda.synchronize(dev)
        # every rank must run the same step (same collectives): graphs only if all ranks captured
        ok = torch.tensor([1 if use_graph else 0], dtype=torch.int32,
                          device=dev if torch.distributed.get_backend() == "nccl" else "cpu")
        torch.distributed.all_reduce(ok, op=torch.distributed.ReduceOp.MIN)
        use_graph = bool(ok.item())
    streams = None
    if use_graph:   # the whole frame as one HIP graph replay (no per-kernel host launches, no host sync)
        if not shard_rays:
            # n frames in flight on this one model (apn_amd.pipeline.FramePipeline): n captures of the
            # frame, each in a per-frame workspace of its own, frame i on stream i % n
            from apn_amd.pipeline import FramePipeline
            pipe = FramePipeline(model, t_arg, rk, n=args.in_flight, poses=poses, Ks=Ks, get_skeleton=True,
                                 readback=None)
            replay_pipeline(pipe, views, max(2, len(views)))
            pipe.overflowed()   # clears the flag: the timed frames' own is read after the loop
        else:
            streams = [torch.cuda.Stream(dev) for _ in shard_graphs]
            comm = torch.cuda.Stream(dev)
            replay_sharded(shard_graphs, views, max(2, len(views)), streams, comm)
            for g in shard_graphs:
                g.overflowed()
        torch.cuda.synchronize(dev)
    mem["with_frames_in_flight_bytes"] = torch.cuda.memory_allocated(dev)
    mem["per_frame_workspace_bytes"] = ([sum(b.numel() * b.element_size() for b in ws.bufs.values())
                                         for ws in pipe.workspaces] if pipe is not None else None)

    # stage / MLP-kernel timings come from HIP events on eager frames (events are not recorded
    # inside a graph replay); the timed loop below runs the step as configured
    model.timing = {}
    if use_graph:
        for i in range(min(args.steps, 10)):
            eager_step(i)
        torch.cuda.synchronize(dev)
    timing, model.timing = model.timing, None
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    host_s = 0.0
    if not use_graph:
        model.timing = timing
    eager_infos = []
    if pipe is not None:   # captured frames without a collective, n in flight on one model
        out, host_s = replay_pipeline(pipe, views, args.steps)
    elif use_graph:   # ray shards, frames in flight, one collective stream
        out, host_s = replay_sharded(shard_graphs, views, args.steps, streams, comm)
    else:
        for i in range(args.steps):
            h0 = time.perf_counter()
            out = eager_step(i)
            host_s += time.perf_counter() - h0
            if model._last_info is not None:
                eager_infos.append(model._last_info)
    torch.cuda.synchronize(dev)
    if not use_graph:
        timing, model.timing = model.timing, None
    # the timed frames are never read: a replay that dropped samples past the captured capacity
    # would be timed short. The graph ORs every replay's overflow flag on the device; read it once.
    # (eager frames: the device frame_info of each timed frame, kept by the loop below)
    if use_graph:
        overflowed = pipe.overflowed() if pipe is not None else any([bool(g.overflowed()) for g in shard_graphs])
    else:
        overflowed = any(bool(i[2]) for i in torch.stack(eager_infos).cpu()) if eager_infos else False
    n_timed = min(args.steps, 10) if use_graph else args.steps
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed, float(overflowed)], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed, overflowed = float(t[0]), bool(t[1] > 0)
    if overflowed:
        log(f"[rank {rank}] WARNING: a timed frame overflowed its sample capacity (dropped samples)")
    serial_ms = same_view_ms = None
    n_flight = pipe.n if pipe is not None else (len(shard_graphs) if use_graph else 1)

    def timed(fn):
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize(dev)
        a = time.perf_counter()
        fn()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - a) / args.steps * 1e3
    if pipe is not None:
        # the same views one frame at a time (each frame waits for the previous one): the
        # reference for the in-flight gain; and view 0 replayed every frame (the earlier headline)
        serial_ms = timed(lambda: replay_pipeline(pipe, views, args.steps, serial=True))
        same_view_ms = timed(lambda: replay_pipeline(pipe, views[:1], args.steps))
        log(f"[rank {rank}] frames in flight {n_flight}, {len(views)} distinct views: "
            f"{elapsed / args.steps * 1e3:.3f} ms/frame; one at a time {serial_ms:.3f} ms/frame; "
            f"view 0 only {same_view_ms:.3f} ms/frame")
    elif use_graph and len(views) > 1:
        same_view_ms = timed(lambda: replay_sharded(shard_graphs, views[:1], args.steps, streams, comm))
    full_mlp_ms = None
    if world == 1 and pipe is not None and model.early_termination and not args.no_full_mlp_leg:
        # the same frames with the neighbour MLP on EVERY kept sample (the reference's work: no early
        # ray termination), n in flight on their own pipeline: the gain of apn_point_mlp_ert
        from apn_amd.pipeline import FramePipeline
        model.early_termination = False
        try:
            pfull = FramePipeline(model, t_arg, rk, n=args.in_flight, poses=poses, Ks=Ks, get_skeleton=True,
                                  readback=None)
            replay_pipeline(pfull, views, 2)
            torch.cuda.synchronize(dev)
            tf0 = time.perf_counter()
            replay_pipeline(pfull, views, args.steps)
            torch.cuda.synchronize(dev)
            full_mlp_ms = (time.perf_counter() - tf0) / args.steps * 1e3
            del pfull
        finally:
            model.early_termination = True
        log(f"[rank {rank}] full MLP (no early ray termination): {full_mlp_ms:.3f} ms/frame")
    from apn_amd import _lib
    lib = _lib.load()
    debug_lib = hasattr(lib, "apn_debug_knn_stats")   # APN_HIP_LIB = libapn_hip_debug.so (tools/ A/B runs)
    variant = int(lib.apn_set_mlp_variant(-1))        # the library's kernel selection (out of range: query)
    if debug_lib and variant in (2, 3, 5):   # timed MLP variants of the debug build: per-phase cycle split
        import ctypes
        ph = (ctypes.c_uint64 * 6)()
        _lib.call("apn_debug_mlp_phase_cycles", ph)
        tot = sum(ph[:4]) or 1
        log("[mlp phases] " + ", ".join(f"{n} {100 * ph[i] / tot:.1f}%" for i, n in
                                        enumerate(["gather", "layer1", "layers2-4", "epilogue"]))
            + f"; cycles/tile {tot / max(ph[4], 1):.0f}, in-loop share {tot / max(ph[5], 1):.3f}")
    stage_ms = {}
    marks = timing.get("marks", [])
    for (_, a), (name, b) in zip(marks[:-1], marks[1:]):
        if name != "frame":
            stage_ms[name] = stage_ms.get(name, 0.0) + a.elapsed_time(b) / n_timed
    log(f"[rank {rank}] stage ms/frame (HIP events, eager frames): " + ", ".join(f"{k} {v:.3f}" for k, v in stage_ms.items()))
    ev = timing.get("mlp_events", [])
    mlp_ms = sum(e[0].elapsed_time(e[1]) for e in ev) / max(len(ev), 1)
    S_last = int(ev[-1][2].item()) if ev else stats.get("kept_samples", 0)   # the last eager frame's
    S_kept = mean_kept(ev, S_last)   # per frame, over the timed eager frames' views
    pass_rows = mlp_pass_rows(ev, S_kept)
    S_mlp = sum(pass_rows)   # the samples the MLP ran on (early ray termination: those the compositing reads)
    mlp_stage_ms = mlp_ms
    pass_ms = mlp_pass_ms(timing)
    if pass_ms is not None:   # the MLP kernel launches alone (HIP events around each pass's launches)
        mlp_ms = sum(pass_ms)
    kept_total = S_kept * (world if not shard_rays else 1)
    shard_diag = None
    if shard_rays:
        # N>1 diagnostics: every rank's stage times, the tile all-gather alone (HIP events around
        # the collective on the current stream, this frame's tile shape) and the per-frame work every
        # rank replicates (skinning, bbox, kNN grid build)
        from apn_amd.shard import RAY_BLOCK, TILE_WIDTH, gather_blocks
        n_local = model.last_ray_count
        tile = torch.zeros(n_local, TILE_WIDTH, device=dev)
        info = torch.zeros(4, dtype=torch.int32, device=dev)
        gather_blocks(tile, R, world, RAY_BLOCK, info=info)
        torch.distributed.barrier()
        g0, g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        g0.record()
        for _ in range(10):
            gather_blocks(tile, R, world, RAY_BLOCK, info=info)
        g1.record()
        torch.cuda.synchronize(dev)
        ag_ms = g0.elapsed_time(g1) / 10
        mine = {"rank": rank, "world_size": torch.distributed.get_world_size(), "device": device_identity(dev),
                "rays": n_local, "kept_samples": S_kept, "mlp_samples": S_mlp, "allgather_ms": round(ag_ms, 4),
                "replicated_ms": round(sum(stage_ms.get(k, 0.0) for k in ("lbs", "bbox", "grid")), 4),
                "stage_ms": {k: round(v, 4) for k, v in stage_ms.items()}}
        per_rank = [None] * world
        torch.distributed.all_gather_object(per_rank, mine)
        kept_total = sum(p["kept_samples"] for p in per_rank)
        shard_diag = {"per_rank": per_rank, "allgather_ms_max": max(p["allgather_ms"] for p in per_rank),
                      "world_size": torch.distributed.get_world_size(),
                      "distinct_devices": len({(p["device"].get("hostname"), p["device"].get("pci_bus_id"),
                                                p["device"].get("uuid")) for p in per_rank}),
                      "rerenders": getattr(model, "sharded_rerenders", 0),
                      "note": "stage_ms from HIP events on eager shard frames; allgather_ms = one gather_blocks "
                              "(the frame's tile all-gather) alone, mean of 10; replicated_ms = lbs + bbox + grid, "
                              "the per-frame stages every rank runs on the whole cloud"}
        log(f"[rank {rank}] all-gather {ag_ms:.3f} ms/frame, replicated stages {mine['replicated_ms']:.3f} ms/frame")
    log(f"[rank {rank}] host time inside step() {1e3 * host_s / args.steps:.3f} ms/step "
        f"({'graph replay' if use_graph else 'eager launches'}; device {1e3 * elapsed / args.steps:.3f} ms/step)")
    if debug_lib and os.environ.get("APN_KNN_MODE") == "3":   # kNN query-class counters (debug build)
        import ctypes
        st = (ctypes.c_uint64 * 20)()
        _lib.call("apn_debug_knn_stats", st)
        names = ["stop2h", "chord_reject", "stop4h", "stop_r", "reject_r"]
        tot_cyc = sum(st[4 * i + 1] for i in range(5)) or 1
        for i, nm in enumerate(names):
            n = st[4 * i] or 1
            log(f"[knn {nm}] queries/frame {st[4 * i] / args.steps:.0f} cycles share {100 * st[4 * i + 1] / tot_cyc:.1f}% "
                f"cycles/query {st[4 * i + 1] / n:.0f} rows/query {st[4 * i + 2] / n:.1f} pts/query {st[4 * i + 3] / n:.1f}")
    if debug_lib and os.environ.get("APN_KNN_STATS"):   # mode-8/9 pass-B counters (per hard list, debug build)
        import ctypes
        st = (ctypes.c_uint64 * 20)()
        _lib.call("apn_debug_knn_stats", st)
        n = args.steps + args.warmup
        for lst, nm in enumerate(["from r/2", "from r"]):
            v = st[10 * lst: 10 * lst + 9]
            q = max(v[0], 1)
            log(f"[knn pass B {nm}] queries/frame {v[0] / n:.0f}, done at r/2 {v[1] / q:.3f}, survive {v[2] / q:.3f}, "
                f"r/2 scan rows+pts iters/query {v[3] / q:.1f}+{v[4] / q:.1f}, r scan {v[5] / q:.1f}+{v[6] / q:.1f}, "
                f"rejected after full r scan {v[7] / q:.3f} ({v[8] / max(v[7], 1):.1f} iters each)")
    if rank != 0:
        if world > 1:
            torch.distributed.destroy_process_group()
        return

    d_in = 191  # pose embedding folded into the bias for ZJU; F_alg still counts the reference D_in
    if model.pose_embedding_dim > 0:
        d_in = 191 + model.pose_embedding_dim
    flop = S_mlp * flop_per_kept_sample(d_in)
    achieved = flop / (mlp_ms * 1e-3) / 1e12 if mlp_ms > 0 else 0.0
    executed = (sum(mfma_executed_flop(int(round(r)), variant) for r in pass_rows) / (mlp_ms * 1e-3) / 1e12
                if mlp_ms > 0 else 0.0)
    if variant in (1, 2):
        kernel, peak, mfma_peak = "k_point_mlp (fp32 MFMA)", FP32_MFMA_PEAK_TFLOPS, FP32_MFMA_PEAK_TFLOPS
        peak_note = "peak = FP32 matrix peak"
    else:
        kernel = ("k_point_mlp_h4 (3-term fp16-split MFMA, 128-row tiles)" if variant in (0, 5)
                  else "k_point_mlp_h3 (3-term fp16-split MFMA, 64-row tiles)")
        peak, mfma_peak = SPLIT3_PEAK_TFLOPS, FP16_MFMA_PEAK_TFLOPS
        peak_note = "peak = fp16 dense MFMA peak / 3 (three fp16 MFMA terms per fp32-accurate product)"
    from apn_amd.ops import mlp_range_fallback
    # the split kernel's range guard hands a launch to the FP32 MFMA kernel; the line says if it fired
    wss = [model._ws_eager] + (pipe.workspaces if pipe is not None else [])
    mlp_fallback = (any(bool(mlp_range_fallback(w.bufs["mlp_w"])) for w in wss if "mlp_w" in w.bufs)
                    if any("mlp_w" in w.bufs for w in wss) else None)
    traffic, traffic_src = latest_traffic("point_mlp_traffic")
    ms_per_step = elapsed / args.steps * 1e3
    mlp_total = kept_total if len(pass_rows) == 1 else (S_mlp if shard_rays else S_mlp * world)
    if shard_rays and len(pass_rows) > 1:
        mlp_total = sum(p.get("mlp_samples", p["kept_samples"]) for p in shard_diag["per_rank"])
    frame_roof = frame_roofline(scene.cfg.N, scene.cfg.J, R, mlp_total * flop_per_kept_sample(d_in), ms_per_step,
                                world if shard_rays else 1)
    value = (1 if shard_rays else world) * args.steps * R / elapsed
    cpu = psnr = same = None
    if world == 1 and not args.no_cpu_baseline:
        # the frame the oracle legs compare: view 0 (the scene's own time and camera)
        if pipe is not None:
            h = submit_view(pipe, views, 0)
            pipe.join()
            out = h.device()
        else:
            out = eager_step(0)
        torch.cuda.synchronize(dev)
        try:
            cpu, ref, sel, (orc, sub, t_cpu) = cpu_baseline(model, scene, args.cpu_rows, torch.get_num_threads())
            psnr = psnr_vs_oracle(out, ref, sel)
            same = same_cloud_error(out, rk, model.last_palette_perm, orc, sub, t_cpu, sel)
        except Exception as e:  # never lose the GPU line over the baseline leg
            log(f"cpu baseline failed: {e!r}")
    knn = None
    if world == 1:
        try:
            knn = knn_report(model, S_last, stats.get("inbbox_samples"), stage_ms.get("knn", 0.0))
        except Exception as e:  # never lose the GPU line over a diagnostic
            log(f"knn work report failed: {e!r}")
    vp = None
    if world == 1 and use_graph and not args.no_viewpoints:
        try:
            vp = viewpoint_rate(model, scene, dev, in_flight=args.in_flight)
            log(f"[render_viewpoints] {vp['ms_per_frame']:.3f} ms/frame over {vp['views']} views "
                f"({vp['frames_in_flight']} in flight, host readback)")
        except Exception as e:  # never lose the GPU line over a diagnostic
            log(f"render_viewpoints leg failed: {e!r}")
    others = None
    if world == 1 and args.config == "C2" and not args.no_other_configs:
        others = other_configs(dev, args.in_flight)
    line = {
        "metric": f"rendered rays/sec at {scene.cfg.W}x{scene.cfg.H}, {scene.cfg.N // 1000}k pts, {scene.cfg.J} bones",
        "value": value, "unit": "rays/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": ms_per_step, "higher_is_better": True,
        "scaling": "strong" if shard_rays else "weak", "vs_baseline": None,
        "dtype": "fp32", "data": "synthetic (procedural SMPL-24 capsule cloud, random-init networks)",
        "library": lib.apn_version().decode(),
        "mlp_arithmetic": ("fp32 as 3 fp16 MFMA terms (hi*hi+hi*lo+lo*hi), fp32 accumulate; parity vs the fp32 "
                           "oracle <= 3e-7 on alpha/rgb" if variant in (0, 3, 4, 5) else "fp32 MFMA (v_mfma_f32_16x16x4_f32)"),
        "config": {"workload": S.CONFIGS[args.config].name + f" ({args.config})", "rays_per_frame": R,
                   "points": scene.cfg.N, "bones": scene.cfg.J, "inbbox_samples": stats.get("inbbox_samples"),
                   "kept_samples": S_kept,
                   "early_ray_termination": len(pass_rows) > 1,
                   "mlp_samples": S_mlp, "mlp_rows_per_pass": pass_rows,
                   "parallelism": (f"rays x{world} ({SH.DEFAULT_SPLIT} split"
                                   + (f" of {SH.RAY_BLOCK}-ray blocks" if SH.DEFAULT_SPLIT == "blocks" else "")
                                   + f") + {backend} all_gather_into_tensor of the per-ray tiles"
                                   if shard_rays else f"frames x{world} (no data-path collective)")
                   if world > 1 else "single",
                   "step": (("each rank's blocks replayed as one HIP graph (shard.capture_sharded), then the "
                             "all-gather" + (f"; {n_flight} frames in flight (one model's shard graphs, each in its "
                                             "own per-frame workspace, on as many streams, the all-gathers in frame "
                                             "order on one collective stream)" if n_flight > 1 else "") if shard_rays
                             else "whole frame replayed as one HIP graph (TemporalPoints.capture_frame)"
                             + (f"; {n_flight} frames in flight on ONE model (apn_amd.pipeline.FramePipeline: the "
                                "frame captured into n per-frame workspaces, canonical tables and the layer-1 "
                                "projection shared; frame i on stream i % n)" if n_flight > 1 else "")) if use_graph
                            else "eager launches"),
                   "frames_in_flight": n_flight,
                   "distinct_views": len(views),
                   "views": ("every timed frame a new view, cycling through the distinct_views frames of "
                             "synthetic.view_sweep: time t0 + 0.6 i / n and the camera orbited by 360 i / n "
                             "degrees about the subject (view 0 = t 0.3, the scene's camera); the view's rays, "
                             "pose and intrinsics, resident on the device, copied into the frame's input buffers "
                             "per frame" if len(views) > 1 else "one view replayed"),
                   "same_view_ms_per_step": same_view_ms,
                   "memory": mem,
                   "serial_ms_per_step": serial_ms,
                   "full_mlp_ms_per_step": full_mlp_ms,
                   "timed_frames_overflowed": overflowed,
                   "mlp_fp32_fallback_fired": mlp_fallback},
        "roofline": {"bound": "mfma", "kernel": kernel, "achieved": achieved, "peak": peak,
                     "unit": "TFLOP/s", "frac": achieved / peak,
                     "traffic": traffic.get("bytes_per_launch") if traffic else None,
                     "traffic_source": (f"{traffic_src}: PMC passes (FETCH_SIZE / WRITE_SIZE, gfx950 read "
                                        f"correction) over bench.py on an earlier build (kernel avg "
                                        f"{traffic.get('avg_ms', float('nan')):.2f} ms then); NOT measured in this run"
                                        if traffic else None),
                     "flop_per_launch": flop, "avg_launch_ms": mlp_ms,
                     "per_pass": ({"rows": pass_rows, "ms": [round(v, 4) for v in pass_ms]} if pass_ms else None),
                     "mlp_stage_ms": mlp_stage_ms,
                     "note": "achieved = reference F_alg (SURVEY.md 8(d), fp32 flops) per sample x the samples the "
                             "MLP kernel ran on in the frame (mlp_samples: with early ray termination the kept "
                             "samples the compositing reads, over the passes' launches) / those launches' summed "
                             "time (avg_launch_ms: HIP events recorded by apn_point_mlp_ert on the launch stream "
                             "around each pass's launches, mean over the timed eager frames; per_pass lists both); "
                             "mlp_stage_ms = the whole stage (direct-blend kernel, pass-list kernels, launches); "
                             + peak_note + "; the kernel issues fewer MFMA flops than F_alg (per-point layer-1 "
                             "projection, folded rgb head): executed_tflops / mfma_util",
                     "executed_tflops": executed,
                     "mfma_util": executed / mfma_peak},
        "frame_roofline_frac": frame_roof["frac"],
        "frame_roofline": frame_roof,
        "stage_ms": {k: round(v, 4) for k, v in stage_ms.items()},
        **({"knn": knn} if knn is not None else {}),
        **({"shards": shard_diag} if shard_diag is not None else {}),
        "cpu_baseline": cpu,
        "psnr_vs_oracle": psnr,
        "same_cloud_vs_oracle": same,
        **({"render_viewpoints": vp} if vp is not None else {}),
        **({"other_configs": others} if others is not None else {}),
    }
    emit(line, args)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
