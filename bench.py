#!/usr/bin/env python
"""bench.py — forward+backward renders/s of the DGE 3DGS rasterizer hot path.

Workload (BASELINE.json configs[1], "c2"): 1.0M Gaussians (SH degree 3),
512x512, fp32, one render() forward + its backward per view, seeded synthetic
scene and orbit cameras of SURVEY.md §8(d) (no network: data = synthetic).
A step = every rank renders its `--views-per-rank` views, then runs one
backward of their summed loss (the reference's batch step: threestudio/systems/
DGE.py renders the batch's views and back-propagates the summed loss), the
gradients accumulated into the shared parameters, and, for N > 1, ONE
all-reduce of the flat parameter-gradient bucket (RCCL) — of the rows nonzero
on some rank only (GradBucket.allreduce: ~24% of the 236 MB for 24 views).  The
views run on `--streams` HIP streams (default 3, dge_amd.multiview.render_views:
one view's latency-bound blend tails overlap the others' work; the in-kernel
gradient accumulation orders only the per-Gaussian passes across streams);
`--per-view-backward` runs each view's backward right after its forward
instead.  Per-GPU work
is fixed, so scaling is weak and value = all views rendered / max-rank time.

Prints ONE JSON line (rank 0) with the contract keys plus `roofline` (the
dominant kernel, timed live with HIP events on its stream through the C ABI's
stage profiler) and `cpu_baseline` (the oracle, a CPU restatement of the
reference, timed on this host's cores on a bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "forward+backward renders/sec @512×512, 1.0M Gaussians; achieved HBM GB/s"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
CLOCK_HZ = 2.4e9        # MI355X peak engine clock
N_SIMDS = 256 * 4       # 256 CUs x 4 SIMDs


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--points", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=512)
    ap.add_argument("--height", type=int, default=512)
    ap.add_argument("--sh-degree", type=int, default=3)
    ap.add_argument("--views-per-rank", type=int, default=3)
    ap.add_argument("--streams", type=int, default=3,
                    help="HIP streams the views alternate over (default 3: one per view of a 3-view step, so "
                         "one view's latency-bound blend tails overlap the others' work)")
    ap.add_argument("--per-view-backward", dest="batch_backward", action="store_false",
                    help="each view's backward right after its forward (default: all forwards, then one "
                         "backward of the summed loss -- the reference's order, DGE.py:170-239, 617-699)")
    ap.add_argument("--batch-backward", dest="batch_backward", action="store_true", help=argparse.SUPPRESS)
    ap.set_defaults(batch_backward=True)
    ap.add_argument("--exact", dest="speculate", action="store_false",
                    help="size every view's binning buffer from its instance count read back to the host (the "
                         "reference's per-view sync, rasterizer_impl.cu:236-239) instead of from the counts seen "
                         "before (render_views(speculate=True), checked once per step)")
    ap.add_argument("--scan-live", action="store_true",
                    help="N > 1: find the all-reduce's live rows by reading the gradient bucket after the backward "
                         "(GradBucket.allreduce) instead of agreeing on the forwards' blended Gaussians before it")
    ap.add_argument("--sync-union", action="store_true",
                    help="distributed step: wait for the union's size inside allreduce_end (GradBucket's default) "
                         "instead of deferring that check to the next step")
    ap.add_argument("--serial-zero", action="store_true",
                    help="zero the gradient bucket on the default stream before the forwards (default: on the first "
                         "view's stream beside the forwards, GradBucket.zero(stream=...))")
    ap.add_argument("--opacity-mean", type=float, default=0.0,
                    help="raw opacity N(mean, std) of the synthetic scene (profiling: -2 / 1 is the c2_high_live leg's)")
    ap.add_argument("--opacity-std", type=float, default=1.5)
    ap.add_argument("--cpu-baseline-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="OpenMP threads of the CPU baseline (default 0: every core this process may use)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--no-side-legs", action="store_true",
                    help="skip the extra legs (unchanged-DGE render() path, high-live-fraction scene)")
    return ap.parse_args()


def stage_bytes(stage, P, M, K, Kb, HW, tiles, live=None):
    """Algorithmic bytes per launch of each stage."""
    if stage == "preprocess":  # read xyz, scale, rot, opacity, SH; write the geometry record
        return P * (12 + 12 + 16 + 4 + 12 * M) + P * (8 + 16 + 16 + 4 + 1 + 4 + 4 + 4 + 4)
    if stage == "render_fwd":  # per instance: id + xy + conic/opacity + rgb/depth; per pixel: color, depth, T, n
        return K * (4 + 8 + 16 + 16) + HW * 24 + tiles * 8
    if stage == "render_bwd":  # per instance in the backward window: gather 44 B + 48-B record; per pixel 20 B
        return Kb * (4 + 8 + 16 + 16 + 48) + HW * 20 + tiles * 12
    if stage == "gauss_bwd":
        # every Gaussian: touched byte + radii (4), dL/dmean2D written (12, a fresh tensor);
        # each live Gaussian (visible with >= 1 record; the others have exactly zero gradients):
        # params in (xyz 12, scale 12, rot 16, opacity 4, SH 12 M), clamped 1, tiles/first slot 8,
        # its slots' flags 4 n, its records 48 each, and the 59-float (3+3+4+1+3M) gradient
        # read-modify-written into the shared .grad (fused accumulation: read + write)
        L, F, R = live["live"], live["flag_words"], live["records"]
        return P * (1 + 4 + 12) + L * (12 + 12 + 16 + 4 + 12 * M + 1 + 8) + 4 * F + 48 * R + \
            L * 2 * 4 * (3 + 3 + 4 + 1 + 3 * M)
    return None


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(args, argv=None, child_cmd=None) -> int:
    """`--gpus N` (N > 1) without a launcher: start N rank processes of this script, one per GPU, over a
    127.0.0.1 rendezvous (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their environment, as
    torch.distributed.run sets them), and return the first nonzero exit code (0 when all succeed).
    Nothing here touches the GPU (torch.cuda.device_count() does not initialise HIP on this image): the
    parent never creates a HIP context, so the ranks own their devices.  Rank 0 prints the JSON line.
    A rank that fails ends the others (their exact PIDs) instead of leaving them in a collective."""
    import subprocess

    n = args.gpus
    ndev = torch.cuda.device_count()
    env0 = dict(os.environ)
    env0.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE=str(n),
                DGE_AMD_BENCH_SPAWNED="1")
    if ndev < n and "DGE_AMD_BENCH_BACKEND" not in env0:
        # (a rehearsal of N ranks on fewer cards: RCCL refuses two ranks on one device, gloo does not)
        print(f"[bench] {n} ranks on {ndev} visible GPU(s): gloo backend (rehearsal)", file=sys.stderr)
        env0["DGE_AMD_BENCH_BACKEND"] = "gloo"
    cmd = child_cmd or [sys.executable, os.path.abspath(__file__)] + list(sys.argv[1:] if argv is None else argv)
    procs = []
    for r in range(n):
        env = dict(env0, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen(cmd, env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:  # (a failed rank leaves the others waiting in a collective)
                    q.terminate()
        if live:
            time.sleep(0.05)
    return rc


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"[bench] note: WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE", file=sys.stderr)
    # one rank per GPU; LOCAL_RANK beyond the visible count wraps (a rehearsal of N ranks on fewer cards)
    gpu = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    # DGE_AMD_BENCH_DIST=1: a process group (and the full sparse all-reduce protocol) even for one rank,
    # to rehearse the RCCL path on a one-GPU box under torch.distributed.run --nproc-per-node 1
    rehearse = os.environ.get("DGE_AMD_BENCH_DIST") == "1"
    distributed = world > 1 or rehearse
    # the views' and the collective's streams before RCCL creates its own: HIP deals the process's
    # GPU_MAX_HW_QUEUES hardware queues to streams round-robin, and a view stream sharing the caller's
    # queue runs that view behind the first one (measured on the one-rank RCCL rehearsal)
    from dge_amd.multiview import _collective_stream, view_streams
    if distributed:
        # (the step off the null stream: under RCCL the null stream shared its hardware queue with the first
        # pool stream, and the second view then ran behind the first one)
        torch.cuda.set_stream(torch.cuda.Stream(device=dev))
    view_streams(dev, args.streams)
    if distributed:
        _collective_stream(dev)
    if distributed:
        backend = os.environ.get("DGE_AMD_BENCH_BACKEND", "nccl")  # nccl = RCCL on ROCm; gloo for rehearsals
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")  # (rehearsal ranks on one host: loopback)
            dist.init_process_group(backend)

    from dge_amd import _native, _C
    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_renderer import PipelineParams, render
    from dge_amd.multiview import GradBucket
    from dge_amd.scene import synthetic_scene

    P, W, H, V = args.points, args.width, args.height, args.views_per_rank
    scene = synthetic_scene(P, sh_degree=args.sh_degree, seed=0, device=dev,
                            opacity_mean=args.opacity_mean, opacity_std=args.opacity_std).requires_grad_(True)
    n_total = V * world
    cams = [orbit_camera(k, n_total, W, H, device=dev) for k in range(rank * V, (rank + 1) * V)]
    gen = torch.Generator(device="cpu").manual_seed(1)
    seeds = [(torch.randn(3, H, W, generator=gen) * 1e-3).to(dev) for _ in range(V)]
    bg = torch.zeros(3, device=dev)
    pipe = PipelineParams()
    # (DGE_AMD_BUCKET_ROWS=0: the flat concatenated bucket instead of the row-major one — an A/B switch)
    bucket = GradBucket(scene.parameters(), rows=None if os.environ.get("DGE_AMD_BUCKET_ROWS", "1") != "0" else False)

    min_world = 1 if rehearse else 2

    coll_evs = []  # (start, end) events around each timed step's gradient collective, on the main stream

    def step(timed=False):
        run_views(args, cams, scene, pipe, bg, seeds, bucket, min_world=min_world if distributed else None)
        if distributed:
            if timed:
                a = torch.cuda.Event(enable_timing=True)
                a.record()
            if args.batch_backward and not args.scan_live:
                # the union-size check waits for the forwards: deferred to the next step's run_views, after
                # that step's forwards are issued (GradBucket.allreduce_finalize; the timed region ends with it)
                bucket.allreduce_end(defer_check=not args.sync_union)
            else:
                bucket.allreduce(min_world=min_world)
            if timed:
                b = torch.cuda.Event(enable_timing=True)
                b.record()
                coll_evs.append((a, b))

    def step_one_stream():
        # the kernels in isolation (one stream, nothing concurrent): what the per-stage and roofline
        # durations are taken from -- on several streams an event pair also times the other streams' work
        run_views(args, cams, scene, pipe, bg, seeds, bucket, streams=1)

    # instance counts of this rank's views (deterministic; outside the timed region)
    Ks, Kbs, lives = [], [], []
    with torch.no_grad():
        for cam in cams:
            from dge_amd.gaussian_renderer import _settings
            s = _settings(cam, bg, 1.0, scene.active_sh_degree)
            K, color, depth, radii, geom, binning, img = _C.rasterize_gaussians(
                s.bg, scene.get_xyz, torch.empty(0, device=dev), scene.get_opacity, scene.get_scaling,
                scene.get_rotation, 1.0, torch.empty(0, device=dev), s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy,
                H, W, scene.get_features, scene.active_sh_degree, s.campos, False, False)
            off = _native.lib().gs_buffer_offset(b"image", b"tile_last", P, W, H, K)
            tiles = ((W + 15) // 16) * ((H + 15) // 16)
            tl = img[off:off + 4 * tiles].view(torch.int32)
            Ks.append(int(K))
            Kbs.append(int(tl.sum().item()))
            # one reference-ABI backward: which Gaussians got records (gauss_bwd's live set)
            _C.rasterize_gaussians_backward(
                s.bg, scene.get_xyz, radii, torch.empty(0, device=dev), scene.get_scaling, scene.get_rotation, 1.0,
                torch.empty(0, device=dev), s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, seeds[len(Ks) - 1],
                scene.get_features, scene.active_sh_degree, s.campos, geom, K, binning, img, False)
            toff = _native.lib().gs_buffer_offset(b"geometry", b"touched", P, W, H, K)
            touched = geom[toff:toff + P]
            toffs = _native.lib().gs_buffer_offset(b"geometry", b"tiles_touched", P, W, H, K)
            tt = geom[toffs:toffs + 4 * P].view(torch.int32)
            foff = _native.lib().gs_buffer_offset(b"binning", b"rec_flags", P, W, H, K)
            recs = int((binning[foff:foff + 4 * K] != 0).sum().item()) if K else 0
            lv = (touched != 0) & (radii > 0)
            lives.append({"live": int(lv.sum().item()), "flag_words": int(tt[lv].sum().item()), "records": recs})
    torch.cuda.synchronize()

    # stage calibration (untimed, one stream): every stage bracketed by events, for the per-stage times
    calib = {}
    blend = ["render_fwd", "render_bwd"]
    if not args.no_profile:
        for _ in range(2):  # (first launches load code objects: keep them out of the stage times)
            step_one_stream()
        _native.profile_stages(None)
        _native.profile_enable(True)
        _native.profile_collect()  # reset
        for _ in range(2):
            step_one_stream()
        torch.cuda.synchronize()
        calib = {n: (ms, c) for n, (ms, c) in _native.profile_collect().items() if c}
        _native.profile_enable(False)
    # the W warmup steps run right before the timed region (after the calibration above), so the timed
    # steps start in the steady state the warmup built: the caching allocator's per-stream pools, the
    # staging slots, the clocks
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    m0 = torch.cuda.memory_stats(dev)
    main_stream = torch.cuda.current_stream(dev)
    # per-step timing: one timing event on the main stream after each step (every view stream and the
    # backward join it there) and the host clock when each step's issue returns
    # (fence-free timing events, gs_timer_*: a torch event's record flushes the L2 for the host — a marker
    # in the caller's queue between a step's last gradient writes and the next step's first kernel)
    evs = [_native.StepTimer() for _ in range(args.steps + 1)]
    host_t = []
    wait0 = _native.lib().gs_host_wait_ns()
    t0 = time.perf_counter()
    evs[0].record(main_stream)
    for i in range(args.steps):
        step(timed=True)
        evs[i + 1].record(main_stream)
        host_t.append(time.perf_counter())
    bucket.allreduce_finalize()  # (the last step's deferred union check, inside the timed region)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    dt = time.perf_counter() - t0
    host_wait_s = (_native.lib().gs_host_wait_ns() - wait0) * 1e-9
    step_ms = [evs[i].elapsed_ms(evs[i + 1]) for i in range(args.steps)]
    # the packed SUM (gather, RCCL all-reduce, scatter) on the main stream behind each step's backward
    coll_ms = [a.elapsed_time(b) for a, b in coll_evs]
    host_ms = [1e3 * (b - a) for a, b in zip([t0] + host_t[:-1], host_t)]
    m1 = torch.cuda.memory_stats(dev)
    # caching-allocator activity inside the timed region (device allocations there cost a hipMalloc each)
    alloc_stats = {k: int(m1.get(k, 0) - m0.get(k, 0)) for k in ("num_device_alloc", "num_device_free",
                                                                   "num_alloc_retries")}
    alloc_stats["reserved_gb"] = round(m1.get("reserved_bytes.all.current", 0) / 2**30, 2)
    # roofline leg (timed, one stream): the two blend kernels bracketed by HIP events on their launch
    # stream, live, over iso_steps steps of the same workload with the views on one stream
    prof, iso = {}, None
    if not args.no_profile:
        iso_steps = max(5, min(args.steps, 20))
        _native.profile_stages(blend)
        _native.profile_enable(True)
        _native.profile_collect()
        torch.cuda.synchronize()
        ti = time.perf_counter()
        for _ in range(iso_steps):
            step_one_stream()
        torch.cuda.synchronize()
        iso = {"steps": iso_steps, "renders_per_s": round(iso_steps * V / (time.perf_counter() - ti), 3)}
        prof = _native.profile_collect()
        _native.profile_enable(False)
        _native.profile_stages(None)
    rank_dt = dt
    if distributed:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        # every rank's own time (rank 0 reports them beside the max the value is taken from)
        allt = torch.zeros(world, device=dev, dtype=torch.float64)
        allt[rank] = rank_dt
        dist.all_reduce(allt, op=dist.ReduceOp.SUM)
        rank_times = [round(float(x), 5) for x in allt.tolist()]

    renders = args.steps * V * world
    value = renders / dt
    ms_per_step = 1000.0 * dt / args.steps

    HW = W * H
    tiles = ((W + 15) // 16) * ((H + 15) // 16)
    M = (args.sh_degree + 1) ** 2
    K = float(np.mean(Ks))
    Kb = float(np.mean(Kbs))
    live = {k: float(np.mean([d[k] for d in lives])) for k in lives[0]}
    stages = {n: ms / cnt for n, (ms, cnt) in calib.items()}
    rooflines = {}
    pmc = {}
    pmc_path = os.path.join(HERE, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc_path):
        try:
            with open(pmc_path) as fh:
                pmc = json.load(fh)
        except Exception:
            pmc = {}
    for name in blend:  # both blend kernels, timed live in the one-stream roofline leg
        ms, cnt = prof.get(name, (0.0, 0))
        if not cnt:
            continue
        avg = ms / cnt
        stages[name] = avg
        b = stage_bytes(name, P, M, K, Kb, HW, tiles, live)
        achieved = b / (avg * 1e-3) / 1e9
        r = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
             "frac": round(achieved / HBM_PEAK_GBPS, 5), "traffic": None, "kernel": name,
             "algorithmic_bytes_per_launch": int(b), "avg_ms": round(avg, 4)}
        tr = pmc.get(name) or {}
        if tr.get("bytes_per_launch"):
            r["traffic"] = tr["bytes_per_launch"]
            r["traffic_over_algorithmic"] = round(tr["bytes_per_launch"] / b, 3)
        if tr.get("valu_insts_per_launch"):
            # VALU issue fraction: wave64 VALU instructions x 2 SIMD cycles / (kernel cycles at the 2.4 GHz
            # peak clock x 1024 SIMDs) -- what bounds these kernels instead of HBM
            vf = tr["valu_insts_per_launch"] * 2.0 / (avg * 1e-3 * CLOCK_HZ * N_SIMDS)
            r["valu_issue_frac"] = round(vf, 4)
            # what bounds the kernel: a resource it keeps over half busy, else latency (dependent chains,
            # the tail of the longest quadrants) -- the blend kernels' case, DESIGN.md §4.3-4.4
            r["limit"] = "hbm" if r["frac"] > 0.5 else "valu" if vf > 0.5 else "latency"
        if tr.get("build"):
            r["pmc_build"] = tr["build"]
            # the PMC pass measured the kernel sources this run was built from (else the traffic is stale)
            from dge_amd._native import source_stamp

            r["pmc_build_current"] = tr["build"] == source_stamp()
        rooflines[name] = r
    roofline = max(rooflines.values(), key=lambda r: r["avg_ms"]) if rooflines else None

    legs = {}
    if not args.no_side_legs and world == 1:
        legs = side_legs(args, scene, cams, seeds, bg, pipe, bucket, step, dev)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(scene, cams[0], seeds[0], bg, args)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "renders/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic",
            "config": {"workload": f"c2: {P / 1e6:.2f}M Gaussians (SH deg {args.sh_degree}), {W}x{H}, fp32 fwd+bwd",
                       "gaussians": P, "width": W, "height": H, "views_per_rank": V, "streams": args.streams,
                       "parallelism": f"views sharded x{world}" + (
                           f", {os.environ.get('DGE_AMD_BENCH_BACKEND', 'nccl').replace('nccl', 'RCCL')} "
                           "sparse-row grad all-reduce" if world > 1 else "")},
            "num_rendered_mean": int(K),
            "live_gaussians_mean": int(live["live"]),
            "gradient_records_mean": int(live["records"]),
            "backward_window_instances_mean": int(Kb),
            # a MODEL, not measured traffic: SURVEY.md §8(d)'s B = 828 P + 200 K + 44 HW bytes per render
            # (the reference's traffic) x renders/s per GPU
            "modeled_gbps_survey_bytes_whole_render": round((828.0 * P + 200.0 * K + 44.0 * HW) * value / world / 1e9, 2),
            "stages_ms": {k: round(v, 4) for k, v in stages.items()},
            "roofline": roofline,
            "rooflines": rooflines,
            # the leg the rooflines and stages_ms come from: the same step with the views on one stream
            "roofline_leg": iso,
            "allocator_timed_region": alloc_stats,
            # per-step GPU time between main-stream events (the step's views and backward joined), its spread,
            # and the host's issue time per step with the part spent blocked on the instance-count read-back
            "step_ms": _spread(step_ms),
            "host_ms_per_step": {"issue": round(1e3 * (host_t[-1] - t0) / args.steps, 4),
                                 "wait": round(1e3 * host_wait_s / args.steps, 4),
                                 "busy": round((1e3 * (host_t[-1] - t0) - 1e3 * host_wait_s) / args.steps, 4),
                                 "per_step": _spread(host_ms)},
            "legs": legs,
            "cpu_baseline": cpu,
        }
        if distributed:
            c50 = float(np.percentile(coll_ms, 50)) if coll_ms else 0.0
            s50 = float(np.percentile(step_ms, 50))
            line["distributed"] = {
                "backend": os.environ.get("DGE_AMD_BENCH_BACKEND", "nccl").replace("nccl", "RCCL"),
                "launch": "bench.py spawned its ranks" if os.environ.get("DGE_AMD_BENCH_SPAWNED") else
                          "external launcher (torch.distributed.run)",
                "rank_seconds": rank_times, "max_rank_seconds": round(dt, 5),
                # the gradient collective of a step (pack, SUM, unpack on the main stream), its share of the step
                "collective_ms": _spread(coll_ms), "collective_share_p50": round(c50 / max(s50, 1e-9), 4)}
        print(json.dumps(line), flush=True)
    if distributed:
        dist.destroy_process_group()


def _spread(xs):
    """p50 / p90 / max (and the index of the max) of per-step milliseconds."""
    a = np.asarray(xs, dtype=np.float64)
    if a.size == 0:
        return None
    out = {"p50": round(float(np.percentile(a, 50)), 4), "p90": round(float(np.percentile(a, 90)), 4),
           "min": round(float(a.min()), 4), "max": round(float(a.max()), 4), "argmax": int(a.argmax()),
           "max_over_p50": round(float(a.max() / max(np.percentile(a, 50), 1e-9)), 3)}
    if a.size > 2:
        # the first timed step starts from the drained GPU the timing contract's synchronize leaves, so
        # it also carries the host's issue time to its first launch: the spread of the others beside it
        rest = a[1:]
        out["max_over_p50_after_first"] = round(float(rest.max() / max(np.percentile(rest, 50), 1e-9)), 3)
    return out


def run_views(args, cams, scene, pipe, bg, seeds, bucket, streams=None, min_world=None):
    """One step's renders: zero the bucket, forward every view, backward (see the module docstring).
    min_world (distributed steps): the sparse all-reduce's union of live rows is agreed on between the
    forwards and the backward (GradBucket.allreduce_begin; the caller runs allreduce_end).  With
    speculated binning capacities the step ends with the batch's check (its one host wait, on the
    views' preprocess) and runs again in the rare case a view overflowed its capacity."""
    from dge_amd.multiview import render_backward_views, render_views

    streams = args.streams if streams is None else streams
    if not args.batch_backward:
        bucket.zero()
        render_backward_views(cams, scene, pipe, bg, seeds, streams=streams)
        return
    for attempt in range(2):
        # the bucket's fill runs on the first view's stream behind that view's forward, beside the others'
        # (only the backward's gradient writes wait for it: GradBucket.zero(stream=...))
        side = streams > 1 and not args.serial_zero
        if not side:
            bucket.zero()
        outs = render_views(cams, scene, pipe, bg, streams=streams, speculate=args.speculate)
        if side:
            from dge_amd.multiview import view_streams

            # (zero() first runs the previous step's deferred union check, its forwards done by now; a fix-up
            # it enqueues writes the bucket, so the fill then also waits for it.)  The view stream already waits
            # for everything the caller's stream held before this step (the forward's fork: the previous step's
            # gradient writes), so the fill needs no event of its own there — one system-fenced marker less in
            # the caller's queue per step
            bucket.zero(stream=view_streams(torch.cuda.current_stream().device, streams)[1])
        if attempt == 0 and min_world is not None and not args.scan_live:
            # (the union's MAX also carries this batch's overflow flag: a re-render below is agreed on)
            bucket.allreduce_begin([o.get("_live_rows") for o in outs], min_world=min_world, views=outs)
        torch.autograd.backward([o["render"] for o in outs], seeds)
        if outs.check():
            return
        # a view's instance count outgrew its speculated capacity: the step again, locally (the capacity
        # grew); the other ranks learn it from the flag and re-agree on the rows in allreduce_end
    raise RuntimeError("render_views: the binning capacity check failed twice")


def _time(fn, steps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return time.perf_counter() - t0


def side_legs(args, scene, cams, seeds, bg, pipe, bucket, step, dev):
    """Extra legs, timed after the main region on the same box (not the headline value):
    * dge_unchanged_render: the path DGE takes with only install_alias() -- its own render()
      (gaussian_renderer/__init__.py:90-140: the torch getters, torch.cat of the SH, GaussianRasterizer /
      _RasterizeGaussians) -- reproduced by render() with the fused raw-parameter path off;
    * c2_high_live: c2 with raw opacity N(-2, 1) instead of N(0, 1.5): most Gaussians translucent, so far
      more of them reach the backward (the live-set backward is not only judged at ~7% live);
    * dge_semantic_forward: DGE's second, gradient-free render of every view (DGE.py:198-204: the edit
      mask as override_color, thresholded norm), batched like the training renders, forward only;
    * dge_step_with_semantic: the c2 step plus those semantic renders (the DGE loop's per-view work)."""
    from dge_amd.cameras import orbit_camera
    from dge_amd.multiview import GradBucket, render_backward_views
    from dge_amd.scene import synthetic_scene

    legs = {}
    steps = max(5, min(args.steps, 20))
    V = len(cams)
    prev = os.environ.get("DGE_AMD_FUSED")
    os.environ["DGE_AMD_FUSED"] = "0"

    # (autograd's own accumulation here, not the fused in-kernel one: a flat bucket of contiguous .grad
    # tensors — into the row-major bucket's strided .grad views AccumulateGrad warns about the layout)
    flat_bucket = GradBucket(scene.parameters(), rows=False)

    def unchanged():
        # DGE renders its views one after another on the caller's stream (DGE.py:179-222).  (On the views'
        # streams each view's torch getter nodes would run on its own stream while feeding the one
        # AccumulateGrad node per parameter: autograd's stream-mismatch warning, round 3's stderr.)
        run_views(args, cams, scene, pipe, bg, seeds, flat_bucket, streams=1)

    try:
        for _ in range(3):
            unchanged()
        dt = _time(unchanged, steps)
    finally:
        if prev is None:
            os.environ.pop("DGE_AMD_FUSED", None)
        else:
            os.environ["DGE_AMD_FUSED"] = prev
    legs["dge_unchanged_render"] = {"value": round(steps * V / dt, 3), "unit": "renders/s",
                                    "path": "torch getters + cat + _RasterizeGaussians (fused path off), one stream"}
    del flat_bucket
    bucket.attach()

    hl = synthetic_scene(args.points, sh_degree=args.sh_degree, seed=0, device=dev, opacity_mean=-2.0,
                         opacity_std=1.0).requires_grad_(True)
    hb = GradBucket(hl.parameters())

    def hstep():
        run_views(args, cams, hl, pipe, bg, seeds, hb)

    for _ in range(3):
        hstep()
    from dge_amd import _native
    _native.profile_stages(None)
    _native.profile_enable(True)
    _native.profile_collect()
    run_views(args, cams, hl, pipe, bg, seeds, hb, streams=1)  # (stage times in isolation: one stream)
    torch.cuda.synchronize()
    st = {n: round(ms / c, 4) for n, (ms, c) in _native.profile_collect().items() if c}
    _native.profile_enable(False)
    dt = _time(hstep, steps)
    # live fraction of view 0 (Gaussians with a gradient: nonzero opacity gradient after one backward)
    hb.zero()
    render_backward_views(cams[:1], hl, pipe, bg, seeds[:1], streams=1)
    live = float((hl._opacity.grad != 0).float().mean().item())
    legs["c2_high_live"] = {"value": round(steps * V / dt, 3), "unit": "renders/s", "live_fraction": round(live, 4),
                            "opacity": "raw N(-2, 1)", "stages_ms": st}
    del hl, hb

    # DGE's semantic render (gradient-free, override_color = the Gaussian mask, DGE.py:198-204): a 20%
    # mask, the views batched on the step's streams, no autograd (forward-only kernels)
    from dge_amd.multiview import render_views
    gm = torch.rand(args.points, generator=torch.Generator().manual_seed(5)) < 0.2
    colors = gm.to(dev)[:, None].float().repeat(1, 3)

    def sem():
        with torch.no_grad():
            outs = render_views(cams, scene, pipe, bg, streams=args.streams, override_color=colors)
            return [torch.norm(o["render"], dim=0) > 0.8 for o in outs]

    for _ in range(3):
        sem()
    dt = _time(sem, steps)
    legs["dge_semantic_forward"] = {"value": round(steps * V / dt, 3), "unit": "renders/s",
                                    "path": "render_views(override_color=mask), no_grad, forward only"}

    # DGE's own loop, unchanged, on the render() that install_alias(fused_render=True) gives it:
    # threestudio/systems/DGE.py forward() :170-239 per view (training render, radii max, the semantic
    # render with the mask as override_color, its norm > 0.8 map, the masked visualisation — a boolean
    # index, i.e. a host sync per view — the stacks), then the masked l1 of training_step (:672) and ONE
    # backward; .grad set to None first (the optimizer's zero_grad).  No edit of DGE's code: its per-view
    # host sync is part of what it costs.
    from dge_amd.gaussian_renderer import render as fused_render
    gts = [torch.rand(H_, W_, 3, generator=torch.Generator().manual_seed(50 + i)).to(dev)
           for i, (H_, W_) in enumerate([(args.height, args.width)] * V)]
    gm_dev = gm.to(dev)

    def dge_loop():
        for p in scene.parameters():
            p.grad = None
        prev_mask, scene.mask = scene.mask, gm_dev
        try:
            images, masks = [], []
            radii = None
            for i, cam in enumerate(cams):
                pkg = fused_render(cam, scene, pipe, bg)
                image, r = pkg["render"], pkg["radii"]
                radii = r if i == 0 else torch.max(r, radii)
                pkg["depth_3dgs"].permute(1, 2, 0)
                sm = fused_render(cam, scene, pipe, bg, override_color=scene.mask[..., None].float().repeat(1, 3))["render"]
                sm = torch.norm(sm, dim=0) > 0.8
                viz = image.detach().clone().permute(1, 2, 0)
                viz[sm] = 0.40 * viz[sm] + 0.60 * torch.tensor([1.0, 0.0, 0.0], device=dev)
                masks.append(sm)
                images.append(image.permute(1, 2, 0))
            images = torch.stack(images, 0)
            m = torch.stack(masks, 0)[..., None].float()
            loss = torch.nn.functional.l1_loss(images * m, torch.stack(gts, 0) * m)
            loss.backward()
        finally:
            scene.mask = prev_mask

    from dge_amd import gaussian_renderer as GR
    hits0 = GR._RECOLOR_HITS
    for _ in range(3):
        dge_loop()
    dt = _time(dge_loop, steps)
    hits = GR._RECOLOR_HITS - hits0
    dt_lazy = None
    recolor = GR._RECOLOR
    GR._RECOLOR = False  # (the semantic render in full: lazy forward-only kernels, its own binning)
    try:
        for _ in range(2):
            dge_loop()
        dt_full = _time(dge_loop, steps)
    finally:
        GR._RECOLOR = recolor
    lazy = GR._LAZY_OVERRIDE
    GR._LAZY_OVERRIDE, GR._RECOLOR = False, False  # (and with the backward's bookkeeping: the round-3 path)
    try:
        for _ in range(2):
            dge_loop()
        dt_lazy = _time(dge_loop, steps)
    finally:
        GR._LAZY_OVERRIDE, GR._RECOLOR = lazy, recolor
    legs["dge_loop_unchanged"] = {
        "value": round(steps * V / dt, 3), "unit": "views/s",
        "path": "DGE.py forward() per view (fused render(), semantic render, boolean-mask viz: a host sync per "
                "view) + masked l1 + one backward, install_alias(fused_render=True), no code edit",
        "semantic_recolor_hits": hits,
        "semantic_full_render_value": round(steps * V / dt_full, 3),
        "semantic_eager_value": round(steps * V / dt_lazy, 3)}
    for p in scene.parameters():
        p.grad = None
    bucket.attach()

    def step_sem():
        step()
        sem()

    for _ in range(3):
        step_sem()
    dt = _time(step_sem, steps)
    legs["dge_step_with_semantic"] = {"value": round(steps * V / dt, 3), "unit": "views/s",
                                      "path": "the c2 step (fwd+bwd renders) + the semantic forward of each view"}
    # BASELINE.json's other single-GPU configs and SURVEY.md §8(f) F3, timed here so the driver's run records them
    torch.cuda.empty_cache()
    for name, fn in (("c4_hd_forward", leg_c4), ("c5_local_edit", leg_c5), ("f3_adam", leg_adam)):
        legs[name] = fn(dev, steps, 3)
        torch.cuda.empty_cache()
    return legs


def _timed(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def _stages(fn, n=3):
    from dge_amd import _native

    _native.profile_stages(None)
    _native.profile_enable(True)
    _native.profile_collect()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    prof = _native.profile_collect()
    _native.profile_enable(False)
    return {k: round(ms / c, 4) for k, (ms, c) in prof.items() if c}


def leg_c4(dev, steps, warmup):
    """configs[3]: 2.5M Gaussians, 1920x1080, forward only (render() without autograd: 8160 tiles, the
    two-level binning; rasterizer_impl.cu:179-285)."""
    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_renderer import PipelineParams, render
    from dge_amd.scene import synthetic_scene

    P, W, H = 2_500_000, 1920, 1080
    sc = synthetic_scene(P, seed=2, device=dev)
    cam = orbit_camera(0, 1, W, H, device=dev)
    bg = torch.zeros(3, device=dev)

    def fwd():
        with torch.no_grad():
            render(cam, sc, PipelineParams(), bg)

    dt = _timed(fwd, steps, warmup)
    return {"workload": "c4: 2.5M Gaussians, 1920x1080, fp32 forward only", "value": round(1.0 / dt, 2),
            "unit": "renders/s", "ms_per_render": round(1e3 * dt, 3), "stages_ms": _stages(fwd)}


def leg_c5(dev, steps, warmup):
    """configs[4]: 1.0M scene, localize on a 200k mask (the x-sorted first 20%), SH stored fp16, fp32
    covariance inputs, 512x512 forward + backward through render() (gaussian_model.py:221-258 localize)."""
    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_renderer import PipelineParams, render
    from dge_amd.scene import synthetic_scene

    P, Psub, W, H = 1_000_000, 200_000, 512, 512
    sc = synthetic_scene(P, seed=0, device=dev)
    sc._features_dc = sc._features_dc.half()
    sc._features_rest = sc._features_rest.half()
    mask = torch.zeros(P, dtype=torch.bool, device=dev)
    mask[torch.argsort(sc._xyz[:, 0])[:Psub]] = True
    sc.mask, sc.localize = mask, True
    sc.requires_grad_(True)
    cam = orbit_camera(0, 1, W, H, device=dev)
    g = torch.randn(3, H, W, device=dev, generator=torch.Generator(device=dev).manual_seed(5)) * 1e-3
    bg = torch.zeros(3, device=dev)

    def step():
        for p in sc.parameters():
            p.grad = None
        (render(cam, sc, PipelineParams(), bg)["render"] * g).sum().backward()

    dt = _timed(step, steps, warmup)
    return {"workload": "c5: 1.0M scene, localize 200k (x-sorted 20%), fp16 SH, 512x512 fwd+bwd",
            "value": round(1.0 / dt, 2), "unit": "renders/s", "ms_per_render": round(1e3 * dt, 3),
            "stages_ms": _stages(step)}


def leg_adam(dev, steps, warmup):
    """the optimizer step over a 1.0M-Gaussian GaussianModel (six groups, 59 floats per
    Gaussian, gaussian_model.py:336-394): FusedAdam (one gfx950 kernel) against torch.optim.Adam (foreach)."""
    from dge_amd.optim import FusedAdam

    P = 1_000_000
    shapes = [(P, 3), (P, 1, 3), (P, 15, 3), (P, 1), (P, 3), (P, 4)]
    lrs = [1.6e-4, 0.0125, 0.0125 / 20, 0.05, 0.005, 0.001]
    out = {"workload": "F3: Adam step over 1.0M Gaussians (59 floats each)", "unit": "GB/s algorithmic",
           "bytes_per_step": 59 * P * 28}
    gen = torch.Generator(device=dev).manual_seed(7)
    for name, cls in (("fused", FusedAdam), ("torch_foreach", torch.optim.Adam)):
        ps = [torch.nn.Parameter(torch.randn(s, device=dev, generator=gen)) for s in shapes]
        for p in ps:
            p.grad = torch.randn(p.shape, device=dev, generator=gen) * 1e-3
        opt = cls([{"params": [p], "lr": lr} for p, lr in zip(ps, lrs)], lr=0.0, eps=1e-15)
        dt = _timed(opt.step, steps, warmup)
        out[name] = {"ms": round(1e3 * dt, 4), "algorithmic_GBps": round(out["bytes_per_step"] / dt / 1e9, 1)}
        del opt, ps
    out["value"] = out["fused"]["algorithmic_GBps"]
    out["speedup"] = round(out["torch_foreach"]["ms"] / out["fused"]["ms"], 2)
    return out


def cpu_baseline(scene, cam, seed, bg, args):
    """The oracle (CPU restatement of the reference) on the same scene/view, bounded to ~N seconds."""
    try:
        from oracle import oracle as O
    except Exception as e:  # pragma: no cover
        return {"error": f"oracle unavailable: {e}"}
    usable = _usable_cpus()
    threads = max(1, args.cpu_threads if args.cpu_threads > 0 else usable["usable"])
    O.set_threads(threads)
    from dge_amd.gaussian_renderer import _settings
    s = _settings(cam, bg, 1.0, scene.active_sh_degree)
    with torch.no_grad():
        xyz, op, sh = scene.get_xyz.cpu().numpy(), scene.get_opacity.cpu().numpy(), scene.get_features.cpu().numpy()
        scl, rot = scene.get_scaling.cpu().numpy(), scene.get_rotation.cpu().numpy()
    g = seed.cpu().numpy()
    n, t0 = 0, time.perf_counter()
    while True:
        _, _, _, _, st = O.forward(s, xyz, op, shs=sh, scales=scl, rotations=rot)
        O.backward(st, g, magnitudes=False)
        del st
        n += 1
        el = time.perf_counter() - t0
        if el >= args.cpu_baseline_seconds or n >= 50:
            break
    model = ""
    try:
        with open("/proc/cpuinfo") as fh:
            for ln in fh:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": round(n / el, 4), "unit": "renders/s", "cores": threads, "kind": "port", "cpu_model": model,
            "affinity_cpus": usable["affinity"], "os_cpu_count": usable["cpu_count"], "cgroup_cpus": usable["cgroup"],
            "sample": f"{n} fwd+bwd render(s) of the c2 scene, view 0, oracle/gs_oracle.c with {threads} OpenMP threads"}


def _usable_cpus():
    """The host cores this process may use: its CPU affinity set, capped by a cgroup CPU quota (cpu.max)
    when one is set; os.cpu_count() (the whole machine) beside them."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return {"usable": min(aff, quota) if quota else aff, "affinity": aff, "cpu_count": os.cpu_count(),
            "cgroup": quota}


if __name__ == "__main__":
    main()
