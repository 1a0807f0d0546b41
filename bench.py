#!/usr/bin/env python3
"""Benchmark: Mrays/s (+ Msamples/s) of the MI355X per-pixel integration path.

Workload (BASELINE.json configs[2], the config the north-star target is quoted on):
bunny.sp at 1920x1080, 256 samples per pixel, DirectLighting (the reference's default integrator
for a scene file that names none: main.cpp:387-392), SAH BVH.  One step = one full frame.
With --gpus N > 1 (one process per GPU via torch.distributed.run) the frame's 8x8 tiles are
sharded across ranks (TileScheduler order, interleaved) and gathered to rank 0 with a single
RCCL gather at frame end: strong scaling (fixed total work).

Prints ONE JSON line (rank 0) with roofline and cpu_baseline objects; see DESIGN.md §Measurement.
"""
from __future__ import annotations

import argparse
import math
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# oracle/build_ref.sh: the reference's CMake flags (-std=gnu++20 -mfma -mavx2) with -O2 in place of
# CMake's empty build type (no -O); -ffp-contract=off keeps the -O0 build's IEEE arithmetic
REF_BUILD = "g++ 11.4 -std=gnu++20 -O2 -ffp-contract=off -mfma -mavx2 (oracle/build_ref.sh)"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
MT_BYTES_PER_DRAW = 24.0  # 8 B draw read + (2496 B twist read + 2496 B write) / 312
PIXEL_BYTES = 12.0  # one float3 radiance store per pixel


# BASELINE.json configs: scene writer, file name, default width / height / spp / integrator, data note.
SCENES = {
    "bunny": dict(writer="write_bunny_scene", file="bunny.sp", w=1920, h=1080, spp=256, integrator="direct_lighting",
                  data="synthetic (bunny-like PLY generated in-process; scene parameters of scenes/bunny.sp)"),
    "bunny_scan": dict(writer="write_bunny_scan_scene", file="bunny_scan.sp", w=1920, h=1080, spp=256,
                       integrator="direct_lighting",
                       data="synthetic scan-like bunny (cupped ears, surface relief; scenes.bunny_scan_mesh), robustness "
                            "variant of configs[2]; scene parameters of scenes/bunny.sp"),
    "spheres": dict(writer="write_material_spheres_scene", file="material_spheres_ibl.sp", w=1024, h=1024, spp=64,
                    integrator="direct_lighting",
                    data="synthetic 4096x2048 HDR night map in place of clarens_night_02_4k.pfm; scene parameters of "
                         "scenes/material_spheres.sp"),
    "lucy": dict(writer="write_lucy_scene", file="lucy.sp", w=1920, h=1080, spp=256, integrator="direct_lighting",
                 data="synthetic 28.05M-triangle lucy-like PLY generated in-process; scene parameters of scenes/lucy.sp"),
    "elf": dict(writer="write_elf_scene", file="elf.sp", w=4096, h=4096, spp=1024, integrator="iterative_rrnee",
                data="synthetic 1.0M-triangle figure as binary STL generated in-process; scene parameters of "
                     "scenes/elf.sp + max_depth 16"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", default="bunny", choices=sorted(SCENES),
                    help="bunny = configs[2] (default, the north-star workload); spheres = configs[1]; "
                         "lucy = configs[3]; elf = configs[4]")
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--integrator", default=None)
    ap.add_argument("--bvh", type=int, default=0, help="0 = SAH, 1 = reference median split")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget for the CPU baseline sample")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads for the CPU baseline (0 = this process's CPU share: OMP_NUM_THREADS when set, "
                         "else os.cpu_count())")
    ap.add_argument("--cpu-scaling-seconds", type=float, default=3.0,
                    help="N = 1: budget per leg of the reference's thread-scaling sample (1 thread and the CPU "
                         "share); 0 = skip")
    ap.add_argument("--parity-seconds", type=float, default=6.0,
                    help="N > 1: CPU budget for the parity sample of the gathered frame")
    ap.add_argument("--pg-timeout", type=float, default=1800.0,
                    help="N > 1: collective timeout (s) of the process group; only the render and the gather "
                         "run inside it -- rank 0's reference scene build and parity run after teardown")
    ap.add_argument("--launch-selftest", action="store_true",
                    help="test hook: spawn the ranks like --gpus N does, join a gloo group, no GPU work")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--pipeline", default="auto", choices=["auto", "megakernel", "wavefront", "chunks"])
    ap.add_argument("--waves", type=int, default=0,
                    help="megakernel occupancy variant (sp_render_params.waves_per_simd; 0 = automatic)")
    ap.add_argument("--tail-fraction", type=float, default=0.0,
                    help="megakernel tail chunks (sp_render_params.tail_fraction): 0 automatic, < 0 off, else the fraction")
    ap.add_argument("--tile-order-factor", type=float, default=0.0,
                    help="megakernel tile order (sp_render_params.tile_order_factor): 0 automatic, > 0 always, < 0 queue order")
    ap.add_argument("--per-lane-queries", action="store_true",
                    help="IterativeRRNEE: walk every ray on its own lane (SP_RENDER_PER_LANE_QUERIES; comparison)")
    ap.add_argument("--sim-world", type=int, default=0,
                    help="diagnostic: render only one rank's shard of an N-GPU run on this one GPU (per-GPU load at N)")
    ap.add_argument("--sim-rank", type=int, default=0,
                    help="with --sim-world N: the rank whose shard is rendered (0..N-1); -1 = every rank's shard in "
                         "turn, one diagnostic JSON line with per-rank times and max/mean (no CPU baseline)")
    ap.add_argument("--traffic-json", default=None,
                    help="tools/pmc_traffic.py output of this workload (default profiles/pmc_bench_<scene>[_shard<N>].json)")
    ap.add_argument("--valu-json", default=None,
                    help="tools/pmc_valu.py output of a PMC pass of this workload (VALU-issue roofline; default "
                         "profiles/pmc_valu_bench_<scene>[_shard<N>].json)")
    a = ap.parse_args()
    if a.sim_world > 1 and not -1 <= a.sim_rank < a.sim_world:
        ap.error("--sim-rank must be -1 or in [0, --sim-world)")
    # tools/gpu_pmc_*.sh output names (PMC passes profile rank 0's shard)
    # the per-rank workload the counters must describe: a --sim-world shard, or with --gpus N rank 0's
    # shard of N (the PMC passes profile `--sim-world N`, the same tiles and calls)
    a.shard_n = a.sim_world if a.sim_world > 1 else (a.gpus if a.gpus > 1 else 0)
    tag = a.scene + (f"_shard{a.shard_n}" if a.shard_n > 1 else "") + (f"_r{a.sim_rank}" if a.sim_world > 1 and a.sim_rank > 0 else "")
    a.traffic_json = a.traffic_json or os.path.join(ROOT, "profiles", f"pmc_bench_{tag}.json")
    a.valu_json = a.valu_json or os.path.join(ROOT, "profiles", f"pmc_valu_bench_{tag}.json")
    sc = SCENES[a.scene]
    a.width = a.width or sc["w"]
    a.height = a.height or sc["h"]
    a.spp = a.spp or sc["spp"]
    a.integrator = a.integrator or sc["integrator"]
    return a


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_command(argv, n: int, port: int) -> list:
    """One process per GPU: torch.distributed.run on this node, rendezvous on 127.0.0.1."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def self_launch(args) -> int:
    """`python bench.py --gpus N` without a launcher: start the N ranks as CHILD processes and
    exit with their status.  Runs before anything touches the GPU (no exec from a GPU process)."""
    cmd = launch_command(sys.argv[1:], args.gpus, free_port())
    print(f"bench: launching {args.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    import subprocess
    return subprocess.run(cmd).returncode


def affinity_cpus() -> int:
    """CPUs the scheduler lets this process run on (os.sched_getaffinity)."""
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return os.cpu_count() or 1


def cpu_share() -> int:
    """CPUs this process may use: the GPU box gives each GPU a share (OMP_NUM_THREADS), while
    os.cpu_count() reports the whole machine there; never more than the affinity mask allows."""
    n = min(os.cpu_count() or 1, affinity_cpus())
    omp = os.environ.get("OMP_NUM_THREADS", "")
    return max(1, min(n, int(omp))) if omp.isdigit() and int(omp) > 0 else n


class _CpuStats:
    """RenderStats stand-in of the SP_BENCH_CPU_RENDER test hook (oracle render on the host)."""

    def __init__(self, st, ms):
        self.rays, self.shadow_rays, self.samples = int(st["rays"]), int(st["shadow_rays"]), int(st["samples"])
        self.rng_draws, self.kernel_ms, self.pipeline, self.primary_hits = 0, ms, 1, 0
        self.stage_ms, self.parts, self.stack_depth, self.launches = (ms, 0.0, 0.0, 0.0), 1, 0, 1


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.launch_selftest:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo")
        t = torch.tensor([float(rank)])
        dist.all_reduce(t)
        if rank == 0:
            print(json.dumps({"launch_selftest": True, "world": dist.get_world_size(), "rank_sum": float(t[0])}),
                  flush=True)
        dist.destroy_process_group()
        return
    import datetime

    import torch

    dist = None
    # SP_BENCH_SHARED_DEVICE=1 (test hook): every rank renders on cuda:0 and the ranks talk over
    # gloo with host copies -- the N>1 flow on a one-GPU box (RCCL needs one GPU per rank).
    # SP_BENCH_CPU_RENDER=1 (test hook, no GPU): the CPU oracle renders each rank's shard and the
    # ranks talk over gloo -- the orchestration (timeouts, teardown before rank 0's reference work)
    # exercised on CPU (tests/test_multi_rank.py).
    cpu_render = os.environ.get("SP_BENCH_CPU_RENDER") == "1"
    shared = world > 1 and (os.environ.get("SP_BENCH_SHARED_DEVICE") == "1" or cpu_render)
    pg_timeout = datetime.timedelta(seconds=args.pg_timeout)
    if world > 1:
        import torch.distributed as dist

        if shared:
            local = 0
            if not cpu_render:
                torch.cuda.set_device(0)
            dist.init_process_group("gloo", timeout=pg_timeout)
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"), timeout=pg_timeout)
        world = dist.get_world_size()
    else:
        if not cpu_render:
            torch.cuda.set_device(0)
        local = 0
    cdev = "cpu" if shared else f"cuda:{local}"  # where the collectives' tensors live
    rdev = "cpu" if cpu_render else f"cuda:{local}"  # where the render output lives

    def sync():
        if not cpu_render:
            torch.cuda.synchronize()

    import simplepath_amd as sp
    from simplepath_amd import scenes

    scene_dir = os.path.join(tempfile.gettempdir(), f"sp_bench_{os.getuid()}")
    writer, fname = SCENES[args.scene]["writer"], SCENES[args.scene]["file"]
    if rank == 0:
        getattr(scenes, writer)(scene_dir)
    if dist is not None:
        dist.barrier()
    path = os.path.join(scene_dir, fname)
    scene = sp.Scene.from_file(path)
    scene.set_resolution(args.width, args.height)
    if not cpu_render:
        scene.upload(device=local, bvh_mode=args.bvh)
    integ = sp.string_to_integrator_type(args.integrator)

    from simplepath_amd import shard

    sched = sp.ColumnMajorTileScheduler(args.width, args.height)
    n_tiles = sched.get_num_tiles()
    my_tiles = shard.shard_tiles(n_tiles, rank, world)
    per_rank = shard.per_rank_capacity(n_tiles, world)
    if args.sim_world > 1 and world == 1:
        if args.sim_rank < 0:
            return sim_all_ranks(args, scene, integ, n_tiles, rdev)
        my_tiles = shard.shard_tiles(n_tiles, args.sim_rank, args.sim_world)
        per_rank = shard.per_rank_capacity(n_tiles, args.sim_world)
    out = torch.zeros((per_rank, 64, 3), dtype=torch.float32, device=rdev)
    gathered, frame = None, None
    if dist is not None and rank == 0:
        gathered = [torch.zeros((per_rank, 64, 3), dtype=torch.float32, device=cdev) for _ in range(world)]
        frame = torch.zeros((n_tiles, 64, 3), dtype=torch.float32, device=cdev)
    stream = None if cpu_render else torch.cuda.current_stream().cuda_stream
    gather_ms = []

    def render():
        if cpu_render:
            from tests import _oracle
            t = time.perf_counter()
            tiles, st = _oracle.render(scene, integ, args.spp, my_tiles, threads=2, variant="glibc")
            out[: len(my_tiles)] = torch.from_numpy(tiles)
            return _CpuStats(st, (time.perf_counter() - t) * 1e3)
        return sp.render_tiles_device(scene, integ, args.spp, my_tiles, out.data_ptr(), stream,
                                      pipeline=args.pipeline, stage_timing=True, waves_per_simd=args.waves,
                                      per_lane_queries=args.per_lane_queries, tile_order_factor=args.tile_order_factor,
                                      tail_fraction=args.tail_fraction)

    def step():
        st = render()
        if dist is not None:  # single RCCL gather of the tile buffers at frame end
            if cpu_render:
                t = time.perf_counter()
                shard.gather_frame(out, n_tiles, rank, world, dist, gathered, frame)
                gather_ms.append((time.perf_counter() - t) * 1e3)
                return st
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            shard.gather_frame(out if not shared else out.cpu(), n_tiles, rank, world, dist, gathered, frame)
            e1.record()
            gather_ms.append((e0, e1))
        return st

    for _ in range(args.warmup):
        step()
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    stats, step_s = [], []
    for _ in range(args.steps):
        ts = time.perf_counter()
        stats.append(step())  # stage timing reads the render's events back: each step has finished here
        step_s.append(time.perf_counter() - ts)
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    rays = sum(s.rays for s in stats)
    samples = sum(s.samples for s in stats)
    draws = sum(s.rng_draws for s in stats)
    kernel_ms = sum(s.kernel_ms for s in stats) / max(1, len(stats))
    timed_gathers = gather_ms[-args.steps:] if gather_ms else []
    g_ms = (sum(g if isinstance(g, float) else g[0].elapsed_time(g[1]) for g in timed_gathers) / len(timed_gathers)
            if timed_gathers else 0.0)
    rank_info = None
    if dist is not None:
        t = torch.tensor([elapsed, float(rays), float(samples), float(draws)], dtype=torch.float64, device=cdev)
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        elapsed = float(mx[0])
        rays, samples, draws = float(t[1]), float(t[2]), float(t[3])
        mine = torch.tensor([float(len(my_tiles)), g_ms, kernel_ms], dtype=torch.float64, device=cdev)
        every = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(every, mine)
        rank_info = [{"rank": r, "tiles": int(v[0]), "gather_ms": round(float(v[1]), 3),
                      "render_ms": round(float(v[2]), 2)} for r, v in enumerate(x.cpu().numpy() for x in every)]
        # Every rank leaves the group here.  What follows on rank 0 -- the reference scene build
        # (minutes for lucy's 28 M triangles) and the parity check of the gathered frame -- needs
        # no collective, so no rank waits on it inside a collective timeout.
        dist.barrier()
        dist.destroy_process_group()
    if rank != 0:
        return
    stall = float(os.environ.get("SP_BENCH_POST_STALL_S", "0") or 0)  # test hook: a slow reference build
    if stall > 0:
        time.sleep(stall)

    mrays = rays / elapsed / 1e6
    msamples = samples / elapsed / 1e6
    roofline = None if cpu_render else roofline_of(stats, min(len(my_tiles) * 64, args.width * args.height), args,
                                                   kernel_ms, scene.device_bytes())

    cpu = None
    parity = None
    if not args.no_cpu:
        # the reference library logs to stdout (base/Logger.cpp); keep stdout for the JSON line
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            if world == 1:  # the CPU baseline is timed at N=1 only
                cpu, parity = cpu_baseline(scene, path, integ, args, out, my_tiles, args.cpu_seconds)
                if args.cpu_scaling_seconds > 0 and cpu is not None and cpu["kind"] == "reference":
                    cpu["thread_scaling"] = cpu_thread_scaling(path, integ, args, my_tiles, cpu)
            else:  # parity of the GATHERED frame (all ranks' tiles, after the RCCL gather)
                _, parity = cpu_baseline(scene, path, integ, args, frame, np.arange(n_tiles, dtype=np.int32),
                                         args.parity_seconds)
                parity["frame"] = "gathered"
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)

    line = {
        "metric": "Mrays/sec (+ Msamples/sec) at fixed spp; per-pixel L2 vs CPU ref",
        "value": round(mrays, 2),
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        # wall time of each timed step (rank 0; render + gather), to show run-to-run spread
        "step_ms": {"min": round(min(step_s) * 1e3, 3), "max": round(max(step_s) * 1e3, 3)},
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": SCENES[args.scene]["data"],
        "config": {"workload": f"{fname} {args.width}x{args.height} @ {args.spp} spp, {args.integrator}",
                   "width": args.width, "height": args.height, "spp": args.spp, "integrator": args.integrator,
                   "bvh": "sah" if args.bvh == 0 else "reference", "tiles": int(n_tiles),
                   "pipeline": "cpu-oracle (test hook)" if cpu_render else
                               ["auto", "megakernel", "wavefront", "chunks"][stats[-1].pipeline],
                   "parallelism": f"tiles{world}"},
        "msamples_per_s": round(msamples, 3),
        "rays_per_step": rays / args.steps,
        "roofline": roofline,
        "cpu_baseline": cpu,
        "parity": parity,
        # which library ran (SP_LIB_PATH can swap it): path, content hash of its sources, .so hash
        "library": None if cpu_render else sp._abi.build_identity(),
    }
    if dist is not None:
        line["world_size"] = world
        if shared:
            line["test_shared_device"] = True  # not a multi-GPU measurement
        if cpu_render:
            line["test_cpu_render"] = True  # oracle on the host: orchestration test, not a measurement
        line["gather_ms"] = round(g_ms, 3)
        ms_step = elapsed / args.steps * 1e3
        render = [r["render_ms"] for r in rank_info]
        # per-rank render time: slowest over mean (1.0 = perfectly balanced shards); the gather's
        # share of a step (rank 0's gather, HIP events around the RCCL call)
        line["imbalance"] = round(max(render) / max(1e-9, sum(render) / len(render)), 4)
        line["gather_frac"] = round(g_ms / max(1e-9, ms_step), 5)
        line["ranks"] = rank_info
        if stall > 0:
            line["test_post_stall_s"] = stall
    print(json.dumps(line), flush=True)
    os.dup2(2, 1)  # exit-time log summaries of the reference library go to stderr


def sim_all_ranks(args, scene, integ, n_tiles, rdev):
    """--sim-world N --sim-rank -1: every rank's shard of an N-rank frame rendered on this one GPU in
    turn (warm-up, then --steps timed frames each; the same tiles and calls a rank makes, no
    collective), so the per-rank balance of the partition can be measured without N GPUs.  Prints
    one diagnostic line: per-rank ms per frame, render-kernel ms, rays; max / mean of each."""
    import torch

    import simplepath_amd as sp
    from simplepath_amd import shard

    stream = torch.cuda.current_stream().cuda_stream
    per_rank = shard.per_rank_capacity(n_tiles, args.sim_world)
    out = torch.zeros((per_rank, 64, 3), dtype=torch.float32, device=rdev)
    ranks = []
    for r in range(args.sim_world):
        tiles = shard.shard_tiles(n_tiles, r, args.sim_world)

        def render():
            return sp.render_tiles_device(scene, integ, args.spp, tiles, out.data_ptr(), stream, pipeline=args.pipeline,
                                          stage_timing=True, waves_per_simd=args.waves,
                                          tile_order_factor=args.tile_order_factor, tail_fraction=args.tail_fraction)
        for _ in range(args.warmup):
            render()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st = [render() for _ in range(args.steps)]
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / args.steps * 1e3
        rays = sum(x.rays for x in st) / args.steps
        ranks.append({"rank": r, "tiles": int(len(tiles)), "ms_per_frame": round(ms, 3),
                      "kernel_ms": round(sum(x.kernel_ms for x in st) / args.steps, 3),
                      "rays": int(rays), "mrays_per_s": round(rays / ms / 1e3, 2),
                      "pipeline": ["auto", "megakernel", "wavefront", "chunks"][st[-1].pipeline]})
        print(json.dumps(ranks[-1]), file=sys.stderr, flush=True)

    def imb(key):
        v = [x[key] for x in ranks]
        return round(max(v) / (sum(v) / len(v)), 4)
    line = {"diag": "sim_ranks", "scene": args.scene, "width": args.width, "height": args.height, "spp": args.spp,
            "integrator": args.integrator, "sim_world": args.sim_world, "shard": "interleaved (shard.shard_tiles)",
            "steps": args.steps, "warmup": args.warmup, "ranks": ranks,
            "imbalance_ms": imb("ms_per_frame"), "imbalance_rays": imb("rays"),
            "frame_ms_at_n": max(x["ms_per_frame"] for x in ranks),
            "library": sp._abi.build_identity()}
    print(json.dumps(line), flush=True)


def stage_bytes(st, pixels):
    """Algorithmic HBM bytes of each wavefront stage for one frame (DESIGN.md "Roofline").
    pixels = pixels in flight; per-pixel-sample SoA records: hit 16 B, shading point 16 B,
    shadow record 32 B per ray, rstate 4 B, queue entry 4 B, running sum 12 B (read + write)."""
    spp = max(1, st.samples // max(1, pixels))
    ps = pixels * spp
    hits, shadow, draws = st.primary_hits, st.shadow_rays, st.rng_draws
    return {
        "wf_primary": ps * 16 + (st.rays - shadow - hits) * 24,      # hit record; light-only sum RMW (upper bound)
        "wf_shade": ps * (16 + 8) + hits * (16 + 4) + shadow * 32 + draws * MT_BYTES_PER_DRAW,
        "wf_shadow": shadow * (16 + 4 + 24 + 32),
    }


def pmc_of_this_build(doc):
    """A committed PMC pass counts for this line only if it profiled the library this process
    loaded: its sp_build_id (tools/pmc_traffic.py / pmc_valu.py read it from the profiled bench
    runs) must equal the loaded build's.  Passes of another build -- or of none recorded -- give
    null traffic / valu, so a line never quotes counters of code it did not run."""
    try:
        import simplepath_amd as sp
        mine = sp._abi.build_identity()["build_id"]
    except Exception:
        return False
    return doc.get("sp_build_id") is not None and doc.get("sp_build_id") == mine


def valu_of(args, kernel):
    """VALU-issue roofline of `kernel` from a committed PMC pass of the same workload
    (tools/gpu_pmc_valu.sh -> tools/pmc_valu.py): issue cycles of its VALU instructions (f32/int
    2, f64 4, transcendental 8 cycles per wave-instruction, measured on gfx950) over 1024 SIMDs x
    its cycles.  None when no pass of this workload is committed."""
    try:
        with open(args.valu_json) as fh:
            vj = json.load(fh)
    except (OSError, ValueError):
        return None
    if (vj.get("width"), vj.get("height"), vj.get("spp"), vj.get("scene", "bunny"), vj.get("sim_world", 0)) != \
            (args.width, args.height, args.spp, args.scene, args.shard_n):
        return None
    if not pmc_of_this_build(vj):
        return None
    k = vj.get("kernels", {}).get(kernel)
    if not k:
        return None
    return {"frac": round(k["valu_frac"], 4), "wait_frac": round(k.get("wait_frac", 0.0), 4),
            "lane_util": round(k.get("lane_util", 0.0), 4), "kernel": kernel, "sp_build_id": vj["sp_build_id"],
            "valu_insts_per_launch": k["valu_insts"], "kernel_ms_profiled": round(k["ms_profiled"], 4),
            "source": os.path.relpath(args.valu_json, ROOT)}


def traffic_source(args, tj):
    return None if tj is None else {"file": os.path.relpath(args.traffic_json, ROOT), "sp_build_id": tj.get("sp_build_id")}


def roofline_of(stats, pixels, args, kernel_ms, scene_bytes=0):
    """Roofline of the dominant kernel: algorithmic bytes per launch / average launch duration
    (HIP events on the render stream, recorded around every launch inside the timed region).
    Algorithmic bytes: the RNG state traffic (24 B per draw), the output, and the resident scene
    (BVH nodes, primitive records, normals, ...) read at least once per frame -- 22 MB for bunny,
    ~2 GB for lucy's 28 M triangles, which do not fit the 256 MiB Infinity Cache."""
    st = stats[-1]
    n = len(stats)
    traffic, tj = None, None
    if os.path.exists(args.traffic_json):
        try:
            with open(args.traffic_json) as fh:
                tj = json.load(fh)
            if (tj.get("width") == args.width and tj.get("height") == args.height and tj.get("spp") == args.spp
                    and tj.get("scene", "bunny") == args.scene and tj.get("sim_world", 0) == args.shard_n
                    and pmc_of_this_build(tj)):
                traffic = tj.get("hbm_bytes_per_launch")
            else:
                tj = None
        except Exception:
            traffic, tj = None, None
    if st.pipeline == 3:  # sample chunks (sp_chunk.hip): the frame's kernels, timed together
        samples = st.samples
        # draws at 24 B (read + the twist of its generation), the hit record written once and read
        # by ck_count and ck_shade, the 2-byte draw count, radiance written once and summed
        alg = st.rng_draws * MT_BYTES_PER_DRAW + samples * (16 * 3 + 2 * 2 + 12 * 2) + pixels * PIXEL_BYTES + scene_bytes
        achieved = alg / (kernel_ms * 1e-3) / 1e9
        # fused form: (ck_camera, unless the camera pass runs in the fused queue: 2 launches), then the
        # counts and the chunks in sp_fused_kernel, ck_sum
        fused = st.launches <= 3
        kernels = (("ck_camera+" if st.launches == 3 else "") + "sp_fused_kernel+ck_sum") if fused \
            else "ck_camera+ck_count+ck_shade+ck_sum"
        if tj is not None:  # the frame's kernels together, like the time
            traffic = sum(v["hbm_bytes_per_launch"] for k, v in tj.get("kernels", {}).items()
                          if k.startswith("ck_") or (fused and k == "sp_fused_kernel")) or traffic
        return {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic, "kernel": kernels,
                "traffic_source": traffic_source(args, tj),
                "scene_bytes": scene_bytes,
                "kernel_ms": round(kernel_ms, 3), "alg_bytes_per_launch": alg,
                # the shading kernel: most of the frame's time
                "valu": valu_of(args, "sp_fused_kernel" if fused else "ck_shade")}
    if st.pipeline == 1 or args.integrator != "direct_lighting":  # megakernel
        # stage_ms[0]: the render kernel alone, [1]: the tile-order probe + partition before it
        # (HIP events on the render stream; sp_render_stats)
        render_ms = sum(s.stage_ms[0] for s in stats) / n
        probe_ms = sum(s.stage_ms[1] for s in stats) / n
        if not render_ms > 0:
            render_ms, probe_ms = kernel_ms, 0.0
        # with tail chunks (sp_render_stats.tail_tiles > 0) the render kernel is sp_tail_kernel, and
        # the same events also hold chunk_sum (ck_sum, ~0.1 ms).  The algorithmic bytes stay the
        # frame's (the tail tiles' hit records and per-sample radiance are not counted: the same
        # frame, the same bytes, whichever way it is scheduled)
        kname = "sp_tail_kernel" if st.tail_tiles > 0 else "sp_render_kernel"
        alg = st.rng_draws * MT_BYTES_PER_DRAW + pixels * PIXEL_BYTES + scene_bytes
        achieved = alg / (render_ms * 1e-3) / 1e9
        if tj is not None and kname in tj.get("kernels", {}):
            traffic = tj["kernels"][kname]["hbm_bytes_per_launch"]
        return {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic, "kernel": kname,
                "traffic_source": traffic_source(args, tj),
                "scene_bytes": scene_bytes, "tail_tiles": st.tail_tiles, "tail_chunks": st.tail_chunks,
                "kernel_ms": round(render_ms, 3), "probe_ms": round(probe_ms, 3), "alg_bytes_per_launch": alg,
                "valu": valu_of(args, kname)}
    names = ["wf_init+wf_resolve", "wf_primary", "wf_shade", "wf_shadow"]
    tot = [sum(s.stage_ms[k] for s in stats) / n for k in range(4)]
    spp = args.spp
    by = stage_bytes(st, pixels)
    # stage events time part 0, which holds about 1 / parts of the interleaved tiles
    tiles = (pixels + 63) // 64
    frac0 = 1.0 / max(1, st.parts)  # blocks of tiles dealt round-robin: about 1 / parts
    by = {k: v * frac0 for k, v in by.items()}
    stages = {}
    for k in (1, 2, 3):
        ms_launch = tot[k] / spp
        b_launch = by[names[k]] / spp
        stages[names[k]] = {"ms_per_launch": round(ms_launch, 4), "frame_ms": round(tot[k], 2),
                            "alg_bytes_per_launch": b_launch,
                            "gbs": round(b_launch / max(ms_launch, 1e-9) / 1e6, 1)}
    stages[names[0]] = {"frame_ms": round(tot[0], 3)}
    dom = max((1, 2, 3), key=lambda k: tot[k])
    d = stages[names[dom]]
    achieved = d["gbs"]
    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic, "kernel": names[dom],
            "parts": st.parts, "part0_fraction": round(frac0, 4),
            "kernel_ms": d["ms_per_launch"], "alg_bytes_per_launch": d["alg_bytes_per_launch"],
            "frame_kernel_ms": round(kernel_ms, 2), "stages": stages, "valu": valu_of(args, names[dom])}


def _ref_lib():
    """oracle/_ref/libsp_ref.so: the reference's own render path built from its sources (test
    infrastructure, present when the reference was available at build time)."""
    import ctypes as C
    path = os.path.join(ROOT, "oracle", "_ref", "libsp_ref.so")
    if not os.path.exists(path):
        return None
    L = C.CDLL(path)
    L.ref_scene_create.restype = C.c_void_p
    L.ref_scene_create.argtypes = [C.c_char_p, C.c_int, C.c_int]
    L.ref_scene_free.argtypes = [C.c_void_p]
    L.ref_render_tiles.restype = C.c_int
    L.ref_render_tiles.argtypes = [C.c_void_p, C.c_int, C.c_uint32, C.POINTER(C.c_int32), C.c_int64, C.c_int,
                                   C.POINTER(C.c_float)]
    return L


def cpu_thread_scaling(scene_path, integ, args, my_tiles, cpu):
    """The reference's own thread scaling on this host: the same random tiles at 1 thread and at
    the process's CPU share, a few seconds each.  The reference's default is hardware_concurrency()
    threads (main.cpp:314); the GPU box's pool rules give one GPU's process a 16-CPU share although
    the affinity mask shows the whole machine, so the whole-host rate is reported as a linear
    extrapolation of the share's per-thread rate -- an upper bound, labelled as such, not a
    measurement."""
    import ctypes as C
    ref = _ref_lib()
    if ref is None:
        return None
    ref_scene = ref.ref_scene_create(scene_path.encode(), args.width, args.height)
    if not ref_scene:
        return None
    order = np.random.default_rng(99).permutation(np.asarray(my_tiles)).astype(np.int32)
    share = args.cpu_threads if args.cpu_threads > 0 else cpu_share()
    from tests import _oracle
    legs = {}
    try:
        for threads in sorted({1, share}):
            done, t_used, chunk = 0, 0.0, threads
            while t_used < args.cpu_scaling_seconds and done < order.size:
                ids = np.ascontiguousarray(order[done:done + chunk])
                out = np.zeros((ids.size, 64, 3), dtype=np.float32)
                t0 = time.perf_counter()
                rc = ref.ref_render_tiles(ref_scene, int(integ), args.spp, ids.ctypes.data_as(C.POINTER(C.c_int32)),
                                          ids.size, threads, out.ctypes.data_as(C.POINTER(C.c_float)))
                t_used += time.perf_counter() - t0
                assert rc == 0
                done += ids.size
                chunk *= 2
            legs[threads] = (done, t_used)
    finally:
        ref.ref_scene_free(ref_scene)
    # rays of each leg's tiles from the oracle (bit-exact twin of the reference)
    res = {}
    s = sp_scene_for(scene_path, args)
    for threads, (done, t_used) in legs.items():
        _, st = _oracle.render(s, integ, args.spp, np.ascontiguousarray(order[:done]), threads=share, variant="glibc")
        res[threads] = {"tiles": done, "s": round(t_used, 2), "mrays_per_s": round(st["rays"] / t_used / 1e6, 4)}
    one, sh = res[1]["mrays_per_s"], res[share]["mrays_per_s"]
    host = affinity_cpus()
    return {"legs": {str(k): v for k, v in res.items()},
            "efficiency_at_share": round(sh / (one * share), 4) if one > 0 else None,
            "full_host_threads": host,
            "full_host_linear_estimate_mrays_per_s": round(sh / share * host, 3),
            "note": "estimate, not a measurement: the box's CPU share is %d of %d CPUs" % (share, host)}


def sp_scene_for(scene_path, args):
    import simplepath_amd as sp
    s = sp.Scene.from_file(scene_path)
    s.set_resolution(args.width, args.height)
    return s


def cpu_baseline(scene, scene_path, integ, args, gpu_out, my_tiles, budget_s):
    """CPU baseline on a bounded sample of the same frame (whole 8x8 tiles spread over the image,
    same spp and integrator, about --cpu-seconds of work): the reference itself (oracle/_ref,
    kind "reference") when built, else the C oracle (kind "port").  Ray counts come from the
    oracle on the same tiles (identical control flow: the two are bit-exact, tests/
    test_oracle_vs_ref.py), which also checks the GPU frame on those tiles."""
    import ctypes as C

    import simplepath_amd as sp
    from tests import _oracle

    n_tiles = sp.TileScheduler(args.width, args.height).get_num_tiles()
    threads = args.cpu_threads if args.cpu_threads > 0 else cpu_share()
    rng = np.random.default_rng(1234)
    order = rng.permutation(np.asarray(my_tiles)).astype(np.int32)  # tiles this GPU rendered (a shard with --sim-world)
    ref = _ref_lib()
    ref_scene = None
    build_s = None
    if ref is not None:  # parse + BVH build outside the timed region, as the reference's main does
        t_build = time.perf_counter()
        ref_scene = ref.ref_scene_create(scene_path.encode(), args.width, args.height)
        build_s = time.perf_counter() - t_build
        if not ref_scene:
            ref = None
    kind = "reference" if ref is not None else "port"

    def run(ids):
        if ref is not None:
            out = np.zeros((ids.size, 64, 3), dtype=np.float32)
            rc = ref.ref_render_tiles(ref_scene, int(integ), args.spp, ids.ctypes.data_as(C.POINTER(C.c_int32)),
                                      ids.size, threads, out.ctypes.data_as(C.POINTER(C.c_float)))
            assert rc == 0
            return out
        out, _ = _oracle.render(scene, integ, args.spp, ids, threads=threads, variant="glibc")
        return out

    done, t_used, chunk, tiles_out = [], 0.0, threads, []
    while t_used < budget_s and len(done) < order.size:
        ids = np.ascontiguousarray(order[len(done):len(done) + chunk])
        t0 = time.perf_counter()
        tiles_out.append(run(ids))
        dt = time.perf_counter() - t0
        t_used += dt
        done.extend(ids.tolist())
        if dt < budget_s / 8:
            chunk *= 2
    if ref_scene:
        ref.ref_scene_free(ref_scene)
    ids = np.array(done, dtype=np.int32)
    orc, st = _oracle.render(scene, integ, args.spp, ids, threads=threads, variant="glibc")
    base = np.concatenate(tiles_out, axis=0)
    cpu = {"value": round(st["rays"] / t_used / 1e6, 4), "unit": "Mrays/s", "cores": threads, "kind": kind,
           "sample": f"{len(done)} random 8x8 tiles of the same frame @ {args.spp} spp ({st['samples']} samples, "
                     f"{t_used:.1f} s, " + ("oracle/_ref/libsp_ref.so = reference sources" if ref is not None
                                             else "oracle liboracle_glibc.so") + ")",
           "msamples_per_s": round(st["samples"] / t_used / 1e6, 5), "host_cores": os.cpu_count(),
           "affinity_cpus": affinity_cpus(),
           "ref_scene_build_s": None if build_s is None else round(build_s, 2),  # parse + BVH, not timed
           "build": REF_BUILD if ref is not None else "oracle/Makefile: gcc -O2 -mavx2 -mfma -ffp-contract=off"}
    parity = {"vs": kind, "tiles": len(done)}
    if ref is not None:
        parity["oracle_bitexact_vs_reference"] = bool(np.array_equal(orc.view(np.uint32), base.view(np.uint32)))
    if gpu_out is not None:
        gpu = gpu_out.cpu().numpy()
        pos = {int(t): i for i, t in enumerate(my_tiles)}
        g = np.stack([gpu[pos[t]] for t in done])
        diff = np.linalg.norm((g - base).ravel())
        norm = np.linalg.norm(base.ravel())
        parity.update({"rel_l2": float(diff / max(norm, 1e-30)),
                       "bitexact_pixel_frac": float(np.mean(np.all(g == base, axis=-1)))})
    return cpu, parity


if __name__ == "__main__":
    main()
