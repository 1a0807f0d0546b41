#!/usr/bin/env python3
"""Host memory and wall time of N concurrent scene loads + SAH BVH builds, as N ranks of
`bench.py --gpus N` do before their first render (sp_scene_load + the upload's host BVH build).

    python tools/host_build_mem.py --scene lucy --ranks 8 [--threads 16]

Each rank is a child process: parse the scene (PLY/STL reading, FileParser), then build the SAH
BVH and its 8-wide form on the host (sp_scene_bvh_build_info, the same builders sp_scene_upload
runs; no device).  Reports each rank's wall time and peak RSS, and the machine's peak of used
memory (MemTotal - MemAvailable) sampled every 0.2 s while the ranks run."""
import argparse
import json
import multiprocessing as mp
import os
import resource
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def used_bytes():
    info = {}
    with open("/proc/meminfo") as fh:
        for line in fh:
            k, v = line.split(":", 1)
            info[k] = int(v.split()[0]) * 1024
    return info["MemTotal"] - info["MemAvailable"]


def rank_job(path, threads, q):
    os.environ["OMP_NUM_THREADS"] = str(threads)
    import simplepath_amd as sp
    t0 = time.perf_counter()
    s = sp.Scene.from_file(path)
    t1 = time.perf_counter()
    info = s.bvh_build_info(0)
    t2 = time.perf_counter()
    q.put({"load_s": round(t1 - t0, 2), "bvh_s": round(t2 - t1, 2),
           "peak_rss_gb": round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6, 3), "bvh": info})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="lucy")
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--workdir", default="/tmp/sp_host_build")
    a = ap.parse_args()
    from simplepath_amd import scenes
    path = {"lucy": scenes.write_lucy_scene, "elf": scenes.write_elf_scene, "bunny": scenes.write_bunny_scene}[a.scene](a.workdir)
    base = used_bytes()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    t0 = time.perf_counter()
    procs = [ctx.Process(target=rank_job, args=(path, a.threads, q)) for _ in range(a.ranks)]
    for p in procs:
        p.start()
    peak = 0
    while any(p.is_alive() for p in procs):
        peak = max(peak, used_bytes() - base)
        time.sleep(0.2)
    wall = time.perf_counter() - t0
    res = [q.get() for _ in procs]
    print(json.dumps({"scene": a.scene, "ranks": a.ranks, "threads_per_rank": a.threads, "cpus": os.cpu_count(),
                      "wall_s": round(wall, 1), "machine_peak_used_gb": round(peak / 1e9, 2),
                      "sum_rank_peak_rss_gb": round(sum(r["peak_rss_gb"] for r in res), 2),
                      "per_rank": [{k: r[k] for k in ("load_s", "bvh_s", "peak_rss_gb")} for r in res],
                      "bvh": res[0]["bvh"]}))


if __name__ == "__main__":
    main()
