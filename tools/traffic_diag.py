#!/usr/bin/env python3
"""Summarise a -DSP_TRAFFIC_DIAG render (sp_path.hpp SP_TD): the SP_TILE_DIAG file's u64 slots
16 + 2k / 17 + 2k hold, per source k, the distinct 128-byte lines the wave-level accesses touched
and the bytes the lanes asked for.  With the bench line of the same run (rays, draws) and an
optional FETCH_SIZE / WRITE_SIZE total (bytes per frame), prints the table of requests by source.

Usage: python3 tools/traffic_diag.py <diag.bin> <bench.json> [fetch_bytes write_bytes]"""
import json
import sys

import numpy as np

NAMES = ["8-wide BVH nodes", "wide-leaf triangles", "binary slot records", "closest-hit records",
         "RNG draws (own stream)", "RNG touches (LDS-DMA)", "RNG served-estimate reads", "twists (read+write)",
         "seeding"]
BOUNCE = 9  # IterativeRRNEE: wave bounce iterations, and the lanes alive in them


def main(path, bench, fetch=None, write=None):
    v = np.fromfile(path, dtype=np.uint64)[16:16 + 2 * len(NAMES)].astype(np.float64)
    with open(bench) as fh:
        b = json.loads([x for x in fh.read().splitlines() if x.startswith("{")][-1])
    rays = b.get("rays_per_step") or 0.0
    tot_lines = sum(v[0::2])
    print(f"{'source':28s} {'lines':>10s} {'line GB':>9s} {'share':>6s} {'lane GB':>9s} {'B/ray':>8s}")
    for k, n in enumerate(NAMES):
        lines, by = v[2 * k], v[2 * k + 1]
        print(f"{n:28s} {lines:10.3e} {lines * 128 / 1e9:9.1f} {lines / max(tot_lines, 1):6.3f} {by / 1e9:9.1f} "
              f"{lines * 128 / max(rays, 1):8.1f}")
    print(f"{'total':28s} {tot_lines:10.3e} {tot_lines * 128 / 1e9:9.1f}")
    it, live = np.fromfile(path, dtype=np.uint64)[16 + 2 * BOUNCE:18 + 2 * BOUNCE].astype(np.float64)
    if it:
        print(f"IterativeRRNEE bounce iterations {it:.4e} (wave-level), live lanes per iteration {live / it:.2f} "
              f"of 64 (lock-step efficiency {live / (64 * it):.3f})")
    if fetch is not None:
        print(f"counters: FETCH {float(fetch) / 1e9:.1f} GB, WRITE {float(write) / 1e9:.1f} GB per frame")


if __name__ == "__main__":
    main(*sys.argv[1:])
