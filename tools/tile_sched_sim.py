#!/usr/bin/env python3
"""Replay a SP_TILE_DIAG megakernel timeline (tools/tile_diag.py) as greedy list scheduling: each
of the W persistent waves takes the next tile of an order as soon as it is free, tiles taking the
durations measured.  Compares the measured queue order with longest-first (perfect knowledge)
and with cost classes of a given count and ratio (sp_mega.hip tile_order_kernel), with the
estimates perturbed by log-normal noise -- how much of the frame's tail an order can remove.

Usage: python3 tools/tile_sched_sim.py diag.bin [waves=4096]"""
import heapq
import sys

import numpy as np


def simulate(dur, order, waves):
    h = [0.0] * waves
    heapq.heapify(h)
    for i in order:
        heapq.heappush(h, heapq.heappop(h) + dur[i])
    return max(h)


def classes(est, k, factor, ratio):
    thr = factor * est.mean()
    c = np.zeros(len(est), int)
    for j in range(k - 1):
        c += est <= thr * ratio ** j
    return c


def main(path, waves=4096):
    waves = int(waves)
    rec = np.fromfile(path, dtype=np.uint64).reshape(-1, 8)
    rec = rec[rec[:, 1] > 0]
    dur = (rec[:, 1].astype(np.int64) - rec[:, 0].astype(np.int64)) / 1e5  # ms (s_memrealtime 100 MHz)
    item = rec[:, 3].astype(np.int64)
    slot = np.arange(len(dur))
    print(f"work / waves {dur.sum() / waves:.1f} ms, longest tile {dur.max():.1f} ms")
    print(f"measured queue order: {simulate(dur, np.argsort(item), waves):.1f} ms")
    rng = np.random.default_rng(1)
    for noise in (0.0, 0.15, 0.3):
        est = dur * np.exp(rng.normal(0.0, noise, len(dur)))
        row = [f"longest-first {simulate(dur, np.argsort(-est), waves):.1f}"]
        for k, f, r in ((6, 2, 0.5), (12, 2, 0.5 ** 0.5), (24, 4, 0.5 ** 0.25), (32, 4, 0.5 ** 0.2)):
            row.append(f"{k} classes x{r:.3f} {simulate(dur, np.lexsort((slot, classes(est, k, f, r))), waves):.1f}")
        print(f"estimate noise {noise}: " + "; ".join(row))


if __name__ == "__main__":
    main(*sys.argv[1:])
