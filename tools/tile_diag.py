#!/usr/bin/env python3
"""Analyse a SP_TILE_DIAG megakernel timeline (sp_mega.hpp: per tile slot {t0, t1, wave, item},
s_memrealtime at 100 MHz).  Usage: python3 tools/tile_diag.py diag.bin
Prints tile durations, tiles per persistent wave and the number of tiles in flight over the
launch, which separates a load-imbalance tail from a uniformly slow render."""
import sys

import numpy as np


def main(path):
    rec = np.fromfile(path, dtype=np.uint64).reshape(-1, 4)
    rec = rec[rec[:, 1] > 0]
    t0 = rec[:, 0].astype(np.int64)
    t1 = rec[:, 1].astype(np.int64)
    base = t0.min()
    t0 -= base
    t1 -= base
    dur = (t1 - t0) / 100.0  # us
    span = t1.max() / 100.0
    waves = np.unique(rec[:, 2])
    print(f"tiles={len(rec)} waves={len(waves)} tiles/wave={len(rec) / len(waves):.2f} span={span / 1000:.2f}ms")
    print(f"tile us: mean={dur.mean():.0f} p10={np.percentile(dur, 10):.0f} p50={np.median(dur):.0f} "
          f"p90={np.percentile(dur, 90):.0f} max={dur.max():.0f}")
    busy = dur.sum() / 100.0 * 100.0
    bins = 20
    edges = np.linspace(0, t1.max(), bins + 1)
    inflight = []
    for b in range(bins):
        lo, hi = edges[b], edges[b + 1]
        ov = np.clip(np.minimum(t1, hi) - np.maximum(t0, lo), 0, None).sum()
        inflight.append(ov / (hi - lo))
    print("in flight per 5% of span:", " ".join(f"{x:.0f}" for x in inflight))
    print(f"mean in flight={busy / span:.0f} peak={max(inflight):.0f}; "
          f"span if peak held throughout={dur.sum() / max(inflight) / 1000:.2f}ms")
    last = t0.argmax()
    print(f"last tile started at {t0[last] / 1e5:.2f}ms and ran {dur[last] / 1000:.2f}ms")


if __name__ == "__main__":
    main(sys.argv[1])
