#!/usr/bin/env python3
"""Analyse a SP_TILE_DIAG megakernel timeline (sp_mega.hpp: per tile slot {t0, t1, wave, item,
4 stage shader-clock totals of a -DSP_MEGA_PROF build}, s_memrealtime at 100 MHz).  Usage: python3 tools/tile_diag.py diag.bin
Prints tile durations, tiles per persistent wave and the number of tiles in flight over the
launch, which separates a load-imbalance tail from a uniformly slow render."""
import sys

import numpy as np


def main(path):
    rec = np.fromfile(path, dtype=np.uint64).reshape(-1, 8)
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
    prof = rec[:, 4:8].astype(np.float64)
    if prof.sum() > 0:  # -DSP_MEGA_PROF build: per stage, the slowest lane's shader clocks
        tot = prof.sum(axis=1)
        slow = np.argsort(-dur)[: max(1, len(dur) // 100)]
        names = ["trace", "light_sample", "material_eval", "occlusion"]
        for label, sel in (("all tiles", slice(None)), ("slowest 1%", slow)):
            share = prof[sel].sum(axis=0) / max(1.0, tot[sel].sum())
            print(f"{label}: " + " ".join(f"{n}={s:.2f}" for n, s in zip(names, share)) +
                  f"  (stage clocks / (tile wall us * 100): {tot[sel].mean() / max(1.0, dur[sel].mean() * 100):.1f})")
    last = t0.argmax()
    print(f"last tile started at {t0[last] / 1e5:.2f}ms and ran {dur[last] / 1000:.2f}ms")


if __name__ == "__main__":
    main(sys.argv[1])
