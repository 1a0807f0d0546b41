#!/usr/bin/env python3
"""Compare the tile-order probe's per-tile times with the render's own tile durations.

Inputs are SP_TILE_DIAG timelines (sp_mega.hpp records, s_memrealtime at 100 MHz) written by a
build that also dumps the probe's tile times next to them as <diag>.probe (float32 per tile slot;
the diagnostic patch is profiles/r05/tile_order/probe_dump.patch).  Prints, in log space, how far
the probe time and the blended estimate (sp_mega.hip tile_est) stray from the render's duration,
and -- given two runs -- how far two probes of the same tiles stray from each other, which is the
part of the error the probe's own timing noise explains.  Then replays the render durations as list
scheduling (tools/tile_sched_sim.py) in the class order those estimates give.

Usage: python3 tools/probe_vs_render.py tiles_x diag1.bin [diag2.bin]"""
import sys

import numpy as np

from tile_sched_sim import classes, simulate


def load(path):
    rec = np.fromfile(path, dtype=np.uint64).reshape(-1, 8)
    dur = (rec[:, 1].astype(np.int64) - rec[:, 0].astype(np.int64)) / 100.0  # us, per slot
    probe = np.fromfile(path + ".probe", dtype=np.float32).astype(np.float64)
    return dur, probe, rec


def blend(t, tx):
    # sp_mega.hip tile_est: the larger of the row and the column blend
    n = len(t)
    i = np.arange(n)
    l, r = t[np.maximum(i - 1, 0)], t[np.minimum(i + 1, n - 1)]
    u = t[np.where(i >= tx, i - tx, i)]
    d = t[np.where(i + tx < n, i + tx, i)]
    return np.maximum(0.25 * (l + r) + 0.5 * t, 0.25 * (u + d) + 0.5 * t)


def spread(a, b):
    ok = (a > 0) & (b > 0)
    x = np.log(a[ok] / a[ok].mean()) - np.log(b[ok] / b[ok].mean())
    return x.std(), np.corrcoef(np.log(a[ok]), np.log(b[ok]))[0, 1]


def main(tx, paths):
    runs = [load(p) for p in paths]
    for p, (dur, probe, rec) in zip(paths, runs):
        waves = len(np.unique(rec[:, 2]))
        est = blend(probe, tx)
        print(f"== {p}: {len(dur)} tiles, {waves} waves, span {(rec[:, 1].max() - rec[:, 0].min()) / 1e5:.1f} ms")
        for name, e in (("probe time", probe), ("blended estimate", est)):
            s, c = spread(e, dur)
            print(f"  {name:17s} vs render duration: log-ratio sd {s:.3f}, log correlation {c:.3f}")
        s, c = spread(blend(dur, tx), dur)
        print(f"  {'render blended':17s} vs render duration: log-ratio sd {s:.3f}, log correlation {c:.3f}")
        work = dur.sum() / waves / 1000
        print(f"  replay (ms): work/waves {work:.1f}; longest-first {simulate(dur, np.argsort(-dur, kind='stable'), waves) / 1000:.1f}")
        for name, e in (("probe time", probe), ("blended estimate", est), ("exact duration", dur)):
            c = classes(e, 24, 2.0, 2 ** -0.25)
            print(f"    24 classes on {name:16s} {simulate(dur, np.argsort(c, kind='stable'), waves) / 1000:.1f}")
    if len(runs) == 2:
        s, c = spread(runs[0][1], runs[1][1])
        print(f"probe vs probe (two runs): log-ratio sd {s:.3f}, log correlation {c:.3f}")
        s, c = spread(runs[0][0], runs[1][0])
        print(f"render vs render (two runs): log-ratio sd {s:.3f}, log correlation {c:.3f}")


if __name__ == "__main__":
    main(int(sys.argv[1]), sys.argv[2:])
