#!/usr/bin/env python3
"""Analyse a SP_WAVE_DIAG per-wave timeline (sp_wave.hip diag_record).

Usage: python3 tools/wave_diag.py diag.bin n_pixel_waves
Prints, for the primary and shadow launches: wave durations, node steps per wave, and the
average number of resident waves (sum of wave lifetimes / launch span)."""
import sys

import numpy as np


def summarize(name, rec):
    rec = rec[rec[:, 1] > 0]
    if rec.size == 0:
        print(name, "no records")
        return
    t0, t1 = rec[:, 0].astype(np.int64), rec[:, 1].astype(np.int64)
    dur_us = (t1 - t0) / 100.0  # s_memrealtime: 100 MHz
    span_us = (t1.max() - t0.min()) / 100.0
    steps = (rec[:, 2] & 0xffffffff).astype(np.int64)
    lanes = (rec[:, 2] >> 32).astype(np.int64)
    hw = (rec[:, 3] & 0xffffffff).astype(np.int64)
    xcc = (rec[:, 3] >> 32).astype(np.int64) & 0xf
    cu = (hw >> 8) & 0xf
    se = (hw >> 13) & 0x7
    print(f"{name}: waves={len(rec)} span={span_us:.1f}us resident_avg={dur_us.sum() / span_us:.0f} "
          f"dur_us mean={dur_us.mean():.1f} p50={np.median(dur_us):.1f} p99={np.percentile(dur_us, 99):.1f} "
          f"max={dur_us.max():.1f}")
    print(f"   steps mean={steps.mean():.1f} p50={np.median(steps):.0f} p99={np.percentile(steps, 99):.0f} "
          f"max={steps.max()}  lanes mean={lanes.mean():.1f}  us/step={dur_us.sum() / max(1, steps.sum()):.3f}")
    # concurrency over time (per 1 us bins)
    b0 = ((t0 - t0.min()) // 100).astype(np.int64)
    b1 = ((t1 - t0.min()) // 100).astype(np.int64)
    conc = np.zeros(b1.max() + 2)
    np.add.at(conc, b0, 1)
    np.add.at(conc, b1 + 1, -1)
    conc = np.cumsum(conc)
    print(f"   concurrency max={conc.max():.0f} mean={conc[:-1].mean():.0f}; distinct (xcc,se,cu)="
          f"{len(set(zip(xcc.tolist(), se.tolist(), cu.tolist())))}")
    q = np.percentile(conc[:-1], [10, 50, 90])
    print(f"   concurrency p10/p50/p90 = {q[0]:.0f}/{q[1]:.0f}/{q[2]:.0f}")


def main():
    a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 4)
    n = int(sys.argv[2])
    summarize("wf_primary", a[:n])
    summarize("wf_shadow", a[n:])


if __name__ == "__main__":
    main()
