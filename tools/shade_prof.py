#!/usr/bin/env python3
"""Stage breakdown of wf_shade from a SP_WAVE_DIAG dump of a -DSP_SHADE_PROF build.

Usage: python3 tools/shade_prof.py diag.bin
Per wave: t0 start, t1 after rng load + twist-ahead, t2 after finish_hit, t3 after light
sampling, t4 after material eval, t5 end (latest lane).  s_memrealtime ticks at 100 MHz."""
import sys

import numpy as np

rec = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 8)[:, :6].astype(np.int64)
rec = rec[(rec[:, 0] > 0) & (rec[:, 5] > 0)]
t0 = rec[:, 0]
names = ["rng load+prepare", "hit + finish_hit", "light_sample", "material_eval", "rest (records)"]
prev = t0.copy()
print(f"waves={len(rec)} span_us={(rec[:, 5].max() - t0.min()) / 100:.1f} wave_us mean={(rec[:, 5] - t0).mean() / 100:.2f}")
for k, nm in enumerate(names, start=1):
    cur = np.where(rec[:, k] > 0, rec[:, k], prev)
    d = (cur - prev) / 100.0
    print(f"  {nm:20s} mean={d.mean():8.2f} us  p50={np.median(d):8.2f}  p99={np.percentile(d, 99):8.2f}")
    prev = np.maximum(prev, cur)
