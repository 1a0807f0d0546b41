#!/usr/bin/env python3
"""Summarise a -DSP_WAVE_PROF render (sp_path.hpp SP_WPROF regions): the SP_TILE_DIAG file's first
16 u64 hold, per region k, the waves' shader clocks inside it (2k) and clocks x active lanes (2k+1).
Prints each region's share of the sample time (region 0) and its lane occupancy."""
import sys

import numpy as np

NAMES = ["sample (integrate)", "glossy rho estimate", "closest-hit queries", "shadow / MIS queries",
         "merged queries: walk steps", "merged queries: whole pass", "closest-hit walk steps", "any-hit walk steps"]


def main(path):
    v = np.fromfile(path, dtype=np.uint64)[:16].astype(np.float64)
    total = max(v[0], 1.0)
    for k, name in enumerate(NAMES):
        cyc, lane = v[2 * k], v[2 * k + 1]
        occ = lane / (64.0 * cyc) if cyc else 0.0
        print(f"{name:26s} wave-clocks {cyc:.4e}  share of sample {cyc / total:6.3f}  lane occupancy {occ:.3f}")
    if v[0]:
        rest = v[0] - v[2] - v[4] - v[6] - v[10]  # regions 1, 2, 3 and the merged pass (4 lies inside 5)
        rest_l = v[1] - v[3] - v[5] - v[7] - v[11]
        print(f"{'rest of the sample':26s} wave-clocks {rest:.4e}  share of sample {rest / total:6.3f}  "
              f"lane occupancy {rest_l / (64.0 * rest) if rest else 0.0:.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
