#!/usr/bin/env python3
"""Sum rocprofv3 --pmc counters per kernel over every dispatch under a directory.

Usage: python3 tools/pmc_sum.py <dir> [kernel-substring ...]
Prints one line per kernel: dispatches, each counter's sum, and derived ratios when the
counters are there (wait / inst-wait fraction of wave cycles, I-cache miss rate).
"""
import collections
import csv
import glob
import os
import sys


def main():
    root = sys.argv[1]
    want = sys.argv[2:]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row["Kernel_Name"].split("(")[0]
                if want and not any(w in k for w in want):
                    continue
                per[k][row["Counter_Name"]] += float(row["Counter_Value"])
                disp[k].add((f, row["Dispatch_Id"]))
    for k, c in sorted(per.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        extra = {}
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if n in c:
                    extra[n.replace("SQ_", "").lower() + "_frac"] = round(c[n] / wc, 4)
        h, m = c.get("SQC_ICACHE_HITS"), c.get("SQC_ICACHE_MISSES")
        if h is not None and m is not None and h + m > 0:
            extra["icache_miss_rate"] = round(m / (h + m), 5)
        vals = " ".join(f"{n}={v:.4g}" for n, v in sorted(c.items()))
        print(f"{k[:48]:48s} n={len(disp[k])} {vals} {extra}")


if __name__ == "__main__":
    main()
