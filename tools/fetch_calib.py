#!/usr/bin/env python3
"""FETCH_SIZE / WRITE_SIZE calibration from tools/ubench/fetch_calib (see its header).

Usage: python3 tools/fetch_calib.py <dir with p1 (FETCH_SIZE) and p2 (WRITE_SIZE) passes> <out.json>
Prints, per access width, counter KiB x 1024 / bytes moved: the factor to divide the raw counter
by (FETCH_SIZE of a 16 B/lane stream is documented at 0.5 on gfx950).
"""
import collections
import csv
import glob
import json
import os
import sys

BYTES = 2 << 30


def per_kernel(root, counter):
    v = collections.defaultdict(float)
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] != counter:
                    continue
                v[row["Kernel_Name"].split("(")[0].replace("void ", "")] += float(row["Counter_Value"])
    return v


def main():
    root, out = sys.argv[1], sys.argv[2]
    fetch = per_kernel(os.path.join(root, "p1"), "FETCH_SIZE")
    write = per_kernel(os.path.join(root, "p2"), "WRITE_SIZE")
    res = {"bytes_per_kernel": BYTES, "fetch_counter_over_bytes": {}, "write_counter_over_bytes": {}}
    for k, kib in fetch.items():
        if k.startswith("rd"):
            res["fetch_counter_over_bytes"][k] = kib * 1024.0 / BYTES
    for k, kib in write.items():
        if k.startswith("wr"):
            res["write_counter_over_bytes"][k] = kib * 1024.0 / BYTES
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
