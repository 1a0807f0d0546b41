#!/usr/bin/env python3
"""HBM traffic per launch from rocprofv3 FETCH_SIZE / WRITE_SIZE passes (tools/gpu_pmc_traffic.sh).

Correction (MI355X_MICROARCH.md "HBM"): FETCH_SIZE reports half the bytes of coalesced reads on
gfx950 -> doubled; WRITE_SIZE is exact.  Both are in KiB.  Calibrated on this code's own
patterns: wf_init's 8-byte-per-lane MT seeding stores (known 2512 B per pixel) and wf_resolve's
4-byte-per-lane reads (known 12 B per pixel) reproduce their byte counts with these factors.

Usage: python3 tools/pmc_traffic.py <pmc dir with p1 (FETCH) and p2 (WRITE)> <width> <height> <spp> <out.json>
"""
import re
import collections
import csv
import glob
import json
import os
import sys


def kernel_key(name):
    """'void spd::wf_shade<4>(spd::Scene, ...)' -> 'wf_shade' (template instances merged;
    '(anonymous namespace)::' dropped)."""
    k = name.replace("(anonymous namespace)::", "")
    if k.startswith("void "):
        k = k[5:]
    return k.split("(")[0].split("<")[0].split("::")[-1]


def per_kernel(root, counter):
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] == counter:
                    vals[kernel_key(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    return vals


def build_id_of_passes(root):
    """sp_build_id of the library the profiled bench runs loaded (their JSON lines, p*.json beside
    the counter directories); None unless every pass ran the same build."""
    ids = set()
    for f in sorted(glob.glob(os.path.join(root, "p*.json"))):
        try:
            with open(f) as fh:
                line = [x for x in fh.read().splitlines() if x.startswith("{")][-1]
            ids.add((json.loads(line).get("library") or {}).get("build_id"))
        except (OSError, ValueError, IndexError):
            ids.add(None)
    return ids.pop() if len(ids) == 1 else None


def main():
    root, w, h, spp, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
    scene = sys.argv[6] if len(sys.argv) > 6 else "bunny"  # bench.py --scene of the profiled run
    sim_world = int(sys.argv[7]) if len(sys.argv) > 7 else 0  # bench.py --sim-world of the profiled run
    fetch = per_kernel(os.path.join(root, "p1"), "FETCH_SIZE")
    write = per_kernel(os.path.join(root, "p2"), "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        if k.startswith("__amd") or "at::" in k:
            continue
        f, wr = fetch.get(k, []), write.get(k, [])
        n = max(len(f), len(wr), 1)
        fb = 2.0 * 1024.0 * sum(f) / max(len(f), 1)
        wb = 1024.0 * sum(wr) / max(len(wr), 1)
        kernels[re.sub(r"\bspd::(mt_blk\d+::)?", "", k)] = {"dispatches": n, "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
                                           "hbm_bytes_per_launch": fb + wb}
    dom = "wf_shade" if "wf_shade" in kernels else max(kernels, key=lambda k: kernels[k]["hbm_bytes_per_launch"])
    res = {"sp_build_id": build_id_of_passes(root), "width": w, "height": h, "spp": spp, "scene": scene, "sim_world": sim_world, "kernel": dom,
           "hbm_bytes_per_launch": kernels[dom]["hbm_bytes_per_launch"], "kernels": kernels,
           "correction": "FETCH_SIZE x2 (gfx950 half-count), WRITE_SIZE x1, KiB -> bytes"}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
