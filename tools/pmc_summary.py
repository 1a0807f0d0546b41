#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (tools/gpu_pmc.sh) per kernel.

Usage: python3 tools/pmc_summary.py gpurun_out/pmc [--json out.json]

Sums every counter over all dispatches of a kernel (one pass per counter set), then derives:
  valu_util   = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES     share of wave time issuing VALU
  lane_util   = SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU)   active lanes per VALU op
  wait_frac   = SQ_WAIT_ANY / SQ_WAVE_CYCLES             share of wave time in s_waitcnt
  hbm_bytes   = (FETCH_SIZE + WRITE_SIZE) * 1024         TCC->EA traffic, KB units
                 (MI355X_MICROARCH.md: gfx950 FETCH_SIZE is reported in KB; see the HBM section
                  for the 64B/128B request accounting -- raw values are kept alongside)
"""
import collections
import csv
import glob
import json
import os
import sys


def load(root):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    calls = collections.defaultdict(set)
    dur = collections.defaultdict(dict)
    for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row["Kernel_Name"].split("(")[0]
                per[name][row["Counter_Name"]] += float(row["Counter_Value"])
                calls[name].add((f, row["Dispatch_Id"]))
                dur[name][(f, row["Dispatch_Id"])] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
                per[name]["_vgpr"] = float(row["VGPR_Count"])
                per[name]["_sgpr"] = float(row["SGPR_Count"])
                per[name]["_lds"] = float(row["LDS_Block_Size"])
    return per, calls, dur


def derive(c):
    d = {}
    wc = c.get("SQ_WAVE_CYCLES", 0.0)
    if wc:
        d["valu_util"] = c.get("SQ_ACTIVE_INST_VALU", 0.0) / wc
        d["wait_frac"] = c.get("SQ_WAIT_ANY", 0.0) / wc
        d["active_any_frac"] = c.get("SQ_ACTIVE_INST_ANY", 0.0) / wc
    if c.get("SQ_ACTIVE_INST_VALU"):
        d["lane_util"] = c.get("SQ_THREAD_CYCLES_VALU", 0.0) / (64.0 * c["SQ_ACTIVE_INST_VALU"])
    if "FETCH_SIZE" in c or "WRITE_SIZE" in c:
        d["hbm_bytes"] = (c.get("FETCH_SIZE", 0.0) + c.get("WRITE_SIZE", 0.0)) * 1024.0
    if c.get("TCC_HIT_sum", 0.0) + c.get("TCC_MISS_sum", 0.0):
        d["l2_hit"] = c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    if c.get("SQ_WAVES"):
        d["valu_insts_per_wave"] = c.get("SQ_INSTS_VALU", 0.0) / c["SQ_WAVES"]
    return d


def main():
    root = sys.argv[1]
    per, calls, dur = load(root)
    out = {}
    for name in sorted(per, key=lambda n: -sum(dur[n].values())):
        if name.startswith("__amd") or "at::native" in name:
            continue
        c = per[name]
        n_calls = len({k[1] for k in calls[name]} ) or 1
        passes = len({k[0] for k in calls[name]}) or 1
        ms = sum(dur[name].values()) / 1e6 / passes
        out[name] = {"dispatches_per_pass": len(calls[name]) // passes, "avg_ms_per_pass": ms,
                     "counters": {k: v for k, v in c.items()}, "derived": derive(c)}
        dv = out[name]["derived"]
        print(f"{name}: dispatches/pass={len(calls[name]) // passes} ms/pass={ms:.2f} VGPR={c['_vgpr']:.0f} "
              f"SGPR={c['_sgpr']:.0f} LDS={c['_lds']:.0f}")
        print("   " + "  ".join(f"{k}={v:.3g}" for k, v in sorted(c.items()) if not k.startswith("_")))
        print("   " + "  ".join(f"{k}={v:.3f}" for k, v in dv.items()))
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
