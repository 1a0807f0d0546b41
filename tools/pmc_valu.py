#!/usr/bin/env python3
"""VALU-issue roofline per kernel from rocprofv3 --pmc passes of the bench (tools/gpu_pmc_valu.sh).

The shading kernels do exact glibc-libm arithmetic (f32 + f64) and move few bytes, so their
roofline is the SIMDs' VALU issue rate, not HBM.  Per launch:

  valu_cycles = 2 * (VALU - F64 - TRANS)   wave64 f32 / int32 / logic
              + 4 * (FMA_F64 + ADD_F64 + MUL_F64 + INT64)
              + 8 * TRANS_F32
              + 16 * TRANS_F64
  cycles per wave-instruction per SIMD measured on gfx950 by tools/ubench/valu_rate.hip
  (profiles/r02/valu_rate.txt, 4-8 waves per SIMD): v_mul_f32 / v_xor_b32 2.2-2.4, v_mul_f64 /
  v_add_f64 4.2, v_exp_f32 8.2 (INT64 and f64 transcendentals by analogy: 4 and 16)
  kernel_cycles = GRBM_GUI_ACTIVE / 8     (rocprofv3 sums the 8 XCDs' busy cycles; microarch guide)
  valu_frac   = valu_cycles / (1024 SIMDs * kernel_cycles)

SQ_INSTS_* count wave-instructions.  Under --pmc every dispatch runs alone, so kernel_cycles is the
kernel's own duration (no overlap with the other part's kernels as in the timed bench).
Also per kernel: lane_util = SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU), wait_frac =
SQ_WAIT_ANY / SQ_WAVE_CYCLES, L1 tag lookups per VMEM instruction = TCP_TOTAL_ACCESSES_sum /
SQ_INSTS_VMEM_RD.

Usage: python3 tools/pmc_valu.py <pmc dir with p1..pN> <width> <height> <spp> <out.json>
"""
import collections
import csv
import glob
import json
import os
import sys

N_SIMD = 1024  # 256 CUs x 4 SIMDs


def kernel_key(name):
    """'void spd::wf_shade<4>(spd::Scene, ...)' -> 'wf_shade' (template instances merged;
    '(anonymous namespace)::' dropped)."""
    k = name.replace("(anonymous namespace)::", "")
    if k.startswith("void "):
        k = k[5:]
    return k.split("(")[0].split("<")[0].split("::")[-1]


def load(root):
    """{kernel: {counter: [per-dispatch values]}} and {kernel: [durations ns]} over all passes."""
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    durs = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
        seen = set()
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = kernel_key(row["Kernel_Name"])
                vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
                key = (row["Dispatch_Id"], k)
                if key not in seen:
                    seen.add(key)
                    durs[k].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    return vals, durs


def mean(x):
    return sum(x) / len(x) if x else 0.0


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
    vals, durs = load(root)
    res = {}
    for k, c in vals.items():
        if k.startswith("__amd") or "at::" in k:
            continue
        m = {n: mean(v) for n, v in c.items()}
        if "SQ_INSTS_VALU" not in m or not m.get("GRBM_GUI_ACTIVE"):
            continue
        f64 = sum(m.get(n, 0.0) for n in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                                           "SQ_INSTS_VALU_INT64"))
        t32, t64 = m.get("SQ_INSTS_VALU_TRANS_F32", 0.0), m.get("SQ_INSTS_VALU_TRANS_F64", 0.0)
        rest = max(0.0, m["SQ_INSTS_VALU"] - f64 - t32 - t64)
        vcyc = 2.0 * rest + 4.0 * f64 + 8.0 * t32 + 16.0 * t64
        kcyc = m["GRBM_GUI_ACTIVE"] / 8.0
        d = {"dispatches": len(c["SQ_INSTS_VALU"]), "valu_insts": m["SQ_INSTS_VALU"], "valu_cycles": vcyc,
             "kernel_cycles": kcyc, "valu_frac": vcyc / (N_SIMD * kcyc),
             "ms_profiled": mean(durs[k]) / 1e6, "clock_ghz": kcyc / (mean(durs[k]) * 1e-9) / 1e9 if durs[k] else None,
             "insts": {n.replace("SQ_INSTS_", ""): v for n, v in m.items() if n.startswith("SQ_INSTS")}}
        if m.get("SQ_ACTIVE_INST_VALU"):
            d["lane_util"] = m.get("SQ_THREAD_CYCLES_VALU", 0.0) / (64.0 * m["SQ_ACTIVE_INST_VALU"])
        if m.get("SQ_WAVE_CYCLES"):
            d["wait_frac"] = m.get("SQ_WAIT_ANY", 0.0) / m["SQ_WAVE_CYCLES"]
            d["valu_active_frac_per_wave"] = m.get("SQ_ACTIVE_INST_VALU", 0.0) / m["SQ_WAVE_CYCLES"]
        if m.get("SQ_INSTS_VMEM_RD") and m.get("TCP_TOTAL_ACCESSES_sum"):
            d["l1_lookups_per_vmem_rd"] = m["TCP_TOTAL_ACCESSES_sum"] / m["SQ_INSTS_VMEM_RD"]
        for n in ("TCP_PENDING_STALL_CYCLES_sum", "TA_TA_BUSY_sum", "SQ_WAVES"):
            if n in m:
                d[n] = m[n]
        res[k] = d
    doc = {"sp_build_id": build_id_of_passes(root), "width": w, "height": h, "spp": spp, "scene": scene, "sim_world": sim_world, "model": __doc__.split("Usage:")[0].strip(), "kernels": res}
    with open(out, "w") as fh:
        json.dump(doc, fh, indent=1)
    for k, d in sorted(res.items(), key=lambda x: -x[1]["valu_cycles"] * x[1]["dispatches"]):
        print(f"{k:14s} n={d['dispatches']:5d} ms={d['ms_profiled']:.3f} valu_frac={d['valu_frac']:.3f} "
              f"insts/launch={d['valu_insts']:.3g} lane_util={d.get('lane_util', 0):.3f} "
              f"wait={d.get('wait_frac', 0):.3f} l1/vmem={d.get('l1_lookups_per_vmem_rd', 0):.1f} "
              f"clk={d['clock_ghz'] or 0:.2f}")


if __name__ == "__main__":
    main()
