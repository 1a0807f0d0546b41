#!/usr/bin/env python3
"""Instruction mix per innermost loop of a kernel's ISA (hipcc -S output), attributing every
instruction to the loop LLVM's comments place its basic block in ("This Loop Header: Depth=d",
"in Loop: Header=BBx_y").

Usage: python3 tools/isa_loops.py <kernel.s> [loop-header]   (with a header: its opcode histogram)
The DirectLighting kernel's ISA: hipcc --offload-arch=gfx950 <the Makefile's flags> -S
--offload-device-only -c simplepath_amd/csrc/hip/sp_mega_direct.hip, then the lines of
sp_render_kernel<6, 4>."""
import collections
import re
import sys


def blocks(lines):
    cur = "top"
    for l in lines:
        s = l.strip()
        if re.match(r"^\.LBB\d+_\d+:|^; %bb\.\d+:", s):
            m = re.search(r"Header=(BB\d+_\d+) Depth=(\d+)", s)
            m2 = re.search(r"This Loop Header: Depth=(\d+)", s)
            lab = s.split(":")[0].lstrip(".").replace("LBB", "BB")
            cur = lab if m2 else (m.group(1) if m else "top")
            continue
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        yield cur, s.split()[0]


def main(path, header=None):
    lines = open(path).read().split("\n")
    if header:
        c = collections.Counter(op for loop, op in blocks(lines) if loop == header)
        for op, n in c.most_common(50):
            print(op, n)
        return
    stats = collections.defaultdict(collections.Counter)
    for loop, op in blocks(lines):
        c = stats[loop]
        c["n"] += 1
        if op.startswith("v_readlane"):
            c["readlane"] += 1
        elif op.startswith("v_writelane"):
            c["writelane"] += 1
        elif op.startswith("scratch_"):
            c["scratch"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
        elif op.startswith("v_"):
            c["valu"] += 1
        if "f64" in op:
            c["f64"] += 1
    for k, c in sorted(stats.items(), key=lambda x: -x[1]["n"])[:30]:
        print(k, dict(c))


if __name__ == "__main__":
    main(*sys.argv[1:])
