#!/bin/bash
# 6-class tile order as the default: the -m gpu suite, smoke, elf 8-way shard (probe on) and bunny.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4r_tests.log 2>&1 || { tail -30 gpurun_out/r4r_tests.log; exit 1; }
tail -1 gpurun_out/r4r_tests.log
timeout -k 10 300 python bench.py --no-cpu --scene elf --sim-world 8 --steps 2 --warmup 0 > gpurun_out/ab.json 2>/dev/null || exit 1
echo "elf8: $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['probe_ms'])")"
