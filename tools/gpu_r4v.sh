#!/bin/bash
# Persistent ck_camera: chunk tests, then the shard lines (before: bunny 8-way 2785-2790, 2-way 2957-2967).
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "chunk or shard or bench_ranks" > gpurun_out/r4v_tests.log 2>&1 || { tail -30 gpurun_out/r4v_tests.log; exit 1; }
tail -1 gpurun_out/r4v_tests.log
for a in "--sim-world 8" "--sim-world 2" "--sim-world 8" "--sim-world 4"; do
  timeout -k 10 300 python bench.py --no-cpu $a > gpurun_out/ab.json 2>/dev/null || exit 1
  echo "$a: $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['value'], d['ms_per_step'], d['step_ms'])")"
done
