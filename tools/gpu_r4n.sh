#!/bin/bash
# Fused seeding in the sample-chunk replay (ck_count): the -m gpu suite, then the shard lines.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not bench_ranks" > gpurun_out/r4n_tests.log 2>&1 || { tail -30 gpurun_out/r4n_tests.log; exit 1; }
tail -1 gpurun_out/r4n_tests.log
for a in "--sim-world 8" "--scene lucy --sim-world 8" "--sim-world 8" "--scene elf --sim-world 8 --steps 2 --warmup 0"; do
  timeout -k 10 300 python bench.py --no-cpu $a > gpurun_out/ab.json 2>/dev/null || exit 1
  echo "$a: $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['value'], d['ms_per_step'], d['step_ms'])")"
done
