#!/bin/bash
# Occupancy-variant sweep of the DirectLighting render kernel on the bench workload.
set -o pipefail
cd "$(dirname "$0")"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for v in ${VARIANTS:-1 2 3 4}; do
  SP_KERNEL_VARIANT=$v timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/bench_v$v.json 2> gpurun_out/bench_v$v.err || { echo "variant $v failed"; tail -5 gpurun_out/bench_v$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bench_v$v.json'));print('variant $v', d['value'], 'Mrays/s', d['ms_per_step'], 'ms', d['roofline']['kernel_ms'])"
done
