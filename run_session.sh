#!/bin/bash
# GPU session: parity tests, then one bench line per BENCH_ARGS entry (";"-separated).
set -o pipefail
cd "$(dirname "$0")"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -v "^Debug" gpurun_out/pytest_gpu.log | tail -15
[ $rc -eq 0 ] || exit $rc
i=0
IFS=';' read -ra BA <<< "${BENCH_ARGS:-}"
for a in "${BA[@]}"; do
  i=$((i+1))
  timeout -k 10 600 python bench.py $a > gpurun_out/bench_$i.json 2> gpurun_out/bench_$i.err
  rc=$?; echo "[bench $a] exit $rc"; cat gpurun_out/bench_$i.json; grep -v "^Debug" gpurun_out/bench_$i.err | tail -3
  [ $rc -eq 0 ] || exit $rc
done
