#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
TESTS="${TESTS:-shared or merged or rrnee or waves_per_simd}" bash -c 'timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$TESTS" > gpurun_out/r4h_tests.log 2>&1' || { tail -30 gpurun_out/r4h_tests.log; exit 1; }
tail -1 gpurun_out/r4h_tests.log
for r in 1 2; do
for v in "" "--per-lane-queries"; do
  timeout -k 10 200 python bench.py --no-cpu $v > gpurun_out/ab.json 2>/dev/null || exit 1
  echo "bunny $v: $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])")"
  timeout -k 10 200 python bench.py --no-cpu --scene elf --width 1024 --height 1024 --spp 16 $v > gpurun_out/ab.json 2>/dev/null || exit 1
  echo "elf $v: $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['value'], d['ms_per_step'])")"
done
done
bash tools/gpu_r4g.sh
