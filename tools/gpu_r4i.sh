#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${TESTS:-merged or rrnee or waves_per_simd or clipped or full_scale_tiles}" > gpurun_out/r4i_tests.log 2>&1 || { tail -30 gpurun_out/r4i_tests.log; exit 1; }
tail -1 gpurun_out/r4i_tests.log
for r in 1 2; do
for v in "" "--per-lane-queries"; do
  timeout -k 10 200 python bench.py --no-cpu --scene elf --width 1024 --height 1024 --spp 16 $v > gpurun_out/ab.json 2>/dev/null || exit 1
  echo "elf $v: $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['value'], d['ms_per_step'])")"
done
done
timeout -k 10 200 python bench.py --no-cpu > gpurun_out/ab.json 2>/dev/null || exit 1
echo "bunny: $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['value'], d['ms_per_step'])")"
