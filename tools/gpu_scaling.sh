#!/bin/bash
# Per-GPU load at N ranks, simulated on one GPU (bench.py --sim-world); AUTO pipeline, tile order on/off.
set -o pipefail
mkdir -p gpurun_out/scal
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/scal/tests.log 2>&1 || { tail -30 gpurun_out/scal/tests.log; exit 1; }
tail -3 gpurun_out/scal/tests.log
for n in 1 2 4 8; do
  timeout -k 10 120 python -u bench.py --no-cpu --steps 3 --warmup 1 --sim-world $n > gpurun_out/scal/auto_$n.json 2> gpurun_out/scal/auto_$n.err || exit 1
  echo "auto N=$n $(python -c "import json;d=json.load(open('gpurun_out/scal/auto_$n.json'));print(d['value'],d['ms_per_step'],d.get('config',{}).get('pipeline'))")"
done
for n in 2 4 8; do
  SP_TILE_ORDER=0 timeout -k 10 120 python -u bench.py --no-cpu --steps 3 --warmup 1 --sim-world $n > gpurun_out/scal/noord_$n.json 2> gpurun_out/scal/noord_$n.err || exit 1
  echo "noorder N=$n $(python -c "import json;d=json.load(open('gpurun_out/scal/noord_$n.json'));print(d['value'],d['ms_per_step'])")"
done
