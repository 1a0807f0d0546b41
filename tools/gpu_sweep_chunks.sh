#!/bin/bash
# Chunks-per-pixel sweep on the chunk pipeline shards: tools/gpu_sweep_chunks.sh "<N:chunks ...>"
set -o pipefail
mkdir -p gpurun_out/swc
for nc in $1; do
  n=${nc%%:*}; c=${nc##*:}
  SP_CHUNKS=$c timeout -k 10 150 python -u bench.py --no-cpu --steps 2 --warmup 1 --pipeline chunks --sim-world $n > gpurun_out/swc/$n.$c.json 2> gpurun_out/swc/$n.$c.err || exit 1
  echo "N=$n chunks=$c $(python -c "import json;d=json.load(open('gpurun_out/swc/$n.$c.json'));print(d['value'],d['ms_per_step'])")"
done
