#!/bin/bash
# Tile order: 2 classes (_build) vs 6 classes (_build_k6) vs 6 classes from a 2-sample probe (_build_k6p2).
set -o pipefail
for r in 1 2; do
for b in _build _build_k6 _build_k6p2; do
  L=$PWD/simplepath_amd/$b/libsimplepath_hip.so
  SP_LIB_PATH=$L timeout -k 10 200 python bench.py --no-cpu > gpurun_out/ab.json 2>/dev/null || exit 1
  echo "bunny $b: $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['probe_ms'])")"
done
done
for b in _build _build_k6 _build_k6p2 _build _build_k6; do
  L=$PWD/simplepath_amd/$b/libsimplepath_hip.so
  SP_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu --scene lucy > gpurun_out/ab.json 2>/dev/null || exit 1
  echo "lucy $b: $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['probe_ms'])")"
done
