#!/bin/bash
# Tile order: 2 cost classes (_build, round 3) vs 4 / 6 classes by halving thresholds (descending).
set -o pipefail
for r in 1 2; do
for b in _build _build_k6 _build_k4; do
  L=$PWD/simplepath_amd/$b/libsimplepath_hip.so
  SP_LIB_PATH=$L timeout -k 10 200 python bench.py --no-cpu > gpurun_out/ab.json 2>/dev/null || exit 1
  echo "bunny $b: $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])")"
done
done
SP_LIB_PATH=$PWD/simplepath_amd/_build_k6/libsimplepath_hip.so SP_TILE_DIAG=gpurun_out/td_k6.bin timeout -k 10 200 python bench.py --no-cpu --steps 1 --warmup 1 > gpurun_out/td_k6.json && python tools/tile_diag.py gpurun_out/td_k6.bin || exit 1
for b in _build _build_k6 _build_k4; do
  L=$PWD/simplepath_amd/$b/libsimplepath_hip.so
  SP_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu --scene lucy > gpurun_out/ab.json 2>/dev/null || exit 1
  echo "lucy $b: $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])")"
done
