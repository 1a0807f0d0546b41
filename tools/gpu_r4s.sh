#!/bin/bash
# Tile order forced where AUTO leaves queue order (spheres 1024^2 @ 64 spp: 4 tiles per wave; elf
# 1024^2 @ 16 spp), and the factor on bunny.
set -o pipefail
run() { timeout -k 10 300 python bench.py --no-cpu "$@" > gpurun_out/ab.json 2>/dev/null || exit 1
  echo "$*: $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], r['kernel_ms'], r.get('probe_ms'))")"; }
for r in 1 2; do
  run --scene spheres
  run --scene spheres --tile-order-factor 2
  run --scene elf --width 1024 --height 1024 --spp 16
  run --scene elf --width 1024 --height 1024 --spp 16 --tile-order-factor 2
  run --tile-order-factor 2
  run --tile-order-factor 4
  run --tile-order-factor 1
done
