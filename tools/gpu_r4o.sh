#!/bin/bash
# IterativeRRNEE occupancy re-check after the RNG layout and seeding changes (bench.py --waves).
set -o pipefail
for r in 1 2; do
for w in 3 4 2; do
  timeout -k 10 200 python bench.py --no-cpu --scene elf --width 1024 --height 1024 --spp 16 --waves $w > gpurun_out/ab.json 2>/dev/null || exit 1
  echo "elf waves $w: $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['value'], d['ms_per_step'])")"
done
done
for w in 3 4; do
  timeout -k 10 300 python bench.py --no-cpu --scene elf --sim-world 8 --steps 2 --warmup 0 --waves $w > gpurun_out/ab.json 2>/dev/null || exit 1
  echo "elf8 waves $w: $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['value'], d['ms_per_step'])")"
done
