#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
for r in 1 2; do
for b in _build _build_p16 _build_p64; do
  SP_LIB_PATH=$PWD/simplepath_amd/$b/libsimplepath_hip.so timeout -k 10 200 python bench.py --no-cpu --scene elf --width 1024 --height 1024 --spp 16 > gpurun_out/ab.json 2>/dev/null || exit 1
  echo "elf $b: $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['value'], d['ms_per_step'])")"
done
done
for w in 2 4; do
  timeout -k 10 200 python bench.py --no-cpu --scene elf --width 1024 --height 1024 --spp 16 --waves $w > gpurun_out/ab.json 2>/dev/null || exit 1
  echo "elf waves $w: $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['value'], d['ms_per_step'])")"
done
timeout -k 10 400 python bench.py --scene elf --steps 2 --warmup 0 --sim-world 8 --cpu-seconds 8 > gpurun_out/elf8.json 2> gpurun_out/elf8.err || { tail -5 gpurun_out/elf8.err; exit 1; }
echo "elf shard8: $(python -c "import json;d=json.load(open('gpurun_out/elf8.json'));print(d['value'], d['ms_per_step'], d['step_ms'], d['cpu_baseline']['value'], d['parity'])")"
