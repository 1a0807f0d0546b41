#!/bin/bash
# Wave-level region profile (-DSP_WAVE_PROF build in simplepath_amd/_ab/wprof, tools/wprof.py).
#   WPROF_RUNS  ";"-separated bench.py argument lists (default: elf 1024^2 @ 16 spp; bunny 1080p)
set -o pipefail
mkdir -p gpurun_out/wprof
lib=$PWD/simplepath_amd/_ab/wprof/libsimplepath_hip.so
IFS=';' read -ra RN <<< "${WPROF_RUNS:---scene elf --width 1024 --height 1024 --spp 16;--spp 64}"
i=0
for a in "${RN[@]}"; do
  i=$((i+1))
  SP_LIB_PATH=$lib SP_TILE_DIAG=gpurun_out/wprof/d$i.bin timeout -k 10 200 python -u bench.py --no-cpu --steps 1 --warmup 0 $a \
    > gpurun_out/wprof/b$i.json 2> gpurun_out/wprof/b$i.err || { tail -5 gpurun_out/wprof/b$i.err; exit 1; }
  echo "== $a: $(python -c "import json;d=json.load(open('gpurun_out/wprof/b$i.json'));print(d['value'],'Mrays/s',d['config']['pipeline'])")"
  python tools/wprof.py gpurun_out/wprof/d$i.bin
done
