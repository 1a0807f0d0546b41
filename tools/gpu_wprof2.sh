#!/bin/bash
# Wave-level region profiles of several -DSP_WAVE_PROF builds on one workload (tools/wprof.py).
#   LIBS        space-separated build dirs (default: simplepath_amd/_ab/wprof)
#   WPROF_ARGS  bench.py arguments (default: elf 1024^2 @ 16 spp)
set -o pipefail
mkdir -p gpurun_out/wprof
i=0
for b in ${LIBS:-simplepath_amd/_ab/wprof}; do
  i=$((i+1))
  SP_LIB_PATH=$PWD/$b/libsimplepath_hip.so SP_TILE_DIAG=gpurun_out/wprof/d$i.bin timeout -k 10 200 python -u bench.py --no-cpu --steps 1 --warmup 0 ${WPROF_ARGS:---scene elf --width 1024 --height 1024 --spp 16} \
    > gpurun_out/wprof/b$i.json 2> gpurun_out/wprof/b$i.err || { tail -5 gpurun_out/wprof/b$i.err; exit 1; }
  echo "== $b: $(python -c "import json;d=json.load(open('gpurun_out/wprof/b$i.json'));print(d['value'],'Mrays/s',d['config']['pipeline'])")"
  python tools/wprof.py gpurun_out/wprof/d$i.bin | tee gpurun_out/wprof/w$i.txt
done
