#!/bin/bash
# Wave profiles of the DirectLighting megakernel, shared vs per-lane shadow walks (bunny 64 spp).
set -o pipefail
mkdir -p gpurun_out/wprof
for v in "" "--per-lane-queries"; do
  SP_LIB_PATH=$PWD/simplepath_amd/_build_wprof/libsimplepath_hip.so SP_TILE_DIAG=gpurun_out/wprof/dl.bin timeout -k 10 200 python -u bench.py --no-cpu --steps 1 --warmup 0 --spp 64 $v > gpurun_out/wprof/dl.json 2> gpurun_out/wprof/dl.err || { tail -5 gpurun_out/wprof/dl.err; exit 1; }
  echo "== bunny 64 spp $v: $(python -c "import json;d=json.load(open('gpurun_out/wprof/dl.json'));print(d['value'],'Mrays/s')")"
  python tools/wprof.py gpurun_out/wprof/dl.bin
done
