#!/bin/bash
# stage profile of the megakernel's tiles (-DSP_MEGA_PROF build) at N=1 and the 8-way shard
set -o pipefail
mkdir -p gpurun_out/mp
lib=$PWD/simplepath_amd/_ab/mprof/libsimplepath_hip.so
for n in 1 8; do
  SP_LIB_PATH=$lib SP_TILE_DIAG=gpurun_out/mp/d$n.bin timeout -k 10 150 python -u bench.py --no-cpu --steps 1 --warmup 0 --pipeline megakernel --sim-world $n > gpurun_out/mp/b$n.json 2> gpurun_out/mp/b$n.err || exit 1
  echo "== N=$n"; python tools/tile_diag.py gpurun_out/mp/d$n.bin
done
