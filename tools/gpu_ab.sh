#!/bin/bash
# A/B timing of library builds: tools/gpu_ab.sh <build_dir>...  (bunny; megakernel N=1, sim-world 8; wavefront N=1)
set -o pipefail
mkdir -p gpurun_out/ab
for b in "$@"; do
  lib=$PWD/simplepath_amd/$b/libsimplepath_hip.so
  for cfg in "megakernel 1" "megakernel 8" "wavefront 1"; do
    set -- $cfg
    SP_LIB_PATH=$lib timeout -k 10 120 python -u bench.py --no-cpu --steps 2 --warmup 1 --pipeline $1 --sim-world $2 > gpurun_out/ab/$b.$1.$2.json 2> gpurun_out/ab/$b.$1.$2.err || exit 1
    echo "$b $1 N=$2 $(python -c "import json;d=json.load(open('gpurun_out/ab/$b.$1.$2.json'));print(d['value'],d['ms_per_step'])")"
  done
done
