#!/bin/bash
# A/B of library builds on the chunk pipeline shards: tools/gpu_ab_chunks.sh <build_dir>...
set -o pipefail
mkdir -p gpurun_out/abc
for b in "$@"; do
  for n in 8 4; do
    SP_LIB_PATH=$PWD/simplepath_amd/$b/libsimplepath_hip.so timeout -k 10 150 python -u bench.py --no-cpu --steps 2 --warmup 1 --pipeline chunks --sim-world $n > gpurun_out/abc/$b.$n.json 2> gpurun_out/abc/$b.$n.err || exit 1
    echo "$b N=$n $(python -c "import json;d=json.load(open('gpurun_out/abc/$b.$n.json'));print(d['value'],d['ms_per_step'])")"
  done
done
