#!/bin/bash
# Sample-chunk RNG store: interleaved words (_build) vs 4-word lane blocks with the grouped twist (_build_c4).
set -o pipefail
export TMPDIR=/tmp
run() { b=$1; shift; SP_LIB_PATH=$PWD/simplepath_amd/$b/libsimplepath_hip.so timeout -k 10 300 python bench.py --no-cpu "$@" > gpurun_out/ab.json 2>/dev/null || exit 1
  echo "$b $*: $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['value'], d['ms_per_step'], d.get('stage_ms'))")"; }
for r in 1 2; do for b in _build _build_c4; do run $b --sim-world 8; run $b --sim-world 2; done; done
SP_LIB_PATH=$PWD/simplepath_amd/_build_c4/libsimplepath_hip.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "chunk or shard" > gpurun_out/r4u_tests.log 2>&1 || { tail -30 gpurun_out/r4u_tests.log; exit 1; }
tail -1 gpurun_out/r4u_tests.log
