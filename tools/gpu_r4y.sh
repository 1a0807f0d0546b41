#!/bin/bash
# One-pass twist (_build, SP_TWIST_FUSED 1) vs the two-part twist (_build_ti2): the -m gpu suite,
# then bunny, elf 1024^2 @ 16 spp and bunny's 8-way shard, alternating.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not bench_ranks" > gpurun_out/r4y_tests.log 2>&1 || { tail -30 gpurun_out/r4x_tests.log; exit 1; }
tail -1 gpurun_out/r4y_tests.log
run() { b=$1; shift; SP_LIB_PATH=$PWD/simplepath_amd/$b/libsimplepath_hip.so timeout -k 10 300 python bench.py --no-cpu "$@" > gpurun_out/ab.json 2>/dev/null || exit 1
  echo "$b $*: $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['value'], d['ms_per_step'])")"; }
for r in 1 2; do for b in _build _build_ti2; do
  run $b; run $b --scene elf --width 1024 --height 1024 --spp 16; run $b --sim-world 8
done; done
