#!/bin/bash
# Tile cost estimate: probe time (_build) vs blended with the queue neighbours' (_build_sm); then the
# -m gpu suite on _build.
set -o pipefail
export TMPDIR=/tmp
run() { b=$1; shift; SP_LIB_PATH=$PWD/simplepath_amd/$b/libsimplepath_hip.so timeout -k 10 300 python bench.py --no-cpu "$@" > gpurun_out/ab.json 2>/dev/null || exit 1
  echo "$b $*: $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], r['kernel_ms'], r.get('probe_ms'))")"; }
for r in 1 2; do for b in _build _build_sm; do run $b; done; done
for b in _build _build_sm; do run $b --scene lucy; done
for b in _build _build_sm; do run $b --scene elf --sim-world 8 --steps 2 --warmup 0; done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4t_tests.log 2>&1 || { tail -30 gpurun_out/r4t_tests.log; exit 1; }
tail -1 gpurun_out/r4t_tests.log
