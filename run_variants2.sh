#!/bin/bash
# Bench the same configuration ($BENCH_ARGS) against library builds listed in $LIBS (dirs under simplepath_amd/).
set -o pipefail
cd "$(dirname "$0")"
mkdir -p gpurun_out
export TMPDIR=/tmp
for d in $LIBS; do
  SP_LIB_PATH=$PWD/simplepath_amd/$d/libsimplepath_hip.so timeout -k 10 300 python bench.py $BENCH_ARGS > gpurun_out/var_$d.json 2> gpurun_out/var_$d.err || { echo "$d failed"; tail -3 gpurun_out/var_$d.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/var_$d.json'));print('$d', d['value'], {k:v.get('ms_per_launch') for k,v in d['roofline'].get('stages',{}).items()})"
done
