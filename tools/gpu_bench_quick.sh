#!/bin/bash
# Quick perf check: the default bench line without the CPU baseline, $1 repeats (default 2).
set -o pipefail
mkdir -p gpurun_out/quick
for i in $(seq 1 ${1:-2}); do
  timeout -k 10 200 python -u bench.py --no-cpu ${BENCH_ARGS:-} > gpurun_out/quick/b$i.json 2> gpurun_out/quick/b$i.err || { tail -5 gpurun_out/quick/b$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/quick/b$i.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],{k:v.get('ms_per_launch') for k,v in r.get('stages',{}).items()})"
done
