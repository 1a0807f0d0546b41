#!/bin/bash
# A/B of environment settings on one box: bench.py --no-cpu for each ";"-separated entry of
# $CONFIGS (e.g. "SP_X=0;SP_X=1"), repeated $REPEAT times in alternation.
set -o pipefail
mkdir -p gpurun_out/ab
IFS=';' read -ra CF <<< "${CONFIGS:-}"
for r in $(seq 1 ${REPEAT:-2}); do
  for cfg in "${CF[@]}"; do
    env $cfg timeout -k 10 200 python -u bench.py --no-cpu ${BENCH_ARGS:-} > gpurun_out/ab/b.json 2> gpurun_out/ab/b.err || { tail -5 gpurun_out/ab/b.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ab/b.json'));r=d['roofline'];print('$cfg |', d['value'],d['ms_per_step'],{k:v.get('ms_per_launch') for k,v in r.get('stages',{}).items()})"
  done
done
