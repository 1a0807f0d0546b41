#!/bin/bash
# Quick perf check: tests then one bench line per configuration given in $CONFIGS (env-prefixed).
set -o pipefail
cd "$(dirname "$0")"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
i=0
while IFS= read -r cfg; do
  [ -z "$cfg" ] && continue
  i=$((i+1))
  env $cfg timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu > gpurun_out/qb_$i.json 2> gpurun_out/qb_$i.err
  rc=$?; echo "[$cfg] exit $rc"; python3 -c "
import json,sys; d=json.load(open('gpurun_out/qb_$i.json')); r=d['roofline']
print(d['value'], 'Mrays/s', d['ms_per_step'], 'ms', {k:(v.get('ms_per_launch'),v.get('frame_ms')) for k,v in r.get('stages',{}).items()})"
  [ $rc -eq 0 ] || exit $rc
done <<< "$CONFIGS"
