#!/bin/bash
# bench the default frame under several env settings: tools/gpu_env_sweep.sh "A=1 B=2" "A=2" ...
set -o pipefail
mkdir -p gpurun_out/sw
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 150 python -u bench.py --no-cpu --steps 2 --warmup 1 $SWEEP_ARGS > gpurun_out/sw/r$i.json 2> gpurun_out/sw/r$i.err || exit 1
  echo "[$cfg] $(python -c "import json;d=json.load(open('gpurun_out/sw/r$i.json'));s=d['roofline']['stages'];print(d['value'],d['ms_per_step'],{k:v.get('ms_per_launch') for k,v in s.items()})")"
done
