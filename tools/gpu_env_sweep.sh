#!/bin/bash
# bench under several env settings: SWEEP_ARGS="bench args" SWEEP_TAG=x tools/gpu_env_sweep.sh "A=1 B=2" "A=2" ...
set -o pipefail
mkdir -p gpurun_out/sw
i=0
for cfg in "$@"; do
  i=$((i+1))
  f=gpurun_out/sw/${SWEEP_TAG:-r}$i
  env $cfg timeout -k 10 150 python -u bench.py --no-cpu --steps 2 --warmup 1 $SWEEP_ARGS > $f.json 2> $f.err || exit 1
  echo "[$cfg $SWEEP_ARGS] $(python -c "import json;d=json.load(open('$f.json'));print(d['value'],d['ms_per_step'],d['config']['pipeline'])")"
done
