#!/bin/bash
# Memory-pipeline PMC passes (TA/TD/TCP) on a reduced bench; one counter set per rocprofv3 run.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/pmc2}
mkdir -p $OUT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
ARGS="--steps 1 --warmup 0 --no-cpu --spp ${SPP:-8}"
cd /tmp
i=0
while IFS= read -r set; do
  [ -z "$set" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $R/$OUT/p$i -o run -- python3 $R/bench.py $ARGS > $R/$OUT/p$i.json 2> $R/$OUT/p$i.err || { echo "pmc pass $i failed"; tail -5 $R/$OUT/p$i.err; exit 1; }
done <<< "$SETS"
echo done
