#!/bin/bash
# rocprofv3 kernel-trace summary of one bench configuration ($BENCH_ARGS) -> gpurun_out/$NAME
set -o pipefail
cd "$(dirname "$0")/.."
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${NAME:-prof} -o run -- python3 $R/bench.py $BENCH_ARGS > $R/gpurun_out/${NAME:-prof}.json 2> $R/gpurun_out/${NAME:-prof}.err
rc=$?; echo "rocprof exit $rc"; cat $R/gpurun_out/${NAME:-prof}.json | head -c 600; echo
head -12 $R/gpurun_out/${NAME:-prof}/run_kernel_stats.csv | cut -c1-220
