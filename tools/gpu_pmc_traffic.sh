#!/bin/bash
# FETCH_SIZE and WRITE_SIZE (separate passes: they cannot share one) on the default bench frame,
# then per-launch HBM bytes per kernel -> gpurun_out/pmc_bench_bunny.json.
set -o pipefail
cd "$(dirname "$0")/.."
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmct
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmct/p1 -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > $R/gpurun_out/pmct/p1.json 2> $R/gpurun_out/pmct/p1.err || { echo "fetch pass failed"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmct/p2 -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > $R/gpurun_out/pmct/p2.json 2> $R/gpurun_out/pmct/p2.err || { echo "write pass failed"; exit 1; }
cd $R && python3 tools/pmc_traffic.py gpurun_out/pmct 1920 1080 256 gpurun_out/pmc_bench_bunny.json > /dev/null && echo done
