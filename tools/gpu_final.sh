#!/bin/bash
# Round-end measurement in one call: the PMC passes of every config workload on this build
# (tools/gpu_pmc_all.sh), copied into profiles/ so the lines below cite them, then the -m gpu
# suite, smoke, the default bench line and its rocprof summary (tools/gpu_check.sh PROF=1) into
# gpurun_out/${OUT:-final}.  The config lines (tools/gpu_configs.sh) run in a second call.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
env -u TAG bash tools/gpu_pmc_all.sh || exit 1
cp gpurun_out/pmc_bench_*.json gpurun_out/pmc_valu_bench_*.json profiles/ || exit 1
PROF=1 bash tools/gpu_check.sh ${OUT:-final}
