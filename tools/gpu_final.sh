#!/bin/bash
# Round-end measurement.  STAGES (default "pmc check"; run "configs" in a second call):
#   pmc      the VALU and HBM-traffic PMC passes of every config workload on this build
#            (tools/gpu_pmc_all.sh, WORKLOADS to narrow it), copied into profiles/ so the lines
#            run after them cite counters of the same build (bench.py checks sp_build_id);
#   check    the -m gpu suite, smoke, the default bench line with the CPU baseline and its rocprofv3
#            --kernel-trace --stats summary (tools/gpu_check.sh PROF=1) into gpurun_out/${OUT:-final};
#   configs  every config line (tools/gpu_configs.sh; CONFIGS to narrow it) with the reference CPU
#            path and parity beside it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
for stage in ${STAGES:-pmc check}; do
  case $stage in
    pmc) env -u TAG bash tools/gpu_pmc_all.sh || exit 1
         cp gpurun_out/pmc_bench_*.json gpurun_out/pmc_valu_bench_*.json profiles/ || exit 1 ;;
    check) PROF=1 bash tools/gpu_check.sh ${OUT:-final} || exit 1 ;;
    configs) bash tools/gpu_configs.sh || exit 1 ;;
    *) echo "unknown stage $stage"; exit 2 ;;
  esac
done
