#!/bin/bash
# The VALU-roofline and HBM-traffic PMC passes (tools/gpu_pmc_valu.sh, tools/gpu_pmc_traffic.sh) of
# every workload in WORKLOADS ("scene:simworld" pairs, default: all the config lines), so that the
# bench lines run AFTER them cite counters of the same build (bench.py checks sp_build_id).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
for w in ${WORKLOADS:-bunny:0 spheres:0 bunny_scan:0 bunny:2 bunny:4 bunny:8 lucy:0 lucy:8 elf:8}; do
  sc=${w%%:*}; sw=${w##*:}
  SCENE=$sc SIMW=$sw bash tools/gpu_pmc_valu.sh > gpurun_out/pmcv_$sc$sw.log 2>&1 || { tail -5 gpurun_out/pmcv_$sc$sw.log; exit 1; }
  tail -1 gpurun_out/pmcv_$sc$sw.log
  SCENE=$sc SIMW=$sw bash tools/gpu_pmc_traffic.sh > gpurun_out/pmct_$sc$sw.log 2>&1 || { tail -5 gpurun_out/pmct_$sc$sw.log; exit 1; }
  tail -1 gpurun_out/pmct_$sc$sw.log
done
