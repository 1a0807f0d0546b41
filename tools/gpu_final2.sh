#!/bin/bash
# Round-end measurement, part 2: the default line's VALU and HBM-traffic PMC passes (bunny), then
# config lines (CONFIGS) with their own PMC passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
if [ -z "${SKIP_BUNNY:-}" ]; then
  SCENE=bunny bash tools/gpu_pmc_valu.sh > gpurun_out/final2_valu.log 2>&1 || { tail -5 gpurun_out/final2_valu.log; exit 1; }
  tail -2 gpurun_out/final2_valu.log
  SCENE=bunny bash tools/gpu_pmc_traffic.sh > gpurun_out/final2_traffic.log 2>&1 || { tail -5 gpurun_out/final2_traffic.log; exit 1; }
  tail -1 gpurun_out/final2_traffic.log
fi
PMC=1 TRAFFIC=1 CONFIGS="${CONFIGS:-spheres bunny_scan}" bash tools/gpu_configs.sh
