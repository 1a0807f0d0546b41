#!/bin/bash
# Round 6, call A: timing-only bounds (SP_XP_*) and the occluder-cache default, A/B on one box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/r6
B=simplepath_amd
SMOKE=1 RUNS="$B/_build;$B/_ab/occ1;$B/_ab/dup1;$B/_ab/dup2;$B/_ab/flibm" bash tools/gpu_ab.sh > gpurun_out/r6/ab_bunny.log 2>&1 \
  || { tail -20 gpurun_out/r6/ab_bunny.log; exit 1; }
cat gpurun_out/r6/ab_bunny.log
RUNS="$B/_build;$B/_ab/flibm;$B/_ab/srvfree;$B/_ab/dup1" WORKLOADS="--scene elf --width 1024 --height 1024 --spp 16" \
  bash tools/gpu_ab.sh > gpurun_out/r6/ab_elf.log 2>&1 || { tail -20 gpurun_out/r6/ab_elf.log; exit 1; }
cat gpurun_out/r6/ab_elf.log
