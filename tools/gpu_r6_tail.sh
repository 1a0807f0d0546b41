#!/bin/bash
# Round 6: the megakernel's tail chunks -- bit-identity against the plain megakernel, then an A/B of
# the tail fraction on bunny (tools/gpu_ab.sh, alternating passes on one box).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/r6tail
B=simplepath_amd/_build
timeout -k 10 180 python -u tools/tail_check.py bunny 8 > gpurun_out/r6tail/check.log 2>&1 || { cat gpurun_out/r6tail/check.log; exit 1; }
cat gpurun_out/r6tail/check.log
RUNS=${RUNS:-"$B SP_TAIL_FRAC=0;$B SP_TAIL_FRAC=0.05;$B SP_TAIL_FRAC=0.08;$B SP_TAIL_FRAC=0.12 SP_TAIL_CHUNKS=64"} \
  WORKLOADS=${WORKLOADS:-} bash tools/gpu_ab.sh > gpurun_out/r6tail/ab.log 2>&1 || { tail -20 gpurun_out/r6tail/ab.log; exit 1; }
cat gpurun_out/r6tail/ab.log
