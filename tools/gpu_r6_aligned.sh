#!/bin/bash
# Round 6: aligned-pair draws for the glossy estimate (SP_RHO_ALIGNED / SP_SERVED_ALIGNED A/B
# builds in simplepath_amd/_ab/) -- the parity suites on each variant, then bunny and elf A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/r6al
B=simplepath_amd
for v in algn algnsrv; do
  SP_LIB_PATH=$R/$B/_ab/$v/libsimplepath_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_tail.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6al/tests_$v.log 2>&1 \
    || { tail -30 gpurun_out/r6al/tests_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r6al/tests_$v.log)"
done
RUNS="$B/_build;$B/_ab/algn;$B/_ab/algnsrv" WORKLOADS="; --scene elf --width 1024 --height 1024 --spp 16; --scene elf --sim-world 8 --steps 1 --warmup 1" REPEAT=2 \
  bash tools/gpu_ab.sh > gpurun_out/r6al/ab.log 2>&1 || { tail -20 gpurun_out/r6al/ab.log; exit 1; }
cat gpurun_out/r6al/ab.log
