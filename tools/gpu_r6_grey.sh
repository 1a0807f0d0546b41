#!/bin/bash
# Round 6: the rho estimate computes one colour channel for a grey microfacet colour
# (rho_accumulate, SP_RHO_GREY) -- parity suites on the new product build, then A/B against the
# previous build (simplepath_amd/_ab/base) on bunny, spheres and elf.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/r6grey
B=simplepath_amd
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_tail.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6grey/tests.log 2>&1 \
  || { tail -30 gpurun_out/r6grey/tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/r6grey/tests.log)"
RUNS="$B/_ab/base;$B/_build" WORKLOADS="; --scene elf --width 1024 --height 1024 --spp 16; --scene lucy --width 1920 --height 1080 --spp 256" REPEAT=3 \
  bash tools/gpu_ab.sh > gpurun_out/r6grey/ab.log 2>&1 || { tail -20 gpurun_out/r6grey/ab.log; exit 1; }
cat gpurun_out/r6grey/ab.log
