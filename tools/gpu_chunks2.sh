#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/ck2
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi_rank.py -m gpu -x -q --timeout 200 --timeout-method thread -k "chunks or two_ranks" > gpurun_out/ck2/tests.log 2>&1 || { tail -40 gpurun_out/ck2/tests.log; exit 1; }
tail -2 gpurun_out/ck2/tests.log
SWEEP_TAG=s8 SWEEP_ARGS="--pipeline chunks --sim-world 8" bash tools/gpu_env_sweep.sh "SP_CHUNK_FUSED=1" "SP_EVAL_WAVES=4" "SP_EVAL_WAVES=3" "SP_EVAL_WAVES=2" || exit 1
SWEEP_TAG=s2 SWEEP_ARGS="--pipeline chunks --sim-world 2" bash tools/gpu_env_sweep.sh "SP_EVAL_WAVES=4" "SP_EVAL_WAVES=3" || exit 1
SWEEP_TAG=s4 SWEEP_ARGS="--pipeline chunks --sim-world 4" bash tools/gpu_env_sweep.sh "SP_EVAL_WAVES=4" "SP_EVAL_WAVES=3" || exit 1
