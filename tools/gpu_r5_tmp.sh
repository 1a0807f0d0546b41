set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5b
SP_LIB_PATH=$PWD/simplepath_amd/_build_pk2/libsimplepath_hip.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "packet or sah or wide_bvh or full_scale_bunny" > gpurun_out/r5b/tests.log 2>&1 || { tail -30 gpurun_out/r5b/tests.log; exit 1; }
tail -1 gpurun_out/r5b/tests.log
RUNS="simplepath_amd/_build;simplepath_amd/_build_pk2" WORKLOADS="; --sim-world 8" bash tools/gpu_ab.sh
LIBS="simplepath_amd/_build_wprof simplepath_amd/_build_wprof_pk2" WPROF_ARGS="--spp 64" bash tools/gpu_wprof2.sh
