#!/bin/bash
# Round-4 A/B of the IterativeRRNEE query sharing: tests, then elf 1024^2 @ 16 spp for each build
# (_build: merged + shadow passes with work sharing; _build_nosteal; _build_noshadow; per-lane
# queries), then wave profiles of elf and bunny 64 spp (-DSP_WAVE_PROF build).
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${TESTS:-rrnee or merged or clipped or full_scale_tiles or every_integrator or image_environment or wide_bvh or forced_stackless or bunny_frame}" > gpurun_out/r4e_tests.log 2>&1 || { tail -30 gpurun_out/r4e_tests.log; exit 1; }
tail -1 gpurun_out/r4e_tests.log
for r in 1 2; do
for v in "_build" "_build_nosteal" "_build_noshadow" "_build --per-lane-queries"; do
  read -r b extra <<< "$v"
  SP_LIB_PATH=$PWD/simplepath_amd/$b/libsimplepath_hip.so timeout -k 10 200 python bench.py --no-cpu --scene elf --width 1024 --height 1024 --spp 16 $extra > gpurun_out/ab.json 2>/dev/null || exit 1
  echo "$v: $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['value'], d['ms_per_step'])")"
done
done
LIBS="simplepath_amd/_build_wprof" bash tools/gpu_wprof2.sh && LIBS="simplepath_amd/_build_wprof" WPROF_ARGS="--spp 64" bash tools/gpu_wprof2.sh
