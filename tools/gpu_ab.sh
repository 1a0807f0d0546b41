#!/bin/bash
# A/B of library builds and environment settings (tools/gpu_ab.sh) on one box, bench.py --no-cpu in alternation.
#   RUNS   ";"-separated entries "builddir [VAR=value ...]" (default: simplepath_amd/_build_base;
#          simplepath_amd/_build), repeated REPEAT times (default 2)
#   TESTS  if set, the -m gpu tests matching it (-k) run first on the in-tree build
#   PMC    if set (a counter list), one --pmc pass per entry at PMC_SPP spp (default 16)
#   BENCH_ARGS  extra bench.py flags
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
IFS=';' read -ra RN <<< "${RUNS:-simplepath_amd/_build_base;simplepath_amd/_build}"
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$TESTS" > gpurun_out/ab/tests.log 2>&1 \
    || { tail -30 gpurun_out/ab/tests.log; exit 1; }
  tail -1 gpurun_out/ab/tests.log
fi
for r in $(seq 1 ${REPEAT:-2}); do
  for e in "${RN[@]}"; do
    read -r lib envs <<< "$e"
    env SP_LIB_PATH=$R/$lib/libsimplepath_hip.so $envs timeout -k 10 200 python -u bench.py --no-cpu ${BENCH_ARGS:-} > gpurun_out/ab/b.json 2> gpurun_out/ab/b.err \
      || { tail -5 gpurun_out/ab/b.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ab/b.json'));r=d['roofline'];print('$e |', d['value'],d['ms_per_step'],{k:v.get('ms_per_launch') for k,v in r.get('stages',{}).items()})"
  done
done
if [ -n "${PMC:-}" ]; then
  i=0
  for e in "${RN[@]}"; do
    i=$((i+1))
    read -r lib envs <<< "$e"
    (cd /tmp && env SP_LIB_PATH=$R/$lib/libsimplepath_hip.so $envs timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $PMC --output-format csv \
       -d $R/gpurun_out/ab/pmc_$i -o run -- python3 $R/bench.py --no-cpu --steps 1 --warmup 0 --spp ${PMC_SPP:-16} ${BENCH_ARGS:-} \
       > $R/gpurun_out/ab/pmc_$i.json 2> $R/gpurun_out/ab/pmc_$i.err) || { echo "pmc $e failed"; tail -5 gpurun_out/ab/pmc_$i.err; exit 1; }
    echo "== pmc $i: $e"
    python3 tools/pmc_sum.py gpurun_out/ab/pmc_$i wf_ ck_ sp_mega | head -8
  done
fi
