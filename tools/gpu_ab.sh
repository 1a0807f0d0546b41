#!/bin/bash
# A/B of library builds and environment settings on one box, bench.py --no-cpu in alternation.
#   RUNS       ";"-separated entries "builddir [VAR=value ...]" (default: simplepath_amd/_ab/base;
#              simplepath_amd/_build), repeated REPEAT times (default 2)
#   WORKLOADS  ";"-separated bench.py argument sets, each run for every entry (default: one set,
#              BENCH_ARGS).  E.g. WORKLOADS="; --scene elf --width 1024 --height 1024 --spp 16; --sim-world 8"
#              is bunny, elf 1024^2 @ 16 spp and bunny's 8-way shard -- the round-4 A/B triple.
#   TESTS      if set, the -m gpu tests matching it (-k) run first on the in-tree build ("all": every one)
#   SMOKE      if set, __graft_entry__.smoke() runs first
#   PMC        if set (a counter list), one --pmc pass per entry at PMC_SPP spp (default 16)
#   BENCH_ARGS extra bench.py flags (every workload)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
IFS=';' read -ra RN <<< "${RUNS:-simplepath_amd/_ab/base;simplepath_amd/_build}"
IFS=';' read -ra WL <<< "${WORKLOADS:-}"
[ ${#WL[@]} -eq 0 ] && WL=("")
if [ -n "${SMOKE:-}" ]; then
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
fi
if [ -n "${TESTS:-}" ]; then
  K=(-k "$TESTS"); [ "$TESTS" = all ] && K=()
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${K[@]}" > gpurun_out/ab/tests.log 2>&1 \
    || { tail -30 gpurun_out/ab/tests.log; exit 1; }
  tail -1 gpurun_out/ab/tests.log
fi
for r in $(seq 1 ${REPEAT:-2}); do
  for w in "${WL[@]}"; do
    for e in "${RN[@]}"; do
      read -r lib envs <<< "$e"
      env SP_LIB_PATH=$R/$lib/libsimplepath_hip.so $envs timeout -k 10 300 python -u bench.py --no-cpu ${BENCH_ARGS:-} $w > gpurun_out/ab/b.json 2> gpurun_out/ab/b.err \
        || { tail -5 gpurun_out/ab/b.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/ab/b.json'));r=d['roofline'];print('$e |$w |', d['value'],d['ms_per_step'],r.get('kernel_ms'),r.get('probe_ms'),{k:v.get('ms_per_launch') for k,v in r.get('stages',{}).items()})"
    done
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
