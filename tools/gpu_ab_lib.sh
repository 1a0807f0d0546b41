#!/bin/bash
# A/B of builds of the library on one box: $LIBS (build dirs; default
# simplepath_amd/_build_base and the in-tree build), bench.py --no-cpu in alternation, $REPEAT rounds.  With $TESTS set,
# the -m gpu tests matching it (-k) run first on the in-tree build.  With $PMC set (a counter
# list), one --pmc pass per build at $PMC_SPP spp follows.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
LIBS=${LIBS:-simplepath_amd/_build_base simplepath_amd/_build}
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$TESTS" > gpurun_out/ab/tests.log 2>&1 \
    || { tail -30 gpurun_out/ab/tests.log; exit 1; }
  tail -1 gpurun_out/ab/tests.log
fi
for r in $(seq 1 ${REPEAT:-2}); do
  for lib in $LIBS; do
    SP_LIB_PATH=$R/$lib/libsimplepath_hip.so timeout -k 10 200 python -u bench.py --no-cpu ${BENCH_ARGS:-} > gpurun_out/ab/b.json 2> gpurun_out/ab/b.err \
      || { tail -5 gpurun_out/ab/b.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ab/b.json'));r=d['roofline'];print('$lib |', d['value'],d['ms_per_step'],{k:v.get('ms_per_launch') for k,v in r.get('stages',{}).items()})"
  done
done
if [ -n "${PMC:-}" ]; then
  for lib in $LIBS; do
    tag=$(basename $lib)
    (cd /tmp && SP_LIB_PATH=$R/$lib/libsimplepath_hip.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $PMC --output-format csv \
       -d $R/gpurun_out/ab/pmc_$tag -o run -- python3 $R/bench.py --no-cpu --steps 1 --warmup 0 --spp ${PMC_SPP:-16} ${BENCH_ARGS:-} \
       > $R/gpurun_out/ab/pmc_$tag.json 2> $R/gpurun_out/ab/pmc_$tag.err) || { echo "pmc $tag failed"; tail -5 gpurun_out/ab/pmc_$tag.err; exit 1; }
    python3 tools/pmc_sum.py gpurun_out/ab/pmc_$tag wf_ ck_ sp_mega | head -20
  done
fi
