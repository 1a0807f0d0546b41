#!/bin/bash
# GPU check: the -m gpu suite, smoke(), the default bench line (N=1, with the CPU baseline) and,
# with PROF=1, a rocprofv3 --kernel-trace --stats summary of the same bench command.
# Usage (from the repo root): gpurun -- bash tools/gpu_check.sh [outdir]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
out=gpurun_out/${1:-check}
mkdir -p "$out"
export TMPDIR=/tmp
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 \
    || { tail -40 "$out/tests.log"; exit 1; }
  tail -2 "$out/tests.log"
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || { tail -20 "$out/smoke.log"; exit 1; }
  tail -1 "$out/smoke.log"
fi
timeout -k 10 300 python -u bench.py ${BENCH_ARGS:-} > "$out/bench.json" 2> "$out/bench.err" || { tail -20 "$out/bench.err"; exit 1; }
cat "$out/bench.json"
if [ -n "${PROF:-}" ]; then
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$out/rocprof -o run -- python3 $R/bench.py --no-cpu ${BENCH_ARGS:-} > $R/$out/rocprof_bench.json 2> $R/$out/rocprof.err) \
    || { echo "rocprof run failed"; tail -5 $out/rocprof.err; exit 1; }
  head -4 $out/rocprof/run_kernel_stats.csv | cut -c1-200
fi
