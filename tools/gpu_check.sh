#!/bin/bash
# GPU check: the -m gpu suite, smoke(), and the default bench line (N=1, with the CPU baseline).
# Usage (from the repo root): gpurun -- bash tools/gpu_check.sh [outdir]
set -o pipefail
out=gpurun_out/${1:-check}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 \
  || { tail -40 "$out/tests.log"; exit 1; }
tail -2 "$out/tests.log"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || { tail -20 "$out/smoke.log"; exit 1; }
tail -1 "$out/smoke.log"
timeout -k 10 300 python -u bench.py > "$out/bench.json" 2> "$out/bench.err" || { tail -20 "$out/bench.err"; exit 1; }
cat "$out/bench.json"
