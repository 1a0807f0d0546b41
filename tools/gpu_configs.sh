#!/bin/bash
# GPU tests, then the BASELINE configs beyond the default line: lucy 1080p@256 (N=1 and the 8-way
# shard), elf 4096^2@1024 max-depth 16 (the 8-way shard), spheres (N=1), the scan-like bunny (N=1),
# bunny's 2/4/8-way shards.  SKIP_TESTS=1 skips the test suite.
set -o pipefail
mkdir -p gpurun_out/cfg
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/cfg/tests.log 2>&1 || { tail -30 gpurun_out/cfg/tests.log; exit 1; }
  tail -2 gpurun_out/cfg/tests.log
fi
run() { # name, args
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu "$@" > gpurun_out/cfg/$n.json 2> gpurun_out/cfg/$n.err || { tail -5 gpurun_out/cfg/$n.err; exit 1; }
  echo "$n $(python -c "import json;d=json.load(open('gpurun_out/cfg/$n.json'));print(d['value'],d['ms_per_step'],d['config']['pipeline'],d['config']['workload'])")"
}
run spheres --scene spheres --steps 2 --warmup 1
run bunny_scan --scene bunny_scan --steps 2 --warmup 1
for n in 2 4 8; do run bunny_shard$n --steps 2 --warmup 1 --sim-world $n; done
run lucy1 --scene lucy --steps 2 --warmup 1
run lucy8 --scene lucy --steps 2 --warmup 1 --sim-world 8
run elf8 --scene elf --steps 1 --warmup 0 --sim-world 8
