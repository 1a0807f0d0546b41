#!/bin/bash
# full GPU test suite, smoke(), and the AUTO bench line at N=1 and at the 2/4/8-way shards
set -o pipefail
mkdir -p gpurun_out/rd
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/rd/tests.log 2>&1 || { tail -40 gpurun_out/rd/tests.log; exit 1; }
tail -2 gpurun_out/rd/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/rd/smoke.log 2>&1 || { tail -20 gpurun_out/rd/smoke.log; exit 1; }
tail -1 gpurun_out/rd/smoke.log
for n in 1 2 4 8; do
  timeout -k 10 150 python -u bench.py --no-cpu --steps 3 --warmup 1 --sim-world $n > gpurun_out/rd/a$n.json 2> gpurun_out/rd/a$n.err || { tail -5 gpurun_out/rd/a$n.err; exit 1; }
  echo "auto N=$n $(python -c "import json;d=json.load(open('gpurun_out/rd/a$n.json'));print(d['value'],d['ms_per_step'],d['config']['pipeline'])")"
done
