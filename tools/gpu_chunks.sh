#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/ck
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "chunks" > gpurun_out/ck/tests.log 2>&1 || { tail -40 gpurun_out/ck/tests.log; exit 1; }
tail -2 gpurun_out/ck/tests.log
for n in 8 4 2; do
  timeout -k 10 150 python -u bench.py --no-cpu --steps 2 --warmup 1 --pipeline chunks --sim-world $n > gpurun_out/ck/c$n.json 2> gpurun_out/ck/c$n.err || { tail -5 gpurun_out/ck/c$n.err; exit 1; }
  echo "chunks N=$n $(python -c "import json;d=json.load(open('gpurun_out/ck/c$n.json'));print(d['value'],d['ms_per_step'],d['config']['pipeline'])")"
done
export TMPDIR=/tmp; R=$PWD
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ckp -o run -- python3 $R/bench.py --no-cpu --steps 2 --warmup 1 --pipeline chunks --sim-world 8 > $R/gpurun_out/ckp.json 2> $R/gpurun_out/ckp.err && cut -c1-120 $R/gpurun_out/ckp/run_kernel_stats.csv | head -5
