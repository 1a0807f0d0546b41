#!/bin/bash
# GPU session: parity tests, then bench with both pipelines, then rocprof kernel stats.
set -o pipefail
cd "$(dirname "$0")"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu -s > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/bench_wave.json 2> gpurun_out/bench_wave.err
rc=$?; echo "bench wave exit $rc"; cat gpurun_out/bench_wave.json; tail -3 gpurun_out/bench_wave.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu --pipeline megakernel > gpurun_out/bench_mega.json 2> gpurun_out/bench_mega.err
rc=$?; echo "bench mega exit $rc"; cat gpurun_out/bench_mega.json
[ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_wave -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/prof_wave.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof_wave.err
echo "rocprof exit $?"
