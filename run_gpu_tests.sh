#!/bin/bash
# One GPU session: build check, GPU tests, smoke, short bench, rocprof summary.
set -o pipefail
cd "$(dirname "$0")"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu -s > gpurun_out/pytest_gpu.log 2>&1
echo "pytest exit $?"
