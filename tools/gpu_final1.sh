#!/bin/bash
# Round-end measurement, part 1: the -m gpu suite, smoke, the default bench line with the CPU
# baseline, and a rocprofv3 kernel-trace summary of the same bench command (PROF=1).
set -o pipefail
PROF=1 bash tools/gpu_check.sh ${TAG:-final1} || exit 1
