#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration (tools/ubench/fetch_calib.hip) -> gpurun_out/calib/fetch_calib.json
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/calib && (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/calib/p1 -o run -- $GRAFT_REPO_ROOT/tools/ubench/fetch_calib > $GRAFT_REPO_ROOT/gpurun_out/calib/p1.log 2>&1) && (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/calib/p2 -o run -- $GRAFT_REPO_ROOT/tools/ubench/fetch_calib > $GRAFT_REPO_ROOT/gpurun_out/calib/p2.log 2>&1) && python3 tools/fetch_calib.py gpurun_out/calib gpurun_out/calib/fetch_calib.json
