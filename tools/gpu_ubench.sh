#!/bin/bash
# Calibration microbenchmarks, built from source on the box (tools/ubench/*.hip -> tools/ubench/_build):
#   valu_rate   SIMD cycles per VALU wave-instruction class (tools/pmc_valu.py's cycle model)
#   fetch_calib FETCH_SIZE / WRITE_SIZE per byte read / written (tools/pmc_traffic.py's correction)
# Outputs gpurun_out/calib/{valu_rate.txt,fetch_calib.json}.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
B=tools/ubench/_build
mkdir -p $B gpurun_out/calib
for t in valu_rate fetch_calib; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 tools/ubench/$t.hip -o $B/$t || exit 1
done
timeout -k 10 120 $B/valu_rate > gpurun_out/calib/valu_rate.txt 2>&1 || { tail -5 gpurun_out/calib/valu_rate.txt; exit 1; }
cat gpurun_out/calib/valu_rate.txt
(cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/calib/p1 -o run -- $R/$B/fetch_calib > $R/gpurun_out/calib/p1.log 2>&1) \
  && (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/calib/p2 -o run -- $R/$B/fetch_calib > $R/gpurun_out/calib/p2.log 2>&1) \
  && python3 tools/fetch_calib.py gpurun_out/calib gpurun_out/calib/fetch_calib.json
