#!/bin/bash
# Requests by source (-DSP_TRAFFIC_DIAG build, LIB) for bench workloads (";"-separated WORKLOADS):
# one render each with SP_TILE_DIAG, then tools/traffic_diag.py.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/td
IFS=';' read -ra WL <<< "${WORKLOADS:- }"
i=0
for w in "${WL[@]}"; do
  i=$((i+1))
  SP_LIB_PATH=$R/${LIB:-simplepath_amd/_ab/td}/libsimplepath_hip.so SP_TILE_DIAG=gpurun_out/td/d$i.bin timeout -k 10 600 \
    python -u bench.py --no-cpu --steps 1 --warmup 0 $w > gpurun_out/td/b$i.json 2> gpurun_out/td/b$i.err || { tail -5 gpurun_out/td/b$i.err; exit 1; }
  echo "== $w: $(python -c "import json;d=json.load(open('gpurun_out/td/b$i.json'));print(d['value'],'Mrays/s',d['config']['pipeline'],d['rays_per_step'],'rays')")"
  python3 tools/traffic_diag.py gpurun_out/td/d$i.bin gpurun_out/td/b$i.json | tee gpurun_out/td/t$i.txt
done
