#!/bin/bash
# FETCH / WRITE traffic passes where the scene does not fit the caches: lucy (1 GPU and the 8-way
# shard) and elf (8-way shard).
set -o pipefail
export TMPDIR=/tmp
SCENE=lucy bash tools/gpu_pmc_traffic.sh || exit 1
SCENE=lucy SIMW=8 bash tools/gpu_pmc_traffic.sh || exit 1
SCENE=elf SIMW=8 bash tools/gpu_pmc_traffic.sh || exit 1
for t in lucy lucy_shard8 elf_shard8; do python3 -c "
import json;d=json.load(open('gpurun_out/pmc_bench_$t.json'))
print('$t', {k:(round(v['fetch_bytes_per_launch']/1e9,2), round(v['write_bytes_per_launch']/1e9,2)) for k,v in d['kernels'].items()})"; done
