#!/bin/bash
# PMC passes (separate runs, kernel-trace only) on a reduced bench (same frame, 32 spp).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
ARGS="--steps 1 --warmup 0 --no-cpu --spp ${SPP:-32}"
cd /tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS" \
           "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $R/gpurun_out/pmc/p$i -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmc/p$i.json 2> $R/gpurun_out/pmc/p$i.err || { echo "pmc pass $i failed"; tail -5 $R/gpurun_out/pmc/p$i.err; exit 1; }
done
echo done
