#!/bin/bash
# PMC passes for the VALU roofline and traversal metrics on the bench frame (one counter set per
# rocprofv3 run, kernel-trace only), then tools/pmc_valu.py -> gpurun_out/pmc_valu_<tag>.json.
#   SPP (default 256: the bench config) and BENCH_ARGS (extra bench.py flags) select the workload.
set -o pipefail
cd "$(dirname "$0")/.."
R=$GRAFT_REPO_ROOT
OUT=gpurun_out/pmcv_${TAG:-bench}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --no-cpu --spp ${SPP:-256} ${BENCH_ARGS:-}"
cd /tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_INT64 GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
           "TCP_TOTAL_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $R/$OUT/p$i -o run -- python3 $R/bench.py $ARGS > $R/$OUT/p$i.json 2> $R/$OUT/p$i.err || { echo "pmc pass $i failed"; tail -5 $R/$OUT/p$i.err; exit 1; }
  echo "pass $i done"
done
cd $R && python3 tools/pmc_valu.py $OUT ${W:-1920} ${H:-1080} ${SPP:-256} gpurun_out/pmc_valu_${TAG:-bench}.json
