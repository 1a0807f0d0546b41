#!/bin/bash
# PMC passes for the VALU roofline and traversal metrics on one bench workload (one counter set
# per rocprofv3 run, kernel-trace only), then tools/pmc_valu.py -> gpurun_out/pmc_valu_bench_<TAG>.json
# (the file bench.py reads as profiles/pmc_valu_bench_<scene>.json).  Workload: SCENE (default
# bunny), W / H / SPP (the scene's bench config), SIMW (--sim-world), BENCH_ARGS (extra flags).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
SCENE=${SCENE:-bunny}
SIMW=${SIMW:-0}
if [ "$SIMW" -gt 1 ]; then TAG=${TAG:-${SCENE}_shard$SIMW}; else TAG=${TAG:-$SCENE}; fi
OUT=gpurun_out/pmcv_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
W=${W:-$(python3 -c "import bench;print(bench.SCENES['$SCENE']['w'])")}
H=${H:-$(python3 -c "import bench;print(bench.SCENES['$SCENE']['h'])")}
SPP=${SPP:-$(python3 -c "import bench;print(bench.SCENES['$SCENE']['spp'])")}
ARGS="--steps 1 --warmup 0 --no-cpu --scene $SCENE --width $W --height $H --spp $SPP --sim-world ${SIMW:-0} ${BENCH_ARGS:-}"
cd /tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_INT64 GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
           "TCP_TOTAL_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $R/$OUT/p$i -o run -- python3 $R/bench.py $ARGS > $R/$OUT/p$i.json 2> $R/$OUT/p$i.err || { echo "pmc pass $i failed"; tail -5 $R/$OUT/p$i.err; exit 1; }
  echo "pass $i done"
done
cd $R && python3 tools/pmc_valu.py $OUT $W $H $SPP gpurun_out/pmc_valu_bench_$TAG.json $SCENE ${SIMW:-0}
