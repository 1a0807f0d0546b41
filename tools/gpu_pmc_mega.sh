#!/bin/bash
# SQ issue/stall breakdown of the megakernel (N=1 full frame and the 8-GPU shard)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pm
for n in 1 8; do
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES --kernel-include-regex sp_render -d gpurun_out/pm/a$n -o pmc -- python3 bench.py --no-cpu --steps 1 --warmup 0 --pipeline megakernel --sim-world $n > gpurun_out/pm/a$n.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES --kernel-include-regex sp_render -d gpurun_out/pm/b$n -o pmc -- python3 bench.py --no-cpu --steps 1 --warmup 0 --pipeline megakernel --sim-world $n > gpurun_out/pm/b$n.log 2>&1 || exit 1
done
find gpurun_out/pm -name "*counter_collection.csv" | head
