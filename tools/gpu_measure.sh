#!/bin/bash
# Round measurement set for the current build:
#   the bench workload (bunny 1080p @ 256 spp): VALU-roofline PMC passes, FETCH/WRITE traffic
#   passes, a rocprofv3 kernel-trace summary of the bench command;
#   elf 1024^2 @ 16 spp (IterativeRRNEE megakernel): VALU passes and a bench line.
# Outputs under gpurun_out/; copy what is judged to profiles/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
bash tools/gpu_pmc_valu.sh || exit 1
bash tools/gpu_pmc_traffic.sh || exit 1
mkdir -p gpurun_out/stats
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/stats/bench -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu > $R/gpurun_out/stats/bench.json 2> $R/gpurun_out/stats/bench.err) || { echo "stats run failed"; exit 1; }
echo "stats done"
SCENE=elf TAG=elf_1k W=1024 H=1024 SPP=16 bash tools/gpu_pmc_valu.sh || exit 1
timeout -k 10 300 python3 bench.py --no-cpu --scene elf --width 1024 --height 1024 --spp 16 > gpurun_out/elf_1k.json 2> gpurun_out/elf_1k.err || exit 1
echo "elf 1k: $(python3 -c "import json;d=json.load(open('gpurun_out/elf_1k.json'));print(d['value'],d['ms_per_step'])")"
