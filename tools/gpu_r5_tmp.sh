set -o pipefail
export TMPDIR=/tmp
LIBS="simplepath_amd/_build_wprof_nr simplepath_amd/_build_wprof" bash tools/gpu_wprof2.sh
WORKLOADS="--scene elf --width 1024 --height 1024 --spp 16" bash tools/gpu_traffic_diag.sh
