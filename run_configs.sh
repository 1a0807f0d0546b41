#!/bin/bash
# Per-configuration bench lines (configs[1], [3], [4]; lucy/elf as one rank's shard of the 8-GPU run).
set -o pipefail
cd "$(dirname "$0")"
mkdir -p gpurun_out/configs
export TMPDIR=/tmp
run() {
  name=$1; shift
  timeout -k 10 300 python bench.py --no-cpu "$@" > gpurun_out/configs/$name.json 2> gpurun_out/configs/$name.err
  rc=$?; echo "[$name] exit $rc"; cut -c1-260 gpurun_out/configs/$name.json
  return $rc
}
run spheres --scene spheres --steps 2 --warmup 1 &&
run lucy1 --scene lucy --steps 2 --warmup 1 &&
run lucy8 --scene lucy --sim-world 8 --steps 2 --warmup 1 &&
run elf8 --scene elf --sim-world 8 --steps 1 --warmup 0
