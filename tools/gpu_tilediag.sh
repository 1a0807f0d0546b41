#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/td
for n in 1 2 8; do
  for o in 0 1; do
    SP_TILE_ORDER=$o SP_TILE_DIAG=gpurun_out/td/mega_${n}_$o.bin timeout -k 10 120 python -u bench.py --no-cpu --steps 1 --warmup 0 --pipeline megakernel --sim-world $n > gpurun_out/td/mega_${n}_$o.json 2> gpurun_out/td/mega_${n}_$o.err || exit 1
    echo "== N=$n order=$o"; python tools/tile_diag.py gpurun_out/td/mega_${n}_$o.bin
  done
done
