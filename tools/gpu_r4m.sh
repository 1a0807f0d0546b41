#!/bin/bash
# Seeding: rng_seed_twisted (generation 1 written from two seed chains, _build) vs seed + twist
# (_build_sf0); both with the probe's once-per-lane seeding.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not bench_ranks" > gpurun_out/r4m_tests.log 2>&1 || { tail -30 gpurun_out/r4m_tests.log; exit 1; }
tail -1 gpurun_out/r4m_tests.log
for r in 1 2; do
for b in _build _build_sf0; do
  L=$PWD/simplepath_amd/$b/libsimplepath_hip.so
  SP_LIB_PATH=$L timeout -k 10 200 python bench.py --no-cpu > gpurun_out/ab.json 2>/dev/null || exit 1
  echo "bunny $b: $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['probe_ms'])")"
  SP_LIB_PATH=$L timeout -k 10 200 python bench.py --no-cpu --scene elf --width 1024 --height 1024 --spp 16 > gpurun_out/ab.json 2>/dev/null || exit 1
  echo "elf $b: $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['value'], d['ms_per_step'])")"
done
done
