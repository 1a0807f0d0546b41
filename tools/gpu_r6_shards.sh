#!/bin/bash
# Round 6, call B: every rank's shard at 8 ranks (bench.py --sim-world 8 --sim-rank -1) for bunny,
# lucy and elf, and the stride-list tile-order A/B on elf's shard.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/r6
for sc in ${SHARD_SCENES:-bunny lucy elf}; do
  st=3; wu=1; [ $sc = elf ] && st=1
  timeout -k 10 600 python -u bench.py --scene $sc --sim-world 8 --sim-rank -1 --steps $st --warmup $wu \
     > gpurun_out/r6/ranks_$sc.json 2> gpurun_out/r6/ranks_$sc.err || { tail -5 gpurun_out/r6/ranks_$sc.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r6/ranks_$sc.json'));print('$sc', d['imbalance_ms'], d['imbalance_rays'], [r['ms_per_frame'] for r in d['ranks']])"
done
if [ -n "${STRIDE_AB:-}" ]; then
  B=simplepath_amd
  RUNS="$B/_build;$B/_ab/strow0" WORKLOADS="--scene elf --sim-world 8 --steps 2 --warmup 1" bash tools/gpu_ab.sh \
    > gpurun_out/r6/ab_strow.log 2>&1 || { tail -20 gpurun_out/r6/ab_strow.log; exit 1; }
  cat gpurun_out/r6/ab_strow.log
fi
