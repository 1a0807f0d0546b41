#!/bin/bash
# The BASELINE configs beyond the default line, each with the reference CPU path timed beside it
# (cpu_baseline, kind "reference") and parity of the GPU frame against it:
#   spheres (configs[1], N=1), lucy (configs[3]: the 1-GPU frame and one rank's 8-way shard),
#   elf (configs[4]: one rank's 8-way shard), bunny's 2/4/8-way shards, the scan-like bunny.
# CONFIGS selects a subset (space-separated names); PMC=1 adds the VALU-roofline PMC passes of
# each line's workload (tools/gpu_pmc_valu.sh), TRAFFIC=1 the FETCH_SIZE / WRITE_SIZE passes
# (tools/gpu_pmc_traffic.sh), so roofline.valu / roofline.traffic are filled on a rerun.
# Every line times 3 steps (step_ms: min / max).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/cfg
declare -A A=(
  [spheres]="--scene spheres --steps 3 --warmup 1"
  [bunny_scan]="--scene bunny_scan --steps 3 --warmup 1"
  [bunny_shard2]="--steps 3 --warmup 1 --sim-world 2"
  [bunny_shard4]="--steps 3 --warmup 1 --sim-world 4"
  [bunny_shard8]="--steps 3 --warmup 1 --sim-world 8"
  [lucy1]="--scene lucy --steps 3 --warmup 1"
  [lucy8]="--scene lucy --steps 3 --warmup 1 --sim-world 8"
  [elf8]="--scene elf --steps 3 --warmup 0 --sim-world 8"
)
for n in ${CONFIGS:-spheres bunny_scan bunny_shard2 bunny_shard4 bunny_shard8 lucy1 lucy8 elf8}; do
  timeout -k 10 1000 python -u bench.py ${A[$n]} ${BENCH_ARGS:-} > gpurun_out/cfg/$n.json 2> gpurun_out/cfg/$n.err || { tail -5 gpurun_out/cfg/$n.err; exit 1; }
  echo "$n $(python -c "import json;d=json.load(open('gpurun_out/cfg/$n.json'));c=d['cpu_baseline'] or {};p=d['parity'] or {};print(d['value'],d['ms_per_step'],d['config']['pipeline'],'cpu',c.get('value'),'parity',p.get('rel_l2'),p.get('bitexact_pixel_frac'))")"
  if [ -n "${PMC:-}" ]; then
    sc=$(python -c "import sys;a=sys.argv[1:];print(a[a.index('--scene')+1] if '--scene' in a else 'bunny')" ${A[$n]})
    sw=$(python -c "import sys;a=sys.argv[1:];print(a[a.index('--sim-world')+1] if '--sim-world' in a else 0)" ${A[$n]})
    SCENE=$sc SIMW=$sw bash tools/gpu_pmc_valu.sh > gpurun_out/cfg/pmc_$n.log 2>&1 || { tail -5 gpurun_out/cfg/pmc_$n.log; exit 1; }
    tail -2 gpurun_out/cfg/pmc_$n.log
  fi
  if [ -n "${TRAFFIC:-}" ]; then
    sc=$(python -c "import sys;a=sys.argv[1:];print(a[a.index('--scene')+1] if '--scene' in a else 'bunny')" ${A[$n]})
    sw=$(python -c "import sys;a=sys.argv[1:];print(a[a.index('--sim-world')+1] if '--sim-world' in a else 0)" ${A[$n]})
    SCENE=$sc SIMW=$sw bash tools/gpu_pmc_traffic.sh > gpurun_out/cfg/traffic_$n.log 2>&1 || { tail -5 gpurun_out/cfg/traffic_$n.log; exit 1; }
    tail -1 gpurun_out/cfg/traffic_$n.log
  fi
done
