#!/bin/bash
# FETCH_SIZE and WRITE_SIZE (separate passes: they cannot share one) on one bench workload, then
# per-launch HBM bytes per kernel -> gpurun_out/pmc_bench_<TAG>.json (the file bench.py reads as
# profiles/pmc_bench_<scene>.json).  Workload: SCENE (default bunny), W / H / SPP (the scene's bench
# config), SIMW (--sim-world, default 0), BENCH_ARGS (extra bench.py flags).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
SCENE=${SCENE:-bunny}
SIMW=${SIMW:-0}
if [ "$SIMW" -gt 1 ]; then TAG=${TAG:-${SCENE}_shard$SIMW}; else TAG=${TAG:-$SCENE}; fi
OUT=gpurun_out/pmct_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
W=${W:-$(python3 -c "import bench;print(bench.SCENES['$SCENE']['w'])")}
H=${H:-$(python3 -c "import bench;print(bench.SCENES['$SCENE']['h'])")}
SPP=${SPP:-$(python3 -c "import bench;print(bench.SCENES['$SCENE']['spp'])")}
ARGS="--steps 1 --warmup 0 --no-cpu --scene $SCENE --width $W --height $H --spp $SPP --sim-world ${SIMW:-0} ${BENCH_ARGS:-}"
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $R/$OUT/p1 -o run -- python3 $R/bench.py $ARGS > $R/$OUT/p1.json 2> $R/$OUT/p1.err || { echo "fetch pass failed"; tail -5 $R/$OUT/p1.err; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $R/$OUT/p2 -o run -- python3 $R/bench.py $ARGS > $R/$OUT/p2.json 2> $R/$OUT/p2.err || { echo "write pass failed"; tail -5 $R/$OUT/p2.err; exit 1; }
cd $R && python3 tools/pmc_traffic.py $OUT $W $H $SPP gpurun_out/pmc_bench_$TAG.json $SCENE ${SIMW:-0} > /dev/null && echo "traffic $TAG done"
