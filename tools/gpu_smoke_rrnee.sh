#!/bin/bash
# One small IterativeRRNEE render per build (elf_small 40x56 @ 2 spp, SAH: the shared-walk path)
# compared with the per-lane walks; stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
for b in ${LIBS:-simplepath_amd/_build}; do
  SP_LIB_PATH=$PWD/$b/libsimplepath_hip.so timeout -k 10 120 python -u - <<'PY' || exit 1
import os, tempfile, numpy as np
import simplepath_amd as sp
from simplepath_amd import scenes
d = tempfile.mkdtemp()
s = sp.Scene.from_file(scenes.write_elf_scene(d, n=24, max_depth=16, name="elf_small.sp"))
s.set_resolution(40, 56)
s.upload(0, 0)
a, st = sp.render_tiles(s, "iterative_rrnee", 2)
b, bt = sp.render_tiles(s, "iterative_rrnee", 2, per_lane_queries=True)
print(os.environ["SP_LIB_PATH"].split("/")[-2], "same:", np.array_equal(a.view(np.uint32), b.view(np.uint32)), st.rays, bt.rays, st.rng_draws, bt.rng_draws)
PY
done
