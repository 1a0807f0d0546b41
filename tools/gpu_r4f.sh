#!/bin/bash
# DirectLighting shared shadow walks: a small smoke, the parity tests that cover the megakernel,
# then bunny 1080p @ 256 spp shared vs per-lane walks (alternating), and elf 1024^2 @ 16 spp.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 120 python -u -c "
import tempfile, numpy as np, simplepath_amd as sp
from simplepath_amd import scenes
s = sp.Scene.from_file(scenes.write_bunny_scene(tempfile.mkdtemp())); s.set_resolution(64, 40); s.upload(0, 0)
a, st = sp.render_tiles(s, 'direct_lighting', 2, pipeline='megakernel')
b, bt = sp.render_tiles(s, 'direct_lighting', 2, pipeline='megakernel', per_lane_queries=True)
print('smoke shared == per-lane:', np.array_equal(a.view(np.uint32), b.view(np.uint32)), st.rays, bt.rays)
" || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${TESTS:-shared or merged or waves_per_simd or wavefront_equals or sample_chunks_equal or full_scale_bunny or tile_order or two_threads or bitexact}" > gpurun_out/r4f_tests.log 2>&1 || { tail -30 gpurun_out/r4f_tests.log; exit 1; }
tail -1 gpurun_out/r4f_tests.log
for r in 1 2; do
for v in "" "--per-lane-queries"; do
  timeout -k 10 200 python bench.py --no-cpu $v > gpurun_out/ab.json 2>/dev/null || exit 1
  echo "bunny $v: $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])")"
done
done
timeout -k 10 200 python bench.py --no-cpu --scene elf --width 1024 --height 1024 --spp 16 > gpurun_out/ab.json 2>/dev/null || exit 1
echo "elf: $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['value'], d['ms_per_step'])")"
