"""Diagnostic: where does the HIP path leave the oracle on the full elf config?  Renders a few
golden tiles under several settings on the GPU and on the CPU oracle (device libm) and prints
bit-exact pixel fractions."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import simplepath_amd as sp  # noqa: E402
from simplepath_amd import scenes  # noqa: E402
from tests import _oracle  # noqa: E402

g = np.load(os.path.join(ROOT, "tests", "golden", "elf_full_tiles.npz"))
d = f"/tmp/sp_full_scale_{os.getuid()}"


def run(label, path, w, h, ids, spp, integ=5, pipeline="megakernel", bvh=1):
    s = sp.Scene.from_file(path)
    s.set_resolution(w, h)
    s.upload(0, bvh)
    out, st = sp.render_tiles(s, integ, spp, ids, pipeline=pipeline)
    o, ost = _oracle.render(s, integ, spp, ids, threads=16, variant="spm")
    frac = float(np.mean(np.all(out == o, axis=-1)))
    print(f"{label:40s} spp {spp:5d} {pipeline:10s} bitexact {frac:.4f} rays {st.rays} vs {ost['rays']} "
          f"samples {st.samples} vs {ost['samples']}", flush=True)


full = scenes.write_elf_scene(d, n=290, max_depth=16)
small = scenes.write_elf_scene(d, n=24, max_depth=16, name="elf_small.sp")
ids = g["tile_ids"].astype(np.int32)
run("full 4096 all 26 golden tiles", full, 4096, 4096, ids[:4], 1024)
run("full 4096 all 26 golden tiles", full, 4096, 4096, ids, 1024)
run("full 4096 all 26 golden tiles", full, 4096, 4096, ids, 256)
run("full 4096 all 26 golden tiles", full, 4096, 4096, ids, 1024, pipeline="wavefront")
