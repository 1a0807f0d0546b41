#!/usr/bin/env python3
"""GPU check of the megakernel's tail chunks (sp_mega.hpp tail_prep / tail_chunk): renders a frame
with tail chunks off and on (SP_TAIL_FRAC / SP_TAIL_CHUNKS, read per render call) and requires
bit-identical images and identical ray / shadow / sample / draw counts.

Usage: python3 tools/tail_check.py [scene=bunny] [spp=8] [width=1920] [height=1080]"""
import os
import sys
import tempfile

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import simplepath_amd as sp  # noqa: E402
from simplepath_amd import scenes  # noqa: E402


def main(scene="bunny", spp="8", width="1920", height="1080"):
    spp, width, height = int(spp), int(width), int(height)
    d = tempfile.mkdtemp()
    path = {"bunny": scenes.write_bunny_scene, "lucy": scenes.write_lucy_scene}[scene](d)
    sc = sp.Scene.from_file(path)
    sc.set_resolution(width, height)
    sc.upload(device=0)
    n = sp.ColumnMajorTileScheduler(width, height).get_num_tiles()
    tiles = np.arange(n, dtype=np.int32)
    out = torch.zeros((n, 64, 3), dtype=torch.float32, device="cuda:0")
    stream = torch.cuda.current_stream().cuda_stream

    def run(frac, chunks):
        os.environ["SP_TAIL_FRAC"] = str(frac)
        os.environ["SP_TAIL_CHUNKS"] = str(chunks)
        out.zero_()
        st = sp.render_tiles_device(sc, "direct_lighting", spp, tiles, out.data_ptr(), stream, stage_timing=True,
                                    tile_order_factor=2.0)
        torch.cuda.synchronize()
        return out.cpu().numpy().copy(), (st.rays, st.shadow_rays, st.samples, st.rng_draws), st.launches

    ref, cref, lref = run(0, 32)
    ok = True
    for frac, chunks in ((0.05, 32), (0.05, 3), (0.2, 1), (1.0, spp), (0.01, 64)):
        img, cnt, launches = run(frac, chunks)
        same = np.array_equal(img.view(np.uint32), ref.view(np.uint32))
        print(f"{scene} {width}x{height} @ {spp}: tail {frac} x {chunks} chunks: bit-identical {same}, "
              f"counts {cnt} vs {cref} {'ok' if cnt == cref else 'DIFFER'}, launches {launches} vs {lref}", flush=True)
        if not same:
            diff = np.nonzero(np.any(img != ref, axis=2))
            print("  differing tiles:", np.unique(diff[0])[:20], "pixels", len(diff[0]))
        ok = ok and same and cnt == cref and launches == lref + 1
    print("TAIL_CHECK", "PASS" if ok else "FAIL")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main(*sys.argv[1:]))
