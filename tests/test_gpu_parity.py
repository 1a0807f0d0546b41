"""GPU parity: the HIP path through the C-ABI against the CPU oracle on the same seeded inputs.

Bar (DESIGN.md "Parity chain"):
  * bit-exact against the oracle with the reference-order BVH (both libm builds of the oracle:
    the device libm is an exact emulation of glibc's float libm);
  * with the SAH BVH (visiting order differs only on exactly-equal hit distances): rel L2 < 1e-4
    and >= 99.9% of pixels bit-exact.
"""
import os

import numpy as np
import pytest

import simplepath_amd as sp
from tests import _oracle

pytestmark = pytest.mark.gpu

REL_L2_TOL = 1e-4  # BASELINE.json north_star: per-pixel L2 error < 1e-4 vs CPU


def rel_l2(a, b):
    return float(np.linalg.norm((a - b).ravel()) / max(np.linalg.norm(b.ravel()), 1e-30))


def load(scene_dir, name, w, h, bvh, **upload_options):
    s = sp.Scene.from_file(os.path.join(scene_dir, name))
    s.set_resolution(w, h)
    s.upload(device=0, bvh_mode=bvh, **upload_options)
    return s


@pytest.mark.parametrize("pipeline", ["megakernel", "wavefront", "chunks"])
def test_bunny_direct_lighting_bitexact(scene_dir, pipeline):
    s = load(scene_dir, "bunny.sp", 64, 40, bvh=1)
    g, gst = sp.render_tiles(s, "direct_lighting", 4, pipeline=pipeline)
    assert gst.pipeline == sp.PIPELINES[pipeline]
    c, cst = _oracle.render(s, 6, 4, variant="spm")
    assert gst.samples == cst["samples"] == 64 * 40 * 4
    assert gst.rays == cst["rays"] and gst.shadow_rays == cst["shadow_rays"]
    assert np.array_equal(g.view(np.uint32), c.view(np.uint32)), rel_l2(g, c)


@pytest.mark.parametrize("pipeline", ["megakernel", "wavefront", "chunks"])
def test_bunny_scan_bitexact(scene_dir, pipeline):
    # the scan-like bunny (cupped ears, surface relief; scenes.bunny_scan_mesh), reference BVH order
    s = load(scene_dir, "bunny_scan.sp", 64, 40, bvh=1)
    g, gst = sp.render_tiles(s, "direct_lighting", 3, pipeline=pipeline)
    c, cst = _oracle.render(s, 6, 3, variant="spm")
    assert gst.rays == cst["rays"] and gst.shadow_rays == cst["shadow_rays"]
    assert np.array_equal(g.view(np.uint32), c.view(np.uint32)), rel_l2(g, c)


@pytest.mark.parametrize("integrator", ["direct_lighting", "brute_force", "brute_force_iterative",
                                        "brute_force_iterative_rr", "iterative_rrnee", "whitted", "mandelbrot"])
def test_every_integrator_bitexact(scene_dir, integrator):
    s = load(scene_dir, "material_spheres.sp", 24, 48, bvh=1)
    g, _ = sp.render_tiles(s, integrator, 3)
    c, _ = _oracle.render(s, sp.string_to_integrator_type(integrator), 3, variant="spm")
    same = np.array_equal(g.view(np.uint32), c.view(np.uint32))
    assert same, (integrator, rel_l2(g, c))


def test_bunny_multibounce_bitexact(scene_dir):
    s = load(scene_dir, "bunny.sp", 32, 24, bvh=1)
    g, _ = sp.render_tiles(s, "iterative_rrnee", 2)
    c, _ = _oracle.render(s, 5, 2, variant="spm")
    assert np.array_equal(g.view(np.uint32), c.view(np.uint32)), rel_l2(g, c)


def test_sah_bvh_within_tolerance(scene_dir):
    s = load(scene_dir, "bunny.sp", 64, 40, bvh=0)
    g, _ = sp.render_tiles(s, "direct_lighting", 4)
    c, _ = _oracle.render(s, 6, 4, variant="spm")
    assert rel_l2(g, c) < REL_L2_TOL
    assert np.mean(np.all(g == c, axis=-1)) > 0.999


def test_tile_subset_order_independent(scene_dir):
    s = load(scene_dir, "bunny.sp", 70, 35, bvh=0)  # clipped border tiles
    full, _ = sp.render_tiles(s, "direct_lighting", 2)
    ids = np.array([13, 0, 7, 44 % full.shape[0], 5], dtype=np.int32)
    part, _ = sp.render_tiles(s, "direct_lighting", 2, ids)
    assert np.array_equal(part, full[ids])
    img = sp.tiles_to_image(70, 35, full)
    assert img.shape == (35, 70, 3)
    # lanes outside the image are written as zero
    last = full[-1].reshape(64, 3)
    assert (last == 0).any()


@pytest.mark.parametrize("integrator", ["direct_lighting", "iterative_rrnee"])
def test_vs_glibc_oracle_bitexact(scene_dir, integrator):
    # reference semantics (glibc float libm): the device libm is an exact emulation
    s = load(scene_dir, "bunny.sp", 48, 32, bvh=1)
    g, _ = sp.render_tiles(s, integrator, 4)
    c, _ = _oracle.render(s, sp.string_to_integrator_type(integrator), 4, variant="glibc")
    r = rel_l2(g, c)
    frac = float(np.mean(np.all(g == c, axis=-1)))
    print(f"GPU vs glibc-libm oracle ({integrator}): rel_l2={r:.3e} bitexact_pixels={frac:.4f}")
    assert np.array_equal(g.view(np.uint32), c.view(np.uint32))


@pytest.mark.parametrize("integrator", ["direct_lighting", "brute_force_iterative_rr", "iterative_rrnee", "whitted",
                                        "brute_force"])
@pytest.mark.parametrize("guide", ["1", "0"])
def test_image_environment_light_bitexact(scene_dir, integrator, guide):
    # ImageBasedEnvironmentLight: Distribution2D sampling (guide tables, or the replayed libstdc++
    # upper_bound: sp_upload_params.env_replay), MIS pdf, escaping-ray lookups
    s = load(scene_dir, "material_spheres_ibl.sp", 24, 48, bvh=1, env_replay=guide == "0")
    g, gst = sp.render_tiles(s, integrator, 4)
    c, cst = _oracle.render(s, sp.string_to_integrator_type(integrator), 4, variant="glibc")
    assert gst.rays == cst["rays"] and gst.shadow_rays == cst["shadow_rays"]
    assert np.array_equal(g.view(np.uint32), c.view(np.uint32)), (integrator, rel_l2(g, c))


@pytest.mark.parametrize("scene,bvh", [("bunny.sp", 0), ("material_spheres.sp", 1), ("material_spheres_ibl.sp", 0)])
def test_wavefront_equals_megakernel(scene_dir, scene, bvh):
    # the two device pipelines run the same floating-point sequence per pixel
    s = load(scene_dir, scene, 72, 40, bvh=bvh)
    m, mst = sp.render_tiles(s, "direct_lighting", 5, pipeline="megakernel")
    w, wst = sp.render_tiles(s, "direct_lighting", 5, pipeline="wavefront")
    assert np.array_equal(m.view(np.uint32), w.view(np.uint32)), rel_l2(w, m)
    assert (mst.rays, mst.shadow_rays, mst.samples, mst.rng_draws) == \
        (wst.rays, wst.shadow_rays, wst.samples, wst.rng_draws)
    assert wst.launches == 3 + 4 * 5 and mst.launches in (1, 3)  # 3: tile-order probe + partition + render


@pytest.mark.parametrize("scene,bvh,chunks,replay", [("bunny.sp", 0, "0", "0"), ("bunny.sp", 1, "3", "0"),
                                                     ("bunny.sp", 0, "5", "1"), ("material_spheres_ibl.sp", 0, "7", "0"),
                                                     ("material_spheres.sp", 1, "16", "0"), ("closed_room.sp", 0, "4", "0")])
@pytest.mark.parametrize("fused", ["1", "0"])
def test_sample_chunks_equal_megakernel(scene_dir, monkeypatch, scene, bvh, chunks, replay, fused):
    # each pixel's samples split into chunks that start from generator snapshots: every sample
    # sees the same stream words, the sum keeps sample order -> bit-identical image and identical
    # ray / draw counts.  Chunk counts that do not divide spp (13) leave a short last chunk; "0" =
    # automatic (16 for this many tiles).  Draw counts come from the camera pass, or from the
    # Light::sample replay (image light, or SP_CHUNK_REPLAY=1).
    # With known counts the fused form (SP_CK_FUSED, default) runs the camera pass, the counts and the
    # chunks in one queue (sp_fused_kernel, sp_mega.hpp), then ck_sum: 2 launches.
    monkeypatch.setenv("SP_CHUNK_REPLAY", replay)
    monkeypatch.setenv("SP_CK_FUSED", fused)
    s = load(scene_dir, scene, 72, 40, bvh=bvh)
    m, mst = sp.render_tiles(s, "direct_lighting", 13, pipeline="megakernel")
    c, cst = sp.render_tiles(s, "direct_lighting", 13, pipeline="chunks", chunks_per_pixel=int(chunks))
    known = replay == "0" and scene != "material_spheres_ibl.sp"
    assert cst.pipeline == 3 and cst.launches == (2 if fused == "1" and known else 4)
    assert np.array_equal(m.view(np.uint32), c.view(np.uint32)), rel_l2(c, m)
    assert (mst.rays, mst.shadow_rays, mst.samples, mst.rng_draws) == \
        (cst.rays, cst.shadow_rays, cst.samples, cst.rng_draws)


def test_sample_chunks_tile_subset_matches_oracle(scene_dir):
    # a ragged tile subset (a rank's shard) through the chunk pipeline vs the CPU oracle
    s = load(scene_dir, "bunny.sp", 100, 60, bvh=1)
    tiles = np.arange(1, sp.TileScheduler(100, 60).get_num_tiles(), 2, dtype=np.int32)
    g, gst = sp.render_tiles(s, "direct_lighting", 6, tiles, pipeline="chunks")
    c, cst = _oracle.render(s, sp.string_to_integrator_type("direct_lighting"), 6, tiles, variant="spm")
    assert gst.rays == cst["rays"] and gst.shadow_rays == cst["shadow_rays"]
    assert np.array_equal(g.view(np.uint32), c.view(np.uint32)), rel_l2(g, c)


def test_wavefront_two_parts(scene_dir):
    # >= 32768 pixels in flight: two interleaved parts on two streams (ragged: odd tile count)
    s = load(scene_dir, "bunny.sp", 264, 128, bvh=0)
    m, _ = sp.render_tiles(s, "direct_lighting", 2, pipeline="megakernel")
    w, wst = sp.render_tiles(s, "direct_lighting", 2, pipeline="wavefront")
    assert wst.parts == 2
    assert np.array_equal(m.view(np.uint32), w.view(np.uint32)), rel_l2(w, m)
    ids = np.arange(sp.TileScheduler(264, 128).get_num_tiles(), dtype=np.int32)[::-1].copy()
    r, rst = sp.render_tiles(s, "direct_lighting", 2, ids, pipeline="wavefront")
    assert rst.parts == 2
    assert np.array_equal(r, w[ids])


def test_wavefront_tile_chunks(scene_dir, monkeypatch):
    # a tiny state budget forces several tile chunks per call; result must not change
    s = load(scene_dir, "bunny.sp", 64, 48, bvh=0)
    ids = np.arange(sp.TileScheduler(64, 48).get_num_tiles() - 1, -1, -1, dtype=np.int32)
    ref, _ = sp.render_tiles(s, "direct_lighting", 3, ids, pipeline="wavefront")
    monkeypatch.setenv("SP_WAVE_MAX_GB", "0.0016")  # ~5 tiles per chunk
    a, ast = sp.render_tiles(s, "direct_lighting", 3, ids, pipeline="wavefront")
    b, _ = sp.render_tiles(s, "direct_lighting", 3, None, pipeline="wavefront")
    assert ast.launches > 3 + 3 * 3
    assert np.array_equal(a, ref)
    assert np.array_equal(b[ids], ref)


def test_mandelbrot_full_frame_vs_reference(scene_dir):
    # the test integrator needs no scene queries: whole 96x64 frame, 2 spp, bit-exact
    from tests import test_oracle_vs_ref as R
    s = load(scene_dir, "bunny.sp", 96, 64, bvh=1)
    g, st = sp.render_tiles(s, "mandelbrot", 2)
    assert st.rays == 0 and st.rng_draws == 0
    c, _ = _oracle.render(s, sp.string_to_integrator_type("mandelbrot"), 2, variant="glibc")
    assert np.array_equal(g.view(np.uint32), c.view(np.uint32)), rel_l2(g, c)
    assert g.max() > 0.0


def test_wavefront_rejects_other_integrators(scene_dir):
    s = load(scene_dir, "bunny.sp", 16, 16, bvh=0)
    for integ in ("whitted", "brute_force", "mandelbrot", "iterative_rrnee", "brute_force_iterative"):
        with pytest.raises(sp.SimplePathError):
            sp.render_tiles(s, integ, 1, pipeline="wavefront")


@pytest.mark.parametrize("scene,w,h,integrator,spp", [("bunny.sp", 64, 40, "direct_lighting", 4),
                                                      ("bunny.sp", 32, 24, "iterative_rrnee", 2),
                                                      ("material_spheres.sp", 24, 48, "whitted", 3),
                                                      ("material_spheres.sp", 24, 48, "brute_force_iterative_rr", 3),
                                                      ("material_spheres_ibl.sp", 24, 48, "direct_lighting", 4),
                                                      ("material_spheres_ibl.sp", 24, 48, "iterative_rrnee", 3),
                                                      ("lucy_small.sp", 40, 56, "direct_lighting", 3),
                                                      ("elf_small.sp", 40, 56, "iterative_rrnee", 2)])
def test_vs_reference_build_bitexact(scene_dir, scene, w, h, integrator, spp):
    # the HIP path against the reference's own code (oracle/_ref, built from its sources)
    from tests import test_oracle_vs_ref as R
    if not os.path.exists(R.REF_LIB):
        pytest.skip("oracle/_ref not built (reference sources were not available)")
    import ctypes as C
    L = C.CDLL(R.REF_LIB)
    L.ref_render.restype = C.c_int
    L.ref_render.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_uint32, C.POINTER(C.c_int32), C.c_int64,
                             C.c_int, C.POINTER(C.c_float)]
    L.ref_last_error.restype = C.c_char_p
    s = load(scene_dir, scene, w, h, bvh=1)
    g, _ = sp.render_tiles(s, integrator, spp)
    ids = np.arange(g.shape[0], dtype=np.int32)
    r = R.ref_render(L, os.path.join(scene_dir, scene), w, h, sp.string_to_integrator_type(integrator), spp, ids)
    assert np.array_equal(g.view(np.uint32), r.view(np.uint32)), rel_l2(g, r)


@pytest.mark.parametrize("scene,w,h", [("bunny.sp", 64, 40), ("lucy_small.sp", 40, 56), ("elf_small.sp", 40, 56)])
def test_wide_bvh_vs_binary(scene_dir, scene, w, h):
    # 8-wide quantised BVH (SAH default) vs the binary SAH walk: same rays traced (any-hit is
    # exact, closest hit differs only on exactly equal distances) and the oracle tolerance
    s0 = load(scene_dir, scene, w, h, bvh=0, wide_bvh=False)
    b, bst = sp.render_tiles(s0, "direct_lighting", 4)
    s1 = load(scene_dir, scene, w, h, bvh=0)
    a, ast = sp.render_tiles(s1, "direct_lighting", 4)
    c, _ = _oracle.render(s1, 6, 4, variant="spm")
    assert rel_l2(a, c) < REL_L2_TOL and rel_l2(b, c) < REL_L2_TOL
    assert np.mean(np.all(a == b, axis=-1)) > 0.999


@pytest.mark.parametrize("integrator", ["brute_force", "whitted"])
def test_deep_recursion_bitexact(scene_dir, integrator):
    # max_depth 40 > the 32 in-register recursion levels: deeper levels live in global records
    s = load(scene_dir, "closed_room.sp", 16, 16, bvh=1)
    g, gst = sp.render_tiles(s, integrator, 2)
    c, cst = _oracle.render(s, sp.string_to_integrator_type(integrator), 2, variant="glibc")
    assert gst.rays == cst["rays"]
    assert np.array_equal(g.view(np.uint32), c.view(np.uint32)), rel_l2(g, c)
    if integrator == "brute_force":
        assert gst.rays > 16 * 16 * 2 * 20  # mean path length > 20: many paths go past level 32


@pytest.mark.parametrize("integrator,pipeline", [("direct_lighting", "megakernel"), ("direct_lighting", "wavefront"),
                                                 ("direct_lighting", "chunks"), ("iterative_rrnee", "megakernel"),
                                                 ("whitted", "megakernel")])
def test_degenerate_deep_bvh_stackless_bitexact(scene_dir, integrator, pipeline):
    # a reference BVH 172 levels deep (the reference's recursion is unbounded, BVHAccelerator.h:
    # 62-77): past the LDS budget, so every walk climbs parent links instead of a stack -- same
    # nodes, same order, same box tests: bit-exact against the oracle and the reference build
    s = load(scene_dir, "wedge_strip.sp", 64, 48, bvh=1)
    assert s.bvh_info()["depth"] == 172
    g, gst = sp.render_tiles(s, integrator, 3, pipeline=pipeline)
    assert gst.stack_depth == 0  # stackless
    t = sp.string_to_integrator_type(integrator)
    c, cst = _oracle.render(s, t, 3, variant="glibc")
    assert gst.rays == cst["rays"] and gst.shadow_rays == cst["shadow_rays"]
    assert np.array_equal(g.view(np.uint32), c.view(np.uint32)), rel_l2(g, c)
    assert g.max() > 0.0


@pytest.mark.parametrize("scene,w,h", [("bunny.sp", 64, 40), ("lucy_small.sp", 40, 56), ("material_spheres_ibl.sp", 24, 48)])
@pytest.mark.parametrize("integrator", ["direct_lighting", "iterative_rrnee"])
def test_forced_stackless_walk(scene_dir, monkeypatch, scene, w, h, integrator):
    # the parent-link walk forced on ordinary scenes (sp_upload_params.walk, and the SP_STACKLESS
    # test override) -- bit-exact vs the oracle on the reference BVH, and bit-identical to the
    # stack walk on the SAH binary BVH (near-first order)
    s = load(scene_dir, scene, w, h, bvh=1, stackless=True)
    g, gst = sp.render_tiles(s, integrator, 3)
    assert gst.stack_depth == 0
    c, _ = _oracle.render(s, sp.string_to_integrator_type(integrator), 3, variant="spm")
    assert np.array_equal(g.view(np.uint32), c.view(np.uint32)), rel_l2(g, c)
    monkeypatch.setenv("SP_STACKLESS", "1")
    a, ast = sp.render_tiles(load(scene_dir, scene, w, h, bvh=0), integrator, 3)
    monkeypatch.delenv("SP_STACKLESS")
    # the stackless scene walks the binary SAH BVH for any-hit too
    b, bst = sp.render_tiles(load(scene_dir, scene, w, h, bvh=0, wide_bvh=False), integrator, 3)
    assert ast.stack_depth == 0 and bst.stack_depth > 0
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), rel_l2(a, b)
    assert (ast.rays, ast.shadow_rays, ast.rng_draws) == (bst.rays, bst.shadow_rays, bst.rng_draws)


@pytest.mark.parametrize("scene,w,h,spp", [("elf_small.sp", 70, 35, 3), ("material_spheres.sp", 70, 35, 3),
                                           ("bunny.sp", 37, 21, 2)])
def test_rrnee_clipped_border_tiles_bitexact(scene_dir, scene, w, h, spp):
    # IterativeRRNEE with estimates served across the wave on image sizes that are not multiples
    # of 8: the lanes of a border tile that fall outside the image never enter integrate(), so the
    # served requests must be dealt to the lanes that are there (sp_path.hpp serve_rho)
    s = load(scene_dir, scene, w, h, bvh=1)
    g, gst = sp.render_tiles(s, "iterative_rrnee", spp)
    c, cst = _oracle.render(s, sp.string_to_integrator_type("iterative_rrnee"), spp, variant="spm")
    assert gst.rays == cst["rays"] and gst.shadow_rays == cst["shadow_rays"]
    assert np.isfinite(g).all()
    assert np.array_equal(g.view(np.uint32), c.view(np.uint32)), rel_l2(g, c)


@pytest.mark.parametrize("scene,w,h,spp", [("elf_small.sp", 40, 56, 3), ("elf_small.sp", 70, 35, 2),
                                           ("material_spheres.sp", 24, 48, 3), ("material_spheres_ibl.sp", 24, 48, 3),
                                           ("bunny.sp", 64, 40, 2), ("lucy_small.sp", 40, 56, 2),
                                           ("closed_room.sp", 16, 16, 2)])
def test_rrnee_merged_queries_equal_per_lane(scene_dir, scene, w, h, spp):
    # IterativeRRNEE on SAH scenes deals each bounce's MIS-ray and next closest-hit BVH walks over
    # the wave (sp_path.hpp mq_run); SP_RENDER_PER_LANE_QUERIES walks every ray on its own lane.
    # Same queries, same walks: bit-identical images and identical ray / shadow / draw counts
    # (material_spheres: two lights -- only the last light's MIS ray joins the pass; closed_room:
    # max_depth 40; a clipped size)
    s = load(scene_dir, scene, w, h, bvh=0)
    a, ast = sp.render_tiles(s, "iterative_rrnee", spp)
    b, bst = sp.render_tiles(s, "iterative_rrnee", spp, per_lane_queries=True)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), rel_l2(a, b)
    assert (ast.rays, ast.shadow_rays, ast.samples, ast.rng_draws) == (bst.rays, bst.shadow_rays, bst.samples, bst.rng_draws)
    c, _ = _oracle.render(s, sp.string_to_integrator_type("iterative_rrnee"), spp, variant="spm")
    assert rel_l2(a, c) < REL_L2_TOL
