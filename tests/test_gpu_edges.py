"""Edge cases of the drop-in boundary on the device, against the CPU oracle (bit for bit with the
reference-order BVH): images smaller than one tile, duplicate ids in a tile list, a scene without
lights, max_depth 0 and 1 for every integrator, and a long sample chain (many mt19937_64
generations per pixel) -- the corners main.cpp's render loop can reach with a valid .sp file."""
import os

import numpy as np
import pytest

import simplepath_amd as sp
from simplepath_amd import scenes
from tests import _oracle

pytestmark = pytest.mark.gpu

INTEGRATORS = ["direct_lighting", "brute_force", "brute_force_iterative", "brute_force_iterative_rr",
               "iterative_rrnee", "whitted"]


def load(path, w, h, bvh=1):
    s = sp.Scene.from_file(path)
    s.set_resolution(w, h)
    s.upload(device=0, bvh_mode=bvh)
    return s


def oracle(s, integrator, spp, tiles=None):
    img, st = _oracle.render(s, sp.string_to_integrator_type(integrator), spp, tiles, variant="spm")
    return img, st


def same_bits(a, b):
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("w,h", [(1, 1), (7, 3), (9, 17)])
@pytest.mark.parametrize("pipeline", ["megakernel", "wavefront", "chunks"])
def test_images_smaller_than_a_tile(scene_dir, w, h, pipeline):
    # one partial tile (or a few): the lanes outside the image never render, their slots stay zero
    s = load(os.path.join(scene_dir, "bunny.sp"), w, h)
    g, gst = sp.render_tiles(s, "direct_lighting", 3, pipeline=pipeline)
    c, cst = oracle(s, "direct_lighting", 3)
    assert gst.rays == cst["rays"] and gst.shadow_rays == cst["shadow_rays"]
    assert same_bits(g, c)
    assert sp.tiles_to_image(w, h, g).shape == (h, w, 3)


@pytest.mark.parametrize("w,h", [(1, 1), (7, 3)])
def test_tiny_images_multibounce(scene_dir, w, h):
    s = load(os.path.join(scene_dir, "bunny.sp"), w, h)
    g, gst = sp.render_tiles(s, "iterative_rrnee", 4)
    c, cst = oracle(s, "iterative_rrnee", 4)
    assert gst.rays == cst["rays"] and same_bits(g, c)


@pytest.mark.parametrize("pipeline", ["megakernel", "chunks"])
def test_duplicate_tile_ids(scene_dir, pipeline):
    # a tile listed twice is rendered twice from its pixels' own seeds: both rows equal the frame's
    s = load(os.path.join(scene_dir, "bunny.sp"), 40, 24)
    full, _ = sp.render_tiles(s, "direct_lighting", 2, pipeline=pipeline)
    ids = np.array([5, 5, 0, 14, 5], dtype=np.int32)
    part, st = sp.render_tiles(s, "direct_lighting", 2, ids, pipeline=pipeline)
    assert same_bits(part, full[ids])
    assert st.samples == ids.size * 64 * 2  # 40 x 24: every tile is whole


def test_scene_without_lights(scene_dir, tmp_path):
    # no light at all: direct lighting is black everywhere, the multi-bounce paths find no emitter;
    # the light accelerator is empty on the device
    d = str(tmp_path)
    text = scenes.bunny_sp(scenes.ensure_bunny_ply(d))
    i = text.index("sphere_light {")
    text = text[:i] + text[text.index("}", i) + 1:]
    path = os.path.join(d, "bunny_dark.sp")
    with open(path, "w") as fh:
        fh.write(text)
    s = load(path, 24, 16)
    for integrator in ("direct_lighting", "iterative_rrnee"):
        g, gst = sp.render_tiles(s, integrator, 2)
        c, cst = oracle(s, integrator, 2)
        assert gst.rays == cst["rays"] and same_bits(g, c), integrator
        assert not np.any(g), integrator


@pytest.mark.parametrize("max_depth", [0, 1])
@pytest.mark.parametrize("integrator", INTEGRATORS)
def test_max_depth_zero_and_one(tmp_path, max_depth, integrator):
    path = scenes.write_closed_room_scene(str(tmp_path), max_depth=max_depth, name=f"room_{max_depth}.sp")
    s = load(path, 16, 16)
    g, gst = sp.render_tiles(s, integrator, 3)
    c, cst = oracle(s, integrator, 3)
    assert gst.rays == cst["rays"] and gst.shadow_rays == cst["shadow_rays"]
    assert same_bits(g, c), (integrator, max_depth)


@pytest.mark.timeout(300)
def test_long_sample_chain(scene_dir):
    # 600 samples on a glossy-heavy tile: each pixel's stream runs through ~40 mt19937_64
    # generations, so every twist path (ahead of a sample, inside a reservation, at a draw) is taken
    s = load(os.path.join(scene_dir, "bunny.sp"), 16, 8)
    ids = np.array([0], dtype=np.int32)
    for integrator, pipelines in (("direct_lighting", ("megakernel", "chunks")), ("iterative_rrnee", ("megakernel",))):
        c, cst = oracle(s, integrator, 600, ids)
        draws = set()
        for pipeline in pipelines:
            g, gst = sp.render_tiles(s, integrator, 600, ids, pipeline=pipeline)
            draws.add(gst.rng_draws)
            assert gst.rays == cst["rays"] and same_bits(g, c), (integrator, pipeline)
        assert len(draws) == 1 and draws.pop() > 64 * 312, integrator  # more than one generation per pixel


@pytest.mark.parametrize("pipeline", ["megakernel", "chunks"])
def test_coloured_microfacet_reflectance(scene_dir, pipeline):
    # every glossy material a scene file makes has a white microfacet colour, and the rho estimate
    # computes one channel for a grey one (sp_path.hpp rho_accumulate); a host-built scene may give
    # any colour: here one glossy material coloured and the others grey, so waves hold both kinds
    a = sp.Scene.from_file(os.path.join(scene_dir, "bunny.sp"))
    a.set_resolution(40, 24)
    d = a.desc()
    glossy = [k for k in range(d.info.num_materials) if d.materials[k].kind == 1]
    assert len(glossy) >= 2
    for k in glossy[:: 2]:
        d.materials[k].microfacet_r[0], d.materials[k].microfacet_r[1], d.materials[k].microfacet_r[2] = 0.9, 0.5, 0.2
    s = sp.Scene.from_desc(d)
    s.upload(device=0, bvh_mode=1)
    for integrator in ["direct_lighting", "iterative_rrnee"] if pipeline == "megakernel" else ["direct_lighting"]:
        g, gst = sp.render_tiles(s, integrator, 3, pipeline=pipeline)
        c, cst = oracle(s, integrator, 3)
        assert gst.rays == cst["rays"] and same_bits(g, c), integrator
