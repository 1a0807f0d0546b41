"""Pin the CPU oracle to the reference itself.

oracle/_ref/libsp_ref.so is the reference's render path compiled from the sources under
/root/reference (oracle/build_ref.sh + oracle/ref_harness.cpp): the reference's own Scene,
BVHAccelerator, shapes, materials, lights, samplers and integrators, driven by main.cpp's
per-pixel loop.  The C oracle built against glibc's float libm (liboracle_glibc.so: reference
semantics) must reproduce it bit for bit; the GPU is in turn checked bit-exact against the oracle
(tests/test_gpu_parity.py), closing the chain reference == oracle == HIP path.

The library exists only where the reference sources were available at build time (this
container); elsewhere these tests skip.
"""
import ctypes as C
import os

import numpy as np
import pytest

import simplepath_amd as sp
from tests import _oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_LIB = os.path.join(ROOT, "oracle", "_ref", "libsp_ref.so")


@pytest.fixture(scope="module")
def ref():
    if not os.path.exists(REF_LIB):
        if os.path.isdir("/root/reference"):
            import subprocess
            subprocess.run(["bash", os.path.join(ROOT, "oracle", "build_ref.sh")], check=True, timeout=1200)
        else:
            pytest.skip("reference sources not present: oracle/_ref not built")
    L = C.CDLL(REF_LIB)
    L.ref_render.restype = C.c_int
    L.ref_render.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_uint32, C.POINTER(C.c_int32), C.c_int64,
                             C.c_int, C.POINTER(C.c_float)]
    L.ref_last_error.restype = C.c_char_p
    return L


def ref_render(L, path, w, h, integrator, spp, ids):
    ids = np.ascontiguousarray(ids, dtype=np.int32)
    out = np.zeros((ids.size, 64, 3), dtype=np.float32)
    rc = L.ref_render(path.encode(), w, h, integrator, spp, ids.ctypes.data_as(C.POINTER(C.c_int32)), ids.size, 8,
                      out.ctypes.data_as(C.POINTER(C.c_float)))
    assert rc == 0, L.ref_last_error()
    return out


def oracle_render(path, w, h, integrator, spp, ids):
    s = sp.Scene.from_file(path)
    s.set_resolution(w, h)
    out, _ = _oracle.render(s, integrator, spp, ids, variant="glibc")
    return out


def same(a, b):
    return np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_bunny_direct_lighting(ref, scene_dir):
    path = os.path.join(scene_dir, "bunny.sp")
    ids = np.arange(sp.TileScheduler(64, 40).get_num_tiles(), dtype=np.int32)
    r = ref_render(ref, path, 64, 40, 6, 4, ids)
    o = oracle_render(path, 64, 40, 6, 4, ids)
    assert same(r, o), float(np.abs(r - o).max())
    assert r.max() > 0.0


def test_bunny_clipped_tiles_and_order(ref, scene_dir):
    path = os.path.join(scene_dir, "bunny.sp")
    n = sp.TileScheduler(70, 35).get_num_tiles()
    ids = np.array([n - 1, 3, 0, n // 2], dtype=np.int32)  # ragged border tiles, any order
    r = ref_render(ref, path, 70, 35, 6, 3, ids)
    o = oracle_render(path, 70, 35, 6, 3, ids)
    assert same(r, o)


@pytest.mark.parametrize("integrator", ["direct_lighting", "brute_force", "brute_force_iterative",
                                        "brute_force_iterative_rr", "iterative_rrnee", "whitted", "mandelbrot"])
def test_spheres_every_integrator(ref, scene_dir, integrator):
    path = os.path.join(scene_dir, "material_spheres.sp")
    t = sp.string_to_integrator_type(integrator)
    ids = np.arange(sp.TileScheduler(24, 48).get_num_tiles(), dtype=np.int32)
    r = ref_render(ref, path, 24, 48, t, 3, ids)
    o = oracle_render(path, 24, 48, t, 3, ids)
    assert same(r, o), (integrator, float(np.abs(r - o).max()))


def test_bunny_multibounce(ref, scene_dir):
    path = os.path.join(scene_dir, "bunny.sp")
    ids = np.arange(0, sp.TileScheduler(32, 24).get_num_tiles(), dtype=np.int32)
    r = ref_render(ref, path, 32, 24, 5, 2, ids)
    o = oracle_render(path, 32, 24, 5, 2, ids)
    assert same(r, o)


@pytest.mark.parametrize("integrator", ["direct_lighting", "brute_force_iterative_rr", "iterative_rrnee", "whitted",
                                        "brute_force"])
def test_image_environment_light(ref, scene_dir, integrator):
    """scenes/material_spheres.sp with its ImageBasedEnvironmentLight (synthetic HDR map with
    clamped, infinite, negative and black texels): light sampling through Distribution2D,
    the light pdf of the MIS integrator, and radiance lookups of escaping rays."""
    path = os.path.join(scene_dir, "material_spheres_ibl.sp")
    t = sp.string_to_integrator_type(integrator)
    ids = np.arange(sp.TileScheduler(24, 48).get_num_tiles(), dtype=np.int32)
    r = ref_render(ref, path, 24, 48, t, 4, ids)
    o = oracle_render(path, 24, 48, t, 4, ids)
    assert same(r, o), (integrator, float(np.abs(r - o).max()), int(np.sum(r != o)))
    assert r.max() > 0.0


@pytest.mark.parametrize("scene,integrator,spp", [("bunny_scan.sp", "direct_lighting", 3),
                                                  ("lucy_small.sp", "direct_lighting", 3),
                                                  ("elf_small.sp", "direct_lighting", 3),
                                                  ("elf_small.sp", "iterative_rrnee", 2)])
def test_figure_scenes(ref, scene_dir, scene, integrator, spp):
    """lucy.sp (PLY with a scene rotation) and elf.sp (binary STL: std::map vertex welding,
    file face normals; max_depth 16) with their constant environment lights."""
    path = os.path.join(scene_dir, scene)
    t = sp.string_to_integrator_type(integrator)
    ids = np.arange(sp.TileScheduler(40, 56).get_num_tiles(), dtype=np.int32)
    r = ref_render(ref, path, 40, 56, t, spp, ids)
    o = oracle_render(path, 40, 56, t, spp, ids)
    assert same(r, o), (scene, integrator, float(np.abs(r - o).max()))
    assert r.max() > 0.0


@pytest.mark.parametrize("integrator", ["brute_force", "whitted", "iterative_rrnee"])
def test_deep_recursion(ref, scene_dir, integrator):
    """Closed room, max_depth 40: recursive paths run to the depth limit."""
    path = os.path.join(scene_dir, "closed_room.sp")
    t = sp.string_to_integrator_type(integrator)
    ids = np.arange(sp.TileScheduler(16, 16).get_num_tiles(), dtype=np.int32)
    r = ref_render(ref, path, 16, 16, t, 2, ids)
    o = oracle_render(path, 16, 16, t, 2, ids)
    assert same(r, o), (integrator, float(np.abs(r - o).max()))
    assert r.max() > 0.0


@pytest.mark.parametrize("integrator", ["direct_lighting", "iterative_rrnee"])
def test_degenerate_deep_bvh(ref, scene_dir, integrator):
    """A wedge strip whose reference BVH nests 172 levels (shapes/BVHAccelerator.h:62-77 recurses
    without bound): the oracle's recursive walk and the reference agree bit for bit."""
    path = os.path.join(scene_dir, "wedge_strip.sp")
    t = sp.string_to_integrator_type(integrator)
    ids = np.arange(sp.TileScheduler(64, 48).get_num_tiles(), dtype=np.int32)
    r = ref_render(ref, path, 64, 48, t, 3, ids)
    o = oracle_render(path, 64, 48, t, 3, ids)
    assert same(r, o), (integrator, float(np.abs(r - o).max()))
    assert r.max() > 0.0
