"""The C-ABI library loads and exports every symbol include/simplepath_hip.h declares."""
import os
import re

import simplepath_amd as sp
from simplepath_amd import _abi

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "simplepath_hip.h")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(sp_[a-z0-9_]+)\s*\(", text)))


def test_every_declared_symbol_is_exported():
    L = sp.lib()
    names = declared_symbols()
    assert len(names) >= 20
    for n in names:
        assert hasattr(L, n), n
    assert set(names) == set(_abi.SIGNATURES), set(names) ^ set(_abi.SIGNATURES)


def test_integrator_names_match_reference():
    # Integrators/Integrator.cpp:25-51
    for name, val in _abi.INTEGRATORS.items():
        assert sp.string_to_integrator_type(name) == val
        assert sp.string_to_integrator_type("  " + name + " ") == val
    try:
        sp.string_to_integrator_type("path_guiding")
        raise AssertionError("expected failure")
    except sp.SimplePathError as e:
        assert "Unknown integrator type" in str(e)


def test_tile_scheduler_column_major_order():
    # base/TileScheduler.h:72-86: x = i % tiles_x, y = i / tiles_x, 8x8 tiles, clipped count
    s = sp.ColumnMajorTileScheduler(20, 11)
    assert s.get_num_tiles() == 3 * 2
    assert [s.tile_origin(i) for i in range(6)] == [(0, 0), (8, 0), (16, 0), (0, 8), (8, 8), (16, 8)]
    got = [s.get_next_tile() for _ in range(7)]
    assert got == [0, 1, 2, 3, 4, 5, None]


def test_render_requires_upload(scene_dir):
    scene = sp.Scene.from_file(os.path.join(scene_dir, "bunny.sp"))
    try:
        sp.render_tiles(scene, "direct_lighting", 1, [0])
        raise AssertionError("expected SP_ERR_STATE")
    except sp.SimplePathError as e:
        assert e.code == _abi.SP_ERR_STATE


def test_abi_version_and_struct_layout():
    # ABI 4: sp_render_params grew the device tile list, occupancy and chunk fields; the ctypes
    # mirror must match the header's layout.  ABI 5 (same layout): sp_build_id, per-scene
    # serialisation of renders.
    import ctypes as C
    text = open(HEADER).read()
    # ABI 6: tail_fraction takes the first reserved word (same size); the stats grew two words.
    assert re.search(r"#define SP_ABI_VERSION 6\b", text)
    assert C.sizeof(_abi.sp_render_params) == 72  # gcc on include/simplepath_hip.h: 72, 40, 60, 64, 68, 32, 88
    assert _abi.sp_render_params.d_tile_ids.offset == 40 and _abi.sp_render_params.tile_order_factor.offset == 60
    assert _abi.sp_render_params.tail_fraction.offset == 64 and _abi.sp_render_params.reserved.offset == 68
    assert C.sizeof(_abi.sp_upload_params) == 32
    assert C.sizeof(_abi.sp_render_stats) == 88


def test_upload_params_validated_before_the_device(scene_dir):
    # argument errors come back as SP_ERR_ARG before any device is touched (this container has none)
    import ctypes as C
    scene = sp.Scene.from_file(os.path.join(scene_dir, "bunny.sp"))
    for field, value in (("walk", 7), ("bvh_mode", 2), ("sah_leaf", 9), ("stack_max_levels", -1), ("binary_closest", 2)):
        p = _abi.sp_upload_params()
        setattr(p, field, value)
        assert _abi.lib().sp_scene_upload_ex(scene.handle, 0, C.byref(p)) == _abi.SP_ERR_ARG, field
    p = _abi.sp_upload_params()
    p.reserved = 3
    assert _abi.lib().sp_scene_upload_ex(scene.handle, 0, C.byref(p)) == _abi.SP_ERR_ARG


def test_build_identity():
    # the bench records which library ran: path, content hash of its sources, hash of the .so
    ident = _abi.build_identity()
    assert re.fullmatch(r"[0-9a-f]{16}", ident["build_id"]), ident
    assert re.fullmatch(r"[0-9a-f]{16}", ident["so_sha256_16"]), ident
    assert ident["path"].endswith("libsimplepath_hip.so")
