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
