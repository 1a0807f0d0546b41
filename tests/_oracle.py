"""TEST INFRASTRUCTURE: ctypes binding of the CPU oracle (oracle/_build/liboracle_*.so)."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
_libs = {}


def build() -> None:
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True, timeout=600)


def load(variant: str = "spm"):
    """variant 'glibc' = reference semantics; 'spm' = product device libm on the host."""
    if variant not in _libs:
        path = os.path.join(ORACLE_DIR, "_build", f"liboracle_{variant}.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        L.orc_render.restype = C.c_int
        L.orc_render.argtypes = [C.c_void_p, C.c_int, C.c_uint32, C.POINTER(C.c_int32), C.c_int64, C.c_int,
                                 C.POINTER(C.c_float), C.POINTER(C.c_uint64)]
        L.orc_mt_stream.restype = None
        L.orc_mt_stream.argtypes = [C.c_uint32, C.c_int, C.POINTER(C.c_float)]
        L.orc_rsqrt.restype = C.c_float
        L.orc_rsqrt.argtypes = [C.c_float]
        _libs[variant] = L
    return _libs[variant]


def render(scene, integrator: int, spp: int, tile_ids=None, threads: int = 8, variant: str = "spm"):
    """Render tiles on the CPU oracle; returns (tiles [n,64,3], stats dict)."""
    from simplepath_amd import TileScheduler
    L = load(variant)
    desc = scene.desc()
    ids = None if tile_ids is None else np.ascontiguousarray(tile_ids, dtype=np.int32)
    n = ids.size if ids is not None else TileScheduler(scene.width, scene.height).get_num_tiles()
    out = np.zeros((max(n, 1), 64, 3), dtype=np.float32)
    st = (C.c_uint64 * 3)()
    rc = L.orc_render(C.byref(desc), int(integrator), int(spp),
                      None if ids is None else ids.ctypes.data_as(C.POINTER(C.c_int32)),
                      0 if ids is None else ids.size, threads, out.ctypes.data_as(C.POINTER(C.c_float)), st)
    assert rc == 0, rc
    return out[:n], {"rays": st[0], "shadow_rays": st[1], "samples": st[2]}
