"""ctypes mirror of include/simplepath_hip.h (the C-ABI boundary).

Only plain pointers and sizes cross the boundary.  The library is built in-tree
(simplepath_amd/_build/libsimplepath_hip.so); importing this module fails loudly when it is
missing -- there is no CPU fallback on the product path.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# SP_LIB_PATH: an alternative build of the same library (experiments, e.g. compile-time variants)
LIB_PATH = os.environ.get("SP_LIB_PATH") or os.path.join(_HERE, "_build", "libsimplepath_hip.so")

SP_OK = 0
SP_ERR_PARSE, SP_ERR_IO, SP_ERR_ARG, SP_ERR_HIP, SP_ERR_UNSUPPORTED, SP_ERR_STATE = -1, -2, -3, -4, -5, -6

INTEGRATORS = {
    "mandelbrot": 1,
    "brute_force": 2,
    "brute_force_iterative": 3,
    "brute_force_iterative_rr": 4,
    "iterative_rrnee": 5,
    "direct_lighting": 6,
    "whitted": 7,
}


class sp_affine(C.Structure):
    _fields_ = [("vx", C.c_float * 3), ("vy", C.c_float * 3), ("vz", C.c_float * 3), ("p", C.c_float * 3)]


class sp_linear(C.Structure):
    _fields_ = [("vx", C.c_float * 3), ("vy", C.c_float * 3), ("vz", C.c_float * 3)]


class sp_material_desc(C.Structure):
    _fields_ = [
        ("kind", C.c_int32), ("base", C.c_int32),
        ("lambert_albedo", C.c_float * 3), ("microfacet_r", C.c_float * 3),
        ("alpha_x", C.c_float), ("alpha_y", C.c_float), ("microfacet_ior", C.c_float),
        ("sample_visible_area", C.c_int32), ("coat_ior", C.c_float), ("coat_color", C.c_float * 3),
    ]


class sp_xform_shape(C.Structure):
    _fields_ = [("object_to_world", sp_affine), ("world_to_object", sp_affine),
                ("normal_to_world", sp_linear), ("material", C.c_int32), ("kind", C.c_int32)]


class sp_light_desc(C.Structure):
    _fields_ = [("kind", C.c_int32), ("image", C.c_int32), ("radiance", C.c_float * 3),
                ("object_to_world", sp_affine), ("world_to_object", sp_affine),
                ("normal_to_world", sp_linear)]


class sp_env_image(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("pixels", C.POINTER(C.c_float)),
                ("max_radiance", C.c_float), ("reserved", C.c_int32),
                ("light_to_world", sp_linear), ("world_to_light", sp_linear)]


class sp_camera_desc(C.Structure):
    _fields_ = [("transform", sp_affine), ("film_width", C.c_int32), ("film_height", C.c_int32)]


class sp_scene_info(C.Structure):
    _fields_ = [
        ("image_width", C.c_int32), ("image_height", C.c_int32),
        ("russian_roulette_depth", C.c_int32), ("max_depth", C.c_int32),
        ("integrator_type", C.c_int32), ("num_triangles", C.c_int32), ("num_vertices", C.c_int32),
        ("num_shapes", C.c_int32), ("num_lights", C.c_int32), ("num_materials", C.c_int32),
        ("output_file_name", C.c_char * 256),
    ]


class sp_scene_desc(C.Structure):
    _fields_ = [
        ("info", sp_scene_info), ("camera", sp_camera_desc),
        ("vertices", C.POINTER(C.c_float)), ("normals", C.POINTER(C.c_float)),
        ("indices", C.POINTER(C.c_uint32)), ("tri_material", C.POINTER(C.c_int32)),
        ("shapes", C.POINTER(sp_xform_shape)),
        ("prim_kind", C.POINTER(C.c_int32)), ("prim_index", C.POINTER(C.c_int32)), ("num_prims", C.c_int64),
        ("lights", C.POINTER(sp_light_desc)), ("materials", C.POINTER(sp_material_desc)),
        ("env_images", C.POINTER(sp_env_image)), ("num_env_images", C.c_int32), ("reserved", C.c_int32),
    ]


class sp_render_params(C.Structure):
    _fields_ = [
        ("integrator", C.c_int32), ("samples_per_pixel", C.c_uint32),
        ("tile_ids", C.POINTER(C.c_int32)), ("num_tiles", C.c_int64),
        ("stream", C.c_void_p), ("bvh_mode", C.c_int32), ("flags", C.c_int32),
        # ABI 4
        ("d_tile_ids", C.c_void_p), ("waves_per_simd", C.c_int32), ("chunks_per_pixel", C.c_int32),
        ("chunk_max_gb", C.c_float),
        # ABI 5
        ("tile_order_factor", C.c_float),
        # ABI 6
        ("tail_fraction", C.c_float), ("reserved", C.c_int32),
    ]


SP_WALK_AUTO, SP_WALK_STACKLESS = 0, 1


class sp_upload_params(C.Structure):
    _fields_ = [("bvh_mode", C.c_int32), ("walk", C.c_int32), ("stack_max_levels", C.c_int32),
                ("no_wide_bvh", C.c_int32), ("env_replay", C.c_int32), ("sah_leaf", C.c_int32),
                ("binary_closest", C.c_int32), ("reserved", C.c_int32)]


class sp_render_stats(C.Structure):
    _fields_ = [("rays", C.c_uint64), ("shadow_rays", C.c_uint64), ("samples", C.c_uint64),
                ("rng_draws", C.c_uint64), ("kernel_ms", C.c_float), ("pipeline", C.c_int32),
                ("launches", C.c_int32), ("primary_hits", C.c_uint64), ("stage_ms", C.c_float * 4),
                ("parts", C.c_int32), ("stack_depth", C.c_int32), ("tail_tiles", C.c_int32), ("tail_chunks", C.c_int32)]


class sp_bvh_info(C.Structure):
    _fields_ = [("depth", C.c_int32), ("wide_depth", C.c_int32), ("light_depth", C.c_int32),
                ("stack_depth", C.c_int32), ("nodes", C.c_int64), ("slots", C.c_int64)]


# Every symbol declared in include/simplepath_hip.h, with its ctypes signature.
SIGNATURES = {
    "sp_version": (C.c_char_p, []),
    "sp_build_id": (C.c_char_p, []),
    "sp_last_error": (C.c_char_p, []),
    "sp_string_to_integrator": (C.c_int, [C.c_char_p, C.POINTER(C.c_int32)]),
    "sp_scene_load": (C.c_int, [C.c_char_p, C.POINTER(C.c_void_p)]),
    "sp_scene_load_string": (C.c_int, [C.c_char_p, C.c_char_p, C.POINTER(C.c_void_p)]),
    "sp_scene_from_desc": (C.c_int, [C.POINTER(sp_scene_desc), C.POINTER(C.c_void_p)]),
    "sp_scene_free": (None, [C.c_void_p]),
    "sp_scene_get_info": (C.c_int, [C.c_void_p, C.POINTER(sp_scene_info)]),
    "sp_scene_get_desc": (C.c_int, [C.c_void_p, C.POINTER(sp_scene_desc)]),
    "sp_scene_set_resolution": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32]),
    "sp_tile_count": (C.c_int, [C.c_int32, C.c_int32, C.POINTER(C.c_int64)]),
    "sp_tile_origin": (C.c_int, [C.c_int32, C.c_int32, C.c_int64, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "sp_device_count": (C.c_int, [C.POINTER(C.c_int32)]),
    "sp_scene_upload": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32]),
    "sp_scene_upload_ex": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(sp_upload_params)]),
    "sp_render_tiles": (C.c_int, [C.c_void_p, C.POINTER(sp_render_params), C.c_void_p, C.POINTER(sp_render_stats)]),
    "sp_render_tiles_host": (C.c_int, [C.c_void_p, C.POINTER(sp_render_params), C.POINTER(C.c_float),
                                       C.POINTER(sp_render_stats)]),
    "sp_scene_bvh_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "sp_scene_device_bytes": (C.c_int, [C.c_void_p, C.POINTER(C.c_int64)]),
    "sp_scene_bvh_build_info": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(sp_bvh_info)]),
    "sp_tiles_to_image": (C.c_int, [C.c_int32, C.c_int32, C.POINTER(C.c_int32), C.c_int64,
                                    C.POINTER(C.c_float), C.POINTER(C.c_float)]),
    "sp_write_pfm": (C.c_int, [C.c_char_p, C.c_int32, C.c_int32, C.POINTER(C.c_float)]),
    "sp_rsqrt_table_get": (C.c_int, [C.POINTER(C.c_uint32), C.c_int64, C.POINTER(C.c_int32), C.POINTER(C.c_uint32),
                                     C.POINTER(C.c_uint32)]),
    "sp_rsqrt_table_set": (C.c_int, [C.POINTER(C.c_uint32), C.c_int32, C.c_uint32, C.c_uint32]),
    "sp_rsqrt_table_info": (C.c_int, [C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "sp_host_rsqrt_emulated": (C.c_float, [C.c_float]),
}

_lib = None


def lib():
    """Load the in-tree HIP library (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: build it with `make -C simplepath_amd` or __graft_entry__.build(); "
                "the MI355X path has no CPU fallback")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def build_identity() -> dict:
    """Which library this process runs: its path, the build's content hash (sp_build_id, ABI 5)
    and the SHA-256 prefix of the .so file itself -- recorded in every bench line, so a swapped
    library (SP_LIB_PATH) is visible."""
    import hashlib
    L = lib()
    with open(LIB_PATH, "rb") as f:
        so_sha = hashlib.sha256(f.read()).hexdigest()[:16]
    return {"path": os.path.relpath(os.path.realpath(LIB_PATH), os.path.dirname(_HERE)),
            "build_id": L.sp_build_id().decode(), "so_sha256_16": so_sha,
            "default": os.path.realpath(LIB_PATH) == os.path.realpath(os.path.join(_HERE, "_build", "libsimplepath_hip.so"))}


class SimplePathError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code


def check(rc: int) -> None:
    if rc != SP_OK:
        raise SimplePathError(rc, lib().sp_last_error().decode(errors="replace"))
