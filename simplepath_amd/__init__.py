"""simplepath_amd -- MI355X-native per-pixel integration path of kjeffery/SimplePath.

Host-side mirror of the reference's Scene / Integrator / TileScheduler interface
(base/Scene.h, Integrators/Integrator.h, base/TileScheduler.h, main.cpp:77-142) over the
C-ABI in include/simplepath_hip.h.  All integration runs in HIP kernels on the GPU; this module
only parses arguments, owns handles and moves buffers.

    scene = Scene.from_file("bunny.sp")          # sp::parse_file (base/FileParser.cpp:929)
    scene.upload(device=0)                       # BVH build + HBM residency
    sched = ColumnMajorTileScheduler(scene.width, scene.height)
    img, stats = render(scene, "direct_lighting", num_pixel_samples=256)   # main.cpp:109 render()
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from . import _abi
from ._abi import INTEGRATORS, SimplePathError, check, lib

__all__ = [
    "Scene", "TileScheduler", "ColumnMajorTileScheduler", "RenderStats", "render", "render_tiles",
    "render_tiles_device", "tiles_to_image", "write_pfm", "string_to_integrator_type", "INTEGRATORS",
    "SimplePathError", "k_tile_dimension", "rsqrt_table", "set_rsqrt_table",
]

k_tile_dimension = 8  # base/Tile.h:10


def string_to_integrator_type(s: str) -> int:
    """Integrators/Integrator.cpp:25 -- raises on unknown names like the reference."""
    out = C.c_int32()
    check(lib().sp_string_to_integrator(s.encode(), C.byref(out)))
    return out.value


@dataclass
class RenderStats:
    rays: int
    shadow_rays: int
    samples: int
    rng_draws: int
    kernel_ms: float
    pipeline: int = 0
    launches: int = 0
    primary_hits: int = 0
    stage_ms: tuple = (0.0, 0.0, 0.0, 0.0)
    parts: int = 1
    stack_depth: int = 0
    tail_tiles: int = 0   # megakernel: tiles rendered as tail chunks (ABI 6)
    tail_chunks: int = 0  # ... sample chunks per such tile


class Scene:
    """base/Scene.h:48 -- parsed scene, optionally resident in HBM."""

    def __init__(self, handle: C.c_void_p):
        self._h = handle
        self._device = None

    @classmethod
    def from_file(cls, path: str) -> "Scene":
        h = C.c_void_p()
        check(lib().sp_scene_load(path.encode(), C.byref(h)))
        return cls(h)

    @classmethod
    def from_string(cls, text: str, base_dir: str = ".") -> "Scene":
        h = C.c_void_p()
        check(lib().sp_scene_load_string(text.encode(), base_dir.encode(), C.byref(h)))
        return cls(h)

    @classmethod
    def from_desc(cls, desc: _abi.sp_scene_desc) -> "Scene":
        """Scene::Scene from an already-built, flattened scene (sp_scene_from_desc: copied)."""
        h = C.c_void_p()
        check(lib().sp_scene_from_desc(C.byref(desc), C.byref(h)))
        return cls(h)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _abi._lib is not None:
            _abi._lib.sp_scene_free(h)
            self._h = None

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    def info(self) -> _abi.sp_scene_info:
        i = _abi.sp_scene_info()
        check(lib().sp_scene_get_info(self._h, C.byref(i)))
        return i

    def desc(self) -> _abi.sp_scene_desc:
        d = _abi.sp_scene_desc()
        check(lib().sp_scene_get_desc(self._h, C.byref(d)))
        return d

    @property
    def width(self) -> int:
        return self.info().image_width

    @property
    def height(self) -> int:
        return self.info().image_height

    @property
    def integrator_type(self) -> int:
        return self.info().integrator_type

    def set_resolution(self, width: int, height: int) -> None:
        check(lib().sp_scene_set_resolution(self._h, width, height))

    def upload(self, device: int = 0, bvh_mode: int = 0, stackless: bool = False, stack_max_levels: int = 0,
               wide_bvh: bool = True, env_replay: bool = False, sah_leaf: int = 0,
               binary_closest: bool = False) -> None:
        """bvh_mode 0 = SAH (throughput), 1 = the reference's median-split BVH (tie-exact order).
        The other options (sp_upload_params) change how the same image is computed, never the
        image: the parent-link walk, the LDS-stack depth budget, the image-light guide tables, the
        SAH leaf size.  On the SAH BVH, wide_bvh / binary_closest choose the 8-wide or binary walks,
        which can only differ in which of two primitives at exactly equal distance wins."""
        p = _abi.sp_upload_params()
        p.bvh_mode = bvh_mode
        p.walk = _abi.SP_WALK_STACKLESS if stackless else _abi.SP_WALK_AUTO
        p.stack_max_levels = stack_max_levels
        p.no_wide_bvh = 0 if wide_bvh else 1
        p.binary_closest = 1 if binary_closest else 0
        p.env_replay = 1 if env_replay else 0
        p.sah_leaf = sah_leaf
        check(lib().sp_scene_upload_ex(self._h, device, C.byref(p)))
        self._device = device

    def bvh_info(self):
        d, n, s = C.c_int32(), C.c_int64(), C.c_int64()
        check(lib().sp_scene_bvh_info(self._h, C.byref(d), C.byref(n), C.byref(s)))
        return {"depth": d.value, "nodes": n.value, "slots": s.value}

    def device_bytes(self) -> int:
        """HBM bytes of the uploaded scene (sp_scene_device_bytes)."""
        b = C.c_int64()
        check(lib().sp_scene_device_bytes(self._h, C.byref(b)))
        return b.value

    def bvh_build_info(self, bvh_mode: int = 0) -> dict:
        """Host-only BVH build statistics (no device): what upload(bvh_mode) would build."""
        i = _abi.sp_bvh_info()
        check(lib().sp_scene_bvh_build_info(self._h, bvh_mode, C.byref(i)))
        return {k: getattr(i, k) for k, _ in _abi.sp_bvh_info._fields_}


class TileScheduler:
    """base/TileScheduler.h:18 -- tiles of k_tile_dimension^2 pixels over the image extents."""

    def __init__(self, width: int, height: int):
        self.width, self.height = width, height
        self._counter = 0

    def get_num_tiles(self) -> int:
        n = C.c_int64()
        check(lib().sp_tile_count(self.width, self.height, C.byref(n)))
        return n.value

    def tile_origin(self, tile: int):
        x, y = C.c_int32(), C.c_int32()
        check(lib().sp_tile_origin(self.width, self.height, tile, C.byref(x), C.byref(y)))
        return x.value, y.value


class ColumnMajorTileScheduler(TileScheduler):
    """base/TileScheduler.h:59 -- tile index order x = i % tiles_x, y = i / tiles_x, pass clamp."""

    def __init__(self, width: int, height: int, pass_clamp: int = 1):
        super().__init__(width, height)
        self.pass_clamp = pass_clamp

    def get_next_tile(self) -> Optional[int]:
        n = self.get_num_tiles()
        c = self._counter
        self._counter += 1
        if c // n >= self.pass_clamp:
            return None
        return c % n

    def shard(self, rank: int, world: int) -> np.ndarray:
        """Tiles owned by `rank` of `world` (interleaved: balanced cost across ranks; shard.py)."""
        from .shard import shard_tiles
        return shard_tiles(self.get_num_tiles(), rank, world)


PIPELINES = {"auto": 0, "megakernel": 1, "wavefront": 2, "chunks": 3}
STAGE_TIMING = 4  # SP_RENDER_STAGE_TIMING
PER_LANE_QUERIES = 8  # SP_RENDER_PER_LANE_QUERIES (ABI 5)


def _params(integrator, spp, tile_ids: Optional[np.ndarray], stream=None, pipeline="auto",
            stage_timing=False, waves_per_simd=0, chunks_per_pixel=0, chunk_max_gb=0.0,
            tile_order_factor=0.0, per_lane_queries=False, tail_fraction=0.0) -> tuple:
    if isinstance(integrator, str):
        integrator = string_to_integrator_type(integrator)
    p = _abi.sp_render_params()
    p.integrator = int(integrator or 0)
    p.samples_per_pixel = int(spp)
    keep = None
    if tile_ids is not None:
        keep = np.ascontiguousarray(tile_ids, dtype=np.int32)
        p.tile_ids = keep.ctypes.data_as(C.POINTER(C.c_int32))
        p.num_tiles = keep.size
    p.stream = stream
    p.flags = ((PIPELINES[pipeline] if isinstance(pipeline, str) else int(pipeline)) | (STAGE_TIMING if stage_timing else 0)
               | (PER_LANE_QUERIES if per_lane_queries else 0))
    p.waves_per_simd = int(waves_per_simd)
    p.chunks_per_pixel = int(chunks_per_pixel)
    p.chunk_max_gb = float(chunk_max_gb)
    p.tile_order_factor = float(tile_order_factor)
    p.tail_fraction = float(tail_fraction)
    return p, keep


def _stats(s: _abi.sp_render_stats) -> RenderStats:
    return RenderStats(s.rays, s.shadow_rays, s.samples, s.rng_draws, s.kernel_ms, s.pipeline, s.launches,
                       s.primary_hits, tuple(s.stage_ms), s.parts, s.stack_depth, s.tail_tiles, s.tail_chunks)


def render_tiles(scene: Scene, integrator, num_pixel_samples: int, tile_ids: Optional[Sequence[int]] = None,
                 pipeline="auto", **options):
    """Render tiles on the GPU; returns (tile-packed radiance [n,64,3] float32, RenderStats).
    options: waves_per_simd, chunks_per_pixel, chunk_max_gb (sp_render_params, ABI 4),
    tile_order_factor (ABI 5: 0 automatic, > 0 forced with that factor, < 0 queue order),
    tail_fraction (ABI 6: megakernel tail chunks, 0 automatic, < 0 off, else the fraction of tiles),
    per_lane_queries (ABI 5: IterativeRRNEE without the merged query pass -- the comparison path)."""
    p, keep = _params(integrator, num_pixel_samples, None if tile_ids is None else np.asarray(tile_ids),
                      pipeline=pipeline, **options)
    n = keep.size if keep is not None else TileScheduler(scene.width, scene.height).get_num_tiles()
    out = np.zeros((max(n, 1), 64, 3), dtype=np.float32)
    st = _abi.sp_render_stats()
    check(lib().sp_render_tiles_host(scene.handle, C.byref(p), out.ctypes.data_as(C.POINTER(C.c_float)), C.byref(st)))
    return out[:n], _stats(st)


def render_tiles_device(scene: Scene, integrator, num_pixel_samples: int, tile_ids, out_ptr: int, stream=None,
                        pipeline="auto", stage_timing=False, stats=True, d_tile_ids: int = 0,
                        num_tiles: int = 0, **options):
    """Render into a caller-owned device buffer (e.g. a torch.cuda tensor's data_ptr()).
    tile_ids: host tile list (None: d_tile_ids, a device pointer to num_tiles int32 ids, or every
    tile).  With stats=False (and no stage timing) the render is only enqueued on `stream`: the
    call returns without waiting (returns None); a host tile list is copied before it returns."""
    p, keep = _params(integrator, num_pixel_samples, None if tile_ids is None else np.asarray(tile_ids), stream,
                      pipeline, stage_timing, **options)
    if d_tile_ids:
        p.d_tile_ids = C.c_void_p(d_tile_ids)
        p.num_tiles = int(num_tiles)
    if not stats:
        check(lib().sp_render_tiles(scene.handle, C.byref(p), C.c_void_p(out_ptr), None))
        return None
    st = _abi.sp_render_stats()
    check(lib().sp_render_tiles(scene.handle, C.byref(p), C.c_void_p(out_ptr), C.byref(st)))
    return _stats(st)


def tiles_to_image(width: int, height: int, tiles: np.ndarray, tile_ids: Optional[np.ndarray] = None) -> np.ndarray:
    img = np.zeros((height, width, 3), dtype=np.float32)
    t = np.ascontiguousarray(tiles, dtype=np.float32)
    ids = None if tile_ids is None else np.ascontiguousarray(tile_ids, dtype=np.int32)
    check(lib().sp_tiles_to_image(width, height,
                                  None if ids is None else ids.ctypes.data_as(C.POINTER(C.c_int32)),
                                  0 if ids is None else ids.size,
                                  t.ctypes.data_as(C.POINTER(C.c_float)), img.ctypes.data_as(C.POINTER(C.c_float))))
    return img


def rsqrt_table() -> dict:
    """The RSQRTSS table scenes are built and rendered with (sp_rsqrt_table_get)."""
    bits, zero, den = C.c_int32(), C.c_uint32(), C.c_uint32()
    check(lib().sp_rsqrt_table_get(None, 0, C.byref(bits), C.byref(zero), C.byref(den)))
    entries = np.zeros(2 << bits.value, dtype=np.uint32)
    check(lib().sp_rsqrt_table_get(entries.ctypes.data_as(C.POINTER(C.c_uint32)), entries.size, None, None, None))
    return {"entries": entries, "bits": bits.value, "zero_result": zero.value, "denorm_result": den.value}


def set_rsqrt_table(table: Optional[dict]) -> None:
    """Emulate another CPU's RSQRTSS (a table from rsqrt_table() there); None: this host's."""
    if table is None:
        check(lib().sp_rsqrt_table_set(None, 0, 0, 0))
        return
    e = np.ascontiguousarray(table["entries"], dtype=np.uint32)
    if e.size != 2 << int(table["bits"]):
        raise ValueError("RSQRTSS table: entries must hold 2 << bits words")
    check(lib().sp_rsqrt_table_set(e.ctypes.data_as(C.POINTER(C.c_uint32)), int(table["bits"]),
                                   int(table["zero_result"]), int(table["denorm_result"])))


def write_pfm(path: str, image: np.ndarray) -> None:
    """Image/Image.cpp:40 write_pfm."""
    img = np.ascontiguousarray(image, dtype=np.float32)
    check(lib().sp_write_pfm(path.encode(), img.shape[1], img.shape[0], img.ctypes.data_as(C.POINTER(C.c_float))))


def render(scene: Scene, integrator=None, num_pixel_samples: int = 1):
    """main.cpp:109 render(): whole frame, returns (image HxWx3, RenderStats)."""
    tiles, st = render_tiles(scene, integrator or 0, num_pixel_samples)
    return tiles_to_image(scene.width, scene.height, tiles), st
