"""The C-ABI render boundary on the device (include/simplepath_hip.h, ABI 4):

  * stream order -- sp_render_tiles without stats only enqueues: two renders and a dependent
    kernel queue back to back on one stream with no host wait, and the result is bit-exact;
  * the device tile list (d_tile_ids): nothing crosses to the host;
  * the occupancy request (waves_per_simd) and the chunk count (chunks_per_pixel) change how the
    image is computed, never the image;
  * argument validation (reserved fields, unknown flags, both tile lists, occupancy ranges).
"""
import os

import numpy as np
import pytest
import torch

import simplepath_amd as sp
from simplepath_amd import _abi

pytestmark = pytest.mark.gpu


def load(scene_dir, name, w, h, bvh=0):
    s = sp.Scene.from_file(os.path.join(scene_dir, name))
    s.set_resolution(w, h)
    s.upload(device=0, bvh_mode=bvh)
    return s


def test_stream_ordered_renders_and_dependent_kernel(scene_dir):
    s = load(scene_dir, "bunny.sp", 256, 160)
    n = sp.TileScheduler(256, 160).get_num_tiles()
    a_ids = np.arange(0, n, 2, dtype=np.int32)
    b_ids = np.arange(1, n, 2, dtype=np.int32)
    ref_a, _ = sp.render_tiles(s, "direct_lighting", 16, a_ids, pipeline="megakernel")
    ref_b, _ = sp.render_tiles(s, "direct_lighting", 16, b_ids, pipeline="megakernel")
    dev = torch.device("cuda:0")
    d_a = torch.from_numpy(a_ids).to(dev)
    d_b = torch.from_numpy(b_ids).to(dev)
    out_a = torch.zeros((a_ids.size, 64, 3), dtype=torch.float32, device=dev)
    out_b = torch.zeros_like(out_a)
    stream = torch.cuda.Stream()
    torch.cuda.synchronize()
    with torch.cuda.stream(stream):
        for out, d in ((out_a, d_a), (out_b, d_b)):
            r = sp.render_tiles_device(s, "direct_lighting", 16, None, out.data_ptr(), stream.cuda_stream,
                                       pipeline="megakernel", stats=False, d_tile_ids=d.data_ptr(),
                                       num_tiles=d.numel())
            assert r is None
        busy = not stream.query()  # the renders were only enqueued: the stream still has work
        both = out_a + out_b       # a dependent kernel behind them, still without a host wait
    stream.synchronize()
    assert busy, "sp_render_tiles waited for the render although no stats were requested"
    assert np.array_equal(out_a.cpu().numpy().view(np.uint32), ref_a.view(np.uint32))
    assert np.array_equal(out_b.cpu().numpy().view(np.uint32), ref_b.view(np.uint32))
    assert np.array_equal(both.cpu().numpy(), ref_a + ref_b)


@pytest.mark.parametrize("pipeline", ["megakernel", "chunks", "wavefront"])
def test_device_tile_list(scene_dir, pipeline):
    s = load(scene_dir, "bunny.sp", 96, 64, bvh=1)
    ids = np.random.default_rng(3).permutation(sp.TileScheduler(96, 64).get_num_tiles())[:37].astype(np.int32)
    ref, rst = sp.render_tiles(s, "direct_lighting", 4, ids, pipeline=pipeline)
    d = torch.from_numpy(ids).cuda()
    out = torch.zeros((ids.size, 64, 3), dtype=torch.float32, device="cuda:0")
    st = sp.render_tiles_device(s, "direct_lighting", 4, None, out.data_ptr(), torch.cuda.current_stream().cuda_stream,
                                pipeline=pipeline, d_tile_ids=d.data_ptr(), num_tiles=ids.size)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), ref.view(np.uint32))
    assert (st.rays, st.shadow_rays, st.samples, st.rng_draws) == (rst.rays, rst.shadow_rays, rst.samples, rst.rng_draws)


@pytest.mark.parametrize("integrator,waves", [("direct_lighting", (1, 2, 3, 4)), ("iterative_rrnee", (2, 3, 4))])
def test_waves_per_simd_variants_identical(scene_dir, integrator, waves):
    s = load(scene_dir, "elf_small.sp", 40, 56)
    ref, rst = sp.render_tiles(s, integrator, 3, pipeline="megakernel")
    for w in waves:
        out, st = sp.render_tiles(s, integrator, 3, pipeline="megakernel", waves_per_simd=w)
        assert np.array_equal(out.view(np.uint32), ref.view(np.uint32)), w
        assert (st.rays, st.rng_draws) == (rst.rays, rst.rng_draws)


def test_chunks_per_pixel_identical(scene_dir):
    s = load(scene_dir, "bunny.sp", 72, 40)
    ref, _ = sp.render_tiles(s, "direct_lighting", 9, pipeline="megakernel")
    for c in (1, 2, 4, 9):
        out, st = sp.render_tiles(s, "direct_lighting", 9, pipeline="chunks", chunks_per_pixel=c)
        assert st.pipeline == sp.PIPELINES["chunks"]
        assert np.array_equal(out.view(np.uint32), ref.view(np.uint32)), c


def test_chunk_budget_falls_back_under_auto(scene_dir):
    # a budget too small for the chunk buffers: AUTO renders with the megakernel, an explicit
    # request is refused
    s = load(scene_dir, "bunny.sp", 72, 40)
    out, st = sp.render_tiles(s, "direct_lighting", 4, chunk_max_gb=1e-6)
    assert st.pipeline == sp.PIPELINES["megakernel"]
    with pytest.raises(sp.SimplePathError):
        sp.render_tiles(s, "direct_lighting", 4, pipeline="chunks", chunk_max_gb=1e-6)


def test_render_params_validation(scene_dir):
    s = load(scene_dir, "bunny.sp", 32, 32)
    bad = [dict(waves_per_simd=5), dict(waves_per_simd=-1)]
    for kw in bad:
        with pytest.raises(sp.SimplePathError):
            sp.render_tiles(s, "direct_lighting", 1, **kw)
    with pytest.raises(sp.SimplePathError):
        sp.render_tiles(s, "whitted", 1, waves_per_simd=3)  # one variant only
    with pytest.raises(sp.SimplePathError):
        sp.render_tiles(s, "iterative_rrnee", 1, waves_per_simd=1)
    with pytest.raises(sp.SimplePathError):
        sp.render_tiles(s, "direct_lighting", 1, chunks_per_pixel=-2)
    import ctypes as C
    for field, value in (("reserved", 1), ("flags", 64), ("tail_fraction", 1.5), ("tail_fraction", float("nan"))):
        p, keep = sp._params("direct_lighting", 1, None)
        setattr(p, field, value)
        out = torch.zeros((16, 64, 3), dtype=torch.float32, device="cuda:0")
        rc = _abi.lib().sp_render_tiles(s.handle, C.byref(p), C.c_void_p(out.data_ptr()), None)
        assert rc == _abi.SP_ERR_ARG, field
    d = torch.zeros(4, dtype=torch.int32, device="cuda:0")
    p, keep = sp._params("direct_lighting", 1, np.arange(4))
    p.d_tile_ids = C.c_void_p(d.data_ptr())
    out = torch.zeros((4, 64, 3), dtype=torch.float32, device="cuda:0")
    assert _abi.lib().sp_render_tiles(s.handle, C.byref(p), C.c_void_p(out.data_ptr()), None) == _abi.SP_ERR_ARG


def test_upload_options_are_part_of_the_residency(scene_dir):
    # re-uploading with other accelerator options really rebuilds (the options are part of the
    # cache key), and every option gives the same image on the reference BVH
    s = sp.Scene.from_file(os.path.join(scene_dir, "material_spheres_ibl.sp"))
    s.set_resolution(24, 48)
    s.upload(0, 1)
    ref, rst = sp.render_tiles(s, "iterative_rrnee", 3)
    for kw in (dict(env_replay=True), dict(stackless=True), dict(stack_max_levels=1), dict(wide_bvh=False)):
        s.upload(0, 1, **kw)
        out, st = sp.render_tiles(s, "iterative_rrnee", 3)
        assert np.array_equal(out.view(np.uint32), ref.view(np.uint32)), kw
        if kw.get("stackless") or kw.get("stack_max_levels"):
            assert st.stack_depth == 0
        else:
            assert st.stack_depth == rst.stack_depth


@pytest.mark.parametrize("integrator", ["direct_lighting", "iterative_rrnee", "whitted"])
def test_tile_order_probe_is_invisible(scene_dir, integrator):
    # the megakernel's tile order (a one-sample probe pass, then the slow tiles first) changes only
    # which wave renders which tile and when: images and ray / draw counts equal queue order's,
    # also for a tile subset in a shuffled order
    s = load(scene_dir, "bunny.sp", 640, 512)  # 5120 tiles: more than the persistent waves (4096)
    # forced (tile_order_factor): AUTO uses it from 6 tiles per wave and 128 spp (IterativeRRNEE: 4, 16)
    ref, rst = sp.render_tiles(s, integrator, 2, pipeline="megakernel", tile_order_factor=2.0)
    # probe, partition, render; integrators without a probe kernel (sp_probe_*.hip) keep queue order
    # (+ the in-order sum of the tail chunks: DirectLighting with the order renders its most expensive
    # tiles as sample chunks, tests/test_gpu_tail.py)
    assert rst.launches == (1 if integrator == "whitted" else 3 + (rst.tail_tiles > 0))
    assert (rst.tail_tiles > 0) == (integrator == "direct_lighting")
    off, ost = sp.render_tiles(s, integrator, 2, pipeline="megakernel", tile_order_factor=-1.0)
    assert ost.launches == 1
    assert np.array_equal(ref.view(np.uint32), off.view(np.uint32))
    assert (rst.rays, rst.shadow_rays, rst.samples, rst.rng_draws) == (ost.rays, ost.shadow_rays, ost.samples, ost.rng_draws)
    for factor in (0.5, 1.0, 4.0):
        ids = np.random.default_rng(int(factor * 10)).permutation(ref.shape[0]).astype(np.int32)
        sub, _ = sp.render_tiles(s, integrator, 2, ids, pipeline="megakernel", tile_order_factor=factor)
        assert np.array_equal(sub.view(np.uint32), ref[ids].view(np.uint32)), factor


@pytest.mark.parametrize("integrator", ["direct_lighting", "iterative_rrnee"])
def test_tile_order_on_strided_lists(scene_dir, integrator):
    # a host list in image order with a constant stride (a rank's interleaved shard) gets the
    # neighbour-blended estimate (sp_capi.hip order_neighbours: the tile below when the stride
    # divides tiles_x, else left / right only); the list as a whole frame (stride 1), a stride that
    # divides the 160 tiles per row (2, 4) and one that does not (3) all render the frame's rows
    s = load(scene_dir, "bunny.sp", 1280, 1024)  # 20480 tiles, 160 per row
    ref, _ = sp.render_tiles(s, integrator, 2, pipeline="megakernel", tile_order_factor=-1.0)
    for k in (1, 2, 3, 4):
        ids = np.arange(k - 1, ref.shape[0], k, dtype=np.int32)
        sub, st = sp.render_tiles(s, integrator, 2, ids, pipeline="megakernel", tile_order_factor=2.0)
        assert st.launches == 3 + (st.tail_tiles > 0), k  # the order ran: more tiles than persistent waves
        assert (st.tail_tiles > 0) == (integrator == "direct_lighting"), k
        assert np.array_equal(sub.view(np.uint32), ref[ids].view(np.uint32)), k


@pytest.mark.parametrize("pipeline", ["megakernel", "chunks", "wavefront"])
def test_device_ids_outside_the_image_render_zeros(scene_dir, pipeline):
    # a device tile list is not checked on the host: ids outside [0, tiles) -- negative ones too --
    # render as zeros and add nothing to the ray counts
    s = load(scene_dir, "bunny.sp", 72, 40, bvh=1)
    n = sp.TileScheduler(72, 40).get_num_tiles()
    good = np.array([3, 0, n - 1], dtype=np.int32)
    ref, rst = sp.render_tiles(s, "direct_lighting", 3, good, pipeline=pipeline)
    ids = np.array([3, -1, 0, n, -n, n - 1, -9], dtype=np.int32)
    d = torch.from_numpy(ids).cuda()
    out = torch.full((ids.size, 64, 3), 7.0, dtype=torch.float32, device="cuda:0")
    st = sp.render_tiles_device(s, "direct_lighting", 3, None, out.data_ptr(), torch.cuda.current_stream().cuda_stream,
                                pipeline=pipeline, d_tile_ids=d.data_ptr(), num_tiles=ids.size)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    valid = [0, 2, 5]
    assert np.array_equal(o[valid].view(np.uint32), ref.view(np.uint32))
    assert not o[[1, 3, 4, 6]].any()
    assert (st.rays, st.shadow_rays, st.samples) == (rst.rays, rst.shadow_rays, rst.samples)


@pytest.mark.parametrize("integrator", ["direct_lighting", "iterative_rrnee"])
def test_one_scene_two_threads_two_streams(scene_dir, integrator):
    # the reference's render() shares one Scene across host threads (main.cpp:122-130); two threads
    # render disjoint tile sets of one scene on two streams without waiting (stats off) -- the
    # scene serialises them, and each result equals a single-threaded call bit for bit
    import threading
    s = load(scene_dir, "bunny.sp", 160, 96)
    n = sp.TileScheduler(160, 96).get_num_tiles()
    sets = [np.arange(0, n, 2, dtype=np.int32), np.arange(1, n, 2, dtype=np.int32)]
    refs = [sp.render_tiles(s, integrator, 4, ids, pipeline="megakernel")[0] for ids in sets]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = [torch.zeros((ids.size, 64, 3), dtype=torch.float32, device="cuda:0") for ids in sets]
    errors = []
    torch.cuda.synchronize()

    def work(k):
        try:
            for _ in range(3):
                ids = sets[k].copy()
                sp.render_tiles_device(s, integrator, 4, ids, outs[k].data_ptr(), streams[k].cuda_stream,
                                       pipeline="megakernel", stats=False)
                ids[:] = -5  # the host list may be reused as soon as the call returns
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=work, args=(k,)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    torch.cuda.synchronize()
    assert not errors, errors
    for k in range(2):
        assert np.array_equal(outs[k].cpu().numpy().view(np.uint32), refs[k].view(np.uint32)), k


def test_scene_device_bytes(scene_dir):
    # sp_scene_device_bytes: the resident scene's HBM bytes (bench.py counts them in the
    # algorithmic bytes of a frame); at least the triangle records of both BVH layouts
    s = load(scene_dir, "bunny.sp", 64, 40)
    info = s.bvh_info()
    b = s.device_bytes()
    assert b >= 2 * info["slots"] * 48 and b < 200e6
    s.upload(device=0, bvh_mode=1)  # the reference BVH alone: no 8-wide copy
    assert 0 < s.device_bytes() < b
