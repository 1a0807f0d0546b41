"""The DirectLighting megakernel's tail chunks (sp_mega.hpp tail_prep / tail_chunk):
the most expensive tiles of the tile order are rendered as sample chunks at the end of the
persistent queue.  Only which wave computes which samples, and when, changes -- every sample sees
the same stream words and floating-point sequence and each pixel's samples are summed in order --
so images and ray / draw counts must equal the plain megakernel's bit for bit, and the CPU
oracle's with the reference-order BVH (main.cpp:86-103: one tile's pixels x samples)."""
import math
import os

import numpy as np
import pytest

import simplepath_amd as sp
from simplepath_amd import scenes
from tests import _oracle

pytestmark = pytest.mark.gpu

W, H = 640, 512  # 5120 tiles: more than the 4096 persistent waves, so the tile order can run


def load(path, bvh=0, w=W, h=H):
    s = sp.Scene.from_file(path)
    s.set_resolution(w, h)
    s.upload(device=0, bvh_mode=bvh)
    return s


def same_bits(a, b):
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


def counts(st):
    return (st.rays, st.shadow_rays, st.samples, st.rng_draws)


@pytest.fixture
def tail_chunks(monkeypatch):
    def set_chunks(n):
        monkeypatch.setenv("SP_TAIL_CHUNKS", str(n))
    return set_chunks


@pytest.mark.parametrize("spp", [3, 8])
def test_tail_chunks_are_invisible(scene_dir, tail_chunks, spp):
    s = load(os.path.join(scene_dir, "bunny.sp"))
    n = sp.TileScheduler(W, H).get_num_tiles()
    ref, rst = sp.render_tiles(s, "direct_lighting", spp, pipeline="megakernel", tile_order_factor=2.0, tail_fraction=-1.0)
    assert rst.tail_tiles == 0 and rst.launches == 3
    for frac, chunks in ((0.05, 64), (0.12, 2), (0.5, 3), (1.0, 1)):
        tail_chunks(chunks)
        img, st = sp.render_tiles(s, "direct_lighting", spp, pipeline="megakernel", tile_order_factor=2.0,
                                  tail_fraction=frac)
        k = min(n, math.ceil(float(np.float32(frac)) * n - 1e-3))
        len_ = -(-spp // min(chunks, spp))
        assert st.tail_tiles == k and st.tail_chunks == -(-spp // len_), (frac, chunks)
        assert st.launches == 4  # probe, partition, render with tail chunks, the in-order sum
        assert counts(st) == counts(rst), (frac, chunks)
        assert same_bits(img, ref), (frac, chunks)


def test_tail_chunks_on_caller_lists(scene_dir):
    # shuffled subsets and duplicate ids: chunk slot k maps to the list slot order[k], whose tile the
    # caller named; a duplicated tile gets two slots (two stores), both equal to the frame's row
    s = load(os.path.join(scene_dir, "bunny.sp"))
    ref, _ = sp.render_tiles(s, "direct_lighting", 3, pipeline="megakernel", tile_order_factor=-1.0)
    rng = np.random.default_rng(7)
    ids = rng.permutation(ref.shape[0])[:4600].astype(np.int32)
    ids = np.concatenate([ids, ids[:300]])  # 300 duplicates
    sub, st = sp.render_tiles(s, "direct_lighting", 3, ids, pipeline="megakernel", tile_order_factor=2.0,
                              tail_fraction=0.25)
    assert st.tail_tiles == math.ceil(float(np.float32(0.25)) * ids.size - 1e-3)
    assert same_bits(sub, ref[ids])


def test_tail_chunks_match_the_oracle(scene_dir):
    # reference-order BVH: the whole frame, tail tiles included, bit for bit with the CPU oracle
    s = load(os.path.join(scene_dir, "bunny.sp"), bvh=1)
    img, st = sp.render_tiles(s, "direct_lighting", 2, pipeline="megakernel", tile_order_factor=2.0, tail_fraction=0.3)
    assert st.tail_tiles > 0
    c, cst = _oracle.render(s, sp.string_to_integrator_type("direct_lighting"), 2, variant="spm")
    assert (st.rays, st.shadow_rays) == (cst["rays"], cst["shadow_rays"])
    assert same_bits(img, c)


@pytest.mark.parametrize("bvh", [0, 1])
def test_tail_chunks_with_an_image_light(scene_dir, tail_chunks, bvh):
    # with an image light a sample's draw count depends on the drawn numbers (Light::sample), so
    # each prep item replays Light::sample on the stream itself to place the chunk starts
    s = load(os.path.join(scene_dir, "material_spheres_ibl.sp"), bvh=bvh, w=640, h=512)
    off, ost = sp.render_tiles(s, "direct_lighting", 5, pipeline="megakernel", tile_order_factor=-1.0)
    for frac, chunks in ((0.5, 2), (1.0, 5), (0.2, 64)):
        tail_chunks(chunks)
        img, st = sp.render_tiles(s, "direct_lighting", 5, pipeline="megakernel", tile_order_factor=2.0,
                                  tail_fraction=frac)
        assert st.tail_tiles > 0 and st.launches == 4
        assert same_bits(img, off) and counts(st) == counts(ost), (frac, chunks)


@pytest.mark.parametrize("max_depth", [0, 1])
def test_tail_chunks_max_depth(tmp_path, max_depth):
    # max_depth 0: no camera ray is traced and nothing is drawn (integrate_direct returns black)
    path = scenes.write_closed_room_scene(str(tmp_path), max_depth=max_depth, name=f"room_{max_depth}.sp")
    s = load(path)
    ref, rst = sp.render_tiles(s, "direct_lighting", 4, pipeline="megakernel", tile_order_factor=2.0, tail_fraction=-1.0)
    img, st = sp.render_tiles(s, "direct_lighting", 4, pipeline="megakernel", tile_order_factor=2.0, tail_fraction=0.4)
    assert st.tail_tiles > 0
    assert counts(st) == counts(rst) and same_bits(img, ref)


def test_auto_takes_the_tail_on_a_two_way_shard(scene_dir):
    # AUTO: DirectLighting from 3 tiles per persistent wave and 128 spp (no image light) runs the
    # megakernel with its tile order and tail chunks -- a 2-GPU shard of the 1080p frame (16200
    # tiles) included, which the sample chunks rendered before ABI 6; same image either way
    from simplepath_amd import shard
    s = load(os.path.join(scene_dir, "bunny.sp"), w=1920, h=1080)
    ids = shard.shard_tiles(sp.TileScheduler(1920, 1080).get_num_tiles(), 0, 2)
    img, st = sp.render_tiles(s, "direct_lighting", 128, ids)
    assert st.pipeline == sp.PIPELINES["megakernel"] and st.tail_tiles > 0
    ck, cst = sp.render_tiles(s, "direct_lighting", 128, ids, pipeline="chunks")
    assert counts(st) == counts(cst) and same_bits(img, ck)
    _, ost = sp.render_tiles(s, "direct_lighting", 8, ids, tail_fraction=-1.0)
    assert ost.pipeline == sp.PIPELINES["chunks"]  # tail off (or below 128 spp): the old rule


@pytest.mark.parametrize("front_div,cam_block", [("1", "32"), ("64", "5"), ("100000", "1000")])
def test_fused_sample_chunks(scene_dir, monkeypatch, front_div, cam_block):
    # the sample-chunk pipeline's fused form: ck_camera, then every tile's prep (stream positions,
    # generations into the store) and its chunks in one queue, prep g + P dealt after tile g's chunks
    # (P = persistent waves / SP_CK_FRONT_DIV: all preps first, some ahead, one ahead); equal to the
    # four-kernel form and the plain megakernel
    s = load(os.path.join(scene_dir, "bunny.sp"))
    ids = np.arange(0, sp.TileScheduler(W, H).get_num_tiles(), 2, dtype=np.int32)  # 2560 tiles
    ref, rst = sp.render_tiles(s, "direct_lighting", 6, ids, pipeline="megakernel", tile_order_factor=-1.0)
    monkeypatch.setenv("SP_CK_FRONT_DIV", front_div)
    monkeypatch.setenv("SP_CK_CAM_BLOCK", cam_block)  # camera items of 32, 5 (ragged) or all samples
    img, st = sp.render_tiles(s, "direct_lighting", 6, ids, pipeline="chunks", chunks_per_pixel=3)
    assert st.launches == 2 and counts(st) == counts(rst) and same_bits(img, ref)  # the camera pass in the queue
    monkeypatch.setenv("SP_CK_CAMFOLD", "0")
    img, st = sp.render_tiles(s, "direct_lighting", 6, ids, pipeline="chunks", chunks_per_pixel=3)
    assert st.launches == 3 and counts(st) == counts(rst) and same_bits(img, ref)  # ck_camera before the queue
    monkeypatch.setenv("SP_CK_FUSED", "0")
    four, fst = sp.render_tiles(s, "direct_lighting", 6, ids, pipeline="chunks", chunks_per_pixel=3)
    assert fst.launches == 4 and counts(fst) == counts(rst) and same_bits(four, ref)


def test_tail_chunks_with_replayed_counts(scene_dir, monkeypatch, tail_chunks):
    # SP_CHUNK_REPLAY=1: the preps replay Light::sample on the stream (the image-light form,
    # sp_tail_kernel<4, true>) for sphere lights as well -- same chunk starts, same image
    s = load(os.path.join(scene_dir, "bunny.sp"))
    ref, rst = sp.render_tiles(s, "direct_lighting", 6, pipeline="megakernel", tile_order_factor=-1.0)
    monkeypatch.setenv("SP_CHUNK_REPLAY", "1")
    for frac, chunks in ((0.3, 4), (1.0, 6)):
        tail_chunks(chunks)
        img, st = sp.render_tiles(s, "direct_lighting", 6, pipeline="megakernel", tile_order_factor=2.0,
                                  tail_fraction=frac)
        assert st.tail_tiles > 0 and counts(st) == counts(rst) and same_bits(img, ref), (frac, chunks)


def test_tail_chunks_within_the_budget(scene_dir):
    # the tail buffers (hit records, radiance, each tail pixel's stream generations) count against
    # chunk_max_gb like the sample chunks': over it, the frame renders without tail chunks
    s = load(os.path.join(scene_dir, "bunny.sp"))
    ref, rst = sp.render_tiles(s, "direct_lighting", 3, pipeline="megakernel", tile_order_factor=2.0, tail_fraction=-1.0)
    img, st = sp.render_tiles(s, "direct_lighting", 3, pipeline="megakernel", tile_order_factor=2.0, tail_fraction=0.5,
                              chunk_max_gb=1e-3)
    assert st.tail_tiles == 0 and st.launches == 3
    assert counts(st) == counts(rst) and same_bits(img, ref)
