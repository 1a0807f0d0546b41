"""The bench's N>1 flow with real device renders: two rank processes share one GPU (the
collective runs over gloo on host copies; on a node each rank owns a GPU and bench.py gathers
over RCCL with the same shard.gather_frame), each renders its interleaved shard with the HIP
path, and the frame assembled on rank 0 must equal one process rendering every tile, bit for
bit.  Shards this small run on the sample-chunk pipeline (AUTO below 24000 tiles), the full
frame here on the wavefront, so this also checks that the two agree through the multi-rank path."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist

from tests._ranks import file_init_method, spawn_ranks

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, init_method, scene_path, w, h, spp, result_path):
    import datetime
    import sys

    sys.path.insert(0, ROOT)
    dist.init_process_group("gloo", init_method=init_method, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=120))
    import simplepath_amd as sp
    from simplepath_amd import shard

    scene = sp.Scene.from_file(scene_path)
    scene.set_resolution(w, h)
    scene.upload(device=0, bvh_mode=0)
    n = sp.TileScheduler(w, h).get_num_tiles()
    mine = shard.shard_tiles(n, rank, world)
    tiles, st = sp.render_tiles(scene, "direct_lighting", spp, mine)
    assert st.pipeline == 3  # AUTO: sample chunks for a shard this small
    local = torch.zeros((shard.per_rank_capacity(n, world), 64, 3), dtype=torch.float32)
    local[: len(mine)] = torch.from_numpy(tiles)
    frame = shard.gather_frame(local, n, rank, world, dist)
    if rank == 0:
        np.save(result_path, frame.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_ranks_on_device_match_single_process(scene_dir, tmp_path):
    import simplepath_amd as sp

    w, h, spp, world = 200, 120, 2, 2  # 375 tiles: ragged shards (188 + 187)
    path = os.path.join(scene_dir, "bunny.sp")
    out = str(tmp_path / "frame.npy")
    spawn_ranks(_worker, (world, file_init_method(tmp_path), path, w, h, spp, out), world, 270)
    frame = np.load(out)
    scene = sp.Scene.from_file(path)
    scene.set_resolution(w, h)
    scene.upload(device=0, bvh_mode=0)
    ref, st = sp.render_tiles(scene, "direct_lighting", spp, pipeline="wavefront")
    assert st.pipeline == 2
    assert frame.shape == ref.shape
    assert np.array_equal(frame.view(np.uint32), ref.view(np.uint32))


def _nccl_worker(rank, world, init_method, result_path):
    """Renders its shard on device `rank`, gathers the CUDA tile buffers over RCCL."""
    import datetime
    import sys

    sys.path.insert(0, ROOT)
    torch.cuda.set_device(rank)
    dist.init_process_group("nccl", init_method=init_method, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=120),
                            device_id=torch.device(f"cuda:{rank}"))
    from simplepath_amd import shard

    n = 45
    mine = shard.shard_tiles(n, rank, world)
    local = torch.full((shard.per_rank_capacity(n, world), 64, 3), -1.0, dtype=torch.float32, device=f"cuda:{rank}")
    # tile t holds the value t in every lane: the assembled frame must be tile-ordered
    local[: len(mine)] = torch.from_numpy(mine.astype(np.float32)).to(f"cuda:{rank}")[:, None, None]
    frame = shard.gather_frame(local, n, rank, world, dist, collective=True)
    if rank == 0:
        assert frame.is_cuda
        np.save(result_path, frame.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(180)
@pytest.mark.parametrize("world", [1, 2])
def test_rccl_gather_frame_on_device(tmp_path, world):
    # the frame-end collective bench.py times: dist.gather of CUDA tensors over nccl (= RCCL);
    # world 1 runs the same collective through a one-rank group, world 2 needs two GPUs
    if torch.cuda.device_count() < world:
        pytest.skip(f"needs {world} GPUs")
    out = str(tmp_path / "frame.npy")
    spawn_ranks(_nccl_worker, (world, file_init_method(tmp_path), out), world, 150)
    frame = np.load(out)
    assert frame.shape == (45, 64, 3)
    assert np.array_equal(frame, np.broadcast_to(np.arange(45, dtype=np.float32)[:, None, None], frame.shape))
