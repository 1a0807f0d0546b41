"""Multi-rank frame assembly on CPU (gloo, world_size 2): each rank renders its shard of tiles
(here with the CPU oracle -- the GPU path is not available on CPU, the sharding / gather logic
is the same code bench.py runs over RCCL), the frame-end gather brings them to rank 0, and the
assembled frame must equal a single-process render of all tiles."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist

from tests._ranks import file_init_method, spawn_ranks

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, init_method, scene_path, w, h, spp, result_path):
    import sys
    sys.path.insert(0, ROOT)
    import datetime
    dist.init_process_group("gloo", init_method=init_method, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=120))
    import simplepath_amd as sp
    from simplepath_amd import shard
    from tests import _oracle

    scene = sp.Scene.from_file(scene_path)
    scene.set_resolution(w, h)
    n = sp.TileScheduler(w, h).get_num_tiles()
    mine = shard.shard_tiles(n, rank, world)
    local = torch.zeros((shard.per_rank_capacity(n, world), 64, 3), dtype=torch.float32)
    tiles, _ = _oracle.render(scene, 6, spp, mine, threads=2, variant="glibc")
    local[: len(mine)] = torch.from_numpy(tiles)
    frame = shard.gather_frame(local, n, rank, world, dist)
    if rank == 0:
        np.save(result_path, frame.numpy())
    else:
        assert frame is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_gather_frame_matches_single_process(scene_dir, tmp_path, world):
    import simplepath_amd as sp
    from tests import _oracle

    w, h, spp = 40, 24, 2  # 15 tiles: ragged shards for world 2 (8 + 7) and world 3
    path = os.path.join(scene_dir, "bunny.sp")
    out = str(tmp_path / "frame.npy")
    spawn_ranks(_worker, (world, file_init_method(tmp_path), path, w, h, spp, out), world, 270)
    frame = np.load(out)
    scene = sp.Scene.from_file(path)
    scene.set_resolution(w, h)
    ref, _ = _oracle.render(scene, 6, spp, None, threads=4, variant="glibc")
    assert frame.shape == ref.shape
    assert np.array_equal(frame.view(np.uint32), ref.view(np.uint32))


def test_shards_partition_the_frame():
    from simplepath_amd import shard
    for n in (1, 7, 32400):
        for world in (1, 2, 3, 8):
            parts = [shard.shard_tiles(n, r, world) for r in range(world)]
            allt = np.sort(np.concatenate(parts))
            assert np.array_equal(allt, np.arange(n))
            assert max(len(p) for p in parts) == shard.per_rank_capacity(n, world)


def test_bench_launcher_spawns_ranks():
    # `python bench.py --gpus 2` without torchrun: bench.py starts the ranks itself (as child
    # processes, before any GPU call) through torch.distributed.run on 127.0.0.1
    import json
    import subprocess
    import sys

    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-selftest"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line == {"launch_selftest": True, "world": 2, "rank_sum": 1.0}


def test_bench_launch_command():
    sys_path = os.path.join(ROOT, "bench.py")
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", sys_path)
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    cmd = b.launch_command(["--gpus", "8", "--steps", "3"], 8, 29555)
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"]


@pytest.mark.timeout(400)
def test_bench_rank0_reference_work_after_teardown(scene_dir):
    """bench.py --gpus 2 (CPU oracle renders, gloo): rank 0's post-render work -- the reference
    scene build and the parity check of the gathered frame, minutes for lucy -- runs after every
    rank has left the process group.  A stall of 3x the collective timeout must not abort the run
    (before round 3 the other ranks waited in a barrier inside that timeout)."""
    import json
    import subprocess
    import sys

    env = dict(os.environ, SP_BENCH_CPU_RENDER="1", SP_BENCH_POST_STALL_S="15", OMP_NUM_THREADS="2")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--width", "40", "--height", "24", "--spp", "2", "--pg-timeout", "5",
                        "--parity-seconds", "1"],
                       capture_output=True, text=True, timeout=380, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["test_cpu_render"] and line["test_post_stall_s"] == 15.0 and line["world_size"] == 2
    assert sum(x["tiles"] for x in line["ranks"]) == line["config"]["tiles"] == 15
    assert line["imbalance"] >= 1.0 and 0.0 <= line["gather_frac"] < 1.0
    p = line["parity"]
    assert p["frame"] == "gathered" and p["tiles"] > 0 and p["rel_l2"] == 0.0
