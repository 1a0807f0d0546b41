"""bench.py's N>1 flow on one GPU: `python bench.py --gpus 2` starts its two ranks itself
(torch.distributed.run as a child process), each renders its interleaved shard on the device,
rank 0 gathers the frame and checks a sample of the GATHERED tiles against the reference build.
SP_BENCH_SHARED_DEVICE=1 puts both ranks on cuda:0 and their collectives on gloo (RCCL needs one
GPU per rank); everything else is the code the driver's multi-GPU run executes."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(400)
def test_bench_two_ranks_gathered_frame():
    env = dict(os.environ, SP_BENCH_SHARED_DEVICE="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--width", "256", "--height", "160", "--spp", "4", "--parity-seconds", "2"],
                       capture_output=True, text=True, timeout=380, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["world_size"] == 2 and line["test_shared_device"]
    assert sorted(x["rank"] for x in line["ranks"]) == [0, 1]
    assert sum(x["tiles"] for x in line["ranks"]) == line["config"]["tiles"] == 32 * 20
    p = line["parity"]
    assert p["frame"] == "gathered" and p["tiles"] > 0
    assert p["rel_l2"] < 1e-4 and p["bitexact_pixel_frac"] >= 0.999
    assert line["cpu_baseline"] is None  # timed at N=1 only


@pytest.mark.timeout(600)
def test_bench_eight_ranks_ragged_shards():
    # the driver's 8-GPU launch shape rehearsed on one device: `bench.py --gpus 8` starts 8 ranks,
    # each renders its interleaved shard (33 x 17 = 561 tiles: ragged, 71 or 70 per rank; AUTO
    # picks the sample chunks for such shards), rank 0 gathers and checks the GATHERED frame;
    # the N > 1 line reports per-rank tiles and render times, imbalance and the gather's share
    env = dict(os.environ, SP_BENCH_SHARED_DEVICE="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "2", "--warmup", "1",
                        "--width", "260", "--height", "130", "--spp", "8", "--parity-seconds", "3"],
                       capture_output=True, text=True, timeout=580, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 8 and line["world_size"] == 8 and line["test_shared_device"]
    ranks = sorted(line["ranks"], key=lambda x: x["rank"])
    assert [x["rank"] for x in ranks] == list(range(8))
    tiles = [x["tiles"] for x in ranks]
    assert sum(tiles) == line["config"]["tiles"] == 33 * 17 and max(tiles) - min(tiles) == 1
    assert all(x["render_ms"] > 0 for x in ranks)
    assert line["imbalance"] >= 1.0 and 0.0 <= line["gather_frac"] < 1.0
    assert line["config"]["pipeline"] == "chunks"
    p = line["parity"]
    assert p["frame"] == "gathered" and p["tiles"] > 0
    assert p["rel_l2"] < 1e-4 and p["bitexact_pixel_frac"] >= 0.999
