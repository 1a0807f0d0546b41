"""Rank processes for the multi-rank tests, with a deadline and no port race.

The ranks rendezvous through a FileStore in the test's tmp dir (`file://` init method) instead of
a TCP port picked by bind-then-release, which another process can take in between.  The parent
joins with a deadline: a rank stuck in a collective is killed and the test fails with a
TimeoutError naming the ranks still alive, instead of holding the whole suite."""
import os
import time

import torch.multiprocessing as mp


def file_init_method(tmp_path, name="rdzv"):
    path = os.path.join(str(tmp_path), name)
    if os.path.exists(path):
        os.remove(path)
    return "file://" + path


def spawn_ranks(fn, args, nprocs, timeout_s):
    ctx = mp.start_processes(fn, args=args, nprocs=nprocs, join=False, start_method="spawn")
    deadline = time.monotonic() + timeout_s
    while not ctx.join(timeout=2.0):  # raises ProcessRaisedException / ProcessExitedException
        if time.monotonic() > deadline:
            alive = [r for r, p in enumerate(ctx.processes) if p.is_alive()]
            for p in ctx.processes:
                if p.is_alive():
                    p.kill()
            for p in ctx.processes:
                p.join(10)
            raise TimeoutError(f"ranks {alive} still running after {timeout_s} s")
