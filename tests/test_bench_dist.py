"""CPU tests of bench.py's multi-GPU plumbing (gloo, world_size 2): the only
collectives (MAX time, SUM frames) and the LPT sharding of config 5."""
import os
import socket
import sys

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        el, fr = bench.reduce_over_ranks(dist, 1.0 + rank, 100 * (rank + 1))
        q.put((rank, el, fr))
    finally:
        dist.destroy_process_group()


def test_reduce_over_ranks_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, el, fr in res:
        assert el == 2.0  # max over ranks
        assert fr == 300  # sum over ranks


def test_reduce_over_ranks_single():
    assert bench.reduce_over_ranks(None, 1.5, 7) == (1.5, 7)


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_shard_lpt_balanced_and_complete(world):
    costs = [((i * 7919) % 97) + 1.0 for i in range(1000)]
    parts = bench.shard_lpt(costs, world)
    assert sorted(i for p in parts for i in p) == list(range(1000))
    loads = [sum(costs[i] for i in p) for p in parts]
    assert max(loads) - min(loads) <= max(costs)


def test_host_cpu_share_slices_affinity():
    # run in a child: the helper pins the calling process when local_world > 1
    import subprocess, sys, os
    code = ("import sys, os; sys.path.insert(0, %r); import bench; "
            "n = len(os.sched_getaffinity(0)); a = bench.host_cpu_share(0, 1); "
            "b = bench.host_cpu_share(1, 2); m = len(os.sched_getaffinity(0)); "
            "print(n, a, b, m)") % os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.check_output([sys.executable, "-c", code], text=True).split()
    n, a, b, m = map(int, out)
    assert a == min(16, n)
    if n >= 2:
        assert b == min(16, n // 2) and m == n // 2
