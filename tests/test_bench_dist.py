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
        bad = bench.sum_over_ranks(dist, rank + 1)
        q.put((rank, el, fr, bad))
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
    for rank, el, fr, bad in res:
        assert el == 2.0  # max over ranks
        assert fr == 300  # sum over ranks
        assert bad == 3  # output-check counters summed over ranks


def test_reduce_over_ranks_single():
    assert bench.reduce_over_ranks(None, 1.5, 7) == (1.5, 7)


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_shard_lpt_balanced_and_complete(world):
    costs = [((i * 7919) % 97) + 1.0 for i in range(1000)]
    parts = bench.shard_lpt(costs, world)
    assert sorted(i for p in parts for i in p) == list(range(1000))
    loads = [sum(costs[i] for i in p) for p in parts]
    assert max(loads) - min(loads) <= max(costs)


def _mixed_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # configs[4]: 65,536 stills over `world` GPUs, per-GPU --frames = 65536 / world
        mine, items = bench.rank_batch("mixed", 65536 // world, world, rank)
        shards = [None] * world
        dist.all_gather_object(shards, mine)
        cost = sum(len(items[i][0]) + 0.02 * items[i][2] for i in mine)
        el, fr = bench.reduce_over_ranks(dist, 10.0 + rank, len(mine))
        q.put((rank, shards, len(items), cost, el, fr))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_mixed_configs4_flow_gloo(world):
    """bench.py's configs[4] flow over the full 65,536-item list: every rank builds the same
    global list, the LPT shards are disjoint and complete, the frame SUM and time MAX are right."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mixed_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=300) for _ in procs), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    shards = res[0][1]
    assert all(r[1] == shards for r in res)  # every rank computed the same partition
    flat = [i for sh in shards for i in sh]
    assert len(flat) == 65536 and sorted(flat) == list(range(65536))
    for rank, sh, total, cost, el, fr in res:
        assert total == 65536
        assert sh[rank] == shards[rank]
        assert el == 10.0 + world - 1  # max over ranks
        assert fr == 65536  # sum over ranks
    costs = [r[3] for r in res]
    assert max(costs) - min(costs) <= 0.01 * max(costs)  # LPT: balanced shards


def test_verify_outputs_against_manifest():
    """bench.py's post-timing output check: every committed bench stream is in the manifest, the
    oracle's own JPEG passes, a flipped byte and an unknown stream are counted."""
    import glob
    import hashlib
    import json
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import oracle_py as O
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    man = json.load(open(os.path.join(root, "tests", "golden", "bench_manifest.json")))
    for wl in bench.WORKLOADS.values():
        if wl["streams"]:
            for f in glob.glob(os.path.join(root, wl["streams"])):
                assert hashlib.md5(open(f, "rb").read()).hexdigest() in man, f
    for pat, *_ in bench.MIXED_SETS.values():
        for f in glob.glob(os.path.join(root, pat)):
            assert hashlib.md5(open(f, "rb").read()).hexdigest() in man, f
    s = open(os.path.join(root, "tests", "golden", "bench264", "avc1080_00.h264"), "rb").read()
    j = O.transcode(s)
    batch = [s, s, b"unknown"]
    out = bytearray(j + j + j)
    offs, lens = [0, len(j), 2 * len(j)], [len(j)] * 3
    assert bench.verify_outputs(batch, out, offs, lens, man) == (3, 0, 1)
    out[len(j) + 100] ^= 1
    assert bench.verify_outputs(batch, out, offs, lens, man) == (3, 1, 1)
