"""Multi-rank path on CPU (gloo, world_size 2): the round-robin genome sharding
used by bench.py covers every genome exactly once with no data-path collective,
and the max-over-ranks timing reduction agrees on every rank."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from kf2vecfsw_amd.counter import synth_ids
    g0, gs = bench.shard_ids(n, rank, world)
    ids = synth_ids(n, g0, gs)
    t = torch.tensor([0.5 + rank], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    gathered = [None] * world
    dist.all_gather_object(gathered, ids)
    q.put((rank, ids, float(t), gathered))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_round_robin_shards_cover_all_genomes(world):
    n = 7
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    all_ids = sorted(i for _, ids, _, _ in res for i in ids)
    assert all_ids == list(range(n * world))               # disjoint, complete
    for rank, ids, tmax, gathered in res:
        assert ids == list(range(rank, n * world, world))  # round robin
        assert tmax == 0.5 + (world - 1)                    # max over ranks
