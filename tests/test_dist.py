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


def _plan_worker(rank, world, port, total, per, q):
    """One rank of bench.py's configs[3] run: its sub-batch plan, the ids it would
    generate, and the all-gathered plans of every rank."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    plan = bench.shard_plan(total, rank, world, per)
    mine = sorted(a + i * st for a, st, c in plan for i in range(c))
    n_sb = torch.tensor([float(len(plan))])
    dist.all_reduce(n_sb, op=dist.ReduceOp.MAX)
    counts = [None] * world
    dist.all_gather_object(counts, [c for _, _, c in plan])
    q.put((rank, mine, len(plan), float(n_sb), counts))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_configs3_50k_shards_disjoint_and_complete(world):
    """bench.py's N>1 workload (BASELINE configs[3]): the 50,000 genome ids are
    split round-robin (genome g on rank g mod N) into per-rank sub-batches of at
    most 6,250; over the ranks of a gloo group the ids are disjoint and complete,
    each rank's are exactly g % N == r, and every rank has the same number of
    sub-batches (the streamed mode's barriers line up)."""
    import bench
    total, per = bench.CONFIG3_GENOMES, bench.SUB_BATCH
    if world == 1:
        plan = bench.shard_plan(total, 0, 1, per)
        ids = [a + i * st for a, st, c in plan for i in range(c)]
        assert ids == list(range(total)) and len(plan) == 8 and all(c <= per for _, _, c in plan)
        return
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_plan_worker, args=(r, world, port, total, per, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    all_ids = [i for _, mine, _, _, _ in res for i in mine]
    assert len(all_ids) == total and sorted(all_ids) == list(range(total))
    for rank, mine, nsb, nsb_max, counts in res:
        assert mine == list(range(rank, total, world))
        assert nsb == nsb_max == -(-(total // world) // per)
        assert all(c <= per for row in counts for c in row)


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


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_cli_file_shards_balanced_and_grouped(world):
    """get_frequencies -gpus N / torchrun: every file in exactly one shard, files of
    one sample name together (last-file-wins stays inside a shard), shards in input
    order, and byte loads within one largest group of each other."""
    import numpy as np
    from kf2vecfsw_amd.main import shard_files
    rng = np.random.default_rng(world)
    sizes = [int(x) for x in rng.integers(1, 10_000_000, size=97)]
    samples = [f"s{int(i)}" for i in rng.integers(0, 80, size=97)]
    shards = shard_files(sizes, samples, world)
    assert len(shards) == world
    assert sorted(i for sh in shards for i in sh) == list(range(97))
    for sh in shards:
        assert sh == sorted(sh)
    owner = {}
    for r, sh in enumerate(shards):
        for i in sh:
            assert owner.setdefault(samples[i], r) == r
    loads = [sum(sizes[i] for i in sh) for sh in shards]
    biggest = max(sum(sizes[i] for i in range(97) if samples[i] == s) for s in set(samples))
    assert max(loads) - min(loads) <= biggest


def test_cli_shard_spec_from_env(monkeypatch):
    from types import SimpleNamespace
    from kf2vecfsw_amd.main import _shard_spec, build_parser
    a = build_parser().parse_args(["get_frequencies", "-input_dir", "i", "-output_dir", "o", "-gpus", "4"])
    assert a.gpus == 4
    monkeypatch.delenv("KF_SHARD", raising=False)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert _shard_spec(SimpleNamespace(gpus=1)) is None
    monkeypatch.setenv("WORLD_SIZE", "4")
    monkeypatch.setenv("RANK", "2")
    assert _shard_spec(SimpleNamespace(gpus=1)) == (2, 4)       # a torchrun rank
    assert _shard_spec(SimpleNamespace(gpus=4)) is None         # -gpus spawns its own children
    monkeypatch.setenv("KF_SHARD", "3,8")
    assert _shard_spec(SimpleNamespace(gpus=1)) == (3, 8)       # a -gpus child


def test_cli_gpus_validation(monkeypatch, tmp_path):
    """-gpus N under torchrun is refused (every rank would count everything); -gpus
    larger than the visible GPUs is refused; visible_gpus reads the env masks
    without initialising HIP."""
    from kf2vecfsw_amd import main as M
    monkeypatch.delenv("KF_SHARD", raising=False)
    monkeypatch.delenv("KF_SHARD_DEVICE", raising=False)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1")
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES", raising=False)
    n = M.visible_gpus()
    assert n <= 2
    a = M.build_parser().parse_args(["get_frequencies", "-input_dir", str(tmp_path), "-output_dir", str(tmp_path),
                                     "-gpus", "4"])
    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(ValueError, match="torchrun"):
        M.get_frequencies(a)
    monkeypatch.setenv("WORLD_SIZE", "1")
    with pytest.raises(ValueError, match="visible"):
        M.get_frequencies(a)
    # HIP's mask applies on top of ROCR's: the smallest of the set masks wins
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "0,1,2,3")
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0")
    assert M.visible_gpus() <= 1
    # no mask and no readable KFD topology: unknown, not 0 (no check then)
    for v in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    if not os.path.isdir("/sys/class/kfd/kfd/topology/nodes"):
        assert M.visible_gpus() is None
