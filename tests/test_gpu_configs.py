"""GPU parity of the BASELINE.json workloads themselves:

* configs[1] at full size -- 1,000 synthetic 5 Mbp genomes generated in HBM by
  kf_synth_fasta (5.06 GB), counted by the k=7 kernel in one kf_count_batch --
  every genome's 8,192 counts and total bit-exact against the oracle run on the
  same bytes (OpenMP over the host's CPUs), with and without N runs;
* configs[3]'s code path -- bench.py's Workload (round-robin shard plan,
  device-generated sub-batches, resident and streamed modes) in-process at a
  small total, every genome of every sub-batch checked against the oracle --
  and one rank's full share (6,250 x 5 Mbp, 31.6 GB in one launch) at ranks 0
  and 7 of 8.

The reference counts with Jellyfish (kf2vec/main.py:309-323); the oracle is its
restatement pinned by the toy goldens (tests/test_oracle_golden.py)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu

SEED = 20260101


@pytest.fixture(scope="module")
def torch_dev(native):
    import torch
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the gpu tests need an MI355X")
    return torch.device("cuda:0")


def host_threads() -> int:
    sys.path.insert(0, ROOT)
    import bench
    return bench.usable_cpus()[0]


@pytest.mark.parametrize("n_period", [0, 3])
def test_configs1_full_batch_every_genome(torch_dev, oracle, n_period):
    """BASELINE configs[1]: 1,000 x 5 Mbp at k=7, every genome bit-exact (n_period=3:
    N runs of 1-100 bases in about a third of the 4 KiB blocks, which reset k-mers)."""
    import torch
    from kf2vecfsw_amd import counter as C
    n, L, k = 1000, 5_000_000, 7
    db = C.synth_device_batch(n, L, SEED, width=80, n_period=n_period, device=torch_dev)
    kc = C.KmerCounter(k, torch_dev)
    cnt, tot = kc.count(db)
    torch.cuda.synchronize()
    counts, totals = C.counts_to_numpy(cnt), tot.cpu().numpy()
    del cnt, tot
    off = db.off.cpu().numpy().view(np.uint64)
    host = db.data.cpu().numpy()
    del db
    torch.cuda.empty_cache()
    if n_period == 0:
        assert (totals == L - k + 1).all()                          # analytic: no N, one record
    else:
        assert (totals < L - k + 1).all() and (totals > L // 2).all()
    # the device generator writes what the oracle's generator writes (first, last,
    # and genomes around workgroup span boundaries)
    grid = kc.launch_info()[0]
    span = int(off[-1]) // grid
    picks = {0, n - 1} | {int(np.searchsorted(off, b * span, side="right")) - 1 for b in (1, 77, 128, grid - 1)}
    for i in sorted(picks):
        exp = oracle.synth_genome(i, SEED + i, L, 80, n_period, int(off[i + 1] - off[i]))
        assert host[off[i]: off[i + 1]].tobytes() == exp, i
    # every genome against the oracle on the same bytes
    oc, ot = oracle.count_many_parts(host, off, k, 1, host_threads(), 1 << 20)
    assert np.array_equal(ot, totals)
    bad = np.nonzero((oc != counts).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} genomes differ, e.g. {bad[:8].tolist()}"


@pytest.mark.parametrize("resident", [True, False])
@pytest.mark.parametrize("rank,world", [(0, 1), (2, 3)])
def test_configs3_shard_path(torch_dev, oracle, resident, rank, world):
    """bench.py's configs[3] machinery at total=64, sub-batch 16: the shard plan of
    rank `rank` of `world` (ids g % world == rank), sub-batches generated on the
    device, counted resident (one step = every sub-batch) or streamed (each
    sub-batch generated then timed on its own), every genome of every sub-batch
    bit-exact vs the oracle and every total analytic."""
    sys.path.insert(0, ROOT)
    import bench
    args = bench.parse_args(["--workload", "configs3", "--total-genomes", "64", "--sub-batch", "16",
                             "--seq-len", "300000", "--verify", "16"])
    W = bench.Workload(args, torch_dev, rank, world)
    ids = [a + i * st for a, st, c in W.plan for i in range(c)]
    assert ids == list(range(rank, 64, world))
    assert all(c <= 16 for _, _, c in W.plan) and W.nsb == -(-len(ids) // 16)
    m = W.measure(7, 2, 1, resident, picks=16, picks_rest=16)
    assert m["ok"]
    assert len(m["launch_ms"]) == 2 * W.nsb
    assert m["el"] > 0


@pytest.mark.parametrize("rank", [0, 7])
def test_configs3_rank_share_full_size(torch_dev, oracle, rank):
    """BASELINE configs[3] at its per-GPU size: rank `rank` of
    the 8-GPU run owns the 6,250 genome ids g < 50,000 with g mod 8 == rank
    (6,250 x 5 Mbp = 31.6 GB), generated on the device by bench.py's own Workload
    and counted at k=7 in ONE kf_count_batch, exactly the launch each rank times.
    Every total is analytic and every genome's row bit-exact against the oracle
    on the same bytes, copied back in host chunks of 500 genomes (the host never
    holds the whole batch).  Reference: the per-file loop this shards,
    kf2vec/main.py:301-357."""
    import torch
    sys.path.insert(0, ROOT)
    import bench
    from kf2vecfsw_amd import counter as C
    args = bench.parse_args(["--workload", "configs3"])
    W = bench.Workload(args, torch_dev, rank, 8)
    assert W.nsb == 1 and W.n == 6250 and W.plan == [(rank, 8, 6250)]
    assert W.fits(7)
    db = W.gen(0)
    L, k = args.seq_len, 7
    assert db.n == 6250 and db.data.numel() > 31.6e9
    kc = C.KmerCounter(k, torch_dev)
    cnt, tot = kc.count(db)
    torch.cuda.synchronize()
    totals = tot.cpu().numpy()
    assert (totals == L - k + 1).all()
    off = db.off.cpu().numpy().view(np.uint64)
    threads = host_threads()
    step = 500
    for g0 in range(0, db.n, step):
        g1 = min(db.n, g0 + step)
        host = db.data[int(off[g0]): int(off[g1])].cpu().numpy()
        if g0 == 0 or g1 == db.n:   # the generator's bytes are the oracle generator's (ids rank + 8 i)
            for i in (g0, g1 - 1):
                g = rank + 8 * i
                exp = oracle.synth_genome(g, SEED + g, L, 80, 0, int(off[i + 1] - off[i]))
                assert host[int(off[i] - off[g0]): int(off[i + 1] - off[g0])].tobytes() == exp, i
        oc, ot = oracle.count_many_parts(host, off[g0: g1 + 1] - off[g0], k, 1, threads, 1 << 20)
        assert np.array_equal(ot, totals[g0:g1]), g0
        got = C.counts_to_numpy(cnt[g0:g1])
        bad = np.nonzero((oc != got).any(axis=1))[0]
        assert bad.size == 0, f"rank {rank}: {bad.size} genomes differ, e.g. {(bad[:8] + g0).tolist()}"
        del host, oc, got
    del cnt, tot, db
    torch.cuda.empty_cache()


@pytest.mark.parametrize("n_period", [0, 3])
def test_configs4_full_batch_every_genome(torch_dev, oracle, n_period):
    """BASELINE configs[4]: k=11 (4^11 codes, 2,098,176 columns: the bucket kernel,
    bins far beyond the LDS) over the same 1,000 x 5 Mbp device-generated batch as
    the bench, every genome's row and total bit-exact against the oracle
    (kf2vec/main.py:291-296 is the reference's large-k vocab branch; the counts
    are Jellyfish's, main.py:309-323).  The rows are compared 100 genomes at a
    time so the host holds ~1 GB of each side at once."""
    import torch
    from kf2vecfsw_amd import counter as C
    n, L, k = 1000, 5_000_000, 11
    db = C.synth_device_batch(n, L, SEED, width=80, n_period=n_period, device=torch_dev)
    kc = C.KmerCounter(k, torch_dev)
    cnt, tot = kc.count(db)
    torch.cuda.synchronize()
    totals = tot.cpu().numpy()
    off = db.off.cpu().numpy().view(np.uint64)
    host = db.data.cpu().numpy()
    del db
    if n_period == 0:
        assert (totals == L - k + 1).all()
    else:
        assert (totals < L - k + 1).all() and (totals > L // 2).all()
    threads = host_threads()
    step = 100
    for g0 in range(0, n, step):
        g1 = min(n, g0 + step)
        sub = off[g0: g1 + 1] - off[g0]
        oc, ot = oracle.count_many_parts(host[int(off[g0]): int(off[g1])], sub, k, 1, threads, 4 << 20)
        assert np.array_equal(ot, totals[g0:g1]), g0
        got = C.counts_to_numpy(cnt[g0:g1])
        bad = np.nonzero((oc != got).any(axis=1))[0]
        assert bad.size == 0, f"k=11: {bad.size} genomes differ, e.g. {(bad[:8] + g0).tolist()}"
        del oc, got
    del cnt, tot
    torch.cuda.empty_cache()


@pytest.mark.parametrize("k", [16, 31])
def test_sparse_bench_size_every_genome(torch_dev, oracle, k):
    """bench.py's `sparse` workload at its own size: 64 x 5 Mbp device-generated
    genomes (324 M keys), every genome's present canonical k-mers and counts
    bit-exact against the oracle's sort-based restatement (OpenMP over genomes);
    k=16 is the u32-key path, k=31 the u64 one (get_kmers, kf2vec/main.py:133-172)."""
    import torch
    from kf2vecfsw_amd import counter as C
    n, L = 64, 5_000_000
    db = C.synth_device_batch(n, L, SEED, width=80, device=torch_dev)
    off = C.synth_layout(n, L)
    sc = C.SparseCounter(k, torch_dev)
    keys, cnts, nu = sc.count(db, int(off[-1]))
    torch.cuda.synchronize()
    gk = keys.cpu().numpy().view(np.uint64)
    gc = cnts.cpu().numpy().view(np.uint32)
    gn = nu.cpu().numpy().view(np.uint64)
    host = db.data.cpu().numpy()
    del keys, cnts, nu, db, sc
    torch.cuda.empty_cache()
    ek, ec, en = oracle.sparse_count_many(host[: int(off[-1])], off, k, 1, host_threads())
    assert np.array_equal(gn, en)
    for g in range(n):
        a, m = int(off[g]), int(en[g])
        assert np.array_equal(gk[a: a + m], ek[a: a + m]), (k, g)
        assert np.array_equal(gc[a: a + m], ec[a: a + m]), (k, g)
        assert int(ec[a: a + m].sum(dtype=np.uint64)) == L - k + 1


@pytest.mark.parametrize("k", [16, 31])
def test_sparse_many_big_buckets_every_genome(torch_dev, oracle, k):
    """Genomes long enough that their low buckets (canonical keys skew low: the
    minimum of a code and its reverse complement) exceed a chunk: 6 x 24 Mbp, so
    hundreds of big buckets go through the overflow sort beside ordinary chunks
    in one call. Every genome bit-exact against the oracle (get_kmers,
    kf2vec/main.py:133-172)."""
    import torch
    from kf2vecfsw_amd import counter as C
    n, L = 6, 24_000_000
    db = C.synth_device_batch(n, L, SEED + 7, width=80, device=torch_dev)
    off = C.synth_layout(n, L)
    sc = C.SparseCounter(k, torch_dev)
    keys, cnts, nu = sc.count(db, int(off[-1]))
    torch.cuda.synchronize()
    gk = keys.cpu().numpy().view(np.uint64)
    gc = cnts.cpu().numpy().view(np.uint32)
    gn = nu.cpu().numpy().view(np.uint64)
    host = db.data.cpu().numpy()
    del keys, cnts, nu, db, sc
    torch.cuda.empty_cache()
    ek, ec, en = oracle.sparse_count_many(host[: int(off[-1])], off, k, 1, host_threads())
    assert np.array_equal(gn, en), (gn[:4], en[:4])
    for g in range(n):
        a, m = int(off[g]), int(en[g])
        assert np.array_equal(gk[a: a + m], ek[a: a + m]), (k, g)
        assert np.array_equal(gc[a: a + m], ec[a: a + m]), (k, g)
        assert int(ec[a: a + m].sum(dtype=np.uint64)) == L - k + 1
