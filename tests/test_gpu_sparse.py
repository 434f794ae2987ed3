"""GPU parity of the sparse counter (kf_sparse_count: get_kmers at k = 2..31,
reference kf2vec/main.py:112-176) against the oracle's sort-based restatement
(oracle/kmer_oracle.c oracle_sparse_count) and against the dense counter where
both exist (k <= 12).  Keys and counts must be bit-exact."""
import numpy as np
import pytest

import gen

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev(native):
    import torch
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible: the gpu tests need an MI355X")
    return torch.device("cuda:0")


_sparse = {}


def sparse_counter(k, dev):
    from kf2vecfsw_amd.counter import SparseCounter
    if k not in _sparse:
        _sparse[k] = SparseCounter(k, dev)
    return _sparse[k]


def run_sparse(blobs, k, dev, fmt=0):
    import torch
    from kf2vecfsw_amd import counter as C
    hb = C.pack_genomes(blobs, fmt=fmt)
    sc = sparse_counter(k, dev)
    keys, cnts, nu = sc.count(C.to_device(hb, dev), int(hb.off[-1]))
    torch.cuda.synchronize()
    return sc.to_host(keys, cnts, nu, hb.off)


def check(oracle, blobs, k, got, fmt=0, tag=""):
    for i, b in enumerate(blobs):
        ek, ec = oracle.sparse_count(b, k, fmt)
        gk, gc = got[i]
        assert gk.size == ek.size, (tag, i, k, gk.size, ek.size)
        if not (np.array_equal(gk, ek) and np.array_equal(gc, ec)):
            bad = np.nonzero((gk != ek) | (gc != ec))[0][:5]
            pytest.fail(f"{tag} genome {i} k={k}: {bad.size}+ rows differ, first {bad.tolist()}: "
                        f"got {gk[bad].tolist()}/{gc[bad].tolist()} want {ek[bad].tolist()}/{ec[bad].tolist()}")


@pytest.mark.parametrize("k", [2, 3, 5, 8, 12, 13, 15, 16, 17, 21, 25, 31])
def test_sparse_random_fasta_vs_oracle(torch_dev, oracle, k):
    """Multi-record FASTA with N runs, IUPAC, lowercase, CRLF, blank lines,
    1-column lines; plus an empty genome, a header-only one and one shorter than k."""
    rng = np.random.default_rng(1000 + k)
    blobs = [gen.random_fasta(rng, int(rng.integers(0, 30000)), n_rate=0.02, iupac_rate=0.002, lower=0.1,
                              crlf_rate=0.2, poly_rate=0.5) for _ in range(6)]
    blobs += [b"", b">only a header\n", b">s\nACG\n", b"ACGTTGCA" * 5]
    check(oracle, blobs, k, run_sparse(blobs, k, torch_dev), tag="random")


@pytest.mark.parametrize("k", [13, 31])
def test_sparse_fastq(torch_dev, oracle, k):
    rng = np.random.default_rng(77 + k)
    blobs = [gen.random_fastq(rng, 150, n_rate=0.01, multiline=bool(i % 2)) for i in range(3)]
    check(oracle, blobs, k, run_sparse(blobs, k, torch_dev, fmt=2), fmt=2, tag="fastq")


@pytest.mark.parametrize("k", [3, 7, 9, 11, 12])
def test_sparse_equals_dense_rows(torch_dev, k):
    """k <= 12: the sparse counter's keys are exactly the dense counter's non-zero
    bins (same lexicographic order), with the same counts."""
    import torch
    from kf2vecfsw_amd import counter as C
    rng = np.random.default_rng(5 + k)
    blobs = [gen.random_fasta(rng, int(rng.integers(1000, 200000)), n_rate=0.01, lower=0.05) for _ in range(5)]
    got = run_sparse(blobs, k, torch_dev)
    kc = C.KmerCounter(k, torch_dev)
    dense, _ = kc.count(C.to_device(C.pack_genomes(blobs), torch_dev))
    torch.cuda.synchronize()
    dense = C.counts_to_numpy(dense)
    _, col2rep = C.tables(k)
    # col2rep is the kf code (A0 C1 T2 G3) of each column's canonical k-mer; map to standard codes
    kf2std = np.array([0, 1, 3, 2], np.uint64)
    rep = col2rep.astype(np.uint64)
    std = np.zeros_like(rep)
    rc = np.zeros_like(rep)
    for i in range(k):
        d = kf2std[((rep >> np.uint64(2 * i)) & np.uint64(3)).astype(np.intp)]
        std |= d << np.uint64(2 * i)
        rc |= (np.uint64(3) - d) << np.uint64(2 * (k - 1 - i))
    std = np.minimum(std, rc)   # the class's lexicographically smaller member
    for i in range(len(blobs)):
        nz = np.nonzero(dense[i])[0]
        assert np.array_equal(got[i][0], std[nz]), i
        assert np.array_equal(got[i][1], dense[i][nz]), i


def test_sparse_tile_boundaries_and_many_genomes(torch_dev, oracle):
    """Genome lengths around the tiles (8,192 slots for u64 keys, 16,384 for u32;
    the lengths around round 4's 4,096 / 8,192 tiles stay in the list) and 300
    small genomes in one batch (many tiles, many look-back chains)."""
    rng = np.random.default_rng(9)
    blobs = []
    for L in [1, 2046, 2047, 2048, 2049, 4095, 4096, 4097, 6143, 6145, 8191, 8192, 8193, 12289, 16383, 16385]:
        s = gen.random_seq(rng, L).tobytes()
        blobs.append(s[:L])
    blobs += [gen.random_fasta(rng, int(rng.integers(0, 3000))) for _ in range(300)]
    for k in (13, 31):
        check(oracle, blobs, k, run_sparse(blobs, k, torch_dev), tag=f"tiles k={k}")


def test_sparse_ragged_tile_counts_interleaved_order(torch_dev, oracle):
    """Genomes of 0 to ~60 tiles next to each other: the single-sweep passes
    ticket tiles in (index in genome, genome) order, so short genomes drop out
    of the rotation while long ones go on; one genome alone (no reordering)."""
    rng = np.random.default_rng(77)
    sizes = [0, 250_000, 1, 3000, 120_000, 0, 9000, 500_000, 17, 40_000]
    blobs = [gen.random_seq(rng, L).tobytes()[:L] if L else b"" for L in sizes]
    for k in (16, 31):
        check(oracle, blobs, k, run_sparse(blobs, k, torch_dev), tag=f"ragged k={k}")
        check(oracle, blobs[7:8], k, run_sparse(blobs[7:8], k, torch_dev), tag=f"single k={k}")


def test_sparse_more_genomes_than_the_order_table(torch_dev, oracle):
    """5,000 genomes in one batch (past KF_SPARSE_ORDER_MAXN = 4,096: tiles run
    in plain order)."""
    rng = np.random.default_rng(78)
    blobs = [gen.random_seq(rng, int(L)).tobytes()[: int(L)] for L in rng.integers(0, 400, 5000)]
    check(oracle, blobs, 21, run_sparse(blobs, 21, torch_dev), tag="n5000")


def test_sparse_low_complexity_runs(torch_dev, oracle):
    """One key for a whole genome (poly-A: a single run of ~1M), two-key genomes,
    and dinucleotide repeats: a run crossing hundreds of tiles."""
    blobs = [b">a\n" + b"A" * 1000000 + b"\n", b"ACACACACAC" * 50000, b"TTTTTTTTTTTTTTTTTTTTTTTTT\n" * 4000,
             b">x\n" + b"ACGT" * 100000]
    for k in (13, 16, 17, 31):
        check(oracle, blobs, k, run_sparse(blobs, k, torch_dev), tag=f"lowcx k={k}")


def test_sparse_newline_runs_and_breaks(torch_dev, oracle):
    """Long runs of blank lines between bases (windows span them), and '\\r' / N
    breaks right at a thread's 8-byte boundary."""
    blobs = [b">a\n" + b"ACGTACGTACGTAC" + b"\n" * 100000 + b"GTACGTTGCAACGT\n",
             b"ACGTACG\nTACGTACGTAC\r\nGTACGTACGTACG\n" * 500,
             (b"ACGTACGN" * 3000), b"\n" * 5000]
    for k in (13, 20):
        check(oracle, blobs, k, run_sparse(blobs, k, torch_dev), tag=f"nl k={k}")


def test_sparse_large_genomes_k31(torch_dev, oracle):
    """Two 5 Mbp device-synthesised genomes (BASELINE configs[1] genome size) at
    k = 31 and 21 against the oracle."""
    import torch
    from kf2vecfsw_amd import counter as C
    db = C.synth_device_batch(2, 5_000_000, 4242, device=torch_dev)
    off = C.synth_layout(2, 5_000_000)
    host = db.data.cpu().numpy()
    for k in (21, 31):
        sc = sparse_counter(k, torch_dev)
        keys, cnts, nu = sc.count(db, int(off[-1]))
        torch.cuda.synchronize()
        got = sc.to_host(keys, cnts, nu, off)
        blobs = [host[int(off[i]): int(off[i + 1])].tobytes() for i in range(2)]
        check(oracle, blobs, k, got, tag=f"synth k={k}")
        # every window of a 5 Mbp N-free genome is counted
        assert int(got[0][1].sum(dtype=np.uint64)) == 5_000_000 - k + 1


@pytest.mark.parametrize("k", [13, 21, 31])
def test_cli_get_kmers_large_k_vs_oracle(torch_dev, toy, oracle, tmp_path, k):
    """`get_kmers -k 13..31` .npy == main.py:147-172 restated on the oracle's
    present k-mers (rows in lexicographic order)."""
    from kf2vecfsw_amd import main as M
    inp, out = tmp_path / "in", tmp_path / "out"
    inp.mkdir()
    small = [t for t in toy if len(t[2]) < 1_000_000]   # the Python restatement is per character
    for name, sample, data, exp in small:
        (inp / name).write_bytes(data)
    M.main(["get_kmers", "-input_dir", str(inp), "-output_dir", str(out), "-k", str(k)])
    for name, sample, data, exp in small:
        m = np.load(out / f"{sample}_k{k}.npy")
        keys, cnts = oracle.sparse_count(data, k)
        ref = oracle.kmers_matrix_from_dump(list(zip(oracle.std_code_text(keys, k), cnts.tolist())), k)
        assert m.dtype == np.float32 and m.shape == (keys.size, k + 1), sample
        assert np.array_equal(m, ref), sample


def test_sparse_rejects_bad_offsets(torch_dev):
    """Offsets past batch_bytes or decreasing: nothing is written, every genome's
    count comes back as UINT64_MAX and SparseCounter.to_host raises."""
    import torch
    from kf2vecfsw_amd import _native as N
    from kf2vecfsw_amd import counter as C
    hb = C.pack_genomes([b">a\nACGTACGTACGTACGT\n", b">b\nGGGGCCCCAAAATTTT\n"])
    db = C.to_device(hb, torch_dev)
    sc = sparse_counter(13, torch_dev)
    keys, cnts, nu = sc.count(db, int(hb.off[-1]) - 16)      # offsets end past batch_bytes
    torch.cuda.synchronize()
    assert (nu.cpu().numpy() == -1).all()
    with pytest.raises(N.NativeError):
        sc.to_host(keys, cnts, nu, hb.off)
    bad = db.off.clone()
    bad[1] = bad[2] + 16                                       # decreasing
    db2 = C.DeviceBatch(db.data, bad, db.excl, db.n, db.n_excl)
    keys, cnts, nu = sc.count(db2, int(hb.off[-1]) + 64)
    torch.cuda.synchronize()
    assert (nu.cpu().numpy() == -1).all()


def _combine(terms):
    """sum of coef x (keys, counts) sparse vectors -> sorted keys, int64 counts (zeros dropped)."""
    keys = np.unique(np.concatenate([t[1] for t in terms]))
    acc = np.zeros(keys.size, np.int64)
    for coef, k_, c_ in terms:
        acc[np.searchsorted(keys, k_)] += coef * c_.astype(np.int64)
    nz = acc != 0
    return keys[nz], acc[nz]


def test_get_kmers_5gib_file_in_pieces(torch_dev, oracle, tmp_path):
    """get_kmers -k 21 on ONE ~5 GiB FASTA (a 4.7 Gbp record,
    far past the sparse counter's 4 GiB per call, then a 0.3 Gbp record): the file
    is counted in 1 GiB pieces with a (k-1)-position overlap (main.fasta_pieces)
    and the pieces' sorted results merged on the device.  The records repeat two
    random 3 Mbp segments, so the expected counts follow from the oracle on short
    strings: record 1 = (AB)^m -> m cnt(AB) + (m-1) J(BA), J(BA) = cnt(ABA) -
    cnt(AB) - cnt(A); record 2 = A^n -> n cnt(A) + (n-1) (cnt(AA) - 2 cnt(A)).
    The .npy must equal main.py:147-176 applied to those counts, bit for bit,
    and the counts sum to the analytic window total.  The reference's Jellyfish
    takes any file size (kf2vec/main.py:133-145)."""
    import os
    import shutil
    from kf2vecfsw_amd import main as M
    k, W = 21, 80
    rng = np.random.default_rng(5150)
    A, B = gen.random_seq(rng, 3_000_000), gen.random_seq(rng, 3_000_000)
    m1, m2 = 780, 100
    base = "/dev/shm" if os.access("/dev/shm", os.W_OK) else str(tmp_path)
    work = os.path.join(base, f"kf_5gib_{os.getpid()}")
    os.makedirs(os.path.join(work, "in"))
    try:
        path = os.path.join(work, "in", "big.fna")
        ab, a = gen.wrap(np.concatenate([A, B]), W), gen.wrap(A, W)   # 6 Mbp and 3 Mbp: whole lines
        with open(path, "wb") as f:
            f.write(b">r1 (AB)^780\n")
            for _ in range(m1):
                f.write(ab)
            f.write(b">r2 A^100\n")
            for _ in range(m2):
                f.write(a)
        size = os.path.getsize(path)
        assert size > 5 * 10 ** 9 and size > (1 << 32)
        M.main(["get_kmers", "-input_dir", os.path.join(work, "in"), "-output_dir", os.path.join(work, "out"),
                "-k", str(k)])
        got = np.load(os.path.join(work, "out", f"big_k{k}.npy"))
        s = lambda x: oracle.sparse_count(b">x\n" + x.tobytes(), k)
        cA, cAB, cABA, cAA = s(A), s(np.concatenate([A, B])), s(np.concatenate([A, B, A])), s(np.concatenate([A, A]))
        ek, ec = _combine([(m1, *cAB), (m1 - 1, *cABA), (-(m1 - 1), *cAB), (-(m1 - 1), *cA),
                           (m2, *cA), (m2 - 1, *cAA), (-2 * (m2 - 1), *cA)])
        assert int(ec.sum()) == (m1 * 6_000_000 - k + 1) + (m2 * 3_000_000 - k + 1)
        exp = M.sparse_kmers_matrix(ek.astype(np.uint64), ec, k)
        assert got.shape == exp.shape and np.array_equal(got, exp)
    finally:
        shutil.rmtree(work, ignore_errors=True)
