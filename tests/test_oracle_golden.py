"""Pins the CPU oracle (oracle/) against every golden vector the reference holds
for this path: the 7 toy `.kf` files with their `.fna` (get_frequencies,
normalised), the 3 chunk `.kf` files (get_chunks -> get_frequencies -raw_cnt,
kf2vec/main.py:869-881) and the vocab files (main.py:278-296)."""
import gzip
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, TOY


def test_oracle_toy_kf_byte_exact(oracle, toy):
    assert len(toy) == 7
    for name, sample, data, exp in toy:
        c, total = oracle.count(data, 7)
        assert int(c.sum()) == total
        assert oracle.kf_line(sample, c).encode() == exp, name


@pytest.mark.parametrize("sample", ["G000830275", "G000830295", "G000402355"])
def test_oracle_chunks_raw_byte_exact(oracle, sample):
    fna = gzip.open(os.path.join(TOY, "train_tree_fna", sample + ".fna.gz")).read()
    exp = gzip.open(os.path.join(TOY, "train_tree_chunks", sample + ".kf.gz")).read().decode()
    rows = exp.splitlines(keepends=True)
    got = {}
    for name, seq in oracle.chunk_windows(fna, sample):
        c, _ = oracle.count(b">w\n" + seq + b"\n", 7)
        got[name] = oracle.kf_line(name, c, raw_cnt=True)
    assert len(got) == len(rows)
    for r in rows:
        assert got[r.split(",", 1)[0]] == r


def test_oracle_vocab_matches_reference_files(oracle):
    ref = json.load(open(os.path.join(GOLDEN, "vocab_sha256.json")))["vocab"]
    for k, (n, sha, _) in ref.items():
        t = oracle.vocab_text(int(k))
        assert t.count(b"\n") == n == oracle.nbins(int(k))
        assert hashlib.sha256(t).hexdigest() == sha


def test_oracle_small_cases(oracle):
    # hand-checked: ACGT has k=2 mers AC, CG, GT -> canonical AC, CG, AC
    c, t = oracle.count(b">x\nACGT\n", 2)
    vocab = oracle.vocab_text(2).split()
    got = {vocab[i].decode(): int(v) for i, v in enumerate(c) if v}
    assert got == {"AC": 2, "CG": 1} and t == 3
    # line breaks are transparent, records and N break k-mers
    a, _ = oracle.count(b">x\nAC\nGT\n", 2)
    assert (a == c).all()
    b, tb = oracle.count(b">x\nAC\n>y\nGT\n", 2)
    assert tb == 2
    n, tn = oracle.count(b">x\nACNGT\n", 2)
    assert tn == 2
    low, _ = oracle.count(b">x\nacgt\n", 2)
    assert (low == c).all()
    # FASTQ: only sequence lines count, quality may contain ACGT
    fq, tq = oracle.count(b"@r1\nACGT\n+\nACGT\n@r2\nAC\nGT\n+\nII\nII\n", 2)
    assert tq == 3 + 3
    # empty genome
    z, tz = oracle.count(b"", 7)
    assert tz == 0 and not z.any()


def test_kf_values_quirks(oracle):
    c = np.array([3, 0, 1], dtype=np.uint32)
    assert oracle.kf_values(c, raw_cnt=True) == ["3.0", "0.0", "1.0"]
    assert oracle.kf_values(np.array([3, 2, 1]), raw_cnt=True) == ["3", "2", "1"]
    assert oracle.kf_values(np.array([3, 2, 1]), pseudocount=True, raw_cnt=True) == ["3.5", "2.5", "1.5"]
    assert oracle.kf_values(np.array([1, 1, 2])) == ["0.25", "0.25", "0.5"]
    assert oracle.kf_values(np.zeros(2)) == ["nan", "nan"]


def test_oracle_synth_spec(oracle):
    g = oracle.synth_genome(3, 20260101 + 3, 1000, 80)
    assert g.startswith(b">syn_3\n")
    lines = g.split(b"\n")
    assert all(len(x) == 80 for x in lines[1:-2]) and len(lines[-2]) == 40
    assert set(b"".join(lines[1:])) <= set(b"ACGT")
    gn = oracle.synth_genome(3, 7, 300000, 80, n_period=2)
    assert b"N" in gn


@pytest.mark.parametrize("part", [3, 64, 1000, 1 << 20])
def test_oracle_parts_equal_whole_genomes(oracle, part):
    """bench.py's CPU baseline counts each genome in parts (OpenMP over genome x
    part, context rebuilt from a line start): it must equal the per-genome scan on
    ragged FASTA (headers, blank lines, 1-base lines, N, CRLF, lowercase) and FASTQ."""
    import gen
    rng = np.random.default_rng(31 + part)
    blobs = [gen.random_fasta(rng, int(rng.integers(0, 12000)), max_records=6, n_rate=0.003, lower=0.05,
                              crlf_rate=0.1, iupac_rate=0.001, poly_rate=0.01) for _ in range(12)]
    blobs += [b"", b">h\n", b"\n\n\n\n", b">x\n" + b"\n" * 50 + b"ACGTACGTAC\n" * 3 + b"\n" * 40 + b"GGTTACA\n",
              gen.random_fastq(rng, 50, n_rate=0.01)]
    off = np.cumsum([0] + [len(b) for b in blobs]).astype(np.uint64)
    buf = np.frombuffer(b"".join(blobs) + b"\0", np.uint8)
    for k in ((3, 7) if part < 1000 else (3, 7, 11)):   # (each part merges a whole row)
        c1, t1 = oracle.count_many(buf, off, k, 0, 4)
        c2, t2 = oracle.count_many_parts(buf, off, k, 0, 4, part)
        assert np.array_equal(c1, c2) and np.array_equal(t1, t2), (k, part)


# ---------------------------------------------------------------------------
# tests/golden/ref_postproc: the reference's own get_frequencies / get_kmers
# post-processing (kf2vec/main.py:250-373, 112-184), run in the build container
# by tests/golden/ref_postproc/make_fixtures.py on inputs the toy set lacks
# ---------------------------------------------------------------------------
REFPP = os.path.join(GOLDEN, "ref_postproc")


def _refpp():
    return json.load(open(os.path.join(REFPP, "manifest.json")))


def _refpp_input(rel):
    return gzip.open(os.path.join(REFPP, rel)).read()


def test_refpp_kf_modes_oracle_and_product_formatter(oracle):
    """-pseudocount, -raw_cnt, both, on ragged / all-bins-present / tiny /
    low-complexity genomes at k = 3..9, plus the empty genome: the oracle's
    restatement AND the product's C++ formatter (kf_format_kf, host code) give the
    reference's bytes."""
    from kf2vecfsw_amd.main import format_kf
    m = _refpp()
    cases = m["kf"] + [e for e in m["errors"] if "file" in e]
    assert len(cases) == 44
    for e in cases:
        exp = gzip.open(os.path.join(REFPP, e["file"])).read()
        data = _refpp_input(e["input"]) if "input" in e else b""
        name = e.get("sample", "empty")
        c, _ = oracle.count(data, e["k"])
        assert oracle.kf_line(name, c, e["pseudocount"], e["raw_cnt"]).encode() == exp, e["file"]
        assert format_kf(name, c, e["pseudocount"], e["raw_cnt"]) == exp, e["file"]


def test_refpp_int_text_quirks_are_covered():
    """The fixtures hold both integer-text cases of raw mode (every bin present;
    empty dump) and their float counterparts."""
    m = _refpp()
    firsts = {e["file"]: gzip.open(os.path.join(REFPP, e["file"])).read().split(b",")[1]
              for e in m["kf"] + [e for e in m["errors"] if "file" in e]}
    assert firsts["kf/dense_k3_raw.kf.gz"].isdigit()
    assert firsts["kf/empty_k7_raw.kf.gz"] == b"0"
    assert firsts["kf/empty_k7.kf.gz"] == b"nan"
    assert b"." in firsts["kf/ragged_k7_raw.kf.gz"] and b"." in firsts["kf/dense_k3_pseudo_raw.kf.gz"]


def test_refpp_npy_oracle_and_product(oracle):
    """get_kmers .npy: digits A0 T1 C2 G3 + float32 count / float32 sum, rows in
    the dump's order (sorted canonical here): the oracle's restatement and the
    product's kmers_matrix equal the reference's arrays bit for bit."""
    from kf2vecfsw_amd.main import kmers_matrix
    m = _refpp()
    assert len(m["npy"]) == 6
    for e in m["npy"]:
        exp = np.load(os.path.join(REFPP, e["file"]), allow_pickle=False)
        c, _ = oracle.count(_refpp_input(e["input"]), e["k"])
        ref = oracle.kmers_matrix_from_dump(oracle.dump_lines(c, e["k"]), e["k"])
        assert exp.dtype == np.float32 and np.array_equal(ref, exp), e["file"]
        got = kmers_matrix(c, e["k"])
        assert got.dtype == np.float32 and np.array_equal(got, exp), e["file"]


def test_sparse_oracle_equals_dense_oracle(oracle):
    """oracle_sparse_count (sort + run-length, any k <= 31) against the pinned dense
    restatement: the same present k-mers and counts for k = 2..9 on a toy genome."""
    import gzip
    data = gzip.open(os.path.join(TOY, "test_fna", "G000402355sub.fna.gz")).read()
    for k in range(2, 10):
        keys, cnts = oracle.sparse_count(data, k)
        c, tot = oracle.count(data, k)
        nz = np.nonzero(c)[0]
        vocab = oracle.vocab_text(k).split()
        assert [vocab[i].decode() for i in nz] == oracle.std_code_text(keys, k)
        assert np.array_equal(c[nz], cnts) and int(cnts.sum()) == tot
