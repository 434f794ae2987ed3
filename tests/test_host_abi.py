"""CPU tests of the C-ABI library: it loads, exports every symbol of
include/kf2vec_gpu.h, and its host half (bin tables, vocab, record index,
`.kf` formatter/writer) matches the oracle.  No device calls."""
import ctypes
import gzip
import os
import re

import numpy as np
import pytest

from conftest import ROOT, TOY
import gen


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "kf2vec_gpu.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(kf_\w+)\s*\(", txt, re.M)))


def test_exports_every_header_symbol(native):
    from kf2vecfsw_amd import _native
    syms = header_symbols()
    assert len(syms) >= 13
    for s in syms:
        assert hasattr(native, s), s
    assert set(syms) == set(_native.SIGNATURES), "ctypes signatures out of sync with the header"
    assert native.kf_abi_version() == 1


def test_tables_match_oracle(native, oracle):
    from kf2vecfsw_amd import counter as C
    for k in range(2, 12):
        c2c, c2r = C.tables(k)
        x = np.arange(1 << (2 * k), dtype=np.uint64)
        s = x ^ ((x >> np.uint64(1)) & np.uint64(int("01" * k, 2)))   # kf code -> lexicographic code
        assert (c2c == oracle.rank_std(k)[s]).all(), k
        nb = C.num_bins(k)
        assert nb == oracle.nbins(k)
        assert (c2c[c2r] == np.arange(nb)).all()
        # the representative is min(code, revcomp(code)) in kf code
        rc = np.zeros_like(x)
        y = x.copy()
        for _ in range(k):
            rc = (rc << np.uint64(2)) | ((y & np.uint64(3)) ^ np.uint64(2))
            y >>= np.uint64(2)
        assert (c2r == np.minimum(x, rc)[c2r]).all()


def test_vocab_text_matches_oracle(native, oracle):
    from kf2vecfsw_amd import counter as C
    for k in range(3, 12):
        assert C.vocab_text(k) == oracle.vocab_text(k)


def test_format_kf_matches_reference_goldens(native, oracle):
    from kf2vecfsw_amd.main import format_kf
    for fd, kd in [("train_tree_fna", "train_tree_kf"), ("test_fna", "test_kf")]:
        for f in sorted(os.listdir(os.path.join(TOY, fd))):
            sample = f[:-3].rsplit(".f", 1)[0]
            c, _ = oracle.count(gzip.open(os.path.join(TOY, fd, f)).read(), 7)
            exp = gzip.open(os.path.join(TOY, kd, sample + ".kf.gz")).read()
            assert format_kf(sample, c) == exp


@pytest.mark.parametrize("pseudo", [False, True])
@pytest.mark.parametrize("raw", [False, True])
def test_format_kf_modes_match_oracle(native, oracle, pseudo, raw):
    from kf2vecfsw_amd.main import format_kf
    rng = np.random.default_rng(7)
    cases = [rng.integers(0, 2 ** 32 - 1, size=4000, dtype=np.uint64).astype(np.uint32),
             rng.integers(0, 3, size=8192).astype(np.uint32),
             rng.integers(1, 100, size=2080).astype(np.uint32),          # all bins present -> int dtype
             np.zeros(32, np.uint32), np.ones(1, np.uint32),
             (rng.pareto(1.0, size=8192) * 10).astype(np.uint32)]
    # the writer's eight-column single-digit path: groups broken by 9/10/1023/1024/
    # 2^31, ragged tails, all-present and all-zero rows of every length to 33
    for n in range(0, 34):
        c = rng.poisson(1.2, size=n).astype(np.uint32)
        if n:
            c[rng.integers(0, n)] = rng.choice([9, 10, 1023, 1024, 2 ** 31, 2 ** 32 - 1])
        cases += [c, c + 1, np.zeros(n, np.uint32), np.full(n, 9, np.uint32)]
    for c in cases:
        assert format_kf("s", c, pseudo, raw).decode() == oracle.kf_line("s", c, pseudo, raw)


def test_write_kf_files(native, oracle, tmp_path):
    from kf2vecfsw_amd.main import write_kf_files
    rng = np.random.default_rng(3)
    c = rng.integers(0, 50, size=(9, 512)).astype(np.uint32)
    names = ["g%d" % i for i in range(9)]
    write_kf_files(str(tmp_path), names, c, False, False, 4)
    for i, n in enumerate(names):
        assert (tmp_path / (n + ".kf")).read_text() == oracle.kf_line(n, c[i])


def test_index_records_fasta_semantics(native, oracle):
    """Index + device semantics (newline-transparent, excluded = reset) count
    exactly what the oracle's own FASTA parser counts."""
    from kf2vecfsw_amd import counter as C
    rng = np.random.default_rng(11)
    for t in range(40):
        data = gen.random_fasta(rng, int(rng.integers(0, 3000)), n_rate=0.01, iupac_rate=0.002, lower=0.1,
                                crlf_rate=0.2)
        base = int(rng.integers(0, 1 << 40))
        iv, fmt = C.index_records(np.frombuffer(data, np.uint8), 0, base)
        assert fmt == 1 and (np.diff(iv.astype(np.int64)) > 0).all() if iv.size else True
        k = int(rng.integers(2, 9))
        got = gen.model_count(data, iv, base, k, oracle.rank_std(k))
        exp = oracle.count(data, k, 1)
        assert got[1] == exp[1] and (got[0] == exp[0]).all(), t


def test_index_records_fastq_semantics(native, oracle):
    from kf2vecfsw_amd import counter as C
    rng = np.random.default_rng(12)
    for t in range(20):
        data = gen.random_fastq(rng, int(rng.integers(0, 30)), n_rate=0.01, multiline=bool(t % 2))
        iv, fmt = C.index_records(np.frombuffer(data, np.uint8), 0, 0)
        if data:
            assert fmt == 2
        k = int(rng.integers(2, 9))
        got = gen.model_count(data, iv, 0, k, oracle.rank_std(k))
        exp = oracle.count(data, k, 0)
        assert got[1] == exp[1] and (got[0] == exp[0]).all(), t


def test_index_records_range_error(native):
    from kf2vecfsw_amd import _native as N
    data = b">a\nAC\n>b\nGT\n>c\nTT\n"
    out = np.zeros(2, np.uint64)
    n = ctypes.c_uint64(0)
    rc = N.lib().kf_index_records(data, len(data), 0, 0, out.ctypes.data, 1, ctypes.byref(n), None)
    assert rc == N.KF_ERANGE and n.value == 3
    assert N.lib().kf_last_error().decode().startswith("record index needs")


def test_count_batch_rejects_bad_args(native):
    from kf2vecfsw_amd import _native as N
    L = N.lib()
    assert L.kf_count_batch(None, None, 1, None, 0, None, None, 7, None, None, 0, None) == N.KF_EINVAL
    assert L.kf_count_batch(None, None, 1, None, 0, None, None, 13, None, None, 0, None) == N.KF_EINVAL
    assert b"k out of range" in L.kf_last_error()
    assert L.kf_count_batch(None, None, 0, None, 0, None, None, 7, None, None, 0, None) == N.KF_OK


def test_chunk_window_plan_counts():
    """get_chunks window plan (main.py:813-818 + seqkit sliding's whole windows):
    the number of windows for contig lengths around the 10 kbp boundaries."""
    from kf2vecfsw_amd import chunks as CH
    for L in [9999, 10000, 10001, 19999, 20000, 25000, 1241422]:
        n, step = CH.window_plan(L)
        assert n == (0 if L < 10000 else len(range(0, L - 10000 + 1, step)))
        if n:
            assert (n - 1) * step + 10000 <= L and 0 < step <= 10000


def test_chunk_record_regions(native):
    """Sequence regions after each header line and the contig ids (first word,
    trailing CR dropped) that name the windows."""
    import numpy as np
    from kf2vecfsw_amd import chunks as CH
    data = np.frombuffer(b"junk\n>c1 desc\r\nACGT\nAC\n>c2\nGG\n>\n\n>c4 x", np.uint8)
    se, ids = CH.record_regions(data)
    assert ids == ["c1", "c2", "", "c4"]
    regs = [data[int(se[2 * i]): int(se[2 * i + 1])].tobytes() for i in range(len(ids))]
    assert regs == [b"ACGT\nAC\n", b"GG\n", b"\n", b""]
    # consecutive header lines (empty records) are merged by kf_index_records: each
    # line is still its own record, so b's windows are named after b
    data = np.frombuffer(b">a\n>b y\r\n>c\nACGT\n>d\n>e", np.uint8)
    se, ids = CH.record_regions(data)
    assert ids == ["a", "b", "c", "d", "e"]
    regs = [data[int(se[2 * i]): int(se[2 * i + 1])].tobytes() for i in range(len(ids))]
    assert regs == [b"", b"", b"ACGT\n", b"", b""]


def test_get_kmers_matrix_matches_reference_restatement(native, oracle):
    """kmers_matrix (product) == main.py:147-172 restated, fed the dump implied by the counts."""
    from kf2vecfsw_amd.main import kmers_matrix
    data = gzip.open(os.path.join(TOY, "test_fna", "G000830275sub.fna.gz")).read()
    for k in (3, 7, 9):
        c, _ = oracle.count(data, k)
        got = kmers_matrix(c, k)
        exp = oracle.kmers_matrix_from_dump(oracle.dump_lines(c, k), k)
        assert got.dtype == np.float32 and got.shape == exp.shape
        assert np.array_equal(got, exp)
        # permutation invariance: a shuffled dump gives the same rows (as a set)
        lines = oracle.dump_lines(c, k)
        rng = np.random.default_rng(k)
        shuf = oracle.kmers_matrix_from_dump([lines[i] for i in rng.permutation(len(lines))], k)
        key = lambda m: m[np.lexsort(m[:, ::-1].T)]
        assert np.array_equal(key(got), key(shuf))


@pytest.mark.parametrize("pseudo", [False, True])
@pytest.mark.parametrize("raw", [False, True])
def test_features_handoff_equals_kf_text_round_trip(native, pseudo, raw):
    """counter.features (in-memory hand-off) == parsing the `.kf` line the writer
    produces, times the trainers' scaler: bit for bit (CPU torch).  Python's
    float() is correctly rounded, like pandas' float_precision="round_trip"; the
    GPU twin also bounds pandas' default parser (<= 1 ulp)."""
    import torch
    from kf2vecfsw_amd import counter as C
    from kf2vecfsw_amd.main import format_kf
    rng = np.random.default_rng(21)
    rows = np.stack([rng.integers(0, 300, size=2080), (rng.pareto(1.0, size=2080) * 10).astype(np.int64),
                     np.zeros(2080, np.int64), np.full(2080, 2 ** 32 - 7)]).astype(np.uint32)
    got = C.features(torch.from_numpy(rows.view(np.int32)), pseudo, raw, scaler=10000.0).numpy()
    for i, r in enumerate(rows):
        vals = format_kf("s", r, pseudo, raw).decode().rstrip("\n").split(",")[1:]
        exp = np.array([float(x) for x in vals]) * 10000.0
        assert np.array_equal(got[i], exp, equal_nan=True), i


def test_features_handoff_float32_equals_trainers_pandas_path(native):
    """What the trainers feed their models is `torch.from_numpy(df.values *
    1e4).float()` with df from my_read_csv (utils.py:436-437: pandas' DEFAULT
    parser, not correctly rounded; train_model_set.py:291, 620).  counter.features
    (...).float() equals that except where the parse's <= ~1e-12 relative error
    crosses a float32 rounding boundary: there the two differ by one float32 ulp
    (the hand-off's value is the correctly rounded one).  Bound: <= 1 ulp, in at
    most 1 entry per 100,000 (measured: 1 of 786,432 here)."""
    import io

    import pandas as pd
    import torch
    from kf2vecfsw_amd import counter as C
    from kf2vecfsw_amd.main import format_kf
    rng = np.random.default_rng(23)
    n_diff = n_all = 0
    for t in range(48):
        row = rng.integers(0, int(rng.choice([3, 50, 2000, 100000])), size=8192).astype(np.uint32)
        for pseudo in (False, True):
            got = C.features(torch.from_numpy(row[None].view(np.int32)), pseudo, False, scaler=1e4).float().numpy()[0]
            df = pd.read_csv(io.BytesIO(format_kf(f"s{t}", row, pseudo)), index_col=0, header=None, sep=",")
            exp = torch.from_numpy(df.values * 1e4).float().numpy()[0]
            ulp = np.abs(got.view(np.int32).astype(np.int64) - exp.view(np.int32).astype(np.int64))
            assert int(ulp.max()) <= 1, (t, pseudo)
            n_diff += int(np.count_nonzero(ulp))
            n_all += ulp.size
    assert n_diff <= n_all // 100_000, (n_diff, n_all)


def test_write_kf_segments_append_and_arenas(native, oracle, tmp_path):
    """kf_write_kf_segments (get_chunks' writer): several files at once, rows in
    order, a segment appended to the file an earlier call started, raw counts
    above and below the formatter's text table (1,024), and enough rows for the
    per-thread 16 MiB formatting arenas to roll over."""
    import ctypes
    from kf2vecfsw_amd import _native as N
    rng = np.random.default_rng(31)
    nb = 8192
    rows = rng.integers(0, 4, size=(700, nb)).astype(np.uint32)
    rows[:, ::97] = rng.integers(1000, 5000, size=rows[:, ::97].shape)
    names = [f"s.part_c{i % 3}.part_c{i % 3}_sliding__{i + 1}-{i + 10000}" for i in range(700)]
    paths = [str(tmp_path / f"g{j}.kf") for j in range(3)]

    def call(seg_paths, row0, app, lo, hi):
        enc = [n.encode() for n in names[lo:hi]]
        r0 = np.asarray(row0, np.int32)
        ap = np.asarray(app, np.uint8)
        sub = np.ascontiguousarray(rows[lo:hi])
        rc = N.lib().kf_write_kf_segments(len(seg_paths), (ctypes.c_char_p * len(seg_paths))(*[p.encode() for p in seg_paths]),
                                          r0.ctypes.data, ap.ctypes.data, (ctypes.c_char_p * len(enc))(*enc),
                                          None, None, None, 0, sub.ctypes.data, nb, 0, 1, 3)
        assert rc == 0, N.lib().kf_last_error()

    # launch 1: g0 rows 0..299, g1 rows 300..399; launch 2: g1 continues (append) 400..549, g2 550..699
    call(paths[:2], [0, 300, 400], [0, 0], 0, 400)
    call(paths[1:], [0, 150, 300], [1, 0], 400, 700)
    exp = ["".join(oracle.kf_line(names[i], rows[i], raw_cnt=True) for i in range(a, b))
           for a, b in [(0, 300), (300, 550), (550, 700)]]
    for p, e in zip(paths, exp):
        assert open(p).read() == e
    # a truncating segment replaces an earlier file
    call(paths[:1], [0, 1], [0], 0, 1)
    assert open(paths[0]).read() == oracle.kf_line(names[0], rows[0], raw_cnt=True)


def test_write_kf_segments_generated_names(native, oracle, tmp_path):
    """kf_write_kf_segments with names built by the writer from contig prefixes and
    window positions (get_chunks' rows: "<sample>.part_<cid>.part_<cid>_sliding__<s+1>-<s+10000>")."""
    import ctypes
    from kf2vecfsw_amd import _native as N
    from kf2vecfsw_amd import chunks as CH
    rng = np.random.default_rng(32)
    rows = rng.integers(0, 3, size=(40, 512)).astype(np.uint32)
    pre = ["g.part_c1.part_c1_sliding__", "g.part_x y.part_x y_sliding__"]
    rpre = np.asarray([0] * 25 + [1] * 15, np.uint32)
    rpos = np.asarray(list(range(0, 25 * 9930, 9930)) + list(range(0, 15 * 9990, 9990)), np.uint64)
    path = str(tmp_path / "g.kf")
    r0 = np.asarray([0, 40], np.int32)
    enc = [p.encode() for p in pre]
    rc = N.lib().kf_write_kf_segments(1, (ctypes.c_char_p * 1)(path.encode()), r0.ctypes.data, None, None,
                                      (ctypes.c_char_p * 2)(*enc), rpre.ctypes.data, rpos.ctypes.data, CH.CHUNK_SZ,
                                      rows.ctypes.data, 512, 0, 1, 4)
    assert rc == 0, N.lib().kf_last_error()
    names = [pre[p] + "{}-{}".format(s + 1, s + CH.CHUNK_SZ) for p, s in zip(rpre.tolist(), rpos.tolist())]
    assert open(path).read() == "".join(oracle.kf_line(n, r, raw_cnt=True) for n, r in zip(names, rows))


def test_sparse_kmers_matrix_matches_reference_restatement(native, oracle):
    """get_kmers at k > 12: sparse_kmers_matrix (product) on the oracle's present
    k-mers == main.py:147-172 restated on the same k-mers as `dump -c` lines."""
    from kf2vecfsw_amd.main import sparse_kmers_matrix
    data = gzip.open(os.path.join(TOY, "test_fna", "G000830275sub.fna.gz")).read()
    for k in (13, 21, 31):
        keys, cnts = oracle.sparse_count(data, k)
        got = sparse_kmers_matrix(keys, cnts, k)
        exp = oracle.kmers_matrix_from_dump(list(zip(oracle.std_code_text(keys, k), cnts.tolist())), k)
        assert got.dtype == np.float32 and got.shape == exp.shape == (keys.size, k + 1)
        assert np.array_equal(got, exp)
    assert sparse_kmers_matrix(np.zeros(0, np.uint64), np.zeros(0, np.uint32), 21).shape == (0, 22)


def test_sparse_count_rejects_bad_args(native):
    """kf_sparse_count argument checks (no kernel is launched) and the workspace size."""
    from kf2vecfsw_amd import _native as N
    L = N.lib()
    assert L.kf_sparse_count(None, None, 1, 100, None, 0, 32, None, 0, None, None, None, None) == N.KF_EINVAL
    assert L.kf_sparse_count(None, None, 1, 100, None, 0, 1, None, 0, None, None, None, None) == N.KF_EINVAL
    assert L.kf_sparse_count(None, None, 0, 0, None, 0, 21, None, 0, None, None, None, None) == N.KF_OK
    assert L.kf_sparse_count(None, None, 1, 100, None, 0, 21, None, 0, None, None, None, None) == N.KF_EINVAL
    assert b"null" in L.kf_last_error()
    assert L.kf_sparse_count(None, None, 1, 1 << 32, None, 0, 21, None, 0, None, None, None, None) == N.KF_EINVAL
    assert L.kf_sparse_workspace_bytes(32, 100, 1) == 0
    w16, w17 = L.kf_sparse_workspace_bytes(16, 1 << 20, 4), L.kf_sparse_workspace_bytes(17, 1 << 20, 4)
    assert (1 << 20) * 8 < w16 < w17   # u32 keys up to k = 16, u64 above; upos + histograms on top


@pytest.mark.parametrize("pseudo", [0, 1])
def test_write_kf_segments16_equals_u32(native, oracle, tmp_path, pseudo):
    """kf_write_kf_segments16 (u16 rows, get_chunks' copy-back width) writes the same
    bytes as the u32 writer: counts 0..9 (SIMD text), up to 65,535, rows with no
    zero column (integer text) and an all-zero row; pseudocount on and off."""
    import ctypes
    from kf2vecfsw_amd import _native as N
    rng = np.random.default_rng(33)
    nb = 2080   # not a multiple of 8: the scalar tail too
    rows = rng.integers(0, 4, size=(60, nb)).astype(np.uint32)
    rows[:, ::13] = rng.integers(0, 65536, size=rows[:, ::13].shape)
    rows[5] = rng.integers(1, 9, size=nb)
    rows[6] = 0
    names = [f"w{i}" for i in range(60)]
    enc = (ctypes.c_char_p * 60)(*[n.encode() for n in names])
    r0 = np.asarray([0, 25, 60], np.int32)
    out = {}
    for tag, arr, fn in (("u32", rows, N.lib().kf_write_kf_segments),
                         ("u16", np.ascontiguousarray(rows.astype(np.uint16)), N.lib().kf_write_kf_segments16)):
        paths = [str(tmp_path / f"{tag}_{j}.kf") for j in range(2)]
        rc = fn(2, (ctypes.c_char_p * 2)(*[p.encode() for p in paths]), r0.ctypes.data, None, enc, None, None, None,
                0, arr.ctypes.data, nb, pseudo, 1, 3)
        assert rc == 0, N.lib().kf_last_error()
        out[tag] = [open(p).read() for p in paths]
    assert out["u16"] == out["u32"]
    assert out["u32"][0] == "".join(oracle.kf_line(names[i], rows[i], pseudocount=bool(pseudo), raw_cnt=True)
                                    for i in range(25))


def test_pack_files_without_index(native, tmp_path):
    """pack_files(index=False): a FASTA batch comes back unindexed (excl None: the
    device indexes it); a batch holding a FASTQ file is indexed on the host, FASTA
    files included, exactly as with index=True."""
    from kf2vecfsw_amd import counter as C
    fa = tmp_path / "a.fna"
    fa.write_bytes(b">a\nACGT\n>b\nGG\n")
    fb = tmp_path / "b.fa"
    fb.write_bytes(b"ACGT\n>c x\nTT")
    fq = tmp_path / "c.fq"
    fq.write_bytes(b"@r1\nACGT\n+\nIIII\n")
    hb = C.pack_files([str(fa), str(fb)], pin=False, threads=1, index=False)
    assert hb.excl is None and hb.n == 2
    assert hb.seq_chars() == C.pack_files([str(fa), str(fb)], pin=False, threads=1).seq_chars()
    mixed = C.pack_files([str(fa), str(fq), str(fb)], pin=False, threads=1, index=False)
    ref = C.pack_files([str(fa), str(fq), str(fb)], pin=False, threads=1)
    assert mixed.excl is not None and np.array_equal(mixed.excl, ref.excl)


def test_read_files_pieces_padding_and_errors(native, tmp_path):
    """kf_read_files (the CLI readers' native path): every file lands at its slot
    whatever the piece size (pieces smaller than a file, files smaller than a
    piece, empty files), the slot tails are '\\n', and a file that changed size
    since it was stat'ed fails loudly naming it."""
    import ctypes
    import gen
    from kf2vecfsw_amd import _native as N
    from kf2vecfsw_amd import counter as C
    rng = np.random.default_rng(44)
    blobs = [gen.random_fasta(rng, int(rng.integers(0, 200000))) for _ in range(9)] + [b"", b">x\nAC\n"]
    paths = []
    for i, b in enumerate(blobs):
        p = tmp_path / f"g{i}.fna"
        p.write_bytes(b)
        paths.append(str(p))
    ref = C.pack_genomes(blobs, pin=False)
    for piece, threads in ((4096, 1), (4096, 8), (1 << 16, 3), (1 << 30, 8)):
        hb = C.pack_files(paths, pin=False, threads=threads, piece=piece, index=True)
        assert np.array_equal(hb.data.numpy()[: int(hb.off[-1])], ref.data.numpy()[: int(ref.off[-1])])
        assert np.array_equal(hb.excl, ref.excl)
    sizes = np.array([len(b) for b in blobs], np.uint64)
    off = C._layout(list(sizes))
    dst = np.zeros(int(off[-1]), np.uint8)
    sizes[3] += 1   # stale size
    enc = (ctypes.c_char_p * len(paths))(*[p.encode() for p in paths])
    rc = native.kf_read_files(enc, len(paths), sizes.ctypes.data, off.ctypes.data, dst.ctypes.data, 4096, 4)
    assert rc == N.KF_EINVAL and b"g3.fna" in native.kf_last_error()
