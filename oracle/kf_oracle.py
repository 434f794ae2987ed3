"""TEST INFRASTRUCTURE ONLY -- the checker, never the product path.

Python side of the oracle: a ctypes handle on the C restatement
(oracle/kmer_oracle.c) plus restatements of the post-processing that the
reference does in pandas after Jellyfish returns:

* ``kf_line``            -- kf2vec/main.py:323-357 (dump -> merge -> pseudocount ->
                            normalise -> ``astype(str)`` -> one ``.kf`` line);
* ``vocab_text``         -- the sorted canonical vocab files loaded at main.py:278-296;
* ``chunk_windows``      -- the ``get_chunks`` window plan, main.py:726-838
                            (seqtk linearise, awk N-run collapse, seqkit length
                            filter, ``seqkit sliding`` windows) used to pin
                            raw-count mode against toy_example/train_tree_chunks.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module.
"""
from __future__ import annotations

import ctypes
import math
import os
import re
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "libkmer_oracle.so")
_lib = None


def build() -> str:
    """Compile oracle/kmer_oracle.c (make -C oracle)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_SO) or os.path.getmtime(_SO) < os.path.getmtime(
                os.path.join(_HERE, "kmer_oracle.c")):
            build()
        L = ctypes.CDLL(_SO)
        u64, i32, vp = ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p
        L.oracle_nbins.restype = u64
        L.oracle_nbins.argtypes = [i32]
        L.oracle_rank_std.argtypes = [i32, vp]
        L.oracle_vocab.argtypes = [i32, vp]
        L.oracle_count.argtypes = [vp, u64, i32, i32, vp, vp, vp]
        L.oracle_count_many.argtypes = [vp, vp, i32, i32, i32, vp, vp, vp, i32]
        L.oracle_count_many_parts.argtypes = [vp, vp, i32, i32, i32, vp, vp, vp, i32, u64]
        L.oracle_max_threads.restype = i32
        L.oracle_synth_header_len.restype = u64
        L.oracle_synth_header_len.argtypes = [ctypes.c_int64]
        L.oracle_synth_genome.argtypes = [ctypes.c_int64, u64, u64, i32, u64, vp, u64]
        L.oracle_sparse_count.argtypes = [vp, u64, i32, i32, vp, vp, vp]
        L.oracle_sparse_count_many.argtypes = [vp, vp, i32, i32, i32, vp, vp, vp, i32]
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def nbins(k: int) -> int:
    return int(lib().oracle_nbins(k))


_rank_cache: dict[int, np.ndarray] = {}


def rank_std(k: int) -> np.ndarray:
    if k not in _rank_cache:
        r = np.zeros(1 << (2 * k), dtype=np.uint32)
        assert lib().oracle_rank_std(k, _ptr(r)) == 0
        _rank_cache[k] = r
    return _rank_cache[k]


def vocab_text(k: int) -> bytes:
    buf = np.zeros(nbins(k) * (k + 1), dtype=np.uint8)
    assert lib().oracle_vocab(k, _ptr(buf)) == 0
    return buf.tobytes()


def count(data: bytes | np.ndarray, k: int, fmt: int = 0) -> tuple[np.ndarray, int]:
    """Counts of one genome in vocab (column) order, and the total."""
    a = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    a = np.ascontiguousarray(a, dtype=np.uint8)
    c = np.zeros(nbins(k), dtype=np.uint32)
    t = ctypes.c_uint64(0)
    assert lib().oracle_count(_ptr(a), a.size, k, fmt, _ptr(rank_std(k)), _ptr(c), ctypes.byref(t)) == 0
    return c, int(t.value)


def count_many(buf: np.ndarray, off: np.ndarray, k: int, fmt: int = 0, threads: int = 0):
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    n = off.size - 1
    c = np.zeros((n, nbins(k)), dtype=np.uint32)
    t = np.zeros(n, dtype=np.uint64)
    assert lib().oracle_count_many(_ptr(buf), _ptr(off), n, k, fmt, _ptr(rank_std(k)),
                                   _ptr(c), _ptr(t), threads) == 0
    return c, t


def count_many_parts(buf: np.ndarray, off: np.ndarray, k: int, fmt: int = 0, threads: int = 0,
                     part_bytes: int = 1 << 20):
    """As count_many, OpenMP over (genome, part) pairs of about part_bytes each
    (bench.py's CPU baseline: every host thread busy whatever the genome count)."""
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    n = off.size - 1
    c = np.zeros((n, nbins(k)), dtype=np.uint32)
    t = np.zeros(n, dtype=np.uint64)
    assert lib().oracle_count_many_parts(_ptr(buf), _ptr(off), n, k, fmt, _ptr(rank_std(k)),
                                         _ptr(c), _ptr(t), threads, part_bytes) == 0
    return c, t


def synth_genome(g: int, seed: int, seq_len: int, width: int = 80, n_period: int = 0,
                 size: int | None = None) -> bytes:
    h = int(lib().oracle_synth_header_len(g))
    need = h + seq_len + (seq_len + width - 1) // width
    size = need if size is None else size
    out = np.zeros(size, dtype=np.uint8)
    assert lib().oracle_synth_genome(g, seed, seq_len, width, n_period, _ptr(out), size) == 0
    return out.tobytes()


# ---------------------------------------------------------------------------
# Post-processing restatement (kf2vec/main.py:323-357)
# ---------------------------------------------------------------------------
def kf_values(counts: np.ndarray, pseudocount: bool = False, raw_cnt: bool = False) -> list[str]:
    """``my_merged_counts["counts"].astype(str).to_list()`` (main.py:327-345).

    dtype quirks of the reference: ``pd.merge(vocab, dump, how='left')`` keeps the
    int64 dtype of the dump's count column when every vocab k-mer is present in
    the dump (no NaN introduced), otherwise it becomes float64 (NaN -> fillna(0)).
    So raw counts print as "54" when no bin is empty and "54.0" otherwise.
    """
    c = np.asarray(counts, dtype=np.int64)
    # ... and an empty dump (no k-mer at all): pandas reads an object column, the
    # merge leaves NaN everywhere and fillna(0) fills in the int 0, so raw counts
    # print "0" (pinned by tests/golden/ref_postproc/kf/empty_k7_raw.kf.gz)
    is_int = bool(c.size) and (bool((c > 0).all()) or not c.any())
    if pseudocount:                                   # main.py:332-334
        v = c.astype(np.float64) + 0.5
        is_int = False
    else:
        v = c if is_int else c.astype(np.float64)
    if not raw_cnt:                                   # main.py:340-342
        with np.errstate(invalid="ignore", divide="ignore"):
            v = v / v.sum()                           # int/int -> float64 true division
        is_int = False
    if is_int:
        return [str(x) for x in v.tolist()]
    return [repr(float(x)) for x in np.asarray(v, dtype=np.float64).tolist()]


def kf_line(name: str, counts: np.ndarray, pseudocount: bool = False, raw_cnt: bool = False) -> str:
    """One ``<sample>.kf`` file body (main.py:350-357)."""
    return "{},".format(name) + ",".join(kf_values(counts, pseudocount, raw_cnt)) + "\n"


def sample_name(fname: str) -> str:
    """main.py:275"""
    return fname.rsplit(".f", 1)[0]


# ---------------------------------------------------------------------------
# get_chunks window plan (kf2vec/main.py:726-838), used to pin raw-count mode.
# ---------------------------------------------------------------------------
CHUNK_SZ = 10000      # main.py:100
CHUNK_CNT_THR = 5     # main.py:101


def fasta_records(data: bytes) -> list[tuple[str, bytes]]:
    """seqtk seq -l 0: (header line without '>', linear sequence)."""
    recs = []
    name, seq = None, []
    for line in data.split(b"\n"):
        if line.endswith(b"\r"):     # seqtk's kseq strips a trailing CR
            line = line[:-1]
        if line.startswith(b">"):
            if name is not None:
                recs.append((name, b"".join(seq)))
            name, seq = line[1:].decode(), []
        elif name is not None:
            seq.append(line)
    if name is not None:
        recs.append((name, b"".join(seq)))
    return recs


_NRUN = re.compile(rb"[N|n]+")   # awk gsub(/[N|n]+/,"N") (main.py:740) -- '|' included
_GAPS = re.compile(rb"[- \t.]")  # seqkit seq -g default gap letters


def chunk_windows(fna: bytes, sample: str) -> list[tuple[str, bytes]]:
    """(chunk sample name, window sequence) in the order get_chunks concatenates
    them (contig order = FASTA order here; the reference uses os.listdir order of
    the split contig files, main.py:792, so row order across contigs is unpinned)."""
    out = []
    for hdr, seq in fasta_records(fna):
        seq = _NRUN.sub(b"N", seq)                     # main.py:740-742
        seq = _GAPS.sub(b"", seq)                      # seqkit seq -g (gap letters "- \\t.")
        if len(seq) < CHUNK_SZ:                        # seqkit seq -m 10000 (main.py:753)
            continue
        cid = hdr.split()[0]
        L = len(seq)
        tc = math.ceil(L / CHUNK_SZ)                   # main.py:813-818
        ov = int(math.ceil((tc * CHUNK_SZ - L) / (tc - 1))) if tc != 1 else 0
        step = CHUNK_SZ - ov
        s = 0
        while s + CHUNK_SZ <= L:                       # seqkit sliding (non-greedy)
            w = "{}_sliding:{}-{}".format(cid, s + 1, s + CHUNK_SZ)
            name = "{}.part_{}.part_{}".format(sample, cid, w).replace("sliding:", "sliding__")
            out.append((name, seq[s:s + CHUNK_SZ]))
            s += step
    return out


# ---------------------------------------------------------------------------
# get_kmers (kf2vec/main.py:112-184): sparse present-k-mer matrix for FSW
# ---------------------------------------------------------------------------
GET_KMERS_CODE = {ord("A"): 0, ord("T"): 1, ord("C"): 2, ord("G"): 3}   # main.py:118


def kmers_matrix_from_dump(dump_lines: list[tuple[str, int]], k: int) -> np.ndarray:
    """Restates main.py:147-172 for `jellyfish dump -c -t` lines (kmer, count) in
    whatever order Jellyfish emits them: rows = k digits (A0 T1 C2 G3) + float32
    count / float32 sum."""
    kmer_data, counts = [], []
    for seq, cnt in dump_lines:
        if all(b in "ATCG" for b in seq):                        # main.py:154
            kmer_data.append([GET_KMERS_CODE[ord(b)] for b in seq])   # :156
            counts.append(int(cnt))
    if not kmer_data:
        return np.zeros((0, k + 1), dtype=np.float32)
    kmer_matrix = np.array(kmer_data, dtype=np.float32)            # :165
    counts_array = np.array(counts, dtype=np.float32)              # :166
    normalized = counts_array / np.sum(counts_array)               # :169
    return np.column_stack((kmer_matrix, normalized))             # :172


def sparse_count(data: bytes | np.ndarray, k: int, fmt: int = 0) -> tuple[np.ndarray, np.ndarray]:
    """Present canonical k-mers of one genome at any k <= 31 (what `jellyfish
    count -C` + `dump -c` give get_kmers, main.py:133-160), ascending by standard
    2-bit code (lexicographic), and their counts (kmer_oracle.c oracle_sparse_count)."""
    a = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    a = np.ascontiguousarray(a, dtype=np.uint8)
    keys = np.zeros(max(a.size, 1), dtype=np.uint64)
    cnt = np.zeros(max(a.size, 1), dtype=np.uint32)
    n = ctypes.c_uint64(0)
    assert lib().oracle_sparse_count(_ptr(a), a.size, k, fmt, _ptr(keys), _ptr(cnt), ctypes.byref(n)) == 0
    return keys[: n.value].copy(), cnt[: n.value].copy()


def sparse_count_many(buf: np.ndarray, off: np.ndarray, k: int, fmt: int = 0, threads: int = 0):
    """sparse_count of every genome of a packed batch (OpenMP over genomes), in
    the device counter's layout: (keys uint64[off[n]], counts uint32[off[n]],
    nuniq uint64[n]) with genome g's k-mers at [off[g], off[g] + nuniq[g])."""
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    n = off.size - 1
    tot = max(int(off[-1]), 1)
    keys = np.zeros(tot, dtype=np.uint64)
    cnt = np.zeros(tot, dtype=np.uint32)
    nu = np.zeros(max(n, 1), dtype=np.uint64)
    assert lib().oracle_sparse_count_many(_ptr(buf), _ptr(off), n, k, fmt, _ptr(keys), _ptr(cnt), _ptr(nu),
                                          threads) == 0
    return keys, cnt, nu[:n]


def std_code_text(keys: np.ndarray, k: int) -> list[str]:
    """k-mer strings of standard 2-bit codes (A0 C1 G2 T3, first base most significant)."""
    keys = np.asarray(keys, dtype=np.uint64)
    sh = 2 * np.arange(k - 1, -1, -1, dtype=np.uint64)
    chars = np.frombuffer(b"ACGT", np.uint8)[((keys[:, None] >> sh[None, :]) & np.uint64(3)).astype(np.intp)]
    return [r.tobytes().decode() for r in chars]


def dump_lines(counts: np.ndarray, k: int) -> list[tuple[str, int]]:
    """The `jellyfish dump -c` content implied by a count vector (vocab order)."""
    vocab = vocab_text(k).split()
    return [(vocab[i].decode(), int(c)) for i, c in enumerate(counts) if c]
