"""Host-side driver of the device k-mer counter.

Mirrors the per-file work of kf2vec's ``get_frequencies`` (reference
kf2vec/main.py:301-357) for a whole batch of genomes at once:

* :func:`pack_genomes` / :func:`pack_files` lay several FASTA/FASTQ files out
  back to back in one (pinned) host buffer and build the record index
  (``kf_index_records``) -- the device-side replacement of the ``jellyfish
  count`` input (main.py:309-311);
* :class:`KmerCounter` owns the per-k bin tables on the device (the vocab of
  main.py:278-296) and runs ``kf_count_batch`` on PyTorch-ROCm tensors, giving
  the ``n_genomes x nbins`` count matrix in vocab column order -- what the
  reference gets from ``jellyfish dump -c`` + the left-merge (main.py:317-328).

PyTorch is used for device memory and streams only.
"""
from __future__ import annotations

import ctypes
import dataclasses
import os
from typing import Sequence

import numpy as np
import torch

from . import _native as N

ALIGN = 16  # genome starts are 16-byte aligned inside a batch ('\n' padding)


def num_bins(k: int) -> int:
    return int(N.lib().kf_num_bins(k))


def tables(k: int) -> tuple[np.ndarray, np.ndarray]:
    """(code2col[4^k], col2rep[nbins]) -- see include/kf2vec_gpu.h kf_tables."""
    nb = num_bins(k)
    code2col = np.empty(1 << (2 * k), dtype=np.uint32)
    col2rep = np.empty(nb, dtype=np.uint32)
    n = ctypes.c_uint64(0)
    N.check(N.lib().kf_tables(k, code2col.ctypes.data, col2rep.ctypes.data, ctypes.byref(n)), "kf_tables")
    assert n.value == nb
    return code2col, col2rep


def vocab_text(k: int) -> bytes:
    nb = num_bins(k)
    buf = np.empty(nb * (k + 1), dtype=np.uint8)
    w = ctypes.c_uint64(0)
    N.check(N.lib().kf_vocab_text(k, buf.ctypes.data, buf.size, ctypes.byref(w)), "kf_vocab_text")
    return buf[: w.value].tobytes()


def index_records(data: np.ndarray, fmt: int = N.KF_FMT_AUTO, base: int = 0) -> tuple[np.ndarray, int]:
    """Excluded (non-sequence) byte ranges of one file, as a flat [s0,e0,s1,e1,...]
    uint64 array offset by ``base``; also returns the detected format."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    cap = 64
    while True:
        out = np.empty(2 * cap, dtype=np.uint64)
        n = ctypes.c_uint64(0)
        f = ctypes.c_int(0)
        rc = N.lib().kf_index_records(data.ctypes.data, data.size, fmt, base, out.ctypes.data, cap,
                                      ctypes.byref(n), ctypes.byref(f))
        if rc == N.KF_ERANGE:
            cap = int(n.value)
            continue
        N.check(rc, "kf_index_records")
        return out[: 2 * n.value], int(f.value)


@dataclasses.dataclass
class HostBatch:
    """Genomes packed back to back: genome g = data[off[g]:off[g+1]]."""
    data: torch.Tensor | None   # uint8, (pinned) host
    off: np.ndarray             # uint64 [n+1]
    excl: np.ndarray | None     # uint64 [2*m] absolute [start, end) pairs; None: FASTA indexed on the device
    names: list[str]
    dev_data: torch.Tensor | None = None   # the bytes already copied to the device (maybe on another stream)
    dev_event: object = None               # ... and the event that copy recorded

    @property
    def n(self) -> int:
        return len(self.off) - 1

    def seq_chars(self) -> int:
        """Sequence characters (excludes header/quality lines and newlines)."""
        d = self.data.numpy()
        nl = int(np.count_nonzero(d[: int(self.off[-1])] == 10))
        excl = self.excl if self.excl is not None else np.concatenate(
            [index_records(d[int(self.off[i]): int(self.off[i + 1])], N.KF_FMT_FASTA, int(self.off[i]))[0]
             for i in range(self.n)] or [np.zeros(0, np.uint64)])
        ex = int((excl[1::2] - excl[0::2]).sum()) if excl.size else 0
        return int(self.off[-1] - self.off[0]) - nl - ex


def _layout(sizes: Sequence[int]) -> np.ndarray:
    off = np.zeros(len(sizes) + 1, dtype=np.uint64)
    pos = 0
    for i, s in enumerate(sizes):
        off[i] = pos
        pos += (int(s) + ALIGN - 1) // ALIGN * ALIGN
    off[-1] = pos
    return off


def _alloc_host(nbytes: int, pin: bool) -> torch.Tensor:
    pin = pin and torch.cuda.is_available()
    return torch.empty(max(nbytes, ALIGN), dtype=torch.uint8, pin_memory=pin)


def pack_genomes(blobs: Sequence[bytes | np.ndarray], names: Sequence[str] | None = None,
                 fmt: int = N.KF_FMT_AUTO, pin: bool = True) -> HostBatch:
    sizes = [len(b) for b in blobs]
    off = _layout(sizes)
    data = _alloc_host(int(off[-1]), pin)
    d = data.numpy()
    d[: int(off[-1])] = 10  # '\n' padding between genomes is transparent
    excl = []
    for i, b in enumerate(blobs):
        a = np.frombuffer(b, dtype=np.uint8) if isinstance(b, (bytes, bytearray, memoryview)) else np.asarray(b, np.uint8)
        lo = int(off[i])
        d[lo: lo + a.size] = a
        iv, _ = index_records(d[lo: lo + a.size], fmt, lo)
        excl.append(iv)
    ex = np.concatenate(excl) if excl else np.zeros(0, np.uint64)
    return HostBatch(data, off, ex.astype(np.uint64), list(names) if names else [str(i) for i in range(len(blobs))])


def pack_files(paths: Sequence[str], names: Sequence[str] | None = None, fmt: int = N.KF_FMT_AUTO,
               pin: bool = True, threads: int = 8, pool=None, times: dict | None = None,
               buf: torch.Tensor | None = None, index: bool = True, piece: int = 1 << 20) -> HostBatch:
    """Read files straight into one (pinned) buffer and index their records.  The
    bytes come from one native call (kf_read_files: pieces of at most `piece`
    bytes read by pread on native threads, as many as `pool` has workers or
    `threads`); FASTQ files (and FASTA ones when index=True) are then indexed by
    the pool (the ctypes index calls release the GIL).
    `buf`: a caller-owned (pinned) buffer of at least the batch's bytes to read
    into instead of a fresh allocation (the caller makes sure no copy still reads it).
    index=False: a batch of FASTA files is not indexed here (excl None: to_device
    finds the header lines on the device, kf_index_fasta); a batch with a FASTQ
    file is indexed on the host all the same."""
    from concurrent.futures import ThreadPoolExecutor
    import time
    t0 = time.perf_counter()
    sizes = [os.path.getsize(p) for p in paths]
    off = _layout(sizes)
    if buf is not None and buf.numel() >= max(int(off[-1]), ALIGN):
        data = buf[: max(int(off[-1]), ALIGN)]
    else:
        data = _alloc_host(int(off[-1]), pin)
    d = data.numpy()
    if times is not None:
        times["alloc_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
    # the bytes: one native call (kf_read_files: pread pieces on native threads)
    nthr = getattr(pool, "_max_workers", None) or max(1, int(threads))
    if paths:
        enc = [os.fsencode(p) for p in paths]
        arr = (ctypes.c_char_p * len(enc))(*enc)
        sz = np.asarray(sizes, dtype=np.uint64)
        N.check(N.lib().kf_read_files(arr, len(enc), sz.ctypes.data, off.ctypes.data, d.ctypes.data,
                                      int(piece), int(nthr)), "kf_read_files")

    def on_host(i: int) -> bool:   # FASTQ (or index=True): the host index
        return index or fmt == N.KF_FMT_FASTQ or (fmt == N.KF_FMT_AUTO and sizes[i] > 0 and d[int(off[i])] == ord("@"))

    def host_index(i: int):
        lo, sz = int(off[i]), sizes[i]
        return index_records(d[lo: lo + sz], fmt, lo)[0] if on_host(i) else None

    if not any(on_host(i) for i in range(len(paths))):   # FASTA only: the device indexes it
        return HostBatch(data, off, None, list(names) if names else list(paths))
    if pool is not None:
        excl = list(pool.map(host_index, range(len(paths))))
    elif threads > 1 and len(paths) > 1:
        with ThreadPoolExecutor(max_workers=min(threads, len(paths))) as ex:
            excl = list(ex.map(host_index, range(len(paths))))
    else:
        excl = [host_index(i) for i in range(len(paths))]
    if not index and all(e is None for e in excl):
        return HostBatch(data, off, None, list(names) if names else list(paths))
    excl = [e if e is not None else index_records(d[int(off[i]): int(off[i]) + sizes[i]], N.KF_FMT_FASTA,
                                                  int(off[i]))[0] for i, e in enumerate(excl)]
    ex = np.concatenate(excl) if excl else np.zeros(0, np.uint64)
    return HostBatch(data, off, ex.astype(np.uint64), list(names) if names else list(paths))


def pack_ranges(ranges: Sequence[tuple[str, int, int]], names: Sequence[str] | None = None, pin: bool = True,
                threads: int = 8, chunk: int = 64 << 20, index: bool = False) -> HostBatch:
    """As pack_files for byte ranges [(path, start, end)] of files (the pieces of
    a file too large for one sparse call, main.fasta_pieces, or get_chunks'
    record-aligned parts, main.record_pieces), read by os.preadv in chunks of
    `chunk` bytes on `threads` threads; FASTA only (index=False: the record index
    is left to the device; index=True: the header lines indexed here)."""
    from concurrent.futures import ThreadPoolExecutor
    sizes = [e - a for _, a, e in ranges]
    off = _layout(sizes)
    data = _alloc_host(int(off[-1]), pin)
    d = data.numpy()
    d[: int(off[-1])] = 10                       # '\n' padding is transparent
    jobs = []
    for i, (p, a, e) in enumerate(ranges):
        for x in range(a, e, chunk):
            jobs.append((p, x, min(e, x + chunk), int(off[i]) + x - a))

    def read(job):
        p, x, y, dst = job
        fd = os.open(p, os.O_RDONLY)
        try:
            got = 0
            mv = memoryview(d[dst: dst + (y - x)])
            while got < y - x:
                r = os.preadv(fd, [mv[got:]], x + got)
                if r <= 0:
                    raise N.NativeError(f"short read on {p}")
                got += r
        finally:
            os.close(fd)

    with ThreadPoolExecutor(max_workers=max(1, int(threads))) as ex:
        list(ex.map(read, jobs))
        excl = None
        if index:
            parts = list(ex.map(lambda i: index_records(d[int(off[i]): int(off[i]) + sizes[i]], N.KF_FMT_FASTA,
                                                        int(off[i]))[0], range(len(ranges))))
            excl = (np.concatenate(parts) if parts else np.zeros(0, np.uint64)).astype(np.uint64)
    return HostBatch(data, off, excl, list(names) if names else [f"{p}:{a}" for p, a, _ in ranges])


@dataclasses.dataclass
class DeviceBatch:
    data: torch.Tensor      # uint8 on device (16-byte aligned)
    off: torch.Tensor       # int64 [n+1]
    excl: torch.Tensor      # int64 [2m]
    n: int
    n_excl: int


def index_on_device(data: torch.Tensor, off: torch.Tensor, n: int, nbytes: int) -> tuple[torch.Tensor, int]:
    """FASTA header lines of a device batch (kf_index_fasta) on the current
    stream: (pairs int64[2m] on the device, m).  Reads m back (one small
    synchronising copy); a table that was too small is grown and the index run
    again, so the result is always complete."""
    dev = data.device
    s = _stream_ptr(dev)
    nb = (nbytes + 4095) // 4096
    scratch = torch.empty(nb + 1, dtype=torch.int32, device=dev)
    npairs = torch.zeros(1, dtype=torch.int64, device=dev)
    # 64 header lines per genome to start (draft assemblies with more contigs
    # re-run once with the exact count; ADVICE r04: a bytes-proportional first
    # guess allocated ~25 % of the batch)
    cap = 64 * n + 4096
    while True:
        excl = torch.empty(max(2 * cap, 2), dtype=torch.int64, device=dev)
        N.check(N.lib().kf_index_fasta(data.data_ptr(), off.data_ptr(), n, nbytes, excl.data_ptr(), cap,
                                       npairs.data_ptr(), scratch.data_ptr(), nb + 1, s), "kf_index_fasta")
        m = int(npairs.item())
        if m <= cap:
            return excl[: 2 * m], m
        cap = m


def to_device(hb: HostBatch, device: torch.device | str = "cuda") -> DeviceBatch:
    """Asynchronous H2D of a batch on the current stream.  The small offset and
    interval tables are staged through pinned memory too: a copy from pageable
    memory would block the host until the stream's earlier copies finish.  A
    batch packed without its record index (excl None) is indexed on the device
    (index_on_device: one small synchronising copy)."""
    dev = torch.device(device)
    if hb.dev_data is not None:   # copied already (get_frequencies' readers, on a copy stream)
        cur = torch.cuda.current_stream(dev)
        if hb.dev_event is not None:
            cur.wait_event(hb.dev_event)
        data = hb.dev_data
        data.record_stream(cur)
    else:
        data = hb.data.to(dev, non_blocking=True)
    if hb.excl is None:
        pin = hb.data is None or hb.data.is_pinned()
        off = torch.from_numpy(hb.off.view(np.int64))
        off = (off.pin_memory() if pin else off).to(dev, non_blocking=pin)
        with torch.cuda.device(dev):
            excl, m = index_on_device(data, off, hb.n, int(hb.off[-1]))
        return DeviceBatch(data, off, excl if m else torch.zeros(2, dtype=torch.int64, device=dev), hb.n, m)
    ex = hb.excl if hb.excl.size else np.zeros(2, np.uint64)
    pin = hb.data is None or hb.data.is_pinned()
    n_off = (hb.off.size + 1) & ~1   # the interval table starts 16-byte aligned
    host = np.zeros(n_off + ex.size, np.int64)
    host[: hb.off.size] = hb.off.view(np.int64)
    host[n_off:] = ex.view(np.int64)
    small = torch.from_numpy(host)
    if pin:
        small = small.pin_memory()
    small = small.to(dev, non_blocking=pin)
    off, excl = small[: hb.off.size], small[n_off:]
    return DeviceBatch(data, off, excl, hb.n, hb.excl.size // 2)


def _stream_ptr(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


_DEV_TABLES: dict = {}   # (k, device index) -> (code2col, col2rep) on the device


class KmerCounter:
    """Canonical k-mer counter for one k on one device (the ``jellyfish count -C
    -m k`` + ``dump -c`` + vocab merge of main.py:309-328)."""

    def __init__(self, k: int, device: torch.device | str = "cuda"):
        if not (N.KF_MIN_K <= k <= N.KF_MAX_K):
            raise ValueError(f"k={k} out of range [{N.KF_MIN_K}, {N.KF_MAX_K}]")
        self.k = k
        self.device = torch.device(device)
        if self.device.type != "cuda" or not torch.cuda.is_available():
            raise N.NativeError("KmerCounter needs a ROCm GPU (no CPU fallback)")
        self.nbins = num_bins(k)
        key = (k, self.device.index if self.device.index is not None else torch.cuda.current_device())
        if key not in _DEV_TABLES:   # immutable: one upload per (k, device) and process
            c2c, c2r = tables(k)
            _DEV_TABLES[key] = (torch.from_numpy(c2c.view(np.int32)).to(self.device),
                                torch.from_numpy(c2r.view(np.int32)).to(self.device))
        self.code2col, self.col2rep = _DEV_TABLES[key]

    def launch_info(self) -> tuple[int, int, int]:
        g, b, l = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        with torch.cuda.device(self.device):
            N.check(N.lib().kf_count_launch_info(self.k, ctypes.byref(g), ctypes.byref(b), ctypes.byref(l)),
                    "kf_count_launch_info")
        return g.value, b.value, l.value

    def reserve(self, max_genomes: int) -> None:
        """Allocate the library's workspace for batches of up to max_genomes now
        (kf_workspace_reserve), so that count() never allocates or synchronises."""
        with torch.cuda.device(self.device):
            N.check(N.lib().kf_workspace_reserve(self.k, int(max_genomes)), "kf_workspace_reserve")

    def alloc_out(self, n: int) -> tuple[torch.Tensor, torch.Tensor]:
        return (torch.empty((n, self.nbins), dtype=torch.int32, device=self.device),
                torch.empty(n, dtype=torch.int64, device=self.device))

    def count(self, db: DeviceBatch, counts: torch.Tensor | None = None, totals: torch.Tensor | None = None,
              accumulate: bool = False, stream: int | None = None) -> tuple[torch.Tensor, torch.Tensor]:
        """Enqueue the count kernel; returns (counts int32[n, nbins] holding uint32
        bit patterns, totals int64[n]) on the device."""
        if counts is None or totals is None:
            counts, totals = self.alloc_out(db.n)
        assert counts.shape == (db.n, self.nbins) and counts.dtype == torch.int32 and counts.is_contiguous()
        assert totals.shape == (db.n,) and totals.dtype == torch.int64
        assert db.data.data_ptr() % 16 == 0
        s = _stream_ptr(self.device) if stream is None else stream
        with torch.cuda.device(self.device):
            N.check(N.lib().kf_count_batch(
                db.data.data_ptr(), db.off.data_ptr(), db.n, db.excl.data_ptr() if db.n_excl else None,
                db.n_excl, self.code2col.data_ptr(), self.col2rep.data_ptr(), self.k,
                counts.data_ptr(), totals.data_ptr(), N.KF_ACCUMULATE if accumulate else 0, s), "kf_count_batch")
        return counts, totals


class SparseCounter:
    """Present canonical k-mers at any k = 2..31 (``kf_sparse_count``): what
    get_kmers reads from ``jellyfish count -C -m k`` + ``dump -c -t``
    (main.py:133-160) -- per genome, the distinct canonical k-mers as standard
    2-bit codes (A0 C1 G2 T3, first base most significant; ascending = the
    lexicographic order of the vocab files) and their counts."""

    def __init__(self, k: int, device: torch.device | str = "cuda"):
        if not (N.KF_MIN_K <= k <= N.KF_SPARSE_MAX_K):
            raise ValueError(f"k={k} out of range [{N.KF_MIN_K}, {N.KF_SPARSE_MAX_K}]")
        self.k = k
        self.device = torch.device(device)
        if self.device.type != "cuda" or not torch.cuda.is_available():
            raise N.NativeError("SparseCounter needs a ROCm GPU (no CPU fallback)")
        self._work = None

    def workspace_bytes(self, batch_bytes: int, n: int) -> int:
        return int(N.lib().kf_sparse_workspace_bytes(self.k, int(batch_bytes), int(n)))

    def count(self, db: DeviceBatch, batch_bytes: int):
        """Enqueue the sparse count of a batch whose genomes end at batch_bytes
        (= off[n]) on the current stream (the outputs and the reused workspace
        belong to that stream's allocator pool, so there is no stream argument);
        returns (keys int64[batch_bytes] holding uint64 codes, counts
        int32[batch_bytes] holding uint32, nuniq int64[n]) on the device: genome
        g's k-mers are keys[off[g] : off[g] + nuniq[g]]."""
        batch_bytes = int(batch_bytes)
        need = self.workspace_bytes(batch_bytes, db.n)
        if self._work is None or self._work.numel() < need:
            self._work = None
            self._work = torch.empty(max(need, 256), dtype=torch.uint8, device=self.device)
        keys = torch.empty(max(batch_bytes, 1), dtype=torch.int64, device=self.device)
        counts = torch.empty(max(batch_bytes, 1), dtype=torch.int32, device=self.device)
        nuniq = torch.zeros(max(db.n, 1), dtype=torch.int64, device=self.device)
        s = _stream_ptr(self.device)
        with torch.cuda.device(self.device):
            N.check(N.lib().kf_sparse_count(
                db.data.data_ptr(), db.off.data_ptr(), db.n, batch_bytes,
                db.excl.data_ptr() if db.n_excl else None, db.n_excl, self.k,
                self._work.data_ptr(), self._work.numel(), keys.data_ptr(), counts.data_ptr(),
                nuniq.data_ptr(), s), "kf_sparse_count")
        return keys, counts, nuniq[: db.n]

    def to_host(self, keys: torch.Tensor, counts: torch.Tensor, nuniq: torch.Tensor,
                off: np.ndarray) -> list[tuple[np.ndarray, np.ndarray]]:
        """Per genome (keys uint64[m], counts uint32[m]) on the host: each genome's
        slice is gathered on the device and the batch copied back once."""
        nu = nuniq.cpu().numpy()
        if nu.size and (nu == -1).any():   # UINT64_MAX: the library refused the offsets
            raise N.NativeError("kf_sparse_count: genome offsets must be non-decreasing and end at or below "
                                "batch_bytes (nothing was counted)")
        if nu.size and (nu == -2).any():   # UINT64_MAX - 1: the device's order check failed
            raise N.NativeError("kf_sparse_count: the sorted keys failed the device's order check")
        if nu.size == 0 or int(nu.sum()) == 0:
            return [(np.zeros(0, np.uint64), np.zeros(0, np.uint32)) for _ in range(nu.size)]
        idx = torch.cat([torch.arange(int(off[g]), int(off[g]) + int(nu[g]), device=keys.device)
                         for g in range(nu.size)])
        hk = keys[idx].cpu().numpy().view(np.uint64)
        hc = counts[idx].cpu().numpy().view(np.uint32)
        out, pos = [], 0
        for g in range(nu.size):
            m = int(nu[g])
            out.append((hk[pos: pos + m], hc[pos: pos + m]))
            pos += m
        return out


def counts_to_numpy(counts: torch.Tensor) -> np.ndarray:
    return counts.cpu().numpy().view(np.uint32)


def features(counts: torch.Tensor, pseudocount: bool = False, raw_cnt: bool = False,
             scaler: float = 1.0) -> torch.Tensor:
    """In-memory hand-off: the float64 feature matrix the
    trainers build from `.kf` files -- `my_read_csv` (utils.py:436-437) then
    `* features_scaler` (train_classifier_model.py:148, train_model_set.py:291) --
    computed on the device from the count matrix, without the text round trip.

    The values are main.py:332-342 (`+0.5` pseudocount, `v / v.sum()` unless raw)
    in float64: the row sums are exact (integers or halves below 2^53) and each
    quotient is correctly rounded, so they equal the numbers the `.kf` text holds
    (`repr` round-trips float64; `pd.read_csv(..., float_precision="round_trip")`
    reads them back bit for bit).  pandas' default parser, which my_read_csv
    uses, is not correctly rounded: about half the entries of a k=7 row read
    differently, by at most ~1e-12 relative (8.7e-13 measured on the toy genomes).  An empty
    genome gives NaN rows (normalised) as the reference's "nan" strings parse.
    """
    c = counts.to(torch.int64)
    c = torch.where(c < 0, c + (1 << 32), c)          # uint32 bit patterns held in int32
    v = c.to(torch.float64)
    if pseudocount:
        v = v + 0.5
    if not raw_cnt:
        v = v / v.sum(dim=1, keepdim=True)
    return v * scaler if scaler != 1.0 else v


def synth_ids(n: int, g0: int = 0, g_stride: int = 1) -> list[int]:
    return [g0 + i * g_stride for i in range(n)]


def synth_layout(n: int, seq_len: int, width: int = 80, g0: int = 0, g_stride: int = 1,
                 align: int = 256) -> np.ndarray:
    """Offsets of n synthetic genomes (kf_synth_fasta layout)."""
    L = N.lib()
    off = np.zeros(n + 1, dtype=np.uint64)
    pos = 0
    for i, g in enumerate(synth_ids(n, g0, g_stride)):
        off[i] = pos
        pos += int(L.kf_synth_genome_bytes(g, seq_len, width, align))
    off[-1] = pos
    return off


def synth_excl(off: np.ndarray, g0: int = 0, g_stride: int = 1) -> np.ndarray:
    """Record index of a synthetic batch: one header line per genome."""
    L = N.lib()
    n = len(off) - 1
    ex = np.empty(2 * n, dtype=np.uint64)
    for i, g in enumerate(synth_ids(n, g0, g_stride)):
        ex[2 * i] = off[i]
        ex[2 * i + 1] = off[i] + int(L.kf_synth_header_len(g)) - 1  # up to the header's '\n'
    return ex


def synth_fasta_bytes(seq_len: int, width: int = 80, g: int = 0) -> int:
    """Unpadded FASTA size of one synthetic genome (header + bases + newlines)."""
    return int(N.lib().kf_synth_header_len(g)) + seq_len + (seq_len + width - 1) // width


def synth_device_batch(n: int, seq_len: int, seed0: int, width: int = 80, n_period: int = 0, g0: int = 0,
                       g_stride: int = 1, device: torch.device | str = "cuda") -> DeviceBatch:
    """Generate n synthetic FASTA genomes (ids g0 + i*g_stride) directly in HBM."""
    dev = torch.device(device)
    off = synth_layout(n, seq_len, width, g0, g_stride)
    ex = synth_excl(off, g0, g_stride)
    data = torch.empty(int(off[-1]), dtype=torch.uint8, device=dev)
    doff = torch.from_numpy(off.view(np.int64)).to(dev)
    dex = torch.from_numpy(ex.view(np.int64)).to(dev)
    s = _stream_ptr(dev)
    with torch.cuda.device(dev):
        for c0 in range(0, n, 65535):
            c1 = min(n, c0 + 65535)
            N.check(N.lib().kf_synth_fasta(data.data_ptr(), doff[c0:].data_ptr(), c1 - c0, g0 + c0 * g_stride,
                                           g_stride, seed0, seq_len, width, n_period, s), "kf_synth_fasta")
    return DeviceBatch(data, doff, dex, n, n)
