"""``get_chunks`` on the device (reference kf2vec/main.py:654-929).

The reference shells out per genome to
* ``seqtk seq -l 0`` to linearise records (:732);
* ``awk gsub(/[N|n]+/,"N")`` to collapse N runs (:740-742);
* ``seqkit seq -m 10000 -g -v`` to drop gaps and contigs < 10 kbp (:753);
* ``seqkit split`` / ``seqkit sliding`` to make 10 kbp windows (:784, :824, :837);
then runs one ``get_frequencies -raw_cnt`` (a Jellyfish pair) per window
(:869-881) and concatenates the rows (:895-915).

Here a genome's bytes go to HBM once; ``kf_chunk_compact`` (csrc/kf_chunks.hip)
does the linearisation, N-run collapse and gap removal of every record in one
pass; the host plans the windows from the record lengths (:813-818);
``kf_chunk_gather`` lays the windows of a batch of genomes out back to back and
one ``kf_count_batch`` counts them all; ``kf_write_kf_rows`` formats a genome's
rows with host threads into its one ``.kf`` file.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _native as N

CHUNK_SZ = 10000       # main.py:100
CHUNK_CNT_THR = 5      # main.py:101


def window_plan(total_length: int) -> tuple[int, int]:
    """(number of windows, step) for a contig of this length (main.py:813-818;
    seqkit sliding keeps only whole windows)."""
    total_chunks = math.ceil(total_length / CHUNK_SZ)
    ovrlap = int(math.ceil((total_chunks * CHUNK_SZ - total_length) / (total_chunks - 1))) \
        if total_chunks != 1 else 0
    step = CHUNK_SZ - ovrlap
    n = 0 if total_length < CHUNK_SZ else (total_length - CHUNK_SZ) // step + 1
    return n, step


def window_name(sample: str, cid: str, s: int) -> str:
    """Row name of the window starting at s (main.py:905-915: `<sample>.part_<cid>.part_<seqkit id>`,
    ':' of seqkit's "_sliding:a-b" replaced by "__")."""
    return "{}.part_{}.part_{}_sliding__{}-{}".format(sample, cid, cid, s + 1, s + CHUNK_SZ)


def record_regions(data: np.ndarray) -> tuple[np.ndarray, list[str]]:
    """Sequence regions [start, end) of the FASTA records (the bytes after each
    header line, up to the next header) and the contig ids (first word of the
    header, seqtk/seqkit id; a trailing '\\r' of the header line is dropped)."""
    iv, _ = _index_fasta(data)
    n = iv.size // 2
    se = np.empty(2 * n, dtype=np.uint64)
    ids = []
    L = data.size
    for r in range(n):
        hs, he = int(iv[2 * r]), int(iv[2 * r + 1])
        se[2 * r] = min(he + 1, L)
        se[2 * r + 1] = int(iv[2 * r + 2]) if r + 1 < n else L
        hdr = data[hs + 1: he].tobytes()
        if hdr.endswith(b"\r"):
            hdr = hdr[:-1]
        w = hdr.split()
        ids.append(w[0].decode(errors="surrogateescape") if w else "")
    return se, ids


def _index_fasta(data: np.ndarray):
    from .counter import index_records
    return index_records(data, N.KF_FMT_FASTA, 0)


@dataclass
class ChunkBatch:
    """Windows of several genomes laid out back to back on the device."""
    buf: torch.Tensor                       # uint8, capacity windows x CHUNK_SZ
    n: int = 0                              # windows so far
    genomes: list = field(default_factory=list)   # (sample, [row names]) in row order

    @property
    def capacity(self) -> int:
        return self.buf.numel() // CHUNK_SZ


class ChunkPipeline:
    """Device pre-pass + window gather + count + row writer for get_chunks."""

    def __init__(self, counter, device: torch.device, capacity_windows: int, threads: int):
        self.counter = counter
        self.device = device
        self.threads = max(1, int(threads))
        self.batch = ChunkBatch(torch.empty(max(1, capacity_windows) * CHUNK_SZ, dtype=torch.uint8, device=device))

    def windows_of(self, data: bytes, sample: str) -> tuple[list[str], np.ndarray, torch.Tensor]:
        """(row names, window starts in the processed sequence, processed sequence
        on the device) of one genome; no window if no contig reaches 10 kbp."""
        host = np.frombuffer(data, dtype=np.uint8)
        se, ids = record_regions(host)
        if se.size == 0:
            return [], np.zeros(0, np.uint64), None
        dev = self.device
        s = torch.cuda.current_stream(dev).cuda_stream
        d_bytes = torch.from_numpy(host.copy()).to(dev, non_blocking=False)
        d_seq = torch.from_numpy(se.view(np.int64)).to(dev)
        d_out = torch.empty(max(host.size, 16), dtype=torch.uint8, device=dev)
        d_se = torch.empty(se.size, dtype=torch.int64, device=dev)
        nwords = (host.size + 4095) // 4096 + 1
        scratch = torch.empty(nwords, dtype=torch.int32, device=dev)
        N.check(N.lib().kf_chunk_compact(d_bytes.data_ptr(), host.size, d_seq.data_ptr(), se.size // 2,
                                         d_out.data_ptr(), d_se.data_ptr(), scratch.data_ptr(), nwords, s),
                "kf_chunk_compact")
        out_se = d_se.cpu().numpy().view(np.uint64)          # (synchronises the stream)
        names, starts = [], []
        for r, cid in enumerate(ids):
            a, b = int(out_se[2 * r]), int(out_se[2 * r + 1])
            L = b - a
            if L < CHUNK_SZ:                                   # seqkit seq -m 10000 (main.py:753)
                continue
            n, step = window_plan(L)
            for i in range(n):
                names.append(window_name(sample, cid, i * step))
                starts.append(a + i * step)
        return names, np.asarray(starts, dtype=np.uint64), d_out

    def add(self, sample: str, names: list[str], starts: np.ndarray, d_seq: torch.Tensor, flush) -> None:
        """Gather a genome's windows into the batch (flushing it first if full)."""
        if self.batch.n + len(names) > self.batch.capacity:
            flush()
            if len(names) > self.batch.capacity:   # one genome larger than the batch: grow it
                self.batch = ChunkBatch(torch.empty(len(names) * CHUNK_SZ, dtype=torch.uint8, device=self.device))
        b = self.batch
        d_src = torch.from_numpy(starts.view(np.int64)).to(self.device)
        dst = b.buf[b.n * CHUNK_SZ:]
        N.check(N.lib().kf_chunk_gather(d_seq.data_ptr(), d_src.data_ptr(), len(names), CHUNK_SZ, dst.data_ptr(),
                                        torch.cuda.current_stream(self.device).cuda_stream), "kf_chunk_gather")
        b.n += len(names)
        b.genomes.append((sample, names))

    def count_and_write(self, output_dir: str, pseudocount: bool, written) -> None:
        """Count every window of the batch in one kf_count_batch and write each
        genome's rows into <output_dir>/<sample>.kf (raw counts, main.py:869-915)."""
        import ctypes
        import os

        from .counter import DeviceBatch, counts_to_numpy
        b = self.batch
        if b.n == 0:
            return
        dev = self.device
        off = torch.arange(0, (b.n + 1) * CHUNK_SZ, CHUNK_SZ, dtype=torch.int64, device=dev)
        db = DeviceBatch(b.buf, off, torch.zeros(2, dtype=torch.int64, device=dev), b.n, 0)
        counts, _ = self.counter.count(db)
        c = counts_to_numpy(counts)
        row = 0
        for sample, names in b.genomes:
            enc = [n.encode(errors="surrogateescape") for n in names]
            arr = (ctypes.c_char_p * len(enc))(*enc)
            rows = np.ascontiguousarray(c[row: row + len(names)])
            N.check(N.lib().kf_write_kf_rows(os.fsencode(os.path.join(output_dir, "{}.kf".format(sample))), arr,
                                             len(enc), rows.ctypes.data, rows.shape[1], int(bool(pseudocount)), 1,
                                             self.threads), "kf_write_kf_rows")
            row += len(names)
            written(sample)
        b.n = 0
        b.genomes = []
