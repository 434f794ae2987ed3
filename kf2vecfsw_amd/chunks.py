"""``get_chunks`` on the device (reference kf2vec/main.py:654-929).

The reference shells out per genome to
* ``seqtk seq -l 0`` to linearise records (:732);
* ``awk gsub(/[N|n]+/,"N")`` to collapse N runs (:740-742);
* ``seqkit seq -m 10000 -g -v`` to drop gaps and contigs < 10 kbp (:753);
* ``seqkit split`` / ``seqkit sliding`` to make 10 kbp windows (:784, :824, :837);
then runs one ``get_frequencies -raw_cnt`` (a Jellyfish pair) per window
(:869-881) and concatenates the rows (:895-915).

Here the genomes are processed in batches of files:
* the files of a batch are read into one pinned buffer by a thread pool and
  their header lines indexed (``kf_index_records``);
* one H2D copy, then ONE ``kf_chunk_compact`` (csrc/kf_chunks.hip) over every
  record of every genome of the batch: linearisation, N-run collapse and gap
  removal;
* ONE device-to-host copy of the processed record bounds per batch; the host
  plans every genome's windows from them (:813-818, numpy);
* the windows are gathered into a device buffer (``kf_chunk_gather``) and
  counted by ``kf_count_batch`` in launches of at most ``max_windows`` windows
  (the count matrix is 4 x bins bytes per window: 32 KiB at k=7, 8 MiB at k=11);
* the count rows come back as uint16 on a copy stream of their own, and a
  writer thread formats and writes each launch's rows while the device counts
  the next launch (``kf_write_kf_segments16``: rows formatted by host threads,
  one file per genome written in parallel, appended when a genome's windows span
  several launches).
"""
from __future__ import annotations

import ctypes
import math
import os
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _native as N

CHUNK_SZ = 10000       # main.py:100
CHUNK_CNT_THR = 5      # main.py:101
assert CHUNK_SZ < 1 << 16   # window counts fit uint16 (count_and_write)
LAUNCH_WINDOWS = 4096  # windows per count launch at most (128 MiB of k=7 counts)

# KF_TRACE=1: stage timeline (host ms since the first event) for tools/chunks_bench.py
TRACE = os.environ.get("KF_TRACE") == "1"
trace: list = []


def _tr(stage: str, t0: float, **kw) -> None:
    if TRACE:
        import time
        trace.append((stage, round(t0 * 1e3, 3), round(time.perf_counter() * 1e3, 3), kw))


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


def _contig_id(hdr: bytes) -> str:
    """seqtk/seqkit id: the first word of the header line ('>' and a trailing '\\r' dropped)."""
    if hdr.endswith(b"\r"):
        hdr = hdr[:-1]
    w = hdr.split()
    return w[0].decode(errors="surrogateescape") if w else ""


def records_from_index(data: np.ndarray, iv: np.ndarray, lo: int, hi: int) -> tuple[list[int], list[str]]:
    """Records of the FASTA bytes data[lo:hi] whose header lines are indexed by iv
    (kf_index_records pairs, absolute positions): [start, end) of each record's
    sequence region (the bytes after its header line, up to the next header) as
    a flat [s0, e0, s1, e1, ...] list, and the contig ids.  kf_index_records
    merges header lines that follow each other (an empty record, ">a\n>b\n..."),
    so every interval is split at its newlines: each line is one header."""
    heads: list[int] = []      # header line starts
    starts: list[int] = []     # sequence region starts
    ids: list[str] = []
    for r in range(iv.size // 2):
        hs, he = int(iv[2 * r]), int(iv[2 * r + 1])
        pos = hs
        for line in data[hs: he].tobytes().split(b"\n"):
            heads.append(pos)
            starts.append(min(pos + len(line) + 1, hi))
            ids.append(_contig_id(line[1:]))
            pos += len(line) + 1
    ends = heads[1:] + [hi]
    out = [0] * (2 * len(ids))
    out[0::2] = starts
    out[1::2] = ends
    return out, ids


def record_regions(data: np.ndarray) -> tuple[np.ndarray, list[str]]:
    """Sequence regions [start, end) of the FASTA records of one genome (the bytes
    after each header line, up to the next header) and the contig ids (first word
    of the header, seqtk/seqkit id; a trailing '\\r' of the header line is
    dropped).  Bytes before the first header belong to no record (seqtk skips them)."""
    from .counter import index_records
    data = np.ascontiguousarray(data, dtype=np.uint8)
    iv, _ = index_records(data, N.KF_FMT_FASTA, 0)
    se, ids = records_from_index(data, iv, 0, data.size)
    return np.asarray(se, dtype=np.uint64), ids


@dataclass
class Genome:
    """One input file of a batch and its fate (the log lines of main.py:761-885).
    Window w starts at starts[w] in the batch's processed sequence and at wpos[w]
    in its contig, whose name prefix is prefixes[wpre[w]]."""
    fname: str
    sample: str
    rec_lo: int = 0                  # its records in the batch's record table
    rec_hi: int = 0
    prefixes: list = field(default_factory=list)   # "<sample>.part_<cid>.part_<cid>_sliding__" per contig
    wpre: np.ndarray | None = None
    wpos: np.ndarray | None = None
    starts: np.ndarray | None = None
    excluded: str | None = None       # "none" (no contig >= 10 kbp) or "few"
    write: bool = True                # False: a later file has the same sample name
    # a file counted in record-aligned parts (main.record_pieces): its parts'
    # rows go to out_name, appended after the first part (cont); only the last
    # part is reported, with the file's windows (total_windows)
    out_name: str | None = None
    cont: bool = False
    last: bool = True
    total_windows: int | None = None

    @property
    def n_windows(self) -> int:
        return 0 if self.starts is None else int(self.starts.size)

    @property
    def names(self) -> list[str]:
        """Row names (main.py:905-915), built here only for tests: the writer builds them."""
        if self.starts is None:
            return []
        return [self.prefixes[int(p)] + "{}-{}".format(int(s) + 1, int(s) + CHUNK_SZ)
                for p, s in zip(self.wpre, self.wpos)]


def shadow(genomes: list[Genome]) -> None:
    """The reference writes genome by genome, so a later file with the same
    sample name replaces an earlier one's .kf: inside a batch, only the last
    written one is counted (across batches the in-order writer does it).  Only a
    file's last part decides: its earlier parts go to its side file anyway."""
    kept = set()
    for gm in reversed(genomes):
        gm.write = True
        if gm.excluded is None and gm.last:
            gm.write = gm.sample not in kept
            kept.add(gm.sample)


class ChunkPipeline:
    """Batched device pre-pass + window plan + count + threaded row writer."""

    def __init__(self, counter, device: torch.device, max_windows: int, threads: int,
                 pseudocount: bool = False):
        self.counter = counter
        self.device = torch.device(device)
        self.threads = max(1, int(threads))
        self.max_windows = max(1, int(max_windows))
        self.pseudocount = bool(pseudocount)
        self.writer = ThreadPoolExecutor(max_workers=1)   # launches are written in order
        self.pending = []
        self._wbuf = None
        # count rows go back on their own stream, so the next batch's H2D (on the
        # compute stream) overlaps them (PCIe is full duplex)
        self.d2h = torch.cuda.Stream(self.device)

    # ------------------------------------------------------------ pre-pass
    def prepare(self, hb, genomes: list[Genome]) -> torch.Tensor:
        """Compact every record of the batch on the device and plan the windows of
        every genome (one device-to-host copy).  Fills genomes[i].names/starts/
        excluded; returns the processed sequence buffer (device)."""
        import time
        t0 = time.perf_counter()
        data = hb.data.numpy()
        rec_se: list[int] = []
        rec_ids: list[str] = []
        ex = hb.excl
        # the batch's header intervals, per genome (sorted, genome by genome)
        bounds = np.searchsorted(ex[0::2], hb.off) if ex.size else np.zeros(hb.off.size, np.int64)
        for g, gm in enumerate(genomes):
            lo, hi = int(hb.off[g]), int(hb.off[g + 1])
            iv = ex[2 * int(bounds[g]): 2 * int(bounds[g + 1])]
            se, ids = records_from_index(data, iv, lo, hi)
            gm.rec_lo = len(rec_ids)
            rec_se += se
            rec_ids += ids
            gm.rec_hi = len(rec_ids)
        n_rec = len(rec_ids)
        _tr("records", t0, n_rec=n_rec)
        t0 = time.perf_counter()
        dev = self.device
        stream = torch.cuda.current_stream(dev)
        total = int(hb.off[-1])
        d_bytes = hb.data.to(dev, non_blocking=True)
        d_out = torch.empty(max(total, 16) + 16, dtype=torch.uint8, device=dev)
        if n_rec:
            host_se = torch.from_numpy(np.asarray(rec_se, dtype=np.int64))
            if hb.data.is_pinned():
                host_se = host_se.pin_memory()
            d_se_in = host_se.to(dev, non_blocking=True)
            d_se = torch.empty(2 * n_rec, dtype=torch.int64, device=dev)
            nwords = (total + 4095) // 4096 + 1
            scratch = torch.empty(nwords, dtype=torch.int32, device=dev)
            N.check(N.lib().kf_chunk_compact(d_bytes.data_ptr(), total, d_se_in.data_ptr(), n_rec, d_out.data_ptr(),
                                             d_se.data_ptr(), scratch.data_ptr(), nwords, stream.cuda_stream),
                    "kf_chunk_compact")
            out_se = d_se.cpu().numpy().view(np.uint64)      # the batch's one synchronising copy
        else:
            out_se = np.zeros(0, np.uint64)
        _tr("h2d_compact_d2h", t0, bytes=total)
        t0 = time.perf_counter()
        for gm in genomes:
            starts, pos_l, pre_l = [], [], []
            for r in range(gm.rec_lo, gm.rec_hi):
                a, b = int(out_se[2 * r]), int(out_se[2 * r + 1])
                L = b - a
                if L < CHUNK_SZ:                                   # seqkit seq -m 10000 (main.py:753)
                    continue
                n, step = window_plan(L)
                cid = rec_ids[r]
                pos = np.arange(n, dtype=np.int64) * step
                starts.append(a + pos)
                pos_l.append(pos)
                pre_l.append(np.full(n, len(gm.prefixes), np.uint32))
                gm.prefixes.append("{}.part_{}.part_{}_sliding__".format(gm.sample, cid, cid))
            cat = (lambda x, t: np.concatenate(x) if x else np.zeros(0, t))
            gm.starts, gm.wpos, gm.wpre = cat(starts, np.int64), cat(pos_l, np.int64), cat(pre_l, np.uint32)
            if not starts:
                gm.excluded = "none"                               # main.py:761-778
            elif gm.n_windows < CHUNK_CNT_THR:
                gm.excluded = "few"                                # main.py:845-860
        shadow(genomes)
        _tr("plan", t0, windows=sum(g.n_windows for g in genomes))
        return d_out

    # ------------------------------------------------------------ count + write
    def count_and_write(self, d_seq: torch.Tensor, genomes: list[Genome], output_dir: str) -> list:
        """Gather, count and (asynchronously) write the windows of the batch's
        kept genomes, at most max_windows per count launch.  Returns the futures
        of the batch's writes."""
        work = [g for g in genomes if g.excluded is None and g.write]
        futs = []
        if not work:
            return futs
        dev = self.device
        # flat window list of the batch, with its genome boundaries
        starts = np.concatenate([g.starts for g in work]).astype(np.int64)
        row0 = np.cumsum([0] + [g.n_windows for g in work])
        total = int(row0[-1])
        d_starts = torch.from_numpy(starts).pin_memory().to(dev, non_blocking=True)
        stream = torch.cuda.current_stream(dev)
        for w0 in range(0, total, self.max_windows):
            w1 = min(total, w0 + self.max_windows)
            nw = w1 - w0
            if self._wbuf is None or self._wbuf.numel() < nw * CHUNK_SZ:
                self._wbuf = torch.empty(nw * CHUNK_SZ, dtype=torch.uint8, device=dev)
            N.check(N.lib().kf_chunk_gather(d_seq.data_ptr(), d_starts[w0:].data_ptr(), nw, CHUNK_SZ,
                                            self._wbuf.data_ptr(), stream.cuda_stream), "kf_chunk_gather")
            from .counter import DeviceBatch
            off = torch.arange(0, (nw + 1) * CHUNK_SZ, CHUNK_SZ, dtype=torch.int64, device=dev)
            db = DeviceBatch(self._wbuf, off, torch.zeros(2, dtype=torch.int64, device=dev), nw, 0)
            counts, _ = self.counter.count(db)
            # a window has at most CHUNK_SZ - k + 1 < 2^16 k-mers: its counts cross
            # PCIe as uint16 bit patterns (half the bytes of the u32 rows)
            c16 = counts.to(torch.int16)
            del counts
            done = torch.cuda.Event()
            done.record(stream)
            self.d2h.wait_event(done)
            host = torch.empty(c16.shape, dtype=torch.int16, pin_memory=True)
            with torch.cuda.stream(self.d2h):
                host.copy_(c16, non_blocking=True)
                c16.record_stream(self.d2h)
                ev = torch.cuda.Event()
                ev.record(self.d2h)
            # the segments of this launch: each genome's rows inside [w0, w1)
            segs = []
            for gi, g in enumerate(work):
                a, b = max(int(row0[gi]), w0), min(int(row0[gi + 1]), w1)
                if a >= b:
                    continue
                segs.append((os.path.join(output_dir, g.out_name or "{}.kf".format(g.sample)), a - w0, b - w0, g,
                             a - int(row0[gi]), g.cont or a > int(row0[gi])))
            args = self._write_args(segs)   # built here: the writer thread only formats + writes
            if len(self.pending) >= 2:      # at most two launches queued for the writer
                self.pending.pop(0).result()
            futs.append(self.writer.submit(self._write, ev, host, args))
            self.pending.append(futs[-1])
            del c16
        return futs

    def _write_args(self, segs):
        """kf_write_kf_segments' arguments for one launch's segments (consecutive
        row ranges): paths, row bounds, append flags and the row-name parts (the
        writer builds the names from contig prefixes and window positions)."""
        import time
        t0 = time.perf_counter()
        if not segs:
            return None
        # consecutive segments of one file (the parts of a file counted in
        # record-aligned parts) are one native segment: the writer opens each
        # segment's file once and lays its rows out from the file's end
        first = [i for i in range(len(segs)) if i == 0 or segs[i][0] != segs[i - 1][0]]
        ends = [segs[j - 1][2] for j in first[1:]] + [segs[-1][2]]
        paths = (ctypes.c_char_p * len(first))(*[os.fsencode(segs[i][0]) for i in first])
        row0 = np.asarray([0] + ends, dtype=np.int32)
        app = np.asarray([1 if segs[i][5] else 0 for i in first], dtype=np.uint8)
        pre, rpre, rpos = [], [], []
        for _, a, b, g, o, _ap in segs:
            rpre.append(g.wpre[o: o + (b - a)].astype(np.uint32) + len(pre))
            rpos.append(g.wpos[o: o + (b - a)].astype(np.uint64))
            pre += g.prefixes
        rpre = np.ascontiguousarray(np.concatenate(rpre), dtype=np.uint32)
        rpos = np.ascontiguousarray(np.concatenate(rpos), dtype=np.uint64)
        enc = [x.encode(errors="surrogateescape") for x in pre]
        arr = (ctypes.c_char_p * len(enc))(*enc)
        _tr("encode_names", t0, rows=int(rpos.size))
        return (len(first), paths, row0, app, enc, arr, rpre, rpos)

    def _write(self, ev, host: torch.Tensor, args) -> None:
        """Format + write one launch's rows, once its counts are on the host."""
        import time
        t0 = time.perf_counter()
        ev.synchronize()
        _tr("wait_d2h", t0)
        if args is None:
            return
        t0 = time.perf_counter()
        n_seg, paths, row0, app, _enc, arr, rpre, rpos = args
        rows = host.numpy().view(np.uint16)
        N.check(N.lib().kf_write_kf_segments16(n_seg, paths, row0.ctypes.data, app.ctypes.data, None, arr,
                                               rpre.ctypes.data, rpos.ctypes.data, CHUNK_SZ, rows.ctypes.data,
                                               rows.shape[1], int(self.pseudocount), 1, self.threads),
                "kf_write_kf_segments16")
        _tr("format_write", t0, segs=n_seg)

    def after_writes(self, fn):
        """Run fn on the writer thread once every write queued so far is done
        (the writer runs in order); returns its future."""
        f = self.writer.submit(fn)
        self.pending.append(f)
        return f

    def drain(self) -> None:
        """Wait for every queued write."""
        while self.pending:
            self.pending.pop(0).result()

    def close(self) -> None:
        self.drain()
        self.writer.shutdown()
