"""Host-side window plan of kf2vec's ``get_chunks`` (reference kf2vec/main.py:654-929).

The reference shells out per genome to
* ``seqtk seq -l 0`` to linearise records (:732);
* ``awk gsub(/[N|n]+/,"N")`` to collapse N runs (:740-742);
* ``seqkit seq -m 10000 -g -v`` to drop short contigs and gaps (:753);
* ``seqkit split`` and ``seqkit sliding`` to make windows (:784, :824, :837).

Then it runs one ``get_frequencies -raw_cnt`` (a Jellyfish pair) per 10 kbp window
(:869-881). Here the plan is computed in memory. All windows of a batch of genomes
become one device batch for ``KmerCounter``: one kernel launch instead of one
Jellyfish process pair per window.
"""
from __future__ import annotations

import math
import re

CHUNK_SZ = 10000       # main.py:100
CHUNK_CNT_THR = 5      # main.py:101

_NRUN = re.compile(rb"[N|n]+")      # awk regex of main.py:740 ('|' is inside the class)
_GAPS = re.compile(rb"[- \t.]")     # seqkit seq -g default gap letters


def fasta_records(data: bytes) -> list[tuple[bytes, bytes]]:
    """``seqtk seq -l 0``: (header line without '>', linear sequence) per record."""
    recs = []
    name, seq = None, []
    for line in data.split(b"\n"):
        if line.endswith(b"\r"):
            line = line[:-1]
        if line.startswith(b">"):
            if name is not None:
                recs.append((name, b"".join(seq)))
            name, seq = line[1:], []
        elif name is not None:
            seq.append(line)
    if name is not None:
        recs.append((name, b"".join(seq)))
    return recs


def window_plan(total_length: int) -> tuple[int, int]:
    """(number of windows, step) for a contig of this length (main.py:813-818)."""
    total_chunks = math.ceil(total_length / CHUNK_SZ)
    ovrlap = int(math.ceil((total_chunks * CHUNK_SZ - total_length) / (total_chunks - 1))) \
        if total_chunks != 1 else 0
    step = CHUNK_SZ - ovrlap
    n = 0 if total_length < CHUNK_SZ else (total_length - CHUNK_SZ) // step + 1   # seqkit sliding, non-greedy
    return n, step


def genome_windows(fna: bytes, sample: str) -> list[tuple[str, bytes]]:
    """(chunk sample name, window bases) in output row order.

    Contigs come in FASTA order. The reference concatenates in the `os.listdir`
    order of its split-contig files (main.py:792), so row order across contigs
    is unpinned there."""
    out = []
    for hdr, seq in fasta_records(fna):
        seq = _GAPS.sub(b"", _NRUN.sub(b"N", seq))
        if len(seq) < CHUNK_SZ:
            continue
        cid = hdr.split()[0].decode(errors="surrogateescape") if hdr.split() else ""
        n, step = window_plan(len(seq))
        for i in range(n):
            s = i * step
            name = "{}.part_{}.part_{}_sliding__{}-{}".format(sample, cid, cid, s + 1, s + CHUNK_SZ)
            out.append((name, seq[s: s + CHUNK_SZ]))
    return out
