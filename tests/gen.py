"""Seeded generators of adversarial FASTA/FASTQ inputs for the parity tests, and a
slow pure-Python model of the device semantics (newline-transparent byte stream
+ excluded record intervals) used on CPU to cross-check kf_index_records
against the oracle's own parser."""
from __future__ import annotations

import numpy as np

BASES = np.frombuffer(b"ACGT", dtype=np.uint8)
IUPAC = np.frombuffer(b"NRYKMSWBDHVnrykmswbdhv-.*", dtype=np.uint8)


def random_seq(rng: np.random.Generator, n: int, gc: float = 0.5, lower: float = 0.0, n_rate: float = 0.0,
               iupac_rate: float = 0.0, poly_rate: float = 0.0) -> np.ndarray:
    p = np.array([(1 - gc) / 2, gc / 2, gc / 2, (1 - gc) / 2])
    s = BASES[rng.choice(4, size=n, p=p)].copy()
    if poly_rate and n:
        for _ in range(rng.poisson(poly_rate * n / 100) + 0):
            st = int(rng.integers(0, n))
            s[st: st + int(rng.integers(5, 200))] = BASES[int(rng.integers(0, 4))]
    if n_rate and n:
        for _ in range(rng.poisson(n_rate * n / 20) + 0):
            st = int(rng.integers(0, n))
            s[st: st + int(rng.integers(1, 40))] = ord("N")
    if iupac_rate and n:
        m = rng.random(n) < iupac_rate
        s[m] = IUPAC[rng.integers(0, IUPAC.size, size=int(m.sum()))]
    if lower and n:
        m = rng.random(n) < lower
        s[m] |= 0x20
    return s


def wrap(seq: np.ndarray, width: int | None, crlf: bool = False) -> bytes:
    nl = b"\r\n" if crlf else b"\n"
    b = seq.tobytes()
    if not width:
        return b + nl
    return b"".join(b[i: i + width] + nl for i in range(0, len(b), width)) if b else b""


def random_fasta(rng: np.random.Generator, total: int, max_records: int = 5, **kw) -> bytes:
    """A multi-record FASTA genome with randomised line widths, headers, blank lines."""
    nrec = int(rng.integers(1, max_records + 1))
    cuts = np.sort(rng.integers(0, total + 1, size=nrec - 1))
    lens = np.diff(np.concatenate([[0], cuts, [total]]))
    out = []
    for i, L in enumerate(lens):
        hl = int(rng.choice([0, 3, 40, 200, 1500]))
        hdr = b">" + bytes(rng.choice(list(b"ACGTNacgt >_|.0123456789"), size=hl).tolist()) + b"\n"
        width = rng.choice([None, 1, 2, 3, 5, 6, 7, 8, 15, 16, 17, 31, 60, 61, 80, 1000])
        crlf = bool(rng.random() < kw.get("crlf_rate", 0.0))
        body = wrap(random_seq(rng, int(L), gc=float(rng.uniform(0.3, 0.7)),
                               lower=kw.get("lower", 0.0), n_rate=kw.get("n_rate", 0.0),
                               iupac_rate=kw.get("iupac_rate", 0.0), poly_rate=kw.get("poly_rate", 0.0)),
                    None if width is None else int(width), crlf)
        if rng.random() < 0.1:
            body = b"\n" + body + b"\n\n"
        out.append(hdr + body)
    data = b"".join(out)
    if rng.random() < 0.1 and data.endswith(b"\n"):
        data = data[:-1]   # unterminated last line
    return data


def random_fastq(rng: np.random.Generator, nreads: int, **kw) -> bytes:
    out = []
    for i in range(nreads):
        L = int(rng.integers(0, 300))
        seq = random_seq(rng, L, lower=kw.get("lower", 0.0), n_rate=kw.get("n_rate", 0.0))
        qual = bytes(rng.choice(list(b"ACGT!#II@+~"), size=L).tolist())
        plus = b"+" if rng.random() < 0.5 else b"+read%d" % i
        if kw.get("multiline") and L > 10:
            w = int(rng.integers(5, 60))
            s = b"".join(seq.tobytes()[j: j + w] + b"\n" for j in range(0, L, w))
            q = b"".join(qual[j: j + w] + b"\n" for j in range(0, L, w))
        else:
            s, q = seq.tobytes() + b"\n", qual + b"\n"
        out.append(b"@read%d extra\n" % i + s + plus + b"\n" + q)
    return b"".join(out)


def model_count(data: bytes, excl: np.ndarray, base: int, k: int, rank_std: np.ndarray) -> tuple[np.ndarray, int]:
    """Device semantics, byte by byte: excluded bytes and non-ACGT reset,
    '\\n' is transparent.  Slow: small inputs only."""
    code = {ord("A"): 0, ord("C"): 1, ord("G"): 2, ord("T"): 3,
            ord("a"): 0, ord("c"): 1, ord("g"): 2, ord("t"): 3}
    ex = np.zeros(len(data), dtype=bool)
    for s, e in excl.reshape(-1, 2):
        ex[int(s) - base: int(e) - base] = True
    nb = int(rank_std.max()) + 1
    counts = np.zeros(nb, dtype=np.uint32)
    mask = (1 << (2 * k)) - 1
    fw = rc = ln = 0
    total = 0
    for i, ch in enumerate(data):
        if ch == 10:
            continue
        c = None if ex[i] else code.get(ch)
        if c is None:
            ln = 0
            continue
        fw = ((fw << 2) | c) & mask
        rc = (rc >> 2) | ((3 - c) << (2 * k - 2))
        ln += 1
        if ln >= k:
            counts[rank_std[min(fw, rc)]] += 1
            total += 1
    return counts, total
