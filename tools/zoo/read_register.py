"""Rejected read path (round 5), kept for re-measurement only -- not imported
by the product.  The files of a batch are mmap'ed and page-locked in place
(hipHostRegister) so the DMA engine copies them from the page cache.  Measured
slower than the native pread reader (18.8 vs 68.9 GB/s
on 16 threads; the CLI took 51-62 ms against 27-31 ms), so it left the CLI in
round 6.  Use with tools/host_register_probe.py."""
from __future__ import annotations

import os
from typing import Sequence

import numpy as np
import torch

from kf2vecfsw_amd import _native as N
from kf2vecfsw_amd.counter import ALIGN, HostBatch, _layout, index_records


class RegisteredFiles:
    """The files of a batch mapped (mmap) and page-locked in place
    (hipHostRegister), so the DMA engine copies them from the page cache: no host
    memcpy of the bytes.  release() after the copies ran."""

    def __init__(self):
        self.maps: list = []   # (mmap, numpy view, registered pointer or 0)

    def add(self, path: str, size: int):
        import mmap
        fd = os.open(path, os.O_RDONLY)
        try:
            m = mmap.mmap(fd, size, prot=mmap.PROT_READ)
        finally:
            os.close(fd)
        a = np.frombuffer(m, dtype=np.uint8)
        rc = int(torch.cuda.cudart().cudaHostRegister(a.ctypes.data, size, 0))   # hipHostRegisterDefault
        self.maps.append((m, a, a.ctypes.data if rc == 0 else 0))
        if rc != 0:
            raise N.NativeError(f"hipHostRegister failed ({rc}) on {path}")
        return a

    def release(self) -> None:
        cr = torch.cuda.cudart()
        for m, a, ptr in self.maps:
            if ptr:
                cr.cudaHostUnregister(ptr)
        self.maps = []


def pack_files_registered(paths: Sequence[str], names: Sequence[str], device: torch.device, stream,
                          fmt: int = N.KF_FMT_AUTO) -> HostBatch:
    """As pack_files, but the bytes go from each file's page-cache pages straight
    to a device batch buffer on `stream` (mmap + hipHostRegister; '\n' padding
    between genomes filled on the device).  FASTQ files are indexed on the host
    from the mapping; a batch of FASTA files leaves its record index to the
    device (excl None).  The returned batch carries `reg` (release it once the
    copies have run: after dev_event)."""
    sizes = [os.path.getsize(p) for p in paths]
    off = _layout(sizes)
    reg = RegisteredFiles()
    excl, fastq = [], False
    with torch.cuda.stream(stream):
        dev = torch.empty(max(int(off[-1]), ALIGN) + ALIGN, dtype=torch.uint8, device=device)
        dev.fill_(10)
        for i, p in enumerate(paths):
            if sizes[i] == 0:
                excl.append(np.zeros(0, np.uint64))
                continue
            a = reg.add(p, sizes[i])
            lo = int(off[i])
            dev[lo: lo + sizes[i]].copy_(torch.from_numpy(a), non_blocking=True)
            if fmt == N.KF_FMT_FASTQ or (fmt == N.KF_FMT_AUTO and a[0] == ord("@")):
                fastq = True
            excl.append(None)
        ev = torch.cuda.Event()
        ev.record(stream)
    if fastq:   # any FASTQ file: the whole batch's record index on the host (from the mappings)
        maps = iter(reg.maps)
        full = []
        for i in range(len(paths)):
            if sizes[i] == 0:
                continue
            a = next(maps)[1]
            full.append(index_records(a, fmt, int(off[i]))[0])
        ex = np.concatenate(full) if full else np.zeros(0, np.uint64)
        hb = HostBatch(None, off, ex.astype(np.uint64), list(names), dev_data=dev, dev_event=ev)
        hb.reg = reg
        return hb
    hb = HostBatch(None, off, None, list(names), dev_data=dev, dev_event=ev)
    hb.reg = reg
    return hb
