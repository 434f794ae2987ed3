"""Host read rate with and without a concurrent H2D stream (is the CLI's read
stage slowed by the DMA reading pinned memory beside it?).  64 bacterial-like
~5 Mbp FASTA files in /dev/shm (tools/e2e_bench.py's generator), read by
counter.pack_files on N threads into a pinned buffer: alone, then while another
thread keeps hipMemcpyAsync H2D copies of a 256 MiB pinned block busy; and the
H2D rate alone and under the reads.
  python tools/read_dma_probe.py [--threads 16] [--reps 5]"""
import argparse
import json
import os
import shutil
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--genomes", type=int, default=64)
    args = ap.parse_args()
    import torch
    from e2e_bench import bacterial_like
    from kf2vecfsw_amd import counter as C
    d = "/dev/shm/kf_probe" if os.access("/dev/shm", os.W_OK) else "/tmp/kf_probe"
    shutil.rmtree(d, ignore_errors=True)
    os.makedirs(d)
    rng = np.random.default_rng(2026)
    paths = []
    for g in range(args.genomes):
        p = os.path.join(d, "B%04d.fna" % g)
        with open(p, "wb") as f:
            f.write(bacterial_like(rng))
        paths.append(p)
    total = sum(os.path.getsize(p) for p in paths)
    dev = torch.device("cuda:0")
    buf = torch.empty(total + (1 << 20), dtype=torch.uint8, pin_memory=True)
    src = torch.empty(256 << 20, dtype=torch.uint8, pin_memory=True)
    dst = torch.empty(256 << 20, dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream(dev)

    def read_once():
        t0 = time.perf_counter()
        C.pack_files(paths, threads=args.threads, buf=buf, index=False)
        return time.perf_counter() - t0

    stop = threading.Event()
    copied = [0, 0.0]

    def dma():
        with torch.cuda.stream(s):
            t0 = time.perf_counter()
            n = 0
            while not stop.is_set():
                for _ in range(4):
                    dst.copy_(src, non_blocking=True)
                s.synchronize()
                n += 4
            copied[0], copied[1] = n * src.numel(), time.perf_counter() - t0

    def h2d_alone(reps=8):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            for _ in range(reps):
                dst.copy_(src, non_blocking=True)
        s.synchronize()
        return reps * src.numel() / (time.perf_counter() - t0) / 1e9

    read_once()
    h2d_alone()
    res = {"bytes": total, "threads": args.threads, "read_alone_GBps": [], "read_under_dma_GBps": [],
           "h2d_alone_GBps": [], "h2d_under_reads_GBps": []}
    for _ in range(args.reps):
        res["read_alone_GBps"].append(round(total / read_once() / 1e9, 1))
        res["h2d_alone_GBps"].append(round(h2d_alone(), 1))
        stop.clear()
        th = threading.Thread(target=dma)
        th.start()
        time.sleep(0.01)
        ts = [read_once() for _ in range(3)]
        stop.set()
        th.join()
        res["read_under_dma_GBps"].append(round(total / min(ts) / 1e9, 1))
        res["h2d_under_reads_GBps"].append(round(copied[0] / copied[1] / 1e9, 1))
    # H2D of the whole batch in ranges of `mb` MiB, on one stream or alternating two
    s2 = torch.cuda.Stream(dev)
    big = torch.empty(total, dtype=torch.uint8, device=dev)
    hsrc = buf[:total]
    res["h2d_chunked_GBps"] = {}
    for mb in (4, 16, 64, 320):
        for ns in (1, 2):
            best = 0.0
            for _ in range(3):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                step = mb << 20
                for i, a in enumerate(range(0, total, step)):
                    st = (s, s2)[i % ns]
                    with torch.cuda.stream(st):
                        big[a: a + step].copy_(hsrc[a: a + step], non_blocking=True)
                torch.cuda.synchronize()
                best = max(best, total / (time.perf_counter() - t0) / 1e9)
            res["h2d_chunked_GBps"][f"{mb}MiB_x{ns}"] = round(best, 1)
    print(json.dumps(res))
    shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
