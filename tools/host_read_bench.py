"""Host side of the CLI path on the GPU box: file read into pinned memory
(readinto, one thread per file) and record indexing, alone and as pack_files
batches, to size the CLI pipeline's reader stage.

  python tools/host_read_bench.py [--genomes 64] [--threads 16]
"""
import argparse
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--genomes", type=int, default=64)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--dir", default="/tmp/kf_hostread")
    a = ap.parse_args()
    from e2e_bench import bacterial_like
    from kf2vecfsw_amd import counter as C
    os.makedirs(a.dir, exist_ok=True)
    rng = np.random.default_rng(1)
    paths = []
    for g in range(a.genomes):
        p = os.path.join(a.dir, "B%04d.fna" % g)
        with open(p, "wb") as f:
            f.write(bacterial_like(rng))
        paths.append(p)
    tot = sum(os.path.getsize(p) for p in paths)
    pool = ThreadPoolExecutor(a.threads)

    def best(fn, reps=4):
        b = 1e9
        for _ in range(reps):
            t = time.perf_counter()
            fn()
            b = min(b, time.perf_counter() - t)
        return b

    res = {}
    res["pack_all"] = tot / best(lambda: C.pack_files(paths, pool=pool)) / 1e9
    q = len(paths) // 4
    quarters = [paths[i * q:(i + 1) * q] for i in range(4)]
    res["pack_quarter"] = (tot / 4) / best(lambda: C.pack_files(quarters[0], pool=pool)) / 1e9
    two = ThreadPoolExecutor(2)
    res["pack_two_quarters_concurrent"] = (tot / 2) / best(
        lambda: list(two.map(lambda ps: C.pack_files(ps, pool=pool), quarters[:2]))) / 1e9
    hb = C.pack_files(paths, pool=pool)
    d = hb.data.numpy()
    t = time.perf_counter()
    for i in range(hb.n):
        C.index_records(d[int(hb.off[i]): int(hb.off[i + 1])], 0, int(hb.off[i]))
    res["index_1thread"] = tot / (time.perf_counter() - t) / 1e9
    print({k: round(v, 2) for k, v in res.items()}, "GB/s")


if __name__ == "__main__":
    main()
