"""Host-side cost of get_chunks' row writer (kf_write_kf_segments) on one launch's
rows: 4096 windows x 8192 columns of Poisson(1.2) counts (a 10 kbp window at k=7),
raw text, 8 segments; written to new files on /dev/shm (tmpfs) and, for the format-only cost,
to /dev/null.

  python tools/fmt_bench.py [--threads 8] [--rows 4096] [--reps 5]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--rows", type=int, default=4096)
    ap.add_argument("--cols", type=int, default=8192)
    ap.add_argument("--segs", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--pseudo", type=int, default=0)
    args = ap.parse_args()
    from kf2vecfsw_amd import _native as N
    rng = np.random.default_rng(1)
    counts = rng.poisson(1.2, size=(args.rows, args.cols)).astype(np.uint32)
    row0 = np.linspace(0, args.rows, args.segs + 1).astype(np.int32)
    app = np.zeros(args.segs, np.uint8)
    pre = (ctypes.c_char_p * 1)(b"sample.part_NC_000913.3.part_NC_000913.3_sliding__")
    rpre = np.zeros(args.rows, np.uint32)
    rpos = (np.arange(args.rows, dtype=np.uint64) * 9990)
    d = "/dev/shm/kf_fmt_bench"
    os.makedirs(d, exist_ok=True)
    res = {"rows": args.rows, "cols": args.cols, "threads": args.threads}
    for tag, mk in [("devnull", lambda g: b"/dev/null"), ("tmpfs", lambda g: os.fsencode(f"{d}/s{g}.kf"))]:
        paths = (ctypes.c_char_p * args.segs)(*[mk(g) for g in range(args.segs)])
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            N.check(N.lib().kf_write_kf_segments(args.segs, paths, row0.ctypes.data, app.ctypes.data, None, pre,
                                                 rpre.ctypes.data, rpos.ctypes.data, 10000, counts.ctypes.data,
                                                 args.cols, args.pseudo, 1, args.threads))
            ts.append(time.perf_counter() - t0)
            if tag == "tmpfs":   # get_chunks writes new files
                sz = sum(os.path.getsize(f"{d}/s{g}.kf") for g in range(args.segs))
                for g in range(args.segs):
                    os.unlink(f"{d}/s{g}.kf")
        res[tag + "_ms"] = round(1e3 * float(np.median(ts)), 2)
    res["bytes"] = sz
    res["tmpfs_GBps"] = round(sz / res["tmpfs_ms"] / 1e6, 2)
    res["format_GBps"] = round(sz / res["devnull_ms"] / 1e6, 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
