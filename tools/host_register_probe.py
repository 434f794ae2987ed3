"""Probe: can the get_frequencies readers hand the page cache straight to the
DMA engine instead of copying every file into pinned memory?

For N files of ~5 MB in /dev/shm, time per file and in aggregate:
  * read:      readinto a reused pinned buffer (what the CLI does today), then H2D;
  * register:  mmap + hipHostRegister of the mapping, H2D from it, unregister;
  * pageable:  H2D from the plain mmap (the runtime stages it itself).

  python tools/host_register_probe.py [--files 64] [--mb 5]
"""
import argparse
import json
import mmap
import os
import shutil
import tempfile
import time

import numpy as np
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=64)
    ap.add_argument("--mb", type=float, default=5.0)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    cr = torch.cuda.cudart()
    work = tempfile.mkdtemp(prefix="kf_probe_", dir="/dev/shm" if os.access("/dev/shm", os.W_OK) else None)
    try:
        size = int(a.mb * (1 << 20))
        paths = []
        rng = np.random.default_rng(1)
        blob = rng.integers(65, 90, size=size, dtype=np.uint8).tobytes()
        for i in range(a.files):
            p = os.path.join(work, f"f{i}.fna")
            with open(p, "wb") as f:
                f.write(blob)
            paths.append(p)
        total = size * a.files
        dst = torch.empty(total + 4096, dtype=torch.uint8, device=dev)
        pinned = torch.empty(total, dtype=torch.uint8, pin_memory=True)
        out = {"files": a.files, "bytes": total}
        s = torch.cuda.Stream(dev)

        def gbps(t):
            return round(total / t / 1e9, 2)

        # read into pinned + one H2D
        res = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            d = pinned.numpy()
            for i, p in enumerate(paths):
                with open(p, "rb", buffering=0) as f:
                    f.readinto(memoryview(d[i * size:(i + 1) * size]))
            t1 = time.perf_counter()
            with torch.cuda.stream(s):
                dst[:total].copy_(pinned, non_blocking=True)
            s.synchronize()
            t2 = time.perf_counter()
            res.append((t1 - t0, t2 - t1))
        r = min(res)
        out["read_pinned_1thread"] = {"read_s": round(r[0], 4), "read_GBps": gbps(r[0]), "h2d_s": round(r[1], 4),
                                      "h2d_GBps": gbps(r[1])}

        # per-thread read rate into pageable vs pinned memory, and 16 threads into pinned
        from concurrent.futures import ThreadPoolExecutor
        pageable = np.empty(total, dtype=np.uint8)

        def read_into(d, i):
            with open(paths[i], "rb", buffering=0) as f:
                f.readinto(memoryview(d[i * size:(i + 1) * size]))

        for name, d in (("pageable", pageable), ("pinned", pinned.numpy())):
            ts = []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                for i in range(len(paths)):
                    read_into(d, i)
                ts.append(time.perf_counter() - t0)
            out[f"read_1thread_{name}_GBps"] = gbps(min(ts))
        for nt in (4, 8, 16):
            ts = []
            with ThreadPoolExecutor(nt) as ex:
                for _ in range(a.reps):
                    t0 = time.perf_counter()
                    list(ex.map(lambda i: read_into(pinned.numpy(), i), range(len(paths))))
                    ts.append(time.perf_counter() - t0)
            out[f"read_{nt}threads_pinned_GBps"] = gbps(min(ts))

        # mmap + hipHostRegister + H2D per file + unregister
        res = []
        for _ in range(a.reps):
            maps, regs = [], []
            t0 = time.perf_counter()
            for p in paths:
                fd = os.open(p, os.O_RDONLY)
                m = mmap.mmap(fd, 0, prot=mmap.PROT_READ)
                os.close(fd)
                arr = np.frombuffer(m, dtype=np.uint8)
                ptr = arr.ctypes.data
                rc = cr.cudaHostRegister(ptr, arr.size, 0)   # hipHostRegisterDefault
                maps.append((m, arr))
                regs.append((ptr, int(rc)))
            t1 = time.perf_counter()
            with torch.cuda.stream(s):
                for i, (m, arr) in enumerate(maps):
                    dst[i * size:(i + 1) * size].copy_(torch.from_numpy(arr), non_blocking=True)
            s.synchronize()
            t2 = time.perf_counter()
            for ptr, rc in regs:
                if rc == 0:
                    cr.cudaHostUnregister(ptr)
            t3 = time.perf_counter()
            for m, arr in maps:
                del arr
            res.append((t1 - t0, t2 - t1, t3 - t2, [rc for _, rc in regs][:3]))
        r = min(res, key=lambda x: x[0] + x[1] + x[2])
        out["mmap_register"] = {"register_s": round(r[0], 4), "register_GBps": gbps(r[0]), "h2d_s": round(r[1], 4),
                                "h2d_GBps": gbps(r[1]), "unregister_s": round(r[2], 4), "rc": r[3],
                                "sum_GBps": gbps(r[0] + r[1] + r[2])}
        # correctness of the registered copy
        out["mmap_register"]["bytes_equal"] = bool(
            (dst[:size].cpu().numpy() == np.frombuffer(blob, np.uint8)).all())

        # pageable mmap H2D (runtime staging)
        res = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            maps = []
            for p in paths:
                fd = os.open(p, os.O_RDONLY)
                m = mmap.mmap(fd, 0, prot=mmap.PROT_READ)
                os.close(fd)
                maps.append((m, np.frombuffer(m, dtype=np.uint8)))
            with torch.cuda.stream(s):
                for i, (m, arr) in enumerate(maps):
                    dst[i * size:(i + 1) * size].copy_(torch.from_numpy(arr), non_blocking=True)
            s.synchronize()
            res.append(time.perf_counter() - t0)
        out["mmap_pageable_h2d"] = {"s": round(min(res), 4), "GBps": gbps(min(res))}
        print(json.dumps(out))
    finally:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
