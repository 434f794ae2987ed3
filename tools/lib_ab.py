"""In-process A/B of kf_count_batch between library builds (ONE process, the same
device batch, interleaved rounds; guide rule: compare on one box, one process).

  python tools/lib_ab.py --libs kf2vecfsw_amd/libkf2vec_gpu.so,tools/zoo/libkf2vec_zoo.so --k 11

Each library is its own ctypes handle (RTLD_LOCAL: separate symbol namespaces,
one HIP runtime).  Counts are compared bit for bit between the libraries.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--k", type=int, default=7)
    ap.add_argument("--genomes", type=int, default=1000)
    ap.add_argument("--seq-len", type=int, default=5_000_000)
    ap.add_argument("--n-period", type=int, default=0)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--env", default="", help="NAME=VAL,... set before the runs")
    args = ap.parse_args()
    for kv in filter(None, args.env.split(",")):
        os.environ[kv.split("=")[0]] = kv.split("=", 1)[1]
    import torch
    from kf2vecfsw_amd import _native as N
    from kf2vecfsw_amd import counter as C
    dev = torch.device("cuda:0")
    db = C.synth_device_batch(args.genomes, args.seq_len, 20260101, n_period=args.n_period, device=dev)
    kc = C.KmerCounter(args.k, dev)   # tables (the product library's)
    libs = []
    for path in args.libs.split(","):
        L = ctypes.CDLL(os.path.join(ROOT, path) if not os.path.isabs(path) else path)
        name, (res, argt) = "kf_count_batch", N.SIGNATURES["kf_count_batch"]
        getattr(L, name).restype, getattr(L, name).argtypes = res, argt
        L.kf_last_error.restype = ctypes.c_char_p
        libs.append((path, L))
    stream = torch.cuda.current_stream(dev)
    outs = {p: kc.alloc_out(db.n) for p, _ in libs}

    def run(L, cnt, tot):
        rc = L.kf_count_batch(db.data.data_ptr(), db.off.data_ptr(), db.n, db.excl.data_ptr(), db.n_excl,
                              kc.code2col.data_ptr(), kc.col2rep.data_ptr(), args.k, cnt.data_ptr(), tot.data_ptr(),
                              0, stream.cuda_stream)
        if rc:
            raise RuntimeError(L.kf_last_error().decode())

    times = {p: [] for p, _ in libs}
    for p, L in libs:
        run(L, *outs[p])   # warm
    torch.cuda.synchronize()
    for _ in range(args.rounds):
        for p, L in libs:
            evs = []
            for _ in range(args.reps):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                run(L, *outs[p])
                b.record(stream)
                evs.append((a, b))
            torch.cuda.synchronize()
            times[p] += [a.elapsed_time(b) for a, b in evs]
    ref = None
    same = True
    for p, _ in libs:
        h = outs[p][0].cpu().numpy()
        t = outs[p][1].cpu().numpy()
        if ref is None:
            ref = (h, t)
        else:
            same &= bool(np.array_equal(ref[0], h) and np.array_equal(ref[1], t))
    fasta = int(db.off[-1].item())
    res = {p: {"median_ms": float(np.median(times[p])), "min_ms": float(np.min(times[p])),
               "Gbases_s": args.genomes * args.seq_len / (np.median(times[p]) * 1e-3) / 1e9} for p, _ in libs}
    print(json.dumps({"k": args.k, "genomes": args.genomes, "bytes": fasta, "counts_equal": same, "results": res},
                     indent=1))
    if not same:
        sys.exit(3)


if __name__ == "__main__":
    main()
