"""Runs kf_count_batch `--reps` times at k on the bench batch (configs[1]:
1,000 synthetic 5 Mbp genomes generated in HBM) with the library KF2VEC_GPU_LIB
points at (default: the product): the program rocprofv3 PMC / kernel-trace
passes wrap (tools/r04_pmc.sh), and a quick per-launch timer.

  KF2VEC_GPU_LIB=tools/ab/libX.so python tools/r04_run.py --k 11 --reps 3
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=11)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--genomes", type=int, default=1000)
    ap.add_argument("--seq-len", type=int, default=5_000_000)
    ap.add_argument("--n-period", type=int, default=0)
    args = ap.parse_args()
    import torch
    from kf2vecfsw_amd import counter as C
    dev = torch.device("cuda:0")
    db = C.synth_device_batch(args.genomes, args.seq_len, 20260101, n_period=args.n_period, device=dev)
    kc = C.KmerCounter(args.k, dev)
    kc.reserve(db.n)
    cnt, tot = kc.alloc_out(db.n)
    stream = torch.cuda.current_stream(dev)
    ms = []
    for _ in range(args.reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        kc.count(db, cnt, tot)
        b.record(stream)
        torch.cuda.synchronize()
        ms.append(round(a.elapsed_time(b), 4))
    ok = bool((tot.cpu().numpy() == args.seq_len - args.k + 1).all()) if not args.n_period else None
    print(json.dumps({"k": args.k, "lib": os.environ.get("KF2VEC_GPU_LIB", "product"), "ms": ms,
                      "totals_analytic": ok}))


if __name__ == "__main__":
    main()
