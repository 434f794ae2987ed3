"""Interleaved A/B timing of count-kernel variants in ONE process (guide §5.4 rule 24).

  python tools/ab_bench.py --variants 0,1 --k 7 --rounds 5 --reps 5 [--genomes 1000]

Each variant is selected with KF_COUNT_VARIANT; the batch (synthetic, device
generated) is shared; outputs are compared bit-for-bit across variants.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,1")
    ap.add_argument("--k", type=int, default=7)
    ap.add_argument("--genomes", type=int, default=1000)
    ap.add_argument("--seq-len", type=int, default=5_000_000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--n-period", type=int, default=0)
    ap.add_argument("--accumulate", action="store_true", help="zero outside the events, accumulate=True")
    ap.add_argument("--weights", default="", help="';'-separated KF_WAVE_WEIGHTS sets, alternated per round")
    ap.add_argument("--env", default="", help="';'-separated sets of NAME=VAL[,NAME=VAL] (e.g. KF_DYN_FRAC=0.8), "
                    "alternated per round like --weights")
    args = ap.parse_args()
    import torch
    from kf2vecfsw_amd import counter as C
    dev = torch.device("cuda:0")
    db = C.synth_device_batch(args.genomes, args.seq_len, 20260101, n_period=args.n_period, device=dev)
    kc = C.KmerCounter(args.k, dev)
    fasta = int(db.off[-1].item())
    wsets = args.weights.split(";") if args.weights else [""]
    if args.env:
        wsets = args.env.split(";")
    env_names = {kv.split("=")[0] for w in wsets for kv in w.split(",") if "=" in kv}
    variants = [(int(v), w) for v in args.variants.split(",") for w in wsets]
    times = {v: [] for v in variants}
    ref = None
    for r in range(args.rounds):
        for v, w in variants:
            os.environ["KF_COUNT_VARIANT"] = str(v)
            if args.env:
                for n in env_names:
                    os.environ.pop(n, None)
                for kv in w.split(","):
                    if "=" in kv:
                        os.environ[kv.split("=")[0]] = kv.split("=", 1)[1]
            elif w:
                os.environ["KF_WAVE_WEIGHTS"] = w
            else:
                os.environ.pop("KF_WAVE_WEIGHTS", None)
            cnt, tot = kc.alloc_out(args.genomes)
            kc.count(db, cnt, tot)  # warm (also selects/caches the variant's grid)
            torch.cuda.synchronize()
            evs = []
            for _ in range(args.reps):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                if args.accumulate:   # count-matrix memset outside the events, atomics-only flushes
                    cnt.zero_()
                    tot.zero_()
                a.record()
                kc.count(db, cnt, tot, accumulate=args.accumulate)   # default: the CLI's and bench.py's call
                b.record()
                evs.append((a, b))
            torch.cuda.synchronize()
            times[(v, w)] += [a.elapsed_time(b) for a, b in evs]
            h = C.counts_to_numpy(cnt)
            if ref is None:
                ref = h
            elif not np.array_equal(ref, h):
                print(f"variant {v}: COUNTS DIFFER from variant {variants[0]}", flush=True)
    out = {}
    for v in variants:
        t = np.array(times[v])
        out[f"{v[0]}" + (f"/{v[1]}" if v[1] else "")] = {"median_ms": float(np.median(t)), "min_ms": float(t.min()),
                  "GBps_median": fasta / (np.median(t) * 1e-3) / 1e9,
                  "Gbases_s": args.genomes * args.seq_len / (np.median(t) * 1e-3) / 1e9,
                  "grid": kc.launch_info() if False else None}
    print(json.dumps({"k": args.k, "genomes": args.genomes, "bytes": fasta, "results": out}, indent=1))


if __name__ == "__main__":
    main()
