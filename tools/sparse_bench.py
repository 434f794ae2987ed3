"""Throughput of the sparse counter (kf_sparse_count: get_kmers at k = 13..31)
on device-resident synthetic genomes, with the oracle's sort-based CPU
restatement timed on one genome beside it.

    python tools/sparse_bench.py --genomes 64 --k 21,31 --reps 5
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--genomes", type=int, default=64)
    ap.add_argument("--seq-len", type=int, default=5_000_000)
    ap.add_argument("--k", default="13,16,17,21,31")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import numpy as np
    import torch
    from kf2vecfsw_amd import counter as C

    dev = torch.device("cuda:0")
    db = C.synth_device_batch(a.genomes, a.seq_len, 99, device=dev)
    off = C.synth_layout(a.genomes, a.seq_len)
    nbytes = int(off[-1])
    bases = a.genomes * a.seq_len
    out = {"genomes": a.genomes, "seq_len": a.seq_len, "batch_bytes": nbytes, "k": {}}
    for k in [int(x) for x in a.k.split(",")]:
        sc = C.SparseCounter(k, dev)
        ms = []
        for r in range(a.reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            keys, cnts, nu = sc.count(db, nbytes)
            e1.record()
            torch.cuda.synchronize()
            if r:
                ms.append(e0.elapsed_time(e1))
        nuh = nu.cpu().numpy()
        try:
            g0 = sc.to_host(keys[: int(off[1])], cnts[: int(off[1])], nu[:1], off[:2])[0]
            ok = int(g0[1].sum(dtype=np.uint64)) == a.seq_len - k + 1
            import kf_oracle as O
            ek, ec = O.sparse_count(db.data[int(off[0]): int(off[1])].cpu().numpy().tobytes(), k)
            ok = ok and bool(np.array_equal(g0[0], ek) and np.array_equal(g0[1], ec))
        except Exception as e:   # profiling ablation builds (KF_SPARSE_ABL) sort wrongly by design
            ok = f"no: {e}"
        med = float(np.median(ms))
        out["k"][k] = {"ms": round(med, 3), "ms_all": [round(x, 3) for x in ms],
                       "Gbases_s": round(bases / med / 1e6, 2),
                       "workspace_GB": round(sc.workspace_bytes(nbytes, a.genomes) / 1e9, 2),
                       "distinct_per_genome": int(nuh.mean()), "totals_ok": ok}
        del keys, cnts, nu, sc
        torch.cuda.empty_cache()
        print(json.dumps({k: out["k"][k]}), file=sys.stderr, flush=True)
    # CPU: the oracle (one thread, qsort) on one genome
    import kf_oracle as O
    g = db.data[int(off[0]): int(off[1])].cpu().numpy().tobytes()
    t0 = time.perf_counter()
    O.sparse_count(g, 31)
    out["cpu_oracle_one_genome_k31_s"] = round(time.perf_counter() - t0, 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
