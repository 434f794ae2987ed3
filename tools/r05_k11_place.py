"""k=11 bucket kernel time against where its scratch (records) lands: in one
process, release and re-reserve the library workspace behind torch pads of
several sizes, then time the launch (profiling build: KF_BUCKET_DEBUG prints the
scratch address).

  KF2VEC_GPU_LIB=kf2vecfsw_amd/libkf2vec_gpu_ablation.so KF_BUCKET_DEBUG=1 python tools/r05_k11_place.py
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=11)
    ap.add_argument("--pads-mb", default="0,2,64,512,1024,0,2,4096,0,8192,2")
    ap.add_argument("--reps", type=int, default=6)
    a = ap.parse_args()
    import torch
    from kf2vecfsw_amd import _native as N
    from kf2vecfsw_amd import counter as C
    dev = torch.device("cuda:0")
    db = C.synth_device_batch(1000, 5_000_000, 20260101, device=dev)
    kc = C.KmerCounter(a.k, dev)
    cnt, tot = kc.alloc_out(db.n)
    stream = torch.cuda.current_stream(dev)
    pads, res = [], []
    for mb in [int(x) for x in a.pads_mb.split(",")]:
        torch.cuda.synchronize()
        N.check(N.lib().kf_workspace_release(), "release")
        if mb:
            pads.append(torch.empty(mb << 20, dtype=torch.uint8, device=dev))
        kc.reserve(db.n)
        kc.count(db, cnt, tot)
        torch.cuda.synchronize()
        ms = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            kc.count(db, cnt, tot)
            e1.record(stream)
            torch.cuda.synchronize()
            ms.append(round(e0.elapsed_time(e1), 4))
        res.append({"pad_mb": mb, "pads_total_mb": sum(p.numel() for p in pads) >> 20,
                    "median_ms": statistics.median(ms), "ms": ms})
        print(json.dumps(res[-1]), flush=True)
    ok = bool((tot.cpu().numpy() == 5_000_000 - a.k + 1).all())
    print(json.dumps({"k": a.k, "totals_ok": ok, "runs": res}))


if __name__ == "__main__":
    main()
