"""k=11: does the bucket kernel's time depend on the order in which its buffers
were allocated?  One process, four steps (profiling build: KF_BUCKET_DEBUG
prints the scratch address):
  A  scratch reserved BEFORE the count matrix (tools/r04_run.py's order);
  B  scratch released and reserved again AFTER the count matrix;
  C  a second count matrix (allocated after the scratch) replaces the first;
  D  scratch reserved again after both.

  KF2VEC_GPU_LIB=kf2vecfsw_amd/libkf2vec_gpu_ablation.so KF_BUCKET_DEBUG=1 python tools/r05_k11_order.py
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from kf2vecfsw_amd import _native as N
    from kf2vecfsw_amd import counter as C
    k = int(os.environ.get("K", "11"))
    dev = torch.device("cuda:0")
    db = C.synth_device_batch(1000, 5_000_000, 20260101, device=dev)
    kc = C.KmerCounter(k, dev)
    stream = torch.cuda.current_stream(dev)

    def timed(cnt, tot, tag, reps=8):
        kc.count(db, cnt, tot)
        torch.cuda.synchronize()
        ms = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            kc.count(db, cnt, tot)
            e1.record(stream)
            torch.cuda.synchronize()
            ms.append(round(e0.elapsed_time(e1), 4))
        ok = bool((tot.cpu().numpy() == 5_000_000 - k + 1).all())
        r = {"step": tag, "median_ms": statistics.median(ms), "ms": ms, "counts_ptr": hex(cnt.data_ptr()),
             "bytes_ptr": hex(db.data.data_ptr()), "totals_ok": ok}
        print(json.dumps(r), flush=True)
        return r

    kc.reserve(db.n)
    cnt, tot = kc.alloc_out(db.n)
    timed(cnt, tot, "A scratch before counts")
    N.check(N.lib().kf_workspace_release(), "release")
    kc.reserve(db.n)
    timed(cnt, tot, "B scratch after counts")
    cnt2, tot2 = kc.alloc_out(db.n)
    timed(cnt2, tot2, "C second counts after scratch")
    timed(cnt, tot, "C' first counts again")
    N.check(N.lib().kf_workspace_release(), "release")
    kc.reserve(db.n)
    timed(cnt2, tot2, "D scratch after both, second counts")
    timed(cnt, tot, "D' first counts")


if __name__ == "__main__":
    main()
