"""Round 4: why the first ~10 k=7 launches after the batch is generated run slower
than the steady state.  Per-launch HIP-event times in
several scenarios, with the GPU's sclk / mclk DPM levels sampled from sysfs by a
host thread (timestamps re-based on the first launch's start event).

  python tools/r04_cold.py [--k 7] [--genomes 1000] > gpurun_out/cold.json
"""
import argparse
import glob
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def dpm_files():
    out = {}
    for f in sorted(glob.glob("/sys/class/drm/card*/device/pp_dpm_*clk")):
        out[os.path.basename(f)[7:] + ":" + f.split("/")[4]] = f
    return out


def read_level(path):
    try:
        for ln in open(path):
            if ln.rstrip().endswith("*"):
                return ln.split(":", 1)[1].strip().rstrip("*").strip()
    except OSError:
        return None
    return None


class Sampler(threading.Thread):
    def __init__(self, files, period=0.002):
        super().__init__(daemon=True)
        self.files, self.period, self.stop, self.rows = files, period, False, []

    def run(self):
        while not self.stop:
            t = time.perf_counter()
            self.rows.append((t, {k: read_level(f) for k, f in self.files.items()}))
            time.sleep(self.period)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=7)
    ap.add_argument("--genomes", type=int, default=1000)
    ap.add_argument("--seq-len", type=int, default=5_000_000)
    args = ap.parse_args()
    import torch
    from kf2vecfsw_amd import _native as N
    from kf2vecfsw_amd import counter as C
    dev = torch.device("cuda:0")
    files = {k: f for k, f in dpm_files().items() if k.startswith(("sclk", "mclk", "fclk", "socclk"))}
    smp = Sampler(files)
    smp.start()
    t_gen0 = time.perf_counter()
    db = C.synth_device_batch(args.genomes, args.seq_len, 20260101, device=dev)
    torch.cuda.synchronize()
    t_gen1 = time.perf_counter()
    kc = C.KmerCounter(args.k, dev)
    out = kc.alloc_out(db.n)
    stream = torch.cuda.current_stream(dev)
    probe_out = torch.zeros(1, dtype=torch.int32, device=dev)
    nbytes = (db.data.numel() // 16) * 16

    def launches(n, tag, pre=None):
        evs = []
        t_host = time.perf_counter()
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        if pre is not None:
            pre()
        for _ in range(n):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            kc.count(db, out[0], out[1])
            b.record(stream)
            evs.append((a, b))
        torch.cuda.synchronize()
        ms = [a.elapsed_time(b) for a, b in evs]
        starts = [e0.elapsed_time(a) for a, _ in evs]
        return {"tag": tag, "t_host": t_host, "ms": [round(x, 4) for x in ms],
                "start_ms": [round(x, 3) for x in starts]}

    def probe(reps):
        def f():
            for _ in range(reps):
                N.check(N.lib().kf_stream_probe(db.data.data_ptr(), nbytes, probe_out.data_ptr(), stream.cuda_stream))
        return f

    def spin(ms):   # compute-only busy kernel (matmul chain), ~ms
        x = torch.randn(4096, 4096, device=dev, dtype=torch.float16)

        def f():
            y = x
            for _ in range(max(1, int(ms / 0.1))):
                y = y @ x
        return f

    def copies(reps):
        dst = torch.empty(nbytes, dtype=torch.uint8, device=dev)

        def f():
            for _ in range(reps):
                dst.copy_(db.data[:nbytes])
        return f

    def count_untimed(reps):
        def f():
            for _ in range(reps):
                kc.count(db, out[0], out[1])
        return f

    res = {"gen_s": round(t_gen1 - t_gen0, 3), "dpm_files": files, "runs": []}
    res["runs"].append(launches(40, "after_gen"))
    for tag, pre in [("idle_none", None), ("idle_probe60_copy6", lambda: (probe(61)(), copies(6)())),
                     ("idle_probe120", probe(120)), ("idle_count30", count_untimed(30)),
                     ("idle_matmul", spin(50)), ("idle_none_b", None)]:
        time.sleep(1.0)
        res["runs"].append(launches(30, tag, pre))
    res["runs"].append(launches(30, "steady"))
    smp.stop = True
    smp.join()
    t0 = res["runs"][0]["t_host"]
    res["dpm"] = [(round((t - t0) * 1e3, 2), v) for t, v in smp.rows]
    for r in res["runs"]:
        r["t_host"] = round((r["t_host"] - t0) * 1e3, 2)
        m = np.array(r["ms"])
        r["summary"] = {"first5": round(float(m[:5].mean()), 4), "first10": round(float(m[:10].mean()), 4),
                        "last10": round(float(m[-10:].mean()), 4), "min": round(float(m.min()), 4)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
