#!/usr/bin/env python3
"""Benchmark of the MI355X k-mer counter (BASELINE.json metric: Gbases/s of the
k-mer -> .kf build at k=7, and achieved HBM GB/s vs the gfx950 peak).

Workload (BASELINE.json configs[1]): per GPU 1,000 synthetic 5 Mbp genomes
(i.i.d. uniform ACGT, 80-column FASTA, header ">syn_<g>", seed 20260101+g),
generated directly in HBM.  Genomes are sharded round-robin over ranks
(rank r owns ids r, r+N, ...); no collective touches the data path.

A step = one pass of the device counter over the rank's resident batch: one
`kf_count_batch` call (k=7) as the CLI makes it, i.e. zeroing the
[genomes x 8192] count matrix and the count kernel.
The default run also times k=11 (BASELINE configs[4]) on the same batch and
reports it under "secondary"; `roofline.traffic` is the measured HBM bytes per
launch (rocprofv3 PMC, tools/pmc_traffic.py) when profiles/ holds it.
`value` = all ranks' sequence characters / max-over-ranks wall time of K steps.
`roofline.achieved` = algorithmic bytes per launch (FASTA bytes read + 4 B x
bins written) / the count kernel's average duration,
timed with HIP events on the launch stream inside the timed region.
The CPU baseline (rank 0, N=1) times the oracle's C restatement (kind "port":
Jellyfish is not installed) on a bounded sample of the same genomes.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--k 7]
  (N>1: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...)
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBPS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
SEED = 20260101


def shard_ids(n_per_rank: int, rank: int, world: int) -> tuple[int, int]:
    """Round-robin shard: rank r owns genome ids r, r+world, r+2*world, ..."""
    return rank, world


def cpu_baseline(args, ids: list[int]) -> dict:
    """Oracle C restatement on host cores over a bounded sample (~10 s of CPU work)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import kf_oracle as O
    O.build()
    threads = int(args.cpu_threads) if args.cpu_threads else min(16, os.cpu_count() or 1)
    n = min(args.cpu_sample_genomes, len(ids))
    blobs = [O.synth_genome(g, SEED + g, args.seq_len, 80) for g in ids[:n]]
    buf = np.frombuffer(b"".join(blobs), dtype=np.uint8)
    off = np.cumsum([0] + [len(b) for b in blobs]).astype(np.uint64)
    O.count_many(buf, off, args.k, 1, threads)          # warm
    t0 = time.perf_counter()
    passes = 0
    while True:
        O.count_many(buf, off, args.k, 1, threads)
        passes += 1
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds or passes >= 1000:
            break
    bases = n * args.seq_len * passes
    cpu = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": round(bases / el / 1e9, 4), "unit": "Gbases/s", "cores": threads, "kind": "port",
            "host": {"nproc": os.cpu_count(), "cpu": cpu, "jellyfish_on_path": bool(shutil.which("jellyfish"))},
            "sample": f"{n} synthetic {args.seq_len // 10**6} Mbp genomes x {passes} passes "
                      f"({el:.1f} s, oracle/kmer_oracle.c OpenMP, k={args.k})"}


def stream_ceiling(torch, data, stream) -> dict:
    """Practical HBM read ceilings on this device, measured on the resident batch
    (SURVEY section 8(d) asks for a measured ceiling beside the spec peak):
    the count kernel's own access pattern with no counting (kf_stream_probe)
    and a device-to-device copy (read + write bytes / time)."""
    from kf2vecfsw_amd import _native as N
    n = (data.numel() // 16) * 16
    out = torch.zeros(1, dtype=torch.int32, device=data.device)
    dst = torch.empty(n, dtype=torch.uint8, device=data.device)

    def timed(fn, reps=5):
        fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(reps):
            fn()
        b.record(stream)
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps * 1e-3

    def probe():
        N.check(N.lib().kf_stream_probe(data.data_ptr(), n, out.data_ptr(), stream.cuda_stream), "kf_stream_probe")

    t_probe = timed(probe)
    t_copy = timed(lambda: dst.copy_(data[:n]))
    del dst
    return {"stream_read_GBps": round(n / t_probe / 1e9, 1), "d2d_copy_GBps": round(2 * n / t_copy / 1e9, 1),
            "bytes": int(n)}


def load_traffic(k: int, workload_tag: str):
    """Measured HBM bytes per launch (tools/pmc_traffic.py output) for this k and
    workload, newest round under profiles/ first; None if not measured."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", f"traffic_k{k}.json")), reverse=True):
        try:
            t = json.load(open(f))
        except (OSError, ValueError):
            continue
        if t.get("k") == k and t.get("workload") == workload_tag:
            return int(t["traffic_bytes"]), os.path.relpath(f, ROOT)
    return None, None


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--k", type=int, default=7)
    ap.add_argument("--genomes-per-gpu", type=int, default=1000)
    ap.add_argument("--seq-len", type=int, default=5_000_000)
    ap.add_argument("--cpu-sample-genomes", type=int, default=64)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--secondary-k", type=int, default=11,
                    help="also time this k on the same batch (BASELINE configs[4]); 0 = off; N=1 only")
    ap.add_argument("--verify", type=int, default=4, help="genomes checked bit-exactly against the oracle")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knob: KF_BENCH_REHEARSE=1 runs every rank on cuda:0 over gloo (one
    # GPU box); the real multi-GPU run uses one GPU per rank over RCCL
    rehearse = os.environ.get("KF_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from kf2vecfsw_amd import build as B
    B.build()
    from kf2vecfsw_amd import counter as C

    n = args.genomes_per_gpu
    g0, gs = shard_ids(n, rank, world)
    ids = C.synth_ids(n, g0, gs)
    db = C.synth_device_batch(n, args.seq_len, SEED, width=80, g0=g0, g_stride=gs, device=dev)
    stream = torch.cuda.current_stream(dev)
    torch.cuda.synchronize(dev)
    fasta_bytes = sum(C.synth_fasta_bytes(args.seq_len, 80, g) for g in ids)
    bases = n * args.seq_len
    workload_tag = f"{n} synthetic {args.seq_len / 1e6:g} Mbp genomes, 80-column FASTA"

    def run(k, steps, warmup):
        """`warmup` untimed + `steps` timed steps at k over the resident batch.
        A step = one kf_count_batch call (count-matrix memset + kernel).  Returns
        (counter, counts, totals, wall s, mean kernel ms by HIP events on the
        launch stream), both max over ranks."""
        kc = C.KmerCounter(k, dev)
        counts, totals = kc.alloc_out(n)

        # the same call the CLI makes (accumulate=False): for k <= 8 it zeroes the
        # count matrix inside kf_count_batch, so the events bracket that memset and
        # the count kernel; the k >= 9 bucket kernels write every row themselves

        def step(ev=None):
            if ev is not None:
                ev[0].record(stream)
            kc.count(db, counts, totals, accumulate=False)
            if ev is not None:
                ev[1].record(stream)

        for _ in range(warmup):
            step()
        torch.cuda.synchronize(dev)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(steps):
            step(evs[i])
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
        if world > 1:
            t = torch.tensor([el, kern_ms], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el, kern_ms = float(t[0]), float(t[1])
        return kc, counts, totals, el, kern_ms

    def verify(k, counts, totals):
        """totals are analytic for N-free synthetic genomes; a few genomes bit-exact vs the oracle"""
        tot = totals.cpu().numpy()
        ok = bool((tot == args.seq_len - k + 1).all())
        if args.verify and rank == 0:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import kf_oracle as O
            cnp = C.counts_to_numpy(counts)
            pick = np.linspace(0, n - 1, min(args.verify, n)).astype(int)
            for i in pick:
                c, t = O.count(O.synth_genome(ids[i], SEED + ids[i], args.seq_len, 80), k)
                ok &= bool((cnp[i] == c).all()) and int(tot[i]) == t
        if world > 1:
            f = torch.tensor([0.0 if ok else 1.0], device=dev)
            dist.all_reduce(f, op=dist.ReduceOp.MAX)
            ok = float(f) == 0.0
        return ok

    kc, counts, totals, el, kern_ms = run(args.k, args.steps, args.warmup)
    ceiling = stream_ceiling(torch, db.data, stream) if rank == 0 else None
    alg_bytes = fasta_bytes + 4 * kc.nbins * n          # per launch
    ok = verify(args.k, counts, totals)
    grid, block, lds = kc.launch_info()
    del counts, totals

    value = bases * world / el * args.steps / 1e9
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    traffic, traffic_src = load_traffic(args.k, workload_tag)
    out = {
        "metric": "Gbases/s k-mer→.kf build at k=7; achieved HBM GB/s vs gfx950 peak",
        "value": round(value, 3),
        "unit": "Gbases/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (device-generated, seeded splitmix64; no datasets)",
        "config": {"workload": f"{'1' if world == 1 else world}xMI355X, k={args.k}, {n} synthetic "
                               f"{args.seq_len / 1e6:g} Mbp genomes per GPU "
                               + ("(BASELINE configs[1])" if world == 1 else
                                  "(BASELINE configs[3] scaling curve, weak: fixed batch per GPU)"),
                   "k": args.k, "genomes_per_gpu": n, "seq_len": args.seq_len, "line_width": 80,
                   "global_batch": n * world, "parallelism": f"round-robin genome shards x{world}, no collective",
                   "kernel_grid": [grid, block], "lds_bytes": lds},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                     "frac": round(achieved / PEAK_HBM_GBPS, 4), "traffic": traffic,
                     "traffic_source": traffic_src,
                     "kernel_ms": round(kern_ms, 4), "alg_bytes_per_launch": int(alg_bytes),
                     "measured_ceiling": ceiling},
        "parity": "ok" if ok else "MISMATCH",
    }
    if args.secondary_k and world == 1 and args.secondary_k != args.k:
        k2 = args.secondary_k
        kc2, c2, t2, el2, km2 = run(k2, max(3, args.steps // 4), 1)
        ok2 = verify(k2, c2, t2)
        ok &= ok2
        alg2 = fasta_bytes + 4 * kc2.nbins * n
        tr2, src2 = load_traffic(k2, workload_tag)
        out["secondary"] = {
            "config": f"1xMI355X, k={k2} (BASELINE configs[4]), same batch",
            "value": round(bases / el2 * max(3, args.steps // 4) / 1e9, 3), "unit": "Gbases/s",
            "ms_per_step": round(el2 / max(3, args.steps // 4) * 1e3, 4),
            "roofline": {"bound": "hbm", "achieved": round(alg2 / (km2 * 1e-3) / 1e9, 1), "peak": PEAK_HBM_GBPS,
                         "unit": "GB/s", "frac": round(alg2 / (km2 * 1e-3) / 1e9 / PEAK_HBM_GBPS, 4),
                         "traffic": tr2, "traffic_source": src2, "kernel_ms": round(km2, 4),
                         "alg_bytes_per_launch": int(alg2)},
            "parity": "ok" if ok2 else "MISMATCH"}
        out["parity"] = "ok" if ok else "MISMATCH"
        del c2, t2
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(args, ids)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
