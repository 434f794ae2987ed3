#!/usr/bin/env python3
"""Benchmark of the MI355X k-mer counter (BASELINE.json metric: Gbases/s of the
k-mer -> .kf build at k=7, and achieved HBM GB/s vs the gfx950 peak).

Workloads (synthetic 5 Mbp genomes: i.i.d. uniform ACGT, 80-column FASTA,
header ">syn_<g>", seed 20260101+g, generated directly in HBM by kf_synth_fasta):
  * N = 1 (default): BASELINE.json configs[1], 1,000 genomes on one GPU;
  * N > 1 (default under torchrun): BASELINE.json configs[3], the 50,000-genome
    batch sharded round-robin -- genome g on rank g mod N, generated on that
    rank's GPU -- with no collective on the data path (`scaling: strong`: the
    total is fixed).  A rank's shard is kept resident in HBM as sub-batches of
    at most --sub-batch genomes (6,250 = the N=8 shard, 31.6 GB); if it does not
    fit (N=1 would need 253 GB) each sub-batch is generated, then timed on its
    own, and the times add up ("resident": false in the config).
  --workload configs1|configs3 forces either.

A step = one pass of the device counter over the rank's resident genomes: one
`kf_count_batch` call (k=7) per sub-batch as the CLI makes it, i.e. zeroing the
[genomes x 8192] count matrix and the count kernel.
The default run also times k=11 (BASELINE configs[4]) on the same batch and
reports it under "secondary"; `roofline.traffic` is the measured HBM bytes per
launch (rocprofv3 PMC, tools/pmc_traffic.py) when profiles/ holds it.
`value` = all ranks' sequence characters / max-over-ranks wall time of K steps.
`roofline.achieved` = algorithmic bytes per launch (FASTA bytes read + 4 B x
bins written) / the count kernel's average duration,
timed with HIP events on the launch stream inside the timed region.
The CPU baseline (rank 0, N=1) times the oracle's C restatement (kind "port":
Jellyfish is not installed) on a bounded sample of the same genomes, OpenMP
over (genome, ~1 MiB part) pairs on every host CPU this process may use
(sched_getaffinity, capped by a cgroup CPU quota if one is set).

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


CONFIG3_GENOMES = 50_000          # BASELINE.json configs[3]
SUB_BATCH = 6_250                 # genomes per resident sub-batch (the N=8 shard)


def shard_ids(n_per_rank: int, rank: int, world: int) -> tuple[int, int]:
    """Round-robin shard: rank r owns genome ids r, r+world, r+2*world, ..."""
    return rank, world


def shard_plan(total: int, rank: int, world: int, per: int = SUB_BATCH) -> list[tuple[int, int, int]]:
    """configs[3]: rank r owns the genome ids g < total with g % world == r (its
    shard, generated on its own GPU), split into sub-batches of at most `per`
    genomes.  Returns [(first id, id stride, count)] per sub-batch; every rank
    gets the same number of sub-batches (trailing ones may be empty), so the
    per-sub-batch barriers of the streamed mode match across ranks."""
    n = len(range(rank, total, world))
    n_max = len(range(0, total, world))
    nsb = max(1, -(-n_max // per))
    out = []
    for j in range(nsb):
        a, b = min(n, j * per), min(n, (j + 1) * per)
        out.append((rank + a * world, world, b - a))
    return out


def usable_cpus() -> tuple[int, dict]:
    """CPUs this process may run on: the affinity mask, capped by a cgroup v2/v1
    CPU quota if one is set (a GPU box may show the whole host in the mask)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    n = aff if quota is None else max(1, min(aff, int(quota)))
    return n, {"nproc": os.cpu_count(), "affinity": aff, "cgroup_cpu_quota": quota}


def cpu_baseline(args, ids: list[int]) -> dict:
    """Oracle C restatement on host cores over a bounded sample (~10 s of CPU work)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import kf_oracle as O
    O.build()
    usable, cpu_info = usable_cpus()
    threads = int(args.cpu_threads) if args.cpu_threads else usable
    n = min(args.cpu_sample_genomes, len(ids))
    blobs = [O.synth_genome(g, SEED + g, args.seq_len, 80) for g in ids[:n]]
    buf = np.frombuffer(b"".join(blobs), dtype=np.uint8)
    off = np.cumsum([0] + [len(b) for b in blobs]).astype(np.uint64)
    # ~8 parts per thread over the sample, 64 KiB..1 MiB each: every thread busy
    part = int(min(1 << 20, max(1 << 16, int(off[-1]) // (8 * threads))))
    O.count_many_parts(buf, off, args.k, 1, threads, part)          # warm
    t0 = time.perf_counter()
    passes = 0
    while True:
        O.count_many_parts(buf, off, args.k, 1, threads, part)
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
            "host": dict(cpu_info, cpu=cpu, jellyfish_on_path=bool(shutil.which("jellyfish"))),
            "sample": f"{n} synthetic {args.seq_len // 10**6} Mbp genomes x {passes} passes "
                      f"({el:.1f} s, oracle/kmer_oracle.c, OpenMP over genome x {part >> 10} KiB parts "
                      f"on {threads} threads, k={args.k})"}


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
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--k", type=int, default=7)
    ap.add_argument("--workload", choices=["auto", "configs1", "configs3"], default="auto",
                    help="auto: configs1 (1,000 genomes per GPU) at N=1, configs3 (50,000 genomes sharded) at N>1")
    ap.add_argument("--genomes-per-gpu", type=int, default=1000, help="configs1 batch per GPU")
    ap.add_argument("--total-genomes", type=int, default=CONFIG3_GENOMES, help="configs3 batch over all GPUs")
    ap.add_argument("--sub-batch", type=int, default=SUB_BATCH, help="configs3 genomes per resident sub-batch")
    ap.add_argument("--max-resident-gb", type=float, default=0.0,
                    help="configs3: HBM budget per rank for resident sub-batches (0 = free memory - 8 GB)")
    ap.add_argument("--seq-len", type=int, default=5_000_000)
    ap.add_argument("--cpu-sample-genomes", type=int, default=64)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every usable host CPU")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--secondary-k", type=int, default=11,
                    help="also time this k on the same batch (BASELINE configs[4]); 0 = off; N=1 only")
    ap.add_argument("--verify", type=int, default=4, help="genomes per rank checked bit-exactly against the oracle")
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

    workload = args.workload if args.workload != "auto" else ("configs1" if world == 1 else "configs3")
    if workload == "configs1":
        g0, gs = shard_ids(args.genomes_per_gpu, rank, world)
        plan = [(g0, gs, args.genomes_per_gpu)]
    else:
        plan = shard_plan(args.total_genomes, rank, world, args.sub_batch)
    n = sum(c for _, _, c in plan)                                  # this rank's genomes
    sb_bytes = [int(C.synth_layout(c, args.seq_len, 80, a, st)[-1]) if c else 0 for a, st, c in plan]
    kmax = max(args.k, args.secondary_k if (world == 1 and args.secondary_k) else 0)
    row_b = 4 * C.num_bins(kmax) + 8
    need = sum(sb_bytes) + row_b * n
    budget = args.max_resident_gb * 1e9 if args.max_resident_gb else torch.cuda.mem_get_info(dev)[0] - 8e9
    resident = need <= budget
    if world > 1:   # every rank takes the same mode (the streamed mode has per-sub-batch barriers)
        f = torch.tensor([0.0 if resident else 1.0], device=dev if not rehearse else "cpu")
        dist.all_reduce(f, op=dist.ReduceOp.MAX)
        resident = float(f) == 0.0
    stream = torch.cuda.current_stream(dev)
    bases = n * args.seq_len
    fasta_bytes = sum(C.synth_fasta_bytes(args.seq_len, 80, a + i * st) for a, st, c in plan for i in range(c))

    def gen(j):
        a, st, c = plan[j]
        if not c:
            return None
        db = C.synth_device_batch(c, args.seq_len, SEED, width=80, g0=a, g_stride=st, device=dev)
        torch.cuda.synchronize(dev)
        return db

    def barrier():
        if world > 1:
            dist.barrier()

    def run(k, steps, warmup, dbs):
        """`warmup` untimed + `steps` timed steps at k over the sub-batches `dbs`
        (None = empty).  A step = one kf_count_batch call (count-matrix memset +
        kernel) per sub-batch.  Returns (counter, outputs, wall s, HIP-event ms of
        every launch on the launch stream)."""
        kc = C.KmerCounter(k, dev)
        outs = [kc.alloc_out(db.n) if db is not None else None for db in dbs]

        def step(evs=None):
            for db, o in zip(dbs, outs):
                if db is None:
                    continue
                if evs is not None:
                    e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                    e[0].record(stream)
                kc.count(db, o[0], o[1], accumulate=False)   # the CLI's call
                if evs is not None:
                    e[1].record(stream)
                    evs.append(e)

        for _ in range(warmup):
            step()
        torch.cuda.synchronize(dev)
        evs = []
        barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            step(evs)
        torch.cuda.synchronize(dev)
        barrier()
        el = time.perf_counter() - t0
        return kc, outs, el, [a.elapsed_time(b) for a, b in evs]

    def verify(k, j, outs, picks):
        """totals are analytic for N-free synthetic genomes; `picks` genomes of
        sub-batch j bit-exact vs the oracle (the checker, outside the timed region)"""
        a, st, c = plan[j]
        ok = True
        for o in outs:
            if o is None:
                continue
            ok &= bool((o[1].cpu().numpy() == args.seq_len - k + 1).all())
        if picks and c:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import kf_oracle as O
            cnp = C.counts_to_numpy(outs[0][0])
            for i in np.linspace(0, c - 1, min(picks, c)).astype(int):
                g = a + int(i) * st
                cc, t = O.count(O.synth_genome(g, SEED + g, args.seq_len, 80), k)
                ok &= bool((cnp[i] == cc).all()) and int(outs[0][1][i]) == t
        return ok

    def all_ok(ok):
        if world > 1:
            f = torch.tensor([0.0 if ok else 1.0], device=dev if not rehearse else "cpu")
            dist.all_reduce(f, op=dist.ReduceOp.MAX)
            ok = float(f) == 0.0
        return ok

    def max_over_ranks(*v):
        if world == 1:
            return v
        t = torch.tensor(v, dtype=torch.float64, device=dev if not rehearse else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return tuple(float(x) for x in t)

    ok = True
    launch_ms = []
    if resident:
        dbs = [gen(j) for j in range(len(plan))]
        kc, outs, el, launch_ms = run(args.k, args.steps, args.warmup, dbs)
        ok &= verify(args.k, 0, outs[:1], args.verify)
        for j in range(1, len(plan)):
            ok &= verify(args.k, j, [outs[j]], 0)
        del outs
    else:
        el = 0.0
        dbs = None
        for j in range(len(plan)):
            db = gen(j)
            kc, outs, e, ms = run(args.k, args.steps, args.warmup, [db])
            el += e
            launch_ms += ms
            ok &= verify(args.k, j, outs, args.verify if j == 0 else 0)
            del outs, db
    kern_ms = float(np.mean(launch_ms)) if launch_ms else 0.0
    el, kern_ms = max_over_ranks(el, kern_ms)
    ok = all_ok(ok)
    ceiling = stream_ceiling(torch, dbs[0].data, stream) if (rank == 0 and resident and dbs and dbs[0] is not None) \
        else None
    nsb = sum(1 for _, _, c in plan if c)
    # per launch (one sub-batch): FASTA bytes read + 4 B x bins written
    alg_bytes = (fasta_bytes + 4 * kc.nbins * n) / max(1, nsb)
    grid, block, lds = kc.launch_info()

    total_bases = bases * world if workload == "configs1" else args.total_genomes * args.seq_len
    value = total_bases / el * args.steps / 1e9
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9 if kern_ms else 0.0
    workload_tag = f"{n // max(1, nsb)} synthetic {args.seq_len / 1e6:g} Mbp genomes, 80-column FASTA"
    traffic, traffic_src = load_traffic(args.k, workload_tag)
    if workload == "configs1":
        wl = (f"{world}xMI355X, k={args.k}, {args.genomes_per_gpu} synthetic {args.seq_len / 1e6:g} Mbp genomes per GPU"
              + (" (BASELINE configs[1])" if world == 1 else " (configs[1] batch on every GPU, weak)"))
        cfg = {"workload": wl, "k": args.k, "genomes_per_gpu": args.genomes_per_gpu, "seq_len": args.seq_len,
               "line_width": 80, "global_batch": args.genomes_per_gpu * world,
               "parallelism": f"round-robin genome shards x{world}, no collective"}
    else:
        wl = (f"{world}xMI355X, k={args.k}, {args.total_genomes} synthetic {args.seq_len / 1e6:g} Mbp genomes sharded "
              f"round-robin (genome g on GPU g mod {world}), no RCCL on the data path (BASELINE configs[3])")
        cfg = {"workload": wl, "k": args.k, "global_batch": args.total_genomes, "genomes_per_gpu": n,
               "seq_len": args.seq_len, "line_width": 80, "sub_batches_per_gpu": nsb,
               "sub_batch": args.sub_batch, "resident": resident,
               "parallelism": f"round-robin genome shards x{world}, no collective"}
    cfg.update({"kernel_grid": [grid, block], "lds_bytes": lds})
    out = {
        "metric": "Gbases/s k-mer→.kf build at k=7; achieved HBM GB/s vs gfx950 peak",
        "value": round(value, 3),
        "unit": "Gbases/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak" if workload == "configs1" else "strong",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (device-generated, seeded splitmix64; no datasets)",
        "config": cfg,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                     "frac": round(achieved / PEAK_HBM_GBPS, 4), "traffic": traffic,
                     "traffic_source": traffic_src, "per_gpu": True,
                     "kernel_ms": round(kern_ms, 4), "alg_bytes_per_launch": int(alg_bytes),
                     "aggregate_achieved": round(achieved * world, 1),
                     "measured_ceiling": ceiling},
        "parity": "ok" if ok else "MISMATCH",
    }
    if args.secondary_k and world == 1 and args.secondary_k != args.k and resident:
        k2 = args.secondary_k
        st2 = max(3, args.steps // 4)
        kc2, o2, el2, ms2 = run(k2, st2, 1, dbs)
        ok2 = verify(k2, 0, o2, args.verify)
        ok &= ok2
        km2 = float(np.mean(ms2))
        alg2 = (fasta_bytes + 4 * kc2.nbins * n) / max(1, nsb)
        tr2, src2 = load_traffic(k2, workload_tag)
        out["secondary"] = {
            "config": f"1xMI355X, k={k2} (BASELINE configs[4]), same batch",
            "value": round(bases / el2 * st2 / 1e9, 3), "unit": "Gbases/s",
            "ms_per_step": round(el2 / st2 * 1e3, 4),
            "roofline": {"bound": "hbm", "achieved": round(alg2 / (km2 * 1e-3) / 1e9, 1), "peak": PEAK_HBM_GBPS,
                         "unit": "GB/s", "frac": round(alg2 / (km2 * 1e-3) / 1e9 / PEAK_HBM_GBPS, 4),
                         "traffic": tr2, "traffic_source": src2, "kernel_ms": round(km2, 4),
                         "alg_bytes_per_launch": int(alg2)},
            "parity": "ok" if ok2 else "MISMATCH"}
        out["parity"] = "ok" if ok else "MISMATCH"
        del o2
    if rank == 0 and world == 1 and not args.no_cpu:
        ids = [a + i * st for a, st, c in plan for i in range(c)]
        out["cpu_baseline"] = cpu_baseline(args, ids)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
