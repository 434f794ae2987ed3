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
`roofline.cold_kernel_ms` is one launch after the GPU has idled for a second
(what a CLI batch that follows host I/O sees), measured after the timed region.
The CPU baseline (rank 0, N=1) times the oracle's C restatement (kind "port":
Jellyfish is not installed) on a bounded sample of the same genomes, OpenMP
over (genome, ~1 MiB part) pairs on every host CPU this process may use
(sched_getaffinity, capped by a cgroup CPU quota if one is set).
`e2e` (rank 0, N=1) is the get_frequencies CLI end to end on 64 bacterial-like
~5 Mbp genome files in tmpfs (BASELINE configs[2] shape): the pipelined CLI
wall time, and the same work run stage by stage (file read, H2D + the FASTA
record index on the device, count, D2H, format + write) to show where the time
goes.
`sparse` (rank 0, N=1) is get_kmers' sparse counter (k=31 by default: the
present canonical k-mers per genome by a device radix sort) on 64 of the
synthetic genomes, genome 0 checked against the oracle.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--k 7]
  (N>1: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...,
   or plain `python bench.py --gpus N`: the process then starts N ranks itself,
   one per GPU, before it touches the GPU, and relays rank 0's line)
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


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); default: WORLD_SIZE under torchrun, else 1.  Without torchrun "
                         "N > 1 starts N rank processes here")
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
    ap.add_argument("--by-k", default="3-12",
                    help="also time every k of this range on the batch (N=1; '' = off): the reference's vocab "
                         "branches k=3..10 (main.py:281-296) plus 11 and 12")
    ap.add_argument("--by-k-steps", type=int, default=5)
    ap.add_argument("--by-k-warmup", type=int, default=3)
    ap.add_argument("--verify", type=int, default=4, help="genomes per rank checked bit-exactly against the oracle")
    ap.add_argument("--e2e-genomes", type=int, default=64, help="CLI end-to-end files (0 = off; N=1 only)")
    ap.add_argument("--e2e-len", type=int, default=5_000_000)
    ap.add_argument("--sparse-k", type=int, default=31, help="get_kmers sparse counter line (0 = off; N=1 only)")
    ap.add_argument("--sparse-genomes", type=int, default=64)
    return ap.parse_args(argv)


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
    """CPUs this process may use (kf2vecfsw_amd.main.usable_cpus: the affinity
    mask capped by a cgroup CPU quota)."""
    from kf2vecfsw_amd.main import usable_cpus as U
    return U()


def _oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import kf_oracle as O
    return O


def cpu_baseline(args, ids: list[int]) -> dict:
    """Oracle C restatement on host cores over a bounded sample (~10 s of CPU work)."""
    O = _oracle()
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


def stream_ceiling(torch, data, stream, reps: int = 5) -> dict:
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

    t_probe = timed(probe, reps)
    t_copy = timed(lambda: dst.copy_(data[:n]), 5)
    del dst
    return {"stream_read_GBps": round(n / t_probe / 1e9, 1), "d2d_copy_GBps": round(2 * n / t_copy / 1e9, 1),
            "bytes": int(n), "probe_reps": reps + 1, "copy_reps": 6}


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


class Workload:
    """One rank's share of the bench workload: configs[1] (one batch of
    --genomes-per-gpu) or configs[3] (the rank's round-robin shard of
    --total-genomes in sub-batches), generated on the device, counted, checked."""

    def __init__(self, args, dev, rank: int = 0, world: int = 1, dist=None, rehearse: bool = False):
        import torch
        from kf2vecfsw_amd import counter as C
        self.args, self.dev, self.rank, self.world, self.dist, self.rehearse = args, dev, rank, world, dist, rehearse
        self.torch, self.C = torch, C
        self.kind = args.workload if args.workload != "auto" else ("configs1" if world == 1 else "configs3")
        if self.kind == "configs1":
            g0, gs = shard_ids(args.genomes_per_gpu, rank, world)
            self.plan = [(g0, gs, args.genomes_per_gpu)]
        else:
            self.plan = shard_plan(args.total_genomes, rank, world, args.sub_batch)
        self.n = sum(c for _, _, c in self.plan)                      # this rank's genomes
        self.nsb = sum(1 for _, _, c in self.plan if c)
        self.sb_bytes = [int(C.synth_layout(c, args.seq_len, 80, a, st)[-1]) if c else 0 for a, st, c in self.plan]
        self.fasta_bytes = sum(C.synth_fasta_bytes(args.seq_len, 80, a + i * st)
                               for a, st, c in self.plan for i in range(c))
        self.stream = torch.cuda.current_stream(dev)

    # ---- collectives (RCCL / gloo: barriers and max-over-ranks only)
    def _tensor(self, v, dtype=None):
        return self.torch.tensor(v, dtype=dtype, device=self.dev if not self.rehearse else "cpu")

    def barrier(self):
        if self.world > 1 and self.dist is not None:
            self.dist.barrier()

    def all_ok(self, ok: bool) -> bool:
        if self.world > 1 and self.dist is not None:
            f = self._tensor([0.0 if ok else 1.0])
            self.dist.all_reduce(f, op=self.dist.ReduceOp.MAX)
            ok = float(f) == 0.0
        return ok

    def max_over_ranks(self, *v):
        if self.world == 1 or self.dist is None:
            return v
        t = self._tensor(v, self.torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return tuple(float(x) for x in t)

    def fits(self, kmax: int) -> bool:
        """Whether every sub-batch (and its count rows at kmax) stays resident."""
        row_b = 4 * self.C.num_bins(kmax) + 8
        need = sum(self.sb_bytes) + row_b * self.n
        a = self.args
        budget = a.max_resident_gb * 1e9 if a.max_resident_gb else self.torch.cuda.mem_get_info(self.dev)[0] - 8e9
        resident = need <= budget
        if self.world > 1:   # every rank takes the same mode (the streamed mode has per-sub-batch barriers)
            resident = self.all_ok(resident)
        return resident

    # ---- device batches and timed passes
    def gen(self, j):
        a, st, c = self.plan[j]
        if not c:
            return None
        db = self.C.synth_device_batch(c, self.args.seq_len, SEED, width=80, g0=a, g_stride=st, device=self.dev)
        self.torch.cuda.synchronize(self.dev)
        return db

    def run(self, k, steps, warmup, dbs, pre=None):
        """`warmup` untimed + `steps` timed steps at k over the sub-batches `dbs`
        (None = empty).  A step = one kf_count_batch call (count-matrix memset +
        kernel) per sub-batch.  `pre(dbs)` runs before the warmup steps.  Returns
        (counter, outputs, wall s, HIP-event ms of every timed launch on the launch
        stream, HIP-event ms of the warmup launches)."""
        torch, stream = self.torch, self.stream
        kc = self.C.KmerCounter(k, self.dev)
        kc.reserve(max((db.n for db in dbs if db is not None), default=0))
        outs = [kc.alloc_out(db.n) if db is not None else None for db in dbs]
        if pre is not None:
            pre(dbs)

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

        wevs = []
        for _ in range(warmup):
            step(wevs)
        torch.cuda.synchronize(self.dev)
        evs = []
        self.barrier()
        torch.cuda.synchronize(self.dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            step(evs)
        torch.cuda.synchronize(self.dev)
        self.barrier()
        el = time.perf_counter() - t0
        return kc, outs, el, [a.elapsed_time(b) for a, b in evs], [a.elapsed_time(b) for a, b in wevs]

    def verify(self, k, j, outs, picks) -> bool:
        """Totals are analytic for N-free synthetic genomes; `picks` genomes of
        sub-batch j (evenly spaced, first and last included; all if picks >= its
        size) bit-exact vs the oracle -- the checker, outside the timed region."""
        a, st, c = self.plan[j]
        ok = True
        for o in outs:
            if o is None:
                continue
            ok &= bool((o[1].cpu().numpy() == self.args.seq_len - k + 1).all())
        if picks and c and outs and outs[0] is not None:
            O = _oracle()
            cnp = self.C.counts_to_numpy(outs[0][0])
            for i in np.unique(np.linspace(0, c - 1, min(picks, c)).astype(int)):
                g = a + int(i) * st
                cc, t = O.count(O.synth_genome(g, SEED + g, self.args.seq_len, 80), k)
                ok &= bool((cnp[i] == cc).all()) and int(outs[0][1][i]) == t
        return ok

    def measure(self, k, steps, warmup, resident, picks, picks_rest=0, keep=False, pre=None):
        """The timed passes at k over this rank's plan: resident (every sub-batch in
        HBM, one step = all of them) or streamed (each sub-batch generated, timed on
        its own, the times added).  `picks` genomes of the first sub-batch and
        `picks_rest` of every other one are checked against the oracle; `pre` (see
        run) before the first timed pass.  Returns a dict with the wall time,
        per-launch ms, the parity verdict of this rank, and (keep=True, resident)
        the batches."""
        res = {"ok": True, "launch_ms": [], "warm_ms": [], "el": 0.0, "dbs": None, "kc": None, "outs": None}
        if resident:
            dbs = [self.gen(j) for j in range(len(self.plan))]
            kc, outs, el, ms, wms = self.run(k, steps, warmup, dbs, pre)
            for j in range(len(self.plan)):
                res["ok"] &= self.verify(k, j, [outs[j]], picks if j == 0 else picks_rest)
            res.update(el=el, launch_ms=ms, warm_ms=wms, kc=kc, dbs=dbs if keep else None,
                       outs=outs if keep else None)
            del outs
        else:
            for j in range(len(self.plan)):
                db = self.gen(j)
                kc, outs, e, ms, wms = self.run(k, steps, warmup, [db], pre if j == 0 else None)
                res["el"] += e
                res["launch_ms"] += ms
                res["warm_ms"] += wms
                res["ok"] &= self.verify(k, j, outs, picks if j == 0 else picks_rest)
                res["kc"] = kc
                del outs, db
        return res


def parse_k_range(spec: str) -> list[int]:
    """"3-12" -> [3..12]; "7,9,11" -> [7, 9, 11]."""
    ks = []
    for part in str(spec).split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            ks += list(range(int(a), int(b) + 1))
        else:
            ks.append(int(part))
    return ks


def by_k_bench(W, dbs, args, workload_tag: str) -> dict:
    """Every k of --by-k on the resident configs[1] batch:
    the batch streamed ~30 times first (the oracle checks of the previous k left
    the GPU idle, and clocks settle over ~20-30 ms of load: profiles/r04/
    v1_cold.json), then --by-k-warmup + --by-k-steps timed kf_count_batch calls,
    the kernel's HIP event time per launch, its roofline (FASTA bytes + 4 B x
    bins per genome, as the headline), the measured traffic when profiles/ holds
    it, and parity: every total analytic plus 2 genomes bit-exact against the
    oracle."""
    import torch
    res = {}

    def prewarm(dbs):
        stream_ceiling(torch, dbs[0].data, W.stream, reps=30)

    for k in parse_k_range(args.by_k):
        kc, o, el, ms, _ = W.run(k, args.by_k_steps, args.by_k_warmup, dbs, pre=prewarm)
        okk = W.verify(k, 0, o, 2)
        km = float(np.mean(ms))
        alg = (W.fasta_bytes + 4 * kc.nbins * W.n) / max(1, W.nsb)
        tr, src = load_traffic(k, workload_tag)
        grid, block, lds = kc.launch_info()
        res[str(k)] = {"kernel_ms": round(km, 4), "kernel_ms_runs": [round(x, 4) for x in ms],
                       "Gbases_s": round(W.n * args.seq_len / (km * 1e-3) / 1e9, 1),
                       "nbins": kc.nbins, "alg_bytes_per_launch": int(alg),
                       "roofline": {"bound": "hbm", "achieved": round(alg / (km * 1e-3) / 1e9, 1),
                                    "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                                    "frac": round(alg / (km * 1e-3) / 1e9 / PEAK_HBM_GBPS, 4),
                                    "traffic": tr, "traffic_source": src},
                       "kernel": ("k1x_kernel<%d>" % k) if k <= 9 else ("bucket_kernel<%d>" % k),
                       "launch": [grid, block, lds], "parity": "ok" if okk else "MISMATCH"}
        del kc, o
        torch.cuda.empty_cache()
    return res


def cold_launch_ms(torch, kc, db, stream, idle_s: float = 1.0) -> float:
    """One launch after the GPU has idled `idle_s` (what a CLI batch sees after host I/O)."""
    out = kc.alloc_out(db.n)
    torch.cuda.synchronize()
    time.sleep(idle_s)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    kc.count(db, out[0], out[1])
    b.record(stream)
    torch.cuda.synchronize()
    return a.elapsed_time(b)


# ---------------------------------------------------------------------------
# e2e: the get_frequencies CLI on real-shaped files (BASELINE configs[2] shape)
# ---------------------------------------------------------------------------
def bacterial_like(rng: np.random.Generator, total: int) -> tuple[bytes, int]:
    """A synthetic bacterial-like assembly (no assemblies offline): 1-80 contigs,
    GC 30-70 %, short N runs, 60/80-column lines, soft-masked stretches.
    Returns the FASTA bytes and its number of sequence characters."""
    ncontig = int(rng.integers(1, 81))
    cuts = np.sort(rng.choice(np.arange(1, total), size=ncontig - 1, replace=False)) if ncontig > 1 else []
    lens = np.diff(np.concatenate([[0], cuts, [total]])).astype(np.int64)
    gc = float(rng.uniform(0.3, 0.7))
    width = int(rng.choice([60, 80]))
    lut = np.frombuffer(b"ACGT", np.uint8)
    p = np.array([(1 - gc) / 2, gc / 2, gc / 2, (1 - gc) / 2])
    out = []
    for i, L in enumerate(lens):
        seq = lut[rng.choice(4, size=int(L), p=p)]
        for _ in range(int(rng.poisson(L * 1e-6)) + 0):
            a = int(rng.integers(0, L))
            seq[a: a + int(rng.integers(1, 40))] = ord("N")
        if rng.random() < 0.3 and L > 2000:
            a = int(rng.integers(0, L - 1000))
            seq[a: a + 1000] |= 0x20
        nl = (int(L) + width - 1) // width
        body = np.full(int(L) + nl, 10, np.uint8)
        idx = np.arange(int(L))
        body[idx + idx // width] = seq
        out.append(b">contig_%d len=%d\n" % (i, L) + body.tobytes())
    return b"".join(out), int(total)


def e2e_bench(args, dev) -> dict:
    """The get_frequencies CLI (kf2vecfsw_amd.main) on --e2e-genomes files in
    tmpfs, k=7: median pipelined wall time of 7 runs after a warm run; then the
    same files stage by stage with a sync between stages.  Four .kf files are
    checked against the oracle (outside the timing)."""
    import contextlib
    import io
    import tempfile

    import torch
    from kf2vecfsw_amd import counter as C
    from kf2vecfsw_amd import main as M
    threads, _ = usable_cpus()
    base = "/dev/shm" if os.access("/dev/shm", os.W_OK) else None
    work = tempfile.mkdtemp(prefix="kf_e2e_", dir=base)
    try:
        inp = os.path.join(work, "in")
        os.makedirs(inp)
        rng = np.random.default_rng(2026)
        bases = 0
        names = []
        for g in range(args.e2e_genomes):
            blob, nb = bacterial_like(rng, args.e2e_len)
            bases += nb
            names.append("B%04d" % g)
            with open(os.path.join(inp, names[-1] + ".fna"), "wb") as f:
                f.write(blob)
        in_bytes = sum(os.path.getsize(os.path.join(inp, n + ".fna")) for n in names)

        def cli(out):
            os.makedirs(out)
            with contextlib.redirect_stdout(io.StringIO()):
                t0 = time.perf_counter()
                # the default -p (mp.cpu_count(), as the reference): what a user gets; the
                # CLI caps it at the usable CPUs (main.host_threads)
                M.main(["get_frequencies", "-input_dir", inp, "-output_dir", out, "-k", str(7)])
                return time.perf_counter() - t0

        # one warm run, then 7 timed: the host side (file reads on a shared box)
        # varies by up to ~30 % run to run
        walls = [cli(os.path.join(work, f"out{r}")) for r in range(8)]
        wall = float(np.median(walls[1:]))
        # stage by stage (one batch of every file, synchronised between stages)
        files = sorted(os.listdir(inp))
        paths = [os.path.join(inp, f) for f in files]
        kc = C.KmerCounter(7, dev)
        stream = torch.cuda.current_stream(dev)
        st = {}
        for rep in range(2):   # the first pass warms the pinned allocator
            t0 = time.perf_counter()
            hb = C.pack_files(paths, [f.rsplit(".f", 1)[0] for f in files], threads=threads, index=False)
            t1 = time.perf_counter()
            db = C.to_device(hb, dev)   # H2D + the record index on the device (kf_index_fasta), as the CLI
            torch.cuda.synchronize(dev)
            t2 = time.perf_counter()
            cnt, _ = kc.count(db)
            torch.cuda.synchronize(dev)
            t3 = time.perf_counter()
            host = torch.empty(cnt.shape, dtype=cnt.dtype, pin_memory=True)
            host.copy_(cnt, non_blocking=True)
            stream.synchronize()
            t4 = time.perf_counter()
            outd = os.path.join(work, f"stage{rep}")
            os.makedirs(outd)
            M.write_kf_files(outd, hb.names, host.numpy().view(np.uint32), False, False, threads)
            t5 = time.perf_counter()
            st = {"read": t1 - t0, "h2d_index": t2 - t1, "count": t3 - t2, "d2h": t4 - t3, "format_write": t5 - t4}
            del hb, db, cnt, host
        O = _oracle()
        ok = True
        for g in np.linspace(0, len(names) - 1, 4).astype(int):
            data = open(os.path.join(inp, names[g] + ".fna"), "rb").read()
            c, _ = O.count(data, 7)
            exp = O.kf_line(names[g], c).encode()
            ok &= open(os.path.join(work, "out1", names[g] + ".kf"), "rb").read() == exp
            ok &= open(os.path.join(work, "stage1", names[g] + ".kf"), "rb").read() == exp
        out_bytes = sum(os.path.getsize(os.path.join(work, "out1", n + ".kf")) for n in names)
        gbs = lambda s: round(bases / s / 1e9, 3)
        return {"workload": f"get_frequencies CLI, k=7, {len(names)} bacterial-like ~{args.e2e_len / 1e6:g} Mbp "
                            f"FASTA files in {'/dev/shm' if base else 'tmp'} (BASELINE configs[2] shape)",
                "bases": bases, "input_bytes": in_bytes, "kf_bytes": out_bytes, "host_threads": threads,
                "cli_wall_s": round(wall, 4), "cli_wall_s_runs": [round(w, 4) for w in walls],
                "value": gbs(wall), "unit": "Gbases/s",
                "stages_s": {k: round(v, 4) for k, v in st.items()},
                "stages_Gbases_s": {k: gbs(v) for k, v in st.items()},
                "stages_sum_s": round(sum(st.values()), 4),
                "pcie_h2d_GBps": round(in_bytes / st["h2d_index"] / 1e9, 1) if st.get("h2d_index") else None,
                "parity": "ok" if ok else "MISMATCH"}
    finally:
        shutil.rmtree(work, ignore_errors=True)


def sparse_bench(args, dev) -> dict:
    """get_kmers' sparse counter (kf_sparse_count, k = 13..31: the present
    canonical k-mers per genome by a device radix sort) on --sparse-genomes of
    the synthetic genomes (ids 0..n-1, resident in HBM), median of 5 launches
    after one warm launch.  Genome 0 is checked against the oracle's restatement
    and every genome's total against seq_len - k + 1 (outside the timing).
    `roofline.achieved` counts the algorithmic bytes (FASTA read + 12 B per
    distinct k-mer written); the design moves the input twice (bucket count,
    bucket scatter), each key once out and once back in (the bucketed keys), and
    12 B per distinct k-mer out (round 5; round 4's LSD sort moved ~2 x 8 B per
    key per 8-bit pass)."""
    import torch
    from kf2vecfsw_amd import counter as C
    k, n, L = args.sparse_k, args.sparse_genomes, args.seq_len
    db = C.synth_device_batch(n, L, SEED, width=80, device=dev)
    off = C.synth_layout(n, L)
    nbytes = int(off[-1])
    sc = C.SparseCounter(k, dev)
    ms = []
    for r in range(6):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        keys, cnts, nu = sc.count(db, nbytes)
        e1.record()
        torch.cuda.synchronize()
        if r:
            ms.append(e0.elapsed_time(e1))
        if r < 5:
            del keys, cnts, nu
    med = float(np.median(ms))
    nuh = nu.cpu().numpy()
    O = _oracle()
    g0 = sc.to_host(keys[: int(off[1])], cnts[: int(off[1])], nu[:1], off[:2])[0]
    ek, ec = O.sparse_count(O.synth_genome(0, SEED, L, 80), k)
    ok = bool(np.array_equal(g0[0], ek) and np.array_equal(g0[1], ec))
    tot = torch.zeros(n, dtype=torch.int64, device=dev)
    c64 = cnts.to(torch.int64) & 0xFFFFFFFF
    for g in range(n):
        tot[g] = c64[int(off[g]): int(off[g]) + int(nuh[g])].sum()
    ok &= bool((tot.cpu().numpy() == L - k + 1).all())
    alg = nbytes + 12 * int(nuh.sum())
    key_b = 4 if k <= 16 else 8
    bucket_bits = min(10, 2 * k)
    r_bits = 2 * k - bucket_bits + 2                  # a chunk spans ~2-4 buckets
    sort_note = ("two 10-bit passes (the whole key)" if r_bits <= 20 else
                 "two 10-bit MSD passes over the top 20 bits + an in-LDS fix-up of runs of equal top bits")
    del keys, cnts, nu, db, sc, tot, c64
    torch.cuda.empty_cache()
    return {"config": f"get_kmers sparse counter, k={k}, {n} synthetic {L / 1e6:g} Mbp genomes resident in HBM "
                      f"(the present canonical k-mers and counts per genome)",
            "value": round(n * L / (med * 1e-3) / 1e9, 3), "unit": "Gbases/s", "ms": round(med, 4),
            "ms_runs": [round(x, 4) for x in ms], "distinct_per_genome": int(nuh.mean()),
            "roofline": {"bound": "hbm", "achieved": round(alg / (med * 1e-3) / 1e9, 1), "peak": PEAK_HBM_GBPS,
                         "unit": "GB/s", "frac": round(alg / (med * 1e-3) / 1e9 / PEAK_HBM_GBPS, 4),
                         "alg_bytes_per_launch": alg,
                         "design_bytes_per_launch": int(nbytes * 2 + n * L * 2 * key_b + 12 * int(nuh.sum())),
                         "note": f"{2 * k}-bit keys: bucket count over the bytes, bucket scatter ({key_b} B per key "
                                 f"out, top {bucket_bits} bits), per-chunk LDS sort ({sort_note}, {key_b} B per key "
                                 f"in) + run-length encoding (12 B per distinct k-mer out)"},
            "parity": "ok" if ok else "MISMATCH"}


def resolve_world(args, env=None) -> tuple[int, bool]:
    """(world size, spawn here?) from --gpus and the launcher's WORLD_SIZE.
    Under a launcher (WORLD_SIZE set) --gpus must match it; without one,
    --gpus N > 1 means this process starts the N ranks itself.  Raises
    SystemExit with a message on a mismatch -- a scaling run must never time
    fewer GPUs than it names."""
    env = os.environ if env is None else env
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        ws = int(ws)
        if args.gpus is not None and args.gpus != ws:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws} (the launcher started {ws} "
                             f"rank(s)); refusing to time a different number of GPUs than named")
        return ws, False
    n = 1 if args.gpus is None else args.gpus
    if n < 1:
        raise SystemExit(f"bench.py: --gpus {n}: need at least one GPU")
    return n, n > 1


def spawn_ranks(n: int, argv: list[str], env=None, timeout_s: float | None = None) -> int:
    """`python bench.py --gpus N` without a launcher: start N rank processes
    (RANK = LOCAL_RANK = r, WORLD_SIZE = N, rendezvous on 127.0.0.1) -- exactly
    what torch.distributed.run would give them -- and relay rank 0's stdout.
    This process never touches the GPU (no HIP call before the children start;
    no exec).  If a rank fails, the others get 60 s to finish, then are
    terminated by PID; ranks still running after `timeout_s` (default
    KF_BENCH_TIMEOUT_S or 1800 s) are terminated too, so a hung rank cannot
    hold the run forever.  Returns the worst exit status (0 if all ranks
    passed; 124 when the overall limit ended the run)."""
    import socket
    import subprocess
    import threading
    env = dict(os.environ if env is None else env)
    from kf2vecfsw_amd.main import visible_gpus   # KFD topology / *_VISIBLE_DEVICES, no HIP init
    avail = visible_gpus(env)   # the masks the children will see
    if env.get("KF_BENCH_REHEARSE") != "1" and avail is not None and n > avail:
        print(f"bench.py: --gpus {n} but only {avail} GPU(s) visible", file=sys.stderr)
        return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), KF_BENCH_SPAWNED="1")
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + argv, env=e,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))

    def relay():
        for line in procs[0].stdout:
            sys.stdout.write(line.decode(errors="replace"))
            sys.stdout.flush()

    t = threading.Thread(target=relay, daemon=True)
    t.start()
    deadline = None
    limit = float(timeout_s if timeout_s is not None else env.get("KF_BENCH_TIMEOUT_S", 1800))
    hard = time.monotonic() + limit
    timed_out = False
    while True:
        rcs = [p.poll() for p in procs]
        if all(rc is not None for rc in rcs):
            break
        if deadline is None and any(rc not in (None, 0) for rc in rcs):
            deadline = time.monotonic() + 60.0
        over = time.monotonic() > hard
        if over or (deadline is not None and time.monotonic() > deadline):
            timed_out = over
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=20)
                except subprocess.TimeoutExpired:
                    p.kill()
            break
        time.sleep(0.2)
    t.join(timeout=10)
    rcs = [p.wait() for p in procs]
    bad = [(r, rc) for r, rc in enumerate(rcs) if rc]
    if timed_out:
        print(f"bench.py: ranks still running after {limit:g} s were terminated", file=sys.stderr)
        return 124
    if bad:
        print("bench.py: rank(s) failed: " + ", ".join(f"rank {r} exit {rc}" for r, rc in bad), file=sys.stderr)
        return max(abs(rc) for _, rc in bad) or 1
    return 0


def main() -> None:
    args = parse_args()
    world, spawn = resolve_world(args)
    if spawn:
        sys.exit(spawn_ranks(world, sys.argv[1:]))

    import torch
    import torch.distributed as dist

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
    from kf2vecfsw_amd import _native as N

    W = Workload(args, dev, rank, world, dist if world > 1 else None, rehearse)
    kmax = max(args.k, args.secondary_k if (world == 1 and args.secondary_k) else 0)
    resident = W.fits(kmax)
    stream = W.stream
    bases = W.n * args.seq_len

    # The measured-ceiling probes run on the generated batch BEFORE the warmup
    # steps: they stream it ~60 times (about 70 ms of HBM traffic), after which
    # the GPU's clocks have settled; right after generation or an idle gap the
    # first ~20 count launches run up to 40 % slower while they settle
    # (profiles/r04/v1_cold.json).  Declared in the JSON ("prewarm"); the launch
    # after an idle second is reported as roofline.cold_kernel_ms.
    ceiling = {}

    def prewarm(dbs):
        db0 = next((d for d in dbs if d is not None), None)
        if db0 is not None:
            ceiling.update(stream_ceiling(torch, db0.data, stream, reps=60))

    m = W.measure(args.k, args.steps, args.warmup, resident, args.verify, keep=True, pre=prewarm)
    ok = m["ok"]
    kc, dbs = m["kc"], m["dbs"]
    kern_ms = float(np.mean(m["launch_ms"])) if m["launch_ms"] else 0.0
    el, kern_ms = W.max_over_ranks(m["el"], kern_ms)
    ok = W.all_ok(ok)
    first = dbs[0] if dbs else None
    cold = cold_launch_ms(torch, kc, first, stream) if (rank == 0 and first is not None) else None
    nsb = W.nsb
    n = W.n
    # per launch (one sub-batch): FASTA bytes read + 4 B x bins written
    alg_bytes = (W.fasta_bytes + 4 * kc.nbins * n) / max(1, nsb)
    grid, block, lds = kc.launch_info()

    total_bases = bases * world if W.kind == "configs1" else args.total_genomes * args.seq_len
    value = total_bases / el * args.steps / 1e9
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9 if kern_ms else 0.0
    workload_tag = f"{n // max(1, nsb)} synthetic {args.seq_len / 1e6:g} Mbp genomes, 80-column FASTA"
    traffic, traffic_src = load_traffic(args.k, workload_tag)
    if W.kind == "configs1":
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
    # what ONE kf_count_batch launch of this rank holds (the largest sub-batch)
    cfg.update({"kernel_grid": [grid, block], "lds_bytes": lds,
                "genomes_per_launch": max(c for _, _, c in W.plan), "bytes_per_launch": max(W.sb_bytes)})
    wm = m["warm_ms"]
    out = {
        "metric": "Gbases/s k-mer→.kf build at k=7; achieved HBM GB/s vs gfx950 peak",
        "value": round(value, 3),
        "unit": "Gbases/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak" if W.kind == "configs1" else "strong",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (device-generated, seeded splitmix64; no datasets)",
        "config": cfg,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                     "frac": round(achieved / PEAK_HBM_GBPS, 4), "traffic": traffic,
                     "traffic_source": traffic_src, "per_gpu": True,
                     "kernel_ms": round(kern_ms, 4), "alg_bytes_per_launch": int(alg_bytes),
                     "aggregate_achieved": round(achieved * world, 1),
                     "cold_kernel_ms": round(cold, 4) if cold is not None else None,
                     "warmup_kernel_ms": [round(x, 4) for x in wm],
                     "measured_ceiling": ceiling or None},
        "prewarm": ("measured_ceiling probes before the warmup steps: kf_stream_probe x{} + {} D2D copies of the "
                    "batch (~70 ms of HBM streaming; clocks settle over the first ~20-30 ms of sustained load, "
                    "profiles/r04/v1_cold.json)".format(ceiling.get("probe_reps"), ceiling.get("copy_reps"))
                    if ceiling else None),
        "parity": "ok" if ok else "MISMATCH",
        "build_id": N.build_id(),
        "ranks": {"world_size_reported": dist.get_world_size() if world > 1 else 1,
                  "backend": (dist.get_backend() if world > 1 else None),
                  "launcher": ("bench.py --gpus (spawned ranks)" if os.environ.get("KF_BENCH_SPAWNED")
                               else "torch.distributed.run" if world > 1 else "single process"),
                  "devices": ("cuda:0 for every rank (KF_BENCH_REHEARSE)" if rehearse
                              else f"cuda:LOCAL_RANK, {world} GPU(s)")},
    }
    if out["ranks"]["world_size_reported"] != world:
        ok = False
        out["parity"] = "MISMATCH"
    if args.secondary_k and world == 1 and args.secondary_k != args.k and resident:
        k2 = args.secondary_k
        st2 = max(3, args.steps // 4)
        kc2, o2, el2, ms2, _ = W.run(k2, st2, 1, dbs)
        ok2 = W.verify(k2, 0, o2, args.verify)
        ok &= ok2
        km2 = float(np.mean(ms2))
        alg2 = (W.fasta_bytes + 4 * kc2.nbins * n) / max(1, nsb)
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
    if args.by_k and world == 1 and resident:
        out["by_k"] = by_k_bench(W, dbs, args, workload_tag)
        ok &= all(v["parity"] == "ok" for v in out["by_k"].values())
        out["parity"] = "ok" if ok else "MISMATCH"
    del dbs, first, m
    if rank == 0 and world == 1 and args.e2e_genomes:
        torch.cuda.empty_cache()
        out["e2e"] = e2e_bench(args, dev)
        ok &= out["e2e"]["parity"] == "ok"
        out["parity"] = "ok" if ok else "MISMATCH"
    if rank == 0 and world == 1 and args.sparse_k:
        out["sparse"] = sparse_bench(args, dev)
        ok &= out["sparse"]["parity"] == "ok"
        out["parity"] = "ok" if ok else "MISMATCH"
    if rank == 0 and world == 1 and not args.no_cpu:
        ids = [a + i * st for a, st, c in W.plan for i in range(c)]
        out["cpu_baseline"] = cpu_baseline(args, ids)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
