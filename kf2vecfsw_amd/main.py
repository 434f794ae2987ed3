"""``python -m kf2vecfsw_amd.main get_frequencies ...`` -- drop-in for the
reference's ``python -m kf2vec.main get_frequencies`` (kf2vec/main.py:250-373,
parser :1023-1038, dispatch :1489-1495).

Same flags, same stdout lines, same ``<sample>.kf`` bytes; the Jellyfish
subprocess pair per file (main.py:309-319) is replaced by one device pass per
batch of files through ``libkf2vec_gpu.so``.  Differences (DESIGN.md "Boundary"):
no ``.jf``/``.dump`` temporaries are created; a device or I/O error raises
instead of being silenced; ``-p`` sizes the host formatting/writing threads.
"""
from __future__ import annotations

import argparse
import ctypes
import multiprocessing as mp
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from . import _native as N

__version__ = "kf2vec 0.1.3 (kf2vecfsw_amd MI355X)"

default_k_len = 7          # main.py:80
min_k_len = 2              # main.py:81
max_k_len = 31             # main.py:82
supported_k = range(3, 12)  # rule-generated vocab (reference ships 3..9; 10 is a missing blob)

FORMATS = [".fq", ".fastq", ".fa", ".fna", ".fasta"]   # main.py:272
_SUFFIXES = tuple(FORMATS)


def list_inputs(input_dir: str) -> tuple[list[str], list[str]]:
    """main.py:272-275: files in os.listdir order and their sample names."""
    # (fnmatch "*" + form on POSIX is a case-sensitive suffix test)
    files_names = [f for f in os.listdir(input_dir) if f.endswith(_SUFFIXES)]
    samples_names = [f.rsplit(".f", 1)[0] for f in files_names]
    return files_names, samples_names


def write_kf_files(output_dir: str, names: list[str], counts: np.ndarray, pseudocount: bool, raw_cnt: bool,
                   threads: int) -> None:
    """Format + write ``<name>.kf`` for every row (main.py:331-357) with C++ threads."""
    counts = np.ascontiguousarray(counts, dtype=np.uint32)
    enc = [os.fsencode(n) for n in names]
    arr = (ctypes.c_char_p * len(enc))(*enc)
    N.check(N.lib().kf_write_kf_files(os.fsencode(output_dir), arr, len(enc), counts.ctypes.data,
                                      counts.shape[1] if counts.ndim == 2 else 0, int(bool(pseudocount)),
                                      int(bool(raw_cnt)), max(1, int(threads))), "kf_write_kf_files")


def format_kf(name: str, counts: np.ndarray, pseudocount: bool = False, raw_cnt: bool = False) -> bytes:
    """One ``.kf`` line (main.py:344-357), formatted by the C++ writer."""
    counts = np.ascontiguousarray(counts, dtype=np.uint32)
    nm = os.fsencode(name)
    cap = len(nm) + 2 + 26 * counts.size
    buf = ctypes.create_string_buffer(cap)
    w = ctypes.c_uint64(0)
    N.check(N.lib().kf_format_kf(nm, counts.ctypes.data, counts.size, int(pseudocount), int(raw_cnt), buf, cap,
                                 ctypes.byref(w)), "kf_format_kf")
    return buf.raw[: w.value]


def _pipeline_budget(paths: list[str], batch_gb, sizes: list[int] | None = None) -> int:
    """Bytes per batch: -batch_gb if given, else about a quarter of the input
    (so reading, copying, counting and writing overlap; 64 x 5 Mbp on two boxes,
    tools/e2e_bench.py: 4 parts 26.1 and 32.9 Gbases/s against 8 parts 22.5 and
    29.8, profiles/r05/v19_e2e_parts.json, v6_e2e_variants.json) within
    [16 MiB, 4 GiB].  KF_BATCH_PARTS overrides the part count."""
    if batch_gb:
        return int(float(batch_gb) * (1 << 30))
    total = sum(sizes) if sizes is not None else sum(os.path.getsize(p) for p in paths)
    parts = int(os.environ.get("KF_BATCH_PARTS", "4"))
    return int(min(max(total // parts, 16 << 20), 4 << 30))


COUNT_BUDGET = 2 << 30   # default count-matrix bytes per batch (device rows; as much again pinned on the host)


def _count_cap(row_bytes: int, batch_gb) -> int:
    """Genomes per batch so that the batch's count matrix (row_bytes per genome:
    4 x bins, 8 MiB at k=11, 33.6 MB at k=12) stays within -batch_gb if given,
    else COUNT_BUDGET (KF_COUNT_BUDGET_MB overrides).  The reference holds one
    genome's counts at a time (main.py:301-357); a batch of many small files must
    not hold thousands of rows."""
    env = os.environ.get("KF_COUNT_BUDGET_MB")
    b = int(float(env) * (1 << 20)) if env else int(float(batch_gb) * (1 << 30)) if batch_gb else COUNT_BUDGET
    return max(1, b // max(1, int(row_bytes)))


def _batches(paths: list[str], budget: int, ramp: bool = False, max_files: int | None = None) -> list[list[int]]:
    """Consecutive files in batches of at most `budget` bytes (a file larger than
    that alone) and at most `max_files` files.  ramp: the first two batches get a
    quarter and a half of the byte budget, so a pipeline's later stages start
    sooner."""
    return _size_batches([os.path.getsize(p) for p in paths], budget, ramp, max_files)


def _size_batches(sizes: list[int], budget: int, ramp: bool = False, max_files: int | None = None) -> list[list[int]]:
    """_batches over item sizes (files, or get_chunks' file parts)."""
    out, cur, size = [], [], 0
    for i, s in enumerate(sizes):
        lim = budget >> max(0, 2 - len(out)) if ramp else budget
        if cur and (size + s > lim or (max_files is not None and len(cur) >= max_files)):
            out.append(cur)
            cur, size = [], 0
        cur.append(i)
        size += s
    if cur:
        out.append(cur)
    return out


def shard_files(sizes: list[int], samples: list[str], world: int) -> list[list[int]]:
    """Byte-balanced shards of the input files for `world` GPUs (section 8(e): genomes
    are independent, no collective).  Files of one sample name stay in one shard,
    so the reference's last-file-wins rule for duplicate names (main.py:357 writes
    in input order) holds inside that shard; groups go largest first to the least
    loaded shard; each shard keeps the input order."""
    groups: dict[str, list[int]] = {}
    for i, s in enumerate(samples):
        groups.setdefault(s, []).append(i)
    load = [0] * world
    out: list[list[int]] = [[] for _ in range(world)]
    for g in sorted(groups.values(), key=lambda g: (-sum(sizes[i] for i in g), g[0])):
        r = min(range(world), key=lambda r: (load[r], r))
        out[r].extend(g)
        load[r] += sum(sizes[i] for i in g)
    return [sorted(o) for o in out]


def _shard_spec(args) -> tuple[int, int] | None:
    """(rank, world) when this process counts one shard: a child of `-gpus N`
    (KF_SHARD="r,N") or one rank of torchrun (RANK / WORLD_SIZE, no -gpus)."""
    e = os.environ.get("KF_SHARD")
    if e:
        r, w = (int(x) for x in e.split(","))
        return r, w
    if getattr(args, "gpus", 1) == 1 and int(os.environ.get("WORLD_SIZE", "1")) > 1:
        return int(os.environ.get("RANK", "0")), int(os.environ["WORLD_SIZE"])
    return None


def _spawn_shards(argv: list[str], world: int) -> int:
    """`-gpus N`: one child process per GPU (cuda:r), each counting shard r; no
    data crosses between them (each writes its own genomes' .kf files).  The
    parent never touches the GPU (KF_SHARD_DEVICE=cuda:0 puts every child on one
    GPU, for rehearsal on a one-GPU box)."""
    import subprocess
    procs = []
    for r in range(world):
        pkg_parent = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        env = dict(os.environ, KF_SHARD=f"{r},{world}",
                   PYTHONPATH=os.pathsep.join(filter(None, [pkg_parent, os.environ.get("PYTHONPATH")])))
        dev = os.environ.get("KF_SHARD_DEVICE") or f"cuda:{r}"
        procs.append(subprocess.Popen([sys.executable, "-m", "kf2vecfsw_amd.main"] + argv + ["-device", dev], env=env))
    return max(abs(p.wait()) for p in procs)


def visible_gpus(env=None) -> int | None:
    """GPUs this process may use, counted without initialising HIP (the -gpus
    parent forks children and must never touch the GPU itself): the GPU nodes of
    the KFD topology (nodes with SIMDs), capped by every one of
    ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES that is set
    (HIP applies its mask on top of ROCR's, so the smallest wins).  None when the
    topology is unreadable and no mask is set: unknown."""
    topo = "/sys/class/kfd/kfd/topology/nodes"
    n_kfd = None
    try:
        n_kfd = 0
        for d in os.listdir(topo):
            try:
                props = open(os.path.join(topo, d, "properties")).read().split("\n")
            except OSError:
                continue
            if any(ln.startswith("simd_count") and ln.split()[-1] != "0" for ln in props):
                n_kfd += 1
    except OSError:
        n_kfd = None
    n = n_kfd
    env = os.environ if env is None else env
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is not None:
            ids = [x for x in v.split(",") if x.strip() != ""]
            n = len(ids) if n is None else min(n, len(ids))
    return n


def usable_cpus() -> tuple[int, dict]:
    """CPUs this process may run on: the affinity mask, capped by a cgroup v2/v1
    CPU quota if one is set (a GPU box may show the whole host in the mask and
    in os.cpu_count(), e.g. 256, against a quota of 16)."""
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


def host_threads(p, world: int = 1) -> int:
    """Host threads of this process (file readers, .kf formatters/writers):
    min(-p, usable CPUs), split evenly over the `world` processes that share the
    host (-gpus N children, torchrun ranks on one node).  The reference hands -p
    to Jellyfish as `-t` (main.py:309) with default mp.cpu_count()
    (main.py:1031-1033), which on a GPU box counts every host CPU, not the
    process's quota: 256 threads on a 16-CPU quota."""
    usable = usable_cpus()[0]
    return max(1, min(max(1, int(p)), usable) // max(1, int(world)))


def _procs_per_host(shard) -> int:
    """Processes of this run sharing this host's CPUs: the -gpus N children (all
    local), or torchrun's ranks on this node (LOCAL_WORLD_SIZE)."""
    if shard is None:
        return 1
    if os.environ.get("KF_SHARD"):
        return shard[1]
    return int(os.environ.get("LOCAL_WORLD_SIZE", shard[1]))


def cli_host_threads(args) -> int:
    """get_frequencies' host threads in this process: -p capped by the usable
    CPUs, shared by the processes of this run on this host."""
    return host_threads(args.p, _procs_per_host(_shard_spec(args)))


def get_frequencies(args) -> None:
    """kf2vec/main.py:250-373 on the GPU (-gpus N: byte-balanced file shards, one
    process per GPU)."""
    import time
    t_entry = time.perf_counter()
    shard = _shard_spec(args)
    lead = shard is None or shard[0] == 0
    if getattr(args, "gpus", 1) != 1 and int(os.environ.get("WORLD_SIZE", "1")) > 1 and not os.environ.get("KF_SHARD"):
        # under torchrun every rank is already one shard: a -gpus spawn per rank
        # would count the whole input on every rank and race on the same .kf files
        raise ValueError("-gpus N cannot be combined with torchrun (WORLD_SIZE > 1): each rank counts its own shard")
    if shard is None and getattr(args, "gpus", 1) != 1:
        world = args.gpus
        avail = visible_gpus()
        if world <= 0:
            if avail is None:
                raise ValueError("-gpus 0: cannot count the visible GPUs (no KFD topology, no *_VISIBLE_DEVICES)")
            world = max(1, avail)
        elif not os.environ.get("KF_SHARD_DEVICE") and avail is not None and world > avail:
            raise ValueError("-gpus {}: only {} GPU(s) visible".format(world, avail))
        if world > 1:
            print("\n==> Starting k-mer counting for {}\n".format(args.input_dir))
            for d in (args.input_dir, args.output_dir):
                if not os.path.exists(d):
                    print("No such directory '{}'".format(d), file=sys.stderr)
                    sys.exit(0)
            sys.stdout.flush()   # before the children write to the same stdout
            rc = _spawn_shards(_child_argv(args), world)
            if rc:
                sys.exit(rc)
            print("\n==> Done processing {}".format(args.input_dir))
            return
    if lead and not os.environ.get("KF_SHARD"):
        print("\n==> Starting k-mer counting for {}\n".format(args.input_dir))

    if not os.path.exists(args.input_dir):            # main.py:255-259 (exit status 0, as the reference)
        print("No such directory '{}'".format(args.input_dir), file=sys.stderr)
        sys.exit(0)
    if not os.path.exists(args.output_dir):           # main.py:262-266
        print("No such directory '{}'".format(args.output_dir), file=sys.stderr)
        sys.exit(0)

    files_names, samples_names = list_inputs(args.input_dir)
    if shard is not None:
        sizes = [os.path.getsize(os.path.join(args.input_dir, f)) for f in files_names]
        mine = shard_files(sizes, samples_names, shard[1])[shard[0]]
        files_names = [files_names[i] for i in mine]
        samples_names = [samples_names[i] for i in mine]
    if args.k not in supported_k:
        # reference: UnboundLocalError at main.py:327 for k without a vocab branch
        raise ValueError("k={} has no vocabulary: supported k are {}..{}".format(
            args.k, supported_k.start, supported_k.stop - 1))

    import torch
    from .counter import KmerCounter, pack_files, to_device

    if shard is not None and not os.environ.get("KF_SHARD"):
        # torchrun: join the host-only gloo group now, before counting, so that a
        # rank that fails later drops its connections and the others' final
        # barrier errors out at once instead of waiting for a rendezvous timeout
        _join_group()
    dflt = f"cuda:{os.environ.get('LOCAL_RANK', '0')}" if shard is not None else "cuda"
    device = torch.device(getattr(args, "device", None) or dflt)
    if not files_names:   # an empty shard
        _finish(args, shard, lead)
        return
    counter = KmerCounter(args.k, device)
    paths = [os.path.join(args.input_dir, f) for f in files_names]
    # the first two batches are a quarter and a half of the others, so that the
    # first H2D and count start sooner
    # ... and at most _count_cap genomes, so the count matrix of a batch (on the
    # device, pinned for the writer, `behind` batches deep) stays bounded at any k
    batch_gb = getattr(args, "batch_gb", None)
    fsz = [os.path.getsize(p) for p in paths]
    asz = [(x + 15) // 16 * 16 for x in fsz]   # bytes in a batch (16-byte aligned files)
    batches = _size_batches(fsz, _pipeline_budget(paths, batch_gb, fsz), ramp=True,
                            max_files=_count_cap(4 * counter.nbins, batch_gb))
    # the reference processes files in order and later ones overwrite earlier
    # ones with the same sample name: keep the last occurrence only
    last = {s: i for i, s in enumerate(samples_names)}
    threads = cli_host_threads(args)
    from collections import deque
    from concurrent.futures import ThreadPoolExecutor

    files_pool = ThreadPoolExecutor(max_workers=threads)
    # KF_TRACE=1: per-batch stage timeline on stderr (host ms; device events ms
    # from the first H2D's start event), for tools/e2e_bench.py
    trace = os.environ.get("KF_TRACE") == "1"
    t_origin = time.perf_counter()
    tr: list = []

    def now_ms():
        return round((time.perf_counter() - t_origin) * 1e3, 3)

    # pinned input slots, reused round robin (a fresh pinned block per batch costs
    # ~1 ms of allocation on the reader's path): batch i reads into slot i mod
    # n_slots once the H2D that last read that slot has completed
    slot_bytes = max(sum(asz[i] for i in b) for b in batches)
    n_slots = min(len(batches), int(os.environ.get("KF_READ_AHEAD", "2")) + 2)
    slots = [torch.empty(max(slot_bytes, 16), dtype=torch.uint8, pin_memory=True) for _ in range(n_slots)]
    slot_ev: list = [None] * n_slots

    def pack(bi, idx):
        t0 = now_ms()
        tm = {}
        j = bi % n_slots
        if slot_ev[j] is not None:
            slot_ev[j].synchronize()
        # FASTA batches are indexed on the device (to_device -> kf_index_fasta):
        # the readers only copy the files
        hb = pack_files([paths[i] for i in idx], [samples_names[i] for i in idx], pool=files_pool, times=tm,
                        buf=slots[j], index=False)
        # the batch goes to the device on the copy stream as soon as it is read,
        # so its H2D overlaps the previous batch's index, count and copy-back
        # (copies issued while the batch is read, 16 MiB at a time from the
        # native readers, measured no faster: DESIGN section 8)
        with torch.cuda.stream(copy_stream):
            hb.dev_data = hb.data.to(device, non_blocking=True)
            hb.dev_event = torch.cuda.Event()
            hb.dev_event.record(copy_stream)
        slot_ev[j] = hb.dev_event   # the slot is free again once this copy has run
        if trace:
            tr.append(("read", idx[0], t0, now_ms(), tm))
        return hb

    # Three-stage pipeline over batches:
    #   readers (2)   : read the next batches into pinned memory (the native
    #                   pool's threads, pieces of 1 MiB) and put each on the copy
    #                   stream as soon as it is read; as many
    #                   batches are queued for them as there are pinned slots, so
    #                   the reads (and the copies behind them) run back to back
    #                   whatever this thread is doing (r06 KF_TRACE: with only
    #                   the next two queued, the third read started when this
    #                   thread took batch 0, after its ~2.5 ms of set-up, and the
    #                   copy stream idled 1.5 ms)
    #   this thread   : record index + count + D2H of batch i on a side stream
    #   writer thread : wait for batch i's copy-back, format + write its .kf files
    # The prints stay in the reference's per-file order (main.py:332-341).
    stream = torch.cuda.Stream(device)
    copy_stream = torch.cuda.Stream(device)
    # two readers: one read call's tail (its last pieces, the files' opens) and
    # the writer's formatting leave host threads idle that a second batch's read
    # fills
    reader = ThreadPoolExecutor(max_workers=int(os.environ.get("KF_READERS", "2")))
    writer = ThreadPoolExecutor(max_workers=1)
    ahead = n_slots   # batches queued for the readers (read, or copied, but not yet counted)
    reads = deque(reader.submit(pack, i, batches[i]) for i in range(min(ahead, len(batches))))
    # While the first batches are read: the side stream's first event and launch
    # and the device block for a batch (the caching allocator keeps it for this
    # stream) would otherwise cost ~2 ms between the first read and its H2D
    # (KF_TRACE: got 0 -> issue 0, tools/e2e_bench.py).
    big = slot_bytes
    with torch.cuda.stream(copy_stream):   # the batches' device blocks come from the copy stream's pool
        warm = torch.empty(big + 16, dtype=torch.uint8, device=device)
        warm[:16].zero_()
        del warm
    with torch.cuda.stream(stream):
        torch.cuda.Event(enable_timing=True).record(stream)
    copy_stream.synchronize()
    stream.synchronize()
    writes = []
    # batches whose .kf files may still be waiting for the writer: each holds a
    # pinned count matrix (4 x bins B per genome), so the backlog is bounded
    behind = max(1, int(os.environ.get("KF_WRITE_BEHIND", "2")))

    def write(ev, host, names):
        ev.synchronize()
        t0 = now_ms()
        c = host.numpy().view(np.uint32)
        write_kf_files(args.output_dir, names, c, args.pseudocount, args.raw_cnt, threads)
        if trace:
            tr.append(("write", names[0] if names else "", t0, now_ms()))

    evs = []
    for bi, idx in enumerate(batches):
        t_wait = now_ms()
        hb = reads.popleft().result()
        if trace:
            tr.append(("got", bi, t_wait, now_ms()))
        if bi + ahead < len(batches):   # its slot is batch bi's, free once bi's copy has run
            reads.append(reader.submit(pack, bi + ahead, batches[bi + ahead]))
        with torch.cuda.stream(stream):
            if trace:
                e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
                e[0].record(stream)
                evs.append((bi, now_ms(), e))
            db = to_device(hb, device)
            del hb
            if trace:
                e[1].record(stream)
                th = [now_ms()]
            counts, _ = counter.count(db, stream=stream.cuda_stream)
            if trace:
                e[2].record(stream)
                th.append(now_ms())
            keep = [j for j, i in enumerate(idx) if last[samples_names[i]] == i]
            rows = counts if len(keep) == len(idx) else counts[torch.tensor(keep, device=device)]
            host = torch.empty(rows.shape, dtype=rows.dtype, pin_memory=True)
            if trace:
                th.append(now_ms())
            host.copy_(rows, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(stream)
            if trace:
                e[3].record(stream)
                th.append(now_ms())
        for i in idx:
            if args.pseudocount:                       # main.py:332-333
                print(">>> Adding pseudocounts. Sample: {}".format(files_names[i]))
            if not args.raw_cnt:                       # main.py:340-341
                print(">>> Normalizing. Sample: {}".format(files_names[i]))
        if bi >= behind:   # backpressure: at most `behind` batches queued for the writer
            writes[bi - behind].result()
        writes.append(writer.submit(write, ev, host, [samples_names[idx[j]] for j in keep]))
        del host, rows, counts, db
        if trace:
            th.append(now_ms())
            tr.append(("issue", bi, th))   # after: to_device, count, pinned alloc, D2H, prints+submit
    for w in writes:
        w.result()
    t_written = now_ms()
    reader.shutdown()
    writer.shutdown()
    files_pool.shutdown()
    if trace and evs:
        base_cpu = evs[0][1]
        e00 = evs[0][2][0]
        for bi, t_issue, e in evs:   # device times re-based on the first start event's host time
            d = [round(base_cpu + e00.elapsed_time(x), 3) for x in e]
            tr.append(("gpu", bi, t_issue, {"h2d": d[:2], "count": d[1:3], "d2h": d[2:4]}))
        import json
        print(json.dumps({"kf_trace": tr, "total_ms": now_ms(), "written_ms": t_written,
                          "setup_ms": round((t_origin - t_entry) * 1e3, 3)}), file=sys.stderr)

    _finish(args, shard, lead)


def _join_group() -> None:
    """Host-only gloo group of the torchrun ranks (nothing on the data path)."""
    import datetime

    import torch.distributed as dist
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # a rank may wait here for the slowest shard's counting: a long timeout
        dist.init_process_group("gloo", timeout=datetime.timedelta(hours=6))


def _finish(args, shard, lead: bool) -> None:
    """torchrun ranks meet in a gloo barrier (host only, nothing crosses) so rank 0
    prints the reference's last line after every shard is written."""
    if shard is not None and not os.environ.get("KF_SHARD"):
        import torch.distributed as dist
        _join_group()
        dist.barrier()
    if lead and not os.environ.get("KF_SHARD"):
        print("\n==> Done processing {}".format(args.input_dir))


def _child_argv(args) -> list[str]:
    """The get_frequencies command line of a -gpus child (its shard and device
    come from KF_SHARD and -device)."""
    a = ["get_frequencies", "-input_dir", args.input_dir, "-output_dir", args.output_dir, "-k", str(args.k),
         "-p", str(args.p)]
    if args.pseudocount:
        a.append("-pseudocount")
    if args.raw_cnt:
        a.append("-raw_cnt")
    if getattr(args, "batch_gb", None):
        a += ["-batch_gb", str(args.batch_gb)]
    return a


# ---------------------------------------------------------------------------
# get_kmers (main.py:112-184): sparse present-k-mer matrices for the FSW trainer
# ---------------------------------------------------------------------------
_GET_KMERS_DIGIT = {ord("A"): 0, ord("T"): 1, ord("C"): 2, ord("G"): 3}   # main.py:118
_digit_tables: dict = {}


def vocab_digits(k: int) -> np.ndarray:
    """uint8 [nbins, k]: the vocab k-mers as get_kmers digits (A0 T1 C2 G3)."""
    if k not in _digit_tables:
        from .counter import vocab_text
        v = np.frombuffer(vocab_text(k), dtype=np.uint8).reshape(-1, k + 1)[:, :k]
        lut = np.zeros(256, dtype=np.uint8)
        for ch, d in _GET_KMERS_DIGIT.items():
            lut[ch] = d
        _digit_tables[k] = lut[v]
    return _digit_tables[k]


def kmers_matrix(counts: np.ndarray, k: int) -> np.ndarray:
    """float32 [n_present, k+1]: digits of each present canonical k-mer + count /
    total (main.py:165-172).  Rows in vocab (sorted canonical) order; the
    reference's rows follow Jellyfish's hash order, which its FSW consumer
    (models.py:60-64) does not depend on.  While the TOTAL k-mer count (the
    float32 sum) stays below 2^24, that sum is exact in any order, so the
    weights equal the reference's bit for bit.  Above 2^24 total k-mers (genomes
    over ~17 Mbp) np.sum's pairwise float32 result depends on row order, and the
    reference's own result then depends on Jellyfish's hash order: parity there
    is unpinned (no fixture covers it)."""
    counts = np.asarray(counts)
    nz = np.nonzero(counts)[0]
    if nz.size == 0:
        return np.zeros((0, k + 1), dtype=np.float32)
    c = counts[nz].astype(np.float32)
    norm = c / np.sum(c)
    return np.column_stack((vocab_digits(k)[nz].astype(np.float32), norm))


_STD_TO_DIGIT = np.array([0, 2, 3, 1], dtype=np.uint8)   # standard code A0 C1 G2 T3 -> get_kmers digit


def sparse_kmers_matrix(keys: np.ndarray, counts: np.ndarray, k: int) -> np.ndarray:
    """kmers_matrix for the sparse counter (k up to 31): keys are the present
    canonical k-mers as ascending standard 2-bit codes, so the rows come in the
    same (lexicographic) order as kmers_matrix's vocab order."""
    if keys.size == 0:
        return np.zeros((0, k + 1), dtype=np.float32)
    shifts = (2 * np.arange(k - 1, -1, -1, dtype=np.uint64))
    digits = _STD_TO_DIGIT[((keys[:, None] >> shifts[None, :]) & np.uint64(3)).astype(np.intp)]
    c = counts.astype(np.float32)
    norm = c / np.sum(c)                                   # main.py:169
    return np.column_stack((digits.astype(np.float32), norm))


MAX_CALL_BYTES = (1 << 32) - 1   # kf_sparse_count / kf_chunk_compact: 32-bit offsets per call


def _refuse_huge_files(paths: list[str], what: str) -> None:
    """The sparse counter takes one genome per call slice with 32-bit offsets:
    a FASTQ file of 4 GiB or more (get_kmers -k 13..31 cuts only FASTA files into
    pieces) is refused up front, before any output is written, not partway
    through a directory."""
    big = [p for p in paths if os.path.getsize(p) > MAX_CALL_BYTES - 16]
    if big:
        raise ValueError("{}: input file(s) of 4 GiB or more are not supported (per-call 32-bit offsets): {}".format(
            what, ", ".join(os.path.basename(p) for p in big[:5])))


SPLIT_BYTES = 1 << 30   # get_kmers' sparse path: FASTA files above this are counted in pieces


def _line_start(f, pos: int) -> int:
    """Offset of the first byte of the line holding byte `pos`."""
    step = 1 << 16
    hi = pos
    while hi > 0:
        lo = max(0, hi - step)
        blk = os.pread(f, hi - lo, lo)
        j = blk.rfind(b"\n")
        if j >= 0:
            return lo + j + 1
        hi = lo
    return 0


def _overlap_start(fd: int, s: int, k: int) -> int:
    """The byte where a piece whose windows end at or after s must start: k-1
    sequence positions before s (newlines are transparent, every other byte is a
    position), or just after a header line, or the file start."""
    w = 1 << 12
    while True:
        lo = max(0, s - w)
        blk = os.pread(fd, s - lo, lo)
        need, q, o, short = k - 1, len(blk), s, False
        while q > 0 and need > 0:
            q -= 1
            if blk[q] == 10:                          # into the line before: a header ends the walk
                ls = blk.rfind(b"\n", 0, q) + 1
                if ls == 0 and lo > 0:
                    short = True
                    break
                if blk[ls: ls + 1] == b">":
                    return lo + q + 1
                continue
            need -= 1
            o = lo + q
        if not short and (need == 0 or lo == 0):
            o = 0 if need > 0 else o
            if o < s and os.pread(fd, 1, o) == b">":   # a '>' inside a line must not start a piece
                o -= 1                                 # (the device index would take it for a header)
            return o
        w <<= 2


def fasta_pieces(path: str, k: int, piece: int = SPLIT_BYTES) -> list[tuple[int, int]]:
    """Byte ranges [(o_i, e_i)] that count a large FASTA file in pieces (each below
    the sparse counter's 32-bit offsets) with every window counted exactly once.
    Piece i owns the windows ending in [s_i, s_{i+1}) (s_0 = 0, the last ends at
    the file end; a cut s_i lies on a sequence line, moved past a header line).
    Its bytes start k-1 sequence positions earlier, at o_i (_overlap_start):
    fewer than k positions before s_i, so no window ends there, and every window
    ending at or after s_i has its context.  Windows never span a header, so
    pieces never need more.  Jellyfish counts a file of any size in one hash
    (kf2vec/main.py:133-145); this is the device counter's way there."""
    size = os.path.getsize(path)
    if size <= piece:
        return [(0, size)]
    cuts = [0]
    fd = os.open(path, os.O_RDONLY)
    try:
        for i in range(1, -(-size // piece)):
            s = i * piece
            ls = _line_start(fd, s)
            if os.pread(fd, 1, ls) == b">":           # a header line: cut after it
                rest = s
                while True:
                    blk = os.pread(fd, 1 << 16, rest)
                    j = blk.find(b"\n")
                    if j >= 0 or not blk:
                        s = rest + (j + 1 if j >= 0 else len(blk))
                        break
                    rest += len(blk)
            if s >= size or s <= cuts[-1]:
                continue
            cuts.append(s)
        return [(_overlap_start(fd, c, k) if c else 0, cuts[i + 1] if i + 1 < len(cuts) else size)
                for i, c in enumerate(cuts)]
    finally:
        os.close(fd)


def _next_record(fd: int, pos: int, size: int) -> int:
    """Offset of the first header line ('>' at a line start) at or after pos
    (pos > 0), or size if there is none."""
    step = 1 << 20
    q = pos - 1                       # the byte before pos: a '\n' there makes pos a line start
    while q < size:
        blk = os.pread(fd, min(step, size - q), q)
        j = blk.find(b"\n>")
        if j >= 0:
            return q + j + 1
        if len(blk) < 2:
            return size
        q += len(blk) - 1             # (a "\n>" across the block edge)
    return size


def record_pieces(path: str, piece: int | None = None) -> list[tuple[int, int]]:
    """Byte ranges [(a_i, e_i)] that cut a FASTA file into parts of about
    `piece` bytes at record starts (header lines), so every part holds whole
    records: get_chunks' windows never span a record, so its parts are counted
    independently (a part's rows follow the previous part's, in file order).
    Bytes before the first header stay in part 0 (no record: seqtk skips them).
    A single record longer than `piece` stays whole.  The reference's
    seqtk/seqkit chain reads a file of any size (kf2vec/main.py:726-760)."""
    piece = SPLIT_BYTES if piece is None else piece
    size = os.path.getsize(path)
    if size <= piece:
        return [(0, size)]
    cuts = [0]
    fd = os.open(path, os.O_RDONLY)
    try:
        while True:
            c = _next_record(fd, cuts[-1] + piece, size)
            if c >= size:
                break
            cuts.append(c)
    finally:
        os.close(fd)
    return [(c, cuts[i + 1] if i + 1 < len(cuts) else size) for i, c in enumerate(cuts)]


def _merge_sorted_counts(parts: list) -> tuple:
    """Union of per-piece (keys int64, counts) device tensors with equal keys'
    counts summed (int64: a merged count may pass 2^32); keys ascending."""
    import torch
    keys = torch.cat([p[0] for p in parts])
    cnts = torch.cat([p[1].to(torch.int64) & 0xFFFFFFFF for p in parts])
    if keys.numel() == 0:
        return keys, cnts
    ks, order = torch.sort(keys)
    u, inv = torch.unique_consecutive(ks, return_inverse=True)
    out = torch.zeros(u.numel(), dtype=torch.int64, device=keys.device).index_add_(0, inv, cnts[order])
    return u, out


def get_kmers(args) -> None:
    """kf2vec/main.py:112-184 on the GPU (the *.fna of input_dir in batches).
    k <= 12: the dense counter's rows, non-zero bins kept; k = 13..31 (the rest
    of the reference's 2..31): the sparse counter (device radix sort of every
    window's canonical code, kf_sparse_count); a FASTA file above SPLIT_BYTES
    goes through it in pieces (fasta_pieces) whose sorted results are merged on
    the device, so no file size is refused."""
    import glob

    import torch
    from .counter import KmerCounter, SparseCounter, counts_to_numpy, pack_files, pack_ranges, to_device

    if not os.path.exists(args.output_dir):             # main.py:121-122
        os.makedirs(args.output_dir)
    fasta_files = glob.glob(os.path.join(args.input_dir, "*.fna"))   # main.py:124
    if not fasta_files:
        return
    device = torch.device(getattr(args, "device", None) or "cuda")
    sparse = args.k > N.KF_MAX_K
    if sparse:   # FASTQ content (first byte '@') is not cut: its record state does not split
        fq = [p for p in fasta_files if os.path.getsize(p) > SPLIT_BYTES and open(p, "rb").read(1) == b"@"]
        _refuse_huge_files(fq, "get_kmers -k {} (kf_sparse_count, FASTQ content)".format(args.k))
    counter = SparseCounter(args.k, device) if sparse else KmerCounter(args.k, device)
    batch_gb = float(getattr(args, "batch_gb", 4.0) or 4.0)
    budget = int(batch_gb * (1 << 30))
    if sparse:   # ~21 (k <= 16) / ~29 device bytes per input byte with the outputs; 32-bit offsets
        budget = min(budget, 1 << 30)
    # dense k <= 12: the whole count matrix comes back to the host, 4 x bins per
    # genome whatever its size (33.6 MB at k=12): at most -batch_gb of it per batch
    cap = None if sparse else _count_cap(4 * counter.nbins, batch_gb)
    if sparse and any(os.path.getsize(p) > SPLIT_BYTES for p in fasta_files):
        _get_kmers_pieces(args, fasta_files, counter, device, budget)
        return
    for idx in _batches(fasta_files, budget, max_files=cap):
        paths = [fasta_files[i] for i in idx]
        names = [os.path.basename(p).replace(".fna", "") for p in paths]   # main.py:127
        hb = pack_files(paths, names, threads=host_threads(10))   # the reference's `jellyfish count -t 10`
        if sparse:
            keys, cnts, nu = counter.count(to_device(hb, device), int(hb.off[-1]))
            per = counter.to_host(keys, cnts, nu, hb.off)
            del keys, cnts, nu
        else:
            counts, _ = counter.count(to_device(hb, device))
            c = counts_to_numpy(counts)
        for j, base_name in enumerate(names):
            print(f"--- Processing {base_name} ---")
            m = sparse_kmers_matrix(per[j][0], per[j][1], args.k) if sparse else kmers_matrix(c[j], args.k)
            if m.shape[0] == 0:
                print(f"Warning: No valid ATCG k-mers found in {base_name}")
                continue
            output_path = os.path.join(args.output_dir, f"{base_name}_k{args.k}.npy")
            np.save(output_path, m)
            print(f"Saved: {output_path} (Shape: {m.shape})")


def _get_kmers_pieces(args, fasta_files: list[str], counter, device, budget: int) -> None:
    """get_kmers' sparse path with files above SPLIT_BYTES: every file as its
    fasta_pieces, the pieces in batches of at most `budget` bytes, a file's
    piece results kept on the device until its last piece is counted, then
    merged (_merge_sorted_counts) and written as main.py:147-176 does."""
    import torch
    from .counter import pack_ranges, to_device
    units = []                                    # (file index, start, end)
    for fi, p in enumerate(fasta_files):
        for a, e in fasta_pieces(p, args.k):
            units.append((fi, a, e))
    last = {fi: j for j, (fi, _, _) in enumerate(units)}
    pending: dict = {}
    batch, size = [], 0

    def run(batch):
        hb = pack_ranges([(fasta_files[fi], a, e) for fi, a, e in batch], threads=host_threads(10))
        db = to_device(hb, device)
        keys, cnts, nu = counter.count(db, int(hb.off[-1]))
        nuh = nu.cpu().numpy()
        if nuh.size and ((nuh == -1).any() or (nuh == -2).any()):
            counter.to_host(keys, cnts, nu, hb.off)   # raises the library's error
        for j, (fi, _, _) in enumerate(batch):
            lo, m = int(hb.off[j]), int(nuh[j])
            pending.setdefault(fi, []).append((keys[lo: lo + m].clone(), cnts[lo: lo + m].clone()))
        del keys, cnts, nu, db, hb

    def finish(fi):
        k_, c_ = _merge_sorted_counts(pending.pop(fi))
        base_name = os.path.basename(fasta_files[fi]).replace(".fna", "")   # main.py:127
        print(f"--- Processing {base_name} ---")
        m = sparse_kmers_matrix(k_.cpu().numpy().view(np.uint64), c_.cpu().numpy(), args.k)
        if m.shape[0] == 0:
            print(f"Warning: No valid ATCG k-mers found in {base_name}")
            return
        output_path = os.path.join(args.output_dir, f"{base_name}_k{args.k}.npy")
        np.save(output_path, m)
        print(f"Saved: {output_path} (Shape: {m.shape})")

    done = 0
    for j, u in enumerate(units):
        n = u[2] - u[1]
        if batch and size + n > budget:
            run(batch)
            batch, size = [], 0
            while done < len(fasta_files) and last[done] < j:
                finish(done)
                done += 1
        batch.append(u)
        size += (n + 15) // 16 * 16
    if batch:
        run(batch)
    while done < len(fasta_files):
        finish(done)
        done += 1


# ---------------------------------------------------------------------------
# get_chunks (main.py:654-929): raw-count rows of 10 kbp windows per genome
# ---------------------------------------------------------------------------
def _hms(seconds: float) -> tuple[int, int, int]:
    m, s = divmod(int(seconds), 60)
    h, m = divmod(m, 60)
    return h, m, s


def get_chunks(args) -> None:
    """kf2vec/main.py:654-929 in batches of genome files: each batch is read and
    header-indexed by host threads, linearised / N-collapsed / gap-filtered on the
    device in one pass (kf_chunk_compact), its windows planned from one copy of
    the record bounds, gathered and counted in launches of bounded size, and
    written by a writer thread while the device counts the next launch -- instead
    of seqtk + awk + seqkit per genome and one Jellyfish pair per window.

    Log lines: the reference's per-genome lines ("Start processing", "Done chunk
    processing" or "Excluded ...", "Done computing k-mer frequences") come in its
    order, genome by genome, once the genome's rows are written (so a genome's
    three lines are logged together, after its batch is counted)."""
    import logging
    import time

    from . import chunks as CH
    from .counter import KmerCounter, pack_files, pack_ranges

    CH.TRACE = os.environ.get("KF_TRACE") == "1"
    since = time.time()
    if not os.path.exists(args.input_dir):
        print("No such directory '{}'".format(args.input_dir), file=sys.stderr)
        sys.exit(0)
    if not os.path.exists(args.output_dir):
        print("No such directory '{}'".format(args.output_dir), file=sys.stderr)
        sys.exit(0)
    log = logging.getLogger("kf2vecfsw_amd.get_chunks")
    log.setLevel(logging.INFO)
    log.handlers[:] = [logging.FileHandler(os.path.join(args.output_dir, "get_chunks_{}.log".format(
        os.path.basename(os.path.normpath(args.input_dir)))), "w+"), logging.StreamHandler(sys.stdout)]
    for h in log.handlers:
        h.setFormatter(logging.Formatter("%(message)s"))

    def stamp(msg):
        hrs, _min, sec = _hms(time.time() - since)
        log.info(msg + " Time: {:02d}:{:02d}:{:02d}\n".format(hrs, _min, sec))

    stamp("\n==> Making a list of sample names.")
    files_names, samples_names = list_inputs(args.input_dir)
    stamp("\n==> Start processing samples.")
    if args.k not in supported_k:
        raise ValueError("k={} has no vocabulary: supported k are {}..{}".format(
            args.k, supported_k.start, supported_k.stop - 1))
    import torch
    device = torch.device(getattr(args, "device", None) or "cuda")
    counter = KmerCounter(args.k, device)
    budget = int(float(getattr(args, "batch_gb", 1.0) or 1.0) * (1 << 30))
    # windows per count launch: the window bytes AND the count matrix (4 x bins
    # per window, 8 MiB at k=11) within the budget
    # and at most CH.LAUNCH_WINDOWS, so the writer formats one launch while the
    # device counts and copies back the next
    max_windows = max(1, min(budget // CH.CHUNK_SZ, budget // (4 * counter.nbins), CH.LAUNCH_WINDOWS))
    threads = host_threads(args.p)
    pipe = CH.ChunkPipeline(counter, device, max_windows, threads, args.pseudocount)
    paths = [os.path.join(args.input_dir, f) for f in files_names]
    # units: whole files, or the record-aligned parts of a file above SPLIT_BYTES
    # (each part below kf_chunk_compact's 32-bit offsets; a single record of 4 GiB
    # or more is refused before anything is written)
    units = []   # (file index, start, end, part, parts)
    for fi, p in enumerate(paths):
        pcs = record_pieces(p)
        for j, (a, e) in enumerate(pcs):
            if e - a > MAX_CALL_BYTES - 16:
                raise ValueError("get_chunks (kf_chunk_compact): a FASTA record of 4 GiB or more is not supported "
                                 "(per-call 32-bit offsets): {} at byte {}".format(files_names[fi], a))
            units.append((fi, a, e, j, len(pcs)))
    # input batches of units: about a quarter of the input each (the first two
    # smaller, so the writer starts sooner), so that reading and preparing one
    # batch overlaps writing the previous one, within the budget (and below 4 GiB
    # of processed sequence: kf_chunk_compact's offsets)
    usz = [e - a for _, a, e, _, _ in units]
    batches = _size_batches(usz, min(budget, 3 << 30, max(sum(usz) // 4, 16 << 20)), ramp=True)
    files_pool = ThreadPoolExecutor(max_workers=threads)
    reader = ThreadPoolExecutor(max_workers=1)

    def read(idx):
        t0 = time.perf_counter()
        us = [units[u] for u in idx]
        names = [samples_names[fi] for fi, _, _, _, _ in us]
        if all(n == 1 for *_, n in us):
            hb = pack_files([paths[fi] for fi, *_ in us], names, fmt=N.KF_FMT_FASTA, pool=files_pool)
        else:
            hb = pack_ranges([(paths[fi], a, e) for fi, a, e, _, _ in us], names, threads=threads, index=True)
        CH._tr("read", t0, files=len(idx))
        return hb

    # a file in several parts: windows and long contigs so far; written to a
    # side file that replaces <sample>.kf after its last part (or is removed if
    # the file is excluded or a later file of the same name replaces it)
    acc: dict = {}

    def settle(genomes, us):
        """The parts' exclusions and names; returns the side-file steps for the
        writer: (before this batch's rows) a stale side file of a file whose first
        part is here removed, (after them) the move of a file whose last part is."""
        lasts, first = [], []
        for gm, (fi, _a, _e, j, n) in zip(genomes, us):
            if n == 1:
                continue
            if j == 0:
                first.append(os.path.join(args.output_dir, "{}.kf.parts".format(gm.sample)))
            nw, longc = acc.get(fi, (0, False))
            nw, longc = nw + gm.n_windows, longc or gm.n_windows > 0
            acc[fi] = (nw, longc)
            gm.out_name = "{}.kf.parts".format(gm.sample)
            gm.cont, gm.last = j > 0, j == n - 1
            if not gm.last:
                gm.excluded = None    # decided by the last part
                continue
            gm.total_windows = nw
            gm.excluded = "none" if not longc else ("few" if nw < CH.CHUNK_CNT_THR else None)
            lasts.append(gm)
        CH.shadow(genomes)
        moves = []
        for gm in lasts:
            side = os.path.join(args.output_dir, gm.out_name)
            final = os.path.join(args.output_dir, "{}.kf".format(gm.sample))

            def move(side=side, final=final, keep=gm.excluded is None and gm.write):
                if keep:
                    os.replace(side, final)
                elif os.path.exists(side):
                    os.remove(side)
            moves.append(move)

        def clear(paths=first):
            for p in paths:
                if os.path.exists(p):
                    os.remove(p)
        return clear, moves

    def report(genomes):
        for gm in genomes:
            if not gm.last:
                continue
            log.info("\n==> Start processing. Sample: {}".format(gm.fname))                   # main.py:703
            log.info(">>> Formatting to single line. Sample: {}".format(gm.fname))            # :728
            log.info(">>> Replacing stretches of N. Sample: {}".format(gm.fname))             # :737
            log.info(">>> Filtering contigs below threshold {}. Sample: {}".format(CH.CHUNK_SZ, gm.fname))   # :746
            if gm.excluded == "none":                                                         # :761-778
                stamp("\n==> Excluded {}. No contigs above threshold length.".format(gm.fname))
                continue
            log.info(">>> Splitting into contigs. Sample: {}".format(gm.fname))               # :783
            log.info(">>> Getting contig ids. Sample: {}".format(gm.fname))                   # :789
            log.info(">>> Computing contig statistics. Sample: {}".format(gm.fname))          # :799
            if gm.excluded == "few":                                                          # :845-860
                stamp("\n==> Excluded {}. {} chunks is too low. {} is required.".format(
                    gm.fname, gm.n_windows if gm.total_windows is None else gm.total_windows, CH.CHUNK_CNT_THR))
                continue
            stamp("\n==> Done chunk processing for {}.".format(gm.fname))                    # :866
            # the reference runs get_frequencies on the genome's chunk directory here
            # (main.py:869-881), which prints its first and last lines to stdout
            chunk_dir = os.path.join(args.output_dir, "{}_chunks".format(gm.sample))
            print("\n==> Starting k-mer counting for {}\n".format(chunk_dir))
            print("\n==> Done processing {}".format(chunk_dir))
            stamp("\n==> Done computing k-mer frequences for {}.".format(gm.fname))          # :885

    nxt = reader.submit(read, batches[0]) if batches else None
    prev = None   # (genomes, write futures) of the previous batch, logged once written
    for bi, idx in enumerate(batches):
        t0 = time.perf_counter()
        hb = nxt.result()
        CH._tr("wait_read", t0, batch=bi)
        if bi + 1 < len(batches):
            nxt = reader.submit(read, batches[bi + 1])
        genomes = [CH.Genome(files_names[units[u][0]], samples_names[units[u][0]]) for u in idx]
        d_seq = pipe.prepare(hb, genomes)
        clear, moves = settle(genomes, [units[u] for u in idx])
        t0 = time.perf_counter()
        pipe.after_writes(clear)
        futs = pipe.count_and_write(d_seq, genomes, args.output_dir)
        futs += [pipe.after_writes(f) for f in moves]   # in the writer's order: before the next batch's writes
        CH._tr("issue_counts", t0, launches=len(futs))
        del hb, d_seq
        if prev is not None:
            for f in prev[1]:
                f.result()
            report(prev[0])
        prev = (genomes, futs)
    if prev is not None:
        for f in prev[1]:
            f.result()
        report(prev[0])
    pipe.close()
    reader.shutdown()
    files_pool.shutdown()
    stamp("\n==> Done getting chunks.")
    if CH.TRACE:
        import json
        print(json.dumps({"kf_chunks_trace": CH.trace}), file=sys.stderr)
        CH.trace.clear()


def build_parser() -> argparse.ArgumentParser:
    parser = argparse.ArgumentParser(description="K-mer frequency to distance\n{}".format(__version__),
                                     formatter_class=argparse.RawDescriptionHelpFormatter)
    parser.add_argument("-v", "--version", action="version", version="{}".format(__version__))
    sub = parser.add_subparsers(title="commands", dest="{commands}",
                                description="get_kmers                Extract k-mers and their frequencies from "
                                            "FASTA files\n"
                                            "get_frequencies          Extract k-mer frequency from a reference "
                                            "genome-skims or assemblies\n"
                                            "get_chunks               Extract chunks from reference assemblies\n")
    pf = sub.add_parser("get_frequencies", description="Process a library of reference genome-skims or assemblies")
    pf.add_argument("-input_dir", help="Directory of input genomes or assemblies "
                                       "(dir of .fastq/.fq/.fa/.fna/.fasta files)")
    pf.add_argument("-output_dir", help="Directory for k-mer frequency outputs (dir for .kf files)")
    pf.add_argument("-k", type=int, choices=list(range(min_k_len, max_k_len + 1)), default=default_k_len,
                    help="K-mer length [{}-{}]. Default: {}".format(min_k_len, max_k_len, default_k_len),
                    metavar="K")
    pf.add_argument("-p", type=int, choices=list(range(1, mp.cpu_count() + 1)), default=mp.cpu_count(),
                    help="Max number of processors to use [1-{0}]. Default for this machine: {0}".format(
                        mp.cpu_count()), metavar="P")
    pf.add_argument("-pseudocount", action="store_true",
                    help="Computes k-mer counts with 0.5 pseudocount added to each frequency value")
    pf.add_argument("-raw_cnt", action="store_true", help="Computes raw k-mer counts without normalization")
    pf.add_argument("-batch_gb", type=float, default=None,
                    help="Input bytes per device batch (GiB). Default: about a quarter of the input, 16 MiB..4 GiB")
    pf.add_argument("-device", default=None, help="torch device (default: cuda)")
    pf.add_argument("-gpus", type=int, default=1,
                    help="GPUs to shard the files over, one process each (0 = every visible GPU). Default: 1. "
                         "Under torchrun each rank counts its own shard.")
    pf.set_defaults(func=get_frequencies)

    pk = sub.add_parser("get_kmers", description="Extract kmers and frequencies from FASTA files")
    pk.add_argument("-input_dir", help="Directory of input genomes or assemblies (dir of .fna files)")
    pk.add_argument("-output_dir", help="Directory for k-mer outputs (.npy files)")
    pk.add_argument("-k", type=int, choices=list(range(min_k_len, max_k_len + 1)), default=default_k_len,
                    help="K-mer length [{}-{}]. Default: {}".format(min_k_len, max_k_len, default_k_len),
                    metavar="K")
    pk.add_argument("-batch_gb", type=float, default=4.0, help="Input bytes per device batch (GiB)")
    pk.add_argument("-device", default=None, help="torch device (default: cuda)")
    pk.set_defaults(func=get_kmers)

    pc = sub.add_parser("get_chunks", description="Extract chunks from reference assemblies")
    pc.add_argument("-input_dir", help="Directory of input genomes or assemblies")
    pc.add_argument("-output_dir", help="Directory for chunked k-mer counts (.kf files)")
    pc.add_argument("-k", type=int, choices=list(range(min_k_len, max_k_len + 1)), default=default_k_len,
                    help="K-mer length [{}-{}]. Default: {}".format(min_k_len, max_k_len, default_k_len),
                    metavar="K")
    pc.add_argument("-p", type=int, choices=list(range(1, mp.cpu_count() + 1)), default=mp.cpu_count(),
                    help="Max number of processors to use", metavar="P")
    pc.add_argument("-pseudocount", action="store_true",
                    help="Computes k-mer counts with 0.5 pseudocount added to each frequency value")
    pc.add_argument("-batch_gb", type=float, default=1.0, help="Window bytes per device batch (GiB)")
    pc.add_argument("-device", default=None, help="torch device (default: cuda)")
    pc.set_defaults(func=get_chunks)
    return parser


_PARSER: list = []   # (mp.cpu_count() it was built for, parser)


def _parser() -> argparse.ArgumentParser:
    """build_parser(), kept for later calls in the process (a library caller that
    runs the CLI per directory; building it costs ~1-3 ms), rebuilt if the CPU
    count its -p choices were made for has changed."""
    n = mp.cpu_count()
    if not _PARSER or _PARSER[0][0] != n:
        _PARSER[:] = [(n, build_parser())]
    return _PARSER[0][1]


def main(argv=None) -> None:
    parser = _parser()
    args = parser.parse_args(argv)
    if os.environ.get("KF_SHARD"):
        # a -gpus child shares its parent's stdout with the other shards: one
        # write per line, so concurrent shards never split each other's lines
        sys.stdout.reconfigure(line_buffering=True)
    if hasattr(args, "func"):
        args.func(args)
    else:
        parser.print_help()


if __name__ == "__main__":
    main()
