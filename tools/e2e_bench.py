"""End-to-end `get_frequencies` on a directory of bacterial-like FASTA files
(BASELINE.json configs[2]: 1xMI355X, k=7, 64 bacterial .fna ~5 Mbp each).

No bacterial assemblies are available offline, so genomes are synthesised on the host:
* 1-80 contigs;
* GC 30-70 %;
* N runs;
* 60- or 80-column lines;
* soft-masked (lowercase) stretches.

Steps:
1. Time the CLI path: file read + record index + H2D + kernel + D2H + `.kf` write.
2. Time each phase separately.
3. Check every `.kf` byte-for-byte against the oracle (CPU restatement).

  python tools/e2e_bench.py [--genomes 64] [--threads 16] [--dir /tmp/kf_e2e]
"""
import argparse
import json
import os
import shutil
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def bacterial_like(rng, total=5_000_000):
    import gen
    ncontig = int(rng.integers(1, 81))
    cuts = np.sort(rng.choice(np.arange(1, total), size=ncontig - 1, replace=False)) if ncontig > 1 else []
    lens = np.diff(np.concatenate([[0], cuts, [total]]))
    gc = float(rng.uniform(0.3, 0.7))
    width = int(rng.choice([60, 80]))
    out = []
    for i, L in enumerate(lens):
        seq = gen.random_seq(rng, int(L), gc=gc, n_rate=2e-5)
        if rng.random() < 0.3 and L > 2000:      # a soft-masked stretch
            a = int(rng.integers(0, L - 1000))
            seq[a: a + 1000] |= 0x20
        out.append(b">contig_%d len=%d\n" % (i, L) + gen.wrap(seq, width))
    return b"".join(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--genomes", type=int, default=64)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--dir", default="/dev/shm/kf_e2e" if os.access("/dev/shm", os.W_OK) else "/tmp/kf_e2e")
    ap.add_argument("--modes", default="read", help="variants to A/B in one process: name[:ENV=VAL[+ENV=VAL]],... "
                    "(e.g. read,r1:KF_READERS=1)")
    ap.add_argument("--k", type=int, default=7)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch
    import kf_oracle as O
    from kf2vecfsw_amd import counter as C
    from kf2vecfsw_amd import main as M

    inp, out = os.path.join(args.dir, "in"), os.path.join(args.dir, "out")
    shutil.rmtree(args.dir, ignore_errors=True)
    os.makedirs(inp)
    os.makedirs(out)
    rng = np.random.default_rng(2026)
    t0 = time.perf_counter()
    sizes = []
    for g in range(args.genomes):
        b = bacterial_like(rng)
        sizes.append(len(b))
        with open(os.path.join(inp, "B%04d.fna" % g), "wb") as f:
            f.write(b)
    gen_s = time.perf_counter() - t0

    cli = ["get_frequencies", "-input_dir", inp, "-output_dir", out, "-k", str(args.k), "-p", str(args.threads)]
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        M.main(cli)                   # warm: runtime init, kernel load, page cache
    # A/B in one process: each read mode pipelined (auto batch size), and one batch
    variants = {}
    for spec in [m for m in args.modes.split(",") if m]:
        name, _, envs = spec.partition(":")
        env = dict(kv.split("=", 1) for kv in envs.split("+") if kv)
        variants[name] = env
    modes = list(variants)
    base_env = {k: os.environ.get(k) for e in variants.values() for k in e}

    def set_env(m):
        for k, v in base_env.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        os.environ.update(variants[m])
    walls = {m: [] for m in modes}
    walls["one_batch"] = []
    parity_modes = {}
    for _ in range(args.reps):
        for m in modes:
            set_env(m)
            t0 = time.perf_counter()
            with contextlib.redirect_stdout(io.StringIO()):
                M.main(cli)
            walls[m].append(time.perf_counter() - t0)
        set_env(modes[0])
        t0 = time.perf_counter()
        with contextlib.redirect_stdout(io.StringIO()):
            M.main(cli + ["-batch_gb", "64"])
        walls["one_batch"].append(time.perf_counter() - t0)
    for m in modes:   # each mode's files against the oracle (below: the last run's)
        set_env(m)
        o2 = out + "_" + m
        os.makedirs(o2, exist_ok=True)
        with contextlib.redirect_stdout(io.StringIO()):
            M.main(["get_frequencies", "-input_dir", inp, "-output_dir", o2, "-k", str(args.k), "-p", str(args.threads)])
        parity_modes[m] = o2
    cli_s = min(walls[modes[0]])
    # one traced pipelined run per mode: per-batch stage timeline (KF_TRACE=1, stderr)
    trace = {}
    for m in modes:
        buf = io.StringIO()
        os.environ["KF_TRACE"] = "1"
        set_env(m)
        with contextlib.redirect_stderr(buf), contextlib.redirect_stdout(io.StringIO()):
            M.main(cli)
        del os.environ["KF_TRACE"]
        trace[m] = [json.loads(line) for line in buf.getvalue().splitlines() if line.startswith('{"kf_trace"')]
    set_env(modes[0])

    # phase breakdown on the same files
    dev = torch.device("cuda:0")
    files, samples = M.list_inputs(inp)
    paths = [os.path.join(inp, f) for f in files]
    kc = C.KmerCounter(args.k, dev)
    ph = {}
    t = time.perf_counter(); hb = C.pack_files(paths, samples, threads=args.threads); ph["read+index"] = time.perf_counter() - t
    t = time.perf_counter(); db = C.to_device(hb, dev); torch.cuda.synchronize(); ph["h2d"] = time.perf_counter() - t
    t = time.perf_counter(); cnt, tot = kc.count(db); torch.cuda.synchronize(); ph["kernel"] = time.perf_counter() - t
    t = time.perf_counter(); c = C.counts_to_numpy(cnt); ph["d2h"] = time.perf_counter() - t
    t = time.perf_counter(); M.write_kf_files(out, samples, c, False, False, args.threads); ph["format+write"] = time.perf_counter() - t
    bases = hb.seq_chars()

    # parity: every .kf against the oracle
    ok = 0
    for f, s in zip(files, samples):
        data = open(os.path.join(inp, f), "rb").read()
        oc, _ = O.count(data, args.k)
        exp = O.kf_line(s, oc).encode()
        ok += all(open(os.path.join(d, s + ".kf"), "rb").read() == exp for d in [out] + list(parity_modes.values()))
    res = {"config": f"1xMI355X, k={args.k}, {args.genomes} bacterial-like .fna (~5 Mbp, 1-80 contigs)",
           "bytes": int(sum(sizes)), "seq_chars": int(bases), "gen_s": round(gen_s, 2),
           "cli_wall_s": round(cli_s, 4), "cli_Gbases_s": round(bases / cli_s / 1e9, 3),
           "cli_wall_s_all": {k: [round(x, 4) for x in v] for k, v in walls.items()},
           "cli_Gbases_s_best": {k: round(bases / min(v) / 1e9, 3) for k, v in walls.items()},
           "phases_s": {k: round(v, 5) for k, v in ph.items()},
           "kernel_Gbases_s": round(bases / ph["kernel"] / 1e9, 1),
           "h2d_GBps": round(sum(sizes) / ph["h2d"] / 1e9, 1),
           "parity_kf_byte_exact": f"{ok}/{len(files)}",
           "trace_pipelined": trace}
    print(json.dumps(res))
    shutil.rmtree(args.dir, ignore_errors=True)
    if ok != len(files):
        sys.exit(1)


if __name__ == "__main__":
    main()
