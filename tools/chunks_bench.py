"""Windows/s of `get_chunks` (reference kf2vec/main.py:654-929) end to end through
the CLI: file read, device pre-pass (kf_chunk_compact), window plan, gather,
one kf_count_batch per batch, row writer.  The reference's own log of the toy
run records ~64 ms per 10 kbp chunk (toy_example/train_tree_chunks/
get_chunks_train_tree_fna.log:16,19: 125 chunks of G000830275 in ~8 s).

  python tools/chunks_bench.py [--genomes 64] [--reps 3]

Inputs: the 4 toy train genomes (tests/golden, ~5 Mbp) and N synthetic
bacterial-like genomes (1-80 contigs, N runs, 60/80 columns; ~5 Mbp each).
Every output row of the toy run is checked against the reference's committed
chunk files (358 rows).
"""
import argparse
import contextlib
import gzip
import io
import json
import os
import shutil
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--genomes", type=int, default=64)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--dir", default="/dev/shm/kf_chunks_bench" if os.access("/dev/shm", os.W_OK)
                    else "/tmp/kf_chunks_bench")
    ap.add_argument("--threads", type=int, default=16)
    args = ap.parse_args()
    from kf2vecfsw_amd import main as M
    from test_gpu_parity import _bacterial_like
    toy = os.path.join(ROOT, "tests", "golden", "toy")
    shutil.rmtree(args.dir, ignore_errors=True)
    sets = {}
    d = os.path.join(args.dir, "toy")
    os.makedirs(d)
    for f in sorted(os.listdir(os.path.join(toy, "train_tree_fna"))):
        open(os.path.join(d, f[:-3]), "wb").write(gzip.open(os.path.join(toy, "train_tree_fna", f)).read())
    sets["toy"] = d
    d = os.path.join(args.dir, "bact")
    os.makedirs(d)
    rng = np.random.default_rng(2026)
    for g in range(args.genomes):
        open(os.path.join(d, "B%04d.fna" % g), "wb").write(_bacterial_like(rng, 5_000_000))
    sets["bacterial_like"] = d
    res = {}
    traces = {}
    for name, inp in sets.items():
        walls = []
        for r in range(args.reps + 1):
            out = os.path.join(args.dir, f"out_{name}")
            shutil.rmtree(out, ignore_errors=True)
            os.makedirs(out)
            t0 = time.perf_counter()
            os.environ["KF_TRACE"] = "1" if r == args.reps else "0"
            err = io.StringIO()
            with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(err):
                M.main(["get_chunks", "-input_dir", inp, "-output_dir", out, "-k", "7", "-p", str(args.threads)])
            for ln in err.getvalue().splitlines():
                if ln.startswith('{"kf_chunks_trace"'):
                    tr = json.loads(ln)["kf_chunks_trace"]
                    t_first = min(e[1] for e in tr) if tr else 0
                    traces[name] = [(e[0], round(e[1] - t_first, 2), round(e[2] - t_first, 2), e[3]) for e in tr]
            if r:   # the first run warms the runtime and the page cache
                walls.append(time.perf_counter() - t0)
        rows = sum(open(os.path.join(out, f)).read().count("\n") for f in os.listdir(out) if f.endswith(".kf"))
        kfb = sum(os.path.getsize(os.path.join(out, f)) for f in os.listdir(out) if f.endswith(".kf"))
        ok = None
        if name == "toy":
            ok = True
            for f in sorted(os.listdir(os.path.join(toy, "train_tree_chunks"))):
                exp = gzip.open(os.path.join(toy, "train_tree_chunks", f)).read().decode().splitlines(True)
                got = open(os.path.join(out, f[:-3])).read().splitlines(True)
                ok &= sorted(got) == sorted(exp)
        w = float(np.median(walls))
        res[name] = {"windows": rows, "wall_s_median": round(w, 4), "windows_per_s": round(rows / w, 1),
                     "ms_per_window": round(w / rows * 1e3, 4),
                     "vs_reference_64ms_per_chunk": round(0.064 / (w / rows), 1),
                     "kf_bytes": kfb, "kf_GBps": round(kfb / w / 1e9, 2), "walls": [round(x, 4) for x in walls],
                     "reference_rows_match": ok}
    shutil.rmtree(args.dir, ignore_errors=True)
    res["trace_last_run"] = traces
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
