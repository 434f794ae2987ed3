"""Timeline of the get_frequencies CLI on bench.py's e2e input (64 bacterial-like
~5 Mbp files in /dev/shm): KF_TRACE=1 stage events of the last of 4 runs, and the
wall time of each run.

  python tools/r04_e2e_trace.py [--genomes 64] [--parts 8]
"""
import argparse
import contextlib
import io
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--genomes", type=int, default=64)
    ap.add_argument("--parts", default="8")
    ap.add_argument("--threads", type=int, default=0)
    args = ap.parse_args()
    import bench
    from kf2vecfsw_amd import main as M
    threads = args.threads or bench.usable_cpus()[0]
    work = tempfile.mkdtemp(prefix="kf_tr_", dir="/dev/shm" if os.access("/dev/shm", os.W_OK) else None)
    try:
        inp = os.path.join(work, "in")
        os.makedirs(inp)
        rng = np.random.default_rng(2026)
        for g in range(args.genomes):
            open(os.path.join(inp, "B%04d.fna" % g), "wb").write(bench.bacterial_like(rng, 5_000_000)[0])
        res = {}
        for parts in args.parts.split(","):   # "P" or "P:A" (KF_READ_AHEAD = A)
            os.environ["KF_BATCH_PARTS"] = parts.split(":")[0]
            os.environ["KF_READ_AHEAD"] = parts.split(":")[1] if ":" in parts else "2"
            walls, trace = [], None
            for r in range(4):
                out = os.path.join(work, f"o{parts}_{r}")
                os.makedirs(out)
                os.environ["KF_TRACE"] = "1" if r == 3 else "0"
                err = io.StringIO()
                with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(err):
                    t0 = time.perf_counter()
                    M.main(["get_frequencies", "-input_dir", inp, "-output_dir", out, "-k", "7", "-p", str(threads)])
                    walls.append(round((time.perf_counter() - t0) * 1e3, 2))
                for ln in err.getvalue().splitlines():
                    if ln.startswith("{\"kf_trace\""):
                        trace = json.loads(ln)
            res[parts] = {"walls_ms": walls, "trace": trace}
        print(json.dumps(res))
    finally:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
