"""Repeat get_chunks (whole files, then record-aligned parts) on the inputs of
tests/test_gpu_parity.py::test_cli_get_chunks_record_parts_equal_whole_files,
with a faulthandler stack dump (and exit) if one call takes over 60 s: a
diagnostic for a one-off silent stall seen on the GPU box (r06 v11).
  python tools/chunks_stress.py [--iters 10]"""
import argparse
import faulthandler
import os
import shutil
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    import contextlib
    import io
    import gen
    from test_gpu_parity import _chunk_genome
    from kf2vecfsw_amd import main as M
    rng = np.random.default_rng(7070)
    work = tempfile.mkdtemp(prefix="kf_chunks_stress_")
    inp = os.path.join(work, "in")
    os.makedirs(inp)
    short = lambda n: b"".join(b">s%d\n" % i + gen.wrap(gen.random_seq(rng, 9000), 80) for i in range(n))
    files = {f"g{i}.fna": _chunk_genome(rng, int(rng.integers(3, 10))) for i in range(5)}
    files["few.fna"] = short(4) + b">long\n" + gen.wrap(gen.random_seq(rng, 21000), 60) + short(3)
    files["none.fna"] = short(8)
    files["dupa.fna"] = _chunk_genome(rng, 8)
    files["dupa.fa"] = b">d\n" + gen.wrap(gen.random_seq(rng, 70000), 70)
    for name, b in files.items():
        with open(os.path.join(inp, name), "wb") as f:
            f.write(b)
    split = M.SPLIT_BYTES
    try:
        for it in range(args.iters):
            for tag, sb in (("whole", split), ("parts", 30000)):
                M.SPLIT_BYTES = sb
                out = os.path.join(work, f"{tag}{it}")
                os.makedirs(out)
                faulthandler.dump_traceback_later(60, exit=True)
                t0 = time.perf_counter()
                with contextlib.redirect_stdout(io.StringIO()):
                    M.main(["get_chunks", "-input_dir", inp, "-output_dir", out, "-k", "7"])
                faulthandler.cancel_dump_traceback_later()
                print(it, tag, round(time.perf_counter() - t0, 3), flush=True)
    finally:
        M.SPLIT_BYTES = split
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
