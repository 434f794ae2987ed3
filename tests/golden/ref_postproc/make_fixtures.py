#!/usr/bin/env python3
"""Generates tests/golden/ref_postproc/ -- golden vectors of the REFERENCE's own
post-processing for the `.kf` modes and the `.npy` layer that the toy fixtures do
not cover.  Run in the build container only (it reads /root/reference, which
does not exist on the GPU box); the tests read the committed outputs.

How: the reference package is imported from /root/reference with two
throwaway stub modules for its absent third-party imports (`treeswift`,
kf2vec/main.py:27-28, and `fswlib`, kf2vec/models.py:4 -- neither is used by
the functions run here), and its own functions are called:

  * kf2vec.main.get_frequencies (main.py:250-373): vocab read, pd.merge + fillna,
    `+0.5` pseudocount, normalisation, `astype(str)`, the `.kf` write;
  * kf2vec.main.get_kmers (main.py:112-184): dump parse, A0/T1/C2/G3 digits,
    float32 weights, np.save.

Jellyfish (`kmer-jellyfish` 1.1.12, kf2vec_env.yml:35) is absent from this image,
so a `jellyfish` stand-in on PATH answers `count -m K ... -C IN -o OUT` and
`dump -c [-t] JF` with the canonical counts of oracle/kmer_oracle.c, which
tests/test_oracle_golden.py pins byte-exactly against the reference's 7 toy
`.kf` files.  Its dump lists k-mers in sorted (vocab) order; Jellyfish's own
order is its hash order, which the `.kf` path erases (the merge onto the vocab)
and which the `.npy` consumer does not depend on (models.py:60-64).

So these fixtures pin the reference's pandas/numpy post-processing
(main.py:323-357, 147-176) on inputs the toy set lacks: -pseudocount,
-pseudocount -raw_cnt, -raw_cnt on a genome with every bin present (the
reference then prints integers: pd.merge keeps int64 when no NaN appears),
several k, and what the reference does with an empty genome.

  python tests/golden/ref_postproc/make_fixtures.py
"""
from __future__ import annotations

import argparse
import gzip
import hashlib
import io
import json
import os
import shutil
import sys
import tempfile
import traceback

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(os.path.dirname(HERE)))
REF = "/root/reference"
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))

# genome name -> (k, modes); modes are (pseudocount, raw_cnt) pairs
MODES = [(False, False), (True, False), (False, True), (True, True)]


def make_inputs() -> dict[str, bytes]:
    import gen
    rng = np.random.default_rng(20260317)
    g = {}
    # ragged multi-record genome with N runs, lowercase, CRLF: many empty bins at k=7
    g["ragged"] = gen.random_fasta(rng, 30000, max_records=5, n_rate=0.003, lower=0.05, crlf_rate=0.2,
                                   poly_rate=0.01)
    # every k=3 / k=4 bin present (20 kbp uniform): the int64 raw-count quirk
    g["dense"] = b">dense\n" + gen.wrap(gen.random_seq(rng, 20000), 60)
    # a few k-mers only (most bins empty), 0 < total
    g["tiny"] = b">t\nACGTACGTTTGA\n>u\nNNNACGGT\n"
    # low complexity: large counts in few bins
    g["polyA"] = b">a\n" + gen.wrap(np.frombuffer(b"A" * 5000 + b"AC" * 3000, np.uint8), 70)
    return g


def write_stubs(d: str) -> None:
    with open(os.path.join(d, "treeswift.py"), "w") as f:
        f.write("# build-container stub: kf2vec/main.py:27-28 imports it; unused by get_frequencies/get_kmers\n"
                "def read_tree_newick(*a, **k):\n    raise RuntimeError('treeswift stub')\n")
    with open(os.path.join(d, "fswlib.py"), "w") as f:
        f.write("# build-container stub: kf2vec/models.py:4 imports it; unused by get_frequencies/get_kmers\n"
                "class FSWEmbedding:\n    def __init__(self, *a, **k):\n        raise RuntimeError('fswlib stub')\n")


JELLYFISH = r'''#!/usr/bin/env python3
# build-container stand-in for `jellyfish count ... -C` / `jellyfish dump -c [-t]`
# (canonical counts of oracle/kmer_oracle.c; dump in sorted canonical order)
import json, sys
sys.path.insert(0, %(oracle)r)
import kf_oracle as O
a = sys.argv[1:]
if a[0] == "count":
    k = int(a[a.index("-m") + 1]); out = a[a.index("-o") + 1]; inp = a[-3] if a[-2] == "-o" else a[a.index("-C") + 1]
    c, _ = O.count(open(inp, "rb").read(), k)
    vocab = O.vocab_text(k).split()
    json.dump({"k": k, "rows": [[vocab[i].decode(), int(x)] for i, x in enumerate(c) if x]}, open(out, "w"))
elif a[0] == "dump":
    sep = "\t" if "-t" in a else " "
    d = json.load(open(a[-1]))
    sys.stdout.write("".join(f"{km}{sep}{n}\n" for km, n in d["rows"]))
else:
    sys.exit(2)
'''


def main() -> None:
    if not os.path.isdir(os.path.join(REF, "kf2vec")):
        sys.exit("needs the reference at /root/reference (build container only)")
    import kf_oracle as O
    O.build()
    work = tempfile.mkdtemp(prefix="kf_ref_fix_")
    stubs, bindir = os.path.join(work, "stubs"), os.path.join(work, "bin")
    os.makedirs(stubs)
    os.makedirs(bindir)
    write_stubs(stubs)
    jf = os.path.join(bindir, "jellyfish")
    with open(jf, "w") as f:
        f.write(JELLYFISH % {"oracle": os.path.join(REPO, "oracle")})
    os.chmod(jf, 0o755)
    os.environ["PATH"] = bindir + os.pathsep + os.environ["PATH"]
    sys.path.insert(0, stubs)
    sys.path.insert(0, REF)
    import kf2vec.main as RM   # the reference itself

    inputs = make_inputs()
    out_in = os.path.join(HERE, "inputs")
    os.makedirs(out_in, exist_ok=True)
    for name, b in inputs.items():
        with gzip.GzipFile(os.path.join(out_in, name + ".fna.gz"), "wb", mtime=0) as f:
            f.write(b)
    import pandas
    manifest = {"generator": "tests/golden/ref_postproc/make_fixtures.py", "reference": "kf2vec/main.py:250-373, 112-184",
                "pandas": pandas.__version__, "numpy": np.__version__, "kf": [], "npy": [], "errors": []}
    kf_dir = os.path.join(HERE, "kf")
    npy_dir = os.path.join(HERE, "npy")
    os.makedirs(kf_dir, exist_ok=True)
    os.makedirs(npy_dir, exist_ok=True)
    cases = [("ragged", k) for k in (3, 5, 7, 9)] + [("dense", k) for k in (3, 4, 7)] + \
            [("tiny", 7), ("polyA", 6), ("polyA", 8)]
    for name, k in cases:
        for pseudo, raw in MODES:
            d_in, d_out = os.path.join(work, "in"), os.path.join(work, "out")
            shutil.rmtree(d_in, ignore_errors=True)
            shutil.rmtree(d_out, ignore_errors=True)
            os.makedirs(d_in)
            os.makedirs(d_out)
            with open(os.path.join(d_in, name + ".fna"), "wb") as f:
                f.write(inputs[name])
            args = argparse.Namespace(input_dir=d_in, output_dir=d_out, k=k, p=2, pseudocount=pseudo, raw_cnt=raw)
            with open(os.devnull, "w") as dn:
                so = sys.stdout
                sys.stdout = dn
                try:
                    RM.get_frequencies(args)
                finally:
                    sys.stdout = so
            body = open(os.path.join(d_out, name + ".kf"), "rb").read()
            tag = f"{name}_k{k}" + ("_pseudo" if pseudo else "") + ("_raw" if raw else "")
            with gzip.GzipFile(os.path.join(kf_dir, tag + ".kf.gz"), "wb", mtime=0) as f:
                f.write(body)
            manifest["kf"].append({"file": f"kf/{tag}.kf.gz", "input": f"inputs/{name}.fna.gz", "sample": name, "k": k,
                                   "pseudocount": pseudo, "raw_cnt": raw,
                                   "sha256": hashlib.sha256(body).hexdigest()})
    # an empty genome: what the reference does with an empty dump (pandas reads
    # no rows; the merge leaves every bin NaN -> fillna(0) on an object column)
    for pseudo, raw in MODES:
        d_in, d_out = os.path.join(work, "ein"), os.path.join(work, "eout")
        shutil.rmtree(d_in, ignore_errors=True)
        shutil.rmtree(d_out, ignore_errors=True)
        os.makedirs(d_in)
        os.makedirs(d_out)
        open(os.path.join(d_in, "empty.fna"), "wb").close()
        args = argparse.Namespace(input_dir=d_in, output_dir=d_out, k=7, p=2, pseudocount=pseudo, raw_cnt=raw)
        err = None
        so = sys.stdout
        sys.stdout = io.StringIO()
        try:
            RM.get_frequencies(args)
        except Exception as e:   # noqa: BLE001 -- the reference's own failure is the fixture
            err = f"{type(e).__module__}.{type(e).__name__}: {e}"
        finally:
            sys.stdout = so
        tag = "empty_k7" + ("_pseudo" if pseudo else "") + ("_raw" if raw else "")
        ent = {"case": "empty genome", "k": 7, "pseudocount": pseudo, "raw_cnt": raw, "reference_raises": err}
        kf = os.path.join(d_out, "empty.kf")
        if os.path.exists(kf):
            body = open(kf, "rb").read()
            with gzip.GzipFile(os.path.join(kf_dir, tag + ".kf.gz"), "wb", mtime=0) as f:
                f.write(body)
            ent.update(file=f"kf/{tag}.kf.gz", sha256=hashlib.sha256(body).hexdigest(),
                       first_values=body.split(b",")[1:4])
            ent["first_values"] = [x.decode() for x in ent["first_values"]]
        manifest["errors"].append(ent)
    # get_kmers .npy (writes its .jf into the CWD, main.py:128)
    for k in (5, 7):
        d_in, d_out = os.path.join(work, "kin"), os.path.join(work, "kout")
        shutil.rmtree(d_in, ignore_errors=True)
        shutil.rmtree(d_out, ignore_errors=True)
        os.makedirs(d_in)
        for name in ("ragged", "tiny", "polyA"):
            with open(os.path.join(d_in, name + ".fna"), "wb") as f:
                f.write(inputs[name])
        args = argparse.Namespace(input_dir=d_in, output_dir=d_out, k=k)
        cwd = os.getcwd()
        os.chdir(work)
        so = sys.stdout
        sys.stdout = io.StringIO()
        try:
            RM.get_kmers(args)
        finally:
            sys.stdout = so
            os.chdir(cwd)
        for name in ("ragged", "tiny", "polyA"):
            m = np.load(os.path.join(d_out, f"{name}_k{k}.npy"), allow_pickle=False)
            dst = os.path.join(npy_dir, f"{name}_k{k}.npy")
            np.save(dst, m)
            manifest["npy"].append({"file": f"npy/{name}_k{k}.npy", "input": f"inputs/{name}.fna.gz", "k": k,
                                    "shape": list(m.shape), "dtype": str(m.dtype),
                                    "row_order": "jellyfish stand-in dump order = sorted canonical (vocab) order"})
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    shutil.rmtree(work, ignore_errors=True)
    print(f"wrote {len(manifest['kf'])} .kf, {len(manifest['npy'])} .npy fixtures; errors: {manifest['errors']}")


if __name__ == "__main__":
    try:
        main()
    except Exception:
        traceback.print_exc()
        sys.exit(1)
