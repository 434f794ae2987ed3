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
import fnmatch
import multiprocessing as mp
import os
import sys

import numpy as np

from . import _native as N

__version__ = "kf2vec 0.1.3 (kf2vecfsw_amd MI355X)"

default_k_len = 7          # main.py:80
min_k_len = 2              # main.py:81
max_k_len = 31             # main.py:82
supported_k = range(3, 12)  # rule-generated vocab (reference ships 3..9; 10 is a missing blob)

FORMATS = [".fq", ".fastq", ".fa", ".fna", ".fasta"]   # main.py:272


def list_inputs(input_dir: str) -> tuple[list[str], list[str]]:
    """main.py:272-275: files in os.listdir order and their sample names."""
    files_names = [f for f in os.listdir(input_dir)
                   if True in (fnmatch.fnmatch(f, "*" + form) for form in FORMATS)]
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


def _batches(paths: list[str], budget: int) -> list[list[int]]:
    out, cur, size = [], [], 0
    for i, p in enumerate(paths):
        s = os.path.getsize(p)
        if cur and size + s > budget:
            out.append(cur)
            cur, size = [], 0
        cur.append(i)
        size += s
    if cur:
        out.append(cur)
    return out


def get_frequencies(args) -> None:
    """kf2vec/main.py:250-373 on the GPU."""
    print("\n==> Starting k-mer counting for {}\n".format(args.input_dir))

    if not os.path.exists(args.input_dir):            # main.py:255-259 (exit status 0, as the reference)
        print("No such directory '{}'".format(args.input_dir), file=sys.stderr)
        sys.exit(0)
    if not os.path.exists(args.output_dir):           # main.py:262-266
        print("No such directory '{}'".format(args.output_dir), file=sys.stderr)
        sys.exit(0)

    files_names, samples_names = list_inputs(args.input_dir)
    if args.k not in supported_k:
        # reference: UnboundLocalError at main.py:327 for k without a vocab branch
        raise ValueError("k={} has no vocabulary: supported k are {}..{}".format(
            args.k, supported_k.start, supported_k.stop - 1))

    import torch
    from .counter import KmerCounter, counts_to_numpy, pack_files, to_device

    device = torch.device(getattr(args, "device", None) or "cuda")
    counter = KmerCounter(args.k, device)
    budget = int(float(getattr(args, "batch_gb", 4.0) or 4.0) * (1 << 30))
    paths = [os.path.join(args.input_dir, f) for f in files_names]
    # the reference processes files in order and later ones overwrite earlier
    # ones with the same sample name: keep the last occurrence only
    last = {s: i for i, s in enumerate(samples_names)}
    for idx in _batches(paths, budget):
        hb = pack_files([paths[i] for i in idx], [samples_names[i] for i in idx])
        db = to_device(hb, device)
        counts, _ = counter.count(db)
        c = counts_to_numpy(counts)
        keep = []
        for j, i in enumerate(idx):
            if args.pseudocount:                       # main.py:332-333
                print(">>> Adding pseudocounts. Sample: {}".format(files_names[i]))
            if not args.raw_cnt:                       # main.py:340-341
                print(">>> Normalizing. Sample: {}".format(files_names[i]))
            if last[samples_names[i]] == i:
                keep.append(j)
        write_kf_files(args.output_dir, [samples_names[idx[j]] for j in keep], c[keep],
                       args.pseudocount, args.raw_cnt, args.p)

    print("\n==> Done processing {}".format(args.input_dir))


def build_parser() -> argparse.ArgumentParser:
    parser = argparse.ArgumentParser(description="K-mer frequency to distance\n{}".format(__version__),
                                     formatter_class=argparse.RawDescriptionHelpFormatter)
    parser.add_argument("-v", "--version", action="version", version="{}".format(__version__))
    sub = parser.add_subparsers(title="commands", dest="{commands}",
                                description="get_frequencies          Extract k-mer frequency from a reference "
                                            "genome-skims or assemblies\n")
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
    pf.add_argument("-batch_gb", type=float, default=4.0, help="Input bytes per device batch (GiB). Default: 4")
    pf.add_argument("-device", default=None, help="torch device (default: cuda)")
    pf.set_defaults(func=get_frequencies)
    return parser


def main(argv=None) -> None:
    parser = build_parser()
    args = parser.parse_args(argv)
    if hasattr(args, "func"):
        args.func(args)
    else:
        parser.print_help()


if __name__ == "__main__":
    main()
