"""Debug the sparse counter's MSD path on small inputs against the oracle."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def run(blobs, k):
    import torch
    from kf2vecfsw_amd import counter as C
    dev = torch.device("cuda:0")
    hb = C.pack_genomes(blobs)
    sc = C.SparseCounter(k, dev)
    keys, cnts, nu = sc.count(C.to_device(hb, dev), int(hb.off[-1]))
    torch.cuda.synchronize()
    return sc.to_host(keys, cnts, nu, hb.off)


def main():
    import gen
    import kf_oracle as O
    cases = {
        "plain": lambda r: [gen.random_fasta(r, 20000)],
        "plain_big": lambda r: [gen.random_seq(r, 100000).tobytes()],
        "polyA_small": lambda r: [b"A" * 5000],
        "polyA_big": lambda r: [b"A" * 50000],
        "poly_runs": lambda r: [gen.random_fasta(r, 20000, poly_rate=0.5)],
        "two": lambda r: [gen.random_seq(r, 9000).tobytes(), gen.random_seq(r, 9000).tobytes()],
    }
    for k in (12, 13, 21):
        for name, mk in cases.items():
            blobs = mk(np.random.default_rng(7))
            got = run(blobs, k)
            msg = []
            for i, b in enumerate(blobs):
                ek, ec = O.sparse_count(b, k)
                gk, gc = got[i]
                ok = gk.size == ek.size and np.array_equal(gk, ek) and np.array_equal(gc, ec)
                srt = bool(np.all(np.diff(gk.astype(np.int64)) > 0)) if gk.size > 1 else True
                msg.append(f"g{i}: ok={ok} n={gk.size}/{ek.size} sorted={srt} sum={int(gc.sum())}/{int(ec.sum())}")
                if not ok:
                    m = min(gk.size, ek.size)
                    bad = np.nonzero((gk[:m] != ek[:m]) | (gc[:m] != ec[:m]))[0]
                    msg.append(f"   first bad {bad[:6].tolist()} got {gk[bad[:6]].tolist()} want {ek[bad[:6]].tolist()}")
            print(k, name, " | ".join(msg), flush=True)


if __name__ == "__main__":
    main()
