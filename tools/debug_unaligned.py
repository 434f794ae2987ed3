"""Debug helper: reproduce test_unaligned_genome_offsets[k] and report per-genome diffs."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'tests'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'oracle'))
import numpy as np, torch
import gen, kf_oracle as O
from test_gpu_parity import run_batch
k = int(sys.argv[1]) if len(sys.argv) > 1 else 3
dev = torch.device('cuda:0')
rng = np.random.default_rng(7 * k)
sizes = [0, 1, 5, 15, 16, 17, 33, 1023, 1024, 1025, 3000, 70000]
blobs = [gen.random_fasta(rng, s, max_records=3, n_rate=0.001) for s in sizes * 3]
rng.shuffle(blobs)
gaps = rng.integers(0, 40, size=len(blobs))
off = [0]
for b, g in zip(blobs, gaps):
    off.append(off[-1] + len(b) + int(g))
counts, totals = run_batch(blobs, k, dev, offsets=off)
vocab = O.vocab_text(k).split()
for i, b in enumerate(blobs):
    c, t = O.count(b, k)
    if int(totals[i]) != t or not (counts[i] == c).all():
        d = counts[i].astype(np.int64) - c
        print(f"genome {i} off={off[i]}..{off[i+1]} len={len(b)} gpu_total={int(totals[i])} oracle={t}")
        for j in np.nonzero(d)[0][:10]:
            print("   bin", j, vocab[j].decode(), "diff", int(d[j]))
        print("   repr:", repr(b[:300]))
        # same genome alone, aligned and at the same offset mod 16
        for lead in (0, off[i] % 1024, off[i] % 16):
            cc, tt = run_batch([b"A"*0, b] if False else [b], k, dev, offsets=[0, len(b)] if lead == 0 else None)
            print("   alone lead", lead, "total", int(tt[0]), "ok" if (cc[0] == c).all() else "BAD")
