"""Read-ceiling probe (kf_stream_probe) over a bench-sized device buffer: median and
best of 10 launches for 1 and 2 workgroups per CU (KF_PROBE_WGS_PER_CU)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kf2vecfsw_amd import _native as N  # noqa: E402

n = 5_062_656_000
d = torch.empty(n + 4096, dtype=torch.uint8, device="cuda")
d.fill_(0x41)
out = torch.zeros(1, dtype=torch.int32, device="cuda")
for rnd in range(2):
    for wpc in ("1", "2"):
        os.environ["KF_PROBE_WGS_PER_CU"] = wpc
        ts = []
        for _ in range(10):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            N.check(N.lib().kf_stream_probe(d.data_ptr(), n, out.data_ptr(), None), "kf_stream_probe")
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        t = np.array(ts)
        print(f"round {rnd} wgs/cu {wpc}: median {n / np.median(t) / 1e6:.0f} GB/s, best {n / t.min() / 1e6:.0f} GB/s",
              flush=True)
