"""HBM read rate of the count kernel's access pattern (kf_stream_probe) at 1 and 2
1024-thread workgroups per CU: how much streaming rate 16 waves per CU keep.
  python tools/probe_occ.py [--gb 5]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=5.0)
    args = ap.parse_args()
    import torch
    from kf2vecfsw_amd import _native as N
    n = int(args.gb * 1e9) // 1024 * 1024
    data = torch.ones(n, dtype=torch.uint8, device="cuda")
    out = torch.zeros(1, dtype=torch.int32, device="cuda")
    for wpc in ("2", "1", "2", "1"):
        os.environ["KF_PROBE_WGS_PER_CU"] = wpc
        N.check(N.lib().kf_stream_probe(data.data_ptr(), n, out.data_ptr(), None), "probe")
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(5):
            N.check(N.lib().kf_stream_probe(data.data_ptr(), n, out.data_ptr(), None), "probe")
        b.record()
        torch.cuda.synchronize()
        t = a.elapsed_time(b) / 5
        print(f"WGs/CU {wpc}: {t:.3f} ms  {n / t / 1e6:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
