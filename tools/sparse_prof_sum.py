"""Per-kernel times of the sparse counter's last call at each k in a rocprofv3
--kernel-trace CSV of tools/sparse_bench.py (one call = sp_tiles .. sp_nuniq).

  python tools/sparse_prof_sum.py gpurun_out/r04/v36_prof/run_kernel_trace.csv
"""
import csv
import re
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    seq = [(r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6,
            int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if "sp_" in r["Kernel_Name"]]
    starts = [i for i, x in enumerate(seq) if "sp_tiles" in x[0]] + [len(seq)]
    calls = [seq[a:b] for a, b in zip(starts, starts[1:])]
    # the last call of each key type / pass count: group by the number of dispatches
    last = {}
    for c in calls:
        last[(len(c), any("sp_emit_kernel<unsigned long>" in n for n, *_ in c))] = c
    for key, c in sorted(last.items()):
        agg = {}
        for n, ms, _, _ in c:
            m = re.search(r"(sp_\w+?)[<(]", n)
            a = agg.setdefault(m.group(1), [0.0, 0])
            a[0] += ms
            a[1] += 1
        span = (c[-1][3] - c[0][2]) / 1e6
        print(f"{'u64' if key[1] else 'u32'} {key[0]} dispatches, first start to last end {span:.3f} ms:",
              {k: (round(v[0], 3), v[1]) for k, v in agg.items()})


if __name__ == "__main__":
    main()
