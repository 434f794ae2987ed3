"""Summarise rocprofv3 --pmc counter_collection.csv files: per-dispatch mean of each
counter for kernels matching a pattern."""
import csv, glob, sys, collections, os
root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
pat = sys.argv[2] if len(sys.argv) > 2 else "count_kernel"
vals = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if pat not in r["Kernel_Name"]:
            continue
        per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (d, c), v in per.items():
        vals[c].append(v)
for c, v in sorted(vals.items()):
    print(f"{c:28s} mean/dispatch {sum(v)/len(v):16.4g}  (n={len(v)})")
