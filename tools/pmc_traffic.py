"""HBM traffic per launch of the count kernel from rocprofv3 PMC passes.

Reads the FETCH_SIZE and WRITE_SIZE passes written by tools/pmc_variant.sh
(one counter per pass, as MI355X_MICROARCH.md "rocprofv3 PMC slots" requires)
and applies that guide's gfx950 corrections:
  * FETCH_SIZE is in KiB and reports half the bytes of a wide coalesced
    streaming read (16 B per lane) -> bytes = FETCH_SIZE x 1024 x 2;
  * WRITE_SIZE is in KiB -> bytes = WRITE_SIZE x 1024.

  python tools/pmc_traffic.py gpurun_out/pmcv1 --kernel "count_kernel<7, 1>" --k 7 \
      --out profiles/r01/traffic_k7.json
bench.py reports `roofline.traffic` from the JSON for its k.
"""
import argparse
import collections
import csv
import glob
import json
import os


def per_dispatch(root, pat):
    vals = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            if pat not in r["Kernel_Name"]:
                continue
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (_, c), v in per.items():
            vals[c].append(v)
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--k", type=int, required=True)
    ap.add_argument("--workload", default="1000 synthetic 5 Mbp genomes, 80-column FASTA")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    v = per_dispatch(a.root, a.kernel)
    fetch = sum(v["FETCH_SIZE"]) / len(v["FETCH_SIZE"]) * 1024 * 2
    write = sum(v["WRITE_SIZE"]) / len(v["WRITE_SIZE"]) * 1024
    out = {"k": a.k, "kernel": a.kernel, "workload": a.workload,
           "fetch_bytes": round(fetch), "write_bytes": round(write), "traffic_bytes": round(fetch + write),
           "dispatches": len(v["FETCH_SIZE"]),
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes; "
                     "FETCH_SIZE x 1024 x 2 (gfx950 half-count of 16-B/lane reads), WRITE_SIZE x 1024"}
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
