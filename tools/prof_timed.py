"""The bench's timed k1x_kernel<7> / bucket_kernel<11> dispatches out of a
rocprofv3 --kernel-trace run of `bench.py --gpus 1 --steps S --warmup W`.

The summary's per-kernel average mixes in the e2e CLI's small launches; the
configs[1] launches are the ones over 0.5 ms (k=7) in order: W warm-up, S timed,
then the cold launch after an idle second.

  python tools/prof_timed.py gpurun_out/r04/v20_prof/run_kernel_trace.csv --steps 20 --warmup 5 \
      --bench gpurun_out/r04/v20_prof_bench.json --out profiles/r04/v20_kernel_trace_timed.json
"""
import argparse
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--bench", default=None, help="the profiled bench's JSON line (for its event times)")
    ap.add_argument("--out", required=True)
    ap.add_argument("--by-k-warmup", type=int, default=3)
    ap.add_argument("--by-k-steps", type=int, default=5)
    a = ap.parse_args()
    k7, k11 = [], []
    per_kernel = {}   # every count kernel's dispatches in order (bench.py's by_k runs come last)
    for r in csv.DictReader(open(a.trace)):
        name = r["Kernel_Name"]
        for tag in ("k1x_kernel<", "bucket_kernel<"):
            if tag in name:
                kk = tag + name.split(tag, 1)[1].split(">", 1)[0] + ">"
                per_kernel.setdefault(kk, []).append(
                    (int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
        ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        if "k1x_kernel<7>" in r["Kernel_Name"] and ms > 0.5:
            k7.append((int(r["Start_Timestamp"]), ms))
        elif "bucket_kernel<11>" in r["Kernel_Name"]:
            k11.append((int(r["Start_Timestamp"]), ms))
    k7 = [m for _, m in sorted(k7)]
    k11 = [m for _, m in sorted(k11)]
    W, S = a.warmup, a.steps
    out = {
        "command": f"rocprofv3 --kernel-trace --stats -- python3 bench.py --gpus 1 --steps {S} --warmup {W}",
        "k1x_kernel<7> dispatches on the configs[1] batch (>0.5 ms), in order": [round(x, 4) for x in k7],
        "warmup_ms": [round(x, 4) for x in k7[:W]],
        "timed_mean_ms": round(sum(k7[W:W + S]) / max(1, len(k7[W:W + S])), 4),
        "timed_n": len(k7[W:W + S]),
        "cold_launch_ms": round(k7[W + S], 4) if len(k7) > W + S else None,
        "bucket_kernel<11> dispatches, in order": [round(x, 4) for x in k11],
    }
    n_by = a.by_k_warmup + a.by_k_steps
    out["by_k timed dispatches (the last --by-k-steps of each kernel; HIP-event kernel_ms beside)"] = {}
    for kk, v in sorted(per_kernel.items()):
        ms = [m for _, m in sorted(v)][-n_by:][a.by_k_warmup:]
        out["by_k timed dispatches (the last --by-k-steps of each kernel; HIP-event kernel_ms beside)"][kk] = {
            "rocprof_mean_ms": round(sum(ms) / max(1, len(ms)), 4), "ms": [round(x, 4) for x in ms]}
    if a.bench:
        b = json.loads(open(a.bench).read().strip().splitlines()[-1])
        out["bench_json_kernel_ms (HIP events around the launch)"] = b["roofline"]["kernel_ms"]
        out["bench_json_secondary_kernel_ms"] = b["secondary"]["roofline"]["kernel_ms"]
        for k, v in (b.get("by_k") or {}).items():
            d = out["by_k timed dispatches (the last --by-k-steps of each kernel; HIP-event kernel_ms beside)"]
            if v["kernel"] in d:
                d[v["kernel"]]["bench_json_kernel_ms"] = v["kernel_ms"]
                d[v["kernel"]]["bench_json_frac"] = v["roofline"]["frac"]
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if not isinstance(v, list)}))


if __name__ == "__main__":
    main()
