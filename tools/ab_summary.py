"""Print the medians of a tools/lib_ab.py JSON file: python tools/ab_summary.py FILE..."""
import json
import sys

for path in sys.argv[1:]:
    t = open(path).read()
    d = json.loads(t[t.index("{"):])
    print(path, "k=%d" % d["k"], "counts_equal=%s" % d["counts_equal"])
    for p, v in d["results"].items():
        print("  %-40s %8.3f ms (min %.3f)" % (p.split("/")[-1], v["median_ms"], v["min_ms"]))
