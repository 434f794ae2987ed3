"""Summarise a kernel's ISA (tools/isa.sh output): spills by basic block, and the
fast-path blocks (>= 20 LDS adds) with their VALU / SALU / LDS counts.
  python tools/isa_stat.py /tmp/isa_v22.s [kernel-substring]"""
import re
import sys

path = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "count_kernel"
s = open(path).read()
m = re.search(r"\n(_Z\S*" + re.escape(pat) + r"\S*):[^\n]*\n", s)
body = s[m.end():s.index(".Lfunc_end", m.end())].split("\n")
blocks, cur = [], ["entry", []]
for l in body:
    mm = re.match(r"^(\.LBB\S+):(.*)", l)
    if mm:
        blocks.append(cur)
        cur = [mm.group(1) + mm.group(2)[:60], []]
    elif re.match(r"\s+[a-z_0-9]+", l) and not l.strip().startswith(";"):
        cur[1].append(l.strip())
blocks.append(cur)
tot = {"scratch": 0, "wl": 0}
for name, ins in blocks:
    sc = sum(1 for x in ins if x.startswith("scratch_") or ("buffer_" in x and "s[0:3]" in x))
    wl = sum(1 for x in ins if x.startswith(("v_writelane", "v_readlane")))
    nds = sum(1 for x in ins if x.startswith("ds_add"))
    tot["scratch"] += sc
    tot["wl"] += wl
    if sc or nds >= 20:
        print(f"{name[:70]:70s} n={len(ins):4d} valu={sum(1 for x in ins if x.startswith('v_')):4d} "
              f"salu={sum(1 for x in ins if x.startswith('s_')):3d} ds_add={nds:2d} scratch={sc} lane_rw={wl}")
print("total scratch ops", tot["scratch"], "readlane/writelane", tot["wl"])
