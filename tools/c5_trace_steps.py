"""Per-step kernel time of a rocprofv3 kernel trace of tools/c5_steps.py: wall, kernel sum, GPU-busy union and the
kernels by total time. python tools/c5_trace_steps.py <dir with c5_kernel_trace.csv and steps.log> [step] [top]"""
import collections
import csv
import re
import sys

d = sys.argv[1]
want = int(sys.argv[2]) if len(sys.argv) > 2 else None
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
steps = []
for line in open(d + "/steps.log"):
    m = re.match(r"step (\d+) ([\d.]+) ms monotonic_ns (\d+) (\d+)", line)
    if m:
        steps.append((int(m.group(3)), int(m.group(4))))
rows = list(csv.DictReader(open(d + "/c5_kernel_trace.csv")))


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"^void ", "", name)
    depth, out = 0, ""
    for ch in name:  # drop the argument list, keep template arguments
        if ch == "(" and depth == 0 and out:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out += ch
    return out[:80]


for si, (a, b) in enumerate(steps):
    if si == 0 or (want is not None and si != want):
        continue
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows
          if a <= int(r["Start_Timestamp"]) < b]
    iv = sorted((s, e) for s, e, _ in ks)
    busy, cs, ce = 0, None, None
    for s, e in iv:
        if ce is None or s > ce:
            if ce is not None:
                busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if ce is not None:
        busy += ce - cs
    print("step %d: wall %.1f ms, kernel sum %.1f ms, GPU busy %.1f ms, %d launches"
          % (si, (b - a) / 1e6, sum(e - s for s, e, _ in ks) / 1e6, busy / 1e6, len(ks)))
    agg, cnt = collections.defaultdict(float), collections.Counter()
    for s, e, n in ks:
        agg[short(n)] += (e - s) / 1e6
        cnt[short(n)] += 1
    for n, v in sorted(agg.items(), key=lambda x: -x[1])[:top]:
        print("  %-80s %4d %8.2f" % (n, cnt[n], v))
