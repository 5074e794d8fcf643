"""Per-queue timeline of one C5 step from a rocprofv3 kernel trace of tools/c5_steps.py: merged runs of the same
kernel (> 0.3 ms) with start / end relative to the step. python tools/c5_timeline.py <trace dir> [step]"""
import csv
import re
import sys

d = sys.argv[1]
want = int(sys.argv[2]) if len(sys.argv) > 2 else 2
steps = []
for line in open(d + "/steps.log"):
    m = re.match(r"step (\d+) ([\d.]+) ms monotonic_ns (\d+) (\d+)", line)
    if m:
        steps.append((int(m.group(3)), int(m.group(4))))
a, b = steps[want]
rows = [r for r in csv.DictReader(open(d + "/c5_kernel_trace.csv")) if a <= int(r["Start_Timestamp"]) < b]


def short(n):
    n = re.sub(r"\(anonymous namespace\)::|dq::|void ", "", n)
    return n[:n.index("(")] if "(" in n else n


print("step %d: %.1f ms" % (want, (b - a) / 1e6))
for q in sorted(set((r["Queue_Id"], r["Stream_Id"]) for r in rows)):
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows
                if (r["Queue_Id"], r["Stream_Id"]) == q)
    runs = []
    for s, e, n in ks:
        if runs and runs[-1][2] == n and s - runs[-1][1] < 200000:
            runs[-1][1] = e
            runs[-1][3] += 1
        else:
            runs.append([s, e, n, 1])
    print("queue %s stream %s: busy %.1f ms" % (q[0], q[1], sum(e - s for s, e, _ in ks) / 1e6))
    for s, e, n, c in runs:
        if e - s > 300000:
            print("   %6.1f-%6.1f %-45s x%d" % ((s - a) / 1e6, (e - a) / 1e6, n[:45], c))
