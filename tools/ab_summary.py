"""Side-by-side kernel times of tools/ab_run.sh variants: python tools/ab_summary.py TAG NVARIANTS [TOPN]
(total ms per kernel name over the profiled run, from each variant's rocprofv3 kernel stats)."""
import csv
import os
import sys

tag, nv = sys.argv[1], int(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 15
tables = []
for i in range(1, nv + 1):
    p = os.path.join("gpurun_out", "%s_%d" % (tag, i), "p_kernel_stats.csv")
    t = {}
    if os.path.exists(p):
        for r in csv.DictReader(open(p)):
            nm = r["Name"]
            for pre in ("void ", "(anonymous namespace)::", "dq::"):
                nm = nm.replace(pre, "")
            name = nm.split("(")[0][-60:]
            t[name] = t.get(name, (0, 0.0))
            t[name] = (t[name][0] + int(r["Calls"]), t[name][1] + float(r["TotalDurationNs"]) / 1e6)
    tables.append(t)
names = sorted({n for t in tables for n in t}, key=lambda n: -max(t.get(n, (0, 0.0))[1] for t in tables))
print("%-60s" % "kernel" + "".join("%16s" % ("v%d ms(calls)" % (i + 1)) for i in range(nv)))
for n in names[:top]:
    print("%-60s" % n + "".join("%10.2f(%4d)" % (t.get(n, (0, 0.0))[1], t.get(n, (0, 0.0))[0]) for t in tables))
print("%-60s" % "TOTAL (excl. synth/copies)" + "".join(
    "%16.2f" % sum(v[1] for k, v in t.items() if "synth" not in k and "rocclr" not in k) for t in tables))
