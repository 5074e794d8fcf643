"""Per-kernel SQ counter totals of tools/ab_pmc.sh variants: python tools/sq_summary.py TAG NVARIANTS [KERNEL_SUBSTR ...]
Prints, per kernel and variant, the counters summed over its dispatches plus the derived ratios
VALU-busy = SQ_ACTIVE_INST_VALU / SQ_BUSY_CYCLES-normalised and instructions per wave."""
import csv
import os
import re
import sys
from collections import defaultdict


def load(path):
    tot = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(path)):
        nm = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("dq::", ""))
        nm = nm.replace("void ", "")[-56:]
        tot[nm][r["Counter_Name"]] += float(r["Counter_Value"])
    return tot


def main():
    tag, nv = sys.argv[1], int(sys.argv[2])
    subs = sys.argv[3:]
    tables = [load(os.path.join("gpurun_out", "%s_%d" % (tag, i), "p_counter_collection.csv")) for i in range(1, nv + 1)]
    names = sorted({n for t in tables for n in t}, key=lambda n: -max(t[n].get("SQ_BUSY_CYCLES", 0) for t in tables))
    for n in names:
        if subs and not any(s in n for s in subs):
            continue
        if "rocclr" in n or "synth" in n:
            continue
        print(n)
        for i, t in enumerate(tables):
            c = t.get(n)
            if not c:
                continue
            w = max(c.get("SQ_WAVES", 1), 1)
            print("  v%d " % (i + 1) + " ".join("%s=%.3g" % (k.replace("SQ_", ""), v) for k, v in sorted(c.items())))
            print("     per wave: VALU %.0f LDS %.0f SALU %.0f | WAIT_ANY/BUSY %.2f WAIT_LDS/BUSY %.2f ACTIVE_VALU/BUSY %.2f"
                  % (c.get("SQ_INSTS_VALU", 0) / w, c.get("SQ_INSTS_LDS", 0) / w, c.get("SQ_INSTS_SALU", 0) / w,
                     c.get("SQ_WAIT_ANY", 0) / max(c.get("SQ_BUSY_CYCLES", 1), 1),
                     c.get("SQ_WAIT_INST_LDS", 0) / max(c.get("SQ_BUSY_CYCLES", 1), 1),
                     c.get("SQ_ACTIVE_INST_VALU", 0) / max(c.get("SQ_BUSY_CYCLES", 1), 1)))


main()
