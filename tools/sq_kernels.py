"""Per-kernel SQ counter totals of one or more rocprofv3 --pmc counter_collection CSVs (same run, different counter
sets), with derived ratios: python tools/sq_kernels.py CSV [CSV ...] [--top N] [--match SUBSTR]"""
import argparse
import csv
import re
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    tot = defaultdict(lambda: defaultdict(float))
    for path in a.csv:
        for r in csv.DictReader(open(path)):
            nm = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("dq::", ""))
            nm = nm.replace("void ", "")
            key = r["Counter_Name"]
            if key == "SQ_WAVES" and key in tot[nm] and path != a.csv[0]:
                continue  # SQ_WAVES of the first pass only
            tot[nm][key] += float(r["Counter_Value"])
    rows = sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_BUSY_CYCLES", kv[1].get("SQ_WAVE_CYCLES", 0)))
    for nm, c in rows[:a.top]:
        if a.match and a.match not in nm:
            continue
        w = max(c.get("SQ_WAVES", 1), 1)
        b = max(c.get("SQ_BUSY_CYCLES", 1), 1)
        wc = max(c.get("SQ_WAVE_CYCLES", 1), 1)
        print(nm[:64])
        print("   per wave: " + " ".join("%s=%.0f" % (k.replace("SQ_INSTS_", ""), v / w) for k, v in sorted(c.items())
                                        if k.startswith("SQ_INSTS")))
        print("   busy=%.3g  WAIT_ANY/BUSY=%.2f WAIT_LDS/BUSY=%.2f ACTIVE_VALU/BUSY=%.2f  WAIT_INST_ANY/WAVE_CYC=%.2f "
              "ACTIVE_ANY/WAVE_CYC=%.2f ACTIVE_LDS/WAVE_CYC=%.2f bank_conf/LDS=%.2f"
              % (b, c.get("SQ_WAIT_ANY", 0) / b, c.get("SQ_WAIT_INST_LDS", 0) / b, c.get("SQ_ACTIVE_INST_VALU", 0) / b,
                 c.get("SQ_WAIT_INST_ANY", 0) / wc, c.get("SQ_ACTIVE_INST_ANY", 0) / wc,
                 c.get("SQ_ACTIVE_INST_LDS", 0) / wc,
                 c.get("SQ_LDS_BANK_CONFLICT", 0) / max(c.get("SQ_INSTS_LDS", 1), 1)))


if __name__ == "__main__":
    main()
