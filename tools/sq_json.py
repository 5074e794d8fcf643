"""rocprofv3 --pmc counter_collection.csv -> the SQ-counter JSON layout bench.py reads (profiles/<round>/
suite10_sq_counters_*.json: {"runs": {tag: {kernel: {counter: value per launch}}}}).

python tools/sq_json.py TAG OUT.json CSV [CSV ...] [--match SUBSTR] [--values-per-launch V]

Each counter is the mean over the kernel's dispatches (one dq_scan call launches each heavy kernel once, so the mean is
the per-call value); with --values-per-launch, VALU_per_value = SQ_INSTS_VALU * 64 / V is added."""
import argparse
import collections
import csv
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("out")
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--match", default="scan_heavy8_kernel")
    ap.add_argument("--values-per-launch", type=float, default=0.0)
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for path in a.csv:
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"]
            if a.match not in name:
                continue
            tot[name][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[name].add((path, r["Dispatch_Id"]))
    run = {}
    for name, ctrs in tot.items():
        n = len(disp[name])
        d = {c: v / n for c, v in sorted(ctrs.items())}
        d["dispatches"] = n
        if a.values_per_launch and "SQ_INSTS_VALU" in d:
            d["VALU_per_value"] = d["SQ_INSTS_VALU"] * 64 / a.values_per_launch
        run[name] = d
    doc = {"note": a.note, "runs": {}}
    if os.path.exists(a.out):
        doc = json.load(open(a.out))
    doc["runs"][a.tag] = run
    json.dump(doc, open(a.out, "w"), indent=1)
    print(json.dumps(run, indent=1))


if __name__ == "__main__":
    main()
