"""HBM traffic of one dq_scan call from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE), per
MI355X_MICROARCH.md (HBM section): both counters are in KiB; on gfx950 FETCH_SIZE reports half the
bytes of wide (16 B/lane) coalesced streaming reads, so it is doubled; WRITE_SIZE is exact.

    python tools/pmc_traffic.py FETCH.csv WRITE.csv --rows 1e9 --out profiles/r01/c2_traffic.json

Only the engine's scan kernels are summed (synthetic-data generators and torch fills excluded);
the per-call figure divides by the number of finalize_kernel dispatches (one per dq_scan call).
"""
import argparse
import csv
import json

SCAN_KERNELS = ("scan_values_kernel", "scan_heavy8_kernel", "scan_bits_kernel", "predicate_kernel", "reduce_partials_kernel",
                "reduce_hll_kernel", "finalize_kernel", "pred_simple_kernel", "where_masks_kernel")
# --all-engine: every kernel except the input generators and torch / runtime fills and copies
NOT_ENGINE = ("synth_", "at::native", "__amd_rocclr", "elementwise_kernel")


def per_kernel(path, all_engine=False):
    out = {}
    calls = 0
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if "finalize_kernel" in name:
            calls += 1
        keep = not any(k in name for k in NOT_ENGINE) if all_engine else any(k in name for k in SCAN_KERNELS)
        if keep:
            out[name] = out.get(name, 0.0) + float(r["Counter_Value"]) * 1024.0
    return out, calls


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--rows", type=float, required=True)
    ap.add_argument("--bytes-per-row", type=float, default=65.0)
    ap.add_argument("--out", required=True)
    ap.add_argument("--calls", type=int, default=0, help="invocations profiled (default: finalize_kernel dispatches)")
    ap.add_argument("--all-engine", action="store_true", help="every engine kernel (grouping, KLL, strings, casts)")
    a = ap.parse_args()
    f, calls = per_kernel(a.fetch, a.all_engine)
    w, calls_w = per_kernel(a.write, a.all_engine)
    if a.calls:
        calls = calls_w = a.calls
    assert calls == calls_w and calls > 0, (calls, calls_w)
    fetch = 2.0 * sum(f.values()) / calls  # gfx950: FETCH_SIZE counts half of 16-B/lane streaming reads
    write = sum(w.values()) / calls
    alg = a.bytes_per_row * a.rows
    res = {"calls": calls, "rows": a.rows, "fetch_bytes_per_call": fetch, "write_bytes_per_call": write,
           "traffic_bytes_per_call": fetch + write, "algorithmic_bytes_per_call": alg,
           "traffic_over_algorithmic": (fetch + write) / alg,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; KiB x 1024; "
                     "FETCH_SIZE x 2 (gfx950 wide-read correction, MI355X_MICROARCH.md); %s"
                     % ("every engine kernel (generators excluded)" if a.all_engine else "scan kernels only"),
           "per_kernel_fetch": {k: 2.0 * v / calls for k, v in f.items()},
           "per_kernel_write": {k: v / calls for k, v in w.items()},
           "sources": [a.fetch, a.write]}
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
