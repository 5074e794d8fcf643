"""Secondary measurements for the other BASELINE.json configs (one JSON line each, single GPU):

  c3     ApproxCountDistinct(k) + Correlation(x, y) + Completeness over 1e9 rows (k = splitmix64 mod 2^30,
         x, y ~ sum-of-uniforms normals, 1 % nulls)                                  24.4 B/row
  c4     Uniqueness / Distinctness / UniqueValueRatio / CountDistinct / Entropy on 1e9 int64 keys with
         exactly 1e8 distinct (5e7 x 19 + 5e7 x 1), checked against the closed forms   8 B/row (+ table)
  kll    KLLSketch(x) (sketch 2048, shrinking 0.64) over 1e9 fp64 rows [kll_nulls: 1 % nulls]  8 B/row
  suite10  the north-star "10-analyzer" fused scan: C2 columns + Compliance(c_i > 0), ApproxCountDistinct(c_i),
         Correlation(c_2k, c_2k+1)                                                    65 B/row

    python tools/bench_configs.py --config c4 [--rows 1e9] [--steps 5]
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PEAK = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", required=True, choices=["c3", "c4", "suite10", "s10_nocorr", "corr4", "hll8", "c2", "kll",
                                                         "kll_nulls", "c2where", "c5"])
    ap.add_argument("--rows", type=float, default=1e9)
    ap.add_argument("--distinct", type=float, default=1e8)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    args = ap.parse_args()
    import torch
    import deequ_amd as D
    import deequ_amd.native as N
    from deequ_amd import engine
    from deequ_amd.table import Table, Column
    import bench

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    ctx = engine.ctx()
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    R = int(args.rows)

    def col(name, kind, seed, spark_type, nulls=True):
        dt = torch.float64 if spark_type == N.TYPE_DOUBLE else torch.int64
        v = torch.empty(R, dtype=dt, device=dev)
        ctx.synth_column(kind, seed, 0, R, v.data_ptr())
        c = Column(name, spark_type, None, None, length=R)
        c.device = {"values": v}
        if nulls:
            m = torch.zeros((R + 63) // 64 * 8, dtype=torch.uint8, device=dev)
            ctx.synth_validity(seed + 0x100, 0, R, 10, m.data_ptr())
            c.device["validity"] = m
        return c

    if args.config == "c3":  # the columns of bench.bench_c3
        t = Table([col("k", 5, 0xC3000001, N.TYPE_LONG), col("x", 6, 0xC3000002, N.TYPE_DOUBLE),
                   col("y", 7, 0xC3000002, N.TYPE_DOUBLE)])
        analyzers = [D.ApproxCountDistinct("k"), D.Correlation("x", "y"), D.Completeness("k")]
        bytes_per_row = 3 * (8 + 1 / 8)
    elif args.config == "c2where":
        t = bench.build_shard(torch, N, ctx, 0, R, dev)
        w = "c4 < 0"
        analyzers = [D.Size(w)]
        for c in t.columns:
            analyzers += [D.Completeness(c, w), D.Mean(c, w), D.Sum(c, w), D.Minimum(c, w), D.Maximum(c, w),
                          D.StandardDeviation(c, w)]
        bytes_per_row = 8 * (8 + 1 / 8)
    elif args.config == "c5":
        t, nbytes = bench.c5_shard(torch, N, ctx, dev, R)
        analyzers = None
        bytes_per_row = nbytes / R
    elif args.config in ("s10_nocorr", "corr4", "hll8", "c2"):
        # cost breakdown of suite10 (diagnostics)
        t = bench.build_shard(torch, N, ctx, 0, R, dev)
        names = list(t.columns)
        analyzers = []
        if args.config in ("s10_nocorr", "c2"):
            analyzers += bench.c2_analyzers(D, names)
        if args.config == "s10_nocorr":
            analyzers += [D.Compliance("pos_%s" % c, "%s > 0" % c) for c in names]
        if args.config in ("s10_nocorr", "hll8"):
            analyzers += [D.ApproxCountDistinct(c) for c in names]
        if args.config == "corr4":
            analyzers += [D.Correlation(names[2 * i], names[2 * i + 1]) for i in range(4)]
        bytes_per_row = 8 * (8 + 1 / 8)
    elif args.config in ("kll", "kll_nulls"):
        # KLLSketch (default sketch 2048 / 0.64) over one fp64 column, N(100, 15^2)
        t = Table([col("x", 3, 0x5EED0003, N.TYPE_DOUBLE, nulls=args.config == "kll_nulls")])
        analyzers = [D.KLLSketch("x")]
        bytes_per_row = 8 + (1 / 8 if args.config == "kll_nulls" else 0)
    elif args.config == "suite10":
        t = bench.build_shard(torch, N, ctx, 0, R, dev)
        names = list(t.columns)
        analyzers = bench.c2_analyzers(D, names)
        analyzers += [D.Compliance("pos_%s" % c, "%s > 0" % c) for c in names]
        analyzers += [D.ApproxCountDistinct(c) for c in names]
        analyzers += [D.Correlation(names[2 * i], names[2 * i + 1]) for i in range(4)]
        bytes_per_row = 8 * (8 + 1 / 8)
    else:
        keys = torch.empty(R, dtype=torch.int64, device=dev)
        ctx.synth_freq_keys(R, int(args.distinct), 0, R, keys.data_ptr())
        c = Column("k", N.TYPE_LONG, None, None, length=R)
        c.device = {"values": keys}
        t = Table([c])
        analyzers = [D.Uniqueness(["k"]), D.Distinctness(["k"]), D.UniqueValueRatio(["k"]), D.CountDistinct(["k"]),
                     D.Entropy("k")]
        bytes_per_row = 8.0
    ctx.synchronize()

    def run():
        if analyzers is None:  # c5: the 3-pass ColumnProfiler
            return D.ColumnProfiler.profile(t)
        return D.AnalysisRunner.onData(t).addAnalyzers(analyzers).run()

    for _ in range(args.warmup):
        res = run()
    torch.cuda.synchronize()
    times = []
    for _ in range(args.steps):
        t0 = time.perf_counter()
        res = run()
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    sec = float(np.median(times))
    out = {"config": args.config, "rows": R, "analyzers": len(analyzers or []), "ms": sec * 1e3, "rows_per_s": R / sec,
           "algorithmic_GBps": bytes_per_row * R / sec / 1e9, "frac_of_peak": bytes_per_row * R / sec / 1e9 / PEAK,
           "note": "end-to-end AnalysisRunner.run() wall time (plan + kernels + host metrics), median of %d"
                   % args.steps}
    if args.config == "c4":
        Dn = int(args.distinct)
        half = Dn // 2
        big = (R - half) / half
        exact_ent = math.fsum([-half * (big / R) * math.log(big / R), -half * (1 / R) * math.log(1 / R)])
        got = {type(a).__name__: res.metric(a).value.get() for a in analyzers}
        out["check"] = {"Uniqueness": got["Uniqueness"] == half / R, "Distinctness": got["Distinctness"] == Dn / R,
                        "UniqueValueRatio": got["UniqueValueRatio"] == 0.5, "CountDistinct": got["CountDistinct"] == Dn,
                        "Entropy_rel_err": abs(got["Entropy"] - exact_ent) / exact_ent}
    elif analyzers:
        out["sample_metrics"] = {repr(a): repr(res.metric(a).value.get())[:200] for a in analyzers[:3]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
