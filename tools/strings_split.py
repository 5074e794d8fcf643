"""Cost split of the C5 string pass (one 1.25e8-row chunk, the 10 UTF-8 columns): dq_scan wall time with
Completeness only, + DataType, + ApproxCountDistinct, and all three — which share of scan_strings_kernel each op takes.

    python tools/strings_split.py [rows] [rounds]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import bench
import deequ_amd as D
import deequ_amd.native as N
from deequ_amd import engine

rows = int(float(sys.argv[1])) if len(sys.argv) > 1 else 125_000_000
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = torch.device("cuda", 0)
t, _ = bench.c5_shard(torch, N, engine.ctx(), dev, rows)
names = [n for n, _ in bench.C5_STRINGS]
sets = {
    "completeness": lambda n: [D.Completeness(n)],
    "datatype": lambda n: [D.Completeness(n), D.DataType(n)],
    "hll": lambda n: [D.Completeness(n), D.ApproxCountDistinct(n)],
    "all": lambda n: [D.Completeness(n), D.ApproxCountDistinct(n), D.DataType(n)],
    "lengths": lambda n: [D.MinLength(n), D.MaxLength(n)],
}
best = {}
for r in range(rounds + 1):
    for name, mk in sets.items():
        an = [a for n in names for a in mk(n)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        D.AnalysisRunner.onData(t).addAnalyzers(an).run()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        if r:
            best[name] = min(best.get(name, 1e9), ms)
for name, ms in best.items():
    print("%-14s %8.2f ms  (%d string columns x %d rows, best of %d)" % (name, ms, len(names), rows, rounds), flush=True)
