"""String pass of the C5 shard (pass 1's Completeness / ApproxCountDistinct / DataType over the 10 UTF-8 columns of
one 1.25e8-row chunk): dq_scan time with the string scan at 4 vs 8 workgroups per CU (DQ_STR_WG_PER_CU), interleaved.

    python tools/strings_ab.py [rows] [rounds]
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
an = []
for n in names:
    an += [D.Completeness(n), D.ApproxCountDistinct(n), D.DataType(n)]
ref = None
for r in range(rounds + 1):
    for per_cu in ("4", "8"):
        os.environ["DQ_STR_WG_PER_CU"] = per_cu
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ctx = D.AnalysisRunner.onData(t).addAnalyzers(an).run()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        vals = {repr(a): ctx.metric(a).value.get() for a in an}
        vals = {k: (v.values if hasattr(v, "values") else v) for k, v in vals.items()}
        if ref is None:
            ref = repr(sorted(vals.items()))
        assert repr(sorted(vals.items())) == ref, "metrics differ"
        print("round %d: %s workgroups per CU: %.2f ms (%d string columns x %d rows)" % (r, per_cu, ms, len(names), rows),
              flush=True)
os.environ.pop("DQ_STR_WG_PER_CU", None)
