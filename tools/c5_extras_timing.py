"""Wall time of the C5 extras (ApproxQuantile(0.5) x 10 numeric columns, Uniqueness / Entropy of s_cat100 and of
s_text0) one analyzer group at a time on the C5 shard, printed as they finish:
python tools/c5_extras_timing.py [rows] [group,group...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import bench
import deequ_amd as D
import deequ_amd.native as N
from deequ_amd import engine

rows = int(float(sys.argv[1])) if len(sys.argv) > 1 else 250_000_000
t, _ = bench.c5_shard(torch, N, engine.ctx(), torch.device("cuda", 0), rows)
print("table ready", flush=True)
groups = {"quantiles": [D.ApproxQuantile(n, 0.5) for n, _ in bench.C5_NUMERIC],
          "cat100": [D.Uniqueness(["s_cat100"]), D.Entropy("s_cat100")],
          "text0": [D.Uniqueness(["s_text0"]), D.Entropy("s_text0")]}
only = sys.argv[2].split(",") if len(sys.argv) > 2 else list(groups)
for rep in range(2):
    for name, an in groups.items():
        if name not in only:
            continue
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ctx = D.AnalysisRunner.onData(t).addAnalyzers(an).run()
        torch.cuda.synchronize()
        print("%s rep %d: %.1f ms %s" % (name, rep, (time.perf_counter() - t0) * 1e3,
                                          [str(ctx.metric(a).value)[:60] for a in an[:2]]), flush=True)
