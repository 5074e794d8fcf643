"""Wall time of Uniqueness / Entropy of the C5 free-text column over a 2-chunk shard (the whole-shard grouping over
the chunks concatenated in HBM): python tools/text_group_timing.py [rows] [chunk_rows]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import bench
import deequ_amd as D
import deequ_amd.native as N
from deequ_amd import engine

rows = int(float(sys.argv[1])) if len(sys.argv) > 1 else 50_000_000
chunk = int(float(sys.argv[2])) if len(sys.argv) > 2 else rows // 2
t, _ = bench.c5_shard(torch, N, engine.ctx(), torch.device("cuda", 0), rows, chunk_rows=chunk)
print("table ready", flush=True)
for col in ("s_cat100", "s_text0"):
    an = [D.Uniqueness([col]), D.Entropy(col)]
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        whole = t.concat([col]) if hasattr(t, "concat") else t
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        ft = engine.frequencies(whole, [col])
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        s = ft.summary(None)
        t3 = time.perf_counter()
        ctx = D.AnalysisRunner.onData(t).addAnalyzers(an).run()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        print("%s rep %d: concat %.1f ms, build %.1f ms, summary %.1f ms, runner %.1f ms; groups %d %s" % (
            col, rep, (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, (t4 - t3) * 1e3, s["num_groups"],
            [str(ctx.metric(a).value)[:40] for a in an]), flush=True)
        del ft, whole
