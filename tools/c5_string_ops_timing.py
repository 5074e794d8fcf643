"""Device time of the profiler's pass-1 string ops per C5 string column, split by op (Completeness + DataType,
ApproxCountDistinct, all three): python tools/c5_string_ops_timing.py [rows] [reps] [all: the all-columns run only]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
import deequ_amd as D  # noqa: E402
import deequ_amd.native as N  # noqa: E402
from deequ_amd import engine  # noqa: E402

rows = int(float(sys.argv[1])) if len(sys.argv) > 1 else 125_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
names = [n for n, _ in bench.C5_STRINGS]
t, _ = bench.c5_shard(torch, N, engine.ctx(), torch.device("cuda", 0), rows, chunk_rows=rows, only=set(names))
torch.cuda.synchronize()


def timed(an):
    D.AnalysisRunner.onData(t).addAnalyzers(an).run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        D.AnalysisRunner.onData(t).addAnalyzers(an).run()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


for c in (names if len(sys.argv) <= 3 or sys.argv[3] != "all" else []):
    a = timed([D.Completeness(c), D.DataType(c)])
    b = timed([D.ApproxCountDistinct(c)])
    both = timed([D.Completeness(c), D.DataType(c), D.ApproxCountDistinct(c)])
    print("%-9s dtype %.2f ms  hll %.2f ms  all %.2f ms" % (c, a, b, both), flush=True)
allc = []
for c in names:
    allc += [D.Completeness(c), D.DataType(c), D.ApproxCountDistinct(c)]
print("all columns, one run: %.2f ms" % timed(allc), flush=True)
