"""Host timeline of one C5-shard ColumnProfiler run: wall-clock enter / exit marks (device synchronised at each mark)
of the profiler's stages, to place the GPU-idle gaps of the kernel trace.

    python tools/c5_host_timeline.py [rows]
"""
import functools
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import bench
import deequ_amd as D
import deequ_amd.native as N
from deequ_amd import engine, runners, profiles

rows = int(float(sys.argv[1])) if len(sys.argv) > 1 else 250_000_000
t, _ = bench.c5_shard(torch, N, engine.ctx(), torch.device("cuda", 0), rows)
D.ColumnProfiler.profile(t)
torch.cuda.synchronize()

marks = []
T0 = [0.0]


def wrap(obj, name, label):
    f = getattr(obj, name)

    @functools.wraps(f)
    def g(*a, **k):
        torch.cuda.synchronize()
        marks.append((time.perf_counter() - T0[0], "enter " + label))
        out = f(*a, **k)
        torch.cuda.synchronize()
        marks.append((time.perf_counter() - T0[0], "exit  " + label))
        return out
    setattr(obj, name, staticmethod(g) if isinstance(obj.__dict__.get(name), staticmethod) else g)


wrap(runners.AnalysisRunner, "doAnalysisRun", "doAnalysisRun")
wrap(runners.AnalysisRunner, "runOnAggregatedStates", "runOnAggregatedStates")
wrap(runners.KLLRunner, "computeKLLSketchesInExtraPass", "KLL extra pass")
wrap(N.Context, "scan", "dq_scan")
wrap(N.Context, "kll_sketch_columns", "dq_kll_sketch_columns")
wrap(N.Context, "cast_column", "dq_cast_column")
wrap(engine, "frequencies", "engine.frequencies")
wrap(profiles.ColumnProfiler, "_extract_numeric", "_extract_numeric")
wrap(profiles.ColumnProfiler, "_extract_generic", "_extract_generic")
torch.cuda.synchronize()
T0[0] = time.perf_counter()
D.ColumnProfiler.profile(t)
torch.cuda.synchronize()
total = time.perf_counter() - T0[0]
prev = 0.0
for ts, what in marks:
    print("%8.2f ms (+%6.2f)  %s" % (ts * 1e3, (ts - prev) * 1e3, what))
    prev = ts
print("total %.2f ms (with a device synchronisation at every mark)" % (total * 1e3))
