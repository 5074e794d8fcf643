"""Wall time of ChunkedTable.concat of the C5 grouping key columns (the HBM concatenation a chunked grouping run
performs before its build) and the grouping run with and without it: python tools/c5_concat_timing.py [rows] [reps]"""
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

rows = int(float(sys.argv[1])) if len(sys.argv) > 1 else 250_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
t, _ = bench.c5_shard(torch, N, engine.ctx(), torch.device("cuda", 0), rows, only={"s_text0", "s_cat100"})
torch.cuda.synchronize()
for cols in (["s_text0"], ["s_cat100"]):
    t.concat(cols)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        c = t.concat(cols)
        del c
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / reps * 1e3
    for mode in ("concat", "parted"):
        if mode == "concat":
            os.environ["DQ_GROUP_CONCAT"] = "1"
        else:
            os.environ.pop("DQ_GROUP_CONCAT", None)
        run = lambda: D.AnalysisRunner.onData(t).addAnalyzers([D.Uniqueness(cols), D.Entropy(cols[0])]).run()  # noqa
        run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            run()
        torch.cuda.synchronize()
        print("%s concat %.2f ms, Uniqueness + Entropy run (%s) %.2f ms"
              % (cols[0], el, mode, (time.perf_counter() - t0) / reps * 1e3), flush=True)
