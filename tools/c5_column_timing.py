"""Per-column device time of the C5 chunk's histogram builds (Histogram's frequencies, include_nulls) and casts:
python tools/c5_column_timing.py [rows] [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
import deequ_amd.native as N  # noqa: E402
from deequ_amd import engine  # noqa: E402

rows = int(float(sys.argv[1])) if len(sys.argv) > 1 else 125_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
t, _ = bench.c5_shard(torch, N, engine.ctx(), torch.device("cuda", 0), rows, chunk_rows=rows,
                      only={"s_cat50", "s_bool", "s_cat100", "s_int", "s_dec", "s_mixnum", "s_text0"})
torch.cuda.synchronize()


def timed(label, fn):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    print("%-28s %8.3f ms" % (label, (time.perf_counter() - t0) * 1e3 / reps), flush=True)


for name in ("s_cat50", "s_bool", "s_cat100"):
    timed("histogram %s" % name, lambda: engine.frequencies(t, [name], True).summary(None))
dev = torch.device("cuda", 0)
for name, to in (("s_int", N.TYPE_LONG), ("s_dec", N.TYPE_DOUBLE), ("s_mixnum", N.TYPE_DOUBLE)):
    vals = torch.empty(rows, dtype=torch.int64 if to == N.TYPE_LONG else torch.float64, device=dev)
    mask = torch.zeros((rows + 63) // 64 * 8, dtype=torch.uint8, device=dev)
    timed("cast %s" % name, lambda: engine.ctx().cast_column(t[name].native(), rows, to, vals.data_ptr(),
                                                             mask.data_ptr()))
