"""KLL extra pass over the C5 shard's 10 numeric columns (5 % nulls) + 3 cast columns' worth of fp64 data: one
dq_kll_sketch per column vs one dq_kll_sketch_columns call (parallel host schedules, one round trip), the latter with
every column's compaction chain spread over the context's 4 streams (DQ_KLL_PER_COLUMN=1) and batched (one launch per
level and class over all columns); bytes compared,
wall time per pass (device synchronised), interleaved rounds.

    python tools/kll_ab.py [rows] [rounds] [no12]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import deequ_amd.native as N  # noqa: E402
from deequ_amd import engine  # noqa: E402
from deequ_amd.table import Column  # noqa: E402

os.environ.setdefault("DQ_KLL_TIMING", "1")
if len(sys.argv) > 3 and sys.argv[3] == "no12":  # padded power-of-two compaction classes only (read once per process)
    os.environ["DQ_KLL_NO_E12"] = "1"
rows = int(float(sys.argv[1])) if len(sys.argv) > 1 else 125_000_000
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
ctx = engine.ctx()
dev = torch.device("cuda", 0)
cols = []
for j in range(13):
    kind = bench.C5_NUMERIC[j % len(bench.C5_NUMERIC)][1]
    dt = torch.float64 if kind in (1, 2, 3, 6, 7) else torch.int64
    v = torch.empty(rows, dtype=dt, device=dev)
    ctx.synth_column(kind, 0xC5000000 + j, 0, rows, v.data_ptr())
    m = torch.zeros((rows + 63) // 64 * 8, dtype=torch.uint8, device=dev)
    ctx.synth_validity(0xC5200000 + j, 0, rows, 50, m.data_ptr())
    c = Column("c%d" % j, N.TYPE_DOUBLE if dt == torch.float64 else N.TYPE_LONG, None, None, length=rows)
    c.device = {"values": v, "validity": m}
    cols.append(c)
ctx.synchronize()
nat = [c.native() for c in cols]
for r in range(rounds + 1):
    ctx.synchronize()
    t0 = time.perf_counter()
    single = [ctx.kll_sketch(x, rows, 2048, 0.64) for x in nat]
    ctx.synchronize()
    t1 = time.perf_counter()
    os.environ["DQ_KLL_PER_COLUMN"] = "1"  # one launch chain per column, spread over 4 streams
    serial = ctx.kll_sketch_columns(nat, rows, 2048, 0.64)
    ctx.synchronize()
    del os.environ["DQ_KLL_PER_COLUMN"]
    t2 = time.perf_counter()
    batch = ctx.kll_sketch_columns(nat, rows, 2048, 0.64)
    ctx.synchronize()
    t3 = time.perf_counter()
    assert batch == single and serial == single, "batched KLL bytes differ"
    print("round %d: 13 x dq_kll_sketch %.1f ms, dq_kll_sketch_columns per-column chains on 4 streams %.1f ms, "
          "batched (one launch per level and class) %.1f ms "
          "(%d rows per column)" % (r, (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, rows), flush=True)
