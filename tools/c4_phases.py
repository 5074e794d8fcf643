"""Host-side phase timing of the C4 frequency build (engine.frequencies / summary / release), for the
allocation-overhead study in DESIGN.md. Usage: python tools/c4_phases.py [rows] [steps]"""
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import deequ_amd.native as N
from deequ_amd import engine
from deequ_amd.table import Table, Column

rows = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
ctx = engine.ctx()
keys = torch.empty(rows, dtype=torch.int64, device="cuda")
ctx.synth_freq_keys(rows, rows // 10, 0, rows, keys.data_ptr())
ctx.synchronize()
c = Column("k", N.TYPE_LONG, None, None, length=rows)
c.device = {"values": keys}
t = Table([c])
for i in range(steps):
    t0 = time.perf_counter()
    ft = engine.frequencies(t, ["k"])
    t1 = time.perf_counter()
    s = ft.summary(None)
    t2 = time.perf_counter()
    ft.close() if hasattr(ft, "close") else None
    del ft
    ctx.synchronize()
    t3 = time.perf_counter()
    print("step %d: build %.2f ms, summary %.2f ms, release %.2f ms, groups %d" %
          (i, (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, s["num_groups"]), flush=True)
