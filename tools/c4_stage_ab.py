"""A/B of the fast grouping build's run staging on C4 (1e9 int64 keys, 1e8 distinct): configurations of
DQ_FREQ_STAGE ("p1tile,p1line,p2tile,p2line"; line 0 = run-granular writes) interleaved round by round, each build
timed on the wall clock to the context's synchronize (as bench.py's c4 line) and checked against C4's closed forms.

    python tools/c4_stage_ab.py [rows] [rounds] [cfg ...]
"""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import deequ_amd.native as N  # noqa: E402
from deequ_amd import engine  # noqa: E402
from deequ_amd.table import Column, Table  # noqa: E402

rows = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
cfgs = sys.argv[3:] or ["4096,0,8192,0", "4096,16,4096,16", "4096,8,4096,8", "2048,16,2048,16", "2048,8,4096,16"]
ctx = engine.ctx()
keys = torch.empty(rows, dtype=torch.int64, device="cuda")
ctx.synth_freq_keys(rows, rows // 10, 0, rows, keys.data_ptr())
ctx.synchronize()
c = Column("k", N.TYPE_LONG, None, None, length=rows)
c.device = {"values": keys}
t = Table([c])
times = {k: [] for k in cfgs}
for r in range(rounds + 1):
    for cfg in cfgs:
        os.environ["DQ_FREQ_STAGE"] = cfg
        ctx.synchronize()
        t0 = time.perf_counter()
        ft = engine.frequencies(t, ["k"])
        s = ft.summary(None)
        ctx.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        ok = s["num_groups"] == rows // 10 and s["num_unique"] == rows // 20 and s["max_count"] == 19
        if not ok:
            print("cfg %s: WRONG summary %s" % (cfg, s), flush=True)
            sys.exit(1)
        del ft
        if r > 0:  # round 0 warms every configuration up
            times[cfg].append(ms)
        print("round %d cfg %-18s build+summary %.2f ms" % (r, cfg, ms), flush=True)
for cfg in cfgs:
    print("cfg %-18s median %.2f ms min %.2f ms" % (cfg, statistics.median(times[cfg]), min(times[cfg])), flush=True)
