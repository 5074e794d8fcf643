"""Narrow-key A/B for the fast grouping build: the frequency table of 1e9 keys with ~1e8 distinct, as int64 keys
inside a 2^30 window (narrow: 32-bit offsets in the partition buffers) and as int32 keys, against the same build
with 64-bit partition keys (DQ_FREQ_WIDE=1), interleaved. Also the C4 keys themselves (full 64-bit mixed values:
the sample sends them to the 64-bit path) to show the sampling costs nothing there."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import bench
import deequ_amd.native as N
from deequ_amd import engine
from deequ_amd.table import Column, Table

total = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
dev = torch.device("cuda:0")
engine.set_device(0)
ctx = engine.ctx()
stream = torch.cuda.Stream(dev)
torch.cuda.set_stream(stream)
ctx.set_stream(stream.cuda_stream)
keys = torch.empty(total, dtype=torch.int64, device=dev)
ctx.synth_freq_keys(total, total // 10, 0, total, keys.data_ptr())
ctx.synchronize()
cases = {"c4_mixed64": (keys, N.TYPE_LONG),
         "int64_window": (keys & ((1 << 30) - 1), N.TYPE_LONG),
         "int32": ((keys & ((1 << 30) - 1)).to(torch.int32), N.TYPE_INT)}
del keys
for name, (v, ty) in cases.items():
    c = Column("k", ty, None, None, length=total)
    c.device = {"values": v}
    t = Table([c])
    res = {}
    for wide in ("0", "1", "0", "1"):
        if wide == "1":
            os.environ["DQ_FREQ_WIDE"] = "1"
        else:
            os.environ.pop("DQ_FREQ_WIDE", None)

        def step(ev):
            if ev is not None:
                ev[0].record(stream)
            ft = engine.frequencies(t, ["k"])
            s = ft.summary(None)
            if ev is not None:
                ev[1].record(stream)
            del ft
            res.setdefault(wide, []).append(s)
            return s

        _, ms, _ = bench.timed(torch, None, 1, 5, 1, stream, step)
        print("%-14s %s %8.3f ms" % (name, "wide  " if wide == "1" else "narrow", ms), flush=True)
    a, b = res["0"][-1], res["1"][-1]
    assert all(a[k] == b[k] for k in ("num_rows", "num_groups", "num_unique", "max_count")), (a, b)
    print("%-14s summaries equal: groups %d" % (name, a["num_groups"]), flush=True)
os.environ.pop("DQ_FREQ_WIDE", None)
