"""Timing experiment harness: the C4 frequency build 3x (results unchecked), for rocprofv3 kernel stats A/B."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from deequ_amd import engine
from deequ_amd.table import Table, Column
import deequ_amd.native as N

total = 1_000_000_000
ctx = engine.ctx()
keys = torch.empty(total, dtype=torch.int64, device="cuda")
ctx.synth_freq_keys(total, total // 10, 0, total, keys.data_ptr())
ctx.synchronize()
c = Column("k", N.TYPE_LONG, None, None, length=total)
c.device = {"values": keys}
t = Table([c])
for _ in range(3):
    try:
        ft = engine.frequencies(t, ["k"])
        print(ft.summary(None))
        del ft
    except Exception as e:
        print("error", e)
torch.cuda.synchronize()
