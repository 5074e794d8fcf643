"""Debug: DataType histograms of the C5 numeric-looking string columns vs a host classification."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import bench
import deequ_amd as D
import deequ_amd.native as N
from deequ_amd import engine
from deequ_amd.table import unpack_validity

rows = int(float(sys.argv[1]))
ctx = engine.ctx()
t, nb = bench.c5_shard(torch, N, ctx, torch.device("cuda", 0), rows)
for name in ("s_int", "s_dec"):
    m = D.DataType(name).calculate(t)
    print(name, {k: v.absolute for k, v in m.value.get().values.items()}, flush=True)
    c = t[name]
    off = c.device["offsets"].cpu().numpy().astype(np.int64)
    data = c.device["values"].cpu().numpy()[:off[-1]]
    valid = unpack_validity(c.device["validity"].cpu().numpy(), rows)
    ok = ((data >= ord('0')) & (data <= ord('9'))) | (data == ord('-')) | (data == ord('.'))
    bad_bytes = np.nonzero(~ok)[0]
    print("  bad bytes", len(bad_bytes), bad_bytes[:10], flush=True)
    if len(bad_bytes):
        rows_bad = np.searchsorted(off, bad_bytes, side="right") - 1
        print("  bad rows", np.unique(rows_bad)[:10], [bytes(data[off[r]:off[r + 1]]) for r in np.unique(rows_bad)[:5]])
    # which rows does the device call String? bisect by running DataType on slices
    lens = np.diff(off)
    print("  len hist", np.bincount(lens)[:10], flush=True)
