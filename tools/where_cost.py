"""Cost of a `where` filter on the C2 suite (1e9 rows). Prints the dq_scan HIP-event time without / with `where`
(the filter produced by its own column's scan, DQ_WHERE_FUSED=1, and by where_masks_kernel with the filter column a
consumer, DQ_WHERE_FUSED=0, interleaved), and a where-only Compliance."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import bench
import deequ_amd as D
import deequ_amd.native as N
from deequ_amd import engine

rows = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
dev = torch.device("cuda:0")
engine.set_device(0)
ctx = engine.ctx()
stream = torch.cuda.Stream(dev)
torch.cuda.set_stream(stream)
ctx.set_stream(stream.cuda_stream)
t = bench.build_shard(torch, N, ctx, 0, rows, dev)
names = list(t.columns)
cases = {"c2": bench.c2_analyzers(D, names)}
# every analyzer of the C2 suite under `where c4 < 0` (c4 is an int64 column)
w = "c4 < 0"
cw = [D.Size(w)]
for c in names:
    cw += [D.Completeness(c, w), D.Mean(c, w), D.Sum(c, w), D.Minimum(c, w), D.Maximum(c, w), D.StandardDeviation(c, w)]
cases["c2_where_c4<0"] = cw
cases["compliance_c4<0"] = [D.Compliance("neg", "c4 < 0")]
cases["compliance_c4<0_or_c5>1"] = [D.Compliance("neg", "c4 < 0 OR c5 > 1")]
runs = [(name, an, None) for name, an in cases.items()]
runs += [("c2_where_c4<0 fused=%s" % f, cw, f) for f in ("1", "0", "1", "0")]
for name, an, fused in runs:
    if fused is not None:
        os.environ["DQ_WHERE_FUSED"] = fused
    wl = bench.ScanWorkload(torch, N, D, ctx, t, an, stream, dev, 1, "nccl")
    _, ms, _ = bench.timed(torch, None, 1, 10, 2, stream, wl.step)
    print("%-26s %8.3f ms  %.3e rows/s" % (name, ms, rows / ms * 1e3), flush=True)
