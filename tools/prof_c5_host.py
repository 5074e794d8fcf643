"""Host-side profile of one C5-shard ColumnProfiler run (cProfile; GPU waits show up inside the ctypes calls)."""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import bench
import deequ_amd as D
import deequ_amd.native as N
from deequ_amd import engine

rows = int(float(sys.argv[1])) if len(sys.argv) > 1 else 100_000_000
t, _ = bench.c5_shard(torch, N, engine.ctx(), torch.device("cuda", 0), rows)
D.ColumnProfiler.profile(t)
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
D.ColumnProfiler.profile(t)
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("cumulative").print_stats(45)
st.sort_stats("tottime").print_stats(25)
