"""Run bench.py's C5-shard workload alone: python tools/c5_shard.py [rows] [steps]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import bench
import deequ_amd as D
import deequ_amd.native as N
from deequ_amd import engine

rows = int(float(sys.argv[1])) if len(sys.argv) > 1 else 10_000_000
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
print(json.dumps(bench.bench_c5(torch, N, D, engine.ctx(), torch.device("cuda", 0), rows, steps)), flush=True)
