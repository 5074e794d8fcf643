"""K full C5 steps (the 3-pass ColumnProfiler + the extra analyzers) on the 2.5e8-row shard, for PMC passes:
python tools/c5_steps.py [rows] [K] — one progress line per step (the generators run first and are excluded by
tools/pmc_traffic.py --all-engine)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import bench
import deequ_amd as D
import deequ_amd.native as N
from deequ_amd import engine

rows = int(float(sys.argv[1])) if len(sys.argv) > 1 else 250_000_000
k = int(sys.argv[2]) if len(sys.argv) > 2 else 2
t, _ = bench.c5_shard(torch, N, engine.ctx(), torch.device("cuda", 0), rows)
extras = bench.c5_extra_analyzers(D)
print("table ready", flush=True)
import threading  # noqa: E402
low = {"free": float("inf")}
stop = threading.Event()


def sample():  # the lowest free device memory seen during the steps (every ~2 ms)
    torch.cuda.set_device(0)
    while not stop.is_set():
        low["free"] = min(low["free"], torch.cuda.mem_get_info()[0])
        time.sleep(0.002)


sampler = threading.Thread(target=sample, daemon=True)
sampler.start()
for i in range(k):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    m0 = time.monotonic_ns()
    bench.c5_step(D, t, extras)
    torch.cuda.synchronize()
    free, total = torch.cuda.mem_get_info()
    print("step %d %.1f ms monotonic_ns %d %d free_gb %.1f" % (i, (time.perf_counter() - t0) * 1e3, m0,
                                                               time.monotonic_ns(), free / 1e9), flush=True)
stop.set()
sampler.join()
print("lowest free device memory during the steps: %.1f GB" % (low["free"] / 1e9), flush=True)
