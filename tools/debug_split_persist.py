"""Debug: the split merged-state persist / load flow of tests/test_gpu_chunked.py, printing the loaded block's buffers
before the weighted build."""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np

import deequ_amd as D
from deequ_amd import groups as G
from test_gpu_chunked import _data, _chunked

data, types = _data(40_000, seed=13)
full, ct = _chunked(data, types, [0, 17_000, 40_000])
G.STRING_KEY_LIMIT = 4096
a = D.Uniqueness(["s", "k"])
st = a.computeStateFrom(ct.chunks[0]).sum(a.computeStateFrom(ct.chunks[1]))
ft = st.device_table()
print("split tables", type(ft).__name__, len(getattr(ft, "tables", [])), flush=True)
blk = ft.distinct_block()
for c in blk.columns:
    print("distinct col", c.name, c.spark_type, c.length, None if c.offsets is None else (c.offsets.dtype, len(c.offsets), int(c.offsets[-1])),
          None if c.values is None else (c.values.dtype, len(c.values)), None if c.validity is None else len(c.validity), flush=True)
print("counts", len(blk.counts), int(blk.counts.sum()), flush=True)
d = tempfile.mkdtemp()
provider = D.HdfsStateProvider(None, d)
provider.persist(a, st)
back = provider.load(a)
f = back.frequencies
print("loaded", type(f).__name__, back.numRows, flush=True)
for c in f.columns:
    print("loaded col", c.name, c.spark_type, c.length, None if c.offsets is None else (c.offsets.dtype, len(c.offsets), int(c.offsets[-1])),
          None if c.values is None else (c.values.dtype, len(c.values)), None if c.validity is None else len(c.validity),
          getattr(c, "offsets64", None), flush=True)
print("counts", len(f.counts), f.counts.dtype, flush=True)
print("metric", a.computeMetricFrom(back).value, flush=True)
