"""Time the steps of tests/test_gpu_c5_grouping_scale.py one by one (progress printed as it goes):
python tools/c5_group_oracle_timing.py [rows] [column]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import torch  # noqa: E402
import bench  # noqa: E402
import deequ_amd as D  # noqa: E402
import deequ_amd.native as N  # noqa: E402
from deequ_amd import engine  # noqa: E402
import oracle as O  # noqa: E402

rows = int(float(sys.argv[1])) if len(sys.argv) > 1 else 250_000_000
name = sys.argv[2] if len(sys.argv) > 2 else "s_text0"
t0 = time.time()


def say(*a):
    print("[%7.2f s]" % (time.time() - t0), *a, flush=True)


t, _ = bench.c5_shard(torch, N, engine.ctx(), torch.device("cuda", 0), rows, only={name})
torch.cuda.synchronize()
say("shard")
for an in ([D.Uniqueness([name]), D.Entropy(name), D.CountDistinct([name])], [D.Histogram(name)]):
    os.environ["DQ_RUN_SERIAL"] = "1"
    before = engine.ctx().freq_paths()
    r = D.AnalysisRunner.onData(t).addAnalyzers(an).run()
    torch.cuda.synchronize()
    after = engine.ctx().freq_paths()
    say("run", [str(a) for a in an], {k: after[k] - before[k] for k in after if after[k] != before[k]},
        [str(r.metric(a).value)[:80] for a in an])
    del os.environ["DQ_RUN_SERIAL"]
    r = D.AnalysisRunner.onData(t).addAnalyzers(an).run()
    torch.cuda.synchronize()
    say("run with helpers")
parts = []
for ch in getattr(t, "chunks", [t]):
    c = ch[name]
    parts.append((c.device["values"].cpu().numpy(), c.device["offsets"].cpu().numpy(), c.device["validity"].cpu().numpy(),
                  c.length))
say("copied to host")
o = O.group_strings_raw(parts, ["a", "b"])
say("oracle", o["num_groups"], o["valid_rows"], o["null_rows"], len(o["count_values"]))
