"""bench.py's own rank launcher (VERDICT r04 missing #2): `--gpus N` without torch.distributed.run starts N rank
processes with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, and rank 0's line reports n_gpus = N. Checked on the
CPU with the hidden --launch-check mode (gloo rendezvous + one all-reduce, no GPU call)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=240, env=env)
    return p


@pytest.mark.parametrize("n", [1, 2, 3])
def test_gpus_flag_starts_that_many_ranks(n):
    p = _run(["--gpus", str(n), "--launch-check", "--dist-backend", "gloo"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout  # only rank 0 prints
    assert lines[0]["n_gpus"] == n
    assert lines[0]["ranks_sum"] == n * (n + 1) // 2  # every rank took part in the all-reduce
    assert lines[0]["local_rank"] == 0


@pytest.mark.parametrize("n", [1, 2])
def test_default_is_baselines_one_billion_row_table(n):
    """BASELINE: "synthetic 1B-row tables at 1/2/4/8 GPUs" -- the default splits 1e9 rows over the ranks (strong
    scaling); --scaling weak stays an explicit option."""
    p = _run(["--gpus", str(n), "--launch-check", "--dist-backend", "gloo", "--device-override", "0"])
    assert p.returncode == 0, p.stderr[-2000:]
    cfg = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")][0]["config"]
    assert cfg["rows"] == 1_000_000_000 and cfg["scaling"] == "strong"
    assert abs(cfg["rows_per_gpu"] - 1_000_000_000 / n) <= 2048
    p = _run(["--gpus", str(n), "--launch-check", "--dist-backend", "gloo", "--scaling", "weak"])
    cfg = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")][0]["config"]
    assert cfg["rows"] == n * 1_000_000_000 and cfg["rows_per_gpu"] == 1_000_000_000


def test_world_size_mismatch_is_refused():
    p = _run(["--gpus", "2", "--launch-check"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0
