"""bench.py reads committed PMC summaries (profiles/<round>/*_traffic_*.json) into its lines: every lookup it makes
must resolve against the committed files without raising (a summary in another layout once crashed the C4 line)."""
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_committed_traffic_summaries_resolve():
    for pattern, rows in (("c2_traffic_*.json", 1_000_000_000), ("c3_traffic_*.json", 1_000_000_000),
                          ("c4_traffic_*.json", 1_000_000_000), ("c5_traffic_*.json", 250_000_000),
                          ("suite10_traffic_*.json", 1_000_000_000), ("c2where_traffic_*.json", 1_000_000_000)):
        for need in ("traffic_bytes_per_call", "total_GB_per_call"):
            found = bench.committed_json(pattern, rows, need=need)
            if found:
                assert float(found[0][need]) > 0, (pattern, found[1])
    assert bench.measured_traffic(1_000_000_000) is not None
    for path in glob.glob(os.path.join(ROOT, "profiles", "*", "*_traffic_*.json")):
        d = json.load(open(path))
        assert "traffic_bytes_per_call" in d or "total_GB_per_call" in d, path
