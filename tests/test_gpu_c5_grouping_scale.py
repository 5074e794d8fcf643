"""BASELINE config C5's general-key (string) grouping pinned to an exact oracle at the size it runs.

The 2.5e8-row C5 shard bench.py times (two 1.25e8-row chunks, ChunkedTable) is grouped on its free-text column
s_text0 (1-20 bytes, ~1.9e8 groups) and its 100-value column s_cat100: Uniqueness, Entropy, CountDistinct (one
frequency table over the chunks' key columns concatenated in HBM with int64 offsets) and Histogram (per-chunk tables
merged as FrequenciesAndNumRows.sum, A/GroupingAnalyzers.scala:127-147). The oracle groups the same device bytes in
C by exact byte-string equality (oracle_group_strings: 24-byte packed keys, bucketed, sorted, run-length counted --
no fingerprint). Group counts, unique groups and CountDistinct are compared exactly, Uniqueness bit-exact, Entropy
within 1e-12, Histogram's bins and every detail count exactly (top-N as a multiset: ties are broken arbitrarily,
A/Histogram.scala:113-117). dq_freq_path_count proves the large build's paths ran: the exact count pass with per-row
keys and two-word tuples, keys past 15 bytes compared by bytes, and split buckets. The ten ApproxQuantile(0.5)
values of the same run lie inside the GK rank bound of the exact ranks over the device columns
(A/GroupingAnalyzers.scala:53-79, A/Uniqueness.scala:29-36, A/Entropy.scala:28-42, A/CountDistinct.scala:24-34,
A/Histogram.scala:41-117, A/ApproxQuantile.scala:28-103)."""
import math

import numpy as np
import pytest

import deequ_amd as D
import oracle as O

pytestmark = pytest.mark.gpu

ROWS = 250_000_000
STRINGS = ("s_text0", "s_cat100")


@pytest.fixture(scope="module")
def shard():
    import torch
    import bench
    import deequ_amd.native as N
    from deequ_amd import engine
    names = set(STRINGS) | {n for n, _ in bench.C5_NUMERIC}
    t, _ = bench.c5_shard(torch, N, engine.ctx(), torch.device("cuda", 0), ROWS, only=names)
    assert len(t.chunks) == 2
    yield t
    del t
    torch.cuda.empty_cache()


def _oracle_groups(t, name, queries):
    parts = []
    for ch in t.chunks:
        c = ch[name]
        parts.append((c.device["values"].cpu().numpy(), c.device["offsets"].cpu().numpy(),
                      c.device["validity"].cpu().numpy(), c.length))
    got = O.group_strings_raw(parts, queries)
    del parts
    return got


def _paths(before):
    from deequ_amd import engine
    after = engine.ctx().freq_paths()
    return {k: after[k] - before[k] for k in after if after[k] != before[k]}


@pytest.mark.parametrize("name", STRINGS)
def test_c5_string_grouping_against_exact_oracle(shard, name, monkeypatch):
    from deequ_amd import engine
    t = shard
    an = [D.Uniqueness([name]), D.Entropy(name), D.CountDistinct([name]), D.Histogram(name)]
    monkeypatch.setenv("DQ_RUN_SERIAL", "1")  # every build on this thread's context: its path counters
    before = engine.ctx().freq_paths()
    res = D.AnalysisRunner.onData(t).addAnalyzers(an).run()
    paths = _paths(before)
    monkeypatch.delenv("DQ_RUN_SERIAL")
    for a in an:
        assert res.metric(a).value.isSuccess, (a, res.metric(a).value)
    hist = res.metric(D.Histogram(name)).value.get()
    queries = [k for k in hist.values if k != "NullValue"]
    o = _oracle_groups(t, name, queries)
    assert o["valid_rows"] + o["null_rows"] == ROWS
    exp = O.group_summary_from_count_groups(o["count_values"], o["count_groups"], o["valid_rows"])
    # Uniqueness = unique groups / numRows (rows with a non-NULL key), bit-exact; CountDistinct = groups
    assert res.metric(D.Uniqueness([name])).value.get() == exp["num_unique"] / o["valid_rows"]
    assert res.metric(D.CountDistinct([name])).value.get() == float(exp["num_groups"])
    ent = res.metric(D.Entropy(name)).value.get()
    assert abs(ent - exp["entropy"]) <= 1e-12 * exp["entropy"], (ent, exp["entropy"])
    # Histogram: NULL rows are the "NullValue" bin (no generated key spells it), every detail count exact
    assert hist.numberOfBins == exp["num_groups"] + (1 if o["null_rows"] else 0)
    got_counts = {k: v.absolute for k, v in hist.values.items()}
    assert got_counts.pop("NullValue") == o["null_rows"]
    assert got_counts == dict(zip(queries, o["query_counts"].tolist()))
    for k, v in hist.values.items():
        assert v.ratio == v.absolute / ROWS, k
    # the details are the top-N counts of all bins (the NULL bin included): equal as multisets
    allc = np.repeat(o["count_values"], np.minimum(o["count_groups"], len(hist.values) + 1))
    allc = np.sort(np.append(allc, o["null_rows"]))[::-1][:len(hist.values)]
    assert sorted((v.absolute for v in hist.values.values()), reverse=True) == allc.tolist()
    assert len(hist.values) == min(1000, hist.numberOfBins)
    if name == "s_text0":  # the large general build: every path it needs ran
        assert exp["num_groups"] > 1e8
        for p in ("exact", "partitioned", "long_tuples", "split_buckets"):
            assert paths.get(p, 0) >= 1, (p, paths)
        assert t.concat([name])[name].offsets64
    else:
        assert exp["num_groups"] == 100 and paths.get("small_optimistic", 0) >= 1, paths
    # the same analyzers with the builds on helper contexts (the default): identical metrics
    again = D.AnalysisRunner.onData(t).addAnalyzers(an).run()
    for a in an:
        assert again.metric(a).value.get() == res.metric(a).value.get() or isinstance(a, D.Histogram), a
    assert again.metric(D.Histogram(name)).value.get().numberOfBins == hist.numberOfBins


def test_c5_quantiles_at_scale_inside_the_rank_bound(shard):
    """ApproxQuantile(0.5) of the ten numeric columns over the 2.5e8-row shard (the chunks read as parts): the value's
    exact rank interval over the device columns (Java Double.compare order, NULL rows excluded) meets the GK bound
    ceil(0.01 n) around rank ceil(0.5 n)."""
    import bench
    t = shard
    an = [D.ApproxQuantile(n, 0.5) for n, _ in bench.C5_NUMERIC]
    res = D.AnalysisRunner.onData(t).addAnalyzers(an).run()
    for a in an:
        v = res.metric(a).value.get()
        lt = le = n = 0
        k = O._java_keys(np.array([v], dtype=np.float64))[0]
        for ch in t.chunks:
            c = ch[a.column]
            vals = c.device["values"].cpu().numpy()
            mask = np.unpackbits(c.device["validity"].cpu().numpy(), bitorder="little")[:c.length].astype(bool)
            keys = O._java_keys(vals[mask].astype(np.float64))
            lt += int((keys < k).sum())
            le += int((keys <= k).sum())
            n += int(mask.sum())
        lo, hi = lt + 1, le
        target = max(1, math.ceil(0.5 * n))
        slack = math.ceil(0.01 * n) + 1
        assert lo <= hi and lo - slack <= target <= hi + slack, (a, v, lo, hi, target)
