"""HdfsStateProvider (A/StateProvider.scala:72-312) on the local file system: host logic only.

Mirrors T/analyzers/StateProviderTest.scala on states built directly (the GPU-computed variant is in
test_gpu_state_provider.py) plus the byte layouts the reference's DataOutputStream writes. The file
identifier (`MurmurHash3.stringHash(analyzer.toString, 42)`) has no golden value in the reference's
tests: its restatement is checked for the properties the layout relies on (parity unpinned)."""
import os
import struct

import pytest

import deequ_amd as D
from deequ_amd.analyzers import FrequenciesAndNumRows
from deequ_amd.quantiles import PercentileDigest, QuantileSummaries, Stats
from deequ_amd.state_provider import StateAlreadyExistsError, murmur3_string_hash
from deequ_amd.runners import AnalysisRunner, Analysis


def _states():
    words = [(i * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF for i in range(52)]
    digest = PercentileDigest(QuantileSummaries(10000, 0.01, [Stats(1.5, 1, 0), Stats(2.5, 2, 0)], 3))
    return [
        (D.Size(), D.NumMatches(5)),
        (D.Completeness("att1"), D.NumMatchesAndCount(4, 5)),
        (D.Compliance("att1", "att1 = 'b'"), D.NumMatchesAndCount(2, 5)),
        (D.PatternMatch("att1", D.Patterns.EMAIL), D.NumMatchesAndCount(0, 5)),
        (D.Sum("price"), D.SumState(12.25)),
        (D.Mean("price"), D.MeanState(12.25, 5)),
        (D.Minimum("price"), D.MinState(-0.0)),
        (D.Maximum("price"), D.MaxState(float("inf"))),
        (D.StandardDeviation("price"), D.StandardDeviationState(5.0, 2.45, 1.0 / 3.0)),
        (D.MaxLength("att1"), D.MaxState(7.0)),
        (D.MinLength("att1"), D.MinState(1.0)),
        (D.DataType("item"), D.DataTypeHistogram(1, 2, 3, 0, 4)),
        (D.ApproxCountDistinct("att1"), D.ApproxCountDistinctState(words)),
        (D.Correlation("count", "price"), D.CorrelationState(5.0, 1.0, 2.0, 0.5, 2.0, 3.0)),
    ], (D.ApproxQuantile("price", 0.5), D.ApproxQuantileState(digest))


def test_scala_string_hash_properties():
    # odd/even lengths take the pair path and the mixLast tail; results are signed 32-bit ints
    vals = [murmur3_string_hash(s) for s in ["", "a", "ab", "abc", "Size(None)", "Completeness(att1,None)"]]
    assert all(-(1 << 31) <= v < (1 << 31) for v in vals)
    assert len(set(vals)) == len(vals)
    assert murmur3_string_hash("Size(None)", 42) != murmur3_string_hash("Size(None)", 43)
    # UTF-16 code units, not UTF-8 bytes: a supplementary character is two units
    assert murmur3_string_hash("\U0001F600") != murmur3_string_hash("éé")


def test_restores_every_state_from_the_filesystem(tmp_path):
    provider = D.HdfsStateProvider(None, str(tmp_path / "states"))
    scans, (aq, aq_state) = _states()
    for a, s in scans:
        provider.persist(a, s)
        assert provider.load(a) == s, a
    provider.persist(aq, aq_state)
    got = provider.load(aq).percentileDigest.quantileSummaries
    want = aq_state.percentileDigest.quantileSummaries
    assert (got.compressThreshold, got.relativeError, got.count) == (want.compressThreshold, want.relativeError,
                                                                     want.count)
    assert got.sampled == want.sampled


def test_byte_layouts_match_java_data_output_stream(tmp_path):
    prefix = str(tmp_path / "p")
    provider = D.HdfsStateProvider(None, prefix)
    a = D.Mean("price")
    provider.persist(a, D.MeanState(1.5, 7))
    raw = open("%s-%d.bin" % (prefix, murmur3_string_hash(str(a), 42)), "rb").read()
    assert raw == struct.pack(">d", 1.5) + struct.pack(">q", 7)
    dt = D.DataType("item")
    provider.persist(dt, D.DataTypeHistogram(1, 2, 3, 4, 5))
    raw = open("%s-%s.bin" % (prefix, provider.toIdentifier(dt)), "rb").read()
    assert raw[:4] == struct.pack(">i", 40) and raw[4:] == struct.pack(">5q", 1, 2, 3, 4, 5)
    hll = D.ApproxCountDistinct("att1")
    provider.persist(hll, D.ApproxCountDistinctState([0xFFFFFFFFFFFFFFFF] + [0] * 51))
    raw = open("%s-%s.bin" % (prefix, provider.toIdentifier(hll)), "rb").read()
    assert raw[:4] == struct.pack(">i", 416) and raw[4:12] == b"\xff" * 8


def test_frequency_state_round_trip_and_overwrite(tmp_path):
    prefix = str(tmp_path / "f")
    freq = {("a",): 2, ("b",): 1, (None,): 3}
    state = FrequenciesAndNumRows(freq, 6, ["att1"])
    provider = D.HdfsStateProvider(None, prefix, numPartitionsForHistogram=2)
    u = D.Uniqueness("att1")
    provider.persist(u, state)
    back = provider.load(u)
    assert back.as_dict() == freq and back.numRows == 6 and back.columns == ["att1"]
    assert os.path.isdir("%s-%s-frequencies.pqt" % (prefix, provider.toIdentifier(u)))
    with pytest.raises(StateAlreadyExistsError, match="already exists"):
        provider.persist(u, state)
    two = {("a", 1): 1, ("b", 2): 4}
    u2 = D.Uniqueness(["att1", "count"])
    provider.persist(u2, FrequenciesAndNumRows(two, 5, ["att1", "count"]))
    assert provider.load(u2).as_dict() == two

    over = D.HdfsStateProvider(None, prefix, allowOverwrite=True)
    over.persist(u, FrequenciesAndNumRows({("a",): 2}, 2, ["att1"]))
    assert over.load(u).as_dict() == {("a",): 2} and over.load(u).numRows == 2


def test_scalar_state_overwrite_guard(tmp_path):
    provider = D.HdfsStateProvider(None, str(tmp_path / "s"))
    provider.persist(D.Size(), D.NumMatches(1))
    with pytest.raises(StateAlreadyExistsError):
        provider.persist(D.Size(), D.NumMatches(2))
    D.HdfsStateProvider(None, str(tmp_path / "s"), allowOverwrite=True).persist(D.Size(), D.NumMatches(2))
    assert provider.load(D.Size()) == D.NumMatches(2)


def test_unsupported_analyzer_raises(tmp_path):
    provider = D.HdfsStateProvider(None, str(tmp_path / "k"))
    with pytest.raises(ValueError, match="Unable to persist state"):
        provider.persist(D.KLLSketch("x"), object())
    with pytest.raises(ValueError, match="Unable to load state"):
        provider.load(D.KLLSketch("x"))


def test_run_on_aggregated_states_from_two_persisted_partitions(tmp_path):
    """StateAggregationIntegrationTest shape: two partitions' states persisted on disk, merged with
    AnalysisRunner.runOnAggregatedStates (no data scan, host only)."""
    p1 = D.HdfsStateProvider(None, str(tmp_path / "part1"))
    p2 = D.HdfsStateProvider(None, str(tmp_path / "part2"))
    size, comp, mean, uniq = D.Size(), D.Completeness("att1"), D.Mean("price"), D.Uniqueness("att1")
    p1.persist(size, D.NumMatches(3))
    p2.persist(size, D.NumMatches(2))
    p1.persist(comp, D.NumMatchesAndCount(3, 3))
    p2.persist(comp, D.NumMatchesAndCount(1, 2))
    p1.persist(mean, D.MeanState(6.0, 3))
    p2.persist(mean, D.MeanState(4.0, 2))
    p1.persist(uniq, FrequenciesAndNumRows({("a",): 2, ("b",): 1}, 3, ["att1"]))
    p2.persist(uniq, FrequenciesAndNumRows({("a",): 1, ("c",): 1}, 2, ["att1"]))
    schema = D.Table.from_pydict({"att1": ["a", "b", "a"], "price": [1.0, 2.0, 3.0]}).schema
    ctx = AnalysisRunner.runOnAggregatedStates(schema, Analysis([size, comp, mean]), [p1, p2])
    assert ctx.metric(size).value.get() == 5.0
    assert ctx.metric(comp).value.get() == 0.8
    assert ctx.metric(mean).value.get() == 2.0
    # string-keyed frequency states load as key columns + counts and merge by concatenation (their metric is the
    # weighted GPU build: tests/test_gpu_state_provider.py); the joined groups are the outer join's
    merged = p1.load(uniq).sum(p2.load(uniq))
    assert merged.numRows == 5 and merged.as_dict() == {("a",): 3, ("b",): 1, ("c",): 1}


def test_run_on_aggregated_states_folds_kll_sketches_in_loader_order():
    """runOnAggregatedStates folds the KLL states of several columns on a thread pool (the library merge releases the
    GIL): each column's metric equals the one of its states summed in loader order by the restated Python merge."""
    import numpy as np
    import oracle as O
    from deequ_amd.kll import KLLState, bucket_distribution
    from deequ_amd.runners import InMemoryStateProvider
    rng = np.random.default_rng(4)
    names = ["c%d" % i for i in range(5)]
    loaders = [InMemoryStateProvider() for _ in range(3)]
    raw = {}
    for n in names:
        for j, p in enumerate(loaders):
            b = O.kll_state_bytes(rng.normal(j, 1 + j, 20_000 + 1000 * j), 256, 0.64)
            raw[(n, j)] = b
            p.persist(D.KLLSketch(n, D.KLLParameters(256, 0.64, 10)), KLLState.fromBytes(b))
    schema = D.Table.from_pydict({n: [1.0] for n in names}).schema
    for ncols in (5, 1):  # several KLL columns (the thread pool) and one (folded in place)
        an = [D.KLLSketch(n, D.KLLParameters(256, 0.64, 10)) for n in names[:ncols]]
        ctx = AnalysisRunner.runOnAggregatedStates(schema, Analysis(an + [D.Size()]), loaders)
        for a, n in zip(an, names):
            exp = KLLState.fromBytes(raw[(n, 0)])
            for j in (1, 2):
                exp = exp.sum_restated(KLLState.fromBytes(raw[(n, j)]))
            assert ctx.metric(a).value.get() == bucket_distribution(exp, 10)


def test_float_grouping_keys_merge_bitwise_across_persisted_states(tmp_path):
    """Frequencies of a double grouping column loaded from disk join the in-memory state with Spark's
    grouping equality (bitwise, NaN canonical, -0.0 != 0.0): repeated values merge, -0.0 and 0.0 stay
    apart, NaNs merge (plain float keys never equalled GroupFloat keys)."""
    from deequ_amd.engine import GroupFloat
    nan = float("nan")
    a = D.FrequenciesAndNumRows({(GroupFloat(1.5),): 2, (GroupFloat(-0.0),): 1, (GroupFloat(nan),): 1}, 4, ["x"])
    provider = D.HdfsStateProvider(None, str(tmp_path / "st"))
    an = D.CountDistinct(["x"])
    provider.persist(an, D.FrequenciesAndNumRows({(1.5,): 3, (0.0,): 1, (float("nan"),): 2}, 6, ["x"]))
    loaded = provider.load(an)
    for merged in (a.sum(loaded), loaded.sum(a)):
        d = merged.as_dict()
        assert merged.numRows == 10
        assert d[(GroupFloat(1.5),)] == 5
        assert d[(GroupFloat(nan),)] == 3
        assert d[(GroupFloat(-0.0),)] == 1 and d[(GroupFloat(0.0),)] == 1
        assert len(d) == 4
    # two loaded states (runOnAggregatedStates): NaN keys merge, signed zeros do not
    provider2 = D.HdfsStateProvider(None, str(tmp_path / "st2"))
    provider2.persist(an, D.FrequenciesAndNumRows({(-0.0,): 1, (float("nan"),): 1}, 2, ["x"]))
    d = loaded.sum(provider2.load(an)).as_dict()
    assert d[(GroupFloat(nan),)] == 3 and d[(GroupFloat(-0.0),)] == 1 and d[(GroupFloat(0.0),)] == 1


def test_date_keyed_frequency_state_round_trip(tmp_path):
    """A single DATE key persisted from its canonical (key, count) arrays (Arrow has no int64 -> date32
    cast) and read back as pairs, NULL group included."""
    import numpy as np
    import deequ_amd.native as N
    from deequ_amd import engine
    days = np.array([-3, 0, 18000, 2 ** 31 - 1], dtype=np.int64)
    pf = engine.PairFrequencies(N.TYPE_DATE, engine.canonical_keys(N.TYPE_DATE, days), [1, 2, 3, 4], 12, 2, 0, ["d"])
    state = FrequenciesAndNumRows(pf, 12, ["d"])
    provider = D.HdfsStateProvider(None, str(tmp_path / "dt"))
    u = D.CountDistinct(["d"])
    provider.persist(u, state)
    back = provider.load(u).frequencies
    assert isinstance(back, engine.PairFrequencies) and back.key_type == N.TYPE_DATE
    got = sorted(zip(back.keys.tolist(), back.counts.tolist()))
    assert got == sorted(zip(days.tolist(), [1, 2, 3, 4])) and back.null_count == 2 and back.num_rows == 12


def test_histogram_identity_and_tostring():
    """case class Histogram(column, binningUdf, maxDetailBins): the UDF takes part in equality and toString
    (the HdfsStateProvider file id hashes that string); Scala renders Double fields with Double.toString."""
    f, g = (lambda s: s), (lambda s: s)
    assert repr(D.Histogram("c")) == "Histogram(c,None,1000)"
    assert D.Histogram("c", f) != D.Histogram("c", g) and D.Histogram("c", f) == D.Histogram("c", f)
    assert D.Histogram("c", f) != D.Histogram("c") and len({D.Histogram("c", f), D.Histogram("c", g)}) == 2
    assert repr(D.ApproxQuantile("c", 0.5, 1e-4)) == "ApproxQuantile(c,0.5,1.0E-4)"
    ctx_keys = {D.Histogram("c", f): 1, D.Histogram("c", g): 2}
    assert ctx_keys[D.Histogram("c", g)] == 2


def test_split_by_key_keeps_keys_together_under_the_offset_limit():
    """A merged string state past the int32 Arrow offsets is built in key-disjoint splits: every copy of
    a key lands in one split, the counts are preserved and each split stays under the (injected) byte limit."""
    import numpy as np
    import deequ_amd.native as N
    from deequ_amd import groups as G
    from deequ_amd.table import Column, pack_validity

    def block(keys, counts, valid):
        data = b"".join(k.encode() for k in keys)
        off = np.zeros(len(keys) + 1, dtype=np.int64)
        np.cumsum([len(k.encode()) for k in keys], out=off[1:])
        col = Column("s", N.TYPE_STRING, np.frombuffer(data, np.uint8), pack_validity(np.array(valid)),
                     off.astype(np.int32), length=len(keys))
        return G.GroupBlock([col, Column("k", N.TYPE_LONG, np.arange(len(keys), dtype=np.int64) % 3, None)],
                            np.array(counts, dtype=np.int64))

    keys = ["key-%05d" % i for i in range(400)]
    a = block(keys[:300], range(1, 301), [i % 17 != 0 for i in range(300)])
    b = block(keys[200:], range(1, 201), [i % 13 != 0 for i in range(200)])
    parts = G.BlockParts([a, b], a.schema())
    assert parts.split_by_key(limit=10 ** 9) == [parts]
    splits = parts.split_by_key(limit=1000)
    assert len(splits) > 1 and all(s.key_bytes() < 1000 for s in splits)
    assert sum(s.size for s in splits) == parts.size
    assert sum(int(s.counts.sum()) for s in splits) == int(parts.counts.sum())
    owner = {}
    for i, s in enumerate(splits):
        for key in s.keys():
            assert owner.setdefault(key, i) == i, key  # a key never spans two splits
