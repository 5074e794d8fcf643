"""ChunkedTable runs (row chunks whose states merge through runOnAggregatedStates, R/AnalysisRunner.scala:385-460)
against the single-table run: duplicated analyzers, a grouping that fails on every chunk, and merged string states
built in key-disjoint splits."""
import numpy as np
import pytest

import deequ_amd as D
from deequ_amd import groups as G
from deequ_amd import runners
from deequ_amd.table import Table

pytestmark = pytest.mark.gpu


def _close(a, b):
    return a == b or abs(a - b) <= 1e-12 * max(1.0, abs(b))


def _data(n=20_000, seed=3):
    rng = np.random.default_rng(seed)
    s = [None if rng.random() < 0.05 else "v%d" % int(v) for v in rng.integers(0, 3000, n)]
    k = [int(v) for v in rng.integers(0, 500, n)]
    x = [None if rng.random() < 0.1 else float(v) for v in rng.normal(size=n)]
    return {"s": s, "k": k, "x": x}, {"s": "string", "k": "long", "x": "double"}


def _chunked(data, types, cuts):
    full = Table.from_pydict(data, types=types).to_device()
    chunks = [Table.from_pydict({c: v[a:b] for c, v in data.items()}, types=types).to_device()
              for a, b in zip(cuts, cuts[1:])]
    return full, D.ChunkedTable(chunks)


def test_duplicated_analyzers_merge_once():
    """VerificationSuite does not dedupe its constraints' analyzers (M/VerificationSuite.scala): two constraints on
    one Size or one Uniqueness must not add each chunk's state twice."""
    data, types = _data()
    full, ct = _chunked(data, types, [0, 7_000, 13_000, 20_000])
    an = [D.Size(), D.Size(), D.Uniqueness(["s"]), D.Uniqueness(["s"]), D.Sum("k"), D.Sum("k"), D.Entropy("k"),
          D.CountDistinct(["s", "k"]), D.CountDistinct(["s", "k"])]
    want = D.AnalysisRunner.onData(full).addAnalyzers(an).run()
    got = D.AnalysisRunner.onData(ct).addAnalyzers(an).run()
    for a in an:
        w, g = want.metric(a).value.get(), got.metric(a).value.get()
        assert _close(g, w), (a, g, w)
    assert got.metric(D.Size()).value.get() == 20_000


def test_grouping_failing_on_every_chunk_returns_failure_metrics(monkeypatch):
    """A grouping whose frequencies fail on every chunk keeps the chunk failure metrics; the other analyzers of the
    run still succeed (no 'requirement failed' from the merge)."""
    data, types = _data()
    _, ct = _chunked(data, types, [0, 10_000, 20_000])
    real = runners.computeFrequencies

    def failing(table, cols, *args, **kw):
        if list(cols) == ["s"]:
            raise RuntimeError("injected grouping failure")
        return real(table, cols, *args, **kw)

    monkeypatch.setattr(runners, "computeFrequencies", failing)
    an = [D.Size(), D.Uniqueness(["s"]), D.Distinctness(["s"]), D.Entropy("k"), D.Mean("x")]
    got = D.AnalysisRunner.onData(ct).addAnalyzers(an).run()
    for a in (D.Uniqueness(["s"]), D.Distinctness(["s"])):
        v = got.metric(a).value
        assert not v.isSuccess, a
    assert got.metric(D.Size()).value.get() == 20_000
    assert got.metric(D.Entropy("k")).value.isSuccess and got.metric(D.Mean("x")).value.isSuccess


def test_merged_string_state_split_under_the_offset_limit(monkeypatch):
    """A merged string / multi-column state whose key bytes reach the int32 Arrow offsets is built in key-disjoint
    splits (the limit injected small here): the metrics equal the single-table run, with NULL keys and validity
    joined on the device."""
    data, types = _data(60_000, seed=9)
    full, ct = _chunked(data, types, [0, 25_000, 41_000, 60_000])
    an = [D.Uniqueness(["s"]), D.Distinctness(["s", "k"]), D.UniqueValueRatio(["s"]), D.CountDistinct(["s", "k"]),
          D.Entropy("s")]
    want = D.AnalysisRunner.onData(full).addAnalyzers(an).run()
    monkeypatch.setattr(G, "STRING_KEY_LIMIT", 4096)
    got = D.AnalysisRunner.onData(ct).addAnalyzers(an).run()
    for a in an:
        w, g = want.metric(a).value.get(), got.metric(a).value.get()
        assert _close(g, w), (a, g, w)
    # the merged state really was split
    st = D.Uniqueness(["s", "k"]).computeStateFrom(ct.chunks[0]).sum(
        D.Uniqueness(["s", "k"]).computeStateFrom(ct.chunks[1]))
    assert isinstance(st.frequencies, G.BlockParts)
    assert len(st.frequencies.split_by_key()) > 1
    assert isinstance(st.device_table(), D.analyzers.SplitFrequencies)


def test_split_merged_state_persists_and_loads_back(monkeypatch, tmp_path):
    """a merged string / multi-column state built as key-disjoint splits (the int32 offset limit injected
    small) persists through HdfsStateProvider as its distinct groups and loads back to the same metrics
    (A/StateProvider.scala:187-262 layouts; FrequenciesAndNumRows.sum, A/GroupingAnalyzers.scala:127-147)."""
    data, types = _data(40_000, seed=13)
    full, ct = _chunked(data, types, [0, 17_000, 40_000])
    monkeypatch.setattr(G, "STRING_KEY_LIMIT", 4096)
    a = D.Uniqueness(["s", "k"])
    st = a.computeStateFrom(ct.chunks[0]).sum(a.computeStateFrom(ct.chunks[1]))
    assert isinstance(st.device_table(), D.analyzers.SplitFrequencies)
    want = a.computeMetricFrom(st).value.get()
    provider = D.HdfsStateProvider(None, str(tmp_path / "split"))
    provider.persist(a, st)
    back = provider.load(a)
    assert back.numRows == st.numRows
    assert _close(a.computeMetricFrom(back).value.get(), want)
    full_state = a.computeStateFrom(full)
    assert _close(a.computeMetricFrom(full_state).value.get(), want)


@pytest.mark.parametrize("lengths", [(4096, 8, 1000), (1001, 77, 3), (64, 0, 129)])
def test_device_concat_equals_host_concat(lengths):
    """ChunkedTable.concat in HBM (byte-wise validity when chunk lengths are multiples of 8, else bit repacking; int64
    string offsets rebased in place) equals the host concatenation bit for bit, chunks with and without NULLs."""
    import torch
    from deequ_amd.table import ChunkedTable, unpack_validity
    rng = np.random.default_rng(sum(lengths))
    chunks = []
    for i, n in enumerate(lengths):
        words = ["w%d" % rng.integers(0, 50) * int(rng.integers(0, 3)) for _ in range(n)]
        s = [None if (i != 1 and rng.random() < 0.2) else w for w in words]
        x = [None if (i == 0 and rng.random() < 0.3) else float(v) for v in rng.normal(size=n)]
        chunks.append(Table.from_pydict({"s": s, "x": x}, types={"s": "string", "x": "double"}))
    host = ChunkedTable(chunks).concat(["s", "x"])
    for c in chunks:
        c.to_device(0)
    dev = ChunkedTable(chunks).concat(["s", "x"])
    n = sum(lengths)
    for name in ("s", "x"):
        hc, dc = host[name], dev[name]
        hv = unpack_validity(hc.validity, n)
        dvb = dc.device.get("validity")
        dv = np.ones(n, dtype=bool) if dvb is None else unpack_validity(dvb.cpu().numpy(), n)
        assert np.array_equal(hv, dv), name
        if dvb is not None:
            assert len(dvb) % 8 == 0
        if name == "s":
            assert np.array_equal(dc.device["offsets"].cpu().numpy(), np.asarray(hc.offsets, dtype=np.int64))
            data = dc.device["values"].cpu().numpy()
            assert bytes(data[:len(hc.values)]) == bytes(hc.values) and not data[len(hc.values):].any()
        else:
            got = dc.device["values"].cpu().numpy().view(np.float64)
            assert np.array_equal(got[hv], np.asarray(hc.values)[hv])
    torch.cuda.synchronize()


def _helper_threads():
    import threading
    return [t for t in threading.enumerate() if t.name.startswith("dq-helper")]


def test_failure_beside_a_running_grouping_helper(monkeypatch):
    """a failure on the main thread of a chunked run while a grouping build runs on its helper context.
    (1) One chunk's fused scan fails: its scanning analyzers keep that chunk's failure metric
    (R/AnalysisRunner.scala:320-323), the grouping analyzers computed beside it succeed. (2) The state merge raises:
    the run raises only after every helper has finished, and no aux context stays leased. (3) A follow-up run is
    correct."""
    from deequ_amd import native as N
    data, types = _data(400_000, seed=5)
    full, ct = _chunked(data, types, [0, 150_000, 400_000])
    an = [D.Size(), D.Mean("x"), D.Uniqueness(["s"]), D.Entropy("k"), D.CountDistinct(["s", "k"])]
    want = D.AnalysisRunner.onData(full).addAnalyzers(an).run()
    real_run = runners.ScanBatch.run

    def failing_scan(self, *a, **kw):
        if self.data.nrows == 250_000:
            raise RuntimeError("injected scan failure")
        return real_run(self, *a, **kw)
    monkeypatch.setattr(runners.ScanBatch, "run", failing_scan)
    got = D.AnalysisRunner.onData(ct).addAnalyzers(an).run()
    for a in (D.Size(), D.Mean("x")):
        assert not got.metric(a).value.isSuccess, a
        assert "injected scan failure" in str(got.metric(a).value.exception), a
    for a in (D.Uniqueness(["s"]), D.Entropy("k"), D.CountDistinct(["s", "k"])):
        assert _close(got.metric(a).value.get(), want.metric(a).value.get()), a
    assert not _helper_threads() and not N._aux_leased
    monkeypatch.setattr(runners.ScanBatch, "run", real_run)

    def failing_merge(*a, **kw):
        raise RuntimeError("injected merge failure")
    monkeypatch.setattr(runners.AnalysisRunner, "runOnAggregatedStates", staticmethod(failing_merge))
    with pytest.raises(RuntimeError, match="injected merge failure"):
        D.AnalysisRunner.onData(ct).addAnalyzers(an).run()
    assert not _helper_threads() and not N._aux_leased
    monkeypatch.undo()
    got = D.AnalysisRunner.onData(ct).addAnalyzers(an).run()
    for a in an:
        assert _close(got.metric(a).value.get(), want.metric(a).value.get()), a
