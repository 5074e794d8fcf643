"""Parquet/Arrow-ingested tables through the GPU engine give the same metrics as the row-built
table (host buffers and HBM-resident buffers), including sliced Arrow arrays."""
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

import deequ_amd as D
from deequ_amd.table import Table
from test_arrow_ingest import ROWS, NAMES, arrow_table

pytestmark = pytest.mark.gpu

ANALYZERS = [D.Size(), D.Completeness("att1"), D.Completeness("flag"), D.Mean("price"), D.Sum("count"),
             D.Minimum("count"), D.Maximum("price"), D.StandardDeviation("price"), D.MaxLength("att1"),
             D.MinLength("att1"), D.ApproxCountDistinct("att1"), D.DataType("item"), D.Uniqueness("att1"),
             D.Entropy("count"), D.Compliance("price", "price > 10")]


def metrics(table):
    ctx = D.AnalysisRunner.onData(table).addAnalyzers(ANALYZERS).run()
    return {str(a): ctx.metric(a).value.get() if ctx.metric(a).value.isSuccess else repr(ctx.metric(a).value)
            for a in ANALYZERS}


@pytest.mark.parametrize("resident", [False, True])
def test_parquet_table_metrics_equal_row_table(tmp_path, resident):
    want = metrics(Table.from_rows(ROWS, NAMES, ["string", "string", "int", "double", "boolean"]))
    p = str(tmp_path / "t.parquet")
    pq.write_table(arrow_table(), p, row_group_size=4)
    t = Table.from_parquet(p)
    if resident:
        t.to_device(0)
    assert metrics(t) == want


def test_sliced_arrow_table_metrics():
    want = metrics(Table.from_rows(ROWS[1:5], NAMES, ["string", "string", "int", "double", "boolean"]))
    assert metrics(Table.from_arrow(arrow_table().slice(1, 4))) == want


@pytest.mark.parametrize("resident", [False, True])
def test_parquet_table_states_match_oracle(tmp_path, resident):
    """The GPU states of the Parquet-ingested table (host buffers, and resident in HBM) against the oracle reading the
    same Arrow buffers with its own decoder, and the oracle on the row-built table: ingest and engine both checked
    against an independent restatement (not GPU against GPU)."""
    import oracle as O
    from test_gpu_scan import assert_state_parity
    rows_table = Table.from_rows(ROWS, NAMES, ["string", "string", "int", "double", "boolean"])
    p = str(tmp_path / "t.parquet")
    pq.write_table(arrow_table(), p, row_group_size=4)
    t = Table.from_parquet(p)
    if resident:
        t.to_device(0)
    scan = [a for a in ANALYZERS if not isinstance(a, (D.Uniqueness, D.Entropy))]
    for a in scan:
        got = a.computeStateFrom(t)
        if isinstance(a, (D.MinLength, D.MaxLength, D.DataType)):  # integer fields: exact, field by field
            exp = O.expected_state(t, a)
            assert (got is None and exp is None) or \
                tuple(getattr(got, f) for f in exp.fields) == exp.key(), (a, got, exp)
        else:
            assert_state_parity(t, a, got)
        e_ingest, e_rows = O.expected_state(t, a), O.expected_state(rows_table, a)
        assert (e_ingest is None and e_rows is None) or e_ingest == e_rows, (a, e_ingest, e_rows)
