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
