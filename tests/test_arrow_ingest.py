"""Arrow / parquet ingest (Table.from_arrow, Table.from_parquet): the host step before the C-ABI
(SURVEY.md §8f rank 1). Host logic only: buffers must decode to the same rows as the row-built
Table, including sliced arrays (non-zero Arrow offsets), nulls and multi-chunk columns."""
import datetime
import decimal

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from deequ_amd import native as N
from deequ_amd.table import Table

ROWS = [("1", "a", 17, 1.3, True), ("2", None, 12, 76.0, False), ("3", "b", None, 89.0, None),
        ("4", "bé", 12, None, True), ("5", None, 1, 1.0, False), ("6", "", 21, 78.0, True)]
NAMES = ["item", "att1", "count", "price", "flag"]


def arrow_table():
    cols = list(zip(*ROWS))
    return pa.table({"item": pa.array(cols[0]), "att1": pa.array(cols[1]), "count": pa.array(cols[2], pa.int32()),
                     "price": pa.array(cols[3], pa.float64()), "flag": pa.array(cols[4], pa.bool_())})


def rows_of(t):
    return list(zip(*[t[n].to_pylist() for n in t.columns]))


def test_from_arrow_matches_row_built_table():
    t = Table.from_arrow(arrow_table())
    assert [c.spark_type for c in t.columns.values()] == [N.TYPE_STRING, N.TYPE_STRING, N.TYPE_INT, N.TYPE_DOUBLE,
                                                          N.TYPE_BOOLEAN]
    assert rows_of(t) == ROWS
    assert t["item"].validity is None and t["att1"].validity is not None


@pytest.mark.parametrize("start,length", [(1, 4), (3, 3), (5, 1), (2, 0)])
def test_sliced_and_chunked_arrays(start, length):
    sliced = arrow_table().slice(start, length)
    assert rows_of(Table.from_arrow(sliced)) == ROWS[start:start + length]
    chunked = pa.concat_tables([arrow_table().slice(0, 2), arrow_table().slice(2)])
    assert rows_of(Table.from_arrow(chunked)) == ROWS


def test_temporal_decimal_and_dictionary_columns():
    tbl = pa.table({
        "d": pa.array([datetime.date(2020, 1, 2), None], pa.date32()),
        "ts": pa.array([1_500, None], pa.timestamp("ms")),
        "dec": pa.array([decimal.Decimal("12.50"), decimal.Decimal("-0.25")], pa.decimal128(6, 2)),
        "cat": pa.array(["x", "y"]).dictionary_encode(),
        "l": pa.array([2**40, -1], pa.int64()),
    })
    t = Table.from_arrow(tbl)
    assert t["d"].spark_type == N.TYPE_DATE and int(t["d"].values[0]) == 18263
    assert t["ts"].spark_type == N.TYPE_TIMESTAMP and int(t["ts"].values[0]) == 1_500_000
    assert t["ts"].to_pylist()[1] is None
    assert t["dec"].spark_type == N.TYPE_DECIMAL and list(t["dec"].values) == [1250, -25]
    assert t["dec"].type_name == "DecimalType(6,2)"
    assert t["cat"].to_pylist() == ["x", "y"]
    assert t["l"].to_pylist() == [2**40, -1]
    with pytest.raises(ValueError, match="exceeds"):
        Table.from_arrow(pa.table({"big": pa.array([decimal.Decimal(1)], pa.decimal128(30, 2))}))


def test_from_parquet_round_trip(tmp_path):
    p = str(tmp_path / "t.parquet")
    pq.write_table(arrow_table(), p, row_group_size=2)
    t = Table.from_parquet(p)
    assert rows_of(t) == ROWS
    assert rows_of(Table.from_parquet(p, columns=["price", "att1"])) == [(r[3], r[1]) for r in ROWS]
    assert t.schema["count"] == "IntegerType"


def test_chunked_table_schema_and_rows():
    """ChunkedTable (row chunks of one schema: Arrow record batches / DataFrame partitions): rows add up, the schema
    is the chunks' common one, and chunks of different schemas are refused."""
    import pytest
    from deequ_amd.table import ChunkedTable, Table
    a = Table.from_pydict({"x": [1, 2, None], "s": ["a", None, "c"]})
    b = Table.from_pydict({"x": [4], "s": ["d"]})
    ct = ChunkedTable([a, b])
    assert ct.nrows == 4 and ct.count() == 4
    assert list(ct.schema.items()) == list(a.schema.items()) and ct.fieldNames == ["x", "s"] and "s" in ct
    with pytest.raises(ValueError):
        ChunkedTable([a, Table.from_pydict({"x": [1.5], "s": ["e"]})])
    with pytest.raises(ValueError):
        ChunkedTable([])
