"""GPU parity of the Spark SQL surface beyond Check.scala's generated predicates (VERDICT r04 missing #4): CASE WHEN
(searched and simple), if, RLIKE / REGEXP (the device regex engine inside the predicate VM), lower / upper / trim /
ltrim / rtrim / substring, isnan / nanvl / abs, nvl / ifnull, year / month / dayofmonth of DATE and TIMESTAMP columns
and DATE literals — as Compliance predicates and as `where` filters (A/Compliance.scala:49-52,
A/Analyzer.scala:409-432), against the oracle's own parser and evaluator (oracle/oracle.py) with SQL three-valued
logic. Bar: exact counts (NumMatchesAndCount / NumMatches)."""
import numpy as np
import pytest

import deequ_amd as D
from deequ_amd.table import Table, _column_from_pylist
import oracle as O

pytestmark = pytest.mark.gpu

PREDICATES = [
    "CASE WHEN k > 5 THEN 'big' WHEN k = 5 THEN 'five' ELSE 'small' END = 'big'",
    "CASE WHEN k > 5 THEN 1 END = 1",
    "CASE k WHEN 1 THEN TRUE WHEN 2 THEN FALSE END",
    "CASE WHEN s IS NULL THEN 0 WHEN length(s) > 3 THEN 2 ELSE 1 END >= 1",
    "if(x > 0, k, -k) > 2",
    "s RLIKE '^[a-z]+$'", "s RLIKE '\\\\d'", "s NOT RLIKE 'o{2}'", "s REGEXP '(?i)^AB'", "s RLIKE ''",
    "lower(s) RLIKE '^ab'", "upper(s) RLIKE 'FOO'", "k RLIKE '^-'", "k RLIKE '7$'",
    "lower(s) = 'abc'", "upper(s) = 'FOO BAR'", "lower(s) LIKE 'a%c'", "upper(s) LIKE '%É%'", "lower(s) > 'm'",
    "lower(s) IN ('abc', 'xyz')", "length(lower(s)) = 3",
    "trim(s) = 'abc'", "ltrim(s) LIKE 'a%'", "rtrim(s) LIKE '% '", "length(trim(s)) < length(s)",
    "substring(s, 2, 2) = 'bc'", "substring(s, -2) = 'yz'", "substr(s, 0, 1) = 'a'", "substring(s, 3) = ''",
    "isnan(x)", "NOT isnan(x) AND x > 0", "nanvl(x, -1) < 0", "abs(x) < 0.5", "abs(k) >= 7",
    "nvl(k, 100) > 50", "ifnull(x, 0) = 0",
    "year(d) = 2020", "month(d) IN (1, 2, 12)", "dayofmonth(d) = 29", "year(d) < 1900",
    "d >= DATE '2000-03-01' AND d < DATE '2020-01-01'",
    "year(ts) = 2021", "month(ts) = 6 OR day(ts) = 31",
]


def surface_table(n, seed=29):
    rng = np.random.default_rng(seed)
    words = ["abc", "ABC", "Abc", " abc", "abc ", "  abc  ", "xyz", "foo bar", "FOO", "foo", "ab1", "a2c", "",
             "ÉCOLE", "école", "zzz", "m", "ab", "xy yz", "boo"]
    s = [None if rng.random() < 0.08 else words[rng.integers(len(words))] for _ in range(n)]
    k = [None if rng.random() < 0.05 else int(v) for v in rng.integers(-9, 10, n)]
    xs = rng.normal(0.0, 1.0, n)
    xs[rng.random(n) < 0.05] = np.nan
    x = [None if rng.random() < 0.05 else float(v) for v in xs]
    # dates across the 1582 cutover, leap days and month ends; timestamps over 2019-2023 (UTC)
    days = rng.integers(-150_000, 20_000, n)
    modern = rng.random(n) < 0.5
    days[modern] = rng.integers(10_900, 18_300, int(modern.sum()))
    leap = np.array([18321, 11016, 18686, 10956, 10957, 18262, 18627], dtype=np.int64)  # 2020-02-29, 2000-02-29, ...
    days[::37] = leap[rng.integers(0, len(leap), len(days[::37]))]
    d = [None if rng.random() < 0.05 else int(v) for v in days]
    ts = [None if rng.random() < 0.05 else int(v) for v in rng.integers(1_546_300_800_000_000, 1_703_980_800_000_000, n)]
    return Table([_column_from_pylist("s", "string", s), _column_from_pylist("k", "long", k),
                  _column_from_pylist("x", "double", x), _column_from_pylist("d", "date", d),
                  _column_from_pylist("ts", "timestamp", ts)])


def _states(t, analyzers):
    batch = D.ScanBatch(t)
    offs = [a.addOps(batch) for a in analyzers]
    res = batch.run()
    return [a.fromAggregationResult(res, o) for a, o in zip(analyzers, offs)]


@pytest.mark.parametrize("device", [False, True])
def test_sql_surface_compliance_matches_oracle(device):
    t = surface_table(6000)
    if device:
        t.to_device(0)
    analyzers = [D.Compliance("p%d" % i, p) for i, p in enumerate(PREDICATES)]
    for a, g in zip(analyzers, _states(t, analyzers)):
        assert g == O.expected_state(t, a), (a.predicate, g, O.expected_state(t, a))


def test_sql_surface_as_where_filters():
    """The same functions in `where` (conditionalSelection): Size, Mean and Completeness under each filter."""
    t = surface_table(4000, seed=31)
    wheres = ["lower(s) = 'abc'", "s RLIKE '^[a-z]{3}$'", "CASE WHEN x > 0 THEN k ELSE 0 END > 3", "year(d) >= 2000",
              "isnan(x) OR x IS NULL", "trim(s) <> s"]
    analyzers = []
    for w in wheres:
        analyzers += [D.Size(w), D.Mean("k", w), D.Completeness("s", w)]
    for a, g in zip(analyzers, _states(t, analyzers)):
        e = O.expected_state(t, a)
        assert (g is None and e is None) or g == e, (a, g, e)


def test_rlike_budget_failure_is_loud():
    """A value past the regex engine's backtracking budget inside the predicate VM fails the batch, never a count."""
    t = Table([_column_from_pylist("s", "string", ["x" * 40, "ok"])])
    m = D.Compliance("c", "s RLIKE '(x+x+)+y'").calculate(t)
    assert m.value.isFailure
