"""Predicate compiler (Spark SQL strings -> dq_predicate postfix programs). CPU only."""
import pytest

import deequ_amd.native as N
from deequ_amd.expr import compile_predicate, PredicateSyntaxError, UnresolvedColumnError


COLS = {"item": 0, "att1": 1, "att2": 2}


def ops(text):
    p = compile_predicate(text, COLS)
    code = list(p._code)
    return [(code[i], code[i + 1]) for i in range(0, len(code), 2)]


def test_reference_predicates_compile():
    # the predicates the reference tests use
    for t in ["item IN ('1', '2')", "att1 > 3", "att1 > 2", "att2 = 0", "att1 < 4", "item != '6'",
              "unique < 4".replace("unique", "att1"), "att1 = 'b'", "att1 != ''", "att1 != 'dddd'",
              "att1 IS NULL OR att2 IS NOT NULL", "NOT (att1 >= 2 AND att2 <= 5)", "att1 BETWEEN 1 AND 3",
              "coalesce(att1, 0) > 1", "att1 LIKE '%fac%ets'", "length(item) >= 2", "att1 + att2 * 2 > 3",
              "`att1` <=> NULL", "att1 NOT IN (1, 2)", "CAST(item AS DOUBLE) > 1.5", "att1 == 3", "att1 <> 3"]:
        p = compile_predicate(t, COLS)
        assert len(p._code) % 2 == 0 and len(p._code) > 0, t


def test_postfix_shape():
    assert ops("att1 > 3") == [(N.P_COL, 1), (N.P_CONST, 0), (N.P_GT, 0)]
    assert ops("item IN ('1', '2')") == [(N.P_COL, 0), (N.P_CONST, 0), (N.P_CONST, 1), (N.P_IN, 2)]
    assert ops("att1 > 1 AND att2 < 2 OR att1 IS NULL")[-1] == (N.P_OR, 0)
    assert ops("NOT att1 > 1")[-1] == (N.P_NOT, 0)


def test_precedence_and_or():
    # a OR b AND c == a OR (b AND c)
    o = ops("att1 = 1 OR att1 = 2 AND att2 = 3")
    assert o[-1] == (N.P_OR, 0) and o[-2] == (N.P_AND, 0)


def test_unknown_column_is_an_analysis_error():
    with pytest.raises(UnresolvedColumnError):
        compile_predicate("attNoSuchColumn > 3", COLS)


def test_syntax_errors():
    for t in ["att1 >", "(att1 > 1", "att1 > 1)", "att1 LIKE att2", "frobnicate(att1)"]:
        with pytest.raises(PredicateSyntaxError):
            compile_predicate(t, COLS)


def test_string_constants_pool():
    p = compile_predicate("item = 'héllo' OR item = 'it''s'", COLS)
    pool = bytes(p._strings[:p._strings_len])
    assert "héllo".encode() in pool and b"it's" in pool
