"""The exact string GROUP BY oracle (oracle_group_strings, test infrastructure) against a plain Python count on the
CPU: empty strings, NULLs, keys of every length up to 23 bytes, non-ASCII UTF-8, row-range parts with their own
int32 offsets, low and high cardinality; a key past 23 bytes is refused rather than mis-grouped."""
import collections
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import oracle as O  # noqa: E402


def _part(strings):
    valid = np.array([s is not None for s in strings], dtype=bool)
    enc = [(s or "").encode() for s in strings]
    offs = np.zeros(len(enc) + 1, dtype=np.int32)
    offs[1:] = np.cumsum([len(e) for e in enc])
    data = np.frombuffer(b"".join(enc) + b"\0", dtype=np.uint8)
    bits = np.packbits(valid, bitorder="little")
    return data, offs, bits, len(strings)


@pytest.mark.parametrize("distinct", [3, 500, 50_000])
def test_group_strings_equals_a_python_count(distinct):
    rng = np.random.default_rng(distinct)
    base = ["", "a", "é", "NullValue", "x" * 23, "y" * 16, "z" * 15, "€uro"]
    words = base + ["w%d-%s" % (i, "q" * int(i % 12)) for i in range(distinct)]
    parts, allrows = [], []
    for n in (30_000, 0, 41_000):
        idx = rng.integers(0, len(words), n)
        rows = [None if rng.random() < 0.04 else words[i] for i in idx]
        parts.append(_part(rows))
        allrows += rows
    cnt = collections.Counter(r for r in allrows if r is not None)
    queries = ["", "a", "NullValue", "x" * 23, "absent", words[-1]]
    got = O.group_strings_raw(parts, queries)
    assert got["valid_rows"] == sum(cnt.values())
    assert got["null_rows"] == sum(r is None for r in allrows)
    assert got["num_groups"] == len(cnt)
    cc = collections.Counter(cnt.values())
    assert dict(zip(got["count_values"].tolist(), got["count_groups"].tolist())) == dict(cc)
    assert got["query_counts"].tolist() == [cnt.get(q, 0) for q in queries]
    s = O.group_summary_from_count_groups(got["count_values"], got["count_groups"], got["valid_rows"])
    ref = O.group_summary_from_counts(np.array(list(cnt.values())), got["valid_rows"])
    assert s == ref


def test_group_strings_refuses_long_keys():
    with pytest.raises(ValueError):
        O.group_strings_raw([_part(["ok", "k" * 24])])
