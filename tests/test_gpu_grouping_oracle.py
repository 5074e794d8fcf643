"""Every grouping build pinned DIRECTLY to the oracle at the sizes where it runs.

The fast build (partition1_fast -> scatter2_fast -> build_kernel) only runs from 2^24 rows on one fixed-width key
column; its narrow-key variants (32-bit offsets around a sampled base) and the optimistic one-pass small build of
general keys only run at millions of rows. Here each of them is compared with the C oracle's count(*) GROUP BY
(oracle_group_counts: canonical keys, a radix sort and a run length — A/GroupingAnalyzers.scala:53-79) on the same
rows: the whole exported (key, count) multiset bit-exact, the fused summary (groups, unique groups, NULL rows) exact and
the entropy within 1e-12 (A/GroupingAnalyzers.scala:83-120, A/Entropy.scala:28-42). The build-path counters
(dq_freq_path_count) prove which build produced the table that was checked."""
import zlib

import numpy as np
import pytest

import deequ_amd.native as N
from deequ_amd import engine
from deequ_amd.table import Table, Column, pack_validity
import oracle as O

pytestmark = pytest.mark.gpu

TYPES = {np.dtype(np.float64): N.TYPE_DOUBLE, np.dtype(np.int64): N.TYPE_LONG, np.dtype(np.int32): N.TYPE_INT,
         np.dtype(np.float32): N.TYPE_FLOAT}


def _paths_delta(before):
    after = engine.ctx().freq_paths()
    return {k: after[k] - before[k] for k in after if after[k] != before[k]}


def _device_table(v, valid_bits):
    import torch
    col = Column("k", TYPES[v.dtype], None, None, length=len(v))
    col.device = {"values": torch.from_numpy(v).cuda()}
    if valid_bits is not None:
        col.device["validity"] = torch.from_numpy(valid_bits).cuda()
    return Table([col])


def _check_against_oracle(v, valid_bits, want_paths, include_nulls=(False,)):
    """Build the table on the GPU and compare it with oracle_group_counts over the same buffers."""
    n = len(v)
    okeys, ocounts, onulls = O.group_counts_raw(TYPES[v.dtype], v, valid_bits, n)
    exp = O.group_summary_from_counts(ocounts, n - onulls)
    t = _device_table(v, valid_bits)
    for inul in include_nulls:
        before = engine.ctx().freq_paths()
        ft = engine.frequencies(t, ["k"], inul)
        paths = _paths_delta(before)
        for p in want_paths:
            assert paths.get(p, 0) >= 1, (want_paths, paths)
        if "fast_done" not in want_paths:
            assert "fast_done" not in paths, paths
        s = ft.summary(None)
        assert s["null_count"] == (onulls if inul else 0)
        assert s["num_rows"] == (n if inul else n - onulls)
        assert (s["num_groups"] - (1 if inul and onulls else 0), s["num_unique"] - (1 if inul and onulls == 1 else 0)) \
            == (exp["num_groups"], exp["num_unique"]), (s, exp)
        assert s["max_count"] == max(int(ocounts.max()) if len(ocounts) else 0, onulls if inul else 0)
        if not inul:
            assert abs(s["entropy"] - exp["entropy"]) <= 1e-12 * max(1.0, exp["entropy"]), (s["entropy"], exp)
        k, c = ft.export_pairs()
        ku = k.view(np.uint64)
        o = np.argsort(ku, kind="stable")
        assert np.array_equal(ku[o], okeys), "exported keys differ from the oracle's"
        assert np.array_equal(c[o], ocounts), "exported counts differ from the oracle's"
        del ft
    return paths


def _value_mixing_to_all_ones():
    """The int64 whose splitmix64 finalizer is 2^64 - 1 (the EMPTY slot marker of the device tables)."""
    m = (1 << 64) - 1

    def inv(a):
        x = a
        for _ in range(6):
            x = (x * (2 - a * x)) & m
        return x

    def unxorshift(z, k):
        r = z
        for _ in range(64 // k + 1):
            r = z ^ (r >> k)
        return r & m
    z = unxorshift(m, 31)
    z = (z * inv(0x94D049BB133111EB)) & m
    z = unxorshift(z, 27)
    z = (z * inv(0xBF58476D1CE4E5B9)) & m
    z = unxorshift(z, 30)
    return z - (1 << 64) if z >= 1 << 63 else z


N_FAST = 32_000_000  # above the fast build's 2^24-row threshold


def _case(case, n=N_FAST):
    rng = np.random.default_rng(zlib.crc32(case.encode()))
    valid = None
    if case == "uniform":  # full-width keys, ~3e6 distinct, repeats: the 64-bit fast path
        pool = rng.integers(-2 ** 63, 2 ** 63 - 1, 3_000_000, dtype=np.int64)
        v = pool[rng.integers(0, len(pool), n)]
        v[::1_000_003] = _value_mixing_to_all_ones()
        return v, None, ["fast", "fast_done"]
    if case == "heavy_hitter":  # 40 % one key: more spilled keys than the spill buffer holds -> the exact path
        v = np.where(rng.random(n) < 0.4, 12345, rng.integers(-2 ** 62, 2 ** 62, n)).astype(np.int64)
        return v, None, ["fast", "exact"]
    if case == "spilled_hitters":  # 5 % / 1 % / 2000 x 0.05 % keys past their buckets' slack: spilled, fast path
        v = rng.integers(-2 ** 62, 2 ** 62, n)
        u = rng.random(n)
        v[u < 0.05] = 777
        v[(u >= 0.05) & (u < 0.06)] = -1
        mid = (u >= 0.06) & (u < 0.16)
        v[mid] = rng.integers(0, 2000, int(mid.sum())) * 1_000_003
        valid = rng.random(n) > 0.01
        return v.astype(np.int64), valid, ["fast", "fast_done", "fast_spill"]
    if case == "double_nulls_nan_negzero":
        v = rng.integers(-2_000_000, 2_000_000, n).astype(np.float64) / 8.0
        v[rng.random(n) < 0.01] = np.nan
        nan2 = rng.random(n) < 0.002  # a non-canonical NaN payload groups with NaN
        v[nan2] = np.frombuffer(np.uint64(0x7FF8000000000123).tobytes(), np.float64)[0]
        v[rng.random(n) < 0.01] = -0.0
        v[rng.random(n) < 0.01] = 0.0
        valid = rng.random(n) > 0.01
        return v, valid, ["fast", "fast_done", "fast_spill"]
    if case == "narrow_window":  # 8-byte keys inside a 2^31 window far from zero
        v = rng.integers(-5_000_000_000 - 3_000_000, -5_000_000_000, n, dtype=np.int64)
        valid = rng.random(n) > 0.02
        return v, valid, ["fast_narrow", "fast_done"]
    if case == "narrow_outlier":  # a key outside the sampled window on a row the sample skips: 64-bit restart
        v = rng.integers(0, 2_000_000, n, dtype=np.int64)
        v[12345] = 1 << 40  # n / 65536 = 488: not on the sample's stride
        v[777777] = -(1 << 40)
        return v, None, ["fast_narrow", "fast", "fast_done"]
    if case == "int32":
        v = rng.integers(-2 ** 31, 2 ** 31, n, dtype=np.int64).astype(np.int32)
        v[::4] = rng.integers(-500, 500, len(v[::4]), dtype=np.int32)  # 8000 rows a key: past a bucket's slack
        valid = rng.random(n) > 0.05
        return v, valid, ["fast_narrow", "fast_done", "fast_spill"]
    if case == "float32":
        v = (rng.integers(-3_000_000, 3_000_000, n) / 4.0).astype(np.float32)
        v[rng.random(n) < 0.01] = np.nan
        v[rng.random(n) < 0.01] = -0.0
        return v, None, ["fast_narrow", "fast_done", "fast_spill"]
    raise KeyError(case)


@pytest.mark.parametrize("case", ["uniform", "heavy_hitter", "spilled_hitters", "double_nulls_nan_negzero", "narrow_window",
                                  "narrow_outlier", "int32", "float32"])
def test_fast_build_against_oracle(case):
    v, valid, paths = _case(case)
    bits = None if valid is None else pack_validity(valid)
    _check_against_oracle(v, bits, paths, include_nulls=(False, True) if valid is not None else (False,))


def test_c4_generator_with_nulls_against_oracle():
    """The C4 key generator (D distinct keys, D/2 of them 19 times) with 1 % NULLs at 1e8 rows — no
    closed form covers it — against the oracle, on the 64-bit fast path bench.py times."""
    import torch
    R, Dn = 100_000_000, 10_000_000
    keys = O.synth_freq_keys(R, Dn, 0, R)
    ctx = engine.ctx()
    dev = torch.empty(R, dtype=torch.int64, device="cuda")
    ctx.synth_freq_keys(R, Dn, 0, R, dev.data_ptr())  # the device generator equals the oracle's
    vbits = torch.zeros((R + 63) // 64 * 8, dtype=torch.uint8, device="cuda")
    ctx.synth_validity(0x5EED0C4, 0, R, 10, vbits.data_ptr())
    ctx.synchronize()
    assert np.array_equal(dev.cpu().numpy(), keys)
    del dev
    bits = vbits.cpu().numpy()
    _check_against_oracle(keys, bits, ["fast", "fast_done"], include_nulls=(False, True))


@pytest.mark.parametrize("distinct", [60, 3000, 1_000_000])
def test_optimistic_small_build_against_oracle(distinct):
    """General (string) keys at 5e6 rows: the one-pass small build tried without the sizing pass. It produces the
    table itself at 60 distinct; at 3000 / 1e6 it gives up and the sized path builds it. Both against the oracle."""
    import pyarrow as pa
    rng = np.random.default_rng(distinct)
    n = 5_000_000
    words = np.array(["v%07d" % i for i in range(distinct)], dtype=object)
    idx = rng.integers(0, distinct, n)
    valid = rng.random(n) > 0.03
    t = Table.from_arrow(pa.table({"s": pa.array(words[idx], type=pa.string(), mask=~valid)}))
    t.to_device(0)
    before = engine.ctx().freq_paths()
    ft = engine.frequencies(t, ["s"], False)
    paths = _paths_delta(before)
    if distinct == 60:
        assert paths.get("small_optimistic", 0) == 1 and "exact" not in paths, paths
    else:
        assert paths.get("small", 0) >= 1 and "small_optimistic" not in paths and paths.get("exact", 0) >= 1, paths
    # oracle: the same rows grouped from the raw index column (word i <-> index i), in C
    okeys, ocounts, onulls = O.group_counts_raw(N.TYPE_LONG, idx.astype(np.int64), pack_validity(valid), n)
    exp = O.group_summary_from_counts(ocounts, n - onulls)
    s = ft.summary(None)
    assert (s["num_rows"], s["num_groups"], s["num_unique"]) == (n - onulls, exp["num_groups"], exp["num_unique"])
    assert abs(s["entropy"] - exp["entropy"]) <= 1e-12 * max(1.0, exp["entropy"])
    got = ft.to_dict()
    want = {("v%07d" % int(k),): int(c) for k, c in zip(okeys.view(np.int64), ocounts)}
    assert got == want


@pytest.mark.parametrize("n", [200_000, 5_000_000])
@pytest.mark.parametrize("include_nulls", [False, True])
def test_small_build_one_string_column_short_and_long_keys(n, include_nulls, monkeypatch):
    """The small build of one string key column holds keys of <= 15 bytes as two words (hashed from them and verified
    against the representative's words in LDS); longer keys go through the byte path. Keys of every length 0-40, the
    literal "NullValue" (a Histogram groups NULL rows with it) and NULLs, at the sized (2e5 rows) and the optimistic
    (5e6 rows) small build: the groups equal a Python count and the byte-path build (DQ_SMALL_NO_STR1)."""
    import collections
    import pyarrow as pa
    rng = np.random.default_rng(n + include_nulls)
    base = ["", "a", "NullValue", "NullValu", "NullValuee", "x" * 15, "y" * 16, "z" * 40, "é" * 5, "é" * 8]
    words = np.array(base + ["w%d-%s" % (i, "q" * int(i % 37)) for i in range(290)], dtype=object)
    idx = rng.integers(0, len(words), n)
    valid = rng.random(n) > 0.03
    t = Table.from_arrow(pa.table({"s": pa.array(words[idx], type=pa.string(), mask=~valid)}))
    t.to_device(0)
    before = engine.ctx().freq_paths()
    got = engine.frequencies(t, ["s"], include_nulls).to_dict()
    paths = _paths_delta(before)
    assert paths.get("small_optimistic" if n >= 1 << 22 else "small", 0) >= 1, paths
    monkeypatch.setenv("DQ_SMALL_NO_STR1", "1")
    ref = engine.frequencies(t, ["s"], include_nulls).to_dict()
    assert got == ref
    exp = collections.Counter()
    for w, v in zip(words[idx], valid):
        if v:
            exp[(w,)] += 1
        elif include_nulls:
            exp[(None,)] += 1
    assert sum(got.values()) == sum(exp.values())
    if include_nulls:  # NULL rows and "NullValue" rows are one group (the Histogram's NullFieldReplacement)
        nv = exp.pop((None,), 0) + exp.pop(("NullValue",), 0)
        gnv = got.get((None,), 0) + got.get(("NullValue",), 0)
        assert gnv == nv
        got = {k: c for k, c in got.items() if k not in ((None,), ("NullValue",))}
    assert got == dict(exp)
