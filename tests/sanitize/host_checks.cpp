// Host-only checks of libdq's pure host code under AddressSanitizer + UndefinedBehaviorSanitizer (tests/sanitize/
// Makefile builds deequ_amd/csrc/host_algebra.cpp and dq_parse.h with -DDQ_HOST_ONLY): the state algebra
// (dq_state_merge / dq_state_fold, A/*State.sum), the HLL++ estimate (dq_hll_count), Spark's hash of a value
// (dq_spark_hash64), the Spark / Java string parsers (dq_parse.h) on exactly-sized heap buffers, and the row-shard
// arithmetic of multi-device contexts (shard_bounds / shard_columns). Exit 0 = every check held and no sanitizer
// report (the build aborts on the first one).
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <random>
#include <string>
#include <vector>

#include "../../include/dq.h"
#include "../../deequ_amd/csrc/dq_common.h"
#include "../../deequ_amd/csrc/dq_parse.h"

namespace dq {
void shard_bounds(int64_t nrows, int ndev, int i, int64_t* row0, int64_t* count);
void shard_columns(const dq_column* columns, int ncols, int64_t row0, int64_t count, dq_column* out,
                   std::vector<std::vector<int32_t>>& scratch);
}

static int failures = 0;
#define CHECK(c)                                                          \
    do {                                                                  \
        if (!(c)) {                                                       \
            fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, #c); \
            ++failures;                                                   \
        }                                                                 \
    } while (0)

static std::mt19937_64 rng(12345);

static double rand_double() {
    switch (rng() % 8) {
        case 0: return NAN;
        case 1: return -0.0;
        case 2: return INFINITY;
        case 3: return -INFINITY;
        default: return std::uniform_real_distribution<double>(-1e6, 1e6)(rng);
    }
}

static dq_state rand_state(int kind) {
    dq_state s;
    memset(&s, 0, sizeof(s));
    s.kind = kind;
    s.present = rng() % 5 != 0;
    switch (kind) {
        case DQ_OP_SIZE: s.u.num_matches.num_matches = (int64_t)(rng() >> 20); break;
        case DQ_OP_COMPLETENESS: case DQ_OP_COMPLIANCE:
            s.u.num_matches_and_count.num_matches = (int64_t)(rng() >> 24);
            s.u.num_matches_and_count.count = (int64_t)(rng() >> 22);
            break;
        case DQ_OP_MEAN:
            s.u.mean.isum = (int64_t)rng();
            s.u.mean.exact = rng() % 2;
            s.u.mean.sum = s.u.mean.exact ? (double)s.u.mean.isum : rand_double();
            s.u.mean.count = (int64_t)(rng() >> 30);
            break;
        case DQ_OP_SUM: case DQ_OP_MINIMUM: case DQ_OP_MAXIMUM:
            s.u.dbl.isum = (int64_t)rng();
            s.u.dbl.exact = kind == DQ_OP_SUM ? (int)(rng() % 2) : 0;
            s.u.dbl.value = s.u.dbl.exact ? (double)s.u.dbl.isum : rand_double();
            break;
        case DQ_OP_STANDARD_DEVIATION:
            s.u.stddev.n = (double)(rng() % 1000);
            s.u.stddev.avg = rand_double();
            s.u.stddev.m2 = fabs(rand_double());
            break;
        case DQ_OP_CORRELATION:
            s.u.corr.n = (double)(rng() % 1000);
            s.u.corr.x_avg = rand_double();
            s.u.corr.y_avg = rand_double();
            s.u.corr.ck = rand_double();
            s.u.corr.x_mk = fabs(rand_double());
            s.u.corr.y_mk = fabs(rand_double());
            break;
        case DQ_OP_APPROX_COUNT_DISTINCT:
            for (int w = 0; w < DQ_HLL_NUM_WORDS; ++w) s.u.hll.words[w] = (int64_t)rng();
            break;
        case DQ_OP_DATATYPE:
            s.u.datatype.num_null = (int64_t)(rng() >> 30);
            s.u.datatype.num_string = (int64_t)(rng() >> 30);
            break;
        default: break;
    }
    return s;
}

static void check_state_algebra() {
    const int kinds[] = {DQ_OP_SIZE, DQ_OP_COMPLETENESS, DQ_OP_COMPLIANCE, DQ_OP_MEAN, DQ_OP_SUM, DQ_OP_MINIMUM,
                         DQ_OP_MAXIMUM, DQ_OP_STANDARD_DEVIATION, DQ_OP_CORRELATION, DQ_OP_APPROX_COUNT_DISTINCT,
                         DQ_OP_DATATYPE, DQ_OP_MIN_LENGTH, DQ_OP_MAX_LENGTH};
    for (int it = 0; it < 20000; ++it) {
        const int kind = kinds[rng() % (sizeof(kinds) / sizeof(kinds[0]))];
        const int nparts = 1 + (int)(rng() % 9), nops = 1 + (int)(rng() % 4);
        std::vector<dq_state> st((size_t)nparts * nops), out(nops);  // exactly sized: ASan sees any overrun
        for (auto& x : st) x = rand_state(kind);
        const int rc = dq_state_fold(st.data(), nparts, nops, out.data());
        CHECK(rc == DQ_OK || kind == DQ_OP_MIN_LENGTH || kind == DQ_OP_MAX_LENGTH || rc == DQ_ERR_UNSUPPORTED);
        if (rc == DQ_OK && kind == DQ_OP_SIZE) {  // the Long counts of the present parts add up
            for (int i = 0; i < nops; ++i) {
                int64_t want = 0;
                bool any = false;
                for (int r = 0; r < nparts; ++r) {
                    const dq_state& x = st[(size_t)r * nops + i];
                    if (x.present) { want += x.u.num_matches.num_matches; any = true; }
                }
                CHECK(out[i].present == (any ? 1 : 0) || !any);
                if (any) CHECK(out[i].u.num_matches.num_matches == want);
            }
        }
        if (rc == DQ_OK && kind == DQ_OP_APPROX_COUNT_DISTINCT && st[0].present && st.back().present) {
            // register max is commutative
            dq_state ab, ba;
            CHECK(dq_state_merge(&st[0], &st.back(), &ab) == DQ_OK && dq_state_merge(&st.back(), &st[0], &ba) == DQ_OK);
            CHECK(memcmp(ab.u.hll.words, ba.u.hll.words, sizeof(ab.u.hll.words)) == 0);
        }
    }
    dq_state a = rand_state(DQ_OP_SIZE), b = rand_state(DQ_OP_MEAN), o;
    CHECK(dq_state_merge(&a, &b, &o) == DQ_ERR_INVALID_ARGUMENT);  // kinds differ
    CHECK(dq_state_fold(nullptr, 2, 1, &o) == DQ_ERR_INVALID_ARGUMENT);
}

static void check_hll_count() {
    for (int it = 0; it < 20000; ++it) {
        std::vector<int64_t> w(DQ_HLL_NUM_WORDS);
        const int mode = (int)(rng() % 4);
        for (auto& x : w) {
            uint64_t v = rng();
            if (mode == 0) v = 0;                              // all registers 0: linear counting
            if (mode == 1) v &= 0x0410410410410410ULL;         // small registers
            if (mode == 2) v = 0x0FFFFFFFFFFFFFFFULL;          // every register 63: the Java int-shift quirk
            x = (int64_t)v;
        }
        const double e = dq_hll_count(w.data());
        // registers >= 32 hit the reference's Java int shift (1 << Midx wraps): any value, no UB; below, a count
        if (mode <= 1) CHECK(e == e && e >= 0.0);
    }
}

static void check_hashes() {
    for (int len = 0; len <= 300; ++len) {
        std::vector<uint8_t> b(len);
        for (auto& c : b) c = (uint8_t)rng();
        const int64_t h1 = dq_spark_hash64(DQ_TYPE_STRING, b.data(), len);
        const int64_t h2 = dq_spark_hash64(DQ_TYPE_STRING, b.data(), len);
        CHECK(h1 == h2);
    }
    const int types[] = {DQ_TYPE_BOOLEAN, DQ_TYPE_BYTE, DQ_TYPE_SHORT, DQ_TYPE_INT, DQ_TYPE_LONG, DQ_TYPE_FLOAT,
                         DQ_TYPE_DOUBLE, DQ_TYPE_DATE, DQ_TYPE_TIMESTAMP, DQ_TYPE_DECIMAL};
    for (int t : types) {
        const int w = (t == DQ_TYPE_BOOLEAN || t == DQ_TYPE_BYTE) ? 1 : t == DQ_TYPE_SHORT ? 2 :
                      (t == DQ_TYPE_INT || t == DQ_TYPE_DATE || t == DQ_TYPE_FLOAT) ? 4 : 8;
        for (int it = 0; it < 1000; ++it) {
            std::vector<uint8_t> cell(w);  // one cell, exactly its width
            for (auto& c : cell) c = (uint8_t)rng();
            (void)dq_spark_hash64(t, cell.data(), w);
        }
    }
    CHECK(dq_spark_hash64(DQ_TYPE_LONG, nullptr, 8) == 0);
}

static void check_parsers() {
    const char* alphabet = "0123456789+-.eEdDfF Na Infty\t";
    const size_t na = strlen(alphabet);
    const char* fixed[] = {"", "-", "+", ".", "1", "-0", "9223372036854775807", "-9223372036854775808",
                           "9223372036854775808", "12.5", "1e308", "1e309", "4.9e-324", "NaN", "-Infinity",
                           " 42 ", "0x1p3", "123456789012345678901234567890", "1.7976931348623157e308d", "2.5f"};
    for (const char* f : fixed) {
        const int n = (int)strlen(f);
        std::vector<uint8_t> b(f, f + n);
        int64_t l;
        double d;
        bool slow = false;
        (void)dq::spark_string_to_long(b.data(), n, l);
        (void)dq::java_parse_double(b.data(), n, d, slow);
    }
    for (int it = 0; it < 200000; ++it) {
        const int n = (int)(rng() % 40);
        std::vector<uint8_t> b(n);  // exactly n bytes: a read past the end is reported
        for (auto& c : b) c = (uint8_t)alphabet[rng() % na];
        int64_t l;
        double d;
        bool slow = false;
        (void)dq::spark_string_to_long(b.data(), n, l);
        const bool ok = dq::java_parse_double(b.data(), n, d, slow);
        if (ok && !slow && n > 0) {  // finite decimal literals round-trip through strtod (correct rounding)
            std::string s(b.begin(), b.end());
            bool plain = s.find_first_not_of("0123456789+-.eE") == std::string::npos;
            if (plain) {
                char* end = nullptr;
                const double r = strtod(s.c_str(), &end);
                if (end && *end == 0 && r == r) CHECK(memcmp(&r, &d, 8) == 0 || (r == 0 && d == 0));
            }
        }
    }
}

static void check_shards() {
    for (int it = 0; it < 5000; ++it) {
        const int64_t nrows = (int64_t)(rng() % 200000);
        const int ndev = 1 + (int)(rng() % 8);
        int64_t covered = 0;
        for (int i = 0; i < ndev; ++i) {
            int64_t r0, cnt;
            dq::shard_bounds(nrows, ndev, i, &r0, &cnt);
            CHECK(r0 % 2048 == 0 || cnt == 0);
            CHECK(r0 == covered || cnt == 0);
            CHECK(cnt >= 0 && r0 + cnt <= nrows);
            covered += cnt;
        }
        CHECK(covered == nrows);
    }
    for (int it = 0; it < 200; ++it) {
        const int64_t n = 1 + (int64_t)(rng() % 20000);
        std::vector<int32_t> offs(n + 1, 0);
        for (int64_t r = 0; r < n; ++r) offs[r + 1] = offs[r] + (int32_t)(rng() % 7);
        std::vector<uint8_t> data(offs[n] + 1);
        std::vector<int64_t> vals(n);
        std::vector<uint8_t> valid((n + 7) / 8);
        dq_column cols[2];
        memset(cols, 0, sizeof(cols));
        cols[0].spark_type = DQ_TYPE_STRING;
        cols[0].length = n;
        cols[0].values = data.data();
        cols[0].offsets = offs.data();
        cols[0].validity = valid.data();
        cols[1].spark_type = DQ_TYPE_LONG;
        cols[1].length = n;
        cols[1].values = vals.data();
        const int ndev = 1 + (int)(rng() % 5);
        for (int i = 0; i < ndev; ++i) {
            int64_t r0, cnt;
            dq::shard_bounds(n, ndev, i, &r0, &cnt);
            dq_column out[2];
            std::vector<std::vector<int32_t>> scratch;
            dq::shard_columns(cols, 2, r0, cnt, out, scratch);
            CHECK(out[0].length == cnt && out[0].offsets[0] == 0);
            if (cnt) {
                CHECK(out[0].offsets[cnt] == offs[r0 + cnt] - offs[r0]);
                CHECK((const uint8_t*)out[0].values == data.data() + offs[r0]);
                CHECK((const int64_t*)out[1].values == vals.data() + r0);
                CHECK(out[0].validity == valid.data() + r0 / 8);
            }
        }
    }
}

int main() {
    check_state_algebra();
    check_hll_count();
    check_hashes();
    check_parsers();
    check_shards();
    if (failures) {
        fprintf(stderr, "%d check(s) failed\n", failures);
        return 1;
    }
    printf("host_checks: ok\n");
    return 0;
}
