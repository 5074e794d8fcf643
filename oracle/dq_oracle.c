/*
 * dq_oracle.c — CPU restatement of deequ's scan-shareable aggregations (TEST INFRASTRUCTURE).
 *
 * This file is the parity oracle for the MI355X engine. Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it; the product (deequ_amd/) never does.
 *
 * It restates, row by row and in Spark's sequential per-partition order, the aggregates deequ
 * builds (paths under /root/reference/src/main/scala/com/amazon/deequ/analyzers/):
 *   count / sum / min / max        Size.scala:33-47, Completeness.scala:38-41, Mean.scala:36-40,
 *                                  Sum.scala:34-37, Minimum.scala:34-37, Maximum.scala:34-37
 *                                  (Spark 2.2 Sum: Long accumulator for integral inputs, Double for
 *                                  fractional; Min/Max order NaN above every number)
 *   stddev (n, avg, m2)            catalyst/StatefulStdDevPop.scala:24-34 — Spark CentralMomentAgg
 *                                  update: n' = n+1; d = x-avg; dN = d/n'; avg += dN; m2 += d*(d-dN)
 *   correlation                    catalyst/StatefulCorrelation.scala:24-49 — Spark Corr update
 *   HLL++ registers + estimate     catalyst/StatefulHyperloglogPlus.scala:89-298 (P = 9, XXH64 seed 42)
 * plus an "exact" two-pass long-double mean/m2 used to judge fp64 tolerances, and the synthetic
 * splitmix64 generators of SURVEY.md §8d (same formulas as deequ_amd/csrc/synth.hip).
 *
 * Spark-side pieces (CentralMomentAgg, Corr, XXH64) are third-party (spark-catalyst_2.11:2.2.2,
 * pom.xml:73-83) and absent from /root/reference; XXH64 is pinned against the python `xxhash`
 * package, the rest against the reference's known-answer tests (tests/golden/).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>

#include "hll_bias_p9.h"

/* ---- XXH64 (standard; Spark's XXH64.hashInt / hashLong / hashUnsafeBytes) --------------------- */
static const uint64_t XP1 = 0x9E3779B185EBCA87ULL, XP2 = 0xC2B2AE3D27D4EB4FULL, XP3 = 0x165667B19E3779F9ULL,
                      XP4 = 0x85EBCA77C2B2AE63ULL, XP5 = 0x27D4EB2F165667C5ULL;

static uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static uint64_t avalanche(uint64_t h) {
    h ^= h >> 33; h *= XP2; h ^= h >> 29; h *= XP3; h ^= h >> 32;
    return h;
}
static uint64_t rd64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }
static uint32_t rd32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }
static uint64_t xround(uint64_t acc, uint64_t in) { acc += in * XP2; acc = rotl(acc, 31); return acc * XP1; }

uint64_t oracle_xxh64(const uint8_t* p, int64_t len, uint64_t seed) {
    const uint8_t* end = p + len;
    uint64_t h;
    if (len >= 32) {
        uint64_t v1 = seed + XP1 + XP2, v2 = seed + XP2, v3 = seed, v4 = seed - XP1;
        while (p + 32 <= end) {
            v1 = xround(v1, rd64(p)); v2 = xround(v2, rd64(p + 8));
            v3 = xround(v3, rd64(p + 16)); v4 = xround(v4, rd64(p + 24));
            p += 32;
        }
        h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
        uint64_t vs[4] = {v1, v2, v3, v4};
        for (int i = 0; i < 4; ++i) { h ^= xround(0, vs[i]); h = h * XP1 + XP4; }
    } else {
        h = seed + XP5;
    }
    h += (uint64_t)len;
    for (; p + 8 <= end; p += 8) { h ^= xround(0, rd64(p)); h = rotl(h, 27) * XP1 + XP4; }
    if (p + 4 <= end) { h ^= (uint64_t)rd32(p) * XP1; h = rotl(h, 23) * XP2 + XP3; p += 4; }
    for (; p < end; ++p) { h ^= (uint64_t)(*p) * XP5; h = rotl(h, 11) * XP1; }
    return avalanche(h);
}

/* Spark type codes (include/dq.h dq_spark_type). */
enum { T_BOOLEAN = 1, T_BYTE, T_SHORT, T_INT, T_LONG, T_FLOAT, T_DOUBLE, T_STRING, T_DATE, T_TIMESTAMP, T_DECIMAL };

/* XxHash64Function.hash(value, type, 42) for a fixed-width value given as raw bytes. */
uint64_t oracle_spark_hash(int spark_type, const void* v) {
    uint8_t b[8];
    switch (spark_type) {
        case T_BOOLEAN: { int32_t x = *(const uint8_t*)v ? 1 : 0; memcpy(b, &x, 4); return oracle_xxh64(b, 4, 42); }
        case T_BYTE: { int32_t x = *(const int8_t*)v; memcpy(b, &x, 4); return oracle_xxh64(b, 4, 42); }
        case T_SHORT: { int32_t x = *(const int16_t*)v; memcpy(b, &x, 4); return oracle_xxh64(b, 4, 42); }
        case T_INT: case T_DATE: return oracle_xxh64((const uint8_t*)v, 4, 42);
        case T_FLOAT: {
            float f = *(const float*)v;
            uint32_t u = 0x7fc00000u;          /* Float.floatToIntBits canonical NaN */
            if (f == f) memcpy(&u, &f, 4);
            memcpy(b, &u, 4);
            return oracle_xxh64(b, 4, 42);
        }
        case T_DOUBLE: {
            double d = *(const double*)v;
            uint64_t u = 0x7ff8000000000000ULL; /* Double.doubleToLongBits canonical NaN */
            if (d == d) memcpy(&u, &d, 8);
            memcpy(b, &u, 8);
            return oracle_xxh64(b, 8, 42);
        }
        default: return oracle_xxh64((const uint8_t*)v, 8, 42); /* LONG, TIMESTAMP, DECIMAL unscaled */
    }
}

/* ---- one column, Spark order ---------------------------------------------------------------- */
typedef struct {
    int64_t n;          /* rows counted (valid and where-true) */
    int64_t isum;       /* integral: Long sum with wrap-around */
    double dsum;        /* fractional: Double sum in row order */
    int64_t imin, imax;
    double dmin, dmax;  /* Spark ordering: NaN greatest */
    double w_n, w_avg, w_m2;          /* CentralMomentAgg, row order */
    double ex_mean, ex_m2;            /* exact two-pass in long double */
} oracle_col;

static int elem_size(int t) {
    switch (t) {
        case T_BOOLEAN: case T_BYTE: return 1;
        case T_SHORT: return 2;
        case T_INT: case T_DATE: case T_FLOAT: return 4;
        default: return 8;
    }
}
static int is_frac(int t) { return t == T_FLOAT || t == T_DOUBLE; }
static int64_t as_i64(int t, const uint8_t* p) {
    switch (t) {
        case T_BOOLEAN: return *p ? 1 : 0;
        case T_BYTE: return *(const int8_t*)p;
        case T_SHORT: { int16_t x; memcpy(&x, p, 2); return x; }
        case T_INT: case T_DATE: { int32_t x; memcpy(&x, p, 4); return x; }
        default: { int64_t x; memcpy(&x, p, 8); return x; }
    }
}
static double as_f64(int t, const uint8_t* p, int scale) {
    if (t == T_FLOAT) { float f; memcpy(&f, p, 4); return (double)f; }
    if (t == T_DOUBLE) { double d; memcpy(&d, p, 8); return d; }
    if (t == T_DECIMAL) {
        double s = 1.0;
        for (int i = 0; i < scale; ++i) s *= 10.0;
        return (double)as_i64(t, p) / s;
    }
    return (double)as_i64(t, p);
}
/* Spark's NaN-aware "a > b" for doubles (Utils.nanSafeCompareDoubles). */
static int nan_gt(double a, double b) {
    if (a != a) return b == b;
    if (b != b) return 0;
    return a > b;
}

/* mask[i] != 0: row i is non-null and its `where` is TRUE. */
void oracle_column(int spark_type, int decimal_scale, const void* values, const uint8_t* mask, int64_t nrows,
                   oracle_col* out) {
    const uint8_t* v = (const uint8_t*)values;
    const int es = elem_size(spark_type);
    oracle_col r;
    memset(&r, 0, sizeof(r));
    r.imin = INT64_MAX;
    r.imax = INT64_MIN;
    r.dmin = NAN;
    r.dmax = NAN;
    int first = 1;
    long double s = 0.0L;
    for (int64_t i = 0; i < nrows; ++i) {
        if (!mask[i]) continue;
        const uint8_t* p = v + i * es;
        const double x = as_f64(spark_type, p, decimal_scale);
        r.n++;
        if (is_frac(spark_type)) {
            r.dsum += x;
            if (first || nan_gt(r.dmin, x)) r.dmin = x;
            if (first || nan_gt(x, r.dmax)) r.dmax = x;
        } else {
            const int64_t xi = as_i64(spark_type, p);
            r.isum = (int64_t)((uint64_t)r.isum + (uint64_t)xi);
            if (xi < r.imin) r.imin = xi;
            if (xi > r.imax) r.imax = xi;
        }
        first = 0;
        /* CentralMomentAgg update (input cast to Double) */
        const double n1 = r.w_n + 1.0;
        const double delta = x - r.w_avg;
        const double deltaN = delta / n1;
        r.w_avg += deltaN;
        r.w_m2 += delta * (delta - deltaN);
        r.w_n = n1;
        s += (long double)x;
    }
    if (r.n > 0) {
        const long double mean = s / (long double)r.n;
        long double m2 = 0.0L;
        for (int64_t i = 0; i < nrows; ++i) {
            if (!mask[i]) continue;
            const long double d = (long double)as_f64(spark_type, v + i * es, decimal_scale) - mean;
            m2 += d * d;
        }
        r.ex_mean = (double)mean;
        r.ex_m2 = (double)m2;
    }
    *out = r;
}

typedef struct {
    double n, x_avg, y_avg, ck, x_mk, y_mk;   /* Spark Corr update, row order */
    double ex_ck, ex_x_mk, ex_y_mk;           /* exact two-pass */
} oracle_corr;

void oracle_correlation(int tx, int sx, const void* xv, int ty, int sy, const void* yv, const uint8_t* mask,
                        int64_t nrows, oracle_corr* out) {
    const uint8_t* xp = (const uint8_t*)xv;
    const uint8_t* yp = (const uint8_t*)yv;
    const int ex = elem_size(tx), ey = elem_size(ty);
    oracle_corr r;
    memset(&r, 0, sizeof(r));
    long double sxl = 0.0L, syl = 0.0L;
    for (int64_t i = 0; i < nrows; ++i) {
        if (!mask[i]) continue;
        const double x = as_f64(tx, xp + i * ex, sx), y = as_f64(ty, yp + i * ey, sy);
        const double n1 = r.n + 1.0;
        const double dx = x - r.x_avg;
        const double dy = y - r.y_avg;
        r.x_avg += dx / n1;
        r.y_avg += dy / n1;
        r.ck += dx * (y - r.y_avg);
        r.x_mk += dx * (x - r.x_avg);
        r.y_mk += dy * (y - r.y_avg);
        r.n = n1;
        sxl += x;
        syl += y;
    }
    if (r.n > 0) {
        const long double mx = sxl / (long double)r.n, my = syl / (long double)r.n;
        long double ck = 0, xm = 0, ym = 0;
        for (int64_t i = 0; i < nrows; ++i) {
            if (!mask[i]) continue;
            const long double dx = (long double)as_f64(tx, xp + i * ex, sx) - mx;
            const long double dy = (long double)as_f64(ty, yp + i * ey, sy) - my;
            ck += dx * dy;
            xm += dx * dx;
            ym += dy * dy;
        }
        r.ex_ck = (double)ck;
        r.ex_x_mk = (double)xm;
        r.ex_y_mk = (double)ym;
    }
    *out = r;
}

/* ---- HLL++ (StatefulHyperloglogPlus.update, P = 9) ------------------------------------------- */
static void hll_add(uint8_t* regs, uint64_t x) {
    const uint32_t idx = (uint32_t)(x >> 55);
    const uint64_t w = (x << 9) | (1ULL << 8);
    const uint8_t pw = (uint8_t)(__builtin_clzll(w) + 1);
    if (pw > regs[idx]) regs[idx] = pw;
}

void oracle_hll_fixed(int spark_type, const void* values, const uint8_t* mask, int64_t nrows, uint8_t* regs512) {
    const uint8_t* v = (const uint8_t*)values;
    const int es = elem_size(spark_type);
    for (int64_t i = 0; i < nrows; ++i)
        if (mask[i]) hll_add(regs512, oracle_spark_hash(spark_type, v + i * es));
}

void oracle_hll_strings(const uint8_t* data, const int32_t* offsets, const uint8_t* mask, int64_t nrows,
                        uint8_t* regs512) {
    for (int64_t i = 0; i < nrows; ++i)
        if (mask[i]) hll_add(regs512, oracle_xxh64(data + offsets[i], offsets[i + 1] - offsets[i], 42));
}

/* 6-bit registers, 10 per 64-bit word (StatefulHyperloglogPlus.update word layout). */
void oracle_hll_pack(const uint8_t* regs512, int64_t* words52) {
    for (int w = 0; w < 52; ++w) {
        uint64_t word = 0;
        for (int k = 0; k < 10; ++k) {
            const int idx = w * 10 + k;
            if (idx < 512) word |= (uint64_t)(regs512[idx] & 63) << (6 * k);
        }
        words52[w] = (int64_t)word;
    }
}

static double estimate_bias(double e) {
    int lo = 0, hi = DQ_HLL_P9_N - 1, nearest = -1;
    while (lo <= hi) {            /* java.util.Arrays.binarySearch */
        const int mid = (lo + hi) >> 1;
        if (DQ_HLL_P9_RAW[mid] < e) lo = mid + 1;
        else if (DQ_HLL_P9_RAW[mid] > e) hi = mid - 1;
        else { nearest = mid; break; }
    }
    if (nearest < 0) nearest = lo;
    int low = nearest - 6 + 1;
    if (low < 0) low = 0;
    int high = low + 6;
    if (high > DQ_HLL_P9_N) high = DQ_HLL_P9_N;
    while (high < DQ_HLL_P9_N) {
        const double dh = e - DQ_HLL_P9_RAW[high], dl = e - DQ_HLL_P9_RAW[low];
        if (!(dh * dh < dl * dl)) break;
        ++low;
        ++high;
    }
    double s = 0.0;
    for (int i = low; i < high; ++i) s += DQ_HLL_P9_BIAS[i];
    return s / (high - low);
}

/* DeequHyperLogLogPlusPlusUtils.count, with Scala's Int shift `1 << Midx` (distance mod 32). */
double oracle_hll_count(const int64_t* words52) {
    const double M = 512.0;
    const double alphaM2 = (0.7213 / (1.0 + 1.079 / M)) * M * M;
    double zInverse = 0.0, V = 0.0;
    int idx = 0;
    for (int w = 0; w < 52; ++w) {
        for (int k = 0; k < 10 && idx < 512; ++k, ++idx) {
            const int m = (int)(((uint64_t)words52[w] >> (6 * k)) & 63);
            const int32_t p2 = (int32_t)(1u << (m & 31));
            zInverse += 1.0 / (double)p2;
            if (m == 0) V += 1.0;
        }
    }
    double est;
    const double e = alphaM2 / zInverse;
    const double corrected = e < 5.0 * M ? e - estimate_bias(e) : e;
    if (V > 0) {
        const double H = M * log(M / V);
        est = H <= DQ_HLL_P9_THRESHOLD ? H : corrected;
    } else {
        est = corrected;
    }
    return floor(est + 0.5);
}

/* ---- synthetic inputs (identical to deequ_amd/csrc/synth.hip) ------------------ */
uint64_t oracle_splitmix64(uint64_t seed, uint64_t i) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static double sum12(uint64_t seed, uint64_t row) {
    double s = 0.0;
    for (int j = 0; j < 12; ++j) {
        const uint64_t h = oracle_splitmix64(seed ^ (0xA5A5A5A5ULL * (uint64_t)(j + 1)), row);
        s = s + (double)(h >> 16) * 0x1.0p-48;
    }
    return s;
}

void oracle_synth_column(int kind, uint64_t seed, int64_t row0, int64_t n, void* out) {
    for (int64_t i = 0; i < n; ++i) {
        const uint64_t row = (uint64_t)(row0 + i);
        const uint64_t h = oracle_splitmix64(seed, row);
        switch (kind) {
            case 1: ((double*)out)[i] = (double)((int64_t)(h % 513ULL) - 256) * 0x1.0p-8; break;
            case 2: ((double*)out)[i] = (double)(h >> 11) * 0x1.0p-53; break;
            case 3: { volatile double t = sum12(seed, row) - 6.0; volatile double u = 15.0 * t;
                      ((double*)out)[i] = 100.0 + u; break; }
            case 4: ((int64_t*)out)[i] = (int64_t)(int32_t)(uint32_t)(h >> 32); break;
            case 5: ((int64_t*)out)[i] = (int64_t)(h & ((1ULL << 30) - 1)); break;
            case 6: ((double*)out)[i] = sum12(seed, row) - 6.0; break;
            case 7: { volatile double x = sum12(seed, row) - 6.0;
                      volatile double e = sum12(seed ^ 0x5A5A5A5A5A5A5A5AULL, row) - 6.0;
                      volatile double a = 0.6 * x; volatile double b = 0.8 * e;
                      ((double*)out)[i] = a + b; break; }
            default: break;
        }
    }
}

void oracle_synth_validity(uint64_t seed, int64_t row0, int64_t n, int permille, uint8_t* mask) {
    for (int64_t i = 0; i < n; ++i)
        mask[i] = (int)(oracle_splitmix64(seed, (uint64_t)(row0 + i)) % 1000ULL) >= permille;
}

/* ---- CPU baseline leg: the Spark-order per-row work only (count, sum, min, max, CentralMomentAgg)
 * over a fixed-width column with a validity mask; returns rows visited. Used by bench.py. -------- */
int64_t oracle_scan_spark(int spark_type, const void* values, const uint8_t* valid, int64_t nrows, double* out5) {
    const uint8_t* v = (const uint8_t*)values;
    const int es = elem_size(spark_type);
    const int frac = is_frac(spark_type);
    int64_t n = 0, isum = 0, imin = INT64_MAX, imax = INT64_MIN;
    double dsum = 0.0, dmin = NAN, dmax = NAN, wn = 0.0, wavg = 0.0, wm2 = 0.0;
    for (int64_t i = 0; i < nrows; ++i) {
        if (!valid[i]) continue;
        const uint8_t* p = v + i * es;
        const double x = as_f64(spark_type, p, 0);
        if (frac) {
            dsum += x;
            if (n == 0 || nan_gt(dmin, x)) dmin = x;
            if (n == 0 || nan_gt(x, dmax)) dmax = x;
        } else {
            const int64_t xi = as_i64(spark_type, p);
            isum = (int64_t)((uint64_t)isum + (uint64_t)xi);
            if (xi < imin) imin = xi;
            if (xi > imax) imax = xi;
        }
        ++n;
        const double n1 = wn + 1.0, delta = x - wavg, deltaN = delta / n1;
        wavg += deltaN;
        wm2 += delta * (delta - deltaN);
        wn = n1;
    }
    out5[0] = (double)n;
    out5[1] = frac ? dsum : (double)isum;
    out5[2] = frac ? dmin : (double)imin;
    out5[3] = frac ? dmax : (double)imax;
    out5[4] = wn > 0 ? sqrt(wm2 / wn) : NAN;
    return nrows;
}

/* Config-C4 frequency keys (same formula as deequ_amd/csrc/synth.hip). */
void oracle_synth_freq_keys(int64_t total, int64_t distinct, int64_t row0, int64_t n, int64_t* out) {
    const uint64_t half = (uint64_t)(distinct / 2 > 0 ? distinct / 2 : 1);
    for (int64_t i = 0; i < n; ++i) {
        const uint64_t r = (uint64_t)(row0 + i);
        const uint64_t j = (uint64_t)(((unsigned __int128)r * 0x9E3779B1ULL) % (uint64_t)total);
        const uint64_t k = j < (uint64_t)distinct ? j : (j - (uint64_t)distinct) % half;
        uint64_t z = k;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        out[i] = (int64_t)(z ^ (z >> 31));
    }
}

/* ---- streamed parity of the generated BASELINE workloads (C2 / suite10 / C3) -------------------
 * The columns are regenerated row by row from the counter-based generators above (never held in
 * memory), so 1e9-row configurations are checked in one pass over OpenMP threads. Everything the
 * reference computes exactly is exact here: counts, Long sums (wrap-around), min/max, Compliance
 * counts, HLL registers (XXH64 hashLong/hashInt, StatefulHyperloglogPlus.scala:89-112). Moments and
 * correlation are the EXACT values (shifted sums in long double with Kahan-Babuska compensation),
 * the yardstick the north star's 1e-12 tolerance is applied to; they restate what
 * CentralMomentAgg / Corr converge to (StandardDeviation.scala:37-44, Correlation.scala:37-52). */
typedef struct {
    int32_t kind;        /* synth kind (1..7) */
    int32_t spark_type;  /* T_DOUBLE or T_LONG */
    uint64_t seed;
    uint64_t vseed;      /* validity seed */
    int32_t permille;    /* P(null) in 1/1000; < 0: no validity bitmap */
    int32_t hll;         /* 1: HLL++ registers */
    int32_t pred_gt0;    /* 1: Compliance(col > 0) count */
    int32_t pad;
} oracle_gen_spec;

typedef struct {
    int64_t n, nnan, isum, imin, imax, pred_true;
    double dmin, dmax;
    double ex_sum, ex_mean, ex_m2;
    /* Spark's own arithmetic order: per partition a sequential Double sum and CentralMomentAgg update, the
     * partitions' states merged in partition order (Sum: +, StandardDeviationState.sum). The deviation of these
     * from ex_* is the reference's own error at this size. */
    double sp_sum, sp_mean, sp_m2;
    uint8_t regs[512];
} oracle_gen_col;

typedef struct {
    double n, x_avg, y_avg, ck, x_mk, y_mk;
} oracle_gen_corr;

typedef struct { long double s, c; } kbn;
static void kbn_add(kbn* a, long double x) {
    const long double t = a->s + x;
    if (fabsl(a->s) >= fabsl(x)) a->c += (a->s - t) + x;
    else a->c += (x - t) + a->s;
    a->s = t;
}
static long double kbn_val(const kbn* a) { return a->s + a->c; }

/* One generated value: its raw 8 bytes, and its value cast to (long) double as Spark casts it. */
static uint64_t synth_raw(int kind, uint64_t seed, uint64_t row) {
    uint64_t v;
    oracle_synth_column(kind, seed, (int64_t)row, 1, &v);
    return v;
}
static long double raw_value(int spark_type, uint64_t raw) {
    if (spark_type == T_DOUBLE) { double d; memcpy(&d, &raw, 8); return (long double)d; }
    return (long double)(double)(int64_t)raw;
}

/* XXH64.hashLong / hashInt of the canonical value (C/StatefulHyperloglogPlus.scala:93). */
static uint64_t hash_long(uint64_t v) {
    uint64_t h = 42 + XP5 + 8;
    h ^= rotl(v * XP2, 31) * XP1;
    h = rotl(h, 27) * XP1 + XP4;
    return avalanche(h);
}

typedef struct {
    int64_t n, nnan, isum, imin, imax, pred_true;
    double dmin, dmax;
    int first;
    kbn s1, s2, sum;
    uint8_t regs[512];
} gen_acc;

typedef struct { int64_t n; kbn sx, sy, sxx, syy, sxy; } corr_acc;

/* A `where` filter or Compliance predicate over the generated columns: leaves `column <op> constant` combined by
 * one AND or OR, in SQL three-valued logic (A/Analyzer.scala:409-432, A/Compliance.scala:49-52): a leaf over a NULL
 * value is NULL; AND is FALSE if any leaf is FALSE, else NULL if any is NULL; OR is TRUE if any leaf is TRUE, else
 * NULL if any is NULL. A DOUBLE column compares as double with Spark's NaN ordering (NaN = NaN, NaN above every
 * number); a LONG column compares as long against a long constant (is_dbl = 0) or as double (is_dbl = 1). */
typedef struct {
    int32_t col, op, is_dbl, pad;   /* op: 0 <, 1 <=, 2 =, 3 !=, 4 >, 5 >= */
    int64_t ci;
    double cd;
} oracle_gen_leaf;

typedef struct {
    int32_t nleaves;                /* 1..4 */
    int32_t comb;                   /* 0 AND, 1 OR */
    oracle_gen_leaf leaf[4];
} oracle_gen_pred;

/* -1 NULL, 0 FALSE, 1 TRUE */
static int gen_leaf(const oracle_gen_leaf* l, const oracle_gen_spec* specs, const int* valid, const uint64_t* raw) {
    if (!valid[l->col]) return -1;
    int c;
    if (specs[l->col].spark_type == T_DOUBLE || l->is_dbl) {
        double x;
        if (specs[l->col].spark_type == T_DOUBLE) memcpy(&x, &raw[l->col], 8);
        else x = (double)(int64_t)raw[l->col];
        const double y = l->cd;
        c = nan_gt(x, y) ? 1 : (nan_gt(y, x) ? -1 : 0);
    } else {
        const int64_t x = (int64_t)raw[l->col];
        c = x < l->ci ? -1 : (x > l->ci ? 1 : 0);
    }
    switch (l->op) {
        case 0: return c < 0;
        case 1: return c <= 0;
        case 2: return c == 0;
        case 3: return c != 0;
        case 4: return c > 0;
        default: return c >= 0;
    }
}

static int gen_pred(const oracle_gen_pred* p, const oracle_gen_spec* specs, const int* valid, const uint64_t* raw) {
    int any_null = 0;
    for (int i = 0; i < p->nleaves; ++i) {
        const int v = gen_leaf(&p->leaf[i], specs, valid, raw);
        if (v < 0) any_null = 1;
        else if (p->comb == 0 && v == 0) return 0;
        else if (p->comb == 1 && v == 1) return 1;
    }
    return any_null ? -1 : (p->comb == 0 ? 1 : 0);
}

/* where: NULL = no filter. where_counts[0..1] = rows with `where` TRUE / NOT NULL (Size(where) and the presence rule
 * of conditionalCount). Every column / pair aggregate runs over rows with `where` TRUE (conditionalSelection).
 * pred_counts[2 i + 0..1] = rows with `where` TRUE and predicate i TRUE / NOT NULL (Compliance numerator and its
 * presence). */
int oracle_generated_suite_ex(int ncols, const oracle_gen_spec* specs, int64_t row0, int64_t nrows, int npairs,
                              const int32_t* pairs, int threads, const oracle_gen_pred* where, int npreds,
                              const oracle_gen_pred* preds, oracle_gen_col* out, oracle_gen_corr* corr_out,
                              int64_t* where_counts, int64_t* pred_counts) {
    if (ncols <= 0 || ncols > 64 || nrows <= 0 || npreds < 0 || npreds > 16) return -1;
    if (where && (where->nleaves < 1 || where->nleaves > 4)) return -1;
    for (int i = 0; i < npreds; ++i)
        if (preds[i].nleaves < 1 || preds[i].nleaves > 4) return -1;
    long double shift[64];
    for (int c = 0; c < ncols; ++c) shift[c] = raw_value(specs[c].spark_type, synth_raw(specs[c].kind, specs[c].seed, (uint64_t)row0));
    gen_acc* acc = (gen_acc*)calloc((size_t)ncols, sizeof(gen_acc));
    corr_acc* cacc = (corr_acc*)calloc((size_t)(npairs > 0 ? npairs : 1), sizeof(corr_acc));
    if (!acc || !cacc) return -2;
    for (int c = 0; c < ncols; ++c) {
        acc[c].imin = INT64_MAX;
        acc[c].imax = INT64_MIN;
        acc[c].first = 1;
    }
    int64_t wt = 0, wnn = 0, pc[32];
    memset(pc, 0, sizeof(pc));
    /* kSparkParts contiguous row partitions (Spark's partitioning of a range scan); each is walked in row order */
    enum { kSparkParts = 64 };
    const int64_t psize = (nrows + kSparkParts - 1) / kSparkParts;
    typedef struct { double n, avg, m2, sum; } spark_acc;
    spark_acc* sacc = (spark_acc*)calloc((size_t)kSparkParts * (size_t)ncols, sizeof(spark_acc));
    if (!sacc) return -2;
    if (threads <= 0) threads = 1;
#pragma omp parallel num_threads(threads)
    {
        gen_acc* la = (gen_acc*)calloc((size_t)ncols, sizeof(gen_acc));
        corr_acc* lc = (corr_acc*)calloc((size_t)(npairs > 0 ? npairs : 1), sizeof(corr_acc));
        for (int c = 0; c < ncols; ++c) {
            la[c].imin = INT64_MAX;
            la[c].imax = INT64_MIN;
            la[c].first = 1;
        }
        double* x = (double*)malloc(sizeof(double) * (size_t)ncols);
        int* ok = (int*)malloc(sizeof(int) * (size_t)ncols);
        int* valid = (int*)malloc(sizeof(int) * (size_t)ncols);
        uint64_t* raw = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)ncols);
        int64_t lwt = 0, lwnn = 0, lpc[32];
        memset(lpc, 0, sizeof(lpc));
#pragma omp for schedule(dynamic, 1)
        for (int64_t k = 0; k < kSparkParts; ++k) {
            const int64_t lo = row0 + k * psize;
            int64_t hi = lo + psize;
            if (hi > row0 + nrows) hi = row0 + nrows;
            spark_acc* sa = sacc + k * ncols;
            for (int64_t r = lo; r < hi; ++r) {
                for (int c = 0; c < ncols; ++c) {
                    const oracle_gen_spec* sp = &specs[c];
                    valid[c] = sp->permille < 0 || (int)(oracle_splitmix64(sp->vseed, (uint64_t)r) % 1000ULL) >= sp->permille;
                    raw[c] = synth_raw(sp->kind, sp->seed, (uint64_t)r);
                }
                int sel = 1;
                if (where) {
                    const int w = gen_pred(where, specs, valid, raw);
                    sel = w == 1;
                    lwt += w == 1;
                    lwnn += w >= 0;
                } else {
                    ++lwt;
                    ++lwnn;
                }
                if (!sel) continue;
                for (int i = 0; i < npreds; ++i) {
                    const int v = gen_pred(&preds[i], specs, valid, raw);
                    lpc[2 * i] += v == 1;
                    lpc[2 * i + 1] += v >= 0;
                }
                for (int c = 0; c < ncols; ++c) {
                    const oracle_gen_spec* sp = &specs[c];
                    ok[c] = valid[c];
                    if (!ok[c]) continue;
                    double v;
                    memcpy(&v, &raw[c], 8);
                    gen_acc* a = &la[c];
                    a->n++;
                    if (sp->spark_type == T_DOUBLE) {
                        if (v != v) a->nnan++;
                        if (a->first || nan_gt(a->dmin, v)) a->dmin = v;
                        if (a->first || nan_gt(v, a->dmax)) a->dmax = v;
                        kbn_add(&a->sum, (long double)v);
                        if (sp->pred_gt0 && (v > 0.0 || v != v)) a->pred_true++;
                        if (sp->hll) hll_add(a->regs, hash_long(v == v ? raw[c] : 0x7ff8000000000000ULL));
                        x[c] = v;
                    } else {
                        const int64_t iv = (int64_t)raw[c];
                        a->isum = (int64_t)((uint64_t)a->isum + (uint64_t)iv);
                        if (iv < a->imin) a->imin = iv;
                        if (iv > a->imax) a->imax = iv;
                        if (sp->pred_gt0 && iv > 0) a->pred_true++;
                        if (sp->hll) hll_add(a->regs, hash_long((uint64_t)iv));
                        x[c] = (double)iv;
                    }
                    a->first = 0;
                    {   /* Spark order inside the partition: Sum, CentralMomentAgg.update (C/StatefulStdDevPop.scala) */
                        spark_acc* q = &sa[c];
                        if (sp->spark_type == T_DOUBLE) q->sum += x[c];
                        const double n1 = q->n + 1.0, delta = x[c] - q->avg, deltaN = delta / n1;
                        q->avg += deltaN;
                        q->m2 += delta * (delta - deltaN);
                        q->n = n1;
                    }
                    const long double d = (long double)x[c] - shift[c];
                    kbn_add(&a->s1, d);
                    kbn_add(&a->s2, d * d);
                }
                for (int p = 0; p < npairs; ++p) {
                    const int cx = pairs[2 * p], cy = pairs[2 * p + 1];
                    if (!ok[cx] || !ok[cy]) continue;
                    const long double kx = shift[cx], ky = shift[cy];
                    const long double dx = (long double)x[cx] - kx, dy = (long double)x[cy] - ky;
                    corr_acc* q = &lc[p];
                    q->n++;
                    kbn_add(&q->sx, dx);
                    kbn_add(&q->sy, dy);
                    kbn_add(&q->sxx, dx * dx);
                    kbn_add(&q->syy, dy * dy);
                    kbn_add(&q->sxy, dx * dy);
                }
            }
        }
#pragma omp critical
        {
            wt += lwt;
            wnn += lwnn;
            for (int i = 0; i < 2 * npreds; ++i) pc[i] += lpc[i];
            for (int c = 0; c < ncols; ++c) {
                gen_acc* a = &acc[c];
                const gen_acc* b = &la[c];
                if (b->n == 0) continue;
                a->n += b->n;
                a->nnan += b->nnan;
                a->pred_true += b->pred_true;
                a->isum = (int64_t)((uint64_t)a->isum + (uint64_t)b->isum);
                if (b->imin < a->imin) a->imin = b->imin;
                if (b->imax > a->imax) a->imax = b->imax;
                if (a->first || nan_gt(a->dmin, b->dmin)) a->dmin = b->dmin;
                if (a->first || nan_gt(b->dmax, a->dmax)) a->dmax = b->dmax;
                a->first = 0;
                kbn_add(&a->s1, kbn_val(&b->s1));
                kbn_add(&a->s2, kbn_val(&b->s2));
                kbn_add(&a->sum, kbn_val(&b->sum));
                for (int i = 0; i < 512; ++i)
                    if (b->regs[i] > a->regs[i]) a->regs[i] = b->regs[i];
            }
            for (int p = 0; p < npairs; ++p) {
                cacc[p].n += lc[p].n;
                kbn_add(&cacc[p].sx, kbn_val(&lc[p].sx));
                kbn_add(&cacc[p].sy, kbn_val(&lc[p].sy));
                kbn_add(&cacc[p].sxx, kbn_val(&lc[p].sxx));
                kbn_add(&cacc[p].syy, kbn_val(&lc[p].syy));
                kbn_add(&cacc[p].sxy, kbn_val(&lc[p].sxy));
            }
        }
        free(la);
        free(lc);
        free(x);
        free(ok);
        free(valid);
        free(raw);
    }
    if (where_counts) {
        where_counts[0] = wt;
        where_counts[1] = wnn;
    }
    for (int i = 0; i < 2 * npreds && pred_counts; ++i) pred_counts[i] = pc[i];
    for (int c = 0; c < ncols; ++c) {
        const gen_acc* a = &acc[c];
        oracle_gen_col* o = &out[c];
        memset(o, 0, sizeof(*o));
        o->n = a->n;
        o->nnan = a->nnan;
        o->isum = a->isum;
        o->imin = a->imin;
        o->imax = a->imax;
        o->pred_true = a->pred_true;
        o->dmin = a->n ? a->dmin : NAN;
        o->dmax = a->n ? a->dmax : NAN;
        memcpy(o->regs, a->regs, 512);
        {   /* partitions merged in order: Double +, StandardDeviationState.sum (A/StandardDeviation.scala:37-44) */
            double n = 0.0, avg = 0.0, m2 = 0.0, sum = 0.0;
            for (int k = 0; k < kSparkParts; ++k) {
                const spark_acc* q = &sacc[k * ncols + c];
                sum += q->sum;
                if (q->n == 0.0) continue;
                const double nn = n + q->n, delta = q->avg - avg, deltaN = nn == 0.0 ? 0.0 : delta / nn;
                m2 = m2 + q->m2 + delta * deltaN * n * q->n;
                avg = avg + deltaN * q->n;
                n = nn;
            }
            o->sp_sum = specs[c].spark_type == T_DOUBLE ? sum : (double)a->isum;
            o->sp_mean = avg;
            o->sp_m2 = m2;
        }
        if (a->n > 0) {
            const long double k = shift[c];
            const long double n = (long double)a->n, s1 = kbn_val(&a->s1), s2 = kbn_val(&a->s2);
            o->ex_sum = specs[c].spark_type == T_DOUBLE ? (double)kbn_val(&a->sum) : (double)(k * n + s1);
            o->ex_mean = (double)(k + s1 / n);
            o->ex_m2 = (double)(s2 - s1 * s1 / n);
        }
    }
    for (int p = 0; p < npairs; ++p) {
        const corr_acc* q = &cacc[p];
        oracle_gen_corr* o = &corr_out[p];
        memset(o, 0, sizeof(*o));
        o->n = (double)q->n;
        if (q->n == 0) continue;
        const int cx = pairs[2 * p], cy = pairs[2 * p + 1];
        const long double kx = shift[cx], ky = shift[cy];
        const long double n = (long double)q->n;
        const long double sx = kbn_val(&q->sx), sy = kbn_val(&q->sy);
        o->x_avg = (double)(kx + sx / n);
        o->y_avg = (double)(ky + sy / n);
        o->ck = (double)(kbn_val(&q->sxy) - sx * sy / n);
        o->x_mk = (double)(kbn_val(&q->sxx) - sx * sx / n);
        o->y_mk = (double)(kbn_val(&q->syy) - sy * sy / n);
    }
    free(acc);
    free(cacc);
    free(sacc);
    return 0;
}

int oracle_generated_suite(int ncols, const oracle_gen_spec* specs, int64_t row0, int64_t nrows, int npairs,
                           const int32_t* pairs, int threads, oracle_gen_col* out, oracle_gen_corr* corr_out) {
    return oracle_generated_suite_ex(ncols, specs, row0, nrows, npairs, pairs, threads, NULL, 0, NULL, out, corr_out,
                                     NULL, NULL);
}

/* ---- CPU baseline legs of bench.py (restated per-row work of the reference, timed on the host) ----------------
 * suite10: one column's Spark-order row loop for every op of the north-star suite on it: count, Sum (Long wrap /
 * Double), NaN-largest Min / Max, CentralMomentAgg update, Compliance(col > 0) and the HLL++ register update
 * (XXH64 hashLong of the value, StatefulHyperloglogPlus.update); pairs add the Spark Corr update. Returns rows. */
int64_t oracle_scan_suite10_col(int spark_type, const void* values, const uint8_t* valid, int64_t nrows,
                                uint8_t* regs512, double* out6) {
    const uint8_t* v = (const uint8_t*)values;
    const int frac = spark_type == T_DOUBLE;
    int64_t n = 0, isum = 0, imin = INT64_MAX, imax = INT64_MIN, pt = 0;
    double dsum = 0.0, dmin = NAN, dmax = NAN, wn = 0.0, wavg = 0.0, wm2 = 0.0;
    for (int64_t i = 0; i < nrows; ++i) {
        if (!valid[i]) continue;
        uint64_t raw;
        memcpy(&raw, v + 8 * i, 8);
        double x;
        if (frac) {
            memcpy(&x, &raw, 8);
            dsum += x;
            if (n == 0 || nan_gt(dmin, x)) dmin = x;
            if (n == 0 || nan_gt(x, dmax)) dmax = x;
            pt += (x > 0.0 || x != x);
            hll_add(regs512, hash_long(x == x ? raw : 0x7ff8000000000000ULL));
        } else {
            const int64_t xi = (int64_t)raw;
            x = (double)xi;
            isum = (int64_t)((uint64_t)isum + (uint64_t)xi);
            if (xi < imin) imin = xi;
            if (xi > imax) imax = xi;
            pt += xi > 0;
            hll_add(regs512, hash_long(raw));
        }
        ++n;
        const double n1 = wn + 1.0, delta = x - wavg, deltaN = delta / n1;
        wavg += deltaN;
        wm2 += delta * (delta - deltaN);
        wn = n1;
    }
    out6[0] = (double)n;
    out6[1] = frac ? dsum : (double)isum;
    out6[2] = frac ? dmin : (double)imin;
    out6[3] = frac ? dmax : (double)imax;
    out6[4] = wn > 0 ? sqrt(wm2 / wn) : NAN;
    out6[5] = (double)pt;
    return nrows;
}

int64_t oracle_corr_spark(int tx, const void* xv, const uint8_t* vx, int ty, const void* yv, const uint8_t* vy,
                          int64_t nrows, double* out6) {
    const uint8_t* xp = (const uint8_t*)xv;
    const uint8_t* yp = (const uint8_t*)yv;
    double n = 0, xa = 0, ya = 0, ck = 0, xm = 0, ym = 0;
    for (int64_t i = 0; i < nrows; ++i) {
        if (!vx[i] || !vy[i]) continue;
        const double x = as_f64(tx, xp + 8 * i, 0), y = as_f64(ty, yp + 8 * i, 0);
        const double n1 = n + 1.0, dx = x - xa, dy = y - ya;
        xa += dx / n1;
        ya += dy / n1;
        ck += dx * (y - ya);
        xm += dx * (x - xa);
        ym += dy * (y - ya);
        n = n1;
    }
    out6[0] = n; out6[1] = xa; out6[2] = ya; out6[3] = ck; out6[4] = xm; out6[5] = ym;
    return nrows;
}

/* C4: the grouping hash aggregate (count(*) GROUP BY key) as a single-threaded open-addressing table over the
 * canonical 64-bit keys (Spark's HashAggregate per partition); returns the number of groups. table: cap slots of
 * (key, count) pairs, cap a power of two larger than the distinct keys; used marks occupied slots. */
int64_t oracle_count_keys(const int64_t* keys, int64_t n, int64_t* table, uint8_t* used, int64_t cap) {
    memset(used, 0, (size_t)cap);
    int64_t groups = 0;
    const uint64_t mask = (uint64_t)cap - 1;
    for (int64_t i = 0; i < n; ++i) {
        uint64_t z = (uint64_t)keys[i];
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        uint64_t p = (z ^ (z >> 31)) & mask;
        for (;;) {
            if (!used[p]) {
                used[p] = 1;
                table[2 * p] = keys[i];
                table[2 * p + 1] = 1;
                ++groups;
                break;
            }
            if (table[2 * p] == keys[i]) {
                ++table[2 * p + 1];
                break;
            }
            p = (p + 1) & mask;
        }
    }
    return groups;
}

/* count(*) GROUP BY one fixed-width key column, the grouping step of FrequencyBasedAnalyzer.computeFrequencies
 * (analyzers/GroupingAnalyzers.scala:53-79: `data.select(cols).where(atLeastOne non-null).groupBy(cols).count()`)
 * for a single column, restated as a sort + run length over the canonical 64-bit keys: integral values
 * sign-extended, FLOAT / DOUBLE bit patterns with every NaN mapped to Java's canonical NaN and -0.0 kept apart
 * from 0.0 — Spark 2.2 groups rows on the binary UnsafeRow of the key (there is no NormalizeFloatingNumbers rule
 * before Spark 3.0), whose float cells are written through floatToIntBits / doubleToLongBits: NaN is canonical,
 * -0.0 is not. NULL rows are not grouped
 * (their count is returned in *null_rows). `valid`: LSB-first bitmap, NULL = every row valid. On return keys[0..g)
 * holds the distinct canonical keys in ascending unsigned order and counts[0..g) their Long counts; the return
 * value is g. keys / counts must hold n entries; scratch is n 64-bit words. */
int64_t oracle_group_counts(int spark_type, const void* values, const uint8_t* valid, int64_t n, int64_t* keys,
                            int64_t* counts, uint64_t* scratch, int64_t* null_rows) {
    const uint8_t* v = (const uint8_t*)values;
    const int w = elem_size(spark_type);
    uint64_t* a = (uint64_t*)keys;
    int64_t m = 0, nulls = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (valid && !((valid[i >> 3] >> (i & 7)) & 1)) {
            ++nulls;
            continue;
        }
        const uint8_t* p = v + i * w;
        uint64_t k;
        if (spark_type == T_DOUBLE) {
            double d;
            memcpy(&d, p, 8);
            if (d != d) k = 0x7ff8000000000000ULL; else memcpy(&k, p, 8);
        } else if (spark_type == T_FLOAT) {
            float f;
            uint32_t u;
            memcpy(&f, p, 4);
            if (f != f) u = 0x7fc00000u; else memcpy(&u, p, 4);
            k = u;
        } else {
            k = (uint64_t)as_i64(spark_type, p);
        }
        a[m++] = k;
    }
    *null_rows = nulls;
    /* LSD radix sort, 16-bit digits; a digit every key shares is skipped */
    uint64_t* src = a;
    uint64_t* dst = scratch;
    static int64_t hist[65536];
    for (int shift = 0; shift < 64; shift += 16) {
        memset(hist, 0, sizeof(hist));
        for (int64_t i = 0; i < m; ++i) hist[(src[i] >> shift) & 0xFFFF]++;
        int single = 0;
        for (int d = 0; d < 65536; ++d)
            if (hist[d] == m) single = 1;
        if (single) continue;
        int64_t at = 0;
        for (int d = 0; d < 65536; ++d) {
            const int64_t c = hist[d];
            hist[d] = at;
            at += c;
        }
        for (int64_t i = 0; i < m; ++i) dst[hist[(src[i] >> shift) & 0xFFFF]++] = src[i];
        uint64_t* t = src;
        src = dst;
        dst = t;
    }
    if (src != a) memcpy(a, src, (size_t)m * 8);
    int64_t g = 0;
    for (int64_t i = 0; i < m;) {
        int64_t j = i + 1;
        while (j < m && a[j] == a[i]) ++j;
        a[g] = a[i];
        counts[g] = j - i;
        ++g;
        i = j;
    }
    return g;
}

/* count(*) GROUP BY one UTF-8 string key column given as row-range parts (the row chunks of a ChunkedTable, each with
 * its own int32 Arrow offsets, bytes and LSB-first validity bitmap), the grouping step of
 * FrequencyBasedAnalyzer.computeFrequencies (A/GroupingAnalyzers.scala:53-79) for a string key: groups are equal
 * BYTE STRINGS. No fingerprint decides equality: every key of <= 23 bytes is packed with its length into a 24-byte
 * record, the records are distributed over 65536 buckets (a hash of the record picks the bucket -- placement only),
 * each bucket is sorted (qsort over the three words) and run-length counted. A key longer than 23 bytes makes the
 * call return -2 (the C5 text columns hold 1-20 bytes).
 * Out: *valid_rows / *null_rows; the distinct group counts cc_vals[0..*ncc) with their multiplicities cc_mult (the
 * "counts of counts": num_groups = sum(cc_mult), unique = cc_mult at 1, the entropy terms per distinct count); for
 * each of the nq query keys (int64 offsets into q_bytes) its exact count (0 when absent) in q_counts. Returns the
 * number of groups, -1 on allocation failure, -2 on a key past 23 bytes, -3 when *ncc is too small. */
typedef struct { uint64_t w[3]; } skey_t;

static int skey_cmp(const void* a, const void* b) {
    const skey_t* x = (const skey_t*)a;
    const skey_t* y = (const skey_t*)b;
    for (int i = 0; i < 3; ++i)
        if (x->w[i] != y->w[i]) return x->w[i] < y->w[i] ? -1 : 1;
    return 0;
}

static int skey_pack(const uint8_t* p, int64_t len, skey_t* k) {
    if (len < 0 || len > 23) return 0;
    uint8_t b[24];
    memset(b, 0, sizeof(b));
    memcpy(b, p, (size_t)len);
    b[23] = (uint8_t)len;
    memcpy(k->w, b, 24);
    return 1;
}

static uint32_t skey_bucket(const skey_t* k) {
    uint64_t h = k->w[0] * 0x9E3779B97F4A7C15ULL ^ k->w[1] * 0xC2B2AE3D27D4EB4FULL ^ k->w[2] * 0x165667B19E3779F9ULL;
    h ^= h >> 31;
    h *= 0xBF58476D1CE4E5B9ULL;
    h ^= h >> 29;
    return (uint32_t)(h >> 48);
}

int64_t oracle_group_strings(int nparts, const uint8_t* const* bytes, const int32_t* const* offsets,
                             const uint8_t* const* valid, const int64_t* rows, int64_t* valid_rows, int64_t* null_rows,
                             int64_t* cc_vals, int64_t* cc_mult, int64_t* ncc, const uint8_t* q_bytes,
                             const int64_t* q_offsets, int64_t nq, int64_t* q_counts) {
    enum { NB = 65536, SMALL = 4096 };
    int64_t n = 0;
    for (int p = 0; p < nparts; ++p) n += rows[p];
    uint16_t* bk = (uint16_t*)malloc((size_t)(n ? n : 1) * sizeof(uint16_t));
    int nt = 1;
#pragma omp parallel
#pragma omp single
    nt = omp_get_num_threads();
    int64_t* th_hist = (int64_t*)calloc((size_t)nt * NB, sizeof(int64_t));
    int64_t* bstart = (int64_t*)malloc((NB + 1) * sizeof(int64_t));
    int64_t* th_nulls = (int64_t*)calloc((size_t)nt, sizeof(int64_t));
    int bad = 0;
    if (!bk || !th_hist || !bstart || !th_nulls) {
        free(bk); free(th_hist); free(bstart); free(th_nulls);
        return -1;
    }
    /* pass A: each row's bucket (0xFFFF + NULL flag kept apart: a NULL row is marked by its validity bit) */
#pragma omp parallel num_threads(nt) reduction(| : bad)
    {
        const int t = omp_get_thread_num();
        int64_t* hist = th_hist + (size_t)t * NB;
        int64_t base = 0;
        for (int p = 0; p < nparts; ++p) {
            const int64_t lo = rows[p] * t / nt, hi = rows[p] * (t + 1) / nt;
            for (int64_t i = lo; i < hi; ++i) {
                if (valid[p] && !((valid[p][i >> 3] >> (i & 7)) & 1)) {
                    th_nulls[t]++;
                    continue;
                }
                skey_t k;
                if (!skey_pack(bytes[p] + offsets[p][i], (int64_t)offsets[p][i + 1] - offsets[p][i], &k)) {
                    bad = 1;
                    continue;
                }
                const uint32_t b = skey_bucket(&k);
                bk[base + i] = (uint16_t)b;
                hist[b]++;
            }
            base += rows[p];
        }
    }
    if (bad) {
        free(bk); free(th_hist); free(bstart); free(th_nulls);
        return -2;
    }
    int64_t nulls = 0;
    for (int t = 0; t < nt; ++t) nulls += th_nulls[t];
    const int64_t m = n - nulls;
    /* bucket starts, and each thread's write cursor per bucket (thread order inside a bucket) */
    int64_t at = 0;
    for (int b = 0; b < NB; ++b) {
        bstart[b] = at;
        for (int t = 0; t < nt; ++t) {
            const int64_t c = th_hist[(size_t)t * NB + b];
            th_hist[(size_t)t * NB + b] = at;
            at += c;
        }
    }
    bstart[NB] = at;
    skey_t* rec = (skey_t*)malloc((size_t)(m ? m : 1) * sizeof(skey_t));
    if (!rec) {
        free(bk); free(th_hist); free(bstart); free(th_nulls);
        return -1;
    }
    /* pass B: the records into their buckets */
#pragma omp parallel num_threads(nt)
    {
        const int t = omp_get_thread_num();
        int64_t* cur = th_hist + (size_t)t * NB;
        int64_t base = 0;
        for (int p = 0; p < nparts; ++p) {
            const int64_t lo = rows[p] * t / nt, hi = rows[p] * (t + 1) / nt;
            for (int64_t i = lo; i < hi; ++i) {
                if (valid[p] && !((valid[p][i >> 3] >> (i & 7)) & 1)) continue;
                skey_t k;
                skey_pack(bytes[p] + offsets[p][i], (int64_t)offsets[p][i + 1] - offsets[p][i], &k);
                rec[cur[bk[base + i]]++] = k;
            }
            base += rows[p];
        }
    }
    free(bk);
    /* sort every bucket, run-length count, counts of counts per thread (small counts in an array, the rest listed) */
    int64_t* small = (int64_t*)calloc((size_t)nt * SMALL, sizeof(int64_t));
    int64_t** big = (int64_t**)calloc((size_t)nt, sizeof(int64_t*));
    int64_t* nbig = (int64_t*)calloc((size_t)nt, sizeof(int64_t));
    int64_t* capbig = (int64_t*)calloc((size_t)nt, sizeof(int64_t));
    int64_t groups = 0;
    int oom = 0;
#pragma omp parallel num_threads(nt) reduction(+ : groups) reduction(| : oom)
    {
        const int t = omp_get_thread_num();
        int64_t* sm = small + (size_t)t * SMALL;
#pragma omp for schedule(dynamic, 64)
        for (int b = 0; b < NB; ++b) {
            skey_t* r = rec + bstart[b];
            const int64_t c = bstart[b + 1] - bstart[b];
            int64_t same = 1;
            while (same < c && skey_cmp(&r[same], &r[0]) == 0) ++same;
            if (same < c) qsort(r, (size_t)c, sizeof(skey_t), skey_cmp);
            for (int64_t i = 0; i < c;) {
                int64_t j = i + 1;
                while (j < c && skey_cmp(&r[j], &r[i]) == 0) ++j;
                const int64_t cnt = j - i;
                ++groups;
                if (cnt < SMALL) {
                    sm[cnt]++;
                } else {
                    if (nbig[t] == capbig[t]) {
                        capbig[t] = capbig[t] ? 2 * capbig[t] : 64;
                        int64_t* nb = (int64_t*)realloc(big[t], (size_t)capbig[t] * sizeof(int64_t));
                        if (!nb) { oom = 1; break; }
                        big[t] = nb;
                    }
                    big[t][nbig[t]++] = cnt;
                }
                i = j;
            }
        }
    }
    int64_t rc = oom ? -1 : groups;
    if (!oom) {
        /* counts of counts: merge the threads' small arrays, sort the big counts */
        int64_t k = 0;
        for (int64_t c = 1; c < SMALL && rc >= 0; ++c) {
            int64_t mult = 0;
            for (int t = 0; t < nt; ++t) mult += small[(size_t)t * SMALL + c];
            if (!mult) continue;
            if (k >= *ncc) { rc = -3; break; }
            cc_vals[k] = c;
            cc_mult[k++] = mult;
        }
        int64_t tot = 0;
        for (int t = 0; t < nt; ++t) tot += nbig[t];
        int64_t* all = (int64_t*)malloc((size_t)(tot ? tot : 1) * sizeof(int64_t));
        if (!all) rc = -1;
        if (rc >= 0) {
            int64_t a = 0;
            for (int t = 0; t < nt; ++t) for (int64_t i = 0; i < nbig[t]; ++i) all[a++] = big[t][i];
            for (int64_t i = 1; i < tot; ++i) {  /* insertion sort: few large counts */
                const int64_t v = all[i];
                int64_t j = i - 1;
                while (j >= 0 && all[j] > v) { all[j + 1] = all[j]; --j; }
                all[j + 1] = v;
            }
            for (int64_t i = 0; i < tot && rc >= 0;) {
                int64_t j = i + 1;
                while (j < tot && all[j] == all[i]) ++j;
                if (k >= *ncc) { rc = -3; break; }
                cc_vals[k] = all[i];
                cc_mult[k++] = j - i;
                i = j;
            }
        }
        free(all);
        *ncc = k;
    }
    /* the query keys: binary search in their bucket */
    for (int64_t q = 0; q < nq && rc >= 0; ++q) {
        skey_t k;
        q_counts[q] = 0;
        if (!skey_pack(q_bytes + q_offsets[q], q_offsets[q + 1] - q_offsets[q], &k)) continue;
        const uint32_t b = skey_bucket(&k);
        const skey_t* r = rec + bstart[b];
        int64_t lo = 0, hi = bstart[b + 1] - bstart[b];
        while (lo < hi) {  /* first record >= k */
            const int64_t mid = (lo + hi) / 2;
            if (skey_cmp(&r[mid], &k) < 0) lo = mid + 1; else hi = mid;
        }
        int64_t j = lo;
        while (j < bstart[b + 1] - bstart[b] && skey_cmp(&r[j], &k) == 0) ++j;
        q_counts[q] = j - lo;
    }
    *valid_rows = m;
    *null_rows = nulls;
    for (int t = 0; t < nt; ++t) free(big[t]);
    free(big); free(nbig); free(capbig); free(small); free(rec); free(th_hist); free(bstart); free(th_nulls);
    return rc;
}
