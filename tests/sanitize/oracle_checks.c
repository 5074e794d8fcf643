/* The CPU oracle (oracle/dq_oracle.c) under AddressSanitizer + UBSan: every entry point on exactly-sized heap
 * buffers (random values, NaN / +-inf / -0.0, nulls, empty inputs, ragged strings). Exit 0 = no report. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct { int64_t n, isum; double dsum; int64_t imin, imax; double dmin, dmax, w_n, w_avg, w_m2, ex_mean, ex_m2; } oc_col;
typedef struct { double n, x_avg, y_avg, ck, x_mk, y_mk, ex_ck, ex_x_mk, ex_y_mk; } oc_corr;
typedef struct { int32_t kind, spark_type; uint64_t seed, vseed; int32_t permille, hll, pred_gt0, pad; } oc_spec;
typedef struct { int64_t n, nnan, isum, imin, imax, pred_true; double dmin, dmax, ex_sum, ex_mean, ex_m2, sp_sum, sp_mean, sp_m2; uint8_t regs[512]; } oc_gcol;
typedef struct { double n, x_avg, y_avg, ck, x_mk, y_mk; } oc_gcorr;
typedef struct { int32_t col, op, is_dbl, pad; int64_t ci; double cd; } oc_leaf;
typedef struct { int32_t nleaves, comb; oc_leaf leaf[4]; } oc_pred;

uint64_t oracle_xxh64(const uint8_t* p, int64_t len, uint64_t seed);
uint64_t oracle_spark_hash(int spark_type, const void* v);
void oracle_column(int spark_type, int decimal_scale, const void* values, const uint8_t* mask, int64_t nrows, oc_col* out);
void oracle_correlation(int tx, int sx, const void* xv, int ty, int sy, const void* yv, const uint8_t* mask,
                        int64_t nrows, oc_corr* out);
void oracle_hll_fixed(int spark_type, const void* values, const uint8_t* mask, int64_t nrows, uint8_t* regs512);
void oracle_hll_strings(const uint8_t* data, const int32_t* offsets, const uint8_t* mask, int64_t nrows, uint8_t* regs512);
void oracle_hll_pack(const uint8_t* regs512, int64_t* words52);
double oracle_hll_count(const int64_t* words52);
int64_t oracle_scan_spark(int spark_type, const void* values, const uint8_t* valid, int64_t nrows, double* out5);
void oracle_synth_column(int kind, uint64_t seed, int64_t row0, int64_t n, void* out);
void oracle_synth_validity(uint64_t seed, int64_t row0, int64_t n, int permille, uint8_t* mask);
void oracle_synth_freq_keys(int64_t total, int64_t distinct, int64_t row0, int64_t n, int64_t* out);
int oracle_generated_suite_ex(int ncols, const oc_spec* specs, int64_t row0, int64_t nrows, int npairs,
                              const int32_t* pairs, int threads, const oc_pred* where, int npreds, const oc_pred* preds,
                              oc_gcol* out, oc_gcorr* corr_out, int64_t* where_counts, int64_t* pred_counts);

static uint64_t st = 88172645463325252ULL;
static uint64_t rnd(void) { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; }
static double rdbl(void) {
    switch (rnd() % 8) { case 0: return NAN; case 1: return -0.0; case 2: return INFINITY; case 3: return -INFINITY; default: return (double)(int64_t)(rnd() >> 11) * 1e-9; }
}

int main(void) {
    const int types[] = {1, 2, 3, 4, 5, 6, 7, 9, 10, 11};
    const int widths[] = {1, 1, 2, 4, 8, 4, 8, 4, 8, 8};
    for (int it = 0; it < 3000; ++it) {
        const int64_t n = (int64_t)(rnd() % 300);
        const int ti = (int)(rnd() % 10), t = types[ti], w = widths[ti];
        uint8_t* vals = malloc(n * w + 1);
        uint8_t* mask = malloc(n + 1);
        for (int64_t i = 0; i < n; ++i) {
            if (t == 7) { double d = rdbl(); memcpy(vals + i * 8, &d, 8); }
            else if (t == 6) { float f = (float)rdbl(); memcpy(vals + i * 4, &f, 4); }
            else for (int b = 0; b < w; ++b) vals[i * w + b] = (uint8_t)rnd();
            mask[i] = rnd() % 4 != 0;
        }
        oc_col c;
        oracle_column(t, t == 11 ? 2 : 0, vals, mask, n, &c);
        uint8_t regs[512] = {0};
        oracle_hll_fixed(t, vals, mask, n, regs);
        int64_t words[52];
        oracle_hll_pack(regs, words);
        (void)oracle_hll_count(words);
        for (int64_t i = 0; i < n; ++i) (void)oracle_spark_hash(t, vals + i * w);
        if (t == 7 || t == 5) {
            double o5[5];
            (void)oracle_scan_spark(t, vals, mask, n, o5);
            oc_corr cr;
            oracle_correlation(t, 0, vals, t, 0, vals, mask, n, &cr);
        }
        free(vals);
        free(mask);
    }
    for (int it = 0; it < 500; ++it) {  /* ragged strings */
        const int64_t n = (int64_t)(rnd() % 100);
        int32_t* offs = malloc(sizeof(int32_t) * (n + 1));
        offs[0] = 0;
        for (int64_t i = 0; i < n; ++i) offs[i + 1] = offs[i] + (int32_t)(rnd() % 70);
        uint8_t* data = malloc(offs[n] + 1);
        for (int32_t i = 0; i < offs[n]; ++i) data[i] = (uint8_t)rnd();
        uint8_t* mask = malloc(n + 1);
        for (int64_t i = 0; i < n; ++i) mask[i] = rnd() % 3 != 0;
        uint8_t regs[512] = {0};
        oracle_hll_strings(data, offs, mask, n, regs);
        for (int64_t i = 0; i < n; ++i) (void)oracle_xxh64(data + offs[i], offs[i + 1] - offs[i], 42);
        free(offs);
        free(data);
        free(mask);
    }
    {   /* generators and the streamed suite (with a compound where and a Compliance predicate) */
        double* d = malloc(sizeof(double) * 1000);
        int64_t* k = malloc(sizeof(int64_t) * 1000);
        uint8_t* m = malloc(1000);
        for (int kind = 1; kind <= 7; ++kind) oracle_synth_column(kind, 7, 3, 1000, kind == 4 || kind == 5 ? (void*)k : (void*)d);
        oracle_synth_validity(9, 0, 1000, 10, m);
        oracle_synth_freq_keys(1000, 100, 0, 1000, k);
        oc_spec sp[3] = {{1, 7, 1, 2, 10, 1, 1, 0}, {4, 5, 3, 4, 10, 1, 1, 0}, {3, 7, 5, 6, -1, 0, 0, 0}};
        int32_t pairs[2] = {0, 2};
        oc_pred where = {2, 1, {{0, 0, 1, 0, 0, 0.0}, {1, 4, 0, 0, 5, 5.0}}};
        oc_pred pr = {1, 0, {{2, 5, 1, 0, 0, 100.0}}};
        oc_gcol out[3];
        oc_gcorr co[1];
        int64_t wc[2], pc[2];
        if (oracle_generated_suite_ex(3, sp, 11, 70001, 1, pairs, 2, &where, 1, &pr, out, co, wc, pc) != 0) return 1;
        if (oracle_generated_suite_ex(3, sp, 0, 5, 1, pairs, 1, NULL, 0, NULL, out, co, NULL, NULL) != 0) return 1;
        free(d);
        free(k);
        free(m);
    }
    printf("oracle_checks: ok\n");
    return 0;
}
