// cast.hip — Spark Cast of a column to LONG / DOUBLE on gfx950 (one lane per row).
//
// Replaces ColumnProfiler.castColumn (M/profiles/ColumnProfiler.scala:346-355, called from
// castNumericStringColumns :427-445 for columns whose DataType pass inferred Integral / Fractional):
// `data(name).cast(LongType | DoubleType)`. The parsers are the device restatements in dq_parse.h;
// NULL rows and strings that do not parse become NULL. HBM-bound byte work: the offsets and bytes are
// read once, 8 B of value + 1 bit of validity written per row; validity words are assembled with a
// wave ballot (64 rows per wave = one 64-bit word, LSB-first).
#include <hip/hip_runtime.h>

#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <thread>
#include <vector>

#include "dq_common.h"
#include "dq_internal.h"
#include "dq_parse.h"

namespace dq {

constexpr int kCastBlock = 256;

// Numeric sources: element kind + decimal scale (Spark Decimal, compact form: value = unscaled / 10^scale).
struct CastSource {
    const void* values;
    const uint8_t* bytes;      // STRING
    const int32_t* offsets;    // STRING
    const uint64_t* validity;
    int32_t elem;              // ET_* (ET_NONE for STRING)
    int32_t decimal_scale;
    int64_t pow10;             // 10^scale
};

// java (long) of a double: NaN -> 0, saturating (Scala Double.toLong, Spark 2.2 Cast double -> long).
__device__ __forceinline__ int64_t java_d2l(double d) {
    if (d != d) return 0;
    if (d >= 9223372036854775807.0) return INT64_MAX;
    if (d <= -9223372036854775808.0) return INT64_MIN;
    return (int64_t)d;
}

// Bytes of one wave's 64 consecutive strings staged in LDS by coalesced dword loads (the parsers then read LDS, not
// scattered HBM bytes); a longer range is parsed from HBM directly.
constexpr int kCastStageWords = 512;

// ---- short numeric strings without per-byte branches (r06) ---------------------------------------------------------
// The numeric-looking string columns a profile casts hold short plain numbers ("-4999", "123.45"). For a string of
// <= 15 bytes the lane assembles its bytes as two words (aligned dword loads, from the wave's LDS stage when there is
// one) and runs one DFA step per byte position, wave-uniform up to the wave's longest such string, with selects only:
// [+|-] digits* [. digits*]. That grammar is all of UTF8String.toLong at this length (the value fits: 15 digits), so
// LONG is decided here; for DOUBLE it is the plain-decimal subset of Double.parseDouble, whose value is the integer of
// all its digits (< 10^15, exact in a double) divided by 10^(fraction digits) (exact): one correctly rounded IEEE
// division, i.e. Java's correctly rounded result (Clinger's fast path). Anything else (whitespace, exponents, NaN /
// Infinity, suffixes, hex, longer strings) takes the general parsers of dq_parse.h as before.
struct ShortNum {
    bool fast;      // the DFA decided the row (LONG: always for <= 15 bytes; DOUBLE: the plain-decimal form)
    bool ok;        // parsed (else NULL)
    int64_t v;      // LONG
    double d;       // DOUBLE
};

__device__ __forceinline__ uint32_t cast_dw(const uint8_t* a, int k) {
    return *reinterpret_cast<const uint32_t*>(a + 4 * k);
}

// Returns the row's short-number parse; `len` <= 15 is the caller's condition for `eligible`. `maxlen` is the wave's
// largest eligible length (wave-uniform loop bound).
__device__ __forceinline__ ShortNum cast_short_number(const uint8_t* s, int len, bool eligible, int maxlen,
                                                      bool to_double) {
    uint64_t x0 = 0, x1 = 0;
    if (eligible && len > 0) {
        const uint8_t* a = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(s) & ~(uintptr_t)3);
        const uint32_t sh = (uint32_t)(s - a);
        const int ndw = (int)((sh + (uint32_t)len + 3) >> 2);
        uint32_t w[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) w[k] = k < ndw ? cast_dw(a, k) : 0u;
        x0 = (uint64_t)__builtin_amdgcn_alignbyte(w[1], w[0], sh) |
             ((uint64_t)__builtin_amdgcn_alignbyte(w[2], w[1], sh) << 32);
        x1 = (uint64_t)__builtin_amdgcn_alignbyte(w[3], w[2], sh) |
             ((uint64_t)__builtin_amdgcn_alignbyte(w[4], w[3], sh) << 32);
    }
    uint64_t mi = 0;      // LONG: the digits before the point
    double md = 0.0;      // DOUBLE: every digit
    double p10 = 1.0;     // 10^(fraction digits)
    int nd = 0;
    bool dot = false, neg = false, sg = false, bad = false;
    for (int i = 0; i < maxlen; ++i) {  // wave-uniform bound
        const bool act = eligible && i < len;
        const uint64_t word = i < 8 ? x0 : x1;
        const uint32_t c = (uint32_t)(word >> (8 * (i & 7))) & 0xFFu;
        const uint32_t dg = c - (uint32_t)'0';
        const bool isd = act && dg < 10u;
        const bool isdot = act && c == (uint32_t)'.' && !dot;
        const bool sgn = act && i == 0 && (c == (uint32_t)'+' || c == (uint32_t)'-');
        bad |= act && !isd && !isdot && !sgn;
        neg |= sgn && c == (uint32_t)'-';
        sg |= sgn;
        mi = isd && !dot ? mi * 10ull + dg : mi;
        md = isd ? __builtin_fma(md, 10.0, (double)dg) : md;
        p10 = isd && dot ? p10 * 10.0 : p10;
        nd += isd ? 1 : 0;
        dot |= isdot;
    }
    ShortNum r;
    if (!to_double) {
        // UTF8String.toLong: "" and a lone sign are NULL; a bad character is NULL; otherwise the truncated integer
        r.fast = eligible;
        r.ok = !bad && len > 0 && !(len == 1 && sg);
        r.v = neg ? (int64_t)(0ull - mi) : (int64_t)mi;
        r.d = 0.0;
    } else {
        r.fast = eligible && !bad && nd > 0;
        r.ok = r.fast;
        const double q = md / p10;
        r.d = neg ? -q : q;
        r.v = 0;
    }
    return r;
}

template <bool STRING>
__global__ void __launch_bounds__(kCastBlock)
cast_kernel(CastSource c, int64_t nrows, int to_double, void* __restrict__ values_out,
            uint64_t* __restrict__ validity_out, unsigned int* __restrict__ slow_flag, int no_short) {
    __shared__ uint32_t stage[STRING ? kCastBlock / 64 : 1][STRING ? kCastStageWords : 1];
    const int64_t stride = (int64_t)gridDim.x * kCastBlock;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int64_t base = (int64_t)blockIdx.x * kCastBlock; base < nrows; base += stride) {
        const int64_t r = base + threadIdx.x;
        bool ok = false;
        double d = 0.0;
        int64_t v = 0;
        const uint8_t* sbase = nullptr;  // STRING: the staged copy of this wave's bytes, based at a0
        int64_t a0 = 0;
        // the row's validity and (STRING) its offsets, loaded before the staging: with the wave's range bounds they
        // are one memory round trip, not a third one after the stage's barrier
        const bool rin = r < nrows;
        const bool rvalid = rin && (c.validity == nullptr || ((c.validity[r >> 6] >> (r & 63)) & 1ull));
        int32_t ro = 0, rlen = 0;
        if (STRING && rin) {
            ro = c.offsets[r];
            rlen = c.offsets[r + 1] - ro;
        }
        if (STRING) {
            const int64_t w0 = base + 64 * wave;
            if (w0 < nrows) {
                const int64_t wl = w0 + 64 < nrows ? w0 + 64 : nrows;
                const int64_t b0 = c.offsets[w0], b1 = c.offsets[wl];
                a0 = b0 & ~(int64_t)3;
                const int64_t nwords = (b1 - a0 + 3) >> 2;  // dwords holding [b0, b1): nothing past the last byte
                if (nwords <= kCastStageWords) {
                    const uint32_t* src = reinterpret_cast<const uint32_t*>(c.bytes + a0);
                    for (int64_t i = lane; i < nwords; i += 64) stage[wave][i] = src[i];
                    sbase = reinterpret_cast<const uint8_t*>(&stage[wave][0]);
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
        }
        ShortNum sn;
        sn.fast = false;
        if (STRING && !no_short) {
            const bool elig = rvalid && rlen <= 15;
            int ml = elig ? rlen : 0;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) ml = max(ml, __shfl_xor(ml, o, 64));
            const uint8_t* s = sbase ? sbase + (ro - a0) : c.bytes + ro;
            sn = cast_short_number(s, rlen, elig, ml, to_double != 0);
            if (sn.fast) {
                ok = sn.ok;
                d = sn.d;
                v = sn.v;
            }
        }
        if (rvalid && !sn.fast) {
            if (STRING) {
                const int32_t o = ro;
                const int len = rlen;
                const uint8_t* s = sbase ? sbase + (o - a0) : c.bytes + o;
                if (to_double) {
                    bool slow = false;
                    ok = java_parse_double(s, len, d, slow);
                    if (slow) atomicOr(slow_flag, 1u);
                } else {
                    ok = spark_string_to_long(s, len, v);
                }
            } else {
                ok = true;
                switch (c.elem) {
                    case ET_F64: d = static_cast<const double*>(c.values)[r]; v = java_d2l(d); break;
                    case ET_F32: d = (double)static_cast<const float*>(c.values)[r]; v = java_d2l(d); break;
                    case ET_I64: {
                        const int64_t x = static_cast<const int64_t*>(c.values)[r];
                        if (c.decimal_scale) {  // Decimal.toDouble / Decimal.toLong (truncating)
                            d = (double)x / (double)c.pow10;
                            v = x / c.pow10;
                        } else {
                            d = (double)x;
                            v = x;
                        }
                        break;
                    }
                    case ET_I32: v = static_cast<const int32_t*>(c.values)[r]; d = (double)v; break;
                    case ET_I16: v = static_cast<const int16_t*>(c.values)[r]; d = (double)v; break;
                    case ET_I8: v = static_cast<const int8_t*>(c.values)[r]; d = (double)v; break;
                    default: v = static_cast<const uint8_t*>(c.values)[r] ? 1 : 0; d = (double)v; break;
                }
            }
        }
        if (r < nrows) {
            if (to_double) static_cast<double*>(values_out)[r] = ok ? d : 0.0;
            else static_cast<int64_t*>(values_out)[r] = ok ? v : 0;
        }
        const unsigned long long ball = __ballot(ok);
        if ((threadIdx.x & 63) == 0 && r < nrows) validity_out[r >> 6] = ball;
        if (STRING) __builtin_amdgcn_wave_barrier();  // every lane's parse done before the next group's staging
    }
}

hipStream_t ctx_stream(dq_ctx* ctx);
int ctx_device(dq_ctx* ctx);
int ctx_fail(dq_ctx* ctx, int code, const char* msg);
int ctx_cus(dq_ctx* ctx);

}  // namespace dq

namespace {
// Per-call device buffers from the context's scratch cache: a hipFree per cast waited for the whole device, so a cast
// stalled behind every other context's running kernels (the C5 step's casts sat idle for ~20 ms between columns).
struct CBuffers {
    dq_ctx* ctx;
    std::vector<std::pair<void*, size_t>> ptrs;
    explicit CBuffers(dq_ctx* c) : ctx(c) {}
    ~CBuffers() {
        for (const auto& p : ptrs) dq::scratch_release(ctx, p.first, p.second);
    }
    hipError_t alloc(void** p, size_t bytes) {
        bytes = std::max<size_t>(bytes, 16);
        *p = dq::scratch_alloc(ctx, bytes);
        if (!*p) return hipErrorOutOfMemory;
        ptrs.push_back({*p, bytes});
        return hipSuccess;
    }
};
}  // namespace

#define CA_HIP(ctx, expr)                                                                         \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess) return dq::ctx_fail((ctx), DQ_ERR_DEVICE, hipGetErrorString(e_));   \
    } while (0)

extern "C" {

static int cast_single(dq_ctx* ctx, const dq_column* column, int64_t nrows, int32_t to_type, void* values_dev,
                       uint8_t* validity_dev);

int dq_cast_column(dq_ctx* ctx, const dq_column* column, int64_t nrows, int32_t to_type, void* values_out,
                   uint8_t* validity_out) {
    if (!ctx || !column || nrows < 0 || column->length != nrows || (nrows > 0 && (!values_out || !validity_out)))
        return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_cast_column: invalid arguments");
    const int nsub = dq::ctx_num_subs(ctx);
    if (nsub == 0) return cast_single(ctx, column, nrows, to_type, values_out, validity_out);
    // multi-device context: host column in, host results out; each device casts its contiguous row shard (2048-row
    // aligned, so its validity words start on a word boundary) and copies its slice of the results back
    if (column->flags & DQ_COL_DEVICE) return dq::ctx_fail(ctx, DQ_ERR_UNSUPPORTED, "a multi-device context takes host columns");
    std::vector<int> rc(nsub, DQ_OK);
    std::vector<std::string> err(nsub);
    std::vector<dq_column> cols(nsub, *column);
    std::vector<std::vector<std::vector<int32_t>>> scratch(nsub);
    std::vector<std::thread> th;
    for (int i = 0; i < nsub; ++i) {
        int64_t r0 = 0, cnt = 0;
        dq::shard_bounds(nrows, nsub, i, &r0, &cnt);
        dq::shard_columns(column, 1, r0, cnt, &cols[i], scratch[i]);
        th.emplace_back([&, i, r0, cnt]() {
            if (cnt == 0) return;
            dq_ctx* sub = dq::ctx_sub(ctx, i);
            void* dv = nullptr;
            void* dm = nullptr;
            const size_t vb = (size_t)cnt * 8, mb = (size_t)(cnt + 63) / 64 * 8;
            if (hipSetDevice(dq::ctx_device(sub)) != hipSuccess || hipMalloc(&dv, vb) != hipSuccess ||
                hipMalloc(&dm, mb) != hipSuccess) {
                rc[i] = DQ_ERR_OUT_OF_MEMORY;
            } else {
                rc[i] = cast_single(sub, &cols[i], cnt, to_type, dv, (uint8_t*)dm);
                if (rc[i] == DQ_OK &&
                    (hipMemcpy((uint8_t*)values_out + (size_t)r0 * 8, dv, vb, hipMemcpyDeviceToHost) != hipSuccess ||
                     hipMemcpy(validity_out + (size_t)r0 / 8, dm, mb, hipMemcpyDeviceToHost) != hipSuccess))
                    rc[i] = DQ_ERR_DEVICE;
            }
            if (dv) (void)hipFree(dv);
            if (dm) (void)hipFree(dm);
        });
    }
    for (auto& x : th) x.join();
    for (int i = 0; i < nsub; ++i)
        if (rc[i] != DQ_OK) return dq::ctx_fail(ctx, rc[i], "dq_cast_column: a device's shard failed");
    return DQ_OK;
}

static int cast_single(dq_ctx* ctx, const dq_column* column, int64_t nrows, int32_t to_type, void* values_dev,
                       uint8_t* validity_dev) {
    const int t = column->spark_type;
    const bool is_string = t == DQ_TYPE_STRING;
    if (is_string && !column->offsets)
        return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_cast_column: string column without offsets");
    if (!is_string && !(t == DQ_TYPE_BOOLEAN || t == DQ_TYPE_BYTE || t == DQ_TYPE_SHORT || t == DQ_TYPE_INT ||
                        t == DQ_TYPE_LONG || t == DQ_TYPE_FLOAT || t == DQ_TYPE_DOUBLE || t == DQ_TYPE_DECIMAL))
        return dq::ctx_fail(ctx, DQ_ERR_UNSUPPORTED, "dq_cast_column: source type cannot be cast to a number here");
    if (t == DQ_TYPE_DECIMAL && (column->decimal_precision > 18 || column->decimal_scale < 0 || column->decimal_scale > 18))
        return dq::ctx_fail(ctx, DQ_ERR_UNSUPPORTED, "dq_cast_column: decimal precision > 18 unsupported");
    if (to_type != DQ_TYPE_LONG && to_type != DQ_TYPE_DOUBLE)
        return dq::ctx_fail(ctx, DQ_ERR_UNSUPPORTED, "dq_cast_column: target type must be LONG or DOUBLE");
    if (((uintptr_t)values_dev & 7) || ((uintptr_t)validity_dev & 7))
        return dq::ctx_fail(ctx, DQ_ERR_ALIGNMENT, "dq_cast_column: output buffers must be 8-B aligned");
    if (nrows == 0) return DQ_OK;
    CA_HIP(ctx, hipSetDevice(dq::ctx_device(ctx)));
    hipStream_t s = dq::ctx_stream(ctx);
    CBuffers buf(ctx);
    if (column->flags & DQ_COL_OFFSETS64)
        return dq::ctx_fail(ctx, DQ_ERR_UNSUPPORTED, "dq_cast_column: int64 string offsets are for the grouping builds only");
    dq::CastSource c;
    memset(&c, 0, sizeof(c));
    c.elem = is_string ? dq::ET_NONE : dq::elem_of(t);
    c.decimal_scale = t == DQ_TYPE_DECIMAL ? column->decimal_scale : 0;
    c.pow10 = 1;
    for (int i = 0; i < c.decimal_scale; ++i) c.pow10 *= 10;
    if (column->flags & DQ_COL_DEVICE) {
        c.values = column->values;
        c.bytes = (const uint8_t*)column->values;
        c.offsets = column->offsets;
        c.validity = (const uint64_t*)column->validity;
    } else {
        void *b = nullptr, *o = nullptr, *m = nullptr;
        if (is_string) {
            const int32_t total = column->offsets[nrows];
            CA_HIP(ctx, buf.alloc(&b, (size_t)total + 16));
            CA_HIP(ctx, buf.alloc(&o, sizeof(int32_t) * (size_t)(nrows + 1)));
            if (total > 0) CA_HIP(ctx, hipMemcpyAsync(b, column->values, (size_t)total, hipMemcpyHostToDevice, s));
            CA_HIP(ctx, hipMemcpyAsync(o, column->offsets, sizeof(int32_t) * (size_t)(nrows + 1), hipMemcpyHostToDevice, s));
        } else {
            const size_t vb = (size_t)nrows * dq::elem_size(c.elem);
            CA_HIP(ctx, buf.alloc(&b, vb));
            CA_HIP(ctx, hipMemcpyAsync(b, column->values, vb, hipMemcpyHostToDevice, s));
        }
        if (column->validity) {
            const size_t bb = (size_t)(nrows + 63) / 64 * 8;
            CA_HIP(ctx, buf.alloc(&m, bb));
            CA_HIP(ctx, hipMemsetAsync(m, 0, bb, s));
            CA_HIP(ctx, hipMemcpyAsync(m, column->validity, (size_t)(nrows + 7) / 8, hipMemcpyHostToDevice, s));
        }
        c.values = b;
        c.bytes = (const uint8_t*)b;
        c.offsets = (const int32_t*)o;
        c.validity = (const uint64_t*)m;
    }
    unsigned int* dslow = nullptr;
    CA_HIP(ctx, buf.alloc((void**)&dslow, sizeof(unsigned int)));
    CA_HIP(ctx, hipMemsetAsync(dslow, 0, sizeof(unsigned int), s));
    const int64_t blocks = (nrows + dq::kCastBlock - 1) / dq::kCastBlock;
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(blocks, (int64_t)dq::ctx_cus(ctx) * 16));
    const int to_double = to_type == DQ_TYPE_DOUBLE ? 1 : 0;
    const int no_short = getenv("DQ_CAST_NO_SHORT") ? 1 : 0;  // A/B and tests: every row through dq_parse.h
    if (is_string)
        hipLaunchKernelGGL(dq::cast_kernel<true>, dim3(grid), dim3(dq::kCastBlock), 0, s, c, nrows, to_double, values_dev,
                           (uint64_t*)validity_dev, dslow, no_short);
    else
        hipLaunchKernelGGL(dq::cast_kernel<false>, dim3(grid), dim3(dq::kCastBlock), 0, s, c, nrows, to_double,
                           values_dev, (uint64_t*)validity_dev, dslow, no_short);
    CA_HIP(ctx, hipGetLastError());
    unsigned int slow = 0;
    CA_HIP(ctx, hipMemcpyAsync(&slow, dslow, sizeof(slow), hipMemcpyDeviceToHost, s));
    CA_HIP(ctx, hipStreamSynchronize(s));
    if (slow)
        return dq::ctx_fail(ctx, DQ_ERR_UNSUPPORTED,
                            "dq_cast_column: a value needs the arbitrary-precision path of Double.parseDouble "
                            "(hexadecimal literal, or > 19 significant digits on a rounding boundary)");
    return DQ_OK;
}

}  // extern "C"
