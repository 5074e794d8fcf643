// strings.hip — the string-shaped scan ops of the fused pass (gfx950 / CDNA4).
//
// Per (column, where) "string slot", one lane per row:
//   MinLength / MaxLength    min/max(length(when(where, col))) — UTF-8 character count
//                            (A/MinLength.scala:28-30, A/MaxLength.scala:28-30)
//   DataType                 StatefulDataType.update (C/StatefulDataType.scala:58-69): the value cast to
//                            string, classified by the full-match regexes
//                            FRACTIONAL ^(-|\+)? ?\d*\.\d*$, INTEGRAL ^(-|\+)? ?\d*$, BOOLEAN ^(true|false)$
//                            (:36-38), in that order; rows outside `where` count as NULL
//                            (conditionalSelection, A/DataType.scala:146-148)
//   ApproxCountDistinct      XxHash64(UTF-8 bytes, seed 42) into HLL++ registers (P = 9) in LDS
//                            (C/StatefulHyperloglogPlus.scala:89-112) — the register partials share the
//                            fixed-width HLL arrays, so reduce_hll / finalize pack them the same way.
// Non-string columns only reach this kernel for DataType, whose string cast is decided from the value
// (Java's Long/Double/Float/BigDecimal.toString rules, see numeric_class).
// Byte work, no MFMA: bytes are read as aligned little-endian dwords (adjacent lanes own adjacent
// strings, so a wave's loads share cache lines); per-block partials are folded in a fixed order.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdlib.h>

#include <algorithm>

#include "dq_common.h"
#include "dq_internal.h"

namespace dq {

namespace {

__device__ __forceinline__ uint32_t load_word(const uint8_t* base, int64_t aligned_off) {
    return *reinterpret_cast<const uint32_t*>(base + aligned_off);
}

__device__ __forceinline__ uint8_t byte_at(const uint8_t* base, int64_t off) { return base[off]; }

// UTF-8 characters (non-continuation bytes) in [o0, o1) — UTF8String.numChars for valid UTF-8.
__device__ int64_t utf8_length(const uint8_t* data, int64_t o0, int64_t o1) {
    if (o1 <= o0) return 0;
    int64_t cont = 0;
    const int64_t w0 = o0 & ~(int64_t)3;
    for (int64_t w = w0; w < o1; w += 4) {
        uint32_t x = load_word(data, w);
        uint32_t mask = 0xFFFFFFFFu;
        if (w < o0) mask &= 0xFFFFFFFFu << (8 * (o0 - w));
        if (w + 4 > o1) mask &= 0xFFFFFFFFu >> (8 * (w + 4 - o1));
        // continuation byte: bit 7 set, bit 6 clear
        const uint32_t c = x & ~(x << 1) & 0x80808080u & mask;
        cont += __popc(c);
    }
    return (o1 - o0) - cont;
}

// XXH64.hashUnsafeBytes over data[o0, o1) (seed 42), reading bytes through dword loads.
__device__ __forceinline__ uint64_t le64_at(const uint8_t* data, int64_t p) {
    const int64_t a = p & ~(int64_t)3;
    const int sh = (int)(p - a) * 8;
    const uint32_t w0 = load_word(data, a), w1 = load_word(data, a + 4), w2 = load_word(data, a + 8);
    const uint64_t lo = sh ? (((uint64_t)w1 << (32 - sh)) | (w0 >> sh)) : w0;
    const uint64_t hi = sh ? (((uint64_t)w2 << (32 - sh)) | (w1 >> sh)) : w1;
    return (lo & 0xFFFFFFFFull) | (hi << 32);
}
__device__ __forceinline__ uint32_t le32_at(const uint8_t* data, int64_t p) {
    const int64_t a = p & ~(int64_t)3;
    const int sh = (int)(p - a) * 8;
    const uint32_t w0 = load_word(data, a);
    if (!sh) return w0;
    const uint32_t w1 = load_word(data, a + 4);
    return (uint32_t)((((uint64_t)w1 << 32) | w0) >> sh);
}

__device__ uint64_t xxh64_utf8(const uint8_t* data, int64_t o0, int64_t o1, uint64_t seed) {
    const int64_t len = o1 - o0;
    int64_t p = o0;
    uint64_t h;
    if (len >= 32) {
        uint64_t v1 = seed + P64_1 + P64_2, v2 = seed + P64_2, v3 = seed, v4 = seed - P64_1;
        const int64_t limit = o1 - 32;
        do {
            v1 = xxh_round(v1, le64_at(data, p));
            v2 = xxh_round(v2, le64_at(data, p + 8));
            v3 = xxh_round(v3, le64_at(data, p + 16));
            v4 = xxh_round(v4, le64_at(data, p + 24));
            p += 32;
        } while (p <= limit);
        h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
        h = xxh_merge_round(h, v1);
        h = xxh_merge_round(h, v2);
        h = xxh_merge_round(h, v3);
        h = xxh_merge_round(h, v4);
    } else {
        h = seed + P64_5;
    }
    h += (uint64_t)len;
    while (p + 8 <= o1) {
        h ^= xxh_round(0, le64_at(data, p));
        h = rotl64(h, 27) * P64_1 + P64_4;
        p += 8;
    }
    if (p + 4 <= o1) {
        h ^= (uint64_t)le32_at(data, p) * P64_1;
        h = rotl64(h, 23) * P64_2 + P64_3;
        p += 4;
    }
    while (p < o1) {
        h ^= (uint64_t)byte_at(data, p) * P64_5;
        h = rotl64(h, 11) * P64_1;
        ++p;
    }
    return xxh_fmix(h);
}

enum DtClass : int { DT_NULL = 0, DT_FRACTIONAL = 1, DT_INTEGRAL = 2, DT_BOOLEAN = 3, DT_STRING = 4 };

// First position in [i, o1) that is not an ASCII digit (o1 if none), four bytes per step: a byte b is a digit iff
// t = b ^ 0x30 is < 10, i.e. neither t's bit 7 nor bit 7 of (t & 0x7F) + 0x76 is set (no carry crosses a byte).
__device__ __forceinline__ int64_t skip_digits(const uint8_t* data, int64_t i, int64_t o1) {
    while (i < o1) {
        const int64_t a = i & ~(int64_t)3;
        const int k = (int)(i - a);
        const uint32_t t = (load_word(data, a) >> (8 * k)) ^ 0x30303030u;
        const uint32_t nd = (((t & 0x7F7F7F7Fu) + 0x76767676u) | t) & 0x80808080u;
        const int nb = (int)(o1 - i < 4 - k ? o1 - i : 4 - k);  // bytes of this word inside the string
        if (nd) {
            const int pos = __builtin_ctz(nd) >> 3;
            if (pos < nb) return i + pos;
        }
        i += nb;
    }
    return o1;
}

// StatefulDataType's three full-match regexes over the UTF-8 bytes.
__device__ int classify_string(const uint8_t* data, int64_t o0, int64_t o1) {
    int64_t i = o0;
    if (i < o1) {
        const uint8_t c = byte_at(data, i);
        if (c == '-' || c == '+') ++i;
    }
    if (i < o1 && byte_at(data, i) == ' ') ++i;
    i = skip_digits(data, i, o1);
    if (i == o1) return DT_INTEGRAL;  // includes "" and a lone sign
    if (byte_at(data, i) == '.') {
        i = skip_digits(data, i + 1, o1);
        if (i == o1) return DT_FRACTIONAL;
    }
    const int64_t n = o1 - o0;
    if (n == 4 && byte_at(data, o0) == 't' && byte_at(data, o0 + 1) == 'r' && byte_at(data, o0 + 2) == 'u' &&
        byte_at(data, o0 + 3) == 'e')
        return DT_BOOLEAN;
    if (n == 5 && byte_at(data, o0) == 'f' && byte_at(data, o0 + 1) == 'a' && byte_at(data, o0 + 2) == 'l' &&
        byte_at(data, o0 + 3) == 's' && byte_at(data, o0 + 4) == 'e')
        return DT_BOOLEAN;
    return DT_STRING;
}

// DataType of a non-string value through Spark's cast to string:
//   boolean -> "true"/"false"; integral -> digits; double/float -> Java toString, which is plain
//   ("d.ddd", FRACTIONAL) exactly for 0 and 1e-3 <= |x| < 1e7 and "d.dddE±n" / "NaN" / "Infinity"
//   (STRING) otherwise; decimal -> BigDecimal.toString: scale 0 -> digits (INTEGRAL), otherwise
//   plain with a point (FRACTIONAL) unless the adjusted exponent is < -6 (scientific, STRING);
//   date / timestamp -> "yyyy-MM-dd..." (STRING).
__device__ __forceinline__ int numeric_class(const StrSlot& s, int64_t row) {
    switch (s.spark_type) {
        case DQ_TYPE_BOOLEAN: return DT_BOOLEAN;
        case DQ_TYPE_BYTE: case DQ_TYPE_SHORT: case DQ_TYPE_INT: case DQ_TYPE_LONG: return DT_INTEGRAL;
        case DQ_TYPE_DOUBLE: {
            const double x = static_cast<const double*>(s.values)[row];
            const double a = fabs(x);
            return (x == 0.0 || (a >= 1e-3 && a < 1e7)) ? DT_FRACTIONAL : DT_STRING;  // NaN/inf fail both
        }
        case DQ_TYPE_FLOAT: {
            const float x = static_cast<const float*>(s.values)[row];
            const float a = fabsf(x);
            return (x == 0.0f || (a >= 1e-3f && a < 1e7f)) ? DT_FRACTIONAL : DT_STRING;
        }
        case DQ_TYPE_DECIMAL: {
            if (s.decimal_scale == 0) return DT_INTEGRAL;
            const int64_t v = static_cast<const int64_t*>(s.values)[row];
            uint64_t m = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
            int digits = 1;
            while (m >= 10) {
                m /= 10;
                ++digits;
            }
            return (digits - 1 - s.decimal_scale) < -6 ? DT_STRING : DT_FRACTIONAL;
        }
        default: return DT_STRING;  // DATE, TIMESTAMP
    }
}

__device__ __forceinline__ int64_t shfl_down_i64s(int64_t x, int off) {
    int lo = (int)(uint32_t)(uint64_t)x, hi = (int)(uint32_t)((uint64_t)x >> 32);
    lo = __shfl_down(lo, off, 64);
    hi = __shfl_down(hi, off, 64);
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

}  // namespace

// One row's string ops over data[o0, o1) — `data` is the column's bytes in HBM, or the wave's staged copy in LDS.
__device__ __forceinline__ void string_row(const StrSlot& s, const uint8_t* data, int64_t o0, int64_t o1, bool want_hll,
                                           int64_t& mn, int64_t& mx, int64_t (&dt)[5], uint32_t* regs) {
    if (s.flags & SF_LEN) {
        const int64_t len = utf8_length(data, o0, o1);
        mn = len < mn ? len : mn;
        mx = len > mx ? len : mx;
    }
    if (s.flags & SF_DTYPE) dt[classify_string(data, o0, o1)] += 1;
    if (want_hll) {
        const uint64_t x = xxh64_utf8(data, o0, o1, SPARK_HLL_SEED);
        atomicMax(&regs[hll_index(x)], hll_rank(x));
    }
}

// Bytes of one wave's 64 consecutive strings staged in LDS (coalesced dword loads of the whole byte range instead of
// each lane's scattered byte / dword loads); ranges longer than this are read from HBM directly.
#ifndef DQ_STR_B128
#define DQ_STR_B128 1
#endif
#ifndef DQ_STR_STAGE
#define DQ_STR_STAGE 256  // words per 64-row group (r06: with DQ_STR_R 8, the same 32 KB of LDS per workgroup as 4 x 512)
#endif
constexpr int kStrStageWords = DQ_STR_STAGE;

// ---- the staged form: 32-bit byte positions into the wave's LDS words -----------------------------------------------
// The same ops as above over a staged range (< 2 KiB, so positions are 32-bit: the int64 position arithmetic of the
// HBM form doubles every add / compare), unaligned words assembled with one v_alignbyte each, the string's first word
// held for the sign / space / boolean tests, and the 1-3 byte hash tail taken from one word. The stage holds >= 12
// bytes past the range, so a word read past a string's end stays inside it.
__device__ __forceinline__ uint32_t st_word(const uint32_t* st, int p) {  // bytes p .. p + 3
    const int a = p >> 2;
    return __builtin_amdgcn_alignbyte(st[a + 1], st[a], (uint32_t)(p & 3));
}
__device__ __forceinline__ uint64_t st_dword(const uint32_t* st, int p) {  // bytes p .. p + 7
    const int a = p >> 2;
    const uint32_t sh = (uint32_t)(p & 3), w0 = st[a], w1 = st[a + 1], w2 = st[a + 2];
    return ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32) | __builtin_amdgcn_alignbyte(w1, w0, sh);
}

__device__ __forceinline__ int st_utf8_length(const uint32_t* st, int o0, int o1) {
    int cont = 0;
    for (int w = o0 & ~3; w < o1; w += 4) {
        const uint32_t x = st[w >> 2];
        uint32_t mask = 0xFFFFFFFFu;
        if (w < o0) mask &= 0xFFFFFFFFu << (8 * (o0 - w));
        if (w + 4 > o1) mask &= 0xFFFFFFFFu >> (8 * (w + 4 - o1));
        cont += __popc(x & ~(x << 1) & 0x80808080u & mask);
    }
    return (o1 - o0) - cont;
}

__device__ __forceinline__ uint64_t st_xxh64(const uint32_t* st, int o0, int o1, uint64_t seed) {
    const int len = o1 - o0;
    int p = o0;
    uint64_t h;
    if (len >= 32) {
        uint64_t v1 = seed + P64_1 + P64_2, v2 = seed + P64_2, v3 = seed, v4 = seed - P64_1;
        const int limit = o1 - 32;
        do {
            v1 = xxh_round(v1, st_dword(st, p));
            v2 = xxh_round(v2, st_dword(st, p + 8));
            v3 = xxh_round(v3, st_dword(st, p + 16));
            v4 = xxh_round(v4, st_dword(st, p + 24));
            p += 32;
        } while (p <= limit);
        h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
        h = xxh_merge_round(h, v1);
        h = xxh_merge_round(h, v2);
        h = xxh_merge_round(h, v3);
        h = xxh_merge_round(h, v4);
    } else {
        h = seed + P64_5;
    }
    h += (uint64_t)len;
    while (p + 8 <= o1) {
        h ^= xxh_round(0, st_dword(st, p));
        h = rotl64(h, 27) * P64_1 + P64_4;
        p += 8;
    }
    if (p + 4 <= o1) {
        h ^= (uint64_t)st_word(st, p) * P64_1;
        h = rotl64(h, 23) * P64_2 + P64_3;
        p += 4;
    }
    if (p < o1) {  // 1-3 bytes, from one word
        uint32_t w = st_word(st, p);
        const int r = o1 - p;
#pragma unroll
        for (int i = 0; i < 3; ++i)
            if (i < r) {
                h ^= (uint64_t)(w & 0xFFu) * P64_5;
                h = rotl64(h, 11) * P64_1;
                w >>= 8;
            }
    }
    return xxh_fmix(h);
}

__device__ __forceinline__ int st_skip_digits(const uint32_t* st, int i, int o1) {
    while (i < o1) {
        const int k = i & 3;
        const uint32_t t = (st[i >> 2] >> (8 * k)) ^ 0x30303030u;
        const uint32_t nd = (((t & 0x7F7F7F7Fu) + 0x76767676u) | t) & 0x80808080u;
        const int nb = o1 - i < 4 - k ? o1 - i : 4 - k;
        if (nd) {
            const int pos = __builtin_ctz(nd) >> 3;
            if (pos < nb) return i + pos;
        }
        i += nb;
    }
    return o1;
}

__device__ __forceinline__ int st_classify(const uint32_t* st, int o0, int o1) {
    const int n = o1 - o0;
    const uint32_t w = st_word(st, o0);  // the first 4 bytes (garbage past n)
    const uint32_t c0 = w & 0xFFu;
    const int sgn = (n > 0 && (c0 == '-' || c0 == '+')) ? 1 : 0;
    const int sp = (n > sgn && ((w >> (8 * sgn)) & 0xFFu) == ' ') ? 1 : 0;
    int i = st_skip_digits(st, o0 + sgn + sp, o1);
    if (i == o1) return DT_INTEGRAL;  // includes "" and a lone sign
    if (((st[i >> 2] >> (8 * (i & 3))) & 0xFFu) == '.') {
        i = st_skip_digits(st, i + 1, o1);
        if (i == o1) return DT_FRACTIONAL;
    }
    if (n == 4 && w == 0x65757274u) return DT_BOOLEAN;                                          // "true"
    if (n == 5 && w == 0x736C6166u && ((st[(o0 + 4) >> 2] >> (8 * ((o0 + 4) & 3))) & 0xFFu) == 'e')  // "false"
        return DT_BOOLEAN;
    return DT_STRING;
}

// dt[c] += 1 with static indices only (a dynamic index into the register array would put it in scratch)
__device__ __forceinline__ void dt_add(int64_t (&dt)[5], int c) {
#pragma unroll
    for (int k = 1; k < 5; ++k) dt[k] += c == k ? 1 : 0;
}

template <bool LEN, bool DT, bool HLL>
__device__ __forceinline__ void st_string_row(const uint32_t* st, int o0, int o1, int64_t& mn, int64_t& mx,
                                              int64_t (&dt)[5], uint32_t* regs) {
    if constexpr (LEN) {
        const int64_t len = st_utf8_length(st, o0, o1);
        mn = len < mn ? len : mn;
        mx = len > mx ? len : mx;
    }
    if constexpr (DT) dt_add(dt, st_classify(st, o0, o1));
    if constexpr (HLL) {
        const uint64_t x = st_xxh64(st, o0, o1, SPARK_HLL_SEED);
        atomicMax(&regs[hll_index(x)], hll_rank(x));
    }
}

// One slot's string rows, kStrR groups of 64 consecutive rows per wave and step (lane L takes rows base + 64 j + L): all
// their offsets and validity words are loaded first, then the step's whole byte range is staged in the wave's LDS words
// by buffer loads issued 8 per lane at a time (out-of-range words read as 0), so one step costs two dependent memory
// round trips for 64 kStrR rows instead of two per 64. Ranges longer than the stage are read from HBM per lane.
// (r06: 8 groups of 256 words, one step = 512 rows per wave, 12.70 ms against 13.26 ms for 4 groups of 512 words on the
// ten C5 string columns of a 1.25e8-row chunk; 16 x 256 words: 21 ms. profiles/r06/c5_strings_r8_ab_r06af.txt)
#ifndef DQ_STR_R
#define DQ_STR_R 8
#endif
constexpr int kStrR = DQ_STR_R;

template <bool LEN, bool DT, bool HLL>
__device__ __forceinline__ void string_groups(const uint8_t* __restrict__ data, const int32_t* __restrict__ offsets,
                                              const uint64_t* __restrict__ validity, const uint64_t* __restrict__ where_t,
                                              int64_t nrows, int64_t base0, int64_t stride, int lane, uint32_t* stage,
                                              int64_t& n, int64_t& mn, int64_t& mx, int64_t (&dt)[5], uint32_t* regs) {
    constexpr int G = 64 * kStrR;
    for (int64_t base = base0; base < nrows; base += stride) {
        const int64_t last = base + G < nrows ? base + G : nrows;
        const int64_t b0 = offsets[base], b1 = offsets[last];
        bool on[kStrR];
        int32_t o[kStrR], e[kStrR];
#pragma unroll
        for (int j = 0; j < kStrR; ++j) {
            const int64_t row = base + 64 * j + lane;
            bool v = row < nrows;
            if (v) {
                v = validity == nullptr || ((validity[row >> 6] >> (row & 63)) & 1ull);
                if (where_t) v = v && ((where_t[row >> 6] >> (row & 63)) & 1ull);
            }
            on[j] = v;
            o[j] = row < nrows ? offsets[row] : 0;
            e[j] = row < nrows ? offsets[row + 1] : 0;
            n += v ? 1 : 0;
        }
        const int64_t a0 = b0 & ~(int64_t)3;
        const int nwords = (int)((b1 + 12 - a0 + 3) >> 2);
        if (nwords <= kStrR * kStrStageWords) {
            const __amdgpu_buffer_rsrc_t r =
                __builtin_amdgcn_make_buffer_rsrc((void*)(data + a0), (short)0, nwords * 4, 0x00020000);
#if DQ_STR_B128
            // 16-byte loads and LDS stores (two per lane per 512 words instead of eight 4-byte ones); words past the
            // range read as 0 (the buffer's size) and the stage holds whole 512-word blocks
            // (a load straddling the range end is split into dword loads, so no load crosses the buffer's size)
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            for (int i0 = 0; i0 < nwords; i0 += 64 * 8) {
                u32x4 w[2];
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int c = i0 + 4 * (64 * u + lane);
                    if (c + 4 <= nwords) {
                        w[u] = __builtin_amdgcn_raw_buffer_load_b128(r, c * 4, 0, 0);
                    } else {
                        w[u] = u32x4{0u, 0u, 0u, 0u};
                        for (int k = 0; k < 3; ++k)
                            if (c + k < nwords) w[u][k] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(r, (c + k) * 4, 0, 0);
                    }
                }
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int c = i0 + 4 * (64 * u + lane);
                    if (c < nwords) *reinterpret_cast<u32x4*>(&stage[c]) = w[u];
                }
            }
#else
            for (int i0 = 0; i0 < nwords; i0 += 64 * 8) {
                uint32_t w[8];
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    w[u] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(r, (i0 + 64 * u + lane) * 4, 0, 0);
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (i0 + 64 * u + lane < nwords) stage[i0 + 64 * u + lane] = w[u];
            }
#endif
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int j = 0; j < kStrR; ++j)
                if (on[j]) st_string_row<LEN, DT, HLL>(stage, (int)(o[j] - a0), (int)(e[j] - a0), mn, mx, dt, regs);
            __builtin_amdgcn_wave_barrier();
        } else {
#pragma unroll
            for (int j = 0; j < kStrR; ++j)
                if (on[j]) {
                    if constexpr (LEN) {
                        const int64_t len = utf8_length(data, o[j], e[j]);
                        mn = len < mn ? len : mn;
                        mx = len > mx ? len : mx;
                    }
                    if constexpr (DT) dt_add(dt, classify_string(data, o[j], e[j]));
                    if constexpr (HLL) {
                        const uint64_t x = xxh64_utf8(data, o[j], e[j], SPARK_HLL_SEED);
                        atomicMax(&regs[hll_index(x)], hll_rank(x));
                    }
                }
        }
    }
}

__global__ void __launch_bounds__(kBlock)
scan_strings_kernel(const StrSlot* __restrict__ slots, int nslots, int64_t nrows, int gstride,
                    StrPartial* __restrict__ partials, uint8_t* __restrict__ hll_partials) {
    __shared__ uint32_t regs[kHllRegs];
    __shared__ StrPartial red[kBlock / 64];
    __shared__ __attribute__((aligned(16))) uint32_t stage[kBlock / 64][kStrR * kStrStageWords];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int si = 0; si < nslots; ++si) {
        const StrSlot s = slots[si];
        const bool str = s.spark_type == DQ_TYPE_STRING;
        const bool want_hll = (s.flags & SF_HLL) && str;
        if (want_hll) {
            for (int i = tid; i < kHllRegs; i += kBlock) regs[i] = 0;
            __syncthreads();
        }
        int64_t n = 0, mn = INT64_MAX, mx = INT64_MIN;
        int64_t dt[5] = {0, 0, 0, 0, 0};
        const int64_t stride = (int64_t)gridDim.x * kBlock;
        const int64_t base0 = (int64_t)blockIdx.x * kBlock + wave * 64;
        auto row_on = [&](int64_t b) {  // validity (and `where`) of row b + lane
            const int64_t row = b + lane;
            bool on = row < nrows;
            if (on) {
                on = s.validity == nullptr || ((s.validity[row >> 6] >> (row & 63)) & 1ull);
                if (s.where_t) on = on && ((s.where_t[row >> 6] >> (row & 63)) & 1ull);
            }
            return on;
        };
        // (r04: software-pipelining this loop — the next group's words and the group after's offsets in registers while
        // the current group is hashed — made the C5 string pass 25 % slower, profiles/r04/c5_ab_r04g.txt)
        if (str) {
            const int fl = ((s.flags & SF_LEN) ? 1 : 0) | ((s.flags & SF_DTYPE) ? 2 : 0) | (want_hll ? 4 : 0);
            const int64_t sbase0 = ((int64_t)blockIdx.x * (kBlock / 64) + wave) * (64 * kStrR);
            const int64_t sstride = (int64_t)gridDim.x * kBlock * kStrR;
            switch (fl) {  // the slot's ops as template flags: no per-row flag tests
#define DQ_STR_CASE(F) \
    case F: string_groups<(F & 1) != 0, (F & 2) != 0, (F & 4) != 0>(s.data, s.offsets, s.validity, s.where_t, nrows, \
                                                                    sbase0, sstride, lane, stage[wave], n, mn, mx, dt, regs); \
        break;
                DQ_STR_CASE(0) DQ_STR_CASE(1) DQ_STR_CASE(2) DQ_STR_CASE(3)
                DQ_STR_CASE(4) DQ_STR_CASE(5) DQ_STR_CASE(6) DQ_STR_CASE(7)
#undef DQ_STR_CASE
            }
        } else {
            for (int64_t b = base0; b < nrows; b += stride) {
                const bool on = row_on(b);
                n += on ? 1 : 0;
                if (on && (s.flags & SF_DTYPE)) dt_add(dt, numeric_class(s, b + lane));
            }
        }
        // wave64 tree, then the 4 waves in a fixed order
#pragma unroll 1
        for (int off = 32; off > 0; off >>= 1) {
            const int64_t on_ = shfl_down_i64s(n, off), omn = shfl_down_i64s(mn, off), omx = shfl_down_i64s(mx, off);
            int64_t odt[5];
#pragma unroll
            for (int k = 0; k < 5; ++k) odt[k] = shfl_down_i64s(dt[k], off);
            if (lane < off) {
                n += on_;
                mn = omn < mn ? omn : mn;
                mx = omx > mx ? omx : mx;
#pragma unroll
                for (int k = 0; k < 5; ++k) dt[k] += odt[k];
            }
        }
        if (lane == 0) {
            red[wave].n = n;
            red[wave].minlen = mn;
            red[wave].maxlen = mx;
            for (int k = 0; k < 5; ++k) red[wave].dt[k] = dt[k];
        }
        __syncthreads();
        if (tid == 0) {
            StrPartial p = red[0];
            for (int w = 1; w < kBlock / 64; ++w) {
                p.n += red[w].n;
                p.minlen = red[w].minlen < p.minlen ? red[w].minlen : p.minlen;
                p.maxlen = red[w].maxlen > p.maxlen ? red[w].maxlen : p.maxlen;
                for (int k = 0; k < 5; ++k) p.dt[k] += red[w].dt[k];
            }
            partials[(int64_t)si * gstride + blockIdx.x] = p;
        }
        if (want_hll) {
            __syncthreads();
            uint8_t* dst = hll_partials + ((int64_t)s.hll_slot * gstride + blockIdx.x) * kHllRegs;
            for (int i = tid; i < kHllRegs; i += kBlock) dst[i] = (uint8_t)regs[i];
        }
        __syncthreads();
    }
}

// One thread per string op: fold its slot's block partials in block order, write the dq_state.
__global__ void finalize_strings_kernel(const StrOpMap* __restrict__ ops, int nops, const StrPartial* __restrict__ partials,
                                        int nblocks, int gstride, int64_t nrows, dq_state* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nops) return;
    const StrOpMap om = ops[i];
    int64_t n = 0, mn = INT64_MAX, mx = INT64_MIN;
    int64_t dt[5] = {0, 0, 0, 0, 0};
    for (int b = 0; b < nblocks; ++b) {
        const StrPartial p = partials[(int64_t)om.slot * gstride + b];
        n += p.n;
        mn = p.minlen < mn ? p.minlen : mn;
        mx = p.maxlen > mx ? p.maxlen : mx;
        for (int k = 1; k < 5; ++k) dt[k] += p.dt[k];
    }
    dq_state* st = out + om.op;
    for (int w = 0; w < DQ_HLL_NUM_WORDS; ++w) st->u.hll.words[w] = 0;
    st->kind = om.kind;
    switch (om.kind) {
        case DQ_OP_MIN_LENGTH:
            st->u.dbl.value = (double)mn;
            st->present = n > 0;
            break;
        case DQ_OP_MAX_LENGTH:
            st->u.dbl.value = (double)mx;
            st->present = n > 0;
            break;
        default: {  // DQ_OP_DATATYPE: the UDAF buffer is never NULL; rows outside where / NULL are numNull
            st->u.datatype.num_fractional = dt[DT_FRACTIONAL];
            st->u.datatype.num_integral = dt[DT_INTEGRAL];
            st->u.datatype.num_boolean = dt[DT_BOOLEAN];
            st->u.datatype.num_string = dt[DT_STRING];
            st->u.datatype.num_null = nrows - (dt[1] + dt[2] + dt[3] + dt[4]);
            st->present = 1;
            break;
        }
    }
}

// 4 workgroups per CU (DQ_STR_WG_PER_CU: 8, twice the resident waves, measured 2-3 % slower on the C5 string pass,
// profiles/r03/strings_grid_ab_r03s.log).
int string_scan_grid(int cus, int64_t nrows) {
    const int per_cu = getenv("DQ_STR_WG_PER_CU") ? std::max(1, atoi(getenv("DQ_STR_WG_PER_CU"))) : 4;
    const int64_t want = (nrows + (int64_t)kBlock * kStrR - 1) / ((int64_t)kBlock * kStrR);
    const int64_t cap = (int64_t)cus * per_cu;
    return (int)(want < 1 ? 1 : (want < cap ? want : cap));
}

void launch_string_scan(const StrSlot* slots, int nslots, int64_t nrows, int grid, int gstride, StrPartial* partials,
                        uint8_t* hll_partials, hipStream_t s) {
    if (nslots == 0) return;
    hipLaunchKernelGGL(scan_strings_kernel, dim3(grid), dim3(kBlock), 0, s, slots, nslots, nrows, gstride, partials,
                       hll_partials);
}

void launch_finalize_strings(const StrOpMap* ops, int nops, const StrPartial* partials, int nblocks, int gstride,
                             int64_t nrows, dq_state* out, hipStream_t s) {
    if (nops == 0) return;
    hipLaunchKernelGGL(finalize_strings_kernel, dim3((nops + 63) / 64), dim3(64), 0, s, ops, nops, partials, nblocks,
                       gstride, nrows, out);
}

}  // namespace dq
