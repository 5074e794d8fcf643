// freq.hip — HBM-resident frequency tables for the grouping analyzers (gfx950).
//
// Replaces FrequencyBasedAnalyzer.computeFrequencies (A/GroupingAnalyzers.scala:53-79):
//   SELECT cols, COUNT(*) WHERE c1 IS NOT NULL OR ... GROUP BY cols     (+ numRows = that WHERE's count)
// and the fused aggregation over the table (runAnalyzersForParticularGrouping,
// R/AnalysisRunner.scala:480-548): #groups, #(count == 1), sum -(c/N) ln(c/N), plus Histogram's
// variant (A/Histogram.scala:54-70: every row counts, NULL is the "NullValue" group) and top-N.
//
// Table: 2^b regions x kRegion slots of 16 bytes {u64 key, u64 count} (Spark counts with Long); a key lives in
// region key & (2^b - 1) and probes linearly from its top bits. Keys:
//   * fast path (one fixed-width key column): key = mix(canonical 64-bit value), mix = the bijective
//     splitmix64 finalizer, so distinct values never collide; the one value that maps to the EMPTY
//     marker is counted in a side counter. Spark groups on binary row equality: NaN is
//     canonicalised (UnsafeRow.setDouble), -0.0 and 0.0 stay distinct.
//   * general path (several key columns or strings): a 64-bit fingerprint over (null flag, value)
//     of every key column, plus the group's smallest row index; a verification pass compares every
//     row with its group's representative row and the build is redone with a new seed if two
//     distinct keys ever shared a fingerprint, so results are exact.
// Build = partitioned aggregation, no global atomics on the hot path; b is chosen from an HLL estimate of the
// distinct keys so a region holds <= kRegionTarget of them:
//   * fast build (one fixed-width key column, >= 2^24 rows, unweighted): partition1_fast reads the rows and
//     scatters the keys into 256 partitions x 8 XCD sub-regions of fixed capacity, each 4096-key tile ordered by
//     digit in LDS and its per-digit runs reserved with one atomicAdd per digit; scatter2_fast splits every
//     partition on the next digit bits into the 2^b buckets the same way. No count pass; a bucket that would
//     overflow (heavy hitters) sends the build to the exact path;
//   * exact build (weighted, multi-column, string keys, small inputs, the fallback): extract_count (per-workgroup
//     digit histograms + sizing) -> partition1 -> count2 / scan2 / scatter2 with deterministic offsets, or compact
//     + rocPRIM radix sort on the low b bits for tables outside the two-pass range;
//   * build_kernel: one workgroup per bucket (heavy buckets split into slices) aggregates its keys in an LDS
//     table and stores region `bucket` (a slice merges into it with global atomics); a whole-bucket item also
//     writes its part of the grouping summary (#groups, #count == 1, max count, entropy terms).
// Summaries, radix-select top-N, exports, the K8 merge (weighted rebuild of both tables' pairs), MutualInformation
// (joint table + marginal lookups) and the multi-device exchange are table scans with per-workgroup partials folded
// in a fixed order (deterministic).
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <type_traits>
#include <vector>

#include <rocprim/device/device_radix_sort.hpp>

#include "dq_common.h"
#include "dq_internal.h"

using namespace dq;

namespace {

constexpr int kMaxKeys = 16;
constexpr uint64_t kEmpty = ~0ull;
constexpr int kSizingRegs = 4096;  // HLL registers used only to size the table
constexpr int kFreqBlock = 256;
constexpr int kDigitBins = 256;    // radix partition: first pass on the low 8 bits of the key
#ifndef DQ_PART_TILE
#define DQ_PART_TILE 4096
#endif
constexpr int kPartTile = DQ_PART_TILE;  // keys per workgroup tile of the partition scatters (16 per lane), general path
// fast pass 1 tile (keys per workgroup tile); measured on C4 end to end (profiles/r02/c4_p1_tile_r02bh.log):
// 2048 -> 15.2-15.5 ms, 4096 -> 13.8-13.9 ms, 8192 -> 17.5 ms
constexpr int kP1TileFast = 4096;
// (r06: 4096 keys, 16 per lane, half the LDS and fewer VGPRs: C4 13.9 -> 14.3 ms, profiles/r06/c4_p2_tile_ab_r06av.txt)
#ifndef DQ_P2_TILE
#define DQ_P2_TILE 8192
#endif
constexpr int kPartTileFast = DQ_P2_TILE;  // second pass, fast path: 32 per lane, so a tile's 256 per-digit runs average 256 B
                                   // (measured: scatter2 5.85 -> 4.88 ms on C4; partition1 slows down at 8192)
constexpr int kPass2Item = 65536;  // keys per work item of the second partition pass
constexpr int kScanBlocks = 1024;  // workgroups of the table-scan kernels (upper bound: the scratch is sized for it)

// Grid of the summary / MutualInformation table scans. The sums are exact fixed point (SummaryPartial), so any
// grid gives the same bits; DQ_FREQ_SUMMARY_GRID (1..kScanBlocks) changes it to prove that (tests/).
int summary_grid() {
    const char* e = getenv("DQ_FREQ_SUMMARY_GRID");
    const int v = e ? atoi(e) : kScanBlocks;
    return v >= 1 && v <= kScanBlocks ? v : kScanBlocks;
}
constexpr int kRegion = 4096;      // slots per bucket region (the LDS table of one workgroup)
// Distinct keys per bucket the bucket count aims at (load <= ~0.63). rocPRIM sorts 8 bits per pass
// on gfx950, so 1e8 distinct keys take b = 16 (2 passes) rather than 17 (3 passes). (Measured on C4: a
// target of 3200 -- b = 15, load 0.75 -- halves the table but the LDS probing makes the build 3.2 -> 4.5 ms.)
constexpr int kRegionTarget = 2600;
constexpr int64_t kSliceRows = 1 << 18;  // rows per build work item (larger buckets are split)

struct KeyCol {
    const void* values;
    const uint8_t* validity;
    const int32_t* offsets;
    const int64_t* offsets64;  // DQ_COL_OFFSETS64: int64 offsets instead (a column past 2^31 bytes)
    int32_t spark_type;
    int32_t elem;
    // dq_frequencies_parts: rows >= split live in a second part (its own buffers, its row split + i); 0 = one part
    int64_t split;
    const void* values2;
    const uint8_t* validity2;
    const int32_t* offsets2;
};

// Row r's UTF-8 bytes of a string key column: start pointer and length.
__host__ __device__ __forceinline__ const uint8_t* str_span(const KeyCol& c, int64_t r, int& len) {
    int64_t o0, o1;
    if (c.split && r >= c.split) {  // the second part (int32 offsets of its own)
        const int64_t q = r - c.split;
        o0 = c.offsets2[q];
        len = (int)(c.offsets2[q + 1] - o0);
        return static_cast<const uint8_t*>(c.values2) + o0;
    }
    if (c.offsets64) {
        o0 = c.offsets64[r];
        o1 = c.offsets64[r + 1];
    } else {
        o0 = c.offsets[r];
        o1 = c.offsets[r + 1];
    }
    len = (int)(o1 - o0);
    return static_cast<const uint8_t*>(c.values) + o0;
}

struct KeySpec {
    KeyCol cols[kMaxKeys];
    int32_t ncols;
    int32_t fast;          // single fixed-width key column
    int32_t include_nulls; // Histogram semantics
    int32_t string_null_is_value;  // Histogram on a string column: NULL == "NullValue"
    uint64_t seed;         // fingerprint seed (general path)
    const long long* weights;  // per-row counts (pre-aggregated (key, count) input), nullptr = 1 per row
    uint64_t fp_mask;      // general-path fingerprint bits kept (~0; the collision tests narrow it: DQ_FREQ_FP_MASK)
};

// A group: 64-bit key and its 64-bit count (Spark counts with Long: a key seen >= 2^32 times is exact).
struct Slot {
    unsigned long long key;
    unsigned long long count;
};

__device__ __forceinline__ unsigned long long row_weight(const KeySpec& ks, int64_t r) {
    return ks.weights ? (unsigned long long)ks.weights[r] : 1ull;
}

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

__host__ __device__ constexpr uint64_t mul_inverse(uint64_t a) {  // a^-1 mod 2^64 for odd a (Newton)
    uint64_t x = a;
    for (int i = 0; i < 6; ++i) x *= 2 - a * x;
    return x;
}

__host__ __device__ __forceinline__ uint64_t unxorshift(uint64_t z, int s) {
    uint64_t x = z;
    for (int i = 0; i < 64 / s + 1; ++i) x = z ^ (x >> s);
    return x;
}

// Inverse of mix64: the canonical value behind a fast-path key.
__host__ __device__ __forceinline__ uint64_t unmix64(uint64_t z) {
    constexpr uint64_t i2 = mul_inverse(0x94D049BB133111EBULL), i1 = mul_inverse(0xBF58476D1CE4E5B9ULL);
    z = unxorshift(z, 31);
    z *= i2;
    z = unxorshift(z, 27);
    z *= i1;
    z = unxorshift(z, 30);
    return z;
}

// Probe start of a key inside its region: its top bits (the region is chosen by the low bits).
__device__ __forceinline__ unsigned int region_probe(uint64_t h) { return (unsigned int)(h >> 52) & (kRegion - 1); }

__device__ __forceinline__ bool is_valid(const KeyCol& c, int64_t r) {
    if (c.split && r >= c.split) {
        r -= c.split;
        return c.validity2 == nullptr || ((c.validity2[r >> 3] >> (r & 7)) & 1);
    }
    return c.validity == nullptr || ((c.validity[r >> 3] >> (r & 7)) & 1);
}

// Canonical 64-bit value of a fixed-width cell (the grouping equality of Spark's UnsafeRow bytes).
__device__ __forceinline__ uint64_t canonical(const KeyCol& c, int64_t r) {
    const void* vals = c.values;
    if (c.split && r >= c.split) {
        r -= c.split;
        vals = c.values2;
    }
    switch (c.elem) {
        case ET_U8: return static_cast<const uint8_t*>(vals)[r] ? 1ull : 0ull;
        case ET_I8: return (uint64_t)(int64_t) static_cast<const int8_t*>(vals)[r];
        case ET_I16: return (uint64_t)(int64_t) static_cast<const int16_t*>(vals)[r];
        case ET_I32: return (uint64_t)(int64_t) static_cast<const int32_t*>(vals)[r];
        case ET_F32: return (uint64_t)float_to_int_bits(static_cast<const float*>(vals)[r]);
        case ET_F64: return double_to_long_bits(static_cast<const double*>(vals)[r]);
        default: return static_cast<const uint64_t*>(vals)[r];
    }
}

__device__ __constant__ const uint8_t kNullValue[9] = {'N', 'u', 'l', 'l', 'V', 'a', 'l', 'u', 'e'};

// Little-endian loads of string bytes through aligned dwords (a lane's byte-by-byte loads were the general path's
// bottleneck); only dwords holding at least one byte of [p, p + n) are read, so nothing past a buffer is touched.
__device__ __forceinline__ uint32_t dw_at(const uint8_t* a) { return *reinterpret_cast<const uint32_t*>(a); }

__device__ __forceinline__ uint64_t dev_le64(const uint8_t* p) {  // 8 readable bytes at p
    const uint8_t* a = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(p) & ~(uintptr_t)3);
    const int sh = (int)(p - a) * 8;
    const uint32_t w0 = dw_at(a), w1 = dw_at(a + 4);
    if (!sh) return (uint64_t)w0 | ((uint64_t)w1 << 32);
    const uint32_t w2 = dw_at(a + 8);
    const uint64_t lo = ((uint64_t)w1 << 32 | w0) >> sh, hi = ((uint64_t)w2 << 32 | w1) >> sh;
    return (lo & 0xFFFFFFFFull) | (hi << 32);
}

__device__ __forceinline__ uint32_t dev_le32(const uint8_t* p) {  // 4 readable bytes at p
    const uint8_t* a = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(p) & ~(uintptr_t)3);
    const int sh = (int)(p - a) * 8;
    const uint32_t w0 = dw_at(a);
    if (!sh) return w0;
    return (uint32_t)((((uint64_t)dw_at(a + 4) << 32) | w0) >> sh);
}

// xxh_bytes (dq_common.h) with the loads above: the same hash.
__device__ uint64_t dev_xxh_bytes(const uint8_t* p, int64_t len, uint64_t seed) {
    const uint8_t* end = p + len;
    uint64_t h;
    if (len >= 32) {
        const uint8_t* limit = end - 32;
        uint64_t v1 = seed + P64_1 + P64_2, v2 = seed + P64_2, v3 = seed, v4 = seed - P64_1;
        do {
            v1 = xxh_round(v1, dev_le64(p));
            v2 = xxh_round(v2, dev_le64(p + 8));
            v3 = xxh_round(v3, dev_le64(p + 16));
            v4 = xxh_round(v4, dev_le64(p + 24));
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
    while (p + 8 <= end) {
        h ^= xxh_round(0, dev_le64(p));
        h = rotl64(h, 27) * P64_1 + P64_4;
        p += 8;
    }
    if (p + 4 <= end) {
        h ^= (uint64_t)dev_le32(p) * P64_1;
        h = rotl64(h, 23) * P64_2 + P64_3;
        p += 4;
    }
    while (p < end) {
        h ^= (uint64_t)(*p) * P64_5;
        h = rotl64(h, 11) * P64_1;
        ++p;
    }
    return xxh_fmix(h);
}

// Key of row r: returns false when the row does not take part (all key columns NULL, grouping
// semantics); `null_group` = the row belongs to the fast path's NULL group (Histogram semantics).
__device__ __forceinline__ bool row_key(const KeySpec& ks, int64_t r, uint64_t& h, bool& null_group) {
    null_group = false;
    if (ks.fast) {
        const KeyCol& c = ks.cols[0];
        if (!is_valid(c, r)) {
            if (!ks.include_nulls) return false;
            null_group = true;
            return true;
        }
        h = mix64(canonical(c, r));
        return true;
    }
    bool any = false;
    uint64_t acc = ks.seed;
    for (int i = 0; i < ks.ncols; ++i) {
        const KeyCol& c = ks.cols[i];
        uint64_t ch;
        if (is_valid(c, r)) {
            any = true;
            if (c.spark_type == DQ_TYPE_STRING) {
                int len;
                const uint8_t* p = str_span(c, r, len);
                ch = dev_xxh_bytes(p, len, ks.seed);
            } else {
                ch = xxh_long(canonical(c, r), ks.seed);
            }
        } else if (ks.string_null_is_value) {
            any = true;
            ch = xxh_bytes(kNullValue, 9, ks.seed);
        } else {
            ch = 0x6A09E667F3BCC909ULL;  // NULL component
        }
        acc = mix64(acc + P64_1 * (uint64_t)(i + 1) + ch);
    }
    if (!any && !ks.include_nulls) return false;
    h = (acc == kEmpty ? kEmpty - 1 : acc) & ks.fp_mask;
    return true;
}

// Exact equality of two rows' keys (null-safe, A/GroupingAnalyzers.scala:149-151).
__device__ bool rows_equal(const KeySpec& ks, int64_t a, int64_t b) {
    for (int i = 0; i < ks.ncols; ++i) {
        const KeyCol& c = ks.cols[i];
        bool va = is_valid(c, a), vb = is_valid(c, b);
        if (c.spark_type == DQ_TYPE_STRING) {
            const uint8_t* pa;
            const uint8_t* pb;
            int la, lb;
            if (va) { pa = str_span(c, a, la); }
            else if (ks.string_null_is_value) { pa = kNullValue; la = 9; va = true; }
            else { pa = nullptr; la = 0; }
            if (vb) { pb = str_span(c, b, lb); }
            else if (ks.string_null_is_value) { pb = kNullValue; lb = 9; vb = true; }
            else { pb = nullptr; lb = 0; }
            if (va != vb) return false;
            if (!va) continue;
            if (la != lb) return false;
            int k = 0;
            for (; k + 8 <= la; k += 8)
                if (dev_le64(pa + k) != dev_le64(pb + k)) return false;
            if (k + 4 <= la) {
                if (dev_le32(pa + k) != dev_le32(pb + k)) return false;
                k += 4;
            }
            for (; k < la; ++k)
                if (pa[k] != pb[k]) return false;
        } else {
            if (va != vb) return false;
            if (va && canonical(c, a) != canonical(c, b)) return false;
        }
    }
    return true;
}

// ---- build counters --------------------------------------------------------------------------------
struct Counters {
    unsigned long long num_rows;   // rows taking part (numRows)
    unsigned long long sentinel;   // fast path: rows whose mixed key equals kEmpty
    unsigned long long nulls;      // fast path + include_nulls: NULL rows
    unsigned long long overflow;   // probe limit hit: rebuild bigger
    unsigned long long mismatch;   // general path verification: fingerprint collisions
    unsigned long long pad[3];     // [0] [1] fast path spill overflow; [2] general count pass: string keys > 15 bytes
    unsigned long long narrow_miss;  // fast path, narrow keys: 8-byte keys outside the 32-bit window
    unsigned long long spilled;      // fast path: keys past a full bucket, appended to the spill buffer
};

__device__ __forceinline__ unsigned long long block_sum_u64(unsigned long long v, unsigned long long* lds4) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    if ((threadIdx.x & 63) == 0) lds4[threadIdx.x >> 6] = v;
    __syncthreads();
    unsigned long long s = 0;
    if (threadIdx.x == 0)
        for (int w = 0; w < kFreqBlock / 64; ++w) s += lds4[w];
    __syncthreads();
    return s;
}

// General path: every row must equal its group's representative row.
__global__ void __launch_bounds__(kFreqBlock)
verify_kernel(KeySpec ks, int64_t nrows, const Slot* __restrict__ slots, const unsigned long long* __restrict__ reps,
              int bits, Counters* __restrict__ ctr) {
    __shared__ unsigned long long red[kFreqBlock / 64];
    unsigned long long bad = 0;
    const int64_t stride = (int64_t)gridDim.x * kFreqBlock;
    for (int64_t r = (int64_t)blockIdx.x * kFreqBlock + threadIdx.x; r < nrows; r += stride) {
        uint64_t h;
        bool ng;
        if (!row_key(ks, r, h, ng) || ng || h == kEmpty) continue;
        const uint64_t base = (h & ((1ull << bits) - 1)) * kRegion;
        unsigned int p = region_probe(h);
        bool found = false;
        for (int probe = 0; probe < kRegion; ++probe) {
            const uint64_t pos = base + p;
            if (slots[pos].key == h) {
                // a group's representative is its own smallest row: no bytes to compare (most rows of a
                // high-cardinality key)
                const int64_t rep = (int64_t)reps[pos];
                if (rep != r && !rows_equal(ks, r, rep)) ++bad;
                found = true;
                break;
            }
            if (slots[pos].key == kEmpty) break;
            p = (p + 1) & (kRegion - 1);
        }
        if (!found) ++bad;
    }
    bad = block_sum_u64(bad, red);
    if (threadIdx.x == 0 && bad) atomicAdd(&ctr->mismatch, bad);
}

// ---- partitioned build ---------------------------------------------------------------------------
// Pass 1a (count): over a contiguous chunk of rows per workgroup, the side counters, the sizing HLL
// and the number of rows whose key goes to the table (per workgroup, for the write offsets).
__device__ __forceinline__ void chunk_of(int64_t nrows, int64_t& r0, int64_t& r1) {
    const int64_t per = (nrows + gridDim.x - 1) / gridDim.x;
    r0 = (int64_t)blockIdx.x * per;
    r1 = r0 + per < nrows ? r0 + per : nrows;
    if (r0 > nrows) r0 = nrows;
}

// One string key column: a key of <= 15 bytes as two exact words (see the small build below).
constexpr uint64_t kTupleNull = ~0ull, kTupleLong = ~0ull - 1;
__device__ __forceinline__ bool short_key_tuple(const KeySpec& ks, int64_t r, uint64_t& b0, uint64_t& b1) {
    const KeyCol& c = ks.cols[0];
    if (!is_valid(c, r)) {
        if (ks.string_null_is_value) {  // "NullValue"
            b0 = 0x756C61566C6C754EULL;
            b1 = 0x65ull | (9ull << 56);
        } else {
            b0 = b1 = kTupleNull;
        }
        return true;
    }
    int len;
    const uint8_t* p = str_span(c, r, len);
    if (len > 15) {
        b0 = b1 = kTupleLong;
        return false;
    }
    const uint8_t* a = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(p) & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(p - a);
    const int ndw = (int)((sh + (uint32_t)len + 3) >> 2);  // only dwords holding bytes of [p, p + len): <= 5
    uint32_t w[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) w[k] = k < ndw ? dw_at(a + 4 * k) : 0u;
    uint64_t x0 = (uint64_t)__builtin_amdgcn_alignbyte(w[1], w[0], sh) |
                  ((uint64_t)__builtin_amdgcn_alignbyte(w[2], w[1], sh) << 32);
    uint64_t x1 = (uint64_t)__builtin_amdgcn_alignbyte(w[3], w[2], sh) |
                  ((uint64_t)__builtin_amdgcn_alignbyte(w[4], w[3], sh) << 32);
    if (len < 8) {
        x0 &= len ? (~0ull >> (64 - 8 * len)) : 0ull;
        x1 = 0;
    } else {
        x1 &= len > 8 ? (~0ull >> (64 - 8 * (len - 8))) : 0ull;
    }
    b0 = x0;
    b1 = x1 | ((uint64_t)len << 56);
    return true;
}

__global__ void __launch_bounds__(kFreqBlock)
extract_count_kernel(KeySpec ks, int64_t nrows, unsigned long long* __restrict__ block_keep,
                     uint8_t* __restrict__ regs_part, Counters* __restrict__ ctr, unsigned int* __restrict__ hist1,
                     int tile_rows, unsigned long long* __restrict__ hrow, unsigned long long* __restrict__ tup) {
    __shared__ unsigned int lds[kSizingRegs];
    __shared__ unsigned int dh[kDigitBins];
    __shared__ unsigned long long red[kFreqBlock / 64];
    for (int i = threadIdx.x; i < kSizingRegs; i += kFreqBlock) lds[i] = 0;
    for (int i = threadIdx.x; i < kDigitBins; i += kFreqBlock) dh[i] = 0;
    __syncthreads();
    unsigned long long taken = 0, sent = 0, nulls = 0, kept = 0, longk = 0;
    constexpr int U = 4;  // rows in flight per lane
    // tiles of kPartTile rows interleaved over the workgroups (tile g, g + G, ...): all workgroups stream
    // through one narrow address window, as the partition scatter that replays the same tiles does
    const int64_t ntiles = (nrows + tile_rows - 1) / tile_rows;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x)
    for (int64_t rb = tile * tile_rows + threadIdx.x, r1 = min((tile + 1) * (int64_t)tile_rows, nrows); rb < r1;
         rb += (int64_t)kFreqBlock * U) {
        uint64_t hv[U];
        bool ok[U], ngv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t r = rb + (int64_t)u * kFreqBlock;
            ngv[u] = false;
            hv[u] = 0;
            ok[u] = r < r1 && row_key(ks, r, hv[u], ngv[u]);
        }
        if (hrow)  // each row's key for the partition pass (kEmpty: the row takes no part in the table)
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t r = rb + (int64_t)u * kFreqBlock;
                if (r < r1) hrow[r] = ok[u] && !ngv[u] ? hv[u] : kEmpty;
            }
        if (tup)  // one string key column: each row's key as two exact words (kTupleLong past 15 bytes) for the checks
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t r = rb + (int64_t)u * kFreqBlock;
                if (r < r1 && ok[u] && !ngv[u]) {
                    uint64_t b0, b1;
                    short_key_tuple(ks, r, b0, b1);
                    tup[2 * r] = b0;
                    tup[2 * r + 1] = b1;
                    longk += b1 == kTupleLong;
                }
            }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!ok[u]) continue;
            const unsigned long long w = row_weight(ks, rb + (int64_t)u * kFreqBlock);
            taken += w;
            if (ngv[u]) { nulls += w; continue; }
            const uint64_t h = hv[u];
            if (h == kEmpty) { sent += w; continue; }
            ++kept;
            // h is already a mixed 64-bit key (splitmix64 finalizer / fingerprint): use its bits directly
            const unsigned int idx = (unsigned int)(h >> 52);
            const unsigned int rank = (unsigned int)__clzll((long long)((h << 12) | (1ull << 11))) + 1u;
            if (rank > lds[idx]) atomicMax(&lds[idx], rank);
            if (hist1) atomicAdd(&dh[(unsigned int)h & (kDigitBins - 1)], 1u);
        }
    }
    taken = block_sum_u64(taken, red);
    sent = block_sum_u64(sent, red);
    nulls = block_sum_u64(nulls, red);
    kept = block_sum_u64(kept, red);
    if (tup) longk = block_sum_u64(longk, red);
    if (threadIdx.x == 0) {
        block_keep[blockIdx.x] = kept;
        if (taken) atomicAdd(&ctr->num_rows, taken);
        if (sent) atomicAdd(&ctr->sentinel, sent);
        if (nulls) atomicAdd(&ctr->nulls, nulls);
        if (longk) atomicAdd(&ctr->pad[2], longk);
    }
    // this workgroup's sizing registers, one byte each; sizing_reduce_kernel takes the max over workgroups
    // (a global atomicMax per register per workgroup contends on 4096 addresses)
    for (int i = threadIdx.x; i < kSizingRegs / 4; i += kFreqBlock) {
        const unsigned int w = lds[4 * i] | (lds[4 * i + 1] << 8) | (lds[4 * i + 2] << 16) | (lds[4 * i + 3] << 24);
        reinterpret_cast<unsigned int*>(regs_part + (uint64_t)blockIdx.x * kSizingRegs)[i] = w;
    }
    if (hist1)
        for (int i = threadIdx.x; i < kDigitBins; i += kFreqBlock) hist1[(uint64_t)blockIdx.x * kDigitBins + i] = dh[i];
}

// Max over workgroups of the per-workgroup sizing registers: grid (kSizingRegs / 256, G), each thread
// folds a run of workgroups for one register.
__global__ void __launch_bounds__(256)
sizing_reduce_kernel(const uint8_t* __restrict__ regs_part, int ngroups, int nregs, unsigned int* __restrict__ regs) {
    const int reg = blockIdx.x * 256 + threadIdx.x;
    const int per = (ngroups + gridDim.y - 1) / gridDim.y;
    const int g0 = blockIdx.y * per, g1 = min(ngroups, g0 + per);
    unsigned int m = 0;
    for (int g = g0; g < g1; ++g) m = max(m, (unsigned int)regs_part[(uint64_t)g * nregs + reg]);
    if (m) atomicMax(&regs[reg], m);
}

// Pass 1b (write): the same tiles again; keys (and row indices) compacted in tile order at the
// workgroup's offset — no shared counter, deterministic layout.
__global__ void __launch_bounds__(kFreqBlock)
extract_write_kernel(KeySpec ks, int64_t nrows, const unsigned long long* __restrict__ block_off,
                     unsigned long long* __restrict__ hs, unsigned long long* __restrict__ rows, int tile_rows) {
    __shared__ unsigned int wave_cnt[kFreqBlock / 64];
    unsigned long long base = block_off[blockIdx.x];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t ntiles = (nrows + tile_rows - 1) / tile_rows;  // the count pass's tiles
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x)
    for (int64_t t0 = tile * tile_rows, r1 = min(t0 + (int64_t)tile_rows, nrows); t0 < r1; t0 += kFreqBlock) {
        const int64_t r = t0 + threadIdx.x;
        uint64_t h = 0;
        bool ng = false;
        const bool keep = r < r1 && row_key(ks, r, h, ng) && !ng && h != kEmpty;
        const unsigned long long bal = __ballot(keep);
        if (lane == 0) wave_cnt[wave] = (unsigned int)__popcll(bal);
        __syncthreads();
        unsigned long long off = base, tile = 0;
        for (int w = 0; w < kFreqBlock / 64; ++w) {
            if (w < wave) off += wave_cnt[w];
            tile += wave_cnt[w];
        }
        if (keep) {
            const unsigned long long at = off + __popcll(bal & ((1ull << lane) - 1ull));
            hs[at] = h;
            if (rows) rows[at] = (unsigned long long)r;
        }
        base += tile;
        __syncthreads();
    }
}

// bounds[b] = first index of bucket b in the keys sorted on their low `bits` bits.
__global__ void bucket_bounds_kernel(const unsigned long long* __restrict__ hs, uint64_t n, int bits, uint64_t nbuckets,
                                     unsigned long long* __restrict__ bounds) {
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b > nbuckets) return;
    if (b == nbuckets) { bounds[b] = n; return; }
    if (bits == 0) { bounds[b] = 0; return; }
    const uint64_t mask = nbuckets - 1;
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if ((hs[mid] & mask) < b) lo = mid + 1; else hi = mid;
    }
    bounds[b] = lo;
}


// ---- radix partition (replaces extract-write + a device radix sort) -------------------------------
// Pass 1 scatters every kept key into one of 256 partitions by its low 8 bits, straight from the rows
// (the count pass above already produced each workgroup's per-digit counts). Pass 2 splits each
// partition by the next (bits - 8) bits. Both scatters stage a 4096-key tile in LDS ordered by digit, so
// the global writes are runs per digit rather than single scattered words. Within a digit the order is
// the arrival order through LDS atomics — irrelevant to the per-bucket aggregation that follows.

// Per digit d: exclusive prefix over workgroups of hist[g][d] -> off[g][d], and the digit total.
__global__ void __launch_bounds__(256)
digit_scan_kernel(const unsigned int* __restrict__ hist, int ngroups, int nbins, unsigned long long* __restrict__ off,
                  unsigned long long* __restrict__ totals) {
    __shared__ unsigned long long part[256];
    const int d = blockIdx.x;
    // each thread owns a contiguous run of groups
    const int per = (ngroups + 255) / 256;
    const int g0 = threadIdx.x * per, g1 = min(ngroups, g0 + per);
    unsigned long long sum = 0;
    for (int g = g0; g < g1; ++g) sum += hist[(uint64_t)g * nbins + d];
    part[threadIdx.x] = sum;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {  // inclusive Hillis-Steele scan over the 256 thread sums
        const unsigned long long v = threadIdx.x >= o ? part[threadIdx.x - o] : 0ull;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    unsigned long long run = threadIdx.x ? part[threadIdx.x - 1] : 0ull;
    for (int g = g0; g < g1; ++g) {
        off[(uint64_t)g * nbins + d] = run;
        run += hist[(uint64_t)g * nbins + d];
    }
    if (threadIdx.x == 255) totals[d] = part[255];
}

// One tile (<= kPartTile keys in registers, digit per key) -> LDS staging ordered by digit -> global
// runs at cursor[digit]. `bins` <= BINS. Returns after the cursors advanced.
template <int BINS, bool GENERAL, int TILE>
__device__ __forceinline__ void scatter_tile(const uint64_t (&h)[TILE / kFreqBlock],
                                             const uint64_t (&rw)[TILE / kFreqBlock], const bool (&keep)[TILE / kFreqBlock],
                                             int shift, unsigned int mask, unsigned int* hist, unsigned int* start,
                                             unsigned long long* cursor, unsigned long long* sh, unsigned long long* sr,
                                             unsigned long long* __restrict__ out_h, unsigned long long* __restrict__ out_r) {
    constexpr int PER = TILE / kFreqBlock;
    unsigned int rank[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j)
        rank[j] = keep[j] ? atomicAdd(&hist[(unsigned int)(h[j] >> shift) & mask], 1u) : 0u;
    __syncthreads();
    // exclusive scan of hist -> start: each thread sums a run of BINS / 256 bins, wave-level inclusive
    // scan of the run sums (shuffles), then the 4 wave totals
    constexpr int RUN = BINS / kFreqBlock > 0 ? BINS / kFreqBlock : 1;
    __shared__ unsigned int wsum[kFreqBlock / 64];
    unsigned int total;
    {
        const int b0 = threadIdx.x * RUN;
        unsigned int acc = 0;
#pragma unroll
        for (int b = 0; b < RUN; ++b) acc += hist[b0 + b];
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        unsigned int inc = acc;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned int v = __shfl_up(inc, o, 64);
            if (lane >= o) inc += v;
        }
        if (lane == 63) wsum[wave] = inc;
        __syncthreads();
        unsigned int run = inc - acc;
        total = 0;
#pragma unroll
        for (int w = 0; w < kFreqBlock / 64; ++w) {
            if (w < wave) run += wsum[w];
            total += wsum[w];
        }
#pragma unroll
        for (int b = 0; b < RUN; ++b) {
            start[b0 + b] = run;
            run += hist[b0 + b];
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        if (!keep[j]) continue;
        const unsigned int at = start[(unsigned int)(h[j] >> shift) & mask] + rank[j];
        sh[at] = h[j];
        if (GENERAL) sr[at] = rw[j];
    }
    __syncthreads();
    for (unsigned int i = threadIdx.x; i < total; i += kFreqBlock) {
        const unsigned long long hv = sh[i];
        const unsigned int d = (unsigned int)(hv >> shift) & mask;
        const unsigned long long pos = cursor[d] + (i - start[d]);
        out_h[pos] = hv;
        if (GENERAL) out_r[pos] = sr[i];
    }
    __syncthreads();
    for (int b = threadIdx.x; b < BINS; b += kFreqBlock) {
        cursor[b] += hist[b];
        hist[b] = 0;
    }
    __syncthreads();
}

// Pass 1: rows -> 256 partitions (same workgroup chunks as extract_count_kernel).
template <bool GENERAL, int TILE>
__global__ void __launch_bounds__(kFreqBlock)
partition1_kernel(KeySpec ks, int64_t nrows, const unsigned long long* __restrict__ off1,
                  const unsigned long long* __restrict__ totals, unsigned long long* __restrict__ out_h,
                  unsigned long long* __restrict__ out_r, const unsigned long long* __restrict__ hrow) {
    constexpr int PER = TILE / kFreqBlock;
    __shared__ unsigned int hist[kDigitBins], start[kDigitBins];
    __shared__ unsigned long long cursor[kDigitBins];
    __shared__ unsigned long long sh[TILE];
    __shared__ unsigned long long sr[GENERAL ? TILE : 1];
    {
        // cursor[d] = (exclusive scan of the digit totals)[d] + this workgroup's offset inside digit d
        __shared__ unsigned long long tot[kDigitBins];
        tot[threadIdx.x] = totals[threadIdx.x];
        hist[threadIdx.x] = 0;
        __syncthreads();
        for (int o = 1; o < kDigitBins; o <<= 1) {
            const unsigned long long v = threadIdx.x >= o ? tot[threadIdx.x - o] : 0ull;
            __syncthreads();
            tot[threadIdx.x] += v;
            __syncthreads();
        }
        cursor[threadIdx.x] = (threadIdx.x ? tot[threadIdx.x - 1] : 0ull) + off1[(uint64_t)blockIdx.x * kDigitBins + threadIdx.x];
        __syncthreads();
    }
    const int64_t ntiles = (nrows + TILE - 1) / TILE;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t t0 = tile * TILE, r1 = min(t0 + (int64_t)TILE, nrows);
        uint64_t h[PER], rw[PER];
        bool keep[PER];
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int64_t r = t0 + (int64_t)j * kFreqBlock + threadIdx.x;
            if (!GENERAL) {  // one fixed-width key column: its mixed canonical value (row_key's fast path)
                const KeyCol& c = ks.cols[0];
                const bool in = r < r1 && is_valid(c, r);
                h[j] = in ? mix64(canonical(c, r)) : kEmpty;
                keep[j] = in && h[j] != kEmpty;
                rw[j] = 0;
                continue;
            }
            rw[j] = (unsigned long long)r;
            if (hrow) {  // the keys the count pass wrote: no second read and hash of the key columns
                h[j] = r < r1 ? hrow[r] : kEmpty;
                keep[j] = h[j] != kEmpty;
                continue;
            }
            bool ng = false;
            h[j] = 0;
            keep[j] = r < r1 && row_key(ks, r, h[j], ng) && !ng && h[j] != kEmpty;
        }
        scatter_tile<kDigitBins, GENERAL, TILE>(h, rw, keep, 0, kDigitBins - 1, hist, start, cursor, sh, sr, out_h, out_r);
    }
}

struct Pass2Item {
    unsigned long long begin, end;  // range in the pass-1 output (inside one partition)
};

// Pass 2 count: per work item, histogram of the second digit.
template <int BINS>
__global__ void __launch_bounds__(kFreqBlock)
count2_kernel(const Pass2Item* __restrict__ items, const unsigned long long* __restrict__ hs, int shift, unsigned int mask,
              unsigned int* __restrict__ cnt) {
    __shared__ unsigned int hist[BINS];
    for (int b = threadIdx.x; b < BINS; b += kFreqBlock) hist[b] = 0;
    __syncthreads();
    const Pass2Item it = items[blockIdx.x];
    for (unsigned long long i = it.begin + threadIdx.x; i < it.end; i += kFreqBlock)
        atomicAdd(&hist[(unsigned int)(hs[i] >> shift) & mask], 1u);
    __syncthreads();
    for (int b = threadIdx.x; b < BINS; b += kFreqBlock) cnt[(uint64_t)blockIdx.x * BINS + b] = hist[b];
}

// Pass 2 offsets, one workgroup per partition: for each bin, exclusive prefix over the partition's items;
// bins laid out in order inside the partition. Writes off[item][bin] (absolute) and each bucket's range
// (bucket = partition + 256 * bin, i.e. the low `bits` bits of its keys).
template <int BINS>
__global__ void __launch_bounds__(kFreqBlock)
scan2_kernel(const unsigned int* __restrict__ cnt, const int* __restrict__ part_items, const unsigned long long* __restrict__ part_begin,
             int nbins, unsigned long long* __restrict__ off, unsigned long long* __restrict__ bstart,
             unsigned long long* __restrict__ bcount) {
    __shared__ unsigned long long tot[BINS];
    __shared__ unsigned long long runsum[kFreqBlock];
    const int p = blockIdx.x;
    const int i0 = part_items[p], i1 = part_items[p + 1];
    for (int b = threadIdx.x; b < nbins; b += kFreqBlock) {
        unsigned long long run = 0;
        for (int i = i0; i < i1; ++i) {
            const unsigned int c = cnt[(uint64_t)i * BINS + b];
            off[(uint64_t)i * BINS + b] = run;
            run += c;
        }
        tot[b] = run;
    }
    __syncthreads();
    constexpr int RUN = BINS / kFreqBlock > 0 ? BINS / kFreqBlock : 1;
    const int b0 = threadIdx.x * RUN;
    unsigned long long acc = 0;
    for (int b = b0; b < b0 + RUN && b < nbins; ++b) acc += tot[b];
    runsum[threadIdx.x] = acc;
    __syncthreads();
    for (int o = 1; o < kFreqBlock; o <<= 1) {
        const unsigned long long v = threadIdx.x >= o ? runsum[threadIdx.x - o] : 0ull;
        __syncthreads();
        runsum[threadIdx.x] += v;
        __syncthreads();
    }
    unsigned long long base = part_begin[p] + (threadIdx.x ? runsum[threadIdx.x - 1] : 0ull);
    for (int b = b0; b < b0 + RUN && b < nbins; ++b) {
        const uint64_t bucket = (uint64_t)p + (uint64_t)kDigitBins * b;
        bstart[bucket] = base;
        bcount[bucket] = tot[b];
        for (int i = i0; i < i1; ++i) off[(uint64_t)i * BINS + b] += base;
        base += tot[b];
    }
}

// Pass 2 scatter: per work item, keys (and rows) -> their bucket's range.
template <int BINS, bool GENERAL, int TILE>
__global__ void __launch_bounds__(kFreqBlock)
scatter2_kernel(const Pass2Item* __restrict__ items, const unsigned long long* __restrict__ off, const unsigned long long* __restrict__ in_h,
                const unsigned long long* __restrict__ in_r, int shift, unsigned int mask, unsigned long long* __restrict__ out_h,
                unsigned long long* __restrict__ out_r) {
    constexpr int PER = TILE / kFreqBlock;
    __shared__ unsigned int hist[BINS], start[BINS];
    __shared__ unsigned long long cursor[BINS];
    __shared__ unsigned long long sh[TILE];
    __shared__ unsigned long long sr[GENERAL ? TILE : 1];
    const Pass2Item it = items[blockIdx.x];
    for (int b = threadIdx.x; b < BINS; b += kFreqBlock) {
        hist[b] = 0;
        cursor[b] = off[(uint64_t)blockIdx.x * BINS + b];
    }
    __syncthreads();
    for (unsigned long long t0 = it.begin; t0 < it.end; t0 += TILE) {
        uint64_t h[PER], rw[PER];
        bool keep[PER];
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const unsigned long long i = t0 + (unsigned long long)j * kFreqBlock + threadIdx.x;
            keep[j] = i < it.end;
            h[j] = keep[j] ? __builtin_nontemporal_load(&in_h[i]) : 0ull;
            rw[j] = (GENERAL && keep[j]) ? in_r[i] : 0ull;
        }
        scatter_tile<BINS, GENERAL, TILE>(h, rw, keep, shift, mask, hist, start, cursor, sh, sr, out_h, out_r);
    }
}

// ---- fast path (one fixed-width key column, unweighted): partitions of fixed capacity, runs reserved with atomics --
// Pass 1 and pass 2 of the fast path need no count pass over the keys: every bucket gets a fixed capacity (its
// expected share of the keys plus slack), and each tile reserves its per-bucket runs with one global atomicAdd
// per non-empty bucket (256 per 8 K keys at most). The order inside a bucket is then arrival order. That does not
// matter to the aggregation that follows, and the table build already takes LDS insertion order anyway.
// A bucket that would overflow its capacity raises a flag. That happens with heavy hitters: one value repeated on
// a large share of the rows. The host then redoes the build on the exactly-counted path
// (extract_count -> partition1 -> count2 / scan2 / scatter2).

constexpr int kFastRegs = 1024;  // sizing HLL registers of the fast pass 1 (1 KB per workgroup; sizing only)
constexpr int kSketchBits = 9;   // the sizing sketch samples the keys whose low 9 mixed bits are zero (1 / 512)
// Pass-1 run cursors, one per 128-byte line: every workgroup of the chip reserves on the same 256 counters, and
// atomics on one line serialise (16 counters to a line would be 16-way contention on top of the reservation's).
constexpr int kCursorStride = 16;
constexpr int kXcds = 8;  // MI355X: 8 XCDs, workgroup i runs on XCD i % 8
// (r04: splitting each (partition, XCD) sub-region 4 or 8 ways by workgroup, so fewer workgroups share a reservation
// counter, made pass 1 4.6 -> 5.1-5.2 ms on C4, profiles/r04/c4_split_ab_r04j.txt; one sub-region per XCD stays.)
constexpr int kP1Sub = kXcds;  // sub-regions per partition

// Raw bits of a W-byte cell, loaded without any branch on the element type (a runtime switch around the load
// would put a wait after every load: one row in flight per lane); canonical_of() converts after the loads.
template <int W>
__device__ __forceinline__ uint64_t load_bits(const void* values, int64_t r) {
    if (W == 8) return static_cast<const uint64_t*>(values)[r];
    if (W == 4) return static_cast<const uint32_t*>(values)[r];
    if (W == 2) return static_cast<const uint16_t*>(values)[r];
    return static_cast<const uint8_t*>(values)[r];
}

template <int W>
__device__ __forceinline__ uint64_t canonical_of(int elem, uint64_t raw) {
    if (W == 8) {
        if (elem == ET_F64) {
            const bool nan = (raw & 0x7FFFFFFFFFFFFFFFull) > 0x7FF0000000000000ull;
            return nan ? 0x7ff8000000000000ull : raw;
        }
        return raw;
    }
    if (W == 4) {
        if (elem == ET_F32) {
            const bool nan = (raw & 0x7FFFFFFFu) > 0x7F800000u;
            return nan ? 0x7fc00000ull : raw;
        }
        return (uint64_t)(int64_t)(int32_t)(uint32_t)raw;
    }
    if (W == 2) return (uint64_t)(int64_t)(int16_t)(uint16_t)raw;
    return elem == ET_U8 ? (raw ? 1ull : 0ull) : (uint64_t)(int64_t)(int8_t)(uint8_t)raw;
}

// Keys that do not fit their bucket (a key repeated more often than a bucket's slack: NaN, 0, a default value) go
// to one spill buffer as full 64-bit keys, reserved per wave; the build inserts them into the finished table with
// global atomics (spill_insert_kernel). Only a full spill buffer sends the build to the exactly-counted path.
constexpr unsigned long long kPosMask = (1ull << 48) - 1ull;  // partition-buffer positions (2^48 keys)

struct Spill {
    unsigned long long* keys;
    unsigned long long cap;
    unsigned long long* count;  // Counters::spilled
};

// One tile already in registers (h, keep) -> LDS staging ordered by digit -> global runs reserved with atomics:
// digit b's run goes to bucket k = bucket_of(b), at k * cap + atomicAdd(&gcursor[k], hist[b]); the part of a run past
// the bucket's capacity is spilled (to_key(staged word) into `sp`), and a full spill buffer raises *lovf.
// NARROW: the staged word is (digit << 32) | 32-bit payload and the payload is what goes out (narrow keys, below);
// otherwise the staged word is the key itself, its digit (key >> shift) & mask.
template <int BINS, int TILE, bool NARROW, typename BucketOf, typename CounterOf, typename Prefetch, typename OutT,
          typename ToKey>
__device__ __forceinline__ void scatter_tile_reserve(const uint64_t (&h)[TILE / kFreqBlock], unsigned int keepm,
                                                     int shift, unsigned int mask, unsigned int* hist, unsigned int* start,
                                                     unsigned long long* cursor, unsigned long long* sh,
                                                     unsigned long long* __restrict__ gcursor, unsigned long long cap,
                                                     BucketOf bucket_of, CounterOf counter_of, unsigned int* lovf,
                                                     const Spill& sp, ToKey to_key, OutT* __restrict__ out_h,
                                                     Prefetch prefetch) {
    constexpr int PER = TILE / kFreqBlock;
    static_assert(PER <= 32, "keep flags are one bit per key");
    auto digit = [shift, mask](uint64_t v) {
        return NARROW ? (unsigned int)(v >> 32) : (unsigned int)(v >> shift) & mask;
    };
    unsigned int rank[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j)
        rank[j] = ((keepm >> j) & 1u) ? atomicAdd(&hist[digit(h[j])], 1u) : 0u;
    __syncthreads();
    constexpr int RUN = BINS / kFreqBlock > 0 ? BINS / kFreqBlock : 1;
    __shared__ unsigned int wsum[kFreqBlock / 64];
    unsigned int total;
    {
        const int b0 = threadIdx.x * RUN;
        unsigned int acc = 0;
#pragma unroll
        for (int b = 0; b < RUN; ++b) acc += hist[b0 + b];
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        unsigned int inc = acc;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned int v = __shfl_up(inc, o, 64);
            if (lane >= o) inc += v;
        }
        if (lane == 63) wsum[wave] = inc;
        __syncthreads();
        unsigned int run = inc - acc;
        total = 0;
#pragma unroll
        for (int w = 0; w < kFreqBlock / 64; ++w) {
            if (w < wave) run += wsum[w];
            total += wsum[w];
        }
#pragma unroll
        for (int b = 0; b < RUN; ++b) {
            const unsigned int hb = hist[b0 + b];
            start[b0 + b] = run;
            run += hb;
            if (hb) {
                const unsigned long long k = bucket_of(b0 + b);
                const unsigned long long at = atomicAdd(&gcursor[counter_of(b0 + b)], (unsigned long long)hb);
                // staged index i of this digit lands at (k cap + at - start) + i while i < start + fit; both halves in
                // one LDS word (positions < 2^48, staged indices < 2^16), so a key needs one read to place itself
                const unsigned long long fit = at >= cap ? 0ull : (cap - at < hb ? cap - at : (unsigned long long)hb);
                const unsigned long long rel = (k * cap + at - (unsigned long long)(run - hb)) & kPosMask;
                cursor[b0 + b] = rel | ((unsigned long long)(run - hb + fit) << 48);
            }
        }
    }
    __syncthreads();  // start[] / cursor[] of every digit written before any thread places its keys
    // the next tile's loads go out only now: a wait for the reservation atomics above (vmcnt counts loads, stores
    // and atomics in order) would otherwise wait for them too
    prefetch();
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        if (!((keepm >> j) & 1u)) continue;
        sh[start[digit(h[j])] + rank[j]] = h[j];
    }
    __syncthreads();
    if (!*lovf) {  // (uniform: read after the barrier that follows every write of the flag)
        const unsigned int lane = threadIdx.x & 63;
        for (unsigned int i = threadIdx.x; i < total; i += kFreqBlock) {
            const unsigned long long hv = sh[i];
            const unsigned long long cw = cursor[digit(hv)];
            const bool fits = i < (unsigned int)(cw >> 48);
            if (fits) out_h[(cw + i) & kPosMask] = (OutT)hv;
            const unsigned long long sm = __ballot(!fits);
            if (sm) {  // wave-uniform: one reservation per wave for its spilled keys
                const int leader = __ffsll((long long)sm) - 1;
                unsigned long long base = 0;
                if ((int)lane == leader) base = atomicAdd(sp.count, (unsigned long long)__popcll(sm));
                base = __shfl(base, leader, 64);
                if (!fits) {
                    const unsigned long long at = base + __popcll(sm & ((1ull << lane) - 1ull));
                    if (at < sp.cap) sp.keys[at] = to_key(hv);
                    else *lovf = 1u;
                }
            }
        }
    }
    __syncthreads();
    for (int b = threadIdx.x; b < BINS; b += kFreqBlock) hist[b] = 0;
    __syncthreads();
}

// Narrow keys: when every key's canonical value fits 32 bits around a base (keys of <= 4-byte columns always; 8-byte
// integral keys when a sample of the column spans < 2^31), the partition buffers hold the 32-bit offset from the base
// instead of the 64-bit mixed key, and pass 2 / the build re-derive the key as mix64(base + offset): the two partition
// passes move 4 bytes per key instead of 8 in every write and every re-read. An 8-byte key outside the window raises
// Counters::narrow_miss in pass 1 and the build restarts with 64-bit keys.
struct NarrowKey {
    unsigned long long base;
    int sx;  // the offset is sign-extended (<= 4-byte signed columns)
    int pad;
};

__device__ __forceinline__ uint64_t narrow_canon(const NarrowKey& nk, uint32_t p) {
    return nk.base + (nk.sx ? (uint64_t)(int64_t)(int32_t)p : (uint64_t)p);
}

// Fast pass 1: rows -> 256 partitions x 8 XCD sub-regions of `cap` keys each (sub-region (d, x) at (8 d + x) * cap),
// plus the side counters and the sizing registers (per workgroup, reduced by sizing_reduce_kernel). W = the key
// column's cell width, FLT = FLOAT / DOUBLE cells (NaN canonical). The next tile's cells are loaded while the current
// tile is scattered (after its reservation atomics returned). (r04: lane-contiguous rows — 16 consecutive cells per
// lane as 16-byte loads at a 128-byte lane stride, the validity one 16-bit load — cut the VALU work but made the pass
// 4.8 -> 5.4 ms: 64 lines per load instruction; the coalesced layout stays.)
typedef int fq_v4i __attribute__((ext_vector_type(4)));
typedef int fq_v2i __attribute__((ext_vector_type(2)));

template <int W, bool FLT>
__device__ __forceinline__ uint64_t canonical_cell(uint64_t raw) {
    if (W == 8) {
        if (FLT) {
            const bool nan = (raw & 0x7FFFFFFFFFFFFFFFull) > 0x7FF0000000000000ull;
            return nan ? 0x7ff8000000000000ull : raw;
        }
        return raw;
    }
    if (W == 4) {
        if (FLT) {
            const bool nan = (raw & 0x7FFFFFFFu) > 0x7F800000u;
            return nan ? 0x7fc00000ull : raw;
        }
        return (uint64_t)(int64_t)(int32_t)(uint32_t)raw;
    }
    if (W == 2) return (uint64_t)(int64_t)(int16_t)(uint16_t)raw;
    return FLT ? (raw ? 1ull : 0ull) : (uint64_t)(int64_t)(int8_t)(uint8_t)raw;  // W = 1: FLT marks BOOLEAN
}

// The lane's PER = 16 rows of tile t0 (row t0 + 256 j + tid: a wave's loads are 64 consecutive cells, coalesced): raw
// cells and the validity word (bit j = row j's). A full tile takes buffer loads (the tile base in SGPRs, the row
// offset j in the scalar offset: no per-row address arithmetic); the last, partial tile reads row by row.
template <int W>
__device__ __forceinline__ void p1_load(const KeyCol& c, int64_t t0, int64_t nrows, uint64_t (&raw)[16],
                                        unsigned int& vword) {
    constexpr int TILE = 16 * kFreqBlock;
    const int64_t rem = nrows - t0;
    const int tid = (int)threadIdx.x;
    if (rem >= TILE) {
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(static_cast<const char*>(c.values) + t0 * W), (short)0, TILE * W, 0x00020000);
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int so = j * kFreqBlock * W;
            if (W == 8) {
                const fq_v2i x = __builtin_amdgcn_raw_buffer_load_b64(r, tid * 8, so, 0);
                raw[j] = ((uint64_t)(uint32_t)x.y << 32) | (uint32_t)x.x;
            } else if (W == 4) {
                raw[j] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(r, tid * 4, so, 0);
            } else if (W == 2) {
                raw[j] = (uint16_t)__builtin_amdgcn_raw_buffer_load_b16(r, tid * 2, so, 0);
            } else {
                raw[j] = (uint8_t)__builtin_amdgcn_raw_buffer_load_b8(r, tid, so, 0);
            }
        }
        if (c.validity) {
            const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(c.validity + (t0 >> 3)), (short)0, TILE / 8, 0x00020000);
            const unsigned int sh = (unsigned int)tid & 7u;
            unsigned int w = 0;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const unsigned int b = (unsigned int)__builtin_amdgcn_raw_buffer_load_b8(rv, tid >> 3, j * (kFreqBlock / 8), 0);
                w |= ((b >> sh) & 1u) << j;
            }
            vword = w;
        } else {
            vword = 0xFFFFu;
        }
        return;
    }
    vword = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int64_t r = t0 + (int64_t)j * kFreqBlock + tid;
        const bool in = r < nrows;
        raw[j] = in ? load_bits<W>(c.values, r) : 0ull;
        const bool ok = in && (!c.validity || ((c.validity[r >> 3] >> (r & 7)) & 1u));
        vword |= (ok ? 1u : 0u) << j;
    }
}

template <int TILE, int W, bool NARROW, bool FLT>
__global__ void __launch_bounds__(kFreqBlock)  // 41 KB of LDS: 3 workgroups per CU (wide keys: 167 VGPRs fit)
partition1_fast_kernel(KeyCol c, int64_t nrows, int include_nulls, unsigned long long cap,
                       unsigned long long* __restrict__ gcursor, void* __restrict__ out,
                       uint8_t* __restrict__ regs_part, Counters* __restrict__ ctr, NarrowKey nk, Spill sp) {
    static_assert(TILE == 16 * kFreqBlock, "16 rows per lane");
    using OutT = typename std::conditional<NARROW, uint32_t, unsigned long long>::type;
    OutT* __restrict__ out_h = static_cast<OutT*>(out);
    constexpr int PER = TILE / kFreqBlock;
    __shared__ unsigned int hist[kDigitBins], start[kDigitBins];
    __shared__ unsigned long long cursor[kDigitBins];
    __shared__ unsigned long long sh[TILE];
    __shared__ unsigned int regs[kFastRegs];
    __shared__ unsigned long long red[kFreqBlock / 64];
    __shared__ unsigned int lovf;
    for (int i = threadIdx.x; i < kFastRegs; i += kFreqBlock) regs[i] = 0;
    hist[threadIdx.x] = 0;
    if (threadIdx.x == 0) lovf = 0;
    __syncthreads();
    // per-lane counts (a lane sees nrows / (grid x 256) rows: 32 bits), widened once at the end
    unsigned int taken = 0, sent = 0, nulls = 0, miss = 0;
    const int64_t ntiles = (nrows + TILE - 1) / TILE;
    // workgroups are dealt round-robin to the XCDs: each XCD's workgroups fill their own sub-region of every
    // partition, so a reservation counter is shared by 1/8 of the chip (and stays with one XCD's traffic)
    const unsigned int xcd = blockIdx.x % kXcds;
    uint64_t raw[PER];
    unsigned int vword = 0;
    int64_t tile = blockIdx.x;
    if (tile < ntiles) p1_load<W>(c, tile * TILE, nrows, raw, vword);
    for (; tile < ntiles; tile += gridDim.x) {
        const int64_t t0 = tile * TILE;
        uint64_t h[PER];
        uint32_t pay[PER];
        // row masks: valid (rows past the end read as invalid), EMPTY-colliding, narrow-window misses; the counters
        // take their popcounts once per tile
        const unsigned int vm = vword;
        unsigned int em = 0, mm = 0;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const uint64_t canon = canonical_cell<W, FLT>(raw[j]);
            h[j] = mix64(canon);
            em |= (h[j] == kEmpty ? 1u : 0u) << j;
            if (NARROW) {
                const uint64_t off = canon - nk.base;
                pay[j] = (uint32_t)off;
                if (W == 8) mm |= ((off >> 32) != 0 ? 1u : 0u) << j;
            }
        }
        const unsigned int keepm = vm & ~em;
        sent += __popc(vm & em);
        if (NARROW && W == 8) miss += __popc(mm & vm);
        if (include_nulls) {  // Histogram: the NULL rows in range count (as the NULL group)
            const int64_t lrem = nrows - t0 - (int64_t)threadIdx.x;  // row t0 + 256 j + tid is in range iff 256 j < lrem
            unsigned int inm = 0;
#pragma unroll
            for (int j = 0; j < PER; ++j) inm |= ((int64_t)j * kFreqBlock < lrem ? 1u : 0u) << j;
            nulls += __popc(inm & ~vm);
            taken += __popc(inm);
        } else {
            taken += __popc(vm);
        }
        const int64_t next = tile + gridDim.x;
        // the sizing sketch sees the keys whose low kSketchBits bits are zero: a 1/512 sample of the distinct keys
        // (each key is in or out on every row), scaled back on the host. A sparse sample leaves the block below
        // unexecuted by most waves (its instructions run whenever one lane of 64 qualifies). The sample bits lie below
        // every bit a rank can reach but the last 9 of 54 (a forced-zero run inside the rank field would inflate the
        // maxima; reaching it needs 45 zero bits first).
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            if (!((keepm >> j) & 1u) || (h[j] & ((1u << kSketchBits) - 1u))) continue;
            const unsigned int idx = (unsigned int)(h[j] >> 54);
            const unsigned int rank = (unsigned int)__clzll((long long)((h[j] << 10) | (1ull << 9))) + 1u;
            if (rank > regs[idx]) atomicMax(&regs[idx], rank);
        }
        if (NARROW) {
#pragma unroll
            for (int j = 0; j < PER; ++j) h[j] = ((h[j] & (kDigitBins - 1)) << 32) | pay[j];
        }
        scatter_tile_reserve<kDigitBins, TILE, NARROW>(h, keepm, 0, kDigitBins - 1, hist, start, cursor, sh, gcursor, cap,
                                               [xcd](int b) { return (unsigned long long)b * kP1Sub + xcd; },
                                               [xcd](int b) { return ((unsigned long long)b * kP1Sub + xcd) * kCursorStride; },
                                               &lovf, sp, [nk](uint64_t v) {
                                                   return NARROW ? mix64(narrow_canon(nk, (uint32_t)v)) : v;
                                               }, out_h, [&]() {
            if (next < ntiles) p1_load<W>(c, next * TILE, nrows, raw, vword);
        });
    }
    const unsigned long long wtaken = block_sum_u64(taken, red);
    const unsigned long long wsent = block_sum_u64(sent, red);
    const unsigned long long wnulls = block_sum_u64(nulls, red);
    const unsigned long long wmiss = (NARROW && W == 8) ? block_sum_u64(miss, red) : 0ull;
    if (threadIdx.x == 0) {
        if (wtaken) atomicAdd(&ctr->num_rows, wtaken);
        if (wsent) atomicAdd(&ctr->sentinel, wsent);
        if (wnulls) atomicAdd(&ctr->nulls, wnulls);
        if (wmiss) atomicAdd(&ctr->narrow_miss, wmiss);
        if (lovf) atomicAdd(&ctr->pad[0], 1ull);
    }
    for (int i = threadIdx.x; i < kFastRegs / 4; i += kFreqBlock) {
        const unsigned int w = regs[4 * i] | (regs[4 * i + 1] << 8) | (regs[4 * i + 2] << 16) | (regs[4 * i + 3] << 24);
        reinterpret_cast<unsigned int*>(regs_part + (uint64_t)blockIdx.x * kFastRegs)[i] = w;
    }
}

struct FastItem {
    unsigned long long begin, end;  // range of one partition's pass-1 output
    unsigned int part, pad;
};

// Fast pass 2: per work item (a chunk of one partition), keys -> bucket part + 256 * (next bits), bucket k at
// k * cap; its reservation counter is part * bins + b, so a partition's counters share lines only with each other.
// The next tile is loaded before the current one is scattered. Two workgroups per CU (69.6 KB of LDS each) need
// <= 256 VGPRs: the 64-bit 8192-key tile sits at 252-258, and one register over halves the occupancy (r03: C4's
// pass 2 went from 4.2 to 5.1 ms when the NARROW template pushed it to 258), hence the explicit bound.
template <int BINS, int TILE, bool NARROW>
__global__ void __launch_bounds__(kFreqBlock, BINS <= kDigitBins ? 2 : 1)
scatter2_fast_kernel(const FastItem* __restrict__ items, const void* __restrict__ in, unsigned int mask,
                     unsigned long long cap, unsigned long long* __restrict__ gcursor, void* __restrict__ out,
                     Counters* __restrict__ ctr, NarrowKey nk, Spill sp) {
    using KeyT = typename std::conditional<NARROW, uint32_t, unsigned long long>::type;
    const KeyT* __restrict__ in_h = static_cast<const KeyT*>(in);
    KeyT* __restrict__ out_h = static_cast<KeyT*>(out);
    constexpr int PER = TILE / kFreqBlock;
    __shared__ unsigned int hist[BINS], start[BINS];
    __shared__ unsigned long long cursor[BINS];
    __shared__ unsigned long long sh[TILE];
    __shared__ unsigned int lovf;
    const FastItem it = items[blockIdx.x];
    for (int b = threadIdx.x; b < BINS; b += kFreqBlock) hist[b] = 0;
    if (threadIdx.x == 0) lovf = 0;
    __syncthreads();
    const unsigned long long part = it.part;
    KeyT nxt[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const unsigned long long i = it.begin + (unsigned long long)j * kFreqBlock + threadIdx.x;
        nxt[j] = i < it.end ? __builtin_nontemporal_load(&in_h[i]) : (KeyT)kEmpty;
    }
    for (unsigned long long t0 = it.begin; t0 < it.end; t0 += TILE) {
        uint64_t h[PER];
        unsigned int keepm = 0;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            // narrow: the digit comes from the re-derived key, the payload travels on
            h[j] = NARROW ? ((((mix64(narrow_canon(nk, (uint32_t)nxt[j])) >> 8) & mask)) << 32) | (uint64_t)nxt[j]
                          : (uint64_t)nxt[j];
            keepm |= (t0 + (unsigned long long)j * kFreqBlock + threadIdx.x < it.end ? 1u : 0u) << j;
        }
        const unsigned long long n0 = t0 + TILE;
        scatter_tile_reserve<BINS, TILE, NARROW>(h, keepm, 8, mask, hist, start, cursor, sh, gcursor, cap,
                                         [part](int b) { return part + (unsigned long long)kDigitBins * b; },
                                         [part, mask](int b) { return part * (mask + 1ull) + b; }, &lovf, sp,
                                         [nk](uint64_t v) {
                                             return NARROW ? mix64(narrow_canon(nk, (uint32_t)v)) : v;
                                         }, out_h, [&]() {
            if (n0 < it.end) {
#pragma unroll
                for (int j = 0; j < PER; ++j) {
                    const unsigned long long i = n0 + (unsigned long long)j * kFreqBlock + threadIdx.x;
                    nxt[j] = i < it.end ? __builtin_nontemporal_load(&in_h[i]) : (KeyT)kEmpty;
                }
            }
        });
    }
    if (threadIdx.x == 0 && lovf) atomicAdd(&ctr->pad[1], 1ull);
}

// Grouping summary partial. `ent` is the exact fixed-point sum of the entropy (or MutualInformation) terms
// (dq_common.h fx_of): integer adds, so the fold is the same for any slot order, workgroup split or device split.
struct SummaryPartial {
    unsigned long long groups, unique, maxc;
    unsigned int pad;        // build partials: 1 = this region needs the table scan
    unsigned int nonfinite;  // terms that were inf / NaN (the metric is then NaN, as a Spark double sum)
    fx128 ent;
};

__host__ __device__ __forceinline__ void summary_merge(SummaryPartial& a, const SummaryPartial& b) {
    a.groups += b.groups;
    a.unique += b.unique;
    a.maxc = b.maxc > a.maxc ? b.maxc : a.maxc;
    a.nonfinite += b.nonfinite;
    a.ent += b.ent;
}

// Adds one term to a partial: rounded once to fixed point, or counted as non-finite.
__device__ __forceinline__ void summary_add_term(SummaryPartial& p, double term) {
    if (__builtin_isfinite(term) && fabs(term) < 4194304.0)
        p.ent += fx_of(term);
    else
        p.nonfinite++;
}

// -(c/N) ln(c/N): the one definition of an entropy term (A/Entropy.scala:28-42), used by every kernel below.
__device__ __forceinline__ double entropy_term(unsigned long long c, double n) {
    const double q = (double)c / n;
    return -q * log(q);
}

__device__ __forceinline__ SummaryPartial summary_shfl_down(const SummaryPartial& p, int off) {
    SummaryPartial o;
    o.groups = __shfl_down(p.groups, off, 64);
    o.unique = __shfl_down(p.unique, off, 64);
    o.maxc = __shfl_down(p.maxc, off, 64);
    o.pad = __shfl_down(p.pad, off, 64);
    o.nonfinite = __shfl_down(p.nonfinite, off, 64);
    o.ent = fx_shfl_down(p.ent, off);
    return o;
}

// Entropy terms of the side groups the host keeps outside the table (the fast path's EMPTY-colliding value,
// Histogram's NULL group), computed by the same device code as the table's terms.
__global__ void side_terms_kernel(unsigned long long c0, unsigned long long c1, double n, SummaryPartial* out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    SummaryPartial p = {0, 0, 0, 0, 0, 0};
    if (c0) summary_add_term(p, entropy_term(c0, n));
    if (c1) summary_add_term(p, entropy_term(c1, n));
    *out = p;
}

struct BuildItem {
    unsigned long long begin, end;  // range of the sorted keys
    unsigned int bucket;
    unsigned int split;             // 1: the bucket is split over several items (merge with atomics)
};

__global__ void region_init_kernel(const BuildItem* __restrict__ items, int nitems, Slot* __restrict__ slots,
                                   unsigned long long* __restrict__ reps) {
    const BuildItem it = items[blockIdx.x];
    if (!it.split) return;
    Slot* region = slots + (uint64_t)it.bucket * kRegion;
    for (int i = threadIdx.x; i < kRegion; i += blockDim.x) {
        region[i].key = kEmpty;
        region[i].count = 0;
        if (reps) reps[(uint64_t)it.bucket * kRegion + i] = ~0ull;
    }
}

// One work item per workgroup: aggregate the item's keys in an LDS table, then store (whole bucket)
// or merge (slice of a split bucket) it into the bucket's region. Keys are loaded kBuildUnroll at a
// time per lane (independent global loads in flight), and each probe is a single LDS compare-and-
// swap EMPTY -> h whose returned value says inserted / found / occupied.
constexpr int kBuildBlock = 512;
constexpr int kBuildUnroll = 8;

// LDS counts: 32-bit for row counting (a work item holds <= kSliceRows rows), 64-bit for weighted input.
template <typename C, typename R = unsigned long long>
__device__ __forceinline__ bool lds_insert(unsigned long long* lkey, C* lcnt, R* lrep, unsigned long long h, R row, C w,
                                           bool general) {
    unsigned int p = region_probe(h);
    for (int probe = 0; probe < kRegion; ++probe) {
        const unsigned long long prev = atomicCAS(&lkey[p], kEmpty, h);
        if (prev == kEmpty || prev == h) {
            atomicAdd(&lcnt[p], w);
            if (general) atomicMin(&lrep[p], row);
            return true;
        }
        p = (p + 1) & (kRegion - 1);
    }
    return false;
}

// The grouping analyzers' table aggregation (runAnalyzersForParticularGrouping, R/AnalysisRunner.scala:480-548:
// #groups, #(count == 1), max count, sum -(c/N) ln(c/N)) is folded into the build: a whole-bucket item knows its
// region's final counts in LDS, so it writes its summary partial (parts[item]) and the table is never re-read for
// the default N; a slice of a split bucket flags its partial (pad = 1) and the host scans the table instead.
// NARROW: `hs` holds 32-bit narrow-key offsets (fast path), the key is mix64(base + offset).
// REP32 (general keys, < 2^32 - 1 source rows): the representatives as 32-bit rows in LDS (64 instead of 80 KB a
// workgroup, so two fit a CU beside other kernels' workgroups), widened when the region is written.
template <bool GENERAL, bool WEIGHTED, bool NARROW = false, bool REP32 = false>
__global__ void __launch_bounds__(kBuildBlock)
build_kernel(const BuildItem* __restrict__ items, const unsigned long long* __restrict__ hs,
             const unsigned long long* __restrict__ rows, const long long* __restrict__ weights,
             Slot* __restrict__ slots, unsigned long long* __restrict__ reps, Counters* __restrict__ ctr,
             SummaryPartial* __restrict__ parts, double n, NarrowKey nk) {
    const uint32_t* __restrict__ hs32 = reinterpret_cast<const uint32_t*>(hs);
    using C = typename std::conditional<WEIGHTED, unsigned long long, unsigned int>::type;
    using R = typename std::conditional<REP32, unsigned int, unsigned long long>::type;
    __shared__ unsigned long long lkey[kRegion];
    __shared__ C lcnt[kRegion];
    __shared__ R lrep[GENERAL ? kRegion : 1];
    __shared__ unsigned int lovf;
    const BuildItem it = items[blockIdx.x];
    auto wide = [](R r) -> unsigned long long { return r == (R)~0ull ? ~0ull : (unsigned long long)r; };
    for (int i = threadIdx.x; i < kRegion; i += kBuildBlock) {
        lkey[i] = kEmpty;
        lcnt[i] = 0;
        if (GENERAL) lrep[i] = (R)~0ull;
    }
    if (threadIdx.x == 0) lovf = 0;
    __syncthreads();
    bool ok = true;
    constexpr unsigned long long kStep = (unsigned long long)kBuildBlock * kBuildUnroll;
    for (unsigned long long j0 = it.begin + threadIdx.x; j0 < it.end; j0 += kStep) {
        unsigned long long h[kBuildUnroll], rw[kBuildUnroll];
#pragma unroll
        for (int u = 0; u < kBuildUnroll; ++u) {
            const unsigned long long j = j0 + (unsigned long long)u * kBuildBlock;
            if (NARROW)
                h[u] = j < it.end ? mix64(narrow_canon(nk, hs32[j])) : kEmpty;
            else
                h[u] = j < it.end ? hs[j] : kEmpty;
            rw[u] = ((GENERAL || WEIGHTED) && j < it.end) ? rows[j] : 0ull;
        }
        // (r04: issuing the 8 keys' compare-and-swaps before looking at any result made the C4 build 3.1 -> 4.1 ms,
        // profiles/r04/c4_split_ab_r04j.txt; one key at a time stays)
#pragma unroll
        for (int u = 0; u < kBuildUnroll; ++u)
            if (h[u] != kEmpty)
                ok &= lds_insert<C, R>(lkey, lcnt, lrep, h[u], (R)rw[u], WEIGHTED ? (C)weights[rw[u]] : (C)1, GENERAL);
    }
    if (!ok) lovf = 1;
    __syncthreads();
    Slot* region = slots + (uint64_t)it.bucket * kRegion;
    unsigned long long* rrep = GENERAL ? reps + (uint64_t)it.bucket * kRegion : nullptr;
    if (!it.split) {
        SummaryPartial p = {0, 0, 0, 0, 0, 0};
        for (int i = threadIdx.x; i < kRegion; i += kBuildBlock) {
            Slot sl;
            sl.key = lkey[i];
            sl.count = (unsigned long long)lcnt[i];
            region[i] = sl;
            if (GENERAL) rrep[i] = wide(lrep[i]);
            const unsigned long long c = sl.count;
            if (c == 0) continue;
            p.groups++;
            p.unique += c == 1;
            p.maxc = c > p.maxc ? c : p.maxc;
            if (n > 0) summary_add_term(p, entropy_term(c, n));
        }
        if (parts) {
            __shared__ SummaryPartial wred[kBuildBlock / 64];
            const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
            for (int off = 32; off > 0; off >>= 1) {
                const SummaryPartial o = summary_shfl_down(p, off);
                if (lane < off) summary_merge(p, o);
            }
            if (lane == 0) wred[wave] = p;
            __syncthreads();
            if (threadIdx.x == 0) {
                for (int w = 1; w < kBuildBlock / 64; ++w) summary_merge(p, wred[w]);
                p.pad = 0;
                parts[blockIdx.x] = p;
            }
        }
    } else {
        if (parts && threadIdx.x == 0) {
            SummaryPartial z = {0, 0, 0, 1, 0, 0};  // pad = 1: this region needs the table scan
            parts[blockIdx.x] = z;
        }
        bool mok = true;
        for (int i = threadIdx.x; i < kRegion; i += kBuildBlock) {
            const unsigned long long h = lkey[i];
            if (h == kEmpty) continue;
            const unsigned long long cnt = (unsigned long long)lcnt[i];
            unsigned int p = region_probe(h);
            bool done = false;
            for (int probe = 0; probe < kRegion; ++probe) {
                Slot* sl = region + p;
                const unsigned long long prev = atomicCAS(&sl->key, kEmpty, h);
                if (prev == kEmpty || prev == h) {
                    atomicAdd(&sl->count, cnt);
                    if (GENERAL) atomicMin(&rrep[p], wide(lrep[i]));
                    done = true;
                    break;
                }
                p = (p + 1) & (kRegion - 1);
            }
            mok &= done;
        }
        if (!mok) lovf = 1;
        __syncthreads();
    }
    if (threadIdx.x == 0 && lovf) atomicAdd(&ctr->overflow, 1ull);
}

// General keys, verified once the table is final: each work item's (key, row) pairs from the partition buffers
// against their region's representative (the group's smallest row), byte for byte unless the row is the representative.
constexpr int kVerifyBlock = 512;
constexpr int kVerifyRows = 4;  // rows per lane and step, their loads and first probes issued together
__global__ void __launch_bounds__(kVerifyBlock)
verify_items_kernel(const BuildItem* __restrict__ items, const unsigned long long* __restrict__ hs,
                    const unsigned long long* __restrict__ rows, const Slot* __restrict__ slots,
                    const unsigned long long* __restrict__ reps, KeySpec ks, Counters* __restrict__ ctr,
                    const unsigned long long* __restrict__ tup) {
    __shared__ unsigned long long vred[kVerifyBlock / 64];
    const BuildItem it = items[blockIdx.x];
    const Slot* region = slots + (uint64_t)it.bucket * kRegion;
    const unsigned long long* rrep = reps + (uint64_t)it.bucket * kRegion;
    unsigned long long bad = 0;
    constexpr unsigned long long kStep = (unsigned long long)kVerifyBlock * kVerifyRows;
    for (unsigned long long j0 = it.begin + threadIdx.x; j0 < it.end; j0 += kStep) {
        unsigned long long h[kVerifyRows], row[kVerifyRows], rep[kVerifyRows];
        unsigned int p[kVerifyRows];
        bool in[kVerifyRows];
#pragma unroll
        for (int u = 0; u < kVerifyRows; ++u) {
            const unsigned long long j = j0 + (unsigned long long)u * kVerifyBlock;
            in[u] = j < it.end;
            h[u] = in[u] ? hs[j] : kEmpty;
            row[u] = in[u] ? rows[j] : 0;
        }
#pragma unroll
        for (int u = 0; u < kVerifyRows; ++u) {
            p[u] = region_probe(h[u]);
            // the group's slot: most keys sit at their first probe position
            unsigned long long k = in[u] ? region[p[u]].key : h[u];
            for (int probe = 0; in[u] && k != h[u] && probe < kRegion; ++probe) {
                if (k == kEmpty) {
                    in[u] = false;
                    ++bad;  // a key missing from the table
                    break;
                }
                p[u] = (p[u] + 1) & (kRegion - 1);
                k = region[p[u]].key;
            }
        }
#pragma unroll
        for (int u = 0; u < kVerifyRows; ++u) rep[u] = in[u] ? rrep[p[u]] : row[u];
        if (tup) {  // 16-byte tuples of keys <= 15 bytes: equal tuples <=> equal keys; longer keys compare bytes
            uint64_t a0[kVerifyRows], a1[kVerifyRows], c0[kVerifyRows], c1[kVerifyRows];
#pragma unroll
            for (int u = 0; u < kVerifyRows; ++u) {
                const bool need = rep[u] != row[u];
                a0[u] = need ? tup[2 * row[u]] : 0;
                a1[u] = need ? tup[2 * row[u] + 1] : 0;
                c0[u] = need ? tup[2 * rep[u]] : 0;
                c1[u] = need ? tup[2 * rep[u] + 1] : 0;
            }
#pragma unroll
            for (int u = 0; u < kVerifyRows; ++u) {
                if (rep[u] == row[u]) continue;
                if (a1[u] != kTupleLong && c1[u] != kTupleLong) {
                    if (a0[u] != c0[u] || a1[u] != c1[u]) ++bad;
                } else if (!rows_equal(ks, (int64_t)row[u], (int64_t)rep[u])) {
                    ++bad;
                }
            }
            continue;
        }
#pragma unroll
        for (int u = 0; u < kVerifyRows; ++u)
            if (rep[u] != row[u] && !rows_equal(ks, (int64_t)row[u], (int64_t)rep[u])) ++bad;
    }
    for (int off = 32; off > 0; off >>= 1) bad += __shfl_down(bad, off, 64);
    if ((threadIdx.x & 63) == 0) vred[threadIdx.x >> 6] = bad;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long b = 0;
        for (int w = 0; w < kVerifyBlock / 64; ++w) b += vred[w];
        if (b) atomicAdd(&ctr->mismatch, b);
    }
}

// Spilled keys of the fast build (a bucket's share of a heavily repeated key past its slack) into the finished table:
// each workgroup aggregates a chunk of the spill in an LDS table (a heavy key becomes one (key, count) entry) and adds
// the entries to their regions with global compare-and-swap + add (the split-bucket merge of build_kernel). Region r
// of a key is its low `bits` bits, its probe start the top bits, as in every other build. A full region (or a full
// LDS table, whose key is then added on its own) raises Counters::overflow: the build grows, as for any overflow.
constexpr int kSpillChunk = 16384;

__device__ __forceinline__ bool region_add(Slot* __restrict__ slots, int bits, unsigned long long h,
                                           unsigned long long c) {
    Slot* region = slots + (h & ((1ull << bits) - 1ull)) * (unsigned long long)kRegion;
    unsigned int p = region_probe(h);
    for (int probe = 0; probe < kRegion; ++probe) {
        const unsigned long long prev = atomicCAS(&region[p].key, kEmpty, h);
        if (prev == kEmpty || prev == h) {
            atomicAdd(&region[p].count, c);
            return true;
        }
        p = (p + 1) & (kRegion - 1);
    }
    return false;
}

__global__ void __launch_bounds__(kBuildBlock)
spill_insert_kernel(const unsigned long long* __restrict__ spill, unsigned long long nspill, Slot* __restrict__ slots,
                    int bits, Counters* __restrict__ ctr) {
    __shared__ unsigned long long lkey[kRegion];
    __shared__ unsigned int lcnt[kRegion];
    bool ok = true;
    for (unsigned long long c0 = (unsigned long long)blockIdx.x * kSpillChunk; c0 < nspill;
         c0 += (unsigned long long)gridDim.x * kSpillChunk) {
        for (int i = threadIdx.x; i < kRegion; i += kBuildBlock) {
            lkey[i] = kEmpty;
            lcnt[i] = 0;
        }
        __syncthreads();
        const unsigned long long c1 = c0 + kSpillChunk < nspill ? c0 + kSpillChunk : nspill;
        for (unsigned long long j = c0 + threadIdx.x; j < c1; j += kBuildBlock) {
            const unsigned long long h = spill[j];
            if (!lds_insert<unsigned int, unsigned long long>(lkey, lcnt, (unsigned long long*)nullptr, h, 0ull, 1u, false)) ok &= region_add(slots, bits, h, 1ull);
        }
        __syncthreads();
        for (int i = threadIdx.x; i < kRegion; i += kBuildBlock)
            if (lkey[i] != kEmpty) ok &= region_add(slots, bits, lkey[i], (unsigned long long)lcnt[i]);
        __syncthreads();
    }
    if (!ok) atomicAdd(&ctr->overflow, 1ull);
}

// ---- small general tables: one fused pass -------------------------------------------------------------
// When the sizing estimate puts a general-path table (string / multi-column keys, unweighted) in one region (bits = 0,
// <= kRegionTarget distinct keys: the Histograms of low-cardinality columns the ColumnProfiler's third pass computes),
// the extract-write / build / verify passes collapse into one: every workgroup takes a contiguous chunk of rows in
// tiles, inserts each tile's fingerprints into its LDS table (count, smallest row), then checks each of the tile's rows
// against its slot's representative while both rows are still cache-hot (rows arrive in order, so once a tile is
// inserted a representative never changes again); the workgroup tables merge into region 0 with global atomics and
// publish their representatives, which small_check_kernel compares with the final (smallest) one. Exact: a fingerprint
// collision anywhere raises `mismatch` and the build reruns with a new seed; a full table raises `overflow` and the
// build takes the regular path.
// One string key column (the Histograms of the profiler's third pass): a key of <= 15 bytes is held exactly as two
// words (bytes 0-7, bytes 8-14 | length << 56), so a row is verified against its group's representative by comparing
// words with the representative's copy in LDS instead of re-reading both rows' bytes from HBM (half the kernel's time).
// A NULL row of a grouping is one marker, a NULL row of a Histogram the bytes of "NullValue" (string_null_is_value),
// a longer key the "long" marker (verified through rows_equal).
// (kTupleNull / kTupleLong / short_key_tuple: defined before extract_count_kernel, which also writes them)

// XXH64 (seed) of a <= 15-byte key held as short_key_tuple words: the same value as dev_xxh_bytes over its bytes.
__device__ __forceinline__ uint64_t xxh_short_words(uint64_t b0, uint64_t b1, uint64_t seed) {
    const int len = (int)(b1 >> 56);
    uint64_t w0 = b0, w1 = b1 & 0x00FFFFFFFFFFFFFFull;  // the key's bytes 0-7 and 8-14
    uint64_t h = seed + P64_5 + (uint64_t)len;
    int rest = len;
    if (rest >= 8) {
        h ^= xxh_round(0, w0);
        h = rotl64(h, 27) * P64_1 + P64_4;
        w0 = w1;
        w1 = 0;
        rest -= 8;
    }
    if (rest >= 4) {
        h ^= (uint64_t)(uint32_t)w0 * P64_1;
        h = rotl64(h, 23) * P64_2 + P64_3;
        w0 >>= 32;
        rest -= 4;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i)
        if (i < rest) {
            h ^= (w0 & 0xFFull) * P64_5;
            h = rotl64(h, 11) * P64_1;
            w0 >>= 8;
        }
    return xxh_fmix(h);
}

// row_key for one string key column that also returns the key's words (short_key_tuple): one set of loads per row.
__device__ __forceinline__ bool row_key_str1(const KeySpec& ks, int64_t r, uint64_t& h, uint64_t& b0, uint64_t& b1,
                                             bool& is_short) {
    const KeyCol& c = ks.cols[0];
    is_short = short_key_tuple(ks, r, b0, b1);
    uint64_t ch;
    bool any = true;
    if (b0 == kTupleNull && b1 == kTupleNull) {  // NULL row of a grouping
        ch = 0x6A09E667F3BCC909ULL;
        any = false;
    } else if (is_short) {  // valid, or "NullValue" for a Histogram's NULL row
        ch = xxh_short_words(b0, b1, ks.seed);
    } else {
        int len;
        const uint8_t* p = str_span(c, r, len);
        ch = dev_xxh_bytes(p, len, ks.seed);
    }
    const uint64_t acc = mix64(ks.seed + P64_1 * 1ull + ch);
    if (!any && !ks.include_nulls) return false;
    h = (acc == kEmpty ? kEmpty - 1 : acc) & ks.fp_mask;
    return true;
}

constexpr int kSmallTile = 4 * kBuildBlock;
constexpr int kSmallGrid = 768;  // 3 workgroups per CU with the 2048-slot table

#ifndef DQ_SMALL_WAVES
#define DQ_SMALL_WAVES 0  // STR1 A/B: a minimum of waves per SIMD (6: 80 VGPRs + spills, 8: 64 + spills) measured no faster, profiles/r06/small_build_waves_ab_r06s.txt
#endif
template <int LS, bool STR1 = false>  // slots of the workgroup's LDS table; STR1: one string key column
__global__ void __launch_bounds__(kBuildBlock, STR1 && DQ_SMALL_WAVES ? DQ_SMALL_WAVES : 1)
small_build_kernel(KeySpec ks, int64_t nrows, Slot* __restrict__ slots, unsigned long long* __restrict__ reps,
                   unsigned long long* __restrict__ wg_keys, unsigned long long* __restrict__ wg_reps,
                   Counters* __restrict__ ctr, int count_rows) {
    __shared__ unsigned long long lkey[LS];
    __shared__ unsigned int lcnt[LS];
    __shared__ unsigned long long lrep[LS];
    __shared__ unsigned long long lb0[STR1 ? LS : 1], lb1[STR1 ? LS : 1];  // the representative's key words (STR1)
    __shared__ unsigned long long red[kBuildBlock / 64];
    __shared__ unsigned int lovf, lfill, lgone;
    // the build is already lost (another workgroup's table filled): a workgroup that starts now does nothing. On a busy
    // device this kernel's 36-40 KB workgroups get CUs one by one, and the optimistic try over a high-cardinality column
    // took 14 ms to let every late workgroup fill its own table once (0.3 ms alone); small_check_kernel skips too
    if (threadIdx.x == 0) lgone = *(volatile unsigned long long*)&ctr->overflow != 0 ? 1u : 0u;
    __syncthreads();
    if (lgone) return;  // (uniform: read after the barrier)
    for (int i = threadIdx.x; i < LS; i += kBuildBlock) {
        lkey[i] = kEmpty;
        lcnt[i] = 0;
        lrep[i] = ~0ull;
    }
    if (threadIdx.x == 0) lovf = lfill = 0;
    __syncthreads();
    auto start = [](uint64_t h) { return (unsigned int)(h >> 52) & (LS - 1); };
    int64_t r0, r1;
    chunk_of(nrows, r0, r1);
    unsigned long long bad = 0, taken = 0;
    bool ok = true;
    for (int64_t t0 = r0; t0 < r1; t0 += kSmallTile) {
        uint64_t h[4];
        bool take[4];
        uint64_t kb0[STR1 ? 4 : 1], kb1[STR1 ? 4 : 1];
        bool kshort[STR1 ? 4 : 1];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t r = t0 + (int64_t)u * kBuildBlock + threadIdx.x;
            bool ng = false;
            h[u] = kEmpty;
            if constexpr (STR1) {
                take[u] = r < r1 && row_key_str1(ks, r, h[u], kb0[u], kb1[u], kshort[u]) && h[u] != kEmpty;
            } else {
                take[u] = r < r1 && row_key(ks, r, h[u], ng) && !ng && h[u] != kEmpty;
            }
            taken += take[u] ? 1 : 0;
        }
        unsigned int pu[4];  // each row's slot, kept for the verification
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            pu[u] = 0;
            if (!take[u]) continue;
            const unsigned long long row = (unsigned long long)(t0 + (int64_t)u * kBuildBlock + threadIdx.x);
            // past 3/4 full the table counts as overflowing (bounded probe chains when the guess was wrong)
            if (*(volatile unsigned int*)&lfill > (unsigned int)(LS / 4 * 3)) {
                ok = false;
                continue;
            }
            unsigned int p = start(h[u]);
            bool done = false;
            for (int probe = 0; probe < LS; ++probe) {
                // a plain read first: a low-cardinality column finds its key already placed on almost every row, and a
                // 64-bit LDS read is one access (kEmpty or the whole key), so only an empty slot takes the CAS and only
                // a smaller row the atomicMin -- the atomics of many lanes on one hot slot serialise
                unsigned long long prev = *(volatile unsigned long long*)&lkey[p];
                if (prev == kEmpty) prev = atomicCAS(&lkey[p], kEmpty, h[u]);
                if (prev == kEmpty || prev == h[u]) {
                    if (prev == kEmpty) atomicAdd(&lfill, 1u);
                    atomicAdd(&lcnt[p], 1u);
                    if (row < *(volatile unsigned long long*)&lrep[p]) atomicMin(&lrep[p], row);
                    done = true;
                    break;
                }
                p = (p + 1) & (LS - 1);
            }
            pu[u] = p;
            ok &= done;
        }
        if (!ok) lovf = 1;
        __syncthreads();
        if (lovf) break;  // a full table: the build goes elsewhere, stop reading rows (uniform: read after the barrier)
        if constexpr (STR1) {  // each group's representative row (new in this tile) publishes its key words
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int64_t r = t0 + (int64_t)u * kBuildBlock + threadIdx.x;
                if (take[u] && lkey[pu[u]] == h[u] && lrep[pu[u]] == (unsigned long long)r) {
                    lb0[pu[u]] = kb0[u];
                    lb1[pu[u]] = kb1[u];
                }
            }
            __syncthreads();
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (!take[u]) continue;
            const int64_t r = t0 + (int64_t)u * kBuildBlock + threadIdx.x;
            const unsigned int p = pu[u];
            const unsigned long long rep = lrep[p];
            if (lkey[p] != h[u]) {
                ++bad;
            } else if (rep != (unsigned long long)r) {
                bool same;
                if constexpr (STR1) {
                    if (kshort[u] && lb1[p] != kTupleLong) same = lb0[p] == kb0[u] && lb1[p] == kb1[u];
                    else same = rows_equal(ks, r, (int64_t)rep);
                } else {
                    same = rows_equal(ks, r, (int64_t)rep);
                }
                if (!same) ++bad;
            }
        }
        __syncthreads();
    }
    if (!ok) lovf = 1;
    __syncthreads();
    // A full table (here or, already, in another workgroup) discards the build: raise `overflow` now and skip the
    // merge, so an optimistic try over many distinct keys does not probe a full region 0 with every workgroup's
    // groups (kRegion global CAS probes per key).
    __shared__ unsigned int lskip;
    if (threadIdx.x == 0) {
        if (lovf) atomicAdd(&ctr->overflow, 1ull);
        lskip = lovf || *(volatile unsigned long long*)&ctr->overflow != 0;
    }
    __syncthreads();
    const bool skip = lskip != 0;
    // publish this workgroup's groups and merge them into region 0 (kRegion slots; a probe chain past
    // kMergeProbes counts as a full region)
    constexpr int kMergeProbes = 512;
    bool mok = true;
    for (int i = threadIdx.x; i < kRegion; i += kBuildBlock) {
        const unsigned long long key = i < LS && !skip ? lkey[i] : kEmpty;
        wg_keys[(uint64_t)blockIdx.x * kRegion + i] = key;
        wg_reps[(uint64_t)blockIdx.x * kRegion + i] = i < LS && !skip ? lrep[i] : ~0ull;
        if (key == kEmpty) continue;
        unsigned int p = region_probe(key);
        bool done = false;
        for (int probe = 0; probe < kMergeProbes; ++probe) {
            const unsigned long long prev = atomicCAS(&slots[p].key, kEmpty, key);
            if (prev == kEmpty || prev == key) {
                atomicAdd(&slots[p].count, (unsigned long long)lcnt[i]);
                atomicMin(&reps[p], lrep[i]);
                done = true;
                break;
            }
            p = (p + 1) & (kRegion - 1);
        }
        mok &= done;
    }
    __shared__ unsigned int lmfail;
    if (threadIdx.x == 0) lmfail = 0;
    __syncthreads();
    if (!mok) lmfail = 1;
    if (count_rows) {  // numRows when no sizing pass counted it (the optimistic small build)
        for (int off = 32; off > 0; off >>= 1) taken += __shfl_down(taken, off, 64);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = taken;
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long t = 0;
            for (int w = 0; w < kBuildBlock / 64; ++w) t += red[w];
            if (t) atomicAdd(&ctr->num_rows, t);
        }
        __syncthreads();  // `red` is reused below
    }
    for (int off = 32; off > 0; off >>= 1) bad += __shfl_down(bad, off, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = bad;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long b = 0;
        for (int w = 0; w < kBuildBlock / 64; ++w) b += red[w];
        if (b) atomicAdd(&ctr->mismatch, b);
        if (lmfail && !lovf) atomicAdd(&ctr->overflow, 1ull);
    }
}

// Every workgroup's representative of a group against the group's final (smallest-row) representative.
__global__ void __launch_bounds__(kBuildBlock)
small_check_kernel(KeySpec ks, const Slot* __restrict__ slots, const unsigned long long* __restrict__ reps,
                   const unsigned long long* __restrict__ wg_keys, const unsigned long long* __restrict__ wg_reps,
                   Counters* __restrict__ ctr) {
    // a full table discards the build (the caller takes the regular path); the workgroups of small_build_kernel that
    // found the overflow raised at their start published nothing
    if (*(volatile unsigned long long*)&ctr->overflow) return;
    unsigned long long bad = 0;
    for (int i = threadIdx.x; i < kRegion; i += kBuildBlock) {
        const unsigned long long key = wg_keys[(uint64_t)blockIdx.x * kRegion + i];
        if (key == kEmpty) continue;
        const unsigned long long wrep = wg_reps[(uint64_t)blockIdx.x * kRegion + i];
        unsigned int p = region_probe(key);
        int probe = 0;
        for (; probe < kRegion && slots[p].key != key; ++probe) p = (p + 1) & (kRegion - 1);
        if (probe == kRegion) {
            ++bad;
            continue;
        }
        const unsigned long long grep = reps[p];
        if (grep != wrep && !rows_equal(ks, (int64_t)wrep, (int64_t)grep)) ++bad;
    }
    if (bad) atomicAdd(&ctr->mismatch, bad);
}

// ---- table scans ---------------------------------------------------------------------------------

__global__ void __launch_bounds__(kFreqBlock)
summary_kernel(const Slot* __restrict__ slots, uint64_t cap, double n, SummaryPartial* __restrict__ out) {
    __shared__ SummaryPartial red[kFreqBlock];
    const uint64_t chunk = (cap + gridDim.x - 1) / gridDim.x;
    const uint64_t b0 = (uint64_t)blockIdx.x * chunk;
    const uint64_t b1 = b0 + chunk < cap ? b0 + chunk : cap;
    SummaryPartial p = {0, 0, 0, 0, 0, 0};
    for (uint64_t i = b0 + threadIdx.x; i < b1; i += kFreqBlock) {
        const unsigned long long c = slots[i].count;
        if (c == 0) continue;
        p.groups++;
        p.unique += c == 1;
        p.maxc = c > p.maxc ? c : p.maxc;
        if (n > 0) summary_add_term(p, entropy_term(c, n));
    }
    red[threadIdx.x] = p;
    __syncthreads();
    for (int s = kFreqBlock / 2; s > 0; s >>= 1) {
        if (threadIdx.x < s) summary_merge(red[threadIdx.x], red[threadIdx.x + s]);
        __syncthreads();
    }
    if (threadIdx.x == 0) out[blockIdx.x] = red[0];
}

// The summary partial of one region (blockIdx.x -> bucket) of the table.
__global__ void __launch_bounds__(kFreqBlock)
region_summary_kernel(const unsigned int* __restrict__ buckets, const Slot* __restrict__ slots, double n,
                      SummaryPartial* __restrict__ out) {
    __shared__ SummaryPartial red[kFreqBlock];
    const Slot* region = slots + (uint64_t)buckets[blockIdx.x] * kRegion;
    SummaryPartial p = {0, 0, 0, 0, 0, 0};
    for (int i = threadIdx.x; i < kRegion; i += kFreqBlock) {
        const unsigned long long c = region[i].count;
        if (c == 0) continue;
        p.groups++;
        p.unique += c == 1;
        p.maxc = c > p.maxc ? c : p.maxc;
        if (n > 0) summary_add_term(p, entropy_term(c, n));
    }
    red[threadIdx.x] = p;
    __syncthreads();
    for (int st = kFreqBlock / 2; st > 0; st >>= 1) {
        if (threadIdx.x < st) summary_merge(red[threadIdx.x], red[threadIdx.x + st]);
        __syncthreads();
    }
    if (threadIdx.x == 0) out[blockIdx.x] = red[0];
}

// Radix-select step: histogram of 11-bit digit `shift` of counts whose higher bits equal `prefix`.
__global__ void __launch_bounds__(kFreqBlock)
digit_hist_kernel(const Slot* __restrict__ slots, uint64_t cap, int shift, unsigned long long prefix_mask,
                  unsigned long long prefix, unsigned long long* __restrict__ hist) {
    __shared__ unsigned int lds[2048];
    for (int i = threadIdx.x; i < 2048; i += kFreqBlock) lds[i] = 0;
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * kFreqBlock;
    for (uint64_t i = (uint64_t)blockIdx.x * kFreqBlock + threadIdx.x; i < cap; i += stride) {
        const unsigned long long c = slots[i].count;
        if (c == 0 || (c & prefix_mask) != prefix) continue;
        atomicAdd(&lds[(unsigned int)(c >> shift) & 2047u], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 2048; i += kFreqBlock)
        if (lds[i]) atomicAdd(&hist[i], (unsigned long long)lds[i]);
}

// Selection predicate of the compaction kernels: mode 0 = count > t, 1 = count == t, 2 = count > 0.
__device__ __forceinline__ bool selected(unsigned long long c, int mode, unsigned long long t) {
    return mode == 0 ? c > t : (mode == 1 ? c == t : c > 0);
}

__global__ void __launch_bounds__(kFreqBlock)
count_selected_kernel(const Slot* __restrict__ slots, uint64_t cap, int mode, unsigned long long t,
                      unsigned long long* __restrict__ per_block) {
    __shared__ unsigned long long red[kFreqBlock / 64];
    const uint64_t chunk = (cap + gridDim.x - 1) / gridDim.x;
    const uint64_t b0 = (uint64_t)blockIdx.x * chunk;
    const uint64_t b1 = b0 + chunk < cap ? b0 + chunk : cap;
    unsigned long long n = 0;
    for (uint64_t i = b0 + threadIdx.x; i < b1; i += kFreqBlock) n += selected(slots[i].count, mode, t);
    n = block_sum_u64(n, red);
    if (threadIdx.x == 0) per_block[blockIdx.x] = n;
}

// Writes the selected slots of each workgroup's chunk in slot order at out[offset[b] + rank],
// skipping ranks >= limit. key_out gets the slot key (fast) or the representative row (general).
__global__ void __launch_bounds__(kFreqBlock)
compact_kernel(const Slot* __restrict__ slots, const unsigned long long* __restrict__ reps, uint64_t cap, int mode,
               unsigned long long t, const unsigned long long* __restrict__ offsets, unsigned long long limit,
               unsigned long long* __restrict__ key_out, unsigned long long* __restrict__ count_out, int decode) {
    __shared__ unsigned int wave_counts[kFreqBlock / 64];
    const uint64_t chunk = (cap + gridDim.x - 1) / gridDim.x;
    const uint64_t b0 = (uint64_t)blockIdx.x * chunk;
    const uint64_t b1 = b0 + chunk < cap ? b0 + chunk : cap;
    unsigned long long base = offsets[blockIdx.x];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint64_t i0 = b0; i0 < b1; i0 += kFreqBlock) {
        const uint64_t i = i0 + threadIdx.x;
        const bool sel = i < b1 && selected(slots[i].count, mode, t);
        const unsigned long long bal = __ballot(sel);
        const unsigned int before = __popcll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) wave_counts[wave] = __popcll(bal);
        __syncthreads();
        unsigned int wave_off = 0, tile_total = 0;
        for (int w = 0; w < kFreqBlock / 64; ++w) {
            if (w < wave) wave_off += wave_counts[w];
            tile_total += wave_counts[w];
        }
        if (sel) {
            const unsigned long long rank = base + wave_off + before;
            if (rank < limit) {
                key_out[rank] = reps ? reps[i] : (decode ? unmix64(slots[i].key) : slots[i].key);
                count_out[rank] = slots[i].count;
            }
        }
        base += tile_total;
        __syncthreads();
    }
}


// ---- MutualInformation over a joint (x, y) table and the two marginal tables (A/MutualInformation.scala:35-97) --
struct LookupTable {
    const Slot* slots;
    KeySpec ks;
    unsigned long long sentinel;  // fast path: the value whose mixed key is the EMPTY marker
    int bits;
};

// Count of row r's key in table T (0 when r's key is NULL: Spark's equi-join on the marginals drops it).
__device__ __forceinline__ unsigned long long lookup_count(const LookupTable& T, int64_t r) {
    uint64_t h;
    bool ng;
    if (!row_key(T.ks, r, h, ng) || ng) return 0;
    if (h == kEmpty) return T.sentinel;
    const uint64_t base = (h & ((1ull << T.bits) - 1)) * kRegion;
    unsigned int p = region_probe(h);
    for (int probe = 0; probe < kRegion; ++probe) {
        const Slot& sl = T.slots[base + p];
        if (sl.key == h) return sl.count;
        if (sl.key == kEmpty) return 0;
        p = (p + 1) & (kRegion - 1);
    }
    return 0;
}

// sum over joint groups with both keys non-NULL of (pxy/N) ln((pxy/N) / ((px/N)(py/N))): every term rounded once to
// fixed point and the integers added (SummaryPartial), so the sum does not depend on the joint table's slot order
__global__ void __launch_bounds__(kFreqBlock)
mi_kernel(const Slot* __restrict__ slots, const unsigned long long* __restrict__ reps, uint64_t cap, KeySpec jks,
          LookupTable X, LookupTable Y, double n, SummaryPartial* __restrict__ out) {
    __shared__ SummaryPartial red[kFreqBlock];
    const uint64_t chunk = (cap + gridDim.x - 1) / gridDim.x;
    const uint64_t b0 = (uint64_t)blockIdx.x * chunk;
    const uint64_t b1 = b0 + chunk < cap ? b0 + chunk : cap;
    SummaryPartial p = {0, 0, 0, 0, 0, 0};
    for (uint64_t i = b0 + threadIdx.x; i < b1; i += kFreqBlock) {
        const unsigned long long c = slots[i].count;
        if (c == 0) continue;
        const int64_t r = (int64_t)reps[i];
        if (!is_valid(jks.cols[0], r) || !is_valid(jks.cols[1], r)) continue;
        const double px = (double)lookup_count(X, r), py = (double)lookup_count(Y, r);
        const double pxy = (double)c / n;
        p.groups++;
        summary_add_term(p, pxy * log(pxy / ((px / n) * (py / n))));
    }
    red[threadIdx.x] = p;
    __syncthreads();
    for (int st = kFreqBlock / 2; st > 0; st >>= 1) {
        if (threadIdx.x < st) summary_merge(red[threadIdx.x], red[threadIdx.x + st]);
        __syncthreads();
    }
    if (threadIdx.x == 0) out[blockIdx.x] = red[0];
}

// Per source row: the count of its group in T (0 when it takes no part) — the join of the rows with their
// frequencies. The rows are the table's own source rows, so the build's verification covers the fingerprints.
__global__ void __launch_bounds__(kFreqBlock)
row_counts_kernel(LookupTable T, int64_t nrows, long long* __restrict__ out) {
    const int64_t stride = (int64_t)gridDim.x * kFreqBlock;
    for (int64_t r = (int64_t)blockIdx.x * kFreqBlock + threadIdx.x; r < nrows; r += stride)
        out[r] = (long long)lookup_count(T, r);
}

}  // namespace

struct dq_ctx;  // defined in dq_api.cpp; only its device/stream are needed here
extern "C" int dq_set_stream(dq_ctx* ctx, void* stream);
namespace dq {
hipStream_t ctx_stream(dq_ctx* ctx);
int ctx_device(dq_ctx* ctx);
int ctx_fail(dq_ctx* ctx, int code, const char* msg);
}

// Key cells of a set of groups as host columns (values / offsets / validity) plus their counts: the groups a
// device owns in a multi-device table over general keys.
struct GatheredKeys {
    std::vector<std::vector<uint8_t>> values, validity;
    std::vector<std::vector<int32_t>> offsets;
    std::vector<dq_column> cols;
    std::vector<int64_t> counts;
};

struct dq_freq_table {
    int device = 0;
    KeySpec ks;
    Slot* slots = nullptr;
    unsigned long long* reps = nullptr;
    Counters* ctr = nullptr;  // device
    Counters host_ctr;
    uint64_t cap = 0;
    int bits = 0;           // 2^bits bucket regions of kRegion slots
    int fast = 1;
    // multi-device context: the table is the union of per-device parts with disjoint key sets (owner device =
    // hash of the key); part j lives on part_ctx[j]'s GPU
    std::vector<dq_freq_table*> parts;
    std::vector<dq_ctx*> part_ctx;
    int64_t total_rows = 0;
    // general keys on several devices: part j's rows are groups gathered from the shards; part_rows[j][r] is the
    // row of the caller's table that group r stands for (its smallest row), so exported keys stay row indices
    std::vector<std::vector<int64_t>> part_rows;
    std::vector<GatheredKeys> part_keys;  // and the key cells + counts of those groups (MutualInformation)
    // summary folded into the build (default N = the build's numRows), see build_kernel
    int pre_valid = 0;
    int64_t pre_n = -1;
    unsigned long long pre_groups = 0, pre_unique = 0, pre_maxc = 0;
    fx128 pre_ent = 0;
    unsigned int pre_nonfinite = 0;
    int32_t key_type = 0;   // Spark type of the (single) key column, or of the canonical keys of a pair-built table
    int64_t num_rows_override = -1;  // tables built from (key, count) pairs carry the caller's numRows
    int64_t src_rows = -1;  // rows of the source columns (dq_frequencies_ex), -1 for pair-built / merged tables
    int64_t cached_n = -1;  // dq_freq_summarize memo (the table is immutable once built)
    dq_freq_summary cached;
    void* scratch = nullptr;  // device scratch for scans
    size_t scratch_bytes = 0;
    std::vector<void*> staged;  // host key columns copied to HBM (rows are re-read by verify/export)
    // slots / reps come from the building context's scratch cache and go back to it when the table is freed
    // through that context (any other way: hipFree)
    dq_ctx* home = nullptr;
    size_t slots_bytes = 0, reps_bytes = 0;
    // ctr / scratch come from this context's scratch cache (a hipFree waits for the whole device: freeing a table on
    // one thread must not stall while other contexts' kernels run)
    dq_ctx* buf_home = nullptr;
};

namespace {

void release_slots(dq_freq_table* t, dq_ctx* ctx) {
    const bool cache = ctx && ctx == t->home;
    if (t->slots) {
        if (cache) dq::scratch_release(ctx, t->slots, t->slots_bytes); else (void)hipFree(t->slots);
    }
    if (t->reps) {
        if (cache) dq::scratch_release(ctx, t->reps, t->reps_bytes); else (void)hipFree(t->reps);
    }
    t->slots = nullptr;
    t->reps = nullptr;
}

void free_table_buffers(dq_freq_table* t, dq_ctx* ctx) {
    release_slots(t, ctx);
    const bool cache = ctx && ctx == t->buf_home;
    if (t->ctr) {
        if (cache) dq::scratch_release(ctx, t->ctr, sizeof(Counters)); else (void)hipFree(t->ctr);
    }
    if (t->scratch) {
        if (cache) dq::scratch_release(ctx, t->scratch, t->scratch_bytes); else (void)hipFree(t->scratch);
    }
    t->slots = nullptr;
    t->reps = nullptr;
    t->ctr = nullptr;
    t->scratch = nullptr;
    for (void* p : t->staged) (void)hipFree(p);
    t->staged.clear();
}

double hll_raw_estimate(const std::vector<unsigned int>& regs) {
    const double m = (double)regs.size();
    double z = 0.0, zeros = 0.0;
    for (unsigned int r : regs) {
        z += ldexp(1.0, -(int)r);
        zeros += r == 0;
    }
    const double alpha = 0.7213 / (1.0 + 1.079 / m);
    double e = alpha * m * m / z;
    if (e <= 2.5 * m && zeros > 0) e = m * log(m / zeros);
    return e;
}

int scan_grid(uint64_t n) {
    uint64_t g = (n + kFreqBlock - 1) / kFreqBlock;
    return (int)std::max<uint64_t>(1, std::min<uint64_t>(g, 2048));
}

}  // namespace

#define FQ_HIP(ctx, expr)                                                                         \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess) return dq::ctx_fail((ctx), DQ_ERR_DEVICE, hipGetErrorString(e_));   \
    } while (0)

namespace {

struct DevBuf {  // scratch device buffers of one build (the context's scratch cache), released on every path
    dq_ctx* ctx;
    std::vector<std::pair<void*, size_t>> ptrs;
    explicit DevBuf(dq_ctx* c) : ctx(c) {}
    ~DevBuf() {
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

// extract (+ sizing) -> radix sort on `bits` bits of the keys -> per-bucket LDS aggregation.
// A bucket whose distinct keys overflow its region (or a fingerprint collision on the general
// path) restarts the sort/build with more bucket bits (or a new seed).
// Aggregates the bucketed keys (bucket b = keys[bstart[b], bstart[b] + bcount[b])) into one region per
// bucket. Returns DQ_OK with *overflow / *collision set from the device counters.
int build_regions(dq_ctx* ctx, dq_freq_table* t, int64_t nrows, DevBuf& buf, const unsigned long long* sorted,
                  const unsigned long long* srows, const std::vector<unsigned long long>& bstart,
                  const std::vector<unsigned long long>& bcount, int bits, bool* overflow, bool* collision,
                  const NarrowKey* narrow = nullptr, const unsigned long long* spill = nullptr,
                  unsigned long long nspill = 0, const unsigned long long* tup = nullptr) {
    hipStream_t s = dq::ctx_stream(ctx);
    const bool general = !t->fast;
    const bool weighted = t->ks.weights != nullptr;
    const uint64_t nb = 1ull << bits;
    std::vector<BuildItem> items;
    items.reserve(nb);
    for (uint64_t bk = 0; bk < nb; ++bk) {
        const unsigned long long b0 = bstart[bk], b1 = b0 + bcount[bk];
        if (b1 - b0 <= (unsigned long long)kSliceRows) {
            items.push_back(BuildItem{b0, b1, (unsigned int)bk, 0u});
            continue;
        }
        for (unsigned long long x = b0; x < b1; x += kSliceRows)
            items.push_back(BuildItem{x, std::min<unsigned long long>(b1, x + kSliceRows), (unsigned int)bk, 1u});
    }
    const uint64_t cap = nb * kRegion;
    release_slots(t, ctx);
    t->home = ctx;
    t->slots_bytes = cap * sizeof(Slot);
    t->reps_bytes = general ? cap * sizeof(unsigned long long) : 0;
    t->slots = (Slot*)dq::scratch_alloc(ctx, t->slots_bytes);
    if (general && t->slots) t->reps = (unsigned long long*)dq::scratch_alloc(ctx, t->reps_bytes);
    if (!t->slots || (general && !t->reps))
        return dq::ctx_fail(ctx, DQ_ERR_OUT_OF_MEMORY, "frequency table allocation failed");
    t->cap = cap;
    t->bits = bits;
    BuildItem* ditems = nullptr;
    FQ_HIP(ctx, buf.alloc((void**)&ditems, items.size() * sizeof(BuildItem)));
    FQ_HIP(ctx, hipMemcpyAsync(ditems, items.data(), items.size() * sizeof(BuildItem), hipMemcpyHostToDevice, s));
    const int nitems = (int)items.size();
    hipLaunchKernelGGL(region_init_kernel, dim3(nitems), dim3(kFreqBlock), 0, s, ditems, nitems, t->slots, t->reps);
    const long long* w = t->ks.weights;
    SummaryPartial* bparts = nullptr;
    FQ_HIP(ctx, buf.alloc((void**)&bparts, items.size() * sizeof(SummaryPartial)));
    const double build_n = (double)t->host_ctr.num_rows;  // the count pass's numRows (copied before the build)
    // general keys: every row is verified against its group's representative by verify_items_kernel, one workgroup
    // per work item reading the item's (key, row) pairs from the partition buffers with the item's region L2-resident
    // (DQ_FREQ_VERIFY_PASS: a pass over the rows instead, re-hashing each key). r05: comparing inside the build while
    // the table is in LDS cost more (build 7.4 -> 16.7 ms on the C5 text column: the random row reads stall the
    // build's few resident workgroups).
    const int verify_by_items = general && !getenv("DQ_FREQ_VERIFY_PASS") ? 1 : 0;
    if (general && weighted)
        hipLaunchKernelGGL((build_kernel<true, true>), dim3(nitems), dim3(kBuildBlock), 0, s, ditems, sorted, srows, w,
                           t->slots, t->reps, t->ctr, bparts, build_n, NarrowKey{});
    else if (general && nrows < (int64_t)0xFFFFFFFFll && !getenv("DQ_FREQ_REP64"))
        hipLaunchKernelGGL((build_kernel<true, false, false, true>), dim3(nitems), dim3(kBuildBlock), 0, s, ditems, sorted,
                           srows, w, t->slots, t->reps, t->ctr, bparts, build_n, NarrowKey{});
    else if (general)
        hipLaunchKernelGGL((build_kernel<true, false>), dim3(nitems), dim3(kBuildBlock), 0, s, ditems, sorted, srows, w,
                           t->slots, t->reps, t->ctr, bparts, build_n, NarrowKey{});
    else if (weighted)
        hipLaunchKernelGGL((build_kernel<false, true>), dim3(nitems), dim3(kBuildBlock), 0, s, ditems, sorted, srows, w,
                           t->slots, t->reps, t->ctr, bparts, build_n, NarrowKey{});
    else if (narrow)
        hipLaunchKernelGGL((build_kernel<false, false, true>), dim3(nitems), dim3(kBuildBlock), 0, s, ditems, sorted, srows,
                           w, t->slots, t->reps, t->ctr, bparts, build_n, *narrow);
    else
        hipLaunchKernelGGL((build_kernel<false, false>), dim3(nitems), dim3(kBuildBlock), 0, s, ditems, sorted, srows, w,
                           t->slots, t->reps, t->ctr, bparts, build_n, NarrowKey{});
    FQ_HIP(ctx, hipGetLastError());
    if (nspill) {
        const int grid = (int)std::min<unsigned long long>((nspill + kSpillChunk - 1) / kSpillChunk, 2048);
        hipLaunchKernelGGL(spill_insert_kernel, dim3(grid), dim3(kBuildBlock), 0, s, spill, nspill, t->slots, bits, t->ctr);
        FQ_HIP(ctx, hipGetLastError());
    }
    if (verify_by_items && nitems > 0) {
        hipLaunchKernelGGL(verify_items_kernel, dim3((unsigned int)nitems), dim3(kVerifyBlock), 0, s,
                           (const BuildItem*)ditems, sorted, srows, t->slots, t->reps, t->ks, t->ctr, tup);
        FQ_HIP(ctx, hipGetLastError());
    }
    if (general && nrows > 0 && !verify_by_items) {
        const int grid = (int)std::min<int64_t>((nrows + kFreqBlock - 1) / kFreqBlock, 8192);
        hipLaunchKernelGGL(verify_kernel, dim3(grid), dim3(kFreqBlock), 0, s, t->ks, nrows, t->slots, t->reps, bits,
                           t->ctr);
    }
    FQ_HIP(ctx, hipMemcpyAsync(&t->host_ctr, t->ctr, sizeof(Counters), hipMemcpyDeviceToHost, s));
    std::vector<SummaryPartial> hparts(items.size());
    FQ_HIP(ctx, hipMemcpyAsync(hparts.data(), bparts, items.size() * sizeof(SummaryPartial), hipMemcpyDeviceToHost, s));
    FQ_HIP(ctx, hipStreamSynchronize(s));
    // the fused summary (exact fixed-point terms: any fold order gives the same bits) unless a split bucket needs
    // the table scan
    t->pre_valid = 0;
    if (t->host_ctr.overflow == 0 && t->host_ctr.mismatch == 0 && nspill == 0) {  // spilled keys: the table scan
        bool all = true;
        SummaryPartial acc = {0, 0, 0, 0, 0, 0};
        std::vector<unsigned int> split_buckets;
        for (size_t i = 0; i < hparts.size(); ++i) {
            if (hparts[i].pad) {
                split_buckets.push_back(items[i].bucket);
                continue;
            }
            summary_merge(acc, hparts[i]);
        }
        std::sort(split_buckets.begin(), split_buckets.end());
        split_buckets.erase(std::unique(split_buckets.begin(), split_buckets.end()), split_buckets.end());
        if (!split_buckets.empty()) ctx->freq_paths[DQ_FREQ_PATH_SPLIT_BUCKETS]++;
        if (!split_buckets.empty() && !getenv("DQ_FREQ_SPLIT_SCAN")) {
            // the regions of split buckets (merged with atomics) scanned on their own, not the whole table
            unsigned int* dsb = nullptr;
            SummaryPartial* dsp = nullptr;
            const size_t nsb = split_buckets.size();
            FQ_HIP(ctx, buf.alloc((void**)&dsb, nsb * sizeof(unsigned int)));
            FQ_HIP(ctx, buf.alloc((void**)&dsp, nsb * sizeof(SummaryPartial)));
            FQ_HIP(ctx, hipMemcpyAsync(dsb, split_buckets.data(), nsb * sizeof(unsigned int), hipMemcpyHostToDevice, s));
            hipLaunchKernelGGL(region_summary_kernel, dim3((unsigned int)nsb), dim3(kFreqBlock), 0, s,
                               (const unsigned int*)dsb, (const Slot*)t->slots, build_n, dsp);
            FQ_HIP(ctx, hipGetLastError());
            std::vector<SummaryPartial> hsp(nsb);
            FQ_HIP(ctx, hipMemcpyAsync(hsp.data(), dsp, nsb * sizeof(SummaryPartial), hipMemcpyDeviceToHost, s));
            FQ_HIP(ctx, hipStreamSynchronize(s));
            for (const SummaryPartial& p : hsp) summary_merge(acc, p);
        } else if (!split_buckets.empty()) {
            all = false;
        }
        if (all) {
            t->pre_valid = 1;
            t->pre_n = (int64_t)build_n;
            t->pre_groups = acc.groups;
            t->pre_unique = acc.unique;
            t->pre_maxc = acc.maxc;
            t->pre_ent = acc.ent;
            t->pre_nonfinite = acc.nonfinite;
        }
    }
    if (getenv("DQ_DEBUG_FREQ"))
        fprintf(stderr, "[freq] rows=%lld bits=%d items=%zu rows_taken=%llu ovf=%llu mis=%llu\n", (long long)nrows, bits,
                items.size(), t->host_ctr.num_rows, t->host_ctr.overflow, t->host_ctr.mismatch);
    *overflow = t->host_ctr.overflow != 0;
    *collision = t->host_ctr.mismatch != 0;
    if (*overflow) {  // reset for the retry with more buckets
        Counters c = t->host_ctr;
        c.overflow = 0;
        c.mismatch = 0;
        FQ_HIP(ctx, hipMemcpyAsync(t->ctr, &c, sizeof(Counters), hipMemcpyHostToDevice, s));
        FQ_HIP(ctx, hipStreamSynchronize(s));  // `c` lives on this stack frame
    }
    return DQ_OK;
}

// Small general tables (bits = 0): small_build_kernel + small_check_kernel, the table one region. *overflow sends the
// caller to the regular path, *collision to a new seed.
int build_small(dq_ctx* ctx, dq_freq_table* t, int64_t nrows, double est, DevBuf& buf, bool* overflow, bool* collision,
                bool count_rows = false) {
    hipStream_t s = dq::ctx_stream(ctx);
    if (count_rows) FQ_HIP(ctx, hipMemsetAsync(t->ctr, 0, sizeof(Counters), s));
    release_slots(t, ctx);
    t->home = ctx;
    t->slots_bytes = kRegion * sizeof(Slot);
    t->reps_bytes = kRegion * sizeof(unsigned long long);
    t->slots = (Slot*)dq::scratch_alloc(ctx, t->slots_bytes);
    if (t->slots) t->reps = (unsigned long long*)dq::scratch_alloc(ctx, t->reps_bytes);
    if (!t->slots || !t->reps) return dq::ctx_fail(ctx, DQ_ERR_OUT_OF_MEMORY, "frequency table allocation failed");
    t->cap = kRegion;
    t->bits = 0;
    // one string key column and a table the estimate leaves <= 5/8 full at 1024 slots (the profiler's Histograms, or the
    // optimistic try with no estimate): 1024 slots + the representatives' key words, 36 KB of LDS (4 workgroups per CU)
    const bool str1 = t->ks.ncols == 1 && t->ks.cols[0].spark_type == DQ_TYPE_STRING && est <= 640.0 &&
                      !getenv("DQ_SMALL_NO_STR1");
    const int grid = (int)std::max<int64_t>(
        1, std::min<int64_t>(str1 ? kSmallGrid / 3 * 4 : kSmallGrid, (nrows + kSmallTile - 1) / kSmallTile));
    BuildItem* ditem = nullptr;
    unsigned long long *wk = nullptr, *wr = nullptr;
    FQ_HIP(ctx, buf.alloc((void**)&ditem, sizeof(BuildItem)));
    FQ_HIP(ctx, buf.alloc((void**)&wk, (size_t)grid * kRegion * 8));
    FQ_HIP(ctx, buf.alloc((void**)&wr, (size_t)grid * kRegion * 8));
    const BuildItem it = {0ull, 0ull, 0u, 1u};  // split = 1: region_init clears region 0
    FQ_HIP(ctx, hipMemcpyAsync(ditem, &it, sizeof(it), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(region_init_kernel, dim3(1), dim3(kFreqBlock), 0, s, ditem, 1, t->slots, t->reps);
    ctx->freq_paths[DQ_FREQ_PATH_SMALL]++;
    if (str1)
        hipLaunchKernelGGL((small_build_kernel<1024, true>), dim3(grid), dim3(kBuildBlock), 0, s, t->ks, nrows, t->slots,
                           t->reps, wk, wr, t->ctr, count_rows ? 1 : 0);
    // a 2048-slot workgroup table (40 KB of LDS: 3 workgroups per CU instead of 1) when the estimate leaves it <= 5/8 full
    else if (est <= 1280.0)
        hipLaunchKernelGGL((small_build_kernel<2048>), dim3(grid), dim3(kBuildBlock), 0, s, t->ks, nrows, t->slots, t->reps,
                           wk, wr, t->ctr, count_rows ? 1 : 0);
    else
        hipLaunchKernelGGL((small_build_kernel<kRegion>), dim3(grid), dim3(kBuildBlock), 0, s, t->ks, nrows, t->slots,
                           t->reps, wk, wr, t->ctr, count_rows ? 1 : 0);
    hipLaunchKernelGGL(small_check_kernel, dim3(grid), dim3(kBuildBlock), 0, s, t->ks, t->slots, t->reps, wk, wr, t->ctr);
    FQ_HIP(ctx, hipGetLastError());
    FQ_HIP(ctx, hipMemcpyAsync(&t->host_ctr, t->ctr, sizeof(Counters), hipMemcpyDeviceToHost, s));
    FQ_HIP(ctx, hipStreamSynchronize(s));
    t->pre_valid = 0;  // the summary scans the one region
    if (getenv("DQ_DEBUG_FREQ"))
        fprintf(stderr, "[freq small] rows=%lld grid=%d rows_taken=%llu ovf=%llu mis=%llu\n", (long long)nrows, grid,
                t->host_ctr.num_rows, t->host_ctr.overflow, t->host_ctr.mismatch);
    *overflow = t->host_ctr.overflow != 0;
    *collision = t->host_ctr.mismatch != 0;
    if (*overflow || *collision) {  // the caller rebuilds: clear the flags the rebuild reads
        Counters c = t->host_ctr;
        c.overflow = 0;
        c.mismatch = 0;
        FQ_HIP(ctx, hipMemcpyAsync(t->ctr, &c, sizeof(Counters), hipMemcpyHostToDevice, s));
        FQ_HIP(ctx, hipStreamSynchronize(s));  // `c` lives on this stack frame
    }
    return DQ_OK;
}

// Radix-partition path (8 <= bits <= kMaxPartBits): rows -> 256 partitions (pass 1, fed by the count pass's
// per-workgroup digit histograms) -> buckets (pass 2 on the next bits - 8 bits) -> regions.
constexpr int kMaxPartBits = 20;

int build_partitioned(dq_ctx* ctx, dq_freq_table* t, int64_t nrows, DevBuf& buf, int xgrid, const unsigned int* hist1,
                      unsigned long long n, int bits, bool* collision, const unsigned long long* hrow = nullptr,
                      const unsigned long long* tup = nullptr) {
    hipStream_t s = dq::ctx_stream(ctx);
    const bool general = !t->fast || t->ks.weights != nullptr;  // carry row indices (representatives / weights)
    const size_t n_alloc = (size_t)std::max<unsigned long long>(n, 1);
    unsigned long long *off1 = nullptr, *totals = nullptr, *h1 = nullptr, *r1 = nullptr;
    FQ_HIP(ctx, buf.alloc((void**)&off1, sizeof(unsigned long long) * (size_t)xgrid * kDigitBins));
    FQ_HIP(ctx, buf.alloc((void**)&totals, sizeof(unsigned long long) * kDigitBins));
    FQ_HIP(ctx, buf.alloc((void**)&h1, n_alloc * 8));
    if (general) FQ_HIP(ctx, buf.alloc((void**)&r1, n_alloc * 8));
    hipLaunchKernelGGL(digit_scan_kernel, dim3(kDigitBins), dim3(256), 0, s, hist1, xgrid, kDigitBins, off1, totals);
    if (general)
        hipLaunchKernelGGL((partition1_kernel<true, kPartTile>), dim3(xgrid), dim3(kFreqBlock), 0, s, t->ks, nrows,
                           (const unsigned long long*)off1, (const unsigned long long*)totals, h1, r1, hrow);
    else
        hipLaunchKernelGGL((partition1_kernel<false, kPartTile>), dim3(xgrid), dim3(kFreqBlock), 0, s, t->ks, nrows,
                           (const unsigned long long*)off1, (const unsigned long long*)totals, h1, r1,
                           (const unsigned long long*)nullptr);
    FQ_HIP(ctx, hipGetLastError());
    std::vector<unsigned long long> tot(kDigitBins), pbegin(kDigitBins + 1, 0);
    FQ_HIP(ctx, hipMemcpyAsync(tot.data(), totals, sizeof(unsigned long long) * kDigitBins, hipMemcpyDeviceToHost, s));
    FQ_HIP(ctx, hipStreamSynchronize(s));
    for (int d = 0; d < kDigitBins; ++d) pbegin[d + 1] = pbegin[d] + tot[d];
    unsigned long long *h2 = nullptr, *r2 = nullptr;
    for (int grow = 0; grow < 8 && bits <= kMaxPartBits; ++grow, ++bits) {
        std::vector<unsigned long long> bstart, bcount;
        const unsigned long long *sorted = h1, *srows = r1;
        if (bits == 8) {
            bstart.assign(pbegin.begin(), pbegin.begin() + kDigitBins);
            bcount = tot;
        } else {
            const int d2 = bits - 8;
            const int bins = 1 << d2;
            const bool big = bins > kDigitBins;
            const int BINS = big ? 4096 : kDigitBins;
            std::vector<Pass2Item> items;
            std::vector<int> pitems(kDigitBins + 1, 0);
            for (int p = 0; p < kDigitBins; ++p) {
                pitems[p] = (int)items.size();
                for (unsigned long long x = pbegin[p]; x < pbegin[p + 1]; x += kPass2Item)
                    items.push_back(Pass2Item{x, std::min<unsigned long long>(pbegin[p + 1], x + kPass2Item)});
            }
            pitems[kDigitBins] = (int)items.size();
            const int nitems = (int)items.size();
            Pass2Item* ditems = nullptr;
            int* dpitems = nullptr;
            unsigned long long *dpbegin = nullptr, *off2 = nullptr, *dbstart = nullptr, *dbcount = nullptr;
            unsigned int* cnt2 = nullptr;
            const uint64_t nb = 1ull << bits;
            FQ_HIP(ctx, buf.alloc((void**)&ditems, sizeof(Pass2Item) * std::max(nitems, 1)));
            FQ_HIP(ctx, buf.alloc((void**)&dpitems, sizeof(int) * (kDigitBins + 1)));
            FQ_HIP(ctx, buf.alloc((void**)&dpbegin, sizeof(unsigned long long) * kDigitBins));
            FQ_HIP(ctx, buf.alloc((void**)&cnt2, sizeof(unsigned int) * (size_t)std::max(nitems, 1) * BINS));
            FQ_HIP(ctx, buf.alloc((void**)&off2, sizeof(unsigned long long) * (size_t)std::max(nitems, 1) * BINS));
            FQ_HIP(ctx, buf.alloc((void**)&dbstart, sizeof(unsigned long long) * nb));
            FQ_HIP(ctx, buf.alloc((void**)&dbcount, sizeof(unsigned long long) * nb));
            if (nitems)
                FQ_HIP(ctx, hipMemcpyAsync(ditems, items.data(), sizeof(Pass2Item) * nitems, hipMemcpyHostToDevice, s));
            FQ_HIP(ctx, hipMemcpyAsync(dpitems, pitems.data(), sizeof(int) * (kDigitBins + 1), hipMemcpyHostToDevice, s));
            FQ_HIP(ctx, hipMemcpyAsync(dpbegin, pbegin.data(), sizeof(unsigned long long) * kDigitBins, hipMemcpyHostToDevice, s));
            if (!h2) {
                FQ_HIP(ctx, buf.alloc((void**)&h2, n_alloc * 8));
                if (general) FQ_HIP(ctx, buf.alloc((void**)&r2, n_alloc * 8));
            }
            const unsigned int mask = (unsigned int)bins - 1;
            if (big) {
                if (nitems) hipLaunchKernelGGL(count2_kernel<4096>, dim3(nitems), dim3(kFreqBlock), 0, s, ditems, h1, 8, mask, cnt2);
                hipLaunchKernelGGL(scan2_kernel<4096>, dim3(kDigitBins), dim3(kFreqBlock), 0, s, cnt2, dpitems, dpbegin, bins, off2,
                                   dbstart, dbcount);
                if (nitems && general)
                    hipLaunchKernelGGL((scatter2_kernel<4096, true, kPartTile>), dim3(nitems), dim3(kFreqBlock), 0, s, ditems, off2, h1, r1, 8,
                                       mask, h2, r2);
                else if (nitems)
                    hipLaunchKernelGGL((scatter2_kernel<4096, false, kPartTileFast>), dim3(nitems), dim3(kFreqBlock), 0, s, ditems, off2, h1, r1, 8,
                                       mask, h2, r2);
            } else {
                if (nitems) hipLaunchKernelGGL(count2_kernel<kDigitBins>, dim3(nitems), dim3(kFreqBlock), 0, s, ditems, h1, 8, mask, cnt2);
                hipLaunchKernelGGL(scan2_kernel<kDigitBins>, dim3(kDigitBins), dim3(kFreqBlock), 0, s, cnt2, dpitems, dpbegin, bins,
                                   off2, dbstart, dbcount);
                if (nitems && general)
                    hipLaunchKernelGGL((scatter2_kernel<kDigitBins, true, kPartTile>), dim3(nitems), dim3(kFreqBlock), 0, s, ditems, off2, h1, r1,
                                       8, mask, h2, r2);
                else if (nitems)
                    hipLaunchKernelGGL((scatter2_kernel<kDigitBins, false, kPartTileFast>), dim3(nitems), dim3(kFreqBlock), 0, s, ditems, off2, h1, r1,
                                       8, mask, h2, r2);
            }
            FQ_HIP(ctx, hipGetLastError());
            bstart.resize(nb);
            bcount.resize(nb);
            FQ_HIP(ctx, hipMemcpyAsync(bstart.data(), dbstart, sizeof(unsigned long long) * nb, hipMemcpyDeviceToHost, s));
            FQ_HIP(ctx, hipMemcpyAsync(bcount.data(), dbcount, sizeof(unsigned long long) * nb, hipMemcpyDeviceToHost, s));
            FQ_HIP(ctx, hipStreamSynchronize(s));
            sorted = h2;
            srows = r2;
        }
        bool overflow = false;
        const int rc = build_regions(ctx, t, nrows, buf, sorted, srows, bstart, bcount, bits, &overflow, collision,
                                     nullptr, nullptr, 0, tup);
        if (rc != DQ_OK) return rc;
        if (!overflow) return DQ_OK;
    }
    return dq::ctx_fail(ctx, DQ_ERR_DEVICE, "frequency table build did not converge");
}

// Fast path (one fixed-width key column, unweighted, large inputs): fixed-capacity buckets with atomically
// reserved runs (partition1_fast -> scatter2_fast -> regions), no count pass. Sets *done = false, having built
// nothing that the exact path cannot redo, when a bucket overflows its capacity (heavy hitters) or the table is
// too small or too large for the two-pass bucketing.
constexpr int64_t kFastMinRows = 1 << 24;
constexpr int64_t kOptimisticSmallRows = 1 << 22;  // below: the sizing pass is cheap, keep the sized path

// Signed min / max of the canonical values of a strided sample of an 8-byte integral key column (narrow-key choice):
// one sampled row per thread (no dependent load chain), block minima / maxima folded with 64-bit atomics.
constexpr int kNarrowSample = 1 << 16;

__global__ void __launch_bounds__(256)
narrow_sample_kernel(KeyCol c, int64_t nrows, long long* __restrict__ out) {
    __shared__ long long smin[4], smax[4];
    const int64_t stride = nrows / kNarrowSample > 0 ? nrows / kNarrowSample : 1;
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t r = k * stride;
    long long lo = LLONG_MAX, hi = LLONG_MIN;
    if (r < nrows && (!c.validity || ((c.validity[r >> 3] >> (r & 7)) & 1u))) {
        lo = hi = static_cast<const long long*>(c.values)[r];
    }
    for (int o = 32; o > 0; o >>= 1) {
        const long long l2 = __shfl_down(lo, o, 64), h2 = __shfl_down(hi, o, 64);
        lo = l2 < lo ? l2 : lo;
        hi = h2 > hi ? h2 : hi;
    }
    if ((threadIdx.x & 63) == 0) {
        smin[threadIdx.x >> 6] = lo;
        smax[threadIdx.x >> 6] = hi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 4; ++w) {
            lo = smin[w] < lo ? smin[w] : lo;
            hi = smax[w] > hi ? smax[w] : hi;
        }
        atomicMin(&out[0], lo);
        atomicMax(&out[1], hi);
    }
}

// The narrow-key window for the fast path's key column (see NarrowKey), or false for 64-bit keys.
bool choose_narrow(dq_ctx* ctx, const dq_freq_table* t, int64_t nrows, DevBuf& buf, NarrowKey* nk, int* rc) {
    *rc = DQ_OK;
    const KeyCol& c = t->ks.cols[0];
    const ElemType elem = (ElemType)c.elem;
    const int w = elem_size(elem);
    if (getenv("DQ_FREQ_WIDE")) return false;
    if (w <= 4) {  // the canonical value is the cell's 32 bits, sign-extended for the signed types
        *nk = NarrowKey{0ull, (elem == ET_F32 || elem == ET_U8) ? 0 : 1, 0};
        return true;
    }
    if (elem == ET_F64) return false;  // the bit patterns of doubles seldom share 32 high bits
    hipStream_t s = dq::ctx_stream(ctx);
    long long* d = nullptr;
    if (buf.alloc((void**)&d, 2 * sizeof(long long)) != hipSuccess) {
        *rc = dq::ctx_fail(ctx, DQ_ERR_OUT_OF_MEMORY, "narrow-key sample allocation failed");
        return false;
    }
    static const long long init[2] = {LLONG_MAX, LLONG_MIN};
    if (hipMemcpyAsync(d, init, sizeof(init), hipMemcpyHostToDevice, s) != hipSuccess) {
        *rc = dq::ctx_fail(ctx, DQ_ERR_DEVICE, "narrow-key sample failed");
        return false;
    }
    hipLaunchKernelGGL(narrow_sample_kernel, dim3(kNarrowSample / 256), dim3(256), 0, s, c, nrows, d);
    long long mm[2];
    if (hipMemcpyAsync(mm, d, sizeof(mm), hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess) {
        *rc = dq::ctx_fail(ctx, DQ_ERR_DEVICE, "narrow-key sample failed");
        return false;
    }
    if (mm[0] > mm[1]) {  // no valid row in the sample
        *nk = NarrowKey{0ull, 1, 0};
        return true;
    }
    const unsigned long long range = (unsigned long long)mm[1] - (unsigned long long)mm[0];
    if (range >= (1ull << 31)) return false;
    // the window [base, base + 2^32) centred on the sample's range
    *nk = NarrowKey{(unsigned long long)mm[0] - ((0xFFFFFFFFull - range) >> 1), 0, 0};
    return true;
}

int build_fast(dq_ctx* ctx, dq_freq_table* t, int64_t nrows, DevBuf& buf, bool* done, bool allow_narrow = true) {
    *done = false;
    hipStream_t s = dq::ctx_stream(ctx);
    const int xgrid = scan_grid((uint64_t)nrows);
    NarrowKey nk{0ull, 0, 0};
    bool narrow = false;
    if (allow_narrow) {
        int rc = DQ_OK;
        narrow = choose_narrow(ctx, t, nrows, buf, &nk, &rc);
        if (rc != DQ_OK) return rc;
    }
    const size_t ksz = narrow ? 4 : 8;  // bytes per key in the partition buffers
    // pass 1: 256 partitions x 8 XCD sub-regions of cap1 keys (the expected share plus slack for hashing variance
    // and repeated keys)
    constexpr int kSub = kDigitBins * kP1Sub;
    const unsigned long long share = (unsigned long long)(nrows / kSub);
    const unsigned long long cap1 = share + share / 8 + 16384;
    unsigned long long* gc1 = nullptr;
    void* h1 = nullptr;
    unsigned int* regs = nullptr;
    uint8_t* regs_part = nullptr;
    FQ_HIP(ctx, buf.alloc((void**)&gc1, sizeof(unsigned long long) * kSub * kCursorStride));
    FQ_HIP(ctx, buf.alloc((void**)&h1, cap1 * kSub * ksz));
    FQ_HIP(ctx, buf.alloc((void**)&regs, kFastRegs * sizeof(unsigned int)));
    FQ_HIP(ctx, buf.alloc((void**)&regs_part, (size_t)kFastRegs * xgrid));
    // spill buffer: room for a quarter of the rows past full buckets (heavily repeated keys); more sends the build to
    // the exactly-counted path
    Spill sp{nullptr, (unsigned long long)nrows / 4 + (1ull << 20), &t->ctr->spilled};
    FQ_HIP(ctx, buf.alloc((void**)&sp.keys, sp.cap * sizeof(unsigned long long)));
    FQ_HIP(ctx, hipMemsetAsync(gc1, 0, sizeof(unsigned long long) * kSub * kCursorStride, s));
    FQ_HIP(ctx, hipMemsetAsync(regs, 0, kFastRegs * sizeof(unsigned int), s));
    FQ_HIP(ctx, hipMemsetAsync(t->ctr, 0, sizeof(Counters), s));
    const int inul = t->ks.include_nulls ? 1 : 0;
    // (measured: an 8 K-key pass-1 tile runs 8.1 ms against 6.1 ms for 4 K on C4 -- twice the registers)
#define DQ_P1(W, N, F)                                                                                              \
    hipLaunchKernelGGL((partition1_fast_kernel<kP1TileFast, W, N, F>), dim3(xgrid), dim3(kFreqBlock), 0, s,            \
                       t->ks.cols[0], nrows, inul, cap1, gc1, h1, regs_part, t->ctr, nk, sp)
    ctx->freq_paths[narrow ? DQ_FREQ_PATH_FAST_NARROW : DQ_FREQ_PATH_FAST]++;
    {
        const ElemType e1 = (ElemType)t->ks.cols[0].elem;
        const bool flt = e1 == ET_F64 || e1 == ET_F32 || e1 == ET_U8;  // NaN canonical / BOOLEAN 0-1
        switch (elem_size(e1)) {
            case 8:
                if (flt) { if (narrow) DQ_P1(8, true, true); else DQ_P1(8, false, true); }
                else { if (narrow) DQ_P1(8, true, false); else DQ_P1(8, false, false); }
                break;
            case 4:
                if (flt) { if (narrow) DQ_P1(4, true, true); else DQ_P1(4, false, true); }
                else { if (narrow) DQ_P1(4, true, false); else DQ_P1(4, false, false); }
                break;
            case 2:
                if (narrow) DQ_P1(2, true, false); else DQ_P1(2, false, false);
                break;
            default:
                if (flt) { if (narrow) DQ_P1(1, true, true); else DQ_P1(1, false, true); }
                else { if (narrow) DQ_P1(1, true, false); else DQ_P1(1, false, false); }
                break;
        }
    }
#undef DQ_P1
    hipLaunchKernelGGL(sizing_reduce_kernel, dim3(kFastRegs / 256, std::min(xgrid, 64)), dim3(256), 0, s,
                       (const uint8_t*)regs_part, xgrid, kFastRegs, regs);
    FQ_HIP(ctx, hipGetLastError());
    std::vector<unsigned int> hregs(kFastRegs);
    std::vector<unsigned long long> pcount(kSub), pstrided((size_t)kSub * kCursorStride);
    FQ_HIP(ctx, hipMemcpyAsync(hregs.data(), regs, kFastRegs * sizeof(unsigned int), hipMemcpyDeviceToHost, s));
    FQ_HIP(ctx, hipMemcpyAsync(pstrided.data(), gc1, sizeof(unsigned long long) * kSub * kCursorStride,
                               hipMemcpyDeviceToHost, s));
    FQ_HIP(ctx, hipMemcpyAsync(&t->host_ctr, t->ctr, sizeof(Counters), hipMemcpyDeviceToHost, s));
    FQ_HIP(ctx, hipStreamSynchronize(s));
    if (t->host_ctr.pad[0]) return DQ_OK;  // the spill buffer overflowed: the exact path
    if (t->host_ctr.narrow_miss) {  // an 8-byte key outside the sampled window: again with 64-bit keys
        if (getenv("DQ_DEBUG_FREQ"))
            fprintf(stderr, "[freq fast] narrow window missed by %llu rows\n", t->host_ctr.narrow_miss);
        return build_fast(ctx, t, nrows, buf, done, false);
    }
    // a sub-region's reservations past its capacity went to the spill buffer
    for (int q = 0; q < kSub; ++q) pcount[q] = std::min(pstrided[(size_t)q * kCursorStride], cap1);
    const unsigned long long spilled1 = t->host_ctr.spilled;
    unsigned long long n = 0;
    for (unsigned long long c : pcount) n += c;
    const double est = n ? (double)(1u << kSketchBits) * hll_raw_estimate(hregs) : 0.0;  // a 1/512 sample of the keys
    int bits = 0;
    while (bits < 40 && est / (double)(1ull << bits) > (double)kRegionTarget) ++bits;
    if (getenv("DQ_DEBUG_FREQ"))
        fprintf(stderr, "[freq fast] rows=%lld n=%llu est=%.1f bits=%d narrow=%d\n", (long long)nrows, n, est, bits,
                (int)narrow);
    if (bits < 8 || bits > kMaxPartBits) return DQ_OK;
    bits = std::max(bits, 9);  // a partition is 8 sub-regions: the second pass gathers them into buckets
    void* h2 = nullptr;
    size_t h2_bytes = 0;
    for (int grow = 0; grow < 8 && bits <= kMaxPartBits; ++grow, ++bits) {
        std::vector<unsigned long long> bstart, bcount;
        const void* sorted = h1;
        {
            const int bins = 1 << (bits - 8);
            const uint64_t nb = 1ull << bits;
            const unsigned long long per = n / nb;
            const unsigned long long cap2 = per + per / 4 + 2048;
            // work items: chunks of each sub-region, dealt round-robin over the partitions so the workgroups in flight
            // reserve on different buckets' counters
            std::vector<std::vector<FastItem>> by_part(kDigitBins);
            for (int q = 0; q < kSub; ++q) {
                const unsigned long long base = (unsigned long long)q * cap1;
                for (unsigned long long x = 0; x < pcount[q]; x += kPass2Item)
                    by_part[q / kP1Sub].push_back(FastItem{base + x, base + std::min<unsigned long long>(pcount[q], x + kPass2Item),
                                                           (unsigned int)(q / kP1Sub), 0u});
            }
            std::vector<FastItem> items;
            for (size_t round = 0;; ++round) {
                bool any = false;
                for (int p = 0; p < kDigitBins; ++p)
                    if (round < by_part[p].size()) {
                        items.push_back(by_part[p][round]);
                        any = true;
                    }
                if (!any) break;
            }
            const int nitems = (int)items.size();
            FastItem* ditems = nullptr;
            unsigned long long* gc2 = nullptr;
            FQ_HIP(ctx, buf.alloc((void**)&ditems, sizeof(FastItem) * std::max(nitems, 1)));
            FQ_HIP(ctx, buf.alloc((void**)&gc2, sizeof(unsigned long long) * nb));
            if (cap2 * nb * ksz > h2_bytes) {
                h2_bytes = cap2 * nb * ksz;
                FQ_HIP(ctx, buf.alloc((void**)&h2, h2_bytes));
            }
            FQ_HIP(ctx, hipMemsetAsync(gc2, 0, sizeof(unsigned long long) * nb, s));
            // a retry with more buckets keeps pass 1's spilled keys and drops the previous pass 2's
            FQ_HIP(ctx, hipMemcpyAsync(&t->ctr->spilled, &spilled1, sizeof(spilled1), hipMemcpyHostToDevice, s));
            if (nitems) FQ_HIP(ctx, hipMemcpyAsync(ditems, items.data(), sizeof(FastItem) * nitems, hipMemcpyHostToDevice, s));
            const unsigned int mask = (unsigned int)bins - 1;
#define DQ_P2(B, T, N)                                                                                            \
    hipLaunchKernelGGL((scatter2_fast_kernel<B, T, N>), dim3(nitems), dim3(kFreqBlock), 0, s, ditems, h1, mask, cap2, \
                       gc2, h2, t->ctr, nk, sp)
            if (nitems && bins > kDigitBins) {
                if (narrow) DQ_P2(4096, kPartTile, true); else DQ_P2(4096, kPartTile, false);
            } else if (nitems) {
                if (narrow) DQ_P2(kDigitBins, kPartTileFast, true); else DQ_P2(kDigitBins, kPartTileFast, false);
            }
#undef DQ_P2
            FQ_HIP(ctx, hipGetLastError());
            std::vector<unsigned long long> pb(nb);
            FQ_HIP(ctx, hipMemcpyAsync(pb.data(), gc2, sizeof(unsigned long long) * nb, hipMemcpyDeviceToHost, s));
            FQ_HIP(ctx, hipMemcpyAsync(&t->host_ctr, t->ctr, sizeof(Counters), hipMemcpyDeviceToHost, s));
            FQ_HIP(ctx, hipStreamSynchronize(s));
            if (t->host_ctr.pad[1]) return DQ_OK;  // the spill buffer overflowed: the exact path
            bstart.resize(nb);
            bcount.resize(nb);
            for (uint64_t k = 0; k < nb; ++k) {
                bstart[k] = k * cap2;
                bcount[k] = std::min(pb[(k & (kDigitBins - 1)) * (uint64_t)bins + (k >> 8)], cap2);
            }
            sorted = h2;
        }
        bool overflow = false, collision = false;
        const unsigned long long nspill = std::min(t->host_ctr.spilled, sp.cap);
        const int rc = build_regions(ctx, t, nrows, buf, static_cast<const unsigned long long*>(sorted), nullptr, bstart,
                                     bcount, bits, &overflow, &collision, narrow ? &nk : nullptr, sp.keys, nspill);
        if (rc != DQ_OK) return rc;
        if (!overflow) {
            *done = true;
            ctx->freq_paths[DQ_FREQ_PATH_FAST_DONE]++;
            if (nspill) ctx->freq_paths[DQ_FREQ_PATH_FAST_SPILL]++;
            return DQ_OK;
        }
    }
    return DQ_OK;
}

// extract (+ sizing) -> bucketing on the low `bits` bits of the keys -> per-bucket LDS aggregation. Tables of
// 8..20 bucket bits take the radix-partition path; the others compact the keys and sort them on the bucket
// bits with rocPRIM. A bucket whose distinct keys overflow its region (or a fingerprint collision on the
// general path) restarts with more bucket bits (or a new seed).
int build_table(dq_ctx* ctx, dq_freq_table* t, int64_t nrows) {
    hipStream_t s = dq::ctx_stream(ctx);
    DevBuf buf(ctx);
    const bool general = !t->fast || t->ks.weights != nullptr;  // carry row indices (representatives / weights)
    const bool no_partition = getenv("DQ_FREQ_NO_PARTITION") != nullptr;
    if (t->fast && !t->ks.weights && !no_partition && nrows >= kFastMinRows && !getenv("DQ_FREQ_EXACT")) {
        bool done = false;
        const int rc = build_fast(ctx, t, nrows, buf, &done);
        if (rc != DQ_OK || done) return rc;
    }
    // General keys, unweighted: try the one-pass small build first, without the sizing pass (a histogram column the
    // ColumnProfiler sends here has <= 120 distinct values). A workgroup whose LDS table fills stops at once and the
    // build takes the sized path below (the cost of a wrong guess: a few thousand rows per workgroup); a fingerprint
    // collision also goes there (it re-seeds).
    bool many_keys = false;  // the optimistic small build overflowed: a large table, its keys worth keeping per row
    if (general && !t->ks.weights && nrows >= kOptimisticSmallRows && !getenv("DQ_FREQ_NO_SMALL") &&
        !getenv("DQ_FREQ_NO_OPTIMISTIC")) {
        bool overflow = false, collision = false;
        const int rc = build_small(ctx, t, nrows, 0.0, buf, &overflow, &collision, true);
        many_keys = overflow;
        if (rc != DQ_OK) return rc;
        if (!overflow && !collision) {
            ctx->freq_paths[DQ_FREQ_PATH_SMALL_OPTIMISTIC]++;
            return DQ_OK;
        }
    }
    for (int seed_attempt = 0; seed_attempt < 4; ++seed_attempt) {
        unsigned long long *hs = nullptr, *rows = nullptr, *bk = nullptr;
        unsigned int *regs = nullptr, *hist1 = nullptr;
        uint8_t* regs_part = nullptr;
        const size_t n_alloc = (size_t)std::max<int64_t>(nrows, 1);
        const int xgrid = scan_grid((uint64_t)std::max<int64_t>(nrows, 1));
        FQ_HIP(ctx, buf.alloc((void**)&bk, 2 * sizeof(unsigned long long) * xgrid));
        FQ_HIP(ctx, buf.alloc((void**)&regs, kSizingRegs * sizeof(unsigned int)));
        FQ_HIP(ctx, buf.alloc((void**)&regs_part, (size_t)kSizingRegs * xgrid));
        FQ_HIP(ctx, buf.alloc((void**)&hist1, sizeof(unsigned int) * (size_t)xgrid * kDigitBins));
        FQ_HIP(ctx, hipMemsetAsync(bk, 0, 2 * sizeof(unsigned long long) * xgrid, s));
        FQ_HIP(ctx, hipMemsetAsync(regs, 0, kSizingRegs * sizeof(unsigned int), s));
        FQ_HIP(ctx, hipMemsetAsync(t->ctr, 0, sizeof(Counters), s));
        // general keys of a large table: the count pass writes every row's key and the partition pass reads it back
        // (8 B a row instead of reading and hashing the key columns twice)
        unsigned long long* hrow = nullptr;
        if (general && many_keys && !getenv("DQ_FREQ_NO_HROW")) FQ_HIP(ctx, buf.alloc((void**)&hrow, n_alloc * 8));
        // one string key column: its rows as two-word tuples too, so the verification compares 16-byte tuples
        // instead of both rows' offsets and bytes
        unsigned long long* tup = nullptr;
        if (hrow && t->ks.ncols == 1 && t->ks.cols[0].spark_type == DQ_TYPE_STRING && !getenv("DQ_FREQ_NO_TUPLES"))
            FQ_HIP(ctx, buf.alloc((void**)&tup, n_alloc * 16));
        ctx->freq_paths[DQ_FREQ_PATH_EXACT]++;
        if (nrows > 0) {
            hipLaunchKernelGGL(extract_count_kernel, dim3(xgrid), dim3(kFreqBlock), 0, s, t->ks, nrows, bk, regs_part,
                               t->ctr, hist1, kPartTile, hrow, tup);
            hipLaunchKernelGGL(sizing_reduce_kernel, dim3(kSizingRegs / 256, std::min(xgrid, 64)), dim3(256), 0, s,
                               (const uint8_t*)regs_part, xgrid, kSizingRegs, regs);
        }
        FQ_HIP(ctx, hipGetLastError());
        std::vector<unsigned int> hregs(kSizingRegs);
        std::vector<unsigned long long> hkeep(xgrid), hoff(xgrid);
        FQ_HIP(ctx, hipMemcpyAsync(hregs.data(), regs, kSizingRegs * sizeof(unsigned int), hipMemcpyDeviceToHost, s));
        FQ_HIP(ctx, hipMemcpyAsync(hkeep.data(), bk, sizeof(unsigned long long) * xgrid, hipMemcpyDeviceToHost, s));
        FQ_HIP(ctx, hipMemcpyAsync(&t->host_ctr, t->ctr, sizeof(Counters), hipMemcpyDeviceToHost, s));
        FQ_HIP(ctx, hipStreamSynchronize(s));
        if (tup && t->host_ctr.pad[2]) ctx->freq_paths[DQ_FREQ_PATH_LONG_TUPLES]++;
        unsigned long long n = 0;
        for (int g = 0; g < xgrid; ++g) {
            hoff[g] = n;
            n += hkeep[g];
        }
        const double est = n ? hll_raw_estimate(hregs) : 0.0;
        int bits = 0;
        while (bits < 40 && est / (double)(1ull << bits) > (double)kRegionTarget) ++bits;
        if (getenv("DQ_DEBUG_FREQ"))
            fprintf(stderr, "[freq] rows=%lld n=%llu est=%.1f bits=%d\n", (long long)nrows, n, est, bits);
        bool collision = false;
        if (general && !t->ks.weights && bits == 0 && n > 0 && !getenv("DQ_FREQ_NO_SMALL")) {
            bool overflow = false;
            const int rc = build_small(ctx, t, nrows, est, buf, &overflow, &collision);
            if (rc != DQ_OK) return rc;
            if (!overflow && !collision) return DQ_OK;
            if (collision) {
                t->ks.seed = mix64(t->ks.seed + 0x9E3779B97F4A7C15ULL);
                continue;
            }
            collision = false;  // a full table: the regular path below
        }
        if (!no_partition && n > 0 && bits >= 8 && bits <= kMaxPartBits) {
            ctx->freq_paths[DQ_FREQ_PATH_PARTITIONED]++;
            const int rc = build_partitioned(ctx, t, nrows, buf, xgrid, hist1, n, bits, &collision, hrow, tup);
            if (rc != DQ_OK) return rc;
            if (!collision) return DQ_OK;
            t->ks.seed = mix64(t->ks.seed + 0x9E3779B97F4A7C15ULL);
            continue;
        }
        ctx->freq_paths[DQ_FREQ_PATH_SORTED]++;
        FQ_HIP(ctx, buf.alloc((void**)&hs, n_alloc * 8));
        if (general) FQ_HIP(ctx, buf.alloc((void**)&rows, n_alloc * 8));
        if (nrows > 0) {
            FQ_HIP(ctx, hipMemcpyAsync(bk + xgrid, hoff.data(), sizeof(unsigned long long) * xgrid, hipMemcpyHostToDevice, s));
            hipLaunchKernelGGL(extract_write_kernel, dim3(xgrid), dim3(kFreqBlock), 0, s, t->ks, nrows,
                               (const unsigned long long*)(bk + xgrid), hs, rows, kPartTile);
            FQ_HIP(ctx, hipGetLastError());
        }
        unsigned long long *hs2 = nullptr, *rows2 = nullptr;
        FQ_HIP(ctx, buf.alloc((void**)&hs2, n_alloc * 8));
        if (general) FQ_HIP(ctx, buf.alloc((void**)&rows2, n_alloc * 8));
        bool overflow = true;
        for (int grow = 0; grow < 8 && overflow; ++grow, ++bits) {
            // ---- sort on the low `bits` bits: each bucket becomes one contiguous run ----------------
            const unsigned long long* sorted = hs;
            const unsigned long long* srows = rows;
            if (bits > 0 && n > 1) {
                size_t tmp_bytes = 0;
                void* tmp = nullptr;
                if (general) {
                    FQ_HIP(ctx, rocprim::radix_sort_pairs(nullptr, tmp_bytes, hs, hs2, rows, rows2, (size_t)n, 0u,
                                                          (unsigned)bits, s));
                    FQ_HIP(ctx, buf.alloc(&tmp, tmp_bytes));
                    FQ_HIP(ctx, rocprim::radix_sort_pairs(tmp, tmp_bytes, hs, hs2, rows, rows2, (size_t)n, 0u, (unsigned)bits, s));
                    srows = rows2;
                } else {
                    FQ_HIP(ctx, rocprim::radix_sort_keys(nullptr, tmp_bytes, hs, hs2, (size_t)n, 0u, (unsigned)bits, s));
                    FQ_HIP(ctx, buf.alloc(&tmp, tmp_bytes));
                    FQ_HIP(ctx, rocprim::radix_sort_keys(tmp, tmp_bytes, hs, hs2, (size_t)n, 0u, (unsigned)bits, s));
                }
                sorted = hs2;
            }
            const uint64_t nb = 1ull << bits;
            unsigned long long* bounds = nullptr;
            FQ_HIP(ctx, buf.alloc((void**)&bounds, (nb + 1) * 8));
            hipLaunchKernelGGL(bucket_bounds_kernel, dim3((unsigned)((nb + 1 + 255) / 256)), dim3(256), 0, s, sorted,
                               (uint64_t)n, bits, nb, bounds);
            std::vector<unsigned long long> hb(nb + 1), bstart(nb), bcount(nb);
            FQ_HIP(ctx, hipMemcpyAsync(hb.data(), bounds, (nb + 1) * 8, hipMemcpyDeviceToHost, s));
            FQ_HIP(ctx, hipStreamSynchronize(s));
            for (uint64_t b = 0; b < nb; ++b) {
                bstart[b] = hb[b];
                bcount[b] = hb[b + 1] - hb[b];
            }
            const int rc = build_regions(ctx, t, nrows, buf, sorted, srows, bstart, bcount, bits, &overflow, &collision);
            if (rc != DQ_OK) return rc;
        }
        if (overflow) return dq::ctx_fail(ctx, DQ_ERR_DEVICE, "frequency table build did not converge");
        if (!collision) return DQ_OK;
        // 64-bit fingerprint collision on the general path: new seed, rebuild from scratch
        t->ks.seed = mix64(t->ks.seed + 0x9E3779B97F4A7C15ULL);
    }
    return dq::ctx_fail(ctx, DQ_ERR_DEVICE, "frequency table build did not converge");
}


// ---- multi-device grouping: owner-device bucketing of (canonical key, count) pairs -------------------------
__device__ __forceinline__ int pair_owner(uint64_t canon, int nparts) {
    return (int)((mix64(canon) >> 32) % (uint64_t)nparts);
}

__global__ void __launch_bounds__(kFreqBlock)
pair_owner_count_kernel(const long long* __restrict__ keys, int64_t n, int nparts, unsigned long long* __restrict__ counts) {
    __shared__ unsigned int lds[64];
    for (int i = threadIdx.x; i < 64; i += kFreqBlock) lds[i] = 0;
    __syncthreads();
    for (int64_t r = (int64_t)blockIdx.x * kFreqBlock + threadIdx.x; r < n; r += (int64_t)gridDim.x * kFreqBlock)
        atomicAdd(&lds[pair_owner((uint64_t)keys[r], nparts)], 1u);
    __syncthreads();
    for (int i = threadIdx.x; i < nparts; i += kFreqBlock)
        if (lds[i]) atomicAdd(&counts[i], (unsigned long long)lds[i]);
}

__global__ void __launch_bounds__(kFreqBlock)
pair_owner_scatter_kernel(const long long* __restrict__ keys, const long long* __restrict__ cnts, int64_t n, int nparts,
                          unsigned long long* __restrict__ cursors, long long* __restrict__ out_keys,
                          long long* __restrict__ out_cnts) {
    for (int64_t r = (int64_t)blockIdx.x * kFreqBlock + threadIdx.x; r < n; r += (int64_t)gridDim.x * kFreqBlock) {
        const int p = pair_owner((uint64_t)keys[r], nparts);
        const unsigned long long at = atomicAdd(&cursors[p], 1ull);
        out_keys[at] = keys[r];
        out_cnts[at] = cnts[r];
    }
}

struct MultiFreqJob {
    std::vector<const dq_column*> cols;
    std::vector<int64_t> rows;
    int ncols;
    const int32_t* key_columns;
    const dq_freq_options* opt;
    int ndev;
    // per device
    std::vector<dq_freq_table*> local;
    std::vector<int64_t> local_rows, local_nulls;
    std::vector<int64_t*> send_keys, send_cnts, recv_keys, recv_cnts;
    std::vector<int64_t> counts;  // ndev x ndev
};

int multi_local_build(int i, dq_ctx* sub, void* arg) {
    MultiFreqJob* j = static_cast<MultiFreqJob*>(arg);
    dq_freq_table* t = nullptr;
    int rc = dq_frequencies_ex(sub, j->cols[i], j->ncols, j->rows[i], j->key_columns, 1, j->opt, &t);
    if (rc) return rc;
    j->local[i] = t;
    dq_freq_summary su;
    rc = dq_freq_summarize(sub, t, 0, &su);
    if (rc) return rc;
    j->local_rows[i] = su.num_rows;
    j->local_nulls[i] = su.null_count;
    const int64_t g = su.num_groups - (su.null_count ? 1 : 0);
    hipStream_t s = dq::ctx_stream(sub);
    int64_t *ek = nullptr, *ec = nullptr;
    if (hipMalloc(&ek, (size_t)std::max<int64_t>(g, 1) * 8) != hipSuccess ||
        hipMalloc(&ec, (size_t)std::max<int64_t>(g, 1) * 8) != hipSuccess ||
        hipMalloc(&j->send_keys[i], (size_t)std::max<int64_t>(g, 1) * 8) != hipSuccess ||
        hipMalloc(&j->send_cnts[i], (size_t)std::max<int64_t>(g, 1) * 8) != hipSuccess)
        return dq::ctx_fail(sub, DQ_ERR_OUT_OF_MEMORY, "exchange buffers");
    const int64_t got = dq_freq_export_device(sub, t, g, ek, ec);
    if (got < 0) return (int)got;
    unsigned long long* dc = nullptr;
    FQ_HIP(sub, hipMalloc(&dc, sizeof(unsigned long long) * 128));
    FQ_HIP(sub, hipMemsetAsync(dc, 0, sizeof(unsigned long long) * 128, s));
    const int grid = scan_grid((uint64_t)std::max<int64_t>(got, 1));
    if (got) hipLaunchKernelGGL(pair_owner_count_kernel, dim3(grid), dim3(kFreqBlock), 0, s, (const long long*)ek, got,
                                j->ndev, dc);
    std::vector<unsigned long long> h(64);
    FQ_HIP(sub, hipMemcpyAsync(h.data(), dc, 64 * 8, hipMemcpyDeviceToHost, s));
    FQ_HIP(sub, hipStreamSynchronize(s));
    std::vector<unsigned long long> cur(64, 0);
    unsigned long long off = 0;
    for (int p = 0; p < j->ndev; ++p) {
        cur[p] = off;
        j->counts[(size_t)i * j->ndev + p] = (int64_t)h[p];
        off += h[p];
    }
    FQ_HIP(sub, hipMemcpyAsync(dc + 64, cur.data(), 64 * 8, hipMemcpyHostToDevice, s));
    if (got) hipLaunchKernelGGL(pair_owner_scatter_kernel, dim3(grid), dim3(kFreqBlock), 0, s, (const long long*)ek,
                                (const long long*)ec, got, j->ndev, dc + 64, (long long*)j->send_keys[i],
                                (long long*)j->send_cnts[i]);
    FQ_HIP(sub, hipGetLastError());
    FQ_HIP(sub, hipStreamSynchronize(s));
    (void)hipFree(ek);
    (void)hipFree(ec);
    (void)hipFree(dc);
    dq_freq_free(sub, t);
    j->local[i] = nullptr;
    return DQ_OK;
}

struct OwnerBuildJob {
    MultiFreqJob* j;
    int32_t key_type;
    int64_t nulls;
    std::vector<dq_freq_table*> parts;
};

int multi_owner_build(int i, dq_ctx* sub, void* arg) {
    OwnerBuildJob* o = static_cast<OwnerBuildJob*>(arg);
    MultiFreqJob* j = o->j;
    int64_t total = 0;
    for (int src = 0; src < j->ndev; ++src) total += j->counts[(size_t)src * j->ndev + i];
    return dq_freq_from_pairs(sub, o->key_type, j->recv_keys[i], j->recv_cnts[i], total, DQ_FREQ_PAIRS_DEVICE, total,
                              i == 0 ? o->nulls : 0, &o->parts[i]);
}

// ---- general keys (strings, several columns) on a multi-device context -------------------------------------
// Each device pre-aggregates its shard (dq_frequencies_ex on the general path) and exports its groups as
// (smallest row, count). Every group goes to the owner device picked by a hash of its key; the owner gathers
// the key cells of its groups (in row order) and builds the weighted table over them, so the groups of one key
// from every shard merge and the parts are disjoint. Groups are few next to rows, so their key bytes travel
// through host memory; the fixed-width path above moves (key, count) pairs device to device over RCCL.

// Grouping equality on the host: canonical fixed-width bits (NaN canonical, -0.0 != 0.0), string bytes, NULL a
// fixed component (or "NullValue" for a Histogram string column) -- equal keys hash equally.
uint64_t host_key_hash(const dq_column* columns, const int32_t* key_columns, int nkeys, int64_t r, bool null_is_value) {
    uint64_t acc = 0x243F6A8885A308D3ULL;
    for (int i = 0; i < nkeys; ++i) {
        const dq_column& c = columns[key_columns[i]];
        const bool valid = !c.validity || ((c.validity[r >> 3] >> (r & 7)) & 1);
        uint64_t ch;
        if (c.spark_type == DQ_TYPE_STRING) {
            if (valid) {
                const int32_t o0 = c.offsets[r], o1 = c.offsets[r + 1];
                ch = xxh_bytes(static_cast<const uint8_t*>(c.values) + o0, o1 - o0, 42);
            } else {
                ch = null_is_value ? xxh_bytes((const uint8_t*)"NullValue", 9, 42) : 0x6A09E667F3BCC909ULL;
            }
        } else if (valid) {
            uint64_t v;
            switch (elem_of(c.spark_type)) {
                case ET_U8: v = static_cast<const uint8_t*>(c.values)[r] ? 1ull : 0ull; break;
                case ET_I8: v = (uint64_t)(int64_t) static_cast<const int8_t*>(c.values)[r]; break;
                case ET_I16: v = (uint64_t)(int64_t) static_cast<const int16_t*>(c.values)[r]; break;
                case ET_I32: v = (uint64_t)(int64_t) static_cast<const int32_t*>(c.values)[r]; break;
                case ET_F32: v = (uint64_t)float_to_int_bits(static_cast<const float*>(c.values)[r]); break;
                case ET_F64: v = double_to_long_bits(static_cast<const double*>(c.values)[r]); break;
                default: v = static_cast<const uint64_t*>(c.values)[r]; break;
            }
            ch = mix64(v);
        } else {
            ch = 0x6A09E667F3BCC909ULL;
        }
        acc = mix64(acc + 0xC2B2AE3D27D4EB4FULL * (uint64_t)(i + 1) + ch);
    }
    return acc;
}


void gather_keys(const dq_column* columns, const int32_t* key_columns, int nkeys, const std::vector<int64_t>& rows,
                 GatheredKeys& g) {
    const size_t n = rows.size();
    g.values.assign(nkeys, {});
    g.validity.assign(nkeys, {});
    g.offsets.assign(nkeys, {});
    g.cols.assign(nkeys, dq_column());
    for (int i = 0; i < nkeys; ++i) {
        const dq_column& c = columns[key_columns[i]];
        dq_column& o = g.cols[i];
        o = c;
        o.flags = 0;
        o.length = (int64_t)n;
        std::vector<uint8_t>& vb = g.validity[i];
        vb.assign((n + 7) / 8 + 8, 0);
        bool all = true;
        for (size_t k = 0; k < n; ++k) {
            const int64_t r = rows[k];
            const bool valid = !c.validity || ((c.validity[r >> 3] >> (r & 7)) & 1);
            if (valid) vb[k >> 3] |= (uint8_t)(1u << (k & 7)); else all = false;
        }
        o.validity = all ? nullptr : vb.data();
        if (c.spark_type == DQ_TYPE_STRING) {
            std::vector<int32_t>& off = g.offsets[i];
            off.assign(n + 1, 0);
            size_t total = 0;
            for (size_t k = 0; k < n; ++k) {
                total += (size_t)(c.offsets[rows[k] + 1] - c.offsets[rows[k]]);
                off[k + 1] = (int32_t)total;
            }
            g.values[i].assign(total + 16, 0);
            for (size_t k = 0; k < n; ++k) {
                const int32_t o0 = c.offsets[rows[k]], len = c.offsets[rows[k] + 1] - o0;
                if (len) memcpy(g.values[i].data() + off[k], static_cast<const uint8_t*>(c.values) + o0, (size_t)len);
            }
            o.offsets = off.data();
        } else {
            const int w = std::max(1, elem_size(elem_of(c.spark_type)));
            g.values[i].assign(n * w + 16, 0);
            for (size_t k = 0; k < n; ++k)
                memcpy(g.values[i].data() + k * w, static_cast<const uint8_t*>(c.values) + rows[k] * w, (size_t)w);
            o.offsets = nullptr;
        }
        o.values = g.values[i].data();
    }
}

struct GeneralJob {
    const dq_column* columns;       // the caller's (host) columns
    std::vector<std::vector<dq_column>> shard_cols;
    std::vector<int64_t> row0, rows;
    int ncols, nkeys;
    const int32_t* key_columns;
    const dq_freq_options* opt;
    int ndev;
    bool null_is_value;
    std::vector<std::vector<int64_t>> grp_rows, grp_counts;  // per device: exported groups (global rows)
    std::vector<int64_t> local_rows, local_nulls;
    // per owner
    std::vector<std::vector<int64_t>> own_rows, own_counts;
    std::vector<GatheredKeys> own_keys;
    std::vector<dq_freq_table*> parts;
};

int general_local(int i, dq_ctx* sub, void* arg) {
    GeneralJob* j = static_cast<GeneralJob*>(arg);
    dq_freq_table* t = nullptr;
    int rc = dq_frequencies_ex(sub, j->shard_cols[i].data(), j->ncols, j->rows[i], j->key_columns, j->nkeys, j->opt, &t);
    if (rc) return rc;
    dq_freq_summary su;
    rc = dq_freq_summarize(sub, t, 0, &su);
    if (!rc) {
        j->local_rows[i] = su.num_rows;
        j->local_nulls[i] = su.null_count;
        const int64_t g = su.num_groups - (su.null_count ? 1 : 0);
        j->grp_rows[i].assign((size_t)std::max<int64_t>(g, 1), 0);
        j->grp_counts[i].assign((size_t)std::max<int64_t>(g, 1), 0);
        const int64_t got = dq_freq_export(sub, t, g, j->grp_rows[i].data(), j->grp_counts[i].data());
        if (got < 0) {
            rc = (int)got;
        } else {
            j->grp_rows[i].resize((size_t)got);
            j->grp_counts[i].resize((size_t)got);
            for (int64_t& r : j->grp_rows[i]) r += j->row0[i];
        }
    }
    dq_freq_free(sub, t);
    return rc;
}

int general_owner(int i, dq_ctx* sub, void* arg) {
    GeneralJob* j = static_cast<GeneralJob*>(arg);
    GatheredKeys& g = j->own_keys[i];
    gather_keys(j->columns, j->key_columns, j->nkeys, j->own_rows[i], g);
    g.counts = j->own_counts[i];
    std::vector<int32_t> keys(j->nkeys);
    for (int k = 0; k < j->nkeys; ++k) keys[k] = k;
    dq_freq_options o = *j->opt;
    o.weights = j->own_counts[i].empty() ? nullptr : j->own_counts[i].data();
    o.weights_device = 0;
    return dq_frequencies_ex(sub, g.cols.data(), j->nkeys, (int64_t)j->own_rows[i].size(), keys.data(), j->nkeys, &o,
                             &j->parts[i]);
}

int multi_frequencies_general(dq_ctx* ctx, const dq_column* columns, int ncols, int64_t nrows,
                              const int32_t* key_columns, int nkeys, const dq_freq_options* opt, dq_freq_table** out) {
    const int n = (int)ctx->subs.size();
    GeneralJob j;
    j.columns = columns;
    j.ncols = ncols;
    j.nkeys = nkeys;
    j.key_columns = key_columns;
    j.opt = opt;
    j.ndev = n;
    j.null_is_value = (opt->flags & DQ_FREQ_INCLUDE_NULLS) && nkeys == 1 && columns[key_columns[0]].spark_type == DQ_TYPE_STRING;
    j.shard_cols.assign(n, std::vector<dq_column>(std::max(ncols, 1)));
    j.row0.assign(n, 0);
    j.rows.assign(n, 0);
    j.grp_rows.assign(n, {});
    j.grp_counts.assign(n, {});
    j.local_rows.assign(n, 0);
    j.local_nulls.assign(n, 0);
    std::vector<std::vector<std::vector<int32_t>>> scratch(n);
    for (int i = 0; i < n; ++i) {
        dq::shard_bounds(nrows, n, i, &j.row0[i], &j.rows[i]);
        dq::shard_columns(columns, ncols, j.row0[i], j.rows[i], j.shard_cols[i].data(), scratch[i]);
    }
    int rc = dq::for_each_device(ctx, general_local, &j);
    if (rc) return rc;
    // owner of every group; each owner's groups in row order (its smallest row stays the group's smallest row)
    j.own_rows.assign(n, {});
    j.own_counts.assign(n, {});
    std::vector<std::vector<std::pair<int64_t, int64_t>>> own(n);
    for (int i = 0; i < n; ++i)
        for (size_t k = 0; k < j.grp_rows[i].size(); ++k) {
            const int64_t r = j.grp_rows[i][k];
            const int dst = (int)((mix64(host_key_hash(columns, key_columns, nkeys, r, j.null_is_value)) >> 32) % (uint64_t)n);
            own[dst].push_back({r, j.grp_counts[i][k]});
        }
    for (int i = 0; i < n; ++i) {
        std::sort(own[i].begin(), own[i].end());
        for (const auto& rc_ : own[i]) {
            j.own_rows[i].push_back(rc_.first);
            j.own_counts[i].push_back(rc_.second);
        }
    }
    j.parts.assign(n, nullptr);
    j.own_keys.assign(n, GatheredKeys());
    rc = dq::for_each_device(ctx, general_owner, &j);
    if (rc) {
        for (int i = 0; i < n; ++i)
            if (j.parts[i]) dq_freq_free(ctx->subs[i], j.parts[i]);
        return rc;
    }
    dq_freq_table* t = new dq_freq_table();
    t->device = ctx->device;
    memset(&t->ks, 0, sizeof(t->ks));
    t->fast = 0;
    t->key_type = nkeys == 1 ? columns[key_columns[0]].spark_type : 0;
    t->parts = j.parts;
    t->part_ctx = ctx->subs;
    t->part_rows = std::move(j.own_rows);
    t->part_keys = std::move(j.own_keys);  // (moving the inner vectors keeps the column pointers valid)
    int64_t total_rows = 0;
    for (int i = 0; i < n; ++i) total_rows += j.local_rows[i];
    t->total_rows = total_rows;
    *out = t;
    return DQ_OK;
}

int multi_frequencies(dq_ctx* ctx, const dq_column* columns, int ncols, int64_t nrows, const int32_t* key_columns,
                      int nkeys, const dq_freq_options* opt, dq_freq_table** out) {
    for (int c = 0; c < ncols; ++c)
        if (columns[c].flags & (DQ_COL_DEVICE | DQ_COL_OFFSETS64))
            return dq::ctx_fail(ctx, DQ_ERR_UNSUPPORTED, "multi-device grouping takes host columns with int32 offsets");
    if (opt->weights)
        return dq::ctx_fail(ctx, DQ_ERR_UNSUPPORTED, "multi-device grouping: weighted input takes a one-device context");
    for (int k = 0; k < nkeys; ++k)
        if (key_columns[k] < 0 || key_columns[k] >= ncols)
            return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_frequencies: bad key column");
    if (nkeys != 1 || elem_of(columns[key_columns[0]].spark_type) == ET_NONE)
        return multi_frequencies_general(ctx, columns, ncols, nrows, key_columns, nkeys, opt, out);
    const int n = (int)ctx->subs.size();
    MultiFreqJob j;
    j.ncols = ncols;
    j.key_columns = key_columns;
    j.opt = opt;
    j.ndev = n;
    j.local.assign(n, nullptr);
    j.local_rows.assign(n, 0);
    j.local_nulls.assign(n, 0);
    j.send_keys.assign(n, nullptr);
    j.send_cnts.assign(n, nullptr);
    j.recv_keys.assign(n, nullptr);
    j.recv_cnts.assign(n, nullptr);
    j.counts.assign((size_t)n * n, 0);
    std::vector<std::vector<dq_column>> cols(n, std::vector<dq_column>(std::max(ncols, 1)));
    std::vector<std::vector<std::vector<int32_t>>> scratch(n);
    j.rows.resize(n);
    j.cols.resize(n);
    for (int i = 0; i < n; ++i) {
        int64_t r0 = 0;
        dq::shard_bounds(nrows, n, i, &r0, &j.rows[i]);
        dq::shard_columns(columns, ncols, r0, j.rows[i], cols[i].data(), scratch[i]);
        j.cols[i] = cols[i].data();
    }
    auto release = [&]() {
        for (int i = 0; i < n; ++i) {
            (void)hipSetDevice(ctx->subs[i]->device);
            for (int64_t* p : {j.send_keys[i], j.send_cnts[i], j.recv_keys[i], j.recv_cnts[i]})
                if (p) (void)hipFree(p);
            if (j.local[i]) dq_freq_free(ctx->subs[i], j.local[i]);
        }
    };
    int rc = dq::for_each_device(ctx, multi_local_build, &j);  // local pre-aggregation + owner bucketing
    if (rc) { release(); return rc; }
    std::vector<int64_t> send_off((size_t)n * n), recv_off((size_t)n * n);
    for (int i = 0; i < n; ++i) {
        int64_t so = 0, ro = 0;
        for (int p = 0; p < n; ++p) {
            send_off[(size_t)i * n + p] = so;
            so += j.counts[(size_t)i * n + p];
            recv_off[(size_t)i * n + p] = ro;  // receiver i, records from source p
            ro += j.counts[(size_t)p * n + i];
        }
        (void)hipSetDevice(ctx->subs[i]->device);
        if (hipMalloc(&j.recv_keys[i], (size_t)std::max<int64_t>(ro, 1) * 8) != hipSuccess ||
            hipMalloc(&j.recv_cnts[i], (size_t)std::max<int64_t>(ro, 1) * 8) != hipSuccess) {
            release();
            return dq::ctx_fail(ctx, DQ_ERR_OUT_OF_MEMORY, "exchange receive buffers");
        }
    }
    rc = dq::exchange_i64(ctx, j.send_keys, j.recv_keys, j.counts, send_off, recv_off);
    if (!rc) rc = dq::exchange_i64(ctx, j.send_cnts, j.recv_cnts, j.counts, send_off, recv_off);
    if (rc) { release(); return rc; }
    OwnerBuildJob o;
    o.j = &j;
    o.key_type = columns[key_columns[0]].spark_type;
    o.nulls = 0;
    int64_t total_rows = 0;
    for (int i = 0; i < n; ++i) {
        o.nulls += j.local_nulls[i];
        total_rows += j.local_rows[i];
    }
    o.parts.assign(n, nullptr);
    rc = dq::for_each_device(ctx, multi_owner_build, &o);
    release();
    if (rc) {
        for (int i = 0; i < n; ++i)
            if (o.parts[i]) dq_freq_free(ctx->subs[i], o.parts[i]);
        return rc;
    }
    dq_freq_table* t = new dq_freq_table();
    t->device = ctx->device;
    memset(&t->ks, 0, sizeof(t->ks));
    t->fast = 1;
    t->key_type = o.key_type;
    t->parts = o.parts;
    t->part_ctx = ctx->subs;
    t->total_rows = total_rows;
    for (int i = 0; i < n; ++i) {  // the pair arrays die with this call: parts keep only their slots
        o.parts[i]->ks.weights = nullptr;
        o.parts[i]->ks.cols[0].values = nullptr;
    }
    *out = t;
    return DQ_OK;
}

}  // namespace

extern "C" {

int dq_frequencies(dq_ctx* ctx, const dq_column* columns, int ncols, int64_t nrows, const int32_t* key_columns,
                   int nkeys, uint32_t flags, dq_freq_table** out) {
    dq_freq_options o;
    memset(&o, 0, sizeof(o));
    o.flags = flags;
    return dq_frequencies_ex(ctx, columns, ncols, nrows, key_columns, nkeys, &o, out);
}

static int finish_frequencies(dq_ctx* ctx, dq_freq_table* t, int64_t nrows, const dq_freq_options* opt,
                              std::vector<void*>& staged, dq_freq_table** out);

int dq_frequencies_ex(dq_ctx* ctx, const dq_column* columns, int ncols, int64_t nrows, const int32_t* key_columns,
                      int nkeys, const dq_freq_options* opt, dq_freq_table** out) {
    if (!ctx || !out || !opt || nkeys <= 0 || nkeys > kMaxKeys || nrows < 0)
        return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_frequencies: invalid arguments");
    if (!ctx->subs.empty()) return multi_frequencies(ctx, columns, ncols, nrows, key_columns, nkeys, opt, out);
    *out = nullptr;
    const int dev = dq::ctx_device(ctx);
    FQ_HIP(ctx, hipSetDevice(dev));
    hipStream_t s = dq::ctx_stream(ctx);
    dq_freq_table* t = new dq_freq_table();
    t->device = dev;
    t->src_rows = nrows;
    memset(&t->ks, 0, sizeof(t->ks));
    std::vector<void*> staged;
    auto cleanup = [&]() {
        for (void* p : staged) (void)hipFree(p);
    };
    for (int i = 0; i < nkeys; ++i) {
        const int c = key_columns[i];
        if (c < 0 || c >= ncols || columns[c].length != nrows) {
            delete t;
            return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_frequencies: bad key column");
        }
        const dq_column& col = columns[c];
        KeyCol& kc = t->ks.cols[i];
        kc.spark_type = col.spark_type;
        kc.elem = elem_of(col.spark_type);
        const bool off64 = col.spark_type == DQ_TYPE_STRING && (col.flags & DQ_COL_OFFSETS64);
        kc.offsets64 = nullptr;
        if (col.flags & DQ_COL_DEVICE) {
            kc.values = col.values;
            kc.validity = col.validity;
            kc.offsets = off64 ? nullptr : col.offsets;
            kc.offsets64 = off64 ? reinterpret_cast<const int64_t*>(col.offsets) : nullptr;
        } else {
            // stage host buffers (kept alive with the table: rows are re-read by verify / export)
            const int64_t send = (!nrows || col.spark_type != DQ_TYPE_STRING)
                                     ? 0
                                     : (off64 ? reinterpret_cast<const int64_t*>(col.offsets)[nrows]
                                              : (int64_t)col.offsets[nrows]);
            size_t vbytes = col.spark_type == DQ_TYPE_STRING ? (size_t)send
                                                              : (size_t)nrows * std::max(1, elem_size(kc.elem));
            void* v = nullptr;
            FQ_HIP(ctx, hipMalloc(&v, vbytes + 16));
            staged.push_back(v);
            if (vbytes) FQ_HIP(ctx, hipMemcpyAsync(v, col.values, vbytes, hipMemcpyHostToDevice, s));
            kc.values = v;
            if (col.validity) {
                void* vd = nullptr;
                const size_t nb = (size_t)(nrows + 7) / 8;
                FQ_HIP(ctx, hipMalloc(&vd, nb + 8));
                staged.push_back(vd);
                if (nb) FQ_HIP(ctx, hipMemcpyAsync(vd, col.validity, nb, hipMemcpyHostToDevice, s));
                kc.validity = (const uint8_t*)vd;
            }
            if (col.spark_type == DQ_TYPE_STRING) {
                const size_t ow = off64 ? 8 : 4;
                void* od = nullptr;
                FQ_HIP(ctx, hipMalloc(&od, ((size_t)nrows + 1) * ow));
                staged.push_back(od);
                FQ_HIP(ctx, hipMemcpyAsync(od, col.offsets, ((size_t)nrows + 1) * ow, hipMemcpyHostToDevice, s));
                kc.offsets = off64 ? nullptr : (const int32_t*)od;
                kc.offsets64 = off64 ? (const int64_t*)od : nullptr;
            }
        }
        if (kc.elem == ET_NONE && kc.spark_type != DQ_TYPE_STRING) {
            cleanup();
            delete t;
            return dq::ctx_fail(ctx, DQ_ERR_UNSUPPORTED, "dq_frequencies: unsupported key type");
        }
    }
    t->ks.ncols = nkeys;
    return finish_frequencies(ctx, t, nrows, opt, staged, out);
}

// The common tail of dq_frequencies_ex / dq_frequencies_parts: `t->ks.cols[0 .. nkeys)` are set up.
static int finish_frequencies(dq_ctx* ctx, dq_freq_table* t, int64_t nrows, const dq_freq_options* opt,
                              std::vector<void*>& staged, dq_freq_table** out) {
    const uint32_t flags = opt->flags;
    hipStream_t s = dq::ctx_stream(ctx);
    auto cleanup = [&]() {
        for (void* p : staged) (void)hipFree(p);
    };
    if (opt->weights && nrows > 0) {
        if (opt->weights_device) {
            t->ks.weights = reinterpret_cast<const long long*>(opt->weights);
        } else {
            void* w = nullptr;
            FQ_HIP(ctx, hipMalloc(&w, (size_t)nrows * 8));
            staged.push_back(w);
            FQ_HIP(ctx, hipMemcpyAsync(w, opt->weights, (size_t)nrows * 8, hipMemcpyHostToDevice, s));
            t->ks.weights = reinterpret_cast<const long long*>(w);
        }
    }
    const int nkeys = t->ks.ncols;
    t->key_type = opt->key_type ? opt->key_type : t->ks.cols[0].spark_type;
    t->ks.include_nulls = (flags & DQ_FREQ_INCLUDE_NULLS) ? 1 : 0;
    // the fast build reads one fixed-width column's values directly: one part only
    t->ks.fast = (nkeys == 1 && t->ks.cols[0].spark_type != DQ_TYPE_STRING && !t->ks.cols[0].split) ? 1 : 0;
    t->ks.string_null_is_value = (t->ks.include_nulls && nkeys == 1 && t->ks.cols[0].spark_type == DQ_TYPE_STRING);
    t->fast = t->ks.fast;
    t->ks.seed = 0x243F6A8885A308D3ULL;
    t->ks.fp_mask = ~0ull;
    if (const char* m = getenv("DQ_FREQ_FP_MASK")) t->ks.fp_mask = strtoull(m, nullptr, 0);

    t->buf_home = ctx;
    t->ctr = (Counters*)dq::scratch_alloc(ctx, sizeof(Counters));
    if (!t->ctr) {
        cleanup();
        delete t;
        return dq::ctx_fail(ctx, DQ_ERR_OUT_OF_MEMORY, "frequency table allocation failed");
    }
    int rc = build_table(ctx, t, nrows);
    if (rc) {
        cleanup();
        free_table_buffers(t, ctx);
        delete t;
        return rc;
    }
    t->scratch_bytes = kScanBlocks * (sizeof(SummaryPartial) + 3 * sizeof(unsigned long long)) + 2048 * 8 + 256;
    t->scratch = dq::scratch_alloc(ctx, t->scratch_bytes);
    if (!t->scratch) {
        cleanup();
        free_table_buffers(t, ctx);
        delete t;
        return dq::ctx_fail(ctx, DQ_ERR_OUT_OF_MEMORY, "frequency table allocation failed");
    }
    t->staged = staged;
    *out = t;
    return DQ_OK;
}

int dq_frequencies_parts(dq_ctx* ctx, const dq_column* parts, int nparts, int ncols, const int32_t* key_columns,
                         int nkeys, const dq_freq_options* opt, dq_freq_table** out) {
    if (!ctx || !out || !opt || !parts || nparts <= 0 || ncols <= 0 || nkeys <= 0 || nkeys > kMaxKeys)
        return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_frequencies_parts: invalid arguments");
    if (nparts == 1) return dq_frequencies_ex(ctx, parts, ncols, parts[0].length, key_columns, nkeys, opt, out);
    if (nparts != 2 || !ctx->subs.empty() || opt->weights)
        return dq::ctx_fail(ctx, DQ_ERR_UNSUPPORTED,
                            "dq_frequencies_parts: two parts on a one-device context, unweighted (else concatenate)");
    *out = nullptr;
    const int64_t n0 = parts[0].length, n1 = parts[ncols].length;
    FQ_HIP(ctx, hipSetDevice(dq::ctx_device(ctx)));
    dq_freq_table* t = new dq_freq_table();
    t->device = dq::ctx_device(ctx);
    t->src_rows = n0 + n1;
    memset(&t->ks, 0, sizeof(t->ks));
    for (int i = 0; i < nkeys; ++i) {
        const int c = key_columns[i];
        const dq_column* a = c >= 0 && c < ncols ? &parts[c] : nullptr;
        const dq_column* b = c >= 0 && c < ncols ? &parts[ncols + c] : nullptr;
        if (!a || !(a->flags & DQ_COL_DEVICE) || !(b->flags & DQ_COL_DEVICE) || (a->flags & DQ_COL_OFFSETS64) ||
            (b->flags & DQ_COL_OFFSETS64) || a->spark_type != b->spark_type || a->length != n0 || b->length != n1 ||
            (elem_of(a->spark_type) == ET_NONE && a->spark_type != DQ_TYPE_STRING)) {
            delete t;
            return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT,
                                "dq_frequencies_parts: key parts must be device columns of one type, int32 offsets");
        }
        KeyCol& kc = t->ks.cols[i];
        kc.spark_type = a->spark_type;
        kc.elem = elem_of(a->spark_type);
        kc.values = a->values;
        kc.validity = a->validity;
        kc.offsets = a->offsets;
        kc.offsets64 = nullptr;
        if (n0 > 0) {  // an empty first part: the second part alone is the column
            kc.split = n0;
            kc.values2 = b->values;
            kc.validity2 = b->validity;
            kc.offsets2 = b->offsets;
        } else {
            kc.values = b->values;
            kc.validity = b->validity;
            kc.offsets = b->offsets;
        }
    }
    t->ks.ncols = nkeys;
    std::vector<void*> staged;
    return finish_frequencies(ctx, t, n0 + n1, opt, staged, out);
}

int dq_freq_key_kind(const dq_freq_table* t) { return !t ? -1 : (t->fast ? DQ_FREQ_KEYS_VALUES : DQ_FREQ_KEYS_ROWS); }

int dq_freq_summarize(dq_ctx* ctx, const dq_freq_table* t, int64_t entropy_rows, dq_freq_summary* out) {
    if (!ctx || !t || !out) return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_freq_summarize: invalid arguments");
    if (!t->parts.empty()) {
        // union of disjoint per-device tables: counts add, the exact entropy sums (global N) add
        const int64_t n = entropy_rows > 0 ? entropy_rows : t->total_rows;
        dq_freq_summary acc;
        memset(&acc, 0, sizeof(acc));
        fx128 ent = 0;
        bool nonfinite = false;
        for (size_t i = 0; i < t->parts.size(); ++i) {
            dq_freq_summary p;
            const int rc = dq_freq_summarize(t->part_ctx[i], t->parts[i], n, &p);
            if (rc) return dq::ctx_fail(ctx, rc, t->part_ctx[i]->err.c_str());
            acc.num_groups += p.num_groups;
            acc.num_unique += p.num_unique;
            acc.max_count = std::max(acc.max_count, p.max_count);
            acc.null_count += p.null_count;
            ent += (fx128)(((unsigned __int128)(uint64_t)p.entropy_fx_hi << 64) | p.entropy_fx_lo);
            nonfinite |= !std::isfinite(p.entropy);
        }
        acc.num_rows = t->total_rows;
        acc.entropy_rows = n;
        acc.entropy = nonfinite ? NAN : fx_to_double(ent);
        acc.entropy_fx_lo = (uint64_t)ent;
        acc.entropy_fx_hi = (int64_t)(ent >> 64);
        *out = acc;
        return DQ_OK;
    }
    FQ_HIP(ctx, hipSetDevice(t->device));
    hipStream_t s = dq::ctx_stream(ctx);
    const int64_t table_rows = t->num_rows_override >= 0 ? t->num_rows_override : (int64_t)t->host_ctr.num_rows;
    const int64_t n = entropy_rows > 0 ? entropy_rows : table_rows;
    if (t->cached_n == n) {  // one table scan serves every analyzer of the grouping
        *out = t->cached;
        return DQ_OK;
    }
    SummaryPartial acc = {0, 0, 0, 0, 0, 0};
    if (t->pre_valid && t->pre_n == n && !getenv("DQ_FREQ_NO_FUSED_SUMMARY")) {  // folded into the build: no scan
        acc.groups = t->pre_groups;
        acc.unique = t->pre_unique;
        acc.maxc = t->pre_maxc;
        acc.ent = t->pre_ent;
        acc.nonfinite = t->pre_nonfinite;
    } else {
        SummaryPartial* parts = (SummaryPartial*)t->scratch;
        const int grid = summary_grid();
        hipLaunchKernelGGL(summary_kernel, dim3(grid), dim3(kFreqBlock), 0, s, t->slots, t->cap, (double)n, parts);
        FQ_HIP(ctx, hipGetLastError());
        std::vector<SummaryPartial> hp(grid);
        FQ_HIP(ctx, hipMemcpyAsync(hp.data(), parts, sizeof(SummaryPartial) * grid, hipMemcpyDeviceToHost, s));
        FQ_HIP(ctx, hipStreamSynchronize(s));
        for (const SummaryPartial& p : hp) summary_merge(acc, p);
    }
    // side groups: the fast path's EMPTY-colliding value and (Histogram) the NULL group; their terms come from the
    // device's entropy_term like every other group's, so a group's term does not depend on where it is kept
    const unsigned long long side[2] = {t->host_ctr.sentinel, t->host_ctr.nulls};
    for (unsigned long long extra : side) {
        if (!extra) continue;
        acc.groups += 1;
        acc.unique += extra == 1;
        acc.maxc = std::max(acc.maxc, extra);
    }
    if (n > 0 && (side[0] || side[1])) {
        SummaryPartial* d = (SummaryPartial*)t->scratch;
        hipLaunchKernelGGL(side_terms_kernel, dim3(1), dim3(64), 0, s, side[0], side[1], (double)n, d);
        FQ_HIP(ctx, hipGetLastError());
        SummaryPartial hs;
        FQ_HIP(ctx, hipMemcpyAsync(&hs, d, sizeof(hs), hipMemcpyDeviceToHost, s));
        FQ_HIP(ctx, hipStreamSynchronize(s));
        acc.ent += hs.ent;
        acc.nonfinite += hs.nonfinite;
    }
    out->num_rows = table_rows;
    out->num_groups = (int64_t)acc.groups;
    out->num_unique = (int64_t)acc.unique;
    out->entropy = acc.nonfinite ? NAN : fx_to_double(acc.ent);
    out->entropy_fx_lo = (uint64_t)acc.ent;
    out->entropy_fx_hi = (int64_t)(acc.ent >> 64);
    out->entropy_rows = n;
    out->max_count = (int64_t)acc.maxc;
    out->null_count = (int64_t)t->host_ctr.nulls;
    dq_freq_table* mt = const_cast<dq_freq_table*>(t);
    mt->cached = *out;
    mt->cached_n = n;
    return DQ_OK;
}

static int64_t compact(dq_ctx* ctx, const dq_freq_table* t, int mode, unsigned long long thr, uint64_t limit,
                       std::vector<unsigned long long>& keys, std::vector<unsigned long long>& counts) {
    hipStream_t s = dq::ctx_stream(ctx);
    unsigned long long* per_block = (unsigned long long*)((char*)t->scratch + kScanBlocks * sizeof(SummaryPartial));
    unsigned long long* offsets = per_block + kScanBlocks;
    hipLaunchKernelGGL(count_selected_kernel, dim3(kScanBlocks), dim3(kFreqBlock), 0, s, t->slots, t->cap, mode, thr,
                       per_block);
    std::vector<unsigned long long> pb(kScanBlocks), off(kScanBlocks);
    if (hipMemcpyAsync(pb.data(), per_block, kScanBlocks * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return -1;
    unsigned long long total = 0;
    for (int b = 0; b < kScanBlocks; ++b) {
        off[b] = total;
        total += pb[b];
    }
    const uint64_t n = std::min<uint64_t>(total, limit);
    keys.assign(n, 0);
    counts.assign(n, 0);
    if (n == 0) return 0;
    unsigned long long* dk = nullptr;
    unsigned long long* dc = nullptr;
    DevBuf buf(ctx);  // the context's scratch cache: no device-wide wait of a hipFree per export
    if (buf.alloc((void**)&dk, n * 8) != hipSuccess || buf.alloc((void**)&dc, n * 8) != hipSuccess) return -1;
    if (hipMemcpyAsync(offsets, off.data(), kScanBlocks * 8, hipMemcpyHostToDevice, s) != hipSuccess) return -1;
    hipLaunchKernelGGL(compact_kernel, dim3(kScanBlocks), dim3(kFreqBlock), 0, s, t->slots, t->reps, t->cap, mode, thr,
                       offsets, (unsigned long long)n, dk, dc, 0);
    bool ok = hipMemcpyAsync(keys.data(), dk, n * 8, hipMemcpyDeviceToHost, s) == hipSuccess &&
              hipMemcpyAsync(counts.data(), dc, n * 8, hipMemcpyDeviceToHost, s) == hipSuccess &&
              hipStreamSynchronize(s) == hipSuccess;
    return ok ? (int64_t)n : -1;
}

static void decode_keys(const dq_freq_table* t, std::vector<unsigned long long>& keys) {
    if (t->fast)
        for (auto& k : keys) k = unmix64(k);
}

int64_t dq_freq_export(dq_ctx* ctx, const dq_freq_table* t, int64_t capacity, int64_t* keys, int64_t* counts) {
    if (!ctx || !t || capacity < 0 || (capacity > 0 && (!keys || !counts))) return DQ_ERR_INVALID_ARGUMENT;
    if (!t->parts.empty()) {
        int64_t n = 0;
        for (size_t i = 0; i < t->parts.size() && n < capacity; ++i) {
            const int64_t got = dq_freq_export(t->part_ctx[i], t->parts[i], capacity - n, keys + n, counts + n);
            if (got < 0) return dq::ctx_fail(ctx, (int)got, t->part_ctx[i]->err.c_str());
            if (!t->part_rows.empty())
                for (int64_t x = n; x < n + got; ++x) keys[x] = t->part_rows[i][(size_t)keys[x]];
            n += got;
        }
        return n;
    }
    if (hipSetDevice(t->device) != hipSuccess) return DQ_ERR_DEVICE;
    std::vector<unsigned long long> k, c;
    if (compact(ctx, t, 2, 0, (uint64_t)capacity, k, c) < 0) return dq::ctx_fail(ctx, DQ_ERR_DEVICE, "export failed");
    decode_keys(t, k);
    int64_t n = (int64_t)k.size();
    for (int64_t i = 0; i < n; ++i) {
        keys[i] = (int64_t)k[i];
        counts[i] = (int64_t)c[i];
    }
    if (t->host_ctr.sentinel && n < capacity) {
        keys[n] = (int64_t)unmix64(kEmpty);
        counts[n] = (int64_t)t->host_ctr.sentinel;
        ++n;
    }
    return n;
}

int64_t dq_freq_top(dq_ctx* ctx, const dq_freq_table* t, int64_t k, int64_t* keys, int64_t* counts) {
    if (!ctx || !t || k < 0 || (k > 0 && (!keys || !counts))) return DQ_ERR_INVALID_ARGUMENT;
    if (k == 0) return 0;
    if (!t->parts.empty()) {
        // every device's top-k, then the k largest of the candidates (ties: device order, then slot order)
        std::vector<std::pair<int64_t, int64_t>> all;  // (count, key)
        std::vector<int64_t> pk((size_t)k), pc((size_t)k);
        for (size_t i = 0; i < t->parts.size(); ++i) {
            const int64_t got = dq_freq_top(t->part_ctx[i], t->parts[i], k, pk.data(), pc.data());
            if (got < 0) return dq::ctx_fail(ctx, (int)got, t->part_ctx[i]->err.c_str());
            for (int64_t x = 0; x < got; ++x)
                all.push_back({pc[x], t->part_rows.empty() ? pk[x] : t->part_rows[i][(size_t)pk[x]]});
        }
        std::stable_sort(all.begin(), all.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
        const int64_t n = std::min<int64_t>(k, (int64_t)all.size());
        for (int64_t x = 0; x < n; ++x) {
            keys[x] = all[x].second;
            counts[x] = all[x].first;
        }
        return n;
    }
    if (hipSetDevice(t->device) != hipSuccess) return DQ_ERR_DEVICE;
    hipStream_t s = dq::ctx_stream(ctx);
    // Radix select of the k-th largest count over three 11-bit digits.
    unsigned long long* hist = (unsigned long long*)((char*)t->scratch + kScanBlocks * sizeof(SummaryPartial) +
                                                     2 * kScanBlocks * 8);
    unsigned long long prefix = 0, prefix_mask = 0;
    uint64_t remaining = (uint64_t)k;
    std::vector<unsigned long long> h(2048);
    bool exhausted = false;
    for (int shift : {33, 22, 11, 0}) {  // 44-bit counts (>> any row count)
        if (hipMemsetAsync(hist, 0, 2048 * 8, s) != hipSuccess) return DQ_ERR_DEVICE;
        hipLaunchKernelGGL(digit_hist_kernel, dim3(scan_grid(t->cap)), dim3(kFreqBlock), 0, s, t->slots, t->cap, shift,
                           prefix_mask, prefix, hist);
        if (hipMemcpyAsync(h.data(), hist, 2048 * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return DQ_ERR_DEVICE;
        int d = 2047;
        uint64_t acc = 0;
        for (; d >= 0; --d) {
            if (acc + h[d] >= remaining) break;
            acc += h[d];
        }
        if (d < 0) {  // fewer groups than k: take all of them
            exhausted = true;
            break;
        }

        remaining -= acc;
        prefix |= (unsigned long long)d << shift;
        prefix_mask |= 2047ull << shift;
    }
    std::vector<unsigned long long> gk, gc, tk, tc;
    if (exhausted) {
        if (compact(ctx, t, 2, 0, UINT64_MAX, gk, gc) < 0) return DQ_ERR_DEVICE;
    } else {
        if (compact(ctx, t, 0, prefix, UINT64_MAX, gk, gc) < 0) return DQ_ERR_DEVICE;
        if (compact(ctx, t, 1, prefix, remaining, tk, tc) < 0) return DQ_ERR_DEVICE;
    }
    decode_keys(t, gk);
    decode_keys(t, tk);
    std::vector<std::pair<unsigned long long, unsigned long long>> all;  // (count, key)
    for (size_t i = 0; i < gk.size(); ++i) all.push_back({gc[i], gk[i]});
    for (size_t i = 0; i < tk.size(); ++i) all.push_back({tc[i], tk[i]});
    if (t->host_ctr.sentinel) all.push_back({t->host_ctr.sentinel, unmix64(kEmpty)});
    std::stable_sort(all.begin(), all.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
    const int64_t n = std::min<int64_t>(k, (int64_t)all.size());
    for (int64_t i = 0; i < n; ++i) {
        keys[i] = (int64_t)all[i].second;
        counts[i] = (int64_t)all[i].first;
    }
    return n;
}


int64_t dq_freq_export_device(dq_ctx* ctx, const dq_freq_table* t, int64_t capacity, int64_t* keys_dev,
                              int64_t* counts_dev) {
    if (!ctx || !t || capacity < 0 || (capacity > 0 && (!keys_dev || !counts_dev)))
        return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_freq_export_device: invalid arguments");
    if (!t->fast || !t->parts.empty())
        return dq::ctx_fail(ctx, DQ_ERR_UNSUPPORTED, "dq_freq_export_device: needs a single-device table of values");
    FQ_HIP(ctx, hipSetDevice(t->device));
    hipStream_t s = dq::ctx_stream(ctx);
    unsigned long long* per_block = (unsigned long long*)((char*)t->scratch + kScanBlocks * sizeof(SummaryPartial));
    unsigned long long* offsets = per_block + kScanBlocks;
    hipLaunchKernelGGL(count_selected_kernel, dim3(kScanBlocks), dim3(kFreqBlock), 0, s, t->slots, t->cap, 2, 0ull,
                       per_block);
    std::vector<unsigned long long> pb(kScanBlocks), off(kScanBlocks);
    FQ_HIP(ctx, hipMemcpyAsync(pb.data(), per_block, kScanBlocks * 8, hipMemcpyDeviceToHost, s));
    FQ_HIP(ctx, hipStreamSynchronize(s));
    unsigned long long total = 0;
    for (int b = 0; b < kScanBlocks; ++b) {
        off[b] = total;
        total += pb[b];
    }
    const uint64_t n = std::min<uint64_t>(total, (uint64_t)capacity);
    if (n) {
        FQ_HIP(ctx, hipMemcpyAsync(offsets, off.data(), kScanBlocks * 8, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(compact_kernel, dim3(kScanBlocks), dim3(kFreqBlock), 0, s, t->slots, (const unsigned long long*)nullptr,
                           t->cap, 2, 0ull, offsets, (unsigned long long)n, (unsigned long long*)keys_dev,
                           (unsigned long long*)counts_dev, 1);
        FQ_HIP(ctx, hipGetLastError());
    }
    int64_t written = (int64_t)n;
    if (t->host_ctr.sentinel && written < capacity) {
        const int64_t kv[2] = {(int64_t)unmix64(kEmpty), (int64_t)t->host_ctr.sentinel};
        FQ_HIP(ctx, hipMemcpyAsync(keys_dev + written, &kv[0], 8, hipMemcpyHostToDevice, s));
        FQ_HIP(ctx, hipMemcpyAsync(counts_dev + written, &kv[1], 8, hipMemcpyHostToDevice, s));
        ++written;
    }
    FQ_HIP(ctx, hipStreamSynchronize(s));  // kv lives on this stack frame
    return written;
}

int dq_freq_from_pairs(dq_ctx* ctx, int32_t key_spark_type, const int64_t* keys, const int64_t* counts, int64_t n,
                       uint32_t flags, int64_t num_rows, int64_t null_count, dq_freq_table** out) {
    if (!ctx || !out || n < 0 || (n > 0 && (!keys || !counts)) || num_rows < 0 || null_count < 0 ||
        elem_of(key_spark_type) == ET_NONE)
        return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_freq_from_pairs: invalid arguments");
    dq_column col;
    memset(&col, 0, sizeof(col));
    col.spark_type = DQ_TYPE_LONG;  // canonical 64-bit keys (their LONG canonical form is the identity)
    col.length = n;
    col.values = keys;
    col.flags = (flags & DQ_FREQ_PAIRS_DEVICE) ? DQ_COL_DEVICE : 0u;
    dq_freq_options o;
    memset(&o, 0, sizeof(o));
    o.weights = counts;
    o.weights_device = (flags & DQ_FREQ_PAIRS_DEVICE) ? 1u : 0u;
    o.key_type = key_spark_type;
    const int32_t key0 = 0;
    const int rc = dq_frequencies_ex(ctx, &col, 1, n, &key0, 1, &o, out);
    if (rc) return rc;
    (*out)->num_rows_override = num_rows;
    (*out)->host_ctr.nulls = (unsigned long long)null_count;
    (*out)->cached_n = -1;
    return DQ_OK;
}

int dq_freq_merge(dq_ctx* ctx, const dq_freq_table* a, const dq_freq_table* b, dq_freq_table** out) {
    if (!ctx || !a || !b || !out) return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_freq_merge: invalid arguments");
    if (!a->fast || !b->fast || !a->parts.empty() || !b->parts.empty())
        return dq::ctx_fail(ctx, DQ_ERR_UNSUPPORTED,
                            "dq_freq_merge: both tables must be single-device tables of one fixed-width key column");
    if (elem_of(a->key_type) != elem_of(b->key_type) || (a->key_type == DQ_TYPE_DOUBLE) != (b->key_type == DQ_TYPE_DOUBLE))
        return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_freq_merge: key types differ");
    FQ_HIP(ctx, hipSetDevice(a->device));
    dq_freq_summary sa, sb;
    int rc = dq_freq_summarize(ctx, a, 0, &sa);
    if (rc) return rc;
    rc = dq_freq_summarize(ctx, b, 0, &sb);
    if (rc) return rc;
    const int64_t ca = sa.num_groups - (sa.null_count ? 1 : 0), cb = sb.num_groups - (sb.null_count ? 1 : 0);
    DevBuf buf(ctx);
    int64_t *k = nullptr, *c = nullptr;
    FQ_HIP(ctx, buf.alloc((void**)&k, (size_t)std::max<int64_t>(ca + cb, 1) * 8));
    FQ_HIP(ctx, buf.alloc((void**)&c, (size_t)std::max<int64_t>(ca + cb, 1) * 8));
    const int64_t na = dq_freq_export_device(ctx, a, ca, k, c);
    if (na < 0) return (int)na;
    const int64_t nb = dq_freq_export_device(ctx, b, cb, k + na, c + na);
    if (nb < 0) return (int)nb;
    rc = dq_freq_from_pairs(ctx, a->key_type, k, c, na + nb, DQ_FREQ_PAIRS_DEVICE, sa.num_rows + sb.num_rows,
                            sa.null_count + sb.null_count, out);
    if (rc == DQ_OK) {
        // the pair arrays are this call's scratch: the merged table only keeps its slots
        FQ_HIP(ctx, hipStreamSynchronize(dq::ctx_stream(ctx)));
        (*out)->ks.weights = nullptr;
        (*out)->ks.cols[0].values = nullptr;
    }
    return rc;
}

namespace {
int mi_tables(dq_ctx* ctx, const dq_freq_table* joint, const dq_freq_table* x, const dq_freq_table* y, double* mi,
              int32_t* present);

// A multi-device (x, y) table: its parts hold disjoint groups. The joint groups are gathered into one weighted
// table on the context's first device and the marginals are grouped from them -- the reference's own marginal
// tables (jointStats.groupBy(col).agg(sum(count)), A/MutualInformation.scala:50-58).
int mi_composite(dq_ctx* ctx, const dq_freq_table* joint, double* mi, int32_t* present) {
    if (joint->part_keys.size() != joint->parts.size() || joint->part_keys.empty() || joint->part_keys[0].cols.size() != 2)
        return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_freq_mutual_information: needs a two-column joint table");
    // concatenate the parts' groups
    GatheredKeys all;
    all.values.assign(2, {});
    all.validity.assign(2, {});
    all.offsets.assign(2, {});
    all.cols.assign(2, dq_column());
    size_t g = 0;
    for (const GatheredKeys& p : joint->part_keys) g += p.counts.size();
    for (const GatheredKeys& p : joint->part_keys) all.counts.insert(all.counts.end(), p.counts.begin(), p.counts.end());
    for (int c = 0; c < 2; ++c) {
        const dq_column& c0 = joint->part_keys[0].cols[c];
        dq_column& o = all.cols[c];
        o = c0;
        o.length = (int64_t)g;
        all.validity[c].assign((g + 7) / 8 + 8, 0);
        bool any_null = false;
        size_t at = 0;
        if (c0.spark_type == DQ_TYPE_STRING) all.offsets[c].assign(g + 1, 0);
        const int w = std::max(1, elem_size(elem_of(c0.spark_type)));
        for (const GatheredKeys& p : joint->part_keys) {
            const dq_column& pc = p.cols[c];
            const size_t pn = p.counts.size();
            for (size_t k = 0; k < pn; ++k) {
                const bool valid = !pc.validity || ((pc.validity[k >> 3] >> (k & 7)) & 1);
                if (valid) all.validity[c][(at + k) >> 3] |= (uint8_t)(1u << ((at + k) & 7)); else any_null = true;
            }
            if (c0.spark_type == DQ_TYPE_STRING) {
                const size_t base = all.values[c].size();
                const size_t bytes = pn ? (size_t)pc.offsets[pn] : 0;
                all.values[c].insert(all.values[c].end(), static_cast<const uint8_t*>(pc.values),
                                     static_cast<const uint8_t*>(pc.values) + bytes);
                for (size_t k = 0; k < pn; ++k) all.offsets[c][at + k + 1] = (int32_t)(base + pc.offsets[k + 1]);
            } else {
                all.values[c].insert(all.values[c].end(), static_cast<const uint8_t*>(pc.values),
                                     static_cast<const uint8_t*>(pc.values) + pn * w);
            }
            at += pn;
        }
        all.values[c].resize(all.values[c].size() + 16, 0);
        o.values = all.values[c].data();
        o.validity = any_null ? all.validity[c].data() : nullptr;
        o.offsets = c0.spark_type == DQ_TYPE_STRING ? all.offsets[c].data() : nullptr;
        o.flags = 0;
    }
    dq_freq_options opt;
    memset(&opt, 0, sizeof(opt));
    opt.weights = all.counts.empty() ? nullptr : all.counts.data();
    const int32_t kj[2] = {0, 1}, kx[1] = {0}, ky[1] = {1};
    dq_freq_table *J = nullptr, *X = nullptr, *Y = nullptr;
    dq_ctx* c0 = ctx->subs.empty() ? ctx : ctx->subs[0];  // one device: the first of the context
    int rc = dq_frequencies_ex(c0, all.cols.data(), 2, (int64_t)g, kj, 2, &opt, &J);
    if (!rc) rc = dq_frequencies_ex(c0, all.cols.data(), 2, (int64_t)g, kx, 1, &opt, &X);
    if (!rc) rc = dq_frequencies_ex(c0, all.cols.data(), 2, (int64_t)g, ky, 1, &opt, &Y);
    if (!rc) rc = mi_tables(c0, J, X, Y, mi, present);
    if (rc && c0 != ctx) ctx->err = c0->err;
    if (J) dq_freq_free(c0, J);
    if (X) dq_freq_free(c0, X);
    if (Y) dq_freq_free(c0, Y);
    return rc;
}
}  // namespace

int dq_freq_mutual_information(dq_ctx* ctx, const dq_freq_table* joint, const dq_freq_table* x,
                               const dq_freq_table* y, double* mi, int32_t* present) {
    if (!ctx || !joint || !x || !y || !mi || !present)
        return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_freq_mutual_information: invalid arguments");
    if (!joint->parts.empty()) return mi_composite(ctx, joint, mi, present);
    // weighted builds (pre-aggregated groups: a merged or persisted state) are fine when all three share the rows and
    // their weights, as a state's marginals are grouped from its joint groups (A/MutualInformation.scala:50-58)
    const bool wj = joint->ks.weights != nullptr;
    if (joint->fast || joint->ks.ncols != 2 || !joint->reps || x->ks.ncols != 1 || y->ks.ncols != 1 ||
        (x->ks.weights != nullptr) != wj || (y->ks.weights != nullptr) != wj)
        return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT,
                            "dq_freq_mutual_information: needs the (x, y) table and the x / y tables of the same rows");
    return mi_tables(ctx, joint, x, y, mi, present);
}

namespace {
int mi_tables(dq_ctx* ctx, const dq_freq_table* joint, const dq_freq_table* x, const dq_freq_table* y, double* mi,
              int32_t* present) {
    FQ_HIP(ctx, hipSetDevice(joint->device));
    hipStream_t s = dq::ctx_stream(ctx);
    LookupTable X, Y;
    X.slots = x->slots;
    X.ks = x->ks;
    X.sentinel = x->host_ctr.sentinel;
    X.bits = x->bits;
    Y.slots = y->slots;
    Y.ks = y->ks;
    Y.sentinel = y->host_ctr.sentinel;
    Y.bits = y->bits;
    const int64_t n = joint->num_rows_override >= 0 ? joint->num_rows_override : (int64_t)joint->host_ctr.num_rows;
    SummaryPartial* parts = (SummaryPartial*)joint->scratch;
    const int grid = summary_grid();
    hipLaunchKernelGGL(mi_kernel, dim3(grid), dim3(kFreqBlock), 0, s, joint->slots, joint->reps, joint->cap,
                       joint->ks, X, Y, (double)n, parts);
    FQ_HIP(ctx, hipGetLastError());
    std::vector<SummaryPartial> hp(grid);
    FQ_HIP(ctx, hipMemcpyAsync(hp.data(), parts, sizeof(SummaryPartial) * grid, hipMemcpyDeviceToHost, s));
    FQ_HIP(ctx, hipStreamSynchronize(s));
    SummaryPartial acc = {0, 0, 0, 0, 0, 0};
    for (const SummaryPartial& p : hp) summary_merge(acc, p);
    *mi = acc.nonfinite ? NAN : fx_to_double(acc.ent);
    *present = acc.groups > 0 ? 1 : 0;  // sum over zero joined rows is NULL (A/MutualInformation.scala:82-86)
    return DQ_OK;
}
}  // namespace

int dq_freq_row_counts(dq_ctx* ctx, const dq_freq_table* t, int64_t* counts, int64_t nrows, uint32_t flags) {
    if (!ctx || !t || (!counts && nrows > 0))
        return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_freq_row_counts: invalid arguments");
    if (!t->parts.empty() || t->src_rows < 0 || !t->slots)
        return dq::ctx_fail(ctx, DQ_ERR_UNSUPPORTED, "dq_freq_row_counts: needs a single-device table built over rows");
    if (nrows != t->src_rows)
        return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_freq_row_counts: nrows differs from the table's source rows");
    if (nrows == 0) return DQ_OK;
    FQ_HIP(ctx, hipSetDevice(t->device));
    hipStream_t s = dq::ctx_stream(ctx);
    LookupTable T;
    T.slots = t->slots;
    T.ks = t->ks;
    T.sentinel = t->host_ctr.sentinel;
    T.bits = t->bits;
    DevBuf buf(ctx);
    long long* d = reinterpret_cast<long long*>(counts);
    const bool dev_out = (flags & DQ_FREQ_PAIRS_DEVICE) != 0;
    if (!dev_out) FQ_HIP(ctx, buf.alloc((void**)&d, (size_t)nrows * 8));
    hipLaunchKernelGGL(row_counts_kernel, dim3(scan_grid((uint64_t)nrows)), dim3(kFreqBlock), 0, s, T, nrows, d);
    FQ_HIP(ctx, hipGetLastError());
    if (!dev_out) FQ_HIP(ctx, hipMemcpyAsync(counts, d, (size_t)nrows * 8, hipMemcpyDeviceToHost, s));
    FQ_HIP(ctx, hipStreamSynchronize(s));
    return DQ_OK;
}

void dq_freq_free(dq_ctx* ctx, dq_freq_table* t) {
    (void)ctx;
    if (!t) return;
    if (!t->parts.empty()) {
        for (size_t i = 0; i < t->parts.size(); ++i) dq_freq_free(t->part_ctx[i], t->parts[i]);
        delete t;
        return;
    }
    (void)hipSetDevice(t->device);
    // every call on a table returns after its stream's work (or hands device pairs to the caller's stream order);
    // the slots go back to the context's cache in its stream order
    (void)hipStreamSynchronize(dq::ctx_stream(ctx));
    free_table_buffers(t, ctx);
    delete t;
}

}  // extern "C"

// ---- multi-GPU key partitioning --------------------------------------------------------------------
namespace {

constexpr int kMaxParts = 64;

__device__ __forceinline__ int owner_of(uint64_t canon, int nparts) {
    return (int)((mix64(canon) >> 32) % (uint64_t)nparts);
}

__global__ void __launch_bounds__(kFreqBlock)
part_count_kernel(KeyCol c, int64_t nrows, int nparts, unsigned long long* __restrict__ counts) {
    __shared__ unsigned int lds[kMaxParts + 1];
    for (int i = threadIdx.x; i <= kMaxParts; i += kFreqBlock) lds[i] = 0;
    __syncthreads();
    const int64_t stride = (int64_t)gridDim.x * kFreqBlock;
    for (int64_t r = (int64_t)blockIdx.x * kFreqBlock + threadIdx.x; r < nrows; r += stride) {
        if (!is_valid(c, r)) {
            atomicAdd(&lds[kMaxParts], 1u);
            continue;
        }
        atomicAdd(&lds[owner_of(canonical(c, r), nparts)], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i <= kMaxParts; i += kFreqBlock)
        if (lds[i]) atomicAdd(&counts[i], (unsigned long long)lds[i]);
}

// Each workgroup reserves its slice of every bucket with one atomic per bucket, then scatters.
__global__ void __launch_bounds__(kFreqBlock)
part_scatter_kernel(KeyCol c, int64_t nrows, int nparts, unsigned long long* __restrict__ cursors,
                    unsigned long long* __restrict__ out) {
    __shared__ unsigned int cnt[kMaxParts];
    __shared__ unsigned long long base[kMaxParts];
    const int64_t per_block = (nrows + gridDim.x - 1) / gridDim.x;
    const int64_t r0 = (int64_t)blockIdx.x * per_block;
    const int64_t r1 = r0 + per_block < nrows ? r0 + per_block : nrows;
    for (int i = threadIdx.x; i < kMaxParts; i += kFreqBlock) cnt[i] = 0;
    __syncthreads();
    for (int64_t r = r0 + threadIdx.x; r < r1; r += kFreqBlock)
        if (is_valid(c, r)) atomicAdd(&cnt[owner_of(canonical(c, r), nparts)], 1u);
    __syncthreads();
    for (int i = threadIdx.x; i < nparts; i += kFreqBlock) {
        base[i] = cnt[i] ? atomicAdd(&cursors[i], (unsigned long long)cnt[i]) : 0ull;
        cnt[i] = 0;
    }
    __syncthreads();
    for (int64_t r = r0 + threadIdx.x; r < r1; r += kFreqBlock) {
        if (!is_valid(c, r)) continue;
        const uint64_t k = canonical(c, r);
        const int p = owner_of(k, nparts);
        const unsigned int slot = atomicAdd(&cnt[p], 1u);
        out[base[p] + slot] = k;
    }
}

}  // namespace

extern "C" int dq_partition_keys(dq_ctx* ctx, const dq_column* column, int64_t nrows, int nparts, int64_t* keys_dev,
                                 int64_t* part_counts, int64_t* null_rows) {
    if (!ctx || !column || nparts < 1 || nparts > kMaxParts || nrows < 0 || !part_counts ||
        column->length != nrows || elem_of(column->spark_type) == ET_NONE || !(column->flags & DQ_COL_DEVICE) ||
        (nrows > 0 && !keys_dev))
        return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_partition_keys: invalid arguments (device fixed-width column)");
    FQ_HIP(ctx, hipSetDevice(dq::ctx_device(ctx)));
    hipStream_t s = dq::ctx_stream(ctx);
    KeyCol c;
    c.values = column->values;
    c.validity = column->validity;
    c.offsets = nullptr;
    c.offsets64 = nullptr;
    c.spark_type = column->spark_type;
    c.elem = elem_of(column->spark_type);
    unsigned long long* dev = nullptr;
    FQ_HIP(ctx, hipMalloc(&dev, sizeof(unsigned long long) * 2 * (kMaxParts + 1)));
    FQ_HIP(ctx, hipMemsetAsync(dev, 0, sizeof(unsigned long long) * 2 * (kMaxParts + 1), s));
    const int grid = scan_grid((uint64_t)std::max<int64_t>(nrows, 1));
    if (nrows > 0) hipLaunchKernelGGL(part_count_kernel, dim3(grid), dim3(kFreqBlock), 0, s, c, nrows, nparts, dev);
    unsigned long long h[kMaxParts + 1];
    FQ_HIP(ctx, hipMemcpyAsync(h, dev, sizeof(h), hipMemcpyDeviceToHost, s));
    FQ_HIP(ctx, hipStreamSynchronize(s));
    unsigned long long cur[kMaxParts + 1] = {0};
    unsigned long long off = 0;
    for (int p = 0; p < nparts; ++p) {
        cur[p] = off;
        part_counts[p] = (int64_t)h[p];
        off += h[p];
    }
    if (null_rows) *null_rows = (int64_t)h[kMaxParts];
    unsigned long long* cursors = dev + kMaxParts + 1;
    FQ_HIP(ctx, hipMemcpyAsync(cursors, cur, sizeof(unsigned long long) * kMaxParts, hipMemcpyHostToDevice, s));
    if (nrows > 0)
        hipLaunchKernelGGL(part_scatter_kernel, dim3(grid), dim3(kFreqBlock), 0, s, c, nrows, nparts, cursors,
                           (unsigned long long*)keys_dev);
    FQ_HIP(ctx, hipGetLastError());
    FQ_HIP(ctx, hipStreamSynchronize(s));
    (void)hipFree(dev);
    return DQ_OK;
}
