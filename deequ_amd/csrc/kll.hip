// kll.hip — KLLSketch (deequ's deterministic KLL, QuantileNonSample) on gfx950 / CDNA4.
//
// Replaces the per-row `sketch.updateUntyped(row.get(index))` loop of KLLRunner.sketchPartitions
// (R/KLLRunner.scala:148-179) for one partition whose non-NULL values arrive in row order, and
// produces the KLLState bytes the reference reads (A/KLLSketch.scala:56-66: min, max, then the
// KLLSketchSerializer layout, A/catalyst/KLLSketchSerializer.scala:60-80), bit for bit.
//
// Why this parallelises: QuantileNonSample.update / condense (A/QuantileNonSample.scala:80-121)
// decide WHEN and WHICH level compacts from buffer LENGTHS only, never from values, and the
// compactor offset flips on a count-only rule (A/NonSampleCompactor.scala:40-47; the Random offset
// is commented out in the reference). So the whole compaction schedule is a function of n:
//   1. the host replays the count automaton event by event (one event per compaction, ~n/1000),
//      recording for every level h the compactions as (start, L, offset) over that level's
//      arrival stream: a compaction sorts the first L = items - items%2 buffered items (an odd
//      leftover is the newest arrival and stays), keeps every other one from `offset`, and appends
//      them to level h+1's stream. Consecutive compactions of a level therefore sort consecutive,
//      non-overlapping ranges of its stream;
//   2. the GPU runs one launch per level: one workgroup per compaction sorts its range in LDS
//      (bitonic network over java.lang.Double.compare order keys — Scala's `.sorted` with
//      Ordering.Double) and writes the alternate picks into the next level's stream at the
//      position the schedule assigned. All compactions of a level are independent;
//   3. what no compaction consumed is each level's final buffer, copied back in arrival order.
// min/max (UntypedQuantileNonSample.updateUntyped, math.min/max from Int.MaxValue/Int.MinValue) come
// from each level-0 range's sorted ends (+ the final level-0 buffer on the host).
//
// Work: level 0 reads 8 B and writes 4 B per value; each level above handles about half of the
// previous one's items — ~2n sorted items and ~24 B of HBM traffic per value in total.
#include <hip/hip_runtime.h>

#include <math.h>
#include <string.h>

#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <chrono>
#include <thread>
#include <vector>

#include "dq_common.h"
#include "dq_internal.h"

namespace dq {

constexpr int kKllMaxPad = 16384;  // 128 KiB of LDS keys: the largest compaction handled
constexpr int kKllStageBlock = 256;
constexpr int kKllStageRows = 2048;  // rows per workgroup tile of the NULL-compaction pass

__device__ __forceinline__ uint64_t kll_key(double d) {
    uint64_t u = d != d ? 0x7ff8000000000000ULL : (uint64_t)__double_as_longlong(d);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ULL);
}
__device__ __forceinline__ double kll_value(uint64_t k) {
    return __longlong_as_double((long long)((k >> 63) ? (k & 0x7fffffffffffffffULL) : ~k));
}

struct KllColumn {
    const void* values;
    const uint64_t* validity;
    int32_t elem;
};

__device__ __forceinline__ double kll_load(const KllColumn& c, int64_t r) {
    switch (c.elem) {
        case ET_F64: return static_cast<const double*>(c.values)[r];
        case ET_F32: return (double)static_cast<const float*>(c.values)[r];
        case ET_I64: return (double)static_cast<const int64_t*>(c.values)[r];
        case ET_I32: return (double)static_cast<const int32_t*>(c.values)[r];
        case ET_I16: return (double)static_cast<const int16_t*>(c.values)[r];
        default: return (double)static_cast<const int8_t*>(c.values)[r];
    }
}

__device__ __forceinline__ bool kll_valid(const KllColumn& c, int64_t r) {
    return c.validity == nullptr || ((c.validity[r >> 6] >> (r & 63)) & 1ull);
}

// One column's NULL compaction: its tile counts, tile offsets and total (blockIdx.y of the count / scan launches).
struct KllCountJob {
    KllColumn c;
    unsigned int* counts;
    unsigned long long* offs;
    unsigned long long* total;
    double* dense;  // the dense level-0 stream (write pass), null when the column has no non-NULL value
};

// NULL compaction, pass 1: non-NULL rows per 2048-row tile, from the validity words (32 per tile): one lane per word
// (a population count of the word's bits below nrows), a wave covers two tiles, a workgroup eight. (The per-row form —
// every lane testing its rows' bits through 64-bit word loads — took 1.36 ms per 1.25e8-row chunk of 13 columns.)
constexpr int kKllCountTilesPerBlock = kKllStageBlock / 32;
__global__ void __launch_bounds__(kKllStageBlock)
kll_count_kernel(const KllCountJob* __restrict__ jobs, int64_t nrows, int64_t ntiles) {
    const KllColumn c = jobs[blockIdx.y].c;
    unsigned int* __restrict__ tile_counts = jobs[blockIdx.y].counts;
    const int64_t t = (int64_t)blockIdx.x * kKllCountTilesPerBlock + (threadIdx.x >> 5);  // this lane's tile
    const int64_t w = t * (kKllStageRows / 64) + (threadIdx.x & 31);                       // its validity word
    const int64_t r0 = w * 64;
    unsigned int cnt = 0;
    if (t < ntiles && r0 < nrows) {
        const uint64_t bits = c.validity ? c.validity[w] : ~0ull;
        const uint64_t in = nrows - r0 >= 64 ? ~0ull : ((1ull << (nrows - r0)) - 1ull);
        cnt = (unsigned int)__popcll(bits & in);
    }
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) cnt += __shfl_down(cnt, o, 32);
    if ((threadIdx.x & 31) == 0 && t < ntiles) tile_counts[t] = cnt;
}

// NULL compaction, pass 2: non-NULL values as doubles, in row order, from each tile's offset.
__global__ void __launch_bounds__(kKllStageBlock)
kll_write_kernel(KllColumn c, int64_t nrows, const unsigned long long* __restrict__ tile_offsets,
                 double* __restrict__ out) {
    __shared__ unsigned int wsum[kKllStageBlock / 64];
    const int64_t r0 = (int64_t)blockIdx.x * kKllStageRows;
    unsigned long long base = tile_offsets[blockIdx.x];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int64_t rb = r0; rb < r0 + kKllStageRows && rb < nrows; rb += kKllStageBlock) {
        const int64_t r = rb + threadIdx.x;
        const bool v = r < nrows && kll_valid(c, r);
        const unsigned long long ball = __ballot(v);
        const unsigned int before = (unsigned int)__popcll(ball & ((1ull << lane) - 1ull));
        if (lane == 0) wsum[wave] = (unsigned int)__popcll(ball);
        __syncthreads();
        unsigned int wbase = 0, total = 0;
        for (int w = 0; w < kKllStageBlock / 64; ++w) {
            if (w < wave) wbase += wsum[w];
            total += wsum[w];
        }
        if (v) out[base + wbase + before] = kll_load(c, r);
        base += total;
        __syncthreads();
    }
}

// The same for every column of a batched sketch (blockIdx.y = job). Each thread loads its 8 rows of the tile at once
// (rows t + 256 q: every load instruction coalesced), the ballots of all 8 row groups go to LDS together, and one
// barrier later every value knows its dense position: one round trip per tile instead of one per 256 rows.
__global__ void __launch_bounds__(kKllStageBlock)
kll_write_jobs_kernel(const KllCountJob* __restrict__ jobs, int64_t nrows) {
    const KllCountJob& j = jobs[blockIdx.y];
    if (!j.dense) return;
    constexpr int Q = kKllStageRows / kKllStageBlock, NW = kKllStageBlock / 64;
    __shared__ unsigned int wc[Q * NW];
    const KllColumn c = j.c;
    const int64_t r0 = (int64_t)blockIdx.x * kKllStageRows;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    double x[Q];
    unsigned long long bal[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int64_t r = r0 + (int64_t)q * kKllStageBlock + t;
        const bool v = r < nrows && kll_valid(c, r);
        x[q] = v ? kll_load(c, r) : 0.0;
        bal[q] = __ballot(v);
    }
    if (lane == 0) {
#pragma unroll
        for (int q = 0; q < Q; ++q) wc[q * NW + wave] = (unsigned int)__popcll(bal[q]);
    }
    __syncthreads();
    unsigned long long at = j.offs[blockIdx.x];
    double* __restrict__ out = j.dense;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        unsigned int wq = 0, tq = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            const unsigned int n = wc[q * NW + w];
            wq += w < wave ? n : 0u;
            tq += n;
        }
        if ((bal[q] >> lane) & 1ull) out[at + wq + (unsigned int)__popcll(bal[q] & ((1ull << lane) - 1ull))] = x[q];
        at += tq;
    }
}

// NULL compaction, between the passes: exclusive prefix of the tile counts (one workgroup) and the total, so only
// the total travels to the host (the compaction schedule is a function of it).
__global__ void __launch_bounds__(1024)
kll_scan_kernel(const KllCountJob* __restrict__ jobs, int64_t ntiles) {
    const unsigned int* __restrict__ counts = jobs[blockIdx.y].counts;
    unsigned long long* __restrict__ offs = jobs[blockIdx.y].offs;
    unsigned long long* __restrict__ total = jobs[blockIdx.y].total;
    __shared__ unsigned long long part[1024];
    const int t = threadIdx.x;
    const int64_t per = (ntiles + 1023) / 1024;
    const int64_t b0 = t * per, b1 = b0 + per < ntiles ? b0 + per : ntiles;
    unsigned long long acc = 0;
    for (int64_t i = b0; i < b1; ++i) acc += counts[i];
    part[t] = acc;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan of the 1024 thread sums
        const unsigned long long v = t >= o ? part[t - o] : 0ull;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    unsigned long long run = part[t] - acc;
    for (int64_t i = b0; i < b1; ++i) {
        offs[i] = run;
        run += counts[i];
    }
    if (t == 1023) *total = part[1023];
}

// Final buffers: each level's unconsumed tail gathered into one contiguous array (one read-back per sketch).
struct KllTail {
    unsigned long long src;   // device address of the level's first unconsumed item
    unsigned long long len;
    unsigned long long dst;   // index in the gathered array
};
__global__ void __launch_bounds__(256)
kll_gather_kernel(const KllTail* __restrict__ tails, double* __restrict__ out) {
    const KllTail tl = tails[blockIdx.x];
    const double* src = reinterpret_cast<const double*>(tl.src);
    for (unsigned long long i = threadIdx.x; i < tl.len; i += 256) out[tl.dst + i] = src[i];
}

// One compaction, packed in 8 bytes: start of the compacted range in its level's stream (bits 0-39),
// L (bits 40-54, <= 16384) and the compactor offset (bit 63). Compactions consume a level's stream
// contiguously from 0 and every L is even, so the picks go to next-level slot start / 2.
__host__ __device__ inline uint64_t kll_desc(uint64_t start, uint32_t len, uint32_t offset) {
    return start | ((uint64_t)len << 40) | ((uint64_t)offset << 63);
}

// One workgroup of T threads per compaction of one level; the range (<= T*E items, padded with +inf
// keys) is sorted as a merge sort: every thread sorts E consecutive keys in registers (bitonic network,
// compile-time indices), then log2(T) rounds merge pairs of sorted runs through LDS, each thread
// producing E outputs of its merged pair from a merge-path split (binary search on the diagonal) — far
// fewer LDS accesses and barriers than a bitonic network over LDS. The LDS image is padded by one key per
// thread (physical index i + i/E) so thread-contiguous accesses are bank-conflict free. The picks
// sorted[offset + 2j] go straight from registers to the next level's stream; level 0 also folds the
// range's sorted ends into the running min / max keys.
template <int E>
__device__ __forceinline__ void kll_reg_sort(uint64_t (&v)[E]) {
    constexpr int P = E <= 4 ? 4 : (E <= 8 ? 8 : 16);
    uint64_t w[P];
#pragma unroll
    for (int r = 0; r < P; ++r) w[r] = r < E ? v[r] : ~0ull;
#pragma unroll
    for (int size = 2; size <= P; size <<= 1)
#pragma unroll
        for (int stride = size >> 1; stride > 0; stride >>= 1)
#pragma unroll
            for (int r = 0; r < P; ++r) {
                const int q = r ^ stride;
                if (q > r) {
                    const bool asc = (r & size) == 0;
                    const uint64_t a = w[r], b = w[q];
                    const bool sw = (a > b) == asc;
                    w[r] = sw ? b : a;
                    w[q] = sw ? a : b;
                }
            }
#pragma unroll
    for (int r = 0; r < E; ++r) v[r] = w[r];
}

// One merge round of the LDS merge sort: thread t's E keys (registers) are the sorted run it holds; runs of w keys are
// merged pairwise. The thread finds its output window of the merged pair on the merge path (binary search on the
// diagonal), loads the next E keys of both inputs at once (2E independent LDS reads, not a chain of E dependent ones)
// and keeps the E smallest of them with a register network: min against the reversed B window (a bitonic half-cleaner:
// the E smallest of two sorted windows) then a bitonic merge of those E. Equal keys are equal values, so which input a
// tied key comes from does not matter. Out-of-range keys read as ~0 (no key is ~0: kll_key(NaN) = 0xfff8...).
// A round whose merged pairs (2w keys = 2w / E threads) lie inside one wave synchronises that wave only: each wave reads
// just its own part of the LDS image until the first block-wide round (DQ_KLL_BLOCK_ROUNDS=1 builds the block-barrier
// form for A/B).
#ifndef DQ_KLL_BLOCK_ROUNDS
#define DQ_KLL_BLOCK_ROUNDS 0
#endif
__device__ __forceinline__ void kll_round_sync(bool wave_local) {
    if (wave_local && !DQ_KLL_BLOCK_ROUNDS) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
        __syncthreads();
    }
}

template <int E>
__device__ __forceinline__ void kll_merge_round(uint64_t* k, uint64_t (&v)[E], int t, int w) {
    auto at = [](int i) { return i + i / E; };
    const bool wave_local = 2 * w <= 64 * E;
#pragma unroll
    for (int r = 0; r < E; ++r) k[at(t * E + r)] = v[r];
    kll_round_sync(wave_local);
    const int diag = E * (t & (2 * (w / E) - 1));  // offset inside the merged pair (w / E is a power of 2)
    const int A = (t * E) - diag, B = A + w;
    int lo = diag > w ? diag - w : 0, hi = diag < w ? diag : w;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (k[at(A + mid)] <= k[at(B + diag - 1 - mid)]) lo = mid + 1;
        else hi = mid;
    }
    int ai = A + lo, bi = B + diag - lo;
    const int aend = A + w, bend = B + w;
    if constexpr ((E & (E - 1)) != 0) {  // E = 12: the sequential merge (the network below needs a power of two)
        uint64_t ah = ai < aend ? k[at(ai)] : ~0ull, bh = bi < bend ? k[at(bi)] : ~0ull;
#pragma unroll
        for (int r = 0; r < E; ++r) {
            const bool takeA = bi >= bend || (ai < aend && ah <= bh);
            if (takeA) {
                v[r] = ah;
                ++ai;
                ah = ai < aend ? k[at(ai)] : ~0ull;
            } else {
                v[r] = bh;
                ++bi;
                bh = bi < bend ? k[at(bi)] : ~0ull;
            }
        }
        kll_round_sync(wave_local);
        return;
    }
    uint64_t a[E], b[E];
#pragma unroll
    for (int r = 0; r < E; ++r) {
        a[r] = ai + r < aend ? k[at(ai + r)] : ~0ull;
        b[r] = bi + r < bend ? k[at(bi + r)] : ~0ull;
    }
#pragma unroll
    for (int r = 0; r < E; ++r) {
        const uint64_t x = a[r], y = b[E - 1 - r];
        v[r] = x < y ? x : y;
    }
    // v is bitonic (non-increasing after non-decreasing): sort it ascending
#pragma unroll
    for (int stride = E / 2; stride > 0; stride >>= 1)
#pragma unroll
        for (int r = 0; r < E; ++r)
            if ((r & stride) == 0) {
                const uint64_t x = v[r], y = v[r + stride];
                const bool sw = x > y;
                v[r] = sw ? y : x;
                v[r + stride] = sw ? x : y;
            }
    kll_round_sync(wave_local);
}

// ---- the first merge rounds across lanes (E = 8) ---------------------------------------------------------------------
#ifndef DQ_KLL_DPP
#define DQ_KLL_DPP 2  // 0: every round through LDS; 1: w = 8-32 across lanes; 2: also w = 64
#endif
// Merging runs of w = 8 * 2^M keys held by 2^M consecutive lanes needs no LDS: a bitonic merge whose first stage pairs
// lane t's key r with lane t ^ (2^(M+1) - 1)'s key 7 - r (the mirror: the partner run read backwards), then halves
// between lanes t ^ 2^s (same r), then the lane's 8 keys in registers. Partners are DPP lane swizzles (quad_perm /
// row_half_mirror): M = 0, 1, 2 cover w = 8, 16, 32, three of the eight rounds of a 2048-key sort, without their LDS
// writes, reads, merge-path searches and wave barriers. The result is the same sorted sequence.
template <int CTRL>
__device__ __forceinline__ uint64_t kll_dpp64(uint64_t x) {
    const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)x, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(x >> 32), CTRL, 0xF, 0xF, false);
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

// Every key of v against the same-index key of the partner lane (REV: the partner's keys reversed); the lower lane
// of the pair keeps the minima.
template <int CTRL, bool REV>
__device__ __forceinline__ void kll_dpp_stage(uint64_t (&v)[8], bool lower) {
    uint64_t b[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) b[r] = kll_dpp64<CTRL>(v[r]);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const uint64_t x = v[r], y = b[REV ? 7 - r : r];
        v[r] = (x < y) == lower ? x : y;
    }
}

__device__ __forceinline__ void kll_bitonic8(uint64_t (&v)[8]) {  // a bitonic 8 in registers, ascending
#pragma unroll
    for (int stride = 4; stride > 0; stride >>= 1)
#pragma unroll
        for (int r = 0; r < 8; ++r)
            if ((r & stride) == 0) {
                const uint64_t x = v[r], y = v[r + stride];
                const bool sw = x > y;
                v[r] = sw ? y : x;
                v[r + stride] = sw ? x : y;
            }
}

// Rounds w = 8, 16, 32 of the merge sort of kll_compact_*: thread t's 8 sorted keys in, the sorted 64-key run of its
// 8-lane group out.
__device__ __forceinline__ void kll_dpp_rounds(uint64_t (&v)[8], int t) {
    constexpr int kXor1 = 0xB1, kXor2 = 0x4E, kRev4 = 0x1B, kRev8 = 0x141;  // quad_perm [1,0,3,2] / [2,3,0,1] / [3,2,1,0], row_half_mirror
    kll_dpp_stage<kXor1, true>(v, (t & 1) == 0);  // w = 8: lanes t, t ^ 1
    kll_bitonic8(v);
    kll_dpp_stage<kRev4, true>(v, (t & 2) == 0);  // w = 16: lanes t, t ^ 3 mirrored, then t ^ 1
    kll_dpp_stage<kXor1, false>(v, (t & 1) == 0);
    kll_bitonic8(v);
    kll_dpp_stage<kRev8, true>(v, (t & 4) == 0);  // w = 32: lanes t, 7 - t mirrored, then t ^ 2, t ^ 1
    kll_dpp_stage<kXor2, false>(v, (t & 2) == 0);
    kll_dpp_stage<kXor1, false>(v, (t & 1) == 0);
    kll_bitonic8(v);
#if DQ_KLL_DPP >= 2
    constexpr int kRev16 = 0x140, kShl4 = 0x104, kShr4 = 0x114;  // row_mirror, row_shl:4, row_shr:4
    kll_dpp_stage<kRev16, true>(v, (t & 8) == 0);  // w = 64: lanes t, 15 - t mirrored, then t ^ 4 (two row shifts),
    {                                              // t ^ 2, t ^ 1
        const bool lo4 = (t & 4) == 0;
        uint64_t b[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const uint64_t up = kll_dpp64<kShl4>(v[r]), dn = kll_dpp64<kShr4>(v[r]);
            b[r] = lo4 ? up : dn;
        }
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const uint64_t x = v[r], y = b[r];
            v[r] = (x < y) == lo4 ? x : y;
        }
    }
    kll_dpp_stage<kXor2, false>(v, (t & 2) == 0);
    kll_dpp_stage<kXor1, false>(v, (t & 1) == 0);
    kll_bitonic8(v);
#endif
}


// ---- levels above 0: merge the natural runs --------------------------------------------------------------------------
// Level h >= 1's stream is the concatenation of level h-1's pick runs, each sorted (a compaction emits the alternate
// items of its sorted range in order). A compaction range of such a level therefore holds a few maximal non-decreasing
// runs (the level's odd leftover, the tail of one pick run, the head of the next) rather than L unsorted items. The
// workgroup finds the descents (one ballot per wave, one barrier); with at most kKllMaxRuns runs it merges them in
// <= 2 merge-path rounds (a sequential E-step merge per thread, since run lengths are arbitrary) instead of the register
// sort + log2(T) rounds; a range with more descents takes the full sort. The sorted result is the same sequence either
// way (sorting keys is unique), so the picks do not depend on which path ran.
constexpr int kKllMaxRuns = 4;

template <int NW>
struct KllRunScratch {
    int cnt[NW];                       // per wave: descents in its keys (or 1 << 20: too many)
    int pos[NW][kKllMaxRuns - 1];      // their positions, in order
};

// One round over up to two (A, B) pairs tiling [0, n): pair j merges [ps[j], pm[j]) with [pm[j], ps[j + 1]). Thread t
// produces sorted positions [tE, tE + E) of the round's output into v.
template <int E>
__device__ __forceinline__ void kll_merge_pairs(const uint64_t* k, uint64_t (&v)[E], int o, int np, const int (&ps)[3],
                                                const int (&pm)[2]) {
    auto at = [](int i) { return i + i / E; };
    int j = (np > 1 && o >= ps[1]) ? 1 : 0;
    int ai, bi, aend, bend;
    {
        const int a0 = ps[j], b0 = pm[j];
        aend = pm[j];
        bend = ps[j + 1];
        const int diag = o - a0, la = aend - a0, lb = bend - b0;
        int lo = diag > lb ? diag - lb : 0, hi = diag < la ? diag : la;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (k[at(a0 + mid)] <= k[at(b0 + diag - 1 - mid)]) lo = mid + 1;
            else hi = mid;
        }
        ai = a0 + lo;
        bi = b0 + diag - lo;
    }
    uint64_t ah = ai < aend ? k[at(ai)] : ~0ull, bh = bi < bend ? k[at(bi)] : ~0ull;
#pragma unroll
    for (int r = 0; r < E; ++r) {
        if (o + r == bend && j + 1 < np) {  // this thread's window runs into the next pair: merge it from its start
            ++j;
            ai = ps[j];
            aend = pm[j];
            bi = pm[j];
            bend = ps[j + 1];
            ah = ai < aend ? k[at(ai)] : ~0ull;
            bh = bi < bend ? k[at(bi)] : ~0ull;
        }
        const bool takeA = bi >= bend || (ai < aend && ah <= bh);
        if (takeA) {
            v[r] = ah;
            ++ai;
            ah = ai < aend ? k[at(ai)] : ~0ull;
        } else {
            v[r] = bh;
            ++bi;
            bh = bi < bend ? k[at(bi)] : ~0ull;
        }
    }
}

// v = keys [tE, tE + E) of the range in stream order (n = T * E of them, padding ~0 at the end), vprev = key tE - 1.
// Returns false (uniformly) when the range has more than kKllMaxRuns natural runs; otherwise v is sorted as by the
// full merge sort. Ends with a barrier after its last LDS read of k.
template <int T, int E>
__device__ bool kll_natural_sort(uint64_t* k, uint64_t (&v)[E], int t, uint64_t vprev, KllRunScratch<T / 64>& rs) {
    constexpr int n = T * E;
    constexpr int NW = T / 64;
    auto at = [](int i) { return i + i / E; };
    const int lane = t & 63, wave = t >> 6;
    int nd = 0, p = 0;
#pragma unroll
    for (int r = 0; r < E; ++r) {
        const bool d = r == 0 ? (t > 0 && v[0] < vprev) : v[r] < v[r - 1];
        p = (d && nd == 0) ? t * E + r : p;
        nd += d ? 1 : 0;
    }
    const uint64_t m = __ballot(nd > 0);
    const bool many = __ballot(nd > 1) != 0 || __popcll(m) > kKllMaxRuns - 1;
    if (!many && nd == 1) rs.pos[wave][__popcll(m & ((1ull << lane) - 1))] = p;
    if (lane == 0) rs.cnt[wave] = many ? 1 << 20 : (int)__popcll(m);
    __syncthreads();
    int total = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) total += rs.cnt[w];
    if (total > kKllMaxRuns - 1) return false;
    if (total == 0) return true;  // already sorted
    static_assert(kKllMaxRuns == 4, "run starts below are three registers");
    int s[kKllMaxRuns + 1] = {0, n, n, n, n};  // static indices only (no scratch)
    int c = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w)
#pragma unroll
        for (int i = 0; i < kKllMaxRuns - 1; ++i)
            if (i < rs.cnt[w]) {
                const int q = rs.pos[w][i];
                s[1] = c == 0 ? q : s[1];
                s[2] = c == 1 ? q : s[2];
                s[3] = c == 2 ? q : s[3];
                ++c;
            }
    const int R = total + 1;
    // round 1: runs (0, 1) and (2, 3); round 2 (R >= 3): the two results
#pragma unroll
    for (int r = 0; r < E; ++r) k[at(t * E + r)] = v[r];
    __syncthreads();
    {
        const int ps[3] = {0, s[2], n};
        const int pm[2] = {s[1], R == 4 ? s[3] : n};
        kll_merge_pairs<E>(k, v, t * E, R >= 3 ? 2 : 1, ps, pm);
    }
    __syncthreads();
    if (R >= 3) {
#pragma unroll
        for (int r = 0; r < E; ++r) k[at(t * E + r)] = v[r];
        __syncthreads();
        const int ps[3] = {0, n, n};
        const int pm[2] = {s[2], n};
        kll_merge_pairs<E>(k, v, t * E, 1, ps, pm);
        __syncthreads();
    }
    return true;
}

// Batched launches (one launch per level and class over every column of a dq_kll_sketch_columns call): a descriptor's
// bits 55-62 name its column, whose stream / next-level / min-max pointers for this level come from `cols`.
struct KllColPtr {
    const double* src;          // the level's stream; null at level 0 of a column read in place (below)
    double* dst;
    unsigned long long* minmax;
    // level 0 read in place: the raw column and its NULL-compaction tile offsets (kll_count / kll_scan)
    KllColumn raw;
    const unsigned long long* offs;
    int64_t ntiles, nrows;
};

// ---- level 0 in place -----------------------------------------------------------------------------------------------
// A level-0 compaction consumes the dense stream of the column's non-NULL values [start, start + L). Instead of writing
// that stream out (8 B written and re-read per value), the compaction reads the raw column: kll_locate_kernel turns each
// level-0 descriptor's dense range into a row range once (tile offsets + a select inside the tile), and the workgroup
// stages the range's non-NULL values into its LDS image in dense order (ballot prefixes), then sorts as before.

// Row of the d-th non-NULL value (d < the column's non-NULL count): the last tile whose offset is <= d, then the
// (d - offset)-th set validity bit of that tile.
__device__ int64_t kll_row_of(const KllColPtr& cp, uint64_t d) {
    if (!cp.raw.validity) return (int64_t)d;
    int64_t lo = 0, hi = cp.ntiles - 1;
    while (lo < hi) {
        const int64_t mid = (lo + hi + 1) >> 1;
        if (cp.offs[mid] <= d) lo = mid;
        else hi = mid - 1;
    }
    uint64_t need = d - cp.offs[lo];
    const int64_t w0 = lo * (kKllStageRows / 64), wend = (cp.nrows + 63) >> 6;
    for (int64_t w = w0; w < w0 + kKllStageRows / 64 && w < wend; ++w) {
        uint64_t bits = cp.raw.validity[w];
        if (w == wend - 1 && (cp.nrows & 63)) bits &= (1ull << (cp.nrows & 63)) - 1ull;
        const uint64_t c = (uint64_t)__popcll(bits);
        if (need < c) {
            for (uint64_t k = 0; k < need; ++k) bits &= bits - 1ull;  // drop the lowest `need` set bits
            return (w << 6) + (__ffsll((long long)bits) - 1);
        }
        need -= c;
    }
    return cp.nrows;  // not reached for d below the non-NULL count
}

__global__ void __launch_bounds__(256)
kll_locate_kernel(const uint64_t* __restrict__ segs, int n, const KllColPtr* __restrict__ cols,
                  unsigned long long* __restrict__ rows) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint64_t sg = segs[i];
    const KllColPtr cp = cols[(sg >> 55) & 0xFF];
    if (cp.src) return;  // a column read as a stream (zero copy)
    const uint64_t start = sg & ((1ull << 40) - 1);
    const uint32_t len = (uint32_t)((sg >> 40) & 0x7FFF);
    rows[2 * i] = (unsigned long long)kll_row_of(cp, start);
    rows[2 * i + 1] = len ? (unsigned long long)kll_row_of(cp, start + len - 1) + 1ull : rows[2 * i];
}

// Stages the non-NULL values of rows [r0, r1) (exactly `len` of them) as order keys, in row order: place(pos, key).
// Each thread loads RM rows per chunk at once (rows r0 + q T + t: coalesced), the chunk's ballots give every value its
// dense position, one barrier pair per chunk of RM * T rows.
template <int T, bool RAWBITS = false, typename Place>
__device__ __forceinline__ void kll_stage_rows(const KllColumn& c, int64_t r0, int64_t r1, unsigned int* wc,
                                               Place place) {
    constexpr int RM = 8, NW = T / 64, NE = RM * NW;  // NE <= 128: (chunk row, wave) counts
    static_assert(NE <= 128, "two scan entries per lane of wave 0");
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    unsigned int base = 0;
    for (int64_t c0 = r0; c0 < r1; c0 += (int64_t)RM * T) {
        uint64_t key[RM];
        uint64_t bal[RM];
        // row groups of this chunk that hold rows at all (uniform): a range of ~2150 rows is one full chunk of 2048
        // and a tail of ~100, whose other seven groups would otherwise run their address / validity / load work
        const int nq = (int)((r1 - c0 + T - 1) / T < RM ? (r1 - c0 + T - 1) / T : RM);
#pragma unroll
        for (int q = 0; q < RM; ++q) {
            key[q] = 0;
            bal[q] = 0;
            if (q < nq) {
                const int64_t r = c0 + (int64_t)q * T + t;
                const bool v = r < r1 && kll_valid(c, r);
                const double x = v ? kll_load(c, r) : 0.0;
                key[q] = RAWBITS ? (uint64_t)__double_as_longlong(x) : kll_key(x);
                bal[q] = __ballot(v);
            }
        }
        if (lane == 0) {
#pragma unroll
            for (int q = 0; q < RM; ++q) wc[q * NW + wave] = (unsigned int)__popcll(bal[q]);
        }
        __syncthreads();
        // wave 0: exclusive prefix of the counts in (chunk row, wave) order, written back in place; the chunk total in
        // wc[NE]
        if (wave == 0) {
            const unsigned int a0 = lane < NE ? wc[lane] : 0u, b0 = lane + 64 < NE ? wc[lane + 64] : 0u;
            unsigned int a = a0, b = b0;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const unsigned int x = __shfl_up(a, o, 64), y = __shfl_up(b, o, 64);
                if (lane >= o) {
                    a += x;
                    b += y;
                }
            }
            const unsigned int ta = __shfl(a, 63, 64), tb = __shfl(b, 63, 64);
            if (lane < NE) wc[lane] = a - a0;
            if (lane + 64 < NE) wc[lane + 64] = ta + b - b0;
            if (lane == 0) wc[NE] = ta + tb;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < RM; ++q)
            if ((bal[q] >> lane) & 1ull)
                place(base + wc[q * NW + wave] + (unsigned int)__popcll(bal[q] & ((1ull << lane) - 1ull)), key[q]);
        base += wc[NE];
        __syncthreads();
    }
}

// Level 0 read in place: its final buffer (the non-NULL values [pos, pos + len) that no compaction consumed) written
// out densely for the gather, one workgroup per column (blockIdx.x = job).
struct KllTail0Job {
    const KllColPtr* col;  // device pointer to the column's level-0 KllColPtr
    unsigned long long pos, len;
    double* out;
};
__global__ void __launch_bounds__(256)
kll_tail0_kernel(const KllTail0Job* __restrict__ jobs) {
    const KllTail0Job j = jobs[blockIdx.x];
    const KllColPtr cp = *j.col;
    __shared__ long long r0s;
    __shared__ unsigned int wc[8 * 4 + 1];
    if (threadIdx.x == 0) r0s = j.len ? (long long)kll_row_of(cp, j.pos) : cp.nrows;
    __syncthreads();
    // exactly `len` non-NULL values remain from that row to the end of the column
    kll_stage_rows<256, true>(cp.raw, (int64_t)r0s, cp.nrows, wc, [&](unsigned int pos, uint64_t bits) {
        if (pos < j.len) j.out[pos] = __longlong_as_double((long long)bits);  // the values as loaded (NaN payloads)
    });
}

template <typename S, typename D, typename M>
__device__ __forceinline__ void kll_col_ptrs(const KllColPtr* cols, uint64_t sg, S& src, D& dst, M& minmax) {
    if (cols) {
        const KllColPtr cp = cols[(sg >> 55) & 0xFF];
        src = cp.src;
        dst = cp.dst;
        minmax = cp.minmax;
    }
}

template <int T, int E>
__global__ void __launch_bounds__(T)
kll_compact_kernel(const double* __restrict__ src, const uint64_t* __restrict__ segs, double* __restrict__ dst,
                   unsigned long long* __restrict__ minmax, const KllColPtr* __restrict__ cols,
                   const unsigned long long* __restrict__ rows, int runs) {
    constexpr int PAD = T * E;
    __shared__ uint64_t k[PAD + T];
    __shared__ KllRunScratch<T / 64> rsc;
    __shared__ unsigned int wc[8 * (T / 64) + 1];
    const uint64_t sg = segs[blockIdx.x];
    kll_col_ptrs(cols, sg, src, dst, minmax);
    const uint64_t start = sg & ((1ull << 40) - 1);
    const int len = (int)((sg >> 40) & 0x7FFF);
    const int t = threadIdx.x;
    uint64_t v[E];
    bool sorted = false;
    if (rows && !src) {  // level 0 read in place: stage the range's values in dense order (uniform branch)
        auto at = [](int i) { return i + i / E; };
        kll_stage_rows<T>(cols[(sg >> 55) & 0xFF].raw, (int64_t)rows[2 * blockIdx.x], (int64_t)rows[2 * blockIdx.x + 1],
                          wc, [&](unsigned int pos, uint64_t key) { if ((int)pos < len) k[at((int)pos)] = key; });
#pragma unroll
        for (int r = 0; r < E; ++r) {
            const int i = t * E + r;
            v[r] = i < len ? k[at(i)] : ~0ull;
        }
    } else {
        const double* in = src + start;
#pragma unroll
        for (int r = 0; r < E; ++r) {
            const int i = t * E + r;
            v[r] = i < len ? kll_key(in[i]) : ~0ull;
        }
        if (runs) {  // a level above 0: its range is a few sorted runs (uniform branch)
            const int ip = t * E - 1;
            const uint64_t vprev = ip >= 0 && ip < len ? kll_key(in[ip]) : ~0ull;
            sorted = kll_natural_sort<T, E>(k, v, t, vprev, rsc);
        }
    }
    if (!sorted) {
        kll_reg_sort<E>(v);
        int w0 = E;
        if constexpr (E == 8 && DQ_KLL_DPP) {
            kll_dpp_rounds(v, t);
            w0 = DQ_KLL_DPP >= 2 ? 128 : 64;
        }
        for (int w = w0; w < PAD; w <<= 1) kll_merge_round<E>(k, v, t, w);
    }
    // picks: sorted index i = t*E + r with i = offset + 2j, j < len/2
    const int half = len >> 1;
    const int off = (int)(sg >> 63);
    double* out = dst + (start >> 1);
#pragma unroll
    for (int r = 0; r < E; ++r) {
        const int i = t * E + r;
        const int d = i - off;
        if (d >= 0 && (d & 1) == 0 && (d >> 1) < half) out[d >> 1] = kll_value(v[r]);
    }
    if (minmax && len > 0) {
        if (t == 0 && v[0] < *(volatile unsigned long long*)&minmax[0]) atomicMin(&minmax[0], (unsigned long long)v[0]);
        const int last = len - 1;
        if (t == last / E) {
            uint64_t hi = 0;
#pragma unroll
            for (int r = 0; r < E; ++r)
                if (r == last % E) hi = v[r];
            if (hi > *(volatile unsigned long long*)&minmax[1]) atomicMax(&minmax[1], (unsigned long long)hi);
        }
    }
}

// Compactions of L = P + rx items with P = T*E a power of two and 0 <= rx <= kll_xm(T) (the schedule's L sit just above
// powers of two: 2060, 1030, 516, 258, ...): the first P items take the exact-size merge sort above, the rx newest
// ones are sorted apart (wave 0's bitonic over lanes up to 64 of them, else a rank pass: 13.5 % of C5's level-0
// compactions have 65-256 extras, which the padded 3072 class sorted at 2.3x the cost) and merged by rank — a main item
// moves up by the extras strictly below it, an extra lands after the main items <= it.
// (224, which keeps the 2048-key class at 20.4 KB of LDS for 8 workgroups per CU instead of 7, measured the same:
// profiles/r04/c5_kll_ab_r04ab.txt)
__host__ __device__ constexpr int kll_xm(int T) { return T < 256 ? T : 256; }

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t x, int m) {
    const int lo = __shfl_xor((int)(uint32_t)x, m, 64), hi = __shfl_xor((int)(uint32_t)(x >> 32), m, 64);
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

template <int T, int E>
__global__ void __launch_bounds__(T)
kll_compact_x_kernel(const double* __restrict__ src, const uint64_t* __restrict__ segs, double* __restrict__ dst,
                     unsigned long long* __restrict__ minmax, const KllColPtr* __restrict__ cols,
                     const unsigned long long* __restrict__ rows, int runs) {
    constexpr int P = T * E;
    constexpr int XM = kll_xm(T);
    __shared__ uint64_t k[P + T];
    __shared__ uint64_t ex[XM];
    __shared__ unsigned int wc[8 * (T / 64) + 1];
    __shared__ KllRunScratch<T / 64> rsc;
    auto at = [](int i) { return i + i / E; };
    const uint64_t sg = segs[blockIdx.x];
    kll_col_ptrs(cols, sg, src, dst, minmax);
    const uint64_t start = sg & ((1ull << 40) - 1);
    const int len = (int)((sg >> 40) & 0x7FFF);
    const int rx = len - P;  // 0..XM (host-checked)
    const int t = threadIdx.x;
    uint64_t v[E];
    uint64_t xk = ~0ull;
    bool sorted = false;
    if (rows && !src) {  // level 0 read in place (see kll_compact_kernel)
        kll_stage_rows<T>(cols[(sg >> 55) & 0xFF].raw, (int64_t)rows[2 * blockIdx.x], (int64_t)rows[2 * blockIdx.x + 1],
                          wc, [&](unsigned int pos, uint64_t key) {
                              if ((int)pos < P) k[at((int)pos)] = key;
                              else if ((int)pos < len) ex[pos - P] = key;
                          });
#pragma unroll
        for (int r = 0; r < E; ++r) v[r] = k[at(t * E + r)];
        if (t < XM && t < rx) xk = ex[t];
        __syncthreads();  // every extra read before wave 0 sorts them back into ex[]
    } else {
        const double* in = src + start;
#pragma unroll
        for (int r = 0; r < E; ++r) v[r] = kll_key(in[t * E + r]);
        if (t < XM && t < rx) xk = kll_key(in[P + t]);
        if (runs) sorted = kll_natural_sort<T, E>(k, v, t, t > 0 ? kll_key(in[t * E - 1]) : 0ull, rsc);
    }
    if (!sorted) {
        kll_reg_sort<E>(v);
        int w0 = E;
        if constexpr (E == 8 && DQ_KLL_DPP) {
            kll_dpp_rounds(v, t);
            w0 = DQ_KLL_DPP >= 2 ? 128 : 64;
        }
        for (int w = w0; w < P; w <<= 1) kll_merge_round<E>(k, v, t, w);
    }
    // the sorted main array in LDS (the extras' ranks) and the extras sorted by wave 0
#pragma unroll
    for (int r = 0; r < E; ++r) k[at(t * E + r)] = v[r];
    if (rx <= 64) {  // wave 0: bitonic over its lanes (rx is uniform)
        if (t < 64) {
#pragma unroll
            for (int size = 2; size <= 64; size <<= 1)
#pragma unroll
                for (int stride = size >> 1; stride > 0; stride >>= 1) {
                    const uint64_t y = shfl_xor_u64(xk, stride);
                    const bool keep_min = ((t & stride) == 0) == ((t & size) == 0);
                    xk = keep_min ? (y < xk ? y : xk) : (y > xk ? y : xk);
                }
            ex[t] = xk;
        }
    } else {  // up to XM extras: each one's rank among them (ties by arrival), one pass over LDS broadcasts
        if (t < rx) ex[t] = xk;
        __syncthreads();
        int rk = 0;
        if (t < rx)
            for (int j = 0; j < rx; ++j) {
                const uint64_t y = ex[j];
                rk += (y < xk || (y == xk && j < t)) ? 1 : 0;
            }
        __syncthreads();
        if (t < rx) ex[rk] = xk;
    }
    __syncthreads();
    const int half = len >> 1;
    const int off = (int)(sg >> 63);
    double* out = dst + (start >> 1);
    // main items: sorted index t*E + r plus the extras strictly below
    int c = 0, hb = rx;
    while (c < hb) {
        const int mid = (c + hb) >> 1;
        if (ex[mid] < v[0]) c = mid + 1;
        else hb = mid;
    }
#pragma unroll
    for (int r = 0; r < E; ++r) {
        while (c < rx && ex[c] < v[r]) ++c;
        const int d = t * E + r + c - off;
        if (d >= 0 && (d & 1) == 0 && (d >> 1) < half) out[d >> 1] = kll_value(v[r]);
    }
    // extras: their index among the extras plus the main items <= them
    if (t < rx) {
        const uint64_t x = ex[t];
        int lo = 0, hi = P;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (k[at(mid)] <= x) lo = mid + 1;
            else hi = mid;
        }
        const int d = lo + t - off;
        if (d >= 0 && (d & 1) == 0 && (d >> 1) < half) out[d >> 1] = kll_value(x);
    }
    if (minmax && t == 0 && len > 0) {
        uint64_t mn = k[at(0)], mx = k[at(P - 1)];
        if (rx > 0) {
            mn = ex[0] < mn ? ex[0] : mn;
            mx = ex[rx - 1] > mx ? ex[rx - 1] : mx;
        }
        if (mn < *(volatile unsigned long long*)&minmax[0]) atomicMin(&minmax[0], (unsigned long long)mn);
        if (mx > *(volatile unsigned long long*)&minmax[1]) atomicMax(&minmax[1], (unsigned long long)mx);
    }
}

// ---- level 0 on fp64 min / max (r06) ---------------------------------------------------------------------------------
// A level-0 compaction sorts raw values. Sorting them as doubles lets a compare-exchange be one v_min_f64 + one
// v_max_f64 instead of a 64-bit compare and four 32-bit selects of the order keys (the register network, the bitonic
// halves after each lane-exchange round and the LDS merge rounds are most of the kernel's VALU work). IEEE order and
// Java's Double.compare order (Scala's `.sorted` over Ordering.Double, A/QuantileNonSample.scala) differ in two places
// only, both restored by position after the sort, from counts taken before it:
//   * NaN: mapped to +inf (min against +inf: 1 instruction); Java puts every NaN above +inf, so the last nnan sorted
//     positions of the range are NaN (written as the canonical NaN, as kll_value(kll_key(NaN)) does);
//   * -0.0 == +0.0 under IEEE compares (and min / max may return either): Java has -0.0 < +0.0, so of the zeros' sorted
//     positions [nlt0, nlt0 + nzero) the first nneg0 are -0.0 and the rest +0.0 (nlt0 = values below zero, counted
//     after the sort when the range holds a -0.0 at all: the multiset is the same).
// Every other value sorts identically, so the picks, the next level's stream and min / max are bit-identical to the
// order-key sort (tests/test_gpu_kll.py runs both, DQ_KLL_NO_F64=1).
__device__ __forceinline__ double kll_canon_f(double x) { return __builtin_canonicalize(x); }
__device__ __forceinline__ double kll_min_f(double a, double b) { return __builtin_fmin(a, b); }
__device__ __forceinline__ double kll_max_f(double a, double b) { return __builtin_fmax(a, b); }

__device__ __forceinline__ void kll_reg_sort8_f(double (&w)[8]) {
#pragma unroll
    for (int size = 2; size <= 8; size <<= 1)
#pragma unroll
        for (int stride = size >> 1; stride > 0; stride >>= 1)
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const int q = r ^ stride;
                if (q > r) {
                    const double a = w[r], b = w[q];
                    const double lo = kll_min_f(a, b), hi = kll_max_f(a, b);
                    const bool asc = (r & size) == 0;
                    w[r] = asc ? lo : hi;
                    w[q] = asc ? hi : lo;
                }
            }
}

template <int CTRL>
__device__ __forceinline__ double kll_dpp_f(double x) {
    return __longlong_as_double((long long)kll_dpp64<CTRL>((uint64_t)__double_as_longlong(x)));
}

template <int CTRL, bool REV>
__device__ __forceinline__ void kll_dpp_stage_f(double (&v)[8], bool lower) {
    double b[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) b[r] = kll_dpp_f<CTRL>(v[r]);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const double x = v[r], y = b[REV ? 7 - r : r];
        v[r] = (x < y) == lower ? x : y;
    }
}

__device__ __forceinline__ void kll_bitonic8_f(double (&v)[8]) {
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] = kll_canon_f(v[r]);  // after lane moves: one canonicalisation, then min / max
#pragma unroll
    for (int stride = 4; stride > 0; stride >>= 1)
#pragma unroll
        for (int r = 0; r < 8; ++r)
            if ((r & stride) == 0) {
                const double x = v[r], y = v[r + stride];
                v[r] = kll_min_f(x, y);
                v[r + stride] = kll_max_f(x, y);
            }
}

__device__ __forceinline__ void kll_dpp_rounds_f(double (&v)[8], int t) {
    constexpr int kXor1 = 0xB1, kXor2 = 0x4E, kRev4 = 0x1B, kRev8 = 0x141;
    constexpr int kRev16 = 0x140, kShl4 = 0x104, kShr4 = 0x114;
    kll_dpp_stage_f<kXor1, true>(v, (t & 1) == 0);  // w = 8
    kll_bitonic8_f(v);
    kll_dpp_stage_f<kRev4, true>(v, (t & 2) == 0);  // w = 16
    kll_dpp_stage_f<kXor1, false>(v, (t & 1) == 0);
    kll_bitonic8_f(v);
    kll_dpp_stage_f<kRev8, true>(v, (t & 4) == 0);  // w = 32
    kll_dpp_stage_f<kXor2, false>(v, (t & 2) == 0);
    kll_dpp_stage_f<kXor1, false>(v, (t & 1) == 0);
    kll_bitonic8_f(v);
    kll_dpp_stage_f<kRev16, true>(v, (t & 8) == 0);  // w = 64
    {
        const bool lo4 = (t & 4) == 0;
        double b[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const double up = kll_dpp_f<kShl4>(v[r]), dn = kll_dpp_f<kShr4>(v[r]);
            b[r] = lo4 ? up : dn;
        }
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const double x = v[r], y = b[r];
            v[r] = (x < y) == lo4 ? x : y;
        }
    }
    kll_dpp_stage_f<kXor2, false>(v, (t & 2) == 0);
    kll_dpp_stage_f<kXor1, false>(v, (t & 1) == 0);
    kll_bitonic8_f(v);
}

// kll_merge_round for E = 8 over doubles (the LDS image holds double bits; +inf pads).
__device__ __forceinline__ void kll_merge_round8_f(double* k, double (&v)[8], int t, int w) {
    constexpr int E = 8;
    auto at = [](int i) { return i + i / E; };
    const bool wave_local = 2 * w <= 64 * E;
    const double inf = __builtin_huge_val();
#pragma unroll
    for (int r = 0; r < E; ++r) k[at(t * E + r)] = v[r];
    kll_round_sync(wave_local);
    const int diag = E * (t & (2 * (w / E) - 1));
    const int A = (t * E) - diag, B = A + w;
    int lo = diag > w ? diag - w : 0, hi = diag < w ? diag : w;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (k[at(A + mid)] <= k[at(B + diag - 1 - mid)]) lo = mid + 1;
        else hi = mid;
    }
    const int ai = A + lo, bi = B + diag - lo;
    const int aend = A + w, bend = B + w;
    double a[E], b[E];
#pragma unroll
    for (int r = 0; r < E; ++r) {
        a[r] = kll_canon_f(ai + r < aend ? k[at(ai + r)] : inf);
        b[r] = kll_canon_f(bi + r < bend ? k[at(bi + r)] : inf);
    }
#pragma unroll
    for (int r = 0; r < E; ++r) v[r] = kll_min_f(a[r], b[E - 1 - r]);
#pragma unroll
    for (int stride = E / 2; stride > 0; stride >>= 1)
#pragma unroll
        for (int r = 0; r < E; ++r)
            if ((r & stride) == 0) {
                const double x = v[r], y = v[r + stride];
                v[r] = kll_min_f(x, y);
                v[r + stride] = kll_max_f(x, y);
            }
    kll_round_sync(wave_local);
}

// Level-0 compactions of L = P + rx items (P = 8T), as kll_compact_x_kernel, sorting doubles (see above).
template <int T>
__global__ void __launch_bounds__(T)
kll_compact_xf_kernel(const double* __restrict__ src, const uint64_t* __restrict__ segs, double* __restrict__ dst,
                      unsigned long long* __restrict__ minmax, const KllColPtr* __restrict__ cols,
                      const unsigned long long* __restrict__ rows) {
    constexpr int E = 8, P = T * E, XM = kll_xm(T), NW = T / 64;
    __shared__ double k[P + T];
    __shared__ double ex[XM];
    __shared__ unsigned int wc[8 * NW + 1];
    __shared__ int cnt[3];  // NaN, -0.0, below zero
    auto at = [](int i) { return i + i / E; };
    const uint64_t sg = segs[blockIdx.x];
    kll_col_ptrs(cols, sg, src, dst, minmax);
    const uint64_t start = sg & ((1ull << 40) - 1);
    const int len = (int)((sg >> 40) & 0x7FFF);
    const int rx = len - P;  // 0..XM (host-checked)
    const int t = threadIdx.x, lane = t & 63;
    const double inf = __builtin_huge_val();
    if (t < 3) cnt[t] = 0;
    __syncthreads();  // cnt[] cleared before any wave counts into it below
    double v[E];
    double xk = inf;
    if (rows && !src) {  // level 0 read in place: the range's values in dense order, as loaded
        kll_stage_rows<T, true>(cols[(sg >> 55) & 0xFF].raw, (int64_t)rows[2 * blockIdx.x],
                                (int64_t)rows[2 * blockIdx.x + 1], wc, [&](unsigned int pos, uint64_t bits) {
                                    const double x = __longlong_as_double((long long)bits);
                                    if ((int)pos < P) k[at((int)pos)] = x;
                                    else if ((int)pos < len) ex[pos - P] = x;
                                });
#pragma unroll
        for (int r = 0; r < E; ++r) v[r] = k[at(t * E + r)];
        if (t < XM && t < rx) xk = ex[t];
    } else {
        const double* in = src + start;
#pragma unroll
        for (int r = 0; r < E; ++r) v[r] = in[t * E + r];
        if (t < XM && t < rx) xk = in[P + t];
    }
    // counts over the range's values (ballot popcounts, one LDS add per wave), NaN -> +inf
    {
        int nn = 0, nz = 0;
#pragma unroll
        for (int r = 0; r <= E; ++r) {
            const double x = r < E ? v[r] : xk;
            const bool in = r < E || (t < XM && t < rx);
            nn += (int)__popcll(__ballot(in && __builtin_isnan(x)));
            nz += (int)__popcll(__ballot(in && x == 0.0 && __builtin_signbit(x)));
        }
        if (lane == 0 && (nn | nz)) {
            atomicAdd(&cnt[0], nn);
            atomicAdd(&cnt[1], nz);
        }
#pragma unroll
        for (int r = 0; r < E; ++r) v[r] = kll_min_f(kll_canon_f(v[r]), inf);
        xk = kll_min_f(kll_canon_f(xk), inf);
    }
    kll_reg_sort8_f(v);
    kll_dpp_rounds_f(v, t);
    for (int w = 128; w < P; w <<= 1) kll_merge_round8_f(k, v, t, w);
#pragma unroll
    for (int r = 0; r < E; ++r) k[at(t * E + r)] = v[r];
    if (rx <= 64) {  // wave 0: bitonic over its lanes
        if (t < 64) {
#pragma unroll
            for (int size = 2; size <= 64; size <<= 1)
#pragma unroll
                for (int stride = size >> 1; stride > 0; stride >>= 1) {
                    const double y = __longlong_as_double((long long)shfl_xor_u64((uint64_t)__double_as_longlong(xk),
                                                                                    stride));
                    const bool keep_min = ((t & stride) == 0) == ((t & size) == 0);
                    xk = keep_min ? (y < xk ? y : xk) : (y > xk ? y : xk);
                }
            ex[t] = xk;
        }
    } else {  // ranks among the extras (ties by arrival)
        __syncthreads();
        if (t < rx) ex[t] = xk;
        __syncthreads();
        int rk = 0;
        if (t < rx)
            for (int j = 0; j < rx; ++j) {
                const double y = ex[j];
                rk += (y < xk || (y == xk && j < t)) ? 1 : 0;
            }
        __syncthreads();
        if (t < rx) ex[rk] = xk;
    }
    __syncthreads();
    const int nnan = cnt[0], nneg0 = cnt[1];
    int nlt0 = 0;
    if (nneg0) {  // (uniform) the zeros' first position: values below zero, over the same multiset
        __shared__ int lt0;
        if (t == 0) lt0 = 0;
        __syncthreads();
        int c = 0;
#pragma unroll
        for (int r = 0; r < E; ++r) c += (int)__popcll(__ballot(v[r] < 0.0));
        c += (int)__popcll(__ballot(t < rx && ex[t < XM ? t : 0] < 0.0));
        if (lane == 0 && c) atomicAdd(&lt0, c);
        __syncthreads();
        nlt0 = lt0;
    }
    // the Java-order value at sorted position pos (v its IEEE-sorted value there)
    auto fix = [&](double x, int pos) {
        if (pos >= len - nnan) return __longlong_as_double(0x7ff8000000000000LL);
        if (x == 0.0) return pos < nlt0 + nneg0 ? -0.0 : 0.0;
        return x;
    };
    const int half = len >> 1;
    const int off = (int)(sg >> 63);
    double* out = dst + (start >> 1);
    int c = 0, hb = rx;
    while (c < hb) {
        const int mid = (c + hb) >> 1;
        if (ex[mid] < v[0]) c = mid + 1;
        else hb = mid;
    }
#pragma unroll
    for (int r = 0; r < E; ++r) {
        while (c < rx && ex[c] < v[r]) ++c;
        const int pos = t * E + r + c, d = pos - off;
        if (d >= 0 && (d & 1) == 0 && (d >> 1) < half) out[d >> 1] = fix(v[r], pos);
    }
    if (t < rx) {
        const double x = ex[t];
        int lo = 0, hi = P;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (k[at(mid)] <= x) lo = mid + 1;
            else hi = mid;
        }
        const int pos = lo + t, d = pos - off;
        if (d >= 0 && (d & 1) == 0 && (d >> 1) < half) out[d >> 1] = fix(x, pos);
    }
    if (minmax && t == 0 && len > 0) {
        double mn = k[at(0)], mx = k[at(P - 1)];
        if (rx > 0) {
            mn = ex[0] < mn ? ex[0] : mn;
            mx = ex[rx - 1] > mx ? ex[rx - 1] : mx;
        }
        const uint64_t kmn = kll_key(fix(mn, 0)), kmx = kll_key(fix(mx, len - 1));
        if (kmn < *(volatile unsigned long long*)&minmax[0]) atomicMin(&minmax[0], (unsigned long long)kmn);
        if (kmx > *(volatile unsigned long long*)&minmax[1]) atomicMax(&minmax[1], (unsigned long long)kmx);
    }
}

// Compaction classes: (threads, keys per thread), capacity T*E.
struct KllClass {
    int t, e;
};
constexpr KllClass kKllClasses[] = {{64, 4},   {64, 8},   {64, 12},   {64, 16},   {128, 12},  {128, 16},
                                    {256, 12}, {256, 16}, {512, 12},  {512, 16},  {1024, 12}, {1024, 16}};
constexpr int kKllNumClasses = sizeof(kKllClasses) / sizeof(kKllClasses[0]);

// Exact-size classes of kll_compact_x_kernel: P = 256 << j (T, E), for L in [P, P + 64].
// (the 2048-key class as 128 threads x 16 keys: 3 % less time in its own launches, but its 128 extras send twice as many
// compactions to the padded 3072 class; no gain overall, profiles/r04/c5_kll_ab_r04ab.txt)
constexpr KllClass kKllXClasses[] = {{64, 4}, {64, 8}, {128, 8}, {256, 8}, {512, 8}, {1024, 8}, {1024, 16}};
constexpr int kKllNumXClasses = sizeof(kKllXClasses) / sizeof(kKllXClasses[0]);
constexpr int kKllAllClasses = kKllNumClasses + kKllNumXClasses;

int kll_class_of_slow(int len) {
    for (int j = kKllNumXClasses - 1; j >= 0; --j) {
        const int P = kKllXClasses[j].t * kKllXClasses[j].e;
        if (len >= P && len - P <= kll_xm(kKllXClasses[j].t)) return kKllNumClasses + j;
    }
    static const bool no12 = getenv("DQ_KLL_NO_E12") != nullptr;  // A/B: padded power-of-two classes only
    for (int c = 0; c < kKllNumClasses; ++c)
        if (kKllClasses[c].t * kKllClasses[c].e >= len && !(no12 && kKllClasses[c].e == 12)) return c;
    return -1;
}

// kll_class_of_slow tabulated over every compaction length the schedule admits (called per compaction, twice).
int kll_class_of(int len) {
    static const std::vector<int8_t> lut = [] {
        std::vector<int8_t> t(kKllMaxPad + 1);
        for (int l = 0; l <= kKllMaxPad; ++l) t[l] = (int8_t)kll_class_of_slow(l);
        return t;
    }();
    return len >= 0 && len <= kKllMaxPad ? lut[len] : kll_class_of_slow(len);
}

int launch_kll_compact(int cls, const double* src, const uint64_t* segs, int nseg, double* dst,
                       unsigned long long* minmax, hipStream_t s, int level, const KllColPtr* cols = nullptr,
                       const unsigned long long* rows = nullptr) {
    const bool no_runs = getenv("DQ_KLL_NO_RUNS") != nullptr;  // A/B and tests: the full sort at every level
    const int runs = level > 0 && !no_runs ? 1 : 0;
    if (nseg <= 0) return 0;
    const bool no_f64 = getenv("DQ_KLL_NO_F64") != nullptr;  // A/B and tests: order keys at level 0 too
    if (level == 0 && !no_f64) {  // level 0: the E = 8 exact-size classes sort doubles (kll_compact_xf_kernel)
        switch (cls) {
#define KLL_FCASE(C, T) \
    case C: hipLaunchKernelGGL((kll_compact_xf_kernel<T>), dim3(nseg), dim3(T), 0, s, src, segs, dst, minmax, cols, rows); \
        return hipGetLastError() == hipSuccess ? 0 : -1;
            KLL_FCASE(13, 64)
            KLL_FCASE(14, 128)
            KLL_FCASE(15, 256)
            KLL_FCASE(16, 512)
            KLL_FCASE(17, 1024)
#undef KLL_FCASE
            default: break;
        }
    }
    switch (cls) {
#define KLL_CASE(C, T, E) \
    case C: hipLaunchKernelGGL((kll_compact_kernel<T, E>), dim3(nseg), dim3(T), 0, s, src, segs, dst, minmax, cols, rows, runs); break;
        KLL_CASE(0, 64, 4)
        KLL_CASE(1, 64, 8)
        KLL_CASE(2, 64, 12)
        KLL_CASE(3, 64, 16)
        KLL_CASE(4, 128, 12)
        KLL_CASE(5, 128, 16)
        KLL_CASE(6, 256, 12)
        KLL_CASE(7, 256, 16)
        KLL_CASE(8, 512, 12)
        KLL_CASE(9, 512, 16)
        KLL_CASE(10, 1024, 12)
        KLL_CASE(11, 1024, 16)
#undef KLL_CASE
#define KLL_XCASE(C, T, E) \
    case C: \
        hipLaunchKernelGGL((kll_compact_x_kernel<T, E>), dim3(nseg), dim3(T), 0, s, src, segs, dst, minmax, cols, rows, runs); break;
        KLL_XCASE(12, 64, 4)
        KLL_XCASE(13, 64, 8)
        KLL_XCASE(14, 128, 8)
        KLL_XCASE(15, 256, 8)
        KLL_XCASE(16, 512, 8)
        KLL_XCASE(17, 1024, 8)
        KLL_XCASE(18, 1024, 16)
#undef KLL_XCASE
        default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

hipStream_t ctx_stream(dq_ctx* ctx);
int ctx_device(dq_ctx* ctx);
int ctx_fail(dq_ctx* ctx, int code, const char* msg);
int ctx_num_subs(dq_ctx* ctx);
int ctx_side_streams(dq_ctx* ctx, hipStream_t* side, hipEvent_t* fork, hipEvent_t* join);
dq_ctx* ctx_sub(dq_ctx* ctx, int i);
void* ctx_scratch(dq_ctx* ctx, size_t bytes);
void* ctx_pinned_buf(dq_ctx* ctx, size_t bytes);

}  // namespace dq

namespace {

using namespace dq;

struct KBuffers {  // per-call device buffers from the context's scratch cache (no hipMalloc / hipFree per sketch)
    dq_ctx* ctx;
    std::vector<std::pair<void*, size_t>> ptrs;
    explicit KBuffers(dq_ctx* c) : ctx(c) {}
    ~KBuffers() {
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

uint64_t host_key(double d) {
    uint64_t u;
    if (d != d) {
        u = 0x7ff8000000000000ULL;
    } else {
        memcpy(&u, &d, 8);
    }
    return (u >> 63) ? ~u : (u | 0x8000000000000000ULL);
}
double host_value(uint64_t k) {
    uint64_t u = (k >> 63) ? (k & 0x7fffffffffffffffULL) : ~k;
    double d;
    memcpy(&d, &u, 8);
    return d;
}

// QuantileNonSample.capacity (A/QuantileNonSample.scala:87-89).
int kll_capacity(int sketch_size, double f, int h) {
    return 2 * ((int)ceil((double)sketch_size * pow(f, (double)h) / 2.0) + 1);
}

// The count automaton of QuantileNonSample.update/condense/expand for n updates.
struct KllLevel {
    int64_t len = 0;       // buffered items
    int32_t ncomp = 0;     // NonSampleCompactor.numOfCompress
    int32_t offset = 0;    // NonSampleCompactor.offset
    int64_t pos = 0;       // first unconsumed item of this level's stream
    int64_t arrived = 0;   // items appended to this level's stream
    int64_t per_class[32] = {0};                  // compactions per kernel class
};

struct KllSchedule {
    std::vector<KllLevel> levels;
    std::vector<uint64_t>* segs = nullptr;  // every compaction in schedule order, its level in bits 55-62
    int64_t actual = 0;
    int64_t total = 0;
};

constexpr int kKllMaxLevels = 64;

// A bitmask of the levels whose buffer reached capacity makes condense's "lowest full level" one ctz, and an
// update that finds no full level jumps straight to the next level-0 fill (nothing changes in between); the
// compactions go to the caller's buffer (~145k entries for 1e8 items).
bool kll_schedule(int64_t n, int sketch_size, double f, KllSchedule& sc, std::vector<uint64_t>* out) {
    std::vector<uint64_t>& events = *out;
    sc.segs = &events;
    int64_t cap[kKllMaxLevels + 1];
    for (int h = 0; h <= kKllMaxLevels; ++h) cap[h] = kll_capacity(sketch_size, f, h);
    // the levels as plain arrays in the loop (one compaction per iteration), copied into sc.levels at the end
    int64_t len[kKllMaxLevels + 1] = {0}, pos[kKllMaxLevels + 1] = {0}, arrived[kKllMaxLevels + 1] = {0};
    int32_t ncomp[kKllMaxLevels + 1] = {0}, offset[kKllMaxLevels + 1] = {0};
    std::vector<int64_t> per_class((size_t)(kKllMaxLevels + 1) * 32, 0);
    int nlev = 1;
    int64_t total = cap[0], actual = 0;
    uint64_t full = 0;  // bit h: len[h] >= cap[h]
    int64_t rem = n;
    events.resize((size_t)(n / 512 + 1024));
    uint64_t* ev = events.data();
    size_t ne = 0;
    while (rem > 0) {
        // the updates until condense next compacts: past `total`, and (no level full) until level 0 fills — one jump
        // per compaction (condense without a full level changes nothing but the counts)
        int64_t k = std::max<int64_t>(1, total - actual + 1);
        if (full == 0) k = std::max<int64_t>(k, cap[0] - len[0]);
        k = std::min<int64_t>(rem, k);
        len[0] += k;
        arrived[0] += k;
        actual += k;
        rem -= k;
        if (len[0] >= cap[0]) full |= 1ull;
        if (actual <= total || full == 0) continue;
        const int h = __builtin_ctzll(full);
        if (h + 1 >= nlev) {
            if (nlev >= kKllMaxLevels) return false;
            ++nlev;
            total += cap[nlev - 1];
        }
        const int64_t items = len[h];
        const int64_t L = items & ~(int64_t)1;
        if (L > kKllMaxPad) return false;
        const int32_t off = offset[h] ^ (ncomp[h] & 1);  // the offset flips on odd compaction counts
        offset[h] = off;
        if (ne == events.size()) {
            events.resize(events.size() * 2);
            ev = events.data();
        }
        ev[ne++] = kll_desc((uint64_t)pos[h], (uint32_t)L, (uint32_t)off) | ((uint64_t)h << 55);
        ++per_class[(size_t)h * 32 + kll_class_of((int)L)];
        pos[h] += L;
        len[h] = items & 1;
        full &= ~(1ull << h);
        len[h + 1] += L >> 1;
        arrived[h + 1] += L >> 1;
        if (len[h + 1] >= cap[h + 1]) full |= 1ull << (h + 1);
        ncomp[h] += 1;
        actual -= L >> 1;  // = the sum of buffer lengths, as getCompactorItemsCount recomputes it
    }
    events.resize(ne);
    sc.levels.assign(nlev, KllLevel());
    for (int h = 0; h < nlev; ++h) {
        KllLevel& l = sc.levels[h];
        l.len = len[h];
        l.ncomp = ncomp[h];
        l.offset = offset[h];
        l.pos = pos[h];
        l.arrived = arrived[h];
        for (int c = 0; c < 32; ++c) l.per_class[c] = per_class[(size_t)h * 32 + c];
    }
    sc.total = total;
    sc.actual = actual;
    return true;
}

void put_be32(std::vector<uint8_t>& o, int32_t v) {
    for (int i = 3; i >= 0; --i) o.push_back((uint8_t)((uint32_t)v >> (8 * i)));
}
void put_be64(std::vector<uint8_t>& o, uint64_t v) {
    const uint64_t be = __builtin_bswap64(v);
    const size_t at = o.size();
    o.resize(at + 8);
    memcpy(o.data() + at, &be, 8);
}
void put_f64(std::vector<uint8_t>& o, double d) {
    uint64_t u;
    memcpy(&u, &d, 8);
    put_be64(o, u);
}

}  // namespace

#define KL_HIP(ctx, expr)                                                                         \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess) return dq::ctx_fail((ctx), DQ_ERR_DEVICE, hipGetErrorString(e_));   \
    } while (0)

namespace {

// ---- host-side QuantileNonSample.merge over KLLState bytes (A/QuantileNonSample.scala:218-234, condense :94-111,
// NonSampleCompactor.compact A/NonSampleCompactor.scala:42-66; KLLState.sum / mergeUntyped, A/KLLSketch.scala:49-54,
// R/KLLRunner.scala:40-44): the partition sketches of a multi-device context folded in device order.
struct KComp {
    int32_t ncomp = 0, offset = 0;
    std::vector<double> buf;
};
struct KState {
    double gmin = 0, gmax = 0;
    int32_t sketch = 0, cur = 0, actual = 0, total = 0;
    double f = 0;
    std::vector<KComp> c;
};

uint32_t get_be32(const uint8_t* p) { return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]; }
double get_f64(const uint8_t* p) {
    uint64_t u;
    memcpy(&u, p, 8);
    u = __builtin_bswap64(u);
    double d;
    memcpy(&d, &u, 8);
    return d;
}

bool kll_parse(const uint8_t* b, size_t nb, KState& s) {
    size_t at = 0;
    auto need = [&](size_t n) { return at + n <= nb; };
    if (!need(16 + 28)) return false;
    s.gmin = get_f64(&b[0]);
    s.gmax = get_f64(&b[8]);
    at = 16;
    s.sketch = (int32_t)get_be32(&b[at]);
    s.f = get_f64(&b[at + 4]);
    s.cur = (int32_t)get_be32(&b[at + 12]);
    s.actual = (int32_t)get_be32(&b[at + 16]);
    s.total = (int32_t)get_be32(&b[at + 20]);
    const int32_t ncomp = (int32_t)get_be32(&b[at + 24]);
    at += 28;
    if (ncomp < 0 || ncomp > kKllMaxLevels) return false;
    s.c.assign(ncomp, KComp());
    for (int h = 0; h < ncomp; ++h) {
        if (!need(12)) return false;
        s.c[h].ncomp = (int32_t)get_be32(&b[at]);
        s.c[h].offset = (int32_t)get_be32(&b[at + 4]);
        const int32_t len = (int32_t)get_be32(&b[at + 8]);
        at += 12;
        if (len < 0 || !need((size_t)len * 8)) return false;
        s.c[h].buf.resize(len);
        for (int i = 0; i < len; ++i) s.c[h].buf[i] = get_f64(&b[at + 8 * (size_t)i]);
        at += (size_t)len * 8;
    }
    return true;
}

void kll_serialize(const KState& s, std::vector<uint8_t>& o) {
    o.clear();
    size_t need = 16 + 28;
    for (const KComp& c : s.c) need += 12 + 8 * c.buf.size();
    o.reserve(need);
    put_f64(o, s.gmin);
    put_f64(o, s.gmax);
    put_be32(o, s.sketch);
    put_f64(o, s.f);
    put_be32(o, s.cur);
    put_be32(o, s.actual);
    put_be32(o, s.total);
    put_be32(o, (int32_t)s.c.size());
    for (const KComp& c : s.c) {
        put_be32(o, c.ncomp);
        put_be32(o, c.offset);
        put_be32(o, (int32_t)c.buf.size());
        for (double d : c.buf) put_f64(o, d);
    }
}

int32_t kll_items(const KState& s) {
    int64_t n = 0;
    for (int h = 0; h < s.cur && h < (int)s.c.size(); ++h) n += (int64_t)s.c[h].buf.size();
    return (int32_t)n;
}

void kll_expand(KState& s) {
    s.c.push_back(KComp());
    s.cur = (int32_t)s.c.size();
    int64_t t = 0;
    for (int h = 0; h < s.cur; ++h) t += kll_capacity(s.sketch, s.f, h);
    s.total = (int32_t)t;
}

// NonSampleCompactor.compact: the first len = items - items % 2 items sorted (Ordering.Double: -0.0 < 0.0, NaN
// largest), every second from offset (flipped on odd compaction counts) goes up, the odd last item stays.
// The sort is a stable LSD radix sort of (order key, position) pairs, 8-bit digits, passes whose digit is the same for
// every item skipped (a comparison sort with the key computed per compare made the chunk merges of the C5 profiler
// ~1 ms per column).
void kll_sort_stable(const double* v, size_t n, std::vector<double>& out) {
    // a buffer above level 0 is a concatenation of sorted pick runs: with few natural runs, stable pairwise merges
    size_t runs = 1;
    for (size_t i = 1; i < n && runs <= 16; ++i) runs += host_key(v[i]) < host_key(v[i - 1]) ? 1 : 0;
    if (n > 1 && runs <= 16) {
        std::vector<uint64_t> k(n), k2(n);
        std::vector<uint32_t> ix(n), ix2(n);
        std::vector<size_t> bnd{0};
        for (size_t i = 0; i < n; ++i) {
            k[i] = host_key(v[i]);
            ix[i] = (uint32_t)i;
            if (i && k[i] < k[i - 1]) bnd.push_back(i);
        }
        bnd.push_back(n);
        while (bnd.size() > 2) {  // merge runs (0, 1), (2, 3), ...: ties from the earlier run first (stable)
            std::vector<size_t> nb{0};
            for (size_t r = 0; r + 1 < bnd.size(); r += 2) {
                const size_t a0 = bnd[r], a1 = bnd[r + 1], b1 = r + 2 < bnd.size() ? bnd[r + 2] : a1;
                size_t i = a0, j = a1, o = a0;
                while (i < a1 && j < b1) {
                    const bool takeB = k[j] < k[i];
                    k2[o] = takeB ? k[j] : k[i];
                    ix2[o++] = takeB ? ix[j++] : ix[i++];
                }
                for (; i < a1; ++i, ++o) { k2[o] = k[i]; ix2[o] = ix[i]; }
                for (; j < b1; ++j, ++o) { k2[o] = k[j]; ix2[o] = ix[j]; }
                nb.push_back(b1);
            }
            k.swap(k2);
            ix.swap(ix2);
            bnd.swap(nb);
        }
        out.resize(n);
        for (size_t i = 0; i < n; ++i) out[i] = v[ix[i]];
        return;
    }
    std::vector<uint64_t> k(n), k2(n);
    std::vector<uint32_t> ix(n), ix2(n);
    for (size_t i = 0; i < n; ++i) {
        k[i] = host_key(v[i]);
        ix[i] = (uint32_t)i;
    }
    for (int sh = 0; sh < 64; sh += 8) {
        size_t cnt[257] = {0};
        for (size_t i = 0; i < n; ++i) ++cnt[((k[i] >> sh) & 0xFF) + 1];
        bool one = false;
        for (int d = 1; d <= 256; ++d) one = one || cnt[d] == n;
        if (one) continue;  // every item has this digit
        for (int d = 1; d <= 256; ++d) cnt[d] += cnt[d - 1];
        for (size_t i = 0; i < n; ++i) {
            const size_t at = cnt[(k[i] >> sh) & 0xFF]++;
            k2[at] = k[i];
            ix2[at] = ix[i];
        }
        k.swap(k2);
        ix.swap(ix2);
    }
    out.resize(n);
    for (size_t i = 0; i < n; ++i) out[i] = v[ix[i]];
}

void kll_compact(KComp& c, std::vector<double>& out) {
    const size_t items = c.buf.size(), len = items - items % 2;
    if (c.ncomp % 2 == 1) c.offset = 1 - c.offset;
    std::vector<double> srt;
    kll_sort_stable(c.buf.data(), len, srt);
    out.clear();
    for (size_t i = (size_t)c.offset; i < len; i += 2) out.push_back(srt[i]);
    std::vector<double> keep;
    if (items % 2 == 1) keep.push_back(c.buf[items - 1]);
    c.buf.swap(keep);
    c.ncomp += 1;
}

void kll_condense(KState& s) {
    for (size_t h = 0; h < s.c.size(); ++h) {
        if ((int64_t)s.c[h].buf.size() >= kll_capacity(s.sketch, s.f, (int)h)) {
            if ((int)h + 1 >= s.cur) kll_expand(s);
            std::vector<double> out;
            kll_compact(s.c[h], out);
            s.c[h + 1].buf.insert(s.c[h + 1].buf.end(), out.begin(), out.end());
            s.actual = kll_items(s);
            break;
        }
    }
}

// java.lang.Math.max / min on doubles: NaN if either is NaN, -0.0 < 0.0
double java_max(double a, double b) {
    if (a != a || b != b) return NAN;
    return host_key(a) >= host_key(b) ? a : b;
}
double java_min(double a, double b) {
    if (a != a || b != b) return NAN;
    return host_key(a) <= host_key(b) ? a : b;
}

bool kll_merge(KState& a, const KState& b) {
    while (a.cur < b.cur) kll_expand(a);
    for (int i = 0; i < b.cur; ++i) a.c[i].buf.insert(a.c[i].buf.end(), b.c[i].buf.begin(), b.c[i].buf.end());
    a.actual = kll_items(a);
    for (int guard = 0; a.actual >= a.total; ++guard) {
        if (guard > (1 << 20)) return false;
        kll_condense(a);
    }
    a.gmax = java_max(a.gmax, b.gmax);
    a.gmin = java_min(a.gmin, b.gmin);
    return true;
}

}  // namespace

extern "C" {

// KLLState.sum of two serialized states (A/KLLSketch.scala:49-54 -> QuantileNonSample.merge, :218-234): host only.
int64_t dq_kll_merge_states(const uint8_t* a, int64_t na, const uint8_t* b, int64_t nb, uint8_t* out,
                            int64_t capacity) {
    if (!a || !b || na < 0 || nb < 0 || capacity < 0 || (capacity > 0 && !out)) return DQ_ERR_INVALID_ARGUMENT;
    KState x, y;
    if (!kll_parse(a, (size_t)na, x) || !kll_parse(b, (size_t)nb, y))
        return DQ_ERR_INVALID_ARGUMENT;
    if (!kll_merge(x, y)) return DQ_ERR_INVALID_ARGUMENT;
    std::vector<uint8_t> o;
    kll_serialize(x, o);
    if ((int64_t)o.size() <= capacity) memcpy(out, o.data(), o.size());
    return (int64_t)o.size();
}

static int64_t kll_sketch_single(dq_ctx* ctx, const dq_column* column, int64_t nrows, int32_t sketch_size,
                                 double shrinking_factor, uint8_t* state_out, int64_t capacity,
                                 std::vector<uint8_t>* keep);

int64_t dq_kll_sketch(dq_ctx* ctx, const dq_column* column, int64_t nrows, int32_t sketch_size,
                      double shrinking_factor, uint8_t* state_out, int64_t capacity) {
    if (!ctx || !column || nrows < 0 || column->length != nrows || capacity < 0 || (capacity > 0 && !state_out))
        return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_kll_sketch: invalid arguments");
    const int nsub = dq::ctx_num_subs(ctx);
    if (nsub == 0) return kll_sketch_single(ctx, column, nrows, sketch_size, shrinking_factor, state_out, capacity, nullptr);
    // multi-device context: one partition per device (contiguous row shards, KLLRunner.sketchPartitions per
    // partition), sketched concurrently, merged in device order on the host (KLLRunner's reduce of the partition
    // sketches, R/KLLRunner.scala:104-112)
    if (column->flags & DQ_COL_DEVICE) return dq::ctx_fail(ctx, DQ_ERR_UNSUPPORTED, "a multi-device context takes host columns");
    std::vector<std::vector<uint8_t>> parts(nsub);
    std::vector<int64_t> rc(nsub, 0);
    std::vector<dq_column> cols(nsub, *column);
    std::vector<std::vector<std::vector<int32_t>>> scratch(nsub);
    std::vector<std::thread> th;
    for (int i = 0; i < nsub; ++i) {
        int64_t r0 = 0, cnt = 0;
        dq::shard_bounds(nrows, nsub, i, &r0, &cnt);
        dq::shard_columns(column, 1, r0, cnt, &cols[i], scratch[i]);
        th.emplace_back([&, i, cnt]() {
            dq_ctx* sub = dq::ctx_sub(ctx, i);
            if (hipSetDevice(dq::ctx_device(sub)) != hipSuccess) {
                rc[i] = DQ_ERR_DEVICE;
                return;
            }
            rc[i] = kll_sketch_single(sub, &cols[i], cnt, sketch_size, shrinking_factor, nullptr, 0, &parts[i]);
        });
    }
    for (auto& x : th) x.join();
    for (int i = 0; i < nsub; ++i)
        if (rc[i] < 0) return dq::ctx_fail(ctx, (int)rc[i], "dq_kll_sketch: a device's partition failed");
    KState acc;
    if (!kll_parse(parts[0].data(), parts[0].size(), acc)) return dq::ctx_fail(ctx, DQ_ERR_DEVICE, "dq_kll_sketch: malformed partition state");
    for (int i = 1; i < nsub; ++i) {
        KState b;
        if (!kll_parse(parts[i].data(), parts[i].size(), b) || !kll_merge(acc, b))
            return dq::ctx_fail(ctx, DQ_ERR_DEVICE, "dq_kll_sketch: partition merge failed");
    }
    std::vector<uint8_t> o;
    kll_serialize(acc, o);
    if ((int64_t)o.size() <= capacity) memcpy(state_out, o.data(), o.size());
    return (int64_t)o.size();
}

static int kll_sketch_batch(dq_ctx* ctx, const dq_column* columns, int ncols, int64_t nrows, int32_t sketch_size,
                            double shrinking_factor, std::vector<std::vector<uint8_t>>& states);

static int64_t kll_sketch_single(dq_ctx* ctx, const dq_column* column, int64_t nrows, int32_t sketch_size,
                                 double shrinking_factor, uint8_t* state_out, int64_t capacity,
                                 std::vector<uint8_t>* keep) {
    std::vector<std::vector<uint8_t>> st;
    const int rc = kll_sketch_batch(ctx, column, 1, nrows, sketch_size, shrinking_factor, st);
    if (rc != DQ_OK) return rc;
    const std::vector<uint8_t>& o = st[0];
    if (keep) *keep = o;
    else if ((int64_t)o.size() <= capacity) memcpy(state_out, o.data(), o.size());
    return (int64_t)o.size();
}

int64_t dq_kll_sketch_columns(dq_ctx* ctx, const dq_column* columns, int32_t ncols, int64_t nrows, int32_t sketch_size,
                              double shrinking_factor, uint8_t* state_out, int64_t capacity, int64_t* sizes) {
    if (!ctx || ncols < 0 || (ncols > 0 && (!columns || !sizes)) || nrows < 0 || capacity < 0 ||
        (capacity > 0 && !state_out))
        return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_kll_sketch_columns: invalid arguments");
    for (int i = 0; i < ncols; ++i)
        if (columns[i].length != nrows)
            return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_kll_sketch_columns: column length differs from nrows");
    std::vector<std::vector<uint8_t>> st(ncols);
    if (dq::ctx_num_subs(ctx) == 0) {
        const int rc = kll_sketch_batch(ctx, columns, ncols, nrows, sketch_size, shrinking_factor, st);
        if (rc != DQ_OK) return rc;
    } else {  // multi-device context: each column through dq_kll_sketch's per-device partitions
        for (int i = 0; i < ncols; ++i) {
            const int64_t need = dq_kll_sketch(ctx, &columns[i], nrows, sketch_size, shrinking_factor, nullptr, 0);
            if (need < 0) return need;
            st[i].resize((size_t)need);
            const int64_t got = dq_kll_sketch(ctx, &columns[i], nrows, sketch_size, shrinking_factor, st[i].data(), need);
            if (got < 0) return got;
        }
    }
    int64_t total = 0;
    for (int i = 0; i < ncols; ++i) {
        sizes[i] = (int64_t)st[i].size();
        total += sizes[i];
    }
    if (total <= capacity) {
        int64_t at = 0;
        for (int i = 0; i < ncols; ++i) {
            if (!st[i].empty()) memcpy(state_out + at, st[i].data(), st[i].size());
            at += (int64_t)st[i].size();
        }
    }
    return total;
}

// One call's columns, each one partition in row order: the NULL-compaction counts of every column, ONE host round
// trip, the compaction schedules on parallel host threads, every column's dense write + compaction launches + final
// gather queued on the stream, ONE more round trip, then each column's KLLState bytes.
struct KColumnRun {
    KllColumn kc;
    bool zero_copy = false;
    int64_t ntiles = 0, n = 0;
    unsigned long long* doffs = nullptr;
    const double* stream0 = nullptr;
    KllSchedule sc;
    std::vector<uint64_t> events;
    std::vector<int64_t> lbase;
    int64_t ntail = 0;
    size_t pin_at = 0;          // this column's region of the pinned staging area
    double* hgat = nullptr;     // pinned: gathered final buffers, then the 2 min / max keys
    struct Launch {
        size_t level, first, count;
        int cls;
    };
    std::vector<Launch> launches;  // compactions grouped per (level, kernel class)
};

// Runs work(i) for i < n on up to hardware-concurrency host threads (inline when n == 1).
extern "C++" template <typename F>
static void kll_parallel(int n, F work) {
    if (n <= 1) {
        if (n == 1) work(0);
        return;
    }
    std::vector<std::thread> th;
    const int nth = std::min(n, std::max(1, (int)std::thread::hardware_concurrency()));
    for (int w = 0; w < nth; ++w)
        th.emplace_back([&, w]() {
            for (int i = w; i < n; i += nth) work(i);
        });
    for (auto& x : th) x.join();
}

static int kll_sketch_batch(dq_ctx* ctx, const dq_column* columns, int ncols, int64_t nrows, int32_t sketch_size,
                            double shrinking_factor, std::vector<std::vector<uint8_t>>& states) {
    states.assign(ncols, std::vector<uint8_t>());
    if (!(shrinking_factor == shrinking_factor))
        return dq::ctx_fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_kll_sketch: shrinking factor is NaN");
    for (int i = 0; i < ncols; ++i) {
        const int t = columns[i].spark_type;
        if (!(t == DQ_TYPE_BYTE || t == DQ_TYPE_SHORT || t == DQ_TYPE_INT || t == DQ_TYPE_LONG || t == DQ_TYPE_FLOAT ||
              t == DQ_TYPE_DOUBLE))
            return dq::ctx_fail(ctx, DQ_ERR_UNSUPPORTED, "dq_kll_sketch: Cannot handle column type");
    }
    const int dev = dq::ctx_device(ctx);
    KL_HIP(ctx, hipSetDevice(dev));
    hipStream_t s = dq::ctx_stream(ctx);
    KBuffers buf(ctx);
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<KColumnRun> run(ncols);
    const int64_t ntiles = (nrows + kKllStageRows - 1) / kKllStageRows;
    unsigned long long* dtotals = nullptr;
    KL_HIP(ctx, buf.alloc((void**)&dtotals, sizeof(unsigned long long) * std::max(ncols, 1)));
    int ncount = 0;
    std::vector<KllCountJob> jobs;  // every NULL-compacted column's counts: one count and one scan launch for all
    std::vector<int> job_col;
    for (int i = 0; i < ncols; ++i) {
        const dq_column* column = &columns[i];
        KColumnRun& r = run[i];
        r.kc.elem = elem_of(column->spark_type);
        const size_t vbytes = (size_t)nrows * elem_size(r.kc.elem);
        const size_t bbytes = (size_t)(nrows + 63) / 64 * 8;
        if (column->flags & DQ_COL_DEVICE) {
            r.kc.values = column->values;
            r.kc.validity = (const uint64_t*)column->validity;
        } else {
            void *v = nullptr, *m = nullptr;
            KL_HIP(ctx, buf.alloc(&v, vbytes));
            if (nrows) KL_HIP(ctx, hipMemcpyAsync(v, column->values, vbytes, hipMemcpyHostToDevice, s));
            if (column->validity) {
                KL_HIP(ctx, buf.alloc(&m, bbytes));
                KL_HIP(ctx, hipMemsetAsync(m, 0, bbytes, s));
                if (nrows)
                    KL_HIP(ctx, hipMemcpyAsync(m, column->validity, (size_t)(nrows + 7) / 8, hipMemcpyHostToDevice, s));
            }
            r.kc.values = v;
            r.kc.validity = (const uint64_t*)m;
        }
        r.ntiles = ntiles;
        r.zero_copy = r.kc.elem == ET_F64 && r.kc.validity == nullptr;
        if (r.zero_copy) {
            r.stream0 = static_cast<const double*>(r.kc.values);
            r.n = nrows;
        } else if (nrows > 0) {
            unsigned int* dcounts = nullptr;
            KL_HIP(ctx, buf.alloc((void**)&dcounts, sizeof(unsigned int) * ntiles));
            KL_HIP(ctx, buf.alloc((void**)&r.doffs, sizeof(unsigned long long) * ntiles));
            jobs.push_back(KllCountJob{r.kc, dcounts, r.doffs, dtotals + i, nullptr});
            job_col.push_back(i);
            ++ncount;
        }
    }
    if (ncount) {
        KllCountJob* djobs = nullptr;
        KL_HIP(ctx, buf.alloc((void**)&djobs, sizeof(KllCountJob) * jobs.size()));
        KL_HIP(ctx, hipMemcpyAsync(djobs, jobs.data(), sizeof(KllCountJob) * jobs.size(), hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(kll_count_kernel,
                           dim3((unsigned)((ntiles + kKllCountTilesPerBlock - 1) / kKllCountTilesPerBlock),
                                (unsigned)jobs.size()),
                           dim3(kKllStageBlock), 0, s, (const KllCountJob*)djobs, nrows, (int64_t)ntiles);
        hipLaunchKernelGGL(kll_scan_kernel, dim3(1, (unsigned)jobs.size()), dim3(1024), 0, s, (const KllCountJob*)djobs,
                           ntiles);
        KL_HIP(ctx, hipGetLastError());
    }
    if (ncount) {  // one round trip for every column's non-NULL count
        unsigned long long* htotals = static_cast<unsigned long long*>(dq::ctx_pinned_buf(ctx, 8 * (size_t)ncols));
        if (!htotals) return DQ_ERR_OUT_OF_MEMORY;
        KL_HIP(ctx, hipMemcpyAsync(htotals, dtotals, 8 * (size_t)ncols, hipMemcpyDeviceToHost, s));
        KL_HIP(ctx, hipStreamSynchronize(s));
        for (int i = 0; i < ncols; ++i)
            if (!run[i].zero_copy) run[i].n = nrows > 0 ? (int64_t)htotals[i] : 0;
    }
    // columns are independent: their compaction chains go round-robin onto the context's stream and its side streams
    // (forked after the non-NULL counts, joined before the read-back): each column's dense write and compaction chain, so one column's small upper-level launches overlap
    // another's instead of leaving the chip idle between them
    hipStream_t cstreams[1 + 8] = {s};
    hipEvent_t fork_ev = nullptr, join_ev[8] = {};
    int nstreams = 1;
    // several columns: one launch per (level, class) over all of them (below) unless DQ_KLL_PER_COLUMN asks for one
    // launch chain per column (spread over the streams)
    const bool batched = ncols >= 1 && ncols <= 255 && !getenv("DQ_KLL_PER_COLUMN");
    // batched: level 0 of a NULL-compacted column is read in place by its compactions (no dense stream: 8 B written and
    // re-read per value less; DQ_KLL_DENSE=1 writes the dense stream first). r04 measured in place slower end to end
    // (profiles/r04/c5_kll_ab_r04k.txt: the compactions waited for the host schedule that the dense write overlapped);
    // since the schedule automaton runs on plain arrays the two are equal in time on the C5 shard (r05: 125.1 vs
    // 126.9 ms a profile, profiles/r05/c5_kll_inplace_ab_r05ah.txt) and in place moves ~50 GB less, so it is the default.
    const bool inplace = batched && getenv("DQ_KLL_DENSE") == nullptr;
    if (ncols > 1 && !batched && !getenv("DQ_KLL_SERIAL")) {
        const int nside = dq::ctx_side_streams(ctx, cstreams + 1, &fork_ev, join_ev);
        if (nside > 0) {
            nstreams = 1 + std::min(nside, ncols - 1);
            KL_HIP(ctx, hipEventRecord(fork_ev, s));
            for (int j = 1; j < nstreams; ++j) KL_HIP(ctx, hipStreamWaitEvent(cstreams[j], fork_ev, 0));
        }
    }
    // dense level-0 streams go out while the host computes the (count-only) compaction schedules; batched: one launch
    if (batched && !inplace && !jobs.empty()) {
        for (size_t j = 0; j < jobs.size(); ++j) {
            KColumnRun& r = run[job_col[j]];
            if (r.n <= 0) continue;
            KL_HIP(ctx, buf.alloc((void**)&jobs[j].dense, (size_t)r.n * 8));
            r.stream0 = jobs[j].dense;
        }
        KllCountJob* wjobs = nullptr;
        KL_HIP(ctx, buf.alloc((void**)&wjobs, sizeof(KllCountJob) * jobs.size()));
        KL_HIP(ctx, hipMemcpyAsync(wjobs, jobs.data(), sizeof(KllCountJob) * jobs.size(), hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(kll_write_jobs_kernel, dim3((unsigned)ntiles, (unsigned)jobs.size()), dim3(kKllStageBlock), 0, s,
                           (const KllCountJob*)wjobs, nrows);
        KL_HIP(ctx, hipGetLastError());
    }
    for (int i = 0; i < ncols && !batched; ++i) {
        KColumnRun& r = run[i];
        if (r.zero_copy || r.n <= 0) continue;
        double* dense = nullptr;
        KL_HIP(ctx, buf.alloc((void**)&dense, (size_t)r.n * 8));
        hipLaunchKernelGGL(kll_write_kernel, dim3((unsigned)r.ntiles), dim3(kKllStageBlock), 0, cstreams[i % nstreams],
                           r.kc, nrows,
                           (const unsigned long long*)r.doffs, dense);
        KL_HIP(ctx, hipGetLastError());
        r.stream0 = dense;
    }
    const auto t0b = std::chrono::steady_clock::now();
    {
        std::vector<int> ok(ncols, 1);
        kll_parallel(ncols, [&](int i) {
            ok[i] = kll_schedule(run[i].n, sketch_size, shrinking_factor, run[i].sc, &run[i].events);
        });
        for (int i = 0; i < ncols; ++i)
            if (!ok[i])
                return dq::ctx_fail(ctx, DQ_ERR_UNSUPPORTED,
                                    "dq_kll_sketch: sketch parameters need a compaction larger than 16384 items");
    }
    const auto t1 = std::chrono::steady_clock::now();

    if (batched) {
        // every column's compactions grouped per (level, class, column): one launch per (level, class) covers all
        // columns, so the upper levels' small per-column launches (a few workgroups each) become one wide launch
        constexpr size_t NC = kKllAllClasses;
        size_t maxlev = 0;
        for (const KColumnRun& r : run) maxlev = std::max(maxlev, r.sc.levels.size());
        std::vector<size_t> cnt(std::max<size_t>(maxlev * NC * ncols, 1), 0), first(cnt.size(), 0);
        for (int i = 0; i < ncols; ++i)
            for (size_t h = 0; h < run[i].sc.levels.size(); ++h)
                for (size_t c = 0; c < NC; ++c) cnt[(h * NC + c) * ncols + i] = (size_t)run[i].sc.levels[h].per_class[c];
        size_t nseg_all = 0;
        for (size_t q = 0; q < cnt.size(); ++q) {
            first[q] = nseg_all;
            nseg_all += cnt[q];
        }
        // pinned: [descriptors][pointer tables, level-major][min / max init], then per column [tails][finals + min / max]
        const size_t seg_bytes = (nseg_all * 8 + 255) / 256 * 256;
        const size_t tab_bytes = (std::max<size_t>(maxlev, 1) * ncols * sizeof(KllColPtr) + 255) / 256 * 256;
        const size_t mm_bytes = ((size_t)ncols * 16 + 255) / 256 * 256;
        size_t pin_total = seg_bytes + tab_bytes + mm_bytes;
        for (KColumnRun& r : run) {
            const size_t nlev = r.sc.levels.size();
            r.ntail = 0;
            for (const KllLevel& l : r.sc.levels) r.ntail += l.len;
            r.pin_at = pin_total;
            pin_total += (nlev * sizeof(KllTail) + (size_t)r.ntail * 8 + 16 + 255) / 256 * 256;
        }
        uint8_t* pin = static_cast<uint8_t*>(dq::ctx_pinned_buf(ctx, pin_total));
        if (!pin) return DQ_ERR_OUT_OF_MEMORY;
        uint64_t* hsegs = reinterpret_cast<uint64_t*>(pin);
        KllColPtr* htab = reinterpret_cast<KllColPtr*>(pin + seg_bytes);
        unsigned long long* hmm = reinterpret_cast<unsigned long long*>(pin + seg_bytes + tab_bytes);
        kll_parallel(ncols, [&](int i) {
            std::vector<size_t> cur(maxlev * NC);
            for (size_t q = 0; q < cur.size(); ++q) cur[q] = first[q * ncols + i];
            for (const uint64_t d : run[i].events) {  // the level bits give way to the column
                const size_t h = (size_t)((d >> 55) & 0xFF);
                const size_t c = (size_t)kll_class_of((int)((d >> 40) & 0x7FFF));
                hsegs[cur[h * NC + c]++] = (d & ~(0xFFull << 55)) | ((uint64_t)i << 55);
            }
        });
        uint8_t* gdev = nullptr;
        KL_HIP(ctx, buf.alloc((void**)&gdev, seg_bytes + tab_bytes + mm_bytes));
        // level 0 in place: (first row, end row) per descriptor, filled for level 0 by kll_locate_kernel
        unsigned long long* drows = nullptr;
        if (inplace) KL_HIP(ctx, buf.alloc((void**)&drows, std::max<size_t>(nseg_all, 1) * 16));
        std::vector<KllTail0Job> tail0;
        const uint64_t* dsegs = reinterpret_cast<const uint64_t*>(gdev);
        const KllColPtr* dtab = reinterpret_cast<const KllColPtr*>(gdev + seg_bytes);
        unsigned long long* dmm = reinterpret_cast<unsigned long long*>(gdev + seg_bytes + tab_bytes);
        std::vector<KllTail*> dtails(ncols);
        std::vector<double*> dgats(ncols);
        memset(htab, 0, tab_bytes);
        for (int i = 0; i < ncols; ++i) {
            KColumnRun& r = run[i];
            const KllSchedule& sc = r.sc;
            const size_t nlev = sc.levels.size();
            r.lbase.assign(nlev, 0);
            int64_t upper = 0;
            for (size_t h = 1; h < nlev; ++h) {
                r.lbase[h] = upper;
                upper += sc.levels[h].arrived;
            }
            const size_t tail_off = ((size_t)upper * 8 + 255) / 256 * 256;
            const size_t gat_off = tail_off + (nlev * sizeof(KllTail) + 255) / 256 * 256;
            uint8_t* scratch = nullptr;
            KL_HIP(ctx, buf.alloc((void**)&scratch, gat_off + (size_t)r.ntail * 8 + 256));
            double* dup = reinterpret_cast<double*>(scratch);
            dtails[i] = reinterpret_cast<KllTail*>(scratch + tail_off);
            dgats[i] = reinterpret_cast<double*>(scratch + gat_off);
            for (size_t h = 0; h < nlev; ++h)
                htab[h * ncols + i] = KllColPtr{h == 0 ? r.stream0 : dup + r.lbase[h], h + 1 < nlev ? dup + r.lbase[h + 1] : nullptr,
                                                h == 0 ? dmm + 2 * i : nullptr, r.kc, r.doffs, r.ntiles, nrows};
            const bool raw0 = r.stream0 == nullptr && r.n > 0;  // level 0 read in place
            double* tail0_buf = nullptr;
            if (raw0 && sc.levels[0].len > 0) {
                KL_HIP(ctx, buf.alloc((void**)&tail0_buf, (size_t)sc.levels[0].len * 8));
                tail0.push_back(KllTail0Job{dtab + i, (unsigned long long)sc.levels[0].pos,
                                            (unsigned long long)sc.levels[0].len, tail0_buf});
            }
            hmm[2 * i] = ~0ull;
            hmm[2 * i + 1] = 0ull;
            KllTail* htails = reinterpret_cast<KllTail*>(pin + r.pin_at);
            r.hgat = reinterpret_cast<double*>(pin + r.pin_at + nlev * sizeof(KllTail));
            unsigned long long at = 0;
            for (size_t h = 0; h < nlev; ++h) {
                const KllLevel& l = sc.levels[h];
                const double* src = h == 0 ? (raw0 ? tail0_buf : r.stream0 + l.pos) : dup + r.lbase[h] + l.pos;
                htails[h] = KllTail{(unsigned long long)(uintptr_t)src, (unsigned long long)l.len, at};
                at += (unsigned long long)l.len;
            }
        }
        KL_HIP(ctx, hipMemcpyAsync(gdev, pin, seg_bytes + tab_bytes + mm_bytes, hipMemcpyHostToDevice, s));
        if (inplace) {
            // level 0's descriptors are the first NC * ncols groups (level-major): their row ranges, then the final
            // level-0 buffers of the columns read in place
            const size_t n0 = maxlev > 1 ? first[NC * ncols] : nseg_all;
            if (n0)
                hipLaunchKernelGGL(kll_locate_kernel, dim3((unsigned)((n0 + 255) / 256)), dim3(256), 0, s, dsegs, (int)n0,
                                   dtab, drows);
            if (!tail0.empty()) {
                KllTail0Job* dt0 = nullptr;
                KL_HIP(ctx, buf.alloc((void**)&dt0, tail0.size() * sizeof(KllTail0Job)));
                KL_HIP(ctx, hipMemcpyAsync(dt0, tail0.data(), tail0.size() * sizeof(KllTail0Job), hipMemcpyHostToDevice, s));
                hipLaunchKernelGGL(kll_tail0_kernel, dim3((unsigned)tail0.size()), dim3(256), 0, s, (const KllTail0Job*)dt0);
            }
            KL_HIP(ctx, hipGetLastError());
        }
        for (size_t h = 0; h < maxlev; ++h)
            for (size_t c = 0; c < NC; ++c) {
                size_t total = 0;
                for (int i = 0; i < ncols; ++i) total += cnt[(h * NC + c) * ncols + i];
                if (!total) continue;
                const size_t f = first[(h * NC + c) * ncols];
                if (launch_kll_compact((int)c, nullptr, dsegs + f, (int)total, nullptr, nullptr, s, (int)h, dtab + h * ncols,
                                       h == 0 && inplace ? drows + 2 * f : nullptr) != 0)
                    return dq::ctx_fail(ctx, DQ_ERR_DEVICE, "dq_kll_sketch: compaction launch failed");
            }
        for (int i = 0; i < ncols; ++i) {
            KColumnRun& r = run[i];
            const size_t nlev = r.sc.levels.size();
            KL_HIP(ctx, hipMemcpyAsync(dtails[i], pin + r.pin_at, nlev * sizeof(KllTail), hipMemcpyHostToDevice, s));
            if (r.ntail)
                hipLaunchKernelGGL(kll_gather_kernel, dim3((unsigned)nlev), dim3(256), 0, s, (const KllTail*)dtails[i], dgats[i]);
            KL_HIP(ctx, hipGetLastError());
            if (r.ntail)
                KL_HIP(ctx, hipMemcpyAsync(r.hgat, dgats[i], sizeof(double) * (size_t)r.ntail, hipMemcpyDeviceToHost, s));
            KL_HIP(ctx, hipMemcpyAsync(r.hgat + r.ntail, dmm + 2 * i, 16, hipMemcpyDeviceToHost, s));
        }
    } else {
        // pinned staging for every column: [segment descriptors][level tails][gathered final buffers + min / max keys]
        size_t pin_total = 0;
        for (KColumnRun& r : run) {
            const size_t nlev = r.sc.levels.size(), nseg = r.events.size();
            r.ntail = 0;
            for (const KllLevel& l : r.sc.levels) r.ntail += l.len;
            r.pin_at = pin_total;
            pin_total += (nseg * 8 + nlev * sizeof(KllTail) + (size_t)r.ntail * 8 + 16 + 255) / 256 * 256;
        }
        uint8_t* pin = static_cast<uint8_t*>(dq::ctx_pinned_buf(ctx, std::max<size_t>(pin_total, 16)));
        if (!pin) return DQ_ERR_OUT_OF_MEMORY;
        // every column's descriptors grouped per (level, kernel class) straight into its pinned region, on the host threads
        kll_parallel(ncols, [&](int i) {
            KColumnRun& r = run[i];
            const KllSchedule& sc = r.sc;
            const size_t nlev = sc.levels.size();
            uint64_t* hsegs = reinterpret_cast<uint64_t*>(pin + r.pin_at);
            size_t pos = 0;
            std::vector<size_t> cursor(nlev * kKllAllClasses);
            r.launches.clear();
            for (size_t h = 0; h < nlev; ++h) {
                const KllLevel& l = sc.levels[h];
                for (int c = 0; c < kKllAllClasses; ++c) {
                    cursor[h * kKllAllClasses + c] = pos;
                    if (l.per_class[c]) r.launches.push_back({h, pos, (size_t)l.per_class[c], c});
                    pos += (size_t)l.per_class[c];
                }
            }
            for (const uint64_t d : r.events)  // schedule order inside a group
                hsegs[cursor[(size_t)((d >> 55) & 0xFF) * kKllAllClasses + kll_class_of((int)((d >> 40) & 0x7FFF))]++] = d;
        });
        const unsigned long long mm_init[2] = {~0ull, 0ull};
        for (int ci = 0; ci < ncols; ++ci) {
            KColumnRun& r = run[ci];
            hipStream_t cs = cstreams[ci % nstreams];
            KllSchedule& sc = r.sc;
            const size_t nlev = sc.levels.size(), nseg_all = r.events.size();
            r.lbase.assign(nlev, 0);
            int64_t upper = 0;
            for (size_t h = 1; h < nlev; ++h) {
                r.lbase[h] = upper;
                upper += sc.levels[h].arrived;
            }
            // device: [upper levels' streams][segment descriptors][min / max][level tails][gathered final buffers]
            const size_t seg_off = ((size_t)upper * 8 + 255) / 256 * 256;
            const size_t mm_off = seg_off + (nseg_all * 8 + 255) / 256 * 256;
            const size_t tail_off = mm_off + 256;
            const size_t gat_off = tail_off + (nlev * sizeof(KllTail) + 255) / 256 * 256;
            uint8_t* scratch = nullptr;
            KL_HIP(ctx, buf.alloc((void**)&scratch, gat_off + (size_t)r.ntail * 8 + 256));
            double* dup = reinterpret_cast<double*>(scratch);
            uint64_t* dsegs = reinterpret_cast<uint64_t*>(scratch + seg_off);
            unsigned long long* dminmax = reinterpret_cast<unsigned long long*>(scratch + mm_off);
            KllTail* dtails = reinterpret_cast<KllTail*>(scratch + tail_off);
            double* dgat = reinterpret_cast<double*>(scratch + gat_off);
            uint64_t* hsegs = reinterpret_cast<uint64_t*>(pin + r.pin_at);
            KllTail* htails = reinterpret_cast<KllTail*>(pin + r.pin_at + nseg_all * 8);
            r.hgat = reinterpret_cast<double*>(pin + r.pin_at + nseg_all * 8 + nlev * sizeof(KllTail));

            // one launch per (level, kernel class) group; the order inside a level is free because every compaction's
            // input range and output slot are explicit
            if (nseg_all) KL_HIP(ctx, hipMemcpyAsync(dsegs, hsegs, nseg_all * 8, hipMemcpyHostToDevice, cs));
            KL_HIP(ctx, hipMemcpyAsync(dminmax, mm_init, sizeof(mm_init), hipMemcpyHostToDevice, cs));
            for (const KColumnRun::Launch& L : r.launches) {  // a level that compacted always has a level above it
                const size_t h = L.level;
                const double* src = h == 0 ? r.stream0 : dup + r.lbase[h];
                double* dst = dup + r.lbase[h + 1];
                if (launch_kll_compact(L.cls, src, dsegs + L.first, (int)L.count, dst, h == 0 ? dminmax : nullptr, cs, (int)h) != 0)
                    return dq::ctx_fail(ctx, DQ_ERR_DEVICE, "dq_kll_sketch: compaction launch failed");
            }
            // final buffers: one gather, one read-back (completed by the single synchronisation below)
            unsigned long long at = 0;
            for (size_t h = 0; h < nlev; ++h) {
                const KllLevel& l = sc.levels[h];
                const double* src = (h == 0 ? r.stream0 : dup + r.lbase[h]) + l.pos;
                htails[h] = KllTail{(unsigned long long)(uintptr_t)src, (unsigned long long)l.len, at};
                at += (unsigned long long)l.len;
            }
            KL_HIP(ctx, hipMemcpyAsync(dtails, htails, nlev * sizeof(KllTail), hipMemcpyHostToDevice, cs));
            if (r.ntail) hipLaunchKernelGGL(kll_gather_kernel, dim3((unsigned)nlev), dim3(256), 0, cs, (const KllTail*)dtails, dgat);
            KL_HIP(ctx, hipGetLastError());
            if (r.ntail) KL_HIP(ctx, hipMemcpyAsync(r.hgat, dgat, sizeof(double) * (size_t)r.ntail, hipMemcpyDeviceToHost, cs));
            KL_HIP(ctx, hipMemcpyAsync(r.hgat + r.ntail, dminmax, 16, hipMemcpyDeviceToHost, cs));
        }
    }
    for (int j = 1; j < nstreams; ++j) {
        KL_HIP(ctx, hipEventRecord(join_ev[j - 1], cstreams[j]));
        KL_HIP(ctx, hipStreamWaitEvent(s, join_ev[j - 1], 0));
    }
    const auto t2 = std::chrono::steady_clock::now();
    KL_HIP(ctx, hipStreamSynchronize(s));
    if (getenv("DQ_KLL_TIMING")) {
        auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
            return std::chrono::duration<double, std::milli>(b - a).count();
        };
        size_t nseg = 0;
        for (const KColumnRun& r : run) nseg += r.events.size();
        fprintf(stderr, "[dq_kll_sketch] columns=%d rows=%lld compactions=%zu counts %.2f ms, schedules %.2f ms, "
                "staging+launch %.2f ms, device %.2f ms\n", ncols, (long long)nrows, nseg, ms(t0, t0b), ms(t0b, t1),
                ms(t1, t2), ms(t2, std::chrono::steady_clock::now()));
    }

    for (int i = 0; i < ncols; ++i) {
        const KColumnRun& r = run[i];
        const KllSchedule& sc = r.sc;
        const size_t nlev = sc.levels.size();
        std::vector<std::vector<double>> fin(nlev);
        int64_t at = 0;
        for (size_t h = 0; h < nlev; ++h) {
            fin[h].assign(r.hgat + at, r.hgat + at + sc.levels[h].len);
            at += sc.levels[h].len;
        }
        unsigned long long mm[2];
        memcpy(mm, r.hgat + r.ntail, sizeof(mm));
        // UntypedQuantileNonSample.updateUntyped: math.min / math.max folds from Int.MaxValue.toDouble /
        // Int.MinValue.toDouble (java.lang.Math: NaN-propagating, -0.0 < 0.0) = the order-key extremes
        // of every item, NaN if any item is NaN.
        uint64_t kmin = mm[0], kmax = mm[1];
        for (double d : fin[0]) {
            kmin = std::min<uint64_t>(kmin, host_key(d));
            kmax = std::max<uint64_t>(kmax, host_key(d));
        }
        double vmin = 2147483647.0, vmax = -2147483648.0;
        if (r.n > 0) {
            const double lo = host_value(kmin), hi = host_value(kmax);
            if (hi != hi) {
                vmin = vmax = NAN;
            } else {
                vmin = host_key(lo) < host_key(vmin) ? lo : vmin;
                vmax = host_key(hi) > host_key(vmax) ? hi : vmax;
            }
        }
        // ---- KLLState bytes (big-endian ByteBuffer) -----------------------------------------------
        std::vector<uint8_t>& o = states[i];
        put_f64(o, vmin);
        put_f64(o, vmax);
        put_be32(o, sketch_size);
        put_f64(o, shrinking_factor);
        put_be32(o, (int32_t)nlev);              // curNumOfCompactors
        put_be32(o, (int32_t)sc.actual);         // compactorActualSize
        put_be32(o, (int32_t)sc.total);          // compactorTotalSize
        put_be32(o, (int32_t)nlev);              // compactors.length
        for (size_t h = 0; h < nlev; ++h) {
            put_be32(o, sc.levels[h].ncomp);
            put_be32(o, sc.levels[h].offset);
            put_be32(o, (int32_t)fin[h].size());
            for (double d : fin[h]) put_f64(o, d);
        }
    }
    return DQ_OK;
}

}  // extern "C"
