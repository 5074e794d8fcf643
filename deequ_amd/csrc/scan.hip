// scan.hip — the fused scan of all scan-shareable analyzers (gfx950 / CDNA4).
//
// Replaces the single Spark aggregation `data.agg(aggregations...).collect()` issued by
// runScanningAnalyzers (R/AnalysisRunner.scala:289-336). Each op's Spark aggregate is restated in
// SURVEY.md §8a; the per-row semantics implemented here:
//   Size / Completeness / Compliance  A/Size.scala:33-47, A/Completeness.scala:38-41,
//                                     A/Compliance.scala:49-52, where: A/Analyzer.scala:409-432
//   Mean / Sum                        A/Mean.scala:36-40, A/Sum.scala:34-37 (Long sum for integral)
//   Minimum / Maximum                 A/Minimum.scala:34-37, A/Maximum.scala:34-37
//   StandardDeviation                 C/StatefulStdDevPop.scala:24-34 + merge A/StandardDeviation.scala:37-44
//   Correlation                       C/StatefulCorrelation.scala:24-49 + merge A/Correlation.scala:37-52
//   ApproxCountDistinct               C/StatefulHyperloglogPlus.scala:89-112 (XXH64 seed 42, P = 9)
//
// Layout: rows are split into contiguous per-workgroup ranges (multiples of a 2048-row tile).
// Inside a tile each of the 256 lanes owns 8 rows: L = 8/P coalesced loads of P rows
// (P = 16 B / element size: one global_load_dwordx4 per load for 4/8-byte types). The validity
// and `where` bits of those rows come from 64-bit bitmap words (2 distinct words per wave per
// load). Per-lane states are folded per 8-row batch (batch mean + Chan merge: one division per
// batch, not per row), reduced wave64 -> workgroup through shuffles and a 4-entry LDS array, and
// written as one SlotPartial per workgroup. A second launch folds the workgroup partials in a
// fixed order (results are bitwise reproducible run to run). No fp atomics are used.
// HLL registers live in LDS (512 x u32 per column) and are max-merged per workgroup.
#include <hip/hip_runtime.h>

#include <math.h>

#include "dq_common.h"
#include "dq_internal.h"

namespace dq {

// Cache policy of the striped column loads (buffer aux: bit 1 = nt on gfx950): once-read streams, measured
// 2-3 % faster on C2 (profiles/r02/c2_policy_r02ap.log). The lane-owned 64-B runs of scan_heavy8_kernel keep the
// default policy: their four 16-B loads per line rely on the line staying cached (nt made them 1.5x slower).
#ifndef DQ_SCAN_AUX
#define DQ_SCAN_AUX 2
#endif

__device__ __forceinline__ double as_f64(uint64_t u) { return __longlong_as_double((long long)u); }
__device__ __forceinline__ uint64_t f64_bits(double d) { return (uint64_t)__double_as_longlong(d); }

__device__ __forceinline__ uint64_t shfl_down_u64(uint64_t x, int off) {
    int lo = (int)(uint32_t)x, hi = (int)(uint32_t)(x >> 32);
    lo = __shfl_down(lo, off, 64);
    hi = __shfl_down(hi, off, 64);
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
__device__ __forceinline__ int64_t shfl_down_i64(int64_t x, int off) {
    return (int64_t)shfl_down_u64((uint64_t)x, off);
}
__device__ __forceinline__ double shfl_down_f64(double x, int off) {
    return as_f64(shfl_down_u64(f64_bits(x), off));
}

// ------------------------------------------------------------------------------------------------
// Partial-state algebra (the reference's State.sum for each state, applied to lane/workgroup partials)
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void col_init(ColPartial& a) {
    a.n = 0;
    a.nnan = 0;
    a.isum = 0;
    a.imin = INT64_MAX;
    a.imax = INT64_MIN;
    a.dsum = 0.0;
    a.dmin = INFINITY;
    a.dmax = -INFINITY;
    a.mean = 0.0;
    a.m2 = 0.0;
    a.pt = 0;
    a.pad = 0;
}

// StandardDeviationState.sum (A/StandardDeviation.scala:37-44) with an explicit empty side.
__device__ __forceinline__ void moments_merge(int64_t na, double& mean, double& m2, int64_t nb,
                                              double meanb, double m2b) {
    if (nb == 0) return;
    if (na == 0) {
        mean = meanb;
        m2 = m2b;
        return;
    }
    const double n1 = (double)na, n2 = (double)nb;
    const double newN = n1 + n2;
    const double delta = meanb - mean;
    const double deltaN = delta / newN;
    mean = mean + deltaN * n2;
    m2 = m2 + m2b + delta * deltaN * n1 * n2;
}

// Batch-path reciprocal: v_rcp_f64 plus two Newton steps (within 1 ulp) for 1/cnt and 1/n, since
// the per-8-row fold would otherwise spend two full IEEE divisions (div_scale/rcp/fma/div_fmas/
// div_fixup) per batch per column. The moments stay within the 1e-12 relative bound of the Spark per-row Welford order either way.
__device__ __forceinline__ double rcp_refined(double d) {
    double r = __builtin_amdgcn_rcp(d);
    double e = __builtin_fma(-d, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-d, r, 1.0);
    return __builtin_fma(r, e, r);
}

// moments_merge for the per-lane batch fold (nb >= 1 guaranteed by the caller).
__device__ __forceinline__ void moments_merge_batch(int64_t na, double& mean, double& m2, int nb,
                                                    double meanb, double m2b) {
    if (na == 0) {
        mean = meanb;
        m2 = m2b;
        return;
    }
    const double n1 = (double)na, n2 = (double)nb;
    const double newN = n1 + n2;
    const double delta = meanb - mean;
    const double deltaN = delta * rcp_refined(newN);
    mean = mean + deltaN * n2;
    m2 = m2 + m2b + delta * deltaN * n1 * n2;
}

__device__ __forceinline__ void col_merge(ColPartial& a, const ColPartial& b) {
    moments_merge(a.n, a.mean, a.m2, b.n, b.mean, b.m2);
    a.n += b.n;
    a.nnan += b.nnan;
    a.pt += b.pt;
    a.isum = (int64_t)((uint64_t)a.isum + (uint64_t)b.isum);
    a.imin = b.imin < a.imin ? b.imin : a.imin;
    a.imax = b.imax > a.imax ? b.imax : a.imax;
    a.dsum += b.dsum;
    a.dmin = fmin(a.dmin, b.dmin);
    a.dmax = fmax(a.dmax, b.dmax);
}

// CorrelationState.sum (A/Correlation.scala:37-52) with an explicit empty side.
__device__ __forceinline__ void corr_merge(CorrPartial& a, const CorrPartial& b) {
    if (b.n == 0.0) return;
    if (a.n == 0.0) {
        a = b;
        return;
    }
    const double n1 = a.n, n2 = b.n;
    const double newN = n1 + n2;
    const double dx = b.xa - a.xa;
    const double dxN = dx / newN;
    const double dy = b.ya - a.ya;
    const double dyN = dy / newN;
    a.xa = a.xa + dxN * n2;
    a.ya = a.ya + dyN * n2;
    a.ck = a.ck + b.ck + dx * dyN * n1 * n2;
    a.xm = a.xm + b.xm + dx * dxN * n1 * n2;
    a.ym = a.ym + b.ym + dy * dyN * n1 * n2;
    a.n = newN;
}

// corr_merge for the per-lane batch fold (b.n >= 1): one refined reciprocal of the new count replaces the two
// divisions (the batch folds run once per 8 rows per lane; the cross-lane folds keep corr_merge).
__device__ __forceinline__ void corr_merge_batch(CorrPartial& a, const CorrPartial& b) {
    if (a.n == 0.0) {
        a = b;
        return;
    }
    const double n1 = a.n, n2 = b.n;
    const double newN = n1 + n2;
    const double rn = rcp_refined(newN);
    const double dx = b.xa - a.xa;
    const double dxN = dx * rn;
    const double dy = b.ya - a.ya;
    const double dyN = dy * rn;
    a.xa = a.xa + dxN * n2;
    a.ya = a.ya + dyN * n2;
    a.ck = a.ck + b.ck + dx * dyN * n1 * n2;
    a.xm = a.xm + b.xm + dx * dxN * n1 * n2;
    a.ym = a.ym + b.ym + dy * dyN * n1 * n2;
    a.n = newN;
}

__device__ __forceinline__ void slot_init(SlotPartial& p) {
    col_init(p.c[0]);
    col_init(p.c[1]);
    p.corr.n = p.corr.xa = p.corr.ya = p.corr.ck = p.corr.xm = p.corr.ym = 0.0;
    p.wt = p.wnn = p.pt = p.pnn = p.vt = p.pad = 0;
}

__device__ __forceinline__ void slot_merge(SlotPartial& a, const SlotPartial& b) {
    col_merge(a.c[0], b.c[0]);
    col_merge(a.c[1], b.c[1]);
    corr_merge(a.corr, b.corr);
    a.wt += b.wt;
    a.wnn += b.wnn;
    a.pt += b.pt;
    a.pnn += b.pnn;
    a.vt += b.vt;
}

__device__ __forceinline__ void col_shfl(ColPartial& o, const ColPartial& a, int off) {
    o.n = shfl_down_i64(a.n, off);
    o.nnan = shfl_down_i64(a.nnan, off);
    o.isum = shfl_down_i64(a.isum, off);
    o.imin = shfl_down_i64(a.imin, off);
    o.imax = shfl_down_i64(a.imax, off);
    o.dsum = shfl_down_f64(a.dsum, off);
    o.dmin = shfl_down_f64(a.dmin, off);
    o.dmax = shfl_down_f64(a.dmax, off);
    o.mean = shfl_down_f64(a.mean, off);
    o.m2 = shfl_down_f64(a.m2, off);
    o.pt = shfl_down_i64(a.pt, off);
    o.pad = 0;
}

__device__ __forceinline__ void slot_shfl(SlotPartial& o, const SlotPartial& a, int off, int ncols,
                                          bool corr) {
    col_shfl(o.c[0], a.c[0], off);
    if (ncols > 1) col_shfl(o.c[1], a.c[1], off);
    else col_init(o.c[1]);
    if (corr) {
        o.corr.n = shfl_down_f64(a.corr.n, off);
        o.corr.xa = shfl_down_f64(a.corr.xa, off);
        o.corr.ya = shfl_down_f64(a.corr.ya, off);
        o.corr.ck = shfl_down_f64(a.corr.ck, off);
        o.corr.xm = shfl_down_f64(a.corr.xm, off);
        o.corr.ym = shfl_down_f64(a.corr.ym, off);
    } else {
        o.corr.n = o.corr.xa = o.corr.ya = o.corr.ck = o.corr.xm = o.corr.ym = 0.0;
    }
    o.wt = shfl_down_i64(a.wt, off);
    o.wnn = shfl_down_i64(a.wnn, off);
    o.pt = shfl_down_i64(a.pt, off);
    o.pnn = shfl_down_i64(a.pnn, off);
    o.vt = shfl_down_i64(a.vt, off);
    o.pad = 0;
}

// wave64 tree (fixed order) -> 4 wave results in LDS -> lane 0 of wave 0 folds them in order.
__device__ void block_reduce_slot(SlotPartial& acc, SlotPartial* lds4, int ncols, bool corr) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
#pragma unroll 1
    for (int off = 32; off > 0; off >>= 1) {
        SlotPartial other;
        slot_shfl(other, acc, off, ncols, corr);
        if (lane < off) slot_merge(acc, other);
    }
    if (lane == 0) lds4[wave] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kBlock / 64; ++w) slot_merge(acc, lds4[w]);
    }
    __syncthreads();
}

// ------------------------------------------------------------------------------------------------
// Tile loaders. Row of (load j, element k) for lane `tid`: tile + j * 256 * P + tid * P + k.
// ------------------------------------------------------------------------------------------------
template <int P>
__device__ __forceinline__ int64_t row_of(int64_t tile, int tid, int j, int k) {
    return tile + (int64_t)j * (kBlock * P) + (int64_t)tid * P + k;
}

typedef int v4i_t __attribute__((ext_vector_type(4)));
typedef int v2i_t __attribute__((ext_vector_type(2)));

// Buffer descriptor over one tile's bytes (T8/T20: 32-bit per-lane voffset, wave-uniform base
// built from the slot descriptor and the tile index only, so it lives in SGPRs).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(const void* base, int64_t byte_off, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)base + byte_off), (short)0, bytes, 0x00020000);
}

// Bits of a padded bitmap (predicate outputs: always readable up to the tile end).
// SCALAR: a wave's rows of load j span P consecutive bitmap words at a wave-uniform address, read by scalar loads
// (read-only, constant address space) instead of 64-lane vector loads of mostly the same word; each lane then picks
// its word and bits. Used for the `where` bitmaps: with where + validity both on vector loads the where scan ran at
// 8.0 vs 5.25 ms per int64 launch, with both scalar C2 (validity only) lost 0.6 ms (profiles/r02/where_bits_r02bt.log).
template <int P, bool SCALAR = false>
__device__ __forceinline__ uint32_t bits_padded(const uint64_t* __restrict__ bm, int64_t tile, int tid) {
    constexpr int L = 8 / P;
    constexpr uint32_t pm = (1u << P) - 1u;
    if constexpr (SCALAR) {
    typedef const __attribute__((address_space(4))) uint64_t* cptr;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    const cptr base = (cptr)(bm + (tile >> 6)) + wv * P;
    uint32_t m = 0;
#pragma unroll
    for (int j = 0; j < L; ++j) {
        const cptr q = base + j * (kBlock * P / 64);
        // readfirstlane keeps the words uniform: without it the select below folds into one divergent-address load
        auto uword = [&](int i) {
            const uint64_t v = q[i];
            return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32) |
                   (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
        };
        uint64_t word = uword(0);
#pragma unroll
        for (int i = 1; i < P; ++i) {
            const uint64_t wi = uword(i);
            word = ((lane * P) >> 6) == i ? wi : word;
        }
        m |= (uint32_t)((word >> ((lane * P) & 63)) & pm) << (j * P);
    }
    return m;
    }
    const __amdgpu_buffer_rsrc_t r = tile_rsrc(bm, tile >> 3, kTileRows / 8);
    uint32_t m = 0;
#pragma unroll
    for (int j = 0; j < L; ++j) {
        // row0 = tile + j * 256 * P + tid * P; its 64-bit word inside the tile and bit offset:
        const int rel = j * (kBlock * P) + tid * P;
        const v2i_t w = __builtin_amdgcn_raw_buffer_load_b64(r, (rel >> 6) * 8, 0, DQ_SCAN_AUX);
        const uint64_t word = ((uint64_t)(uint32_t)w.y << 32) | (uint32_t)w.x;
        m |= (uint32_t)((word >> (rel & 63)) & pm) << (j * P);
    }
    return m;
}

// Rows of this lane that exist (tail tile).
template <int P>
__device__ __forceinline__ uint32_t in_range_mask(int64_t tile, int tid, int64_t nrows) {
    constexpr int L = 8 / P;
    uint32_t m = 0;
#pragma unroll
    for (int j = 0; j < L; ++j)
#pragma unroll
        for (int k = 0; k < P; ++k)
            if (row_of<P>(tile, tid, j, k) < nrows) m |= 1u << (j * P + k);
    return m;
}

// Validity bits of a user bitmap (exactly ceil(nrows/8) bytes long: bounded in the tail tile).
template <int P>
__device__ __forceinline__ uint32_t bits_valid(const uint64_t* __restrict__ bm, int64_t tile, int tid,
                                               bool full, int64_t nrows) {
    if (bm == nullptr) return full ? 0xFFu : in_range_mask<P>(tile, tid, nrows);
    if (full) return bits_padded<P>(bm, tile, tid);
    const uint8_t* b = reinterpret_cast<const uint8_t*>(bm);
    constexpr int L = 8 / P;
    uint32_t m = 0;
#pragma unroll
    for (int j = 0; j < L; ++j)
#pragma unroll
        for (int k = 0; k < P; ++k) {
            const int64_t r = row_of<P>(tile, tid, j, k);
            if (r < nrows && ((b[r >> 3] >> (r & 7)) & 1)) m |= 1u << (j * P + k);
        }
    return m;
}

// Loads the lane's 8 values in canonical form: int64 for integral storage, double bits for
// FLOAT/DOUBLE. Missing rows (tail) load 0 and are masked off by the caller.
__device__ __forceinline__ uint64_t pack64(int lo, int hi) { return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo; }

template <int P, bool F>
__device__ __forceinline__ void load_values(const ColDesc& c, int64_t tile, int tid, bool full,
                                            int64_t nrows, uint64_t (&v)[8]) {
    constexpr int L = 8 / P;
    // Only the element types a (P, F) kernel can be planned for are compiled into it.
    int e = c.elem;
    if (P == 2) e = F ? ET_F64 : ET_I64;
    if (P == 4) e = F ? ET_F32 : ET_I32;
    if (P == 8 && F && e != ET_F32) e = ET_F64;
    if (full) {
        // One descriptor per tile; lane byte offsets: striped (P = 16 B / elem) or 8 contiguous rows.
        const int esz = (e == ET_F64 || e == ET_I64) ? 8 : (e == ET_F32 || e == ET_I32) ? 4 : (e == ET_I16 ? 2 : 1);
        const __amdgpu_buffer_rsrc_t r = tile_rsrc(c.values, tile * esz, kTileRows * esz);
        if (esz == 8) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                // P == 2: load i covers rows i*512 + 2*tid (+0, +1); P == 8: rows 8*tid + 2i (+0, +1)
                const int voff = P == 8 ? tid * 64 + i * 16 : tid * 16;
                const int soff = P == 8 ? 0 : i * 4096;
                const v4i_t x = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, DQ_SCAN_AUX);
                v[2 * i] = pack64(x.x, x.y);
                v[2 * i + 1] = pack64(x.z, x.w);
            }
            return;
        }
        if (esz == 4) {
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int voff = P == 8 ? tid * 32 + i * 16 : tid * 16;
                const int soff = P == 8 ? 0 : i * 4096;
                const v4i_t x = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, DQ_SCAN_AUX);
                const int xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (e == ET_F32) v[4 * i + k] = f64_bits((double)__int_as_float(xs[k]));
                    else v[4 * i + k] = (uint64_t)(int64_t)xs[k];
                }
            }
            return;
        }
        if (esz == 2) {
            const v4i_t x = __builtin_amdgcn_raw_buffer_load_b128(r, tid * 16, 0, DQ_SCAN_AUX);
            const uint32_t w[4] = {(uint32_t)x.x, (uint32_t)x.y, (uint32_t)x.z, (uint32_t)x.w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                v[2 * i] = (uint64_t)(int64_t)(int16_t)(w[i] & 0xFFFFu);
                v[2 * i + 1] = (uint64_t)(int64_t)(int16_t)(w[i] >> 16);
            }
            return;
        }
        const v2i_t x = __builtin_amdgcn_raw_buffer_load_b64(r, tid * 8, 0, DQ_SCAN_AUX);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t b = ((uint32_t)(i < 4 ? x.x : x.y) >> (8 * (i & 3))) & 0xFFu;
            v[i] = e == ET_I8 ? (uint64_t)(int64_t)(int8_t)b : (uint64_t)b;
        }
        return;
    }
    // Tail tile: bounded element loads.
#pragma unroll
    for (int j = 0; j < L; ++j)
#pragma unroll
        for (int k = 0; k < P; ++k) {
            const int64_t r = row_of<P>(tile, tid, j, k);
            const bool in = r < nrows;
            uint64_t x = 0;
            switch (e) {
                case ET_F64:
                case ET_I64: x = in ? static_cast<const uint64_t*>(c.values)[r] : 0; break;
                case ET_F32: x = f64_bits(in ? (double)static_cast<const float*>(c.values)[r] : 0.0); break;
                case ET_I32: x = (uint64_t)(int64_t)(in ? static_cast<const int32_t*>(c.values)[r] : 0); break;
                case ET_I16: x = (uint64_t)(int64_t)(in ? static_cast<const int16_t*>(c.values)[r] : 0); break;
                case ET_I8: x = (uint64_t)(int64_t)(in ? static_cast<const int8_t*>(c.values)[r] : 0); break;
                default: x = in ? static_cast<const uint8_t*>(c.values)[r] : 0; break;
            }
            v[j * P + k] = x;
        }
}

__device__ __forceinline__ bool is_float_elem(int e) { return e == ET_F32 || e == ET_F64; }

__device__ __forceinline__ double to_double(uint64_t v, bool is_float) {
    return is_float ? as_f64(v) : (double)(int64_t)v;
}

// Spark XxHash64Function.hash(value, dataType, 42) for the canonical lane value.
__device__ __forceinline__ uint64_t spark_hash(uint64_t v, int spark_type) {
    switch (spark_type) {
        case DQ_TYPE_BOOLEAN:
        case DQ_TYPE_BYTE:
        case DQ_TYPE_SHORT:
        case DQ_TYPE_INT:
        case DQ_TYPE_DATE:
            return xxh_int((uint32_t)(int32_t)(int64_t)v, SPARK_HLL_SEED);
        case DQ_TYPE_FLOAT:
            return xxh_int(float_to_int_bits((float)as_f64(v)), SPARK_HLL_SEED);
        case DQ_TYPE_DOUBLE:
            return xxh_long(double_to_long_bits(as_f64(v)), SPARK_HLL_SEED);
        default:  // LONG, TIMESTAMP, DECIMAL(p <= 18): hashLong of the (unscaled) long
            return xxh_long(v, SPARK_HLL_SEED);
    }
}

// Lane-level helpers shared by the striped and the lean kernels (see scan_heavy8_kernel).
// bit k of m as 0 / 0xFFFFFFFF: one v_bfe_i32 (the shift pair it equals is sometimes left as two instructions)
__device__ __forceinline__ uint32_t row_mask(uint32_t m, int k) { return (uint32_t)__builtin_amdgcn_sbfe((int)m, k, 1); }
__device__ __forceinline__ double pack_f64(uint32_t hi, uint32_t lo) { return as_f64(((uint64_t)hi << 32) | lo); }
__device__ __forceinline__ uint32_t hi32(double d) { return (uint32_t)(f64_bits(d) >> 32); }
__device__ __forceinline__ uint32_t lo32(double d) { return (uint32_t)f64_bits(d); }
__device__ __forceinline__ double and_f64(double d, uint32_t mk) { return pack_f64(hi32(d) & mk, lo32(d) & mk); }
// v_min_f64 / v_max_f64 without the compiler's canonicalising v_max_f64 x, x of each operand: a NaN operand is
// dropped (a signalling NaN can make the result NaN; batches with NaN rows take the exact path).
__device__ __forceinline__ double raw_min(double a, double b) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double raw_max(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ uint32_t ffbh_raw(uint32_t x) {  // leading zeros, 0xFFFFFFFF for 0
    uint32_t r;
    asm("v_ffbh_u32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}
// (double)(int64_t)v correctly rounded in 3 instructions (hi * 2^32 is exact; one rounding in the fma)
__device__ __forceinline__ double i64_to_f64(uint64_t v) {
    return __builtin_fma((double)(int32_t)(uint32_t)(v >> 32), 4294967296.0, (double)(uint32_t)v);
}
__device__ __forceinline__ double one_if(uint32_t mk) { return pack_f64(mk & 0x3FF00000u, 0u); }
// x * {1.0, 0.0} as one v_mul_f64: left to itself the compiler turns the multiply by one_if() into two v_and_b32
// of the halves (finite x only, which is all the callers pass)
__device__ __forceinline__ double mul_raw(double a, double b) {
    double r;
    asm("v_mul_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// ------------------------------------------------------------------------------------------------
// Per-lane accumulators, specialised by storage class so only live state occupies VGPRs.
// ------------------------------------------------------------------------------------------------
struct FAcc {  // FLOAT / DOUBLE column
    int64_t n, nnan, pt;
    double sum, mn, mx, mean, m2;
};
struct IAcc {  // integral column (Long sum with wrap-around, integer min/max)
    int64_t n, sum, mn, mx, pt;
    double mean, m2;
    double dmn, dmx;  // striped kernel: extremes of batches whose values are all exact doubles (|x| < 2^53)
};
template <bool F> struct AccOf { using type = IAcc; };
template <> struct AccOf<true> { using type = FAcc; };

__device__ __forceinline__ void acc_init(FAcc& a) {
    a.n = a.nnan = a.pt = 0;
    a.sum = 0.0;
    a.mn = INFINITY;
    a.mx = -INFINITY;
    a.mean = a.m2 = 0.0;
}
__device__ __forceinline__ void acc_init(IAcc& a) {
    a.n = a.sum = a.pt = 0;
    a.mn = INT64_MAX;
    a.mx = INT64_MIN;
    a.mean = a.m2 = 0.0;
    a.dmn = a.dmx = __builtin_nan("");
}
// Folds the double-tracked extremes into the int64 ones before the cross-lane reduction (exact: |x| < 2^53).
__device__ __forceinline__ void acc_finish(FAcc&) {}
__device__ __forceinline__ void acc_finish(IAcc& a) {
    if (a.dmn == a.dmn && (int64_t)a.dmn < a.mn) a.mn = (int64_t)a.dmn;
    if (a.dmx == a.dmx && (int64_t)a.dmx > a.mx) a.mx = (int64_t)a.dmx;
    a.dmn = a.dmx = __builtin_nan("");
}

__device__ __forceinline__ void acc_merge(FAcc& a, const FAcc& b) {
    moments_merge(a.n, a.mean, a.m2, b.n, b.mean, b.m2);
    a.n += b.n;
    a.nnan += b.nnan;
    a.pt += b.pt;
    a.sum += b.sum;
    a.mn = fmin(a.mn, b.mn);
    a.mx = fmax(a.mx, b.mx);
}
__device__ __forceinline__ void acc_merge(IAcc& a, const IAcc& b) {
    moments_merge(a.n, a.mean, a.m2, b.n, b.mean, b.m2);
    a.n += b.n;
    a.pt += b.pt;
    a.sum = (int64_t)((uint64_t)a.sum + (uint64_t)b.sum);
    a.mn = b.mn < a.mn ? b.mn : a.mn;
    a.mx = b.mx > a.mx ? b.mx : a.mx;
}

__device__ __forceinline__ void acc_shfl(FAcc& o, const FAcc& a, int off) {
    o.n = shfl_down_i64(a.n, off);
    o.nnan = shfl_down_i64(a.nnan, off);
    o.pt = shfl_down_i64(a.pt, off);
    o.sum = shfl_down_f64(a.sum, off);
    o.mn = shfl_down_f64(a.mn, off);
    o.mx = shfl_down_f64(a.mx, off);
    o.mean = shfl_down_f64(a.mean, off);
    o.m2 = shfl_down_f64(a.m2, off);
}
__device__ __forceinline__ void acc_shfl(IAcc& o, const IAcc& a, int off) {
    o.n = shfl_down_i64(a.n, off);
    o.sum = shfl_down_i64(a.sum, off);
    o.pt = shfl_down_i64(a.pt, off);
    o.mn = shfl_down_i64(a.mn, off);
    o.mx = shfl_down_i64(a.mx, off);
    o.mean = shfl_down_f64(a.mean, off);
    o.m2 = shfl_down_f64(a.m2, off);
}
__device__ __forceinline__ void corr_shfl(CorrPartial& o, const CorrPartial& a, int off) {
    o.n = shfl_down_f64(a.n, off);
    o.xa = shfl_down_f64(a.xa, off);
    o.ya = shfl_down_f64(a.ya, off);
    o.ck = shfl_down_f64(a.ck, off);
    o.xm = shfl_down_f64(a.xm, off);
    o.ym = shfl_down_f64(a.ym, off);
}

__device__ __forceinline__ void store_empty(ColPartial& p) {
    p.n = p.nnan = p.isum = 0;
    p.imin = INT64_MAX;
    p.imax = INT64_MIN;
    p.dsum = 0.0;
    p.dmin = INFINITY;
    p.dmax = -INFINITY;
    p.mean = p.m2 = 0.0;
    p.pt = p.pad = 0;
}
__device__ __forceinline__ void store_partial(ColPartial& p, const FAcc& a) {
    store_empty(p);
    p.pt = a.pt;
    p.n = a.n;
    p.nnan = a.nnan;
    p.dsum = a.sum;
    p.dmin = a.mn;
    p.dmax = a.mx;
    p.mean = a.mean;
    p.m2 = a.m2;
}
__device__ __forceinline__ void store_partial(ColPartial& p, const IAcc& a) {
    store_empty(p);
    p.pt = a.pt;
    p.n = a.n;
    p.isum = a.sum;
    p.imin = a.mn;
    p.imax = a.mx;
    p.mean = a.mean;
    p.m2 = a.m2;
}
__device__ __forceinline__ void to_partial(ColPartial& p, const FAcc& a) {
    col_init(p);
    p.n = a.n;
    p.nnan = a.nnan;
    p.dsum = a.sum;
    p.dmin = a.mn;
    p.dmax = a.mx;
    p.mean = a.mean;
    p.m2 = a.m2;
}
__device__ __forceinline__ void to_partial(ColPartial& p, const IAcc& a) {
    col_init(p);
    p.n = a.n;
    p.isum = a.sum;
    p.imin = a.mn;
    p.imax = a.mx;
    p.mean = a.mean;
    p.m2 = a.m2;
}

// Per-lane fold of one 8-row batch (Spark's per-row updates restated as a batch + Chan merge).
// Masked rows are sanitised once: to 0.0 for the sum and the moments, to NaN for min / max (v_min_f64 /
// v_max_f64 return the non-NaN operand, so a NaN stand-in drops out exactly like a skipped row; the two
// stand-ins share their low word). NaN values that are valid rows make the batch sum NaN, so they are
// counted only in that (rare, divergent) case: Spark orders NaN above every double, which the finaliser
// applies through nnan (max = NaN if nnan > 0, min = NaN if nnan == n). An inf - inf batch sum also lands
// in that branch and counts zero NaNs.
// 1.0 for a kept row of the batch mask, 0.0 otherwise (the low word of both is 0: one 32-bit select).
__device__ __forceinline__ double on_factor(uint32_t m, int k) {
    return as_f64((uint64_t)(((m >> k) & 1u) ? 0x3FF00000u : 0u) << 32);
}

__device__ __forceinline__ void accumulate(FAcc& a, const uint64_t (&v)[8], uint32_t m, uint32_t flags) {
    const int cnt = __popc(m);
    if (cnt == 0) return;
    if (flags & (CF_STATS | CF_MOMENTS)) {
        double xz[8];
        double s = 0.0, mn = __builtin_nan(""), mx = __builtin_nan("");
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const bool on = (m >> k) & 1u;
            const uint32_t lo = on ? (uint32_t)v[k] : 0u;
            const uint32_t hz = on ? (uint32_t)(v[k] >> 32) : 0u;
            const uint32_t hn = on ? (uint32_t)(v[k] >> 32) : 0x7FF80000u;
            xz[k] = as_f64(((uint64_t)hz << 32) | lo);
            const double xn = as_f64(((uint64_t)hn << 32) | lo);
            s += xz[k];
            mn = fmin(mn, xn);
            mx = fmax(mx, xn);
        }
        if (s != s) {  // a NaN among the valid rows (or inf - inf): count the NaNs exactly
            int nn = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) nn += (((m >> k) & 1u) && as_f64(v[k]) != as_f64(v[k])) ? 1 : 0;
            a.nnan += nn;
        }
        a.sum += s;
        a.mn = fmin(a.mn, mn);
        a.mx = fmax(a.mx, mx);
        if (flags & CF_MOMENTS) {
            const double mb = s * rcp_refined((double)cnt);
            double m2b = 0.0;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                // (x - mean) * {1.0, 0.0}: one 32-bit select builds the factor, exact for the kept rows
                const double d = (xz[k] - mb) * on_factor(m, k);
                m2b = __builtin_fma(d, d, m2b);
            }
            moments_merge_batch(a.n, a.mean, a.m2, cnt, mb, m2b);
        }
    }
    a.n += cnt;
}

// Integral batch: each value converted to double once (3 instructions, exact while |x| < 2^53) for the moments and
// the min / max (raw v_min / v_max over NaN stand-ins; a batch holding a larger magnitude takes the exact int64
// compares instead), the Long sum over bit-cleared values.
template <bool S, bool M>
__device__ __forceinline__ void accumulate_int(IAcc& a, const uint64_t (&v)[8], uint32_t m, int cnt) {
    double xd[8];
    uint64_t bs = 0;
    double mn = __builtin_nan(""), mx = __builtin_nan("");
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t mk = row_mask(m, k);
        xd[k] = i64_to_f64(v[k]);
        if constexpr (S) {
            bs += ((uint64_t)((uint32_t)(v[k] >> 32) & mk) << 32) | ((uint32_t)v[k] & mk);
            const double xn = pack_f64((hi32(xd[k]) & mk) | (~mk & 0x7FF80000u), lo32(xd[k]));
            mn = raw_min(mn, xn);
            mx = raw_max(mx, xn);
        }
    }
    if constexpr (S) {
        a.sum = (int64_t)((uint64_t)a.sum + bs);
        if (__builtin_expect(fabs(mn) >= 9007199254740992.0 || fabs(mx) >= 9007199254740992.0, 0)) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int64_t x = (int64_t)v[k];
                const bool on = (m >> k) & 1u;
                a.mn = (on && x < a.mn) ? x : a.mn;
                a.mx = (on && x > a.mx) ? x : a.mx;
            }
        } else {
            a.dmn = raw_min(a.dmn, mn);
            a.dmx = raw_max(a.dmx, mx);
        }
    }
    if constexpr (M) {
        // Deviations from a shift c, then one reciprocal: with c = the running mean (or, on the lane's first
        // batch, any value of the batch) the Chan merge of (cnt, mean_b, m2_b) into (n, mean, m2) collapses to
        // mean' = c + S1 / n', m2' = m2 + S2 - S1^2 / n' (S1, S2: sums of the shifted deviations; n' = n + cnt).
        double c = a.mean;
        if (a.n == 0) {
            c = 0.0;
#pragma unroll
            for (int k = 7; k >= 0; --k) c = ((m >> k) & 1u) ? xd[k] : c;
        }
        double s1 = 0.0, s2 = 0.0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const double d = (xd[k] - c) * one_if(row_mask(m, k));
            s1 += d;
            s2 = __builtin_fma(d, d, s2);
        }
        const double r = rcp_refined((double)(a.n + cnt));
        a.mean = __builtin_fma(s1, r, c);
        a.m2 += __builtin_fma(-s1 * s1, r, s2);
    }
}
__device__ __forceinline__ void accumulate(IAcc& a, const uint64_t (&v)[8], uint32_t m, uint32_t flags) {
    const int cnt = __popc(m);
    if (cnt == 0) return;
    // the flags are wave-uniform: one branch per batch picks a straight-line body
    const bool stats = (flags & CF_STATS) != 0, moments = (flags & CF_MOMENTS) != 0;
    if (stats && moments) accumulate_int<true, true>(a, v, m, cnt);
    else if (stats) accumulate_int<true, false>(a, v, m, cnt);
    else if (moments) accumulate_int<false, true>(a, v, m, cnt);
    a.n += cnt;
}

// Rows of mask m where `value <op> constant` holds (Spark comparison semantics: integral vs long
// constant compares as long; otherwise as double with NaN above every number and NaN = NaN). Branch-free:
// the comparison's sign selects a bit of the operator's 3-bit truth mask (bit 0: <, bit 1: =, bit 2: >).
__device__ __forceinline__ uint32_t cmp_truth_mask(int op) {
    switch (op) {
        case DQ_P_EQ: return 2u;
        case DQ_P_NE: return 5u;
        case DQ_P_LT: return 1u;
        case DQ_P_LE: return 3u;
        case DQ_P_GT: return 4u;
        default: return 6u;  // GE
    }
}

template <bool F>
__device__ __forceinline__ int fused_pred_count(const ColDesc& c, const uint64_t (&v)[8], uint32_t m) {
    const uint32_t truth = cmp_truth_mask(c.pred_op);  // wave-uniform
    uint32_t hit = 0;
    if (!F && c.pred_kind == FP_LONG) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int64_t x = (int64_t)v[k];
            const uint32_t sel = x < c.pred_i ? 0u : (x > c.pred_i ? 2u : 1u);
            hit |= ((truth >> sel) & 1u) << k;
        }
    } else {
        const double y = c.pred_kind == FP_LONG ? (double)c.pred_i : c.pred_d;
        const bool yn = y != y;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const double x = to_double(v[k], F);
            const bool xn = x != x;
            const uint32_t sel = (xn || yn) ? ((xn && yn) ? 1u : (xn ? 2u : 0u)) : (x < y ? 0u : (x > y ? 2u : 1u));
            hit |= ((truth >> sel) & 1u) << k;
        }
    }
    return __popc(hit & m);
}

template <bool FX, bool FY>
__device__ __forceinline__ void accumulate_corr(CorrPartial& c, const uint64_t (&x)[8], const uint64_t (&y)[8],
                                                uint32_t m) {
    const int cnt = __popc(m);
    if (cnt == 0) return;
    // masked rows become 0.0 once (their bits may be anything, NaN included); the deviations are then masked by
    // a {1.0, 0.0} factor and accumulated with fma
    double xv[8], yv[8];
    double sx = 0.0, sy = 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const bool on = (m >> k) & 1u;
        xv[k] = on ? to_double(x[k], FX) : 0.0;
        yv[k] = on ? to_double(y[k], FY) : 0.0;
        sx += xv[k];
        sy += yv[k];
    }
    CorrPartial b;
    b.n = (double)cnt;
    const double inv = rcp_refined(b.n);  // one reciprocal for both means (instead of two IEEE divisions)
    b.xa = sx * inv;
    b.ya = sy * inv;
    b.ck = b.xm = b.ym = 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const double f = on_factor(m, k);
        const double dx = xv[k] - b.xa, dy = yv[k] - b.ya;
        const double dxf = dx * f, dyf = dy * f;
        b.ck = __builtin_fma(dxf, dy, b.ck);
        b.xm = __builtin_fma(dxf, dx, b.xm);
        b.ym = __builtin_fma(dyf, dy, b.ym);
    }
    corr_merge_batch(c, b);
}

// Hash class of a Spark type for XxHash64Function: 0 = hashInt of the int value, 1 = hashInt of the
// float bits, 2 = hashLong of the double bits, 3 = hashLong of the long value.
__device__ __forceinline__ int hash_class(int spark_type) {
    switch (spark_type) {
        case DQ_TYPE_BOOLEAN: case DQ_TYPE_BYTE: case DQ_TYPE_SHORT: case DQ_TYPE_INT: case DQ_TYPE_DATE: return 0;
        case DQ_TYPE_FLOAT: return 1;
        case DQ_TYPE_DOUBLE: return 2;
        default: return 3;
    }
}

// XXH64 (hashInt / hashLong, seed 42) of a lane value up to the last multiply of the avalanche, then the
// HLL++ register index and rank (C/StatefulHyperloglogPlus.scala:96-100) from the final hash's high word
// alone: with g = h * P3 and x = g ^ (g >> 32), idx = x >>> 55 = g_hi >>> 23 and, whenever g_hi << 9 != 0
// (all but 2^-23 of the values), rank = nlz((x << 9) | 1 << 8) + 1 = nlz32(g_hi << 9) + 1 — so the low half of
// the last 64-bit multiply and the final xor are only computed on that rare path. Bit-identical to
// hll_index(xxh_*(v)) / hll_rank(xxh_*(v)).
template <int HC>
__device__ __forceinline__ uint32_t hll_idx_rank(uint64_t v) {
    uint64_t h;
    if (HC <= 1) {
        const uint32_t iv = HC == 0 ? (uint32_t)(int32_t)(int64_t)v : float_to_int_bits((float)as_f64(v));
        h = SPARK_HLL_SEED + P64_5 + 4ULL;
        h ^= (uint64_t)iv * P64_1;
        h = rotl64(h, 23) * P64_2 + P64_3;
    } else {
        const uint64_t lv = HC == 2 ? double_to_long_bits(as_f64(v)) : v;
        h = SPARK_HLL_SEED + P64_5 + 8ULL;
        h ^= rotl64(lv * P64_2, 31) * P64_1;
        h = rotl64(h, 27) * P64_1 + P64_4;
    }
    h ^= h >> 33;
    h *= P64_2;
    h ^= h >> 29;
    const uint32_t hl = (uint32_t)h, hh = (uint32_t)(h >> 32);
    constexpr uint32_t p3l = (uint32_t)P64_3, p3h = (uint32_t)(P64_3 >> 32);
    const uint32_t ghi = __umulhi(hl, p3l) + hl * p3h + hh * p3l;
    const uint32_t idx = ghi >> 23;
    const uint32_t t = ghi << 9;
    uint32_t rank;
    if (__builtin_expect(t != 0u, 1)) {
        rank = (uint32_t)__clz((int)t) + 1u;
    } else {
        const uint32_t xlo = (hl * p3l) ^ ghi;
        const uint32_t whi = xlo >> 23;
        rank = whi ? (uint32_t)__clz((int)whi) + 1u : 32u + (uint32_t)__clz((int)((xlo << 9) | 256u)) + 1u;
    }
    return idx | (rank << 16);
}

// All 8 lane values are hashed unconditionally (independent multiply chains the scheduler can
// interleave; no divergence), then the valid ones are max-merged into the LDS registers with
// no-return ds_max atomics (fire-and-forget: no LDS latency on the critical path).
template <int HC>
__device__ __forceinline__ void hll_update8(uint32_t* regs, const uint64_t (&v)[8], uint32_t m) {
    // two groups of 4 independent hash chains: enough ILP for the VALU, half the live temporaries
#pragma unroll
    for (int g = 0; g < 8; g += 4) {
        uint32_t packed[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) packed[k] = hll_idx_rank<HC>(v[g + k]);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if ((m >> (g + k)) & 1u) atomicMax(&regs[packed[k] & 0xffffu], packed[k] >> 16);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// The hash class follows from the storage shape except for mixed-width pairs (P = 8): 8-byte
// storage is DOUBLE (2) or LONG / TIMESTAMP / DECIMAL (3), 4-byte FLOAT (1) or INT / DATE (0).
// Resolving it at compile time keeps one hash variant per kernel (instruction-cache footprint).
template <int P, bool F>
__device__ __forceinline__ void hll_update(uint32_t* regs, const uint64_t (&v)[8], uint32_t m, int spark_type) {
    if (m == 0u) return;
    if (P == 2) {
        hll_update8<F ? 2 : 3>(regs, v, m);
        return;
    }
    if (P == 4) {
        hll_update8<F ? 1 : 0>(regs, v, m);
        return;
    }
    switch (hash_class(spark_type)) {  // wave-uniform
        case 0: hll_update8<0>(regs, v, m); break;
        case 1: hll_update8<1>(regs, v, m); break;
        case 2: hll_update8<2>(regs, v, m); break;
        default: hll_update8<3>(regs, v, m); break;
    }
}

// ------------------------------------------------------------------------------------------------
// Value slots: P rows per load, NC columns (2 = Correlation pair), F0/F1 = floating storage.
// Workgroup g handles tiles g, g + G, g + 2G, ... (balanced for any grid size); the next tile's
// loads are issued before the current tile is folded (register double buffer).
// ------------------------------------------------------------------------------------------------
template <int NC, bool F0, bool F1>
struct BlockRed {
    typename AccOf<F0>::type a0[kBlock / 64];
    typename AccOf<F1>::type a1[kBlock / 64];
    CorrPartial cp[kBlock / 64];
    int64_t wt[kBlock / 64], wnn[kBlock / 64];
};

#ifndef DQ_HEAVY_PAIR_MINB
#define DQ_HEAVY_PAIR_MINB 1
#endif
template <int P, int NC, bool F0, bool F1, bool HEAVY>
__global__ void __launch_bounds__(kBlock, (HEAVY && NC > 1) ? DQ_HEAVY_PAIR_MINB : 1)
scan_values_kernel(const SlotDesc* __restrict__ slots, const int32_t* __restrict__ group, int ngroup,
                   int64_t nrows, int64_t ntiles, int gstride, SlotPartial* __restrict__ partials,
                   uint8_t* __restrict__ hll_partials) {
    using A0 = typename AccOf<F0>::type;
    using A1 = typename AccOf<F1>::type;
    __shared__ uint32_t hll_lds[NC][kHllRegs];
    __shared__ BlockRed<NC, F0, F1> red;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int64_t G = gridDim.x;
    for (int gi = 0; gi < ngroup; ++gi) {
        const int s = group[gi];
        const SlotDesc sd = slots[s];
        const ColDesc c0 = sd.col[0];
        const ColDesc c1 = sd.col[1];
        const bool has_where = sd.where_t != nullptr;
        // HLL and fused predicates only exist in the HEAVY instantiations (register budget).
        const bool hll0 = HEAVY && (c0.flags & CF_HLL) != 0;
        const bool hll1 = HEAVY && NC > 1 && (c1.flags & CF_HLL) != 0;
        A0 a0;
        A1 a1;
        acc_init(a0);
        acc_init(a1);
        CorrPartial cp;
        cp.n = cp.xa = cp.ya = cp.ck = cp.xm = cp.ym = 0.0;
        int64_t wt = 0, wnn = 0;
        if (hll0 || hll1) {
            for (int i = tid; i < NC * kHllRegs; i += kBlock) (&hll_lds[0][0])[i] = 0;
            __syncthreads();
        }
        // Folds one loaded tile into the lane state.
        auto fold = [&](int64_t tb, bool full, const uint64_t (&xv)[8], const uint64_t (&yv)[8]) {
            uint32_t mx = bits_valid<P>(c0.validity, tb, tid, full, nrows);
            uint32_t my = NC > 1 ? bits_valid<P>(c1.validity, tb, tid, full, nrows) : 0u;
            if (has_where) {
                const uint32_t w = bits_padded<P, true>(sd.where_t, tb, tid);
                wt += __popc(w);
                wnn += __popc(bits_padded<P, true>(sd.where_nn, tb, tid));
                mx &= w;
                my &= w;
            }
            // Phases are fenced from each other (sched_barrier) so the scheduler cannot interleave
            // them: only one phase's temporaries are live at a time, which keeps the 2-column
            // HEAVY kernels out of AGPR/SGPR spilling.
            accumulate(a0, xv, mx, c0.flags);
            if (HEAVY) __builtin_amdgcn_sched_barrier(0);
            if (HEAVY && c0.pred_kind) a0.pt += fused_pred_count<F0>(c0, xv, mx);
            if (hll0) hll_update<P, F0>(hll_lds[0], xv, mx, c0.spark_type);
            if (NC > 1) {
                if (HEAVY) __builtin_amdgcn_sched_barrier(0);
                accumulate(a1, yv, my, c1.flags);
                if (HEAVY) __builtin_amdgcn_sched_barrier(0);
                if (HEAVY && c1.pred_kind) a1.pt += fused_pred_count<F1>(c1, yv, my);
                if (hll1) hll_update<P, F1>(hll_lds[NC - 1], yv, my, c1.spark_type);
                if (HEAVY) __builtin_amdgcn_sched_barrier(0);
                accumulate_corr<F0, F1>(cp, xv, yv, mx & my);
            }
        };
        // Full tiles: buffer loads only, next tile's loads in flight while the current one folds.
        const int64_t nfull = nrows / kTileRows;
        int64_t t = blockIdx.x;
        uint64_t x[8], y[8], xn[8], yn[8];
        constexpr bool kDoubleBuffer = !(HEAVY && NC > 1);
        if (kDoubleBuffer && t < nfull) {
            load_values<P, F0>(c0, t * kTileRows, tid, true, nrows, x);
            if (NC > 1) load_values<P, F1>(c1, t * kTileRows, tid, true, nrows, y);
        }
        if (!kDoubleBuffer && t < nfull) {
            load_values<P, F0>(c0, t * kTileRows, tid, true, nrows, x);
            load_values<P, F1>(c1, t * kTileRows, tid, true, nrows, y);
        }
        for (; t < nfull; t += G) {
            const int64_t tn = t + G;
            if (!kDoubleBuffer) {
                // Two-column HEAVY kernels: no second register set (it costs 32 VGPRs and drops them to
                // 1 wave/SIMD). Instead the phases run in the order corr(x, y) -> x -> y, and each column's
                // registers are refilled with the next tile's values as soon as that column is done, so the
                // loads of x overlap the work on y and the loads of y the next tile's corr + x work.
                const int64_t tb = t * kTileRows;
                uint32_t mx = bits_valid<P>(c0.validity, tb, tid, true, nrows);
                uint32_t my = bits_valid<P>(c1.validity, tb, tid, true, nrows);
                if (has_where) {
                    const uint32_t w = bits_padded<P, true>(sd.where_t, tb, tid);
                    wt += __popc(w);
                    wnn += __popc(bits_padded<P, true>(sd.where_nn, tb, tid));
                    mx &= w;
                    my &= w;
                }
                accumulate_corr<F0, F1>(cp, x, y, mx & my);
                __builtin_amdgcn_sched_barrier(0);
                accumulate(a0, x, mx, c0.flags);
                __builtin_amdgcn_sched_barrier(0);
                if (c0.pred_kind) a0.pt += fused_pred_count<F0>(c0, x, mx);
                if (hll0) hll_update<P, F0>(hll_lds[0], x, mx, c0.spark_type);
                __builtin_amdgcn_sched_barrier(0);
                if (tn < nfull) load_values<P, F0>(c0, tn * kTileRows, tid, true, nrows, x);
                accumulate(a1, y, my, c1.flags);
                __builtin_amdgcn_sched_barrier(0);
                if (c1.pred_kind) a1.pt += fused_pred_count<F1>(c1, y, my);
                if (hll1) hll_update<P, F1>(hll_lds[NC - 1], y, my, c1.spark_type);
                __builtin_amdgcn_sched_barrier(0);
                if (tn < nfull) load_values<P, F1>(c1, tn * kTileRows, tid, true, nrows, y);
                continue;
            }
            if (tn < nfull) {
                load_values<P, F0>(c0, tn * kTileRows, tid, true, nrows, xn);
                if (NC > 1) load_values<P, F1>(c1, tn * kTileRows, tid, true, nrows, yn);
            }
            fold(t * kTileRows, true, x, y);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                x[k] = xn[k];
                if (NC > 1) y[k] = yn[k];
            }
        }
        // The partial last tile (if any) goes to the workgroup next in the interleave.
        if (nfull < ntiles && blockIdx.x == nfull % G) {
            load_values<P, F0>(c0, nfull * kTileRows, tid, false, nrows, x);
            if (NC > 1) load_values<P, F1>(c1, nfull * kTileRows, tid, false, nrows, y);
            fold(nfull * kTileRows, false, x, y);
        }
        acc_finish(a0);
        acc_finish(a1);
        // wave64 tree, then the 4 wave results in a fixed order.
#pragma unroll 1
        for (int off = 32; off > 0; off >>= 1) {
            A0 o0;
            acc_shfl(o0, a0, off);
            const int64_t owt = shfl_down_i64(wt, off), ownn = shfl_down_i64(wnn, off);
            A1 o1;
            CorrPartial oc;
            if (NC > 1) {
                acc_shfl(o1, a1, off);
                corr_shfl(oc, cp, off);
            }
            if (lane < off) {
                acc_merge(a0, o0);
                wt += owt;
                wnn += ownn;
                if (NC > 1) {
                    acc_merge(a1, o1);
                    corr_merge(cp, oc);
                }
            }
        }
        if (lane == 0) {
            red.a0[wave] = a0;
            red.wt[wave] = wt;
            red.wnn[wave] = wnn;
            if (NC > 1) {
                red.a1[wave] = a1;
                red.cp[wave] = cp;
            }
        }
        __syncthreads();
        if (tid == 0) {
            for (int w = 1; w < kBlock / 64; ++w) {
                acc_merge(a0, red.a0[w]);
                wt += red.wt[w];
                wnn += red.wnn[w];
                if (NC > 1) {
                    acc_merge(a1, red.a1[w]);
                    corr_merge(cp, red.cp[w]);
                }
            }
            // Field-wise stores: a whole SlotPartial temporary would cost ~70 VGPRs here.
            SlotPartial* dst = partials + (int64_t)s * gstride + blockIdx.x;
            store_partial(dst->c[0], a0);
            if (NC > 1) {
                store_partial(dst->c[1], a1);
                dst->corr = cp;
            } else {
                store_empty(dst->c[1]);
                dst->corr.n = dst->corr.xa = dst->corr.ya = dst->corr.ck = dst->corr.xm = dst->corr.ym = 0.0;
            }
            dst->wt = wt;
            dst->wnn = wnn;
            dst->pt = dst->pnn = dst->vt = dst->pad = 0;
        }
        if (hll0 || hll1) {
            for (int c = 0; c < NC; ++c) {
                const int hs = c == 0 ? c0.hll_slot : c1.hll_slot;
                if (hs >= 0 && (c == 0 ? hll0 : hll1)) {
                    uint8_t* dst = hll_partials + ((int64_t)hs * gstride + blockIdx.x) * kHllRegs;
                    for (int i = tid; i < kHllRegs; i += kBlock) dst[i] = (uint8_t)hll_lds[c][i];
                }
            }
        }
        __syncthreads();
    }
}


// ------------------------------------------------------------------------------------------------
// HEAVY slots over 8-byte columns (LONG / TIMESTAMP / DECIMAL storage, DOUBLE): HLL registers, fused
// Compliance `col <op> const`, the moments and Correlation in one pass — the north-star suite, VALU-bound on
// XXH64. Written for the instruction count:
//  * each lane owns 8 consecutive rows of the tile (4 x 16-B loads at a 64-B lane stride), so its validity /
//    where bits are one bitmap byte (no bit gathering);
//  * per-row masks are one v_bfe_i32 (0 / ~0); masked values are cleared with two v_and, min / max use a NaN
//    stand-in built with one v_bfi (raw v_min_f64 / v_max_f64 drop a NaN operand; no canonicalising moves);
//  * integral columns are converted to double once (3 instructions) and that double serves the moments, the
//    correlation and the min / max (exact while |x| < 2^53 — checked per batch, exact int64 fallback);
//  * the fused compare counts hits on the cleared values and corrects the masked rows with the wave-uniform
//    result of `0 <op> const`; HLL updates are unconditional LDS max of (rank & mask) (rank 0 is a no-op); the
//    2^-23 case of a zero rank field takes a per-tile exact re-hash.
// Bit-exact HLL registers, counts, integral sums and min / max; fp64 moments within rounding of the batch order.
// ------------------------------------------------------------------------------------------------

// Fused compare of the cleared value (masked rows hold 0 / 0.0) — Spark semantics (NaN above every number,
// NaN = NaN, -0.0 = 0.0) for a non-NaN double constant; integral columns against a LONG constant compare as long.
template <bool F>
__device__ __forceinline__ uint32_t cmp_hits8(const double (&xd)[8], const uint64_t (&xi)[8], int op, double y,
                                              int64_t yi) {
    uint32_t h = 0;
#define DQ_CMP8(expr) _Pragma("unroll") for (int k = 0; k < 8; ++k) h += (expr) ? 1u : 0u; break;
    if (F) {
        switch (op) {
            case DQ_P_EQ: DQ_CMP8(xd[k] == y)
            case DQ_P_NE: DQ_CMP8(!(xd[k] == y))
            case DQ_P_LT: DQ_CMP8(xd[k] < y)
            case DQ_P_LE: DQ_CMP8(xd[k] <= y)
            case DQ_P_GT: DQ_CMP8(!(xd[k] <= y))
            default: DQ_CMP8(!(xd[k] < y))
        }
    } else {
        switch (op) {
            case DQ_P_EQ: DQ_CMP8((int64_t)xi[k] == yi)
            case DQ_P_NE: DQ_CMP8((int64_t)xi[k] != yi)
            case DQ_P_LT: DQ_CMP8((int64_t)xi[k] < yi)
            case DQ_P_LE: DQ_CMP8((int64_t)xi[k] <= yi)
            case DQ_P_GT: DQ_CMP8((int64_t)xi[k] > yi)
            default: DQ_CMP8((int64_t)xi[k] >= yi)
        }
    }
#undef DQ_CMP8
    return h;
}

// The same count over the whole wave (wave-uniform): each compare is one v_cmp into a lane mask whose popcount the
// scalar unit adds, instead of a compare plus a per-lane add with carry for every value.
template <bool F>
__device__ __forceinline__ uint32_t cmp_hits8_wave(const double (&xd)[8], const uint64_t (&xi)[8], int op, double y,
                                                   int64_t yi) {
    uint32_t h = 0;
#define DQ_CMPW(expr) _Pragma("unroll") for (int k = 0; k < 8; ++k) h += (uint32_t)__popcll(__ballot(expr)); break;
    if (F) {
        switch (op) {
            case DQ_P_EQ: DQ_CMPW(xd[k] == y)
            case DQ_P_NE: DQ_CMPW(!(xd[k] == y))
            case DQ_P_LT: DQ_CMPW(xd[k] < y)
            case DQ_P_LE: DQ_CMPW(xd[k] <= y)
            case DQ_P_GT: DQ_CMPW(!(xd[k] <= y))
            default: DQ_CMPW(!(xd[k] < y))
        }
    } else {
        switch (op) {
            case DQ_P_EQ: DQ_CMPW((int64_t)xi[k] == yi)
            case DQ_P_NE: DQ_CMPW((int64_t)xi[k] != yi)
            case DQ_P_LT: DQ_CMPW((int64_t)xi[k] < yi)
            case DQ_P_LE: DQ_CMPW((int64_t)xi[k] <= yi)
            case DQ_P_GT: DQ_CMPW((int64_t)xi[k] > yi)
            default: DQ_CMPW((int64_t)xi[k] >= yi)
        }
    }
#undef DQ_CMPW
    return h;
}

// XXH64 hashLong (seed 42) of a long (or of doubleToLongBits) up to the final multiply's high word (see hll_idx_rank);
// returns that word: idx = g >> 23, rank field t = g << 9.
__device__ __forceinline__ uint32_t xxh_long_ghi(uint64_t lv) {
    uint64_t h = SPARK_HLL_SEED + P64_5 + 8ULL;
    h ^= rotl64(lv * P64_2, 31) * P64_1;
    h = rotl64(h, 27) * P64_1 + P64_4;
    h ^= h >> 33;
    h *= P64_2;
    h ^= h >> 29;
    const uint32_t hl = (uint32_t)h, hh = (uint32_t)(h >> 32);
    constexpr uint32_t p3l = (uint32_t)P64_3, p3h = (uint32_t)(P64_3 >> 32);
    return __umulhi(hl, p3l) + hl * p3h + hh * p3l;
}

struct HAccF {  // DOUBLE column
    uint32_t n, nnan, pt;
    double sum, mn, mx, mean, m2;
};
struct HAccI {  // 8-byte integral column
    uint32_t n, pt;
    int64_t isum, imn, imx;  // imn / imx: exact fallback of batches with |value| >= 2^53
    double mn, mx, mean, m2;
};
template <bool F> struct HAccOf { using type = HAccI; };
template <> struct HAccOf<true> { using type = HAccF; };

__device__ __forceinline__ void hacc_init(HAccF& a) {
    a.n = a.nnan = a.pt = 0;
    a.sum = 0.0;
    a.mn = a.mx = __builtin_nan("");
    a.mean = a.m2 = 0.0;
}
__device__ __forceinline__ void hacc_init(HAccI& a) {
    a.n = a.pt = 0;
    a.isum = 0;
    a.imn = INT64_MAX;
    a.imx = INT64_MIN;
    a.mn = a.mx = __builtin_nan("");
    a.mean = a.m2 = 0.0;
}
__device__ __forceinline__ void hacc_to(FAcc& o, const HAccF& a) {
    o.n = a.n;
    o.nnan = a.nnan;
    o.pt = a.pt;
    o.sum = a.sum;
    o.mn = a.mn != a.mn ? INFINITY : a.mn;
    o.mx = a.mx != a.mx ? -INFINITY : a.mx;
    o.mean = a.mean;
    o.m2 = a.m2;
}
__device__ __forceinline__ void hacc_to(IAcc& o, const HAccI& a) {
    o.n = a.n;
    o.pt = a.pt;
    o.sum = a.isum;
    o.mn = a.imn;
    o.mx = a.imx;
    if (a.mn == a.mn && (int64_t)a.mn < o.mn) o.mn = (int64_t)a.mn;  // |mn| < 2^53: exact
    if (a.mx == a.mx && (int64_t)a.mx > o.mx) o.mx = (int64_t)a.mx;
    o.mean = a.mean;
    o.m2 = a.m2;
    o.dmn = o.dmx = __builtin_nan("");
}

// Chan merge of one batch (cnt >= 1 rows, mean mb, m2b) into the lane moments.
__device__ __forceinline__ void hmoments_merge(uint32_t na, double& mean, double& m2, uint32_t cnt, double mb,
                                               double m2b) {
    if (na == 0) {
        mean = mb;
        m2 = m2b;
        return;
    }
    const double n1 = (double)na, n2 = (double)cnt;
    const double delta = mb - mean;
    const double deltaN = delta * rcp_refined(n1 + n2);
    mean = __builtin_fma(deltaN, n2, mean);
    m2 = m2 + m2b + delta * deltaN * (n1 * n2);
}

struct HeavyCol {  // wave-uniform description of one column's work in the heavy kernel
    bool stats, moments, hll, pred;
    int op;
    uint32_t zhit;  // 1 if `0 <op> const` holds (masked rows hold 0 / 0.0)
    double y;
    int64_t yi;
};

__device__ __forceinline__ HeavyCol heavy_col_of(const ColDesc& c, bool F) {
    HeavyCol h;
    h.stats = (c.flags & CF_STATS) != 0;
    h.moments = (c.flags & CF_MOMENTS) != 0;
    h.hll = (c.flags & CF_HLL) != 0;
    h.op = c.pred_op;
    h.yi = c.pred_i;
    h.y = c.pred_kind == FP_LONG ? (double)c.pred_i : c.pred_d;
    // fast fused compare: DOUBLE column vs a non-NaN constant, integral column vs a LONG constant
    h.pred = c.pred_kind != FP_NONE && (F ? (h.y == h.y) : c.pred_kind == FP_LONG);
    const double zero = 0.0;
    bool z;
    if (F || c.pred_kind != FP_LONG) {
        switch (h.op) {
            case DQ_P_EQ: z = zero == h.y; break;
            case DQ_P_NE: z = !(zero == h.y); break;
            case DQ_P_LT: z = zero < h.y; break;
            case DQ_P_LE: z = zero <= h.y; break;
            case DQ_P_GT: z = !(zero <= h.y); break;
            default: z = !(zero < h.y); break;
        }
    } else {
        switch (h.op) {
            case DQ_P_EQ: z = 0 == h.yi; break;
            case DQ_P_NE: z = 0 != h.yi; break;
            case DQ_P_LT: z = 0 < h.yi; break;
            case DQ_P_LE: z = 0 <= h.yi; break;
            case DQ_P_GT: z = 0 > h.yi; break;
            default: z = 0 >= h.yi; break;
        }
    }
    h.zhit = z ? 1u : 0u;
    return h;
}

// One column's 8 rows of the tile. xd receives the value as double for the correlation phase (DOUBLE: cleared
// bits; integral: the converted raw value, finite); `fin` is false when a valid DOUBLE row is inf / NaN.
// `need_xd`: stats, moments, the fused compare or the correlation read the values; otherwise (ApproxCountDistinct
// alone) only the hash loop runs.
template <bool F, bool FULL>
__device__ __forceinline__ void heavy_col_rows(typename HAccOf<F>::type& a, const uint64_t (&v)[8], uint32_t m,
                                               const HeavyCol& hc, const ColDesc& c, uint32_t* regs, uint32_t& tmin,
                                               bool need_xd, double (&xd)[8], bool& fin) {
    const uint32_t cnt = __popc(m);
    uint64_t xi[8];  // cleared integral values
    double s = 0.0;
    fin = true;
    uint32_t hm = m;  // rows hashed from their raw bits below
    if (FULL || need_xd) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t mk = row_mask(m, k);
            if constexpr (F) {
                xd[k] = and_f64(as_f64(v[k]), mk);
                s += xd[k];
            } else {
                xi[k] = ((uint64_t)((uint32_t)(v[k] >> 32) & mk) << 32) | ((uint32_t)v[k] & mk);
                xd[k] = i64_to_f64(v[k]);
            }
        }
    } else if (F) {
#pragma unroll
        for (int k = 0; k < 8; ++k) s += as_f64(v[k]);  // NaN detector only (masked rows may raise it spuriously)
    }
    double mn = __builtin_nan(""), mx = __builtin_nan("");
    if (FULL || hc.stats) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t mk = row_mask(m, k);
            // NaN stand-in for masked rows: v_min / v_max drop it
            const double xn = pack_f64((hi32(xd[k]) & mk) | (~mk & 0x7FF80000u), lo32(xd[k]));
            mn = raw_min(mn, xn);
            mx = raw_max(mx, xn);
        }
    }
    if constexpr (F) {
        if (__builtin_expect(!(s - s == 0.0), 0)) {
            fin = false;
            if (s != s) {
                // NaN among the valid rows (or inf - inf): exact NaN count and NaN-free extremes of the batch; the
                // NaN rows leave the raw-bits hash loop and add the canonical NaN's register once (doubleToLongBits)
                uint32_t nanm = 0;
                mn = INFINITY;
                mx = -INFINITY;
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const double x = as_f64(v[k]);
                    const bool on = (m >> k) & 1u;
                    nanm |= (on && x != x) ? (1u << k) : 0u;
                    if (on && x == x) {
                        mn = x < mn ? x : mn;
                        mx = x > mx ? x : mx;
                    }
                }
                const uint32_t nn = __popc(nanm);
                a.nnan += nn;
                if (mn == INFINITY && mx == -INFINITY && nn == cnt) mn = mx = __builtin_nan("");
                hm = m & ~nanm;
                if ((FULL || hc.hll) && nanm) {
                    const uint32_t p = hll_idx_rank<2>(f64_bits(__builtin_nan("")));
                    atomicMax(reinterpret_cast<int*>(&regs[p & 0xffffu]), (int)(p >> 16) - 1);
                }
            }
        }
        if (FULL || hc.stats) {
            a.sum += s;
            a.mn = raw_min(a.mn, mn);
            a.mx = raw_max(a.mx, mx);
        }
    } else {
        if (FULL || hc.stats) {
            int64_t bs = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) bs = (int64_t)((uint64_t)bs + xi[k]);
            a.isum = (int64_t)((uint64_t)a.isum + (uint64_t)bs);
            const bool big = fabs(mn) >= 9007199254740992.0 || fabs(mx) >= 9007199254740992.0;
            if (__builtin_expect(big, 0)) {
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const int64_t x = (int64_t)v[k];
                    const bool on = (m >> k) & 1u;
                    a.imn = (on && x < a.imn) ? x : a.imn;
                    a.imx = (on && x > a.imx) ? x : a.imx;
                }
            } else {
                a.mn = raw_min(a.mn, mn);
                a.mx = raw_max(a.mx, mx);
            }
        }
    }
    if constexpr (!F) {
        if ((FULL || hc.moments) && cnt) {
            // finite values: shifted deviations and one reciprocal (see accumulate_int)
            double c0 = a.mean;
            if (a.n == 0) {
                c0 = 0.0;
#pragma unroll
                for (int k = 7; k >= 0; --k) c0 = ((m >> k) & 1u) ? xd[k] : c0;
            }
            double s1 = 0.0, s2 = 0.0;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const double d = mul_raw(xd[k] - c0, one_if(row_mask(m, k)));
                s1 += d;
                s2 = __builtin_fma(d, d, s2);
            }
            const double r = rcp_refined((double)(a.n + cnt));
            a.mean = __builtin_fma(s1, r, c0);
            a.m2 += __builtin_fma(-s1 * s1, r, s2);
        }
    } else if ((FULL || hc.moments) && cnt && __builtin_expect(fin && a.n != 0, 1)) {
        // finite batch: deviations from the running mean as the integral path, one reciprocal of the new count; masked
        // rows hold 0.0 and get a 0.0 factor. A lane's first batch (and a batch with a valid inf / NaN) takes the
        // batch mean + Chan merge below.
        const double c0 = a.mean;
        double s1 = 0.0, s2 = 0.0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            // xd holds 0.0 on masked rows: xd - c0 f is exactly the rounded deviation on valid rows and 0 on masked
            // ones, one fma instead of a subtract and a multiply
            const double d = __builtin_fma(-c0, one_if(row_mask(m, k)), xd[k]);
            s1 += d;
            s2 = __builtin_fma(d, d, s2);
        }
        const double r = rcp_refined((double)(a.n + cnt));
        a.mean = __builtin_fma(s1, r, c0);
        a.m2 += __builtin_fma(-s1 * s1, r, s2);
    } else if ((FULL || hc.moments) && cnt) {
        const double mb = s * rcp_refined((double)cnt);
        double m2b = 0.0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t mk = row_mask(m, k);
            const double d = and_f64(xd[k] - mb, mk);
            m2b = __builtin_fma(d, d, m2b);
        }
        hmoments_merge(a.n, a.mean, a.m2, cnt, mb, m2b);
    }
    if (FULL) {
        // the tile loop runs with every lane active: the wave's hits go to lane 0's partial (the lane partials are
        // summed at the end); masked rows hold 0 and hit when `0 <op> c` does (zhit): taken off per wave
        uint32_t w = cmp_hits8_wave<F>(xd, xi, hc.op, hc.y, hc.yi);
        if (hc.zhit) {
#pragma unroll
            for (int k = 0; k < 8; ++k) w -= (uint32_t)__popcll(__ballot(!((m >> k) & 1u)));
        }
        if ((threadIdx.x & 63) == 0) a.pt += w;
    } else if (hc.pred) {
        a.pt += cmp_hits8<F>(xd, xi, hc.op, hc.y, hc.yi) - hc.zhit * (8u - cnt);
    }
    else if (c.pred_kind != FP_NONE) a.pt += fused_pred_count<F>(c, v, m);  // NaN constant / mixed kinds
    a.n += cnt;
    if (FULL || hc.hll) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t g = xxh_long_ghi(v[k]);  // DOUBLE: raw bits (NaN rows were taken out of hm above)
            const uint32_t t = g << 9;
            tmin = min(tmin, t);
            // the registers hold rank - 1 as signed ints (-1 = empty): ffbh's -1 for a masked row (and for t == 0) is
            // the no-op, and the + 1 is paid once per register at the end instead of once per value
            atomicMax(reinterpret_cast<int*>(&regs[g >> 23]), (int)ffbh_raw(t & row_mask(hm, k)));
        }
    }
}

// Correlation of the rows valid in both columns (CorrelationState per 8-row batch + Chan merge). xd / yd hold
// finite values on the fast path (cleared DOUBLE rows, converted integral rows), so a {1.0, 0.0} factor selects
// the rows of the pair; a lane whose DOUBLE batch holds a valid inf / NaN clears the bits instead.
template <bool FX, bool FY>
__device__ __forceinline__ void heavy_corr_rows(CorrPartial& cp, const double (&xd)[8], const double (&yd)[8],
                                                uint32_t m, bool fin) {
    const uint32_t cnt = __popc(m);
    if (cnt == 0) return;
    if (__builtin_expect(fin && cp.n != 0.0, 1)) {
        // deviations from the lane's running means (cx, cy): with d = x - cx, e = y - cy over the batch and
        // n' = n + cnt, xAvg' = cx + sum d / n', ck' = ck + sum d e - (sum d)(sum e) / n' (xMk, yMk alike) -- the
        // algebra of the CorrelationState merge (A/Correlation.scala:37-52), one reciprocal per batch. A lane's first
        // batch (and a batch with a valid inf / NaN) takes the batch-mean form below.
        const double cx = cp.xa, cy = cp.ya;
        double sd = 0.0, se = 0.0, sdd = 0.0, see = 0.0, sde = 0.0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const double f = one_if(row_mask(m, k));
            const double d = mul_raw(xd[k] - cx, f), e = mul_raw(yd[k] - cy, f);
            sd += d;
            se += e;
            sdd = __builtin_fma(d, d, sdd);
            see = __builtin_fma(e, e, see);
            sde = __builtin_fma(d, e, sde);
        }
        const double n1 = cp.n + (double)cnt;
        const double r = rcp_refined(n1);
        const double sdr = sd * r, ser = se * r;
        cp.xa = __builtin_fma(sd, r, cx);
        cp.ya = __builtin_fma(se, r, cy);
        cp.ck += __builtin_fma(-sd, ser, sde);
        cp.xm += __builtin_fma(-sd, sdr, sdd);
        cp.ym += __builtin_fma(-se, ser, see);
        cp.n = n1;
        return;
    }
    CorrPartial b;
    b.n = (double)cnt;
    b.ck = b.xm = b.ym = 0.0;
    const double inv = rcp_refined(b.n);
    {
        double xv[8], yv[8];
        double sx = 0.0, sy = 0.0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t mk = row_mask(m, k);
            xv[k] = and_f64(xd[k], mk);
            yv[k] = and_f64(yd[k], mk);
            sx += xv[k];
            sy += yv[k];
        }
        b.xa = sx * inv;
        b.ya = sy * inv;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t mk = row_mask(m, k);
            const double dx = and_f64(xv[k] - b.xa, mk), dy = and_f64(yv[k] - b.ya, mk);
            b.ck = __builtin_fma(dx, dy, b.ck);
            b.xm = __builtin_fma(dx, dx, b.xm);
            b.ym = __builtin_fma(dy, dy, b.ym);
        }
    }
    corr_merge_batch(cp, b);
}

// The rare path of the HLL update: exact index / rank of every valid row of the lane (max is idempotent).
template <bool F>
__device__ __forceinline__ void heavy_hll_exact(uint32_t* regs, const uint64_t (&v)[8], uint32_t m) {
    for (int k = 0; k < 8; ++k)
        if ((m >> k) & 1u) {
            const uint32_t p = hll_idx_rank<F ? 2 : 3>(v[k]);
            atomicMax(reinterpret_cast<int*>(&regs[p & 0xffffu]), (int)(p >> 16) - 1);
        }
}

// Lane's 8 consecutive rows of a full tile and their validity byte.
__device__ __forceinline__ void heavy_load(const ColDesc& c, int64_t t, int tid, uint64_t (&v)[8]) {
    const __amdgpu_buffer_rsrc_t r = tile_rsrc(c.values, t * kTileRows * 8, kTileRows * 8);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const v4i_t x = __builtin_amdgcn_raw_buffer_load_b128(r, tid * 64 + i * 16, 0, 0);
        v[2 * i] = pack64(x.x, x.y);
        v[2 * i + 1] = pack64(x.z, x.w);
    }
}
__device__ __forceinline__ uint32_t heavy_bits(const uint64_t* bm, int64_t t, int tid) {
    return bm ? (uint32_t)reinterpret_cast<const uint8_t*>(bm)[t * (kTileRows / 8) + tid] : 0xFFu;
}
// The partial last tile: bounded loads, rows past the end masked off.
__device__ __forceinline__ uint32_t heavy_tail(const ColDesc& c, int64_t t, int tid, int64_t nrows, uint64_t (&v)[8]) {
    const int64_t r0 = t * kTileRows + (int64_t)tid * 8;
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int64_t r = r0 + k;
        const bool in = r < nrows;
        v[k] = in ? static_cast<const uint64_t*>(c.values)[r] : 0ull;
        const bool ok = in && (c.validity == nullptr ||
                               ((reinterpret_cast<const uint8_t*>(c.validity)[r >> 3] >> (r & 7)) & 1));
        m |= (ok ? 1u : 0u) << k;
    }
    return m;
}

// ---- `where` producer (WhereOut, dq_internal.h) ----------------------------------------------------------------------
// The lane's 8 consecutive rows of one 8-byte column against one PredSimple term: TRUE / NOT-NULL row bytes (Spark
// comparison: NaN = NaN and above every number for double compares, long compares for integral vs long constant).
template <bool F>
__device__ __forceinline__ void where_term8(const PredTerm& q, const uint64_t (&v)[8], uint32_t valid, uint32_t inr,
                                            uint32_t& t, uint32_t& n) {
    if (q.op == DQ_P_IS_NULL || q.op == DQ_P_IS_NOT_NULL) {
        t = (q.op == DQ_P_IS_NULL ? ~valid : valid) & inr;
        n = inr;
        return;
    }
    const uint32_t truth = cmp_truth_mask(q.op);  // bit 0: <, bit 1: =, bit 2: >
    uint32_t hit = 0;
    if (!F && !q.dbl) {
        const int64_t y = q.ci;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int64_t x = (int64_t)v[k];
            const uint32_t sel = x < y ? 0u : (x > y ? 2u : 1u);
            hit |= ((truth >> sel) & 1u) << k;
        }
    } else {
        const double y = q.cd;
        const bool yn = y != y;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const double x = F ? as_f64(v[k]) : (double)(int64_t)v[k];
            const bool xn = x != x;
            const uint32_t sel = (xn || yn) ? ((xn && yn) ? 1u : (xn ? 2u : 0u)) : (x < y ? 0u : (x > y ? 2u : 1u));
            hit |= ((truth >> sel) & 1u) << k;
        }
    }
    n = valid & inr;
    t = hit & n;
}

// The PredSimple postfix over 8-row bytes, SQL three-valued logic on a byte stack in two 64-bit registers (depth <=
// kWhereStack, checked on the host). Returns TRUE bits in the low byte, NOT-NULL bits in the next.
template <bool F>
__device__ __forceinline__ uint32_t where_eval8(const PredSimple& P, const uint64_t (&v)[8], uint32_t valid,
                                                uint32_t inr) {
    uint64_t st = 0, sn = 0;
    const int nb = P.nb;
    for (int i = 0; i < nb; ++i) {  // wave-uniform
        const int o = P.b[i];
        if (o >= 0) {
            uint32_t t, n;
            where_term8<F>(P.t[o], v, valid, inr, t, n);
            st = (st << 8) | t;
            sn = (sn << 8) | n;
        } else if (o == kPB_NOT) {
            const uint64_t t = st & 0xFFu, n = sn & 0xFFu;
            st = (st & ~0xFFull) | (n & ~t);
        } else {
            const uint64_t tc = st & 0xFFu, nc = sn & 0xFFu;
            st >>= 8;
            sn >>= 8;
            const uint64_t ta = st & 0xFFu, na = sn & 0xFFu;
            uint64_t rt, rn;
            if (o == kPB_AND) {
                const uint64_t f = (na & ~ta) | (nc & ~tc);  // a FALSE side decides
                rt = ta & tc;
                rn = f | (na & nc);
            } else {
                rt = ta | tc;
                rn = rt | (na & nc);
            }
            st = (st & ~0xFFull) | rt;
            sn = (sn & ~0xFFull) | rn;
        }
    }
    return (uint32_t)(st & 0xFFu) | ((uint32_t)(sn & 0xFFu) << 8);
}

// Four lanes' row bytes -> one dword (rows 32 q .. 32 q + 31 of the tile) in every lane of the quad.
__device__ __forceinline__ uint32_t quad_pack(uint32_t byte, int lane) {
    uint32_t p = byte << (8 * (lane & 3));
    p |= (uint32_t)__builtin_amdgcn_mov_dpp((int)p, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    p |= (uint32_t)__builtin_amdgcn_mov_dpp((int)p, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
    return p;
}

// Bitmap bytes [b0, b0 + 4) of a user validity bitmap of exactly vbytes bytes (bounded in the tail tile).
__device__ __forceinline__ uint32_t valid_dword(const uint64_t* vb, int64_t b0, int64_t vbytes, bool full) {
    if (vb == nullptr) return 0xFFFFFFFFu;
    const uint8_t* b = reinterpret_cast<const uint8_t*>(vb);
    if (full) return *reinterpret_cast<const uint32_t*>(b + b0);
    uint32_t d = 0;
    for (int i = 0; i < 4; ++i)
        if (b0 + i < vbytes) d |= (uint32_t)b[b0 + i] << (8 * i);
    return d;
}

// Full tiles: the first kWherePf consumers' validity dwords of tile t are loaded together with the tile's values
// (prefetch), so the mask stores never wait on a load issued after the next tile's prefetch (vmcnt is in order).
constexpr int kWherePf = 8;

// A producer slot's WhereOut fields read once at the slot's start into wave-uniform registers: read through `wo` inside
// the tile loop, every pointer was reloaded after each mask store (a store may alias the WhereOut) and every store
// waited on that reload.
struct WhereRegs {
    const WhereOut* wo;
    int nm, bitmaps;
    const uint64_t* valid[kWherePf];
    uint64_t* mask[kWherePf];
    uint64_t* where_t;
    uint64_t* where_nn;
};
__device__ __forceinline__ WhereRegs where_regs(const WhereOut* __restrict__ wo) {
    WhereRegs r;
    r.wo = wo;
    r.nm = wo ? wo->nmasks : 0;
    r.bitmaps = wo ? wo->bitmaps : 0;
#pragma unroll
    for (int k = 0; k < kWherePf; ++k) {
        r.valid[k] = wo && k < r.nm ? wo->valid[k] : nullptr;
        r.mask[k] = wo && k < r.nm ? wo->mask[k] : nullptr;
    }
    r.where_t = wo ? wo->where_t : nullptr;
    r.where_nn = wo ? wo->where_nn : nullptr;
    return r;
}

__device__ __forceinline__ void where_prefetch(const WhereRegs& W, int64_t t, int tid, uint32_t (&vd)[kWherePf]) {
    const int64_t b0 = t * (kTileRows / 8) + tid;
#pragma unroll
    for (int k = 0; k < kWherePf; ++k) vd[k] = (k < W.nm && (tid & 3) == 0) ? valid_dword(W.valid[k], b0, 0, true) : 0u;
}

// Writes a full tile's producer outputs from the prefetched validity (stores only; consumers past kWherePf load).
__device__ __forceinline__ void where_emit_full(const WhereRegs& W, int64_t t, int tid, uint32_t w, uint32_t wn,
                                                const uint32_t (&vd)[kWherePf]) {
    const int lane = tid & 63;
    const uint32_t pw = quad_pack(w, lane);
    const uint32_t pn = quad_pack(wn, lane);
    if ((lane & 3) != 0) return;
    const int64_t b0 = t * (kTileRows / 8) + tid;
#pragma unroll
    for (int k = 0; k < kWherePf; ++k)
        if (k < W.nm) *reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(W.mask[k]) + b0) = vd[k] & pw;
    for (int m = kWherePf; m < W.nm; ++m) {  // wave-uniform, rare
        const uint32_t v = valid_dword(W.wo->valid[m], b0, 0, true);
        *reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(W.wo->mask[m]) + b0) = v & pw;
    }
    if (W.bitmaps) {
        *reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(W.where_t) + b0) = pw;
        *reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(W.where_nn) + b0) = pn;
    }
}

// Writes the producer's outputs for tile t: per consumer valid & where TRUE, and the where bitmaps if asked for.
__device__ __forceinline__ void where_emit(const WhereRegs& W, int64_t t, int tid, uint32_t w, uint32_t wn, bool full,
                                           int64_t vbytes) {
    const int lane = tid & 63;
    const uint32_t pw = quad_pack(w, lane);
    const uint32_t pn = quad_pack(wn, lane);
    if ((lane & 3) != 0) return;
    const int64_t b0 = t * (kTileRows / 8) + tid;  // this quad's first bitmap byte
    const int nm = W.nm;
    const WhereOut* __restrict__ wo = W.wo;
    // 8 consumers at a time: their validity loads are all in flight before the first store waits on one
    for (int m0 = 0; m0 < nm; m0 += 8) {  // wave-uniform
        uint32_t vd[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) vd[k] = m0 + k < nm ? valid_dword(wo->valid[m0 + k], b0, vbytes, full) : 0u;
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (m0 + k < nm) *reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(wo->mask[m0 + k]) + b0) = vd[k] & pw;
    }
    if (W.bitmaps) {
        *reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(W.where_t) + b0) = pw;
        *reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(W.where_nn) + b0) = pn;
    }
}

// FULL: every column has stats, moments, HLL and a fast fused compare, pairs have the correlation, no `where`
// (the north-star suite) — the per-flag branches compile away.
// WP (NC == 1): the slot is a `where` producer (sd.wout): its column's values and validity evaluate the filter, the
// filter masks the slot's own rows and goes out as consumer masks (where_emit).
// Minimum waves per SIMD for the north-star (FULL) instance. r06: 3 (168 VGPRs, 284 B of spills a lane) made suite10
// 21.1 -> 34.9 ms (profiles/r06/suite10_minwaves_ab_r06ak.txt); the 256-VGPR, 2-wave form stays.
#ifndef DQ_HEAVY8_MINW
#define DQ_HEAVY8_MINW 1
#endif
template <int NC, bool F0, bool F1, bool FULL, bool WP = false>
__global__ void __launch_bounds__(kBlock, FULL ? DQ_HEAVY8_MINW : 1)
scan_heavy8_kernel(const SlotDesc* __restrict__ slots, const int32_t* __restrict__ group, int ngroup, int64_t nrows,
                   int64_t ntiles, int gstride, SlotPartial* __restrict__ partials, uint8_t* __restrict__ hll_partials) {
    using A0 = typename HAccOf<F0>::type;
    using A1 = typename HAccOf<F1>::type;
    __shared__ uint32_t hll_lds[NC][kHllRegs];
    __shared__ BlockRed<NC, F0, F1> red;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int64_t G = gridDim.x;
    for (int gi = 0; gi < ngroup; ++gi) {
        const int s = group[gi];
        const SlotDesc sd = slots[s];
        const ColDesc c0 = sd.col[0];
        const ColDesc c1 = sd.col[1];
        const HeavyCol h0 = heavy_col_of(c0, F0);
        const HeavyCol h1 = heavy_col_of(c1, F1);
        const bool corr = NC > 1 && (FULL || sd.corr);
        const bool has_where = WP || (!FULL && sd.where_t != nullptr);
        const WhereOut* __restrict__ wo = sd.wout;
        const WhereRegs wr = where_regs(WP ? wo : nullptr);
        const int64_t vbytes = (nrows + 7) >> 3;
        const bool need0 = corr || h0.stats || h0.moments || c0.pred_kind != FP_NONE;
        const bool need1 = corr || h1.stats || h1.moments || c1.pred_kind != FP_NONE;
        A0 a0;
        A1 a1;
        hacc_init(a0);
        hacc_init(a1);
        CorrPartial cp;
        cp.n = cp.xa = cp.ya = cp.ck = cp.xm = cp.ym = 0.0;
        uint32_t wt = 0, wnn = 0;
        for (int i = tid; i < NC * kHllRegs; i += kBlock) (&hll_lds[0][0])[i] = 0xFFFFFFFFu;  // rank - 1 = -1
        __syncthreads();
        auto fold = [&](const uint64_t (&x)[8], const uint64_t (&y)[8], uint32_t mx, uint32_t my, uint32_t w,
                        uint32_t wn) {
            if (has_where) {
                wt += __popc(w);
                wnn += __popc(wn);
                mx &= w;
                my &= w;
            }
            uint32_t tmin = 0xFFFFFFFFu;
            double xd[8], yd[8];
            bool fx = true, fy = true;
            heavy_col_rows<F0, FULL>(a0, x, mx, h0, c0, hll_lds[0], tmin, need0, xd, fx);
            if (NC > 1) {
                heavy_col_rows<F1, FULL>(a1, y, my, h1, c1, hll_lds[NC - 1], tmin, need1, yd, fy);
                if (corr) heavy_corr_rows<F0, F1>(cp, xd, yd, mx & my, fx && fy);
            }
            if (__builtin_expect(tmin == 0u, 0)) {
                if (FULL || h0.hll) heavy_hll_exact<F0>(hll_lds[0], x, mx);
                if (NC > 1 && (FULL || h1.hll)) heavy_hll_exact<F1>(hll_lds[NC - 1], y, my);
            }
        };
        const int64_t nfull = nrows / kTileRows;
        int64_t t = blockIdx.x;
        uint64_t x[8], y[8];
        uint32_t bx = 0xFF, by = 0xFF, bw = 0xFF, bn = 0xFF;
        uint32_t vdc[WP ? kWherePf : 1], vdn[WP ? kWherePf : 1];
        if constexpr (WP) {
            if (t < nfull) where_prefetch(wr, t, tid, vdc);
        }
        if (t < nfull) {
            heavy_load(c0, t, tid, x);
            bx = heavy_bits(c0.validity, t, tid);
            if (NC > 1) {
                heavy_load(c1, t, tid, y);
                by = heavy_bits(c1.validity, t, tid);
            }
            if (has_where && !WP) {
                bw = heavy_bits(sd.where_t, t, tid);
                bn = heavy_bits(sd.where_nn, t, tid);
            }
        }
        for (; t < nfull; t += G) {
            const int64_t tn = t + G;
            uint64_t xn[8], yn[8];
            uint32_t nbx = 0xFF, nby = 0xFF, nbw = 0xFF, nbn = 0xFF;
            if constexpr (WP) {  // the filter of this tile and its mask stores go out before the next tile's loads
                const uint32_t e = where_eval8<F0>(wo->prog, x, bx, 0xFFu);
                bw = e & 0xFFu;
                bn = e >> 8;
                where_emit_full(wr, t, tid, bw, bn, vdc);
            }
            if (tn < nfull) {
                heavy_load(c0, tn, tid, xn);
                nbx = heavy_bits(c0.validity, tn, tid);
                if (NC > 1) {
                    heavy_load(c1, tn, tid, yn);
                    nby = heavy_bits(c1.validity, tn, tid);
                }
                if (has_where && !WP) {
                    nbw = heavy_bits(sd.where_t, tn, tid);
                    nbn = heavy_bits(sd.where_nn, tn, tid);
                }
                if constexpr (WP) where_prefetch(wr, tn, tid, vdn);
            }
            fold(x, y, bx, by, bw, bn);
            if constexpr (WP) {
#pragma unroll
                for (int k = 0; k < kWherePf; ++k) vdc[k] = vdn[k];
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                x[k] = xn[k];
                if (NC > 1) y[k] = yn[k];
            }
            bx = nbx;
            by = nby;
            bw = nbw;
            bn = nbn;
        }
        if (nfull < ntiles && blockIdx.x == nfull % G) {
            const uint32_t mx = heavy_tail(c0, nfull, tid, nrows, x);
            const uint32_t my = NC > 1 ? heavy_tail(c1, nfull, tid, nrows, y) : 0u;
            uint32_t w = 0, wn = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int64_t r = nfull * kTileRows + (int64_t)tid * 8 + k;
                const bool in = r < nrows;
                w |= (in ? 1u : 0u) << k;
            }
            if (WP) {
                const uint32_t e = where_eval8<F0>(wo->prog, x, mx, w);
                wn = e >> 8;
                w = e & 0xFFu;
                where_emit(wr, nfull, tid, w, wn, false, vbytes);
            } else if (has_where) {
                wn = w & heavy_bits(sd.where_nn, nfull, tid);
                w &= heavy_bits(sd.where_t, nfull, tid);
            } else {
                wn = w;
            }
            if (NC == 1) {
#pragma unroll
                for (int k = 0; k < 8; ++k) y[k] = 0;
            }
            fold(x, y, mx, my, w, wn);
        }
        // lane states -> the scan's partial structs, then the shared wave / workgroup reduction
        typename AccOf<F0>::type r0;
        typename AccOf<F1>::type r1;
        hacc_to(r0, a0);
        if (NC > 1) hacc_to(r1, a1);
        else acc_init(r1);
        int64_t lwt = wt, lwnn = wnn;
#pragma unroll 1
        for (int off = 32; off > 0; off >>= 1) {
            typename AccOf<F0>::type o0;
            acc_shfl(o0, r0, off);
            const int64_t owt = shfl_down_i64(lwt, off), ownn = shfl_down_i64(lwnn, off);
            typename AccOf<F1>::type o1;
            CorrPartial oc;
            if (NC > 1) {
                acc_shfl(o1, r1, off);
                corr_shfl(oc, cp, off);
            }
            if (lane < off) {
                acc_merge(r0, o0);
                lwt += owt;
                lwnn += ownn;
                if (NC > 1) {
                    acc_merge(r1, o1);
                    corr_merge(cp, oc);
                }
            }
        }
        if (lane == 0) {
            red.a0[wave] = r0;
            red.wt[wave] = lwt;
            red.wnn[wave] = lwnn;
            if (NC > 1) {
                red.a1[wave] = r1;
                red.cp[wave] = cp;
            }
        }
        __syncthreads();
        if (tid == 0) {
            for (int w = 1; w < kBlock / 64; ++w) {
                acc_merge(r0, red.a0[w]);
                lwt += red.wt[w];
                lwnn += red.wnn[w];
                if (NC > 1) {
                    acc_merge(r1, red.a1[w]);
                    corr_merge(cp, red.cp[w]);
                }
            }
            SlotPartial* dst = partials + (int64_t)s * gstride + blockIdx.x;
            store_partial(dst->c[0], r0);
            if (NC > 1) {
                store_partial(dst->c[1], r1);
                dst->corr = cp;
            } else {
                store_empty(dst->c[1]);
                dst->corr.n = dst->corr.xa = dst->corr.ya = dst->corr.ck = dst->corr.xm = dst->corr.ym = 0.0;
            }
            dst->wt = lwt;
            dst->wnn = lwnn;
            dst->pt = dst->pnn = dst->vt = dst->pad = 0;
        }
        for (int c = 0; c < NC; ++c) {
            const bool hl = c == 0 ? h0.hll : h1.hll;
            const int hs = c == 0 ? c0.hll_slot : c1.hll_slot;
            if (hl && hs >= 0) {
                uint8_t* dst = hll_partials + ((int64_t)hs * gstride + blockIdx.x) * kHllRegs;
                for (int i = tid; i < kHllRegs; i += kBlock) dst[i] = (uint8_t)(hll_lds[c][i] + 1u);
            }
        }
        __syncthreads();
    }
}


// Bits-only slots (Size(where), Completeness of an unread column, Compliance): one 64-row bitmap
// word per lane per step, tiles interleaved over workgroups like the value kernels.
__global__ void __launch_bounds__(kBlock)
scan_bits_kernel(const SlotDesc* __restrict__ slots, const int32_t* __restrict__ group, int ngroup, int64_t nrows,
                 int64_t ntiles, int gstride, SlotPartial* __restrict__ partials) {
    __shared__ SlotPartial red[kBlock / 64];
    (void)ntiles;
    const int64_t nwords_total = (nrows + 63) >> 6;
    for (int gi = 0; gi < ngroup; ++gi) {
        const int s = group[gi];
        const SlotDesc sd = slots[s];
        const uint8_t* vb = reinterpret_cast<const uint8_t*>(sd.bits_valid);
        SlotPartial acc;
        slot_init(acc);
        // every lane of the grid takes bitmap words in turn (a 2048-row tile is only 32 words: a tile per workgroup
        // left 7 of its 8 waves idle)
        for (int64_t w = (int64_t)blockIdx.x * kBlock + threadIdx.x; w < nwords_total; w += (int64_t)gridDim.x * kBlock) {
            {
                const int64_t base = w << 6;
                const int64_t nin = nrows - base;
                const uint64_t range = nin >= 64 ? ~0ull : ((1ull << nin) - 1ull);
                const uint64_t wtb = sd.where_t ? sd.where_t[w] : range;
                const uint64_t wnb = sd.where_t ? sd.where_nn[w] : range;
                acc.wt += __popcll(wtb);
                acc.wnn += __popcll(wnb);
                if (sd.pred_t) {
                    acc.pt += __popcll(wtb & sd.pred_t[w]);
                    acc.pnn += __popcll(wtb & sd.pred_nn[w]);
                }
                if (vb) {
                    uint64_t vw;
                    if (nin >= 64) {
                        vw = sd.bits_valid[w];
                    } else {
                        vw = 0;
                        for (int64_t b = 0; b < (nin + 7) / 8; ++b) vw |= (uint64_t)vb[(base >> 3) + b] << (8 * b);
                        vw &= range;
                    }
                    acc.vt += __popcll(wtb & vw);
                }
            }
        }
        block_reduce_slot(acc, red, 1, false);
        if (threadIdx.x == 0) partials[(int64_t)s * gstride + blockIdx.x] = acc;
    }
}

// Folds each slot's workgroup partials in a fixed order.
__global__ void __launch_bounds__(kBlock)
reduce_partials_kernel(const SlotPartial* __restrict__ partials, const int32_t* __restrict__ nblocks_of,
                       int gstride, SlotPartial* __restrict__ finals) {
    __shared__ SlotPartial red[kBlock / 64];
    const int s = blockIdx.x;
    const int nb = nblocks_of[s];
    SlotPartial acc;
    slot_init(acc);
    for (int b = threadIdx.x; b < nb; b += kBlock) slot_merge(acc, partials[(int64_t)s * gstride + b]);
    block_reduce_slot(acc, red, 2, true);
    if (threadIdx.x == 0) finals[s] = acc;
}

__global__ void __launch_bounds__(kHllRegs)
reduce_hll_kernel(const uint8_t* __restrict__ hll_partials, const int32_t* __restrict__ nblocks_of, int gstride,
                  uint8_t* __restrict__ hll_final) {
    const int h = blockIdx.x;
    const int r = threadIdx.x;
    const int nb = nblocks_of[h];
    uint32_t m = 0;
    for (int b = 0; b < nb; ++b) {
        const uint32_t v = hll_partials[((int64_t)h * gstride + b) * kHllRegs + r];
        m = v > m ? v : m;
    }
    hll_final[(int64_t)h * kHllRegs + r] = (uint8_t)m;
}

__device__ __forceinline__ double pow10i(int scale) {
    double d = 1.0;
    for (int i = 0; i < scale; ++i) d *= 10.0;
    return d;
}

// Builds each op's dq_state from its slot (fromAggregationResult + ifNoNullsIn of every analyzer).
__global__ void finalize_kernel(const OpMap* __restrict__ ops, int nops, const SlotPartial* __restrict__ finals,
                                const uint8_t* __restrict__ hll_final, dq_state* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nops) return;
    const OpMap om = ops[i];
    dq_state* st = out + i;
    for (int w = 0; w < DQ_HLL_NUM_WORDS; ++w) st->u.hll.words[w] = 0;
    st->kind = om.kind;
    int present = 0;
    SlotPartial sp;
    if (om.slot >= 0) sp = finals[om.slot];
    else slot_init(sp);
    const ColPartial& c = sp.c[om.colpos > 0 ? 1 : 0];
    // conditionalCount(where) (A/Analyzer.scala:426-432): count(*), or sum(cast(where AS long)),
    // which is NULL when no row has a non-null `where` value.
    // The where counts live in the op's own slot, or in the slot of the filter's producer (masked `where`).
    int64_t wt = sp.wt, wnn = sp.wnn;
    if (om.has_where && om.wslot >= 0 && om.wslot != om.slot) {
        wt = finals[om.wslot].wt;
        wnn = finals[om.wslot].wnn;
    }
    const int64_t cond_count = om.has_where ? wt : om.nrows;
    const bool cond_count_present = om.has_where ? (wnn > 0) : true;
    const double scale = om.decimal_scale > 0 ? pow10i(om.decimal_scale) : 1.0;
    switch (om.kind) {
        case DQ_OP_SIZE:
            st->u.num_matches.num_matches = cond_count;
            present = cond_count_present;
            break;
        case DQ_OP_COMPLETENESS: {
            // sum(cast(isNotNull(when(where, col)) AS int)): NULL only over zero rows.
            const int64_t matches = om.from_bits == 1 ? sp.vt : (om.from_bits == 2 ? cond_count : c.n);
            st->u.num_matches_and_count.num_matches = matches;
            st->u.num_matches_and_count.count = cond_count;
            present = (om.nrows > 0) && cond_count_present;
            break;
        }
        case DQ_OP_COMPLIANCE:
            // sum(cast(when(where, pred) AS int)): NULL when no row has where TRUE and pred non-null.
            // Fused `col <op> const` (from_bits == 3): pred is non-null exactly where col is.
            st->u.num_matches_and_count.num_matches = om.from_bits == 3 ? c.pt : sp.pt;
            st->u.num_matches_and_count.count = cond_count;
            present = (om.from_bits == 3 ? c.n > 0 : sp.pnn > 0) && cond_count_present;
            break;
        case DQ_OP_MEAN:
            st->u.mean.sum = om.is_float ? c.dsum : (double)c.isum / scale;
            st->u.mean.count = c.n;
            st->u.mean.isum = c.isum;
            st->u.mean.exact = (!om.is_float && om.decimal_scale == 0) ? 1 : 0;
            present = c.n > 0;
            break;
        case DQ_OP_SUM:
            st->u.dbl.value = om.is_float ? c.dsum : (double)c.isum / scale;
            st->u.dbl.isum = c.isum;
            st->u.dbl.exact = (!om.is_float && om.decimal_scale == 0) ? 1 : 0;
            present = c.n > 0;
            break;
        case DQ_OP_MINIMUM:
            if (om.is_float) st->u.dbl.value = (c.nnan == c.n) ? NAN : c.dmin;
            else st->u.dbl.value = (double)c.imin / scale;
            present = c.n > 0;
            break;
        case DQ_OP_MAXIMUM:
            if (om.is_float) st->u.dbl.value = (c.nnan > 0) ? NAN : c.dmax;
            else st->u.dbl.value = (double)c.imax / scale;
            present = c.n > 0;
            break;
        case DQ_OP_STANDARD_DEVIATION:
            st->u.stddev.n = (double)c.n;
            st->u.stddev.avg = c.mean / scale;
            st->u.stddev.m2 = c.m2 / (scale * scale);
            present = c.n > 0;
            break;
        case DQ_OP_CORRELATION:
            st->u.corr.n = sp.corr.n;
            st->u.corr.x_avg = om.colpos ? sp.corr.ya : sp.corr.xa;
            st->u.corr.y_avg = om.colpos ? sp.corr.xa : sp.corr.ya;
            st->u.corr.ck = sp.corr.ck;
            st->u.corr.x_mk = om.colpos ? sp.corr.ym : sp.corr.xm;
            st->u.corr.y_mk = om.colpos ? sp.corr.xm : sp.corr.ym;
            present = sp.corr.n > 0.0;
            break;
        case DQ_OP_APPROX_COUNT_DISTINCT: {
            // 6-bit registers, 10 per word, LSB first (C/StatefulHyperloglogPlus.scala:99-109).
            const uint8_t* regs = hll_final + (int64_t)om.hll_slot * kHllRegs;
            for (int w = 0; w < DQ_HLL_NUM_WORDS; ++w) {
                uint64_t word = 0;
                for (int k = 0; k < 10; ++k) {
                    const int idx = w * 10 + k;
                    if (idx < kHllRegs) word |= (uint64_t)(regs[idx] & 63u) << (6 * k);
                }
                st->u.hll.words[w] = (int64_t)word;
            }
            present = 1;  // the HLL aggregate is never null (nullable = false)
            break;
        }
        default:
            break;
    }
    st->present = present;
}

// ------------------------------------------------------------------------------------------------
// Launchers
// ------------------------------------------------------------------------------------------------
template <int P, int NC, bool F0, bool F1>
static const void* values_kernel_ptr(int heavy) {
    return heavy ? reinterpret_cast<const void*>(&scan_values_kernel<P, NC, F0, F1, true>)
                 : reinterpret_cast<const void*>(&scan_values_kernel<P, NC, F0, F1, false>);
}

static const void* values_kernel_for(int P, int nc, bool f0, bool f1, int heavy) {
    // 8-byte columns: HEAVY slots and Correlation pairs take the lean kernel (heavy == 2: every flag on, no `where`);
    // the striped kernel's pair instantiation runs at 1 wave / SIMD (255 VGPRs), this one at 2
    if (heavy == 3) {  // `where` producer over one 8-byte column
        if (P != 2 || nc != 1 || f1) return nullptr;
        return f0 ? reinterpret_cast<const void*>(&scan_heavy8_kernel<1, true, false, false, true>)
                  : reinterpret_cast<const void*>(&scan_heavy8_kernel<1, false, false, false, true>);
    }
    if ((heavy || nc == 2) && P == 2) {
#define DQ_HK(n, a, b) \
    if (nc == n && f0 == a && f1 == b) \
        return heavy == 2 ? reinterpret_cast<const void*>(&scan_heavy8_kernel<n, a, b, true>) \
                          : reinterpret_cast<const void*>(&scan_heavy8_kernel<n, a, b, false>);
        DQ_HK(1, false, false) DQ_HK(1, true, false)
        DQ_HK(2, false, false) DQ_HK(2, false, true) DQ_HK(2, true, false) DQ_HK(2, true, true)
#undef DQ_HK
    }
#define DQ_VK(p, n, a, b) \
    if (P == p && nc == n && f0 == a && f1 == b) return values_kernel_ptr<p, n, a, b>(heavy);
    // P = 2 (8-byte elements): HEAVY slots went to scan_heavy8_kernel above
#define DQ_VK2(n, a, b) \
    if (P == 2 && nc == n && f0 == a && f1 == b) return reinterpret_cast<const void*>(&scan_values_kernel<2, n, a, b, false>);
    DQ_VK2(1, false, false) DQ_VK2(1, true, false)
    DQ_VK2(2, false, false) DQ_VK2(2, false, true) DQ_VK2(2, true, false) DQ_VK2(2, true, true)
#undef DQ_VK2
    DQ_VK(4, 1, false, false) DQ_VK(4, 1, true, false)
    DQ_VK(8, 1, false, false) DQ_VK(8, 1, true, false)
    DQ_VK(4, 2, false, false) DQ_VK(4, 2, false, true) DQ_VK(4, 2, true, false) DQ_VK(4, 2, true, true)
    DQ_VK(8, 2, false, false) DQ_VK(8, 2, false, true) DQ_VK(8, 2, true, false) DQ_VK(8, 2, true, true)
#undef DQ_VK
    return nullptr;
}

int scan_group_blocks_per_cu(int kind, int P, int nc, bool f0, bool f1, int heavy) {
    const void* k = kind == SK_BITS ? reinterpret_cast<const void*>(&scan_bits_kernel) : values_kernel_for(P, nc, f0, f1, heavy);
    if (!k) return 0;
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, kBlock, 0) != hipSuccess || n <= 0) n = 1;
    return n;
}

int launch_scan_group(int kind, int P, int nc, bool f0, bool f1, int heavy, const SlotDesc* slots, const int32_t* group,
                      int ngroup, int64_t nrows, int64_t ntiles, int gstride, int grid, SlotPartial* partials,
                      uint8_t* hll_partials, hipStream_t s) {
    if (kind == SK_BITS) {
        hipLaunchKernelGGL(scan_bits_kernel, dim3(grid), dim3(kBlock), 0, s, slots, group, ngroup, nrows, ntiles,
                           gstride, partials);
        return 0;
    }
    const void* k = values_kernel_for(P, nc, f0, f1, heavy);
    if (!k) return -1;
    void* args[] = {(void*)&slots, (void*)&group, (void*)&ngroup, (void*)&nrows, (void*)&ntiles,
                    (void*)&gstride, (void*)&partials, (void*)&hll_partials};
    return hipLaunchKernel(k, dim3(grid), dim3(kBlock), args, 0, s) == hipSuccess ? 0 : -1;
}

void launch_reduce_partials(const SlotPartial* partials, const int32_t* nblocks_of, int nslots, int gstride,
                            SlotPartial* finals, hipStream_t s) {
    hipLaunchKernelGGL(reduce_partials_kernel, dim3(nslots), dim3(kBlock), 0, s, partials, nblocks_of, gstride, finals);
}

void launch_reduce_hll(const uint8_t* hll_partials, const int32_t* nblocks_of, int nhll, int gstride,
                       uint8_t* hll_final, hipStream_t s) {
    if (nhll == 0) return;
    hipLaunchKernelGGL(reduce_hll_kernel, dim3(nhll), dim3(kHllRegs), 0, s, hll_partials, nblocks_of, gstride,
                       hll_final);
}

void launch_finalize(const OpMap* ops, int nops, const SlotPartial* finals, const uint8_t* hll_final,
                     dq_state* out, hipStream_t s) {
    const int tb = 64;
    hipLaunchKernelGGL(finalize_kernel, dim3((nops + tb - 1) / tb), dim3(tb), 0, s, ops, nops, finals, hll_final,
                       out);
}

}  // namespace dq
