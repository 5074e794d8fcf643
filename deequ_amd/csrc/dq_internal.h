// dq_internal.h — layouts shared by the host runtime (dq_api.cpp) and the HIP kernels.
//
// The fused scan works on "slots". A slot is one pass over one or two columns (two for a
// Correlation pair) under one `where` mask, or a bits-only pass over validity/predicate bitmaps
// (Size(where), Completeness of an otherwise unread column, Compliance). Every op of the batch
// is answered from the final slot partial it maps to (OpMap), so every column is read once.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dq.h"

namespace dq {

constexpr int kBlock = 256;          // threads per workgroup (4 wave64)
constexpr int kRowsPerThread = 8;    // rows per thread per tile
constexpr int kTileRows = kBlock * kRowsPerThread;  // 2048 rows = 32 bitmap words per tile
constexpr int kMaxSlots = 256;
constexpr int kHllRegs = 512;

// Element storage classes of the fused scan.
enum ElemType : int32_t {
    ET_U8 = 0,   // BOOLEAN
    ET_I8 = 1,   // BYTE
    ET_I16 = 2,  // SHORT
    ET_I32 = 3,  // INT, DATE
    ET_I64 = 4,  // LONG, TIMESTAMP, DECIMAL (unscaled)
    ET_F32 = 5,  // FLOAT
    ET_F64 = 6,  // DOUBLE
    ET_NONE = 7
};

enum ColFlags : uint32_t {
    CF_STATS = 1u,    // count/sum/min/max (+ NaN count)
    CF_MOMENTS = 2u,  // (n, avg, m2) Welford/Chan state
    CF_HLL = 4u,      // HLL++ registers
};

// Row mapping inside a 2048-row tile: L loads of P consecutive rows per thread, L * P = 8.
// Striped (coalesced) for a single element size; pairs of different sizes use P = 8.
// A Compliance predicate `column <op> constant` evaluated inside the value scan (no extra pass).
enum FusedPredKind : int32_t { FP_NONE = 0, FP_LONG = 1, FP_DOUBLE = 2 };

struct ColDesc {
    const void* values;
    const uint64_t* validity;  // nullptr = all valid
    int32_t spark_type;
    int32_t elem;              // ElemType
    uint32_t flags;            // ColFlags
    int32_t hll_slot;          // index into the HLL partial arrays, -1 = none
    int32_t pred_op;           // dq_pred_opcode DQ_P_EQ..DQ_P_GE of the fused predicate
    int32_t pred_kind;         // FusedPredKind
    int64_t pred_i;            // constant (FP_LONG)
    double pred_d;             // constant (FP_DOUBLE)
};

enum SlotKind : int32_t {
    SK_VALUES = 0,
    SK_BITS = 1,
    SK_WHERE = 2,  // holds the TRUE / NOT-NULL row counts of a `where` evaluated by where_masks_kernel (not a scan launch)
};

struct WhereOut;

struct SlotDesc {
    ColDesc col[2];
    const uint64_t* where_t;   // where evaluated TRUE   (padded bitmap) or nullptr
    const uint64_t* where_nn;  // where evaluated NOT NULL
    const uint64_t* pred_t;    // SK_BITS: predicate TRUE, or nullptr
    const uint64_t* pred_nn;   // SK_BITS: predicate NOT NULL
    const uint64_t* bits_valid;// SK_BITS: validity to count (Completeness), nullptr = none
    int32_t kind;              // SlotKind
    int32_t ncols;             // SK_VALUES: 1 or 2
    int32_t corr;              // compute CorrelationState of (col0, col1)
    int32_t rows_per_load;     // P: 2, 4 or 8
    const WhereOut* wout;      // where producer: this slot's scan evaluates a `where` from col[0] (scan_heavy8_kernel)
};

struct ColPartial {
    int64_t n;     // valid & where-true rows
    int64_t nnan;  // of which NaN (floating columns)
    int64_t isum;  // integral sum (Spark LongType wrap-around)
    int64_t imin, imax;
    double dsum;
    double dmin, dmax;  // NaN-free min/max (NaN handled through nnan, Spark orders NaN largest)
    double mean, m2;    // Welford/Chan state over the same rows (n)
    int64_t pt;         // rows of n where the fused predicate is TRUE
    int64_t pad;
};

struct CorrPartial {
    double n, xa, ya, ck, xm, ym;
};

struct SlotPartial {
    ColPartial c[2];
    CorrPartial corr;
    int64_t wt;    // rows with where TRUE (or all rows if no where)
    int64_t wnn;   // rows with where NOT NULL
    int64_t pt;    // SK_BITS: rows with where TRUE and predicate TRUE
    int64_t pnn;   // SK_BITS: rows with where TRUE and predicate NOT NULL
    int64_t vt;    // SK_BITS: rows with where TRUE and bits_valid set
    int64_t pad;
};

// How each op is answered from a final slot partial.
struct OpMap {
    int32_t kind;        // dq_op_kind
    int32_t slot;        // slot index
    int32_t colpos;      // 0/1 inside the slot
    int32_t has_where;
    int32_t is_float;    // column is FLOAT/DOUBLE
    int32_t hll_slot;    // ApproxCountDistinct register set
    int32_t decimal_scale;
    int32_t from_bits;   // Completeness answered from a bits-only slot (vt) instead of c[colpos].n
    int32_t wslot;       // slot whose wt / wnn are the op's conditionalCount (its `where`); -1 = no where
    int32_t pad;
    int64_t nrows;       // count(*) of the batch
};

// String-shaped ops (strings.hip): one slot per (column, where).
enum StrFlags : uint32_t {
    SF_LEN = 1u,    // MinLength / MaxLength (UTF-8 characters)
    SF_DTYPE = 2u,  // DataType histogram
    SF_HLL = 4u,    // ApproxCountDistinct over UTF-8 bytes
};

struct StrSlot {
    const uint8_t* data;       // STRING: UTF-8 bytes (4-byte aligned, >= 16 readable bytes past the end)
    const int32_t* offsets;    // STRING: nrows + 1 offsets
    const void* values;        // fixed width (DataType of a non-string column)
    const uint64_t* validity;  // nullptr = all valid
    const uint64_t* where_t;   // where TRUE (padded bitmap) or nullptr
    int32_t spark_type;
    int32_t decimal_scale;
    uint32_t flags;            // StrFlags
    int32_t hll_slot;          // shared numbering with the fixed-width HLL partials, -1 = none
};

struct StrPartial {
    int64_t n;                 // rows with the value non-NULL and where TRUE
    int64_t minlen, maxlen;
    int64_t dt[5];             // DataType classes (index 0 unused: NULLs are derived)
};

struct StrOpMap {
    int32_t op;                // index into the dq_state output
    int32_t kind;              // DQ_OP_MIN_LENGTH / DQ_OP_MAX_LENGTH / DQ_OP_DATATYPE
    int32_t slot;
    int32_t pad;
};

// Predicate VM limits.
constexpr int kPredStack = 16;

struct PredColumn {
    const void* values;
    const uint64_t* validity;
    const int32_t* offsets;
    int32_t spark_type;
    int32_t elem;
    int32_t decimal_scale;
    int32_t pad;
};

struct PredProgram {
    const int32_t* code;
    const dq_const* consts;
    const uint8_t* strings;
    int32_t code_len;
    int32_t n_consts;
};

// A predicate that is a boolean combination (AND / OR / NOT) of leaves `column <op> constant` and `column IS [NOT]
// NULL` over fixed-width numeric columns (IN lists of constants become OR chains of `=`): each leaf is evaluated into
// a (TRUE, NOT-NULL) bit pair per row and the combination runs on a per-lane bit stack, all in registers
// (pred_simple_kernel). Everything else runs on the general VM (predicate_kernel).
constexpr int kPredTerms = 16;
constexpr int kPredBCode = 64;
constexpr int8_t kPB_AND = -1, kPB_OR = -2, kPB_NOT = -3;
struct PredTerm {
    int32_t col;
    int32_t op;   // DQ_P_EQ..DQ_P_GE, DQ_P_IS_NULL, DQ_P_IS_NOT_NULL
    int32_t dbl;  // compare as double (Spark NaN ordering) instead of as long
    int32_t pad;
    int64_t ci;
    double cd;
};
struct PredSimple {
    int32_t nterms;
    int32_t nb;
    PredTerm t[kPredTerms];
    int8_t b[kPredBCode];  // postfix: >= 0 pushes term b[i]; kPB_AND / kPB_OR / kPB_NOT
};

// A `where` evaluated inside the scan (simple predicates): instead of TRUE / NOT-NULL bitmaps that every
// slot under the filter re-reads and pop-counts, the producer writes one mask per consumer column, valid & where TRUE,
// which that column's scan then reads in place of its validity (running the no-`where` kernels). The producer is the
// scan of the filter's own column when the filter reads only that 8-byte column (scan_heavy8_kernel, WP) or else a
// pass of its own (where_masks_kernel); either also counts the TRUE / NOT-NULL rows (conditionalCount) into a slot
// partial, and writes the bitmaps only when bits / string slots read them.
constexpr int kWhereMasks = 32;
constexpr int kWhereStack = 8;  // fused producer: 8-row bytes on a 64-bit stack
struct WhereOut {
    PredSimple prog;                      // fused producer: every term's column is the slot's col[0]
    int32_t nmasks;
    int32_t bitmaps;                      // 1: write where_t / where_nn
    uint64_t* where_t;                    // padded bitmaps (pwords words)
    uint64_t* where_nn;
    const uint64_t* valid[kWhereMasks];   // consumer column validity (nullptr = all valid; exactly ceil(nrows/8) bytes)
    uint64_t* mask[kWhereMasks];          // out: valid & where TRUE, padded bitmap
};

inline int elem_of(int32_t spark_type) {
    switch (spark_type) {
        case DQ_TYPE_BOOLEAN: return ET_U8;
        case DQ_TYPE_BYTE: return ET_I8;
        case DQ_TYPE_SHORT: return ET_I16;
        case DQ_TYPE_INT:
        case DQ_TYPE_DATE: return ET_I32;
        case DQ_TYPE_LONG:
        case DQ_TYPE_TIMESTAMP:
        case DQ_TYPE_DECIMAL: return ET_I64;
        case DQ_TYPE_FLOAT: return ET_F32;
        case DQ_TYPE_DOUBLE: return ET_F64;
        default: return ET_NONE;
    }
}
inline int elem_size(int e) {
    switch (e) {
        case ET_U8: case ET_I8: return 1;
        case ET_I16: return 2;
        case ET_I32: case ET_F32: return 4;
        case ET_I64: case ET_F64: return 8;
        default: return 0;
    }
}
inline int rows_per_load_of(int e) {
    int s = elem_size(e);
    return s == 8 ? 2 : (s == 4 ? 4 : 8);
}

}  // namespace dq

#ifdef __cplusplus
#include <map>
#include <mutex>
#include <string>
#include <vector>
// The context behind the C-ABI. A single-device context owns one stream, a device arena and pinned staging;
// a multi-device context (dq_open_devices) owns one single-device sub-context per GPU and, when the devices
// are distinct, one RCCL communicator per GPU for the frequency-table exchange.
struct dq_ctx {
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    std::string err;
    // Device arena, re-used by every call (grown outside of any timed/captured region).
    uint8_t* arena = nullptr;
    size_t arena_cap = 0;
    // Pinned host staging for plan uploads and state downloads.
    uint8_t* pinned = nullptr;
    size_t pinned_cap = 0;
    int cus = 256;
    // Side streams: scan launches of different shapes (and the string scan) run concurrently, forked from and
    // joined back to `stream` by events, so a VALU-heavy shape shares the CUs with a memory-bound one.
    int hip_priority = 0;  // HIP stream priority of own_stream and the side streams (dq_set_priority)
    static constexpr int kSide = 3;
    hipStream_t side[kSide] = {};
    hipEvent_t fork_ev = nullptr;
    hipEvent_t join_ev[kSide] = {};
    std::map<int, int> occupancy;  // launch shape -> workgroups per CU
    int64_t scan_launches = 0;
    int64_t kernel_launches[DQ_KERNEL_COUNT] = {};  // by dq_scan_kernel
    int64_t freq_paths[DQ_FREQ_PATH_COUNT] = {};     // by dq_freq_path
    // Released device scratch of the grouping builds (multi-GB partition buffers and tables), re-used in stream
    // order instead of a hipMalloc / hipFree pair per call; bounded, freed at dq_close and on allocation failure.
    struct CachedBlock {
        void* ptr;
        size_t bytes;
        hipStream_t stream;  // the stream of its last use
    };
    std::vector<CachedBlock> scratch_free;  // guarded by scratch_mu: a table may be freed from another thread
    size_t scratch_cached = 0;
    std::mutex scratch_mu;
    // multi-device
    std::vector<dq_ctx*> subs;   // one per device (empty: single-device context)
    std::vector<int> devices;
    void* comms = nullptr;       // ncclComm_t[ndev] when the devices are distinct, else nullptr (copy transport)
};
#endif

namespace dq {

// Cached device scratch (see dq_ctx::scratch_free): a block of >= bytes (best fit, at most twice the request)
// or a new hipMalloc; nullptr when the device is out of memory even after the cache was released.
void* scratch_alloc(dq_ctx* ctx, size_t bytes);
// Hand a block back to the cache (its last use was queued on the ctx stream).
void scratch_release(dq_ctx* ctx, void* ptr, size_t bytes);
// Release the cached blocks beyond keep_bytes (oldest first).
void scratch_trim(dq_ctx* ctx, size_t keep_bytes = 0);

// Context accessors for the .hip translation units (dq_api.cpp).
hipStream_t ctx_stream(dq_ctx* ctx);
int ctx_device(dq_ctx* ctx);
int ctx_fail(dq_ctx* ctx, int code, const char* msg);
int ctx_cus(dq_ctx* ctx);
int ctx_num_subs(dq_ctx* ctx);       // devices of a multi-device context (dq_open_devices), 0 for a single-device one
dq_ctx* ctx_sub(dq_ctx* ctx, int i);  // the single-device context of device i of a multi-device one

// Multi-device orchestration (multi.cpp).
int multi_scan(dq_ctx* ctx, const dq_column* const* shard_columns, const int64_t* shard_rows, int ncols,
               const dq_op* ops, int nops, const dq_predicate* preds, int npreds, dq_state* out);
// Row bounds of shard i of n rows over ndev devices (contiguous, 2048-row aligned).
void shard_bounds(int64_t nrows, int ndev, int i, int64_t* row0, int64_t* count);
// Host columns -> per-shard column views (string offsets rebased into `scratch`).
void shard_columns(const dq_column* columns, int ncols, int64_t row0, int64_t count, dq_column* out,
                   std::vector<std::vector<int32_t>>& scratch);
void close_subs(dq_ctx* ctx);
// Run fn(i, sub) on every device of a multi-device context concurrently; returns the first error.
int for_each_device(dq_ctx* ctx, int (*fn)(int, dq_ctx*, void*), void* arg);
// All-to-all of int64 records between the devices of a multi-device context: send[i] holds, for every
// destination j, counts[i * ndev + j] records starting at send_off[i * ndev + j]; recv[j] receives them
// ordered by source device at recv_off[j * ndev + i]. RCCL (ncclSend / ncclRecv in one group) when the
// devices are distinct, device-to-device copies when a device repeats.
int exchange_i64(dq_ctx* ctx, const std::vector<int64_t*>& send, const std::vector<int64_t*>& recv,
                 const std::vector<int64_t>& counts, const std::vector<int64_t>& send_off,
                 const std::vector<int64_t>& recv_off);

// Kernel launchers (defined in the .hip files).
// One launch per slot shape (kind, P, column count, float/integral storage); each launch walks its
// slots with tiles interleaved over `grid` workgroups and writes partials[slot * gstride + block].
int launch_scan_group(int kind, int P, int nc, bool f0, bool f1, int heavy, const SlotDesc* slots,
                      const int32_t* group, int ngroup, int64_t nrows, int64_t ntiles, int gstride, int grid,
                      SlotPartial* partials, uint8_t* hll_partials, hipStream_t s);
int scan_group_blocks_per_cu(int kind, int P, int nc, bool f0, bool f1, int heavy);
void launch_reduce_partials(const SlotPartial* partials, const int32_t* nblocks_of, int nslots, int gstride,
                            SlotPartial* finals, hipStream_t s);
void launch_reduce_hll(const uint8_t* hll_partials, const int32_t* nblocks_of, int nhll, int gstride,
                       uint8_t* hll_final, hipStream_t s);
void launch_finalize(const OpMap* ops, int nops, const SlotPartial* finals, const uint8_t* hll_final,
                     dq_state* out, hipStream_t s);
void launch_pred_simple(const PredSimple& prog, const PredColumn* cols_dev, int64_t nrows, int64_t padded_words,
                        uint64_t* out_t, uint64_t* out_nn, hipStream_t s);
// Standalone `where` producer: masks / bitmaps of WhereOut (its terms' columns index cols_dev) and per-block row
// counts into partials[wslot * gstride + block] for `grid` blocks.
void launch_where_masks(const WhereOut* wo_dev, const PredSimple& prog, const PredColumn* cols_dev, int64_t nrows,
                        int64_t padded_words, SlotPartial* partials, int wslot, int gstride, int grid, hipStream_t s);
// rx: the program holds RLIKE (the kernel variant with the regex engine; a value past its backtracking budget sets
// *status).
void launch_predicate(const PredProgram* prog_dev, bool rx, int32_t* status, const PredColumn* cols_dev, int64_t nrows,
                      int64_t padded_words, uint64_t* out_t, uint64_t* out_nn, hipStream_t s);
int string_scan_grid(int cus, int64_t nrows);
void launch_string_scan(const StrSlot* slots, int nslots, int64_t nrows, int grid, int gstride, StrPartial* partials,
                        uint8_t* hll_partials, hipStream_t s);
void launch_finalize_strings(const StrOpMap* ops, int nops, const StrPartial* partials, int nblocks, int gstride,
                             int64_t nrows, dq_state* out, hipStream_t s);
void launch_regex(const PredColumn& col, const int32_t* image_dev, int64_t nrows, int64_t padded_words,
                  uint64_t* out_t, uint64_t* out_nn, int32_t* status, hipStream_t s);
void launch_synth_column(int kind, uint64_t seed, int64_t row0, int64_t nrows, void* out, hipStream_t s);
void launch_synth_freq_keys(int64_t total, int64_t distinct, int64_t row0, int64_t nrows, int64_t* out, hipStream_t s);
void launch_synth_string_lengths(int kind, uint64_t seed, int64_t row0, int64_t nrows, int32_t* lens, hipStream_t s);
void launch_synth_string_bytes(int kind, uint64_t seed, int64_t row0, int64_t nrows, const int32_t* offsets, void* bytes,
                               hipStream_t s);
void launch_synth_validity(uint64_t seed, int64_t row0, int64_t nrows, int permille, uint8_t* out,
                           hipStream_t s);

}  // namespace dq
