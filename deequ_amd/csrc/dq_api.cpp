// dq_api.cpp — host runtime behind include/dq.h.
//
// Plans a batch of deequ ops into fused-scan slots (one HBM read per column), evaluates `where`
// / Compliance predicates into bitmaps, launches the kernels on the context's stream and turns
// the final slot partials into per-op states. Mirrors, per entry point:
//   dq_scan            runScanningAnalyzers            R/AnalysisRunner.scala:289-336
//   dq_state_merge     State.sum / Analyzers.merge     A/Analyzer.scala:367-386 (+ each state's sum)
//   dq_hll_count       DeequHyperLogLogPlusPlusUtils   C/StatefulHyperloglogPlus.scala:210-298
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <string>
#include <tuple>
#include <vector>
#include <vector>

#include "dq_common.h"
#include "dq_internal.h"

#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

namespace {
// DQ_SEGV_TRACE=1: a host-side fault of the library prints its native backtrace (addresses into libdq.so, resolved
// with addr2line against the same build) before the process dies -- the host code's equivalent of a GPU printf.
void dq_segv_trace(int sig) {
    void* frames[64];
    const int n = backtrace(frames, 64);
    const char msg[] = "[dq] fatal signal, native backtrace:\n";
    (void)!write(2, msg, sizeof(msg) - 1);
    backtrace_symbols_fd(frames, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}
struct DqSegvTrace {
    DqSegvTrace() {
        if (getenv("DQ_SEGV_TRACE")) signal(SIGSEGV, dq_segv_trace);
    }
} dq_segv_trace_init;
}  // namespace


using namespace dq;


namespace {

int fail(dq_ctx* ctx, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    if (ctx) ctx->err = buf;
    return code;
}

#define DQ_HIP(ctx, expr)                                                                         \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess)                                                                     \
            return fail((ctx), DQ_ERR_DEVICE, "%s failed: %s", #expr, hipGetErrorString(e_));     \
    } while (0)

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// DQ_PRED_VM=1: every predicate on the general VM (A/B and cross-checks of the simple-predicate kernel).
bool pred_vm_forced() {
    const char* e = getenv("DQ_PRED_VM");
    return e && e[0] == '1';
}

// DQ_SCAN_CONCURRENT=1: the scan's launch shapes run concurrently on side streams (read per call).
bool scan_concurrency() {
    const char* e = getenv("DQ_SCAN_CONCURRENT");
    return e && e[0] == '1';
}

// Recognises the predicates pred_simple_kernel evaluates (see PredSimple): a symbolic run of the postfix program.
bool compile_simple_predicate(const dq_predicate& pr, const dq_column* columns, int ncols, PredSimple& out) {
    memset(&out, 0, sizeof(out));
    enum { E_COL, E_CONST, E_BOOL };
    struct Ent { int kind, idx; bool neg = false; };  // neg: a constant under unary minus (`x < -1`)
    std::vector<Ent> st;
    auto fixed_numeric = [&](int c) {
        if (c < 0 || c >= ncols) return false;
        switch (columns[c].spark_type) {
            case DQ_TYPE_BOOLEAN: case DQ_TYPE_BYTE: case DQ_TYPE_SHORT: case DQ_TYPE_INT: case DQ_TYPE_DATE:
            case DQ_TYPE_LONG: case DQ_TYPE_TIMESTAMP: case DQ_TYPE_FLOAT: case DQ_TYPE_DOUBLE: return true;
            default: return false;
        }
    };
    auto emit = [&](int b) {
        if (out.nb >= kPredBCode) return false;
        out.b[out.nb++] = (int8_t)b;
        return true;
    };
    auto term = [&](int col, int op, int k, bool neg = false) -> int {  // k: constant index, or -1 for IS [NOT] NULL
        if (out.nterms >= kPredTerms) return -1;
        PredTerm& q = out.t[out.nterms];
        q.col = col;
        q.op = op;
        if (k >= 0) {
            const dq_const& c = pr.consts[k];
            const int ty = columns[col].spark_type;
            q.dbl = (ty == DQ_TYPE_FLOAT || ty == DQ_TYPE_DOUBLE || c.tag == DQ_V_DOUBLE) ? 1 : 0;
            // Spark's UnaryMinus on a literal: a Long negates with wrap-around, a Double flips its sign
            q.ci = neg ? (int64_t)(0ull - (uint64_t)c.i64) : c.i64;
            q.cd = c.tag == DQ_V_DOUBLE ? (neg ? -c.f64 : c.f64) : (double)q.ci;
        }
        return out.nterms++;
    };
    auto flip = [](int op) {
        switch (op) {
            case DQ_P_LT: return (int)DQ_P_GT;
            case DQ_P_LE: return (int)DQ_P_GE;
            case DQ_P_GT: return (int)DQ_P_LT;
            case DQ_P_GE: return (int)DQ_P_LE;
            default: return op;
        }
    };
    auto const_ok = [&](int k) {
        if (k < 0 || k >= pr.n_consts) return false;
        const int tag = pr.consts[k].tag;
        return tag == DQ_V_BOOL || tag == DQ_V_LONG || tag == DQ_V_DOUBLE;
    };
    for (int pc = 0; pc + 1 < pr.code_len; pc += 2) {
        const int op = pr.code[pc], arg = pr.code[pc + 1];
        switch (op) {
            case DQ_P_COL:
                if (!fixed_numeric(arg)) return false;
                st.push_back({E_COL, arg});
                break;
            case DQ_P_CONST:
                if (!const_ok(arg)) return false;
                st.push_back({E_CONST, arg});
                break;
            case DQ_P_EQ: case DQ_P_NE: case DQ_P_LT: case DQ_P_LE: case DQ_P_GT: case DQ_P_GE: {
                if (st.size() < 2) return false;
                const Ent b = st.back(); st.pop_back();
                const Ent a = st.back(); st.pop_back();
                int k;
                if (a.kind == E_COL && b.kind == E_CONST) k = term(a.idx, op, b.idx, b.neg);
                else if (a.kind == E_CONST && b.kind == E_COL) k = term(b.idx, flip(op), a.idx, a.neg);
                else return false;
                if (k < 0 || !emit(k)) return false;
                st.push_back({E_BOOL, 0});
                break;
            }
            case DQ_P_IS_NULL: case DQ_P_IS_NOT_NULL: {
                if (st.empty() || st.back().kind != E_COL) return false;
                const int k = term(st.back().idx, op, -1);
                st.pop_back();
                if (k < 0 || !emit(k)) return false;
                st.push_back({E_BOOL, 0});
                break;
            }
            case DQ_P_AND: case DQ_P_OR: {
                if (st.size() < 2 || st[st.size() - 1].kind != E_BOOL || st[st.size() - 2].kind != E_BOOL) return false;
                st.pop_back();
                if (!emit(op == DQ_P_AND ? kPB_AND : kPB_OR)) return false;
                break;
            }
            case DQ_P_NOT:
                if (st.empty() || st.back().kind != E_BOOL || !emit(kPB_NOT)) return false;
                break;
            case DQ_P_NEG: {  // -constant (a LONG / DOUBLE literal): folded into the leaf's constant
                if (st.empty() || st.back().kind != E_CONST) return false;
                const int tag = pr.consts[st.back().idx].tag;
                if (tag != DQ_V_LONG && tag != DQ_V_DOUBLE) return false;
                st.back().neg = !st.back().neg;
                break;
            }
            case DQ_P_IN: {  // x IN (c1..cn) with non-NULL constants == (x = c1) OR ... OR (x = cn)
                const int n = arg;
                if (n < 1 || (int)st.size() < n + 1) return false;
                const size_t base = st.size() - n - 1;
                if (st[base].kind != E_COL) return false;
                for (int i = 0; i < n; ++i) {
                    if (st[base + 1 + i].kind != E_CONST) return false;
                    const int k = term(st[base].idx, DQ_P_EQ, st[base + 1 + i].idx, st[base + 1 + i].neg);
                    if (k < 0 || !emit(k)) return false;
                    if (i > 0 && !emit(kPB_OR)) return false;
                }
                st.resize(base);
                st.push_back({E_BOOL, 0});
                break;
            }
            default:
                return false;
        }
        if (st.size() > 24) return false;
    }
    return st.size() == 1 && st[0].kind == E_BOOL && out.nterms > 0;
}

// Which kernel a launch group runs (mirrors values_kernel_for in scan.hip).
int scan_kernel_family(int kind, int P, int nc, int heavy) {
    if (kind == SK_BITS) return DQ_KERNEL_BITS;
    if (heavy == 3) return DQ_KERNEL_WHERE_FUSED;
    if ((heavy || nc == 2) && P == 2) return heavy == 2 ? DQ_KERNEL_HEAVY8_FULL : DQ_KERNEL_HEAVY8;
    return heavy ? DQ_KERNEL_STRIPED_HEAVY : DQ_KERNEL_STRIPED;
}

int ensure_side_streams(dq_ctx* ctx) {
    if (ctx->fork_ev) return DQ_OK;
    for (int i = 0; i < dq_ctx::kSide; ++i) {
        DQ_HIP(ctx, hipStreamCreateWithPriority(&ctx->side[i], hipStreamNonBlocking, ctx->hip_priority));
        DQ_HIP(ctx, hipEventCreateWithFlags(&ctx->join_ev[i], hipEventDisableTiming));
    }
    DQ_HIP(ctx, hipEventCreateWithFlags(&ctx->fork_ev, hipEventDisableTiming));
    return DQ_OK;
}

// Bump allocator over the context arena. Two passes: measure, then (after growth) assign.
struct Bump {
    size_t off = 0;
    uint8_t* base = nullptr;
    void* take(size_t bytes, size_t align = 256) {
        off = align_up(off, align);
        void* p = base ? base + off : nullptr;
        off += bytes;
        return p;
    }
};

int ensure_arena(dq_ctx* ctx, size_t bytes) {
    if (bytes <= ctx->arena_cap) return DQ_OK;
    if (ctx->arena) {
        DQ_HIP(ctx, hipStreamSynchronize(ctx->stream));
        DQ_HIP(ctx, hipFree(ctx->arena));
        ctx->arena = nullptr;
        ctx->arena_cap = 0;
    }
    size_t cap = std::max(bytes, (size_t)64 << 20);
    if (hipMalloc(&ctx->arena, cap) != hipSuccess) {
        ctx->arena = nullptr;
        return fail(ctx, DQ_ERR_OUT_OF_MEMORY, "device arena allocation of %zu bytes failed", cap);
    }
    ctx->arena_cap = cap;
    return DQ_OK;
}

int ensure_pinned(dq_ctx* ctx, size_t bytes) {
    if (bytes <= ctx->pinned_cap) return DQ_OK;
    if (ctx->pinned) {
        DQ_HIP(ctx, hipStreamSynchronize(ctx->stream));
        DQ_HIP(ctx, hipHostFree(ctx->pinned));
        ctx->pinned = nullptr;
        ctx->pinned_cap = 0;
    }
    size_t cap = std::max(bytes, (size_t)1 << 20);
    DQ_HIP(ctx, hipHostMalloc((void**)&ctx->pinned, cap, hipHostMallocDefault));
    ctx->pinned_cap = cap;
    return DQ_OK;
}

bool is_numeric_type(int t) {
    // Preconditions.isNumeric (A/Analyzer.scala:329-343)
    return t == DQ_TYPE_BYTE || t == DQ_TYPE_SHORT || t == DQ_TYPE_INT || t == DQ_TYPE_LONG ||
           t == DQ_TYPE_FLOAT || t == DQ_TYPE_DOUBLE || t == DQ_TYPE_DECIMAL;
}
bool is_fixed_width(int t) { return elem_of(t) != ET_NONE; }

int64_t padded_words_for(int64_t nrows) {
    const int64_t tiles = std::max<int64_t>(1, (nrows + kTileRows - 1) / kTileRows);
    return tiles * (kTileRows / 64);
}

}  // namespace

namespace dq {
hipStream_t ctx_stream(dq_ctx* ctx) { return ctx->stream; }
int ctx_device(dq_ctx* ctx) { return ctx->device; }
int ctx_cus(dq_ctx* ctx) { return ctx->cus; }
int ctx_fail(dq_ctx* ctx, int code, const char* msg) { return fail(ctx, code, "%s", msg); }
int ctx_num_subs(dq_ctx* ctx) { return (int)ctx->subs.size(); }
// The context's side streams (created on first use) with its fork event and one join event per side stream; returns
// their number, 0 when they cannot be created.
int ctx_side_streams(dq_ctx* ctx, hipStream_t* side, hipEvent_t* fork, hipEvent_t* join) {
    if (ensure_side_streams(ctx) != DQ_OK) return 0;
    for (int i = 0; i < dq_ctx::kSide; ++i) {
        side[i] = ctx->side[i];
        join[i] = ctx->join_ev[i];
    }
    *fork = ctx->fork_ev;
    return dq_ctx::kSide;
}
dq_ctx* ctx_sub(dq_ctx* ctx, int i) { return ctx->subs[i]; }
// The context's device arena / pinned staging buffer, grown to `bytes` (NULL + error set on failure).
// Used by one call at a time (a ctx is not re-entrant); work queued on the ctx stream stays ordered.
void* ctx_scratch(dq_ctx* ctx, size_t bytes) { return ensure_arena(ctx, bytes) == DQ_OK ? ctx->arena : nullptr; }
void* ctx_pinned_buf(dq_ctx* ctx, size_t bytes) {
    if (ensure_pinned(ctx, bytes) != DQ_OK) return nullptr;
    if (hipStreamSynchronize(ctx->stream) != hipSuccess) return nullptr;  // earlier copies from it are done
    return ctx->pinned;
}

constexpr size_t kScratchCacheCap = size_t(48) << 30;  // idle bytes kept for re-use

// Every open single-device context, so an allocation that fails can release the idle scratch of the device's
// other contexts (helper contexts keep their caches between runs).
std::mutex g_ctx_mu;
std::vector<dq_ctx*> g_ctxs;

void register_ctx(dq_ctx* ctx) {
    std::lock_guard<std::mutex> g(g_ctx_mu);
    g_ctxs.push_back(ctx);
}

void unregister_ctx(dq_ctx* ctx) {
    std::lock_guard<std::mutex> g(g_ctx_mu);
    g_ctxs.erase(std::remove(g_ctxs.begin(), g_ctxs.end(), ctx), g_ctxs.end());
}

void free_blocks(int device, const std::vector<dq_ctx::CachedBlock>& blocks) {
    if (blocks.empty()) return;
    (void)hipSetDevice(device);
    for (const dq_ctx::CachedBlock& b : blocks) {
        (void)hipStreamSynchronize(b.stream);  // its last use was queued there
        (void)hipFree(b.ptr);
    }
}

// Take the cached blocks beyond keep_bytes (oldest first) out of the cache under its lock.
std::vector<dq_ctx::CachedBlock> take_blocks(dq_ctx* ctx, size_t keep_bytes) {
    std::vector<dq_ctx::CachedBlock> out;
    std::lock_guard<std::mutex> g(ctx->scratch_mu);
    size_t i = 0;
    while (ctx->scratch_cached > keep_bytes && i < ctx->scratch_free.size()) {
        out.push_back(ctx->scratch_free[i]);
        ctx->scratch_cached -= ctx->scratch_free[i].bytes;
        ++i;
    }
    ctx->scratch_free.erase(ctx->scratch_free.begin(), ctx->scratch_free.begin() + i);
    return out;
}

void scratch_trim(dq_ctx* ctx, size_t keep_bytes) { free_blocks(ctx->device, take_blocks(ctx, keep_bytes)); }

// Release the idle scratch of the device's other contexts (an allocation of `ctx` failed).
void trim_device_peers(dq_ctx* ctx) {
    std::vector<dq_ctx::CachedBlock> blocks;
    {
        std::lock_guard<std::mutex> g(g_ctx_mu);
        for (dq_ctx* o : g_ctxs) {
            if (o == ctx || o->device != ctx->device) continue;
            std::vector<dq_ctx::CachedBlock> b = take_blocks(o, 0);
            blocks.insert(blocks.end(), b.begin(), b.end());
        }
    }
    free_blocks(ctx->device, blocks);
}

void* scratch_alloc(dq_ctx* ctx, size_t bytes) {
    bytes = std::max<size_t>(bytes, 256);
    {
        std::unique_lock<std::mutex> g(ctx->scratch_mu);
        int best = -1;
        for (int i = 0; i < (int)ctx->scratch_free.size(); ++i) {
            const size_t b = ctx->scratch_free[i].bytes;
            if (b >= bytes && b <= 2 * bytes && (best < 0 || b < ctx->scratch_free[best].bytes)) best = i;
        }
        if (best >= 0) {
            dq_ctx::CachedBlock blk = ctx->scratch_free[best];
            ctx->scratch_free.erase(ctx->scratch_free.begin() + best);
            ctx->scratch_cached -= blk.bytes;
            g.unlock();
            // last used on another stream (dq_set_stream since): that work must be done before this stream reuses it
            if (blk.stream != ctx->stream && hipStreamSynchronize(blk.stream) != hipSuccess) {
                (void)hipFree(blk.ptr);
                return nullptr;
            }
            return blk.ptr;
        }
    }
    void* p = nullptr;
    if (hipMalloc(&p, bytes) == hipSuccess) return p;
    (void)hipGetLastError();
    scratch_trim(ctx);  // the cache may hold what this allocation needs
    if (hipMalloc(&p, bytes) == hipSuccess) return p;
    (void)hipGetLastError();
    trim_device_peers(ctx);  // then the idle caches of the device's other contexts
    if (hipMalloc(&p, bytes) == hipSuccess) return p;
    (void)hipGetLastError();
    return nullptr;
}

void scratch_release(dq_ctx* ctx, void* ptr, size_t bytes) {
    if (!ptr) return;
    bytes = std::max<size_t>(bytes, 256);
    {
        std::lock_guard<std::mutex> g(ctx->scratch_mu);
        ctx->scratch_free.push_back(dq_ctx::CachedBlock{ptr, bytes, ctx->stream});
        ctx->scratch_cached += bytes;
    }
    scratch_trim(ctx, kScratchCacheCap);  // beyond the cap: the oldest blocks (their stream's queued work first)
}
}  // namespace dq

// =================================================================================================
// C-ABI
// =================================================================================================
extern "C" {

int dq_abi_version(void) { return DQ_ABI_VERSION; }

dq_ctx* dq_open(int device, int* status) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        if (status) *status = DQ_ERR_NO_DEVICE;
        return nullptr;
    }
    if (device < 0 || device >= n) {
        if (status) *status = DQ_ERR_INVALID_ARGUMENT;
        return nullptr;
    }
    if (hipSetDevice(device) != hipSuccess) {
        if (status) *status = DQ_ERR_DEVICE;
        return nullptr;
    }
    dq_ctx* ctx = new dq_ctx();
    ctx->device = device;
    if (hipStreamCreateWithFlags(&ctx->own_stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        if (status) *status = DQ_ERR_DEVICE;
        return nullptr;
    }
    ctx->stream = ctx->own_stream;
    register_ctx(ctx);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
        ctx->cus = prop.multiProcessorCount;
    if (status) *status = DQ_OK;
    return ctx;
}

void dq_close(dq_ctx* ctx) {
    if (!ctx) return;
    if (!ctx->subs.empty()) close_subs(ctx);
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    unregister_ctx(ctx);
    scratch_trim(ctx);
    if (ctx->arena) (void)hipFree(ctx->arena);
    if (ctx->pinned) (void)hipHostFree(ctx->pinned);
    for (int i = 0; i < dq_ctx::kSide; ++i) {
        if (ctx->side[i]) (void)hipStreamDestroy(ctx->side[i]);
        if (ctx->join_ev[i]) (void)hipEventDestroy(ctx->join_ev[i]);
    }
    if (ctx->fork_ev) (void)hipEventDestroy(ctx->fork_ev);
    if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
    delete ctx;
}

const char* dq_last_error(const dq_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int dq_set_stream(dq_ctx* ctx, void* stream) {
    if (!ctx) return DQ_ERR_INVALID_ARGUMENT;
    ctx->stream = stream ? (hipStream_t)stream : ctx->own_stream;
    return DQ_OK;
}

int dq_set_priority(dq_ctx* ctx, int priority) {
    if (!ctx || priority < -1 || priority > 1) return DQ_ERR_INVALID_ARGUMENT;
    for (dq_ctx* sub : ctx->subs) {
        const int rc = dq_set_priority(sub, priority);
        if (rc) return fail(ctx, rc, "device %d: %s", sub->device, sub->err.c_str());
    }
    DQ_HIP(ctx, hipSetDevice(ctx->device));
    int least = 0, greatest = 0;
    DQ_HIP(ctx, hipDeviceGetStreamPriorityRange(&least, &greatest));
    const int want = priority > 0 ? greatest : priority < 0 ? least : std::min(std::max(0, greatest), least);
    if (want == ctx->hip_priority) return DQ_OK;
    // the old streams' queued work first: cached scratch blocks and events are re-tagged to the new streams
    DQ_HIP(ctx, hipStreamSynchronize(ctx->own_stream));
    for (int i = 0; i < dq_ctx::kSide; ++i)
        if (ctx->side[i]) DQ_HIP(ctx, hipStreamSynchronize(ctx->side[i]));
    hipStream_t fresh = nullptr;
    DQ_HIP(ctx, hipStreamCreateWithPriority(&fresh, hipStreamNonBlocking, want));
    const hipStream_t old = ctx->own_stream;
    {
        std::lock_guard<std::mutex> g(ctx->scratch_mu);
        for (dq_ctx::CachedBlock& b : ctx->scratch_free)
            if (b.stream == old) b.stream = fresh;
    }
    if (ctx->stream == old) ctx->stream = fresh;
    ctx->own_stream = fresh;
    (void)hipStreamDestroy(old);
    ctx->hip_priority = want;
    for (int i = 0; i < dq_ctx::kSide; ++i) {
        if (!ctx->side[i]) continue;
        (void)hipStreamDestroy(ctx->side[i]);
        DQ_HIP(ctx, hipStreamCreateWithPriority(&ctx->side[i], hipStreamNonBlocking, want));
    }
    return DQ_OK;
}

void dq_scratch_trim(dq_ctx* ctx, int64_t keep_bytes) {
    if (!ctx) return;
    for (dq_ctx* sub : ctx->subs) dq_scratch_trim(sub, keep_bytes);
    scratch_trim(ctx, (size_t)std::max<int64_t>(keep_bytes, 0));
}

int dq_synchronize(dq_ctx* ctx) {
    if (!ctx) return DQ_ERR_INVALID_ARGUMENT;
    for (dq_ctx* sub : ctx->subs) {
        const int rc = dq_synchronize(sub);
        if (rc) return fail(ctx, rc, "device %d: %s", sub->device, sub->err.c_str());
    }
    DQ_HIP(ctx, hipSetDevice(ctx->device));
    DQ_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return DQ_OK;
}

int64_t dq_scan_launch_count(const dq_ctx* ctx) { return ctx ? ctx->scan_launches : -1; }

int64_t dq_scan_kernel_launches(const dq_ctx* ctx, int32_t kernel) {
    if (!ctx || kernel < 0 || kernel >= DQ_KERNEL_COUNT) return -1;
    int64_t n = ctx->kernel_launches[kernel];
    for (const dq_ctx* sub : ctx->subs) n += sub->kernel_launches[kernel];
    return n;
}

int64_t dq_freq_path_count(const dq_ctx* ctx, int32_t path) {
    if (!ctx || path < 0 || path >= DQ_FREQ_PATH_COUNT) return -1;
    int64_t n = ctx->freq_paths[path];
    for (const dq_ctx* sub : ctx->subs) n += sub->freq_paths[path];
    return n;
}

int dq_scan(dq_ctx* ctx, const dq_column* columns, int ncols, int64_t nrows, const dq_op* ops, int nops,
            const dq_predicate* preds, int npreds, dq_state* out, uint32_t flags) {
    if (!ctx) return DQ_ERR_INVALID_ARGUMENT;
    ctx->err.clear();
    if (nops < 0 || ncols < 0 || npreds < 0 || nrows < 0 || (nops > 0 && (!ops || !out)))
        return fail(ctx, DQ_ERR_INVALID_ARGUMENT, "invalid arguments");
    if (nops == 0) return DQ_OK;
    if (!ctx->subs.empty()) {
        // multi-device context: host columns are row-sharded over the devices (multi.cpp)
        if (flags & DQ_SCAN_OUT_DEVICE)
            return fail(ctx, DQ_ERR_UNSUPPORTED, "a multi-device context returns host states (no DQ_SCAN_OUT_DEVICE)");
        for (int c = 0; c < ncols; ++c) {
            if (columns[c].flags & DQ_COL_DEVICE)
                return fail(ctx, DQ_ERR_UNSUPPORTED, "device columns of a multi-device context go through dq_scan_sharded");
            if (columns[c].length != nrows)
                return fail(ctx, DQ_ERR_INVALID_ARGUMENT, "column %d has %lld rows, batch has %lld", c,
                            (long long)columns[c].length, (long long)nrows);
        }
        const int n = (int)ctx->subs.size();
        std::vector<std::vector<dq_column>> cols(n, std::vector<dq_column>(std::max(ncols, 1)));
        std::vector<std::vector<std::vector<int32_t>>> scratch(n);
        std::vector<const dq_column*> ptrs(n);
        std::vector<int64_t> rows(n);
        for (int i = 0; i < n; ++i) {
            int64_t r0 = 0;
            shard_bounds(nrows, n, i, &r0, &rows[i]);
            shard_columns(columns, ncols, r0, rows[i], cols[i].data(), scratch[i]);
            ptrs[i] = cols[i].data();
        }
        return multi_scan(ctx, ptrs.data(), rows.data(), ncols, ops, nops, preds, npreds, out);
    }
    DQ_HIP(ctx, hipSetDevice(ctx->device));

    // ---- validation ---------------------------------------------------------------------------
    for (int c = 0; c < ncols; ++c) {
        const dq_column& col = columns[c];
        if (col.length != nrows)
            return fail(ctx, DQ_ERR_INVALID_ARGUMENT, "column %d has %lld rows, batch has %lld", c,
                        (long long)col.length, (long long)nrows);
        if (col.spark_type < DQ_TYPE_BOOLEAN || col.spark_type > DQ_TYPE_DECIMAL)
            return fail(ctx, DQ_ERR_UNSUPPORTED, "column %d: unknown spark type %d", c, col.spark_type);
        if (col.spark_type == DQ_TYPE_STRING && nrows > 0 && !col.offsets)
            return fail(ctx, DQ_ERR_INVALID_ARGUMENT, "string column %d without offsets", c);
        if (col.flags & DQ_COL_OFFSETS64)
            return fail(ctx, DQ_ERR_UNSUPPORTED, "column %d: int64 string offsets are for the grouping builds only", c);
        if (col.spark_type == DQ_TYPE_DECIMAL && (col.decimal_precision > 18 || col.decimal_scale < 0 || col.decimal_scale > 18))
            return fail(ctx, DQ_ERR_UNSUPPORTED, "column %d: decimal precision > 18 unsupported", c);
        if ((col.flags & DQ_COL_DEVICE) && nrows > 0) {
            const int e = elem_of(col.spark_type);
            // strings: 4-byte aligned UTF-8 (read as dwords), padded by 16 bytes past offsets[length]
            const size_t va = e == ET_NONE ? 4 : (elem_size(e) == 1 ? 8 : 16);
            if (((uintptr_t)col.values % va) != 0 || ((uintptr_t)col.validity % 8) != 0)
                return fail(ctx, DQ_ERR_ALIGNMENT, "device column %d: values must be %zu-byte and validity 8-byte aligned", c, va);
        }
    }
    auto col_ok = [&](int c) { return c >= 0 && c < ncols; };
    std::vector<char> pred_used(npreds, 0);
    std::vector<char> col_used(ncols, 0);
    for (int i = 0; i < nops; ++i) {
        const dq_op& op = ops[i];
        if (op.where >= npreds || op.where < -1) return fail(ctx, DQ_ERR_INVALID_ARGUMENT, "op %d: bad where index", i);
        if (op.where >= 0) pred_used[op.where] = 1;
        switch (op.kind) {
            case DQ_OP_SIZE: break;
            case DQ_OP_COMPLIANCE:
                if (op.predicate < 0 || op.predicate >= npreds)
                    return fail(ctx, DQ_ERR_INVALID_ARGUMENT, "op %d: Compliance needs a predicate", i);
                pred_used[op.predicate] = 1;
                break;
            case DQ_OP_COMPLETENESS:
                if (!col_ok(op.column[0])) return fail(ctx, DQ_ERR_INVALID_ARGUMENT, "op %d: bad column", i);
                col_used[op.column[0]] = 1;
                break;
            case DQ_OP_MEAN: case DQ_OP_SUM: case DQ_OP_MINIMUM: case DQ_OP_MAXIMUM: case DQ_OP_STANDARD_DEVIATION:
                if (!col_ok(op.column[0])) return fail(ctx, DQ_ERR_INVALID_ARGUMENT, "op %d: bad column", i);
                if (!is_numeric_type(columns[op.column[0]].spark_type))
                    return fail(ctx, DQ_ERR_UNSUPPORTED, "op %d: column %d is not numeric", i, op.column[0]);
                col_used[op.column[0]] = 1;
                break;
            case DQ_OP_CORRELATION:
                if (!col_ok(op.column[0]) || !col_ok(op.column[1]))
                    return fail(ctx, DQ_ERR_INVALID_ARGUMENT, "op %d: bad column", i);
                if (!is_numeric_type(columns[op.column[0]].spark_type) || !is_numeric_type(columns[op.column[1]].spark_type))
                    return fail(ctx, DQ_ERR_UNSUPPORTED, "op %d: correlation needs numeric columns", i);
                col_used[op.column[0]] = col_used[op.column[1]] = 1;
                break;
            case DQ_OP_APPROX_COUNT_DISTINCT:
            case DQ_OP_DATATYPE:
                if (!col_ok(op.column[0])) return fail(ctx, DQ_ERR_INVALID_ARGUMENT, "op %d: bad column", i);
                col_used[op.column[0]] = 1;
                break;
            case DQ_OP_MIN_LENGTH: case DQ_OP_MAX_LENGTH:
                if (!col_ok(op.column[0])) return fail(ctx, DQ_ERR_INVALID_ARGUMENT, "op %d: bad column", i);
                if (columns[op.column[0]].spark_type != DQ_TYPE_STRING)
                    return fail(ctx, DQ_ERR_UNSUPPORTED, "op %d: MinLength/MaxLength need a string column", i);
                col_used[op.column[0]] = 1;
                break;
            default:
                return fail(ctx, DQ_ERR_UNSUPPORTED, "op %d: kind %d not implemented by the fused scan", i, op.kind);
        }
    }
    for (int p = 0; p < npreds; ++p) {
        if (!pred_used[p]) continue;
        const dq_predicate& pr = preds[p];
        if (pr.code_len <= 0 || (pr.code_len & 1) || !pr.code)
            return fail(ctx, DQ_ERR_PREDICATE, "predicate %d: empty or odd-length program", p);
        if (pr.code_len == 4 && pr.code[2] == DQ_P_REGEX) {
            const int c = pr.code[1], k = pr.code[3];
            if (pr.code[0] != DQ_P_COL || !col_ok(c) || k < 0 || k >= pr.n_consts || pr.consts[k].tag != DQ_V_STRING ||
                pr.consts[k].str_len < 32 || (pr.consts[k].str_offset & 3) ||
                pr.consts[k].str_offset + pr.consts[k].str_len > pr.strings_len)
                return fail(ctx, DQ_ERR_PREDICATE, "predicate %d: malformed REGEX program", p);
            const int t = columns[c].spark_type;
            if (t < DQ_TYPE_BOOLEAN || t > DQ_TYPE_DECIMAL)
                return fail(ctx, DQ_ERR_UNSUPPORTED, "predicate %d: PatternMatch over this column type is not supported", p);
            if (t == DQ_TYPE_DECIMAL && (columns[c].decimal_scale < 0 || columns[c].decimal_scale > 18))
                return fail(ctx, DQ_ERR_UNSUPPORTED, "predicate %d: PatternMatch over a DECIMAL of scale %d", p,
                            columns[c].decimal_scale);
            col_used[c] = 1;
            continue;
        }
        int depth = 0, maxd = 0;
        for (int k = 0; k < pr.code_len; k += 2) {
            const int op = pr.code[k], arg = pr.code[k + 1];
            if (op == DQ_P_COL) {
                if (!col_ok(arg)) return fail(ctx, DQ_ERR_PREDICATE, "predicate %d: bad column %d", p, arg);
                col_used[arg] = 1;
                ++depth;
            } else if (op == DQ_P_CONST || op == DQ_P_NULL) {
                if (op == DQ_P_CONST && (arg < 0 || arg >= pr.n_consts)) return fail(ctx, DQ_ERR_PREDICATE, "predicate %d: bad constant", p);
                ++depth;
            } else if (op == DQ_P_REGEX) {
                return fail(ctx, DQ_ERR_PREDICATE, "predicate %d: REGEX is only supported as [COL, REGEX]", p);
            } else if (op == DQ_P_IN) {
                depth -= arg;
            } else if (op == DQ_P_COALESCE) {
                depth -= arg - 1;
            } else if (op == DQ_P_CASE) {
                if (arg < 2) return fail(ctx, DQ_ERR_PREDICATE, "predicate %d: CASE without WHEN", p);
                depth -= arg - 1;  // 2 * #WHEN + has ELSE operands -> 1
            } else if (op == DQ_P_SUBSTR) {
                depth -= 2;
            } else if (op == DQ_P_NOT || op == DQ_P_IS_NULL || op == DQ_P_IS_NOT_NULL || op == DQ_P_NEG ||
                       op == DQ_P_LIKE || op == DQ_P_LENGTH || op == DQ_P_CAST_DOUBLE || op == DQ_P_CAST_LONG ||
                       op == DQ_P_CAST_STRING_NUM || op == DQ_P_RLIKE || op == DQ_P_LOWER || op == DQ_P_UPPER ||
                       op == DQ_P_TRIM || op == DQ_P_ISNAN || op == DQ_P_ABS || op == DQ_P_YEAR || op == DQ_P_MONTH ||
                       op == DQ_P_DAY) {
                if (op == DQ_P_LIKE && (arg < 0 || arg >= pr.n_consts)) return fail(ctx, DQ_ERR_PREDICATE, "predicate %d: bad LIKE pattern", p);
                if (op == DQ_P_RLIKE &&
                    (arg < 0 || arg >= pr.n_consts || pr.consts[arg].tag != DQ_V_STRING || pr.consts[arg].str_len < 32 ||
                     (pr.consts[arg].str_offset & 3) || pr.consts[arg].str_offset + pr.consts[arg].str_len > pr.strings_len))
                    return fail(ctx, DQ_ERR_PREDICATE, "predicate %d: malformed RLIKE program", p);
            } else {
                --depth;
            }
            if (depth < 1) return fail(ctx, DQ_ERR_PREDICATE, "predicate %d: stack underflow", p);
            maxd = std::max(maxd, depth);
        }
        if (depth != 1 || maxd > kPredStack) return fail(ctx, DQ_ERR_PREDICATE, "predicate %d: malformed program", p);
    }

    // ---- plan: column uses -> slots -----------------------------------------------------------
    struct Use {
        uint32_t flags = 0;
        int slot = -1, pos = 0, hll = -1;
        int pred_op = 0, pred_kind = FP_NONE, pred_src = -1;  // fused `col <op> const` Compliance predicate
        int64_t pred_i = 0;
        double pred_d = 0.0;
    };
    std::map<std::pair<int, int>, Use> uses;  // (column, where) -> use
    std::vector<int> fused_col(nops, -1);     // Compliance ops answered inside a value slot
    for (int i = 0; i < nops; ++i) {
        const dq_op& op = ops[i];
        const auto key = std::make_pair(op.column[0], op.where);
        switch (op.kind) {
            case DQ_OP_MEAN: case DQ_OP_SUM: case DQ_OP_MINIMUM: case DQ_OP_MAXIMUM: uses[key].flags |= CF_STATS; break;
            case DQ_OP_STANDARD_DEVIATION: uses[key].flags |= CF_MOMENTS; break;
            case DQ_OP_APPROX_COUNT_DISTINCT:
                if (columns[op.column[0]].spark_type != DQ_TYPE_STRING) uses[key].flags |= CF_HLL;
                break;
            case DQ_OP_COMPLIANCE: {
                // `col <op> const` on a non-decimal numeric column: evaluate inside that column's scan.
                const dq_predicate& pr = preds[op.predicate];
                if (pr.code_len != 6) break;
                int a = pr.code[0], aa = pr.code[1], b = pr.code[2], ba = pr.code[3], cmp = pr.code[4];
                if (cmp < DQ_P_EQ || cmp > DQ_P_GE) break;
                if (a == DQ_P_CONST && b == DQ_P_COL) {  // const <op> col  ->  col <op'> const
                    std::swap(a, b);
                    std::swap(aa, ba);
                    if (cmp == DQ_P_LT) cmp = DQ_P_GT;
                    else if (cmp == DQ_P_GT) cmp = DQ_P_LT;
                    else if (cmp == DQ_P_LE) cmp = DQ_P_GE;
                    else if (cmp == DQ_P_GE) cmp = DQ_P_LE;
                }
                if (a != DQ_P_COL || b != DQ_P_CONST || ba < 0 || ba >= pr.n_consts) break;
                const dq_const& k = pr.consts[ba];
                const int t = columns[aa].spark_type;
                if (!(t >= DQ_TYPE_BYTE && t <= DQ_TYPE_DOUBLE) || (k.tag != DQ_V_LONG && k.tag != DQ_V_DOUBLE)) break;
                Use& u = uses[std::make_pair(aa, op.where)];
                const int kind = k.tag == DQ_V_LONG ? FP_LONG : FP_DOUBLE;
                if (u.pred_kind != FP_NONE &&
                    !(u.pred_op == cmp && u.pred_kind == kind && u.pred_i == k.i64 &&
                      (kind == FP_LONG || u.pred_d == k.f64)))
                    break;  // one fused predicate per column scan; others use the predicate VM
                u.pred_op = cmp;
                u.pred_kind = kind;
                u.pred_i = k.i64;
                u.pred_d = k.f64;
                fused_col[i] = aa;
                break;
            }
            default: break;
        }
    }
    std::vector<SlotDesc> slots;
    auto new_slot = [&](int kind) {
        SlotDesc sd;
        memset(&sd, 0, sizeof(sd));
        sd.kind = kind;
        sd.col[0].hll_slot = sd.col[1].hll_slot = -1;
        sd.col[0].elem = sd.col[1].elem = ET_NONE;
        sd.rows_per_load = 8;
        slots.push_back(sd);
        return (int)slots.size() - 1;
    };
    struct PairKey { int x, y, w; bool operator<(const PairKey& o) const { return std::tie(x, y, w) < std::tie(o.x, o.y, o.w); } };
    std::map<PairKey, int> pair_slots;  // (x, y, where) -> slot with corr
    std::vector<std::pair<int, int>> op_slot(nops, {-1, 0});  // slot, colpos (corr: 1 = swapped)
    // Correlation pairs first: fuse both columns' uses into one pair slot when element sizes match.
    for (int i = 0; i < nops; ++i) {
        const dq_op& op = ops[i];
        if (op.kind != DQ_OP_CORRELATION) continue;
        const int x = op.column[0], y = op.column[1], w = op.where;
        auto it = pair_slots.find({x, y, w});
        if (it != pair_slots.end()) { op_slot[i] = {it->second, 0}; continue; }
        it = pair_slots.find({y, x, w});
        if (it != pair_slots.end()) { op_slot[i] = {it->second, 1}; continue; }
        const int ex = elem_of(columns[x].spark_type), ey = elem_of(columns[y].spark_type);
        const int s = new_slot(SK_VALUES);
        slots[s].ncols = 2;
        slots[s].corr = 1;
        slots[s].rows_per_load = elem_size(ex) == elem_size(ey) ? rows_per_load_of(ex) : 8;
        slots[s].col[0].elem = ex;
        slots[s].col[1].elem = ey;
        if (x != y) {
            auto ux = uses.find({x, w}), uy = uses.find({y, w});
            if (ux != uses.end() && ux->second.slot < 0) { ux->second.slot = s; ux->second.pos = 0; }
            if (uy != uses.end() && uy->second.slot < 0) { uy->second.slot = s; uy->second.pos = 1; }
        }
        slots[s].col[0].values = (const void*)(intptr_t)x;  // column index until pointers are known
        slots[s].col[1].values = (const void*)(intptr_t)y;
        slots[s].where_t = (const uint64_t*)(intptr_t)(w + 1);
        pair_slots[{x, y, w}] = s;
        op_slot[i] = {s, 0};
    }
    for (auto& kv : uses) {
        if (kv.second.slot >= 0) continue;
        const int c = kv.first.first, w = kv.first.second;
        const int s = new_slot(SK_VALUES);
        slots[s].ncols = 1;
        slots[s].rows_per_load = rows_per_load_of(elem_of(columns[c].spark_type));
        slots[s].col[0].elem = elem_of(columns[c].spark_type);
        slots[s].col[0].values = (const void*)(intptr_t)c;
        slots[s].where_t = (const uint64_t*)(intptr_t)(w + 1);
        kv.second.slot = s;
        kv.second.pos = 0;
    }
    int nhll = 0;
    for (auto& kv : uses) {
        SlotDesc& sd = slots[kv.second.slot];
        sd.col[kv.second.pos].flags |= kv.second.flags;
        sd.col[kv.second.pos].pred_op = kv.second.pred_op;
        sd.col[kv.second.pos].pred_kind = kv.second.pred_kind;
        sd.col[kv.second.pos].pred_i = kv.second.pred_i;
        sd.col[kv.second.pos].pred_d = kv.second.pred_d;
        if (kv.second.flags & CF_HLL) {
            kv.second.hll = nhll++;
            sd.col[kv.second.pos].hll_slot = kv.second.hll;
        }
    }
    // String-shaped ops -> string slots (column, where): MinLength/MaxLength, DataType, string HLL.
    std::vector<StrSlot> sslots;
    std::map<std::pair<int, int>, int> sslot_of;
    std::vector<int> op_sslot(nops, -1);
    for (int i = 0; i < nops; ++i) {
        const dq_op& op = ops[i];
        const bool str_hll = op.kind == DQ_OP_APPROX_COUNT_DISTINCT && columns[op.column[0]].spark_type == DQ_TYPE_STRING;
        if (!(op.kind == DQ_OP_MIN_LENGTH || op.kind == DQ_OP_MAX_LENGTH || op.kind == DQ_OP_DATATYPE || str_hll)) continue;
        const auto key = std::make_pair(op.column[0], op.where);
        auto it = sslot_of.find(key);
        if (it == sslot_of.end()) {
            StrSlot ss;
            memset(&ss, 0, sizeof(ss));
            ss.spark_type = columns[op.column[0]].spark_type;
            ss.decimal_scale = columns[op.column[0]].decimal_scale;
            ss.hll_slot = -1;
            ss.values = (const void*)(intptr_t)op.column[0];  // column index until pointers are known
            ss.where_t = (const uint64_t*)(intptr_t)(op.where + 1);
            sslots.push_back(ss);
            it = sslot_of.emplace(key, (int)sslots.size() - 1).first;
        }
        StrSlot& ss = sslots[it->second];
        if (op.kind == DQ_OP_DATATYPE) ss.flags |= SF_DTYPE;
        else if (str_hll) {
            ss.flags |= SF_HLL;
            if (ss.hll_slot < 0) ss.hll_slot = nhll++;
        } else ss.flags |= SF_LEN;
        op_sslot[i] = it->second;
    }
    const int nsslots = (int)sslots.size();
    std::vector<StrOpMap> sopmap;
    for (int i = 0; i < nops; ++i) {
        if (op_sslot[i] < 0 || ops[i].kind == DQ_OP_APPROX_COUNT_DISTINCT) continue;
        StrOpMap m;
        m.op = i;
        m.kind = ops[i].kind;
        m.slot = op_sslot[i];
        m.pad = 0;
        sopmap.push_back(m);
    }

    // `where` filters evaluated inside the scan (WhereOut, dq_internal.h): every simple predicate used as a `where`
    // (DQ_WHERE_MASKS=0 or DQ_PRED_VM=1: the bitmap pass for all of them, for A/B runs).
    std::vector<char> wmasked(npreds, 0);
    std::vector<PredSimple> wprog(npreds);
    {
        const char* e = getenv("DQ_WHERE_MASKS");
        const bool masks_on = !pred_vm_forced() && !(e && e[0] == '0');
        for (int i = 0; i < nops && masks_on; ++i) {
            const int p = ops[i].where;
            if (p < 0 || wmasked[p]) continue;
            const dq_predicate& pr = preds[p];
            if (pr.code_len == 4 && pr.code[2] == DQ_P_REGEX) continue;
            if (compile_simple_predicate(pr, columns, ncols, wprog[p])) wmasked[p] = 1;
        }
    }

    // Ops -> OpMap; bits-only slots for Size(where), Completeness of unread columns, Compliance.
    std::vector<OpMap> opmap(nops);
    std::map<std::tuple<int, int, int>, int> bits_slots;  // (kind, col/pred, where) -> slot
    auto bits_slot = [&](int tag, int ref, int w) {
        auto key = std::make_tuple(tag, ref, w);
        auto it = bits_slots.find(key);
        if (it != bits_slots.end()) return it->second;
        const int s = new_slot(SK_BITS);
        slots[s].where_t = (const uint64_t*)(intptr_t)(w + 1);
        slots[s].col[0].values = (const void*)(intptr_t)ref;
        slots[s].col[0].flags = (uint32_t)tag;  // 1 = completeness column, 2 = compliance predicate, 0 = size
        bits_slots[key] = s;
        return s;
    };
    for (int i = 0; i < nops; ++i) {
        const dq_op& op = ops[i];
        OpMap& m = opmap[i];
        memset(&m, 0, sizeof(m));
        m.kind = op.kind;
        m.slot = -1;
        m.hll_slot = -1;
        m.has_where = op.where >= 0;
        m.nrows = nrows;
        const int c = op.column[0];
        if (op.kind != DQ_OP_SIZE && op.kind != DQ_OP_COMPLIANCE && col_ok(c)) {
            const int t = columns[c].spark_type;
            m.is_float = (t == DQ_TYPE_FLOAT || t == DQ_TYPE_DOUBLE);
            m.decimal_scale = t == DQ_TYPE_DECIMAL ? columns[c].decimal_scale : 0;
        }
        m.wslot = -1;
        const bool masked_where = op.where >= 0 && wmasked[op.where];
        switch (op.kind) {
            case DQ_OP_SIZE:
                if (op.where >= 0 && !masked_where) m.slot = bits_slot(0, -1, op.where);
                break;
            case DQ_OP_COMPLIANCE:
                if (fused_col[i] >= 0) {
                    const Use& u = uses.at({fused_col[i], op.where});
                    m.slot = u.slot;
                    m.colpos = u.pos;
                    m.from_bits = 3;  // fused predicate: matches = c.pt, non-null rows = c.n
                } else {
                    m.slot = bits_slot(2, op.predicate, op.where);
                }
                break;
            case DQ_OP_COMPLETENESS: {
                auto it = uses.find({c, op.where});
                if (it != uses.end()) {
                    m.slot = it->second.slot;
                    m.colpos = it->second.pos;
                } else if (columns[c].validity == nullptr) {
                    m.from_bits = 2;  // all rows valid: matches = conditionalCount
                    if (op.where >= 0 && !masked_where) m.slot = bits_slot(0, -1, op.where);
                } else {
                    m.slot = bits_slot(1, c, op.where);
                    m.from_bits = 1;
                }
                break;
            }
            case DQ_OP_CORRELATION:
                m.slot = op_slot[i].first;
                m.colpos = op_slot[i].second;
                break;
            case DQ_OP_MIN_LENGTH: case DQ_OP_MAX_LENGTH: case DQ_OP_DATATYPE:
                break;  // written by finalize_strings_kernel
            default: {
                if (op_sslot[i] >= 0) {  // ApproxCountDistinct of a string column
                    m.hll_slot = sslots[op_sslot[i]].hll_slot;
                    break;
                }
                const Use& u = uses.at({c, op.where});
                m.slot = u.slot;
                m.colpos = u.pos;
                m.hll_slot = u.hll;
                break;
            }
        }
    }
    // Masked `where` plan: the producer (a one-column 8-byte value slot under the filter whose terms read only that
    // column, else an SK_WHERE slot filled by where_masks_kernel), the consumer masks, and whether bits / string
    // slots still read the filter's bitmaps.
    struct WherePlan {
        int producer = -1;           // value slot evaluating the filter inside its scan
        int wslot = -1;              // slot holding the TRUE / NOT-NULL counts
        bool bitmaps = false;
        std::vector<int> mask_col;   // consumer columns, one mask each
    };
    std::vector<WherePlan> wplan(npreds);
    std::vector<std::pair<int, int>> slot_masks(slots.size() * 2, {-1, -1});  // (slot, k) -> (pred, mask index)
    std::vector<int> slot_producer_of(slots.size(), -1);
    auto slot_where = [&](const SlotDesc& sd) { return (int)(intptr_t)sd.where_t - 1; };
    for (int p = 0; p < npreds; ++p) {
        if (!wmasked[p]) continue;
        WherePlan& wp = wplan[p];
        int depth = 0, maxd = 0;
        for (int i = 0; i < wprog[p].nb; ++i) {
            depth += wprog[p].b[i] >= 0 ? 1 : (wprog[p].b[i] == kPB_NOT ? 0 : -1);
            maxd = std::max(maxd, depth);
        }
        // (DQ_WHERE_FUSED=0: every masked filter from where_masks_kernel, the filter column a consumer -- A/B runs)
        const bool fuse_producer = !(getenv("DQ_WHERE_FUSED") && getenv("DQ_WHERE_FUSED")[0] == '0');
        for (int s = 0; s < (int)slots.size() && wp.producer < 0 && maxd <= kWhereStack && fuse_producer; ++s) {
            const SlotDesc& sd = slots[s];
            if (sd.kind != SK_VALUES || sd.ncols != 1 || slot_where(sd) != p) continue;
            const int x = (int)(intptr_t)sd.col[0].values;
            const int t = columns[x].spark_type;
            if (!(t == DQ_TYPE_LONG || t == DQ_TYPE_TIMESTAMP || t == DQ_TYPE_DOUBLE)) continue;
            bool own = true;
            for (int k = 0; k < wprog[p].nterms; ++k) own &= wprog[p].t[k].col == x;
            if (own) wp.producer = s;
        }
        for (int s = 0; s < (int)slots.size(); ++s) {
            SlotDesc& sd = slots[s];
            if (sd.kind == SK_BITS && (slot_where(sd) == p || ((int)sd.col[0].flags == 2 && (int)(intptr_t)sd.col[0].values == p)))
                wp.bitmaps = true;
            if (sd.kind != SK_VALUES || slot_where(sd) != p) continue;
            if (s == wp.producer) continue;
            for (int k = 0; k < sd.ncols; ++k) {
                const int c = (int)(intptr_t)sd.col[k].values;
                auto it = std::find(wp.mask_col.begin(), wp.mask_col.end(), c);
                int mi = (int)(it - wp.mask_col.begin());
                if (it == wp.mask_col.end()) wp.mask_col.push_back(c);
                slot_masks[2 * s + k] = {p, mi};
            }
        }
        for (const StrSlot& ss : sslots)
            if ((int)(intptr_t)ss.where_t - 1 == p) wp.bitmaps = true;
        if ((int)wp.mask_col.size() > kWhereMasks) {  // too many consumers for one producer: the bitmap pass
            wmasked[p] = 0;
            wp = WherePlan();
            for (auto& sm : slot_masks)
                if (sm.first == p) sm = {-1, -1};
            continue;
        }
    }
    // Size(where) / from_bits == 2 Completeness were planned without a bits slot for masked filters: give back the
    // bits slots to filters that fell back above.
    for (int i = 0; i < nops; ++i) {
        const dq_op& op = ops[i];
        if (op.where < 0 || wmasked[op.where] || opmap[i].slot >= 0) continue;
        if (op.kind == DQ_OP_SIZE || (op.kind == DQ_OP_COMPLETENESS && opmap[i].from_bits == 2))
            opmap[i].slot = bits_slot(0, -1, op.where);
    }
    slot_masks.resize(slots.size() * 2, {-1, -1});
    slot_producer_of.resize(slots.size(), -1);
    for (int p = 0; p < npreds; ++p) {
        if (!wmasked[p]) continue;
        WherePlan& wp = wplan[p];
        if (wp.producer >= 0) {
            wp.wslot = wp.producer;
            slot_producer_of[wp.producer] = p;
            slots[wp.producer].where_t = nullptr;
        } else {
            wp.wslot = new_slot(SK_WHERE);
            slot_masks.resize(slots.size() * 2, {-1, -1});
            slot_producer_of.resize(slots.size(), -1);
        }
        for (int s = 0; s < (int)slots.size(); ++s)
            if (slots[s].kind == SK_VALUES && slot_where(slots[s]) == p) slots[s].where_t = nullptr;
    }
    for (int i = 0; i < nops; ++i) {
        const int p = ops[i].where;
        if (p >= 0) opmap[i].wslot = wmasked[p] ? wplan[p].wslot : opmap[i].slot;
    }
    const int nslots = (int)slots.size();
    if (nslots > kMaxSlots) return fail(ctx, DQ_ERR_UNSUPPORTED, "too many slots (%d)", nslots);
    // Predicates evaluated by the VM pass: `where` filters and Compliance predicates not fused into
    // a value scan.
    std::fill(pred_used.begin(), pred_used.end(), 0);
    for (int i = 0; i < nops; ++i) {
        if (ops[i].where >= 0) pred_used[ops[i].where] = 1;
        if (ops[i].kind == DQ_OP_COMPLIANCE && fused_col[i] < 0) pred_used[ops[i].predicate] = 1;
    }
    // pred_used: the predicate gets TRUE / NOT-NULL bitmaps (allocated); pred_pass: a predicate pass writes them (a
    // masked `where` writes them from its producer, only when something reads them)
    std::vector<char> pred_pass(pred_used);
    int nstandalone = 0;
    for (int p = 0; p < npreds; ++p) {
        if (!wmasked[p]) continue;
        pred_pass[p] = 0;
        if (!wplan[p].bitmaps) pred_used[p] = 0;
        if (wplan[p].producer < 0) ++nstandalone;
    }

    // ---- device memory layout -----------------------------------------------------------------
    // Launch groups: one kernel launch per slot shape; each gets a grid sized to fill the chip once.
    const int64_t ntiles = (nrows + kTileRows - 1) / kTileRows;
    struct Group { int kind, P, nc; bool f0, f1; int heavy; int grid; std::vector<int32_t> slots; };
    std::vector<Group> groups;
    auto shape_key = [](int kind, int P, int nc, bool f0, bool f1, int heavy) {
        return (((((kind * 16 + P) * 4 + nc) * 2 + f0) * 2 + f1) * 4 + heavy);
    };
    // heavy 2 (8-byte columns only): every column carries stats, moments, HLL and a fused compare the heavy kernel
    // evaluates on its fast path, pairs carry the correlation, and there is no `where` -> the branch-free variant
    auto full_col = [](const ColDesc& c) {
        const bool fl = c.elem == ET_F64;
        const uint32_t all = CF_STATS | CF_MOMENTS | CF_HLL;
        const bool fast_pred = fl ? (c.pred_kind != FP_NONE && (c.pred_kind == FP_LONG || c.pred_d == c.pred_d))
                                  : c.pred_kind == FP_LONG;
        return (c.flags & all) == all && fast_pred;
    };
    std::map<int, int> group_of;
    for (int s = 0; s < (int)slots.size(); ++s) {
        const SlotDesc& sd = slots[s];
        if (sd.kind == SK_WHERE) continue;
        const bool f0 = sd.kind == SK_VALUES && (sd.col[0].elem == ET_F32 || sd.col[0].elem == ET_F64);
        const bool f1 = sd.kind == SK_VALUES && sd.ncols > 1 && (sd.col[1].elem == ET_F32 || sd.col[1].elem == ET_F64);
        const int P = sd.kind == SK_VALUES ? sd.rows_per_load : 8;
        const int nc = sd.kind == SK_VALUES ? sd.ncols : 1;
        // HLL registers or a fused predicate need the larger (HEAVY) kernel instantiation.
        int heavy = 0;
        for (int k = 0; sd.kind == SK_VALUES && k < sd.ncols; ++k)
            if ((sd.col[k].flags & CF_HLL) || sd.col[k].pred_kind != FP_NONE) heavy = 1;
        if (heavy && P == 2 && sd.where_t == nullptr && (sd.ncols == 1 || sd.corr)) {
            bool full = true;
            for (int k = 0; k < sd.ncols; ++k) full &= full_col(sd.col[k]);
            if (full) heavy = 2;
        }
        if (slot_producer_of[s] >= 0) heavy = 3;
        const int kind = sd.kind;
        const int key = shape_key(kind, P, nc, f0, f1, heavy);
        auto it = group_of.find(key);
        if (it == group_of.end()) {
            int occ;
            auto oc = ctx->occupancy.find(key);
            if (oc != ctx->occupancy.end()) occ = oc->second;
            else occ = ctx->occupancy[key] = std::max(1, scan_group_blocks_per_cu(kind, P, nc, f0, f1, heavy));
            const int64_t grid = std::max<int64_t>(1, std::min<int64_t>(std::max<int64_t>(ntiles, 1), (int64_t)ctx->cus * occ));
            groups.push_back(Group{kind, P, nc, f0, f1, heavy, (int)grid, {}});
            it = group_of.emplace(key, (int)groups.size() - 1).first;
        }
        groups[it->second].slots.push_back(s);
    }
    // concurrent launches: each shape gets its share of the chip so the launches are co-resident
    const int nlaunch = (int)groups.size() + (nsslots ? 1 : 0);
    const bool concurrent = scan_concurrency() && nlaunch > 1 && ensure_side_streams(ctx) == DQ_OK;
    if (concurrent)
        for (Group& g : groups) g.grid = std::max(1, (g.grid + nlaunch - 1) / nlaunch);
    int gstride = 1;
    for (const Group& g : groups) gstride = std::max(gstride, g.grid);
    int sgrid = nsslots ? string_scan_grid(ctx->cus, nrows) : 0;
    if (concurrent && sgrid) sgrid = std::max(1, (sgrid + nlaunch - 1) / nlaunch);
    gstride = std::max(gstride, sgrid);
    // producers first: their masks are read by the other launches
    std::stable_sort(groups.begin(), groups.end(), [](const Group& a, const Group& b) { return (a.heavy == 3) > (b.heavy == 3); });
    std::vector<int32_t> slot_nblocks(std::max<size_t>(slots.size(), 1), 1);
    for (const Group& g : groups)
        for (int32_t s : g.slots) slot_nblocks[s] = g.grid;
    const int64_t wchunks = (padded_words_for(nrows) + 7) / 8;  // where_masks_kernel: 8 words per wave, 4 waves
    const int wgrid = (int)std::max<int64_t>(1, std::min<int64_t>((wchunks + 3) / 4, gstride));
    for (int p = 0; p < npreds; ++p)
        if (wmasked[p] && wplan[p].producer < 0) slot_nblocks[wplan[p].wslot] = wgrid;
    std::vector<int32_t> hll_nblocks(std::max(nhll, 1), 1);
    for (const auto& kv : uses)
        if (kv.second.hll >= 0) hll_nblocks[kv.second.hll] = slot_nblocks[kv.second.slot];
    for (const StrSlot& ss : sslots)
        if (ss.hll_slot >= 0) hll_nblocks[ss.hll_slot] = sgrid;
    const int64_t pwords = padded_words_for(nrows);
    const size_t bitmap_bytes = (size_t)(nrows + 7) / 8;

    std::vector<const void*> dval(ncols, nullptr), dvalid(ncols, nullptr), doffs(ncols, nullptr);
    size_t arena_need = 0;
    std::vector<size_t> stage_off(ncols, 0);
    int npred_pass = 0;
    for (int p = 0; p < npreds; ++p) npred_pass += pred_pass[p];
    for (int pass = 0; pass < 2; ++pass) {
        Bump b;
        b.base = pass ? ctx->arena : nullptr;
        for (int c = 0; c < ncols; ++c) {
            const dq_column& col = columns[c];
            if (!col_used[c]) continue;
            if (col.flags & DQ_COL_DEVICE) {
                dval[c] = col.values;
                dvalid[c] = col.validity;
                doffs[c] = col.offsets;
                continue;
            }
            size_t vbytes;
            if (col.spark_type == DQ_TYPE_STRING) vbytes = nrows > 0 ? (size_t)col.offsets[nrows] : 0;
            else vbytes = (size_t)nrows * elem_size(elem_of(col.spark_type));
            void* v = b.take(vbytes + 16);
            void* vd = col.validity ? b.take(align_up(bitmap_bytes, 8) + 8) : nullptr;
            void* od = col.spark_type == DQ_TYPE_STRING ? b.take(((size_t)nrows + 1) * 4) : nullptr;
            if (pass) {
                if (vbytes) DQ_HIP(ctx, hipMemcpyAsync(v, col.values, vbytes, hipMemcpyHostToDevice, ctx->stream));
                if (vd && bitmap_bytes) DQ_HIP(ctx, hipMemcpyAsync(vd, col.validity, bitmap_bytes, hipMemcpyHostToDevice, ctx->stream));
                if (od) DQ_HIP(ctx, hipMemcpyAsync(od, col.offsets, ((size_t)nrows + 1) * 4, hipMemcpyHostToDevice, ctx->stream));
                dval[c] = v;
                dvalid[c] = col.validity ? vd : nullptr;
                doffs[c] = od;
            }
        }
        // predicate outputs + programs
        std::vector<uint64_t*> pt(npreds, nullptr), pn(npreds, nullptr);
        for (int p = 0; p < npreds; ++p) {
            if (!pred_used[p]) continue;
            pt[p] = (uint64_t*)b.take((size_t)pwords * 8);
            pn[p] = (uint64_t*)b.take((size_t)pwords * 8);
        }
        // masked `where`: the producer's descriptor and one mask per consumer column
        std::vector<WhereOut*> wodev(npreds, nullptr);
        std::vector<std::vector<uint64_t*>> wmask(npreds);
        for (int p = 0; p < npreds; ++p) {
            if (!wmasked[p]) continue;
            wodev[p] = (WhereOut*)b.take(sizeof(WhereOut));
            for (size_t m = 0; m < wplan[p].mask_col.size(); ++m) wmask[p].push_back((uint64_t*)b.take((size_t)pwords * 8));
        }
        void* pcols = b.take(sizeof(PredColumn) * std::max(ncols, 1));
        int32_t* rx_status = (int32_t*)b.take(sizeof(int32_t) * std::max(npreds, 1));
        std::vector<void*> pprog(npreds, nullptr), pcode(npreds, nullptr), pconst(npreds, nullptr), pstr(npreds, nullptr);
        for (int p = 0; p < npreds; ++p) {
            if (!pred_pass[p]) continue;
            pprog[p] = b.take(sizeof(PredProgram));
            pcode[p] = b.take(sizeof(int32_t) * preds[p].code_len);
            pconst[p] = b.take(sizeof(dq_const) * std::max(preds[p].n_consts, 1));
            pstr[p] = b.take(std::max<int64_t>(preds[p].strings_len, 1));
        }
        SlotDesc* dslots = (SlotDesc*)b.take(sizeof(SlotDesc) * std::max(nslots, 1));
        OpMap* dops = (OpMap*)b.take(sizeof(OpMap) * nops);
        SlotPartial* partials = (SlotPartial*)b.take(sizeof(SlotPartial) * (size_t)std::max(nslots, 1) * gstride);
        int32_t* dgroups = (int32_t*)b.take(sizeof(int32_t) * std::max(nslots, 1));
        int32_t* dslot_nb = (int32_t*)b.take(sizeof(int32_t) * slot_nblocks.size());
        int32_t* dhll_nb = (int32_t*)b.take(sizeof(int32_t) * hll_nblocks.size());
        SlotPartial* finals = (SlotPartial*)b.take(sizeof(SlotPartial) * std::max(nslots, 1));
        uint8_t* hllp = (uint8_t*)b.take((size_t)std::max(nhll, 1) * gstride * kHllRegs);
        uint8_t* hllf = (uint8_t*)b.take((size_t)std::max(nhll, 1) * kHllRegs);
        dq_state* dout = (flags & DQ_SCAN_OUT_DEVICE) ? out : (dq_state*)b.take(sizeof(dq_state) * nops);
        StrSlot* dsslots = (StrSlot*)b.take(sizeof(StrSlot) * std::max(nsslots, 1));
        StrPartial* spartials = (StrPartial*)b.take(sizeof(StrPartial) * (size_t)std::max(nsslots, 1) * gstride);
        StrOpMap* dsops = (StrOpMap*)b.take(sizeof(StrOpMap) * std::max<size_t>(sopmap.size(), 1));
        if (!pass) {
            arena_need = b.off;
            int rc = ensure_arena(ctx, arena_need);
            if (rc) return rc;
            // plan bytes uploaded through pinned staging
            size_t pin = sizeof(int32_t) * std::max(npreds, 1) + 32 + sizeof(StrSlot) * std::max(nsslots, 1) + sizeof(StrOpMap) * std::max<size_t>(sopmap.size(), 1) +
                         sizeof(PredColumn) * std::max(ncols, 1) + sizeof(SlotDesc) * std::max(nslots, 1) +
                         sizeof(OpMap) * nops + sizeof(dq_state) * nops + 4 * (slot_nblocks.size() + hll_nblocks.size() + nslots) + 8192;
            for (int p = 0; p < npreds; ++p)
                if (wmasked[p]) pin += sizeof(WhereOut) + 256;
            for (int p = 0; p < npreds; ++p)
                if (pred_pass[p])
                    pin += sizeof(PredProgram) + sizeof(int32_t) * preds[p].code_len +
                           sizeof(dq_const) * std::max(preds[p].n_consts, 1) + std::max<int64_t>(preds[p].strings_len, 1) + 256;
            rc = ensure_pinned(ctx, pin);
            if (rc) return rc;
            continue;
        }
        // ---- pass 1: fill descriptors, upload, launch ------------------------------------------
        // The pinned buffer may still be read by a previous call's async copies: wait for them.
        DQ_HIP(ctx, hipStreamSynchronize(ctx->stream));
        Bump hb;
        hb.base = ctx->pinned;
        auto upload = [&](void* dst, const void* src, size_t n) -> int {
            void* h = hb.take(n, 16);
            memcpy(h, src, n);
            DQ_HIP(ctx, hipMemcpyAsync(dst, h, n, hipMemcpyHostToDevice, ctx->stream));
            return DQ_OK;
        };
        bool any_regex = false;
        if (npred_pass || nstandalone) {
            DQ_HIP(ctx, hipMemsetAsync(rx_status, 0, sizeof(int32_t) * std::max(npreds, 1), ctx->stream));
            std::vector<PredColumn> pc(std::max(ncols, 1));
            for (int c = 0; c < ncols; ++c) {
                memset(&pc[c], 0, sizeof(PredColumn));
                pc[c].values = dval[c];
                pc[c].validity = (const uint64_t*)dvalid[c];
                pc[c].offsets = (const int32_t*)doffs[c];
                pc[c].spark_type = columns[c].spark_type;
                pc[c].elem = elem_of(columns[c].spark_type);
                pc[c].decimal_scale = columns[c].decimal_scale;
            }
            int rc = upload(pcols, pc.data(), sizeof(PredColumn) * pc.size());
            if (rc) return rc;
            for (int p = 0; p < npreds; ++p) {
                if (!pred_pass[p]) continue;
                const dq_predicate& pr = preds[p];
                rc = upload(pcode[p], pr.code, sizeof(int32_t) * pr.code_len);
                if (rc) return rc;
                if (pr.n_consts > 0) {
                    rc = upload(pconst[p], pr.consts, sizeof(dq_const) * pr.n_consts);
                    if (rc) return rc;
                }
                if (pr.strings_len > 0) {
                    rc = upload(pstr[p], pr.strings, (size_t)pr.strings_len);
                    if (rc) return rc;
                }
                PredProgram pg;
                pg.code = (const int32_t*)pcode[p];
                pg.consts = (const dq_const*)pconst[p];
                pg.strings = (const uint8_t*)pstr[p];
                pg.code_len = pr.code_len;
                pg.n_consts = pr.n_consts;
                rc = upload(pprog[p], &pg, sizeof(pg));
                if (rc) return rc;
                if (pr.code_len == 4 && pr.code[2] == DQ_P_REGEX) {
                    const dq_const& k = pr.consts[pr.code[3]];
                    launch_regex(pc[pr.code[1]], (const int32_t*)((const uint8_t*)pstr[p] + k.str_offset), nrows, pwords,
                                 pt[p], pn[p], rx_status + p, ctx->stream);
                    ctx->kernel_launches[DQ_KERNEL_REGEX]++;
                    any_regex = true;
                } else if (PredSimple ps; !pred_vm_forced() && compile_simple_predicate(pr, columns, ncols, ps)) {
                    launch_pred_simple(ps, (const PredColumn*)pcols, nrows, pwords, pt[p], pn[p], ctx->stream);
                    ctx->kernel_launches[DQ_KERNEL_PRED_SIMPLE]++;
                } else {
                    bool rx = false;
                    for (int k = 0; k + 1 < pr.code_len; k += 2) rx |= pr.code[k] == DQ_P_RLIKE;
                    launch_predicate((const PredProgram*)pprog[p], rx, rx_status + p, (const PredColumn*)pcols, nrows,
                                     pwords, pt[p], pn[p], ctx->stream);
                    ctx->kernel_launches[DQ_KERNEL_PRED_VM]++;
                    any_regex |= rx;
                }
                DQ_HIP(ctx, hipGetLastError());
            }
        }
        // masked `where` descriptors; the standalone producers run here, before every scan launch
        for (int p = 0; p < npreds; ++p) {
            if (!wmasked[p]) continue;
            const WherePlan& wp = wplan[p];
            WhereOut wo;
            memset(&wo, 0, sizeof(wo));
            wo.prog = wprog[p];
            wo.nmasks = (int)wp.mask_col.size();
            wo.bitmaps = wp.bitmaps ? 1 : 0;
            wo.where_t = pt[p];
            wo.where_nn = pn[p];
            for (int m = 0; m < wo.nmasks; ++m) {
                wo.valid[m] = (const uint64_t*)dvalid[wp.mask_col[m]];
                wo.mask[m] = wmask[p][m];
            }
            int rc = upload(wodev[p], &wo, sizeof(wo));
            if (rc) return rc;
            if (wp.producer < 0) {
                launch_where_masks(wodev[p], wprog[p], (const PredColumn*)pcols, nrows, pwords, partials, wp.wslot, gstride,
                                   slot_nblocks[wp.wslot], ctx->stream);
                DQ_HIP(ctx, hipGetLastError());
                ctx->kernel_launches[DQ_KERNEL_WHERE_MASKS]++;
            }
        }
        // resolve slot descriptors
        for (int s = 0; s < nslots; ++s) {
            SlotDesc& sd = slots[s];
            const int w = (int)(intptr_t)sd.where_t - 1;
            sd.where_t = w >= 0 ? pt[w] : nullptr;
            sd.where_nn = w >= 0 ? pn[w] : nullptr;
            if (sd.kind == SK_VALUES) {
                for (int k = 0; k < sd.ncols; ++k) {
                    const int c = (int)(intptr_t)sd.col[k].values;
                    sd.col[k].values = dval[c];
                    sd.col[k].validity = (const uint64_t*)dvalid[c];
                    sd.col[k].spark_type = columns[c].spark_type;
                    sd.col[k].elem = elem_of(columns[c].spark_type);
                    const auto& sm = slot_masks[2 * s + k];
                    if (sm.first >= 0) sd.col[k].validity = wmask[sm.first][sm.second];  // valid & where TRUE
                }
                sd.wout = slot_producer_of[s] >= 0 ? wodev[slot_producer_of[s]] : nullptr;
            } else {
                const int tag = (int)sd.col[0].flags;
                const int ref = (int)(intptr_t)sd.col[0].values;
                memset(&sd.col[0], 0, sizeof(ColDesc));
                sd.col[0].hll_slot = -1;
                sd.ncols = 1;
                if (tag == 1) sd.bits_valid = (const uint64_t*)dvalid[ref];
                if (tag == 2) { sd.pred_t = pt[ref]; sd.pred_nn = pn[ref]; }
            }
        }
        int rc = nslots ? upload(dslots, slots.data(), sizeof(SlotDesc) * nslots) : DQ_OK;
        if (rc) return rc;
        rc = upload(dops, opmap.data(), sizeof(OpMap) * nops);
        if (rc) return rc;
        if (nslots) {
            std::vector<int32_t> order;
            for (const Group& g : groups) order.insert(order.end(), g.slots.begin(), g.slots.end());
            rc = upload(dgroups, order.data(), sizeof(int32_t) * order.size());
            if (rc) return rc;
            rc = upload(dslot_nb, slot_nblocks.data(), sizeof(int32_t) * slot_nblocks.size());
            if (rc) return rc;
        }
        if (nsslots) {
            for (StrSlot& ss : sslots) {
                const int c = (int)(intptr_t)ss.values;
                const int w = (int)(intptr_t)ss.where_t - 1;
                ss.values = dval[c];
                ss.data = (const uint8_t*)dval[c];
                ss.offsets = (const int32_t*)doffs[c];
                ss.validity = (const uint64_t*)dvalid[c];
                ss.where_t = w >= 0 ? pt[w] : nullptr;
            }
            rc = upload(dsslots, sslots.data(), sizeof(StrSlot) * nsslots);
            if (rc) return rc;
        }
        // the scan launches: in order on the ctx stream, or one stream each (fork / join) when concurrent
        int used_side = 0;
        auto launch_stream = [&](int i) -> hipStream_t {
            if (!concurrent || i == 0) return ctx->stream;
            const int j = (i - 1) % dq_ctx::kSide;
            used_side = std::max(used_side, j + 1);
            return ctx->side[j];
        };
        int li = 0;
        size_t goff = 0;
        size_t gi = 0;
        auto launch_group = [&](const Group& g, hipStream_t st) -> int {
            if (launch_scan_group(g.kind, g.P, g.nc, g.f0, g.f1, g.heavy, dslots, dgroups + goff, (int)g.slots.size(), nrows,
                                  ntiles, gstride, g.grid, partials, hllp, st) != 0)
                return fail(ctx, DQ_ERR_DEVICE, "scan launch failed for shape (%d,%d,%d)", g.kind, g.P, g.nc);
            DQ_HIP(ctx, hipGetLastError());
            ctx->kernel_launches[scan_kernel_family(g.kind, g.P, g.nc, g.heavy)]++;
            goff += g.slots.size();
            return DQ_OK;
        };
        // `where` producers first, on the ctx stream: every other launch reads their masks
        for (; gi < groups.size() && groups[gi].heavy == 3; ++gi) {
            rc = launch_group(groups[gi], ctx->stream);
            if (rc) return rc;
        }
        if (concurrent) {
            DQ_HIP(ctx, hipEventRecord(ctx->fork_ev, ctx->stream));
            for (int j = 0; j < std::min(nlaunch - 1, dq_ctx::kSide); ++j)
                DQ_HIP(ctx, hipStreamWaitEvent(ctx->side[j], ctx->fork_ev, 0));
        }
        for (; gi < groups.size(); ++gi) {
            rc = launch_group(groups[gi], launch_stream(li++));
            if (rc) return rc;
        }
        if (nsslots) {
            launch_string_scan(dsslots, nsslots, nrows, sgrid, gstride, spartials, hllp, launch_stream(li++));
            DQ_HIP(ctx, hipGetLastError());
            ctx->kernel_launches[DQ_KERNEL_STRINGS]++;
        }
        for (int j = 0; j < used_side; ++j) {
            DQ_HIP(ctx, hipEventRecord(ctx->join_ev[j], ctx->side[j]));
            DQ_HIP(ctx, hipStreamWaitEvent(ctx->stream, ctx->join_ev[j], 0));
        }
        if (nslots) {
            launch_reduce_partials(partials, dslot_nb, nslots, gstride, finals, ctx->stream);
            DQ_HIP(ctx, hipGetLastError());
        }
        if (nslots || nsslots) ctx->scan_launches++;
        if (nhll) {
            rc = upload(dhll_nb, hll_nblocks.data(), sizeof(int32_t) * hll_nblocks.size());
            if (rc) return rc;
            launch_reduce_hll(hllp, dhll_nb, nhll, gstride, hllf, ctx->stream);
            DQ_HIP(ctx, hipGetLastError());
        }
        launch_finalize(dops, nops, finals, hllf, dout, ctx->stream);
        DQ_HIP(ctx, hipGetLastError());
        if (!sopmap.empty()) {
            rc = upload(dsops, sopmap.data(), sizeof(StrOpMap) * sopmap.size());
            if (rc) return rc;
            launch_finalize_strings(dsops, (int)sopmap.size(), spartials, sgrid, gstride, nrows, dout, ctx->stream);
            DQ_HIP(ctx, hipGetLastError());
        }
        if (any_regex) {
            // a row that exhausted the backtracking budget fails the batch (never a silent count)
            int32_t* hs = (int32_t*)hb.take(sizeof(int32_t) * std::max(npreds, 1), 16);
            DQ_HIP(ctx, hipMemcpyAsync(hs, rx_status, sizeof(int32_t) * std::max(npreds, 1), hipMemcpyDeviceToHost, ctx->stream));
            DQ_HIP(ctx, hipStreamSynchronize(ctx->stream));
            for (int p = 0; p < npreds; ++p)
                if (pred_pass[p] && hs[p])
                    return fail(ctx, DQ_ERR_UNSUPPORTED, "predicate %d: regex backtracking limit exceeded", p);
        }
        if (!(flags & DQ_SCAN_OUT_DEVICE)) {
            void* h = hb.take(sizeof(dq_state) * nops, 16);
            DQ_HIP(ctx, hipMemcpyAsync(h, dout, sizeof(dq_state) * nops, hipMemcpyDeviceToHost, ctx->stream));
            DQ_HIP(ctx, hipStreamSynchronize(ctx->stream));
            memcpy(out, h, sizeof(dq_state) * nops);
        } else {
            // Host columns were staged into the arena: keep them alive until the kernels finish.
            bool staged = false;
            for (int c = 0; c < ncols; ++c) staged |= col_used[c] && !(columns[c].flags & DQ_COL_DEVICE);
            if (staged) DQ_HIP(ctx, hipStreamSynchronize(ctx->stream));
        }
    }
    return DQ_OK;
}

// Host columns streamed through HBM in row chunks (tables larger than HBM, or host-resident batches): the copy
// of chunk i + 1 (its own stream, double-buffered device chunks) overlaps the fused scan of chunk i; every chunk's
// states land in device memory and the chunks are folded in row order with the reference merges (the partition
// merge of R/AnalysisRunner.scala:313) — the same result as any other row partitioning.
int dq_scan_streamed(dq_ctx* ctx, const dq_column* columns, int ncols, int64_t nrows, const dq_op* ops, int nops,
                     const dq_predicate* preds, int npreds, dq_state* out, int64_t chunk_rows) {
    if (!ctx || (nops > 0 && (!ops || !out)) || ncols < 0 || nrows < 0 || chunk_rows <= 0)
        return fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_scan_streamed: invalid arguments");
    ctx->err.clear();
    if (!ctx->subs.empty()) return fail(ctx, DQ_ERR_UNSUPPORTED, "dq_scan_streamed takes a single-device context");
    for (int c = 0; c < ncols; ++c)
        if ((columns[c].flags & DQ_COL_DEVICE) || columns[c].length != nrows)
            return fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_scan_streamed: column %d must be a host column of %lld rows", c,
                        (long long)nrows);
    if (nops == 0) return DQ_OK;
    chunk_rows = std::max<int64_t>(kTileRows, chunk_rows / kTileRows * kTileRows);
    if (nrows <= chunk_rows) return dq_scan(ctx, columns, ncols, nrows, ops, nops, preds, npreds, out, 0);
    DQ_HIP(ctx, hipSetDevice(ctx->device));
    const int64_t nchunks = (nrows + chunk_rows - 1) / chunk_rows;
    // device chunk buffers: 2 sets, each sized for the largest chunk of every column
    std::vector<size_t> vcap(ncols, 0), bcap(ncols, 0), ocap(ncols, 0);
    for (int c = 0; c < ncols; ++c) {
        const dq_column& col = columns[c];
        if (col.spark_type == DQ_TYPE_STRING) {
            size_t mx = 0;
            for (int64_t k = 0; k < nchunks; ++k) {
                const int64_t r0 = k * chunk_rows, r1 = std::min(nrows, r0 + chunk_rows);
                mx = std::max<size_t>(mx, (size_t)(col.offsets[r1] - col.offsets[r0]));
            }
            vcap[c] = mx + 16;
            ocap[c] = ((size_t)chunk_rows + 1) * 4;
        } else {
            vcap[c] = (size_t)chunk_rows * elem_size(elem_of(col.spark_type)) + 16;
        }
        if (col.validity) bcap[c] = (size_t)chunk_rows / 8 + 8;
    }
    struct Set { std::vector<void*> v, b, o; hipEvent_t copied, scanned; };
    Set sets[2];
    hipStream_t cstream = nullptr;
    std::vector<void*> allocs;
    dq_state* dstates = nullptr;
    std::vector<std::vector<int32_t>> rebased(2 * std::max(ncols, 1));
    auto cleanup = [&]() {
        (void)hipStreamSynchronize(ctx->stream);
        if (cstream) { (void)hipStreamSynchronize(cstream); (void)hipStreamDestroy(cstream); }
        for (Set& st : sets) {
            if (st.copied) (void)hipEventDestroy(st.copied);
            if (st.scanned) (void)hipEventDestroy(st.scanned);
        }
        for (void* p : allocs) (void)hipFree(p);
    };
    for (Set& st : sets) {
        st.copied = st.scanned = nullptr;
        st.v.assign(ncols, nullptr);
        st.b.assign(ncols, nullptr);
        st.o.assign(ncols, nullptr);
    }
    int rc = DQ_OK;
    auto dalloc = [&](size_t bytes) -> void* {
        void* p = nullptr;
        if (hipMalloc(&p, std::max<size_t>(bytes, 16)) != hipSuccess) return nullptr;
        allocs.push_back(p);
        return p;
    };
    for (Set& st : sets) {
        for (int c = 0; c < ncols && rc == DQ_OK; ++c) {
            if (!(st.v[c] = dalloc(vcap[c]))) rc = DQ_ERR_OUT_OF_MEMORY;
            if (bcap[c] && !(st.b[c] = dalloc(bcap[c]))) rc = DQ_ERR_OUT_OF_MEMORY;
            if (ocap[c] && !(st.o[c] = dalloc(ocap[c]))) rc = DQ_ERR_OUT_OF_MEMORY;
        }
        if (rc == DQ_OK && (hipEventCreateWithFlags(&st.copied, hipEventDisableTiming) != hipSuccess ||
                            hipEventCreateWithFlags(&st.scanned, hipEventDisableTiming) != hipSuccess))
            rc = DQ_ERR_DEVICE;
    }
    if (rc == DQ_OK && !(dstates = (dq_state*)dalloc(sizeof(dq_state) * (size_t)nops * nchunks))) rc = DQ_ERR_OUT_OF_MEMORY;
    if (rc == DQ_OK && hipStreamCreateWithFlags(&cstream, hipStreamNonBlocking) != hipSuccess) rc = DQ_ERR_DEVICE;
    if (rc != DQ_OK) {
        cleanup();
        return fail(ctx, rc, "dq_scan_streamed: chunk buffers of %lld rows do not fit", (long long)chunk_rows);
    }
    auto issue_copy = [&](int64_t k) -> int {
        Set& st = sets[k & 1];
        const int64_t r0 = k * chunk_rows, n = std::min(nrows, r0 + chunk_rows) - r0;
        for (int c = 0; c < ncols; ++c) {
            const dq_column& col = columns[c];
            if (col.spark_type == DQ_TYPE_STRING) {
                std::vector<int32_t>& ro = rebased[(k & 1) * ncols + c];
                ro.resize((size_t)n + 1);
                const int32_t base = col.offsets[r0];
                for (int64_t i = 0; i <= n; ++i) ro[i] = col.offsets[r0 + i] - base;
                if (ro[n]) DQ_HIP(ctx, hipMemcpyAsync(st.v[c], (const uint8_t*)col.values + base, ro[n], hipMemcpyHostToDevice, cstream));
                DQ_HIP(ctx, hipMemcpyAsync(st.o[c], ro.data(), ((size_t)n + 1) * 4, hipMemcpyHostToDevice, cstream));
            } else {
                const size_t es = elem_size(elem_of(col.spark_type));
                DQ_HIP(ctx, hipMemcpyAsync(st.v[c], (const uint8_t*)col.values + r0 * es, (size_t)n * es,
                                           hipMemcpyHostToDevice, cstream));
            }
            if (col.validity)
                DQ_HIP(ctx, hipMemcpyAsync(st.b[c], col.validity + r0 / 8, (size_t)(n + 7) / 8, hipMemcpyHostToDevice, cstream));
        }
        DQ_HIP(ctx, hipEventRecord(st.copied, cstream));
        return DQ_OK;
    };
    rc = issue_copy(0);
    std::vector<dq_column> dcols(std::max(ncols, 1));
    for (int64_t k = 0; k < nchunks && rc == DQ_OK; ++k) {
        Set& st = sets[k & 1];
        if (k + 1 < nchunks) {
            // buffer set (k + 1) & 1 was read by chunk k - 1's scan: wait for it, then start the next copy
            if (k >= 1 && hipEventSynchronize(sets[(k + 1) & 1].scanned) != hipSuccess) { rc = DQ_ERR_DEVICE; break; }
            rc = issue_copy(k + 1);
            if (rc) break;
        }
        if (hipStreamWaitEvent(ctx->stream, st.copied, 0) != hipSuccess) { rc = DQ_ERR_DEVICE; break; }
        const int64_t r0 = k * chunk_rows, n = std::min(nrows, r0 + chunk_rows) - r0;
        for (int c = 0; c < ncols; ++c) {
            dcols[c] = columns[c];
            dcols[c].flags |= DQ_COL_DEVICE;
            dcols[c].length = n;
            dcols[c].values = st.v[c];
            dcols[c].validity = columns[c].validity ? (const uint8_t*)st.b[c] : nullptr;
            dcols[c].offsets = columns[c].spark_type == DQ_TYPE_STRING ? (const int32_t*)st.o[c] : nullptr;
        }
        rc = dq_scan(ctx, dcols.data(), ncols, n, ops, nops, preds, npreds, dstates + (size_t)k * nops, DQ_SCAN_OUT_DEVICE);
        if (rc) break;
        if (hipEventRecord(st.scanned, ctx->stream) != hipSuccess) { rc = DQ_ERR_DEVICE; break; }
    }
    std::vector<dq_state> hst;
    if (rc == DQ_OK) {
        hst.resize((size_t)nops * nchunks);
        if (hipMemcpyAsync(hst.data(), dstates, sizeof(dq_state) * hst.size(), hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
            hipStreamSynchronize(ctx->stream) != hipSuccess)
            rc = DQ_ERR_DEVICE;
    }
    const std::string err = ctx->err;
    cleanup();
    if (rc) return fail(ctx, rc, "%s", err.empty() ? "dq_scan_streamed failed" : err.c_str());
    rc = dq_state_fold(hst.data(), (int)nchunks, nops, out);  // chunks in row order
    if (rc) return fail(ctx, rc, "dq_scan_streamed: state fold failed");
    return DQ_OK;
}

int dq_synth_column(dq_ctx* ctx, int32_t kind, uint64_t seed, int64_t row0, int64_t nrows, void* values_dev) {
    if (!ctx || nrows < 0 || (!values_dev && nrows > 0) || kind < DQ_SYNTH_DYADIC || kind > DQ_SYNTH_GAUSS_CORR)
        return fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_synth_column: invalid arguments");
    if (nrows == 0) return DQ_OK;
    DQ_HIP(ctx, hipSetDevice(ctx->device));
    launch_synth_column(kind, seed, row0, nrows, values_dev, ctx->stream);
    DQ_HIP(ctx, hipGetLastError());
    return DQ_OK;
}

int dq_synth_strings(dq_ctx* ctx, int32_t kind, uint64_t seed, int64_t row0, int64_t nrows, int32_t* offsets_dev,
                     void* bytes_dev, int64_t* total_bytes) {
    if (!ctx || nrows < 0 || !offsets_dev || !total_bytes || kind < DQ_SYNTH_STR_CAT50 || kind > DQ_SYNTH_STR_TEXT)
        return fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_synth_strings: invalid arguments");
    DQ_HIP(ctx, hipSetDevice(ctx->device));
    if (!bytes_dev) {
        // lengths into offsets[1..n], then an exclusive scan on the host (offsets are int32: < 2 GiB of text)
        DQ_HIP(ctx, hipMemsetAsync(offsets_dev, 0, 4, ctx->stream));
        if (nrows) launch_synth_string_lengths(kind, seed, row0, nrows, offsets_dev + 1, ctx->stream);
        DQ_HIP(ctx, hipGetLastError());
        std::vector<int32_t> h((size_t)nrows + 1);
        DQ_HIP(ctx, hipMemcpyAsync(h.data(), offsets_dev, ((size_t)nrows + 1) * 4, hipMemcpyDeviceToHost, ctx->stream));
        DQ_HIP(ctx, hipStreamSynchronize(ctx->stream));
        int64_t acc = 0;
        for (int64_t i = 1; i <= nrows; ++i) {
            acc += h[(size_t)i];
            if (acc > INT32_MAX) return fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_synth_strings: more than 2 GiB of text");
            h[(size_t)i] = (int32_t)acc;
        }
        DQ_HIP(ctx, hipMemcpyAsync(offsets_dev, h.data(), ((size_t)nrows + 1) * 4, hipMemcpyHostToDevice, ctx->stream));
        DQ_HIP(ctx, hipStreamSynchronize(ctx->stream));
        *total_bytes = acc;
        return DQ_OK;
    }
    if (nrows) launch_synth_string_bytes(kind, seed, row0, nrows, offsets_dev, bytes_dev, ctx->stream);
    DQ_HIP(ctx, hipGetLastError());
    return DQ_OK;
}

int dq_synth_freq_keys(dq_ctx* ctx, int64_t total_rows, int64_t distinct, int64_t row0, int64_t nrows, int64_t* keys_dev) {
    if (!ctx || total_rows <= 0 || distinct <= 0 || distinct > total_rows || nrows < 0 || row0 < 0 ||
        row0 + nrows > total_rows || (!keys_dev && nrows > 0))
        return fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_synth_freq_keys: invalid arguments");
    if (nrows == 0) return DQ_OK;
    DQ_HIP(ctx, hipSetDevice(ctx->device));
    launch_synth_freq_keys(total_rows, distinct, row0, nrows, keys_dev, ctx->stream);
    DQ_HIP(ctx, hipGetLastError());
    return DQ_OK;
}

int dq_synth_validity(dq_ctx* ctx, uint64_t seed, int64_t row0, int64_t nrows, int32_t null_permille, uint8_t* validity_dev) {
    if (!ctx || nrows < 0 || (!validity_dev && nrows > 0) || null_permille < 0 || null_permille > 1000)
        return fail(ctx, DQ_ERR_INVALID_ARGUMENT, "dq_synth_validity: invalid arguments");
    if (nrows == 0) return DQ_OK;
    DQ_HIP(ctx, hipSetDevice(ctx->device));
    launch_synth_validity(seed, row0, nrows, null_permille, validity_dev, ctx->stream);
    DQ_HIP(ctx, hipGetLastError());
    return DQ_OK;
}

}  // extern "C"
