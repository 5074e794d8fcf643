// multi.cpp — one context over several GPUs of one node (SURVEY.md §8b "multi-GPU: same calls; ctx
// row-shards internally and performs the merge").
//
// The reference merges partition aggregates inside its single `data.agg(...).collect()`
// (R/AnalysisRunner.scala:313); here the context splits the rows into contiguous 2048-row-aligned shards, one
// per GPU, runs every shard's fused scan concurrently (one host thread per device, each on its device's own
// stream) and folds the per-device states in device order with the reference semigroup merges
// (dq_state_fold = State.sum per state file) — the same result for any device count. Fixed-size states are a
// few KB and land in this process anyway, so they are folded on the host directly; the device-to-device
// traffic that matters is the frequency-table exchange (freq.hip), which goes over RCCL (ncclSend /
// ncclRecv grouped into one all-to-all over xGMI) between distinct GPUs.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <thread>
#include <vector>

#include "dq_common.h"
#include "dq_internal.h"

namespace dq {

// RCCL is bound at run time, on the first multi-GPU context: a process that already carries an RCCL (PyTorch
// ships its own librccl.so.1) shares that one — two copies of the library in one process corrupt each
// other's teardown — and a process without one (a JVM host) loads ROCm's.
struct Rccl {
    ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    bool ok = false;
};

static const Rccl& rccl() {
    static Rccl r = []() {
        Rccl x;
        void* h = dlopen("librccl.so.1", RTLD_LAZY | RTLD_NOLOAD);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_LAZY | RTLD_LOCAL);
        if (!h) h = dlopen("librccl.so.1", RTLD_LAZY | RTLD_LOCAL);
        if (!h) return x;
        x.CommInitAll = (decltype(x.CommInitAll))dlsym(h, "ncclCommInitAll");
        x.CommDestroy = (decltype(x.CommDestroy))dlsym(h, "ncclCommDestroy");
        x.GroupStart = (decltype(x.GroupStart))dlsym(h, "ncclGroupStart");
        x.GroupEnd = (decltype(x.GroupEnd))dlsym(h, "ncclGroupEnd");
        x.Send = (decltype(x.Send))dlsym(h, "ncclSend");
        x.Recv = (decltype(x.Recv))dlsym(h, "ncclRecv");
        x.ok = x.CommInitAll && x.CommDestroy && x.GroupStart && x.GroupEnd && x.Send && x.Recv;
        return x;
    }();
    return r;
}

int for_each_device(dq_ctx* ctx, int (*fn)(int, dq_ctx*, void*), void* arg) {
    const int n = (int)ctx->subs.size();
    std::vector<int> rc(n, DQ_OK);
    std::vector<std::thread> th;
    th.reserve(n);
    for (int i = 0; i < n; ++i)
        th.emplace_back([&, i]() {
            if (hipSetDevice(ctx->subs[i]->device) != hipSuccess) {
                rc[i] = DQ_ERR_DEVICE;
                return;
            }
            rc[i] = fn(i, ctx->subs[i], arg);
        });
    for (auto& t : th) t.join();
    for (int i = 0; i < n; ++i)
        if (rc[i] != DQ_OK) {
            ctx->err = "device " + std::to_string(ctx->subs[i]->device) + ": " + ctx->subs[i]->err;
            return rc[i];
        }
    return DQ_OK;
}

namespace {

struct ScanJob {
    const dq_column* const* cols;
    const int64_t* rows;
    int ncols;
    const dq_op* ops;
    int nops;
    const dq_predicate* preds;
    int npreds;
    std::vector<dq_state>* parts;
};

int scan_one(int i, dq_ctx* sub, void* arg) {
    ScanJob* j = static_cast<ScanJob*>(arg);
    return dq_scan(sub, j->cols[i], j->ncols, j->rows[i], j->ops, j->nops, j->preds, j->npreds,
                   j->parts->data() + (size_t)i * j->nops, 0);
}

}  // namespace

int multi_scan(dq_ctx* ctx, const dq_column* const* shard_cols, const int64_t* shard_rows, int ncols,
               const dq_op* ops, int nops, const dq_predicate* preds, int npreds, dq_state* out) {
    const int n = (int)ctx->subs.size();
    std::vector<dq_state> parts((size_t)n * std::max(nops, 1));
    ScanJob job{shard_cols, shard_rows, ncols, ops, nops, preds, npreds, &parts};
    int rc = for_each_device(ctx, scan_one, &job);
    if (rc) return rc;
    ctx->scan_launches++;
    // device-order fold with the reference merges: deterministic for a given device count
    rc = dq_state_fold(parts.data(), n, nops, out);
    if (rc) ctx->err = "dq_state_fold failed";
    return rc;
}

int exchange_i64(dq_ctx* ctx, const std::vector<int64_t*>& send, const std::vector<int64_t*>& recv,
                 const std::vector<int64_t>& counts, const std::vector<int64_t>& send_off,
                 const std::vector<int64_t>& recv_off) {
    const int n = (int)ctx->subs.size();
    if (ctx->comms) {
        ncclComm_t* comms = static_cast<ncclComm_t*>(ctx->comms);
        if (rccl().GroupStart() != ncclSuccess) { ctx->err = "ncclGroupStart failed"; return DQ_ERR_DEVICE; }
        for (int i = 0; i < n; ++i) {
            dq_ctx* sub = ctx->subs[i];
            for (int j = 0; j < n; ++j) {
                const int64_t c_out = counts[(size_t)i * n + j], c_in = counts[(size_t)j * n + i];
                if (c_out && rccl().Send(send[i] + send_off[(size_t)i * n + j], (size_t)c_out, ncclInt64, j, comms[i],
                                      sub->stream) != ncclSuccess) {
                    rccl().GroupEnd();
                    ctx->err = "ncclSend failed";
                    return DQ_ERR_DEVICE;
                }
                if (c_in && rccl().Recv(recv[i] + recv_off[(size_t)i * n + j], (size_t)c_in, ncclInt64, j, comms[i],
                                     sub->stream) != ncclSuccess) {
                    rccl().GroupEnd();
                    ctx->err = "ncclRecv failed";
                    return DQ_ERR_DEVICE;
                }
            }
        }
        if (rccl().GroupEnd() != ncclSuccess) { ctx->err = "ncclGroupEnd failed"; return DQ_ERR_DEVICE; }
    } else {
        // shards sharing a GPU (RCCL admits one rank per device): plain device copies
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < n; ++j) {
                const int64_t c = counts[(size_t)i * n + j];
                if (!c) continue;
                if (hipSetDevice(ctx->subs[i]->device) != hipSuccess ||
                    hipMemcpyPeerAsync(recv[j] + recv_off[(size_t)j * n + i], ctx->subs[j]->device,
                                       send[i] + send_off[(size_t)i * n + j], ctx->subs[i]->device, (size_t)c * 8,
                                       ctx->subs[i]->stream) != hipSuccess) {
                    ctx->err = "device copy of the exchange failed";
                    return DQ_ERR_DEVICE;
                }
            }
    }
    for (int i = 0; i < n; ++i)
        if (hipSetDevice(ctx->subs[i]->device) != hipSuccess || hipStreamSynchronize(ctx->subs[i]->stream) != hipSuccess) {
            ctx->err = "exchange synchronisation failed";
            return DQ_ERR_DEVICE;
        }
    return DQ_OK;
}

}  // namespace dq

using namespace dq;

extern "C" {

dq_ctx* dq_open_devices(const int* devices, int ndev, int* status) {
    if (!devices || ndev <= 0 || ndev > 64) {
        if (status) *status = DQ_ERR_INVALID_ARGUMENT;
        return nullptr;
    }
    // ndev == 1 is a real one-device multi context (one sub-context, an RCCL communicator of size 1): the
    // sharded path itself, not dq_open
    dq_ctx* ctx = dq_open(devices[0], status);  // the parent: device 0's own context (errors, metadata)
    if (!ctx) return nullptr;
    ctx->devices.assign(devices, devices + ndev);
    for (int i = 0; i < ndev; ++i) {
        int st = DQ_OK;
        dq_ctx* sub = dq_open(devices[i], &st);
        if (!sub) {
            dq_close(ctx);
            if (status) *status = st;
            return nullptr;
        }
        ctx->subs.push_back(sub);
    }
    std::vector<int> sorted(devices, devices + ndev);
    std::sort(sorted.begin(), sorted.end());
    const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
    if (distinct) {
        if (!rccl().ok) {
            dq_close(ctx);
            if (status) *status = DQ_ERR_DEVICE;
            return nullptr;
        }
        ncclComm_t* comms = new ncclComm_t[ndev];
        if (rccl().CommInitAll(comms, ndev, devices) != ncclSuccess) {
            delete[] comms;
            dq_close(ctx);
            if (status) *status = DQ_ERR_DEVICE;
            return nullptr;
        }
        ctx->comms = comms;
    }
    if (status) *status = DQ_OK;
    return ctx;
}

int dq_ctx_num_devices(const dq_ctx* ctx) { return !ctx ? 0 : (ctx->subs.empty() ? 1 : (int)ctx->subs.size()); }

int dq_ctx_uses_rccl(const dq_ctx* ctx) { return ctx && ctx->comms ? 1 : 0; }

int dq_scan_sharded(dq_ctx* ctx, const dq_column* const* shard_columns, const int64_t* shard_rows, int ncols,
                    const dq_op* ops, int nops, const dq_predicate* preds, int npreds, dq_state* out) {
    if (!ctx || !shard_columns || !shard_rows || (nops > 0 && (!ops || !out)) || ncols < 0 || nops < 0)
        return DQ_ERR_INVALID_ARGUMENT;
    ctx->err.clear();
    if (ctx->subs.empty())
        return dq_scan(ctx, shard_columns[0], ncols, shard_rows[0], ops, nops, preds, npreds, out, 0);
    return multi_scan(ctx, shard_columns, shard_rows, ncols, ops, nops, preds, npreds, out);
}

}  // extern "C"

// Called by dq_close for a multi-device context.
namespace dq {
void close_subs(dq_ctx* ctx) {
    if (ctx->comms) {
        ncclComm_t* comms = static_cast<ncclComm_t*>(ctx->comms);
        for (size_t i = 0; i < ctx->subs.size(); ++i) rccl().CommDestroy(comms[i]);
        delete[] comms;
        ctx->comms = nullptr;
    }
    for (dq_ctx* s : ctx->subs) dq_close(s);
    ctx->subs.clear();
}
}  // namespace dq
static_assert(dq::kTileRows == 2048, "host_algebra.cpp shards on 2048-row tiles");
