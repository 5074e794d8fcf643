// freq.hip — frequency tables for the grouping analyzers (placeholder until the HBM hash lands).
#include <hip/hip_runtime.h>

#include "dq_internal.h"

extern "C" {
int dq_frequencies(dq_ctx*, const dq_column*, int, int64_t, const int32_t*, int, uint32_t, dq_freq_table** t) {
    if (t) *t = nullptr;
    return DQ_ERR_UNSUPPORTED;
}
int dq_freq_summarize(dq_ctx*, const dq_freq_table*, int64_t, dq_freq_summary*) { return DQ_ERR_UNSUPPORTED; }
int64_t dq_freq_top(dq_ctx*, const dq_freq_table*, int64_t, int64_t*, int64_t*) { return -1; }
int64_t dq_freq_export(dq_ctx*, const dq_freq_table*, int64_t, int64_t*, int64_t*) { return -1; }
void dq_freq_free(dq_ctx*, dq_freq_table*) {}
}
