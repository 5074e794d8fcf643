#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <stdio.h>
#include <vector>
#include <random>
int main() {
    const size_t n = 65537;
    std::vector<unsigned long long> h(n);
    std::mt19937_64 g(1);
    for (auto& x : h) x = g();
    unsigned long long *a, *b;
    hipMalloc(&a, n * 8); hipMalloc(&b, n * 8);
    hipStream_t s; hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    for (int bits : {6, 13, 64}) {
        hipMemcpy(a, h.data(), n * 8, hipMemcpyHostToDevice);
        size_t tb = 0; void* t = nullptr;
        hipError_t e1 = rocprim::radix_sort_keys(nullptr, tb, a, b, n, 0, bits, s);
        hipMalloc(&t, tb);
        hipError_t e2 = rocprim::radix_sort_keys(t, tb, a, b, n, 0, bits, s);
        hipStreamSynchronize(s);
        std::vector<unsigned long long> o(n);
        hipMemcpy(o.data(), b, n * 8, hipMemcpyDeviceToHost);
        size_t bad = 0;
        for (size_t i = 1; i < n; ++i) { unsigned long long m = bits == 64 ? ~0ull : ((1ull << bits) - 1); if ((o[i] & m) < (o[i - 1] & m)) ++bad; }
        printf("bits=%d e=%d/%d tmp=%zu unsorted=%zu\n", bits, (int)e1, (int)e2, tb, bad);
        hipFree(t);
    }
    return 0;
}
