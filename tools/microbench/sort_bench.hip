// Micro-benchmark of rocprim radix-sort configurations for the build's key sort
// (u64 Morton keys of 2J+1 = 43 bits, u32 payload).  Build: see tools/microbench/Makefile.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            std::printf("%s: %s\n", #x, hipGetErrorString(e_));                      \
            std::exit(1);                                                            \
        }                                                                            \
    } while (0)

template <class Cfg, class K>
float run(const char *name, size_t n, unsigned bits, const K *k_in, K *k_out,
          const uint32_t *v_in, uint32_t *v_out, int reps) {
    size_t bytes = 0;
    CK(rocprim::radix_sort_pairs<Cfg>(nullptr, bytes, k_in, k_out, v_in, v_out, n, 0u, bits));
    void *tmp = nullptr;
    CK(hipMalloc(&tmp, bytes));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 3; ++w)
        CK(rocprim::radix_sort_pairs<Cfg>(tmp, bytes, k_in, k_out, v_in, v_out, n, 0u, bits));
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r)
        CK(rocprim::radix_sort_pairs<Cfg>(tmp, bytes, k_in, k_out, v_in, v_out, n, 0u, bits));
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipFree(tmp));
    std::printf("%-28s n=%9zu bits=%u  %8.1f us\n", name, n, bits, 1e3f * ms / reps);
    return ms / reps;
}

template <unsigned R>
using Onesweep = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<256, 12>,
                                        rocprim::kernel_config<256, 12>, R>,
    0>;
template <unsigned R>
using OnesweepBig = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<256, 12>,
                                        rocprim::kernel_config<256, 16>, R>,
    0>;

int main() {
    const unsigned bits = 43;
    for (size_t n : {(size_t)1000000, (size_t)10000000}) {
        std::vector<uint64_t> hk(n);
        std::vector<uint32_t> hv(n);
        uint64_t s = 88172645463325252ull;
        for (size_t i = 0; i < n; ++i) {
            s ^= s << 13;
            s ^= s >> 7;
            s ^= s << 17;
            hk[i] = s & ((1ull << bits) - 1);
            hv[i] = (uint32_t)i;
        }
        uint64_t *k_in, *k_out;
        uint32_t *v_in, *v_out;
        CK(hipMalloc(&k_in, n * 8));
        CK(hipMalloc(&k_out, n * 8));
        CK(hipMalloc(&v_in, n * 4));
        CK(hipMalloc(&v_out, n * 4));
        CK(hipMemcpy(k_in, hk.data(), n * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(v_in, hv.data(), n * 4, hipMemcpyHostToDevice));
        const int reps = 20;
        run<rocprim::default_config>("default", n, bits, k_in, k_out, v_in, v_out, reps);
        run<Onesweep<4>>("onesweep 4b", n, bits, k_in, k_out, v_in, v_out, reps);
        run<Onesweep<6>>("onesweep 6b", n, bits, k_in, k_out, v_in, v_out, reps);
        run<Onesweep<8>>("onesweep 8b", n, bits, k_in, k_out, v_in, v_out, reps);
        run<Onesweep<7>>("onesweep 7b", n, bits, k_in, k_out, v_in, v_out, reps);
        run<OnesweepBig<8>>("onesweep 8b 256x16", n, bits, k_in, k_out, v_in, v_out, reps);
        run<OnesweepBig<6>>("onesweep 6b 256x16", n, bits, k_in, k_out, v_in, v_out, reps);
        // 32-bit keys (top 32 of the 43) + u32 payload; and the engine-like nearly sorted input
        {
            uint32_t *k32_in, *k32_out;
            CK(hipMalloc(&k32_in, n * 4));
            CK(hipMalloc(&k32_out, n * 4));
            std::vector<uint32_t> h32(n);
            for (size_t i = 0; i < n; ++i) h32[i] = (uint32_t)(hk[i] >> 11);
            CK(hipMemcpy(k32_in, h32.data(), n * 4, hipMemcpyHostToDevice));
            run<rocprim::default_config>("u32 keys default", n, 32, k32_in, k32_out, v_in, v_out, reps);
            std::sort(h32.begin(), h32.end());
            for (size_t i = 0; i + 1 < n; i += 7) std::swap(h32[i], h32[i + 1]);  // local disorder
            CK(hipMemcpy(k32_in, h32.data(), n * 4, hipMemcpyHostToDevice));
            run<rocprim::default_config>("u32 keys nearly sorted", n, 32, k32_in, k32_out, v_in, v_out, reps);
            CK(hipFree(k32_in));
            CK(hipFree(k32_out));
        }
        {
            std::vector<uint64_t> hs = hk;
            std::sort(hs.begin(), hs.end());
            for (size_t i = 0; i + 1 < n; i += 7) std::swap(hs[i], hs[i + 1]);
            CK(hipMemcpy(k_in, hs.data(), n * 8, hipMemcpyHostToDevice));
            run<rocprim::default_config>("u64 nearly sorted", n, bits, k_in, k_out, v_in, v_out, reps);
            CK(hipMemcpy(k_in, hk.data(), n * 8, hipMemcpyHostToDevice));
        }
        // sorted-check of the last run
        std::vector<uint64_t> ok(n);
        CK(hipMemcpy(ok.data(), k_out, n * 8, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (size_t i = 1; i < n; ++i) bad += ok[i - 1] > ok[i];
        std::printf("  last run sorted: %s\n", bad ? "NO" : "yes");
        CK(hipFree(k_in));
        CK(hipFree(k_out));
        CK(hipFree(v_in));
        CK(hipFree(v_out));
    }
    return 0;
}
