// wait_value.hip -- probe for the one-launch LET evaluation: can the exchange
// stream wait (hipStreamWaitValue32) on a counter that the waves of a still-running traversal-like
// kernel increment, and how soon after the round's last wave does the waiting stream go on?
//
// One kernel of B one-wave workgroups (uneven busy loops) adds 1 to a counter at the end of every
// wave (system-scope release); a second stream waits for counter >= B, then stamps the wall clock.
// Prints the wait's delay after the last wave's stamp, for signal memory (hipMallocSignalMemory)
// and plain device memory.  The host gives up after 5 s (a wait that never completes).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>

#define CHK(x)                                                                            \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            std::printf("%s: %s\n", #x, hipGetErrorString(e_));                           \
            std::exit(1);                                                                 \
        }                                                                                 \
    } while (0)

__global__ void k_waves(uint32_t *ctr, int iters, unsigned long long *t_last, uint32_t *sink) {
    uint64_t x = threadIdx.x + 1;
    const int n = iters * (1 + (int)(blockIdx.x % 7));
    for (int i = 0; i < n; ++i) x = x * 6364136223846793005ull + 1442695040888963407ull;
    if (x == 0) sink[threadIdx.x] = 1u;  // (keeps the loop)
    if (threadIdx.x == 0) {
        atomicMax(t_last, (unsigned long long)wall_clock64());
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__global__ void k_stamp(unsigned long long *t) { *t = (unsigned long long)wall_clock64(); }

static int probe(bool signal, uint32_t blocks, int iters) {
    void *p = nullptr;
    if (signal)
        CHK(hipExtMallocWithFlags(&p, 8, hipMallocSignalMemory));
    else
        CHK(hipMalloc(&p, 64));
    uint32_t *ctr = static_cast<uint32_t *>(p);
    unsigned long long *t = nullptr;
    uint32_t *sink = nullptr;
    CHK(hipMalloc(&t, 2 * sizeof(unsigned long long)));
    CHK(hipMalloc(&sink, 64 * sizeof(uint32_t)));
    CHK(hipMemset(ctr, 0, signal ? 8 : 64));
    CHK(hipMemset(t, 0, 2 * sizeof(unsigned long long)));
    CHK(hipDeviceSynchronize());
    hipStream_t a, b;
    CHK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
    CHK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
    CHK(hipStreamWaitValue32(b, ctr, blocks, hipStreamWaitValueGte, 0xFFFFFFFFu));
    k_stamp<<<1, 1, 0, b>>>(t + 1);
    k_waves<<<blocks, 64, 0, a>>>(ctr, iters, t, sink);
    CHK(hipGetLastError());
    const auto t0 = std::chrono::steady_clock::now();
    bool done = false;
    while (std::chrono::steady_clock::now() - t0 < std::chrono::seconds(5)) {
        if (hipStreamQuery(b) == hipSuccess) {
            done = true;
            break;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    CHK(hipStreamSynchronize(a));
    if (!done) {
        std::printf("{\"memory\": \"%s\", \"blocks\": %u, \"released\": false}\n",
                    signal ? "signal" : "device", blocks);
        return 2;  // (the waiting stream is left to the process teardown)
    }
    unsigned long long h[2];
    uint32_t c = 0;
    CHK(hipMemcpy(h, t, sizeof(h), hipMemcpyDeviceToHost));
    CHK(hipMemcpy(&c, ctr, sizeof(c), hipMemcpyDeviceToHost));
    int mhz = 100;
    (void)hipDeviceGetAttribute(&mhz, hipDeviceAttributeWallClockRate, 0);  // kHz
    const double us = (double)((long long)(h[1] - h[0])) / ((double)mhz / 1000.0);
    std::printf("{\"memory\": \"%s\", \"blocks\": %u, \"released\": true, \"count\": %u, "
                "\"wait_after_last_wave_us\": %.2f}\n",
                signal ? "signal" : "device", blocks, c, us);
    CHK(hipStreamDestroy(a));
    CHK(hipStreamDestroy(b));
    CHK(hipFree(t));
    CHK(hipFree(sink));
    CHK(hipFree(p));
    return 0;
}

int main() {
    int can = 0;
    CHK(hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, 0));
    std::printf("{\"can_use_stream_wait_value\": %d}\n", can);
    if (!can) return 0;
    int rc = 0;
    for (uint32_t blocks : {256u, 4096u, 20000u}) {
        rc |= probe(true, blocks, 20000);
        if (rc) return rc;
        rc |= probe(false, blocks, 20000);
        if (rc) return rc;
    }
    return rc;
}
