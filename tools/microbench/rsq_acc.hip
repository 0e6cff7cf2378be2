// Accuracy of the hardware reciprocal square root seeds on gfx950: the largest relative error of
// v_rsq_f64 (the seed of the traversal's exact sqrt sequence, fastmath.hpp) and of v_rsq_f32 on
// the converted operand, against 1/sqrt(x) computed exactly (IEEE sqrt, then a correctly rounded
// division, error <= 1.5 ulp), over random operands in [1, 2^24) -- the physical range of the
// traversal's d2 (soft2 = 1, distances below the 2404-px root).  Build: tools/microbench/Makefile.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            std::printf("%s: %s\n", #x, hipGetErrorString(e_));                      \
            std::exit(1);                                                            \
        }                                                                            \
    } while (0)

__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// max relative error as the bits of a non-negative double (ordered like the values)
__global__ void k_acc(long long n, unsigned long long *worst) {
    unsigned long long w64 = 0, w32 = 0;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x) {
        const unsigned long long r = mix64((unsigned long long)i);
        const double x = __builtin_ldexp(1.0 + (double)(r >> 12) * 0x1p-52, (int)(r % 24));
        const double want = 1.0 / sqrt(x);
        const double a = __builtin_amdgcn_rsq(x);
        const double b = (double)__builtin_amdgcn_rsqf((float)x);
        const double ea = fabs(a - want) / want, eb = fabs(b - want) / want;
        const unsigned long long ba = (unsigned long long)__double_as_longlong(ea);
        const unsigned long long bb = (unsigned long long)__double_as_longlong(eb);
        w64 = ba > w64 ? ba : w64;
        w32 = bb > w32 ? bb : w32;
    }
    atomicMax(worst, w64);
    atomicMax(worst + 1, w32);
}

int main() {
    unsigned long long *d = nullptr, h[2] = {0, 0};
    CK(hipMalloc((void **)&d, sizeof(h)));
    CK(hipMemset(d, 0, sizeof(h)));
    const long long n = 1ll << 30;
    k_acc<<<4096, 256>>>(n, d);
    CK(hipGetLastError());
    CK(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
    double e64, e32;
    std::memcpy(&e64, &h[0], 8);
    std::memcpy(&e32, &h[1], 8);
    std::printf("{\"operands\": %lld, \"v_rsq_f64_max_rel_err\": %.3e, \"log2\": %.2f, "
                "\"v_rsq_f32_max_rel_err\": %.3e, \"log2_f32\": %.2f}\n",
                n, e64, std::log2(e64), e32, std::log2(e32));
    return 0;
}
