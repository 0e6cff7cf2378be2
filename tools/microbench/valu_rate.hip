// Micro-benchmark of the fp64 VALU issue rates that bound k_direct and k_traverse's force
// blocks: v_fma_f64, v_rsq_f64, and the exact point-force sequence of direct.hip (fastmath.hpp)
// with its operands in registers.  Every kernel also reads the shader clock (s_memtime) against
// the 100 MHz constant clock (s_memrealtime), so rates are reported per CU per shader clock.
// Build: see tools/microbench/Makefile.  Run: ./valu_rate
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../../barnes-hut-n-body_amd/csrc/fastmath.hpp"

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            std::printf("%s: %s\n", #x, hipGetErrorString(e_));                      \
            std::exit(1);                                                            \
        }                                                                            \
    } while (0)

constexpr int TB = 256;
constexpr int CHAINS = 8;

struct Clocks {
    unsigned long long shader, real;
};

__device__ __forceinline__ void stamp(Clocks *c, unsigned long long s0, unsigned long long r0) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        c->shader = __builtin_amdgcn_s_memtime() - s0;
        c->real = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

__global__ __launch_bounds__(TB) void k_fma(int iters, double a, double b, double *out, Clocks *c) {
    const unsigned long long s0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    double v[CHAINS];
#pragma unroll
    for (int k = 0; k < CHAINS; ++k) v[k] = threadIdx.x * 1e-3 + k;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < CHAINS; ++k) v[k] = __builtin_fma(v[k], a, b);
    }
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < CHAINS; ++k) s += v[k];
    out[blockIdx.x * TB + threadIdx.x] = s;
    stamp(c, s0, r0);
}

__global__ __launch_bounds__(TB) void k_rsq(int iters, double *out, Clocks *c) {
    const unsigned long long s0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    double v[CHAINS];
#pragma unroll
    for (int k = 0; k < CHAINS; ++k) v[k] = 2.0 + threadIdx.x * 1e-3 + k;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < CHAINS; ++k) v[k] = __builtin_amdgcn_rsq(v[k]);
    }
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < CHAINS; ++k) s += v[k];
    out[blockIdx.x * TB + threadIdx.x] = s;
    stamp(c, s0, r0);
}

// The fast-path point force of direct.hip (4 independent interactions per step, as k_direct's
// unroll): operands in registers, no LDS, so the loop measures the fp64 sequence alone.
__global__ __launch_bounds__(TB) void k_pair(int iters, double soft2, double *out, Clocks *c) {
    const unsigned long long s0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    const double bx = 100.0 + threadIdx.x, by = 50.0 + blockIdx.x % 97, Gm = 80.0 * 0.5;
    double px[4], py[4], pm[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        px[u] = 300.0 + 7.0 * u;
        py[u] = 200.0 - 3.0 * u;
        pm[u] = 0.5 + u;
    }
    double fx = 0.0, fy = 0.0;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const double dx = px[u] - bx, dy = py[u] - by;
            const double r2 = dx * dx + dy * dy + soft2;
            double h;
            const double r = bh::sqrt_rn_inrange_h(r2, h);
            const double invR = bh::rcp_rn_seeded(r, h + h);
            const double invR2 = bh::rcp_rn_seeded(r2, invR * invR);
            const double f = Gm * pm[u] * invR2;
            fx += f * dx * invR;
            fy += f * dy * invR;
            px[u] += 1.0;  // keeps the loop from being hoisted (one fp64 add per interaction)
        }
    }
    out[blockIdx.x * TB + threadIdx.x] = fx + fy;
    stamp(c, s0, r0);
}

int main() {
    int dev = 0, cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    int blocks = cus * 4 * 8 * 64 / TB;  // 8 waves per SIMD (k_pair also at 4: k_direct's C5 grid)
    double *out = nullptr;
    Clocks *c = nullptr;
    CK(hipMalloc(&out, sizeof(double) * blocks * TB));
    CK(hipMalloc(&c, sizeof(Clocks)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto report = [&](const char *name, double ops_per_iter_lane, int iters, auto launch) {
        for (int w = 0; w < 2; ++w) launch();
        CK(hipEventRecord(e0));
        launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        Clocks h{};
        CK(hipMemcpy(&h, c, sizeof(h), hipMemcpyDeviceToHost));
        const double mhz = h.real ? 100.0 * (double)h.shader / (double)h.real : 0.0;
        const double lane_ops = ops_per_iter_lane * iters * (double)blocks * TB;
        const double wave_instr_per_cu_clk = lane_ops / 64.0 / cus / (ms * 1e-3 * mhz * 1e6);
        std::printf("{\"kernel\": \"%s\", \"ms\": %.3f, \"clock_mhz\": %.0f, \"lane_ops_per_s\": %.4g, "
                    "\"wave_ops_per_cu_per_clk\": %.4f}\n",
                    name, ms, mhz, lane_ops / (ms * 1e-3), wave_instr_per_cu_clk);
    };
    const int it = 1 << 14;
    report("v_fma_f64", CHAINS, it, [&] { k_fma<<<blocks, TB>>>(it, 0.999999, 1e-9, out, c); });
    report("v_rsq_f64", CHAINS, it / 4, [&] { k_rsq<<<blocks, TB>>>(it / 4, out, c); });
    // per interaction: the 33 fp64 VALU ops + v_rsq_f64 of k_direct, + 1 add (px[u] += 1)
    report("point_force_interactions", 4, it / 16, [&] { k_pair<<<blocks, TB>>>(it / 16, 1.0, out, c); });
    blocks = cus * 4 * 4 * 64 / TB;  // 4 waves per SIMD: 262 144 bodies, one lane each
    report("point_force_interactions_4waves", 4, it / 16,
           [&] { k_pair<<<blocks, TB>>>(it / 16, 1.0, out, c); });
    CK(hipDeviceSynchronize());
    return 0;
}
