// fp32 3-D all-pairs N-body step — the physics of the reference's only GPU kernel
// (gpu/GPU.kt:101-152, an OpenGL compute shader), MI355X-native.
//
// Per body i:  a_i = sum_{j != i} (G m_j) d_ij / (|d_ij|^2 + soft^2)^{3/2},  d_ij = x_j - x_i
//              v_i += a_i dt;  x_i += v_i dt              (semi-implicit Euler, GPU.kt:145-146)
// in fp32 with the hardware reciprocal square root (GLSL inversesqrt, GPU.kt:140).  The
// reference updates its buffer in place while other invocations still read it (a race); here
// the step reads one buffer and writes the other (double-buffered), as SURVEY §8f asks.
//
// Layout: float4 (x, y, z, m) and float4 (vx, vy, vz, 0) per body, the shader's std430 Body.
// The kernel stages TILE bodies per workgroup in LDS and every lane (one body) reads them as
// broadcasts; two tile bodies per iteration with packed fp32 math (v_pk_fma_f32 / v_pk_mul_f32).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "bh_engine.h"

namespace {

constexpr int TB = 256;
constexpr int TILE = 1024;

typedef float float2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float2_t pk_fma(float2_t a, float2_t b, float2_t c) {
    return __builtin_elementwise_fma(a, b, c);
}

struct Tile {  // SoA so that two consecutive bodies load as one packed float2 per component
    float x[TILE], y[TILE], z[TILE], m[TILE];
};

// acceleration of the lane's body from every body (self excluded by index, GPU.kt:134)
__device__ __forceinline__ void accumulate(const float4 *__restrict__ pm, uint32_t n,
                                           uint32_t self, float3 p, float G, float soft2,
                                           Tile &tile, float3 &acc) {
    float2_t ax = {0.f, 0.f}, ay = {0.f, 0.f}, az = {0.f, 0.f};
    const float2_t px = {p.x, p.x}, py = {p.y, p.y}, pz = {p.z, p.z};
    const float2_t s2 = {soft2, soft2}, g2 = {G, G};
    for (uint32_t t0 = 0; t0 < n; t0 += TILE) {
        const uint32_t cnt = min((uint32_t)TILE, n - t0);
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < TILE; i += TB) {
            const float4 q = i < cnt ? pm[t0 + i] : make_float4(0.f, 0.f, 0.f, 0.f);  // m = 0 pads
            tile.x[i] = q.x;
            tile.y[i] = q.y;
            tile.z[i] = q.z;
            tile.m[i] = q.w;
        }
        __syncthreads();
        // self: its mass enters as 0, so its term is exactly 0 (soft2 > 0 keeps r2 > 0)
        const uint32_t sl = self - t0;
#pragma unroll 4
        for (uint32_t j = 0; j < TILE; j += 2) {
            const float2_t dx = *reinterpret_cast<const float2_t *>(tile.x + j) - px;
            const float2_t dy = *reinterpret_cast<const float2_t *>(tile.y + j) - py;
            const float2_t dz = *reinterpret_cast<const float2_t *>(tile.z + j) - pz;
            float2_t m = *reinterpret_cast<const float2_t *>(tile.m + j);
            if (j == (sl & ~1u)) m = (sl & 1u) ? float2_t{m.x, 0.f} : float2_t{0.f, m.y};
            const float2_t r2 = pk_fma(dz, dz, pk_fma(dy, dy, pk_fma(dx, dx, s2)));
            float2_t inv;
            inv.x = __builtin_amdgcn_rsqf(r2.x);
            inv.y = __builtin_amdgcn_rsqf(r2.y);
            const float2_t inv3 = inv * inv * inv;
            const float2_t s = (g2 * m) * inv3;  // (uG * other.w) * d * invR3
            ax = pk_fma(s, dx, ax);
            ay = pk_fma(s, dy, ay);
            az = pk_fma(s, dz, az);
        }
    }
    acc = make_float3(ax.x + ax.y, ay.x + ay.y, az.x + az.y);
}

__global__ __launch_bounds__(TB) void k_step3d(const float4 *__restrict__ pm_in,
                                               const float4 *__restrict__ vel_in,
                                               float4 *__restrict__ pm_out,
                                               float4 *__restrict__ vel_out, uint32_t n,
                                               float dt, float G, float soft2) {
    __shared__ Tile tile;
    const uint32_t i = blockIdx.x * TB + threadIdx.x;
    const bool valid = i < n;
    const float4 me = valid ? pm_in[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    float3 acc;
    accumulate(pm_in, n, valid ? i : 0xFFFFFFFFu, make_float3(me.x, me.y, me.z), G, soft2, tile,
               acc);
    if (!valid) return;
    float4 v = vel_in[i];
    v.x += acc.x * dt;  // GPU.kt:145-146
    v.y += acc.y * dt;
    v.z += acc.z * dt;
    pm_out[i] = make_float4(me.x + v.x * dt, me.y + v.y * dt, me.z + v.z * dt, me.w);
    vel_out[i] = make_float4(v.x, v.y, v.z, 0.f);
}

__global__ __launch_bounds__(TB) void k_acc3d(const float4 *__restrict__ pm, uint32_t n, float G,
                                              float soft2, float *__restrict__ a3) {
    __shared__ Tile tile;
    const uint32_t i = blockIdx.x * TB + threadIdx.x;
    const bool valid = i < n;
    const float4 me = valid ? pm[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    float3 acc;
    accumulate(pm, n, valid ? i : 0xFFFFFFFFu, make_float3(me.x, me.y, me.z), G, soft2, tile, acc);
    if (!valid) return;
    a3[3 * i] = acc.x;
    a3[3 * i + 1] = acc.y;
    a3[3 * i + 2] = acc.z;
}

}  // namespace

struct bh_nbody3d {
    int device = 0;
    hipStream_t stream = nullptr;
    int64_t n = 0, cap = 0;
    float4 *pm[2] = {nullptr, nullptr};
    float4 *vel[2] = {nullptr, nullptr};
    float *a3 = nullptr;
    int cur = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    float last_ms = 0.f;
    std::string err;
};

namespace {

#define HIPCHK3(h, expr)                                                               \
    do {                                                                               \
        hipError_t _st = (expr);                                                       \
        if (_st != hipSuccess) {                                                       \
            (h)->err = std::string(#expr) + ": " + hipGetErrorString(_st);            \
            return BH_E_DEVICE;                                                        \
        }                                                                              \
    } while (0)

int reserve3d(bh_nbody3d *h, int64_t n) {
    if (n <= h->cap) return BH_OK;
    for (int b = 0; b < 2; ++b) {
        if (h->pm[b]) (void)hipFree(h->pm[b]);
        if (h->vel[b]) (void)hipFree(h->vel[b]);
        h->pm[b] = h->vel[b] = nullptr;
        HIPCHK3(h, hipMalloc((void **)&h->pm[b], sizeof(float4) * n));
        HIPCHK3(h, hipMalloc((void **)&h->vel[b], sizeof(float4) * n));
    }
    if (h->a3) (void)hipFree(h->a3);
    h->a3 = nullptr;
    HIPCHK3(h, hipMalloc((void **)&h->a3, sizeof(float) * 3 * n));
    h->cap = n;
    return BH_OK;
}

}  // namespace

extern "C" {

int bh_nbody3d_create(int device, bh_nbody3d **out) {
    if (!out) return BH_E_INVALID;
    *out = nullptr;
    bh_nbody3d *h = new bh_nbody3d();
    h->device = device;
    if (hipSetDevice(device) != hipSuccess ||
        hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&h->ev0) != hipSuccess || hipEventCreate(&h->ev1) != hipSuccess) {
        delete h;
        return BH_E_DEVICE;
    }
    *out = h;
    return BH_OK;
}

void bh_nbody3d_destroy(bh_nbody3d *h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    for (int b = 0; b < 2; ++b) {
        if (h->pm[b]) (void)hipFree(h->pm[b]);
        if (h->vel[b]) (void)hipFree(h->vel[b]);
    }
    if (h->a3) (void)hipFree(h->a3);
    if (h->ev0) (void)hipEventDestroy(h->ev0);
    if (h->ev1) (void)hipEventDestroy(h->ev1);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

const char *bh_nbody3d_last_error(const bh_nbody3d *h) { return h ? h->err.c_str() : "null handle"; }

int bh_nbody3d_set(bh_nbody3d *h, int64_t n, const float *x, const float *y, const float *z,
                   const float *vx, const float *vy, const float *vz, const float *m) {
    if (!h || n < 0 || n > 0x7FFFFFFF || (n > 0 && (!x || !y || !z || !vx || !vy || !vz || !m)))
        return BH_E_INVALID;
    HIPCHK3(h, hipSetDevice(h->device));
    int rc = reserve3d(h, n > 0 ? n : 1);
    if (rc != BH_OK) return rc;
    std::vector<float4> pm((size_t)n), vel((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        pm[(size_t)i] = make_float4(x[i], y[i], z[i], m[i]);
        vel[(size_t)i] = make_float4(vx[i], vy[i], vz[i], 0.f);
    }
    h->cur = 0;
    h->n = n;
    if (n > 0) {
        HIPCHK3(h, hipMemcpy(h->pm[0], pm.data(), sizeof(float4) * n, hipMemcpyHostToDevice));
        HIPCHK3(h, hipMemcpy(h->vel[0], vel.data(), sizeof(float4) * n, hipMemcpyHostToDevice));
    }
    return BH_OK;
}

int bh_nbody3d_step(bh_nbody3d *h, int32_t k, float dt, float G, float softening) {
    if (!h || k < 0) return BH_E_INVALID;
    HIPCHK3(h, hipSetDevice(h->device));
    if (h->n == 0 || k == 0) return BH_OK;
    const float soft2 = softening * softening;  // GPU.kt:420 uSoftening = softening^2
    const unsigned grid = (unsigned)((h->n + TB - 1) / TB);
    HIPCHK3(h, hipEventRecord(h->ev0, h->stream));
    for (int32_t s = 0; s < k; ++s) {
        const int a = h->cur, b = a ^ 1;
        k_step3d<<<grid, TB, 0, h->stream>>>(h->pm[a], h->vel[a], h->pm[b], h->vel[b],
                                             (uint32_t)h->n, dt, G, soft2);
        h->cur = b;
    }
    HIPCHK3(h, hipGetLastError());
    HIPCHK3(h, hipEventRecord(h->ev1, h->stream));
    HIPCHK3(h, hipEventSynchronize(h->ev1));
    HIPCHK3(h, hipEventElapsedTime(&h->last_ms, h->ev0, h->ev1));
    return BH_OK;
}

int bh_nbody3d_accelerations(bh_nbody3d *h, float G, float softening, float *ax, float *ay,
                             float *az) {
    if (!h || (h->n > 0 && (!ax || !ay || !az))) return BH_E_INVALID;
    HIPCHK3(h, hipSetDevice(h->device));
    if (h->n == 0) return BH_OK;
    const unsigned grid = (unsigned)((h->n + TB - 1) / TB);
    HIPCHK3(h, hipEventRecord(h->ev0, h->stream));
    k_acc3d<<<grid, TB, 0, h->stream>>>(h->pm[h->cur], (uint32_t)h->n, G, softening * softening,
                                        h->a3);
    HIPCHK3(h, hipGetLastError());
    HIPCHK3(h, hipEventRecord(h->ev1, h->stream));
    std::vector<float> a3((size_t)(3 * h->n));
    HIPCHK3(h, hipMemcpyAsync(a3.data(), h->a3, sizeof(float) * 3 * h->n, hipMemcpyDeviceToHost,
                              h->stream));
    HIPCHK3(h, hipStreamSynchronize(h->stream));
    HIPCHK3(h, hipEventElapsedTime(&h->last_ms, h->ev0, h->ev1));
    for (int64_t i = 0; i < h->n; ++i) {
        ax[i] = a3[(size_t)(3 * i)];
        ay[i] = a3[(size_t)(3 * i + 1)];
        az[i] = a3[(size_t)(3 * i + 2)];
    }
    return BH_OK;
}

int bh_nbody3d_get(const bh_nbody3d *h, float *x, float *y, float *z, float *vx, float *vy,
                   float *vz, float *m, int64_t cap, int64_t *n_out) {
    if (!h || cap < 0) return BH_E_INVALID;
    if (n_out) *n_out = h->n;
    if (cap < h->n) return BH_E_CAPACITY;
    if (h->n == 0) return BH_OK;
    if (!x || !y || !z || !vx || !vy || !vz || !m) return BH_E_INVALID;
    std::vector<float4> pm((size_t)h->n), vel((size_t)h->n);
    if (hipSetDevice(h->device) != hipSuccess ||
        hipMemcpy(pm.data(), h->pm[h->cur], sizeof(float4) * h->n, hipMemcpyDeviceToHost) !=
            hipSuccess ||
        hipMemcpy(vel.data(), h->vel[h->cur], sizeof(float4) * h->n, hipMemcpyDeviceToHost) !=
            hipSuccess)
        return BH_E_DEVICE;
    for (int64_t i = 0; i < h->n; ++i) {
        const float4 p = pm[(size_t)i], v = vel[(size_t)i];
        x[i] = p.x;
        y[i] = p.y;
        z[i] = p.z;
        m[i] = p.w;
        vx[i] = v.x;
        vy[i] = v.y;
        vz[i] = v.z;
    }
    return BH_OK;
}

double bh_nbody3d_last_ms(const bh_nbody3d *h) { return h ? (double)h->last_ms : -1.0; }

}  // extern "C"
