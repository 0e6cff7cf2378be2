// launch_floor.hip -- what a short kernel launch costs on the GPU, against the alternatives a small
// tree build could use instead (small body lists: ~12 launches of >= 5 us each).
//
//   chain   K launches back to back on one stream, per launch: 1 wave; 1024 x 256 threads each
//           writing one word; the same chain captured in a hipGraph and replayed
//   events  K launches of 1024 x 256 threads with timing: an event recorded between launches
//           (a marker in the queue) vs events attached to the launches (hipExtLaunchKernelGGL)
//   barrier one launch of B workgroups that meet R times at a grid barrier (one atomic counter and
//           a generation word, agent scope), per barrier: B spread over the XCDs, or B on one XCD
//           (8 B workgroups launched, those with blockIdx % 8 != 0 leave at once)
//
// A barrier poll gives up after ~2^24 tries and counts an error, so a non-resident workgroup
// cannot hang the run.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                            \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            std::printf("%s: %s\n", #x, hipGetErrorString(e_));                           \
            std::exit(1);                                                                 \
        }                                                                                 \
    } while (0)

__global__ void k_empty(uint32_t *p) {
    if (p && threadIdx.x == 1023u) p[0] = 1u;  // never true for the launch shapes used
}
__global__ void k_touch(uint32_t *p) { p[blockIdx.x * blockDim.x + threadIdx.x] = blockIdx.x; }

__device__ __forceinline__ void grid_barrier(uint32_t *count, uint32_t *gen, uint32_t nb,
                                             uint32_t &g, uint32_t *err) {
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t arrived =
            __hip_atomic_fetch_add(count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (arrived == nb - 1u) {
            __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(gen, g + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            uint32_t spins = 0;
            while (__hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) {
                if (++spins > (1u << 24)) {
                    __hip_atomic_fetch_add(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
            }
        }
        g += 1u;
    }
    __syncthreads();
}

__global__ void k_barriers(uint32_t *sync, int rounds, uint32_t nb, uint32_t stride,
                           uint32_t *data) {
    if (blockIdx.x % stride != 0u) return;
    uint32_t g = 0;
    uint32_t *count = sync, *gen = sync + 32, *err = sync + 64;
    for (int r = 0; r < rounds; ++r) {
        data[(blockIdx.x / stride) * blockDim.x + threadIdx.x] += (uint32_t)r;  // a little work
        grid_barrier(count, gen, nb, g, err);
    }
}

static float time_chain(hipStream_t s, int K, dim3 grid, dim3 block, bool touch, uint32_t *buf,
                        bool graph) {
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    hipGraphExec_t exec = nullptr;
    if (graph) {
        hipGraph_t gr;
        CHK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        for (int i = 0; i < K; ++i) {
            if (touch) k_touch<<<grid, block, 0, s>>>(buf);
            else k_empty<<<grid, block, 0, s>>>(nullptr);
        }
        CHK(hipStreamEndCapture(s, &gr));
        CHK(hipGraphInstantiate(&exec, gr, nullptr, nullptr, 0));
        CHK(hipGraphLaunch(exec, s));  // warm
        CHK(hipStreamSynchronize(s));
    }
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        CHK(hipEventRecord(a, s));
        if (graph) {
            CHK(hipGraphLaunch(exec, s));
        } else {
            for (int i = 0; i < K; ++i) {
                if (touch) k_touch<<<grid, block, 0, s>>>(buf);
                else k_empty<<<grid, block, 0, s>>>(nullptr);
            }
        }
        CHK(hipEventRecord(b, s));
        CHK(hipEventSynchronize(b));
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
    }
    return best * 1000.0f / K;  // us per launch
}

// mode 0: no events, 1: hipEventRecord before and after every launch, 2: events attached to the
// launch (hipExtLaunchKernelGGL start / stop)
static float time_events(hipStream_t s, int K, int mode, uint32_t *buf) {
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    hipEvent_t ev[2 * 64];
    for (int i = 0; i < 2 * 64; ++i) CHK(hipEventCreate(&ev[i]));
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        CHK(hipEventRecord(a, s));
        for (int i = 0; i < K; ++i) {
            hipEvent_t e0 = ev[(2 * i) % 128], e1 = ev[(2 * i + 1) % 128];
            if (mode == 1) CHK(hipEventRecord(e0, s));
            if (mode == 2)
                hipExtLaunchKernelGGL(k_touch, dim3(1024), dim3(256), 0, s, e0, e1, 0, buf);
            else
                k_touch<<<1024, 256, 0, s>>>(buf);
            if (mode == 1) CHK(hipEventRecord(e1, s));
        }
        CHK(hipEventRecord(b, s));
        CHK(hipEventSynchronize(b));
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
    }
    if (mode > 0) {  // the last launch's own interval
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, ev[(2 * (K - 1)) % 128], ev[(2 * (K - 1) + 1) % 128]));
        std::printf("{\"probe\": \"event_interval\", \"mode\": %d, \"last_launch_us\": %.2f}\n", mode,
                    ms * 1000.0f);
    }
    return best * 1000.0f / K;
}

static float time_barriers(hipStream_t s, uint32_t nb, uint32_t stride, int rounds, uint32_t *sync,
                           uint32_t *data, uint32_t *err_out) {
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        CHK(hipMemsetAsync(sync, 0, 128 * sizeof(uint32_t), s));
        CHK(hipEventRecord(a, s));
        k_barriers<<<nb * stride, 256, 0, s>>>(sync, rounds, nb, stride, data);
        CHK(hipEventRecord(b, s));
        CHK(hipEventSynchronize(b));
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
        uint32_t err = 0;
        CHK(hipMemcpy(&err, sync + 64, 4, hipMemcpyDeviceToHost));
        *err_out += err;
    }
    return best * 1000.0f;  // us per launch
}

int main() {
    hipStream_t s;
    CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    uint32_t *buf = nullptr, *sync = nullptr, *data = nullptr;
    CHK(hipMalloc(&buf, 1024 * 256 * sizeof(uint32_t)));
    CHK(hipMalloc(&sync, 128 * sizeof(uint32_t)));
    CHK(hipMalloc(&data, 2048 * 256 * sizeof(uint32_t)));
    CHK(hipMemset(data, 0, 2048 * 256 * sizeof(uint32_t)));
    const int K = 200;
    for (int g = 0; g < 2; ++g) {
        const bool graph = g == 1;
        std::printf("{\"probe\": \"chain\", \"graph\": %s, \"shape\": \"1x64 empty\", \"us_per_launch\": %.2f}\n",
                    graph ? "true" : "false", time_chain(s, K, dim3(1), dim3(64), false, buf, graph));
        std::printf("{\"probe\": \"chain\", \"graph\": %s, \"shape\": \"1024x256 one store\", \"us_per_launch\": %.2f}\n",
                    graph ? "true" : "false", time_chain(s, K, dim3(1024), dim3(256), true, buf, graph));
    }
    for (int mode = 0; mode < 3; ++mode)
        std::printf("{\"probe\": \"events\", \"mode\": \"%s\", \"us_per_launch\": %.2f}\n",
                    mode == 0 ? "none" : mode == 1 ? "hipEventRecord around" : "attached (hipExtLaunchKernelGGL)",
                    time_events(s, K, mode, buf));
    const uint32_t nbs[] = {8, 32, 64, 256};
    for (uint32_t nb : nbs) {
        for (uint32_t stride : {1u, 8u}) {
            if (stride == 8u && nb > 32u) continue;  // one XCD holds 32 CUs
            uint32_t err = 0;
            const float t0 = time_barriers(s, nb, stride, 0, sync, data, &err);
            const float t1 = time_barriers(s, nb, stride, 100, sync, data, &err);
            std::printf("{\"probe\": \"grid_barrier\", \"workgroups\": %u, \"one_xcd\": %s, "
                        "\"launch_us\": %.2f, \"us_per_barrier\": %.3f, \"errors\": %u}\n",
                        nb, stride == 8u ? "true" : "false", t0, (t1 - t0) / 100.0f, err);
        }
    }
    CHK(hipDeviceSynchronize());
    return 0;
}
