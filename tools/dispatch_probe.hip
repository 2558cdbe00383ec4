// Per-launch cost of K back-to-back launches of an empty kernel, timed with HIP events on
// the launch stream, four ways ("why K = 20 reads more than K = 2000"):
//   graph        K kernel nodes captured into one hipGraph, one replay
//   graph_gate   the same, the stream held behind a gate kernel until the host has
//                submitted the replay (so host submission is off the event interval)
//   direct       K hipLaunchKernelGGL calls
//   direct_gate  the same behind the gate
// plus the host time of the submitting call(s).
//   hipcc --offload-arch=gfx950 -O2 -o tools/dispatch_probe tools/dispatch_probe.hip
//   ./tools/dispatch_probe [K] [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(2);                                                               \
        }                                                                               \
    } while (0)

__global__ void empty_kernel(float* x) {
    if (x && threadIdx.x == 1024) x[0] = 1.0f;  // never true: keeps the argument live
}

// spins for `ticks` of the 100 MHz realtime clock (a kernel of fixed duration)
__global__ void spin_kernel(unsigned long long ticks) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
}

struct Big {  // a kernel-argument block the size of the step kernel's (KParams + Bufs + StepIO)
    float v[160];
};
__global__ void big_kernel(float* x, Big b) {
    if (x && threadIdx.x == 1024) x[0] = b.v[threadIdx.x & 127];
}

// One wave spins until the host-written word reaches `value` or `ticks` of the 100 MHz
// realtime clock pass (every path exits).
__global__ void gate_kernel(const unsigned* flag, unsigned value, unsigned long long ticks) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < value) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) break;
        __builtin_amdgcn_s_sleep(2);
    }
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    const int K = argc > 1 ? std::atoi(argv[1]) : 20;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 9;
    if (K < 1 || K > 100000 || reps < 1 || reps > 1000) return 2;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    unsigned* flag = nullptr;
    CK(hipHostMalloc((void**)&flag, 64, hipHostMallocCoherent));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, (float*)nullptr);
    CK(hipStreamSynchronize(s));

    hipGraph_t graph;
    hipGraphExec_t exec;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < K; ++i) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, (float*)nullptr);
    CK(hipStreamEndCapture(s, &graph));
    CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    CK(hipGraphLaunch(exec, s));
    CK(hipStreamSynchronize(s));

    unsigned gen = 0;
    const char* names[4] = {"graph", "graph_gate", "direct", "direct_gate"};
    std::printf("{\"k\": %d, \"reps\": %d", K, reps);
    for (int mode = 0; mode < 4; ++mode) {
        const bool gated = mode & 1, direct = mode >= 2;
        std::vector<double> dev, host;
        for (int r = 0; r < reps; ++r) {
            CK(hipStreamSynchronize(s));
            if (gated) {
                ++gen;
                hipLaunchKernelGGL(gate_kernel, dim3(1), dim3(64), 0, s, (const unsigned*)flag, gen, 100000ull);
            }
            CK(hipEventRecord(e0, s));
            const double t0 = now_us();
            if (direct) {
                for (int i = 0; i < K; ++i) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, (float*)nullptr);
            } else {
                CK(hipGraphLaunch(exec, s));
            }
            host.push_back(now_us() - t0);
            CK(hipEventRecord(e1, s));
            if (gated) __atomic_store_n(flag, gen, __ATOMIC_SEQ_CST);
            CK(hipStreamSynchronize(s));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            dev.push_back(ms * 1e3 / K);
        }
        std::sort(dev.begin(), dev.end());
        std::sort(host.begin(), host.end());
        std::printf(", \"%s\": {\"dev_us_per_launch\": %.4f, \"host_us_submit\": %.2f}", names[mode], dev[reps / 2],
                    host[reps / 2]);
    }
    // host cost per direct launch: a 8-B argument vs a 640-B argument block
    Big big{};
    for (int big_arg = 0; big_arg < 2; ++big_arg) {
        std::vector<double> host;
        for (int r = 0; r < reps; ++r) {
            CK(hipStreamSynchronize(s));
            const double t0 = now_us();
            for (int i = 0; i < K; ++i) {
                if (big_arg) hipLaunchKernelGGL(big_kernel, dim3(1), dim3(64), 0, s, (float*)nullptr, big);
                else hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, (float*)nullptr);
            }
            host.push_back((now_us() - t0) / K);
        }
        std::sort(host.begin(), host.end());
        std::printf(", \"host_us_per_launch_%s\": %.3f", big_arg ? "arg640" : "arg8", host[reps / 2]);
    }
    // GPU-bound: K launches of a 4-us kernel (256 waves), graph replay vs direct launches
    {
        hipGraph_t g2;
        hipGraphExec_t x2;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        for (int i = 0; i < K; ++i) hipLaunchKernelGGL(spin_kernel, dim3(256), dim3(64), 0, s, 400ull);
        CK(hipStreamEndCapture(s, &g2));
        CK(hipGraphInstantiate(&x2, g2, nullptr, nullptr, 0));
        CK(hipGraphLaunch(x2, s));
        CK(hipStreamSynchronize(s));
        for (int direct = 0; direct < 2; ++direct) {
            std::vector<double> dev, host;
            for (int r = 0; r < reps; ++r) {
                CK(hipStreamSynchronize(s));
                CK(hipEventRecord(e0, s));
                const double t0 = now_us();
                if (direct) {
                    for (int i = 0; i < K; ++i) hipLaunchKernelGGL(spin_kernel, dim3(256), dim3(64), 0, s, 400ull);
                } else {
                    CK(hipGraphLaunch(x2, s));
                }
                host.push_back((now_us() - t0) / K);
                CK(hipEventRecord(e1, s));
                CK(hipStreamSynchronize(s));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                dev.push_back(ms * 1e3 / K);
            }
            std::sort(dev.begin(), dev.end());
            std::sort(host.begin(), host.end());
            std::printf(", \"spin4us_%s\": {\"dev_us_per_launch\": %.4f, \"host_us_per_launch\": %.3f}",
                        direct ? "direct" : "graph", dev[reps / 2], host[reps / 2]);
        }
        CK(hipGraphExecDestroy(x2));
        CK(hipGraphDestroy(g2));
    }
    std::printf("}\n");
    CK(hipGraphExecDestroy(exec));
    CK(hipGraphDestroy(graph));
    CK(hipHostFree(flag));
    return 0;
}
