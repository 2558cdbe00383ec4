// Latency of dependent scalar loads from the kernel-argument segment vs from ordinary device
// memory (where the step kernel should read its parameter block from).
// One wave per launch walks a 40-step index chain idx = tab[idx] through (a) a 640-B by-value
// argument, (b) a device buffer holding the same table; it records s_memrealtime before and
// after (100 MHz) and writes ticks with a vector store. Graph replay and direct launches.
//   hipcc --offload-arch=gfx950 -O2 -o tools/kernarg_latency tools/kernarg_latency.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                     \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(2);                                                                         \
        }                                                                                         \
    } while (0)

struct Tab {
    unsigned v[160];
};

__global__ void chain_arg(Tab t, unsigned long long* out, int slot) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned idx = t.v[0];
#pragma unroll 1
    for (int i = 0; i < 40; ++i) idx = t.v[idx & 127];
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        out[2 * slot] = t1 - t0;
        out[2 * slot + 1] = idx;
    }
}

__global__ void chain_mem(const Tab* __restrict__ t, unsigned long long* out, int slot) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned idx = t->v[0];
#pragma unroll 1
    for (int i = 0; i < 40; ++i) idx = t->v[idx & 127];
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        out[2 * slot] = t1 - t0;
        out[2 * slot + 1] = idx;
    }
}

int main() {
    Tab h{};
    for (int i = 0; i < 160; ++i) h.v[i] = (unsigned)((i * 37 + 11) % 128);
    Tab* d = nullptr;
    unsigned long long* out = nullptr;
    CK(hipMalloc((void**)&d, sizeof(Tab)));
    CK(hipMemcpy(d, &h, sizeof(Tab), hipMemcpyHostToDevice));
    CK(hipMalloc((void**)&out, 64 * 16));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const int K = 8;
    // direct: slots 0..7 arg, 8..15 mem
    for (int i = 0; i < K; ++i) hipLaunchKernelGGL(chain_arg, dim3(1), dim3(64), 0, s, h, out, i);
    for (int i = 0; i < K; ++i) hipLaunchKernelGGL(chain_mem, dim3(1), dim3(64), 0, s, (const Tab*)d, out, K + i);
    // graph: slots 16..23 arg, 24..31 mem
    hipGraph_t g;
    hipGraphExec_t x;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < K; ++i) hipLaunchKernelGGL(chain_arg, dim3(1), dim3(64), 0, s, h, out, 2 * K + i);
    for (int i = 0; i < K; ++i) hipLaunchKernelGGL(chain_mem, dim3(1), dim3(64), 0, s, (const Tab*)d, out, 3 * K + i);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(x, s));
    CK(hipGraphLaunch(x, s));
    CK(hipStreamSynchronize(s));
    unsigned long long r[64 * 2];
    CK(hipMemcpy(r, out, 4 * K * 16, hipMemcpyDeviceToHost));
    const char* names[4] = {"direct_arg", "direct_mem", "graph_arg", "graph_mem"};
    std::printf("{\"unit\": \"ns per dependent scalar load (40-load chain, 100 MHz clock)\"");
    for (int m = 0; m < 4; ++m) {
        std::printf(", \"%s\": [", names[m]);
        for (int i = 0; i < K; ++i) std::printf("%s%.0f", i ? ", " : "", r[2 * (m * K + i)] * 10.0 / 40.0);
        std::printf("]");
    }
    std::printf("}\n");
    return 0;
}
