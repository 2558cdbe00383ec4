// launch_host_probe.hip — host-side cost of one kernel launch through the HIP runtime's entry
// points (diagnostic, not part of the library): an empty kernel taking a by-value argument block
// of the step kernel's size (~450 B: state / action pointers, N, mode word, KParams, Bufs,
// StepIO), launched K times back to back on one stream with
//   (a) hipLaunchKernelGGL (what rr_step uses),
//   (b) hipModuleLaunchKernel on the hipFunction_t from hipGetFuncBySymbol, arguments as kernelParams,
//   (c) the same with the argument block pre-packed (HIP_LAUNCH_PARAM_BUFFER_POINTER),
//   (d) hipExtLaunchKernel.
// Prints one JSON line: host microseconds per launch (median of 15 rounds of K launches).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

struct Blob {
    float f[96];
    void* p[10];
};

__global__ void empty_kernel(float* state, const float* action, uint32_t n, uint32_t mode, Blob b)
{
    if (n == 0xFFFFFFFFu && threadIdx.x == 0) state[0] = b.f[mode & 63] + action[0];
}

// ~`mode` x 10 ns of wall time per wave (100 MHz realtime clock): keeps the GPU behind the host
// so that launches queue up, as the step kernel's ~4.2 us do against ~2-5 us of host per launch
__global__ void busy_kernel(float* state, const float* action, uint32_t n, uint32_t mode, Blob b)
{
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < mode) __builtin_amdgcn_s_sleep(1);
    if (n == 0xFFFFFFFFu && threadIdx.x == 0) state[0] = b.f[mode & 63] + action[0];
}

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));          \
            return 1;                                                             \
        }                                                                         \
    } while (0)

int main()
{
    const int K = 200, R = 15;
    float* d = nullptr;
    CK(hipMalloc(&d, 4096));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    Blob b;
    std::memset(&b, 0, sizeof(b));
    uint32_t n = 65536, mode = 1;
    float* st = d;
    const float* ac = d + 16;
    hipFunction_t fn = nullptr;
    CK(hipGetFuncBySymbol(&fn, reinterpret_cast<const void*>(&empty_kernel)));
    // pre-packed argument block in the kernel's kernarg layout
    struct alignas(8) Packed {
        float* st;
        const float* ac;
        uint32_t n, mode;
        Blob b;
    } pk{st, ac, n, mode, b};
    size_t pk_size = sizeof(pk);
    void* extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &pk, HIP_LAUNCH_PARAM_BUFFER_SIZE, &pk_size, HIP_LAUNCH_PARAM_END};
    void* params[] = {&st, &ac, &n, &mode, &b};
    const char* names[] = {"hipLaunchKernelGGL", "hipModuleLaunchKernel_params", "hipModuleLaunchKernel_extra",
                           "hipExtLaunchKernel"};
    std::printf("{\"K\": %d, \"arg_bytes\": %zu", K, pk_size);
    for (int v = 0; v < 4; ++v) {
        std::vector<double> us;
        for (int r = 0; r < R + 2; ++r) {
            CK(hipStreamSynchronize(s));
            auto t0 = std::chrono::steady_clock::now();
            for (int k = 0; k < K; ++k) {
                if (v == 0)
                    hipLaunchKernelGGL(empty_kernel, dim3(128), dim3(512), 0, s, st, ac, n, mode, b);
                else if (v == 1)
                    CK(hipModuleLaunchKernel(fn, 128, 1, 1, 512, 1, 1, 0, s, params, nullptr));
                else if (v == 2)
                    CK(hipModuleLaunchKernel(fn, 128, 1, 1, 512, 1, 1, 0, s, nullptr, extra));
                else
                    CK(hipExtLaunchKernel(reinterpret_cast<const void*>(&empty_kernel), dim3(128), dim3(512), params,
                                          0, s, nullptr, nullptr, 0));
            }
            auto t1 = std::chrono::steady_clock::now();
            if (r >= 2) us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count() / K);
        }
        CK(hipStreamSynchronize(s));
        std::sort(us.begin(), us.end());
        std::printf(", \"%s_us\": %.3f", names[v], us[us.size() / 2]);
    }
    // busy kernels (~4 us each): does the host cost per launch grow when the queue backs up?
    for (int kk : {20, 200}) {
        for (uint32_t busy : {0u, 400u}) {
            std::vector<double> us;
            for (int r = 0; r < R + 2; ++r) {
                CK(hipStreamSynchronize(s));
                auto t0 = std::chrono::steady_clock::now();
                for (int k = 0; k < kk; ++k)
                    hipLaunchKernelGGL(busy_kernel, dim3(1024), dim3(256), 0, s, st, ac, n, busy, b);
                auto t1 = std::chrono::steady_clock::now();
                if (r >= 2) us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count() / kk);
            }
            CK(hipStreamSynchronize(s));
            std::sort(us.begin(), us.end());
            std::printf(", \"busy%u_K%d_us\": %.3f", busy, kk, us[us.size() / 2]);
        }
    }
    std::printf("}\n");
    CK(hipGetLastError());
    return 0;
}
