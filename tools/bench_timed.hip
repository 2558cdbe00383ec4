// bench_timed.hip — benchmark-only helper (NOT part of librocket_hip.so's ABI): the event-timed
// direct-launch region of bench.py (--launch loop, and --launch auto below K = 32).
//
//   bt_step_repeat_timed(rr_step, env, actions, n_batches, batch_floats, n_steps, obs, reward,
//                        done, truncated, terms, stream, ev_start, ev_end)
//
// issues n_steps calls of the library's public rr_step (passed as a function pointer, so this
// library links against nothing but the HIP runtime), step t taking action batch t % n_batches,
// with ev_start recorded right before the first launch and ev_end right after the last one.
// The stream is first held behind a one-wave gate kernel that this call releases once the
// first kGateQueued launches are submitted: a direct launch costs ~3 us of host time against
// ~4.1-4.4 us of GPU time per step at N = 65536, so from there on the host stays ahead and the
// events bracket back-to-back launches on the GPU timeline rather than the host's submission
// pace (without the gate the GPU idles while the first launch is submitted, and a stall of the
// submitting thread early in a short region lands inside it). The gate is time-bounded (1 s of
// the 100 MHz realtime clock) and released on every path, so every wave exits.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {
constexpr int64_t kGateQueued = 2;                // launches queued behind the gate before its release
constexpr uint64_t kGateMaxTicks = 100000000ull;  // 1 s of the 100 MHz realtime clock

__global__ __launch_bounds__(64) void gate_kernel(const uint32_t* word, uint32_t gen, uint64_t ticks)
{
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < gen) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) break;
        __builtin_amdgcn_s_sleep(2);
    }
}

uint32_t* g_word = nullptr;  // host-pinned, coherent
uint32_t g_gen = 0;

typedef int (*rr_step_fn)(void*, const float*, float*, float*, uint8_t*, uint8_t*, float*, void*);
}  // namespace

extern "C" {

// 0 on success; < 0: -1 bad argument, -2 HIP error, or the first failing rr_step's code
int bt_step_repeat_timed(void* rr_step, void* env, const float* actions, int64_t n_batches, int64_t batch_floats,
                         int64_t n_steps, float* obs, float* reward, uint8_t* done, uint8_t* truncated, float* terms,
                         void* stream, void* ev_start, void* ev_end)
{
    if (!rr_step || !env || !actions || n_batches <= 0 || n_steps < 0 || !ev_start || !ev_end) return -1;
    hipStream_t s = (hipStream_t)stream;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone) return -1;
    if (!g_word) {
        if (hipHostMalloc((void**)&g_word, 64, hipHostMallocCoherent) != hipSuccess) {
            g_word = nullptr;
            return -2;
        }
        __atomic_store_n(g_word, 0u, __ATOMIC_SEQ_CST);
    }
    const rr_step_fn step = (rr_step_fn)rr_step;
    const uint32_t gen = ++g_gen;
    hipLaunchKernelGGL(gate_kernel, dim3(1), dim3(64), 0, s, (const uint32_t*)g_word, gen, kGateMaxTicks);
    if (hipGetLastError() != hipSuccess) return -2;
    int rc = hipEventRecord((hipEvent_t)ev_start, s) == hipSuccess ? 0 : -2;
    bool held = true;
    for (int64_t t = 0; t < n_steps && rc == 0; ++t) {
        rc = step(env, actions + (t % n_batches) * batch_floats, obs, reward, done, truncated, terms, stream);
        if (held && t + 1 >= kGateQueued) {
            __atomic_store_n(g_word, gen, __ATOMIC_SEQ_CST);
            held = false;
        }
    }
    if (rc == 0 && hipEventRecord((hipEvent_t)ev_end, s) != hipSuccess) rc = -2;
    if (held) __atomic_store_n(g_word, gen, __ATOMIC_SEQ_CST);  // released on every path
    return rc;
}

}  // extern "C"
