// floor_probe.hip — measurement-only probe kernels (NOT part of librocket_hip.so): the latency
// floor of the N = 65 536 step kernel's shape, for the per-wave floor model in DESIGN.md §3.
//
// Every probe launches like step_kernel<6, RK4, AoS, HELP, WPB = 4> at N = 65 536: 256 workgroups
// of 4 main + 4 helper waves (512 threads), the same 30 KiB of static LDS (obs tiles + candidate
// rows), one main wave per SIMD. Variants:
//   kind 0  empty:  the waves start and exit (dispatch + wave launch + end-of-kernel);
//   kind 1  mem:    the step's memory pattern and nothing else — main waves load the counter word,
//                   the 12-B action row, the 14 state planes and v0 through buffer descriptors,
//                   then store the 14 planes + counter (sc1 write-through, as the helper-wave step
//                   kernels), reward / done / truncated (sc1) and the obs rows through the LDS tile
//                   as 16-B stores (sc1); helper waves load the counter word and publish a flag;
//   kind 2+c chain: mem + 32 c dependent-VALU rounds between the loads and the stores (c = 1..4,
//                   template instances so that a kernel trace separates them): 4 independent fma
//                   chains (the step's RK4 has that much ILP), one round = 4 v_fma_f32, straight-line,
//                   so a lone wave issues 128 c more VALU instructions than `mem`.
// fp_launch runs one launch on `stream`; fp_repeat k back-to-back launches.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {
constexpr int kWave = 64, kWPB = 4, kNS = 14;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
using rsrc_t = __amdgpu_buffer_rsrc_t;

__device__ __forceinline__ rsrc_t rsrc(const void* p, uint64_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0,
                                             (int)(bytes >= 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)bytes), 0x00020000);
}

template <int KIND, int CHAIN>
__global__ __launch_bounds__(2 * kWPB * kWave) void probe_kernel(float* state, const float* action, uint32_t n,
                                                                  float* obs, float* reward, uint8_t* done,
                                                                  uint8_t* trunc)
{
    __shared__ __attribute__((aligned(16))) float lds[kWPB][kWave * kNS];
    __shared__ __attribute__((aligned(16))) float cand[kWPB][kWave * 16];
    __shared__ uint32_t cflag[kWPB];
    if constexpr (KIND == 0) {
        if (threadIdx.x == 0) cflag[0] = 0u;  // keeps the LDS allocation
        return;
    } else {
        const uint32_t lane = threadIdx.x & (kWave - 1);
        const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
        const uint32_t plane = n * 4u;
        const rsrc_t st = rsrc(state, (uint64_t)(kNS + 3) * plane);
        if (wv >= (uint32_t)kWPB) {  // helper: counter word -> LDS row, flag
            const uint32_t k = wv - kWPB;
            const uint32_t i = (blockIdx.x * kWPB + k) * kWave + lane;
            const uint32_t cw = __builtin_amdgcn_raw_buffer_load_b32(st, (int)(i * 4u), (int)((kNS + 1) * plane), 0);
            cand[k][lane * 16] = __uint_as_float(cw);
            __hip_atomic_store(&cflag[k], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            return;
        }
        const uint32_t wave_base = (blockIdx.x * kWPB + wv) * kWave;
        const uint32_t i = wave_base + lane, vo = i * 4u;
        const uint32_t cw = __builtin_amdgcn_raw_buffer_load_b32(st, (int)vo, (int)((kNS + 1) * plane), 0);
        const u32x3 a = __builtin_amdgcn_raw_buffer_load_b96(rsrc(action, 3 * plane), (int)(vo * 3u), 0, 0);
        float y[kNS];
#pragma unroll
        for (int j = 0; j < kNS; ++j)
            y[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(st, (int)vo, (int)(j * plane), 0));
        float v0 = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(st, (int)vo, (int)(kNS * plane), 0));
        float c0 = y[0] + __uint_as_float(a.x), c1 = y[1] + __uint_as_float(a.y), c2 = y[2] + __uint_as_float(a.z),
              c3 = v0;
        if constexpr (CHAIN > 0) {
#pragma unroll
            for (int r = 0; r < CHAIN; ++r) {  // 4 independent dependent-fma chains
                c0 = fmaf(c0, 0.999f, y[3]);
                c1 = fmaf(c1, 0.999f, y[4]);
                c2 = fmaf(c2, 0.999f, y[5]);
                c3 = fmaf(c3, 0.999f, y[6]);
            }
        }
        y[0] = c0;
        y[1] = c1;
        y[2] = c2;
        y[13] += c3;
#pragma unroll
        for (int j = 0; j < kNS; ++j)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(y[j]), st, (int)vo, (int)(j * plane), 16);
        __builtin_amdgcn_raw_buffer_store_b32(cw + 1u, st, (int)vo, (int)((kNS + 1) * plane), 16);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(c0 + c1), rsrc(reward, plane), (int)vo, 0, 16);
        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(c2 > 0.0f), rsrc(done, n), (int)i, 0, 16);
        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(c3 > 0.0f), rsrc(trunc, n), (int)i, 0, 16);
        // the obs rows through the wave's LDS tile as 16-B stores (step_kernel's store_obs_tile)
        float2* l2 = reinterpret_cast<float2*>(&lds[wv][lane * kNS]);
#pragma unroll
        for (int j = 0; j < kNS / 2; ++j) l2[j] = make_float2(y[2 * j], y[2 * j + 1]);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const rsrc_t orr = rsrc(obs, (uint64_t)kNS * plane);
        const u32x4* src4 = reinterpret_cast<const u32x4*>(&lds[wv][0]);
        constexpr int NV = kWave * kNS / 4;  // 224 16-B stores per wave
#pragma unroll
        for (int q = 0; q < (NV + kWave - 1) / kWave; ++q) {
            const int k = lane + q * kWave;
            if (k < NV)
                __builtin_amdgcn_raw_buffer_store_b128(src4[k], orr, (int)(k * 16u), (int)(wave_base * kNS * 4u), 16);
        }
        if (lane == 0 && cflag[wv] == 2u) reward[0] = cand[wv][0];  // never true: keeps cand / cflag live
    }
}
}  // namespace

extern "C" {

// kind 0 empty, 1 mem, 2..5 mem + 128 x (kind - 1) VALU; n must be a multiple of 256. Returns 0 or
// a hipError_t (-1: bad argument).
int fp_launch(int kind, float* state, const float* action, int64_t n, float* obs, float* reward, uint8_t* done,
              uint8_t* trunc, void* stream)
{
    if (n <= 0 || n % (kWPB * kWave) != 0 || kind < 0 || kind > 5) return -1;
    const dim3 grid((unsigned)(n / (kWPB * kWave))), block(2 * kWPB * kWave);
    hipStream_t s = (hipStream_t)stream;
#define FP_L(K, C) hipLaunchKernelGGL((probe_kernel<K, C>), grid, block, 0, s, state, action, (uint32_t)n, obs, reward, done, trunc)
    switch (kind) {
        case 0: FP_L(0, 0); break;
        case 1: FP_L(1, 0); break;
        case 2: FP_L(1, 32); break;
        case 3: FP_L(1, 64); break;
        case 4: FP_L(1, 96); break;
        default: FP_L(1, 128); break;
    }
#undef FP_L
    return (int)hipGetLastError();
}

int fp_repeat(int kind, int64_t k, float* state, const float* action, int64_t n, float* obs, float* reward,
              uint8_t* done, uint8_t* trunc, void* stream)
{
    int rc = 0;
    for (int64_t t = 0; t < k && rc == 0; ++t) rc = fp_launch(kind, state, action, n, obs, reward, done, trunc, stream);
    return rc;
}

}  // extern "C"
