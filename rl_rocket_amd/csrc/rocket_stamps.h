// rocket_stamps.h — per-wave phase clocks of the DIAGNOSTIC builds only (-DRR_DIAG_STAMPS;
// tools/step_stamps.py, tools/step_stamps_graph.py, tools/exact_stamps.py, tools/collect_stamps.py).
// Without RR_DIAG_STAMPS every macro expands to nothing, so the shipped library's machine code is
// the same with or without these hooks (tests/test_isa_hash.py).
//
// Phase stamps (step / exact kernels): RR_STAMPS_BEGIN(N) at kernel entry, RR_STAMP(k) after
// phase k (k < N), RR_STAMPS_WRITE(dst, i, lane, ok, rt) at the end: lane 0 gets the cycles from
// entry to stamp 0, lane k those from stamp k - 1 to stamp k, and with rt the lanes N and N + 1 the
// wave's s_memrealtime at entry / at the write (100 MHz, low 32 bits, as float bit patterns); the
// values overwrite dst[i] (a per-env output such as the reward) of the wave's first lanes.
// Accumulated stamps (the collect's step loop): RR_ACC_BEGIN(N), RR_ST(p) adds the cycles since
// the previous stamp to phase p, RR_ACC_WRITE(dst, base, lane, ok) writes phase `lane` to dst[base + lane].
#pragma once

#if defined(RR_DIAG_STAMPS)
#define RR_STAMPS_BEGIN(N)                                                    \
    constexpr int rr_st_n = (N);                                              \
    const uint32_t rr_st_rt0 = (uint32_t)__builtin_amdgcn_s_memrealtime();    \
    const uint32_t rr_st_c0 = (uint32_t)__builtin_amdgcn_s_memtime();         \
    uint32_t rr_st_c[rr_st_n]
#define RR_STAMP(k)                                                           \
    do {                                                                      \
        __builtin_amdgcn_sched_barrier(0);                                    \
        rr_st_c[k] = (uint32_t)__builtin_amdgcn_s_memtime();                  \
        __builtin_amdgcn_sched_barrier(0);                                    \
    } while (0)
// stamp k once the NV values of `arr` are in registers (the loads of a phase have landed)
#define RR_STAMP_AFTER(k, arr, NV)                                            \
    do {                                                                      \
        _Pragma("unroll") for (int rr_j = 0; rr_j < (NV); ++rr_j)             \
            asm volatile("" ::"v"((arr)[rr_j]));                              \
        RR_STAMP(k);                                                          \
    } while (0)
#define RR_STAMPS_WRITE(dst, i, lane, ok, rt)                                 \
    do {                                                                      \
        __builtin_amdgcn_sched_barrier(0);                                    \
        const uint32_t rr_rt1 = (uint32_t)__builtin_amdgcn_s_memrealtime();   \
        float rr_v = (float)(rr_st_c[0] - rr_st_c0);                          \
        _Pragma("unroll") for (int rr_k = 1; rr_k < rr_st_n; ++rr_k)          \
            rr_v = (lane) == (uint32_t)rr_k ? (float)(rr_st_c[rr_k] - rr_st_c[rr_k - 1]) : rr_v; \
        if (rt) {                                                             \
            rr_v = (lane) == (uint32_t)rr_st_n ? __uint_as_float(rr_st_rt0) : rr_v;      \
            rr_v = (lane) == (uint32_t)rr_st_n + 1 ? __uint_as_float(rr_rt1) : rr_v;     \
        }                                                                     \
        if ((lane) < (uint32_t)rr_st_n + ((rt) ? 2u : 0u) && (ok)) (dst)[i] = rr_v;      \
    } while (0)
#define RR_ACC_BEGIN(N)                                                       \
    constexpr int rr_acc_n = (N);                                             \
    uint32_t rr_acc[rr_acc_n] = {};                                           \
    uint32_t rr_acc_prev = (uint32_t)__builtin_amdgcn_s_memtime()
#define RR_ST(p)                                                              \
    do {                                                                      \
        __builtin_amdgcn_sched_barrier(0);                                    \
        const uint32_t rr_t = (uint32_t)__builtin_amdgcn_s_memtime();         \
        rr_acc[p] += rr_t - rr_acc_prev;                                      \
        rr_acc_prev = rr_t;                                                   \
        __builtin_amdgcn_sched_barrier(0);                                    \
    } while (0)
#define RR_ACC_WRITE(dst, base, lane, ok)                                     \
    do {                                                                      \
        float rr_v = 0.0f;                                                    \
        _Pragma("unroll") for (int rr_p = 0; rr_p < rr_acc_n; ++rr_p)         \
            rr_v = (lane) == (uint32_t)rr_p ? (float)rr_acc[rr_p] : rr_v;     \
        if ((lane) < (uint32_t)rr_acc_n && (ok)) (dst)[(base) + (lane)] = rr_v; \
    } while (0)
#else
#define RR_STAMPS_BEGIN(N) static_assert((N) > 0, "")
#define RR_STAMP(k) \
    do {            \
    } while (0)
#define RR_STAMP_AFTER(k, arr, NV) \
    do {                           \
    } while (0)
#define RR_STAMPS_WRITE(dst, i, lane, ok, rt) \
    do {                                      \
    } while (0)
#define RR_ACC_BEGIN(N) static_assert((N) > 0, "")
#define RR_ST(p) \
    do {         \
    } while (0)
#define RR_ACC_WRITE(dst, base, lane, ok) \
    do {                                  \
    } while (0)
#endif
