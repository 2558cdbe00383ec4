// rocket_hip.hip — MI355X (gfx950) kernels and C-ABI for the vectorized rocket env.
//
// One lane = one env. The per-env state lives in HBM as fp32 struct-of-arrays
// planes ([state_dim][N]); one launch of step_kernel does, for every env:
//   action denormalisation   (rocket_env.py:969-981 / :395-406)
//   RK4 integration of the rigid-body ODE over dt with the terminal ground event
//                            (simulator.py:227-294 / :55-130; the reference uses
//                             scipy RK45 + brentq on its dense output)
//   quaternion renormalisation / theta wrap (simulator.py:250 / :77)
//   bounds check, reward shaping, landing check, obs normalisation
//                            (rocket_env.py:690-719, 825-859, 963-1061 / :150-247, 431-476)
//   TimeLimit, auto-reset with an in-kernel RNG, done compaction by wave ballot
// with state kept in registers, the [N][state_dim] observation tile staged through
// LDS so that it leaves the CU as 16-byte coalesced stores.
//
// Element-wise ODE work: no contraction, so no MFMA. The roofline is HBM bytes
// (189 B per 6DOF env-step, 101 B per 3DOF env-step).

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <type_traits>
#include <vector>

#include "rocket_hip.h"
#include "rocket_stamps.h"


namespace {

// Newton iterations of the event root (2: -1.2 % per step, but the oracle-parity margin drops
// from 36x to 3x)
constexpr int kNewtonIters = 3;
// Cache-policy bits of the step kernel's buffer loads / stores (gfx950 CPol: 1 = sc0,
// 2 = nt, 16 = sc1); 0 = default policy. kStAux: library state planes (kernels above
// kHelpMaxN); kOutAux: caller-owned outputs.
constexpr int kLdAux = 0;
constexpr int kStAux = 0;
// state planes of the helper-wave step kernels (N <= kHelpMaxN): sc1 (device-scope write-through)
// where the whole batch's state is a few MB, so the end-of-kernel release has no dirty state
// lines to write back. A/B at N = 65536: direct launches 4.13-4.26 vs 4.34-4.55 us per step,
// hipGraph replays K = 20 4.39-4.41 vs 4.47-4.48, K = 2000 equal; at N = 524288 (plain kernel,
// default policy kept) it had cost 10-25 %.
constexpr int kStAuxHelp = 16;
// caller-owned outputs (obs, reward, done, truncated): sc1 = device-scope write-through, the
// outputs leave L2 while the kernel runs instead of in the end-of-kernel writeback (A/B at
// N = 65536: 5.49 -> 5.18 us; the same bit on the state planes, which the next launch re-reads,
// is slower; nt loads +5 %).
constexpr int kOutAux = 16;
// terminal obs rows (the done lanes' scattered 56 B) of the plain kernels (N > kHelpMaxN): nt.
// Past the MALL, 4-B stores from a few lanes of a wave cost far more than their bytes (one
// partial line each): at 4M envs in steady state (~1.5 % of the envs done per step) the
// terminal rows took ~24 us and the reset v0 ~20 us of a 200 us step. The rows go nt
// (197.5 -> 182.4 us; sc1 200.5, sc1 | nt 200.2); the terminal return / length and v0 are stored
// by every lane of a wave with a done lane, as whole lines, past the MALL (kModeWholeLines; v0:
// 174.3 -> 157.3 us with the rows off; profiles/r04/phase/done_path_ab.txt)
constexpr int kTermAuxLarge = 2;
// largest N stepped with helper waves (step_kernel<..., HELP = true>); RR_HELP_MAX_N in the
// environment overrides it at rr_create (tests select the plain kernel at small N with it)
constexpr int64_t kHelpMaxN = 131072;
// largest N stepped with one main wave per workgroup (helper variant)
constexpr int64_t kNarrowMaxN = 16384;
// exact mode: the one-wave-per-SIMD 6DOF kernel runs up to (CUs x 4 SIMDs x 64 lanes) envs, one
// env per lane; above it the lean two-waves-per-SIMD kernel (rocket_dopri5.inc, solve LEAN). The
// CU count is the device's (rr_create); kExactLeanCUs is the fallback if the query fails
constexpr int64_t kExactLeanCUs = 256;
constexpr int kWave = 64;
constexpr int kBlock = 256;  // threads per workgroup
constexpr int kWavesPerBlock = kBlock / kWave;

// ---------------------------------------------------------------------------
// Physical constants of the reference simulators.
//   6DOF: simulator.py:210-224 — g0 9.81, Isp 360, J = diag(75350.25, 6037675.13,
//         6037675.13), thrust hinge r_T_B = [-15, 0, 0], aero force identically 0.
//   3DOF: simulator.py:36-51, :100-126 — rho 1.225, Cd 0.3, Sref 10.5, alpha = 0
//         (normal force 0), I 6.04e6, lever x_T - x_CG = 30.
// ---------------------------------------------------------------------------
constexpr float kG0 = 9.81f;
constexpr double kIsp = 360.0;
constexpr double kJ1 = 75350.25, kJ2 = 6037675.13, kJ3 = 6037675.13;
constexpr double kRT = -15.0;
constexpr double kDrag3 = 0.5 * 1.225 * 0.3 * 10.5;  // A = Cd * (0.5 rho v^2) * Sref
constexpr double kLever3 = 40.0 - 10.0;               // x_T - x_CG
constexpr double kI3 = 6.04e6;
// folded into the device code as immediates
constexpr float kDmScale = (float)(-1.0 / (9.81 * kIsp));  // dm = T * kDmScale
constexpr float kJinv2 = (float)(1.0 / kJ2), kJinv3 = (float)(1.0 / kJ3);
constexpr float kJd1 = (float)(kJ1 - kJ3), kJd2 = (float)(kJ2 - kJ1);  // (w x Jw)_1 = kJd1 w1 w3, _2 = kJd2 w1 w2
constexpr float kRt = (float)(-kRT);  // tau = r_T_B x T_b = [0, 15 Tbz, -15 Tby]
static_assert(kJ2 == kJ3, "omega_1 is constant only for an axisymmetric body (J2 == J3)");
constexpr float kDrag3f = (float)kDrag3;
constexpr float kLeverOverI3 = (float)(kLever3 / kI3);
constexpr float kHalfPi = 1.57079632679489662f;
constexpr float kTwoPi = 6.28318530717958648f;

// Per-env counter word: TimeLimit steps in the low E bits, episodes started in the high
// 32 - E bits (keys the counter-based reset stream). E = bits of max_episode_steps (10 for the
// reference's TimeLimit 800: 2^22 episodes per env before the episode field wraps), 16 without
// a TimeLimit (KParams.el_mask / ep_shift, counter_bits()).
constexpr int32_t kMaxEpisodeSteps = 0xFFFF;
// step_kernel `mode` word: rr_params.flags plus "the counter word is live" and "the batch is
// past the MALL" (N > kWholeLineMinN: the done path's 4-B scalars leave as whole lines)
constexpr uint32_t kModeCounter = 0x80000000u;
constexpr uint32_t kModeWholeLines = 0x40000000u;
// ~200 B of state, action and outputs per env and step: above ~1M envs a step's working set
// passes the 256 MB MALL and partial lines become DRAM read-modify-writes (at 524 288, inside
// it, the whole-line stores measured 2-4 % slower; at 4 194 304 10 % faster). RR_WHOLE_LINE_MIN_N
// in the environment overrides it at rr_create (tests run the whole-line path at small N)
constexpr int64_t kWholeLineMinN = 1 << 20;

// Device-side constants, derived once on the host from rr_params (see make_kparams).
struct KParams {
    int32_t max_steps;
    uint32_t flags;
    float h, h2, h6;          // dt, dt/2, dt/6
    float ic_low[RR_MAX_STATE];
    float ic_span[RR_MAX_STATE];
    float inv_norm[RR_MAX_STATE];
    float blo[3], bhi[3];     // 6DOF: inclusive position box; 3DOF: x_lo(<=), x_hi(>=), z_hi(>=)
    float max_gimbal, half_thrust;
    float alfa, beta, eta, gamma, delta, kappa, xi;
    float waypoint, land_r2, land_v2;
    // attitude tests on the zyx Euler angles without inverse trig (make_kparams):
    //   |atan2(Y,X)| > L  <=>  X < r cos L ;  |asin(S)| > L  <=>  |S| > sin L
    float att_c[3];           // threshold per axis for "> limit"
    float land_c[3];          // threshold per axis for "< limit"
    uint32_t att_never;       // bit k: "|e_k| > limit" can never hold
    uint32_t land_always;     // bit k: "|e_k| < limit" always holds
    float omega_lt;           // |w| < omega_lim  (float threshold, reference 0.2)
    float zero_h;             // x <= 1e-3 as a float threshold
    uint32_t seed_w[4];       // reset stream key words (rr_seed)
    int64_t id_off;           // global id of env 0 (multi-GPU shards)
    // counter word: elapsed = cw & el_mask, episode = cw >> ep_shift. Last in the struct: placed
    // after `flags` they shifted the fields above and the kernel's kernarg scalar loads regrouped
    // (+2 % per step at N = 65536, A/B r02l)
    uint32_t el_mask, ep_shift;
};

// The parameters read after the integration (reward, bounds, obs). Copied out of the
// kernel arguments once at kernel start and pinned (pin_s) so the compiler cannot
// rematerialise them as scalar loads later: a lone wave per SIMD would otherwise stall
// on ~20 dependent s_load/s_waitcnt round trips inside the reward code (measured with
// per-wave s_memtime stamps in round 1: 2380 cycles for ~150 instructions).
struct HotParams {
    float inv_norm[RR_MAX_STATE];
    float blo[3], bhi[3];
    float half_thrust, alfa, beta, eta, gamma, delta, kappa, xi;
    float waypoint, land_r2, land_v2;
    float att_c[3], land_c[3];
    float omega_lt, zero_h;
    uint32_t att_never, land_always, flags;
};

template <class T>
__device__ __forceinline__ void pin_s(T& x)
{
    asm volatile("" : "+s"(x));
}

template <int NS>
__device__ __forceinline__ HotParams load_hot(const KParams& P)
{
    HotParams H;
#pragma unroll
    for (int j = 0; j < NS; ++j) {
        H.inv_norm[j] = P.inv_norm[j];
        asm volatile("" : "+v"(H.inv_norm[j]));
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        H.blo[j] = P.blo[j];
        H.bhi[j] = P.bhi[j];
        H.att_c[j] = P.att_c[j];
        H.land_c[j] = P.land_c[j];
        asm volatile("" : "+v"(H.blo[j]));
        asm volatile("" : "+v"(H.bhi[j]));
        asm volatile("" : "+v"(H.att_c[j]));
        asm volatile("" : "+v"(H.land_c[j]));
    }
#define RR_HOT(f) \
    H.f = P.f;    \
    pin_s(H.f)
    RR_HOT(half_thrust);
    RR_HOT(alfa);
    RR_HOT(beta);
    RR_HOT(eta);
    RR_HOT(gamma);
    RR_HOT(delta);
    RR_HOT(kappa);
    RR_HOT(xi);
    RR_HOT(waypoint);
    RR_HOT(land_r2);
    RR_HOT(land_v2);
    RR_HOT(omega_lt);
    RR_HOT(zero_h);
    RR_HOT(att_never);
    RR_HOT(land_always);
    RR_HOT(flags);
#undef RR_HOT
    return H;
}

struct Bufs {
    float* state;
    float* v0;
    uint32_t* counter;        // [N] counter word: elapsed in bits 0..E-1, episode above (E = KParams.ep_shift)
    float* ep_ret;
    uint64_t* done_bits;      // [ceil(N/64)] wave ballot of done lanes, one word per wave
    float* term_obs;
    float* term_ret;
    int32_t* term_len;
    int64_t n;
    const KParams* kp;        // device copy of the kernel's KParams: the helper waves read it (see step_kernel),
                              // and every kernel reads the reset-stream key seed_w from it, so rr_seed applies
                              // to every later launch, graph replays included
};

struct StepIO {
    const float* action;
    float* obs;
    float* reward;
    uint8_t* done;
    uint8_t* truncated;
    float* terms;
    int32_t obs_vec_ok;       // obs pointer 16-B aligned: LDS-staged float4 stores
};

__device__ __forceinline__ float frcp(float x) { return __builtin_amdgcn_rcpf(x); }

// packed fp32 pairs (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32 with op_sel swizzles)
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 pk_swap(f2 a) { return __builtin_shufflevector(a, a, 1, 0); }
__device__ __forceinline__ f2 pk_lo(f2 a) { return __builtin_shufflevector(a, a, 0, 0); }
__device__ __forceinline__ f2 pk_hi(f2 a) { return __builtin_shufflevector(a, a, 1, 1); }
__device__ __forceinline__ f2 pk_fma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 pk_his(f2 a, f2 b) { return __builtin_shufflevector(a, b, 1, 3); }  // (a.hi, b.hi)
__device__ __forceinline__ f2 pk_bc(float x) { return f2{x, x}; }


// Raw buffer access (SRSRC descriptor built from wave-uniform values): 32-bit per-lane
// voffset, per-plane offsets in soffset (SGPR) — no per-lane 64-bit address arithmetic.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
using rsrc_t = __amdgpu_buffer_rsrc_t;
__device__ __forceinline__ rsrc_t make_rsrc(const void* p, uint64_t bytes)
{
    const uint32_t nr = bytes >= 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)bytes;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)nr, 0x00020000);
}
__device__ __forceinline__ float bld_f(rsrc_t r, uint32_t voff, uint32_t soff)
{
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, (int)soff, kLdAux));
}
__device__ __forceinline__ uint32_t bld_u(rsrc_t r, uint32_t voff, uint32_t soff)
{
    return __builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, (int)soff, kLdAux);
}
template <int AUX = kStAux>
__device__ __forceinline__ void bst_f(rsrc_t r, float v, uint32_t voff, uint32_t soff)
{
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, (int)voff, (int)soff, AUX);
}
template <int AUX = kStAux>
__device__ __forceinline__ void bst_u(rsrc_t r, uint32_t v, uint32_t voff, uint32_t soff)
{
    __builtin_amdgcn_raw_buffer_store_b32(v, r, (int)voff, (int)soff, AUX);
}
template <int AUX = kStAux>
__device__ __forceinline__ void bst_u8(rsrc_t r, uint8_t v, uint32_t voff)
{
    __builtin_amdgcn_raw_buffer_store_b8(v, r, (int)voff, 0, AUX);
}

// Element idx of a wave-uniform base pointer with a 32-bit byte offset: lowers to the
// saddr + voffset form of global_load/store (no per-lane 64-bit address arithmetic).
template <class T>
__device__ __forceinline__ T& at(T* base, uint32_t idx)
{
    return *reinterpret_cast<T*>(reinterpret_cast<char*>(base) + (uint32_t)(idx * (uint32_t)sizeof(T)));
}
template <class T>
__device__ __forceinline__ const T& at(const T* base, uint32_t idx)
{
    return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + (uint32_t)(idx * (uint32_t)sizeof(T)));
}
__device__ __forceinline__ float frsq(float x) { return __builtin_amdgcn_rsqf(x); }
__device__ __forceinline__ float fsqrt(float x) { return __builtin_amdgcn_sqrtf(x); }  // v_sqrt_f32, no IEEE fixup

// 1 - exp(-x) for x >= 0 without cancellation: Taylor series below 1/8 (truncation
// < 2e-9 relative), v_exp_f32 above (result >= 0.117, so its ulp error stays relative).
__device__ __forceinline__ float one_minus_exp_neg(float x)
{
    const float p = x * (1.0f - x * (0.5f - x * (1.0f / 6.0f - x * (1.0f / 24.0f - x * (1.0f / 120.0f)))));
    const float e = 1.0f - __builtin_amdgcn_exp2f(-x * 1.44269504088896341f);
    return x < 0.125f ? p : e;
}

// ---------------------------------------------------------------------------
// Reset stream: counter-based. The initial condition an env `gid` gets when its episode
// ends at counter word `cw` (episode | steps, unique per env and step) comes from a
// register-resident xorshift128 (Marsaglia 2003) whose four words are chained lowbias32
// mixes of (seed words, gid, cw): no per-env RNG state lives in HBM, the draw needs only
// the counter word (so the step kernel draws it while the state planes are in flight),
// and it is independent of how envs are sharded. After the mixes every draw is 6 full-rate
// shift/xor ops; the top 24 bits of each draw make one uniform (statistics:
// tests/test_gpu_envs.py::test_reset_distribution).
// ---------------------------------------------------------------------------

// 32-bit avalanche mix (lowbias32)
__device__ __forceinline__ uint32_t mix32(uint32_t x)
{
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

struct ResetStream {
    uint32_t x, y, z, w;
    // next uniform in [0, 1) with 24 random bits
    __device__ __forceinline__ float uniform()
    {
        const uint32_t t = x ^ (x << 11);
        x = y;
        y = z;
        z = w;
        w = w ^ (w >> 19) ^ t ^ (t >> 8);
        return (float)(w >> 8) * 0x1p-24f;
    }
};

__device__ __forceinline__ ResetStream reset_stream(const uint32_t* seed_w, int64_t gid, uint32_t cw)
{
    // every state word is a nonlinear function of (gid, cw): a word that depended on gid
    // alone would correlate the components of one env's successive initial conditions
    const uint32_t g = mix32(((uint32_t)gid + seed_w[0]) ^ (uint32_t)((uint64_t)gid >> 32));
    ResetStream r;
    r.x = mix32(g ^ (cw + seed_w[1]));
    r.y = mix32(r.x ^ seed_w[2]);
    r.z = mix32(r.y ^ seed_w[3]);
    r.w = mix32(r.z ^ seed_w[0]);
    return r;
}

template <int MODEL>
struct Dims;
template <>
struct Dims<6> {
    static constexpr int NS = 14, NA = 3, NT = 5, EV = 0;  // event on x (altitude)
};
template <>
struct Dims<3> {
    static constexpr int NS = 7, NA = 2, NT = 6, EV = 1;   // event on z (altitude)
};

// Controls, fixed over one env step.
struct Ctl {
    // 6DOF: body-frame thrust T_b = T [cy cz, sy cz, sz] (simulator.py:311-318, :350-357)
    float tbx, tby, tbz;
    float tau1, tau2;       // r_T_B x T_b (simulator.py:373-378), component 0 is 0
    // 3DOF
    float sd, cd, thrust, dom;
    float dm;               // -T/(g0 Isp)
};

template <int MODEL>
__device__ __forceinline__ Ctl make_ctl(const KParams& P, const float* a)
{
    Ctl c;
    if constexpr (MODEL == 6) {
        float dy = a[0] * P.max_gimbal, dz = a[1] * P.max_gimbal;
        float T = (a[2] + 1.0f) * P.half_thrust;
        float cy = __cosf(dy), sy = __sinf(dy), cz = __cosf(dz), sz = __sinf(dz);
        c.tbx = T * (cy * cz);
        c.tby = T * (sy * cz);
        c.tbz = T * sz;
        c.tau1 = (kRt * kJinv2) * c.tbz;   // J2^-1 tau_1
        c.tau2 = (-kRt * kJinv3) * c.tby;  // J3^-1 tau_2
        c.dm = T * kDmScale;
    } else {
        float d = a[0] * P.max_gimbal;
        float T = (a[1] + 1.0f) * P.half_thrust;
        c.sd = __sinf(d);
        c.cd = __cosf(d);
        c.thrust = T;
        c.dom = -(T * c.sd) * kLeverOverI3;
        c.dm = T * kDmScale;
    }
    return c;
}

// 6DOF RHS, simulator.py:259-294. R(q/|q|) T_b (scipy Rotation.from_quat normalises,
// simulator.py:346) is applied as a quaternion rotation of the UNnormalised q scaled by
// 1/|q|^2 (R is homogeneous of degree 2 in q):  |q|^2 R T_b = |q|^2 T_b + w t + u x t,
// t = 2 u x T_b; the division by |q|^2 folds into the division by the mass.
template <int MODEL>
__device__ __forceinline__ void rhs(const KParams& P, const Ctl& c, const float* s, float* d)
{
    if constexpr (MODEL == 6) {
        const float q0 = s[6], q1 = s[7], q2 = s[8], q3 = s[9];
        const float w1 = s[10], w2 = s[11], w3 = s[12];
        const float qq = q0 * q0 + q1 * q1 + q2 * q2 + q3 * q3;
        const float tx = 2.0f * (q2 * c.tbz - q3 * c.tby);
        const float ty = 2.0f * (q3 * c.tbx - q1 * c.tbz);
        const float tz = 2.0f * (q1 * c.tby - q2 * c.tbx);
        const float Fx = qq * c.tbx + q0 * tx + (q2 * tz - q3 * ty);
        const float Fy = qq * c.tby + q0 * ty + (q3 * tx - q1 * tz);
        const float Fz = qq * c.tbz + q0 * tz + (q1 * ty - q2 * tx);
        const float sc = frcp(qq * s[13]);
        d[0] = s[3];
        d[1] = s[4];
        d[2] = s[5];
        d[3] = Fx * sc - kG0;
        d[4] = Fy * sc;
        d[5] = Fz * sc;
        // dq = 0.5 Omega(w) q with the unnormalised q (simulator.py:287, :362-370)
        const float h1 = 0.5f * w1, h2 = 0.5f * w2, h3 = 0.5f * w3;
        d[6] = -h1 * q1 - h2 * q2 - h3 * q3;
        d[7] = h1 * q0 + h3 * q2 - h2 * q3;
        d[8] = h2 * q0 - h3 * q1 + h1 * q3;
        d[9] = h3 * q0 + h2 * q1 - h1 * q2;
        // dw = J^-1 (tau - w x Jw) (simulator.py:288); J2 == J3 makes dw_1 = 0
        d[10] = 0.0f;
        d[11] = c.tau1 - (kJd1 * kJinv2) * (w1 * w3);
        d[12] = c.tau2 - (kJd2 * kJinv3) * (w1 * w2);
        d[13] = c.dm;
    } else {
        // 3DOF RHS, simulator.py:88-130 (N = 0; the z-drag uses cos(phi): reference quirk)
        const float th = s[2], vx = s[3], vz = s[4];
        float st = __sinf(th), ct = __cosf(th);
        float A = kDrag3f * (vx * vx + vz * vz);
        float cdt = c.cd * ct - c.sd * st;   // cos(delta + phi)
        float sdt = c.sd * ct + c.cd * st;   // sin(delta + phi)
        float im = frcp(s[6]);
        d[0] = vx;
        d[1] = vz;
        d[2] = s[5];
        d[3] = (c.thrust * cdt - A * ct) * im;
        d[4] = (c.thrust * sdt - A * ct) * im - kG0;
        d[5] = c.dom;
        d[6] = c.dm;
    }
}

// 6DOF RK4 specialised to the structure of the RHS (simulator.py:259-294): r and v never
// feed back (the aero force is identically zero, :359-360), so over one step they are
// quadratures of the stage accelerations a_s = R(q_s) T_b / m_s + g:
//   v1 = v0 + h/6 (a1 + 2 a2 + 2 a3 + a4),   r1 = r0 + h v0 + h^2/6 (a1 + a2 + a3)
// (the RK4 update itself, rearranged); m is linear in t (exact at every stage); w1 is
// constant (J2 == J3); q and (w2, w3) take the usual RK4 stages, carried as half-rates
// W = w/2 so dq = Omega(W) q needs no 0.5 factors. Same RK4 solution as the generic form
// (integrate) up to fp32 rounding. f0 = f(y0) for the event path.
// It runs on packed fp32 pairs (v_pk_fma_f32 / v_pk_mul_f32, two lanes'
// worth of fp32 per instruction): a lone wave issues one VALU instruction per 4 cycles
// whatever its width, so pairing the independent components of one env halves the issue
// cost of the quaternion and angular-rate algebra. Pairs: q = (q0,q1),(q2,q3);
// W = (W2,W3); a = (ax,ay), az. Each half rounds exactly like the scalar fma.

// o = y * inv_norm, two components per v_pk_mul_f32
template <int NS>
__device__ __forceinline__ void normalize_obs(const float* y, const float* inv_norm, float* o)
{
#pragma unroll
    for (int j = 0; j + 1 < NS; j += 2) {
        const f2 v = f2{y[j], y[j + 1]} * f2{inv_norm[j], inv_norm[j + 1]};
        o[j] = v.x;
        o[j + 1] = v.y;
    }
    if constexpr (NS % 2) o[NS - 1] = y[NS - 1] * inv_norm[NS - 1];
}

// Packed 6DOF RHS pieces for one step's controls: R(q) T_b / m + g as (ax, ay), az, and
// dq = Omega(W) q with W = w / 2 (pairs (q0,q1), (q2,q3); see rhs for the formulas).
struct Pk6 {
    f2 t2xy, tbxy, t2zn, t2yx, gxy;
    float t2z, tbz;
    __device__ __forceinline__ explicit Pk6(const Ctl& c)
    {
        t2xy = f2{2.0f * c.tbx, 2.0f * c.tby};
        t2z = 2.0f * c.tbz;
        tbxy = f2{c.tbx, c.tby};
        tbz = c.tbz;
        t2zn = f2{t2z, -t2z};
        t2yx = f2{-t2xy.y, t2xy.x};
        gxy = f2{-kG0, 0.0f};
    }
    __device__ __forceinline__ void accel(f2 q01, f2 q23, float m, f2& axy, float& az) const
    {
        const f2 sq = pk_fma(q01, q01, q23 * q23);
        const float qq = sq.x + sq.y;
        // t = 2 u x T_b, u = (q1, q2, q3), with qa = (q2, q1):
        //   (tx, ty) = qa (t2z, -t2z) + q3 (-t2y, t2x),   tz = q1 t2y - q2 t2x
        const f2 qa = __builtin_shufflevector(q23, q01, 0, 3);
        const f2 q3 = pk_hi(q23);
        const f2 txy = pk_fma(qa, t2zn, q3 * t2yx);
        const float tz = fmaf(q01.y, t2xy.y, -q23.x * t2xy.x);
        // F = |q|^2 T_b + q0 t + u x t;  (u x t)_xy = qa (tz, -tz) + q3 (-ty, tx)
        const f2 uxt = pk_fma(qa, f2{tz, -tz}, q3 * (pk_swap(txy) * f2{-1.0f, 1.0f}));
        const f2 Fxy = pk_fma(pk_bc(qq), tbxy, pk_fma(pk_lo(q01), txy, uxt));
        const float Fz = fmaf(qq, tbz, fmaf(q01.x, tz, fmaf(q01.y, txy.y, -q23.x * txy.x)));
        const float sc = frcp(qq * m);
        axy = pk_fma(Fxy, pk_bc(sc), gxy);
        az = Fz * sc;
    }
    // dq = Omega(W) q:
    //   (d0, d1) = (-W1, W1) (q1, q0) + (-W2, W3) (q2, q2) - (W3, W2) (q3, q3)
    //   (d2, d3) = (W2, W3) (q0, q0) + (-W3, W2) (q1, q1) + (W1, -W1) (q3, q2)
    static __device__ __forceinline__ void dq(f2 q01, f2 q23, float W1, f2 W, f2& d01, f2& d23)
    {
        const f2 w1a = {-W1, W1}, w1b = {W1, -W1};
        const f2 Wn = W * f2{-1.0f, 1.0f}, Ws = pk_swap(W), Wsn = Ws * f2{-1.0f, 1.0f};
        d01 = pk_fma(w1a, pk_swap(q01), pk_fma(Wn, pk_lo(q23), -(Ws * pk_hi(q23))));
        d23 = pk_fma(W, pk_lo(q01), pk_fma(Wsn, pk_hi(q01), w1b * pk_swap(q23)));
    }
};

// Full 6DOF RHS f(s) on the packed pieces (the ground-event path's f(y1)).
__device__ __forceinline__ void rhs6_pk(const Ctl& c, const float* s, float* d)
{
    const Pk6 k(c);
    f2 axy, d01, d23;
    float az;
    const f2 q01 = {s[6], s[7]}, q23 = {s[8], s[9]};
    k.accel(q01, q23, s[13], axy, az);
    const float W1 = 0.5f * s[10];
    const f2 W = {0.5f * s[11], 0.5f * s[12]};
    Pk6::dq(q01, q23, W1, W, d01, d23);
    const f2 A = {c.tau1, c.tau2};
    const f2 B = {(-kJd1 * kJinv2) * s[10], (-kJd2 * kJinv3) * s[10]};
    const f2 dw = pk_fma(B, f2{s[12], s[11]}, A);
    d[0] = s[3];
    d[1] = s[4];
    d[2] = s[5];
    d[3] = axy.x;
    d[4] = axy.y;
    d[5] = az;
    d[6] = d01.x;
    d[7] = d01.y;
    d[8] = d23.x;
    d[9] = d23.y;
    d[10] = 0.0f;
    d[11] = dw.x;
    d[12] = dw.y;
    d[13] = c.dm;
}

__device__ __forceinline__ void integrate6_rk4_pk(const KParams& P, const Ctl& c, const float* y0, float* y1,
                                                  float* f0)
{
    const float h = P.h, hh = P.h2, h6 = P.h6, hh6 = P.h * P.h6;
    const Pk6 k(c);
    auto accel = [&](f2 q01, f2 q23, float m, f2& axy, float& az) { k.accel(q01, q23, m, axy, az); };
    const float W1 = 0.5f * y0[10];
    // dW2 = A2 + B2 W3, dW3 = A3 + B3 W2 (half of dw = J^-1 (tau - w x Jw)): pair form
    // dW = A + B swap(W)
    const f2 A = {0.5f * c.tau1, 0.5f * c.tau2};
    const f2 B = {(-2.0f * kJd1 * kJinv2) * W1, (-2.0f * kJd2 * kJinv3) * W1};
    auto dq = [&](f2 q01, f2 q23, f2 W, f2& d01, f2& d23) { Pk6::dq(q01, q23, W1, W, d01, d23); };
    const f2 q01 = {y0[6], y0[7]}, q23 = {y0[8], y0[9]};
    const f2 W0 = {0.5f * y0[11], 0.5f * y0[12]};
    const float m0 = y0[13];
    const float mh = m0 + hh * c.dm, me = m0 + h * c.dm;
    const f2 hh2 = pk_bc(hh), h2 = pk_bc(h);
    f2 a1, a2, a3, a4, k101, k123, k201, k223, k301, k323, k401, k423, l1, l2, l3, l4;
    float a1z, a2z, a3z, a4z;
    // stage 1
    accel(q01, q23, m0, a1, a1z);
    dq(q01, q23, W0, k101, k123);
    l1 = pk_fma(B, pk_swap(W0), A);
    // stage 2
    f2 Ws = pk_fma(hh2, l1, W0);
    f2 qs01 = pk_fma(hh2, k101, q01), qs23 = pk_fma(hh2, k123, q23);
    accel(qs01, qs23, mh, a2, a2z);
    dq(qs01, qs23, Ws, k201, k223);
    l2 = pk_fma(B, pk_swap(Ws), A);
    // stage 3
    Ws = pk_fma(hh2, l2, W0);
    qs01 = pk_fma(hh2, k201, q01);
    qs23 = pk_fma(hh2, k223, q23);
    accel(qs01, qs23, mh, a3, a3z);
    dq(qs01, qs23, Ws, k301, k323);
    l3 = pk_fma(B, pk_swap(Ws), A);
    // stage 4
    Ws = pk_fma(h2, l3, W0);
    qs01 = pk_fma(h2, k301, q01);
    qs23 = pk_fma(h2, k323, q23);
    accel(qs01, qs23, me, a4, a4z);
    dq(qs01, qs23, Ws, k401, k423);
    l4 = pk_fma(B, pk_swap(Ws), A);
    // updates: v1 = v0 + h/6 (a1 + 2 a2 + 2 a3 + a4), r1 = r0 + h v0 + h^2/6 (a1 + a2 + a3)
    const f2 two = pk_bc(2.0f), h62 = pk_bc(h6), hh62 = pk_bc(hh6);
    const f2 v01 = {y0[3], y0[4]}, r01 = {y0[0], y0[1]};
    const f2 s23 = a2 + a3;
    const f2 v1 = pk_fma(h62, pk_fma(two, s23, a1 + a4), v01);
    const f2 r1 = pk_fma(hh62, a1 + s23, pk_fma(h2, v01, r01));
    const float s23z = a2z + a3z;
    y1[0] = r1.x;
    y1[1] = r1.y;
    y1[2] = (y0[2] + h * y0[5]) + hh6 * (a1z + s23z);
    y1[3] = v1.x;
    y1[4] = v1.y;
    y1[5] = y0[5] + h6 * (a1z + a4z + 2.0f * s23z);
    const f2 qe01 = pk_fma(h62, pk_fma(two, k201 + k301, k101 + k401), q01);
    const f2 qe23 = pk_fma(h62, pk_fma(two, k223 + k323, k123 + k423), q23);
    const f2 We = pk_fma(h62, pk_fma(two, l2 + l3, l1 + l4), W0);
    y1[6] = qe01.x;
    y1[7] = qe01.y;
    y1[8] = qe23.x;
    y1[9] = qe23.y;
    y1[10] = y0[10];
    y1[11] = 2.0f * We.x;
    y1[12] = 2.0f * We.y;
    y1[13] = me;
    f0[0] = y0[3];
    f0[1] = y0[4];
    f0[2] = y0[5];
    f0[3] = a1.x;
    f0[4] = a1.y;
    f0[5] = a1z;
    f0[6] = k101.x;
    f0[7] = k101.y;
    f0[8] = k123.x;
    f0[9] = k123.y;
    f0[10] = 0.0f;
    f0[11] = 2.0f * l1.x;
    f0[12] = 2.0f * l1.y;
    f0[13] = c.dm;
}

template <int MODEL, int INTEG>
__device__ __forceinline__ void integrate(const KParams& P, const Ctl& c, const float* y0, float h,
                                          float* y1, float* f0)
{
    constexpr int NS = Dims<MODEL>::NS;
    float k[NS], yt[NS];
    if constexpr (MODEL == 6 && INTEG == RR_INT_RK4) {
        integrate6_rk4_pk(P, c, y0, y1, f0);
        return;
    }
    if constexpr (INTEG == RR_INT_EULER) {
        rhs<MODEL>(P, c, y0, k);
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            f0[j] = k[j];
            y1[j] = y0[j] + h * k[j];
        }
    } else {
        const float hh = 0.5f * h, h6 = h * (1.0f / 6.0f);
        float acc[NS];
        rhs<MODEL>(P, c, y0, k);
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            f0[j] = k[j];
            acc[j] = k[j];
            yt[j] = y0[j] + hh * k[j];
        }
        rhs<MODEL>(P, c, yt, k);
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            acc[j] += 2.0f * k[j];
            yt[j] = y0[j] + hh * k[j];
        }
        rhs<MODEL>(P, c, yt, k);
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            acc[j] += 2.0f * k[j];
            yt[j] = y0[j] + h * k[j];
        }
        rhs<MODEL>(P, c, yt, k);
#pragma unroll
        for (int j = 0; j < NS; ++j) y1[j] = y0[j] + h6 * (acc[j] + k[j]);
    }
}

// Terminal ground event (solve_ivp events=..., terminal, direction 0; scipy
// ivp.find_active_events): sign change of the altitude between the step ends.
// The reference returns its RK45 dense output at the brentq root of the altitude
// (ivp.py handle_events, rk.py RkDenseOutput). Here the step's dense output is the
// cubic Hermite interpolant through (y0, f(y0)) and (y1, f(y1)) — 4th-order like the
// reference's — its altitude root is found by safeguarded Newton, and every state
// component is evaluated there. Explicit Euler (RR_INT_EULER) uses its own continuous extension,
// the line y0 + s h f(y0): root s = x0 / (x0 - x1) (oracle/rocket_oracle.c euler_step).
template <int MODEL, int INTEG>
__device__ __forceinline__ void event_step(const KParams& P, const Ctl& c, const float* y0, const float* f0,
                                           float* y1)
{
    constexpr int EV = Dims<MODEL>::EV;
    constexpr int NS = Dims<MODEL>::NS;
    const float x0 = y0[EV], x1 = y1[EV];
    if (x1 == 0.0f) return;  // root at the step end: state unchanged
    if constexpr (INTEG == RR_INT_EULER) {
        const float sh = (x0 * frcp(x0 - x1)) * P.h;
#pragma unroll
        for (int j = 0; j < NS; ++j) y1[j] = fmaf(sh, f0[j], y0[j]);
        return;
    }
    float f1[NS];
    if constexpr (MODEL == 6) rhs6_pk(c, y1, f1);
    else rhs<MODEL>(P, c, y1, f1);
    // straight-line code (one basic block with the RHS, so the scheduler interleaves the
    // two): x0 == 0 gives the secant guess 0 and H(0) == 0, so s stays 0 (y = y0, as the
    // reference's root at the step start)
    float s;
    {
        const float hv0 = P.h * f0[EV], hv1 = P.h * f1[EV];
        // the altitude's Hermite cubic in monomial form: H(s) = ((c3 s + c2) s + c1) s + c0
        const float dx = x1 - x0;
        const float c2 = 3.0f * dx - (2.0f * hv0 + hv1), c3 = (hv0 + hv1) - 2.0f * dx;
        const float d2 = 2.0f * c2, d3 = 3.0f * c3;
        const bool pos0 = x0 > 0.0f;
        float lo = 0.0f, hi = 1.0f;  // H(lo) has the sign of x0
        s = x0 * frcp(x0 - x1);
        // Newton from the secant guess, kept inside the closed sign bracket [lo, hi]
        // (bisection fallback). A converged iterate sits on a bracket end, so the test is
        // inclusive. Fixed 3 iterations, branch-free (quadratic convergence from the secant
        // guess; the parity tests cover touchdowns down to |v| ~ 1 m/s).
#pragma unroll
        for (int it = 0; it < kNewtonIters; ++it) {
            const float H = fmaf(fmaf(fmaf(c3, s, c2), s, hv0), s, x0);
            const float dH = fmaf(fmaf(d3, s, d2), s, hv0);
            const bool same = (H > 0.0f) == pos0;
            lo = same ? s : lo;
            hi = same ? hi : s;
            float sn = fmaf(-H, frcp(dH), s);
            sn = (sn >= lo && sn <= hi) ? sn : 0.5f * (lo + hi);
            s = (H == 0.0f) ? s : sn;
        }
    }
    // every component at the root: y = y0 + h01 (y1 - y0) + h10 f0 + h11 f1 (cubic Hermite)
    const float s2 = s * s, s3 = s2 * s;
    const float h01 = 3 * s2 - 2 * s3;
    const float h10 = P.h * (s3 - 2 * s2 + s), h11 = P.h * (s3 - s2);
    // two components per v_pk_fma_f32; w1 (6DOF) is constant over the step (J2 == J3) and the
    // mass is linear in t, so exact at the root
    const f2 H01 = {h01, h01}, H10 = {h10, h10}, H11 = {h11, h11};
    auto herm2 = [&](int j, int k) {
        const f2 a = {y0[j], y0[k]}, b = {y1[j], y1[k]};
        const f2 r = pk_fma(H11, f2{f1[j], f1[k]}, pk_fma(H10, f2{f0[j], f0[k]}, pk_fma(H01, b - a, a)));
        y1[j] = r.x;
        y1[k] = r.y;
    };
    herm2(0, 1);
    herm2(2, 3);
    herm2(4, 5);
    if constexpr (MODEL == 6) {
        herm2(6, 7);
        herm2(8, 9);
        herm2(11, 12);
    }
    y1[NS - 1] = fmaf(s * P.h, f0[NS - 1], y0[NS - 1]);
}

// After the step: _normalize_quaternion (simulator.py:250) / _wrapTo2Pi (simulator.py:150-163)
template <int MODEL>
__device__ __forceinline__ void post_integrate(float* y1)
{
    if constexpr (MODEL == 6) {
        // _normalize_quaternion (simulator.py:250)
        const f2 q01 = {y1[6], y1[7]}, q23 = {y1[8], y1[9]};
        const f2 sq = pk_fma(q01, q01, q23 * q23);
        const f2 rn = pk_bc(frsq(sq.x + sq.y));
        const f2 n01 = q01 * rn, n23 = q23 * rn;
        y1[6] = n01.x;
        y1[7] = n01.y;
        y1[8] = n23.x;
        y1[9] = n23.y;
    } else {
        // _wrapTo2Pi (simulator.py:150-163): fmod(fmod(theta, 2pi) + 2pi, 2pi)
        float th = fmodf(y1[2], kTwoPi) + kTwoPi;
        y1[2] = fmodf(th, kTwoPi);
    }
}

// A post-step state with a NaN / inf component ends the episode: the analogue of solve_ivp's
// status -1 (done = bool(status), simulator.py:236-241 -> rocket_env.py:702 / :158). scipy's RK45
// never returns on such a state (a NaN step size passes its `h_abs < min_step` test forever);
// the exact mode and the oracle stop it as TOO_SMALL_STEP (status -1), and here every
// component enters a sum of y_j * 0, which is +-0 for finite y_j and NaN otherwise (no
// overflow of finite values; 7 v_pk_fma_f32 for 6DOF). The terms plane reports status -1.
template <int NS>
__device__ __forceinline__ bool nonfinite(const float* y)
{
    f2 acc = pk_bc(0.0f);
#pragma unroll
    for (int j = 0; j + 1 < NS; j += 2) acc = pk_fma(f2{y[j], y[j + 1]}, pk_bc(0.0f), acc);
    float s = acc.x + acc.y;
    if constexpr (NS % 2) s = fmaf(y[NS - 1], 0.0f, s);
    return !(s == 0.0f);
}

// Sample one initial condition: gym Box.sample (uniform in [low, high], float32),
// then q <- q/|q| (rocket_env.py:672-673); v0 = |IC velocity| (rocket_env.py:989-991).
template <int MODEL, class IP>  // IP: KParams, or anything with its ic_low / ic_span (rol::ResetParams)
__device__ __forceinline__ void sample_ic(const IP& P, ResetStream& k, float* s, float& v0)
{
    constexpr int NS = Dims<MODEL>::NS;
#pragma unroll
    for (int j = 0; j < NS; ++j) s[j] = fmaf(P.ic_span[j], k.uniform(), P.ic_low[j]);
    if constexpr (MODEL == 6) {
        const float rn = frsq(s[6] * s[6] + s[7] * s[7] + s[8] * s[8] + s[9] * s[9]);
        s[6] *= rn;
        s[7] *= rn;
        s[8] *= rn;
        s[9] *= rn;
        v0 = fsqrt(s[3] * s[3] + s[4] * s[4] + s[5] * s[5]);
    } else {
        v0 = fsqrt(s[3] * s[3] + s[4] * s[4]);
    }
}

// Bounds violation on the float32 post-step state: 6DOF Box(lo, hi, float32).contains(r)
// (rocket_env.py:1036-1038, inclusive); 3DOF _check_bounds (rocket_env.py:431-447).
struct BoxParams {
    float blo[3], bhi[3];
};

template <int MODEL, class BP>
__device__ __forceinline__ bool bounds_hit(const BP& P, const float* s)
{
    if constexpr (MODEL == 6) {
        const bool inside = (s[0] >= P.blo[0]) & (s[0] <= P.bhi[0]) & (s[1] >= P.blo[1]) & (s[1] <= P.bhi[1]) &
                            (s[2] >= P.blo[2]) & (s[2] <= P.bhi[2]);
        return !inside;
    } else {
        return (s[0] <= P.blo[0]) | (s[0] >= P.bhi[0]) | (s[1] >= P.bhi[1]);
    }
}

// Reward / done of the reference env on the float32 post-step state.
template <int MODEL>
__device__ __forceinline__ float reward_terms(const HotParams& P, const float* s, const float* a, float v0,
                                              bool& bounds_violation, float* t)
{
    // Branch-free on purpose: the comparisons combine with bitwise & / | and the waypoint
    // cases with selects, so a lone wave runs straight-line code (short-circuit && / ||
    // compiled to ~8 exec-mask branches here).
    if constexpr (MODEL == 6) {
        bounds_violation = bounds_hit<6>(P, s);
        // _compute_vtarg (rocket_env.py:986-1014)
        const bool above = s[0] > P.waypoint;
        const float rh0 = above ? s[0] - P.waypoint : s[0] + 1.0f;
        const float rh1 = above ? s[1] : 0.0f, rh2 = above ? s[2] : 0.0f;
        const float vh0 = s[3] + (above ? 2.0f : 1.0f);
        const float tau_inv = above ? 1.0f / 20.0f : 1.0f / 100.0f;
        float nrh = fsqrt(rh0 * rh0 + rh1 * rh1 + rh2 * rh2);
        float t_go = nrh * frsq(vh0 * vh0 + s[4] * s[4] + s[5] * s[5]);
        float f = (-v0 * frcp(fmaxf(1e-3f, nrh))) * one_minus_exp_neg(t_go * tau_inv);
        float e0 = s[3] - f * rh0, e1 = s[4] - f * rh1, e2 = s[5] - f * rh2;
        t[0] = P.alfa * fsqrt(e0 * e0 + e1 * e1 + e2 * e2);
        // thrust_penalty = beta * T (denormalised, float32)
        t[1] = P.beta * ((a[2] + 1.0f) * P.half_thrust);
        t[2] = P.eta;
        // zyx Euler angles of q (Rotation.as_euler("zyx"), rocket_env.py:852-855, 1047):
        //   a = atan2(-R01, R00), b = asin(R02), c = atan2(-R12, R22)
        const float w = s[6], x = s[7], y = s[8], z = s[9];
        float R00 = w * w + x * x - y * y - z * z;
        float mR01 = 2.0f * (z * w - x * y);
        float R02 = 2.0f * (x * z + y * w);
        float mR12 = 2.0f * (x * w - y * z);
        float R22 = w * w - x * x - y * y + z * z;
        float ra = fsqrt(R00 * R00 + mR01 * mR01);
        float rc = fsqrt(R22 * R22 + mR12 * mR12);
        // q was renormalised after the step (|q|^2 = 1 to fp32 rounding), so sin b = R02
        // without the division by |q|^2 (R00, R22 and the cos b radii are homogeneous)
        float sb = fabsf(R02);
        const bool att = (!(P.att_never & 1u) & (R00 < ra * P.att_c[0])) | (!(P.att_never & 2u) & (sb > P.att_c[1])) |
                         (!(P.att_never & 4u) & (R22 < rc * P.att_c[2]));
        t[3] = att ? P.gamma : 0.0f;
        // _check_landing (rocket_env.py:1040-1061); any() over angles and omega is the reference's
        const bool att_ok = (P.land_always != 0u) | (R00 > ra * P.land_c[0]) | (sb < P.land_c[1]) |
                            (R22 > rc * P.land_c[2]);
        const bool om_ok = (fabsf(s[10]) < P.omega_lt) | (fabsf(s[11]) < P.omega_lt) | (fabsf(s[12]) < P.omega_lt);
        float r2 = s[0] * s[0] + s[1] * s[1] + s[2] * s[2];
        float v2 = s[3] * s[3] + s[4] * s[4] + s[5] * s[5];
        const bool landing = (s[0] <= P.zero_h) & (v2 < P.land_v2) & (r2 < P.land_r2) & att_ok & om_ok;
        t[4] = landing ? P.kappa : 0.0f;
        if (P.flags & RR_FLAG_REWARD_ANNEALING) return t[3] + t[4] - P.xi * (a[2] + 1.0f);
        return t[0] + t[1] + t[2] + t[3] + t[4] + (bounds_violation ? -50.0f : 0.0f);
    } else {
        bounds_violation = bounds_hit<3>(P, s);
        // _compute_vtarg (rocket_env.py:219-247)
        const bool above = s[1] > P.waypoint;
        const float rh0 = above ? s[0] : 0.0f;
        const float rh1 = above ? s[1] - P.waypoint : s[1];
        const float vh1 = s[4] + (above ? 2.0f : 1.0f);
        const float tau_inv = above ? 1.0f / 20.0f : 1.0f / 100.0f;
        float nrh = fsqrt(rh0 * rh0 + rh1 * rh1);
        float nvh = fsqrt(s[3] * s[3] + vh1 * vh1);
        float t_go = nrh * frcp(nvh);
        float f = (-v0 * frcp(fmaxf(1e-3f, nrh))) * one_minus_exp_neg(t_go * tau_inv);
        float e0 = s[3] - f * rh0, e1 = s[4] - f * rh1;
        t[0] = P.alfa * fsqrt(e0 * e0 + e1 * e1);
        t[1] = P.beta * ((a[1] + 1.0f) * P.half_thrust);
        t[2] = P.eta;
        float zeta = fabsf(s[2] - kHalfPi);
        t[3] = zeta > kTwoPi ? P.gamma : 0.0f;
        t[4] = P.delta * fmaxf(0.0f, zeta - kHalfPi);
        // _check_landing (rocket_env.py:449-476)
        float r2 = s[0] * s[0] + s[1] * s[1];
        float v2 = s[3] * s[3] + s[4] * s[4];
        const bool landing = (s[1] <= P.zero_h) & (v2 < P.land_v2) & (r2 < P.land_r2) & (zeta < 0.2f) &
                             (fabsf(s[5]) < P.omega_lt);
        t[5] = landing ? P.kappa : 0.0f;
        if (P.flags & RR_FLAG_REWARD_ANNEALING) return t[3] + t[5] - P.xi * (a[1] + 1.0f);
        return t[0] + t[1] + t[2] + t[3] + t[4] + t[5] + (bounds_violation ? -50.0f : 0.0f);
    }
}

// Write this wave's [64][NS] observation tile through LDS as 16-B coalesced stores.
template <int NS, int EPW>
__device__ __forceinline__ void store_obs_tile(float* lds, const float* o, rsrc_t obs_r, uint32_t wave_base,
                                               int lane, uint32_t nvalid, bool vec_ok)
{
    if (lane >= EPW) {
    } else if constexpr (NS % 2 == 0) {
        float2* l2 = reinterpret_cast<float2*>(lds + lane * NS);
#pragma unroll
        for (int j = 0; j < NS / 2; ++j) l2[j] = make_float2(o[2 * j], o[2 * j + 1]);
    } else {
#pragma unroll
        for (int j = 0; j < NS; ++j) lds[lane * NS + j] = o[j];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t sbase = wave_base * NS * 4u;  // byte offset of the tile (wave-uniform)
    if (vec_ok && nvalid == (uint32_t)EPW) {
        constexpr int NV = EPW * NS / 4;
        const u32x4* src4 = reinterpret_cast<const u32x4*>(lds);
#pragma unroll
        for (int q = 0; q < (NV + kWave - 1) / kWave; ++q) {
            const int k = lane + q * kWave;
            if (NV % kWave == 0 || k < NV)
                __builtin_amdgcn_raw_buffer_store_b128(src4[k], obs_r, (int)(k * 16u), (int)sbase, kOutAux);
        }
    } else {
        const int tot = (int)nvalid * NS;
        for (int k = lane; k < tot; k += kWave) bst_f<kOutAux>(obs_r, lds[k], k * 4u, sbase);
    }
}

// ---------------------------------------------------------------------------
// Step kernels. One launch = one env step of all N envs. Every HBM access goes through a
// buffer descriptor: the per-lane byte offset is one 32-bit VGPR (i*4), plane offsets are
// wave-uniform soffsets (NS*N*4 < 4 GiB, checked at rr_create). The leading four arguments
// are plain pointers / words so that the command processor preloads them into user SGPRs at
// wave launch (-mllvm -amdgpu-kernarg-preload-count, rl_rocket_amd/build.py): the first
// state loads then issue without waiting for scalar loads of the kernarg segment.
// `mode` = rr_params.flags | kModeCounter. ASOA: action layout [NA][N] (RR_FLAG_ACTION_SOA)
// as a template parameter (a runtime branch between the two layouts made the waitcnt pass
// stall the wave on the state loads before it issued the action load).
// ---------------------------------------------------------------------------

// the action row of env `vo / 4` ([N][NA] rows or [NA][N] planes)
template <int NA, bool ASOA>
__device__ __forceinline__ void load_action(rsrc_t act_r, uint32_t vo, uint32_t plane, float* a)
{
    if constexpr (ASOA) {
#pragma unroll
        for (int j = 0; j < NA; ++j) a[j] = bld_f(act_r, vo, j * plane);
    } else if constexpr (NA == 3) {
        const u32x3 v = __builtin_amdgcn_raw_buffer_load_b96(act_r, (int)((vo << 1) + vo), 0, kLdAux);  // 12 B rows
        a[0] = __uint_as_float(v.x);
        a[1] = __uint_as_float(v.y);
        a[2] = __uint_as_float(v.z);
    } else {
        const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(act_r, (int)(vo << 1), 0, kLdAux);  // 8 B rows
        a[0] = __uint_as_float(v.x);
        a[1] = __uint_as_float(v.y);
    }
}

// Simulator*.step (simulator.py:227-257 / :55-80): integrator, terminal ground event,
// quaternion renormalisation / theta wrap. Returns the event flag (solve_ivp status 1).
template <int MODEL, int INTEG>
__device__ __forceinline__ bool physics_step(const KParams& P, const float* a, const float* y0, float* y1)
{
    constexpr int NS = Dims<MODEL>::NS, EV = Dims<MODEL>::EV;
    float f0[NS];
    const Ctl c = make_ctl<MODEL>(P, a);
    integrate<MODEL, INTEG>(P, c, y0, P.h, y1, f0);
    const float g0 = y0[EV], g1 = y1[EV];
    const bool event = (g0 <= 0.0f && g1 >= 0.0f) || (g0 >= 0.0f && g1 <= 0.0f);
    if (event) event_step<MODEL, INTEG>(P, c, y0, f0, y1);
    post_integrate<MODEL>(y1);
    return event;
}

// The counter-word layout and the TimeLimit, read from the kernel arguments once at kernel
// start and pinned in SGPRs (pin_s): read where they are used, after the integration, they
// were scalar loads with a wait in the tail of a lone wave (+2 % per step at N = 65536).
struct CounterLayout {
    uint32_t el_mask, ep_shift;
    int32_t max_steps;
    __device__ __forceinline__ explicit CounterLayout(const KParams& P)
        : el_mask(P.el_mask), ep_shift(P.ep_shift), max_steps(P.max_steps)
    {
        pin_s(el_mask);
        pin_s(ep_shift);
        pin_s(max_steps);
    }
    // gym TimeLimit (main_6DOF.py:21): elapsed += 1; at the limit done = True and
    // info["TimeLimit.truncated"] = not done. Returns the new elapsed count, saturated at el_mask
    // (>= max_steps): an env stepped on past its TimeLimit without a reset keeps reporting
    // done / truncated instead of wrapping into the episode field.
    __device__ __forceinline__ int32_t time_limit(uint32_t cw, bool& done, bool& trunc) const
    {
        const int32_t el = min((int32_t)(cw & el_mask) + 1, (int32_t)el_mask);
        trunc = false;
        if (max_steps > 0 && el >= max_steps) {
            trunc = !done;
            done = true;
        }
        return el;
    }
    // the counter word of a reset env: episode + 1, elapsed 0
    __device__ __forceinline__ uint32_t next_episode(uint32_t cw) const { return ((cw >> ep_shift) + 1u) << ep_shift; }
    // the elapsed field set to `el`
    __device__ __forceinline__ uint32_t with_elapsed(uint32_t cw, int32_t el) const
    {
        return (cw & ~el_mask) | ((uint32_t)el & el_mask);
    }
};

// terminal obs / return / length of a done env (info["terminal_observation"], Monitor):
// row i of [N][NS] as 16-B stores (rows are 4-B aligned; gfx950 buffer stores need only
// dword alignment), NS = 14 -> 3 x 16 B + 8 B, NS = 7 -> 16 B + 12 B. AUX: cache policy
template <int NS, int AUX, bool SCALARS = true>
__device__ __forceinline__ void store_terminal(const Bufs& B, uint32_t i, uint32_t vo, uint32_t plane, const float* o,
                                               float ret, int32_t el)
{
    const rsrc_t tr = make_rsrc(B.term_obs, (uint64_t)NS * plane);
    const uint32_t ro = NS == 14 ? (i << 6) - (i << 3) : i * (NS * 4u);  // i * 56 without v_mul_lo_u32
    auto u4 = [&](int j) {
        return u32x4{__float_as_uint(o[j]), __float_as_uint(o[j + 1]), __float_as_uint(o[j + 2]),
                     __float_as_uint(o[j + 3])};
    };
#pragma unroll
    for (int j = 0; j + 4 <= NS; j += 4) __builtin_amdgcn_raw_buffer_store_b128(u4(j), tr, (int)(ro + j * 4), 0, AUX);
    if constexpr (NS % 4 == 2)
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{__float_as_uint(o[NS - 2]), __float_as_uint(o[NS - 1])}, tr,
                                              (int)(ro + (NS - 2) * 4), 0, AUX);
    else if constexpr (NS % 4 == 3)
        __builtin_amdgcn_raw_buffer_store_b96(
            u32x3{__float_as_uint(o[NS - 3]), __float_as_uint(o[NS - 2]), __float_as_uint(o[NS - 1])}, tr,
            (int)(ro + (NS - 3) * 4), 0, AUX);
    if constexpr (SCALARS) {
        bst_f<AUX>(make_rsrc(B.term_ret, plane), ret, vo, 0);
        bst_u<AUX>(make_rsrc(B.term_len, plane), (uint32_t)el, vo, 0);
    }
}

// per-env step outputs owned by the caller: reward, done (unless they travel in the obs row),
// truncated, optional terms
template <int NT, bool REWARD_DONE = true>
__device__ __forceinline__ void store_outputs(const StepIO& io, uint32_t i, uint32_t vo, uint32_t plane, uint32_t n,
                                              float r, bool done, bool trunc, const float* t, bool bv, float status)
{
    if constexpr (REWARD_DONE) {
        bst_f<kOutAux>(make_rsrc(io.reward, plane), r, vo, 0);
        bst_u8<kOutAux>(make_rsrc(io.done, n), (uint8_t)done, i);
    }
    if (io.truncated) bst_u8<kOutAux>(make_rsrc(io.truncated, n), (uint8_t)trunc, i);
    if (io.terms) {
        const rsrc_t tr = make_rsrc(io.terms, (uint64_t)(NT + 2) * plane);
#pragma unroll
        for (int j = 0; j < NT; ++j) bst_f(tr, t[j], vo, j * plane);
        bst_f(tr, bv ? 1.0f : 0.0f, vo, NT * plane);           // info["bounds_violation"]
        bst_f(tr, status, vo, (NT + 1) * plane);  // solve_ivp status: 1 ground event, -1 non-finite state, 0
    }
}

// The step kernel: one env per lane, 64 envs per wave.
// HELP (N <= kHelpMaxN, about one main wave per SIMD): the auto-reset candidates of main
// wave k are drawn by helper wave WPB + k of the same workgroup (on the same SIMD) into
// cand[k] (row per lane: NS values, v0), published by cflag[k]. A lone wave issues one VALU op
// per 4 cycles and its SIMD can take one per 2 (MI355X_MICROARCH.md, 'vector-instruction ISSUE
// cost'), so the helper's ~190 instructions run beside the main wave's instead of before them
// (they need the counter word, which arrives with the state planes). Without HELP the main
// wave draws the candidate itself right after its counter word lands. Measured and rejected
// (round 2): a helper that also computes reward, obs and every caller-owned output while the
// main wave resets and stores the state (bitwise equal, 4.69 vs 4.31 us per step at N = 65536).
// ROWS (rr_step_rows): obs, reward and done leave as ONE row of NS + 2 fp32 per env
// (obs[NS], reward, done as 0 / 1) through the same LDS tile, e.g. straight into the send
// buffer of the multi-GPU all-gather (rl_rocket_amd.dist.ShardGather).
// rocket_exact.hip compiles this file again for the exact-mode kernels only, rocket_collect.hip for
// the rollout collect kernels only
#if !defined(RR_TU_EXACT) && !defined(RR_TU_COLLECT)
template <int MODEL, int INTEG, bool ASOA, bool HELP, int WPB, bool ROWS>
// amdgpu_waves_per_eu(4): <= 128 VGPRs keeps 4 waves per SIMD at large N
__global__ __launch_bounds__(HELP ? 2 * WPB * kWave : WPB * kWave) __attribute__((amdgpu_waves_per_eu(4))) void step_kernel(
    float* __restrict__ state, const float* __restrict__ action, uint32_t n_envs, uint32_t mode, const KParams P,
    const Bufs B, const StepIO io)
{
    constexpr int NS = Dims<MODEL>::NS, NA = Dims<MODEL>::NA, NT = Dims<MODEL>::NT, EV = Dims<MODEL>::EV;
    constexpr int OW = ROWS ? NS + 2 : NS;  // floats per output row
    __shared__ __attribute__((aligned(16))) float lds[WPB][kWave * OW];
    constexpr int kCandRow = (NS + 1 + 3) / 4 * 4;
    __shared__ __attribute__((aligned(16))) float cand[HELP ? WPB : 1][HELP ? kWave * kCandRow : 1];
    __shared__ uint32_t cflag[WPB];
    const uint32_t lane = threadIdx.x & (kWave - 1);
    // wave index as an SGPR: derived from threadIdx it is a VGPR the compiler cannot prove
    // uniform, and every buffer store with a wave_base soffset became a waterfall loop
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const uint32_t n = n_envs;
    RR_STAMPS_BEGIN(4);  // diagnostic builds only (rocket_stamps.h)
    if constexpr (HELP) {
        if (wv < (uint32_t)WPB && lane == 0) cflag[wv] = 0u;
        __syncthreads();  // flags cleared before any helper can publish
        if (wv >= (uint32_t)WPB) {
            // the helper role reads its parameters through the device copy (B.kp): kernel-argument
            // values it used were loaded in the kernel's entry block and kept live into the main
            // role, where SGPRs are the scarce resource
            const KParams& P = *B.kp;
            const uint32_t k = wv - WPB;  // the main wave this helper serves
            const uint32_t base = (blockIdx.x * WPB + k) * kWave;
            const uint32_t ih = min(base + lane, n - 1);
            const uint32_t cwh = (base < n && (mode & kModeCounter)) ? at(B.counter, ih) : 0u;
            if ((mode & RR_FLAG_AUTO_RESET) && base < n) {
                float s_[NS], v_;
                ResetStream key = reset_stream(P.seed_w, P.id_off + base + lane, cwh);
                sample_ic<MODEL>(P, key, s_, v_);
                float* row = &cand[k][lane * kCandRow];
#pragma unroll
                for (int j = 0; j < NS; ++j) row[j] = s_[j];
                row[NS] = v_;
            }
            __hip_atomic_store(&cflag[k], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            return;
        }
    }
    const uint32_t wave_idx = blockIdx.x * WPB + wv;
    const uint32_t wave_base = wave_idx * kWave;
    if (wave_base >= n) return;  // wave-uniform
    RR_STAMP(0);
    const uint32_t i = wave_base + lane;
    const bool valid = i < n;
    const uint32_t ic = valid ? i : n - 1;
    const uint32_t vo = ic * 4u;           // per-lane byte offset in every fp32/u32 plane
    const uint32_t plane = n * 4u;         // bytes per plane
    const bool use_counter = mode & kModeCounter;
    // state planes, v0, counter and ep_ret are consecutive planes of ONE allocation
    // (rr_create), so a single descriptor (4 SGPRs) serves them all via soffset
    const rsrc_t st_r = make_rsrc(state, (uint64_t)(NS + 3) * plane);
    const uint32_t v0_off = NS * plane, cw_off = (NS + 1) * plane, ret_off = (NS + 2) * plane;
    constexpr int SA = HELP ? kStAuxHelp : kStAux;  // cache policy of the state-buffer stores

    // ---- all loads first (one memory round trip per wave); the counter word first, so the
    // reset candidate below is drawn while the state planes are still in flight ----
    uint32_t cw = use_counter ? bld_u(st_r, vo, cw_off) : 0u;
    float y0[NS], y1[NS], a[NA];
    load_action<NA, ASOA>(make_rsrc(action, (uint64_t)NA * plane), vo, plane, a);
#pragma unroll
    for (int j = 0; j < NS; ++j) y0[j] = bld_f(st_r, vo, j * plane);
    float v0 = bld_f(st_r, vo, v0_off);
    float ret = (mode & RR_FLAG_EPISODE_STATS) ? bld_f(st_r, vo, ret_off) : 0.0f;
    const HotParams H = load_hot<NS>(P);  // scalar loads overlap the HBM latency above
    const CounterLayout CL(P);
    // the kernel-argument lines holding the tail's pointers (outputs, terminal rows) are read
    // here, in the load shadow, so that the scalar reloads after the integration hit the
    // scalar cache instead of missing in the wave's critical tail (HELP kernels: without the
    // helpers' device parameter copy the SGPRs are short, 2-5 spills)
    if constexpr (HELP)
        asm volatile("" ::"s"(io.obs), "s"(io.reward), "s"(io.done), "s"(io.truncated), "s"(B.done_bits),
                     "s"(B.term_obs));
    // the SGPR -> VGPR copies of the pinned per-axis parameters issue here, in the shadow of
    // the state loads; left to the scheduler they landed after the load wait, inside the RK4
    __builtin_amdgcn_sched_barrier(0);
    // SB3 auto-reset candidate of this step, keyed on (gid, counter word): ~190 VALU right
    // after the counter word lands, instead of in the done branch of the waves that finish
    // last. Used by done lanes only. (HELP: drawn by the helper wave instead.)
    float ic_s[NS], ic_v0 = 0.0f;
    if (!HELP && (mode & RR_FLAG_AUTO_RESET)) {
        ResetStream key = reset_stream(B.kp->seed_w, P.id_off + i, cw);
        sample_ic<MODEL>(P, key, ic_s, ic_v0);
    }

    RR_STAMP_AFTER(1, y0, NS);  // the state landed
    const bool event = physics_step<MODEL, INTEG>(P, a, y0, y1);
    const bool nf = nonfinite<NS>(y1);
    bool bv;
    float t[NT];
    const float r = reward_terms<MODEL>(H, y1, a, v0, bv, t);
    bool done = event || bv || nf, trunc;
    int32_t el = CL.time_limit(cw, done, trunc);
    ret += r;
    float o[NS];
    normalize_obs<NS>(y1, H.inv_norm, o);
    RR_STAMP(2);

    // Done compaction: one ballot per wave; lane 0 stores the wave's 64-bit done mask
    // (every wave writes its word each step, so no clearing and no atomics; the host
    // side expands the masks into the sorted index list, rr_fetch_done).
    const bool dv = done && valid;
    const uint64_t m = __ballot(dv);
    if (lane == 0) B.done_bits[wave_idx] = m;
    if (m) {
        // plain kernels past the MALL: the 4-B terminal return / length and the reset v0 leave as
        // whole lines, from every lane of a wave with a done lane (the others' values are not
        // read: terminal rows count at done indices only; their v0 is unchanged)
        if (dv) store_terminal<NS, HELP ? 0 : kTermAuxLarge, HELP>(B, i, vo, plane, o, ret, el);
        if constexpr (!HELP) {
            if ((mode & kModeWholeLines) ? valid : dv) {
                bst_f<0>(make_rsrc(B.term_ret, plane), ret, vo, 0);
                bst_u<0>(make_rsrc(B.term_len, plane), (uint32_t)el, vo, 0);
            }
        }
        if ((mode & RR_FLAG_AUTO_RESET) && dv) {
            if constexpr (HELP) {
                while (__hip_atomic_load(&cflag[wv], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u)
                    __builtin_amdgcn_s_sleep(1);
                const float* row = &cand[wv][lane * kCandRow];
#pragma unroll
                for (int j = 0; j < NS; ++j) y1[j] = row[j];
                v0 = row[NS];
            } else {
#pragma unroll
                for (int j = 0; j < NS; ++j) y1[j] = ic_s[j];
                v0 = ic_v0;
            }
            if (HELP || !(mode & kModeWholeLines)) bst_f<SA>(st_r, v0, vo, v0_off);
            cw = CL.next_episode(cw);
            normalize_obs<NS>(y1, H.inv_norm, o);
            el = 0;
            ret = 0.0f;
        }
        if constexpr (!HELP) {
            if ((mode & kModeWholeLines) && (mode & RR_FLAG_AUTO_RESET) && valid) bst_f<SA>(st_r, v0, vo, v0_off);
        }
    }
    cw = CL.with_elapsed(cw, el);

    if (valid) {
#pragma unroll
        for (int j = 0; j < NS; ++j) bst_f<SA>(st_r, y1[j], vo, j * plane);
        if (use_counter) bst_u<SA>(st_r, cw, vo, (NS + 1) * plane);
        if (mode & RR_FLAG_EPISODE_STATS) bst_f<SA>(st_r, ret, vo, (NS + 2) * plane);
        store_outputs<NT, !ROWS>(io, i, vo, plane, n, r, done, trunc, t, bv, event ? 1.0f : (nf ? -1.0f : 0.0f));
    }
    const uint32_t nvalid = (n - wave_base) < (uint32_t)kWave ? (n - wave_base) : (uint32_t)kWave;
    if constexpr (ROWS) {
        float ow[OW];
#pragma unroll
        for (int j = 0; j < NS; ++j) ow[j] = o[j];
        ow[NS] = r;
        ow[NS + 1] = done ? 1.0f : 0.0f;
        store_obs_tile<OW, kWave>(lds[wv], ow, make_rsrc(io.obs, (uint64_t)OW * plane), wave_base, lane, nvalid,
                                  io.obs_vec_ok);
    } else {
        store_obs_tile<NS, kWave>(lds[wv], o, make_rsrc(io.obs, (uint64_t)NS * plane), wave_base, lane, nvalid,
                                  io.obs_vec_ok);
    }
    // lanes 0..2: barrier / loads / compute cycles; 3: the tail (outputs issued); 4, 5: the wave's
    // s_memrealtime start / end (100 MHz, low 32 bits, bit patterns in the float slots)
    RR_STAMP(3);
    RR_STAMPS_WRITE(io.reward, i, lane, valid, true);
}

template <int MODEL>
__global__ __launch_bounds__(kBlock) void reset_kernel(const KParams P, const Bufs B, const uint8_t* mask,
                                                      float* obs, double* state64)
{
    constexpr int NS = Dims<MODEL>::NS;
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= B.n) return;
    const int64_t n = B.n;
    float s[NS], v0;
    if (mask == nullptr || mask[i]) {
        const uint32_t ep = (B.counter[i] >> P.ep_shift) + 1u;
        ResetStream key = reset_stream(B.kp->seed_w, P.id_off + i, B.counter[i]);
        sample_ic<MODEL>(P, key, s, v0);
#pragma unroll
        for (int j = 0; j < NS; ++j) B.state[(int64_t)j * n + i] = s[j];
        if (state64) {  // RR_INT_DOPRI5
#pragma unroll
            for (int j = 0; j < NS; ++j) state64[(int64_t)j * n + i] = (double)s[j];
        }
        B.v0[i] = v0;
        B.counter[i] = ep << P.ep_shift;
        B.ep_ret[i] = 0.0f;
    } else {
#pragma unroll
        for (int j = 0; j < NS; ++j) s[j] = B.state[(int64_t)j * n + i];
    }
    if (obs) {
#pragma unroll
        for (int j = 0; j < NS; ++j) obs[i * NS + j] = s[j] * P.inv_norm[j];
    }
}

// counter words: clear the elapsed field, keep the episode field (rr_set_state without elapsed)
__global__ __launch_bounds__(kBlock) void clear_elapsed_kernel(uint32_t* counter, int64_t n, uint32_t el_mask)
{
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) counter[i] &= ~el_mask;
}

// Compact the terminal rows of the (sorted) done list for one host copy.
__global__ __launch_bounds__(kBlock) void gather_done_kernel(const int32_t* idx, int64_t count, int ns,
                                                             const float* term_obs, const float* term_ret,
                                                             const int32_t* term_len, const uint8_t* trunc,
                                                             float* g_obs, float* g_ret, int32_t* g_len,
                                                             uint8_t* g_trunc)
{
    const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= count) return;
    const int64_t i = idx[k];
    for (int j = 0; j < ns; ++j) g_obs[k * ns + j] = term_obs[i * ns + j];
    g_ret[k] = term_ret[i];
    g_len[k] = term_len[i];
    if (trunc) g_trunc[k] = trunc[i];
}

// rr_copy_terminal: the terminal rows of the envs done at the last step (done_bits) into
// caller buffers (any may be null); rows of other envs are left untouched
__global__ __launch_bounds__(kBlock) void copy_done_rows_kernel(const uint64_t* done_bits, int64_t n, int ns,
                                                                const float* term_obs, const float* term_ret,
                                                                const int32_t* term_len, float* d_obs, float* d_ret,
                                                                int32_t* d_len)
{
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n || !((done_bits[i / kWave] >> (i % kWave)) & 1ull)) return;
    if (d_obs)
        for (int j = 0; j < ns; ++j) d_obs[i * ns + j] = term_obs[i * ns + j];
    if (d_ret) d_ret[i] = term_ret[i];
    if (d_len) d_len[i] = term_len[i];
}

#endif  // !RR_TU_EXACT && !RR_TU_COLLECT

#ifndef RR_TU_EXACT
// On-device PPO rollout kernels (fused MlpPolicy forward on fp32 MFMA, bootstrap, GAE)
#include "rocket_policy.inc"
#include "rocket_rollout.inc"
// PPO learner (loss + backward of the MlpPolicy on fp32 MFMA, clip + Adam): its types in both
// translation units, its kernels launched from the collect TU (rrc_launch_learner)
#include "rocket_ppo.inc"
#endif  // RR_TU_EXACT

// Exact-integrator mode (RR_INT_DOPRI5): fp64 scipy RK45 restatement, compiled without
// FMA contraction so its roundings follow the reference's numpy arithmetic. Its kernels are
// compiled in the second translation unit (rocket_exact.hip); this one keeps XParams and the
// fp32 <-> fp64 plane conversions.
#pragma clang fp contract(off)
#include "rocket_dopri5.inc"
#pragma clang fp contract(fast)

#ifdef RR_TU_EXACT
}  // namespace

// the exact TU's only entry point (hidden: not part of the C-ABI). bufs / io / xp point to the
// Bufs / StepIO / XParams of the calling TU (same definitions, same layout).
extern "C" __attribute__((visibility("hidden"))) int rrx_launch_exact(int model, int variant, const void* xp,
                                                                        const void* bufs, const void* io,
                                                                        double* state64, unsigned grid, void* stream)
{
    Bufs b;
    StepIO o;
    std::memcpy(&b, bufs, sizeof(Bufs));
    std::memcpy(&o, io, sizeof(StepIO));
    const XParams* x = static_cast<const XParams*>(xp);
    hipStream_t s = (hipStream_t)stream;
    // variant bit 0 = lean (6DOF above one wave per SIMD, the caller's choice): 256 registers, two
    // waves per SIMD hide each other's fp64 latency (147.6 vs 176.6 us at N = 524 288); otherwise the
    // in-loop dense output (no event re-derivation, no spills: 28.9 vs 32.1 us at 65 536,
    // profiles/r04/ab_lean/). Bit 1 = [NA][N] action planes (RR_FLAG_ACTION_SOA).
    const bool lean = variant & 1, soa = variant & 2;
#define RR_LAUNCH_X(M, L, A) \
    hipLaunchKernelGGL((step_exact_kernel<M, L, A>), dim3(grid), dim3(kBlock), 0, s, x, b, o, state64)
    if (model == RR_MODEL_6DOF && lean) {
        if (soa) RR_LAUNCH_X(6, true, true);
        else RR_LAUNCH_X(6, true, false);
    } else if (model == RR_MODEL_6DOF) {
        if (soa) RR_LAUNCH_X(6, false, true);
        else RR_LAUNCH_X(6, false, false);
    } else {
        if (soa) RR_LAUNCH_X(3, false, true);
        else RR_LAUNCH_X(3, false, false);
    }
#undef RR_LAUNCH_X
    return (int)hipGetLastError();
}
#elif defined(RR_TU_COLLECT)
}  // namespace

// the collect TU's only entry point (hidden: not part of the C-ABI): one rr_rollout_collect launch,
// rollout_step_kernel<MODEL, INTEG, PREC, MULTI = true, 2>. kp / bufs / io point to the KParams /
// Bufs / RolloutIO of the calling TU (same definitions, same layout).
extern "C" __attribute__((visibility("hidden"))) int rrc_launch_collect(int model, int integ, int prec,
                                                                          unsigned grid, float* state, uint32_t n,
                                                                          uint32_t mode, const void* kp,
                                                                          const void* bufs, const void* io,
                                                                          void* stream)
{
    KParams p;
    Bufs b;
    RolloutIO o;
    std::memcpy(&p, kp, sizeof(KParams));
    std::memcpy(&b, bufs, sizeof(Bufs));
    std::memcpy(&o, io, sizeof(RolloutIO));
    hipStream_t s = (hipStream_t)stream;
#define RR_COLLECT(M, I, PR)                                                                                  \
    hipLaunchKernelGGL((rollout_step_kernel<M, I, PR, true, 2>), dim3(grid), dim3(rol::Shape<2>::kThreads), 0, \
                       s, state, n, mode, p, b, o)
#define RR_COLLECT_P(M, I)                      \
    do {                                        \
        if (prec == 1) RR_COLLECT(M, I, 1);     \
        else if (prec == 2) RR_COLLECT(M, I, 2); \
        else RR_COLLECT(M, I, 0);               \
    } while (0)
    const bool euler = integ == RR_INT_EULER;
    if (model == RR_MODEL_6DOF && !euler) RR_COLLECT_P(6, RR_INT_RK4);
    else if (model == RR_MODEL_6DOF) RR_COLLECT_P(6, RR_INT_EULER);
    else if (!euler) RR_COLLECT_P(3, RR_INT_RK4);
    else RR_COLLECT_P(3, RR_INT_EULER);
#undef RR_COLLECT_P
#undef RR_COLLECT
    return (int)hipGetLastError();
}

// the learner's launches (hidden: not part of the C-ABI), for rr_ppo_grad / rr_ppo_update /
// rr_clip_adam, which validated the arguments and carved the workspace into `launch` (a PpoLaunch of
// the calling TU). Compiled here with the MFMA accumulators in VGPRs: the gradient kernel's loop
// then moves ~740 fewer registers between AGPRs and VGPRs per launch, bitwise the same gradients
// (profiles/r06/ppo_vf/)
extern "C" __attribute__((visibility("hidden"))) int rrc_launch_learner(const void* launch, void* stream)
{
    PpoLaunch L;
    std::memcpy(&L, launch, sizeof(PpoLaunch));
    hipStream_t s = (hipStream_t)stream;
    if (L.op == 2) {
        const dim3 grid((unsigned)((L.a.start[L.a.n] + kAdamThreads - 1) / kAdamThreads));
        hipLaunchKernelGGL(adam_norm_kernel, grid, dim3(kAdamThreads), 0, s, L.a, L.work);
        hipLaunchKernelGGL(adam_step_kernel, grid, dim3(kAdamThreads), 0, s, L.a, L.work, L.max_norm, L.lr, L.beta1,
                           L.beta2, L.w1, L.w2, L.eps);
        return (int)hipGetLastError();
    }
    const bool update = L.op == 1;
    auto run = [&](auto obs_c, auto act_c) {
        constexpr int O = decltype(obs_c)::value, A = decltype(act_c)::value;
        using PT = ppo::Part<O, A>;
        using K = ppo::Pack<O, A>;
        constexpr int nfin = (PT::SIZE + kFinElems - 1) / kFinElems;
        if (!(update && (L.flags & RR_PPO_CHAINED)))
            hipLaunchKernelGGL((ppo_prep_kernel<O, A>), dim3(ppo::kAdvPart + (2 * K::SIZE + 255) / 256), dim3(256), 0, s,
                               L.advantages, L.idx, L.batch, L.adv_part, L.ps, L.pack);
        hipLaunchKernelGGL((ppo_grad_kernel<O, A>), dim3(L.nwg, 2), dim3(ppo::kThreads), 0, s, L.obs, L.actions,
                           L.old_log_prob, L.advantages, L.returns, L.idx, L.batch, L.clip, L.vf, L.adv_part, L.pack,
                           L.part);
        hipLaunchKernelGGL((ppo_finish_kernel<O, A>), dim3(nfin, 2), dim3(256), 0, s, L.part, L.nwg, L.batch, L.ent,
                           L.ps, L.pg, L.stats, update ? L.normw : nullptr,
                           update ? (const float*)L.a.step[0] : nullptr);
        if (update) {
            const AdvNext nx = {L.advantages, L.next_idx, L.next_idx ? L.next_batch : 0, L.adv_part};
            hipLaunchKernelGGL((adam_chain_kernel<O, A>), dim3(L.nbp + (L.next_idx ? ppo::kAdvPart / 4 : 0)),
                               dim3(kAdamThreads), 0, s, L.a, (const float*)L.normw, 2 * nfin, L.max_norm, L.lr,
                               L.beta1, L.beta2, L.w1, L.w2, L.eps, L.pack, nx, L.nbp);
        }
    };
    if (L.obs_dim == 14) run(std::integral_constant<int, 14>{}, std::integral_constant<int, 3>{});
    else run(std::integral_constant<int, 7>{}, std::integral_constant<int, 2>{});
    return (int)hipGetLastError();
}
#else  // the main translation unit: host side

// defined by the exact / collect translation units; these weak stand-ins (a library built from this
// file alone, e.g. a tools/ A/B variant) make RR_INT_DOPRI5 steps and rr_rollout_collect fail loudly
// instead of failing to load
extern "C" __attribute__((weak, visibility("hidden"))) int rrx_launch_exact(int, int, const void*, const void*,
                                                                          const void*, double*, unsigned, void*)
{
    return (int)hipErrorInvalidDeviceFunction;
}
extern "C" __attribute__((weak, visibility("hidden"))) int rrc_launch_collect(int, int, int, unsigned, float*,
                                                                            uint32_t, uint32_t, const void*,
                                                                            const void*, const void*, void*)
{
    return (int)hipErrorInvalidDeviceFunction;
}
extern "C" __attribute__((weak, visibility("hidden"))) int rrc_launch_learner(const void*, void*)
{
    return (int)hipErrorInvalidDeviceFunction;
}

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
thread_local std::string g_err;

int fail(int code, const std::string& msg)
{
    g_err = msg;
    return code;
}

int hip_fail(hipError_t e, const char* what)
{
    return fail(RR_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

float ceil_f(double d)   // smallest float >= d
{
    float f = (float)d;
    if ((double)f < d) f = std::nextafter(f, INFINITY);
    return f;
}
float floor_f(double d)  // largest float <= d
{
    float f = (float)d;
    if ((double)f > d) f = std::nextafter(f, -INFINITY);
    return f;
}

// 64-bit user seed -> the reset stream's four key words (splitmix64, host side)
void seed_words(uint64_t seed, uint32_t* w)
{
    auto sm = [](uint64_t x) {
        uint64_t z = x + 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    };
    const uint64_t a = sm(seed), b = sm(seed + 0x9E3779B97F4A7C15ull);
    w[0] = (uint32_t)a;
    w[1] = (uint32_t)(a >> 32);
    w[2] = (uint32_t)b;
    w[3] = (uint32_t)(b >> 32);
}

// bits of the elapsed field of the counter word: enough for max_episode_steps (TimeLimit
// 800 -> 10), 16 without a TimeLimit (elapsed then only counts Monitor's episode length)
int counter_bits(int32_t max_episode_steps)
{
    if (max_episode_steps <= 0) return 16;
    int b = 1;
    while (((int64_t)1 << b) <= (int64_t)max_episode_steps) ++b;
    return b;
}

KParams make_kparams(const rr_params& p)
{
    KParams k;
    std::memset(&k, 0, sizeof(k));
    const int ns = p.model == RR_MODEL_6DOF ? 14 : 7;
    k.max_steps = p.max_episode_steps;
    k.flags = p.flags;
    const int eb = counter_bits(p.max_episode_steps);
    k.el_mask = (1u << eb) - 1u;
    k.ep_shift = (uint32_t)eb;
    k.h = (float)p.dt;
    k.h2 = 0.5f * k.h;
    k.h6 = k.h / 6.0f;
    for (int j = 0; j < ns; ++j) {
        k.ic_low[j] = p.ic_low[j];
        k.ic_span[j] = p.ic_high[j] - p.ic_low[j];
        k.inv_norm[j] = (float)(1.0 / p.normalizer[j]);
    }
    // fp32 thresholds equivalent to the reference's float64 comparisons of float32 values
    for (int j = 0; j < 3; ++j) {
        if (p.model == RR_MODEL_6DOF) {  // inside <=> lo <= x <= hi
            k.blo[j] = ceil_f(p.bounds_low[j]);
            k.bhi[j] = floor_f(p.bounds_high[j]);
        } else {                         // out <=> x <= lo | x >= hi
            k.blo[j] = floor_f(p.bounds_low[j]);
            k.bhi[j] = ceil_f(p.bounds_high[j]);
        }
    }
    k.max_gimbal = (float)p.max_gimbal;
    k.half_thrust = (float)(0.5 * p.max_thrust);
    k.alfa = (float)p.alfa;
    k.beta = (float)p.beta;
    k.eta = (float)p.eta;
    k.gamma = (float)p.gamma;
    k.delta = (float)p.delta;
    k.kappa = (float)p.kappa;
    k.xi = (float)p.xi;
    k.waypoint = (float)p.waypoint;
    k.land_r2 = (float)((double)p.landing_radius * p.landing_radius);
    k.land_v2 = (float)((double)p.max_velocity * p.max_velocity);
    const double pi = 3.14159265358979323846;
    for (int ax = 0; ax < 3; ++ax) {
        const double L = p.att_limit[ax], M = p.land_att_limit[ax];
        // limits outside the angle's range make a test constant: |e| > L always holds for L < 0
        // (threshold 2 on axes 0 / 2: X < 2r for every r > 0, since |X| <= r; -1 on axis 1: |S| > -1;
        // the one exception, r == 0 exactly — the pitch singularity — reads false), and |e| < M
        // never holds for M <= 0 (X > 2r and |S| < -1 are never true)
        if (ax == 1) {  // b = asin(R02) in [-pi/2, pi/2]
            if (L >= pi / 2) k.att_never |= 1u << ax;
            else k.att_c[ax] = L < 0 ? -1.0f : (float)std::sin(L);
            if (M > pi / 2) k.land_always |= 1u << ax;
            else k.land_c[ax] = M <= 0 ? -1.0f : (float)std::sin(M);
        } else {        // a, c = atan2(.) in [-pi, pi]
            if (L >= pi) k.att_never |= 1u << ax;
            else k.att_c[ax] = L < 0 ? 2.0f : (float)std::cos(L);
            if (M > pi) k.land_always |= 1u << ax;
            else k.land_c[ax] = M <= 0 ? 2.0f : (float)std::cos(M);
        }
    }
    k.omega_lt = ceil_f(p.omega_lim[0]);
    k.zero_h = floor_f(1e-3);
    seed_words(42, k.seed_w);
    k.id_off = 0;
    return k;
}

XParams make_xparams(const rr_params& p)
{
    XParams x;
    std::memset(&x, 0, sizeof(x));
    x.dt = p.dt;
    const double ms = std::rint(p.dt * 1000.0);
    x.dt_milli = (ms > 0 && std::fabs(p.dt * 1000.0 - ms) < 1e-6) ? ms : 0.0;
    for (int j = 0; j < RR_MAX_STATE; ++j) x.norm[j] = p.normalizer[j];
    for (int j = 0; j < 3; ++j) {
        x.lo[j] = p.bounds_low[j];
        x.hi[j] = p.bounds_high[j];
        x.att_limit[j] = p.att_limit[j];
        x.land_att_limit[j] = p.land_att_limit[j];
        x.omega_lim[j] = p.omega_lim[j];
    }
    x.max_gimbal = p.max_gimbal;
    x.max_thrust = p.max_thrust;
    x.alfa = p.alfa;
    x.beta = p.beta;
    x.eta = p.eta;
    x.gamma = p.gamma;
    x.delta = p.delta;
    x.kappa = p.kappa;
    x.xi = p.xi;
    x.waypoint = p.waypoint;
    x.landing_radius = p.landing_radius;
    x.max_velocity = p.max_velocity;
    x.clamp_h0 = (p.flags & RR_FLAG_SCIPY_H0_CLAMP) ? 1 : 0;
    {
        const double pi = 3.14159265358979323846;
        for (int ax = 0; ax < 3; ++ax) {  // as make_kparams' float thresholds, in fp64
            const double L = p.att_limit[ax], M = p.land_att_limit[ax];
            // constant tests: |e| > L for L < 0 always, |e| < M for M <= 0 never (finish6)
            if (L < 0) x.att_always |= 1u << ax;
            if (M <= 0) x.land_never |= 1u << ax;
            if (ax == 1) {
                if (L >= pi / 2) x.att_never |= 1u << ax;
                else x.att_c[ax] = std::sin(L);
                if (M > pi / 2) x.land_always |= 1u << ax;
                else x.land_c[ax] = std::sin(M);
            } else {
                if (L >= pi) x.att_never |= 1u << ax;
                else x.att_c[ax] = std::cos(L);
                if (M > pi) x.land_always |= 1u << ax;
                else x.land_c[ax] = std::cos(M);
            }
        }
    }
    return x;
}

}  // namespace

struct rr_env {
    int device;
    rr_params p;
    KParams kp;
    XParams xp;
    int ns, na, nt;
    int64_t n, id_off;
    uint64_t steps;
    int64_t help_max_n;       // largest N stepped with helper waves (kHelpMaxN, RR_HELP_MAX_N env override)
    int64_t exact_lean_min_n; // 6DOF exact mode: lean kernel above this N (CUs x 256, RR_EXACT_LEAN_MIN_N)
    int64_t whole_line_min_n; // plain step kernels: whole-line done-path stores above this N (kWholeLineMinN,
                              // RR_WHOLE_LINE_MIN_N)
    float* state;
    float* v0;
    uint32_t* counter;
    float* ep_ret;
    uint64_t* done_bits;
    float* term_obs;
    float* term_ret;
    int32_t* term_len;
    double* state64;    // RR_INT_DOPRI5 only
    bool host_state;    // RR_FLAG_HOST_STATE: `state` (+ v0, counter, ep_ret planes) is pinned host memory
    KParams* d_kp;      // device copy of kp (Bufs.kp)
    XParams* d_xp;      // device copy of xp (RR_INT_DOPRI5: step_exact_kernel reads it where it uses it)
    int32_t* g_idx;     // rr_fetch_done scratch
    float* g_obs;
    float* g_ret;
    int32_t* g_len;
    uint8_t* g_trunc;   // rr_gather_rows scratch
    // the streams the handle's key-reading launches (step, reset, rollout kernels) were queued on,
    // most recent last (stored handles, compared only): rr_seed makes its key copy wait for the work
    // queued on each of them (seed_ev), and for the whole device past kSeedStreams distinct streams
    static constexpr int kSeedStreams = 8;
    void* streams[kSeedStreams];
    int n_streams;
    bool streams_overflow;
    hipEvent_t seed_ev;
};

namespace {

// note that a launch reading the reset-stream key went to `stream` (rr_seed orders its key copy after
// the work queued on every stream noted): a pointer compare per launch, no HIP call
inline void note_stream(rr_env* e, void* stream)
{
    if (e->n_streams > 0 && e->streams[e->n_streams - 1] == stream) return;
    for (int k = 0; k < e->n_streams; ++k)
        if (e->streams[k] == stream) {
            for (int j = k; j + 1 < e->n_streams; ++j) e->streams[j] = e->streams[j + 1];
            e->streams[e->n_streams - 1] = stream;
            return;
        }
    if (e->n_streams < rr_env::kSeedStreams) e->streams[e->n_streams++] = stream;
    else e->streams_overflow = true;
}

Bufs bufs_of(const rr_env* e)
{
    Bufs b;
    b.state = e->state;
    b.v0 = e->v0;
    b.counter = e->counter;
    b.ep_ret = e->ep_ret;
    b.done_bits = e->done_bits;
    b.term_obs = e->term_obs;
    b.term_ret = e->term_ret;
    b.term_len = e->term_len;
    b.n = e->n;
    b.kp = e->d_kp;
    return b;
}

unsigned grid_of(int64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }
int64_t n_words(int64_t n) { return (n + kWave - 1) / kWave; }

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard()
    {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

}  // namespace

extern "C" {

int rr_abi_version(void) { return RR_ABI_VERSION; }

const char* rr_last_error(void) { return g_err.c_str(); }

int rr_create(rr_env** out, const rr_params* p, int64_t n, int64_t env_id_offset, int device)
{
    if (!out || !p) return fail(RR_EINVAL, "rr_create: null argument");
    *out = nullptr;
    if (p->model != RR_MODEL_6DOF && p->model != RR_MODEL_3DOF)
        return fail(RR_EINVAL, "rr_create: model must be 3 or 6");
    if (p->integrator != RR_INT_RK4 && p->integrator != RR_INT_EULER && p->integrator != RR_INT_DOPRI5)
        return fail(RR_EINVAL, "rr_create: unknown integrator");
    const int64_t ns_ = p->model == RR_MODEL_6DOF ? 14 : 7;
    if (n <= 0 || n * (ns_ + 3) * 4 > (int64_t)0xFFFFFFFF)
        return fail(RR_EINVAL, "rr_create: n must be >= 1 and n*state_dim*4 must fit 32-bit buffer offsets");
    if (p->max_episode_steps < 0 || p->max_episode_steps > kMaxEpisodeSteps)
        return fail(RR_EINVAL, "rr_create: max_episode_steps must be in [0, 65535]");
    if (!(p->dt > 0.0)) return fail(RR_EINVAL, "rr_create: dt must be > 0");
    constexpr uint32_t kKnownFlags = RR_FLAG_AUTO_RESET | RR_FLAG_EPISODE_STATS | RR_FLAG_REWARD_ANNEALING |
                                     RR_FLAG_ACTION_SOA | RR_FLAG_SCIPY_H0_CLAMP | RR_FLAG_HOST_STATE;
    if (p->flags & ~kKnownFlags)  // the high bits carry the kernels' internal mode (kModeCounter, ...)
        return fail(RR_EINVAL, "rr_create: unknown flag bits");
    rr_env* e = new (std::nothrow) rr_env();
    if (!e) return fail(RR_ENOMEM, "rr_create: host allocation failed");
    e->device = device;
    e->p = *p;
    e->kp = make_kparams(*p);
    e->xp = make_xparams(*p);
    e->ns = p->model == RR_MODEL_6DOF ? 14 : 7;
    e->na = p->model == RR_MODEL_6DOF ? 3 : 2;
    e->nt = p->model == RR_MODEL_6DOF ? 5 : 6;
    e->n = n;
    e->id_off = env_id_offset;
    DeviceGuard g(device);
    {
        // test / A-B override of the helper-wave threshold: RR_HELP_MAX_N=<n> in the environment
        const char* hv = std::getenv("RR_HELP_MAX_N");
        e->help_max_n = hv ? std::strtoll(hv, nullptr, 10) : kHelpMaxN;
        // the exact mode's lean-kernel threshold: one env per lane of one wave per SIMD of THIS
        // device (a partitioned or smaller part has fewer CUs); RR_EXACT_LEAN_MIN_N overrides it
        // (tests run the lean kernel at small N)
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0)
            cus = (int)kExactLeanCUs;
        const char* lv = std::getenv("RR_EXACT_LEAN_MIN_N");
        e->exact_lean_min_n = lv ? std::strtoll(lv, nullptr, 10) : (int64_t)cus * 4 * kWave;
        // the plain kernels' whole-line done path (tests run it at small N with RR_WHOLE_LINE_MIN_N=0)
        const char* wv = std::getenv("RR_WHOLE_LINE_MIN_N");
        e->whole_line_min_n = wv ? std::strtoll(wv, nullptr, 10) : kWholeLineMinN;
    }
    struct A {
        void** ptr;
        size_t bytes;
    } allocs[] = {
        {(void**)&e->state, sizeof(float) * (e->ns + 3) * n},  // + v0, counter, ep_ret planes
        {(void**)&e->done_bits, sizeof(uint64_t) * n_words(n)},
        {(void**)&e->term_obs, sizeof(float) * e->ns * n},
        {(void**)&e->term_ret, sizeof(float) * n},        {(void**)&e->term_len, sizeof(int32_t) * n},
        {(void**)&e->g_idx, sizeof(int32_t) * n},         {(void**)&e->g_obs, sizeof(float) * e->ns * n},
        {(void**)&e->g_ret, sizeof(float) * n},           {(void**)&e->g_len, sizeof(int32_t) * n},
        {(void**)&e->g_trunc, sizeof(uint8_t) * n},
    };
    const bool exact = p->integrator == RR_INT_DOPRI5;
    e->host_state = (p->flags & RR_FLAG_HOST_STATE) != 0;
    for (auto& a : allocs) {
        if (e->host_state && a.ptr == (void**)&e->state) {
            // fine-grained (coherent) pinned host memory: the kernels' loads and stores go straight
            // to host memory, and the host reads the planes after a stream synchronise
            hipError_t err = hipHostMalloc(a.ptr, a.bytes, hipHostMallocCoherent | hipHostMallocMapped);
            if (err != hipSuccess) {
                *a.ptr = nullptr;
                rr_destroy(e);
                return hip_fail(err, "rr_create: hipHostMalloc (host state)");
            }
            std::memset(*a.ptr, 0, a.bytes);
            continue;
        }
        hipError_t err = hipMalloc(a.ptr, a.bytes);
        if (err != hipSuccess) {
            rr_destroy(e);
            return hip_fail(err, "rr_create: hipMalloc");
        }
        err = hipMemset(*a.ptr, 0, a.bytes);
        if (err != hipSuccess) {
            rr_destroy(e);
            return hip_fail(err, "rr_create: hipMemset");
        }
    }
    if (exact) {
        const size_t bytes = sizeof(double) * e->ns * n;
        hipError_t err = hipMalloc((void**)&e->state64, bytes);
        if (err == hipSuccess) err = hipMemset(e->state64, 0, bytes);
        if (err != hipSuccess) {
            rr_destroy(e);
            return hip_fail(err, "rr_create: hipMalloc (fp64 state)");
        }
    }
    e->v0 = e->state + (size_t)e->ns * n;
    e->counter = reinterpret_cast<uint32_t*>(e->state + (size_t)(e->ns + 1) * n);
    e->ep_ret = e->state + (size_t)(e->ns + 2) * n;
    e->kp.id_off = env_id_offset;
    {
        hipError_t err = hipMalloc((void**)&e->d_kp, sizeof(KParams));
        if (err == hipSuccess) err = hipEventCreateWithFlags(&e->seed_ev, hipEventDisableTiming);
        if (err == hipSuccess) err = hipMalloc((void**)&e->d_xp, sizeof(XParams));
        if (err == hipSuccess) err = hipMemcpy(e->d_xp, &e->xp, sizeof(XParams), hipMemcpyHostToDevice);
        if (err != hipSuccess) {
            rr_destroy(e);
            return hip_fail(err, "rr_create: hipMalloc (params)");
        }
    }
    int rc = rr_seed(e, 42, nullptr);
    if (rc == RR_OK) {
        hipError_t err = hipDeviceSynchronize();
        if (err != hipSuccess) rc = hip_fail(err, "rr_create: sync");
    }
    if (rc != RR_OK) {
        rr_destroy(e);
        return rc;
    }
    *out = e;
    return RR_OK;
}

int rr_destroy(rr_env* e)
{
    if (!e) return RR_OK;
    DeviceGuard g(e->device);
    if (e->host_state && e->state) {
        (void)hipHostFree(e->state);
        e->state = nullptr;
    }
    if (e->seed_ev) (void)hipEventDestroy(e->seed_ev);
    void* ptrs[] = {e->state, e->state64, e->d_kp, e->d_xp, e->done_bits,
                    e->term_obs, e->term_ret, e->term_len, e->g_idx, e->g_obs,  e->g_ret, e->g_len,
                    e->g_trunc};
    for (void* q : ptrs)
        if (q) (void)hipFree(q);
    delete e;
    return RR_OK;
}

int64_t rr_num_envs(const rr_env* e) { return e ? e->n : -1; }
int rr_state_dim(const rr_env* e) { return e ? e->ns : -1; }
int rr_action_dim(const rr_env* e) { return e ? e->na : -1; }

int rr_seed(rr_env* e, uint64_t seed, void* stream)
{
    // The reset stream is counter-based and every kernel reads its key from the device copy of
    // the parameters (Bufs.kp), so the new key applies to every launch that runs after this call
    // — graph replays of launches captured before it included — whatever the batch size. The
    // copy is written in the order of `stream` (the handle's stream: every launch queued on it
    // before this call reads the old key) and the call returns once it has landed. Refused
    // while `stream` is being captured: the key is not a graph node (replays read the key
    // current when they run).
    if (!e) return fail(RR_EINVAL, "rr_seed: null handle");
    DeviceGuard g(e->device);
    hipStream_t s = (hipStream_t)stream;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    hipError_t err = hipStreamIsCapturing(s, &cs);
    if (err != hipSuccess) return hip_fail(err, "rr_seed: hipStreamIsCapturing");
    if (cs != hipStreamCaptureStatusNone)
        return fail(RR_EINVAL, "rr_seed: the stream is being captured into a graph (seed before capturing: "
                               "replays read the key current when they run)");
    // launches of this handle queued on OTHER streams may still read the key: the new key must not
    // land under them. The copy waits, on the device, for the work queued so far on
    // every stream the handle launched on (the per-handle event recorded there now); the usual
    // single-stream caller keeps the plain stream-ordered write. Past kSeedStreams distinct streams
    // the device is synchronised. A stream being captured has run nothing of the capture yet.
    // Graph replays are not launches of the handle: the caller orders them (header).
    // A noted stream the runtime no longer knows (destroyed since: its queued work still runs) is
    // covered by the same device synchronise.
    bool sync_device = e->streams_overflow;
    for (int k = 0; k < e->n_streams && !sync_device; ++k) {
        hipStream_t o = (hipStream_t)e->streams[k];
        if (o == s) continue;
        hipStreamCaptureStatus ocs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(o, &ocs) != hipSuccess) {
            (void)hipGetLastError();
            sync_device = true;
            break;
        }
        if (ocs != hipStreamCaptureStatusNone) continue;
        err = hipEventRecord(e->seed_ev, o);
        if (err == hipSuccess) err = hipStreamWaitEvent(s, e->seed_ev, 0);
        if (err != hipSuccess) return hip_fail(err, "rr_seed: order the key after the handle's other streams");
    }
    if (sync_device) {
        err = hipDeviceSynchronize();
        if (err != hipSuccess) return hip_fail(err, "rr_seed: synchronise the device");
    }
    e->n_streams = 0;  // everything queued so far is ordered before the key copy
    e->streams_overflow = false;
    seed_words(seed, e->kp.seed_w);
    err = hipMemcpyAsync(e->d_kp, &e->kp, sizeof(KParams), hipMemcpyHostToDevice, s);
    if (err == hipSuccess) err = hipStreamSynchronize(s);  // e->kp is pageable host memory: wait until it is read
    return err == hipSuccess ? RR_OK : hip_fail(err, "rr_seed: params upload");
}

int rr_reset(rr_env* e, const uint8_t* mask, float* obs, void* stream)
{
    if (!e) return fail(RR_EINVAL, "rr_reset: null handle");
    const Bufs b = bufs_of(e);
    if (e->p.model == RR_MODEL_6DOF)
        hipLaunchKernelGGL(reset_kernel<6>, dim3(grid_of(e->n)), dim3(kBlock), 0, (hipStream_t)stream, e->kp, b,
                           mask, obs, e->state64);
    else
        hipLaunchKernelGGL(reset_kernel<3>, dim3(grid_of(e->n)), dim3(kBlock), 0, (hipStream_t)stream, e->kp, b,
                           mask, obs, e->state64);
    hipError_t err = hipGetLastError();
    note_stream(e, stream);
    return err == hipSuccess ? RR_OK : hip_fail(err, "rr_reset: launch");
}

}  // extern "C"

namespace {
// one step launch (rr_step / rr_step_repeat; arguments checked by the caller)
template <bool ROWS>
int launch_step(rr_env* e, const float* action, float* obs, float* reward, uint8_t* done, uint8_t* truncated,
                float* terms, void* stream)
{
    StepIO io;
    io.action = action;
    io.obs = obs;
    io.reward = reward;
    io.done = done;
    io.truncated = truncated;
    io.terms = terms;
    io.obs_vec_ok = ((uintptr_t)obs & 15u) == 0;
    const Bufs b = bufs_of(e);
    hipStream_t s = (hipStream_t)stream;
    const bool m6 = e->p.model == RR_MODEL_6DOF;
    const bool euler = e->p.integrator == RR_INT_EULER;
    const dim3 grid(grid_of(e->n)), block(kBlock);
    if (e->p.integrator == RR_INT_DOPRI5) {
        // the exact kernels live in the second translation unit (rocket_exact.hip: compiled with a
        // register-pressure-first scheduler, no scratch spills)
        const int variant = (m6 && e->n > e->exact_lean_min_n ? 1 : 0) | ((e->p.flags & RR_FLAG_ACTION_SOA) ? 2 : 0);
        const hipError_t xe = (hipError_t)rrx_launch_exact(m6 ? RR_MODEL_6DOF : RR_MODEL_3DOF, variant, e->d_xp, &b,
                                                           &io, e->state64, grid.x, s);
        if (xe != hipSuccess) return hip_fail(xe, "rr_step: exact launch");
    } else {
        const uint32_t nn = (uint32_t)e->n;
        const bool counter = e->p.max_episode_steps > 0 || (e->p.flags & (RR_FLAG_EPISODE_STATS | RR_FLAG_AUTO_RESET));
        const uint32_t mode =
            e->p.flags | (counter ? kModeCounter : 0u) | (e->n > e->whole_line_min_n ? kModeWholeLines : 0u);
        const bool soa = e->p.flags & RR_FLAG_ACTION_SOA;
        // small N (at most ~2 main waves per SIMD): helper waves draw the reset candidates
        const bool help = (mode & RR_FLAG_AUTO_RESET) && e->n <= e->help_max_n;
        // up to 16 384 envs one main wave per workgroup (64 + 64 threads): the few workgroups
        // spread over 4x as many CUs (A/B at N = 4 096: -5 % 6DOF); above, 4 main waves
        const bool narrow = e->n <= kNarrowMaxN;
#define RR_LAUNCH(M, I, A)                                                                                          \
    do {                                                                                                             \
        if (help && narrow)                                                                                          \
            hipLaunchKernelGGL((step_kernel<M, I, A, true, 1, ROWS>), dim3((unsigned)((e->n + kWave - 1) / kWave)), \
                               dim3(2 * kWave), 0, s, e->state, action, nn, mode, e->kp, b, io);                     \
        else if (help)                                                                                               \
            hipLaunchKernelGGL((step_kernel<M, I, A, true, kWavesPerBlock, ROWS>), grid, dim3(2 * kBlock), 0, s,     \
                               e->state, action, nn, mode, e->kp, b, io);                                            \
        else                                                                                                         \
            hipLaunchKernelGGL((step_kernel<M, I, A, false, kWavesPerBlock, ROWS>), grid, block, 0, s, e->state,     \
                               action, nn, mode, e->kp, b, io);                                                      \
    } while (0)
        if constexpr (ROWS) {  // row-major actions only (the multi-GPU gather path)
            if (m6 && !euler) RR_LAUNCH(6, RR_INT_RK4, false);
            else if (m6) RR_LAUNCH(6, RR_INT_EULER, false);
            else if (!euler) RR_LAUNCH(3, RR_INT_RK4, false);
            else RR_LAUNCH(3, RR_INT_EULER, false);
        } else if (m6 && !euler) {
            if (soa) RR_LAUNCH(6, RR_INT_RK4, true);
            else RR_LAUNCH(6, RR_INT_RK4, false);
        } else if (m6) {
            if (soa) RR_LAUNCH(6, RR_INT_EULER, true);
            else RR_LAUNCH(6, RR_INT_EULER, false);
        } else if (!euler) {
            if (soa) RR_LAUNCH(3, RR_INT_RK4, true);
            else RR_LAUNCH(3, RR_INT_RK4, false);
        } else {
            if (soa) RR_LAUNCH(3, RR_INT_EULER, true);
            else RR_LAUNCH(3, RR_INT_EULER, false);
        }
#undef RR_LAUNCH
    }
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) return hip_fail(err, "rr_step: launch");
    e->steps++;
    note_stream(e, stream);
    return RR_OK;
}
}  // namespace

extern "C" {

int rr_step(rr_env* e, const float* action, float* obs, float* reward, uint8_t* done, uint8_t* truncated,
            float* terms, void* stream)
{
    if (!e) return fail(RR_EINVAL, "rr_step: null handle");
    if (!action || !obs || !reward || !done) return fail(RR_EINVAL, "rr_step: action/obs/reward/done required");
    return launch_step<false>(e, action, obs, reward, done, truncated, terms, stream);
}

int rr_step_rows(rr_env* e, const float* action, float* rows, uint8_t* truncated, float* terms, void* stream)
{
    if (!e) return fail(RR_EINVAL, "rr_step_rows: null handle");
    if (!action || !rows) return fail(RR_EINVAL, "rr_step_rows: action/rows required");
    if (e->p.integrator == RR_INT_DOPRI5 || (e->p.flags & RR_FLAG_ACTION_SOA))
        return fail(RR_EINVAL, "rr_step_rows: RK4 / Euler envs with [N][action_dim] actions only");
    return launch_step<true>(e, action, rows, nullptr, nullptr, truncated, terms, stream);
}

int rr_step_repeat(rr_env* e, const float* actions, int64_t n_batches, int64_t n_steps, float* obs, float* reward,
                   uint8_t* done, uint8_t* truncated, float* terms, void* stream)
{
    if (!e) return fail(RR_EINVAL, "rr_step_repeat: null handle");
    if (!actions || !obs || !reward || !done) return fail(RR_EINVAL, "rr_step_repeat: actions/obs/reward/done required");
    if (n_batches <= 0 || n_steps < 0) return fail(RR_EINVAL, "rr_step_repeat: n_batches must be >= 1, n_steps >= 0");
    const int64_t batch = e->n * e->na;
    int rc = RR_OK;
    for (int64_t t = 0; t < n_steps && rc == RR_OK; ++t)
        rc = launch_step<false>(e, actions + (t % n_batches) * batch, obs, reward, done, truncated, terms, stream);
    return rc;
}

namespace {

// v0 / counter / episode-return part shared by the fp32 and fp64 setters
hipError_t set_aux(rr_env* e, const float* v0, const int32_t* elapsed, hipStream_t s)
{
    hipError_t err = hipSuccess;
    if (v0) err = hipMemcpyAsync(e->v0, v0, sizeof(float) * e->n, hipMemcpyDefault, s);
    if (err == hipSuccess) {
        if (elapsed) {
            err = hipMemcpyAsync(e->counter, elapsed, sizeof(int32_t) * e->n, hipMemcpyDefault, s);
        } else {  // elapsed steps -> 0, the episode field (reset-stream key) is kept
            hipLaunchKernelGGL(clear_elapsed_kernel, dim3(grid_of(e->n)), dim3(kBlock), 0, s, e->counter, e->n,
                               e->kp.el_mask);
            err = hipGetLastError();
        }
    }
    if (err == hipSuccess) err = hipMemsetAsync(e->ep_ret, 0, sizeof(float) * e->n, s);
    return err;
}

hipError_t get_aux(rr_env* e, float* v0, int32_t* elapsed, hipStream_t s)
{
    hipError_t err = hipSuccess;
    if (v0) err = hipMemcpyAsync(v0, e->v0, sizeof(float) * e->n, hipMemcpyDefault, s);
    if (err == hipSuccess && elapsed)
        err = hipMemcpyAsync(elapsed, e->counter, sizeof(int32_t) * e->n, hipMemcpyDefault, s);
    return err;
}

hipError_t widen_async(const float* src, double* dst, int64_t count, hipStream_t s)
{
    hipLaunchKernelGGL(widen_kernel, dim3(grid_of(count)), dim3(kBlock), 0, s, src, dst, count);
    return hipGetLastError();
}

hipError_t narrow_async(const double* src, float* dst, int64_t count, hipStream_t s)
{
    hipLaunchKernelGGL(narrow_kernel, dim3(grid_of(count)), dim3(kBlock), 0, s, src, dst, count);
    return hipGetLastError();
}

}  // namespace

int rr_set_state(rr_env* e, const float* state_soa, const float* v0, const int32_t* elapsed, void* stream)
{
    if (!e || !state_soa) return fail(RR_EINVAL, "rr_set_state: null argument");
    hipStream_t s = (hipStream_t)stream;
    const int64_t cnt = (int64_t)e->ns * e->n;
    hipError_t err = hipMemcpyAsync(e->state, state_soa, sizeof(float) * cnt, hipMemcpyDefault, s);
    if (err == hipSuccess && e->state64) err = widen_async(e->state, e->state64, cnt, s);
    if (err == hipSuccess) err = set_aux(e, v0, elapsed, s);
    return err == hipSuccess ? RR_OK : hip_fail(err, "rr_set_state");
}

int rr_get_state(rr_env* e, float* state_soa, float* v0, int32_t* elapsed, void* stream)
{
    if (!e) return fail(RR_EINVAL, "rr_get_state: null handle");
    hipStream_t s = (hipStream_t)stream;
    hipError_t err = hipSuccess;
    if (state_soa)
        err = hipMemcpyAsync(state_soa, e->state, sizeof(float) * e->ns * e->n, hipMemcpyDefault, s);
    if (err == hipSuccess) err = get_aux(e, v0, elapsed, s);
    return err == hipSuccess ? RR_OK : hip_fail(err, "rr_get_state");
}

int rr_set_state64(rr_env* e, const double* state_soa, const float* v0, const int32_t* elapsed, void* stream)
{
    if (!e || !state_soa) return fail(RR_EINVAL, "rr_set_state64: null argument");
    hipStream_t s = (hipStream_t)stream;
    const int64_t cnt = (int64_t)e->ns * e->n;
    hipError_t err = hipSuccess;
    if (e->state64) {
        err = hipMemcpyAsync(e->state64, state_soa, sizeof(double) * cnt, hipMemcpyDefault, s);
        if (err == hipSuccess) err = narrow_async(e->state64, e->state, cnt, s);
    } else {
        err = narrow_async(state_soa, e->state, cnt, s);
    }
    if (err == hipSuccess) err = set_aux(e, v0, elapsed, s);
    return err == hipSuccess ? RR_OK : hip_fail(err, "rr_set_state64");
}

int rr_get_state64(rr_env* e, double* state_soa, float* v0, int32_t* elapsed, void* stream)
{
    if (!e) return fail(RR_EINVAL, "rr_get_state64: null handle");
    hipStream_t s = (hipStream_t)stream;
    const int64_t cnt = (int64_t)e->ns * e->n;
    hipError_t err = hipSuccess;
    if (state_soa) {
        if (e->state64)
            err = hipMemcpyAsync(state_soa, e->state64, sizeof(double) * cnt, hipMemcpyDefault, s);
        else
            err = widen_async(e->state, state_soa, cnt, s);
    }
    if (err == hipSuccess) err = get_aux(e, v0, elapsed, s);
    return err == hipSuccess ? RR_OK : hip_fail(err, "rr_get_state64");
}

int rr_counter_bits(const rr_env* e) { return e ? (int)e->kp.ep_shift : RR_EINVAL; }

int rr_get_aux(rr_env* e, uint32_t* counter, float* ep_return, void* stream)
{
    if (!e) return fail(RR_EINVAL, "rr_get_aux: null handle");
    hipStream_t s = (hipStream_t)stream;
    hipError_t err = hipSuccess;
    if (counter) err = hipMemcpyAsync(counter, e->counter, sizeof(uint32_t) * e->n, hipMemcpyDefault, s);
    if (err == hipSuccess && ep_return)
        err = hipMemcpyAsync(ep_return, e->ep_ret, sizeof(float) * e->n, hipMemcpyDefault, s);
    return err == hipSuccess ? RR_OK : hip_fail(err, "rr_get_aux");
}

int rr_set_aux(rr_env* e, const uint32_t* counter, const float* ep_return, void* stream)
{
    if (!e) return fail(RR_EINVAL, "rr_set_aux: null handle");
    hipStream_t s = (hipStream_t)stream;
    hipError_t err = hipSuccess;
    if (counter) err = hipMemcpyAsync(e->counter, counter, sizeof(uint32_t) * e->n, hipMemcpyDefault, s);
    if (err == hipSuccess && ep_return)
        err = hipMemcpyAsync(e->ep_ret, ep_return, sizeof(float) * e->n, hipMemcpyDefault, s);
    return err == hipSuccess ? RR_OK : hip_fail(err, "rr_set_aux");
}

int rr_get_buffers(rr_env* e, rr_buffers* out)
{
    if (!e || !out) return fail(RR_EINVAL, "rr_get_buffers: null argument");
    out->state = e->state;
    out->v0 = e->v0;
    out->elapsed = (int32_t*)e->counter;
    out->ep_return = e->ep_ret;
    out->done_bits = e->done_bits;
    out->terminal_obs = e->term_obs;
    out->terminal_return = e->term_ret;
    out->terminal_len = e->term_len;
    return RR_OK;
}

int rr_host_alloc(void** out, int64_t bytes)
{
    if (!out || bytes <= 0) return fail(RR_EINVAL, "rr_host_alloc: null pointer or bytes <= 0");
    *out = nullptr;
    const hipError_t err = hipHostMalloc(out, (size_t)bytes, hipHostMallocCoherent | hipHostMallocMapped);
    if (err != hipSuccess) {
        *out = nullptr;
        return hip_fail(err, "rr_host_alloc");
    }
    std::memset(*out, 0, (size_t)bytes);
    return RR_OK;
}

int rr_host_free(void* p)
{
    if (!p) return RR_OK;
    const hipError_t err = hipHostFree(p);
    return err == hipSuccess ? RR_OK : hip_fail(err, "rr_host_free");
}

}  // extern "C"

namespace {
// The rows of the env indices `hidx` (ascending) from the given [N][ns] / [N] sources into the
// caller's host arrays (at most `capacity` rows): one index upload, one gather kernel into the
// env's scratch, the copies, one synchronise. Returns the number of indices or an RR_E* code.
int64_t fetch_rows(rr_env* e, const std::vector<int32_t>& hidx, int64_t capacity, const float* src_obs,
                   const float* src_ret, const int32_t* src_len, const uint8_t* src_trunc, int32_t* idx,
                   float* term_obs, float* term_return, int32_t* term_len, uint8_t* trunc_out, hipStream_t s,
                   const char* what)
{
    const int64_t count = (int64_t)hidx.size();
    const int64_t m = std::min<int64_t>(count, capacity);
    if (m == 0) return count;
    if (idx) std::memcpy(idx, hidx.data(), sizeof(int32_t) * m);
    if (term_obs || term_return || term_len || trunc_out) {
        hipError_t err = hipMemcpyAsync(e->g_idx, hidx.data(), sizeof(int32_t) * m, hipMemcpyHostToDevice, s);
        if (err != hipSuccess) return hip_fail(err, what);
        hipLaunchKernelGGL(gather_done_kernel, dim3(grid_of(m)), dim3(kBlock), 0, s, e->g_idx, m, e->ns, src_obs,
                           src_ret, src_len, trunc_out ? src_trunc : nullptr, e->g_obs, e->g_ret, e->g_len, e->g_trunc);
        err = hipGetLastError();
        if (err == hipSuccess && term_obs)
            err = hipMemcpyAsync(term_obs, e->g_obs, sizeof(float) * e->ns * m, hipMemcpyDefault, s);
        if (err == hipSuccess && term_return)
            err = hipMemcpyAsync(term_return, e->g_ret, sizeof(float) * m, hipMemcpyDefault, s);
        if (err == hipSuccess && term_len)
            err = hipMemcpyAsync(term_len, e->g_len, sizeof(int32_t) * m, hipMemcpyDefault, s);
        if (err == hipSuccess && trunc_out)
            err = hipMemcpyAsync(trunc_out, e->g_trunc, sizeof(uint8_t) * m, hipMemcpyDefault, s);
        if (err == hipSuccess) err = hipStreamSynchronize(s);
        if (err != hipSuccess) return hip_fail(err, what);
    }
    return count;
}
}  // namespace

extern "C" {

int64_t rr_fetch_done(rr_env* e, int64_t capacity, int32_t* idx, float* term_obs, float* term_return,
                      int32_t* term_len, void* stream)
{
    if (!e) return fail(RR_EINVAL, "rr_fetch_done: null handle");
    if (capacity < 0) return fail(RR_EINVAL, "rr_fetch_done: negative capacity");
    if (e->steps == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    const int64_t nw = n_words(e->n);
    std::vector<uint64_t> bits(nw);
    hipError_t err = hipMemcpyAsync(bits.data(), e->done_bits, sizeof(uint64_t) * nw, hipMemcpyDeviceToHost, s);
    if (err == hipSuccess) err = hipStreamSynchronize(s);
    if (err != hipSuccess) return hip_fail(err, "rr_fetch_done: done bits");
    std::vector<int32_t> hidx;
    for (int64_t w = 0; w < nw; ++w) {
        uint64_t m = bits[w];
        while (m) {
            const int b = __builtin_ctzll(m);
            hidx.push_back((int32_t)(w * kWave + b));
            m &= m - 1;
        }
    }
    return fetch_rows(e, hidx, capacity, e->term_obs, e->term_ret, e->term_len, nullptr, idx, term_obs, term_return,
                      term_len, nullptr, s, "rr_fetch_done: gather");
}

int64_t rr_gather_rows(rr_env* e, const uint8_t* done, const float* term_obs_src, const float* term_return_src,
                       const int32_t* term_len_src, const uint8_t* truncated_src, int64_t capacity, int32_t* idx,
                       float* term_obs, float* term_return, int32_t* term_len, uint8_t* truncated, void* stream)
{
    if (!e || !done) return fail(RR_EINVAL, "rr_gather_rows: null handle or done flags");
    if (capacity < 0) return fail(RR_EINVAL, "rr_gather_rows: negative capacity");
    if ((term_obs && !term_obs_src) || (term_return && !term_return_src) || (term_len && !term_len_src) ||
        (truncated && !truncated_src))
        return fail(RR_EINVAL, "rr_gather_rows: an output without its source");
    hipStream_t s = (hipStream_t)stream;
    const int64_t n = e->n;
    std::vector<uint64_t> flags((n + 7) / 8, 0);  // the u8 flags, read 8 at a time
    hipError_t err = hipMemcpyAsync(flags.data(), done, (size_t)n, hipMemcpyDefault, s);
    if (err == hipSuccess) err = hipStreamSynchronize(s);
    if (err != hipSuccess) return hip_fail(err, "rr_gather_rows: done flags");
    std::vector<int32_t> hidx;
    const uint8_t* f8 = reinterpret_cast<const uint8_t*>(flags.data());
    for (int64_t w = 0; w < (int64_t)flags.size(); ++w) {
        if (!flags[w]) continue;  // ~1 % of the envs finish per step: most words are zero
        for (int64_t i = 8 * w; i < std::min<int64_t>(8 * w + 8, n); ++i)
            if (f8[i]) hidx.push_back((int32_t)i);
    }
    return fetch_rows(e, hidx, capacity, term_obs_src, term_return_src, term_len_src, truncated_src, idx, term_obs,
                      term_return, term_len, truncated, s, "rr_gather_rows: gather");
}

int rr_copy_terminal(rr_env* e, float* term_obs, float* term_return, int32_t* term_len, void* stream)
{
    if (!e) return fail(RR_EINVAL, "rr_copy_terminal: null handle");
    if (!term_obs && !term_return && !term_len) return RR_OK;
    if (e->steps == 0) return RR_OK;  // no step yet: no done rows
    // only the rows of the envs done at the last step (its done_bits): ~1 % of the rows in steady
    // state, so one pass reads N/8 bytes of masks instead of copying the whole [N][state_dim] buffer
    hipLaunchKernelGGL(copy_done_rows_kernel, dim3(grid_of(e->n)), dim3(kBlock), 0, (hipStream_t)stream,
                       e->done_bits, e->n, e->ns, e->term_obs, e->term_ret, e->term_len, term_obs, term_return,
                       term_len);
    hipError_t err = hipGetLastError();
    return err == hipSuccess ? RR_OK : hip_fail(err, "rr_copy_terminal");
}

// ---- on-device PPO rollout (rocket_policy.inc) ----

}  // extern "C"

template <int O, int A, int P>
struct PolCfg {
    static constexpr int OBS = O, ACT = A, PREC = P;
    using L = pol::Layout<O, A, P>;
};

// f(PolCfg<...>{}) for a supported (obs_dim, act_dim, precision); false otherwise
template <class F>
static bool pol_dispatch(int obs_dim, int act_dim, int precision, F&& f)
{
    if (precision != RR_POLICY_FP32 && precision != RR_POLICY_BF16 && precision != RR_POLICY_FP16X3) return false;
    if (obs_dim == 14 && act_dim == 3) {
        if (precision == RR_POLICY_BF16) f(PolCfg<14, 3, 1>{});
        else if (precision == RR_POLICY_FP16X3) f(PolCfg<14, 3, 2>{});
        else f(PolCfg<14, 3, 0>{});
        return true;
    }
    if (obs_dim == 7 && act_dim == 2) {
        if (precision == RR_POLICY_BF16) f(PolCfg<7, 2, 1>{});
        else if (precision == RR_POLICY_FP16X3) f(PolCfg<7, 2, 2>{});
        else f(PolCfg<7, 2, 0>{});
        return true;
    }
    return false;
}

#define RR_POL_UNSUPPORTED(fn) \
    fail(RR_EINVAL, fn ": supported (obs_dim, act_dim) are (14, 3) and (7, 2), precision RR_POLICY_FP32 / RR_POLICY_BF16 / RR_POLICY_FP16X3")

extern "C" {

int rr_policy_layout(int obs_dim, int act_dim, int precision, int64_t* off)
{
    int size = 0;
    const bool ok = pol_dispatch(obs_dim, act_dim, precision, [&](auto c) {
        using LL = typename decltype(c)::L;
        if (off) {
            const int64_t v[12] = {LL::L1A, LL::B1, LL::L2A, LL::B2, LL::TOWER, LL::PI,
                                   LL::VF,  LL::HA, LL::HV,  LL::HB, LL::VB,    LL::LS};
            for (int k = 0; k < 12; ++k) off[k] = v[k];
        }
        size = LL::SIZE;
    });
    return ok ? size : RR_POL_UNSUPPORTED("rr_policy_layout");
}

int rr_policy_pack(int obs_dim, int act_dim, int precision, const float* const* src, float* params, void* stream)
{
    if (!src || !params) return fail(RR_EINVAL, "rr_policy_pack: null argument");
    PolSrc ps;
    for (int k = 0; k < 13; ++k) {
        if (!src[k]) return fail(RR_EINVAL, "rr_policy_pack: null parameter tensor");
        ps.p[k] = src[k];
    }
    hipStream_t s = (hipStream_t)stream;
    const bool ok = pol_dispatch(obs_dim, act_dim, precision, [&](auto c) {
        using C = decltype(c);
        hipLaunchKernelGGL((policy_pack_kernel<C::OBS, C::ACT, C::PREC>), dim3((C::L::SIZE + 255) / 256), dim3(256),
                           0, s, ps, params);
    });
    if (!ok) return RR_POL_UNSUPPORTED("rr_policy_pack");
    hipError_t err = hipGetLastError();
    return err == hipSuccess ? RR_OK : hip_fail(err, "rr_policy_pack: launch");
}

int rr_policy_act(const float* params, int obs_dim, int act_dim, int precision, int64_t n, int64_t env_id_offset,
                  const float* obs, uint64_t seed, const uint64_t* iter, int t, float* action_env, float* action,
                  float* value, float* log_prob, float* obs_copy, const float* prev_term_obs,
                  const uint8_t* prev_truncated, const float* prev_reward, float gamma, float* reward_out,
                  const uint8_t* done, float* start_out, void* stream)
{
    if (!params || !obs || !iter || !action_env || !action || !value || !log_prob || n <= 0)
        return fail(RR_EINVAL, "rr_policy_act: null argument or n <= 0");
    if (reward_out && (!prev_term_obs || !prev_truncated || !prev_reward))
        return fail(RR_EINVAL, "rr_policy_act: reward_out needs prev_term_obs, prev_truncated, prev_reward");
    if (start_out && !done) return fail(RR_EINVAL, "rr_policy_act: start_out needs done");
    if (((uintptr_t)params & 15) != 0) return fail(RR_EINVAL, "rr_policy_act: params must be 16-B aligned");
    const dim3 grid((unsigned)((n + pol::kEnvsPerBlock - 1) / pol::kEnvsPerBlock)), block(pol::kThreads);
    hipStream_t s = (hipStream_t)stream;
    const uint32_t lo = (uint32_t)seed, hi = (uint32_t)(seed >> 32);
    const bool ok = pol_dispatch(obs_dim, act_dim, precision, [&](auto c) {
        using C = decltype(c);
        hipLaunchKernelGGL((policy_act_kernel<C::OBS, C::ACT, C::PREC>), grid, block, 0, s, params, n, env_id_offset,
                           obs, lo, hi, iter, (uint32_t)t, action_env, action, value, log_prob, obs_copy,
                           prev_term_obs, prev_truncated, prev_reward, gamma, reward_out, done, start_out);
    });
    if (!ok) return RR_POL_UNSUPPORTED("rr_policy_act");
    hipError_t err = hipGetLastError();
    return err == hipSuccess ? RR_OK : hip_fail(err, "rr_policy_act: launch");
}

int rr_policy_bootstrap(const float* params, int obs_dim, int act_dim, int precision, int64_t n,
                        const float* term_obs, const uint8_t* truncated, const float* reward, float gamma,
                        float* reward_out, const float* obs, float* value_out, void* stream)
{
    if (!params || n <= 0) return fail(RR_EINVAL, "rr_policy_bootstrap: null params or n <= 0");
    if (term_obs && (!truncated || !reward || !reward_out))
        return fail(RR_EINVAL, "rr_policy_bootstrap: term_obs needs truncated, reward, reward_out");
    if (!term_obs && !value_out) return fail(RR_EINVAL, "rr_policy_bootstrap: nothing to do");
    if (value_out && !obs) return fail(RR_EINVAL, "rr_policy_bootstrap: value_out needs obs");
    if (((uintptr_t)params & 15) != 0) return fail(RR_EINVAL, "rr_policy_bootstrap: params must be 16-B aligned");
    const dim3 grid((unsigned)((n + pol::kEnvsPerBlock - 1) / pol::kEnvsPerBlock)), block(pol::kThreads);
    hipStream_t s = (hipStream_t)stream;
    const bool ok = pol_dispatch(obs_dim, act_dim, precision, [&](auto c) {
        using C = decltype(c);
        hipLaunchKernelGGL((policy_bootstrap_kernel<C::OBS, C::ACT, C::PREC>), grid, block, 0, s, params, n,
                           term_obs, truncated, reward, gamma, reward_out, obs, value_out);
    });
    if (!ok) return RR_POL_UNSUPPORTED("rr_policy_bootstrap");
    hipError_t err = hipGetLastError();
    return err == hipSuccess ? RR_OK : hip_fail(err, "rr_policy_bootstrap: launch");
}

namespace {
int launch_rollout(rr_env* e, const char* who, bool multi, const float* params, int precision, uint64_t seed,
                   const uint64_t* iter, RolloutIO& io, void* stream)
{
    if (!params || !iter || !io.buf_obs || !io.buf_act || !io.buf_val || !io.buf_logp || !io.buf_start ||
        !io.buf_rew || !io.reward || !io.done)
        return fail(RR_EINVAL, std::string(who) + ": null argument");
    if (((uintptr_t)params & 15) != 0) return fail(RR_EINVAL, std::string(who) + ": params must be 16-B aligned");
    if (precision != RR_POLICY_FP32 && precision != RR_POLICY_BF16 && precision != RR_POLICY_FP16X3)
        return fail(RR_EINVAL,
                    std::string(who) + ": precision must be RR_POLICY_FP32, RR_POLICY_BF16 or RR_POLICY_FP16X3");
    if (e->p.integrator == RR_INT_DOPRI5)
        return fail(RR_EINVAL, std::string(who) + ": RR_INT_DOPRI5 envs step through rr_policy_act + rr_step");
    io.params = params;
    io.iter = iter;
    io.seed_lo = (uint32_t)seed;
    io.seed_hi = (uint32_t)(seed >> 32);
    io.obs_vec_ok = ((uintptr_t)io.obs & 15u) == 0;
    io.buf_obs_vec_ok = ((uintptr_t)io.buf_obs & 15u) == 0;
    const Bufs b = bufs_of(e);
    const uint32_t nn = (uint32_t)e->n;
    const bool counter = e->p.max_episode_steps > 0 || (e->p.flags & (RR_FLAG_EPISODE_STATS | RR_FLAG_AUTO_RESET));
    const uint32_t mode = e->p.flags | (counter ? kModeCounter : 0u);
    const dim3 grid((unsigned)((e->n + rol::kEnvsPerBlock - 1) / rol::kEnvsPerBlock));
    // 64 envs per wave (two 32-env MFMA column tiles). 32 envs per wave (rol::Shape<1>, two waves
    // per SIMD) measured 2-16 % slower at N = 65536 in round 2 and 4-8 % slower in round 4, with or
    // without the second wave's start staggered: the env step's VALU work doubles, and an fp32
    // MFMA holds its SIMD's vector issue, so one wave's MFMAs do not hide the other's VALU work
    // (tools/coissue_probe.hip, profiles/r04/coissue/).
    // The collect kernel (MULTI) lives in the third translation unit (rocket_collect.hip), compiled
    // with the MFMA accumulators in VGPRs (rl_rocket_amd/build.py COLLECT_FLAGS).
    hipStream_t s = (hipStream_t)stream;
    const int prec = precision == RR_POLICY_BF16 ? 1 : precision == RR_POLICY_FP16X3 ? 2 : 0;
    hipError_t err = hipSuccess;
    if (multi) {
        err = (hipError_t)rrc_launch_collect(e->p.model, e->p.integrator, prec, grid.x, e->state, nn, mode, &e->kp,
                                             &b, &io, stream);
    } else {
        const bool m6 = e->p.model == RR_MODEL_6DOF, euler = e->p.integrator == RR_INT_EULER;
#define RR_LAUNCH(M, I, PR)                                                                                     \
    hipLaunchKernelGGL((rollout_step_kernel<M, I, PR, false, 2>), grid, dim3(rol::Shape<2>::kThreads), 0, s, \
                       e->state, nn, mode, e->kp, b, io)
#define RR_LAUNCH_P(M, I)                  \
    do {                                   \
        if (prec == 1) RR_LAUNCH(M, I, 1); \
        else if (prec == 2) RR_LAUNCH(M, I, 2); \
        else RR_LAUNCH(M, I, 0);           \
    } while (0)
        if (m6 && !euler) RR_LAUNCH_P(6, RR_INT_RK4);
        else if (m6) RR_LAUNCH_P(6, RR_INT_EULER);
        else if (!euler) RR_LAUNCH_P(3, RR_INT_RK4);
        else RR_LAUNCH_P(3, RR_INT_EULER);
#undef RR_LAUNCH_P
#undef RR_LAUNCH
        err = hipGetLastError();
    }
    if (err != hipSuccess) return hip_fail(err, (std::string(who) + ": launch").c_str());
    e->steps += io.T;
    note_stream(e, stream);
    return RR_OK;
}
}  // namespace

int rr_rollout_step(rr_env* e, const float* params, int precision, uint64_t seed, const uint64_t* iter, int t,
                    float gamma, float* buf_obs, float* buf_action, float* buf_value, float* buf_log_prob,
                    float* buf_start, float* buf_reward, float* obs, float* reward, uint8_t* done, uint8_t* truncated,
                    float* terms, void* stream)
{
    if (!e) return fail(RR_EINVAL, "rr_rollout_step: null handle");
    RolloutIO io = {};
    io.buf_obs = buf_obs;
    io.buf_act = buf_action;
    io.buf_val = buf_value;
    io.buf_logp = buf_log_prob;
    io.buf_start = buf_start;
    io.buf_rew = buf_reward;
    io.obs = obs;
    io.reward = reward;
    io.done = done;
    io.truncated = truncated;
    io.terms = terms;
    io.t = (uint32_t)t;
    io.gamma = gamma;
    io.T = 1;
    return launch_rollout(e, "rr_rollout_step", false, params, precision, seed, iter, io, stream);
}

int rr_rollout_collect(rr_env* e, const float* params, int precision, uint64_t seed, const uint64_t* iter,
                       int n_steps, float gamma, float gae_lambda, float* buf_obs, float* buf_action,
                       float* buf_value, float* buf_log_prob, float* buf_start, float* buf_reward,
                       float* buf_advantage, float* buf_return, float* last_value, float* last_done,
                       float* last_start, float* obs, float* reward, uint8_t* done, uint8_t* truncated, float* terms,
                       void* stream)
{
    if (!e) return fail(RR_EINVAL, "rr_rollout_collect: null handle");
    if (n_steps <= 0) return fail(RR_EINVAL, "rr_rollout_collect: n_steps must be positive");
    if ((buf_advantage == nullptr) != (buf_return == nullptr))
        return fail(RR_EINVAL, "rr_rollout_collect: buf_advantage and buf_return go together");
    RolloutIO io = {};
    io.buf_obs = buf_obs;
    io.buf_act = buf_action;
    io.buf_val = buf_value;
    io.buf_logp = buf_log_prob;
    io.buf_start = buf_start;
    io.buf_rew = buf_reward;
    io.buf_adv = buf_advantage;
    io.buf_ret = buf_return;
    io.last_value = last_value;
    io.last_done = last_done;
    io.last_start = last_start;
    io.obs = obs;
    io.reward = reward;
    io.done = done;
    io.truncated = truncated;
    io.terms = terms;
    io.t = 0;
    io.T = (uint32_t)n_steps;
    io.gamma = gamma;
    io.lam = gae_lambda;
    return launch_rollout(e, "rr_rollout_collect", true, params, precision, seed, iter, io, stream);
}

int rr_gae(int64_t T, int64_t n, const float* rewards, const float* values, const float* starts,
           const float* last_value, const float* last_done, float gamma, float lam, float* advantages,
           float* returns, void* stream)
{
    if (!rewards || !values || !starts || !last_value || !last_done || !advantages || !returns || T <= 0 || n <= 0)
        return fail(RR_EINVAL, "rr_gae: null argument or empty rollout");
    hipLaunchKernelGGL(gae_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, (hipStream_t)stream,
                       T, n, rewards, values, starts, last_value, last_done, gamma, lam, advantages, returns);
    hipError_t err = hipGetLastError();
    return err == hipSuccess ? RR_OK : hip_fail(err, "rr_gae: launch");
}

namespace {
int64_t ppo_nwg(int64_t batch)
{
    const int64_t tiles = (batch + ppo::kTile - 1) / ppo::kTile;
    const int64_t w = (tiles + ppo::kWaves - 1) / ppo::kWaves;
    return w < 1 ? 1 : (w > ppo::kMaxWG ? ppo::kMaxWG : w);
}

int64_t ppo_part_floats(int obs_dim, int act_dim)
{
    if (obs_dim == 14 && act_dim == 3) return ppo::Part<14, 3>::SIZE;
    if (obs_dim == 7 && act_dim == 2) return ppo::Part<7, 2>::SIZE;
    return 0;
}

int64_t ppo_pack_floats(int obs_dim, int act_dim)
{
    return obs_dim == 14 ? ppo::Pack<14, 3>::SIZE : ppo::Pack<7, 2>::SIZE;
}

// rr_ppo_workspace_size's layout: advantage partial sums | 2 towers x nwg partial-gradient vectors |
// 2 packed tower images (16-B aligned: Part::SIZE % 4 == 0)
void ppo_carve(PpoLaunch& L, int obs_dim, int act_dim, int64_t batch, void* workspace)
{
    L.obs_dim = obs_dim;
    L.nwg = (int)ppo_nwg(batch);
    L.adv_part = (double*)workspace;
    L.part = (float*)((char*)workspace + 2 * ppo::kAdvPart * sizeof(double));
    L.pack = L.part + 2 * (int64_t)L.nwg * ppo_part_floats(obs_dim, act_dim);
}
}  // namespace

int rr_clip_adam_workspace_size(int64_t total_elements, int64_t* bytes)
{
    if (total_elements < 1 || !bytes) return fail(RR_EINVAL, "rr_clip_adam_workspace_size: total_elements >= 1");
    *bytes = ((total_elements + kAdamThreads - 1) / kAdamThreads + 1) * (int64_t)sizeof(float);
    return RR_OK;
}

int rr_clip_adam(int n_tensors, float* const* params, float* const* grads, float* const* exp_avg,
                 float* const* exp_avg_sq, float* const* step, const int64_t* numel, float max_grad_norm,
                 const float* lr, double beta1, double beta2, float eps, void* workspace, int64_t workspace_bytes,
                 void* stream)
{
    if (n_tensors < 1 || n_tensors > 16) return fail(RR_EINVAL, "rr_clip_adam: 1 .. 16 tensors");
    if (!params || !grads || !exp_avg || !exp_avg_sq || !step || !numel || !lr || !workspace)
        return fail(RR_EINVAL, "rr_clip_adam: null argument");
    AdamList a = {};
    a.n = n_tensors;
    for (int t = 0; t < n_tensors; ++t) {
        if (!params[t] || !grads[t] || !exp_avg[t] || !exp_avg_sq[t] || !step[t] || numel[t] < 1)
            return fail(RR_EINVAL, "rr_clip_adam: null or empty tensor");
        a.param[t] = params[t];
        a.grad[t] = grads[t];
        a.exp_avg[t] = exp_avg[t];
        a.exp_avg_sq[t] = exp_avg_sq[t];
        a.step[t] = step[t];
        a.start[t + 1] = a.start[t] + numel[t];
    }
    int64_t need = 0;
    rr_clip_adam_workspace_size(a.start[n_tensors], &need);
    if (workspace_bytes < need) return fail(RR_EINVAL, "rr_clip_adam: workspace smaller than rr_clip_adam_workspace_size");
    PpoLaunch L = {};
    L.op = 2;
    L.a = a;
    L.work = (float*)workspace;
    L.max_norm = max_grad_norm;
    L.lr = lr;
    L.beta1 = (float)beta1;
    L.beta2 = (float)beta2;
    L.w1 = (float)(1.0 - beta1);
    L.w2 = (float)(1.0 - beta2);
    L.eps = eps;
    const hipError_t err = (hipError_t)rrc_launch_learner(&L, stream);
    return err == hipSuccess ? RR_OK : hip_fail(err, "rr_clip_adam: launch");
}

int rr_ppo_workspace_size(int obs_dim, int act_dim, int64_t batch, int64_t* bytes)
{
    const int64_t pf = ppo_part_floats(obs_dim, act_dim);
    if (!pf) return fail(RR_EINVAL, "rr_ppo_workspace_size: supported (obs_dim, act_dim) are (14, 3) and (7, 2)");
    if (batch < 2 || !bytes) return fail(RR_EINVAL, "rr_ppo_workspace_size: batch >= 2 and bytes required");
    // adv partial sums | 2 towers x nwg partial-gradient vectors | 2 packed tower images
    *bytes = (int64_t)(2 * ppo::kAdvPart * sizeof(double)) +
             2 * (ppo_nwg(batch) * pf + ppo_pack_floats(obs_dim, act_dim)) * (int64_t)sizeof(float);
    return RR_OK;
}

int rr_ppo_grad(int obs_dim, int act_dim, const float* const* params, float* const* grads, const float* obs,
                const float* actions, const float* old_log_prob, const float* advantages, const float* returns,
                const int64_t* idx, int64_t batch, float clip_range, float ent_coef, float vf_coef, float* stats,
                void* workspace, int64_t workspace_bytes, void* stream)
{
    int64_t need = 0;
    const int rc = rr_ppo_workspace_size(obs_dim, act_dim, batch, &need);
    if (rc != RR_OK) return rc;
    if (!params || !grads || !obs || !actions || !old_log_prob || !advantages || !returns || !idx || !workspace)
        return fail(RR_EINVAL, "rr_ppo_grad: null argument");
    if (workspace_bytes < need) return fail(RR_EINVAL, "rr_ppo_grad: workspace smaller than rr_ppo_workspace_size");
    if (((uintptr_t)workspace & 15) != 0) return fail(RR_EINVAL, "rr_ppo_grad: workspace must be 16-B aligned");
    if (!(clip_range >= 0.0f)) return fail(RR_EINVAL, "rr_ppo_grad: clip_range must be >= 0");
    PpoLaunch L = {};
    L.op = 0;
    for (int k = 0; k < 13; ++k) {
        if (!params[k] || !grads[k]) return fail(RR_EINVAL, "rr_ppo_grad: null parameter or gradient tensor");
        L.ps.p[k] = params[k];
        L.pg.p[k] = grads[k];
    }
    ppo_carve(L, obs_dim, act_dim, batch, workspace);
    L.obs = obs;
    L.actions = actions;
    L.old_log_prob = old_log_prob;
    L.advantages = advantages;
    L.returns = returns;
    L.idx = idx;
    L.batch = batch;
    L.clip = clip_range;
    L.ent = ent_coef;
    L.vf = vf_coef;
    L.stats = stats;
    const hipError_t err = (hipError_t)rrc_launch_learner(&L, stream);
    return err == hipSuccess ? RR_OK : hip_fail(err, "rr_ppo_grad: launch");
}

int rr_ppo_update_workspace_size(int obs_dim, int act_dim, int64_t batch, int64_t* bytes)
{
    int64_t ppo = 0;
    if (!ppo_part_floats(obs_dim, act_dim))
        return fail(RR_EINVAL, "rr_ppo_update_workspace_size: supported (obs_dim, act_dim) are (14, 3) and (7, 2)");
    if (batch < 2 || !bytes) return fail(RR_EINVAL, "rr_ppo_update_workspace_size: batch >= 2 and bytes required");
    rr_ppo_workspace_size(obs_dim, act_dim, batch, &ppo);
    // + the finish kernel's squared-gradient sums (two towers) and the step count, 16-B rows
    const int64_t fin = (ppo_part_floats(obs_dim, act_dim) + kFinElems - 1) / kFinElems;
    *bytes = (ppo + 15) / 16 * 16 + (2 * fin + 1 + 3) / 4 * 16;
    return RR_OK;
}

int rr_ppo_update(int obs_dim, int act_dim, float* const* params, float* const* grads, float* const* exp_avg,
                  float* const* exp_avg_sq, float* const* step, const float* obs, const float* actions,
                  const float* old_log_prob, const float* advantages, const float* returns, const int64_t* idx,
                  int64_t batch, const int64_t* next_idx, int64_t next_batch, float clip_range, float ent_coef,
                  float vf_coef, float max_grad_norm, const float* lr, double beta1, double beta2, float eps,
                  float* stats, uint32_t flags, void* workspace, int64_t workspace_bytes, void* stream)
{
    int64_t need = 0, ppo_bytes = 0;
    int rc = rr_ppo_update_workspace_size(obs_dim, act_dim, batch, &need);
    if (rc != RR_OK) return rc;
    rr_ppo_workspace_size(obs_dim, act_dim, batch, &ppo_bytes);
    if (!params || !grads || !exp_avg || !exp_avg_sq || !step || !obs || !actions || !old_log_prob || !advantages ||
        !returns || !idx || !lr || !workspace)
        return fail(RR_EINVAL, "rr_ppo_update: null argument");
    if (workspace_bytes < need) return fail(RR_EINVAL, "rr_ppo_update: workspace smaller than rr_ppo_update_workspace_size");
    if (((uintptr_t)workspace & 15) != 0) return fail(RR_EINVAL, "rr_ppo_update: workspace must be 16-B aligned");
    if (!(clip_range >= 0.0f)) return fail(RR_EINVAL, "rr_ppo_update: clip_range must be >= 0");
    if (flags & ~(uint32_t)RR_PPO_CHAINED) return fail(RR_EINVAL, "rr_ppo_update: unknown flag bits");
    if (next_idx && !(next_batch >= 2 && next_batch <= batch))
        return fail(RR_EINVAL, "rr_ppo_update: next_batch must be in [2, batch]");
    const int na = act_dim, no = obs_dim;
    const int64_t numel[13] = {64 * no, 64, 64 * 64, 64, 64 * no, 64, 64 * 64, 64, 64 * na, na, 64, 1, na};
    PpoLaunch L = {};
    L.op = 1;
    L.a.n = 13;
    for (int k = 0; k < 13; ++k) {
        if (!params[k] || !grads[k] || !exp_avg[k] || !exp_avg_sq[k] || !step[k])
            return fail(RR_EINVAL, "rr_ppo_update: null parameter, gradient or optimizer-state tensor");
        L.ps.p[k] = params[k];
        L.pg.p[k] = grads[k];
        L.a.param[k] = params[k];
        L.a.grad[k] = grads[k];
        L.a.exp_avg[k] = exp_avg[k];
        L.a.exp_avg_sq[k] = exp_avg_sq[k];
        L.a.step[k] = step[k];
        L.a.start[k + 1] = L.a.start[k] + numel[k];
        L.a.wstart[k + 1] = L.a.wstart[k] + (numel[k] + kWave - 1) / kWave * kWave;
    }
    ppo_carve(L, obs_dim, act_dim, batch, workspace);
    L.normw = (float*)((char*)workspace + (ppo_bytes + 15) / 16 * 16);
    L.nbp = (int)((L.a.wstart[13] + kAdamThreads - 1) / kAdamThreads);
    L.obs = obs;
    L.actions = actions;
    L.old_log_prob = old_log_prob;
    L.advantages = advantages;
    L.returns = returns;
    L.idx = idx;
    L.next_idx = next_idx;
    L.batch = batch;
    L.next_batch = next_batch;
    L.clip = clip_range;
    L.ent = ent_coef;
    L.vf = vf_coef;
    L.max_norm = max_grad_norm;
    L.lr = lr;
    L.beta1 = (float)beta1;
    L.beta2 = (float)beta2;
    L.w1 = (float)(1.0 - beta1);
    L.w2 = (float)(1.0 - beta2);
    L.eps = eps;
    L.stats = stats;
    L.flags = flags;
    const hipError_t err = (hipError_t)rrc_launch_learner(&L, stream);
    return err == hipSuccess ? RR_OK : hip_fail(err, "rr_ppo_update: launch");
}


}  // extern "C"
#endif  // RR_TU_EXACT
