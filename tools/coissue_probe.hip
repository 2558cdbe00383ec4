// coissue_probe.hip — measurement-only (NOT part of librocket_hip.so): does one wave's fp32 MFMA
// stream (v_mfma_f32_32x32x2_f32, the rollout towers' instruction) leave the SIMD's vector
// issue to a second wave's VALU stream? Two waves per SIMD (256 workgroups x 8 waves), three
// kernels of identical shape:
//   role 0  every wave: `m` rounds of 4 independent fp32 MFMAs        (MFMA alone, 2 waves/SIMD)
//   role 1  every wave: `v` rounds of 4 independent v_fma_f32 chains  (VALU alone, 2 waves/SIMD)
//   role 2  waves 0-3 the MFMA stream, waves 4-7 the VALU stream      (one of each per SIMD)
// role 2 ~ max(half of role 0, half of role 1) means the VALU runs under the MFMAs; ~ their sum
// means the MFMA holds the SIMD's vector issue. Roles 3-5 ask the same of transcendentals
// (v_exp_f32, the rollout towers' tanh):
//   role 3  every wave: `v` rounds of 4 independent v_exp_f32 chains
//   role 4  waves 0-3 the MFMA stream, waves 4-7 the v_exp_f32 stream
//   role 5  every wave: `m` rounds of 4 MFMAs with 2 v_exp_f32 after each MFMA (one stream)
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int ROLE>
__global__ __launch_bounds__(512) void coissue_kernel(float* out, int m, int v, float seed)
{
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
    // waves w and w + 4 of a workgroup share a SIMD (the step kernel's main / helper pairing)
    const bool mfma = ROLE == 0 || ((ROLE == 2 || ROLE == 4) && wv < 4u);
    const bool trans = ROLE == 3 || (ROLE == 4 && wv >= 4u);
    float r = seed + (float)threadIdx.x;
    if (ROLE == 5) {
        f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
        const float a = r, b = r * 0.5f;
        float x0 = r, x1 = r + 1.0f, x2 = r + 2.0f, x3 = r + 3.0f;
        for (int k = 0; k < m; ++k) {
            c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c0, 0, 0, 0);
            x0 = __builtin_amdgcn_exp2f(x0);
            x1 = __builtin_amdgcn_exp2f(x1);
            c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(b, a, c1, 0, 0, 0);
            x2 = __builtin_amdgcn_exp2f(x2);
            x3 = __builtin_amdgcn_exp2f(x3);
            c2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, a, c2, 0, 0, 0);
            x0 = __builtin_amdgcn_exp2f(x0);
            x1 = __builtin_amdgcn_exp2f(x1);
            c3 = __builtin_amdgcn_mfma_f32_32x32x2f32(b, b, c3, 0, 0, 0);
            x2 = __builtin_amdgcn_exp2f(x2);
            x3 = __builtin_amdgcn_exp2f(x3);
            asm volatile("" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));
        }
        r = c0[0] + c1[3] + c2[7] + c3[15] + x0 + x1 + x2 + x3;
    } else if (trans) {
        float x0 = r, x1 = r + 1.0f, x2 = r + 2.0f, x3 = r + 3.0f;
        for (int k = 0; k < v; ++k) {
            x0 = __builtin_amdgcn_exp2f(x0);
            x1 = __builtin_amdgcn_exp2f(x1);
            x2 = __builtin_amdgcn_exp2f(x2);
            x3 = __builtin_amdgcn_exp2f(x3);
            asm volatile("" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));
        }
        r = x0 + x1 + x2 + x3;
    } else if (mfma) {
        f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
        const float a = r, b = r * 0.5f;
        for (int k = 0; k < m; ++k) {
            c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(b, a, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, a, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_f32_32x32x2f32(b, b, c3, 0, 0, 0);
        }
        r = c0[0] + c1[3] + c2[7] + c3[15];
    } else {
        float x0 = r, x1 = r + 1.0f, x2 = r + 2.0f, x3 = r + 3.0f;
        for (int k = 0; k < v; ++k) {
            x0 = fmaf(x0, 0.999f, 0.5f);
            x1 = fmaf(x1, 0.999f, 0.25f);
            x2 = fmaf(x2, 0.999f, 0.125f);
            x3 = fmaf(x3, 0.999f, 0.0625f);
            asm volatile("" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));
        }
        r = x0 + x1 + x2 + x3;
    }
    if (r == 12345.0f) out[blockIdx.x * blockDim.x + threadIdx.x] = r;  // never true: keeps the work
}
}  // namespace

extern "C" int cp_launch(int role, int blocks, float* out, int m, int v, void* stream)
{
    if (role < 0 || role > 5 || blocks <= 0 || m < 0 || v < 0) return -1;
    hipStream_t s = (hipStream_t)stream;
    if (role == 0) hipLaunchKernelGGL(coissue_kernel<0>, dim3(blocks), dim3(512), 0, s, out, m, v, 1.0f);
    else if (role == 1) hipLaunchKernelGGL(coissue_kernel<1>, dim3(blocks), dim3(512), 0, s, out, m, v, 1.0f);
    else if (role == 2) hipLaunchKernelGGL(coissue_kernel<2>, dim3(blocks), dim3(512), 0, s, out, m, v, 1.0f);
    else if (role == 3) hipLaunchKernelGGL(coissue_kernel<3>, dim3(blocks), dim3(512), 0, s, out, m, v, 1.0f);
    else if (role == 4) hipLaunchKernelGGL(coissue_kernel<4>, dim3(blocks), dim3(512), 0, s, out, m, v, 1.0f);
    else hipLaunchKernelGGL(coissue_kernel<5>, dim3(blocks), dim3(512), 0, s, out, m, v, 1.0f);
    return (int)hipGetLastError();
}
