// rocket_collect.hip — the third translation unit of librocket_hip.so: the rollout collect kernels
// (rollout_step_kernel<..., MULTI = true>, rocket_rollout.inc: rr_rollout_collect) and nothing else,
// so that they can be compiled with their own code-generation setting (rl_rocket_amd/build.py
// COLLECT_FLAGS: -amdgpu-mfma-vgpr-form, the MFMA accumulators in VGPRs) without touching the other
// kernels. In the AGPR form every tanh input of the policy towers first crosses back with a
// v_accvgpr_read (384 in the collect loop); in the VGPR form the loop issues 12 % fewer VALU
// instructions and the collect measured 5.5 % faster (profiles/r04/ab_vf/). The same flag on the
// whole main TU would cost the per-step fp16x3 rollout kernels their second wave per SIMD.
#define RR_TU_COLLECT 1
#include "rocket_hip.hip"
