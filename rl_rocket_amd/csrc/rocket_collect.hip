// rocket_collect.hip — the third translation unit of librocket_hip.so: the rollout collect kernels
// (rollout_step_kernel<..., MULTI = true>, rocket_rollout.inc: rr_rollout_collect) and the PPO
// learner's kernels (rocket_ppo.inc: rr_ppo_grad / rr_ppo_update / rr_clip_adam, launched through
// rrc_launch_learner), compiled with their own code-generation setting (rl_rocket_amd/build.py
// COLLECT_FLAGS: -amdgpu-mfma-vgpr-form, the MFMA accumulators in VGPRs) without touching the other
// kernels. In the AGPR form every tanh input of the policy towers first crosses back with a
// v_accvgpr_read (384 in the collect loop); in the VGPR form the loop issues 12 % fewer VALU
// instructions and the collect measured 5.5 % faster (profiles/r04/ab_vf/). The gradient kernel
// moves 1 082 -> 343 registers between the files and its minibatch measured 3 % faster, bitwise
// (profiles/r06/ppo_vf/). The same flag on the whole main TU would cost the per-step fp16x3
// rollout kernels their second wave per SIMD.
#define RR_TU_COLLECT 1
#include "rocket_hip.hip"
