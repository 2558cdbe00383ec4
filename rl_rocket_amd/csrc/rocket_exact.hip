// rocket_exact.hip — the second translation unit of librocket_hip.so: the exact-integrator
// kernels (step_exact_kernel, rocket_dopri5.inc) and nothing else, so that they can be compiled
// with their own scheduler setting (rl_rocket_amd/build.py: -amdgpu-schedule-metric-bias=100,
// register pressure first) without touching the fast kernels' code. With the fast kernels'
// scheduler the 6DOF exact kernel spilled 33 VGPRs to scratch at one wave per SIMD.
#define RR_TU_EXACT 1
#include "rocket_hip.hip"
