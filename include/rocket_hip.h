/*
 * rocket_hip.h — C-ABI of librocket_hip.so, the MI355X-native vectorized
 * rocket-landing env step (gfx950 HIP kernels).
 *
 * The reference has no native boundary: its hot path is the Python gym 0.21
 * Env API (reference my_environment/envs/rocket_env.py). Each entry point below
 * replaces one reference interface, batched over N independent envs that live in
 * HBM in struct-of-arrays fp32 layout:
 *
 *   rr_create      <- Rocket6DOF.__init__ rocket_env.py:511-663 / Rocket.__init__ :27-135
 *                     (kwargs lowered to rr_params on the host, rl_rocket_amd/params.py)
 *   rr_reset       <- Rocket6DOF.reset rocket_env.py:665-688 / Rocket.reset :137-148
 *                     (+ seed(): rocket_env.py:1063-1065 / :478-480)
 *   rr_step        <- Rocket6DOF.step rocket_env.py:690-719 (+ Simulator6DOF.step/RHS
 *                     simulator.py:227-378) / Rocket.step :150-175 (+ simulator.py:55-130),
 *                     fused with gym TimeLimit (main_6DOF.py:21), the SB3 vec-env auto-reset
 *                     and, optionally, RewardAnnealing (wrappers.py:68-86)
 *   rr_set_state / rr_get_state
 *                  <- direct access to Simulator*.state / .t used by the reference's
 *                     callers (env.SIM, rocket_env.py:686, :694; used here for parity
 *                     injection and checkpoint/restore)
 *   rr_fetch_done / rr_copy_terminal / rr_get_buffers
 *                  <- info["terminal_observation"] / Monitor episode stats for done envs
 *                     (SB3 DummyVecEnv / Monitor, main_6DOF.py:18-24)
 *
 * Conventions
 *   - All data pointers are DEVICE pointers (e.g. torch.Tensor.data_ptr()) on the
 *     handle's device, or pinned host memory from rr_host_alloc (zero-copy: the kernels read
 *     and write it directly), owned by the caller unless stated otherwise.
 *   - Every call is asynchronous on the given hipStream_t (pass as void*; NULL = the
 *     default stream). Apart from rr_fetch_done (documented as synchronising), no call
 *     synchronises, allocates or frees after rr_create, so rr_step / rr_reset can be
 *     captured into a hipGraph.
 *   - Return value: 0 on success, < 0 on error (RR_E*); rr_last_error() returns a
 *     thread-local message. No exception or abort crosses the ABI.
 *   - A handle is not thread-safe; use one handle per stream / GPU.
 */
#ifndef ROCKET_HIP_H
#define ROCKET_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RR_ABI_VERSION 12

/* error codes */
#define RR_OK 0
#define RR_EINVAL -1   /* bad argument */
#define RR_EHIP -2     /* HIP runtime error */
#define RR_ENOMEM -3   /* allocation failed */

/* models */
#define RR_MODEL_3DOF 3
#define RR_MODEL_6DOF 6

/* integrators. RK4 is the fast parity mode (fp32 state; matches the reference's
 * adaptive RK45 + terminal ground event to <= 1e-5 floored-relative).
 * EULER is a declared NON-parity speed mode (BASELINE config "3DOF Euler").
 * DOPRI5 is the exact mode: fp64 state and the reference's own integrator
 * (scipy RK45: select_initial_step, DOPRI5 tableau, RMS error controller, dense-output
 * brentq ground event; simulator.py:230-241 / :58-69), per-env adaptive, with the
 * simulator clock t (round(t + dt, 3), simulator.py:245) kept as elapsed_steps * dt. */
#define RR_INT_RK4 0
#define RR_INT_EULER 1
#define RR_INT_DOPRI5 2

/* rr_params.flags */
#define RR_FLAG_AUTO_RESET 0x1        /* reset done envs inside rr_step (SB3 vec-env semantics) */
#define RR_FLAG_EPISODE_STATS 0x2     /* keep per-env episode return (Monitor) */
#define RR_FLAG_REWARD_ANNEALING 0x4  /* reward = attitude + goal - xi*(a_thrust+1)  (wrappers.py:72-86) */
#define RR_FLAG_ACTION_SOA 0x8        /* action laid out [n_act][N] instead of [N][n_act] */
#define RR_FLAG_SCIPY_H0_CLAMP 0x10   /* DOPRI5: scipy >= 1.12 select_initial_step (clamp h0 to
                                         the interval); default = scipy 1.7 (requirements.txt:73) */
#define RR_FLAG_HOST_STATE 0x20       /* the state planes (+ v0, counter words, episode returns) live in
                                         pinned, GPU-coherent host memory instead of HBM: after the
                                         stream is synchronised the host reads them through
                                         rr_get_buffers with no copy. For small N — the single-env gym
                                         shims (rocket_env.py:690-719 called once per env step), whose
                                         step is then one launch + one synchronise with the action and
                                         outputs in rr_host_alloc memory */

#define RR_MAX_STATE 14

/* Per-config constants. Lowered on the host from the reference env kwargs
 * (rl_rocket_amd/params.py restates rocket_env.py:51-123 / :557-658). Values the
 * reference holds as Python floats are double here; the fp32 kernels round them once
 * at rr_create (bounds with the rounding direction that keeps each comparison exact). */
typedef struct rr_params {
    int32_t model;               /* RR_MODEL_3DOF | RR_MODEL_6DOF */
    int32_t integrator;          /* RR_INT_* */
    int32_t max_episode_steps;   /* gym TimeLimit; 0 = none */
    uint32_t flags;              /* RR_FLAG_* */
    double dt;                   /* timestep [s] */
    float ic_low[RR_MAX_STATE];  /* init_space Box low  (float32, rocket_env.py:564-567) */
    float ic_high[RR_MAX_STATE]; /* init_space Box high */
    double normalizer[RR_MAX_STATE]; /* state_normalizer, float64 (rocket_env.py:592-612 / :76-94) */
    double bounds_low[3];        /* 6DOF: position Box low (float32 values, inclusive);
                                    3DOF: [-x_bound, -, -] (x <= -x_bound is out) */
    double bounds_high[3];       /* 6DOF: position Box high; 3DOF: [x_bound, z_bound, -] (>= is out) */
    double max_gimbal;           /* rad */
    double max_thrust;           /* N */
    double alfa, beta, eta, gamma, delta, kappa, xi; /* reward_coeff */
    double waypoint, landing_radius, max_velocity;
    double att_limit[3];         /* trajectory_limits["attitude_limit"] (zyx) */
    double land_att_limit[3];    /* landing_params["landing_attitude_limit"] */
    double omega_lim[3];         /* 0.2 hard-coded in the reference (rocket_env.py:656) */
} rr_params;

/* Library-owned device buffers, valid until rr_destroy. done_bits / terminal_* refer
 * to the MOST RECENT rr_step on the handle (overwritten by the next step). */
typedef struct rr_buffers {
    float* state;          /* [state_dim][N] fp32 SoA */
    float* v0;             /* [N] ||IC velocity|| of the episode (rocket_env.py:989-991) */
    int32_t* elapsed;      /* [N] counter word: TimeLimit steps in bits 0..E-1, episode in bits E..31,
                              E = rr_counter_bits() */
    float* ep_return;      /* [N] running episode return (RR_FLAG_EPISODE_STATS) */
    uint64_t* done_bits;   /* [ceil(N/64)] wave-ballot done masks: bit b of word w <=> env 64w+b done */
    float* terminal_obs;   /* [N][state_dim] final obs of env i, valid where done[i] */
    float* terminal_return;/* [N] episode return of env i, valid where done[i] */
    int32_t* terminal_len; /* [N] episode length of env i, valid where done[i] */
} rr_buffers;

typedef struct rr_env rr_env;

int rr_abi_version(void);
const char* rr_last_error(void);

/* Allocate N envs on `device`. env_id_offset = global id of env 0 (multi-GPU shards
 * use rank*N so every env has its own RNG stream). Envs start un-initialised: call
 * rr_reset before the first rr_step. 1 <= N and N * (state_dim + 3) * 4 <= 2^32 - 1 (the
 * kernels address each plane / row block with 32-bit buffer offsets): at most 63 161 283
 * 6DOF or 107 374 182 3DOF envs per handle, else RR_EINVAL; larger batches are several
 * handles (shards). */
int rr_create(rr_env** out, const rr_params* p, int64_t n, int64_t env_id_offset, int device);
int rr_destroy(rr_env* e);
int64_t rr_num_envs(const rr_env* e);
int rr_state_dim(const rr_env* e);
int rr_action_dim(const rr_env* e);

/* Set the key of the reset stream. Resets are counter-based: when env `gid` ends an episode
 * with counter word `cw` (episode number | elapsed steps), its next initial condition comes
 * from a register-resident xorshift128 whose four words are chained lowbias32 mixes of
 * (the seed's four key words — splitmix64 of `seed` on the host — , gid, cw): deterministic,
 * independent of how envs are sharded over GPUs, and free of per-env RNG state in HBM. The
 * episode field has 32 - rr_counter_bits() bits (22 under the reference's TimeLimit 800), so
 * one env's keys do not repeat for 2^22 episodes. Stream-ordered host call: the key is written
 * in the order of `stream` (launches queued on it before the call read the old key) and the
 * call returns once it has landed (it synchronises `stream`, nothing else); it applies to every
 * launch that runs after it, including replays of hipGraphs captured before it, at every N.
 * Launches of the handle (step / reset / rollout) queued on OTHER streams since the last rr_seed
 * are waited for on the device: the key copy waits on a per-handle event recorded on each of
 * those streams (up to 8 distinct streams; past that, or when one of them no longer exists, the
 * call synchronises the device), so no launch still queued there reads a half-written key, and
 * nothing else on the device is waited for. NOT tracked: replays of hipGraphs (they are not
 * launches of the handle) — the caller orders a replay queued on another stream before the seed
 * (seed on the replay's stream, or synchronise it first).
 * RR_EINVAL while `stream` is being captured into a graph. */
int rr_seed(rr_env* e, uint64_t seed, void* stream);
/* Sample a fresh initial condition for every env where mask[i] != 0 (all when mask is
 * NULL), write the normalised obs [N][state_dim] (obs may be NULL). */
int rr_reset(rr_env* e, const uint8_t* mask, float* obs, void* stream);

/* One env step for all N envs.
 *   action    [N][action_dim] fp32 normalised in [-1,1] (not clipped, like the reference)
 *   obs       [N][state_dim] fp32 out (post-reset obs for done envs under AUTO_RESET)
 *   reward    [N] fp32 out
 *   done      [N] u8 out (ground event | bounds violation | non-finite state | TimeLimit)
 *   truncated [N] u8 out or NULL (TimeLimit.truncated)
 *   terms     [n_terms + 2][N] fp32 out or NULL: info["rewards_dict"] (6DOF 5 terms:
 *             velocity_tracking, thrust_penalty, eta, attitude_constraint, rew_goal;
 *             3DOF 6 terms: ..., attitude_hint, rew_goal), then two planes:
 *             info["bounds_violation"] (0 / 1) and the solve_ivp status: 1 = ground event,
 *             -1 = failure (a post-step state with a NaN / inf component: done, like the
 *             reference's done = bool(status), rocket_env.py:702 / :158), 0 otherwise */
int rr_step(rr_env* e, const float* action, float* obs, float* reward, uint8_t* done, uint8_t* truncated,
            float* terms, void* stream);

/* rr_step with obs, reward and done packed as one fp32 row per env: rows [N][state_dim + 2]
 * = (obs[state_dim], reward, done ? 1 : 0), bitwise the values rr_step writes. One 16-B
 * coalesced tile store per wave, and the row block is exactly the send buffer of the
 * multi-GPU all-gather (rl_rocket_amd.dist.ShardGather), so no copy kernels
 * sit between the step and the collective. truncated / terms as rr_step. RK4 / Euler envs
 * with [N][action_dim] actions. */
int rr_step_rows(rr_env* e, const float* action, float* rows, uint8_t* truncated, float* terms, void* stream);

/* n_steps consecutive rr_step launches on `stream`, step t taking action batch t % n_batches
 * of `actions` ([n_batches][N][action_dim], or [n_batches][action_dim][N] planes with
 * RR_FLAG_ACTION_SOA) — open-loop action sequences already resident on the device (e.g. a
 * benchmark or a replayed plan) without one host call per step. Outputs as rr_step, of the
 * last step. */
int rr_step_repeat(rr_env* e, const float* actions, int64_t n_batches, int64_t n_steps, float* obs, float* reward,
                   uint8_t* done, uint8_t* truncated, float* terms, void* stream);
/* Overwrite / read the per-env state (parity injection, checkpoint / restore).
 * state_soa [state_dim][N] fp32; v0 [N] or NULL (kept on set / skipped on get);
 * elapsed [N] or NULL is the per-env counter word: TimeLimit steps in bits 0..E-1, episodes
 * started in bits E..31 (keys the reset stream), E = rr_counter_bits(e); a plain step count
 * below 2^E is a valid word (episode 0; larger counts would spill into the episode field: the
 * Python layer rejects them). On set, NULL clears the steps and keeps the episode field. The
 * elapsed field saturates at 2^E - 1 (>= max_episode_steps): an env stepped on past its
 * TimeLimit without a reset keeps reporting done / truncated; its Monitor length and, under
 * RR_INT_DOPRI5, its clock t = steps * dt stop there.
 * rr_set_state* zero the Monitor running return (an injected state starts a new segment);
 * rr_get_aux / rr_set_aux round-trip the raw counter words and the running return for a
 * checkpoint. */
int rr_set_state(rr_env* e, const float* state_soa, const float* v0, const int32_t* elapsed, void* stream);
int rr_get_state(rr_env* e, float* state_soa, float* v0, int32_t* elapsed, void* stream);
/* Same with an fp64 state [state_dim][N]. Under RR_INT_DOPRI5 this is the state the
 * integrator carries (the reference's float64 SIM.state); otherwise it is converted
 * to / from the fp32 planes. In DOPRI5 mode elapsed also sets the clock: t = steps*dt. */
int rr_set_state64(rr_env* e, const double* state_soa, const float* v0, const int32_t* elapsed, void* stream);
int rr_get_state64(rr_env* e, double* state_soa, float* v0, int32_t* elapsed, void* stream);
/* Bits E of the elapsed-steps field of the counter word (16 without a TimeLimit). */
int rr_counter_bits(const rr_env* e);
/* Raw counter words [N] and Monitor running returns [N] (either may be NULL). */
int rr_get_aux(rr_env* e, uint32_t* counter, float* ep_return, void* stream);
int rr_set_aux(rr_env* e, const uint32_t* counter, const float* ep_return, void* stream);

/* Pointers to the library-owned buffers (done list of the last step, etc.). */
int rr_get_buffers(rr_env* e, rr_buffers* out);

/* Pinned, GPU-coherent (fine-grained) host memory that the kernels read and write directly:
 * zero-copy step inputs / outputs for small N (the single-env gym shims pass the action and
 * every output of rr_step in it, so a step needs no copy command). Host-only, synchronous;
 * free with rr_host_free. */
int rr_host_alloc(void** out, int64_t bytes);
int rr_host_free(void* p);

/* Host-side retrieval of the last step's done list (SB3 infos: terminal_observation,
 * Monitor episode stats). SYNCHRONISES `stream`. Writes at most `capacity` rows into
 * the HOST arrays (any may be NULL): idx [capacity], term_obs [capacity][state_dim],
 * term_return [capacity], term_len [capacity]; rows are in ascending env order.
 * Returns the number of done envs (>= 0) or an RR_E* code. */
int64_t rr_fetch_done(rr_env* e, int64_t capacity, int32_t* idx, float* term_obs, float* term_return,
                      int32_t* term_len, void* stream);

/* rr_fetch_done for caller-owned per-step snapshots (SB3 infos of a device-output vec env, built
 * after later steps have run): the env indices where done[i] != 0 ([N] u8, device), ascending,
 * and their rows of the given sources — term_obs_src [N][state_dim] f32, term_return_src [N] f32,
 * term_len_src [N] i32, truncated_src [N] u8 (device; e.g. the rows rr_copy_terminal wrote) — into
 * the host arrays idx / term_obs / term_return / term_len / truncated (at most `capacity` rows,
 * any may be NULL; an output needs its source). SYNCHRONISES `stream`. Returns the number of done
 * envs or an RR_E* code. */
int64_t rr_gather_rows(rr_env* e, const uint8_t* done, const float* term_obs_src, const float* term_return_src,
                       const int32_t* term_len_src, const uint8_t* truncated_src, int64_t capacity, int32_t* idx,
                       float* term_obs, float* term_return, int32_t* term_len, uint8_t* truncated, void* stream);

/* Device-to-device copy of the terminal rows of the envs done at the last step (their final
 * obs row [state_dim], episode return, episode length) into the same rows of the caller's
 * [N][state_dim] / [N] / [N] buffers; rows of envs not done are left untouched. Any destination
 * may be NULL. One kernel that reads the last step's done masks. Asynchronous. */
int rr_copy_terminal(rr_env* e, float* term_obs, float* term_return, int32_t* term_len, void* stream);

/* ---- On-device PPO rollouts (BASELINE configs[4]) ----
 * Replace the per-step host work of stable_baselines3 1.6 OnPolicyAlgorithm.collect_rollouts
 * + RolloutBuffer (the reference trains PPO("MlpPolicy", ...), main_6DOF.py:62-69) for
 * an on-device rollout: the MlpPolicy actor-critic (separate pi / vf towers, net_arch
 * [64, 64], tanh, state-independent log_std) runs as one fp32 MFMA launch per step.
 * Supported (obs_dim, act_dim): (14, 3) 6DOF, (7, 2) 3DOF.
 * precision: RR_POLICY_FP32 (default; v_mfma_f32_32x32x2_f32, exact fp32 products. The pack
 * holds the tanh FOLDED into the weights: tanh(x) = 1 - 2 r, r = 1 / (1 + 2^(2 x log2 e)), with
 * W1' = c W1, b1' = c b1, W2' = -2c W2, b2' = c (b2 + row sums of W2), heads W' = -2 W and
 * b' = b + row sums of W (c = 2 log2 e; each folded value computed in fp64 and rounded once to
 * fp32), so a hidden unit is v_exp_f32 + add + v_rcp_f32. The SB3 policy's numbers to a few fp32
 * ulps of each weight and hidden unit: values / means within ~1e-5 of the fp32 MlpPolicy
 * (tests/test_gpu_rollout.py). The PPO learner (rr_ppo_grad) packs and runs the UNfolded tanh,
 * so the rollout's log_prob / value and the learner's recomputation on the same parameters agree
 * to rounding, not bit for bit: at epoch 0 the ratio is 1 and approx_kl 0 only to ~1e-6 / ~1e-12
 * (tests/test_gpu_ppo.py::test_rollout_and_learner_forwards_agree)) or RR_POLICY_BF16 (opt-in; v_mfma_f32_32x32x16_bf16
 * with fp32 accumulation: obs, the tower weights and the first hidden layer rounded to
 * bf16, everything else fp32) or RR_POLICY_FP16X3 (v_mfma_f32_32x32x16_f16 on operands split
 * into two fp16 halves, three MFMAs per k step: ~2^-21 relative products, fp32-level
 * results at ~5x the fp32 MFMA rate). A packed buffer is specific to its precision. */
#define RR_POLICY_FP32 0
#define RR_POLICY_BF16 1
#define RR_POLICY_FP16X3 2

/* Packed parameter buffer for rr_policy_*: returns its size in floats (or RR_EINVAL) and,
 * if off != NULL, the 12 section offsets {L1A, B1, L2A, B2, TOWER, PI, VF, HA, HV, HB, VB,
 * LS} (fragment-ordered layout, rl_rocket_amd/csrc/rocket_policy.inc; filled on the device
 * by rl_rocket_amd.rollout.pack_policy). Host-only. */
int rr_policy_layout(int obs_dim, int act_dim, int precision, int64_t* off);

/* Fill the packed buffer (device, rr_policy_layout floats) from the 13 device fp32 tensors
 * of the actor-critic in PyTorch nn.Linear layouts ([out][in] row-major), src[] being a
 * HOST array of device pointers: pi {W1 [64][obs], b1, W2 [64][64], b2}, vf {W1, b1, W2,
 * b2}, W_action [act][64], b_action, W_value [1][64], b_value, log_std [act]. One launch. */
int rr_policy_pack(int obs_dim, int act_dim, int precision, const float* const* src, float* params, void* stream);

/* One rollout step's policy work (SB3 ActorCriticPolicy.forward + clip, plus the previous
 * step's bookkeeping of collect_rollouts) in one launch:
 *   obs [n][obs_dim] -> action_env [n][act_dim] (clip to [-1, 1], the rr_step input),
 *   action [n][act_dim] (unclipped sample), value [n], log_prob [n], obs_copy [n][obs_dim]
 *   (or NULL; the rollout buffer's obs[t]). The normal draws are counter-based on
 *   (seed, env_id_offset + i, *iter, t): `iter` is a device uint64 the caller advances once
 *   per rollout, so graph replays draw new noise. params 16-B aligned.
 *   If reward_out != NULL: reward_out[i] = prev_reward[i] + gamma * V(prev_term_obs[i])
 *   where prev_truncated[i] (the timeout bootstrap of step t-1; rr_step's outputs and
 *   rr_get_buffers' terminal_obs). If start_out != NULL: start_out[i] = done[i] (episode
 *   start flags of step t). */
int rr_policy_act(const float* params, int obs_dim, int act_dim, int precision, int64_t n, int64_t env_id_offset,
                  const float* obs, uint64_t seed, const uint64_t* iter, int t, float* action_env, float* action,
                  float* value, float* log_prob, float* obs_copy, const float* prev_term_obs,
                  const uint8_t* prev_truncated, const float* prev_reward, float gamma, float* reward_out,
                  const uint8_t* done, float* start_out, void* stream);

/* End of a rollout: reward_out[i] = reward[i] + gamma * V(term_obs[i]) where truncated[i]
 * (TimeLimit.truncated), else reward[i] (skipped when term_obs == NULL); and, if
 * value_out != NULL, value_out[i] = V(obs[i]). */
int rr_policy_bootstrap(const float* params, int obs_dim, int act_dim, int precision, int64_t n,
                        const float* term_obs, const uint8_t* truncated, const float* reward, float gamma,
                        float* reward_out, const float* obs, float* value_out, void* stream);

/* One rollout step in ONE launch: rr_policy_act (without its previous-step bookkeeping) and
 * rr_step fused. For every env i of e: obs = state * normalizer^-1 (the obs rr_step /
 * rr_reset last produced) -> buf_obs [n][obs_dim]; a ~ N(mean, exp(log_std)) with the noise
 * key of rr_policy_act (seed, env id, *iter, t) -> buf_action [n][act_dim] (unclipped),
 * buf_value, buf_log_prob; the env steps with clip(a, -1, 1) (auto-reset, TimeLimit, terminal
 * rows as rr_step); buf_reward[i] = reward + gamma * V(terminal obs) where truncated;
 * buf_start[i] = done[i] as passed in (the previous step's done flags, updated in place to
 * this step's). reward / done (required), truncated / terms (optional) are rr_step's env
 * outputs; obs (optional, NULL to skip) receives the post-step obs. Bitwise the same results
 * as rr_policy_act + rr_step. RK4 / Euler envs (not RR_INT_DOPRI5). */
int rr_rollout_step(rr_env* e, const float* params, int precision, uint64_t seed, const uint64_t* iter, int t,
                    float gamma, float* buf_obs, float* buf_action, float* buf_value, float* buf_log_prob,
                    float* buf_start, float* buf_reward, float* obs, float* reward, uint8_t* done, uint8_t* truncated,
                    float* terms, void* stream);

/* A whole PPO rollout in ONE launch (replaces SB3 OnPolicyAlgorithm.collect_rollouts +
 * RolloutBuffer.compute_returns_and_advantage, stable_baselines3 1.6 on_policy_algorithm.py /
 * buffers.py, driving the reference's env through main_6DOF.py:60-103). Steps t = 0..n_steps-1
 * are exactly rr_rollout_step(t) — same noise key (seed, env id, *iter, t), same env step,
 * bootstrap and buffer writes, now into the [t] slices of [n_steps][n] buffers — with the env
 * state kept in registers between steps; then last_value[i] = V(post-step obs) (as
 * rr_policy_bootstrap), last_done[i] = last_start[i] = float(done[i]) and, when
 * buf_advantage / buf_return are given, the GAE scan of rr_gae(gamma, gae_lambda). Env outputs
 * (obs, reward, done, truncated, terms) are those of the last step. last_* / obs / truncated /
 * terms may be NULL. Bitwise the same results as n_steps rr_rollout_step launches +
 * rr_policy_bootstrap + rr_gae. RK4 / Euler envs. */
int rr_rollout_collect(rr_env* e, const float* params, int precision, uint64_t seed, const uint64_t* iter,
                       int n_steps, float gamma, float gae_lambda, float* buf_obs, float* buf_action,
                       float* buf_value, float* buf_log_prob, float* buf_start, float* buf_reward,
                       float* buf_advantage, float* buf_return, float* last_value, float* last_done,
                       float* last_start, float* obs, float* reward, uint8_t* done, uint8_t* truncated, float* terms,
                       void* stream);

/* RolloutBuffer.compute_returns_and_advantage: rewards / values / starts [T][n] (starts[t]
 * = episode-start flag of step t), last_value / last_done [n] -> advantages, returns [T][n]. */
int rr_gae(int64_t T, int64_t n, const float* rewards, const float* values, const float* starts,
           const float* last_value, const float* last_done, float gamma, float lam, float* advantages,
           float* returns, void* stream);

/* ---- PPO minibatch gradient (the learner half of configs[4]) ----
 * Replaces the loss + loss.backward() of stable_baselines3 1.6 PPO.train for the MlpPolicy
 * actor-critic the reference trains (PPO("MlpPolicy", env, ..., ent_coef=0.01),
 * main_6DOF.py:62-69; SB3 defaults otherwise): for the minibatch idx[0 .. batch) of a device
 * rollout (obs [*][obs_dim], actions [*][act_dim], old_log_prob, advantages, returns [*]),
 *   A = (adv - mean) / (std + 1e-8) (unbiased std), r = exp(log_prob - old_log_prob),
 *   loss = -mean(min(A r, A clamp(r, 1 - clip_range, 1 + clip_range)))
 *          + ent_coef * -sum(0.5 + 0.5 log(2 pi) + log_std) + vf_coef * mean((returns - V)^2),
 * the gradient of loss with respect to the 13 parameter tensors (params / grads: HOST arrays of
 * device fp32 pointers in rr_policy_pack's order and PyTorch layouts) is WRITTEN to grads (not
 * accumulated). stats (device, 5 floats, or NULL): policy_loss, value_loss, entropy,
 * clip_fraction, approx_kl (SB3's logged quantities). Deterministic (fixed-order sums, no
 * atomics); fp32 MFMA, so the gradients equal PyTorch's autograd ones to fp32 summation-order
 * rounding. Three launches on `stream`, capturable in a graph. Supported (obs_dim, act_dim):
 * (14, 3), (7, 2); batch >= 2. workspace: device, 16-B aligned, rr_ppo_workspace_size bytes. */
int rr_ppo_workspace_size(int obs_dim, int act_dim, int64_t batch, int64_t* bytes);
int rr_ppo_grad(int obs_dim, int act_dim, const float* const* params, float* const* grads, const float* obs,
                const float* actions, const float* old_log_prob, const float* advantages, const float* returns,
                const int64_t* idx, int64_t batch, float clip_range, float ent_coef, float vf_coef, float* stats,
                void* workspace, int64_t workspace_bytes, void* stream);

/* torch.nn.utils.clip_grad_norm_(max_grad_norm) + one torch.optim.Adam(capturable=True) step
 * (weight_decay 0, no amsgrad / maximize) over n_tensors (<= 16) fp32 device tensors, in two
 * launches: the rest of SB3 PPO.train's minibatch step after rr_ppo_grad. grads are scaled in
 * place by min(1, max_grad_norm / (||grads|| + 1e-6)) (no clip when max_grad_norm <= 0);
 * exp_avg / exp_avg_sq / step are the optimizer's state tensors (optimizer.state[p]: "exp_avg",
 * "exp_avg_sq", and the device float "step", incremented), updated in place with PyTorch's
 * capturable multi-tensor formulas; lr is a DEVICE float, read at run time (a learning-rate
 * schedule can change it between graph replays). Arrays are host arrays of device pointers;
 * numel[] host. workspace: device, rr_clip_adam_workspace_size(sum of numel) bytes. */
int rr_clip_adam_workspace_size(int64_t total_elements, int64_t* bytes);
int rr_clip_adam(int n_tensors, float* const* params, float* const* grads, float* const* exp_avg,
                 float* const* exp_avg_sq, float* const* step, const int64_t* numel, float max_grad_norm,
                 const float* lr, double beta1, double beta2, float eps, void* workspace, int64_t workspace_bytes,
                 void* stream);

/* One whole PPO minibatch step: rr_ppo_grad followed by rr_clip_adam over the same 13 tensors
 * (rr_ppo_grad's order; exp_avg / exp_avg_sq / step as rr_clip_adam's), replacing SB3 1.6
 * PPO.train's loss.backward(), clip_grad_norm_ and optimizer.step() for one minibatch
 * (main_6DOF.py:62-69) without a multi-GPU all_reduce between them. It takes three launches
 * where the two calls take five:
 *   - the gradient finish also sums the squared gradients for the clip;
 *   - the optimizer step also refreshes the packed tower images of the gradient launch;
 *   - with next_idx (next_batch rows, 2 <= next_batch <= batch) the optimizer launch also sums
 *     the NEXT minibatch's advantage statistics.
 * A call with flags & RR_PPO_CHAINED skips the packing / statistics launch and uses what the
 * previous rr_ppo_update on the same workspace left there. That previous call must have been
 * given next_idx = this idx, next_batch = this batch, and nothing else may have written the
 * parameters since. Without the flag the call packs from the parameters itself (four launches).
 * Arithmetic as the two calls, except that the clip's norm sums the squares in the finish's
 * order. workspace: device, 16-B aligned, rr_ppo_update_workspace_size bytes; lr a device float. */
#define RR_PPO_CHAINED 0x1u
int rr_ppo_update_workspace_size(int obs_dim, int act_dim, int64_t batch, int64_t* bytes);
int rr_ppo_update(int obs_dim, int act_dim, float* const* params, float* const* grads, float* const* exp_avg,
                  float* const* exp_avg_sq, float* const* step, const float* obs, const float* actions,
                  const float* old_log_prob, const float* advantages, const float* returns, const int64_t* idx,
                  int64_t batch, const int64_t* next_idx, int64_t next_batch, float clip_range, float ent_coef,
                  float vf_coef, float max_grad_norm, const float* lr, double beta1, double beta2, float eps,
                  float* stats, uint32_t flags, void* workspace, int64_t workspace_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif
