/*
 * lorenz_env.h -- C-ABI of the MI355X-native vectorised chaotic-ODE env library
 *                 (libgym_lorenz_amd.so).
 *
 * The reference (erererq/gym-lorenz) is pure Python: every env is a gym/gymnasium
 * `Env` whose reset()/step() run scalar NumPy on 3-8 element arrays, one env per
 * object, driven one step at a time by stable-baselines3's DummyVecEnv.  This
 * library replaces exactly that hot path -- the env batch's reset()/step() -- with
 * one HIP kernel launch per batched step, one env per GPU lane.  The Python package
 * `gym_lorenz` (gym-lorenz_amd/gym_lorenz) binds it through ctypes and keeps the
 * reference's per-env classes, ids and SB3 VecEnv surface.
 *
 * Entry point  ->  reference interface it replaces
 *   lz_create / lz_config_init
 *       -> the env constructors: dynamic.py:8-33 (lorenzEnv_transient, 3-state),
 *          lorenz_env_transient.py:253-273 (lorenzEnv_transient, 4-state),
 *          lorenz_env_try_pmsm.py:9-50 (PMSM_Sync_Env),
 *          lorenz_env_try.py:19-48 (HRSyncEnv); plus gym_lorenz/__init__.py:4-23
 *          (registration kwargs max_episode_steps -> max_episode_steps)
 *   lz_reset
 *       -> reset(): dynamic.py:35-47, lorenz_env_transient.py:275-297,
 *          lorenz_env_try_pmsm.py:59-75, lorenz_env_try.py:49-78
 *   lz_step
 *       -> step(action): dynamic.py:61-90, lorenz_env_transient.py:314-373,
 *          lorenz_env_try_pmsm.py:76-184, lorenz_env_try.py:80-179, batched over
 *          the env axis with SB3 DummyVecEnv.step_wait auto-reset semantics
 *          (terminal observation kept, post-reset observation returned)
 *   lz_step_host / lz_resident_step
 *       -> ONE env's step(action) from host memory, the per-env classes'
 *          DummyVecEnv([lambda: gymnasium.make(id)]) path (code/train.py:98-100);
 *          lz_resident_step serves it from a resident kernel (no launch per step)
 *   lz_rollout
 *       -> K consecutive step() calls fused in one launch (state kept in VGPRs)
 *   (legacy, unregistered: lorenz_env_transient1.py:18-104,
 *    lorenz_env_transient2.py:115-240, lorenz_env_transient_pmsm.py:17-133,
 *    lorenz_singlecontrol.py:97-172 -- LZ_SYS_T1 / T2 / TP / SC)
 *   lz_step_vecnorm / lz_vecnorm_apply
 *       -> VecNormalize(DummyVecEnv(...)).step() as the PMSM callers wrap the env
 *          (code/lorenz_pmsm/train.py:118,170, optimize.py:52; SB3 2.7.1
 *          common/vec_env/vec_normalize.py): step + statistics + normalisation
 *   lz_get_state / lz_set_state
 *       -> attribute access env.state1 / state2 / state_master / state_slave /
 *          lambda_coef ... used by code/lorenz_pmsm/test_evaluate.py:99-111
 *   lz_policy_pack_f32 / lz_rollout_policy_f32 / lz_policy_pack[_hidden] /
 *   lz_rollout_policy / lz_gae / lz_episode_starts
 *       -> SB3 OnPolicyAlgorithm.collect_rollouts + RolloutBuffer.compute_returns_and_
 *          advantage for the MlpPolicy learners (code/lorenz_pmsm/train.py:155-178,
 *          optimize.py:36-60 ([64,64] / [128,128]), code/gym_run.py:83 (PPO default
 *          net_arch [64,64]))
 *   lz_attn_policy_pack / lz_rollout_policy_attn
 *       -> the same for code/train.py:52-112 and code/gym_try.py:52-116 (PPO with the
 *          AttentionFeaturesExtractor)
 *   lz_attn_ln_policy_pack / lz_rollout_policy_attn_stack
 *       -> the same for code/lorenz_filter/train.py:54-132 (VecFrameStack(4) + the
 *          residual/LayerNorm extractor)
 *   lz_frame_stack
 *       -> SB3 VecFrameStack.step_wait (code/lorenz_filter/train.py:115)
 *
 * Conventions
 *   - Every function returns an lz_status (0 == LZ_OK).  Nothing throws across
 *     the ABI; lz_last_error() returns a thread-local message for the last failure.
 *   - All buffer pointers are DEVICE pointers on the handle's device (hipMalloc or
 *     torch CUDA tensors), contiguous, row-major.  "T" below is float for
 *     LZ_DTYPE_F32 handles and double for LZ_DTYPE_F64 handles.
 *   - A handle is bound to one device and one HIP stream and is not re-entrant.
 *     Calls are asynchronous on that stream; lz_sync() waits for it.
 *   - Non-finite states are not errors: they reproduce the reference's IEEE
 *     behaviour (overflow to inf/NaN is silently allowed there too).
 *   - hipGraph capture: lz_reset / lz_step / lz_rollout enqueue kernels (and, for
 *     n_done_out, one D2D copy) only -- no allocation, no host sync -- and keep their
 *     RNG call counter and compact-list cursor in device memory (2-slot ping-pong
 *     selected by a host-side call parity).  A captured sequence must therefore hold
 *     an EVEN number of these calls so that every replay starts on the same slot.
 */
#ifndef LORENZ_ENV_H
#define LORENZ_ENV_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: lz_get_state / lz_set_state take (indices, count); lz_config.integrator */
#define LZ_ABI_VERSION 2

typedef enum lz_status {
  LZ_OK = 0,
  LZ_ERR_INVALID = 1,     /* bad argument / config */
  LZ_ERR_UNSUPPORTED = 2, /* combination not supported (e.g. PMSM in fp64) */
  LZ_ERR_HIP = 3,         /* HIP runtime error (message has hipGetErrorString) */
  LZ_ERR_STATE = 4,       /* call order violated (step before the first reset) */
  LZ_ERR_OOM = 5
} lz_status;

typedef enum lz_system {
  LZ_SYS_LORENZ3 = 0, /* dynamic.py: 3-state Lorenz, Euler dt=0.01, additive action */
  LZ_SYS_LORENZ4 = 1, /* lorenz_env_transient.py: 4-state master/slave, dt=0.001 */
  LZ_SYS_PMSM = 2,    /* lorenz_env_try_pmsm.py: PMSM sync, fp32, Adam dual lambda */
  LZ_SYS_HR = 3,      /* lorenz_env_try.py: Hindmarsh-Rose master/slave, RK4 */
  /* legacy, unregistered variants (fp64 in the reference) */
  LZ_SYS_T1 = 4,      /* lorenz_env_transient1.py: one PMSM-form system, additive actions */
  LZ_SYS_T2 = 5,      /* lorenz_env_transient2.py: 4-state master/slave, dt=0.001 */
  LZ_SYS_TP = 6,      /* lorenz_env_transient_pmsm.py: PMSM-form master/slave + noise */
  LZ_SYS_SC = 7       /* lorenz_singlecontrol.py: fixed start, noise only, no action */
} lz_system;

typedef enum lz_dtype { LZ_DTYPE_F32 = 0, LZ_DTYPE_F64 = 1 } lz_dtype;

/* lz_config.integrator.  LZ_INT_EULER is the reference's own integrator for every
 * system (dynamic.py:70-75 forward Euler; HR is RK4 by definition, lorenz_env_try.py:
 * 100-113, whatever this field says).  LZ_INT_RK4 is an opt-in mode of LORENZ3 and
 * LORENZ4 (BASELINE north_star "the dynamic.py RK4 integrator ... RK4 substages in
 * registers"): the classical four-stage step of HRSyncEnv's stage order (k1 = f(s),
 * k2 = f(s + dt/2 k1), k3 = f(s + dt/2 k2), k4 = f(s + dt k3),
 * s += (dt/6.0) (((k1 + 2 k2) + 2 k3) + k4)) applied to the system's own RHS, then the
 * additive action of dynamic.py:73-75 (LORENZ3).  The reference has no RK4 Lorenz, so
 * this mode is pinned to the build's own CPU restatement only ("parity unpinned"). */
typedef enum lz_integrator { LZ_INT_EULER = 0, LZ_INT_RK4 = 1 } lz_integrator;

/* State planes (SoA, one T or int32 element per env) addressable by
 * lz_get_state / lz_set_state.  Reference attribute in brackets. */
enum {
  /* LZ_SYS_LORENZ3 [state1 = x,y,z] */
  LZ_L3_X = 0, LZ_L3_Y = 1, LZ_L3_Z = 2, LZ_L3_STEP = 3,
  /* LZ_SYS_LORENZ4 [state1 = master x1..x4, state2 = slave x1..x4] */
  LZ_L4_M1 = 0, LZ_L4_S1 = 4, LZ_L4_STEP = 8,
  /* LZ_SYS_PMSM [state1 (3), state2 (3), lambda_coef, m_t, v_t: float32;
   *              adam_step, current_step: int32] */
  LZ_PMSM_S1 = 0, LZ_PMSM_S2 = 3, LZ_PMSM_LAMBDA = 6, LZ_PMSM_M = 7, LZ_PMSM_V = 8,
  LZ_PMSM_ADAM_STEP = 9, LZ_PMSM_STEP = 10,
  /* LZ_SYS_HR [state_master (3), state_slave (3), sigma: T;
   *            filtered_action (2): float32; step: int32] */
  LZ_HR_M = 0, LZ_HR_S = 3, LZ_HR_SIGMA = 6, LZ_HR_FA = 7, LZ_HR_STEP = 9,
  /* legacy: LZ_SYS_T1 [state1 = x,y,z]; LZ_SYS_T2 [state1 (4), state2 (4)];
   * LZ_SYS_TP [state1 (3), state2 (3)]; LZ_SYS_SC [state1 = x,y,z]  (all T) */
  LZ_T1_X = 0, LZ_T1_STEP = 3,
  LZ_T2_M1 = 0, LZ_T2_S1 = 4, LZ_T2_STEP = 8,
  LZ_TP_M = 0, LZ_TP_S = 3, LZ_TP_STEP = 6,
  LZ_SC_X = 0, LZ_SC_STEP = 3
};

/* done byte written per env by lz_step / lz_rollout */
#define LZ_DONE_TERMINATED 1u /* the env's own termination condition */
#define LZ_DONE_TRUNCATED 2u  /* max_episode_steps (gymnasium TimeLimit) or PMSM's own
                                 current_step >= max_steps */

/* lz_config.flags */
#define LZ_FLAG_AUTORESET 1u   /* reset done envs inside lz_step (SB3 VecEnv semantics) */
#define LZ_FLAG_ADD_NOISE 2u   /* PMSM / HR ctor kwarg add_noise */
#define LZ_FLAG_EVAL_MODE 4u   /* HR ctor kwarg eval_mode (sigma = 2.0 on reset) */
#define LZ_FLAG_ADD_FILTER 8u  /* HR ctor kwarg add_filter */

#define LZ_MAX_PARAMS 16

typedef struct lz_config {
  int32_t system;            /* lz_system */
  int32_t dtype;             /* lz_dtype; PMSM is float32 only (as the reference) */
  int64_t num_envs;          /* envs owned by this handle (this rank's shard) */
  int64_t global_env_offset; /* first global env id of the shard: keys the RNG, so
                                trajectories do not depend on the GPU count */
  uint64_t seed;             /* Philox key for on-device reset / noise draws */
  int32_t device;            /* HIP device ordinal */
  int32_t max_episode_steps; /* TimeLimit truncation; 0 = none */
  uint32_t flags;            /* LZ_FLAG_* */
  float alpha;               /* PMSM fractional-reward exponent (ctor kwarg alpha) */
  /* System constants, filled with the reference values by lz_config_init:
   *  LORENZ3: sigma, rho, beta, dt, action clip            (dynamic.py:31-33,73-75,63-65)
   *  LORENZ4: a, b, c, dt, action clip, T_end              (lorenz_env_transient.py:270-273,327-330)
   *  PMSM:    sigma, gamma, dt, f_max, lambda_lr, beta1, beta2, eps, err_threshold,
   *           max_steps, term_threshold                    (lorenz_env_try_pmsm.py:12-50)
   *  HR:      a, b, c, d, r, s, I_bias, x_rest, dt, scale, master_scale,
   *           action_alpha, term_threshold                 (lorenz_env_try.py:32-40)
   *  T1:      a, b, -, dt, action clip, T_end              (lorenz_env_transient1.py:21-39)
   *  T2:      a, b, c, dt, action clip, T_end, d, h, action gain, x4 damping
   *                                                        (lorenz_env_transient2.py:118-137)
   *  TP:      a, b, action gain, dt, action clip, T_end, noise std
   *                                                        (lorenz_env_transient_pmsm.py:22-41)
   *  SC:      a, b, -, dt, action clip, T_end, noise std, x0, y0, z0
   *                                                        (lorenz_singlecontrol.py:100-121)
   * lz_config_init sets LZ_FLAG_ADD_NOISE for TP and SC (their noise is unconditional). */
  double params[LZ_MAX_PARAMS];
  /* LORENZ3/4 'done = (t == T)' on a float accumulator (dynamic.py:85-89): the host
   * replays the accumulator; the step index where it fires (-1 = never, which is the
   * case for the reference constants) is stored here by lz_create. Read-only. */
  int32_t t_done_step;
  int32_t reserved[6];       /* reserved[0]: kernel tuning variant (A/B experiments) */
  int32_t integrator;        /* lz_integrator (LZ_INT_EULER = the reference, default) */
} lz_config;

typedef struct lz_info {
  int32_t state_dim;   /* T elements of dynamical state per env */
  int32_t action_dim;  /* actions per env (T elements) */
  int32_t obs_dim;     /* observation T elements per env */
  int32_t init_dim;    /* T elements per env of lz_reset's `init` vector */
  int32_t n_planes;    /* SoA planes addressable by lz_get_state/lz_set_state */
  int32_t bytes_per_env_step; /* algorithmic HBM bytes of one lz_step per env */
  int32_t counts_steps;       /* 1 if the STEP plane is maintained by lz_step */
  int32_t state_io_bytes;     /* of bytes_per_env_step: state planes read + written
                                 (paid once per launch by lz_rollout, not per step) */
} lz_info;

/* Fill *cfg with the reference defaults of `system` (dtype f32, 1 env, seed 0). */
lz_status lz_config_init(lz_config* cfg, int32_t system);

typedef struct lz_handle lz_handle;

lz_status lz_create(const lz_config* cfg, lz_handle** out);
lz_status lz_destroy(lz_handle* h);
lz_status lz_get_info(const lz_handle* h, lz_info* info);
lz_status lz_get_config(const lz_handle* h, lz_config* cfg);

/* Change the Philox key used by subsequent on-device resets / noise draws
 * (SB3 VecEnv.seed()) and rewind the device call counter to 0 (stream-ordered), so
 * that seed(s) followed by reset() draws the same initial states whatever calls came
 * before -- SB3 / gymnasium seed-then-reset reproducibility. */
lz_status lz_set_seed(lz_handle* h, uint64_t seed);

/* Bind the handle to a HIP stream (hipStream_t passed as void*; NULL = default). */
lz_status lz_set_stream(lz_handle* h, void* hip_stream);
lz_status lz_sync(lz_handle* h);

/* Reset the envs selected by `mask` (uint8 [N], NULL = all).
 * init: NULL -> draw initial states on device (Philox keyed by (seed, global env
 *       id, call counter)), with the reference distributions;
 *       else T [N, init_dim] initial states to inject (parity tests, per-env drop-in
 *       classes replaying the reference's host RNG):
 *         LORENZ3 [x,y,z]; LORENZ4 [master(4), slave(4)]; PMSM [state1(3), state2(3)];
 *         HR [master(3), slave(3), sigma].
 * obs_out: T [N, obs_dim] (rows of unselected envs untouched) or NULL. */
lz_status lz_reset(lz_handle* h, const uint8_t* mask, const void* init, void* obs_out);

/* One batched step of every env.
 *   actions   T [N, action_dim]
 *   noise     double [N, 3] injected process noise (PMSM: the N(0,3) draw of
 *             lorenz_env_try_pmsm.py:80, used iff LZ_FLAG_ADD_NOISE; HR: the
 *             N(0,sigma) draw of lorenz_env_try.py:136) or NULL = on-device Philox
 *   obs_out   T [N, obs_dim]   (post-reset obs for envs auto-reset this step)
 *   rew_out   T [N]
 *   done_out  uint8 [N]        LZ_DONE_* bits
 *   done_idx_out      int32 [N] or NULL: compact list of env indices done this step
 *   terminal_obs_out  T [N, obs_dim] or NULL: their pre-reset observations
 *   n_done_out        int32 [1] (device) or NULL: number of entries written
 * Entries of the compact list are in unspecified order. */
lz_status lz_step(lz_handle* h, const void* actions, const double* noise, void* obs_out,
                  void* rew_out, uint8_t* done_out, int32_t* done_idx_out,
                  void* terminal_obs_out, int32_t* n_done_out);

/* One step of a small handle from / to HOST memory, synchronous: actions (float32
 * [N, A]) and optional injected noise (double [N, 3]) are copied into the handle's
 * host staging buffer, which is mapped into the device address space (hipHostMalloc
 * mapped + coherent), lz_step reads them and writes obs | reward | done there over
 * PCIe (no copy launches), the stream is synchronised and the outputs copied out.  The per-env drop-in classes use it -- one call per
 * env.step() of a reference caller that keeps DummyVecEnv([lambda: gymnasium.make(..)])
 * (code/train.py:98-100).  The handle's first call allocates the staging buffers. */
lz_status lz_step_host(lz_handle* h, const float* actions, const double* noise, void* obs_out,
                       void* rew_out, uint8_t* done_out);

/* lz_step_host's contract (same arguments, same results bit for bit -- the same step
 * body, tick for tick) served by a RESIDENT kernel: one launch per process and device
 * serves every handle that calls this (one wave per handle, up to 15 handles; a
 * DummyVecEnv of several drop-in envs -- code/train.py:98-100 -- shares the one launch
 * and its one stream), keeps each handle's state in registers; each call writes its
 * inputs into the handle's mailbox in mapped host memory, then the request number into
 * the handle's own 8-byte word of the server's command line (one 128-B line, one word
 * per member handle; -1 in ANY word stops every wave).  One poller wave reads the whole
 * line with one wave-wide load per poll and hands a changed word to the handle's wave
 * through LDS; the call spins until the reply lands in host memory -- no launch, no
 * stream synchronisation per step.  A
 * handle joining the server restarts it (its state goes back to the planes and every
 * handle is relaunched); a 16th handle steps through lz_step_host instead.  Handles of
 * at most 64 envs without LZ_FLAG_AUTORESET (LZ_ERR_UNSUPPORTED otherwise).  The server
 * exits after LZ_RESIDENT_IDLE_US (default 1000; read at every launch of the server)
 * microseconds without a request to ANY of its handles and is relaunched by the next call (a device-wide synchronize waits
 * for that exit); every other call on a served handle stops it first (all states go
 * back to the planes), as does lz_resident_stop.  Synchronous: LZ_ERR_STATE while the
 * handle's stream is being captured into a graph. */
lz_status lz_resident_step(lz_handle* h, const float* actions, const double* noise,
                           void* obs_out, void* rew_out, uint8_t* done_out);
lz_status lz_resident_stop(lz_handle* h);
/* Host copy of one state plane (N elements, lz_plane_elem_size bytes each) -- what the
 * per-env drop-in classes' state1 / state2 / state_master ... attributes return
 * (code/lorenz_pmsm/test_evaluate.py:123-125 reads them after every step).  While the
 * resident server serves the handle this is its published copy after the last request
 * (no device interaction, the server keeps running); otherwise the plane is copied from
 * the device (synchronous). */
lz_status lz_resident_read_state(lz_handle* h, int32_t plane, void* host_dst);

/* The byte sizes the caller buffers of lz_step (K = 0) or lz_rollout (K >= 1, done list of
 * `cap` entries) must each cover, for a config -- the raw pointers of those calls carry no
 * sizes, and a buffer shorter than this is written past its end on the device (DESIGN
 * §6.2.1: a LORENZ3 obs ring of [N, 3] for the [N, 6] observation).  Host-only, needs no
 * GPU and no handle; gym_lorenz.core.check_buffer applies the same sizes. */
typedef struct lz_io_sizes {
  int64_t actions;      /* float32 [N, A] / [K, N, A]; 0: the system reads none (LORENZ4, SC) */
  int64_t noise;        /* float64 [N, 3]: lz_step's optional injected noise (0 for K >= 1) */
  int64_t obs;          /* T [N, O] / [K, N, O] */
  int64_t rew;          /* T [N] / [K, N] */
  int64_t done;         /* uint8 [N] / [K, N] */
  int64_t done_idx;     /* int32 [N] (step) / int64 [cap] (rollout) */
  int64_t terminal_obs; /* T [N, O] (step) / T [cap, O] (rollout) */
  int64_t n_done;       /* int32 [1] */
} lz_io_sizes;
lz_status lz_io_sizes_for(const lz_config* cfg, int32_t K, int64_t cap, lz_io_sizes* out);

/* K fused steps in ONE launch, state held in registers.  Time-major buffers:
 *   actions T [K, N, action_dim]; obs_out T [K, N, obs_dim]; rew_out T [K, N];
 *   done_out uint8 [K, N]; done_idx_out int64 [cap] (k * N + env) and
 *   terminal_obs_out T [cap, obs_dim], cap entries at most (both NULL = skip);
 *   n_done_out int32 [1] or NULL.  Noise is drawn on device. */
lz_status lz_rollout(lz_handle* h, int32_t K, const void* actions, void* obs_out,
                     void* rew_out, uint8_t* done_out, int64_t* done_idx_out,
                     void* terminal_obs_out, int64_t cap, int32_t* n_done_out);

/* ------------------------------------------------------------------------------
 * Policy in the loop.  The reference's learners drive these envs with
 * stable-baselines3 A2C / PPO "MlpPolicy" actor-critics -- net_arch
 * dict(pi=[128, 128], vf=[128, 128]), activation Tanh, DiagGaussian actions
 * (code/lorenz_pmsm/train.py:155-178 A2C n_steps=16; code/lorenz_filter/train.py:
 * 117-127 and code/gym_try.py:106-116 PPO n_steps=2048, gae_lambda=0.95;
 * code/gym_run.py:79) -- stepping the env through DummyVecEnv one env at a time
 * (SB3 2.7.1 OnPolicyAlgorithm.collect_rollouts + RolloutBuffer).  lz_rollout_policy
 * fuses that whole collection loop into one launch: per step, the policy forward
 * (bf16 MFMA, fp32 accumulate), the Gaussian sample, the action-space clip, the env
 * step with auto-reset, and SB3's truncation bootstrap.  lz_gae is
 * RolloutBuffer.compute_returns_and_advantage.
 * ------------------------------------------------------------------------------ */
#define LZ_POLICY_HIDDEN 128
#define LZ_POLICY_DETERMINISTIC 1u /* action = mean (SB3 predict(deterministic=True)) */
#define LZ_POLICY_BOOTSTRAP 2u     /* reward += gamma * V(terminal obs) when truncated */
#define LZ_POLICY_I8X4 4u          /* the blob is an lz_*policy_pack_i8x4 blob (the float32
                                      attention / MlpPolicy rollouts; see there) */

/* Formats of the float32 / i8x4 policy blobs.  The packers below write a 16-byte format
 * tag into spare bytes of the blob; the float32 / i8x4 rollout kernels compare it with the
 * format their launch implies (entry point + LZ_POLICY_I8X4) and, on a mismatch, run on
 * an all-NaN copy of the blob: every output of the launch is NaN instead of a rollout on
 * misread weights (a float32 blob's bits read as int8 digits, or the reverse). */
enum {
  LZ_BLOB_UNKNOWN = 0,
  LZ_BLOB_MLP_F32 = 1,       /* lz_policy_pack_f32 */
  LZ_BLOB_MLP_I8X4 = 2,      /* lz_policy_pack_i8x4 */
  LZ_BLOB_ATTN_F32 = 3,      /* lz_attn_policy_pack_f32 */
  LZ_BLOB_ATTN_I8X4 = 4,     /* lz_attn_policy_pack_i8x4 */
  LZ_BLOB_ATTN_LN_F32 = 5,   /* lz_attn_ln_policy_pack_f32 */
  LZ_BLOB_ATTN_LN_I8X4 = 6   /* lz_attn_ln_policy_pack_i8x4 */
};
/* The LZ_BLOB_* format of a packed host blob of `size` bytes (LZ_BLOB_UNKNOWN: not a
 * tagged float32 / i8x4 blob, or too small).  Host-only; lets a C-ABI caller check a blob
 * against the flags it is about to launch with. */
int32_t lz_policy_blob_format(const void* host_blob, int64_t size);

/* Float32 weights in torch nn.Linear layout ([out, in], row-major), host memory.
 * Names are the SB3 ActorCriticPolicy state_dict keys. */
typedef struct lz_mlp_policy {
  int32_t obs_dim;     /* 1..8 */
  int32_t act_dim;     /* 1..4 */
  const float* pi_w1;  /* mlp_extractor.policy_net.0.weight [128, obs_dim] */
  const float* pi_b1;  /* mlp_extractor.policy_net.0.bias   [128] */
  const float* pi_w2;  /* mlp_extractor.policy_net.2.weight [128, 128] */
  const float* pi_b2;  /* mlp_extractor.policy_net.2.bias   [128] */
  const float* vf_w1;  /* mlp_extractor.value_net.0.weight  [128, obs_dim] */
  const float* vf_b1;
  const float* vf_w2;  /* mlp_extractor.value_net.2.weight  [128, 128] */
  const float* vf_b2;
  const float* act_w;  /* action_net.weight [act_dim, 128] */
  const float* act_b;  /* action_net.bias   [act_dim] */
  const float* val_w;  /* value_net.weight  [1, 128] */
  const float* val_b;  /* value_net.bias    [1] */
  const float* log_std; /* log_std [act_dim] */
} lz_mlp_policy;

/* Size of the packed policy blob (bf16 MFMA fragments + f32 biases). */
int64_t lz_policy_blob_bytes(void);
/* Pack *p into host_blob (host memory, cap >= lz_policy_blob_bytes()).  The caller
 * copies the blob to the device (e.g. torch.uint8 CUDA tensor) for lz_rollout_policy.
 * Host-only: needs no GPU. */
lz_status lz_policy_pack(const lz_mlp_policy* p, void* host_blob, int64_t cap);
/* lz_policy_pack for net_arch pi=[hidden, hidden] vf=[hidden, hidden], hidden 1..128
 * (code/lorenz_pmsm/optimize.py:36-41 searches 64 and 128): weights [hidden, obs_dim],
 * [hidden, hidden], [act_dim, hidden] ...; zero-padded to the kernel's 128 units, which
 * is exact (padded units are tanh(0) = 0 and carry zero weights). */
lz_status lz_policy_pack_hidden(const lz_mlp_policy* p, int32_t hidden, void* host_blob,
                                int64_t cap);

/* The same policy packed for SB3's own precision (float32 operands, float32
 * accumulation; stable-baselines3 runs these nets in torch float32, code/lorenz_pmsm/
 * train.py:173-178): f32-input MFMA hidden layers (bit-for-bit k-ordered fmaf chains),
 * fmaf-chain heads, tanh from IEEE basic operations -- deterministic and reproduced bit
 * for bit by the C oracle.  hidden 1..128 as lz_policy_pack_hidden.  Host-only. */
int64_t lz_policy_f32_blob_bytes(void);
lz_status lz_policy_pack_f32(const lz_mlp_policy* p, int32_t hidden, void* host_blob, int64_t cap);

typedef struct lz_policy_rollout_args {
  int32_t K;                /* steps (SB3 n_steps) */
  uint32_t flags;           /* LZ_POLICY_* */
  const void* blob;         /* device copy of the packed policy */
  const float* obs_in;      /* [N, O] raw obs the rollout starts from (SB3 _last_obs
                               before normalisation) */
  float* obs_last;          /* [N, O] raw obs after the K steps (may alias obs_in) */
  const double* obs_norm;   /* VecNormalize obs_rms [mean(O), var(O)] (double, device) or
                               NULL: the policy sees clip((o - mean)/sqrt(var + eps),
                               +-clip_obs), frozen for the K steps */
  double norm_eps, clip_obs;
  double gamma;             /* LZ_POLICY_BOOTSTRAP discount */
  float act_low, act_high;  /* action space Box bounds (np.clip before env.step) */
  float* obs_buf;           /* [K, N, O] observations the policy saw (normalised) */
  float* act_buf;           /* [K, N, A] sampled actions (unclipped, as SB3 stores) */
  float* logp_buf;          /* [K, N] log pi(a|s) */
  float* val_buf;           /* [K, N] V(s) */
  float* rew_buf;           /* [K, N] rewards (+ bootstrap) */
  uint8_t* done_buf;        /* [K, N] LZ_DONE_* bits of each step */
  float* last_values;       /* [N] V(normalised obs_last) */
  double* obs_moments;      /* device double [1 + 2*O]: (K*N, sums, sums of squares) of
                               the raw step outputs -- what VecNormalize's K per-step
                               obs_rms updates would see -- or NULL */
  int64_t* done_idx;        /* compact list k*N + env (cap entries) or NULL */
  float* terminal_obs;      /* [cap, O] raw pre-reset observations or NULL */
  int64_t cap;
  int32_t* n_done;          /* int32 [1] device or NULL */
} lz_policy_rollout_args;

/* K policy+env steps in one launch (float32 handles; env state and policy activations
 * in registers, weights in LDS).  The Gaussian sample is Philox keyed by (seed,
 * global env id, call counter + k), purpose 3.  The first call on a handle allocates
 * a small scratch buffer for obs_moments (do not capture that first call). */
lz_status lz_rollout_policy(lz_handle* h, const lz_policy_rollout_args* r);
/* lz_rollout_policy with an lz_policy_pack_f32 blob: the float32 MlpPolicy (replaces
 * SB3's ActorCriticPolicy.forward / predict in the same collect_rollouts loop and in
 * code/lorenz_pmsm/test_evaluate.py:117-120's deterministic closed loop). */
lz_status lz_rollout_policy_f32(lz_handle* h, const lz_policy_rollout_args* r);

/* The same collect under VecNormalize(training=True) in SB3's own order (SB3 2.7.1
 * VecNormalize.step_wait inside collect_rollouts; code/lorenz_pmsm/train.py:170-181
 * A2C n_steps=16 behind VecNormalize(norm_obs=True, norm_reward=False, clip_obs=10)):
 * step k's observation is normalised with obs_rms already updated by step k's whole
 * batch, and a truncated step's terminal observation (bootstrap value) with the
 * statistics that step produced.  One launch per step (the update is a reduction over
 * the batch between two steps) plus a closing launch:
 *   k = 0 .. K-1: [bootstrap of step k-1] normalise obs with obs_rms_state, policy,
 *                 sample, clip, env step (raw obs -> r->obs_last); then obs_rms_state
 *                 is updated in place from float64 tile moments of the raw step obs
 *                 (moments_out == NULL), or moments_out (device double [1 + 2*O]) gets
 *                 the batch moments (n, sums, sums of squares) for the caller's
 *                 all-reduce + lz_rms_update (multi-GPU);
 *   k = K:        the bootstrap of step K-1 and r->last_values.
 * obs_rms_state: the lz_rms state (lz_rms_state: mean[O], var[O], count, contiguous),
 * read and written; r->obs_norm NULL or the same pointer; r->obs_moments NULL.  The
 * batch moments are float64 sums in one fixed order (lz_internal.h PStepArgs; restated
 * by the oracle) -- SB3 sums float32 rows with np.mean / np.var.  Step k reads
 * r->obs_in (k = 0) or r->obs_last.  Call k = 0 .. K in order on one stream. */
lz_status lz_policy_step_f32(lz_handle* h, const lz_policy_rollout_args* r, int32_t k,
                             double* obs_rms_state, double* moments_out);
/* k = 0 .. K of lz_policy_step_f32 with in-place statistics (single GPU). */
lz_status lz_rollout_policy_f32_vn(lz_handle* h, const lz_policy_rollout_args* r,
                                   double* obs_rms_state);

/* The actor-critic of the reference's flagship PPO script, code/train.py:52-112:
 * policy_kwargs = dict(features_extractor_class=AttentionFeaturesExtractor,
 * features_extractor_kwargs=dict(features_dim=64), net_arch=dict(pi=[128, 128],
 * vf=[128, 128])), Tanh nets, one features extractor shared by pi and vf (SB3
 * share_features_extractor=True).  The extractor (code/train.py:56-95): fc1
 * Linear(obs_dim, 128) + ReLU, the 128 units viewed as 8 tokens of 16, a 4-head
 * nn.MultiheadAttention(16) self-attention, the 8 outputs flattened,
 * post_attention_fc Linear(128, 64) + ReLU.  Names are SB3 state_dict keys
 * (prefix features_extractor.). */
typedef struct lz_attn_policy {
  int32_t obs_dim;        /* 1..8 */
  int32_t act_dim;        /* 1..4 */
  const float* fc1_w;     /* features_extractor.fc1.weight [128, obs_dim] */
  const float* fc1_b;     /* features_extractor.fc1.bias [128] */
  const float* in_proj_w; /* features_extractor.attention_layer.in_proj_weight [48, 16] */
  const float* in_proj_b; /* features_extractor.attention_layer.in_proj_bias [48] */
  const float* out_proj_w; /* features_extractor.attention_layer.out_proj.weight [16, 16] */
  const float* out_proj_b; /* features_extractor.attention_layer.out_proj.bias [16] */
  const float* post_w;    /* features_extractor.post_attention_fc.0.weight [64, 128] */
  const float* post_b;    /* features_extractor.post_attention_fc.0.bias [64] */
  const float* pi_w1;     /* mlp_extractor.policy_net.0.weight [128, 64] */
  const float* pi_b1;
  const float* pi_w2;     /* mlp_extractor.policy_net.2.weight [128, 128] */
  const float* pi_b2;
  const float* vf_w1;     /* mlp_extractor.value_net.0.weight [128, 64] */
  const float* vf_b1;
  const float* vf_w2;     /* mlp_extractor.value_net.2.weight [128, 128] */
  const float* vf_b2;
  const float* act_w;     /* action_net.weight [act_dim, 128] */
  const float* act_b;
  const float* val_w;     /* value_net.weight [1, 128] */
  const float* val_b;
  const float* log_std;   /* log_std [act_dim] */
} lz_attn_policy;

/* Size of the packed attention policy blob (bf16 MFMA fragments + f32 biases;
 * out_proj folded into post_attention_fc in float64). */
int64_t lz_attn_policy_blob_bytes(void);
/* Pack *p into host_blob (cap >= lz_attn_policy_blob_bytes()).  Host-only. */
lz_status lz_attn_policy_pack(const lz_attn_policy* p, void* host_blob, int64_t cap);
/* lz_rollout_policy with an lz_attn_policy_pack blob: the same K-step fused rollout
 * with the attention features extractor in front of the two nets (32 envs per wave,
 * one wave per SIMD; the blob is resident in LDS). */
lz_status lz_rollout_policy_attn(lz_handle* h, const lz_policy_rollout_args* r);

/* code/lorenz_filter/train.py:54-132: PPO on VecFrameStack(HR, n_stack=4) with the
 * extractor variant that adds a residual connection and LayerNorm(16) after the
 * attention (x_seq = layer_norm(x_seq + out_proj(attn))) before post_attention_fc.
 * attn.obs_dim is the policy's input width = n_stack * env obs_dim (1..32). */
typedef struct lz_attn_ln_policy {
  lz_attn_policy attn;
  const float* ln_w;      /* features_extractor.layer_norm.weight [16] */
  const float* ln_b;      /* features_extractor.layer_norm.bias [16] */
} lz_attn_ln_policy;

int64_t lz_attn_ln_policy_blob_bytes(void);
lz_status lz_attn_ln_policy_pack(const lz_attn_ln_policy* p, void* host_blob, int64_t cap);

/* The fused rollout with an lz_attn_ln_policy_pack blob on SB3 VecFrameStack(n_stack)
 * observations (n_stack 1 or 4; systems LORENZ3 / PMSM / HR).  The stack of every env
 * lives in registers for the K steps and follows SB3 StackedObservations.update: roll
 * by obs_dim, the new frame last, zeros before the post-reset frame of a done env; the
 * truncation bootstrap values the stacked terminal observation [rolled stack, terminal
 * frame].  r->obs_buf is [K, N, n_stack*O] (the stacked observations the policy saw);
 * r->obs_in / obs_last stay the raw [N, O] frames, r->terminal_obs the raw terminal
 * frames; r->obs_norm and r->obs_moments must be NULL (the reference stacks raw obs).
 * stack_in / stack_out: [N, n_stack*O] float32 device (may alias). */
lz_status lz_rollout_policy_attn_stack(lz_handle* h, const lz_policy_rollout_args* r,
                                       int32_t n_stack, const float* stack_in, float* stack_out);

/* The two attention actor-critics at the precision the reference trains them in (torch
 * float32; code/train.py:101-112, code/lorenz_filter/train.py:117-127): float32
 * operands and accumulation everywhere (f32-input MFMA = k-ordered fmaf chains), the
 * softmax exp / LayerNorm / tanh as fixed IEEE operation sequences -- deterministic and
 * reproduced bit for bit by the C oracle (orc_attn_f32), which agrees with torch's
 * nn.MultiheadAttention / nn.LayerNorm float32 modules to ~1e-6.  Nothing is folded
 * (out_proj runs as its own layer).  hidden 128, features_dim 64.  Host-only packers;
 * obs_dim 1..8 (lz_attn_policy_pack_f32) or stacked input dims 1..32
 * (lz_attn_ln_policy_pack_f32, attn.obs_dim = n_stack * env obs_dim). */
int64_t lz_attn_policy_f32_blob_bytes(void);
lz_status lz_attn_policy_pack_f32(const lz_attn_policy* p, void* host_blob, int64_t cap);
lz_status lz_attn_ln_policy_pack_f32(const lz_attn_ln_policy* p, void* host_blob, int64_t cap);
/* lz_rollout_policy_attn / lz_rollout_policy_attn_stack with those blobs (systems
 * LORENZ3 / PMSM / HR).  The kernel keeps the extractor and one net in LDS and swaps the
 * pi / vf nets into it by LDS-DMA twice per step; a truncated step's bootstrap value is
 * added to its reward by the next step's launch segment (same result). */
lz_status lz_rollout_policy_attn_f32(lz_handle* h, const lz_policy_rollout_args* r);
/* Opt-in precision "i8x4" of the same actor-critics (same blob size, same rollout entry
 * points with LZ_POLICY_I8X4 in lz_policy_rollout_args.flags): the two wide layers of
 * each pi / vf net (64 -> 128, 128 -> 128: three quarters of the policy's multiplies) run
 * as truncated 4-digit fixed-point dot products on the int8 MFMA (v_mfma_i32_16x16x64_i8,
 * digit levels >= 3 summed exactly in int32, recombined with two float32 roundings): every
 * float32 input and weight is the int32 V = rint(v 2^q), |V| <= 2^28 (q per weight row
 * from its largest |w|; per env from its largest feature; 28 for tanh outputs), split into
 * four balanced int8 digits; only the 10 digit products of levels i + j >= 3 (weight
 * >= 2^-24 of the leading one) are summed -- exactly, in int32 (no order, no rounding);
 * levels 0-2 are dropped -- then recombined as fmaf(float(hi), 2^16, float(lo)), i.e.
 * rounded to float32 twice (lo, |lo| up to 2^31, is rounded before the fmaf), + the bias.  Error vs the exact dot product: that of float32's own fmaf
 * chain (tests/test_i8x4_host.py); bit-exact vs the C oracle (orc_attn_i8x4).  A NaN / inf
 * feature makes all of that env's outputs NaN.  The packers refuse non-finite net weights.
 * The extractor, softmax, heads and everything else are the float32 path's. */
lz_status lz_attn_policy_pack_i8x4(const lz_attn_policy* p, void* host_blob, int64_t cap);
/* The same opt-in precision for the float32 MlpPolicy (lz_rollout_policy_f32 with
 * LZ_POLICY_I8X4; not the per-step VecNormalize collect, lz_policy_step_f32): layer 2 of
 * each net (128 -> 128) on v_mfma_i32_32x32x32_i8 as above, layer 1 and the heads as the
 * float32 path; systems LORENZ3 / LORENZ4 / PMSM / HR.  Oracle: orc_mlp_i8x4. */
lz_status lz_policy_pack_i8x4(const lz_mlp_policy* p, int32_t hidden, void* host_blob, int64_t cap);
lz_status lz_attn_ln_policy_pack_i8x4(const lz_attn_ln_policy* p, void* host_blob, int64_t cap);
lz_status lz_rollout_policy_attn_stack_f32(lz_handle* h, const lz_policy_rollout_args* r,
                                           int32_t n_stack, const float* stack_in,
                                           float* stack_out);

/* SB3 RolloutBuffer.compute_returns_and_advantage over time-major [K, N] float32
 * buffers (float32 arithmetic in NumPy's order): advantages and returns out.
 * done = the done bytes of each step (episode_starts shifted by one). */
lz_status lz_gae(int64_t n, int32_t K, const float* rew, const float* values,
                 const uint8_t* done, const float* last_values, double gamma,
                 double gae_lambda, float* advantages, float* returns, int32_t device,
                 void* hip_stream);

/* RolloutBuffer.episode_starts of one collect (SB3 2.7.1 OnPolicyAlgorithm.
 * collect_rollouts: rollout_buffer.add(..., self._last_episode_starts, ...), then
 * _last_episode_starts = dones): starts[0] = last_in, starts[k] = (done[k-1] != 0)
 * as float32 [K, N]; last_out = (done[K-1] != 0), the next collect's last_in (must
 * not alias last_in). */
lz_status lz_episode_starts(int64_t n, int32_t K, const uint8_t* done, const float* last_in,
                            float* starts, float* last_out, int32_t device, void* hip_stream);

/* Read / write one SoA state plane (T or int32 / float32 elements as listed above),
 * stream-ordered on the handle's stream, device buffers:
 *   indices == NULL: the whole plane, N elements (count 0 or N);
 *   indices != NULL: a device int64 [count] list of env ids -- lz_get_state gathers
 *     dst[i] = plane[indices[i]], lz_set_state scatters plane[indices[i]] = src[i]
 *     (one launch, O(count) bytes: a single env's attribute is written without a
 *     whole-plane round trip).  Ids outside [0, N) are skipped by the scatter and read
 *     as zero bits by the gather (validate on the host); with repeated ids in a scatter
 *     it is unspecified which value lands.
 * Replaces the per-env attribute reads / writes of a DummyVecEnv caller:
 * VecEnv.get_attr / set_attr(name, value, indices) and the injection
 * `base_env.state1 = np.array([10, -10, 15])` in code/lorenz_pmsm/test_evaluate.py:100-102. */
lz_status lz_get_state(lz_handle* h, int32_t plane, void* dst, const int64_t* indices, int64_t count);
lz_status lz_set_state(lz_handle* h, int32_t plane, const void* src, const int64_t* indices,
                       int64_t count);

/* Element size in bytes of a plane (4 or 8), or 0 for an invalid plane. */
int32_t lz_plane_elem_size(const lz_handle* h, int32_t plane);

/* ------------------------------------------------------------------------------
 * On-device VecNormalize statistics (stable-baselines3 2.7.1 RunningMeanStd /
 * VecNormalize, common/running_mean_std.py and common/vec_env/vec_normalize.py, as
 * wrapped around the reference envs by code/lorenz_pmsm/train.py:118,170).  Float64
 * statistics on the device; batch moments are plain sums (count, sum, sum of squares)
 * so a multi-GPU caller all-reduces them before lz_rms_update.
 * ------------------------------------------------------------------------------ */
typedef struct lz_rms lz_rms;

/* RunningMeanStd(epsilon=count_init, shape=(dim,)): mean 0, var 1, count count_init. */
lz_status lz_rms_create(int32_t dim, int32_t device, double count_init, lz_rms** out);
lz_status lz_rms_destroy(lz_rms* r);
lz_status lz_rms_set_stream(lz_rms* r, void* hip_stream);
/* Device pointers to the statistics: mean[dim], var[dim], count[1] (double). */
lz_status lz_rms_state(lz_rms* r, double** mean, double** var, double** count);
/* moments_out (device double [1 + 2*dim]) = (n, column sums, column sums of squares)
 * of x [n, dim] (dtype LZ_DTYPE_F32 / F64); deterministic reduction order. */
lz_status lz_rms_moments(lz_rms* r, const void* x, int32_t dtype, int64_t n, double* moments_out);
/* RunningMeanStd.update_from_moments with those moments (possibly all-reduced). */
lz_status lz_rms_update(lz_rms* r, const double* moments);
/* RunningMeanStd.update(x) for x float32 [n, dim] (dim <= 8) in lz_policy_step_f32's
 * moment order (VecNormalize.reset() of the SB3-exact collect); with moments_out
 * non-NULL only the batch moments are written (all-reduce, then lz_rms_update). */
lz_status lz_rms_update_obs(lz_rms* r, const float* x, int64_t n, double* moments_out);
/* y (float32 [n, dim]) = clip((x - mean if center else x) / sqrt(var + eps), -clip, clip)
 * (VecNormalize.normalize_obs with center=1, normalize_reward with center=0). */
lz_status lz_rms_normalize(lz_rms* r, const void* x, int32_t dtype, int64_t n, float* y,
                           int32_t center, double eps, double clip);
/* VecNormalize discounted returns (double [n]): phase 0: returns = returns*gamma + rew;
 * phase 1: returns[done != 0] = 0. */
lz_status lz_returns_update(double* returns, const void* rew, int32_t dtype, const uint8_t* done,
                            int64_t n, double gamma, int32_t phase, int32_t device,
                            void* hip_stream);

/* ------------------------------------------------------------------------------
 * One VecNormalize(VecEnv).step() fused into the env step ("move the
 * running mean/var and obs normalisation into the step kernel epilogue").  SB3 2.7.1
 * VecNormalize.step_wait (common/vec_env/vec_normalize.py) over the outputs of
 * lz_step, in its order:
 *   obs_rms.update(obs)                       (if TRAINING and NORM_OBS)
 *   returns = returns*gamma + reward; ret_rms.update(returns)      (if TRAINING)
 *   obs_out  = NORM_OBS    ? clip((obs - mean)/sqrt(var + eps), +-clip_obs)  : obs
 *   rew_out  = NORM_REWARD ? clip(reward/sqrt(ret_var + eps), +-clip_reward) : reward
 *   terminal observations normalised like obs; returns[done] = 0
 * lz_step_vecnorm runs the env step (its kernel also writes float64 per-workgroup
 * moment partials of the obs and of the updated returns); the partials are reduced in
 * a fixed order (deterministic, no float atomics) -- up to 262,144 envs by every
 * workgroup of lz_vecnorm_apply, above that by a second launch of lz_step_vecnorm --
 * and lz_vecnorm_apply (one launch) applies the two RunningMeanStd updates (workgroup 0
 * writes them back) and writes the normalised outputs.  Call the two as a pair, apply
 * right after step on the same stream: the statistics are updated, and (without a
 * second launch) the step's *n_done_out is written, by the lz_vecnorm_apply launch.
 * With LZ_VN_DEFER the step's second launch publishes *n_done_out and leaves the
 * batch moments (obs: count, sums[O], sumsq[O]; then returns: count, sum, sumsq) in
 * moments for a multi-GPU all-reduce, and lz_vecnorm_apply performs the updates first.  Every
 * pointer is device memory; the statistics are those of the two lz_rms objects (dims
 * O and 1).
 * ------------------------------------------------------------------------------ */
enum {
  LZ_VN_TRAINING = 1,
  LZ_VN_NORM_OBS = 2,
  LZ_VN_NORM_REWARD = 4,
  LZ_VN_DEFER = 8
};

typedef struct lz_vecnorm {
  lz_rms* obs_rms;     /* RunningMeanStd(shape=(obs_dim,)) */
  lz_rms* ret_rms;     /* RunningMeanStd(shape=()) */
  double* returns;     /* [num_envs] discounted returns (VecNormalize.returns) */
  double* moments;     /* [2*obs_dim + 4] batch moments (LZ_VN_DEFER), else NULL */
  double gamma;
  double epsilon;
  double clip_obs;
  double clip_reward;
  uint32_t flags;      /* LZ_VN_* */
  uint32_t reserved;
} lz_vecnorm;

/* lz_step's contract for the raw outputs (obs_out/rew_out/done/compact list) plus the
 * VecNormalize bookkeeping above.  n_done_out (device int32) is required: the compact
 * list is how lz_vecnorm_apply finds the terminal rows to normalise; it is written by
 * the paired lz_vecnorm_apply launch (LZ_VN_DEFER: by this call's second launch). */
lz_status lz_step_vecnorm(lz_handle* h, const lz_vecnorm* vn, const void* actions,
                          void* obs_out, void* rew_out, uint8_t* done_out, int32_t* done_idx_out,
                          void* terminal_obs_out, int32_t* n_done_out);
/* The normalised views: obs_norm float32 [N, O], rew_norm float32 [N]; if done and
 * dones_out are non-NULL, dones_out[i] = (done[i] != 0) (uint8 0/1, SB3's bool
 * dones); if terminal_obs_raw and term_norm are non-NULL, term_norm float32
 * [n_done, O] from terminal_obs_raw [n_done, O], n_done read on the device from
 * n_done (the lz_step_vecnorm output; right after lz_step_vecnorm the count comes
 * from the step itself and this launch writes it to the step's n_done_out). */
lz_status lz_vecnorm_apply(lz_handle* h, const lz_vecnorm* vn, const void* obs_raw,
                           const void* rew_raw, const uint8_t* done, float* obs_norm,
                           float* rew_norm, uint8_t* dones_out, const void* terminal_obs_raw,
                           const int32_t* n_done, float* term_norm);

/* ------------------------------------------------------------------------------
 * VecFrameStack(venv, n_stack) on the device (SB3 2.7.1 common/vec_env/
 * stacked_observations.py StackedObservations, 1-D Box, channels-last), as the
 * reference stacks 4 HR observations (code/lorenz_filter/train.py:113-115).
 * stacked float32 [n, n_stack * obs_dim] (in place), obs float32 [n, obs_dim]:
 *   reset != 0: stacked = 0, last obs_dim columns = obs          (reset())
 *   reset == 0: shift left by obs_dim, rows with done[i] != 0 zeroed, then the last
 *               obs_dim columns = obs                           (update())
 * The stacked terminal observation of a done env is
 * concat(stacked_before[i, obs_dim:], terminal_obs[i]) -- build it before this call.
 * ------------------------------------------------------------------------------ */
lz_status lz_frame_stack(float* stacked, const float* obs, const uint8_t* done, int64_t n,
                         int32_t n_stack, int32_t obs_dim, int32_t reset, int32_t device,
                         void* hip_stream);

/* ------------------------------------------------------------------------------
 * Launch shapes (introspection; host-only, no device work).  Which kernel instantiation
 * and grid a call on this handle would launch -- the launchers choose by env count, CUs
 * and system (one-wave / split-lane / 256-lane rollouts; one wave per tile, the two nets
 * interleaved, or split over actor and critic waves for the policies), so tests can
 * assert that they reach every branch and profiling tools can name the kernel.
 * ------------------------------------------------------------------------------ */
enum {
  LZ_CALL_STEP = 0,                        /* lz_step, noise drawn on the device (noise NULL) */
  LZ_CALL_ROLLOUT = 1,                     /* lz_rollout */
  LZ_CALL_ROLLOUT_POLICY = 2,              /* lz_rollout_policy (bf16 MlpPolicy) */
  LZ_CALL_ROLLOUT_POLICY_F32 = 3,          /* lz_rollout_policy_f32 (LZ_POLICY_I8X4 runs the same
                                              shape: the i8x4 instantiation of the kernel) */
  LZ_CALL_POLICY_STEP_F32 = 4,             /* lz_policy_step_f32 / lz_rollout_policy_f32_vn */
  LZ_CALL_ROLLOUT_POLICY_ATTN = 5,         /* lz_rollout_policy_attn */
  LZ_CALL_ROLLOUT_POLICY_ATTN_STACK = 6,   /* lz_rollout_policy_attn_stack */
  LZ_CALL_ROLLOUT_POLICY_ATTN_F32 = 7,     /* lz_rollout_policy_attn_f32 */
  LZ_CALL_ROLLOUT_POLICY_ATTN_STACK_F32 = 8, /* lz_rollout_policy_attn_stack_f32 */
  LZ_CALL_STEP_NOISE = 9                   /* lz_step with caller-supplied noise (always
                                              k_step: the multi-tile kernel draws on device) */
};
enum {
  LZ_KERNEL_STEP = 1,             /* k_step: one 256-env tile per workgroup */
  LZ_KERNEL_STEP_MULTI = 2,       /* k_step_multi: 2 or 4 tiles per workgroup */
  LZ_KERNEL_ROLLOUT = 3,          /* k_rollout, 256-lane workgroups */
  LZ_KERNEL_ROLLOUT_WAVE = 4,     /* k_rollout, one-wave workgroups */
  LZ_KERNEL_ROLLOUT_SPLIT = 5,    /* k_rollout_split: two lanes per env */
  LZ_KERNEL_POLICY = 6,           /* k_rollout_policy: one wave per env tile, nets in turn */
  LZ_KERNEL_POLICY_PAIR = 7,      /* ... both nets interleaved in one instruction stream */
  LZ_KERNEL_POLICY_PAIR_PIPE = 8, /* ... interleaved, pipelined weight loads */
  LZ_KERNEL_POLICY_SPLIT = 9,     /* k_rollout_policy_f32_split: actor and critic waves */
  LZ_KERNEL_POLICY_STEP = 10,     /* k_policy_step_f32 */
  LZ_KERNEL_POLICY_ATTN = 11,     /* k_rollout_policy<..., kAttn / kAttnLn> (bf16) */
  LZ_KERNEL_POLICY_ATTN_F32 = 12, /* k_rollout_policy_attn_f32 */
  LZ_KERNEL_ROLLOUT_PAIR = 13     /* k_rollout_pair: PMSM, the step split over a lane
                                     pair (SysPMSM::step_pair) */
};
#define LZ_SHAPE_NO_DONE 1u     /* the done-free instantiation (no done can occur) */
#define LZ_SHAPE_GRID_STRIDE 2u /* fewer workgroups than env groups: workgroups loop */

typedef struct lz_launch_shape {
  int32_t kernel;        /* LZ_KERNEL_* */
  int32_t envs_per_wave; /* envs one wave carries (64, 32 or 16) */
  int32_t waves;         /* waves per workgroup */
  int32_t grid;          /* workgroups launched */
  uint32_t flags;        /* LZ_SHAPE_* */
  int32_t groups;        /* env groups of waves x envs_per_wave (> grid: grid-stride) */
} lz_launch_shape;

lz_status lz_get_launch_shape(const lz_handle* h, int32_t call, lz_launch_shape* out);

const char* lz_last_error(void);
int32_t lz_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* LORENZ_ENV_H */
