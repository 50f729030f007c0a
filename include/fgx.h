/*
 * fgx.h — C ABI of libfgx.so, the MI355X (gfx950) black-box rollout engine.
 *
 * Drop-in boundary for the fancy_gym black-box reacher path.  The reference has no native
 * code: each entry point below replaces a *Python* interface of the reference
 * (paths relative to /root/reference/fancy_gym):
 *
 *   fgx_create        make_bb(...) / bb_env_constructor(...)            utils/make_env_helpers.py:68-136,
 *                     (+ BlackBoxWrapper.__init__)                      envs/registry.py:280-309,
 *                                                                       black_box/black_box_wrapper.py:17-88
 *   fgx_reset         BlackBoxWrapper.reset -> env.reset(seed)          black_box/black_box_wrapper.py:258-267,
 *                                                                       base_reacher/base_reacher.py:73-93,
 *                                                                       simple_reacher/simple_reacher.py:46-54,
 *                                                                       hole_reacher/hole_reacher.py:60-112
 *   fgx_step          BlackBoxWrapper.step(action) (+ VectorEnv         black_box/black_box_wrapper.py:170-253
 *                     autoreset)                                        (gymnasium SyncVectorEnv.step [EXT-M])
 *   fgx_step_traj     BlackBoxWrapper.step with the desired trajectory  black_box/black_box_wrapper.py:177-253
 *                     supplied by the caller (get_trajectory skipped)
 *   fgx_trajectory    BlackBoxWrapper.get_trajectory(action)            black_box/black_box_wrapper.py:106-140
 *                     -> MPInterface.get_traj_pos/get_traj_vel          (mp_pytorch, EXTERNAL)
 *   fgx_step_raw      step-based env.step(action) (+ autoreset)         base_reacher/base_reacher_torque.py:20-37,
 *                                                                       base_reacher/base_reacher_direct.py:20-38
 *   fgx_get_state /   env.unwrapped.current_pos/current_vel, goal, hole black_box/raw_interface_wrapper.py:24-44
 *   fgx_set_state     (checkpoint/test access)
 *   fgx_get_tables    basis tables (test/introspection)
 *   fgx_episode_kernel which episode kernel fgx_step launches (introspection / benchmarks)
 *
 * Conventions
 *   - Every array argument is a CALLER-OWNED DEVICE pointer (e.g. torch tensor storage) on the
 *     handle's device, contiguous, row-major with the env index outermost ("[N, ...]").
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream).  All work is
 *     stream-ordered; no call synchronises the host except fgx_create / fgx_destroy.
 *   - Return value: 0 on success, a negative FGX_E* code on error; fgx_last_error() returns a
 *     thread-local message.  Nothing throws across the ABI.
 *   - A handle is bound to one device; calls on one handle are not re-entrant.  Distinct
 *     handles may be driven from distinct threads / processes (one per GPU).
 *   - Floating point: env state is f64 (as the reference's numpy state), MP trajectories f32
 *     (as mp_pytorch's torch f32), observations f32, rewards/returns f64.
 */
#ifndef FGX_H
#define FGX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FGX_ABI_VERSION 8

/* error codes */
#define FGX_OK 0
#define FGX_E_INVALID (-1)   /* bad argument / configuration (reference: ValueError)         */
#define FGX_E_HIP (-2)       /* HIP runtime error                                            */
#define FGX_E_NOMEM (-3)     /* device allocation failed                                     */
#define FGX_E_UNSUPPORTED (-4) /* configuration outside what the engine implements           */

/* env kinds (reference: SimpleReacherEnv = torque; HoleReacherEnv, ViaPointReacherEnv = direct
 * velocity; envs/__init__.py:56-698) */
#define FGX_ENV_SIMPLE 0
#define FGX_ENV_HOLE 1
#define FGX_ENV_VIA 2

/* replanning-schedule clauses (black_box_wrapper.py:233: replanning_schedule(pos, vel, obs,
 * action, t) with t = env steps since reset); a schedule is the OR of up to 4 clauses */
#define FGX_SCHED_EVERY 0        /* t % k == 0            (example_replanning_envs.py:38)       */
#define FGX_SCHED_AT 1           /* t == k                                                      */
#define FGX_SCHED_NORM_PERIOD 2  /* t % max(int(norm(obs[i0:i1])**2 * mul / div), 1) == 0
                                    (crowd_navigation/utils.py:9-10, obs = wrapped f64 obs)     */

/* HoleReacher reward functions (hole_reacher.py:48-58, rew_fct) */
#define FGX_REW_SIMPLE 0     /* hr_simple_reward.py        */
#define FGX_REW_VEL_ACC 1    /* hr_dist_vel_acc_reward.py  */
#define FGX_REW_UNBOUNDED 2  /* hr_unbounded_reward.py     */

/* trajectory validity (ABI 6): the env-side hooks BlackBoxWrapper.step calls before it runs a plan,
 * RawInterfaceWrapper.preprocessing_and_validity_callback / invalid_traj_callback
 * (raw_interface_wrapper.py:55-72,103-121; called at black_box_wrapper.py:178-197).  The reachers
 * keep the identity default (every plan valid, valid_flags = 0); a registered variant can ask for
 * the checks the reference's overriding envs make (table_tennis_env.py:304-309): */
#define FGX_VALID_TAU 1    /* valid_tau_lo <= action[0] <= valid_tau_hi (the raw f32 action, compared in
                              f32 as numpy does a float32 scalar against a Python float); learn_tau  */
#define FGX_VALID_DELAY 2  /* the same for the delay entry action[learn_tau]; learn_delay              */
#define FGX_VALID_POS 4    /* valid_pos_lo[d] <= desired position d <= valid_pos_hi[d] at every sample
                              of the plan (f32 positions against f64 bounds, as numpy compares them) */
/* the artificial transition of an invalid plan (invalid_traj_callback): no env step is taken,
 * trajectory_length = 0, return = invalid_reward, flags = invalid_terminated / invalid_truncated,
 * observation = zeros (the reference default, np.zeros) or the env's current observation */
#define FGX_INVALID_OBS_ZEROS 0
#define FGX_INVALID_OBS_CURRENT 1

/* trajectory generators (reference: trajectory_generator_factory.py:7-21) */
#define FGX_MP_NONE 0   /* step-based env only (fgx_step_raw)                */
#define FGX_MP_PROMP 1
#define FGX_MP_DMP 2
#define FGX_MP_PRODMP 3

/* phase generators (phase_generator_factory.py:9-23) */
#define FGX_PHASE_LINEAR 0
#define FGX_PHASE_EXP 1

/* tracking controllers (controller_factory.py:10-24) */
#define FGX_CTRL_PD 0        /* "motor"    pd_controller.py:21-29  */
#define FGX_CTRL_VEL 1       /* "velocity" vel_controller.py:8-9   */
#define FGX_CTRL_POS 2       /* "position" pos_controller.py:8-9   */

typedef struct fgx_config {
  int32_t abi_version;          /* = FGX_ABI_VERSION                                        */
  int32_t env_kind;             /* FGX_ENV_*                                                */
  int32_t n_links;              /* 1..8 (2 and 5, the registered reachers, have specialised 
                                   kernels; 1, 3, 4, 6, 7, 8 run the logging k_episode)       */
  int32_t random_start;         /* base_reacher.py:81-86                                    */
  int32_t allow_self_collision; /* HoleReacher only                                         */
  int32_t allow_wall_collision; /* HoleReacher only                                         */
  int32_t mp_kind;              /* FGX_MP_*                                                 */
  int32_t phase_kind;           /* FGX_PHASE_*                                              */
  int32_t n_basis;              /* basis functions per dof (without zero padding)          */
  int32_t zero_start;           /* ZeroPaddingNormalizedRBF num_basis_zero_start            */
  int32_t zero_goal;            /* ZeroPaddingNormalizedRBF num_basis_zero_goal             */
  int32_t ctrl_kind;            /* FGX_CTRL_*                                               */
  int32_t T;                    /* samples per plan = round(duration/dt)                    */
  int32_t max_episode_steps;    /* TimeLimit (registry max_episode_steps)                   */
  int32_t replan_period;        /* 0 = none; else replanning_schedule t % period == 0 (see sched_*) */
  int32_t max_planning_times;   /* <= 0 : unlimited                                         */
  int32_t condition_on_desired; /* black_box_wrapper.py:235-237                             */
  int32_t time_aware;           /* TimeAwareObservation appended (utils/wrappers.py:49-63)  */
  int32_t return_context;       /* context-mask the BB observation (black_box_wrapper.py:90-95) */
  int32_t num_basis_outside;    /* RBF centres beyond [0, 1] of the phase on each side (mp_pytorch
                                   NormalizedRBF / ProDMP num_basis_outside; was reserved0 = 0) */
  double dt;                    /* env dt (base_reacher.py:21)                              */
  double duration;              /* BB duration (make_env_helpers.py:110-111)                */
  double tau, delay, alpha_phase; /* phase generator                                        */
  double bandwidth;             /* basis_bandwidth_factor                                   */
  double weights_scale, goal_scale;
  double alpha;                 /* DMP / ProDMP spring constant                             */
  double pc_length;             /* ProDMP pre_compute_length_factor                         */
  double p_gain, d_gain;        /* PD gains                                                 */
  double act_low, act_high;     /* env action-space bounds as stored by gymnasium Box (f32) */
  double hole_width, hole_depth, hole_x; /* NaN = sampled at reset (hole_reacher.py:79-112)  */
  double collision_penalty;     /* HoleReacher / ViaPointReacher reward                     */
  /* ---- ABI 2 */
  int32_t rew_fct;              /* FGX_REW_* (HoleReacher only)                             */
  int32_t learn_tau;            /* phase_generator_kwargs learn_tau: params = [tau, ...]    */
  int32_t learn_delay;          /* learn_delay: params = [(tau,) delay, ...]                */
  int32_t learn_sub_trajectories; /* black_box_kwargs (black_box_wrapper.py:106-113)        */
  double tau_bound_lo, tau_bound_hi;     /* make_env_helpers.py:118-122 ([2 dt, duration])  */
  double delay_bound_lo, delay_bound_hi; /* make_env_helpers.py:124-126 ([0, duration-2dt]) */
  double via_x, via_y;          /* ViaPointReacher via_target (NaN = sampled, viapoint_reacher.py:60-66) */
  double target_x, target_y;    /* ViaPointReacher / SimpleReacher target (NaN = sampled;
                                   viapoint_reacher.py:68-74, simple_reacher.py:85-96)        */
  /* ---- ABI 3: replanning schedule as a clause program (sched_n == 0 and replan_period > 0
   * is the single clause EVERY(replan_period)) */
  int32_t sched_n;
  int32_t sched_kind[4];        /* FGX_SCHED_*                                              */
  int32_t sched_k[4];           /* EVERY: period; AT: step                                  */
  int32_t sched_i0[4], sched_i1[4]; /* NORM_PERIOD: slice of the (time-aware) observation   */
  double sched_mul[4], sched_div[4];
  /* ---- ABI 4: per-joint PD gains (pd_controller.py:16-29 with tuple gains); n_gains = 0 uses
   * the scalars p_gain / d_gain for every joint, else n_gains == n_links */
  int32_t n_gains;
  int32_t reserved1;
  double p_gains[8], d_gains[8];
  /* ---- ABI 6: trajectory validity (FGX_VALID_*, FGX_INVALID_OBS_*) */
  int32_t valid_flags;          /* 0 = every plan valid (the reachers' RawInterfaceWrapper default) */
  int32_t invalid_obs;          /* FGX_INVALID_OBS_*                                        */
  int32_t invalid_terminated, invalid_truncated;
  double invalid_reward;
  double valid_tau_lo, valid_tau_hi, valid_delay_lo, valid_delay_hi;
  double valid_pos_lo[8], valid_pos_hi[8];
  /* ---- ABI 8 */
  double basis_dt;              /* ProDMP basis generator dt (basis_generator_kwargs 'dt',
                                   basis_generator_factory.py:8-23): step of the precompute grid
                                   s_j = j * basis_dt / tau; 0 = the env dt                    */
} fgx_config;

typedef struct fgx_dims {
  int32_t n_envs, dof, obs_dim, ctx_dim, out_obs_dim, n_params, T, table_rows, table_stride;
  int32_t reserved[7];
} fgx_dims;

/* Optional per-step outputs of fgx_step / fgx_step_traj (black_box_wrapper.py:185-249,
 * verbose >= 2).  Any pointer may be NULL.  Rows after trajectory_length are set to NaN (0 for the
 * u8 flags); positions / velocities hold the whole plan (NaN after a learned plan length).
 * (Per-step arrays need n_envs < 2^24: FGX_E_UNSUPPORTED otherwise.)
 * The arrays are TIME- AND COMPONENT-MAJOR (ABI 7): [T, N] (sample k of env e at k*N + e) and
 * [T, X, N] (component x at (k*X + x)*N + e), so that a wave's per-step stores cover consecutive
 * envs; [N, T] / [N, T, X] are transposed / permuted views. */
typedef struct fgx_info {
  float* positions;      /* [T, dof, N]  desired positions                                 */
  float* velocities;     /* [T, dof, N]  desired velocities                                */
  double* step_actions;  /* [T, dof, N]  clipped controller actions                        */
  float* step_obs;       /* [T, obs_dim + time_aware, N]  full (unmasked) observations     */
  double* step_rewards;  /* [T, N]                                                         */
  uint8_t* is_collided;  /* [T, N]  HoleReacher / ViaPointReacher info                     */
  uint8_t* is_success;   /* [T, N]  HoleReacher / ViaPointReacher info                     */
  double* end_effector;  /* [T, 2, N] HoleReacher / ViaPointReacher info                   */
  double* reward_dist;   /* [T, N]  SimpleReacher info                                     */
  double* reward_ctrl;   /* [T, N]  SimpleReacher info                                     */
  int64_t* inner_steps;  /* [FGX_INNER_STEPS_LEN] zero-initialised partial counters: their sum  */
                         /* += the sum of trajectory_length over all envs (ABI 7; one device   */
                         /* atomic per wave / workgroup, spread over FGX_INNER_SLOTS lines)     */
} fgx_info;

/* fgx_info.inner_steps: FGX_INNER_SLOTS counters, FGX_INNER_STRIDE int64 apart (one 128-B line each):
 * a single counter serialised one device-scope atomic per wave (-6% on the 65536-env metric
 * kernel, profiles/r03_count_ab.jsonl) */
#define FGX_INNER_SLOTS 128
#define FGX_INNER_STRIDE 16
#define FGX_INNER_STEPS_LEN (FGX_INNER_SLOTS * FGX_INNER_STRIDE)

const char* fgx_last_error(void);
int fgx_abi_version(void);
/* Hash of the sources (csrc/, include/fgx.h) this library was built from (build provenance). */
const char* fgx_build_id(void);

int fgx_create(const fgx_config* cfg, int64_t n_envs, int device, void** handle);
int fgx_destroy(void* handle);
int fgx_get_dims(void* handle, fgx_dims* out);

/* Reset the envs where mask[i] != 0 (mask NULL = all).  seeds: device u64 [N] or NULL
 * (NULL = continue each env's own PCG64 stream, i.e. reset() without a seed).
 * random_start: -1 = the env's constructor setting, 0 / 1 = reset(options={'random_start': ...})
 * (base_reacher.py:77-86; a non-random reset restores the env's last start angle).
 * obs_out: [N, out_obs_dim] f32 (NULL ok); rows of envs not reset receive their current
 * observation.  seeds and mask, when given, must hold N entries. */
int fgx_reset(void* handle, const uint64_t* seeds, const uint8_t* mask, int32_t random_start, float* obs_out,
              void* stream);

/* One black-box step for all N envs: MP parameters params [N, n_params] f32 ->
 * obs [N, out_obs_dim] f32 (already auto-reset for finished envs), ret [N] f64 (episode-segment
 * return, np.sum aggregation), terminated/truncated [N] u8, traj_len [N] i32,
 * final_obs [N, out_obs_dim] f32 (observation before the auto-reset; may be NULL), info (NULL ok).
 * autoreset != 0 resets envs whose terminated|truncated is set (gymnasium VectorEnv). */
int fgx_step(void* handle, const float* params, float* obs, double* ret, uint8_t* terminated,
             uint8_t* truncated, int32_t* traj_len, float* final_obs, const fgx_info* info,
             int32_t autoreset, void* stream);

/* Same as fgx_step but with caller-supplied desired trajectories pos/vel [N, T, dof] f32. */
int fgx_step_traj(void* handle, const float* des_pos, const float* des_vel, float* obs,
                  double* ret, uint8_t* terminated, uint8_t* truncated, int32_t* traj_len,
                  float* final_obs, const fgx_info* info, int32_t autoreset, void* stream);

/* Desired trajectories for the next plan of every env (initial conditions = current state),
 * pos/vel [N, T, dof] f32 — the MFMA basis x weights GEMM path. */
int fgx_trajectory(void* handle, const float* params, float* des_pos, float* des_vel, void* stream);

/* Step-based env.step for all N envs: actions [N, dof] f32 applied unclipped (as the raw
 * reference env), obs [N, obs_dim] f32, reward [N] f64, terminated/truncated [N] u8,
 * final_obs (NULL ok).  autoreset as in fgx_step. */
int fgx_step_raw(void* handle, const float* actions, float* obs, double* reward,
                 uint8_t* terminated, uint8_t* truncated, float* final_obs, int32_t autoreset,
                 void* stream);

/* State access (tests / checkpoint): q, qd [N, dof] f64, goal [N, 2] f64, hole [N, 3] f64
 * (HoleReacher: x, width, depth; ViaPointReacher: via x, via y, 0), steps [N] i32.
 * Any pointer may be NULL. */
int fgx_get_state(void* handle, double* q, double* qd, double* goal, double* hole, int32_t* steps,
                  void* stream);
int fgx_set_state(void* handle, const double* q, const double* qd, const double* goal,
                  const double* hole, const int32_t* steps, void* stream);

/* Copy the f32 basis tables [table_rows, table_stride] to out (device). */
int fgx_get_tables(void* handle, float* out, void* stream);

/* The kernel fgx_step launches for this handle with the given info level (>= 2: per-step info
 * arrays): 0 = k_episode (one env per lane), 1 = k_episode_jp (one wave per joint),
 * 2 = k_episode_ws (trajectory producer / dynamics consumer wave pairs), 3 = k_episode_jl (one lane
 * per env x joint), 4 = k_episode_w2 (k_episode for two resident waves per SIMD), 5 = k_episode_pair
 * (HoleReacher, two lanes per env), 6 = k_episode_v2 (SimpleReacher + PD with per-step arrays: dynamics
 * and observation-trigonometry waves side by side), 7 = k_episode_v2h (HoleReacher / ViaPointReacher with
 * per-step arrays, n_envs % 256 == 0: the logging body beside a wave that stores its rows), 8 = k_episode_hp
 * (HoleReacher up to info level 1: a producer wave of dynamics feeding two consumer waves of FK /
 * collision / reward / per-step rows through LDS, + k_hp_finish for the epilogue); negative on error.
 * info_level >= 1 means some per-step output pointer is given (the launch then runs k_episode_hp, the
 * logging k_episode, k_episode_v2 or k_episode_v2h, as it does for a config with valid_flags; 2: the
 * verbose-2 rows, planned positions and step observations included).  All nine give
 * bit-identical results; the choice follows measured speed (fgx_dispatch.h, fgx_hp.h).
 * The report is for fgx_step with the handle's own plans and the output sets the Python VectorEnv
 * passes at that level (level >= 2: positions and step observations given, which is the launch's
 * "heavy" predicate); fgx_step_traj (caller-supplied plans) and C callers passing other subsets of
 * the per-step arrays may launch a different kernel of the same nine. */
int fgx_episode_kernel(void* handle, int32_t info_level);

/* Diagnostics (tests): for x[0..n) (device f64), out[4 n] = {sin, cos} of the kernels' sincos
 * (fgx_trig.h, the ocml algorithm with its small-argument reduction inlined) followed by {sin, cos}
 * of the ocml library call, so a test can compare them bit for bit. */
int fgx_selftest_sincos(const double* x, int64_t n, double* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* FGX_H */
