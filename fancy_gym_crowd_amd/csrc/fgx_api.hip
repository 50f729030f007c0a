// fgx_api.hip — C ABI (include/fgx.h) of the MI355X black-box rollout engine.
//
// Host side only does what the reference does once per env construction (make_bb,
// make_env_helpers.py:68-136): validate and flatten the configuration, allocate the SoA env
// state, build the basis tables (on the device), then launch kernels on the caller's stream.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>

#include "../../include/fgx.h"
#include "fgx_kernels.h"
#include "fgx_tables_k.h"
#include "fgx_aux.h"
#include "fgx_dispatch.h"
#include "fgx_learned.h"
#include "fgx_step.h"
#include "fgx_hp.h"

using namespace fgx;

static_assert(kInnerSlots == FGX_INNER_SLOTS && kInnerStride == FGX_INNER_STRIDE, "inner-step counter layout");

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                        \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess) return fail(FGX_E_HIP, std::string(#expr ": ") + hipGetErrorString(_e)); \
  } while (0)

struct Handle {
  fgx_config cfg;
  DevCfg dc;
  DevState st;
  int device;
  float* tables = nullptr;
  double* scratch = nullptr;
  void* state_block = nullptr;
  int ctx_dim = 0;
  // learned tau / delay: per-env tables, plans and plan lengths
  float* env_tab = nullptr;
  float* plan_pos = nullptr;
  float* plan_vel = nullptr;
  int32_t* plan_len = nullptr;
  void* learned_block = nullptr;
  double* obs_scratch = nullptr;   // info_level 2, SimpleReacher: qlog [T][nl][N] + gsave [2][N]
  bool learned() const { return dc.learn_tau || dc.learn_delay; }
};

size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

}  // namespace

// ------------------------------------------------------------------------ dispatch
// The episode kernels are instantiated per env kind in their own translation units
// (fgx_ep_<env>.hip, fgx_ep_<env>_gen.hip) so that the build compiles them in parallel.
#define FGX_FOR_NL(X) X(2) X(5)

// the kernel families of the other link counts (fgx_ep_nl.h); null for 2 and 5
static const NlOps* nl_ops(int nl) {
  switch (nl) {
    case 1: return fgx_nl_ops_1();
    case 3: return fgx_nl_ops_3();
    case 4: return fgx_nl_ops_4();
    case 6: return fgx_nl_ops_6();
    case 7: return fgx_nl_ops_7();
    case 8: return fgx_nl_ops_8();
  }
  return nullptr;
}

// any per-step output, or the validity checks: the logging instantiations (fgx_dispatch.h)
static bool episode_logs(const DevCfg& c, const Outputs& o) {
  return o.positions || o.step_actions || o.step_obs || o.step_rewards || o.is_collided || o.end_effector ||
         o.reward_dist || c.valid_flags != 0;
}

static int launch_episode(const Handle& h, int mp, const float* params, const float* dpos, const float* dvel,
                          const Outputs& o, hipStream_t stream) {
  if (const NlOps* ops = nl_ops(h.dc.nl)) return ops->episode(h.dc, h.st, mp, params, dpos, dvel, o, stream, g_err);
  // HoleReacher up to info level 1: the producer / consumer pipeline (fgx_hp.h)
  if (hp_applies(h.dc, h.st, mp, episode_logs(h.dc, o), o.positions || o.step_obs, h.st.plan_len != nullptr))
    return fgx_launch_episode_hp(h.dc, h.st, mp, params, o, stream, g_err);
  const bool gen = mp != MP_GIVEN && h.dc.nb != 5;   // generic basis-count instantiations
  if (h.dc.env == ENV_SIMPLE)
    return (gen ? fgx_launch_episode_simple_gen : fgx_launch_episode_simple)(h.dc, h.st, mp, params, dpos, dvel, o,
                                                                           stream, g_err);
  if (h.dc.env == ENV_HOLE)
    return (gen ? fgx_launch_episode_hole_gen : fgx_launch_episode_hole)(h.dc, h.st, mp, params, dpos, dvel, o,
                                                                       stream, g_err);
  return (gen ? fgx_launch_episode_via_gen : fgx_launch_episode_via)(h.dc, h.st, mp, params, dpos, dvel, o, stream,
                                                                     g_err);
}

static int launch_reset(const Handle& h, const uint64_t* seeds, const uint8_t* mask, int rs_mode, float* obs,
                        hipStream_t stream) {
  const int threads = 256;
  const int blocks = (int)((h.dc.N + threads - 1) / threads);
#define X(NL)                                                                                                    \
  if (h.dc.nl == NL) {                                                                                           \
    hipLaunchKernelGGL((k_reset<NL>), dim3(blocks), dim3(threads), 0, stream, h.dc, h.st, seeds, mask, rs_mode, obs); \
    HIP_TRY(hipGetLastError());                                                                           \
    return FGX_OK;                                                                                        \
  }
  FGX_FOR_NL(X)
#undef X
  if (const NlOps* ops = nl_ops(h.dc.nl)) return ops->reset(h.dc, h.st, seeds, mask, rs_mode, obs, stream, g_err);
  return fail(FGX_E_UNSUPPORTED, "n_links must be in 1..8");
}

static int launch_traj_env(const Handle& h, const float* params, float* pos, float* vel, hipStream_t stream,
                           float* info_pos = nullptr, float* info_vel = nullptr) {
  const int threads = 256;
  const int blocks = (int)((h.dc.N + threads - 1) / threads);
#define LAUNCH1(MPV, NLV, NBV)                                                                           \
  hipLaunchKernelGGL((k_traj_env<MPV, NLV, NBV>), dim3(blocks), dim3(threads), 0, stream, h.dc, h.st, params, \
                     h.env_tab, pos, vel, h.plan_len, info_pos, info_vel)
#define LAUNCH(MPV, NLV) do { if (h.dc.nb == 5) LAUNCH1(MPV, NLV, 5); else LAUNCH1(MPV, NLV, 0); } while (0)
  const int mp = h.dc.mp, nl = h.dc.nl;
  if (const NlOps* ops = nl_ops(nl))
    return ops->traj_env(h.dc, h.st, params, h.env_tab, pos, vel, h.plan_len, info_pos, info_vel, stream, g_err);
  if (mp == MP_PROMP && nl == 2) LAUNCH(MP_PROMP, 2);
  else if (mp == MP_PROMP && nl == 5) LAUNCH(MP_PROMP, 5);
  else if (mp == MP_DMP && nl == 2) LAUNCH(MP_DMP, 2);
  else if (mp == MP_DMP && nl == 5) LAUNCH(MP_DMP, 5);
  else if (mp == MP_PRODMP && nl == 2) LAUNCH(MP_PRODMP, 2);
  else if (mp == MP_PRODMP && nl == 5) LAUNCH(MP_PRODMP, 5);
  else return fail(FGX_E_UNSUPPORTED, "n_links must be in 1..8");
#undef LAUNCH1
#undef LAUNCH
  HIP_TRY(hipGetLastError());
  return FGX_OK;
}

// ------------------------------------------------------------------------ config -> DevCfg
static int build_devcfg(const fgx_config& c, int64_t N, DevCfg& d, int& ctx_dim) {
  if (c.abi_version != FGX_ABI_VERSION) return fail(FGX_E_INVALID, "abi_version mismatch");
  if (N <= 0) return fail(FGX_E_INVALID, "n_envs must be positive");
  if (c.env_kind != FGX_ENV_SIMPLE && c.env_kind != FGX_ENV_HOLE && c.env_kind != FGX_ENV_VIA)
    return fail(FGX_E_INVALID, "bad env_kind");
  if (c.rew_fct < FGX_REW_SIMPLE || c.rew_fct > FGX_REW_UNBOUNDED) return fail(FGX_E_INVALID, "Unknown reward function");
  if (c.rew_fct != FGX_REW_SIMPLE && c.env_kind != FGX_ENV_HOLE) return fail(FGX_E_INVALID, "rew_fct is a HoleReacher option");
  if (c.sched_n < 0 || c.sched_n > 4) return fail(FGX_E_INVALID, "sched_n must be in [0, 4]");
  for (int j = 0; j < c.sched_n; ++j) {
    const int kd = c.sched_kind[j];
    if (kd == FGX_SCHED_EVERY && c.sched_k[j] <= 0) return fail(FGX_E_INVALID, "schedule period must be positive");
    if (kd == FGX_SCHED_NORM_PERIOD &&
        !(c.sched_i0[j] >= 0 && c.sched_i0[j] < c.sched_i1[j] && c.sched_i1[j] - c.sched_i0[j] <= 8 &&
          c.sched_div[j] != 0.0))
      return fail(FGX_E_INVALID, "norm-period clause: 0 <= i0 < i1 <= i0 + 8, div != 0");
    if (kd < FGX_SCHED_EVERY || kd > FGX_SCHED_NORM_PERIOD) return fail(FGX_E_INVALID, "bad schedule clause kind");
  }
  if (c.learn_sub_trajectories && (c.replan_period > 0 || c.sched_n > 0))   // make_env_helpers.py:91-92
    return fail(FGX_E_INVALID, "Cannot used sub-trajectory learning and replanning together.");
  if (c.learn_sub_trajectories && !c.learn_tau)   // make_env_helpers.py:115-116
    return fail(FGX_E_INVALID, "learn_sub_trajectories requires learn_tau");
  if ((c.learn_tau || c.learn_delay) && c.mp_kind == FGX_MP_NONE)
    return fail(FGX_E_INVALID, "learn_tau / learn_delay need a movement primitive");
  if (c.learn_tau && !(c.tau_bound_lo > 0.0 && c.tau_bound_lo <= c.tau_bound_hi))
    return fail(FGX_E_INVALID, "tau_bound must satisfy 0 < lo <= hi");
  if (c.learn_delay && !(c.delay_bound_lo >= 0.0 && c.delay_bound_lo <= c.delay_bound_hi))
    return fail(FGX_E_INVALID, "delay_bound must satisfy 0 <= lo <= hi");
  if (c.n_links < 1 || c.n_links > kMaxLinks) return fail(FGX_E_INVALID, "n_links out of range");
  if (c.mp_kind < FGX_MP_NONE || c.mp_kind > FGX_MP_PRODMP) return fail(FGX_E_INVALID, "bad mp_kind");
  if (c.ctrl_kind < FGX_CTRL_PD || c.ctrl_kind > FGX_CTRL_POS) return fail(FGX_E_INVALID, "bad ctrl_kind");
  if (c.mp_kind != FGX_MP_NONE) {
    if (c.T <= 0) return fail(FGX_E_INVALID, "T must be positive");
    // the in-register return sum restates numpy's pairwise summation with one recursion level
    if (c.T > 256) return fail(FGX_E_UNSUPPORTED, "plan length T > 256 not supported");
    if (c.n_basis < 1 || c.n_basis > kGenBasis) return fail(FGX_E_UNSUPPORTED, "n_basis must be in [1, 12]");
    if (c.n_basis + c.zero_start + c.zero_goal > kMaxBasis) return fail(FGX_E_INVALID, "too many basis functions");
    // centres (j - o) / (n - 2o - 1) of the unbounded phase (fgx_tables.h rbf64): n - 2o - 1 >= 1
    if (c.num_basis_outside < 0 || c.n_basis + c.zero_start + c.zero_goal - 2 * c.num_basis_outside - 1 < 1)
      return fail(FGX_E_INVALID, "num_basis_outside must satisfy 0 <= o and num_basis - 2 o > 1");
    if (c.mp_kind == FGX_MP_PRODMP && c.phase_kind != FGX_PHASE_EXP)
      return fail(FGX_E_INVALID, "prodmp needs the exp phase generator");   // basis_generator_factory.py:14
    if (!(c.tau > 0.0) || !(c.dt > 0.0) || !std::isfinite(c.tau)) return fail(FGX_E_INVALID, "tau/dt must be positive");
    if (!std::isfinite(c.delay)) return fail(FGX_E_INVALID, "delay must be finite");
    // ProDMP: a negative delay would look up basis rows after the current one (prodmp_delay_index);
    // ProMP / DMP clip the phase max((t - delay) / tau, 0) and take any delay, as the reference does
    if (c.mp_kind == FGX_MP_PRODMP && !(c.delay >= 0.0)) return fail(FGX_E_INVALID, "ProDMP delay must be >= 0");
    if (!(c.basis_dt >= 0.0) || !std::isfinite(c.basis_dt)) return fail(FGX_E_INVALID, "basis_dt must be finite and >= 0");
    if (c.basis_dt > 0.0 && c.basis_dt != c.dt && c.mp_kind != FGX_MP_PRODMP)
      return fail(FGX_E_INVALID, "basis_dt is a ProDMP basis generator option");
  }
  if (c.time_aware && c.return_context) return fail(FGX_E_INVALID, "time_aware with context observation");
  std::memset(&d, 0, sizeof(d));
  d.N = N;
  d.env = c.env_kind;
  d.nl = c.n_links;
  d.random_start = c.random_start;
  d.allow_self = c.allow_self_collision;
  d.allow_wall = c.allow_wall_collision;
  d.mp = c.mp_kind;
  d.phase = c.phase_kind;
  d.nb = c.n_basis;
  d.zs = c.zero_start;
  d.zg = c.zero_goal;
  d.nbo = c.num_basis_outside;
  d.ctrl = c.ctrl_kind;
  d.T = c.T;
  d.max_steps = c.max_episode_steps;
  // replanning schedule program (replan_period alone == one EVERY clause)
  if (c.sched_n > 0) {
    d.sched_n = c.sched_n;
    for (int j = 0; j < c.sched_n; ++j) {
      d.sched_kind[j] = c.sched_kind[j];
      d.sched_k[j] = c.sched_k[j];
      d.sched_i0[j] = c.sched_i0[j];
      d.sched_i1[j] = c.sched_i1[j];
      d.sched_mul[j] = c.sched_mul[j];
      d.sched_div[j] = c.sched_div[j];
      if (c.sched_kind[j] == FGX_SCHED_NORM_PERIOD) d.sched_state = 1;
    }
  } else if (c.replan_period > 0) {
    d.sched_n = 1;
    d.sched_kind[0] = SCHED_EVERY;
    d.sched_k[0] = c.replan_period;
  }
  d.replan = d.sched_n > 0 ? 1 : 0;
  d.max_plans = c.max_planning_times;
  d.cond_desired = c.condition_on_desired;
  d.time_aware = c.time_aware;
  d.return_context = c.return_context;
  const int n = c.n_links;
  d.obs_dim = (c.env_kind == FGX_ENV_SIMPLE) ? 3 * n + 3 : (c.env_kind == FGX_ENV_HOLE ? 3 * n + 4 : 3 * n + 5);
  d.full_dim = d.obs_dim + (c.time_aware ? 1 : 0);
  for (int j = 0; j < c.sched_n; ++j)
    if (c.sched_kind[j] == FGX_SCHED_NORM_PERIOD && c.sched_i1[j] > d.full_dim)
      return fail(FGX_E_INVALID, "norm-period clause slice exceeds the observation");
  // context mask (simple_reacher/mp_wrapper.py:32-40, hole_reacher/mp_wrapper.py:36-46,
  // viapoint_reacher/mp_wrapper.py:27-35)
  int m = 0;
  for (int j = 0; j < 3 * n; ++j)
    if (c.random_start) d.ctx_idx[m++] = j;
  int p = 3 * n;
  if (c.env_kind == FGX_ENV_HOLE) {
    if (std::isnan(c.hole_width)) d.ctx_idx[m++] = p;
    p += 1;
  }
  if (c.env_kind == FGX_ENV_VIA) {
    if (std::isnan(c.via_x)) { d.ctx_idx[m++] = p; d.ctx_idx[m++] = p + 1; }
    p += 2;
  }
  d.ctx_idx[m++] = p;
  d.ctx_idx[m++] = p + 1;
  ctx_dim = m;
  d.out_dim = c.return_context ? ctx_dim : d.full_dim;
  d.n_params = (c.mp_kind == FGX_MP_PROMP) ? n * c.n_basis : n * (c.n_basis + 1);
  if (c.mp_kind == FGX_MP_NONE) d.n_params = 0;
  d.n_params += (c.learn_tau ? 1 : 0) + (c.learn_delay ? 1 : 0);   // params = [tau?, delay?, w...]
  d.learn_tau = c.learn_tau != 0;
  d.learn_delay = c.learn_delay != 0;
  d.sub_traj = c.learn_sub_trajectories != 0;
  d.tau_lo32 = (float)c.tau_bound_lo; d.tau_hi32 = (float)c.tau_bound_hi;
  d.delay_lo32 = (float)c.delay_bound_lo; d.delay_hi32 = (float)c.delay_bound_hi;
  const int max_s0 = (c.replan_period > 0 || c.sched_n > 0) ? c.max_episode_steps : 0;
  d.rows = max_s0 + c.T + 2;
  if (c.mp_kind == FGX_MP_PRODMP) {
    d.stride = 2 * (c.n_basis + 1) + 4;
  } else {
    d.stride = (c.n_basis + 2 + 3) & ~3;   // [basis..., dt32 | sdt, rcp(dt32), pad] (16-B rows)
  }
  if (c.mp_kind == FGX_MP_NONE) { d.rows = 0; d.stride = 0; }
  if ((int64_t)d.rows * d.stride * 4 > 64 * 1024)
    return fail(FGX_E_UNSUPPORTED, "MP tables exceed 64 KiB of LDS (episode / replanning too long)");
  d.rand_width = std::isnan(c.hole_width);
  d.rand_x = std::isnan(c.hole_x);
  d.rand_depth = std::isnan(c.hole_depth);
  d.rew_fct = c.rew_fct;
  if (c.env_kind == FGX_ENV_VIA && std::isnan(c.via_x) != std::isnan(c.via_y))
    return fail(FGX_E_INVALID, "via_target must be given as (x, y) or left unset");
  if (c.env_kind != FGX_ENV_HOLE && std::isnan(c.target_x) != std::isnan(c.target_y))
    return fail(FGX_E_INVALID, "target must be given as (x, y) or left unset");
  d.rand_via = std::isnan(c.via_x);
  d.rand_target = c.env_kind == FGX_ENV_HOLE || std::isnan(c.target_x);   // SimpleReacher / ViaPointReacher target
  d.via_x0 = c.via_x; d.via_y0 = c.via_y;
  d.tgt_x0 = c.target_x; d.tgt_y0 = c.target_y;
  d.dt = c.dt;
  d.tau = c.tau;
  d.delay = c.delay;
  d.alpha_phase = c.alpha_phase;
  d.bandwidth = c.bandwidth;
  d.bdt = c.basis_dt > 0.0 ? c.basis_dt : c.dt;
  // the fine grid's extent: row i looks up rint(max(t_i - delay, 0) / bdt), largest for the smallest
  // delay -- with learn_delay each env's own clipped delay (>= delay_bound_lo, the per-env walk of
  // prodmp_rows_seq), else the static one
  if (c.mp_kind == FGX_MP_PRODMP &&
      prodmp_fine_rows(d.dt, d.bdt, d.rows, d.tau, c.learn_delay ? std::min(d.delay, c.delay_bound_lo) : d.delay) >
          (1 << 20))
    return fail(FGX_E_UNSUPPORTED, "ProDMP precompute grid too fine (basis dt far below the env dt)");
  if (c.n_gains != 0 && c.n_gains != c.n_links)   // p_gains * (des_pos - c_pos) must broadcast
    return fail(FGX_E_INVALID, "per-joint PD gains must have n_links entries");
  for (int k = 0; k < kMaxLinks; ++k) {
    d.pg[k] = c.n_gains ? (k < c.n_links ? c.p_gains[k] : 0.0) : c.p_gain;
    d.dg[k] = c.n_gains ? (k < c.n_links ? c.d_gains[k] : 0.0) : c.d_gain;
  }
  d.act_lo = c.act_low;
  d.act_hi = c.act_high;
  d.act_lo32 = (float)c.act_low;
  d.act_hi32 = (float)c.act_high;
  d.dt32 = (float)c.dt;
  d.rcp_dt = 1.0 / c.dt;          // RN(1/dt): div_rcp64 (Markstein) is exact with it
  d.rcp_dt32 = 1.0f / d.dt32;
  d.tau32 = (float)c.tau;
  d.rcp_tau32 = 1.0f / d.tau32;
  d.hole_w0 = c.hole_width;
  d.hole_d0 = c.hole_depth;
  d.hole_x0 = c.hole_x;
  d.penalty = c.collision_penalty;
  d.weights_scale = c.weights_scale;
  d.goal_scale = c.goal_scale;
  d.alpha = c.alpha;
  d.ws32 = (float)c.weights_scale;
  d.gs32 = (float)c.goal_scale;
  d.alpha32 = (float)c.alpha;
  d.beta32 = (float)(c.alpha / 4);
  // trajectory validity (raw_interface_wrapper.py:55-72,103-121)
  if (c.valid_flags & ~(FGX_VALID_TAU | FGX_VALID_DELAY | FGX_VALID_POS)) return fail(FGX_E_INVALID, "bad valid_flags");
  if (c.valid_flags && c.mp_kind == FGX_MP_NONE) return fail(FGX_E_INVALID, "trajectory validity needs a movement primitive");
  if ((c.valid_flags & FGX_VALID_TAU) && !c.learn_tau) return fail(FGX_E_INVALID, "FGX_VALID_TAU needs learn_tau");
  if ((c.valid_flags & FGX_VALID_DELAY) && !c.learn_delay) return fail(FGX_E_INVALID, "FGX_VALID_DELAY needs learn_delay");
  if (c.invalid_obs != FGX_INVALID_OBS_ZEROS && c.invalid_obs != FGX_INVALID_OBS_CURRENT)
    return fail(FGX_E_INVALID, "bad invalid_obs");
  d.valid_flags = c.valid_flags;
  d.invalid_obs = c.invalid_obs;
  d.invalid_term = c.invalid_terminated != 0;
  d.invalid_trunc = c.invalid_truncated != 0;
  d.invalid_reward = c.invalid_reward;
  d.vtau_lo32 = (float)c.valid_tau_lo; d.vtau_hi32 = (float)c.valid_tau_hi;
  d.vdelay_lo32 = (float)c.valid_delay_lo; d.vdelay_hi32 = (float)c.valid_delay_hi;
  for (int k = 0; k < kMaxLinks; ++k) { d.vpos_lo[k] = c.valid_pos_lo[k]; d.vpos_hi[k] = c.valid_pos_hi[k]; }
  return FGX_OK;
}

__global__ void k_selftest_sincos(const double* x, int64_t n, double* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double s, c;
  fgx_sincos(x[i], &s, &c);
  out[4 * i] = s;
  out[4 * i + 1] = c;
  sincos_ocml(x[i], &s, &c);
  out[4 * i + 2] = s;
  out[4 * i + 3] = c;
}

extern "C" {

const char* fgx_last_error(void) { return g_err.c_str(); }

int fgx_selftest_sincos(const double* x, int64_t n, double* out, void* stream) {
  if (!x || !out || n < 0) return fail(FGX_E_INVALID, "bad argument");
  if (n == 0) return FGX_OK;
  hipLaunchKernelGGL(k_selftest_sincos, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x, n,
                     out);
  HIP_TRY(hipGetLastError());
  return FGX_OK;
}

int fgx_abi_version(void) { return FGX_ABI_VERSION; }

#ifndef FGX_BUILD_ID
#define FGX_BUILD_ID "unknown"
#endif
const char* fgx_build_id(void) { return FGX_BUILD_ID; }

int fgx_create(const fgx_config* cfg, int64_t n_envs, int device, void** handle) {
  if (!cfg || !handle) return fail(FGX_E_INVALID, "null argument");
  *handle = nullptr;
  Handle* h = new Handle();
  h->cfg = *cfg;
  h->device = device;
  int rc = build_devcfg(*cfg, n_envs, h->dc, h->ctx_dim);
  if (rc) { delete h; return rc; }
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) { delete h; return fail(FGX_E_HIP, std::string("hipSetDevice: ") + hipGetErrorString(e)); }
  const int64_t N = n_envs;
  const int nl = cfg->n_links;
  size_t off = 0;
  const size_t o_q = off; off = align_up(off + sizeof(double) * nl * N);
  const size_t o_qd = off; off = align_up(off + sizeof(double) * nl * N);
  const size_t o_goal = off; off = align_up(off + sizeof(double) * 2 * N);
  const size_t o_hole = off; off = align_up(off + sizeof(double) * 3 * N);
  const size_t o_aux = off; off = align_up(off + sizeof(double) * 3 * N);
  const size_t o_steps = off; off = align_up(off + sizeof(int32_t) * N);
  const size_t o_plans = off; off = align_up(off + sizeof(int32_t) * N);
  const size_t o_flags = off; off = align_up(off + sizeof(uint32_t) * N);
  const size_t o_rng = off; off = align_up(off + sizeof(uint64_t) * 5 * N);
  const size_t o_cond = off; off = align_up(off + sizeof(float) * 2 * nl * N);
  const size_t o_seed = off; off = align_up(off + sizeof(uint64_t) * N);
  const size_t o_start = off; off = align_up(off + sizeof(double) * N);
  const size_t o_tab = off; off = align_up(off + sizeof(float) * (size_t)h->dc.rows * h->dc.stride + 16);
  const size_t o_tabt = off; off = align_up(off + sizeof(float) * (size_t)tables_t_rows(h->dc.rows) * h->dc.stride);
  // step rewards of one BB step for the exact pairwise return of terminating envs (L > 128, k_episode);
  // for the direct envs also k_episode_hp's candidate final states (2 consumers x 2 n_links rows, fgx_hp.h)
  const bool direct = cfg->env_kind != FGX_ENV_SIMPLE && cfg->mp_kind != FGX_MP_NONE;
  const bool need_rew = direct || (h->dc.sched_state && cfg->mp_kind != FGX_MP_NONE && h->dc.T > 128);
  const size_t rew_rows = direct ? (size_t)std::max(h->dc.T, 2 * (2 * nl)) : (size_t)h->dc.T;
  const size_t o_rew = off; off = align_up(off + (need_rew ? sizeof(double) * rew_rows * N : 0));
  e = hipMalloc(&h->state_block, off);
  if (e != hipSuccess) { delete h; return fail(FGX_E_NOMEM, std::string("hipMalloc state: ") + hipGetErrorString(e)); }
  char* b = (char*)h->state_block;
  h->st.q = (double*)(b + o_q);
  h->st.qd = (double*)(b + o_qd);
  h->st.goal = (double*)(b + o_goal);
  h->st.hole = (double*)(b + o_hole);
  h->st.aux = (double*)(b + o_aux);
  h->st.steps = (int32_t*)(b + o_steps);
  h->st.plans = (int32_t*)(b + o_plans);
  h->st.flags = (uint32_t*)(b + o_flags);
  h->st.rng = (uint64_t*)(b + o_rng);
  h->st.cond = (float*)(b + o_cond);
  h->tables = (float*)(b + o_tab);
  h->st.rew = need_rew ? (double*)(b + o_rew) : nullptr;
  h->st.plan_len = nullptr;
  h->st.tables = h->tables;
  h->st.tables_t = (const float*)(b + o_tabt);
  h->st.start = (double*)(b + o_start);
  (void)hipMemset(h->state_block, 0, off);
  if (h->learned()) {
    const DevCfg& d0 = h->dc;
    size_t lo = 0;
    const size_t o_et = lo; lo = align_up(lo + sizeof(float) * (size_t)N * d0.rows * d0.stride);
    const size_t o_pp = lo; lo = align_up(lo + sizeof(float) * (size_t)N * d0.T * nl);
    const size_t o_pv = lo; lo = align_up(lo + sizeof(float) * (size_t)N * d0.T * nl);
    const size_t o_pl = lo; lo = align_up(lo + sizeof(int32_t) * N);
    e = hipMalloc(&h->learned_block, lo);
    if (e != hipSuccess) { fgx_destroy(h); return fail(FGX_E_NOMEM, "hipMalloc per-env plans"); }
    char* lb = (char*)h->learned_block;
    h->env_tab = (float*)(lb + o_et);
    h->plan_pos = (float*)(lb + o_pp);
    h->plan_vel = (float*)(lb + o_pv);
    h->plan_len = (int32_t*)(lb + o_pl);
  }
  // basis tables
  const DevCfg& d = h->dc;
  if (d.mp == MP_PROMP || d.mp == MP_DMP) {
    const int thr = 128, blk = (d.rows + thr - 1) / thr;
    hipLaunchKernelGGL(k_tables_rbf, dim3(blk), dim3(thr), 0, 0, d, cfg->tau, cfg->delay, cfg->alpha_phase,
                       cfg->bandwidth, h->tables);
  } else if (d.mp == MP_PRODMP) {
    const int Rf = prodmp_fine_rows(d.dt, d.bdt, d.rows, cfg->tau, cfg->delay);   // fine-grid rows
    e = hipMalloc(&h->scratch, sizeof(double) * (size_t)Rf * 2 * d.nb + 64);
    if (e != hipSuccess) { fgx_destroy(h); return fail(FGX_E_NOMEM, "hipMalloc scratch"); }
    hipLaunchKernelGGL(k_tables_prodmp, dim3(1), dim3(256), 0, 0, d, cfg->tau, cfg->delay, cfg->alpha_phase,
                       cfg->bandwidth, Rf, h->scratch, h->tables);
  }
  if (d.mp != MP_NONE && d.rows > 0) {
    const int n = tables_t_rows(d.rows) * d.stride;
    hipLaunchKernelGGL(k_tables_transpose, dim3((n + 255) / 256), dim3(256), 0, 0, d.rows, d.stride, d.nb, h->tables,
                       (float*)(b + o_tabt));
  }
  e = hipGetLastError();
  if (e != hipSuccess) { fgx_destroy(h); return fail(FGX_E_HIP, std::string("table kernel: ") + hipGetErrorString(e)); }
  // _start_pos[0] of a fresh env (simple_reacher.py:29 zeros; base_reacher.py:34 pi/2), then a
  // deterministic first reset (seed = env index) so that the state is always valid
  uint64_t* seeds = (uint64_t*)(b + o_seed);
  {
    uint64_t* hs = new uint64_t[N];
    double* sp = new double[N];
    for (int64_t i = 0; i < N; ++i) {
      hs[i] = (uint64_t)i;
      sp[i] = cfg->env_kind == FGX_ENV_SIMPLE ? 0.0 : M_PI / 2;
    }
    e = hipMemcpy(seeds, hs, sizeof(uint64_t) * N, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(h->st.start, sp, sizeof(double) * N, hipMemcpyHostToDevice);
    delete[] hs;
    delete[] sp;
    if (e != hipSuccess) { fgx_destroy(h); return fail(FGX_E_HIP, "hipMemcpy seeds"); }
  }
  rc = launch_reset(*h, seeds, nullptr, -1, nullptr, 0);
  if (rc) { fgx_destroy(h); return rc; }
  e = hipDeviceSynchronize();
  if (e != hipSuccess) { fgx_destroy(h); return fail(FGX_E_HIP, std::string("create sync: ") + hipGetErrorString(e)); }
  // NaN-free guard bound of the ProMP fast blocks: the largest row L1 norm of the basis columns
  h->dc.wbound32 = 1e30f;
  if (d.mp == MP_PROMP && d.rows > 0) {
    const size_t n = (size_t)d.rows * d.stride;
    float* ht = new float[n];
    e = hipMemcpy(ht, h->tables, n * sizeof(float), hipMemcpyDeviceToHost);
    double l1max = 0.0;
    for (int i = 0; e == hipSuccess && i < d.rows; ++i) {
      double l1 = 0.0;
      for (int j = 0; j < d.nb; ++j) l1 += std::fabs((double)ht[(size_t)i * d.stride + j]);
      l1max = std::isnan(l1) ? INFINITY : (l1 > l1max ? l1 : l1max);
    }
    delete[] ht;
    if (e != hipSuccess) { fgx_destroy(h); return fail(FGX_E_HIP, "hipMemcpy tables"); }
    h->dc.wbound32 = l1max > 1.0 ? (float)(1e30 / l1max) : 1e30f;   // (inf table: 0, every wave exact)
  }
  *handle = h;
  return FGX_OK;
}

int fgx_destroy(void* handle) {
  Handle* h = (Handle*)handle;
  if (!h) return FGX_OK;
  (void)hipSetDevice(h->device);
  if (h->state_block) (void)hipFree(h->state_block);
  if (h->learned_block) (void)hipFree(h->learned_block);
  if (h->scratch) (void)hipFree(h->scratch);
  if (h->obs_scratch) (void)hipFree(h->obs_scratch);
  delete h;
  return FGX_OK;
}

int fgx_get_dims(void* handle, fgx_dims* out) {
  Handle* h = (Handle*)handle;
  if (!h || !out) return fail(FGX_E_INVALID, "null argument");
  std::memset(out, 0, sizeof(*out));
  out->n_envs = (int32_t)h->dc.N;
  out->dof = h->dc.nl;
  out->obs_dim = h->dc.obs_dim;
  out->ctx_dim = h->ctx_dim;
  out->out_obs_dim = h->dc.out_dim;
  out->n_params = h->dc.n_params;
  out->T = h->dc.T;
  out->table_rows = h->dc.rows;
  out->table_stride = h->dc.stride;
  return FGX_OK;
}

int fgx_reset(void* handle, const uint64_t* seeds, const uint8_t* mask, int32_t random_start, float* obs_out,
              void* stream) {
  Handle* h = (Handle*)handle;
  if (!h) return fail(FGX_E_INVALID, "null handle");
  if (random_start < -1 || random_start > 1) return fail(FGX_E_INVALID, "random_start must be -1, 0 or 1");
  return launch_reset(*h, seeds, mask, random_start, obs_out, (hipStream_t)stream);
}

#ifdef FGX_STAMPS
static unsigned long long* g_stamps = nullptr;
#endif
static Outputs make_outputs(float* obs, double* ret, uint8_t* te, uint8_t* tr, int32_t* tlen, float* fobs,
                            const fgx_info* info, int32_t autoreset) {
  Outputs o;
  std::memset(&o, 0, sizeof(o));
  o.obs = obs; o.ret = ret; o.term = te; o.trunc = tr; o.tlen = tlen; o.final_obs = fobs;
  o.autoreset = autoreset;
  if (info) {
    o.positions = info->positions;
    o.velocities = info->velocities;
    o.step_actions = info->step_actions;
    o.step_obs = info->step_obs;
    o.step_rewards = info->step_rewards;
    o.is_collided = info->is_collided;
    o.is_success = info->is_success;
    o.end_effector = info->end_effector;
    o.reward_dist = info->reward_dist;
    o.reward_ctrl = info->reward_ctrl;
    o.inner_steps = (long long*)info->inner_steps;
  }
#ifdef FGX_STAMPS
  static unsigned long long* stamps = nullptr;   // diagnostics build only (tools/stamps.py)
  if (!stamps && hipMalloc(&stamps, 16384 * 16 * sizeof(unsigned long long)) != hipSuccess) stamps = nullptr;
  o.stamps = stamps;
  g_stamps = stamps;
#endif
  return o;
}

#ifdef FGX_STAMPS
// Copies the section clocks of the last episode launch (n values) to host memory.
extern "C" int fgx_dbg_stamps(unsigned long long* host, int n) {
  if (!g_stamps) return -1;
  return hipMemcpy(host, g_stamps, (size_t)n * sizeof(unsigned long long), hipMemcpyDeviceToHost) == hipSuccess ? 0 : -2;
}
#endif

// per-step info arrays: InfoStage keeps each row's per-sample stride in 32 bits (fgx_device.h):
// N < 2^24 keeps kMaxObs rows of f64 below 4 GB (at 65536 envs the arrays are already 2.4 GB)
static bool info_too_large(const Handle* h, const fgx_info* info) {
  return info && (info->positions || info->step_actions || info->step_obs || info->step_rewards || info->is_collided ||
                  info->end_effector || info->reward_dist) && h->dc.N >= (int64_t(1) << 24);
}

// info_level 2 (per-step observations) on SimpleReacher: the logging k_episode logs q per sample and
// k_info_obs derives the trigonometric observation components from it (fgx_kernels.h); the handle's
// scratch for that is allocated on the first such step that needs it (T * n_links * N + 2 N doubles;
// k_episode_v2 needs none).  A first such step inside a HIP graph capture is refused rather than
// allocating there (hipMalloc would invalidate the capture): run it once before capturing.  Per-step
// observations on one handle must stay on one stream (the scratch is per handle).
static int attach_obs_scratch(Handle* h, Outputs& o, int mp, hipStream_t stream) {
  if (!o.step_obs || h->dc.env != ENV_SIMPLE) return FGX_OK;
  if (episode_kernel_choice(h->dc, mp, true, h->learned()) == EK_V2) return FGX_OK;
  const size_t nq = (size_t)h->dc.T * h->dc.nl * h->dc.N;
  if (!h->obs_scratch) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(stream, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone)
      return fail(FGX_E_INVALID, "the first step with per-step observations allocates its scratch: "
                                 "run it once outside the HIP graph capture");
    const hipError_t e = hipMalloc(&h->obs_scratch, sizeof(double) * (nq + 2 * (size_t)h->dc.N));
    if (e != hipSuccess) {
      h->obs_scratch = nullptr;
      return fail(FGX_E_NOMEM, std::string("hipMalloc per-step observation scratch: ") + hipGetErrorString(e));
    }
  }
  o.qlog = h->obs_scratch;
  o.gsave = h->obs_scratch + nq;
  return FGX_OK;
}

int fgx_step(void* handle, const float* params, float* obs, double* ret, uint8_t* terminated, uint8_t* truncated,
             int32_t* traj_len, float* final_obs, const fgx_info* info, int32_t autoreset, void* stream) {
  Handle* h = (Handle*)handle;
  if (!h) return fail(FGX_E_INVALID, "null handle");
  if (h->dc.mp == MP_NONE) return fail(FGX_E_INVALID, "step-based handle: use fgx_step_raw");
  if (!params || !obs || !ret || !terminated || !truncated || !traj_len) return fail(FGX_E_INVALID, "null output");
  if (info && ((info->positions == nullptr) != (info->velocities == nullptr)))
    return fail(FGX_E_INVALID, "positions and velocities must be given together");
  if (info && ((info->is_collided == nullptr) != (info->is_success == nullptr)))
    return fail(FGX_E_INVALID, "is_collided and is_success must be given together");
  if (info && ((info->reward_dist == nullptr) != (info->reward_ctrl == nullptr)))
    return fail(FGX_E_INVALID, "reward_dist and reward_ctrl must be given together");
  if (info_too_large(h, info)) return fail(FGX_E_UNSUPPORTED, "per-step info arrays need n_envs < 2^24");
  Outputs o = make_outputs(obs, ret, terminated, truncated, traj_len, final_obs, info, autoreset);
  if (const int rc = attach_obs_scratch(h, o, h->learned() ? MP_GIVEN : h->dc.mp, (hipStream_t)stream)) return rc;
  if (h->learned()) {
    // per-env plans first (and, when requested, the time-major info copies), then the episode
    // over the given plans with per-env lengths
    float* P = h->plan_pos;
    float* V = h->plan_vel;
    int rc = launch_traj_env(*h, params, P, V, (hipStream_t)stream, info ? info->positions : nullptr,
                             info ? info->velocities : nullptr);
    if (rc) return rc;
    Handle hh = *h;
    hh.st.plan_len = h->plan_len;
    o.positions = nullptr;
    o.velocities = nullptr;
    // (params only for the validity checks of the raw tau / delay entries)
    return launch_episode(hh, MP_GIVEN, params, P, V, o, (hipStream_t)stream);
  }
  return launch_episode(*h, h->dc.mp, params, nullptr, nullptr, o, (hipStream_t)stream);
}

int fgx_step_traj(void* handle, const float* des_pos, const float* des_vel, float* obs, double* ret,
                  uint8_t* terminated, uint8_t* truncated, int32_t* traj_len, float* final_obs, const fgx_info* info,
                  int32_t autoreset, void* stream) {
  Handle* h = (Handle*)handle;
  if (!h) return fail(FGX_E_INVALID, "null handle");
  if (!des_pos || !des_vel || !obs || !ret || !terminated || !truncated || !traj_len)
    return fail(FGX_E_INVALID, "null argument");
  if (h->dc.T <= 0) return fail(FGX_E_INVALID, "T must be positive");
  if (info && ((info->is_collided == nullptr) != (info->is_success == nullptr)))
    return fail(FGX_E_INVALID, "is_collided and is_success must be given together");
  if (info && ((info->reward_dist == nullptr) != (info->reward_ctrl == nullptr)))
    return fail(FGX_E_INVALID, "reward_dist and reward_ctrl must be given together");
  if (info_too_large(h, info)) return fail(FGX_E_UNSUPPORTED, "per-step info arrays need n_envs < 2^24");
  Outputs o = make_outputs(obs, ret, terminated, truncated, traj_len, final_obs, info, autoreset);
  if (const int rc = attach_obs_scratch(h, o, MP_GIVEN, (hipStream_t)stream)) return rc;
  o.positions = nullptr;
  o.velocities = nullptr;   // the caller already holds the desired trajectories
  return launch_episode(*h, MP_GIVEN, nullptr, des_pos, des_vel, o, (hipStream_t)stream);
}

int fgx_trajectory(void* handle, const float* params, float* des_pos, float* des_vel, void* stream) {
  Handle* h = (Handle*)handle;
  if (!h) return fail(FGX_E_INVALID, "null handle");
  if (!params || !des_pos || !des_vel) return fail(FGX_E_INVALID, "null argument");
  if (h->learned()) return launch_traj_env(*h, params, des_pos, des_vel, (hipStream_t)stream);
  if (const NlOps* ops = nl_ops(h->dc.nl)) return ops->traj(h->dc, h->st, params, des_pos, des_vel, (hipStream_t)stream, g_err);
  return launch_trajectory(h->dc, h->st, params, des_pos, des_vel, (hipStream_t)stream, g_err);
}

int fgx_step_raw(void* handle, const float* actions, float* obs, double* reward, uint8_t* terminated,
                 uint8_t* truncated, float* final_obs, int32_t autoreset, void* stream) {
  Handle* h = (Handle*)handle;
  if (!h) return fail(FGX_E_INVALID, "null handle");
  if (!actions || !obs || !reward || !terminated || !truncated) return fail(FGX_E_INVALID, "null argument");
  if (h->dc.time_aware) return fail(FGX_E_UNSUPPORTED, "step-based envs have no TimeAwareObservation");
  const int threads = kStepRawBlock;
  const int blocks = (int)((h->dc.N + threads - 1) / threads);
  hipStream_t s = (hipStream_t)stream;
  // LDS rows of the workgroup's action / observation slices (k_step_raw)
  const int so = step_raw_stride(h->dc.obs_dim), sa = step_raw_stride(h->dc.nl);
  const size_t lds = sizeof(float) * threads * ((so > sa ? so : sa) + (final_obs ? so : 0));
#define X(NL)                                                                                                  \
  if (h->dc.nl == NL) {                                                                                        \
    if (h->dc.env == ENV_SIMPLE)                                                                               \
      hipLaunchKernelGGL((k_step_raw<ENV_SIMPLE, NL>), dim3(blocks), dim3(threads), lds, s, h->dc, h->st,        \
                         actions, obs, reward, terminated, truncated, final_obs, autoreset);                   \
    else if (h->dc.env == ENV_HOLE)                                                                            \
      hipLaunchKernelGGL((k_step_raw<ENV_HOLE, NL>), dim3(blocks), dim3(threads), lds, s, h->dc, h->st,          \
                         actions, obs, reward, terminated, truncated, final_obs, autoreset);                   \
    else                                                                                                       \
      hipLaunchKernelGGL((k_step_raw<ENV_VIA, NL>), dim3(blocks), dim3(threads), lds, s, h->dc, h->st,           \
                         actions, obs, reward, terminated, truncated, final_obs, autoreset);                   \
    HIP_TRY(hipGetLastError());                                                                                \
    return FGX_OK;                                                                                             \
  }
  FGX_FOR_NL(X)
#undef X
  if (const NlOps* ops = nl_ops(h->dc.nl))
    return ops->step_raw(h->dc, h->st, actions, obs, reward, terminated, truncated, final_obs, autoreset, lds, s, g_err);
  return fail(FGX_E_UNSUPPORTED, "n_links must be in 1..8");
}

int fgx_get_state(void* handle, double* q, double* qd, double* goal, double* hole, int32_t* steps, void* stream) {
  Handle* h = (Handle*)handle;
  if (!h) return fail(FGX_E_INVALID, "null handle");
  return fgx_transpose_state(h->dc, h->st, q, qd, goal, hole, steps, (hipStream_t)stream, g_err);
}

int fgx_set_state(void* handle, const double* q, const double* qd, const double* goal, const double* hole,
                  const int32_t* steps, void* stream) {
  Handle* h = (Handle*)handle;
  if (!h) return fail(FGX_E_INVALID, "null handle");
  return fgx_untranspose_state(h->dc, h->st, q, qd, goal, hole, steps, (hipStream_t)stream, g_err);
}

int fgx_get_tables(void* handle, float* out, void* stream) {
  Handle* h = (Handle*)handle;
  if (!h || !out) return fail(FGX_E_INVALID, "null argument");
  const size_t n = (size_t)h->dc.rows * h->dc.stride;
  if (n) HIP_TRY(hipMemcpyAsync(out, h->tables, n * sizeof(float), hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return FGX_OK;
}

int fgx_episode_kernel(void* handle, int32_t info_level) {
  Handle* h = (Handle*)handle;
  if (!h) return fail(FGX_E_INVALID, "null handle");
  const int mp = h->learned() ? MP_GIVEN : h->dc.mp;
  // the predicate launch_episode_nl uses: any per-step output, or the validity checks
  const bool log = info_level >= 1 || h->dc.valid_flags != 0;
  if (h->dc.nl == 2 || h->dc.nl == 5)
    if (hp_applies(h->dc, h->st, mp, log, info_level >= 2, h->learned())) return EK_HP;
  return episode_kernel_choice(h->dc, mp, log, h->learned());
}

}  // extern "C"
