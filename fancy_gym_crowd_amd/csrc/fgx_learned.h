// fgx_learned.h — per-env movement primitives for learned tau / delay and sub-trajectories
// (included by fgx_api.hip only).
//
// Reference: make_env_helpers.py:115-126 (learn_tau / learn_delay, tau_bound [2 dt, duration],
// delay_bound [0, duration - 2 dt]), black_box_wrapper.py:106-140 (get_trajectory: np.clip of the
// params to the action space, duration=None for learn_sub_trajectories).  The phase, and with it
// the basis tables, differ per env: each thread builds its env's table rows (the same device
// functions as the shared tables, fgx_tables.h) into a per-env scratch slice, evaluates the plan
// with the same Traj code as the episode kernel, and writes it to [N, T, dof]; k_episode<MP_GIVEN>
// then runs the plan with per-env lengths (DevState::plan_len).  Oracle: mp.trajectory_learned.
#pragma once
#include "fgx_kernels.h"
#include "fgx_tables.h"

namespace fgx {

template <int MP, int NL, int NB>
__global__ __launch_bounds__(256) void k_traj_env(DevCfg c, DevState s, const float* __restrict__ params,
                                                  float* env_tab, float* dpos, float* dvel, int32_t* plan_len,
                                                  float* info_pos, float* info_vel) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= c.N) return;
  const int64_t N = c.N;
  const float* p = params + e * c.n_params;
  // np.clip(action, low, high) on the float32 action space (tau, delay bounds; weights unbounded)
  int off = 0;
  double tau = c.tau, delay = c.delay;
  float tau32 = c.tau32;
  if (c.learn_tau) {
    tau32 = np_clipf(p[0], c.tau_lo32, c.tau_hi32);
    tau = (double)tau32;
    off = 1;
  }
  if (c.learn_delay) {
    delay = (double)np_clipf(p[off], c.delay_lo32, c.delay_hi32);
    off += 1;
  }
  int Te = c.T;
  if (c.sub_traj) {   // duration=None: T = round(tau / dt) (np.round: half to even == rint)
    const double r = rint(tau / c.dt);
    Te = (r >= 1.0 && r <= (double)c.T) ? (int)r : (r > (double)c.T ? c.T : 1);
  }
  const int steps = s.steps[e];
  const int s0 = c.replan ? steps : 0;
  double ic_q[NL], ic_qd[NL];
  const bool has_cond = c.cond_desired && (s.flags[e] & 2u);
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    ic_q[k] = has_cond ? (double)s.cond[k * N + e] : s.q[k * N + e];
    ic_qd[k] = has_cond ? (double)s.cond[(NL + k) * N + e] : s.qd[k * N + e];
  }
  // this env's table rows [0, s0 + Te + 2)
  float* tab = env_tab + (size_t)e * c.rows * c.stride;
  const int R = s0 + Te + 2;
  if (MP == MP_PRODMP) {
    prodmp_rows_seq(c, tau, delay, c.alpha_phase, c.bandwidth, R, tab);
  } else {
    for (int i = s0; i < R; ++i) rbf_row(c, i, tau, delay, c.alpha_phase, c.bandwidth, tab + (size_t)i * c.stride);
  }
  Traj<MP, NL, NB, true> tg;
  tg.init(c, p + off, tab, s0, ic_q, ic_qd, Te, tau32, 1.0f / tau32);
  float pos[NL], vel[NL];
  for (int k = 0; k < Te; ++k) {
    tg.at(c, k, pos, vel);
#pragma unroll
    for (int d = 0; d < NL; ++d) {
      dpos[(e * c.T + k) * NL + d] = pos[d];
      dvel[(e * c.T + k) * NL + d] = vel[d];
    }
    if (info_pos) {   // info['positions'/'velocities'], time- and component-major [T, dof, N]
#pragma unroll
      for (int d = 0; d < NL; ++d) {
        info_pos[((int64_t)k * NL + d) * N + e] = pos[d];
        info_vel[((int64_t)k * NL + d) * N + e] = vel[d];
      }
    }
  }
  if (info_pos)   // the plan ends at T_e: NaN beyond (info arrays are [T, dof, N]; rows walked by the wave)
    for (int k = wave_min_active(min(Te, c.T)); k < c.T; ++k)
#pragma unroll
      for (int d = 0; d < NL; ++d) {
        if (k < Te) continue;
        info_pos[((int64_t)k * NL + d) * N + e] = __builtin_nanf("");
        info_vel[((int64_t)k * NL + d) * N + e] = __builtin_nanf("");
      }
  if (plan_len) plan_len[e] = Te;
}

}  // namespace fgx
