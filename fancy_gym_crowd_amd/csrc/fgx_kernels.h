// fgx_kernels.h — the HIP kernels of the rollout engine (gfx950).
//
//   k_tables      basis tables on the absolute-step grid (f64 math, rounded once to f32)
//   k_reset       seeded / unseeded env resets with numpy-exact PCG64 draws
//   k_episode     THE hot kernel: one black-box step (BlackBoxWrapper.step,
//                 black_box_wrapper.py:170-253) per env per thread — MP trajectory evaluation
//                 (basis x weights as a k-ordered f32 fma chain), PD / velocity controller,
//                 clip, reacher dynamics, FK, collisions, reward, TimeLimit, replanning and the
//                 numpy-pairwise return, with env state in registers for all T substeps, then
//                 the VectorEnv auto-reset — one launch per BB step.
//   k_step_raw    one step-based env.step for all envs (the per-substep kernel)
//   k_traj_valu   desired trajectories [N, T, dof] (reference path for k_traj_mfma)
//   k_traj_mfma   desired trajectories as an f32 MFMA GEMM (v_mfma_f32_32x32x2_f32)
#pragma once
#include "fgx_device.h"

namespace fgx {

// ============================================================================ tables
__device__ inline double phase64(const DevCfg& c, double t, double tau, double delay, double alpha_x) {
  double lin = (t - delay) / tau;
  lin = lin > 0.0 ? lin : 0.0;   // np.maximum(x, 0.0)
  if (c.phase == 0) return lin < 1.0 ? lin : 1.0;
  return exp((-alpha_x) * lin);
}

// normalized RBF at phase x, f64, all n = nb + zs + zg columns (oracle/mp.py:rbf64)
__device__ inline void rbf64(const DevCfg& c, double alpha_x, double bw, double x, double* phi) {
  const int n = c.nb + c.zs + c.zg;
  double cen[kMaxBasis + 4], e[kMaxBasis + 4];
  for (int j = 0; j < n; ++j) {
    const double u = (n > 1) ? (double)j / (double)(n - 1) : 0.0;
    cen[j] = (c.phase == 0) ? u : exp((-alpha_x) * u);
  }
  for (int j = 0; j < n; ++j) {
    double d = (n > 1) ? ((j < n - 1) ? cen[j + 1] - cen[j] : cen[n - 1] - cen[n - 2]) : 1.0;
    const double h = bw / (d * d);
    const double dd = x - cen[j];
    e[j] = exp((-h) * (dd * dd) / 2);
  }
  double s;
  if (n < 8) {
    s = e[0] + 0.0;
    for (int j = 1; j < n; ++j) s = s + e[j];
  } else {   // numpy pairwise (8 accumulators, n <= 128)
    double r[8];
    for (int j = 0; j < 8; ++j) r[j] = e[j];
    int i = 8;
    for (; i < n - (n % 8); i += 8)
      for (int j = 0; j < 8; ++j) r[j] = r[j] + e[i + j];
    s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) s = s + e[i];
  }
  for (int j = 0; j < n; ++j) phi[j] = e[j] / s;
}

// ProMP / DMP tables: one thread per row.
__global__ void k_tables_rbf(DevCfg c, double tau, double delay, double alpha_x, double bw, float* tab) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= c.rows) return;
  double phi[kMaxBasis + 4];
  const double t = (double)i * c.dt;
  const double x = phase64(c, t, tau, delay, alpha_x);
  rbf64(c, alpha_x, bw, x, phi);
  float* row = tab + (size_t)i * c.stride;
  if (c.mp == MP_PROMP) {
    for (int j = 0; j < c.nb; ++j) row[j] = (float)(c.weights_scale * phi[c.zs + j]);
    const float t0 = (float)t, t1 = (float)((double)(i + 1) * c.dt);
    row[c.nb] = t1 - t0;
  } else {   // DMP: psi = x * phi ; sdt = f32(s_{i+1}) - f32(s_i)
    for (int j = 0; j < c.nb; ++j) row[j] = (float)(x * phi[c.zs + j]);
    double s0 = (t - delay) / tau, s1 = ((double)(i + 1) * c.dt - delay) / tau;
    s0 = s0 > 0.0 ? s0 : 0.0;
    s1 = s1 > 0.0 ? s1 : 0.0;
    row[c.nb] = (float)s1 - (float)s0;
  }
}

// ProDMP precompute (oracle/mp.py:prodmp_fine64).  Single block; scratch: [rows][2*nb] f64.
__global__ void k_tables_prodmp(DevCfg c, double tau, double alpha_x, double bw, double* dp, float* tab) {
  const int nb = c.nb, R = c.rows, W = 2 * nb;
  const double h = c.dt / tau, a = c.alpha;
  for (int i = threadIdx.x; i < R; i += blockDim.x) {
    const double s = (double)i * h;
    const double x = exp((-alpha_x) * s);
    double phi[kMaxBasis + 4];
    rbf64(c, alpha_x, bw, x, phi);
    const double e = exp(a * s / 2);
    const double k1 = s * e * x, k2 = e * x;
    for (int j = 0; j < nb; ++j) {
      dp[(size_t)i * W + j] = k1 * phi[c.zs + j];
      dp[(size_t)i * W + nb + j] = k2 * phi[c.zs + j];
    }
  }
  __syncthreads();
  // cumulative trapezoid, one thread per column, sequential (same order as the oracle)
  if ((int)threadIdx.x < W) {
    const int j = threadIdx.x;
    double p = 0.0, prev = dp[j];
    dp[j] = 0.0;
    for (int i = 1; i < R; ++i) {
      const double cur = dp[(size_t)i * W + j];
      p = p + h * (prev + cur) / 2;
      dp[(size_t)i * W + j] = p;
      prev = cur;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < R; i += blockDim.x) {
    const double s = (double)i * h;
    const double e = exp(a * s / 2);
    const double y1 = exp((-a) * s / 2);
    const double y2 = s * y1;
    const double dy1 = -a / 2 * y1;
    const double dy2 = -a / 2 * y2 + y1;
    const double q1 = (a * s / 2 - 1) * e + 1;
    const double q2 = a / 2 * (e - 1);
    float* row = tab + (size_t)i * c.stride;
    for (int j = 0; j < nb; ++j) {
      const double p1 = dp[(size_t)i * W + j], p2 = dp[(size_t)i * W + nb + j];
      row[j] = (float)(p2 * y2 - p1 * y1);
      row[nb + 1 + j] = (float)(p2 * dy2 - p1 * dy1);
    }
    row[nb] = (float)(q2 * y2 - q1 * y1);
    row[2 * nb + 1] = (float)(q2 * dy2 - q1 * dy1);
    row[2 * nb + 2] = (float)y1;
    row[2 * nb + 3] = (float)y2;
    row[2 * nb + 4] = (float)dy1;
    row[2 * nb + 5] = (float)dy2;
  }
}

// ============================================================================ obs
// Full env observation (simple_reacher.py:75-83 / hole_reacher.py:296-306) [+ t/max_steps]
template <int NL>
__device__ __forceinline__ void full_obs(const DevCfg& c, const Env<NL>& v, float* o) {
  int p = 0;
  double sn[NL], cs[NL];
#pragma unroll
  for (int k = 0; k < NL; ++k) sincos(v.q[k], &sn[k], &cs[k]);
#pragma unroll
  for (int k = 0; k < NL; ++k) o[p++] = (float)cs[k];
#pragma unroll
  for (int k = 0; k < NL; ++k) o[p++] = (float)sn[k];
#pragma unroll
  for (int k = 0; k < NL; ++k) o[p++] = (float)v.qd[k];
  if (c.env == ENV_HOLE) o[p++] = (float)v.hw;
  o[p++] = (float)(v.jx[NL] - v.gx);
  o[p++] = (float)(v.jy[NL] - v.gy);
  o[p++] = (float)v.steps;
  if (c.time_aware) o[p++] = (float)((double)v.steps / (double)c.max_steps);
}

__device__ __forceinline__ void write_out_obs(const DevCfg& c, const float* full, float* dst) {
  if (c.return_context) {
    for (int j = 0; j < c.out_dim; ++j) dst[j] = full[c.ctx_idx[j]];
  } else {
    for (int j = 0; j < c.out_dim; ++j) dst[j] = full[j];
  }
}

// ============================================================================ state I/O
template <int NL>
__device__ __forceinline__ void load_env(const DevCfg& c, const DevState& s, int64_t e, Env<NL>& v) {
  const int64_t N = c.N;
#pragma unroll
  for (int k = 0; k < NL; ++k) { v.q[k] = s.q[k * N + e]; v.qd[k] = s.qd[k * N + e]; }
  v.gx = s.goal[e]; v.gy = s.goal[N + e];
  v.hx = s.hole[e]; v.hw = s.hole[N + e]; v.hd = s.hole[2 * N + e];
  v.steps = s.steps[e];
  v.flags = s.flags[e];
}

template <int NL>
__device__ __forceinline__ void store_env(const DevCfg& c, const DevState& s, int64_t e, const Env<NL>& v) {
  const int64_t N = c.N;
#pragma unroll
  for (int k = 0; k < NL; ++k) { s.q[k * N + e] = v.q[k]; s.qd[k * N + e] = v.qd[k]; }
  s.goal[e] = v.gx; s.goal[N + e] = v.gy;
  s.hole[e] = v.hx; s.hole[N + e] = v.hw; s.hole[2 * N + e] = v.hd;
  s.steps[e] = v.steps;
  s.flags[e] = v.flags;
}

// ============================================================================ reset
template <int NL>
__global__ __launch_bounds__(256) void k_reset(DevCfg c, DevState s, const uint64_t* seeds, const uint8_t* mask,
                                               float* obs) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= c.N) return;
  if (mask && !mask[e]) return;
  Env<NL> v;
  Pcg64 r = load_rng(s.rng, c.N, e);
  v.reset(c, r, seeds != nullptr, seeds ? seeds[e] : 0);
  store_rng(s.rng, c.N, e, r);
  store_env(c, s, e, v);
  s.plans[e] = 0;
  s.flags[e] = 0;
  if (obs) {
    float full[kMaxObs + 1];
    full_obs(c, v, full);
    write_out_obs(c, full, obs + e * c.out_dim);
  }
}

// ============================================================================ trajectories
// Per-thread desired-trajectory generator (oracle/mp.py:trajectory), f32 throughout.
template <int MP, int NL, int NB>
struct Traj {
  static constexpr int K = (MP == MP_PRODMP) ? NB + 3 : NB;
  float w[NL][K];          // ProMP: w ; DMP: w' ; ProDMP: [w', g', c1, c2]
  float g[NL];             // DMP goal
  float y[NL], z[NL];      // DMP state
  float cur[NL], vprev[NL];// ProMP look-ahead
  const float* tab;
  int stride, s0, T;

  __device__ __forceinline__ static float chain(const float* row, const float* wd) {
    float acc = 0.0f;
#pragma unroll
    for (int j = 0; j < K; ++j) acc = __builtin_fmaf(row[j], wd[j], acc);
    return acc;
  }

  // params: this env's row of the [N, n_params] matrix; q0/qd0 the initial conditions
  __device__ __forceinline__ void init(const DevCfg& c, const float* params, const float* tab_, int s0_,
                                       const double* q0, const double* qd0) {
    tab = tab_; stride = c.stride; s0 = s0_; T = c.T;
    if (MP == MP_PROMP) {
#pragma unroll
      for (int d = 0; d < NL; ++d)
#pragma unroll
        for (int j = 0; j < NB; ++j) w[d][j] = params[d * NB + j];
      const float* r1 = tab + (size_t)(s0 + 1) * stride;
#pragma unroll
      for (int d = 0; d < NL; ++d) { cur[d] = chain(r1, w[d]); vprev[d] = 0.0f; }
    } else if (MP == MP_DMP) {
#pragma unroll
      for (int d = 0; d < NL; ++d) {
#pragma unroll
        for (int j = 0; j < NB; ++j) w[d][j] = params[d * NB + j] * c.ws32;
        g[d] = params[NL * NB + d] * c.gs32;
        y[d] = (float)q0[d];
        z[d] = (float)qd0[d] * c.tau32;
      }
    } else if (MP == MP_PRODMP) {
      const float* rb = tab + (size_t)s0 * stride;
      const float y1 = rb[2 * NB + 2], y2 = rb[2 * NB + 3], dy1 = rb[2 * NB + 4], dy2 = rb[2 * NB + 5];
      const float det = y1 * dy2 - y2 * dy1;
#pragma unroll
      for (int d = 0; d < NL; ++d) {
#pragma unroll
        for (int j = 0; j < NB; ++j) w[d][j] = params[d * (NB + 1) + j] * c.ws32;
        w[d][NB] = params[d * (NB + 1) + NB] * c.gs32;
        float P = 0.0f, V = 0.0f;
#pragma unroll
        for (int j = 0; j <= NB; ++j) {
          P = __builtin_fmaf(rb[j], w[d][j], P);
          V = __builtin_fmaf(rb[NB + 1 + j], w[d][j], V);
        }
        const float A = (float)q0[d] - P;
        const float B = (float)qd0[d] * c.tau32 - V;
        w[d][NB + 1] = (dy2 * A - y2 * B) / det;
        w[d][NB + 2] = (y1 * B - dy1 * A) / det;
      }
    }
  }

  // desired (pos, vel) of plan sample k (row i = s0 + k + 1); call with k = 0, 1, 2, ...
  __device__ __forceinline__ void at(const DevCfg& c, int k, float* pos, float* vel) {
    const int i = s0 + k + 1;
    const float* row = tab + (size_t)i * stride;
    if (MP == MP_PROMP) {
      if (k < T - 1) {
        const float* nrow = row + stride;
        const float dti = row[NB];
#pragma unroll
        for (int d = 0; d < NL; ++d) {
          const float nx = chain(nrow, w[d]);
          pos[d] = cur[d];
          vel[d] = (nx - cur[d]) / dti;
          cur[d] = nx;
          vprev[d] = vel[d];
        }
      } else {
#pragma unroll
        for (int d = 0; d < NL; ++d) { pos[d] = cur[d]; vel[d] = vprev[d]; }
      }
    } else if (MP == MP_DMP) {
      const float sdt = row[NB];
#pragma unroll
      for (int d = 0; d < NL; ++d) {
        pos[d] = y[d];
        vel[d] = z[d] / c.tau32;
        if (k < T - 1) {
          const float f = chain(row, w[d]);
          const float acc = c.alpha32 * (c.beta32 * (g[d] - y[d]) - z[d]) + f;
          z[d] = z[d] + sdt * acc;
          y[d] = y[d] + sdt * z[d];
        }
      }
    } else if (MP == MP_PRODMP) {
      float hp[K], hv[K];
#pragma unroll
      for (int j = 0; j <= NB; ++j) { hp[j] = row[j]; hv[j] = row[NB + 1 + j]; }
      hp[NB + 1] = row[2 * NB + 2]; hp[NB + 2] = row[2 * NB + 3];
      hv[NB + 1] = row[2 * NB + 4]; hv[NB + 2] = row[2 * NB + 5];
#pragma unroll
      for (int d = 0; d < NL; ++d) {
        pos[d] = chain(hp, w[d]);
        vel[d] = chain(hv, w[d]) / c.tau32;
      }
    }
  }
};

// ============================================================================ the BB step
template <int ENV, int MP, int CTRL, int NL, int NB>
__global__ __launch_bounds__(256) void k_episode(DevCfg c, DevState s, const float* __restrict__ params,
                                                 const float* __restrict__ dpos, const float* __restrict__ dvel,
                                                 Outputs o) {
  extern __shared__ float lds_tab[];
  if (MP != MP_GIVEN) {
    const int n = c.rows * c.stride;
    for (int i = threadIdx.x; i < n; i += blockDim.x) lds_tab[i] = s.tables[i];
    __syncthreads();
  }
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= c.N) return;
  const int64_t N = c.N;

  Env<NL> v;
  load_env(c, s, e, v);
  int plans = s.plans[e];
  const int s0 = c.replan ? v.steps : 0;       // init_time = current_traj_steps * dt if replanning

  // initial conditions (black_box_wrapper.py:123-127)
  double ic_q[NL], ic_qd[NL];
  const bool has_cond = c.cond_desired && (v.flags & 2u);
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    ic_q[k] = has_cond ? (double)s.cond[k * N + e] : v.q[k];
    ic_qd[k] = has_cond ? (double)s.cond[(NL + k) * N + e] : v.qd[k];
  }
  Traj<(MP == MP_GIVEN ? MP_NONE : MP), NL, NB> tg;
  if (MP != MP_GIVEN) tg.init(c, params + e * c.n_params, lds_tab, s0, ic_q, ic_qd);

  plans += 1;
  PairwiseSum ps;
  ps.init();
  const int split = c.n_split;
  bool term = false, trunc = false;
  int k = 0;
  float pos[NL], vel[NL];
  const bool log = o.step_actions || o.step_obs || o.step_rewards || o.is_collided || o.reward_dist ||
                   o.positions || o.end_effector;
  for (k = 0; k < c.T; ++k) {
    if (MP == MP_GIVEN) {
#pragma unroll
      for (int d = 0; d < NL; ++d) {
        pos[d] = dpos[(e * c.T + k) * NL + d];
        vel[d] = dvel[(e * c.T + k) * NL + d];
      }
    } else {
      tg.at(c, k, pos, vel);
    }
    // ---- tracking controller + clip (black_box_wrapper.py:201-205)
    double a[NL];
    float a32[NL];
    constexpr bool F32 = (CTRL != CTRL_PD);
#pragma unroll
    for (int d = 0; d < NL; ++d) {
      if (CTRL == CTRL_PD) {
        const double u = c.p_gain * ((double)pos[d] - v.q[d]) + c.d_gain * ((double)vel[d] - v.qd[d]);
        a[d] = np_min(np_max(u, c.act_lo), c.act_hi);
      } else {
        const float u = (CTRL == CTRL_VEL) ? vel[d] : pos[d];
        a32[d] = np_minf(np_maxf(u, c.act_lo32), c.act_hi32);
        a[d] = (double)a32[d];
      }
    }
    // ---- env.step (base_reacher_torque.py:20-37 / base_reacher_direct.py:20-38)
    const int st = v.steps;
    double reward;
    bool coll = false, success = false;
    double rdist = 0.0, rctrl = 0.0;
    if (ENV == ENV_SIMPLE) {
#pragma unroll
      for (int d = 0; d < NL; ++d) {
        const double inc = F32 ? (double)(c.dt32 * a32[d]) : c.dt * a[d];
        v.qd[d] = v.qd[d] + inc;
        v.q[d] = v.q[d] + c.dt * v.qd[d];
      }
      double ctrl;
      if (F32) {
        float s32 = a32[0] * a32[0];
#pragma unroll
        for (int d = 1; d < NL; ++d) s32 = s32 + a32[d] * a32[d];
        ctrl = (double)s32;
      } else {
        ctrl = a[0] * a[0];
#pragma unroll
        for (int d = 1; d < NL; ++d) ctrl = ctrl + a[d] * a[d];
      }
      double dist = 0.0;
      if (st >= 199 || log) v.fk();
      if (st >= 199) dist = -norm2(v.jx[NL] - v.gx, v.jy[NL] - v.gy);
      reward = dist - ctrl;
      rdist = dist;
      rctrl = ctrl;
    } else {
      double acc_cost;
      if (F32 && (v.flags & 1u)) {
        float s32 = 0.0f;
#pragma unroll
        for (int d = 0; d < NL; ++d) {
          const float ac = (a32[d] - (float)v.qd[d]) / c.dt32;
          s32 = (d == 0) ? ac * ac : s32 + ac * ac;
        }
        acc_cost = (double)s32;
      } else {
        acc_cost = 0.0;
#pragma unroll
        for (int d = 0; d < NL; ++d) {
          const double ac = (a[d] - v.qd[d]) / c.dt;
          acc_cost = (d == 0) ? ac * ac : acc_cost + ac * ac;
        }
      }
#pragma unroll
      for (int d = 0; d < NL; ++d) {
        v.qd[d] = a[d];
        const double inc = F32 ? (double)(c.dt32 * a32[d]) : c.dt * v.qd[d];
        v.q[d] = v.q[d] + inc;
      }
      if (F32) v.flags |= 1u;
      v.fk();
      const bool sc = c.allow_self ? false : v.self_collision();
      const bool wc = c.allow_wall ? false : v.wall_collision(c);
      coll = sc || wc;
      if (st == 199 || coll) {
        const double dist = norm2(v.jx[NL] - v.gx, v.jy[NL] - v.gy);
        const double dc = dist * dist;
        reward = __builtin_fma(coll ? 1.0 : 0.0, -c.penalty, __builtin_fma(acc_cost, -5e-8, dc * -1.0));
        success = dist < 0.005 && !coll;
      } else {
        reward = acc_cost * -5e-8;
      }
    }
    v.steps = st + 1;
    term = (ENV == ENV_HOLE) ? coll : false;
    trunc = v.steps >= c.max_steps;
    ps.add(k, reward, split);
    // ---- info (verbose >= 2)
    if (log) {
      const int64_t ek = e * c.T + k;
      if (o.step_actions)
        for (int d = 0; d < NL; ++d) o.step_actions[ek * NL + d] = a[d];
      if (o.positions && MP != MP_GIVEN)
        for (int d = 0; d < NL; ++d) { o.positions[ek * NL + d] = pos[d]; o.velocities[ek * NL + d] = vel[d]; }
      if (o.step_rewards) o.step_rewards[ek] = reward;
      if (o.step_obs) {
        float full[kMaxObs + 1];
        full_obs(c, v, full);
        for (int j = 0; j < c.full_dim; ++j) o.step_obs[ek * c.full_dim + j] = full[j];
      }
      if (ENV == ENV_HOLE) {
        if (o.is_collided) { o.is_collided[ek] = coll; o.is_success[ek] = success; }
        if (o.end_effector) { o.end_effector[ek * 2] = v.jx[NL]; o.end_effector[ek * 2 + 1] = v.jy[NL]; }
      } else if (o.reward_dist) {
        o.reward_dist[ek] = rdist;
        o.reward_ctrl[ek] = rctrl;
      }
    }
    const bool replan_now = c.replan > 0 && ((k + 1 + s0) % c.replan == 0) &&
                            (c.max_plans <= 0 || plans < c.max_plans);
    if (term || trunc || replan_now) {
      if (c.cond_desired) {
#pragma unroll
        for (int d = 0; d < NL; ++d) { s.cond[d * N + e] = pos[d]; s.cond[(NL + d) * N + e] = vel[d]; }
        v.flags |= 2u;
      }
      break;
    }
  }
  const int L = (k < c.T) ? k + 1 : c.T;
  // fill the remaining desired rows for info['positions'] (full plan is reported)
  if (o.positions && MP != MP_GIVEN) {
    for (int kk = L; kk < c.T; ++kk) {
      tg.at(c, kk, pos, vel);
      const int64_t ek = e * c.T + kk;
      for (int d = 0; d < NL; ++d) { o.positions[ek * NL + d] = pos[d]; o.velocities[ek * NL + d] = vel[d]; }
    }
  }
  if (ENV == ENV_SIMPLE && !log) v.fk();
  float full[kMaxObs + 1];
  full_obs(c, v, full);
  o.ret[e] = ps.result(L, split);
  o.term[e] = term;
  o.trunc[e] = trunc;
  o.tlen[e] = L;
  if (o.final_obs) write_out_obs(c, full, o.final_obs + e * c.out_dim);
  if (o.autoreset && (term || trunc)) {
    Pcg64 r = load_rng(s.rng, N, e);
    v.reset(c, r, false, 0);
    store_rng(s.rng, N, e, r);
    plans = 0;
    v.flags = 0;
    full_obs(c, v, full);
  }
  write_out_obs(c, full, o.obs + e * c.out_dim);
  store_env(c, s, e, v);
  s.plans[e] = plans;
}

// ============================================================================ step-based
template <int ENV, int NL>
__global__ __launch_bounds__(256) void k_step_raw(DevCfg c, DevState s, const float* __restrict__ act, float* obs,
                                                  double* rew, uint8_t* term, uint8_t* trunc, float* final_obs,
                                                  int autoreset) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= c.N) return;
  const int64_t N = c.N;
  Env<NL> v;
  load_env(c, s, e, v);
  float a32[NL];
#pragma unroll
  for (int d = 0; d < NL; ++d) a32[d] = act[e * NL + d];
  const int st = v.steps;
  double reward;
  bool coll = false;
  if (ENV == ENV_SIMPLE) {
#pragma unroll
    for (int d = 0; d < NL; ++d) {
      v.qd[d] = v.qd[d] + (double)(c.dt32 * a32[d]);
      v.q[d] = v.q[d] + c.dt * v.qd[d];
    }
    float s32 = a32[0] * a32[0];
#pragma unroll
    for (int d = 1; d < NL; ++d) s32 = s32 + a32[d] * a32[d];
    v.fk();
    const double ctrl = (double)s32;
    reward = (st >= 199) ? -norm2(v.jx[NL] - v.gx, v.jy[NL] - v.gy) - ctrl : -ctrl;
  } else {
    double acc_cost;
    if (v.flags & 1u) {
      float s32 = 0.0f;
#pragma unroll
      for (int d = 0; d < NL; ++d) {
        const float ac = (a32[d] - (float)v.qd[d]) / c.dt32;
        s32 = (d == 0) ? ac * ac : s32 + ac * ac;
      }
      acc_cost = (double)s32;
    } else {
      acc_cost = 0.0;
#pragma unroll
      for (int d = 0; d < NL; ++d) {
        const double ac = ((double)a32[d] - v.qd[d]) / c.dt;
        acc_cost = (d == 0) ? ac * ac : acc_cost + ac * ac;
      }
    }
#pragma unroll
    for (int d = 0; d < NL; ++d) {
      v.qd[d] = (double)a32[d];
      v.q[d] = v.q[d] + (double)(c.dt32 * a32[d]);
    }
    v.flags |= 1u;
    v.fk();
    coll = (c.allow_self ? false : v.self_collision()) || (c.allow_wall ? false : v.wall_collision(c));
    if (st == 199 || coll) {
      const double dist = norm2(v.jx[NL] - v.gx, v.jy[NL] - v.gy);
      reward = __builtin_fma(coll ? 1.0 : 0.0, -c.penalty, __builtin_fma(acc_cost, -5e-8, dist * dist * -1.0));
    } else {
      reward = acc_cost * -5e-8;
    }
  }
  v.steps = st + 1;
  const bool te = (ENV == ENV_HOLE) && coll, tr = v.steps >= c.max_steps;
  float full[kMaxObs + 1];
  full_obs(c, v, full);
  rew[e] = reward;
  term[e] = te;
  trunc[e] = tr;
  if (final_obs) for (int j = 0; j < c.obs_dim; ++j) final_obs[e * c.obs_dim + j] = full[j];
  if (autoreset && (te || tr)) {
    Pcg64 r = load_rng(s.rng, N, e);
    v.reset(c, r, false, 0);
    store_rng(s.rng, N, e, r);
    v.flags = 0;
    full_obs(c, v, full);
  }
  for (int j = 0; j < c.obs_dim; ++j) obs[e * c.obs_dim + j] = full[j];
  store_env(c, s, e, v);
}

// ============================================================================ trajectories
template <int MP, int NL, int NB>
__global__ __launch_bounds__(256) void k_traj_valu(DevCfg c, DevState s, const float* __restrict__ params,
                                                   float* dpos, float* dvel) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= c.N) return;
  const int64_t N = c.N;
  Env<NL> v;
  load_env(c, s, e, v);
  const int s0 = c.replan ? v.steps : 0;
  double ic_q[NL], ic_qd[NL];
  const bool has_cond = c.cond_desired && (v.flags & 2u);
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    ic_q[k] = has_cond ? (double)s.cond[k * N + e] : v.q[k];
    ic_qd[k] = has_cond ? (double)s.cond[(NL + k) * N + e] : v.qd[k];
  }
  Traj<MP, NL, NB> tg;
  tg.init(c, params + e * c.n_params, s.tables, s0, ic_q, ic_qd);
  float pos[NL], vel[NL];
  for (int k = 0; k < c.T; ++k) {
    tg.at(c, k, pos, vel);
#pragma unroll
    for (int d = 0; d < NL; ++d) {
      dpos[(e * c.T + k) * NL + d] = pos[d];
      dvel[(e * c.T + k) * NL + d] = vel[d];
    }
  }
}

}  // namespace fgx
