// fgx_v2.h — k_episode_v2: the verbose-2 black-box step (info_level 2, what fgx.make returns by
// default) for SimpleReacher + PD.
//
// BlackBoxWrapper.step(action, verbose=2) (black_box_wrapper.py:170-253) returns, besides the
// episode-segment return, per-step arrays of the whole plan: desired positions / velocities, the
// clipped actions, the observations and rewards, and SimpleReacher's reward_dist / reward_ctrl lists
// (simple_reacher.py:56-70) — 176 B per env and sample for LongSimpleReacher, 2.31 GB per BB step at
// 65536 envs.  Two things bound it: the bytes (≈ 0.33 ms at the box's ~6.9 TB/s write rate) and the
// observation's trigonometry (cos / sin of every q and FK's cumulative angles: 2 NL - 1 f64 sincos
// per sample and env, ~0.27 ms of full-chip VALU issue).  The logging k_episode puts
// both in one lone wave per SIMD; here they run side by side on the same SIMD:
//   waves 0..3 ("dynamics", one env per lane as k_episode): trajectory, PD, clip, torque Euler step,
//     reward, the epilogue (final observation, TimeLimit, auto-reset), and per sample the rows that
//     need no trigonometry: positions, velocities, step_actions, step_rewards, reward_dist,
//     reward_ctrl and the observation's q̇ / step / time components, each a store of 64 consecutive
//     envs ([T, X, N] rows, include/fgx.h fgx_info); q and the reward go to an LDS ring;
//   waves 4..7 ("observation", the same 64 envs): per sample the observation's trigonometric and
//     end-effector components from the staged q (an exact-checked fast path, DESIGN.md §4.9, else
//     the same Env::fk / fgx_sincos as emit_obs and k_info_obs), and the numpy pairwise return of the
//     staged rewards (handed back through LDS for the epilogue: its accumulators stay off the
//     dynamics waves' registers, which would otherwise spill — and a spill reload waits behind the
//     wave's outstanding stores, vmcnt counting both).
// Wave w and wave w + 4 of a workgroup share a SIMD (profiles/r01_wave_placement.txt), so each SIMD
// interleaves one dynamics and one observation wave; the ring holds kV2Chunk samples, double-buffered,
// one workgroup barrier per chunk (the k_episode_ws protocol with the roles' work reversed).
//
// Every value equals the logging k_episode's (+ k_info_obs): bit-identical results
// (tests/test_gpu_info_rows.py).  Served: ENV_SIMPLE + PD + shared tables, static replanning
// schedules, max_episode_steps <= 200, no validity checks (fgx_dispatch.h).
#pragma once
#include "fgx_jp.h"

namespace fgx {

constexpr int kV2Chunk = 4;   // samples per ring slot
typedef __attribute__((address_space(1))) float gfloat;
typedef __attribute__((address_space(1))) double gdouble;
__device__ __forceinline__ gfloat* gp(float* p) { return (gfloat*)(uintptr_t)p; }
__device__ __forceinline__ gdouble* gp(double* p) { return (gdouble*)(uintptr_t)p; }
// element e of row r (wave-uniform: sample and component) of a [rows, N] array: the row base in SGPRs,
// the lane's byte offset eb = e * sizeof(T) in a VGPR (global_store saddr form; per-step arrays need
// N < 2^24, fgx_step)
template <typename T>
__device__ __forceinline__ void st_row(T* A, int64_t r, int64_t N, uint32_t eb, T x) {
  gchar* rb = uniform_ptr(A + r * N);
  *(__attribute__((address_space(1))) T*)(rb + eb) = x;
}
constexpr int kV2Pairs = 4;   // dynamics / observation wave pairs per workgroup (256 envs)
constexpr int kV2Threads = 128 * kV2Pairs;

// LDS: the basis table, the ring ([pair][2][C][NL + 1][64] doubles: q and the reward of each sample)
// and each env's return
inline size_t v2_lds_bytes(int rows, int stride, int nl) {
  return (((size_t)rows * stride + 3) & ~(size_t)3) * sizeof(float) +
         (size_t)kV2Pairs * 2 * kV2Chunk * (nl + 1) * 64 * sizeof(double) + (size_t)kV2Pairs * 64 * sizeof(double);
}

template <int MP, int NL, int NB>
__global__ __launch_bounds__(kV2Threads) void k_episode_v2(DevCfg c, DevState s, const float* __restrict__ params,
                                                    Outputs o) {
  constexpr int C = kV2Chunk;
  extern __shared__ float4 lds_v2[];
  float* tab = (float*)lds_v2;
  const int tab_f = c.rows * c.stride;
  constexpr int RS = NL + 1;   // ring doubles per sample and lane: q, then the reward
  double* ring = (double*)(lds_v2 + (tab_f + 3) / 4);   // [pair][2][C][RS][64]
  double* rets = ring + (size_t)kV2Pairs * 2 * C * RS * 64;   // [pair][64]
  for (int i = threadIdx.x; i < tab_f; i += blockDim.x) tab[i] = s.tables[i];

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool obs_wave = w >= kV2Pairs;
  const int pair = w & (kV2Pairs - 1);   // (waves w and w + 4 share a SIMD)
  const int64_t N = c.N;
  const int64_t e0 = (int64_t)blockIdx.x * (64 * kV2Pairs) + pair * 64 + lane;
  const bool valid = e0 < N;
  const int64_t e = valid ? e0 : N - 1;   // clamped index: loads stay in bounds, nothing is stored
  double* myring = ring + (size_t)pair * 2 * C * RS * 64;
  auto rq = [&](int b, int i, int d) __attribute__((always_inline)) -> double& { return myring[((b * C + i) * RS + d) * 64 + lane]; };
  const int T = c.T;
  const int nch = (T + C - 1) / C;   // every wave walks all T rows (the plan rows continue after L)
  const int X = c.full_dim;
  const float fnan = __builtin_nanf("");
  const double dnan = __builtin_nan("");
  const uint32_t e4 = (uint32_t)e * 4u, e8 = (uint32_t)e * 8u;   // the lane's byte offset in an f32 / f64 row
  // component x of sample k of a [T, X, N] array is row k X + x
  auto row_of = [&](int k, int x) __attribute__((always_inline)) -> int64_t { return (int64_t)k * X + x; };

  JpSeg sg;
  sg.init(c, s, e, valid);
  const int L = sg.L;
  // numpy pairwise split of the return sum (SimpleReacher never terminates: L is known now)
  const int split = (L > 128) ? ((L / 2) & ~7) : 0;
  __syncthreads();   // table staged

  if (obs_wave) {
    // ------------------------------------------------------------------ observation waves
    const double gx = s.goal[e], gy = s.goal[N + e];   // the episode's goal (the auto-reset comes later)
    float* so = o.step_obs;
    // the episode return: numpy's pairwise sum of the rewards the dynamics waves stage (its 19
    // accumulators live here, off the dynamics waves' registers)
    PairwiseSum ps;
    ps.init();
    // iteration it reads chunk it - 1 (staged before the previous barrier) while the dynamics waves
    // write chunk it into the other buffer
    for (int it = 0; it <= nch; ++it) {
      const int ch = it - 1, b = ch & 1;
      if (it > 0 && valid) {
#pragma unroll
        for (int i = 0; i < C; ++i) {
          const int k = ch * C + i;
          if (k >= T) break;
          if (k < L) ps.add(k, rq(b, i, NL), split);
          if (!so) continue;
          if (k < L) {
            // cos / sin of q (q[0]'s from FK) and end effector - goal, the f32 values k_info_obs
            // computes: a fast path (fgx_sincos_fast; the cumulative angles' cos / sin by angle
            // addition) whose every f32 result is checked against its error bound, else the lane
            // recomputes them exactly
            double q[NL];
#pragma unroll
            for (int d = 0; d < NL; ++d) q[d] = rq(b, i, d);
            float out[2 * NL + 2];
            const bool ok = obs_trig_fast<NL>(q, gx, gy, out);
            if (!ok) {   // (rare: a value near an f32 rounding boundary, or |q| >= 2^20)
              Env<NL> v;
#pragma unroll
              for (int d = 0; d < NL; ++d) v.q[d] = q[d];
              v.fk();
              out[0] = (float)v.c[0];
              out[NL] = (float)v.s[0];
#pragma unroll
              for (int d = 1; d < NL; ++d) {
                double sn, cs;
                fgx_sincos(v.q[d], &sn, &cs);
                out[d] = (float)cs;
                out[NL + d] = (float)sn;
              }
              out[2 * NL] = (float)(v.jx[NL] - gx);
              out[2 * NL + 1] = (float)(v.jy[NL] - gy);
            }
#pragma unroll
            for (int p = 0; p < 2 * NL; ++p) st_row(so, row_of(k, p), N, e4, out[p]);
            st_row(so, row_of(k, 3 * NL), N, e4, out[2 * NL]);
            st_row(so, row_of(k, 3 * NL + 1), N, e4, out[2 * NL + 1]);
          } else {
#pragma unroll
            for (int p = 0; p < 2 * NL; ++p) st_row(so, row_of(k, p), N, e4, fnan);
            st_row(so, row_of(k, 3 * NL), N, e4, fnan);
            st_row(so, row_of(k, 3 * NL + 1), N, e4, fnan);
          }
        }
      }
      __syncthreads();   // chunk it - 1 read; chunk it staged
    }
    rets[pair * 64 + lane] = ps.result(L, split);
    __syncthreads();   // the returns staged
    return;
  }

  // -------------------------------------------------------------------- dynamics waves
  Env<NL> v;
  load_env(c, s, e, v, false);   // SimpleReacher: no hole / reward state
  const int s0 = c.replan ? v.steps : 0;
  Traj<MP, NL, NB> tg;
  {
    double ic_q[NL], ic_qd[NL];
    const bool has_cond = c.cond_desired && (v.flags & 2u);
#pragma unroll
    for (int d = 0; d < NL; ++d) {
      ic_q[d] = has_cond ? (double)s.cond[d * N + e] : v.q[d];
      ic_qd[d] = has_cond ? (double)s.cond[(NL + d) * N + e] : v.qd[d];
    }
    tg.init(c, params + e * c.n_params, tab, s0, ic_q, ic_qd);
  }
  bool trunc = false;
  const double act_lo = __builtin_canonicalize(c.act_lo), act_hi = __builtin_canonicalize(c.act_hi);
  // (every info store is a typed global store, st_row: a generic pointer would make it a FLAT store,
  // which also counts in lgkmcnt, so the ring's LDS waits would wait for the stores)
  const Outputs& oo = o;

  // one row of sample k: the desired state (every lane), then the env step (lanes with k < L)
  auto row = [&](int k, int b, int i) __attribute__((always_inline)) {
    float pos[NL], vel[NL];
    tg.at(c, k, pos, vel);
    if (!valid) return;
    if (oo.positions) {
#pragma unroll
      for (int d = 0; d < NL; ++d) {
        st_row(oo.positions, (int64_t)k * NL + d, N, e4, pos[d]);
        st_row(oo.velocities, (int64_t)k * NL + d, N, e4, vel[d]);
      }
    }
    if (k < L) {
      // tracking controller + clip (black_box_wrapper.py:201-205; np.clip's NaN propagation)
      double a[NL];
      float a32[NL];
#pragma unroll
      for (int d = 0; d < NL; ++d) {
        const double u = fadd(c.pg[d] * fsub((double)pos[d], v.q[d]), c.dg[d] * fsub((double)vel[d], v.qd[d]));
        const double cl = __builtin_fmin(__builtin_fmax(u, act_lo), act_hi);
        a[d] = (u != u) ? u : cl;
        a32[d] = 0.0f;
      }
      const StepOut r = substep<ENV_SIMPLE, false, NL, true>(c, v, a, a32, false);
      trunc = v.steps >= c.max_steps;
      rq(b, i, NL) = r.reward;   // (the observation waves sum the return)
      if (oo.step_actions)
#pragma unroll
        for (int d = 0; d < NL; ++d) st_row(oo.step_actions, (int64_t)k * NL + d, N, e8, a[d]);
      if (oo.step_rewards) st_row(oo.step_rewards, (int64_t)k, N, e8, r.reward);
      if (oo.reward_dist) {
        st_row(oo.reward_dist, (int64_t)k, N, e8, r.rdist);
        st_row(oo.reward_ctrl, (int64_t)k, N, e8, r.rctrl);
      }
      if (oo.step_obs) {   // the components emit_obs computes without trigonometry, in its order
#pragma unroll
        for (int d = 0; d < NL; ++d) st_row(oo.step_obs, row_of(k, 2 * NL + d), N, e4, (float)v.qd[d]);
        st_row(oo.step_obs, row_of(k, 3 * NL + 2), N, e4, (float)v.steps);
        if (c.time_aware)
          st_row(oo.step_obs, row_of(k, 3 * NL + 3), N, e4, (float)((double)v.steps / (double)c.max_steps));
      }
#pragma unroll
      for (int d = 0; d < NL; ++d) rq(b, i, d) = v.q[d];
      if (k == L - 1 && sg.stop && c.cond_desired) {   // black_box_wrapper.py:234-236
#pragma unroll
        for (int d = 0; d < NL; ++d) { s.cond[d * N + e] = pos[d]; s.cond[(NL + d) * N + e] = vel[d]; }
        v.flags |= 2u;
      }
    } else {   // after trajectory_length: NaN rows (the plan rows above continue)
      if (oo.step_actions)
#pragma unroll
        for (int d = 0; d < NL; ++d) st_row(oo.step_actions, (int64_t)k * NL + d, N, e8, dnan);
      if (oo.step_rewards) st_row(oo.step_rewards, (int64_t)k, N, e8, dnan);
      if (oo.reward_dist) {
        st_row(oo.reward_dist, (int64_t)k, N, e8, dnan);
        st_row(oo.reward_ctrl, (int64_t)k, N, e8, dnan);
      }
      if (oo.step_obs) {
#pragma unroll
        for (int d = 0; d < NL; ++d) st_row(oo.step_obs, row_of(k, 2 * NL + d), N, e4, fnan);
        st_row(oo.step_obs, row_of(k, 3 * NL + 2), N, e4, fnan);
        if (c.time_aware) st_row(oo.step_obs, row_of(k, 3 * NL + 3), N, e4, fnan);
      }
    }
  };
  for (int it = 0; it <= nch; ++it) {   // iteration it writes chunk it (the observation waves read it - 1)
    if (it < nch) {
#pragma nounroll
      for (int i = 0; i < C; ++i) {
        const int k = it * C + i;
        if (k < T) row(k, it & 1, i);
      }
    }
    __syncthreads();   // chunk it staged; chunk it - 1 read
  }
  __syncthreads();   // the returns staged
  if (!valid) return;
  // the epilogue needs FK of the final q; a last sample at env step >= 199 has just computed it
  if (!(v.steps - 1 >= 199)) v.fk();
  episode_epilogue(c, s, o, e, v, sg.plans, L, rets[pair * 64 + lane], false, trunc);
}

}  // namespace fgx
