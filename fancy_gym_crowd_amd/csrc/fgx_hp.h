// fgx_hp.h — k_episode_hp: the HoleReacher black-box step as a producer / consumer pipeline.
//
// BlackBoxWrapper.step (black_box_wrapper.py:170-253) over HoleReacher (hole_reacher.py:73-179,
// hr_simple_reward.py:19-53, base_reacher_direct.py:20-38): per plan sample the tracking controller,
// np.clip, the direct-velocity Euler step (q̇ = a, q += dt q̇), FK, the self- and wall-collision tests
// and the reward; the episode segment ends at the first collision.  The dynamics never read the
// collision result (the controller reads q and q̇ only, base_reacher_direct.py:25-27,
// black_box_wrapper.py:202-205): collisions only end the episode and enter the reward.  So the sample
// stream splits exactly, without rollback, into
//   * a producer wave P (one env per lane, as k_episode): plan, controller, clip, Σ acc², Euler — the
//     f64 chain that depends on the previous sample; it writes q and acc_cost of every sample (and the
//     action, the final q̇ candidate) into an LDS ring, chunk by chunk, running up to one chunk ahead;
//   * two consumer waves C0 / C1 on the same 64 envs: C_i takes the samples k ≡ i (mod 2) of each
//     two-sample chunk: FK, self / wall collision, the reward (hr_simple_reward) — the independent,
//     costly part (≈ 3/4 of k_episode's instructions);
//   * the resolution, one chunk later on both consumers (identically): the first sample that collides
//     or reaches the static end (plan end, TimeLimit, replanning sample) ends the segment; every
//     earlier sample counts.
// The return is numpy's pairwise sum (umath pairwise_sum) of the counted rewards, computed online
// although the length L is only known at the end: pairwise slot j = k & 7 is owned by consumer
// j & 1 (= k & 1), which keeps its four slots' accumulators of committed full 8-blocks for the
// level-1 sum (L <= 128) and for every second-half start s = (L/2) & ~7 that an L in (128, 200] can
// give (64, 72, 80, 88, 96); the partial last block's rewards stay in a 16-deep LDS ring until the
// end, and block(0, s) is formed by an LDS exchange when the first s samples have been counted.  The
// sum's rounding sequence is numpy's for every L (== PairwiseSum / pairwise_strided).  No [T][N]
// reward scratch in HBM.
//
// Workgroups of G groups (3 G waves, 64 envs per group): waves 0..G-1 are the producers, G..2G-1
// the consumers C0, 2G..3G-1 the consumers C1 of group w % G; with G = 4 the three waves of a group
// share one SIMD (wave w runs on SIMD w % 4, profiles/r01_wave_placement.txt), one workgroup per CU.
// One LDS-only barrier per two-sample chunk.  The producer reads the basis rows from global memory
// (all lanes the same row: one broadcast request per wave), so LDS holds only the rings.
//
// Served (hp_applies): HoleReacher with the simple reward function, 5 links, 5 basis functions per
// joint, shared tables (no learned tau / delay), static replanning schedules, no
// condition_on_desired, no validity checks, max_episode_steps <= 200; with per-step info arrays
// (info_level 1 / 2, a reward_aggregation reading step_rewards) the INFO instantiation.  Every output,
// every per-step array and the whole env state equal k_episode's bit for bit (tests/test_gpu_hp.py).
#pragma once
#include <cstdlib>
#include <cstring>
#include <string>

#include "fgx_v2.h"

namespace fgx {

constexpr int EK_HP = 8;   // fgx_episode_kernel's id (include/fgx.h)
constexpr int kHpNS = 5;   // second-half starts s = 64, 72, ..., 96 of numpy's split for L in (128, 200]
constexpr int kHpS0 = 64;
constexpr int kHpNR = 2;   // of them in the producer's registers (64, 72); the rest in LDS
constexpr int kHpPA = 10;  // depth of the producer's acc_cost ring (its lead over the resolution + 8)
// candidate final state rows per consumer in the handle's direct-env scratch: q, q̇
template <int NL> __host__ __device__ constexpr int hp_cand_rows() { return 2 * NL; }

// LDS of one group (doubles): the q ring [buf][i][d][lane] and the action ring [buf][i][d][lane] (the
// consumers' input: chunk it in buffer it & 1), the consumers' stop codes [buf][i][lane] (u8), the
// producer's acc_cost ring [k % 10][lane],
// the second-half accumulators of the LDS-held split starts [s][slot][lane], block(0, s) [s][lane]
// and the alive masks [parity] (u64)
template <int NL>
struct HpLayout {
  static constexpr int RQ = 2 * 2 * NL * 64;
  static constexpr int RA = 2 * 2 * NL * 64;
  static constexpr int RS = 2 * 2 * 64 / 8;
  static constexpr int PA = kHpPA * 64;
  static constexpr int BL = (kHpNS - kHpNR) * 8 * 64;
  static constexpr int FF = kHpNS * 64;
  static constexpr int AL = 2;
  static constexpr int SY = 2;   // the group's arrival counters (u32: producer, C0, C1)
  static constexpr int GROUP = RQ + RA + RS + PA + BL + FF + AL + SY;
  static constexpr int oRQ = 0, oRA = RQ, oRS = oRA + RA, oPA = oRS + RS, oBL = oPA + PA,
                       oFF = oBL + BL, oAL = oFF + FF, oSY = oAL + AL;
};

// The chunk barrier of one group (its producer and two consumers) when a workgroup holds several
// groups: a workgroup s_barrier makes every group wait each chunk for the slowest of the four (section
// clocks, profiles/r06_hp_stamps.jsonl: the waves of a four-group workgroup parked 17-45% of their loop
// there).  Each wave publishes its arrival count in the group's LDS word once its own LDS accesses have
// completed, then polls until the other two have arrived (LDS is one memory: a wave that sees the count
// reads the data written before it).  The three waves of a group arrive at the same barriers (the loop
// exits on the group's own alive mask, which all three read after the same barrier); the poll is
// bounded.
__device__ __forceinline__ void hp_group_barrier(uint32_t* cnt, int role, uint32_t target) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if ((threadIdx.x & 63) == 0) __hip_atomic_store(cnt + role, target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  for (int spin = 0; spin < (1 << 24); ++spin) {
    bool all = true;
#pragma unroll
    for (int r = 0; r < 3; ++r) all &= __hip_atomic_load(cnt + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= target;
    if (__builtin_amdgcn_readfirstlane((int)all)) break;
    __builtin_amdgcn_s_sleep(1);
  }
  asm volatile("" ::: "memory");
}

// diagnostics build (-DFGX_STAMPS, tools/hp_stamps.py): per wave (row blockIdx * 3 G + w of the stamp
// buffer) the cycles spent waiting at the chunk barriers and in the loop, and the iteration count
#ifdef FGX_STAMPS
#define FGX_HP_CLK(v) const unsigned long long v = __builtin_readcyclecounter()
#define FGX_HP_BAR(t0) hp_bar += __builtin_readcyclecounter() - (t0)
#define FGX_HP_PUT(i, v)                                                                   \
  do {                                                                                     \
    if (lane == 0 && o.stamps) o.stamps[((size_t)blockIdx.x * 3 * G + w) * 16 + (i)] = (v); \
  } while (0)
#else
#define FGX_HP_CLK(v) do { } while (0)
#define FGX_HP_BAR(t0) do { } while (0)
#define FGX_HP_PUT(i, v) do { } while (0)
#endif

// INFO: the verbose-2 per-step arrays (black_box_wrapper.py:184-189,218-227,244-249) as well: the
// producer writes the plan rows (positions / velocities) as it evaluates them, and at each chunk's
// resolution the rows that need the counted / not-counted decision (step_actions from the action ring,
// step_rewards, step_observations — cos / sin of q through obs_trig_fast, DESIGN.md §4.9 — NaN after
// trajectory_length); the consumers write the env info rows of their samples (end_effector, is_collided,
// is_success); the producer pads those after trajectory_length once every wave has left the loop.
template <int MP, int CTRL, int NL, int NB, int G, bool INFO>
__global__ __launch_bounds__(192 * G) void k_episode_hp(DevCfg c, DevState s, const float* __restrict__ params,
                                                       Outputs o) {
  using Lay = HpLayout<NL>;
  constexpr bool F32 = (CTRL != CTRL_PD);
#ifdef FGX_HP_NO_GSYNC   // (A/B builds) the workgroup barrier for every shape
  constexpr bool GSYNC = false;
#else
  constexpr bool GSYNC = G > 1;   // per-group chunk barriers (hp_group_barrier)
#endif
  extern __shared__ double lds_hp[];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int g = w % G, role = w / G;   // role 0: producer, 1: consumer C0, 2: consumer C1
#ifdef FGX_STAMPS
  unsigned long long hp_bar = 0, hp_res = 0, hp_prod = 0;
  const unsigned long long hp_t0 = __builtin_readcyclecounter();
#endif
  double* gr = lds_hp + (size_t)g * Lay::GROUP;
  uint64_t* al = (uint64_t*)(gr + Lay::oAL);
  uint8_t* rs = (uint8_t*)(gr + Lay::oRS);
  const int64_t N = c.N;
  const int64_t e0 = (int64_t)blockIdx.x * (64 * G) + g * 64 + lane;
  const bool valid = e0 < N;
  const int64_t e = valid ? e0 : N - 1;   // clamped: loads stay in bounds, nothing is stored
  const int T = c.T;
  double* cand = s.rew;   // candidate final states [ci][q | q̇ | |ee - goal|^2][N] (the handle's direct-env scratch)
  constexpr int CR = hp_cand_rows<NL>();

  // ---- every role: the env's static segment end (black_box_wrapper.py:233-239: plan end, TimeLimit,
  // replanning sample); a collision can only end it earlier
  const int steps0 = s.steps[e];
  const int plans = s.plans[e] + 1;
  const bool plans_ok = c.replan && (c.max_plans <= 0 || plans < c.max_plans);
  const int k_replan = plans_ok ? first_static_replan(c, steps0) : -1;
  int Lst = min(T, max(1, c.max_steps - steps0));
  if (k_replan >= 0) Lst = min(Lst, k_replan + 1);
  const int itmax = (T + 1) / 2 + 3;
  {
    const uint64_t vm = __ballot(valid);
    if (role == 0 && lane == 0) al[1] = vm;   // read as "iteration -1" by iteration 0
    if (role == 0 && lane < 3) ((uint32_t*)(gr + Lay::oSY))[lane] = 0u;
  }
  __syncthreads();
  // the loop ends when no env of the group (GSYNC; else of the workgroup) is alive
  auto all_done = [&](int rp) __attribute__((always_inline)) {
    uint64_t any = 0;
    if constexpr (GSYNC) {
      any = al[rp];
    } else {
#pragma unroll
      for (int gg = 0; gg < G; ++gg) any |= ((const uint64_t*)(lds_hp + (size_t)gg * Lay::GROUP + Lay::oAL))[rp];
    }
    return any == 0;
  };
  uint32_t* sy = (uint32_t*)(gr + Lay::oSY);
  auto chunk_barrier = [&](int it) __attribute__((always_inline)) {
    FGX_HP_CLK(tb);
    if constexpr (GSYNC) hp_group_barrier(sy, role, (uint32_t)(it + 1));
    else lds_barrier();
    FGX_HP_BAR(tb);
  };

  if (role != 0) {
    // ================================================================ consumers
    const int ci = role - 1;   // sample k = 2 c + ci of chunk c
    const double gx = s.goal[e], gy = s.goal[N + e];
    // the wall's edges (Env::wall_collision: left / right of the hole, its depth below the ground)
    const double hx = s.hole[e], hw = s.hole[N + e], hd = s.hole[2 * N + e];
    const double w_left = hx - hw / 2, w_right = hx + hw / 2, w_nd = -hd;
    const bool allow_self = c.allow_self != 0, allow_wall = c.allow_wall != 0;
    bool own_done = false;   // this consumer saw a stop sample of the env: the segment ends there or earlier
    for (int it = 0;; ++it) {
      const int rp = (it + 1) & 1;
      if (all_done(rp) || it > itmax) break;
      const int cpk = it - 1;
      const int k = 2 * cpk + ci;
      const bool alive = ((al[rp] >> lane) & 1) && !own_done;
      if (it >= 1 && alive && k < Lst) {
        const double* rq = gr + Lay::oRQ + (size_t)((cpk & 1) * 2 + ci) * NL * 64;
        // FK (base_reacher.py:95-103, Env::fk's operations) fused with the wall test of each link as
        // soon as its start joint and direction exist (hole_reacher.py:126-179, Env::wall_collision's
        // per-link test): only the joint positions stay live for the self-collision test
        // (base_reacher.py:105-119); q is read from the ring as it is needed
        double jx[NL + 1], jy[NL + 1];
        jx[0] = 0.0; jy[0] = 0.0;
        bool lim = false, wc = false;
        double ang = 0.0, x = 0.0, y = 0.0;
        double c0q = 0.0, s0q = 0.0;   // cos / sin of q[0] (the observation's)
#pragma unroll
        for (int d = 0; d < NL; ++d) {
          const double qv = rq[d * 64 + lane];
          lim |= qv > M_PI || qv < -M_PI;   // base_reacher.py:38-39,111
          ang = (d == 0) ? qv : ang + qv;
          double sn, cs;
          fgx_sincos(ang, &sn, &cs);
          if (d == 0) { c0q = cs; s0q = sn; }
          x = (d == 0) ? cs : x + cs;
          y = (d == 0) ? sn : y + sn;
          jx[d + 1] = 0.0 + x;
          jy[d + 1] = 0.0 + y;
          if (!allow_wall && !(jy[d] >= 0.0 && jy[d + 1] >= 0.0 && w_nd <= 0.0))
            wc |= Env<NL>::link_wall(w_left, w_right, w_nd, jx[d], jy[d], cs, sn);
        }
        bool sc = false;
        if (!allow_self) {
          sc = lim;
#pragma unroll
          for (int i = 0; i < NL; ++i)
#pragma unroll
            for (int j = i + 2; j < NL; ++j)
              sc |= (ccw(jx[i], jy[i], jx[j], jy[j], jx[j + 1], jy[j + 1]) !=
                     ccw(jx[i + 1], jy[i + 1], jx[j], jy[j], jx[j + 1], jy[j + 1])) &&
                    (ccw(jx[i], jy[i], jx[i + 1], jy[i + 1], jx[j], jy[j]) !=
                     ccw(jx[i], jy[i], jx[i + 1], jy[i + 1], jx[j + 1], jy[j + 1]));
        }
        const bool coll = sc || wc;   // hr_simple_reward.py:19-53
        const bool stop = coll || k == Lst - 1;
        if constexpr (INFO) {
          // the per-step rows of this sample (black_box_wrapper.py:218-227; the producer rewrites the last
          // sample's reward and pads every row past trajectory_length once the segment's end is known)
          const uint32_t e4 = (uint32_t)e * 4u, e8 = (uint32_t)e * 8u;
          const double* ra = gr + Lay::oRA + (size_t)((cpk & 1) * 2 + ci) * NL * 64;
          if (o.step_actions)
#pragma unroll
            for (int d = 0; d < NL; ++d) st_row(o.step_actions, (int64_t)k * NL + d, N, e8, ra[d * 64 + lane]);
          if (o.step_rewards)   // acc_cost * -5e-8 (hr_simple_reward.py:47)
            st_row(o.step_rewards, (int64_t)k, N, e8, gr[Lay::oPA + (k % kHpPA) * 64 + lane] * -5e-8);
          // the env info (hole_reacher.py:73-77, hr_simple_reward.py:33-53)
          if (o.end_effector) {
            st_row(o.end_effector, (int64_t)k * 2, N, e8, jx[NL]);
            st_row(o.end_effector, (int64_t)k * 2 + 1, N, e8, jy[NL]);
          }
          if (o.is_collided) {
            const bool sg = steps0 + k == 199 || coll;
            const bool succ = sg && norm2(jx[NL] - gx, jy[NL] - gy) < 0.005 && !coll;
            o.is_collided[(int64_t)k * N + e] = coll ? 1 : 0;
            o.is_success[(int64_t)k * N + e] = succ ? 1 : 0;
          }
          if (o.step_obs) {
            // emit_obs (hole_reacher.py:114-124, + TimeAwareObservation): cos q, sin q, q̇, hole width,
            // end effector - goal, steps [, steps / max_steps].  cos / sin of q[0] are FK's first angle's;
            // those of q[1..NL) through fgx_sincos_fast, each f32 checked against its error bound
            // (obs_trig_fast's margin), else the exact fgx_sincos
            const int X = c.full_dim;
            const int64_t r0 = (int64_t)k * X;
            st_row(o.step_obs, r0, N, e4, (float)c0q);
            st_row(o.step_obs, r0 + NL, N, e4, (float)s0q);
#pragma unroll
            for (int d = 1; d < NL; ++d) {
              const double qv = rq[d * 64 + lane];
              double sn, cs;
              fgx_sincos_fast(qv, &sn, &cs);
              bool ok = __builtin_fabs(qv) < 0x1p20;
              float fc = f32_checked(cs, 1e-15, ok), fs = f32_checked(sn, 1e-15, ok);
              if (!ok) {
                fgx_sincos(qv, &sn, &cs);
                fc = (float)cs;
                fs = (float)sn;
              }
              st_row(o.step_obs, r0 + d, N, e4, fc);
              st_row(o.step_obs, r0 + NL + d, N, e4, fs);
            }
#pragma unroll
            for (int d = 0; d < NL; ++d) st_row(o.step_obs, r0 + 2 * NL + d, N, e4, (float)ra[d * 64 + lane]);
            st_row(o.step_obs, r0 + 3 * NL, N, e4, (float)hw);
            st_row(o.step_obs, r0 + 3 * NL + 1, N, e4, (float)(jx[NL] - gx));
            st_row(o.step_obs, r0 + 3 * NL + 2, N, e4, (float)(jy[NL] - gy));
            const int stp = steps0 + k + 1;
            st_row(o.step_obs, r0 + 3 * NL + 3, N, e4, (float)stp);
            if (c.time_aware)
              st_row(o.step_obs, r0 + 3 * NL + 4, N, e4, (float)((double)stp / (double)c.max_steps));
          }
        }
        rs[((cpk & 1) * 2 + ci) * 64 + lane] = (uint8_t)((stop ? 1 : 0) | (coll ? 2 : 0));
        if (stop) {
          // a candidate final state: this sample ends the segment unless an earlier one does
          const double* ra = gr + Lay::oRA + (size_t)((cpk & 1) * 2 + ci) * NL * 64;
          double* cd = cand + (int64_t)(ci * CR) * N + e;
#pragma unroll
          for (int d = 0; d < NL; ++d) {
            cd[(int64_t)d * N] = rq[d * 64 + lane];
            cd[(int64_t)(NL + d) * N] = ra[d * 64 + lane];
          }
          own_done = true;
        }
      }
      chunk_barrier(it);
    }
#ifdef FGX_STAMPS
    FGX_HP_PUT(0, hp_t0);
    FGX_HP_PUT(1, __builtin_readcyclecounter());
    FGX_HP_PUT(8, hp_bar);
    FGX_HP_PUT(10, (unsigned long long)role);
#endif
    // the candidate states and this wave's rows complete before the producer reads the former and
    // overwrites rows past trajectory_length (a workgroup barrier does not wait for stores)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();   // (the candidate states are visible to the producer)
    return;
  }

  // ================================================================== producer
  Env<NL> v;
#pragma unroll
  for (int d = 0; d < NL; ++d) { v.q[d] = s.q[d * N + e]; v.qd[d] = s.qd[d * N + e]; }
  uint32_t flags = s.flags[e];
  const int s0 = c.replan ? steps0 : 0;
  Traj<MP, NL, NB, false, false> tg;
  tg.init(c, params + e * c.n_params, s.tables, s0, v.q, v.qd);
  // every valid lane's plan starts on one row (always without replanning): the basis rows come through
  // scalar loads (the constant address space), else per-lane loads of the same values
  const int s0u = __builtin_amdgcn_readfirstlane(s0);
  const bool s0_uni = __ballot(s0 != s0u) == 0;
  tg.stab = (cfloat_ptr)(uintptr_t)s.tables + (size_t)s0u * tg.str();
  const double act_lo = __builtin_canonicalize(c.act_lo), act_hi = __builtin_canonicalize(c.act_hi);
  const double pen = c.penalty;
  double* pa = gr + Lay::oPA;
  double pgx = 0.0, pgy = 0.0, phw = 0.0;   // (INFO: the observation's goal and hole width)
  if constexpr (INFO) { pgx = s.goal[e]; pgy = s.goal[N + e]; phw = s.hole[N + e]; }
  const uint32_t e4 = (uint32_t)e * 4u, e8 = (uint32_t)e * 8u;
  const int X = c.full_dim;
  const float fnan = __builtin_nanf("");
  const double dnan = __builtin_nan("");
  auto plan_rows = [&](int kk, const float* pos, const float* vel) __attribute__((always_inline)) {
    if constexpr (INFO) {
      if (o.positions)
#pragma unroll
        for (int d = 0; d < NL; ++d) {
          st_row(o.positions, (int64_t)kk * NL + d, N, e4, pos[d]);
          st_row(o.velocities, (int64_t)kk * NL + d, N, e4, vel[d]);
        }
    }
  };
  double* bl = gr + Lay::oBL;
  double* ff = gr + Lay::oFF;
  // resolution state: alive, segment length, terminated
  bool alive = valid;
  int L = 0;
  bool term = false;
  // numpy pairwise accumulators of committed full 8-blocks: level 1 (A) and the second half from
  // s = 64, 72 (B; 80, 88, 96 in LDS).  Every committed sample's reward is acc_cost * -5e-8: the only
  // other reward (a collision, env step 199) is the segment's last one, whose block is committed at
  // the end (hr_simple_reward.py:33-47)
  double A[8], B[kHpNR][8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    A[j] = 0.0;
#pragma unroll
    for (int q = 0; q < kHpNR; ++q) B[q][j] = 0.0;
  }
  auto plain = [&](int kk) __attribute__((always_inline)) { return pa[(kk % kHpPA) * 64 + lane] * -5e-8; };
  // block b8 / 8 into the level-1 sums and the second halves that have started; x(j): reward of 8b + j
  auto commit = [&](int b8, auto x) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const double r = x(j);
      if (b8 < 128) A[j] = (b8 == 0) ? r : A[j] + r;
#pragma unroll
      for (int q = 0; q < kHpNS; ++q) {
        const int sq = kHpS0 + 8 * q;
        if (sq > b8) continue;
        if (q < kHpNR) {
          B[q][j] = (sq == b8) ? r : B[q][j] + r;
        } else {
          double* bp = bl + ((q - kHpNR) * 8 + j) * 64 + lane;
          *bp = (sq == b8) ? r : *bp + r;
        }
      }
    }
  };
  int it_end = 0;
  int kp = 0;   // (INFO) the env's plan rows written so far
  for (int it = 0;; ++it) {
    it_end = it;
    const int rp = (it + 1) & 1;
    if (all_done(rp) || it > itmax) break;
#ifdef FGX_STAMPS
    const unsigned long long tr0 = __builtin_readcyclecounter();
#endif
    // ---- resolve chunk cr = it - 2 (its consumers' stop codes were staged before the last barrier)
    if (it >= 2) {
      const int cr = it - 2;
      if (alive) {
        const uint8_t c0 = rs[((cr & 1) * 2) * 64 + lane], c1 = rs[((cr & 1) * 2 + 1) * 64 + lane];
        if (c0 & 1) { L = 2 * cr + 1; term = (c0 & 2) != 0; alive = false; }
        else if (c1 & 1) { L = 2 * cr + 2; term = (c1 & 2) != 0; alive = false; }
        // samples 8b .. 8b + 7 all counted, none of them the last: commit block b
        if (alive && (cr & 3) == 3) {
          const int b8 = 2 * cr - 6;   // = 8 b
          commit(b8, [&](int j) { return plain(b8 + j); });
          const int sn = b8 + 8;   // block(0, sn) for a split start sn
          if (sn >= kHpS0 && sn <= kHpS0 + 8 * (kHpNS - 1)) ff[((sn - kHpS0) / 8) * 64 + lane] = PairwiseSum::comb(A);
        }
      }
    }
    {
      const uint64_t am = __ballot(alive);
      if (lane == 0) al[it & 1] = am;
    }
#ifdef FGX_STAMPS
    const unsigned long long tr1 = __builtin_readcyclecounter();
    hp_res += tr1 - tr0;
#endif
    // ---- produce chunk it (samples 2 it, 2 it + 1) into buffer it & 1
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int k = 2 * it + i;
      if (alive && k < Lst) {
        float pos[NL], vel[NL];
        if (s0_uni) tg.template at<false, true>(c, k, pos, vel);   // rows by scalar loads: never queued
        else tg.at(c, k, pos, vel);                                // behind the row stores (vmcnt)
        plan_rows(k, pos, vel);
        kp = k + 1;
        // tracking controller + clip (black_box_wrapper.py:201-205; np.clip propagates NaN)
        double a[NL];
        float a32[NL];
#pragma unroll
        for (int d = 0; d < NL; ++d) {
          if (CTRL == CTRL_PD) {
            const double u = fadd(c.pg[d] * fsub((double)pos[d], v.q[d]), c.dg[d] * fsub((double)vel[d], v.qd[d]));
            const double cl = __builtin_fmin(__builtin_fmax(u, act_lo), act_hi);
            a[d] = (u != u) ? u : cl;
            a32[d] = 0.0f;
          } else {
            const float u = (CTRL == CTRL_VEL) ? vel[d] : pos[d];
            a32[d] = np_clipf(u, c.act_lo32, c.act_hi32);
            a[d] = (double)a32[d];
          }
        }
        // np.sum(self._acc ** 2) (hr_simple_reward.py:48), acc = (a - q̇) / dt
        // (base_reacher_direct.py:25): f32 once q̇ holds a float32 array (substep, fgx_kernels.h)
        double acc_cost;
        if (F32 && (flags & 1u)) {
          float sq[NL];
#pragma unroll
          for (int d = 0; d < NL; ++d) {
            const float ac = div_rcp(a32[d] - (float)v.qd[d], c.dt32, c.rcp_dt32);
            sq[d] = ac * ac;
          }
          acc_cost = (double)np_sum<NL, float>([&](int d) { return sq[d]; }, [](float x, float y) { return x + y; });
        } else {
          double sq[NL];
#pragma unroll
          for (int d = 0; d < NL; ++d) {
            const double ac = div_rcp64(a[d] - v.qd[d], c.dt, c.rcp_dt);
            sq[d] = ac * ac;
          }
          acc_cost = np_sum<NL, double>([&](int d) { return sq[d]; }, [](double x, double y) { return x + y; });
        }
        pa[(k % kHpPA) * 64 + lane] = acc_cost;
        double* rq = gr + Lay::oRQ + (size_t)((it & 1) * 2 + i) * NL * 64;
        double* ra = gr + Lay::oRA + (size_t)((it & 1) * 2 + i) * NL * 64;
        // q̇ = a; q += dt q̇ (base_reacher_direct.py:26-27)
#pragma unroll
        for (int d = 0; d < NL; ++d) {
          v.qd[d] = a[d];
          const double inc = F32 ? (double)(c.dt32 * a32[d]) : c.dt * v.qd[d];
          v.q[d] = v.q[d] + inc;
          rq[d * 64 + lane] = v.q[d];
          ra[d * 64 + lane] = v.qd[d];
        }
        if (F32) flags |= 1u;
      }
    }
#ifdef FGX_STAMPS
    hp_prod += __builtin_readcyclecounter() - tr1;
#endif
    chunk_barrier(it);
  }
#ifdef FGX_STAMPS
  FGX_HP_PUT(0, hp_t0);
  FGX_HP_PUT(1, __builtin_readcyclecounter());
  FGX_HP_PUT(8, hp_bar);
  FGX_HP_PUT(9, (unsigned long long)it_end);
  FGX_HP_PUT(10, 0ull);
  FGX_HP_PUT(11, hp_res);
  FGX_HP_PUT(12, hp_prod);
#endif
  if constexpr (INFO) {
    // the rest of every env's plan (black_box_wrapper.py:245-246: the full desired trajectory); the
    // sample index stays wave-uniform (the row stores' base is), lanes join at their own kp
    const int kmin = wave_min(valid ? kp : T);
    for (int k = kmin; k < T; ++k) {
      if (valid && k >= kp) {
        float pos[NL], vel[NL];
        if (s0_uni) tg.template at<false, true>(c, k, pos, vel);
        else tg.at(c, k, pos, vel);
        plan_rows(k, pos, vel);
      }
    }
  }
  __syncthreads();   // the consumers' candidate states and info rows are visible
  // the wave's inner steps: one atomic per wave (all lanes active here)
  if (o.inner_steps) {
    long long sum = valid ? L : 0;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off, 64);
    count_inner(o.inner_steps, sum, lane == 0);
  }
  const int Lmin = wave_min(valid ? L : T);   // (INFO padding: wave-uniform rows from here)
  if (!valid) return;
  const int own = (L - 1) & 1;   // the consumer that ran the last sample
  const double* cd = cand + (int64_t)(own * CR) * N + e;
  // the last sample's reward: np.dot([dist^2, acc, coll], [-1, -5e-8, -penalty]) at a collision or at
  // env step 199, else acc * -5e-8 (hr_simple_reward.py:33-47)
  const double acc_l = pa[((L - 1) % kHpPA) * 64 + lane];
  const bool special = term || steps0 + L - 1 == 199;
  double dist2 = 0.0;
  if (special) {
    // |ee - goal|^2 of the final state (the consumer's candidate): Env::fk once per env rather than at
    // every stop sample a consumer meets (one lane's stop costs the whole wave the branch)
    Env<NL> f;
#pragma unroll
    for (int d = 0; d < NL; ++d) f.q[d] = cd[(int64_t)d * N];
    f.fk();
    const double dist = norm2(f.jx[NL] - s.goal[e], f.jy[NL] - s.goal[N + e]);
    dist2 = dist * dist;
  }
  const double rfin = special ? __builtin_fma(term ? 1.0 : 0.0, -pen, __builtin_fma(acc_l, -5e-8, dist2 * -1.0))
                              : acc_l * -5e-8;
  auto reward_of = [&](int kk) __attribute__((always_inline)) { return kk == L - 1 ? rfin : plain(kk); };
  // ---- the return: numpy pairwise sum of the L counted rewards (umath pairwise_sum: block(0, L) for
  // L <= 128, else block(0, s) + block(s, L - s), s = (L / 2) & ~7; a block of >= 8 = its 8 slot sums
  // combined, then the remainder added in order)
  double ret;
  if (L < 8) {
    ret = 0.0;
    for (int k = 0; k < L; ++k) ret = ret + reward_of(k);
  } else {
    if ((L & 7) == 0) commit(L - 8, [&](int j) { return reward_of(L - 8 + j); });   // the last block
    double r8[8];
    const int sfin = (L > 128) ? ((L / 2) & ~7) : 0;
    const int qs = (sfin - kHpS0) / 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      double x = A[j];
#pragma unroll
      for (int q = 0; q < kHpNS; ++q)
        if (L > 128 && q == qs) x = (q < kHpNR) ? B[q][j] : bl[((q - kHpNR) * 8 + j) * 64 + lane];
      r8[j] = x;
    }
    double u = PairwiseSum::comb(r8);
    for (int k = L & ~7; k < L; ++k) u = u + reward_of(k);
    ret = (L > 128) ? ff[qs * 64 + lane] + u : u;
  }
  if constexpr (INFO) {
    if (o.step_rewards) o.step_rewards[(int64_t)(L - 1) * N + e] = rfin;   // (per-lane row: no st_row)
    // the consumers' rows after trajectory_length (written by them for samples they ran past it, or
    // never written): NaN, 0 for the flags (black_box_wrapper.py:244-249)
    for (int k = Lmin; k < T; ++k) {
      if (k < L) continue;   // (the row index stays wave-uniform for the row stores)
      if (o.step_actions)
#pragma unroll
        for (int d = 0; d < NL; ++d) st_row(o.step_actions, (int64_t)k * NL + d, N, e8, dnan);
      if (o.step_rewards) st_row(o.step_rewards, (int64_t)k, N, e8, dnan);
      if (o.step_obs)
        for (int p = 0; p < X; ++p) st_row(o.step_obs, (int64_t)k * X + p, N, e4, fnan);
      if (o.end_effector) {
        st_row(o.end_effector, (int64_t)k * 2, N, e8, dnan);
        st_row(o.end_effector, (int64_t)k * 2 + 1, N, e8, dnan);
      }
      if (o.is_collided) {
        o.is_collided[(int64_t)k * N + e] = 0;
        o.is_success[(int64_t)k * N + e] = 0;
      }
    }
  }
  // the BB-step outputs; k_hp_finish (below) completes the env: its final state, FK, the final
  // observation and the VectorEnv auto-reset (episode_epilogue)
  o.ret[e] = ret;
  o.term[e] = term;
  o.trunc[e] = steps0 + L >= c.max_steps;
  o.tlen[e] = L;
}

// The episode epilogue of k_episode_hp's envs, one thread per env at full occupancy (in the pipeline
// kernel its registers — PCG64 draws and rejection loops of the reset, FK, two observations — would
// exceed the three-waves-per-SIMD budget): the final state is the candidate of the consumer that ran
// the last sample; outputs, final observation, auto-reset and state write-back as k_episode's
// (episode_epilogue, black_box_wrapper.py:241-253).
template <int NL, bool F32>
__global__ __launch_bounds__(256) void k_hp_finish(DevCfg c, DevState s, Outputs o) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= c.N) return;
  const int64_t N = c.N;
  constexpr int CR = hp_cand_rows<NL>();
  const int L = o.tlen[e];
  const double* cd = s.rew + (int64_t)(((L - 1) & 1) * CR) * N + e;
  Env<NL> f;
  load_env(c, s, e, f);
#pragma unroll
  for (int d = 0; d < NL; ++d) {
    f.q[d] = cd[(int64_t)d * N];
    f.qd[d] = cd[(int64_t)(NL + d) * N];
  }
  f.steps += L;
  if (F32) f.flags |= 1u;
  f.fk();
  episode_epilogue(c, s, o, e, f, s.plans[e] + 1, L, o.ret[e], o.term[e] != 0, o.trunc[e] != 0, false);
}

inline size_t hp_lds_bytes(int nl, int groups) {
  return (size_t)groups * (nl == 5 ? HpLayout<5>::GROUP : HpLayout<2>::GROUP) * sizeof(double);
}
static_assert(4 * HpLayout<5>::GROUP * sizeof(double) <= 160 * 1024, "k_episode_hp: four groups fit one CU's LDS");

// k_episode_hp serves this step (FGX_HP=0 or any FGX_EPISODE_KERNEL but "hp" keep the others: A/B, tests)
// log: some per-step array is written (the INFO instantiation; FGX_V2=0 keeps the logging k_episode)
// heavy: the verbose-2 rows (planned positions / velocities, step observations): k_episode_v2h stays
// faster there (65536 envs: 1026 vs 1637 us, profiles/r05_s9_jlhelper_traj_hpinfo.jsonl), so k_episode_hp takes
// them only when forced (FGX_HP=1); FGX_HP=0 never takes it
inline bool hp_applies(const DevCfg& c, const DevState& s, int mp, bool log, bool heavy, bool per_env_plans) {
  bool force = false;
  if (const char* v = std::getenv("FGX_HP")) {
    if (std::strcmp(v, "0") == 0) return false;
    force = std::strcmp(v, "1") == 0;
  }
  if (heavy && !force) return false;
  // a forced kernel wins (fgx_dispatch.h): any FGX_EPISODE_KERNEL other than "hp" keeps k_episode_hp out
  if (const char* v = std::getenv("FGX_EPISODE_KERNEL"))
    if (*v && std::strcmp(v, "hp") != 0) return false;
  if (log)
    if (const char* v = std::getenv("FGX_V2"))
      if (std::strcmp(v, "0") == 0) return false;
  return c.env == ENV_HOLE && c.rew_fct == REW_SIMPLE && c.nl == 5 && c.nb == 5 &&
         (mp == MP_PROMP || mp == MP_DMP || mp == MP_PRODMP) && !per_env_plans && !c.learn_tau && !c.learn_delay &&
         !c.sched_state && !c.cond_desired && c.valid_flags == 0 && c.max_steps <= 200 && c.T <= 256 &&
         s.rew != nullptr;
}

}  // namespace fgx

// fgx_ep_hp.hip
int fgx_launch_episode_hp(const fgx::DevCfg& c, const fgx::DevState& s, int mp, const float* params,
                          const fgx::Outputs& o, hipStream_t stream, std::string& err);
