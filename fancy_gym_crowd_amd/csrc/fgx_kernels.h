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
//   k_traj_valu   desired trajectories [N, T, dof] (reference path for k_traj_mfma)
//   k_traj_mfma   desired trajectories as an f32 MFMA GEMM (v_mfma_f32_32x32x2_f32)
#pragma once
#include <type_traits>

#include "fgx_device.h"

namespace fgx {

// ============================================================================ obs
// Env observation (simple_reacher.py:75-83 / hole_reacher.py:114-124) [+ t/max_steps,
// utils/wrappers.py:58-59], context-masked when `ctx` (black_box_wrapper.py:90-95), written
// straight to up to two destinations (no private arrays: nothing spills to scratch).
// fresh: v was just reset (Env::reset): q = [q0, +0, ..., +0] and fk() has run, so cos / sin of
// q0 are FK's c[0] / s[0] (the same sincos of the same angle) and those of +0 are exactly 1 / +0.
// fk0: FK is current for q (k_episode's epilogue), so cos / sin of q[0] are c[0] / s[0].
// gcs / gsn (optional): cos / sin of every q[k], computed elsewhere with the same sincos
// s1: element stride of d1 (the per-step observations: the lane's column of the wave's LDS staging
// slots, stride 64, InfoStage)
// skip_q: cos / sin of q[1..NL) are left as NaN placeholders (k_episode_v2h: the storing wave writes
// them, from the staged q, before the row leaves; it skips a NaN q, whose cos / sin are NaN anyway --
// a padded row, or a running env whose state went NaN through NaN parameters)
template <int NL>
__device__ __forceinline__ void emit_obs(const DevCfg& c, const Env<NL>& v, bool ctx, float* d1, float* d2,
                                         bool fresh = false, bool fk0 = false, const double* gcs = nullptr,
                                         const double* gsn = nullptr, int s1 = 1, bool skip_q = false) {
  const bool rs = !ctx || c.random_start;
  int p = 0;
  auto put = [&](float x) {
    if (d1) d1[p * s1] = x;
    if (d2) d2[p] = x;
    ++p;
  };
  if (rs) {
    double sn[NL], cs[NL];
    if (fresh) {
      cs[0] = v.c[0];
      sn[0] = v.s[0];
#pragma unroll
      for (int k = 1; k < NL; ++k) { cs[k] = 1.0; sn[k] = 0.0; }
    } else {
#pragma unroll
      for (int k = 0; k < NL; ++k) {
        if (gcs) { cs[k] = gcs[k]; sn[k] = gsn[k]; }
        else if (k == 0 && fk0) { cs[0] = v.c[0]; sn[0] = v.s[0]; }   // FK's first angle is q[0]
        else if (skip_q) { cs[k] = __builtin_nan(""); sn[k] = __builtin_nan(""); }
        else fgx_sincos(v.q[k], &sn[k], &cs[k]);
      }
    }
#pragma unroll
    for (int k = 0; k < NL; ++k) put((float)cs[k]);
#pragma unroll
    for (int k = 0; k < NL; ++k) put((float)sn[k]);
#pragma unroll
    for (int k = 0; k < NL; ++k) put((float)v.qd[k]);
  }
  if (c.env == ENV_HOLE && (!ctx || c.rand_width)) put((float)v.hw);
  if (c.env == ENV_VIA && (!ctx || c.rand_via)) {   // viapoint_reacher.py:116-126
    put((float)(v.jx[NL] - v.hx));
    put((float)(v.jy[NL] - v.hw));
  }
  put((float)(v.jx[NL] - v.gx));
  put((float)(v.jy[NL] - v.gy));
  if (!ctx) {
    put((float)v.steps);
    if (c.time_aware) put((float)((double)v.steps / (double)c.max_steps));
  }
}

// ============================================================================ state I/O
// hole: the hole / via-point / reward-state arrays take part (SimpleReacher never reads or changes
// them — k_reset zeroes them — so its episode kernels neither load nor store them: no registers
// held across the sample loop for them)
template <int NL>
__device__ __forceinline__ void load_env(const DevCfg& c, const DevState& s, int64_t e, Env<NL>& v,
                                         bool hole = true) {
  const int64_t N = c.N;
#pragma unroll
  for (int k = 0; k < NL; ++k) { v.q[k] = s.q[k * N + e]; v.qd[k] = s.qd[k * N + e]; }
  v.gx = s.goal[e]; v.gy = s.goal[N + e];
  v.ex = v.ey = v.cd = 0.0;
  if (!hole) {
    v.hx = v.hw = v.hd = 0.0;
    v.steps = s.steps[e];
    v.flags = s.flags[e];
    return;
  }
  v.hx = s.hole[e]; v.hw = s.hole[N + e]; v.hd = s.hole[2 * N + e];
  if (c.env == ENV_HOLE && c.rew_fct != REW_SIMPLE) { v.ex = s.aux[e]; v.ey = s.aux[N + e]; v.cd = s.aux[2 * N + e]; }
  v.steps = s.steps[e];
  v.flags = s.flags[e];
}

template <int NL>
__device__ __forceinline__ void store_env(const DevCfg& c, const DevState& s, int64_t e, const Env<NL>& v,
                                          bool hole = true) {
  const int64_t N = c.N;
#pragma unroll
  for (int k = 0; k < NL; ++k) { s.q[k * N + e] = v.q[k]; s.qd[k * N + e] = v.qd[k]; }
  s.goal[e] = v.gx; s.goal[N + e] = v.gy;
  if (!hole) {
    s.steps[e] = v.steps;
    s.flags[e] = v.flags;
    return;
  }
  s.hole[e] = v.hx; s.hole[N + e] = v.hw; s.hole[2 * N + e] = v.hd;
  if (c.env == ENV_HOLE && c.rew_fct != REW_SIMPLE) { s.aux[e] = v.ex; s.aux[N + e] = v.ey; s.aux[2 * N + e] = v.cd; }
  s.steps[e] = v.steps;
  s.flags[e] = v.flags;
}

// ============================================================================ reset
// An unseeded reset of env e in registers (VectorEnv auto-reset: env.reset() without options, so
// the constructor's random_start): the PCG64 stream continues; the start angle is restored
// (random_start False) or drawn and kept (True).  Callers store the env state afterwards.
template <int NL>
__device__ __forceinline__ void autoreset_env(const DevCfg& c, const DevState& s, int64_t e, Env<NL>& v) {
  Pcg64 rg = load_rng(s.rng, c.N, e);
  if (!c.random_start) v.sp = s.start[e];
  v.reset(c, rg, false, 0);
  store_rng(s.rng, c.N, e, rg);
  if (c.random_start) s.start[e] = v.sp;
}

// rs_mode: -1 = the constructor's random_start, 0 / 1 = reset(options={'random_start': ...})
// (base_reacher.py:77-80).  Envs outside the mask are not reset; their current observation is
// written to their obs row.
template <int NL>
__global__ __launch_bounds__(256) void k_reset(DevCfg c, DevState s, const uint64_t* seeds, const uint8_t* mask,
                                               int rs_mode, float* obs) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= c.N) return;
  Env<NL> v;
  if (mask && !mask[e]) {
    if (obs) {
      load_env(c, s, e, v);
      v.fk();
      emit_obs(c, v, c.return_context, obs + e * c.out_dim, nullptr);
    }
    return;
  }
  const bool rs = rs_mode < 0 ? c.random_start != 0 : rs_mode != 0;
  Pcg64 r = load_rng(s.rng, c.N, e);
  v.sp = s.start[e];
  v.reset(c, r, seeds != nullptr, seeds ? seeds[e] : 0, rs);
  store_rng(s.rng, c.N, e, r);
  if (rs) s.start[e] = v.sp;
  store_env(c, s, e, v);
  s.plans[e] = 0;
  s.flags[e] = 0;
  if (obs) emit_obs(c, v, c.return_context, obs + e * c.out_dim, nullptr);
}

// ============================================================================ trajectories
// Per-thread desired-trajectory generator (oracle/mp.py:trajectory), f32 throughout.
// NB: basis functions per dof; NB = 0 is the generic instantiation with the runtime c.nb
// (<= kGenBasis), whose chains run over compile-time slots guarded by j < nb (same fma order).
// DIVREF: divide by tau with the IEEE division (per-env learned tau, for which the reciprocal
// shortcut div_rcp is not verified) instead of div_rcp.
constexpr int kGenBasis = 12;

// PAIRS: the ProDMP joint-pair contraction (PKD) is allowed (k_episode takes it for SimpleReacher:
// -5% at 65536 envs; the register-bound HoleReacher body measured +2% with it,
// profiles/r03_ab_s4.jsonl)
template <int MP, int NL, int NB, bool DIVREF = false, bool PAIRS = true>
struct Traj {
  static constexpr int NBM = NB ? NB : kGenBasis;           // weight slots per dof
  static constexpr int K = (MP == MP_PRODMP) ? NBM + 3 : NBM;
  // ProMP with >= 2 joints runs the basis contraction on joint pairs (v_pk_fma_f32 / v_pk_mul_f32 /
  // v_pk_add_f32: two independent IEEE f32 ops per lane and instruction, so each joint's result is
  // bit-identical to the scalar chain); an odd last joint rides in the low half of a pair whose
  // high half is zero.
  static constexpr bool PK = (MP == MP_PROMP) && NL >= 2;
  // ProDMP with >= 2 joints: the two basis contractions (position, velocity) on joint pairs likewise
#ifdef FGX_NO_PKD   // A/B builds only: the scalar chains
  static constexpr bool PKD = false;
#else
  static constexpr bool PKD = PAIRS && (MP == MP_PRODMP) && NL >= 2;
#endif
  static constexpr int NLP = (NL + 1) / 2;
  float w[(PK || PKD) ? 1 : NL][K]; // ProMP (1 joint): w ; DMP: w' ; ProDMP (1 joint): [w' (NBM slots), g', c1, c2]
  f32x2 wp[PK ? NLP : 1][PK ? NBM : 1];   // ProMP (>= 2 joints): weights of joints (2p, 2p + 1)
  f32x2 wq[PKD ? NLP : 1][PKD ? K : 1];   // ProDMP (>= 2 joints): [w', g', c1, c2] of joints (2p, 2p + 1)
  f32x2 cur2[PK ? NLP : 1], vprev2[PK ? NLP : 1];
  float g[NL];             // DMP goal
  float y[NL], z[NL];      // DMP state
  float cur[NL], vprev[NL];// ProMP look-ahead (1 joint)
  const float* tab;        // row s0 of the basis table: plan sample k reads rows k + 1, k + 2
  cfloat_ptr stab;         // the same row in global memory through the constant address space,
                           // wave-uniform (fast blocks: rows land in SGPRs via s_load)
  int stride, T, nbr;
  float tau32, rtau32;
  // table row stride, compile-time for a fixed basis count (build_devcfg in fgx_api.hip): every
  // row address of an unrolled sample block is then a constant offset from one base
  static constexpr int KS = NB ? ((MP == MP_PRODMP) ? 2 * (NB + 1) + 4 : (NB + 2 + 3) & ~3) : 0;

  // weight j of joint d (any layout)
  __device__ __forceinline__ float wt(int d, int j) const {
    if constexpr (PK) return (d & 1) ? wp[d >> 1][j].y : wp[d >> 1][j].x;
    else if constexpr (PKD) return (d & 1) ? wq[d >> 1][j].y : wq[d >> 1][j].x;
    else return w[d][j];
  }
  __device__ __forceinline__ int nb() const { return NB ? NB : nbr; }
  __device__ __forceinline__ int str() const { return KS ? KS : stride; }
  __device__ __forceinline__ float div_tau(float x) const { return DIVREF ? x / tau32 : div_rcp(x, tau32, rtau32); }

  // k-ordered f32 fma chain over the nb basis slots (== f32-input MFMA numerics)
  template <typename P>
  __device__ __forceinline__ float chain(P row, const float* wd) const {
    float acc = 0.0f;
#pragma unroll
    for (int j = 0; j < NBM; ++j)
      if (NB || j < nbr) acc = __builtin_fmaf(row[j], wd[j], acc);
    return acc;
  }
  // the same chain on a joint pair (the table entry is broadcast to both halves)
  template <typename P>
  __device__ __forceinline__ f32x2 chain2(P row, const f32x2* wd) const {
    f32x2 acc = {0.0f, 0.0f};
#pragma unroll
    for (int j = 0; j < NBM; ++j)
      if (NB || j < nbr) acc = __builtin_elementwise_fma((f32x2)row[j], wd[j], acc);
    return acc;
  }
  // ProDMP: [basis (nb), goal, y1, y2] . [w', g', c1, c2]; h holds the 3 tail entries at NBM..NBM+2
  __device__ __forceinline__ float chain3(const float* h, const float* wd) const {
    float acc = chain(h, wd);
    acc = __builtin_fmaf(h[NBM], wd[NBM], acc);
    acc = __builtin_fmaf(h[NBM + 1], wd[NBM + 1], acc);
    return __builtin_fmaf(h[NBM + 2], wd[NBM + 2], acc);
  }
  // the same chain on a joint pair
  __device__ __forceinline__ f32x2 chain3_2(const float* h, const f32x2* wd) const {
    f32x2 acc = chain2(h, wd);
    acc = __builtin_elementwise_fma((f32x2)h[NBM], wd[NBM], acc);
    acc = __builtin_elementwise_fma((f32x2)h[NBM + 1], wd[NBM + 1], acc);
    return __builtin_elementwise_fma((f32x2)h[NBM + 2], wd[NBM + 2], acc);
  }
  __device__ __forceinline__ f32x2 div_tau2(f32x2 x) const {
    if constexpr (DIVREF) return x / (f32x2)tau32;   // two IEEE divisions
    const f32x2 q = x * rtau32;                       // div_rcp on the pair
    const f32x2 e = __builtin_elementwise_fma(-q, (f32x2)tau32, x);
    return __builtin_elementwise_fma(e, (f32x2)rtau32, q);
  }

  // params: this env's row of the [N, n_params] matrix; q0/qd0 the initial conditions
  __device__ __forceinline__ void init(const DevCfg& c, const float* params, const float* tab_, int s0_,
                                       const double* q0, const double* qd0) {
    init(c, params, tab_, s0_, q0, qd0, c.T, c.tau32, c.rcp_tau32);
  }
  // T_ / tau32_: this plan's length and tau (learned tau, sub-trajectories).  goff: offset of the
  // DMP goal entries in params (default NL * nb; the per-joint generators of k_episode_jp pass
  // params + d * nb and the offset of goal d, c.nl * nb + d - d * nb).
  __device__ __forceinline__ void init(const DevCfg& c, const float* params, const float* tab_, int s0_,
                                       const double* q0, const double* qd0, int T_, float tau32_, float rtau32_,
                                       int goff = -1) {
    stride = c.stride; T = T_; tau32 = tau32_; rtau32 = rtau32_; nbr = c.nb;
    tab = tab_ + (size_t)s0_ * str();
    const int n = nb();
    if (MP == MP_PROMP && PK) {
#pragma unroll
      for (int p = 0; p < NLP; ++p)
#pragma unroll
        for (int j = 0; j < NBM; ++j) {
          wp[p][j].x = (NB || j < n) ? params[2 * p * n + j] : 0.0f;
          wp[p][j].y = ((NB || j < n) && 2 * p + 1 < NL) ? params[(2 * p + 1) * n + j] : 0.0f;
        }
      const float* r1 = tab + str();
#pragma unroll
      for (int p = 0; p < NLP; ++p) { cur2[p] = chain2(r1, wp[p]); vprev2[p] = (f32x2)0.0f; }
    } else if (MP == MP_PROMP) {
#pragma unroll
      for (int d = 0; d < NL; ++d)
#pragma unroll
        for (int j = 0; j < NBM; ++j) w[d][j] = (NB || j < n) ? params[d * n + j] : 0.0f;
      const float* r1 = tab + str();
#pragma unroll
      for (int d = 0; d < NL; ++d) { cur[d] = chain(r1, w[d]); vprev[d] = 0.0f; }
    } else if (MP == MP_DMP) {
#pragma unroll
      for (int d = 0; d < NL; ++d) {
#pragma unroll
        for (int j = 0; j < NBM; ++j) w[d][j] = (NB || j < n) ? params[d * n + j] * c.ws32 : 0.0f;
        g[d] = params[(goff < 0 ? NL * n : goff) + d] * c.gs32;
        y[d] = (float)q0[d];
        z[d] = (float)qd0[d] * tau32;
      }
    } else if (MP == MP_PRODMP) {
      const float* rb = tab;
      const float y1 = rb[2 * n + 2], y2 = rb[2 * n + 3], dy1 = rb[2 * n + 4], dy2 = rb[2 * n + 5];
      const float det = y1 * dy2 - y2 * dy1;
      float hp[NBM + 1], hv[NBM + 1];
#pragma unroll
      for (int j = 0; j < NBM; ++j) {
        hp[j] = (NB || j < n) ? rb[j] : 0.0f;
        hv[j] = (NB || j < n) ? rb[n + 1 + j] : 0.0f;
      }
      hp[NBM] = rb[n];
      hv[NBM] = rb[2 * n + 1];
#pragma unroll
      for (int d = 0; d < NL; ++d) {
        float wd[K];
#pragma unroll
        for (int j = 0; j < NBM; ++j) wd[j] = (NB || j < n) ? params[d * (n + 1) + j] * c.ws32 : 0.0f;
        wd[NBM] = params[d * (n + 1) + n] * c.gs32;
        // P, V = [basis, goal] . [w', g'] (chain over nb + 1 entries)
        float P = __builtin_fmaf(hp[NBM], wd[NBM], chain(hp, wd));
        float V = __builtin_fmaf(hv[NBM], wd[NBM], chain(hv, wd));
        const float A = (float)q0[d] - P;
        const float B = (float)qd0[d] * tau32 - V;
        wd[NBM + 1] = (dy2 * A - y2 * B) / det;
        wd[NBM + 2] = (y1 * B - dy1 * A) / det;
#pragma unroll
        for (int j = 0; j < K; ++j) {
          if constexpr (PKD) {
            if (d & 1) wq[d >> 1][j].y = wd[j];
            else wq[d >> 1][j] = (f32x2){wd[j], 0.0f};   // (an odd last joint: zero high half)
          } else {
            w[d][j] = wd[j];
          }
        }
      }
    }
  }

  // desired (pos, vel) of plan sample k (row s0 + k + 1); call with k = 0, 1, 2, ...
  // MID: the caller guarantees k < T - 1 (no last-sample branch)
  // SC: read the rows through stab (k and stab wave-uniform)
  template <bool MID = false, bool SC = false>
  __device__ __forceinline__ void at(const DevCfg& c, int k, float* pos, float* vel) {
    if constexpr (SC) at_rows<MID>(c, k, stab + (size_t)(k + 1) * str(), pos, vel);
    else at_rows<MID>(c, k, tab + (size_t)(k + 1) * str(), pos, vel);
  }
  template <bool MID, typename RowPtr>
  __device__ __forceinline__ void at_rows(const DevCfg& c, int k, RowPtr row, float* pos, float* vel) {
    const int n = nb();
    if (MP == MP_PROMP && PK) {
      if (MID || k < T - 1) {
        const auto nrow = row + str();
        const float dti = row[n], rdt = row[n + 1];
#pragma unroll
        for (int p = 0; p < NLP; ++p) {
          const f32x2 nx = chain2(nrow, wp[p]);
          const f32x2 x = nx - cur2[p];
          const f32x2 q = x * rdt;                                    // div_rcp on the pair
          const f32x2 er = __builtin_elementwise_fma(-q, (f32x2)dti, x);
          const f32x2 vl = __builtin_elementwise_fma(er, (f32x2)rdt, q);
          pos[2 * p] = cur2[p].x;
          vel[2 * p] = vl.x;
          if (2 * p + 1 < NL) { pos[2 * p + 1] = cur2[p].y; vel[2 * p + 1] = vl.y; }
          cur2[p] = nx;
          vprev2[p] = vl;
        }
      } else {
#pragma unroll
        for (int p = 0; p < NLP; ++p) {
          pos[2 * p] = cur2[p].x;
          vel[2 * p] = vprev2[p].x;
          if (2 * p + 1 < NL) { pos[2 * p + 1] = cur2[p].y; vel[2 * p + 1] = vprev2[p].y; }
        }
      }
    } else if (MP == MP_PROMP) {
      if (MID || k < T - 1) {
        const auto nrow = row + str();
        const float dti = row[n], rdt = row[n + 1];
#pragma unroll
        for (int d = 0; d < NL; ++d) {
          const float nx = chain(nrow, w[d]);
          pos[d] = cur[d];
          vel[d] = div_rcp(nx - cur[d], dti, rdt);
          cur[d] = nx;
          vprev[d] = vel[d];
        }
      } else {
#pragma unroll
        for (int d = 0; d < NL; ++d) { pos[d] = cur[d]; vel[d] = vprev[d]; }
      }
    } else if (MP == MP_DMP) {
      const float sdt = row[n];
#pragma unroll
      for (int d = 0; d < NL; ++d) {
        pos[d] = y[d];
        vel[d] = div_tau(z[d]);
        if (MID || k < T - 1) {
          const float f = chain(row, w[d]);
          const float acc = c.alpha32 * (c.beta32 * (g[d] - y[d]) - z[d]) + f;
          z[d] = z[d] + sdt * acc;
          y[d] = y[d] + sdt * z[d];
        }
      }
    } else if (MP == MP_PRODMP) {
      float hp[K], hv[K];
#pragma unroll
      for (int j = 0; j < NBM; ++j) {
        hp[j] = (NB || j < n) ? row[j] : 0.0f;
        hv[j] = (NB || j < n) ? row[n + 1 + j] : 0.0f;
      }
      hp[NBM] = row[n]; hv[NBM] = row[2 * n + 1];
      hp[NBM + 1] = row[2 * n + 2]; hp[NBM + 2] = row[2 * n + 3];
      hv[NBM + 1] = row[2 * n + 4]; hv[NBM + 2] = row[2 * n + 5];
      if constexpr (PKD) {
#pragma unroll
        for (int p = 0; p < NLP; ++p) {
          const f32x2 ps = chain3_2(hp, wq[p]);
          const f32x2 vs = div_tau2(chain3_2(hv, wq[p]));
          pos[2 * p] = ps.x;
          vel[2 * p] = vs.x;
          if (2 * p + 1 < NL) { pos[2 * p + 1] = ps.y; vel[2 * p + 1] = vs.y; }
        }
      } else {
#pragma unroll
        for (int d = 0; d < NL; ++d) {
          pos[d] = chain3(hp, w[d]);
          vel[d] = div_tau(chain3(hv, w[d]));
        }
      }
    }
  }
};

// ============================================================================ env substep
// One env.step with the (clipped) action a (f64) / a32 (when the action array is float32).
// base_reacher_torque.py:20-37, base_reacher_direct.py:20-38, simple_reacher.py:56-70,
// hole_reacher.py:73-77, hr_simple_reward.py:19-53, hr_dist_vel_acc_reward.py:20-60,
// hr_unbounded_reward.py:17-59, viapoint_reacher.py:79-111.  Returns the reward; FK is
// refreshed for the direct envs always and for SimpleReacher only when the reward needs it or
// `fk_always`.
struct StepOut {
  double reward, rdist, rctrl;
  bool coll, success;
};

// PAIR: k_episode_pair's lane pairs share the FK sincos and the collision tests (pp = lane parity)
template <int ENV, bool F32, int NL, bool MAYFK = true, bool PAIR = false>
__device__ __forceinline__ StepOut substep(const DevCfg& c, Env<NL>& v, const double* a, const float* a32,
                                           bool fk_always, int pp = 0) {
  auto self_c = [&]() { if constexpr (PAIR) return v.self_collision_pair(pp); else return v.self_collision(); };
  auto wall_c = [&]() { if constexpr (PAIR) return v.wall_collision_pair(c, pp); else return v.wall_collision(c); };
  StepOut r;
  r.coll = false;
  r.success = false;
  r.rdist = 0.0;
  const int st = v.steps;
  if (ENV == ENV_SIMPLE) {
#pragma unroll
    for (int d = 0; d < NL; ++d) {
      const double inc = F32 ? (double)(c.dt32 * a32[d]) : c.dt * a[d];
      v.qd[d] = fadd(v.qd[d], inc);
      v.q[d] = fadd(v.q[d], c.dt * v.qd[d]);
    }
    // np.sum(np.square(action)) (simple_reacher.py:60-62): f32 for a float32 action array
    double ctrl;
    if (F32) ctrl = (double)np_sum<NL, float>([&](int d) { return a32[d] * a32[d]; }, [](float x, float y) { return x + y; });
    else ctrl = np_sum<NL, double>([&](int d) { return a[d] * a[d]; }, [](double x, double y) { return fadd(x, y); });
    // MAYFK = false: the caller guarantees st < 199 (fast blocks), no FK code in the loop body
    if (MAYFK && (st >= 199 || fk_always)) v.fk();
    if (MAYFK && st >= 199) r.rdist = -norm2(v.jx[NL] - v.gx, v.jy[NL] - v.gy);
    r.reward = fsub(r.rdist, ctrl);
    r.rctrl = ctrl;
  } else {   // direct velocity control: HoleReacher, ViaPointReacher
    double acc_cost = 0.0;
    if (ENV == ENV_HOLE) {   // ViaPointReacher's reward uses the action, not _acc
      // np.sum(self._acc ** 2) (hr_simple_reward.py:48 and the other reward functions)
      if (F32 && (v.flags & 1u)) {   // qd already holds a float32 array: f32 arithmetic
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
    }
#pragma unroll
    for (int d = 0; d < NL; ++d) {
      v.qd[d] = a[d];
      const double inc = F32 ? (double)(c.dt32 * a32[d]) : c.dt * v.qd[d];
      v.q[d] = v.q[d] + inc;
    }
    if (F32) v.flags |= 1u;
    if constexpr (PAIR) v.fk_pair(pp);
    else v.fk();
    // sum(action**2) == sum(qd**2) after the step (f32 for a float32 action array)
    const double act_sq =
        F32 ? (double)np_sum<NL, float>([&](int d) { return a32[d] * a32[d]; }, [](float x, float y) { return x + y; })
            : np_sum<NL, double>([&](int d) { return a[d] * a[d]; }, [](double x, double y) { return x + y; });
    if (ENV == ENV_VIA) {   // viapoint_reacher.py:79-111
      r.coll = c.allow_self ? false : self_c();
      // 5e-8 * np.sum(action**2): a float32 sum stays float32 (NEP 50)
      const double pen_ctrl = F32 ? (double)(5e-8f * (float)act_sq) : 5e-8 * act_sq;
      if (r.coll) {
        const double dist = norm2(v.jx[NL] - v.gx, v.jy[NL] - v.gy);
        r.reward = (-c.penalty - dist * dist) - pen_ctrl;
      } else {   // reward starts at -inf and stays there (reference behaviour)
        r.reward = -__builtin_inf();
        if (st == 100) r.success = norm2(v.jx[NL] - v.hx, v.jy[NL] - v.hw) < 0.005;
        else if (st == 199) r.success = norm2(v.jx[NL] - v.gx, v.jy[NL] - v.gy) < 0.005;
      }
    } else if (c.rew_fct == REW_VEL_ACC) {   // hr_dist_vel_acc_reward.py:20-60
      if (!(v.flags & 4u)) {
        const bool sc = c.allow_self ? false : self_c();
        const bool wc = c.allow_wall ? false : wall_c();
        if (sc || wc) v.flags |= 4u;
        v.cd = norm2(v.jx[NL] - v.gx, v.jy[NL] - v.gy);
      }
      r.coll = (v.flags & 4u) != 0;
      double dist_cost = 0.0, coll_cost = 0.0;
      if (st == 199) {
        const double dist = norm2(v.jx[NL] - v.gx, v.jy[NL] - v.gy);
        r.success = dist < 0.005 && !r.coll;
        dist_cost = dist * dist;
        coll_cost = r.coll ? v.cd * v.cd : 0.0;
      }
      // np.dot(features, (-1, -1e-4, -1e-6, -penalty, 0)): OpenBLAS forward fma chain
      double d = dist_cost * -1.0;
      d = __builtin_fma(act_sq, -1e-4, d);
      d = __builtin_fma(acc_cost, -1e-6, d);
      d = __builtin_fma(coll_cost, -c.penalty, d);
      r.reward = __builtin_fma(0.0, 0.0, d);   // time_cost = 199 - steps is 0 whenever used
    } else if (c.rew_fct == REW_UNBOUNDED) {   // hr_unbounded_reward.py:17-59
      const bool sc = c.allow_self ? false : self_c();
      const bool wc = c.allow_wall ? false : wall_c();
      r.coll = sc || wc;
      if (st == 180 || r.coll) { v.ex = v.jx[NL]; v.ey = v.jy[NL]; }
      double dr = 0.0;
      if (st == 199 || r.coll) {
        const double dist = norm2(v.ex - v.gx, v.ey - v.gy);
        if (r.coll) dr = 0.25 * exp(-dist);
        else dr = (v.jy[NL] > 0.0) ? exp(-dist) : 1.0 - v.ey;
        r.success = !r.coll;
      }
      r.reward = __builtin_fma(acc_cost, -5e-6, dr * 1.0);
    } else {   // hr_simple_reward.py:19-53
      const bool sc = c.allow_self ? false : self_c();
      const bool wc = c.allow_wall ? false : wall_c();
      r.coll = sc || wc;
      if (st == 199 || r.coll) {
        const double dist = norm2(v.jx[NL] - v.gx, v.jy[NL] - v.gy);
        const double dc = dist * dist;
        // np.dot([dist^2, acc, coll], [-1, -5e-8, -penalty]) == OpenBLAS forward fma chain
        r.reward = __builtin_fma(r.coll ? 1.0 : 0.0, -c.penalty, __builtin_fma(acc_cost, -5e-8, dc * -1.0));
        r.success = dist < 0.005 && !r.coll;
      } else {
        r.reward = acc_cost * -5e-8;
      }
    }
  }
  v.steps = st + 1;
  return r;
}

// ============================================================================ replanning schedule
// Entry idx of the observation the replanning schedule receives (black_box_wrapper.py:233): the
// env obs cast to float32, then TimeAwareObservation's t / max_episode_steps (an f64 entry).
template <int NL>
__device__ inline double obs_entry(const DevCfg& c, const Env<NL>& v, int idx) {
  // register arrays are read through compile-time indices (a runtime index would move the
  // whole env state to scratch memory)
  if (idx < 2 * NL) {
    const int k = idx < NL ? idx : idx - NL;
    double qk = 0.0;
#pragma unroll
    for (int j = 0; j < NL; ++j) qk = (j == k) ? v.q[j] : qk;
    double sn, cs;
    fgx_sincos(qk, &sn, &cs);
    return (double)(float)(idx < NL ? cs : sn);
  }
  if (idx < 3 * NL) {
    double qd = 0.0;
#pragma unroll
    for (int j = 0; j < NL; ++j) qd = (j == idx - 2 * NL) ? v.qd[j] : qd;
    return (double)(float)qd;
  }
  int p = 3 * NL;
  if (c.env == ENV_HOLE) {
    if (idx == p) return (double)(float)v.hw;
    p += 1;
  }
  if (c.env == ENV_VIA) {
    if (idx == p) return (double)(float)(v.jx[NL] - v.hx);
    if (idx == p + 1) return (double)(float)(v.jy[NL] - v.hw);
    p += 2;
  }
  if (idx == p) return (double)(float)(v.jx[NL] - v.gx);
  if (idx == p + 1) return (double)(float)(v.jy[NL] - v.gy);
  if (idx == p + 2) return (double)(float)v.steps;
  return (double)v.steps / (double)c.max_steps;
}

// first plan sample k whose step t = steps + k + 1 satisfies a clause that depends on t only
__device__ inline int first_static_replan(const DevCfg& c, int steps) {
  int kr = 0x7fffffff;
  for (int j = 0; j < c.sched_n; ++j) {
    if (c.sched_kind[j] == SCHED_EVERY) {
      const int P = c.sched_k[j];
      kr = min(kr, P - 1 - (steps % P));
    } else if (c.sched_kind[j] == SCHED_AT) {
      const int kk = c.sched_k[j] - steps - 1;
      if (kk >= 0) kr = min(kr, kk);
    }
  }
  return kr == 0x7fffffff ? -1 : kr;
}

// t % max(int(np.linalg.norm(obs[i0:i1]) ** 2 * mul / div), 1) == 0 for any NORM_PERIOD clause
// (crowd_navigation/utils.py:9-10); the norm is sqrt of the OpenBLAS ddot (forward fma chain)
template <int NL>
__device__ inline bool state_replan(const DevCfg& c, const Env<NL>& v) {
  const int t = v.steps;
  bool hit = false;
  for (int j = 0; j < c.sched_n; ++j) {
    if (c.sched_kind[j] != SCHED_NORM_PERIOD) continue;
    double acc = 0.0;
    for (int i = c.sched_i0[j]; i < c.sched_i1[j]; ++i) {
      const double x = obs_entry(c, v, i);
      acc = (i == c.sched_i0[j]) ? x * x : __builtin_fma(x, x, acc);
    }
    const double n = __builtin_sqrt(acc);
    const double x = (n * n) * c.sched_mul[j] / c.sched_div[j];
    if (!(x == x)) continue;
    const double tr = __builtin_trunc(x);
    if (tr > 4.0e18) continue;             // period beyond any step count
    const long long P = tr >= 1.0 ? (long long)tr : 1;
    hit |= ((long long)t % P) == 0;
  }
  return hit;
}

// BB-step outputs, VectorEnv auto-reset and state write-back of one env (black_box_wrapper.py:
// 241-253; gymnasium SyncVectorEnv autoreset), shared by k_episode and k_episode_jp.  v holds
// the env after its last sample with FK refreshed.  reset_elsewhere (k_episode_jl): an ending env
// only gets its outputs and final observation here; another wave runs its reset.
template <int NL>
__device__ __forceinline__ void episode_epilogue(const DevCfg& c, const DevState& s, const Outputs& o, int64_t e,
                                                 Env<NL>& v, int plans, int L, double ret, bool term, bool trunc,
                                                 bool count = true, const double* gcs = nullptr,
                                                 const double* gsn = nullptr, bool reset_elsewhere = false) {
  const int64_t N = c.N;
  o.ret[e] = ret;
  o.term[e] = term;
  o.trunc[e] = trunc;
  o.tlen[e] = L;
  if (count && o.inner_steps) {   // (count = false: the caller adds L to inner_steps itself)
    if (__ballot(1) == ~0ull) {   // wave-reduce the trajectory lengths: one atomic per (full) wave
      long long sum = L;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off, 64);
      count_inner(o.inner_steps, sum, (threadIdx.x & 63) == 0);
    } else {
      count_inner(o.inner_steps, L, true);
    }
  }
  float* ob = o.obs + e * c.out_dim;
  float* fo = o.final_obs ? o.final_obs + e * c.out_dim : nullptr;
  if (o.autoreset && (term || trunc)) {
    if (fo) emit_obs(c, v, c.return_context, fo, nullptr, false, true, gcs, gsn);
    if (reset_elsewhere) return;   // another thread resets the env and writes its state / obs row
    autoreset_env(c, s, e, v);
    plans = 0;
    v.flags = 0;
    emit_obs(c, v, c.return_context, ob, nullptr, true);
  } else {
    emit_obs(c, v, c.return_context, ob, fo, false, true, gcs, gsn);
  }
  store_env(c, s, e, v, c.env != ENV_SIMPLE);
  s.plans[e] = plans;
}

// ============================================================================ trajectory validity
// RawInterfaceWrapper.preprocessing_and_validity_callback (raw_interface_wrapper.py:55-72) as the
// checks of include/fgx.h FGX_VALID_* (the form of table_tennis_env.py:304-309): the raw learned
// tau / delay entries against their bounds (f32 compares: a float32 action entry against a Python
// float), the desired positions of the whole plan against per-joint bounds (f64 compares of the f32
// positions).  tg: a copy of the plan's generator (advanced here); dpos: caller-given plan.
template <int MP, int NL, typename TrajT>
__device__ inline bool plan_valid(const DevCfg& c, TrajT tg, const float* prow, const float* dpos, int64_t e, int Te) {
  if (prow && (c.valid_flags & VALID_TAU)) {
    const float t = prow[0];
    if (t > c.vtau_hi32 || t < c.vtau_lo32) return false;
  }
  if (prow && (c.valid_flags & VALID_DELAY)) {
    const float dl = prow[c.learn_tau ? 1 : 0];
    if (dl > c.vdelay_hi32 || dl < c.vdelay_lo32) return false;
  }
  if (c.valid_flags & VALID_POS) {
    float pos[NL], vel[NL];
    for (int k = 0; k < Te; ++k) {
      if constexpr (MP == MP_GIVEN) {
#pragma unroll
        for (int d = 0; d < NL; ++d) pos[d] = dpos[(e * c.T + k) * NL + d];
      } else {
        tg.at(c, k, pos, vel);
      }
#pragma unroll
      for (int d = 0; d < NL; ++d)
        if ((double)pos[d] > c.vpos_hi[d] || (double)pos[d] < c.vpos_lo[d]) return false;
    }
  }
  return true;
}

// invalid_traj_callback's artificial transition (raw_interface_wrapper.py:103-121,
// black_box_wrapper.py:194-197): no env step, no plan counted; return / flags from the config, the
// observation zeros (np.zeros, the reference default) or the env's current one; then the VectorEnv
// auto-reset when the artificial flags end the episode.
template <int NL>
__device__ inline void invalid_transition(const DevCfg& c, const DevState& s, const Outputs& o, int64_t e, Env<NL>& v) {
  o.ret[e] = c.invalid_reward;
  o.term[e] = c.invalid_term;
  o.trunc[e] = c.invalid_trunc;
  o.tlen[e] = 0;
  v.fk();
  float* ob = o.obs + e * c.out_dim;
  float* fo = o.final_obs ? o.final_obs + e * c.out_dim : nullptr;
  auto artificial = [&](float* d) {
    if (!d) return;
    if (c.invalid_obs == INVALID_OBS_CURRENT) emit_obs(c, v, c.return_context, d, nullptr);
    else
      for (int i = 0; i < c.out_dim; ++i) d[i] = 0.0f;
  };
  if (o.autoreset && (c.invalid_term || c.invalid_trunc)) {
    artificial(fo);
    autoreset_env(c, s, e, v);
    v.flags = 0;
    emit_obs(c, v, c.return_context, ob, nullptr, true);
    store_env(c, s, e, v, c.env != ENV_SIMPLE);
    s.plans[e] = 0;
  } else {   // the env state and plan count are unchanged
    artificial(ob);
    artificial(fo);
  }
}

// ============================================================================ the BB step
// The body of k_episode (below) and k_episode_w2 (the same code compiled for two resident waves
// per SIMD).
// PAIR (k_episode_pair): two lanes per env (lanes 2i, 2i + 1 hold env i), both running the whole
// step; the FK sincos and the collision tests are divided between them (Env::fk_pair).  Every store
// is made by both lanes with the same value; the inner-step counter takes the even lanes' lengths.
// HELPED (k_episode_v2h): the logging body of waves 0..3 of a 512-thread workgroup whose waves 4..7
// store the per-step rows; the table is staged by the kernel, each sample's rows go to one of two
// staging slots per wave and one LDS-only workgroup barrier per sample hands them over.
template <int ENV, int MP, int CTRL, int NL, int NB, bool LOG, bool PAIR = false, bool HELPED = false>
__device__ __forceinline__ void episode_body(const DevCfg& c, const DevState& s, const float* __restrict__ params,
                                             const float* __restrict__ dpos, const float* __restrict__ dvel,
                                             const Outputs& o) {
  static_assert(!(PAIR && (LOG || ENV == ENV_SIMPLE)), "lane pairs serve the direct envs without per-step info");
  static_assert(!HELPED || (LOG && !PAIR), "the helped body is the logging one");
  extern __shared__ float lds_tab[];
  if (MP != MP_GIVEN && !HELPED) {
    const int n = c.rows * c.stride;
    for (int i = threadIdx.x; i < n; i += blockDim.x) lds_tab[i] = s.tables[i];
    __syncthreads();
  }
  const int64_t tid = (int64_t)blockIdx.x * (HELPED ? 256 : blockDim.x) + threadIdx.x;
  const int64_t e = PAIR ? (tid >> 1) : tid;
  const int pp = PAIR ? (int)(threadIdx.x & 1) : 0;
  if (e >= c.N) return;
  const int64_t N = c.N;
  FGX_STAMP(o, e, 6);
  FGX_STAMP(o, e, 0);

  Env<NL> v;
  load_env(c, s, e, v, ENV != ENV_SIMPLE);
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
  Traj<(MP == MP_GIVEN ? MP_NONE : MP), NL, NB, false, ENV == ENV_SIMPLE> tg;
  if (MP != MP_GIVEN) tg.init(c, params + e * c.n_params, lds_tab, s0, ic_q, ic_qd);

  plans += 1;
  // first sample index k with (k + 1 + s0) % replan == 0 (black_box_wrapper.py:233); the loop
  // stops there unless max_planning_times is exhausted, in which case it never replans again
  const bool plans_ok = c.replan && (c.max_plans <= 0 || plans < c.max_plans);
  const int k_replan = plans_ok ? first_static_replan(c, v.steps) : -1;
  PairwiseSum ps;
  ps.init();
  // plan length and the numpy pairwise split point of the return sum.  SimpleReacher never
  // terminates, so its episode-segment length is known now (plan end, TimeLimit or the
  // replanning sample) and the two-level online sum is exact; the direct envs can stop at any
  // sample (collision) and keep their step rewards in s.rew for lengths above 128.
  const int Te = (MP == MP_GIVEN && s.plan_len) ? s.plan_len[e] : c.T;
  // the per-step info rows L..T-1: the full desired plan (black_box_wrapper.py:245-246), NaN (0 for
  // the flags) in the per-step arrays after trajectory_length; gen: the plan's generator at sample L.
  // The wave walks the rows together (lanes whose env has stopped pad their row beside the running
  // ones) and the staged rows of each sample leave the wave as wide stores (InfoStage::flush).
  InfoStage<NL> ist;
  char* helped_slots = nullptr;   // HELPED: this wave's two staging slots
  int row = 0;                    // HELPED: rows handed over so far
  if constexpr (LOG) {
    const size_t tabf = (MP == MP_GIVEN) ? 0 : (size_t)c.rows * c.stride;
    if constexpr (HELPED) {
      helped_slots = (char*)lds_tab + stage_tab_offset(tabf) +
                     (size_t)(2 * (threadIdx.x >> 6)) * stage_wave_bytes(NL, c.full_dim);
      ist.init_at(c, o, helped_slots, e, MP != MP_GIVEN);
    } else {
      ist.init(c, o, (char*)lds_tab + stage_tab_offset(tabf), e, MP != MP_GIVEN);
    }
  }
  // the staged rows of sample kk leave: as this wave's wide stores, or (HELPED) to the partner wave
  auto emit_row = [&](int kk) __attribute__((always_inline)) {
    if constexpr (HELPED) {
      lds_barrier();
      ++row;
      ist.rebase(helped_slots + (size_t)(row & 1) * stage_wave_bytes(NL, c.full_dim));
    } else {
      ist.flush(kk, o);
    }
  };
  auto pad_row = [&](int kk, auto& gen) {
    const double dnan = __builtin_nan("");
    const float fnan = __builtin_nanf("");
    if (o.positions && MP != MP_GIVEN) {
      float pp[NL], pv[NL];
      gen.at(c, kk, pp, pv);
#pragma unroll
      for (int d = 0; d < NL; ++d) { ist.pos(d, pp[d]); ist.vel(d, pv[d]); }
    }
#pragma unroll
    for (int d = 0; d < NL; ++d) ist.act(d, dnan);
    ist.rew(dnan);
    float* so = ist.obs_row();
    for (int q = 0; q < c.full_dim; ++q) so[q * 64] = fnan;
    if constexpr (HELPED)   // (a NaN q: the storing wave leaves the padding's NaN)
#pragma unroll
      for (int d = 1; d < NL; ++d) ist.ql(d, dnan);
    ist.flags(0, 0);
    ist.ee(dnan, dnan);
    ist.rdc(dnan, dnan);
  };
  // trajectory validity (the logging instantiation serves valid_flags != 0): an invalid plan takes
  // no env step; its lane pads every row in the sample loop below (L = 0), then makes the artificial
  // transition instead of the epilogue
  bool invalid = false;
  if constexpr (LOG) {
    if (c.valid_flags)
      invalid = !plan_valid<MP, NL>(c, tg, params ? params + e * c.n_params : nullptr, dpos, e, Te);
  }
  int split = 0;
  if (ENV == ENV_SIMPLE && !c.sched_state) {
    int Lp = min(Te, max(1, c.max_steps - v.steps));
    if (k_replan >= 0) Lp = min(Lp, k_replan + 1);
    split = (Lp > 128) ? ((Lp / 2) & ~7) : 0;
  }
  // only read back for segments longer than 128 samples (L <= T): shorter plans store nothing
  double* rew_row = ((ENV != ENV_SIMPLE || c.sched_state) && s.rew && c.T > 128) ? s.rew + e : nullptr;
  bool term = false, trunc = false, stop = false;
  float pos[NL], vel[NL];
  // fast blocks are software-pipelined: sample k's f64 controller / dynamics and the f32
  // trajectory evaluation of sample k + 1 (into npos / nvel) form one scheduling region, so the
  // independent f32 and f64 chains interleave and only one look-ahead sample is held in registers
  float npos[NL], nvel[NL];
  bool pre = false;   // npos / nvel hold the desired state of the next sample (wave-uniform)
  constexpr bool F32 = (CTRL != CTRL_PD);

  // One plan sample k: desired state -> controller -> clip -> env.step -> return / info.
  // J = k & 7 when known at compile time (unrolled fast loop), -1 otherwise.  Returns true
  // when the BB step ends after this sample (black_box_wrapper.py:233-239).
  // canonical clip bounds: v_max/v_min need no per-sample canonicalisation of kernel args
  const double act_lo = __builtin_canonicalize(c.act_lo), act_hi = __builtin_canonicalize(c.act_hi);
  auto sample = [&](int k, auto Jtag, auto PHtag, bool fk_always) -> bool {
    constexpr int J = decltype(Jtag)::value;
    constexpr int PH = decltype(PHtag)::value;
    if (MP == MP_GIVEN) {
#pragma unroll
      for (int d = 0; d < NL; ++d) {
        pos[d] = dpos[(e * c.T + k) * NL + d];
        vel[d] = dvel[(e * c.T + k) * NL + d];
      }
    } else if constexpr (J >= 0) {
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int d = 0; d < NL; ++d) { pos[d] = npos[d]; vel[d] = nvel[d]; }
      // fast samples k < lim2 <= T - 2: the look-ahead k + 1 is never the plan's last sample
      tg.template at<true, true>(c, k + 1, npos, nvel);
    } else if (pre) {
#pragma unroll
      for (int d = 0; d < NL; ++d) { pos[d] = npos[d]; vel[d] = nvel[d]; }
      pre = false;
    } else {
      tg.at(c, k, pos, vel);
    }
    // ---- tracking controller + clip (black_box_wrapper.py:201-205)
    double a[NL];
    float a32[NL];
    bool nan_in = false;
#pragma unroll
    for (int d = 0; d < NL; ++d) {
      if (CTRL == CTRL_PD) {
        const double u = fadd(c.pg[d] * fsub((double)pos[d], v.q[d]), c.dg[d] * fsub((double)vel[d], v.qd[d]));
        a[d] = __builtin_fmin(__builtin_fmax(u, act_lo), act_hi);
        nan_in |= (u != u);
        if (LOG || J < 0) a[d] = (u != u) ? u : a[d];
        a32[d] = 0.0f;
      } else {
        const float u = (CTRL == CTRL_VEL) ? vel[d] : pos[d];
        a32[d] = np_clipf(u, c.act_lo32, c.act_hi32);
        a[d] = (double)a32[d];
      }
    }
    // np.clip propagates NaN; max/min do not: fix up (rare, wave-uniform branch).  ProMP fast
    // blocks run only in NaN-free waves (see nan_free below): no check there.
    if (CTRL == CTRL_PD && !(LOG || J < 0) && !(MP == MP_PROMP && J >= 0) &&
        __builtin_expect(__ballot(nan_in) != 0, 0)) {
#pragma unroll
      for (int d = 0; d < NL; ++d) {
        const double u = fadd(c.pg[d] * fsub((double)pos[d], v.q[d]), c.dg[d] * fsub((double)vel[d], v.qd[d]));
        if (u != u) a[d] = u;
      }
    }
    // ---- env.step
    const StepOut r = substep<ENV, F32, NL, (J < 0), PAIR>(c, v, a, a32, fk_always, pp);
    if constexpr (J >= 0) {   // fast blocks: no termination, truncation or replanning inside
      // SimpleReacher below env step 199: reward = 0 - ctrl, pushed as acc - ctrl
      if constexpr (ENV != ENV_SIMPLE) ps.template add_fast<J, (PH & 3)>(r.reward);   // (not reached)
      else if constexpr ((PH & 4) != 0) ps.template sub_partial<J, (PH & 3)>(r.rctrl);   // partial block
      else ps.template sub_fast<J, PH>(r.rctrl);
      return false;
    } else {
      term = (ENV != ENV_SIMPLE) ? r.coll : false;
      trunc = v.steps >= c.max_steps;
      ps.add(k, r.reward, split);
      if (rew_row) rew_row[(int64_t)k * N] = r.reward;
    }
    // ---- info (verbose >= 2, black_box_wrapper.py:220-227): the sample's values into the wave's
    // staging slots (flushed as wide stores once the wave has reconverged, InfoStage)
    if constexpr (LOG) {
#pragma unroll
      for (int d = 0; d < NL; ++d) ist.act(d, a[d]);
      if (MP != MP_GIVEN)
#pragma unroll
        for (int d = 0; d < NL; ++d) { ist.pos(d, pos[d]); ist.vel(d, vel[d]); }
      ist.rew(r.reward);
      if constexpr (ENV == ENV_SIMPLE) {   // (the host always passes o.qlog with step_obs here)
        // SimpleReacher: q for k_info_obs (cos / sin of q, FK's end effector - goal); here the
        // components emit_obs computes without trigonometry, in its order
#pragma unroll
        for (int d = 0; d < NL; ++d) ist.ql(d, v.q[d]);
        float* so = ist.obs_row();
#pragma unroll
        for (int d = 0; d < NL; ++d) so[(2 * NL + d) * 64] = (float)v.qd[d];
        so[(3 * NL + 2) * 64] = (float)v.steps;
        if (c.time_aware) so[(3 * NL + 3) * 64] = (float)((double)v.steps / (double)c.max_steps);
      } else if (o.step_obs) {
        // (FK is current after every logged sample: fk_always; cos / sin of q[0] are FK's)
        emit_obs(c, v, false, ist.obs_row(), nullptr, false, true, nullptr, nullptr, 64, HELPED);
        if constexpr (HELPED)   // cos / sin of q[1..]: the storing wave's (k_episode_v2h)
#pragma unroll
          for (int d = 1; d < NL; ++d) ist.ql(d, v.q[d]);
      }
      if (ENV != ENV_SIMPLE) {
        ist.flags((uint8_t)r.coll, (uint8_t)r.success);
        ist.ee(v.jx[NL], v.jy[NL]);
      } else {
        ist.rdc(r.rdist, r.rctrl);
      }
    }
    bool replan_now = (k == k_replan);
    if (J < 0 && c.sched_state && plans_ok && !replan_now) replan_now = state_replan(c, v);
    if (term || trunc || replan_now) {
      if (c.cond_desired) {
#pragma unroll
        for (int d = 0; d < NL; ++d) { s.cond[d * N + e] = pos[d]; s.cond[(NL + d) * N + e] = vel[d]; }
        v.flags |= 2u;
      }
      return true;
    }
    return false;
  };

  // Hand-levelled fast sample (SimpleReacher + ProMP on joint pairs + PD, the metric kernel).  One
  // wave per SIMD issues from a single instruction stream, so every dependent f64 / f32 op must
  // find independent work between itself and its producer.  The sample is written as levels
  // separated by sched_barriers: each level holds one step of every joint's f64 chain (PD, clip,
  // Euler, sum of squared actions) and one step of every pair's f32 trajectory chain for the NEXT
  // sample (basis contraction, finite difference, div_rcp), so consecutive dependent instructions
  // are >= 8 instructions apart.  The basis rows of the sample after next are loaded with scalar
  // loads one region ahead.  Every operation is the one `sample` performs, in the same order per
  // value: bit-identical results.
  using TrajT = decltype(tg);
  constexpr bool LV = !LOG && ENV == ENV_SIMPLE && MP == MP_PROMP && CTRL == CTRL_PD && NB > 0 && TrajT::PK;
  constexpr int NBL = NB > 0 ? NB : 1;
  constexpr int NLP = (NL + 1) / 2;
  float rb_[NBL];         // basis row k + 3 (trajectory of sample k + 1: its next position)
  float rdti = 0.0f, rrdt = 0.0f;   // dt and 1 / dt of row k + 2
  int rmax = 0;           // last table row reachable through stab (wave-uniform)
  auto lv_load = [&](int k) {   // rows for the region of sample k (clamped: never past the table)
    const int rb = min(k + 3, rmax), rd = min(k + 2, rmax);
#pragma unroll
    for (int j = 0; j < NBL; ++j) rb_[j] = tg.stab[(size_t)rb * TrajT::KS + j];
    rdti = tg.stab[(size_t)rd * TrajT::KS + NBL];
    rrdt = tg.stab[(size_t)rd * TrajT::KS + NBL + 1];
  };
  auto lv_sample = [&](int k, auto Jtag, auto PHtag) {
    constexpr int J = decltype(Jtag)::value;
    constexpr int PH = decltype(PHtag)::value;
    if constexpr (LV) {
      float b[NBL];
#pragma unroll
      for (int j = 0; j < NBL; ++j) b[j] = rb_[j];
      const float dti = rdti, rdt = rrdt;
      __builtin_amdgcn_sched_barrier(0);
      lv_load(k + 1);   // next region's rows (scalar loads in flight during this region)
      double pd[NL], vd[NL], e1[NL], e2[NL], u[NL], a[NL], sq[NL], inc[NL];
      f32x2 acc[NLP], x[NLP], qq[NLP], er[NLP], vl[NLP];
      // A: f32 -> f64 desired state | basis slot 0
#pragma unroll
      for (int d = 0; d < NL; ++d) { pd[d] = (double)npos[d]; vd[d] = (double)nvel[d]; }
#pragma unroll
      for (int p = 0; p < NLP; ++p) acc[p] = __builtin_elementwise_fma((f32x2)b[0], tg.wp[p][0], (f32x2)0.0f);
      __builtin_amdgcn_sched_barrier(0);
      // B: tracking errors | basis slot 1
#pragma unroll
      for (int d = 0; d < NL; ++d) { e1[d] = fsub(pd[d], v.q[d]); e2[d] = fsub(vd[d], v.qd[d]); }
      if constexpr (NBL > 1) {
#pragma unroll
        for (int p = 0; p < NLP; ++p) acc[p] = __builtin_elementwise_fma((f32x2)b[1], tg.wp[p][1], acc[p]);
      }
      __builtin_amdgcn_sched_barrier(0);
      // C: gains | basis slot 2
#pragma unroll
      for (int d = 0; d < NL; ++d) { e1[d] = c.pg[d] * e1[d]; e2[d] = c.dg[d] * e2[d]; }
      if constexpr (NBL > 2) {
#pragma unroll
        for (int p = 0; p < NLP; ++p) acc[p] = __builtin_elementwise_fma((f32x2)b[2], tg.wp[p][2], acc[p]);
      }
      __builtin_amdgcn_sched_barrier(0);
      // D: PD sum | basis slot 3
#pragma unroll
      for (int d = 0; d < NL; ++d) u[d] = fadd(e1[d], e2[d]);
      if constexpr (NBL > 3) {
#pragma unroll
        for (int p = 0; p < NLP; ++p) acc[p] = __builtin_elementwise_fma((f32x2)b[3], tg.wp[p][3], acc[p]);
      }
      __builtin_amdgcn_sched_barrier(0);
      // E: clip low | basis slots 4.. (NaN-free waves only: no np.clip NaN fix-up needed)
#pragma unroll
      for (int d = 0; d < NL; ++d) {
#ifdef FGX_EXP_NOCLIP   // timing experiment only (wrong results): no clip
        (void)act_lo;
#else
        u[d] = __builtin_fmax(u[d], act_lo);
#endif
      }
#pragma unroll
      for (int j = 4; j < NBL; ++j)
#pragma unroll
        for (int p = 0; p < NLP; ++p) acc[p] = __builtin_elementwise_fma((f32x2)b[j], tg.wp[p][j], acc[p]);
      __builtin_amdgcn_sched_barrier(0);
      // F: clip high | finite difference
#pragma unroll
      for (int d = 0; d < NL; ++d) {
#ifdef FGX_EXP_NOCLIP
        a[d] = u[d];
#else
        a[d] = __builtin_fmin(u[d], act_hi);
#endif
      }
#pragma unroll
      for (int p = 0; p < NLP; ++p) x[p] = acc[p] - tg.cur2[p];
      __builtin_amdgcn_sched_barrier(0);
      // G: Euler increment, squared actions | div_rcp quotient
#pragma unroll
      for (int d = 0; d < NL; ++d) { inc[d] = c.dt * a[d]; sq[d] = a[d] * a[d]; }
#pragma unroll
      for (int p = 0; p < NLP; ++p) qq[p] = x[p] * rdt;
      __builtin_amdgcn_sched_barrier(0);
      // H: velocities, ctrl | div_rcp residual
#pragma unroll
      for (int d = 0; d < NL; ++d) v.qd[d] = fadd(v.qd[d], inc[d]);
      double ctrl = fadd(sq[0], sq[1]);
#pragma unroll
      for (int p = 0; p < NLP; ++p) er[p] = __builtin_elementwise_fma(-qq[p], (f32x2)dti, x[p]);
      __builtin_amdgcn_sched_barrier(0);
      // I: position increments, ctrl | div_rcp correction
#pragma unroll
      for (int d = 0; d < NL; ++d) inc[d] = c.dt * v.qd[d];
      if constexpr (NL > 2) ctrl = fadd(ctrl, sq[2]);
#pragma unroll
      for (int p = 0; p < NLP; ++p) vl[p] = __builtin_elementwise_fma(er[p], (f32x2)rdt, qq[p]);
      __builtin_amdgcn_sched_barrier(0);
      // J: positions, ctrl | the next sample's desired state, trajectory state
#pragma unroll
      for (int d = 0; d < NL; ++d) v.q[d] = fadd(v.q[d], inc[d]);
      if constexpr (NL > 3) ctrl = fadd(ctrl, sq[3]);
#pragma unroll
      for (int p = 0; p < NLP; ++p) {
        npos[2 * p] = tg.cur2[p].x;
        nvel[2 * p] = vl[p].x;
        if (2 * p + 1 < NL) { npos[2 * p + 1] = tg.cur2[p].y; nvel[2 * p + 1] = vl[p].y; }
        tg.cur2[p] = acc[p];
        tg.vprev2[p] = vl[p];
      }
      v.steps += 1;
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int d = 4; d < NL; ++d) ctrl = fadd(ctrl, sq[d]);
      __builtin_amdgcn_sched_barrier(0);
      // SimpleReacher below env step 199: reward = 0 - ctrl, pushed as acc - ctrl
      if constexpr ((PH & 4) != 0) ps.template sub_partial<J, (PH & 3)>(ctrl);
      else ps.template sub_fast<J, PH>(ctrl);
    }
  };

  int k = 0;      // per-lane: index of the next sample
  FGX_STAMP(o, e, 1);
  if (!LOG && ENV == ENV_SIMPLE) {   // (HoleReacher's FK + collision body is too large to unroll)
    // fast path: blocks of 8 samples with compile-time return slots and a wave-uniform sample
    // index.  Fast samples must not reach env step 199 (the only SimpleReacher step whose reward
    // needs FK), the TimeLimit or the replanning sample, so no lane leaves the loop early and
    // the blocks carry no per-lane control flow; the wave runs the blocks every lane can take.
    int lim = min(199, c.max_steps - 1) - v.steps;
    if (k_replan >= 0) lim = min(lim, k_replan);
    if (c.sched_state) lim = 0;   // state-dependent replanning: every sample checks the schedule
    // fast samples k < lim2 (sample Te - 1 ends the plan; the look-ahead of the last fast sample
    // must not be it either)
    const int lim2 = min(Te - (MP == MP_GIVEN ? 1 : 2), max(0, lim));
    bool fast_ok = __ballot(1) == ~0ull;   // partial wave (N % 64 != 0): generic path only
    if (MP == MP_PROMP && CTRL == CTRL_PD) {
      // NaN-free waves: the PD control u = p (pos - q) + d (vel - qd) is finite for every sample
      // of the plan when, for every lane, |w| < c.wbound32 and |q|, |qd|, |p|, |d| < 1e150:
      //   |pos| <= max_i sum_j |table_ij| |w_j| < 1e30 (wbound32 = 1e30 / max(1, the table's largest
      //   row L1 norm), which carries weights_scale, fgx_create), |vel| <= 2 |pos| / dt < 2e32
      //   (finite in f32); the clipped |a| <= act_hi = 1000 bounds 200 Euler steps to
      //   |qd| < 1e150 + 2e3, |q| < 3.1e150, so |p (pos - q)|, |d (vel - qd)| < 4e300 and their
      //   sum < 8e300 < DBL_MAX: no inf - inf, no 0 * inf, no overflow.
      // The fast blocks then skip np.clip's NaN fix-up; other waves take the exact generic path.
      bool ok = __builtin_fabs(c.act_lo) <= 1e3 && __builtin_fabs(c.act_hi) <= 1e3 && c.dt <= 1.0;
#pragma unroll
      for (int d = 0; d < NL; ++d) {
        ok = ok && __builtin_fabs(v.q[d]) < 1e150 && __builtin_fabs(v.qd[d]) < 1e150 &&
             __builtin_fabs(c.pg[d]) < 1e150 && __builtin_fabs(c.dg[d]) < 1e150;
#pragma unroll
        for (int j = 0; j < (NB ? NB : kGenBasis); ++j) ok = ok && __builtin_fabsf(tg.wt(d, j)) < c.wbound32;
      }
      if (__ballot(!ok) != 0) fast_ok = false;
    }
    const int usplit = __builtin_amdgcn_readfirstlane(split);
    if (__ballot(split != usplit) != 0) fast_ok = false;   // the block phases need one split per wave
    // fast blocks read the basis rows with scalar loads: one plan start row per wave
    const int s0u = __builtin_amdgcn_readfirstlane(s0);
    if (__ballot(s0 != s0u) != 0) fast_ok = false;
    if constexpr (MP != MP_GIVEN) tg.stab = (cfloat_ptr)(uintptr_t)s.tables + (size_t)s0u * tg.str();
    // nfast full 8-blocks, then the remainder before the first sample that needs the generic
    // path (e.g. 192..198 ahead of step 199) as one partial block of np < 8 samples
    const int lim2_min = wave_min(lim2);
    const int nfast = fast_ok ? lim2_min / 8 : 0;
    const int np = fast_ok ? lim2_min % 8 : 0;
    if constexpr (MP != MP_GIVEN) {
      if (nfast > 0 || np > 0) {   // look-ahead of the first fast sample
        tg.template at<true, true>(c, 0, npos, nvel);
        pre = true;
        if constexpr (LV) {
          rmax = c.rows - 1 - s0u;
          lv_load(0);
        }
      }
    }
    // Two loops: blocks before the pairwise split push into the level-1 sums a[] only, blocks from
    // the split on into the second-half sums b[] only.  (With a split, L > 128 and the result is
    // first + u: a[] and t are dead after the split, so numpy's level-1 adds there are skipped;
    // without one every block is < L <= 128 and in the first loop.)  Each loop keeps one set of 8
    // accumulators live.
#define FGX_SAMPLE(J, PH)                                                                      \
  if constexpr (LV) lv_sample(kb + J, std::integral_constant<int, J>{}, std::integral_constant<int, PH>{}); \
  else sample(kb + J, std::integral_constant<int, J>{}, std::integral_constant<int, PH>{}, false);
#define FGX_BLOCK(PH) \
      FGX_SAMPLE(0, PH) FGX_SAMPLE(1, PH) FGX_SAMPLE(2, PH) FGX_SAMPLE(3, PH) \
      FGX_SAMPLE(4, PH) FGX_SAMPLE(5, PH) FGX_SAMPLE(6, PH) FGX_SAMPLE(7, PH)
    const int nA = usplit > 0 ? min(nfast, usplit / 8) : nfast;
    int kb = 0;
    for (; kb < 8 * nA; kb += 8) { FGX_BLOCK(1) }
    if (usplit > 0 && nfast > nA) {
      ps.first = PairwiseSum::comb(ps.a);   // blocks [0, split)
      for (; kb < 8 * nfast; kb += 8) { FGX_BLOCK(2) }
    }
    k = 8 * nfast;
    ps.sync_tails();   // fast blocks end on complete 8-blocks: tails = combined accumulators
    if (np > 0) {
      if (usplit > 0 && kb >= usplit) {
        if (kb == usplit) ps.first = PairwiseSum::comb(ps.a);   // the partial block opens the second half
#define FGX_PART(J) if (J < np) { FGX_SAMPLE(J, 6) }
        FGX_PART(0) FGX_PART(1) FGX_PART(2) FGX_PART(3) FGX_PART(4) FGX_PART(5) FGX_PART(6)
      } else {
#undef FGX_PART
#define FGX_PART(J) if (J < np) { FGX_SAMPLE(J, 5) }
        FGX_PART(0) FGX_PART(1) FGX_PART(2) FGX_PART(3) FGX_PART(4) FGX_PART(5) FGX_PART(6)
      }
#undef FGX_PART
      k += np;
    }
#undef FGX_BLOCK
#undef FGX_SAMPLE
  }
  FGX_STAMP(o, e, 2);
  int L = 0x7fffffff;   // samples executed (trajectory_length)
  if constexpr (LOG) {
    // the wave walks the plan rows together (k is wave-uniform here: no fast blocks with LOG): a
    // lane whose env has stopped pads its row k beside the samples of the lanes still running, so
    // every info store covers the wave's consecutive envs in one row, then rows k..T-1 of all lanes
    stop = invalid;
    for (;; ++k) {
      const bool act = !stop && k < Te;
      if (__ballot(act) == 0) break;
      if (act) {
        // (defer: FK only where the reward or the replanning schedule reads it, as without LOG)
        stop = sample(k, std::integral_constant<int, -1>{}, std::integral_constant<int, 0>{},
                      ENV == ENV_SIMPLE ? (bool)c.sched_state : true);
      } else {
        L = min(L, k);
        if (k < c.T) pad_row(k, tg);
      }
      if (k < c.T) emit_row(__builtin_amdgcn_readfirstlane(k));
    }
    L = min(L, k);
    for (int kk = __builtin_amdgcn_readfirstlane(k); kk < c.T; ++kk) {
      pad_row(kk, tg);
      emit_row(kk);
    }
    if constexpr (HELPED) lds_barrier();   // the partner has stored the last row
    if (invalid) {
      invalid_transition(c, s, o, e, v);
      return;
    }
    if (ENV == ENV_SIMPLE && o.gsave) { o.gsave[e] = v.gx; o.gsave[N + e] = v.gy; }   // the episode's goal, for k_info_obs
  } else {
    while (!stop && k < Te) {
      stop = sample(k, std::integral_constant<int, -1>{}, std::integral_constant<int, 0>{}, c.sched_state);
      ++k;
    }
    L = k;
  }
  FGX_STAMP(o, e, 3);
  // the epilogue needs FK of the final q; a last sample at env step >= 199 (always a generic one)
  // has just computed it for its reward
  if (ENV == ENV_SIMPLE && !(v.steps - 1 >= 199 && !c.sched_state)) v.fk();
  const double ret = (L > 128 && rew_row) ? pairwise_strided(rew_row, N, L) : ps.result(L, split);
  FGX_STAMP(o, e, 4);
  if constexpr (PAIR) {   // the env's length once: from its even lane
    if (o.inner_steps) {
      long long sum = pp ? 0 : L;
      if (__ballot(1) == ~0ull) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off, 64);
        count_inner(o.inner_steps, sum, (threadIdx.x & 63) == 0);
      } else {
        count_inner(o.inner_steps, sum, true);
      }
    }
  }
  episode_epilogue(c, s, o, e, v, plans, L, ret, term, trunc, !PAIR);
  FGX_STAMP(o, e, 5);
  FGX_STAMP(o, e, 7);
}

// HoleReacher with lane pairs (episode_body PAIR): 2N threads, two resident waves per SIMD (<= 256
// registers), so that 65536 envs fill two waves on each SIMD instead of one
template <int ENV, int MP, int CTRL, int NL, int NB>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_episode_pair(
    DevCfg c, DevState s, const float* __restrict__ params, const float* __restrict__ dpos,
    const float* __restrict__ dvel, Outputs o) {
  episode_body<ENV, MP, CTRL, NL, NB, false, true>(c, s, params, dpos, dvel, o);
}

// k_episode_v2h: the verbose-2 step of the direct envs (HoleReacher, ViaPointReacher).  The logging
// k_episode runs one lone wave per SIMD that computes a sample and then stores its ~30 info rows;
// here waves 0..3 run the same logging body (episode_body HELPED) and hand each sample's staged rows
// to waves 4..7 (wave w + 4 shares wave w's SIMD), which issue the stores (InfoStage::flush, the same
// code and the same bytes), so the dynamics wave never issues a global info store; the storing wave
// also computes the observation's cos / sin of q[1..NL) from the staged q (emit_obs skip_q: the
// same fgx_sincos on the same q; q[0]'s are FK's, computed for the dynamics anyway).  Two staging
// slots per dynamics wave, one LDS-only barrier per sample (s_barrier after lgkmcnt(0): a
// __syncthreads fence would make the storing waves wait for their own stores every sample).  The
// grid covers N with whole workgroups (N % 256 == 0, fgx_dispatch.h): every wave meets every barrier.
template <int ENV, int MP, int CTRL, int NL, int NB>
__global__ __launch_bounds__(512) void k_episode_v2h(DevCfg c, DevState s, const float* __restrict__ params,
                                                     const float* __restrict__ dpos, const float* __restrict__ dvel,
                                                     Outputs o) {
  extern __shared__ float lds_tab[];
  const int tabn = (MP != MP_GIVEN) ? c.rows * c.stride : 0;
  for (int i = threadIdx.x; i < tabn; i += blockDim.x) lds_tab[i] = s.tables[i];
  __syncthreads();   // table staged
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  if (w < 4) {
    episode_body<ENV, MP, CTRL, NL, NB, true, false, true>(c, s, params, dpos, dvel, o);
    return;
  }
  // the storing wave of dynamics wave w - 4: row k from slot k & 1, after the barrier that follows it
  const int pw = w - 4;
  const size_t wb = stage_wave_bytes(NL, c.full_dim);
  char* slots = (char*)lds_tab + stage_tab_offset((size_t)tabn) + (size_t)(2 * pw) * wb;
  InfoStage<NL> ist;
  ist.init_at(c, o, slots, (int64_t)blockIdx.x * 256 + pw * 64 + (threadIdx.x & 63), MP != MP_GIVEN);
  const int lane = threadIdx.x & 63;
  for (int k = 0; k < c.T; ++k) {
    lds_barrier();
    ist.rebase(slots + (size_t)(k & 1) * wb);
    if (o.step_obs) {
      // the observation's cos / sin of q[1..NL) (emit_obs's fgx_sincos on the staged q; for a NaN q --
      // a padded row, or a running env with NaN state -- the NaN placeholder stays, as sincos(NaN))
      float* so = ist.obs_row();
#pragma unroll
      for (int d = 1; d < NL; ++d) {
        const double q = ist.d[(NL + 5 + d) * 64 + lane];
        if (q == q) {
          double sn, cs;
          fgx_sincos(q, &sn, &cs);
          so[d * 64] = (float)cs;
          so[(NL + d) * 64] = (float)sn;
        }
      }
    }
    ist.flush(k, o);
  }
  lds_barrier();
}

inline size_t v2h_lds_bytes(int mp, int rows, int stride, int nl, int full_dim) {
  const size_t tabf = (mp == MP_GIVEN) ? 0 : (size_t)rows * stride;
  return stage_tab_offset(tabf) + 8 * stage_wave_bytes(nl, full_dim);
}

template <int ENV, int MP, int CTRL, int NL, int NB, bool LOG>
__global__ __launch_bounds__(256) void k_episode(DevCfg c, DevState s, const float* __restrict__ params,
                                                 const float* __restrict__ dpos, const float* __restrict__ dvel,
                                                 Outputs o) {
  episode_body<ENV, MP, CTRL, NL, NB, LOG>(c, s, params, dpos, dvel, o);
}

// k_episode capped at 256 registers (two resident waves per SIMD; the 5-link SimpleReacher body
// spills ~30 registers outside its sample loop, the loop itself is unchanged).  Past one round of
// 64-lane waves per SIMD (N > 65536 on 256 CUs) the second wave shares the SIMD's issue slots
// instead of waiting for the next round: ProMP 5 links 131072 envs 139 -> 126 us, 262144 262 ->
// 224 us; within one round the uncapped kernel is faster (76.0 vs 80.4 us at 65536).
template <int ENV, int MP, int CTRL, int NL, int NB, bool LOG>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_episode_w2(
    DevCfg c, DevState s, const float* __restrict__ params, const float* __restrict__ dpos,
    const float* __restrict__ dvel, Outputs o) {
  episode_body<ENV, MP, CTRL, NL, NB, LOG>(c, s, params, dpos, dvel, o);
}

// info_level 2, SimpleReacher: the per-step observation components that need trigonometry -- cos /
// sin of every q (emit_obs: q[0]'s from FK) and the end effector minus the goal -- for every (sample,
// env), one thread each, from the q the logging k_episode logged after every sample and the
// episode's goal; NaN after trajectory_length.  The same FK / sincos / conversions as emit_obs on the
// same q: bit-identical to computing them in the sample loop, where they cost ~9 f64 sincos per
// sample of a lone wave's instruction stream; here they run at full occupancy.
template <int NL>
__global__ __launch_bounds__(256) void k_info_obs(DevCfg c, Outputs o) {
  const int64_t N = c.N;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t t = blockIdx.y;
  if (e >= N) return;
  float* row = o.step_obs + t * c.full_dim * N + e;   // observation component p at row[p * N]
  if (t >= o.tlen[e]) {
    const float fnan = __builtin_nanf("");
#pragma unroll
    for (int p = 0; p < 2 * NL; ++p) row[p * N] = fnan;
    row[3 * NL * N] = fnan;
    row[(3 * NL + 1) * N] = fnan;
    return;
  }
  Env<NL> v;
#pragma unroll
  for (int d = 0; d < NL; ++d) v.q[d] = o.qlog[(t * NL + d) * N + e];
  v.fk();
  row[0] = (float)v.c[0];
  row[NL * N] = (float)v.s[0];
#pragma unroll
  for (int d = 1; d < NL; ++d) {
    double sn, cs;
    fgx_sincos(v.q[d], &sn, &cs);
    row[d * N] = (float)cs;
    row[(NL + d) * N] = (float)sn;
  }
  row[3 * NL * N] = (float)(v.jx[NL] - o.gsave[e]);
  row[(3 * NL + 1) * N] = (float)(v.jy[NL] - o.gsave[N + e]);
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
