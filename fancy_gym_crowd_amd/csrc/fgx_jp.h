// fgx_jp.h — k_episode_jp: the joint-parallel black-box step for SimpleReacher (the metric path).
//
// BlackBoxWrapper.step (black_box_wrapper.py:170-253) over a torque SimpleReacher with a PD
// tracking controller is, per joint d, an independent recurrence
//     desired (pos_d, vel_d)(k)  ->  u_d = p (pos_d - q_d) + d (vel_d - qd_d)  ->  clip
//     qd_d += dt a_d ;  q_d += dt qd_d                         (base_reacher_torque.py:20-37)
// coupled only through the reward  r_k = -dist(ee, goal)[step == 199] - sum_d a_d^2
// (simple_reacher.py:56-70).  k_episode runs one env per lane with every joint in registers:
// 306 registers, one wave per SIMD, so with N <= 65536 envs a SIMD holds at most one wave and
// issues at the single-wave rate (profiles/r01_valu_rates.jsonl).  Here a workgroup owns 64
// envs and runs one wave per joint (lane = env, wave = joint): NL x the waves with no duplicated
// work and a small per-lane state (96 registers, 5 waves per SIMD).
//
// The reward couples the joints: every 8 samples (one "chunk" = one block of numpy's 8-way
// pairwise accumulators) each joint wave writes its a_d^2 to LDS, and the wave owning
// accumulator slot j (j % NL) forms sum_d a_d^2 in joint order, the reward, and pushes it into
// its slots of numpy's pairwise sum (first half / second half / sequential tail, exact for every
// segment length L <= 256).  The one sample whose reward needs forward kinematics (env step 199,
// the last before the TimeLimit) is held back: its sum a^2 goes to wave 0, which gathers q, qd
// and the slot sums after the last chunk, computes FK once, finishes the return and runs the
// shared epilogue (observation, TimeLimit, auto-reset, state write-back).
//
// np.clip propagates NaN, v_max/v_min do not: a chunk runs with the plain clip while recording
// whether any u was NaN (one compare per sample, no branch), and is re-run from its saved start
// state with the NaN-propagating clip if one was.
//
// Every expression rounds exactly as in k_episode / the numpy reference (same operations, same
// order); it serves ENV_SIMPLE + PD + shared tables + info_level < 2 + max_episode_steps <= 200,
// and fgx_dispatch.h picks it over k_episode where it is measured faster (episode_kernel_choice).
#pragma once
#include "fgx_kernels.h"

namespace fgx {

constexpr int kJpChunk = 8;

// LDS: [basis table (f32; first, so that row offsets fit the ds_read2 immediates)]
//      [ex: max(8 NL, 25) rows] [qs: 2 NL rows]   (f64 rows of 64 entries, one per lane / env)
//   ex  chunk exchange: a^2 of slot j, joint d at row j * NL + d; end of step: slot sums A / B /
//       tail of slot j at rows 3 j + {0, 1, 2}, the FK sample's sum a^2 at row 24
//   qs  end of step: q_d at row d, qd_d at row NL + d
template <int NL>
__host__ __device__ constexpr int jp_ex_rows() { return 8 * NL > 25 ? 8 * NL : 25; }
template <int NL>
inline size_t jp_lds_bytes(int rows, int stride) {
  return (size_t)(jp_ex_rows<NL>() + 2 * NL) * 64 * sizeof(double) + (size_t)rows * stride * sizeof(float);
}


// v_max_f64 / v_min_f64 (IEEE maxNum / minNum: a NaN u gives a bound, see the chunk redo); asm so
// that the bounds are not re-canonicalised for every sample
__device__ __forceinline__ double clip_nonan(double u, double lo, double hi) {
  double a;
  asm("v_max_f64 %0, %1, %2\n\tv_min_f64 %0, %0, %3" : "=&v"(a) : "v"(u), "s"(lo), "s"(hi));
  return a;
}

// One env's BB-step segment (the same quantities k_episode derives): trajectory_length L and the
// numpy pairwise layout of rewards[0:L] — [0, hs) first half (L > 128), [hs, bend) 8-way blocks of
// the last half, [bend, L) its sequential tail (hs, bend multiples of 8) — and the sample k_fk
// whose reward needs FK (env step >= 199: with max_steps <= 200 only the segment's last sample).
struct JpSeg {
  int steps, plans, k_replan, L, hs, bend, k_fk;
  uint32_t flags;
  bool stop;   // the segment ends in truncation or a replanning sample (black_box_wrapper.py:233-239)
  __device__ __forceinline__ void init(const DevCfg& c, const DevState& s, int64_t e, bool valid) {
    init_vals(c, s.steps[e], s.flags[e], s.plans[e], valid);
  }
  // the same from the env's stored steps / flags / plan count (values gathered elsewhere)
  __device__ __forceinline__ void init_vals(const DevCfg& c, int steps_, uint32_t flags_, int plans_stored,
                                            bool valid) {
    steps = steps_;
    flags = flags_;
    plans = plans_stored + 1;
    const bool plans_ok = c.replan && (c.max_plans <= 0 || plans < c.max_plans);
    k_replan = plans_ok ? first_static_replan(c, steps) : -1;
    L = min(c.T, max(1, c.max_steps - steps));
    if (k_replan >= 0) L = min(L, k_replan + 1);
    if (!valid) L = 0;
    hs = (L > 128) ? ((L / 2) & ~7) : 0;
    bend = hs + ((L - hs) & ~7);
    k_fk = (valid && steps + L - 1 >= 199) ? L - 1 : 0x7fffffff;
    stop = (steps + L >= c.max_steps) || (k_replan >= 0 && L == k_replan + 1);
  }
};

template <int MP, int NL, int NB>
__global__ __launch_bounds__(NL * 64, 5) void k_episode_jp(DevCfg c, DevState s, const float* __restrict__ params,
                                                           Outputs o) {
  extern __shared__ double lds_jp[];
  float* tab = (float*)lds_jp;
  double* ex = lds_jp + ((size_t)c.rows * c.stride + 1) / 2;   // rows * stride is a multiple of 4
  double* qs = ex + jp_ex_rows<NL>() * 64;
  {
    const int n = c.rows * c.stride;
    for (int i = threadIdx.x; i < n; i += blockDim.x) tab[i] = s.tables[i];
  }
  const int lane = threadIdx.x & 63;
  const int d = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // this wave's joint
  const int64_t N = c.N;
  const int64_t e0 = (int64_t)blockIdx.x * 64 + lane;
  const bool valid = e0 < N;
  const int64_t e = valid ? e0 : N - 1;   // clamped index: loads stay in bounds, nothing is stored

  // ---- the env's segment (every wave reads the same 64 envs: wave reductions agree across waves)
  JpSeg sg;
  sg.init(c, s, e, valid);
  const int Lmin = wave_min_dpp(sg.L), Lmax = wave_max_dpp(sg.L);
  const bool uni = Lmin == Lmax;   // one segment length (hence layout) for the wave: uniform phases
  const int hs_u = __builtin_amdgcn_readfirstlane(sg.hs), bend_u = __builtin_amdgcn_readfirstlane(sg.bend);

  // ---- this lane's joint d
  double pg = c.pg[0], dg = c.dg[0];
#pragma unroll
  for (int j = 1; j < NL; ++j) {
    pg = (j == d) ? c.pg[j] : pg;
    dg = (j == d) ? c.dg[j] : dg;
  }
  const int nb = NB ? NB : c.nb;
  double q = s.q[d * N + e], qd = s.qd[d * N + e];
  float pos = 0.0f, vel = 0.0f;
  Traj<MP, 1, NB> tg;
  {
    const int s0 = c.replan ? sg.steps : 0;   // init_time = current_traj_steps * dt when replanning
    const bool has_cond = c.cond_desired && (sg.flags & 2u);
    const double ic_q = has_cond ? (double)s.cond[d * N + e] : q;
    const double ic_qd = has_cond ? (double)s.cond[(NL + d) * N + e] : qd;
    const float* pe = params + e * c.n_params;
    __syncthreads();   // basis table staged
    if (MP == MP_PRODMP)
      tg.init(c, pe + d * (nb + 1), tab, s0, &ic_q, &ic_qd, c.T, c.tau32, c.rcp_tau32);
    else
      tg.init(c, pe + d * nb, tab, s0, &ic_q, &ic_qd, c.T, c.tau32, c.rcp_tau32, NL * nb + d - d * nb);
  }

  const double act_lo = c.act_lo, act_hi = c.act_hi;
  double cfk = 0.0;   // sum a^2 of the sample that needs FK (owned by the wave of its slot)
  uint64_t nanm = 0;
  // one sample: desired state -> PD -> clip -> torque Euler step; returns a_d^2.  EXACT: np.clip's
  // NaN propagation; otherwise a NaN u is recorded in nanm (chunk redo)
  auto joint_sample = [&](int k, auto mid, auto exact) -> double {
    float p1[1], v1[1];
    tg.template at<decltype(mid)::value>(c, k, p1, v1);
    pos = p1[0];
    vel = v1[0];
    const double u = pg * ((double)pos - q) + dg * ((double)vel - qd);
    double a = clip_nonan(u, act_lo, act_hi);
    if constexpr (decltype(exact)::value) a = (u != u) ? u : a;
    else nanm |= __ballot(u != u);
    qd = qd + c.dt * a;
    q = q + c.dt * qd;
    return a * a;
  };
  // the 8 samples of chunk k0, a^2 straight to LDS
  auto chunk = [&](int k0, auto exact) {
    if (k0 + kJpChunk <= Lmin && k0 + kJpChunk < c.T) {   // every lane, no plan-end sample
#pragma unroll
      for (int j = 0; j < kJpChunk; ++j)
        ex[(j * NL + d) * 64 + lane] = joint_sample(k0 + j, std::true_type{}, exact);
    } else {
#pragma unroll
      for (int j = 0; j < kJpChunk; ++j) {
        double a2 = 0.0;
        if (k0 + j < sg.L) a2 = joint_sample(k0 + j, std::false_type{}, exact);
        ex[(j * NL + d) * 64 + lane] = a2;
      }
    }
  };

  // ---- accumulator slots owned by this wave: j = d + NL * sl
  constexpr int SPW = (kJpChunk + NL - 1) / NL;
  double A[SPW], B[SPW], Tl[SPW];
#pragma unroll
  for (int sl = 0; sl < SPW; ++sl) { A[sl] = -0.0; B[sl] = -0.0; Tl[sl] = 0.0; }   // -0.0 + r == r

  const int nchunks = (Lmax + kJpChunk - 1) / kJpChunk;
  for (int ch = 0; ch < nchunks; ++ch) {
    const int k0 = ch * kJpChunk;
    const double q0 = q, qd0 = qd;
    const Traj<MP, 1, NB> tg0 = tg;
    nanm = 0;
    chunk(k0, std::false_type{});
    if (__builtin_expect(nanm != 0, 0)) {   // a NaN control: redo the chunk with np.clip semantics
      q = q0;
      qd = qd0;
      tg = tg0;
      chunk(k0, std::true_type{});
    }
    __syncthreads();
    // reductions of this wave's slots: sum_d a_d^2 in joint order, reward, pairwise slot sums
#pragma unroll
    for (int sl = 0; sl < SPW; ++sl) {
      const int j = d + NL * sl;
      if (j < kJpChunk) {
        const int k = k0 + j;
        double ctrl = ex[(j * NL) * 64 + lane];
#pragma unroll
        for (int dd = 1; dd < NL; ++dd) ctrl = ctrl + ex[(j * NL + dd) * 64 + lane];
        const double r = 0.0 - ctrl;   // rdist = 0 below env step 199
        if (k == sg.k_fk) {
          cfk = ctrl;                   // reward finished after the loop, with FK
        } else if (uni) {
          if (k < hs_u) A[sl] = A[sl] + r;
          else if (k < bend_u) B[sl] = B[sl] + r;
          else if (k < Lmin) Tl[sl] = r;
        } else {
          if (k < sg.hs) A[sl] = A[sl] + r;
          else if (k < sg.bend) B[sl] = B[sl] + r;
          else if (k < sg.L) Tl[sl] = r;
        }
      }
    }
    __syncthreads();   // reductions done before the next chunk writes ex
  }

  // ---- gather: slot sums, the FK sample's control cost and the joint state to wave 0
  if (valid && sg.stop && c.cond_desired) {   // black_box_wrapper.py:234-236
    s.cond[d * N + e] = pos;
    s.cond[(NL + d) * N + e] = vel;
  }
#pragma unroll
  for (int sl = 0; sl < SPW; ++sl) {
    const int j = d + NL * sl;
    if (j < kJpChunk) {
      ex[(3 * j) * 64 + lane] = A[sl];
      ex[(3 * j + 1) * 64 + lane] = B[sl];
      ex[(3 * j + 2) * 64 + lane] = Tl[sl];
    }
  }
  if (sg.k_fk < sg.L && ((sg.k_fk & 7) % NL) == d) ex[24 * 64 + lane] = cfk;
  qs[d * 64 + lane] = q;
  qs[(NL + d) * 64 + lane] = qd;
  __syncthreads();
  if (d != 0 || !valid) return;

  // ---- wave 0: return and epilogue
  Env<NL> v;
  load_env(c, s, e, v, false);   // SimpleReacher: no hole / reward state
#pragma unroll
  for (int k = 0; k < NL; ++k) { v.q[k] = qs[k * 64 + lane]; v.qd[k] = qs[(NL + k) * 64 + lane]; }
  v.steps = sg.steps + sg.L;
  if (sg.stop && c.cond_desired) v.flags |= 2u;
  v.fk();
  // the last sample at env step 199 (simple_reacher.py:60-62): r = -dist(ee, goal) - sum a^2;
  // it is the last element of the return sum, either the sequential tail's last or slot 7 of the
  // last 8-block (L == bend)
  const int L = sg.L, bend = sg.bend;
  const bool fk_last = sg.k_fk < L;
  const double r_fk = fk_last ? -norm2(v.jx[NL] - v.gx, v.jy[NL] - v.gy) - ex[24 * 64 + lane] : 0.0;
  double sa[8], sb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sa[j] = ex[(3 * j) * 64 + lane]; sb[j] = ex[(3 * j + 1) * 64 + lane]; }
  if (fk_last && L == bend && L >= 8) sb[7] = sb[7] + r_fk;
  double res = (L >= 8) ? PairwiseSum::comb(sb) : 0.0;
  const int ntail = L - bend;
#pragma unroll
  for (int j = 0; j < 8; ++j)
    if (j < ntail) res = res + ((fk_last && j == ntail - 1) ? r_fk : ex[(3 * j + 2) * 64 + lane]);
  if (L > 128) res = PairwiseSum::comb(sa) + res;
  const bool trunc = v.steps >= c.max_steps;
  episode_epilogue(c, s, o, e, v, sg.plans, L, res, false, trunc);
}

}  // namespace fgx
