// fgx_jl.h — k_episode_jl: the joint-lane black-box step for SimpleReacher + PD (the metric path
// and its strong-scaling shards).
//
// BlackBoxWrapper.step (black_box_wrapper.py:170-253) over a torque SimpleReacher with a PD tracking
// controller is, per joint d, an independent recurrence (base_reacher_torque.py:20-37)
//     desired (pos_d, vel_d)(k) -> u_d = p (pos_d - q_d) + d (vel_d - qd_d) -> clip -> qd_d += dt a_d ; q_d += dt qd_d
// coupled only through the reward r_k = -dist(ee, goal)[step == 199] - sum_d a_d^2 (simple_reacher.py:56-70).
//
// k_episode runs one env per lane (all joints in one instruction stream, ~300 registers): at
// N <= 65536 envs per GPU a SIMD holds at most one wave and issues at the lone-wave rate, and at the
// strong-scaling shard sizes (8192-32768 envs per GPU) most SIMDs hold none.  k_episode_jp splits
// the joints over waves but couples them through LDS + workgroup barriers every 8 samples.  Here
// one lane owns one (env, joint): a wave holds G = 64 / NL envs (12 for 5 links, lanes 60-63 idle;
// 32 for 2 links) and the joint coupling never leaves the wave:
//   * per 8-sample chunk every lane writes its 8 a_d^2 to the wave's LDS rows; the lane owning
//     pairwise slot j (j % NL == d) forms sum_d a_d^2 in joint order, the reward 0 - ctrl, and pushes
//     it into its share of numpy's pairwise accumulators (first half / second half / sequential tail,
//     exact for every L <= 200, as k_episode_jp) — ordered by wavefront fences, no barrier;
//   * the trajectory of joint d (Traj<MP, 1, NB>) runs in its own lane: no duplicated work, ~90
//     registers, ~5 waves per SIMD at 65536 envs and 5 x the lanes of k_episode at shard sizes;
//   * the basis rows come through scalar loads (SGPRs) whenever the wave's plans start on one row
//     (always, unless resets desynchronised replanning envs: then per-lane loads, same values).
// After the last chunk the lanes hand q, qd, the slot sums and the FK sample's control cost to one
// thread per env (threads 0..4G-1 of the workgroup, one LDS pass + workgroup barrier), which forms
// FK, the step-199 reward, the return and runs the shared epilogue (k_episode_jp's wave-0 part).
//
// NaN controls: np.clip propagates NaN, v_max / v_min do not: a chunk runs with the plain clip
// while recording any NaN u (one compare per sample), and is re-run from its saved start state with
// the NaN-propagating clip if one was (k_episode_jp).  Every expression rounds exactly as in
// k_episode (same operations, same order): bit-identical results (tests/test_gpu_jl.py).
#pragma once
#include "fgx_jp.h"

namespace fgx {

template <int NL>
struct JlShape {
  static constexpr int G = 64 / NL;             // envs per wave
  static constexpr int WAVES = 4;               // waves per workgroup
  static constexpr int EPB = G * WAVES;         // envs per workgroup
  static constexpr int SPW = (8 + NL - 1) / NL; // pairwise slots owned per lane
  static constexpr int GF = 25 + 2 * NL;        // gathered f64 per env: A, B, tail (8 each), cfk, q, qd
  static constexpr size_t lds_bytes() {
    const size_t ex = (size_t)WAVES * 16 * 64 * sizeof(double);
    const size_t ga = (size_t)GF * EPB * sizeof(double);
    return ex > ga ? ex : ga;
  }
};

// orders this wave's LDS writes before its later reads (and reads before later writes): LDS
// operations of one wave execute in order, so the compiler's ordering is all that is needed
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int MP, int NL, int NB>
__global__ __launch_bounds__(256) void k_episode_jl(DevCfg c, DevState s, const float* __restrict__ params, Outputs o) {
  using S = JlShape<NL>;
  constexpr int G = S::G, EPB = S::EPB, SPW = S::SPW;
  extern __shared__ double lds_jl[];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  double* ex = lds_jl + w * (16 * 64);  // this wave's two chunk buffers: a^2 of sample j at [j * 64 + lane]
  const int g = lane / NL, d = lane - g * NL;
  const int64_t N = c.N;
  const int slot = w * G + g;           // env of this lane within the workgroup
  const int64_t e0 = (int64_t)blockIdx.x * EPB + slot;
  const bool valid = g < G && e0 < N;
  const int64_t e = valid ? e0 : N - 1;   // clamped: loads stay in bounds, nothing is stored
  const uint64_t vmask = __ballot(valid);
  const int64_t wst = ((int64_t)blockIdx.x * S::WAVES + w) * 64;   // diagnostics build: stamp slot of this wave
  FGX_STAMP(o, wst, 6);
  FGX_STAMP(o, wst, 0);

  // ---- the env's segment; wave-uniform bounds over the valid lanes
  JpSeg sg;
  sg.init(c, s, e, valid);
  const int Lmin = wave_min(valid ? sg.L : 0x7fffffff), Lmax = wave_max(valid ? sg.L : 0);
  const int lead = vmask ? __builtin_ctzll(vmask) : 0;

  // ---- this lane's joint
  double pg = c.pg[0], dg = c.dg[0];
#pragma unroll
  for (int j = 1; j < NL; ++j) {
    pg = (j == d) ? c.pg[j] : pg;
    dg = (j == d) ? c.dg[j] : dg;
  }
  const int nb = NB ? NB : c.nb;
  double q = s.q[d * N + e], qd = s.qd[d * N + e];
  Traj<MP, 1, NB> tg;
  const int s0 = c.replan ? sg.steps : 0;   // init_time = current_traj_steps * dt when replanning
  auto init_traj = [&]() __attribute__((always_inline)) {
    const bool has_cond = c.cond_desired && (sg.flags & 2u);
    const double ic_q = has_cond ? (double)s.cond[d * N + e] : q;
    const double ic_qd = has_cond ? (double)s.cond[(NL + d) * N + e] : qd;
    const float* pe = params + e * c.n_params;
    if (MP == MP_PRODMP)
      tg.init(c, pe + d * (nb + 1), s.tables, s0, &ic_q, &ic_qd, c.T, c.tau32, c.rcp_tau32);
    else
      tg.init(c, pe + d * nb, s.tables, s0, &ic_q, &ic_qd, c.T, c.tau32, c.rcp_tau32, NL * nb + d - d * nb);
  };
  init_traj();
  // basis rows through scalar loads when every valid lane's plan starts on the same row
  const int s0u = __builtin_amdgcn_readlane(s0, lead);
  const bool s0_uni = __ballot(valid && s0 != s0u) == 0;
  const cfloat_ptr stab = (cfloat_ptr)(uintptr_t)s.tables + (size_t)s0u * tg.str();
  tg.stab = stab;

  const double act_lo = __builtin_canonicalize(c.act_lo), act_hi = __builtin_canonicalize(c.act_hi);
  const double dt = c.dt;
  double cfk = 0.0;   // sum a^2 of the sample that needs FK (owned by the lane of its slot)
  float posl = 0.0f, vell = 0.0f;   // desired state of the segment's last sample (condition_on_desired)
  uint64_t nanm = 0;

  // desired (pos, vel) of the 8 samples of chunk k0 (samples >= T are never run: left 0).
  // FAST: every sample < T - 1 (no plan-end branch).  ProMP / ProDMP samples are independent fma
  // chains (8-way ILP); DMP is one f32 recurrence that overlaps the previous chunk's f64 chain.
  auto traj = [&](int k0, float* P, float* V, auto fast, auto sc) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float p1[1] = {0.0f}, v1[1] = {0.0f};
      if constexpr (decltype(fast)::value) tg.template at<true, decltype(sc)::value>(c, k0 + j, p1, v1);
      else if (k0 + j < c.T) tg.template at<false, decltype(sc)::value>(c, k0 + j, p1, v1);
      P[j] = p1[0];
      V[j] = v1[0];
    }
  };
  // the joint's PD -> clip -> torque Euler recurrence over chunk k0 (black_box_wrapper.py:201-205,
  // base_reacher_torque.py:20-37): sq[j] = a^2.  FAST: every valid lane runs all 8 samples.  EXACT:
  // np.clip's NaN propagation; otherwise a NaN u is recorded in nanm (the chunk is then re-run)
  auto dyn = [&](int k0, const float* P, const float* V, double* sq, auto fast, auto exact)
      __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sq[j] = 0.0;
      if (decltype(fast)::value || k0 + j < sg.L) {
        const double u = fadd(pg * fsub((double)P[j], q), dg * fsub((double)V[j], qd));
        double a = clip_nonan(u, act_lo, act_hi);
        if constexpr (decltype(exact)::value) a = (u != u) ? u : a;
        else nanm |= __ballot(u != u);
        qd = fadd(qd, dt * a);
        q = fadd(q, dt * qd);
        sq[j] = a * a;
      }
      if (!decltype(fast)::value && k0 + j == sg.L - 1) { posl = P[j]; vell = V[j]; }
    }
  };
  // ---- pairwise slots owned by this lane: j = d + NL * sl (two LDS buffers of 8 rows per wave:
  // chunk ch writes buffer ch & 1 while chunk ch - 1's rows are reduced from the other)
  double A[SPW], B[SPW], Tl[SPW];
#pragma unroll
  for (int sl = 0; sl < SPW; ++sl) { A[sl] = -0.0; B[sl] = -0.0; Tl[sl] = 0.0; }   // -0.0 + r == r
  const int gr = g < G ? g : G - 1;   // idle lanes read (and discard) the last env's rows
  auto write_sq = [&](int ch, const double* sq) __attribute__((always_inline)) {
    double* b = ex + (ch & 1) * 512;
#pragma unroll
    for (int j = 0; j < 8; ++j) b[j * 64 + lane] = sq[j];
  };
  // sum_d a_d^2 in joint order, the reward 0 - ctrl (rdist = 0 below env step 199) and numpy's
  // pairwise slots, branch-free (selects); chunk ch < 0 changes nothing
  auto reduce = [&](int ch) __attribute__((always_inline)) {
    const double* b = ex + (ch & 1) * 512;
#pragma unroll
    for (int sl = 0; sl < SPW; ++sl) {
      const int j = d + NL * sl;
      const bool ok = j < 8 && ch >= 0;
      const int jj = j < 8 ? j : 0;
      const int k = ch * 8 + jj;
      const double* row = b + jj * 64 + gr * NL;
      double ctrl = row[0];
#pragma unroll
      for (int dd = 1; dd < NL; ++dd) ctrl = fadd(ctrl, row[dd]);
      const double r = 0.0 - ctrl;
      const bool fk = ok && k == sg.k_fk;   // reward finished after the loop, with FK
      const bool add = ok && !fk;
      cfk = fk ? ctrl : cfk;
      const double a1 = fadd(A[sl], r), b1 = fadd(B[sl], r);
      A[sl] = (add && k < sg.hs) ? a1 : A[sl];
      B[sl] = (add && k >= sg.hs && k < sg.bend) ? b1 : B[sl];
      Tl[sl] = (add && k >= sg.bend && k < sg.L) ? r : Tl[sl];
    }
  };

  // Generic chunk loop (any wave): chunk ch's f64 recurrence, chunk ch - 1's reduction with
  // per-lane phases (selects), chunk ch + 1's trajectory after the exchange.
  float P[8], V[8], Pn[8], Vn[8];
  double sq[8];
  auto slow_range = [&](int c0, int nchunks, auto sc, auto exact) __attribute__((always_inline)) {
    for (int ch = c0; ch < nchunks; ++ch) {
      const int k0 = ch * 8;
      dyn(k0, P, V, sq, std::false_type{}, exact);
      reduce(ch - 1);
      write_sq(ch, sq);
      wave_lds_sync();
      if (ch + 1 < nchunks) traj(k0 + 8, P, V, std::false_type{}, sc);
    }
    reduce(nchunks - 1);
  };

  // Fast chunk pipeline (waves whose valid lanes share one segment layout and plan start row): one
  // branch-free basic block per chunk that evaluates chunk ch + 1's trajectory (independent f32
  // work, basis rows by scalar loads at constant offsets from one chunk base), runs chunk ch's f64
  // recurrence, reduces chunk ch - 1 into one pairwise phase fixed at compile time (PH 1: the
  // first-half slots A, PH 2: the second-half slots B) and writes chunk ch's rows.  A lone wave
  // per SIMD (shard sizes) issues every instruction, SALU and selects included, at ~6 cycles:
  // nothing here is per-lane control flow.
  float plast = 0.0f, vlast = 0.0f;   // desired state of the last fast sample
  auto traj_fast = [&](int k0, float* Pt, float* Vt) __attribute__((always_inline)) {
    const cfloat_ptr base = tg.stab + (size_t)k0 * tg.str();
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float p1[1], v1[1];
      tg.template at_rows<true>(c, k0 + j, base + (j + 1) * tg.str(), p1, v1);
      Pt[j] = p1[0];
      Vt[j] = v1[0];
    }
  };
  auto reduce_fast = [&](int ch, auto ph) __attribute__((always_inline)) {
    const double* b = ex + (ch & 1) * 512;
#pragma unroll
    for (int sl = 0; sl < SPW; ++sl) {
      const int j = d + NL * sl;
      const int jj = j < 8 ? j : 0;   // (lanes without this slot accumulate a discarded sum)
      const double* row = b + jj * 64 + gr * NL;
      double ctrl = row[0];
#pragma unroll
      for (int dd = 1; dd < NL; ++dd) ctrl = fadd(ctrl, row[dd]);
      const double r = 0.0 - ctrl;
      if constexpr (decltype(ph)::value == 1) A[sl] = fadd(A[sl], r);
      else B[sl] = fadd(B[sl], r);
    }
  };
  auto fast_iter = [&](int ch, const float* Pc, const float* Vc, float* Pt, float* Vt, auto ph)
      __attribute__((always_inline)) {
    const int k0 = ch * 8;
    traj_fast(k0 + 8, Pt, Vt);
    dyn(k0, Pc, Vc, sq, std::true_type{}, std::false_type{});
    if constexpr (decltype(ph)::value != 0) reduce_fast(ch - 1, ph);
    write_sq(ch, sq);
    wave_lds_sync();
    plast = Pc[7];
    vlast = Vc[7];
  };
  // chunks [c0, c1) with reduction phase PH; P / V hold chunk c0's trajectory on entry and chunk
  // c1's on exit (two iterations per trip: the look-ahead buffers swap roles, no copies)
  auto fast_range = [&](int c0, int c1, auto ph) __attribute__((always_inline)) {
    int ch = c0;
    for (; ch + 1 < c1; ch += 2) {
      fast_iter(ch, P, V, Pn, Vn, ph);
      fast_iter(ch + 1, Pn, Vn, P, V, ph);
    }
    if (ch < c1) {
      fast_iter(ch, P, V, Pn, Vn, ph);
#pragma unroll
      for (int j = 0; j < 8; ++j) { P[j] = Pn[j]; V[j] = Vn[j]; }
    }
  };

  // EXACT = false records NaN controls in nanm instead of propagating them; the caller then re-runs
  // the whole segment with EXACT = true on the generic loop.
  auto run = [&](auto sc, auto exact) __attribute__((always_inline)) {
    const int nchunks = (Lmax + 7) / 8;
    if (nchunks == 0) return;
    traj(0, P, V, std::false_type{}, sc);
    int ch = 0;
    if constexpr (decltype(sc)::value && !decltype(exact)::value) {
      if (Lmin == Lmax) {   // one segment layout for the wave: uniform phases
        const int L = Lmin;
        const int hs = __builtin_amdgcn_readlane(sg.hs, lead), bend = __builtin_amdgcn_readlane(sg.bend, lead);
        const int kfk = __builtin_amdgcn_readlane(sg.k_fk, lead);
        // fast iteration ch: chunk ch runs on every lane (8 ch + 8 <= L), chunk ch + 1's samples
        // are below T - 1 (8 ch + 16 < T), and chunk ch - 1 lies before the tail and the FK sample
        // (8 ch <= bend, 8 ch <= kfk)
        int nf = min(L / 8, (c.T - 16 + 7) / 8);
        nf = min(nf, bend / 8 + 1);
        if (kfk < 0x7fffffff) nf = min(nf, kfk / 8 + 1);
        nf = max(0, min(nf, nchunks));
        if (nf > 0) {
          fast_range(0, 1, std::integral_constant<int, 0>{});
          const int na = min(nf, hs / 8 + 1);   // iterations reducing first-half chunks
          fast_range(1, na, std::integral_constant<int, 1>{});
          fast_range(max(1, na), nf, std::integral_constant<int, 2>{});
          ch = nf;
          if (8 * ch == L) { posl = plast; vell = vlast; }
        }
      }
    }
    FGX_STAMP(o, wst, 2);
    slow_range(ch, nchunks, sc, exact);
  };
  // the segment from its start state (re-run after a NaN control)
  auto restart = [&]() __attribute__((always_inline)) {
    q = s.q[d * N + e];
    qd = s.qd[d * N + e];
    init_traj();
    tg.stab = stab;
    cfk = 0.0;
#pragma unroll
    for (int sl = 0; sl < SPW; ++sl) { A[sl] = -0.0; B[sl] = -0.0; Tl[sl] = 0.0; }
  };
  nanm = 0;
  FGX_STAMP(o, wst, 1);
  if (s0_uni) run(std::true_type{}, std::false_type{});
  else run(std::false_type{}, std::false_type{});
  if (__builtin_expect((nanm & vmask) != 0, 0)) {   // a NaN control: np.clip semantics from the start
    wave_lds_sync();
    restart();
    if (s0_uni) run(std::true_type{}, std::true_type{});
    else run(std::false_type{}, std::true_type{});
  }

  if (valid && sg.stop && c.cond_desired) {   // black_box_wrapper.py:234-236
    s.cond[d * N + e] = posl;
    s.cond[(NL + d) * N + e] = vell;
  }

  FGX_STAMP(o, wst, 3);
  // ---- gather per env (SoA [field][EPB]): slot sums, the FK sample's control cost, joint state
  __syncthreads();   // every wave is done with its chunk rows (the gather area overlaps them)
  double* ga = lds_jl;
  if (g < G) {
#pragma unroll
    for (int sl = 0; sl < SPW; ++sl) {
      const int j = d + NL * sl;
      if (j < 8) {
        ga[(3 * j) * EPB + slot] = A[sl];
        ga[(3 * j + 1) * EPB + slot] = B[sl];
        ga[(3 * j + 2) * EPB + slot] = Tl[sl];
      }
    }
    if (sg.k_fk < sg.L && ((sg.k_fk & 7) % NL) == d) ga[24 * EPB + slot] = cfk;
    ga[(25 + d) * EPB + slot] = q;
    ga[(25 + NL + d) * EPB + slot] = qd;
  }
  __syncthreads();

  // ---- one thread per env: return and epilogue
  const int t = threadIdx.x;
  const int64_t et = (int64_t)blockIdx.x * EPB + t;
  const bool tv = t < EPB && et < N;
  if (o.inner_steps) {   // sum of trajectory lengths: one atomic per wave
    JpSeg st;
    st.init(c, s, tv ? et : N - 1, tv);
    long long sum = tv ? st.L : 0;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off, 64);
    if (lane == 0 && sum != 0) atomicAdd((unsigned long long*)o.inner_steps, (unsigned long long)sum);
  }
  FGX_STAMP(o, wst, 4);
  if (!tv) {
    FGX_STAMP(o, wst, 5);
    FGX_STAMP(o, wst, 7);
    return;
  }
  JpSeg st;
  st.init(c, s, et, true);
  Env<NL> v;
  load_env(c, s, et, v, false);   // SimpleReacher: no hole / reward state
#pragma unroll
  for (int k = 0; k < NL; ++k) { v.q[k] = ga[(25 + k) * EPB + t]; v.qd[k] = ga[(25 + NL + k) * EPB + t]; }
  v.steps = st.steps + st.L;
  if (st.stop && c.cond_desired) v.flags |= 2u;
  v.fk();
  // the last sample at env step 199 (simple_reacher.py:60-62): r = -dist(ee, goal) - sum a^2; it is
  // the last element of the return sum, either the sequential tail's last or slot 7 of the last
  // 8-block (L == bend)
  const int L = st.L, bend = st.bend;
  const bool fk_last = st.k_fk < L;
  const double r_fk = fk_last ? -norm2(v.jx[NL] - v.gx, v.jy[NL] - v.gy) - ga[24 * EPB + t] : 0.0;
  double sa[8], sb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sa[j] = ga[(3 * j) * EPB + t]; sb[j] = ga[(3 * j + 1) * EPB + t]; }
  if (fk_last && L == bend && L >= 8) sb[7] = sb[7] + r_fk;
  double res = (L >= 8) ? PairwiseSum::comb(sb) : 0.0;
  const int ntail = L - bend;
#pragma unroll
  for (int j = 0; j < 8; ++j)
    if (j < ntail) res = res + ((fk_last && j == ntail - 1) ? r_fk : ga[(3 * j + 2) * EPB + t]);
  if (L > 128) res = PairwiseSum::comb(sa) + res;
  const bool trunc = v.steps >= c.max_steps;
  episode_epilogue(c, s, o, et, v, st.plans, L, res, false, trunc, false);
  FGX_STAMP(o, wst, 5);
  FGX_STAMP(o, wst, 7);
}

}  // namespace fgx
