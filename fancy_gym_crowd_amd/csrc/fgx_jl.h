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

typedef float jl_f4 __attribute__((ext_vector_type(4)));

// HLP: one joint wave and one helper wave per workgroup (k_episode_jl's helper form, below);
// 1: the helper hands over f32 trajectory chunks and the joint wave writes a^2, 2: f64 chunks (the
// conversions on the helper) and the joint wave writes a (the squares on the helper)
template <int NL, int HLP = 0>
struct JlShape {
  static constexpr int G = 64 / NL;             // envs per wave
  static constexpr int WAVES = HLP ? 1 : 4;     // joint waves per workgroup
  static constexpr int EPB = G * WAVES;         // envs per workgroup
  static constexpr int SPW = (8 + NL - 1) / NL; // pairwise slots owned per lane
  static constexpr int THREADS = 64 * WAVES * (HLP ? 2 : 1);
  // the plain form may add a reset wave after the joint waves (kernel argument rw): the workgroup's
  // VectorEnv auto-resets, run while the joint waves run their episodes
  static constexpr int MAXT = THREADS + (HLP ? 0 : 64);
  // gathered f64 per env: A, B, tail (8 each), cfk, q, qd, then cos / sin of the cumulative angles
  // (FK) and of every q (observation), then the env's stored steps, plan count, flags and goal
  static constexpr int GX = 25 + 6 * NL;
  static constexpr int GF = GX + 5;
  // row stride (doubles) of the a^2 exchange rows.  The owner lane of slot j reads a^2 of joint dd
  // of env g at row j, column g NL + dd; with 64-double rows every row starts on the same bank, so
  // the NL lanes of one env (rows d, d + NL, ...) hit one bank pair: 5-way conflicts for 5 links
  // (PMC SQ_LDS_BANK_CONFLICT = 63% of SQ_LDS_IDX_ACTIVE at 65536 envs,
  // profiles/r02_stall_probe.json).  An odd stride spreads the rows over the banks (modelled
  // ds_read_b64 group cycles per chunk, tools/lds_bank_model.py): 5 links use 60 columns, stride 61
  // (90 -> 40, the LDS footprint shrinks; the 4 idle lanes do not write), 2 links stride 65
  // (32 -> 16, conflict-free; the gather area is larger anyway).  Writes stay conflict-free.
  static constexpr int XS = (G * NL < 64) ? G * NL + 1 : 65;
  // HLP: after the exchange rows, the helper's two trajectory chunk buffers ([buf][PVQ][lane] 16-B
  // quads: HLP 1 P[0..3], P[4..7], V[0..3], V[4..7] as f32; HLP 2 P[0..1] .. V[6..7] as f64) and its
  // hand-over record (the pairwise slots, the look-ahead)
  static constexpr int PVQ = HLP == 2 ? 8 : 4;
  static constexpr size_t ex_bytes() { return ((size_t)WAVES * 16 * XS * sizeof(double) + 15) & ~(size_t)15; }
  static constexpr size_t pv_bytes() { return HLP ? (size_t)2 * PVQ * 64 * 16 : 0; }
  static constexpr size_t ho_bytes() { return HLP ? (size_t)64 * (2 * SPW + 1) * sizeof(double) : 0; }
  static constexpr size_t lds_bytes() {
    const size_t ex = ex_bytes() + pv_bytes() + ho_bytes();
    const size_t ga = (size_t)GF * EPB * sizeof(double);
    return ex > ga ? ex : ga;
  }
};

// gw: envs per wave actually used (<= G; experiments, FGX_JL_GW); LDS slots keep the compile-time
// stride G.
//
// HLP (the helper form; ProMP with the column table only, host-selected): a workgroup is one joint
// wave and one helper wave for the same G envs (lane l of both = env l / NL, joint l % NL).  The two
// waves of a workgroup run on different SIMDs (profiles/r01_wave_placement.txt), and at the shard
// sizes most SIMDs are otherwise idle.  Over the fast chunks the joint wave keeps only the f64
// PD -> clip -> Euler chain (and the a^2 rows); the helper evaluates chunk ch + 1's trajectory into
// an LDS buffer and reduces chunk ch - 1's a^2 rows into the pairwise slots while the joint wave runs
// chunk ch, one workgroup barrier per chunk.  Both waves derive the fast-path decision from the same
// loads (segment bounds, plan start, NaN-free guard), so they agree on the barrier count without
// talking; after the last fast chunk the helper hands the pairwise slots and the look-ahead over and
// the joint wave continues exactly as k_episode_jl (slow chunks, NaN re-run, gather, epilogue), the
// helper wave's threads running the auto-resets of the split group.  Same operations in the same
// order: bit-identical.
//
// rw (plain form, host-chosen): the workgroup has a fifth wave, the reset wave, which runs the
// auto-resets from the launch on (below); otherwise the reset group after the gather does.
template <int MP, int NL, int NB, int HLP = 0>
__global__ __launch_bounds__((JlShape<NL, HLP>::MAXT)) void k_episode_jl(DevCfg c, DevState s,
                                                                       const float* __restrict__ params,
                                                                       Outputs o, int gw, int rw) {
  using S = JlShape<NL, HLP>;
  constexpr int G = S::G, EPB = S::EPB, SPW = S::SPW;
  constexpr int NBL = NB > 0 ? NB : 1;
  extern __shared__ double lds_jl[];
  const int lane = threadIdx.x & 63;
  const bool helper = HLP && (int)(threadIdx.x >> 6) >= S::WAVES;
  const bool rwave = !HLP && rw && (int)(threadIdx.x >> 6) == S::WAVES;
  const int w = helper ? (int)(threadIdx.x >> 6) - S::WAVES : (int)(threadIdx.x >> 6);
  constexpr int XS = S::XS;
  double* ex = lds_jl + w * (16 * XS);  // this wave's two chunk buffers: a^2 of sample j at [j * XS + lane]
  const int g = lane / NL, d = lane - g * NL;
  const int64_t N = c.N;
  const int slot = w * G + g;           // LDS slot of this lane's env
  const int64_t e0 = (int64_t)blockIdx.x * (S::WAVES * gw) + w * gw + g;
  const bool valid = g < gw && e0 < N;
  const int64_t e = valid ? e0 : N - 1;   // clamped: loads stay in bounds, nothing is stored
  const uint64_t vmask = __ballot(valid);
  // diagnostics build: stamp slot of this wave (the helper's: none)
  const int64_t wst = (helper || rwave) ? (int64_t)16384 * 64 : ((int64_t)blockIdx.x * S::WAVES + w) * 64;
  FGX_STAMP(o, wst, 6);
  FGX_STAMP(o, wst, 0);

  // ---- the reset wave (plain form): the VectorEnv auto-reset of every env of the workgroup whose
  // segment ends in truncation (SimpleReacher never terminates).  It depends only on the env's PCG64
  // stream, start angle and segment words -- all known before the episode -- so it runs from the
  // launch on, beside the joint waves (section clocks: as the epilogue's reset group after the
  // gather it was the launch's last ~7.7 k cycles, profiles/r03_stamps_s17.jsonl).  Its inputs are
  // read first; it writes the env state only after the barrier by which every joint wave holds its
  // env's state (q, q̇, segment words, goal) in registers.  It then leaves: the joint waves' later
  // barriers wait on the surviving waves only.
  if constexpr (!HLP) {
    if (rwave) {
      constexpr int NR = (EPB + 63) / 64;
      bool rdo[NR];
      int64_t rer[NR];
      Pcg64 rgs[NR];
      double rsp[NR];
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        const int t1 = lane + 64 * i, tw1 = t1 / G, tg1 = t1 - tw1 * G;
        rer[i] = (int64_t)blockIdx.x * (S::WAVES * gw) + tw1 * gw + tg1;
        rdo[i] = o.autoreset && t1 < EPB && tg1 < gw && rer[i] < N;
        if (rdo[i]) {
          JpSeg sr;
          sr.init(c, s, rer[i], true);
          rdo[i] = sr.steps + sr.L >= c.max_steps;
        }
        rsp[i] = 0.0;
        if (rdo[i]) {
          rgs[i] = load_rng(s.rng, N, rer[i]);
          rsp[i] = s.start[rer[i]];
        }
      }
      __syncthreads();   // R: the joint waves' env state is in their registers
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        if (rdo[i]) {
          const int64_t er = rer[i];
          Env<NL> vr;
          if (!c.random_start) vr.sp = rsp[i];
          vr.reset(c, rgs[i], false, 0);
          store_rng(s.rng, N, er, rgs[i]);
          if (c.random_start) s.start[er] = vr.sp;
          emit_obs(c, vr, c.return_context, o.obs + er * c.out_dim, nullptr, true);
          store_env(c, s, er, vr, false);   // SimpleReacher: no hole / reward state
          s.plans[er] = 0;
        }
      }
      return;
    }
  }

  // the joint's state first: its loads need nothing the segment computes (they are in flight while
  // the segment's loads return and its wave reductions run)
  double q = s.q[d * N + e], qd = s.qd[d * N + e];
  const double q_in = q, qd_in = qd;   // (a NaN re-run restarts from these: the reset wave may have
                                       // overwritten the stored state by then)
  // ---- the env's segment; wave-uniform bounds over the valid lanes
  JpSeg sg;
  sg.init(c, s, e, valid);
  const int Lmin = wave_min_dpp(valid ? sg.L : 0x7fffffff), Lmax = wave_max_dpp(valid ? sg.L : 0);
  const int lead = vmask ? __builtin_ctzll(vmask) : 0;
  FGX_STAMP(o, wst, 12);

  // ---- this lane's joint
  double pg = c.pg[0], dg = c.dg[0];
#pragma unroll
  for (int j = 1; j < NL; ++j) {
    pg = (j == d) ? c.pg[j] : pg;
    dg = (j == d) ? c.dg[j] : dg;
  }
  const int nb = NB ? NB : c.nb;
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
  double gx = 0.0, gy = 0.0;   // the env's goal, for the return thread (FK reward, observation)
  if (d == 0) { gx = s.goal[e]; gy = s.goal[N + e]; }
  if constexpr (!HLP)
    if (rw) __syncthreads();   // R: the reset wave may overwrite the env state after this
  FGX_STAMP(o, wst, 13);
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
  // base_reacher_torque.py:20-37): sq[j] = a^2.  FAST: every valid lane runs all 8 samples.  EXACT
  // 1: np.clip's NaN propagation; 0: a NaN u is recorded in nanm (the segment is then re-run);
  // 2: the wave is NaN-free (proven), neither
  auto dyn = [&](int k0, const float* P, const float* V, double* sq, auto fast, auto exact)
      __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sq[j] = 0.0;
      if (decltype(fast)::value || k0 + j < sg.L) {
        const double u = fadd(pg * fsub((double)P[j], q), dg * fsub((double)V[j], qd));
        double a = __builtin_fmin(__builtin_fmax(u, act_lo), act_hi);   // v_max / v_min: a NaN u gives a bound
        if constexpr (decltype(exact)::value == 1) a = (u != u) ? u : a;
        else if constexpr (decltype(exact)::value == 0) nanm |= __ballot(u != u);
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
    double* b = ex + (ch & 1) * (8 * XS);
    if (G * NL == 64 || lane < G * NL) {   // (rows hold G NL columns: idle lanes must not write)
#pragma unroll
      for (int j = 0; j < 8; ++j) b[j * XS + lane] = sq[j];
    }
  };
  // sum_d a_d^2 in joint order, the reward 0 - ctrl (rdist = 0 below env step 199) and numpy's
  // pairwise slots, branch-free (selects); chunk ch < 0 changes nothing
  auto reduce = [&](int ch) __attribute__((always_inline)) {
    const double* b = ex + (ch & 1) * (8 * XS);
#pragma unroll
    for (int sl = 0; sl < SPW; ++sl) {
      const int j = d + NL * sl;
      const bool ok = j < 8 && ch >= 0;
      const int jj = j < 8 ? j : 0;
      const int k = ch * 8 + jj;
      const double* row = b + jj * XS + gr * NL;
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
  // work, basis rows by scalar loads), runs chunk ch's f64 recurrence, reduces chunk ch - 1 into
  // one pairwise phase fixed at compile time (PH 1: the first-half slots A, PH 2: the second-half
  // slots B) and writes chunk ch's rows.  A lone wave per SIMD (shard sizes) issues every
  // instruction, SALU and selects included, at ~6 cycles: nothing here is per-lane control flow.
  //
  // ProMP (PKT): the chunk's trajectory comes from the column-major table (DevState::tables_t):
  // one 8-row scalar load per basis column and per dt column, the 8 look-ahead positions as 4
  // pairs of samples (v_pk_fma_f32 over two table rows, the same k-ordered fma chain per sample),
  // the forward differences and div_rcp on the same pairs: bit-identical to Traj::at.  Chunks past
  // the plan's end read rows inside the padded table and are never run; the plan's last sample
  // (vel = the previous velocity, Traj::at's k == T - 1 branch) is patched once, in a peeled
  // iteration.  ProMP waves take the fast path only when NaN-free (the k_episode guard), so the
  // fast recurrence records no NaN controls.
  constexpr bool PKT = (MP == MP_PROMP) && NB > 0;
  typedef float f8u __attribute__((ext_vector_type(8), aligned(4)));
  typedef const f8u __attribute__((address_space(4)))* cf8_ptr;
  float plast = 0.0f, vlast = 0.0f;   // desired state of the last fast sample
  // ProMP chunk columns: basis columns j (rows R + 2 ..), dt and 1/dt (rows R + 1 ..) of chunk k0
  struct Cols { f8u b[NBL]; f8u dt, rd; };
  auto traj_load = [&](int k0, Cols& cl) __attribute__((always_inline)) {
    if constexpr (PKT) {
      const int RT = tables_t_rows(c.rows);
      const int R = s0u + k0;   // absolute row of sample k0: its dt row is R + 1, its next basis row R + 2
      const cfloat_ptr tt = (cfloat_ptr)(uintptr_t)s.tables_t;
#pragma unroll
      for (int j = 0; j < NBL; ++j) cl.b[j] = *(cf8_ptr)(tt + (size_t)j * RT + R + 8);
      cl.dt = *(cf8_ptr)(tt + (size_t)NBL * RT + R + 8);
      cl.rd = *(cf8_ptr)(tt + (size_t)(NBL + 1) * RT + R + 8);
    }
  };
  auto traj_fast = [&](int k0, const Cols& cl, float* Pt, float* Vt) __attribute__((always_inline)) {
    if constexpr (PKT) {
      // sample pairs (2i, 2i + 1): rows (R + 2 + 2i, R + 3 + 2i) of basis column j, and the dt / 1/dt
      // entries of rows (R + 1 + 2i, R + 2 + 2i)
      f32x2 acc[4] = {};
#pragma unroll
      for (int j = 0; j < NBL; ++j) {
        const f8u col = cl.b[j];
        const f32x2 wj = (f32x2)tg.w[0][j];
        acc[0] = __builtin_elementwise_fma(__builtin_shufflevector(col, col, 0, 1), wj, acc[0]);
        acc[1] = __builtin_elementwise_fma(__builtin_shufflevector(col, col, 2, 3), wj, acc[1]);
        acc[2] = __builtin_elementwise_fma(__builtin_shufflevector(col, col, 4, 5), wj, acc[2]);
        acc[3] = __builtin_elementwise_fma(__builtin_shufflevector(col, col, 6, 7), wj, acc[3]);
      }
      const f8u dt8 = cl.dt, rd8 = cl.rd;
      const f32x2 rdp[4] = {__builtin_shufflevector(rd8, rd8, 0, 1), __builtin_shufflevector(rd8, rd8, 2, 3),
                            __builtin_shufflevector(rd8, rd8, 4, 5), __builtin_shufflevector(rd8, rd8, 6, 7)};
      const f32x2 dtp[4] = {__builtin_shufflevector(dt8, dt8, 0, 1), __builtin_shufflevector(dt8, dt8, 2, 3),
                            __builtin_shufflevector(dt8, dt8, 4, 5), __builtin_shufflevector(dt8, dt8, 6, 7)};
      float cr[9];
      cr[0] = tg.cur[0];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        cr[2 * i + 1] = acc[i].x;
        cr[2 * i + 2] = acc[i].y;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x2 x = {cr[2 * i + 1] - cr[2 * i], cr[2 * i + 2] - cr[2 * i + 1]};
        const f32x2 rd = rdp[i], dd = dtp[i];
        const f32x2 qv = x * rd;                                     // div_rcp on the pair
        const f32x2 er = __builtin_elementwise_fma(-qv, dd, x);
        const f32x2 vl = __builtin_elementwise_fma(er, rd, qv);
        Pt[2 * i] = cr[2 * i];
        Pt[2 * i + 1] = cr[2 * i + 1];
        Vt[2 * i] = vl.x;
        Vt[2 * i + 1] = vl.y;
      }
      tg.cur[0] = cr[8];
      tg.vprev[0] = Vt[7];
    } else {
      (void)cl;
      const cfloat_ptr base = tg.stab + (size_t)k0 * tg.str();
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float p1[1], v1[1];
        tg.template at_rows<true>(c, k0 + j, base + (j + 1) * tg.str(), p1, v1);
        Pt[j] = p1[0];
        Vt[j] = v1[0];
      }
    }
  };
  auto reduce_load = [&](int ch, double (*rv)[NL]) __attribute__((always_inline)) {
    const double* b = ex + (ch & 1) * (8 * XS);
#pragma unroll
    for (int sl = 0; sl < SPW; ++sl) {
      const int j = d + NL * sl;
      const int jj = j < 8 ? j : 0;   // (lanes without this slot accumulate a discarded sum)
      const double* row = b + jj * XS + gr * NL;
#pragma unroll
      for (int dd = 0; dd < NL; ++dd) rv[sl][dd] = row[dd];
    }
  };
  auto reduce_fast = [&](double (*rv)[NL], auto ph) __attribute__((always_inline)) {
#pragma unroll
    for (int sl = 0; sl < SPW; ++sl) {
      double ctrl = rv[sl][0];
#pragma unroll
      for (int dd = 1; dd < NL; ++dd) ctrl = fadd(ctrl, rv[sl][dd]);
      const double r = 0.0 - ctrl;
      if constexpr (decltype(ph)::value == 1) A[sl] = fadd(A[sl], r);
      else B[sl] = fadd(B[sl], r);
    }
  };
  // the chunk holding the plan's last sample T - 1 (computed as a look-ahead like any other chunk)
  // gets Traj::at's k == T - 1 velocity (the previous one) before it runs: a uniform branch at the
  // top of the iteration, outside the chunk's basic block
  const int cpch = (c.T - 1) / 8, ip = (c.T - 1) & 7;
  auto fast_iter = [&](int ch, float* Pc, float* Vc, float* Pt, float* Vt, auto ph) __attribute__((always_inline)) {
    const int k0 = ch * 8;
    if constexpr (PKT) {
      if (__builtin_expect(ch == cpch, 0)) {
        float prev = vlast;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float vj = Vc[j];
          if (j == ip) Vc[j] = prev;
          prev = vj;
        }
      }
    }
    // issue the chunk's memory reads first (scalar column loads, the previous chunk's LDS rows): their
    // latency runs under the f64 recurrence
    Cols cl;
    traj_load(k0 + 8, cl);
    double rv[SPW][NL];
    if constexpr (decltype(ph)::value != 0) reduce_load(ch - 1, rv);
    __builtin_amdgcn_sched_barrier(0);
    traj_fast(k0 + 8, cl, Pt, Vt);
    dyn(k0, Pc, Vc, sq, std::true_type{}, std::integral_constant<int, PKT ? 2 : 0>{});   // ProMP: NaN-free
    if constexpr (decltype(ph)::value != 0) reduce_fast(rv, ph);
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
  // ProMP NaN-free waves (k_episode's guard): with |w| < c.wbound32 and |q|, |qd|, |p|, |d| < 1e150 every
  // PD control u of the plan is finite, so np.clip's NaN propagation never applies
  bool nan_free = true;
  if constexpr (PKT) {
    bool ok = __builtin_fabs(c.act_lo) <= 1e3 && __builtin_fabs(c.act_hi) <= 1e3 && c.dt <= 1.0 &&
              __builtin_fabs(q) < 1e150 && __builtin_fabs(qd) < 1e150 && __builtin_fabs(pg) < 1e150 &&
              __builtin_fabs(dg) < 1e150;
#pragma unroll
    for (int j = 0; j < NBL; ++j) ok = ok && __builtin_fabsf(tg.w[0][j]) < c.wbound32;
    nan_free = __ballot(valid && !ok) == 0;
  }

  // EXACT = false records NaN controls in nanm instead of propagating them; the caller then re-runs
  // the whole segment with EXACT = true on the generic loop.
  // fast iterations of a wave whose valid lanes share one segment layout (0: none): chunk ch runs
  // on every lane (8 ch + 8 <= L), chunk ch - 1 lies before the tail and the FK sample (8 ch <= bend,
  // 8 ch <= kfk) and, generic trajectories only, chunk ch + 1's samples are below T - 1 (8 ch + 16 < T)
  auto fast_count = [&](int nchunks) __attribute__((always_inline)) -> int {
    if (Lmin != Lmax || !nan_free) return 0;
    const int L = Lmin;
    const int bend = __builtin_amdgcn_readlane(sg.bend, lead);
    const int kfk = __builtin_amdgcn_readlane(sg.k_fk, lead);
    int nf = min(L / 8, bend / 8 + 1);
    if (!PKT) nf = min(nf, (c.T - 16 + 7) / 8);
    if (kfk < 0x7fffffff) nf = min(nf, kfk / 8 + 1);
    return max(0, min(nf, nchunks));
  };
  // ---- HLP: the two sides of the fast chunks
  static_assert(!HLP || PKT, "the helper form runs ProMP's column-table chunks only");
  jl_f4* pvb = (jl_f4*)((char*)lds_jl + S::ex_bytes());                    // [buf][4][lane]
  double* hob = (double*)((char*)lds_jl + S::ex_bytes() + S::pv_bytes());  // [2 SPW + 1][lane]
  auto hl_barrier = [] {   // both waves' LDS operations done, then the workgroup barrier
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  typedef double jl_d2 __attribute__((ext_vector_type(2)));
  auto pv_put = [&](int ch, const float* Pv, const float* Vv) __attribute__((always_inline)) {
    jl_f4* b = pvb + (ch & 1) * (S::PVQ * 64) + lane;
    if constexpr (HLP == 2) {
      jl_d2* bd = (jl_d2*)b;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        bd[i * 64] = (jl_d2){(double)Pv[2 * i], (double)Pv[2 * i + 1]};
        bd[(4 + i) * 64] = (jl_d2){(double)Vv[2 * i], (double)Vv[2 * i + 1]};
      }
    } else {
      b[0] = (jl_f4){Pv[0], Pv[1], Pv[2], Pv[3]};
      b[64] = (jl_f4){Pv[4], Pv[5], Pv[6], Pv[7]};
      b[128] = (jl_f4){Vv[0], Vv[1], Vv[2], Vv[3]};
      b[192] = (jl_f4){Vv[4], Vv[5], Vv[6], Vv[7]};
    }
  };
  auto pv_get = [&](int ch, float* Pv, float* Vv) __attribute__((always_inline)) {
    const jl_f4* b = pvb + (ch & 1) * (S::PVQ * 64) + lane;
    if constexpr (HLP == 2) {
      const jl_d2* bd = (const jl_d2*)b;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const jl_d2 p = bd[i * 64], v = bd[(4 + i) * 64];
        Pv[2 * i] = (float)p[0]; Pv[2 * i + 1] = (float)p[1];
        Vv[2 * i] = (float)v[0]; Vv[2 * i + 1] = (float)v[1];
      }
    } else {
      const jl_f4 p0 = b[0], p1 = b[64], v0 = b[128], v1 = b[192];
#pragma unroll
      for (int j = 0; j < 4; ++j) { Pv[j] = p0[j]; Pv[4 + j] = p1[j]; Vv[j] = v0[j]; Vv[4 + j] = v1[j]; }
    }
  };
  auto pv_get_d = [&](int ch, double* Pd, double* Vd) __attribute__((always_inline)) {   // HLP 2
    const jl_d2* bd = (const jl_d2*)(pvb + (ch & 1) * (S::PVQ * 64) + lane);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const jl_d2 p = bd[i * 64], v = bd[(4 + i) * 64];
      Pd[2 * i] = p[0]; Pd[2 * i + 1] = p[1];
      Vd[2 * i] = v[0]; Vd[2 * i + 1] = v[1];
    }
  };
  // the helper: chunk 0's trajectory (Traj::at through the scalar rows, as run()), then per chunk ch
  // the trajectory of chunk ch + 1 (with the plan-end patch of fast_iter) and the reduction of chunk
  // ch - 1 in fast_range's phases; after the last chunk the hand-over record
  auto helper_fast = [&](int nf, int na) __attribute__((always_inline)) {
    traj(0, P, V, std::false_type{}, std::true_type{});
    float vl = 0.0f;   // fast_iter's vlast: the last (patched) velocity of the previous chunk
    auto patch = [&](int m, float* Vv) __attribute__((always_inline)) {
      if (__builtin_expect(m == cpch, 0)) {
        float prev = vl;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float vj = Vv[j];
          if (j == ip) Vv[j] = prev;
          prev = vj;
        }
      }
    };
    patch(0, V);
    vl = V[7];
    pv_put(0, P, V);
    hl_barrier();
    for (int ch = 0; ch < nf; ++ch) {
      const int k0 = ch * 8;
      Cols cl;
      traj_load(k0 + 8, cl);
      double rv[SPW][NL];
      if (ch >= 1) reduce_load(ch - 1, rv);
      __builtin_amdgcn_sched_barrier(0);
      traj_fast(k0 + 8, cl, Pn, Vn);
      patch(ch + 1, Vn);
      if constexpr (HLP == 2) {   // the joint wave wrote a: the squares here
#pragma unroll
        for (int sl = 0; sl < SPW; ++sl)
#pragma unroll
          for (int dd = 0; dd < NL; ++dd) rv[sl][dd] = rv[sl][dd] * rv[sl][dd];
      }
      vl = Vn[7];
      pv_put(ch + 1, Pn, Vn);
      if (ch >= 1) {
        if (ch < na) reduce_fast(rv, std::integral_constant<int, 1>{});
        else reduce_fast(rv, std::integral_constant<int, 2>{});
      }
      if (ch == nf - 1) {
#pragma unroll
        for (int sl = 0; sl < SPW; ++sl) { hob[sl * 64 + lane] = A[sl]; hob[(SPW + sl) * 64 + lane] = B[sl]; }
        hob[2 * SPW * 64 + lane] = __builtin_bit_cast(double, (f32x2){tg.cur[0], tg.vprev[0]});
      }
      hl_barrier();
    }
  };
  // the joint wave: per chunk the f64 chain on the helper's trajectory; then chunk nf's trajectory
  // (the slow chunks' first) and the hand-over
  auto joint_fast = [&](int nf) __attribute__((always_inline)) {
    hl_barrier();   // chunk 0's trajectory
    for (int ch = 0; ch < nf; ++ch) {
      if constexpr (HLP == 2) {
        // dyn's fast, NaN-free form on the helper's f64 chunk, writing a (the last fast chunk a^2:
        // the slow chunks reduce it here)
        double Pd[8], Vd[8];
        pv_get_d(ch, Pd, Vd);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const double u = fadd(pg * fsub(Pd[j], q), dg * fsub(Vd[j], qd));
          const double a = __builtin_fmin(__builtin_fmax(u, act_lo), act_hi);
          qd = fadd(qd, dt * a);
          q = fadd(q, dt * qd);
          sq[j] = a;
        }
        if (ch == nf - 1) {
#pragma unroll
          for (int j = 0; j < 8; ++j) sq[j] = sq[j] * sq[j];
        }
        plast = (float)Pd[7];
        vlast = (float)Vd[7];
      } else {
        pv_get(ch, P, V);
        dyn(ch * 8, P, V, sq, std::true_type{}, std::integral_constant<int, 2>{});   // ProMP: NaN-free
        plast = P[7];
        vlast = V[7];
      }
      write_sq(ch, sq);
      hl_barrier();
    }
    pv_get(nf, P, V);
#pragma unroll
    for (int sl = 0; sl < SPW; ++sl) { A[sl] = hob[sl * 64 + lane]; B[sl] = hob[(SPW + sl) * 64 + lane]; }
    const f32x2 cv = __builtin_bit_cast(f32x2, hob[2 * SPW * 64 + lane]);
    tg.cur[0] = cv[0];
    tg.vprev[0] = cv[1];
  };
  // both waves decide the helper form's fast chunks from the same values
  auto hlp_chunks = [&](int nchunks) __attribute__((always_inline)) -> int {
    return (HLP && nchunks > 0 && s0_uni && Lmin == Lmax) ? fast_count(nchunks) : 0;
  };

  auto run = [&](auto sc, auto exact) __attribute__((always_inline)) {
    const int nchunks = (Lmax + 7) / 8;
    if (nchunks == 0) return;
    if constexpr (HLP && decltype(sc)::value && decltype(exact)::value == 0) {
      const int nf = hlp_chunks(nchunks);
      if (nf > 0) {
        joint_fast(nf);
        if (8 * nf == Lmin) { posl = plast; vell = vlast; }
        FGX_STAMP(o, wst, 2);
        slow_range(nf, nchunks, sc, exact);
        return;
      }
    }
    traj(0, P, V, std::false_type{}, sc);
    int ch = 0;
    if constexpr (decltype(sc)::value && decltype(exact)::value == 0) {
      if (Lmin == Lmax) {   // one segment layout for the wave: uniform phases
        const int L = Lmin;
        const int hs = __builtin_amdgcn_readlane(sg.hs, lead);
        const int nf = fast_count(nchunks);
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
    q = q_in;
    qd = qd_in;
    init_traj();
    tg.stab = stab;
    cfk = 0.0;
#pragma unroll
    for (int sl = 0; sl < SPW; ++sl) { A[sl] = -0.0; B[sl] = -0.0; Tl[sl] = 0.0; }
  };
  nanm = 0;
  FGX_STAMP(o, wst, 1);
  if (helper) {
    const int nf = hlp_chunks((Lmax + 7) / 8);
    if (nf > 0) helper_fast(nf, min(nf, __builtin_amdgcn_readlane(sg.hs, lead) / 8 + 1));
  } else {
    if (s0_uni) run(std::true_type{}, std::integral_constant<int, 0>{});
    else run(std::false_type{}, std::integral_constant<int, 0>{});
    if (__builtin_expect((nanm & vmask) != 0, 0)) {   // a NaN control: np.clip semantics from the start
      wave_lds_sync();
      restart();
      if (s0_uni) run(std::true_type{}, std::integral_constant<int, 1>{});
      else run(std::false_type{}, std::integral_constant<int, 1>{});
    }
  }

  if (!helper && valid && sg.stop && c.cond_desired) {   // black_box_wrapper.py:234-236
    s.cond[d * N + e] = posl;
    s.cond[(NL + d) * N + e] = vell;
  }

  FGX_STAMP(o, wst, 3);
  // The helper form (no reset wave): the VectorEnv auto-reset of a truncated env depends only on its
  // PCG64 stream and start angle, not on the episode: when the workgroup has a second group of EPB
  // threads (R0 = EPB rounded up to whole waves), those threads run the resets concurrently with the
  // first group's returns and final observations.  Their inputs are loaded here, so that the loads
  // land under the gather.
  constexpr int R0 = (EPB + 63) / 64 * 64;
  const bool SPLIT = !rw && R0 + EPB <= S::THREADS;
  const int t1 = (int)threadIdx.x - R0, tw1 = t1 / G, tg1 = t1 - tw1 * G;
  const int64_t er = (int64_t)blockIdx.x * (S::WAVES * gw) + tw1 * gw + tg1;
  const bool rgrp = SPLIT && o.autoreset && t1 >= 0 && t1 < EPB && tg1 < gw && er < N;
  Pcg64 rg;
  double rsp = 0.0;
  if (rgrp) {
    rg = load_rng(s.rng, N, er);
    rsp = s.start[er];
  }
  // ---- gather per env (SoA [field][EPB]): slot sums, the FK sample's control cost, joint state,
  // the env's segment words and goal
  __syncthreads();   // 1: every wave is done with its chunk rows (the gather area overlaps them)
  double* ga = lds_jl;
  if (!helper && g < G && d == 0) {
    ga[(S::GX + 0) * EPB + slot] = (double)sg.steps;
    ga[(S::GX + 1) * EPB + slot] = (double)(sg.plans - 1);
    ga[(S::GX + 2) * EPB + slot] = (double)sg.flags;
    ga[(S::GX + 3) * EPB + slot] = gx;
    ga[(S::GX + 4) * EPB + slot] = gy;
  }
  if (!helper && g < G) {
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
  __syncthreads();   // 2
  // the epilogue's trigonometry, one joint per lane: cos / sin of the cumulative angle q0 + ... + qd
  // (numpy cumsum order, Env::fk) and of qd itself (the observation, emit_obs)
  if (!helper && g < G) {
    double ang = ga[25 * EPB + slot];
#pragma unroll
    for (int k = 1; k < NL; ++k) {
      const double nx = ang + ga[(25 + k) * EPB + slot];
      ang = (k <= d) ? nx : ang;
    }
    double fs, fc, os_, oc;
    fgx_sincos(ang, &fs, &fc);
    fgx_sincos(q, &os_, &oc);
    ga[(25 + 2 * NL + d) * EPB + slot] = fc;
    ga[(25 + 3 * NL + d) * EPB + slot] = fs;
    ga[(25 + 4 * NL + d) * EPB + slot] = oc;
    ga[(25 + 5 * NL + d) * EPB + slot] = os_;
  }
  __syncthreads();   // 3

  // ---- the reset group: the auto-reset of every env whose segment ends in truncation (SimpleReacher
  // never terminates); nothing in this launch reads the env state after the gather
  FGX_STAMP(o, wst, 4);
  if (rgrp) {
    JpSeg sr;
    sr.init_vals(c, (int)ga[(S::GX + 0) * EPB + t1], (uint32_t)ga[(S::GX + 2) * EPB + t1],
                 (int)ga[(S::GX + 1) * EPB + t1], true);
    if (sr.steps + sr.L >= c.max_steps) {
      Env<NL> vr;
      if (!c.random_start) vr.sp = rsp;
      vr.reset(c, rg, false, 0);
      store_rng(s.rng, N, er, rg);
      if (c.random_start) s.start[er] = vr.sp;
      emit_obs(c, vr, c.return_context, o.obs + er * c.out_dim, nullptr, true);
      store_env(c, s, er, vr, false);   // SimpleReacher: no hole / reward state
      s.plans[er] = 0;
    }
    FGX_STAMP(o, wst, 10);
  }
  // ---- one thread per env: return and epilogue (threads t < EPB), from the LDS gather only
  const int t = threadIdx.x;
  const int tw = t / G, tg_ = t - tw * G;   // slot t = tw * G + tg_
  const int64_t et = (int64_t)blockIdx.x * (S::WAVES * gw) + tw * gw + tg_;
  const bool tv = t < EPB && tg_ < gw && et < N;
  if (o.inner_steps && (t >> 6) < (EPB + 63) / 64) {   // trajectory lengths: one atomic per wave of the group
    long long sum = 0;
    if (tv) {
      JpSeg sq;
      sq.init_vals(c, (int)ga[(S::GX + 0) * EPB + t], (uint32_t)ga[(S::GX + 2) * EPB + t],
                   (int)ga[(S::GX + 1) * EPB + t], true);
      sum = sq.L;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off, 64);
    count_inner(o.inner_steps, sum, lane == 0);
  }
  if (!tv) {
    FGX_STAMP(o, wst, 5);
    FGX_STAMP(o, wst, 7);
    return;
  }
  JpSeg st;
  st.init_vals(c, (int)ga[(S::GX + 0) * EPB + t], (uint32_t)ga[(S::GX + 2) * EPB + t], (int)ga[(S::GX + 1) * EPB + t],
               true);
  Env<NL> v;
  v.hx = v.hw = v.hd = 0.0;
  v.ex = v.ey = v.cd = 0.0;
  v.gx = ga[(S::GX + 3) * EPB + t];
  v.gy = ga[(S::GX + 4) * EPB + t];
  v.flags = st.flags;
#pragma unroll
  for (int k = 0; k < NL; ++k) { v.q[k] = ga[(25 + k) * EPB + t]; v.qd[k] = ga[(25 + NL + k) * EPB + t]; }
  v.steps = st.steps + st.L;
  if (st.stop && c.cond_desired) v.flags |= 2u;
  double fc[NL], fs[NL], oc[NL], os_[NL];
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    fc[k] = ga[(25 + 2 * NL + k) * EPB + t];
    fs[k] = ga[(25 + 3 * NL + k) * EPB + t];
    oc[k] = ga[(25 + 4 * NL + k) * EPB + t];
    os_[k] = ga[(25 + 5 * NL + k) * EPB + t];
  }
  v.fk_given(fc, fs);
  FGX_STAMP(o, wst, 11);
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
  episode_epilogue(c, s, o, et, v, st.plans, L, res, false, trunc, false, oc, os_, SPLIT || rw);
  FGX_STAMP(o, wst, 5);
  FGX_STAMP(o, wst, 7);
}

}  // namespace fgx
