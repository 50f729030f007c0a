// fgx_traj_run.h — k_traj_run: desired trajectories [N, T, dof] (get_trajectory,
// black_box_wrapper.py:119-133) for the plans k_traj_mfma does not take: DMP, replanning plans
// (per-env plan start s0 = steps), condition_on_desired initial conditions, basis counts other than 5.
//
// k_traj_valu (fgx_kernels.h) runs one env per lane and stores each sample's dof floats at that
// env's row: 64 lanes of a store instruction hit 64 runs T * dof * 4 B apart, 20 B each — 0.10 of
// HBM peak (621-628 us for 524 MB at 65536 envs, profiles/r04_kernel_stats_all_final.csv).  Here the
// output is written the way k_traj_mfma writes it (fgx_mfma.h: whole env runs, consecutive lanes on
// consecutive 16-B chunks, no load queued behind the stores):
//   * a 256-thread workgroup walks groups of GE envs; the basis table sits in LDS (rows of different
//     plan starts are random access);
//   * per group, rows [row0, row0 + RC) of every env's run are computed into two LDS regions
//     ([env][row][dof], positions and velocities), one LDS-only barrier, then each wave streams whole
//     env pieces (16-B chunks over consecutive lanes; the env base wave-uniform), one more barrier;
//     with RC >= T a piece is the env's whole run;
//   * ProMP / ProDMP: a sample is a closed form of its table row(s) (Traj::at_rows), so the GE envs'
//     rows are split over the 256 lanes: lane (env = t % GE, part = t / GE) computes a run of
//     consecutive rows.  ProMP's look-ahead (position of the next row, Traj::cur) is re-seeded at the
//     run's first row; a run starting at the plan's last sample starts one row early (its velocity
//     repeats the previous one's, Traj::at);
//   * DMP: the Euler recurrence is sequential per joint, so lane (env = t / dof, joint = t % dof) runs
//     one joint of one env through all of the group's chunks (Traj<DMP, 1>, k_episode_jp's per-joint
//     generator).
// Every value is computed by the same Traj code as k_traj_valu and k_episode: bit-identical.
#pragma once
#include <cstdlib>

#include "fgx_kernels.h"
#include "fgx_mfma.h"

namespace fgx {

constexpr int kTrajRunThreads = 256;

inline int traj_run_cus() {
  static const int n = [] {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
    return cus;
  }();
  return n;
}

// V4: every piece is a whole number of 16-B chunks at a 16-B aligned address (host-checked)
template <int MP, int NL, int NB, bool V4>
__global__ __launch_bounds__(kTrajRunThreads) void k_traj_run(DevCfg c, DevState s, const float* __restrict__ params,
                                                              float* __restrict__ dpos, float* __restrict__ dvel,
                                                              int GE, int RC, int nt, int sep) {
  constexpr bool SEQ = MP == MP_DMP;                   // per-joint lanes through every chunk
  using TrajT = Traj<MP, SEQ ? 1 : NL, NB>;
  extern __shared__ float4 lds_run[];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int64_t N = c.N;
  const int T = c.T;
  const int str = TrajT::KS ? TrajT::KS : c.stride;
  float* tab = (float*)lds_run;
  // (DMP reads its rows from global memory: by scalar loads when the wave's plans start on one row)
  const int tab_f = SEQ ? 0 : c.rows * c.stride;
  const int nthr = blockDim.x;   // 64 .. kTrajRunThreads (host: DMP one wave, else 256)
  for (int i = t; i < tab_f; i += nthr) tab[i] = s.tables[i];
  // LDS floats per env and region (16-B aligned): a 32-float carry area (the tail of the previous
  // chunk that did not reach a 128-B line of the output), then the chunk's rows
  constexpr int CA = 32;
  const int ESR = CA + RC * NL;
  float* rpos = tab + ((tab_f + 3) & ~3);
  float* rvel = rpos + GE * ESR;
  // each array's carried tail per env ([array][env][32]), after the regions (sep: one region for both)
  float* csave = rpos + (sep ? 1 : 2) * GE * ESR;
  const int64_t groups = (N + GE - 1) / GE;
  const int nb = NB ? NB : c.nb;
  auto lds_barrier = [] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  __syncthreads();   // the table staged

  // lane roles (fixed for the launch)
  const int je = SEQ ? t / NL : t % GE;               // env of the group
  const int dl = SEQ ? t - je * NL : 0;               // DMP: the lane's joint
  const int part = SEQ ? 0 : t / GE;                  // ProMP / ProDMP: the lane's run of rows
  const int parts = nthr / GE;
  const bool role = SEQ ? je < GE : part < parts;

  // one region's pieces to out: of rows [row0, row0 + rows) of each env's run, the floats up to the last
  // 128-B line boundary of the output (all of them at the run's end), after the previous chunk's carried
  // tail; the rest (< 32 floats) is carried: copied in front of the region's next rows.  Every line of the
  // output but a run's first and last is then written whole by one piece (tools/wbench.hip: 800-B pieces
  // 4.1-4.7 TB/s aligned against 3.3-4.4 unaligned, profiles/r05_s11_wbench.jsonl)
  auto store_region = [&](float* reg, float* out, int64_t e0, int ne, int row0, int rows, int arr) __attribute__((always_inline)) {
    const bool last = row0 + rows >= T;
    for (int j = wave; j < ne; j += nthr >> 6) {
      const int64_t g0 = (e0 + j) * (int64_t)T * NL;   // the run's first float in out
      // (nt bit 1, A/B: pieces end on rows, as before)
      auto aligned_end = [&](int r) { return (nt & 2) ? r * NL : r * NL - (int)((g0 + (int64_t)r * NL) & 31); };
      const int fs = row0 == 0 ? 0 : aligned_end(row0);
      const int fe = last ? T * NL : aligned_end(row0 + rows);
      gchar* base = uniform_ptr(out + g0 + fs);
      float* src = reg + j * ESR + CA + (fs - row0 * NL);
      const int nf = fe - fs;
      float* cs = csave + (arr * GE + j) * CA;
      {   // the previous chunk's tail of this array in front of the rows (this wave saved it)
        const int ncp = row0 * NL - fs;
        for (int f = lane; f < ncp; f += 64) src[f] = cs[f];
      }
      if constexpr (V4) {
        if (nt & 1) {   // streaming stores
          for (int ch = lane; ch < nf / 4; ch += 64)
            __builtin_nontemporal_store(*reinterpret_cast<const f32x4*>(src + 4 * ch),
                                        (__attribute__((address_space(1))) f32x4*)(base + 16u * (uint32_t)ch));
        } else {
          for (int ch = lane; ch < nf / 4; ch += 64)
            *(__attribute__((address_space(1))) f32x4*)(base + 16u * (uint32_t)ch) = *reinterpret_cast<const f32x4*>(src + 4 * ch);
        }
      } else {
        for (int f = lane; f < nf; f += 64) *(__attribute__((address_space(1))) float*)(base + 4u * (uint32_t)f) = src[f];
      }
      if (!last) {   // the new tail (this wave's LDS ops run in order: the piece was read first)
        const int nc = (row0 + rows) * NL - fe;
        const float* cb = reg + j * ESR + CA + (fe - row0 * NL);
        for (int f = lane; f < nc; f += 64) cs[f] = cb[f];
      }
    }
  };

  for (int64_t grp = blockIdx.x; grp < groups; grp += gridDim.x) {
    const int64_t e0 = grp * GE;
    const int ne = (int)min((int64_t)GE, N - e0);
    const bool act = role && je < ne;
    const int64_t e = e0 + (act ? je : 0);
    // the plan's start row and initial conditions (k_traj_valu)
    int s0 = 0;
    TrajT tg;
    if (act) {
      s0 = c.replan ? s.steps[e] : 0;
      const bool has_cond = c.cond_desired && (s.flags[e] & 2u);
      constexpr int NQ = SEQ ? 1 : NL;
      double ic_q[NQ], ic_qd[NQ];
#pragma unroll
      for (int k = 0; k < NQ; ++k) {
        const int d = SEQ ? dl : k;
        ic_q[k] = has_cond ? (double)s.cond[d * N + e] : s.q[d * N + e];
        ic_qd[k] = has_cond ? (double)s.cond[(NL + d) * N + e] : s.qd[d * N + e];
      }
      if constexpr (SEQ)
        tg.init(c, params + e * c.n_params + dl * nb, s.tables, s0, ic_q, ic_qd, c.T, c.tau32, c.rcp_tau32,
                c.nl * nb + dl - dl * nb);
      else
        tg.init(c, params + e * c.n_params, s.tables, s0, ic_q, ic_qd);
    }
    for (int row0 = 0; row0 < T; row0 += RC) {
      const int rows = min(RC, T - row0);
      if constexpr (SEQ) {
        const uint64_t am = __ballot(act);
        const int s0l = __builtin_amdgcn_readlane(s0, am ? __builtin_ctzll(am) : 0);
        const bool uni = __ballot(act && s0 != s0l) == 0;
        if (act) {
          float pos[1], vel[1];
          float* dp = rpos + je * ESR + CA + dl;
          float* dv = rvel + je * ESR + CA + dl;
          if (uni) {   // rows by scalar loads
            const cfloat_ptr sb = (cfloat_ptr)(uintptr_t)s.tables + (size_t)(s0l + 1) * str;
            for (int k = row0; k < row0 + rows; ++k) {
              tg.template at_rows<false>(c, k, sb + (size_t)k * str, pos, vel);
              dp[(k - row0) * NL] = pos[0];
              dv[(k - row0) * NL] = vel[0];
            }
          } else {     // (plans starting on different rows: per-lane loads)
            for (int k = row0; k < row0 + rows; ++k) {
              tg.template at_rows<false>(c, k, s.tables + (size_t)(s0 + k + 1) * str, pos, vel);
              dp[(k - row0) * NL] = pos[0];
              dv[(k - row0) * NL] = vel[0];
            }
          }
        }
        lds_barrier();
        store_region(rpos, dpos, e0, ne, row0, rows, 0);
        store_region(rvel, dvel, e0, ne, row0, rows, 1);
        lds_barrier();   // every wave's region reads done before the next chunk overwrites it
      } else {
        // WHICH 0: positions and velocities into their regions; 1 / 2 (sep): positions / velocities
        // into the one region (the other half of at_rows is dead code)
        auto comp = [&](auto which) __attribute__((always_inline)) {
          constexpr int W = decltype(which)::value;
          if (!act) return;
          float pos[NL], vel[NL];
          const int rs = (rows + parts - 1) / parts;   // rows per lane
          const int kb = row0 + part * rs, kend = min(kb + rs, row0 + rows);
          if (kb >= kend) return;
          int ka = kb;
          if constexpr (MP == MP_PROMP) {
            // re-seed the look-ahead at row ka (a run starting at the last sample starts one early)
            if (kb == T - 1 && kb > 0) ka = kb - 1;
            tg.T = T - ka;
            const float* r1 = tab + (size_t)(s0 + ka + 1) * str;
            if constexpr (TrajT::PK) {
#pragma unroll
              for (int p = 0; p < TrajT::NLP; ++p) { tg.cur2[p] = tg.chain2(r1, tg.wp[p]); tg.vprev2[p] = (f32x2)0.0f; }
            } else {
#pragma unroll
              for (int d = 0; d < NL; ++d) { tg.cur[d] = tg.chain(r1, tg.w[d]); tg.vprev[d] = 0.0f; }
            }
          }
          float* dp = rpos + je * ESR + CA;
          float* dv = rvel + je * ESR + CA;
          for (int k = ka; k < kend; ++k) {
            tg.template at_rows<false>(c, MP == MP_PROMP ? k - ka : k, tab + (size_t)(s0 + k + 1) * str, pos, vel);
            if (k >= kb) {
#pragma unroll
              for (int d = 0; d < NL; ++d) {
                if constexpr (W == 0) {
                  dp[(k - row0) * NL + d] = pos[d];
                  dv[(k - row0) * NL + d] = vel[d];
                } else {
                  dp[(k - row0) * NL + d] = W == 1 ? pos[d] : vel[d];
                }
              }
            }
          }
        };
        if (!sep) {
          comp(std::integral_constant<int, 0>{});
          lds_barrier();
          store_region(rpos, dpos, e0, ne, row0, rows, 0);
          store_region(rvel, dvel, e0, ne, row0, rows, 1);
          lds_barrier();
        } else {
          comp(std::integral_constant<int, 1>{});
          lds_barrier();
          store_region(rpos, dpos, e0, ne, row0, rows, 0);
          lds_barrier();
          comp(std::integral_constant<int, 2>{});
          lds_barrier();
          store_region(rpos, dvel, e0, ne, row0, rows, 1);
          lds_barrier();
        }
      }
    }
  }
}

// workgroup shape of k_traj_run: GE envs per group, RC rows per chunk (RC >= T: whole runs), nt:
// streaming stores, sep: positions then velocities through one region.  Chosen from the A/B sweeps at
// 65536 envs, T = 200, 5 links (profiles/r05_s10_traj_hpinfo.jsonl, r05_s11_traj_sweep.jsonl, us per
// launch; sessions differ by up to 15%):
//   * ProMP (replanning): whole runs of 8 envs, one region: 105.6 us (both regions 102-122 us);
//   * ProDMP (replanning, a 402-row table in LDS): whole runs of 12 envs, one region, streaming
//     stores: 128.9 us (16 envs x 64 rows, two regions: 151-155; whole runs, two regions: 192-315);
//   * DMP (sequential per joint): one wave of joint lanes (64 / dof envs) x 40 rows, streaming
//     stores: 162-167 us (regular stores 167-190; 12 x 32 / 64 rows: 165-205; 17 / 25 envs: 175-218;
//     pieces ending on 128-B lines or on rows: within the sessions' noise, r05_s12_traj_sweep.jsonl).
//     DMP is sensitive to the workgroups per CU (LDS-bound; its joint lanes fill wave 0, every wave
//     stores): four per CU 272 us, five 169-183 us, one-wave workgroups 480 us (r05_s15..s17_dmp_shapes);
//     its rows by scalar loads instead of an LDS table copy per workgroup: six per CU, 154-165 us
//     (r05_s22_dmp_scalar_rows.jsonl).
// FGX_TRAJ_GE / _RC / _NT=0|1 / _SEP=0|1 / _ALIGN=0 / _THREADS / _PERCU override (A/B).
struct TrajRunShape {
  int GE, RC, nt, sep, threads, per_cu;
  size_t lds;
};
// sep: positions, then velocities through one region (ProMP / ProDMP)
inline size_t traj_run_lds(const DevCfg& c, int GE, int RC, int sep = 0) {
  return (c.mp == MP_DMP ? 0 : (((size_t)c.rows * c.stride + 3) & ~(size_t)3) * 4) +
         (sep ? 1 : 2) * (size_t)GE * (32 + (size_t)RC * c.nl) * 4 +
         2 * (size_t)GE * 32 * 4;
}
inline TrajRunShape traj_run_shape(const DevCfg& c) {
  const int nl = c.nl, T = c.T;
  const size_t budget = 80 * 1024;   // two workgroups per CU
  int GE, RC, nt = 0, sep = 0;
  if (c.mp == MP_DMP) {
    GE = 64 / nl;
    RC = std::min(T, 40);
    nt = 1;
  } else {   // whole runs, positions then velocities through one region
    sep = 1;
    GE = c.mp == MP_PRODMP ? 12 : 8;
    nt = c.mp == MP_PRODMP ? 1 : 0;
    while (GE > 1 && traj_run_lds(c, GE, T, 1) > budget) --GE;
    RC = T;
    if (traj_run_lds(c, GE, T, 1) > budget) {   // a run too long for the region: chunks
      const size_t fixed = traj_run_lds(c, GE, 0, 1);
      const size_t per = budget > fixed ? (budget - fixed) / ((size_t)GE * 4) : 0;
      RC = std::max(4, (int)std::min<size_t>((size_t)T, per / nl));
    }
  }
  if (const char* v = std::getenv("FGX_TRAJ_GE")) GE = std::max(1, std::min(kTrajRunThreads, std::atoi(v)));
  int threads = kTrajRunThreads;   // (DMP: the joint lanes on wave 0; every wave stores)
  if (const char* v = std::getenv("FGX_TRAJ_THREADS")) threads = std::max(1, std::min(4, std::atoi(v) / 64)) * 64;
  if (c.mp == MP_DMP) {
    GE = std::min(GE, kTrajRunThreads / nl);
    threads = std::max(threads, (GE * nl + 63) / 64 * 64);
  } else {
    GE = std::min(GE, threads);
  }
  if (const char* v = std::getenv("FGX_TRAJ_RC")) RC = std::max(1, std::min(T, std::atoi(v)));
  if (const char* v = std::getenv("FGX_TRAJ_NT")) nt = v[0] == '1';
  if (const char* v = std::getenv("FGX_TRAJ_ALIGN"))
    if (v[0] == '0') nt |= 2;
  if (const char* v = std::getenv("FGX_TRAJ_SEP")) sep = v[0] == '1' && c.mp != MP_DMP;
  RC = std::min(RC, T);
  if (RC < T) {   // a chunk spans at least one 128-B line (the carry stays below 32 floats); whole 16-B chunks
    RC = std::max(RC, (32 + nl - 1) / nl);
    while ((RC * nl) % 4 && RC < T) ++RC;
    if (RC < T && (RC * nl) % 4) RC = T;
  }
  const size_t lds = traj_run_lds(c, GE, RC, sep);
  int per_cu = (int)std::max<size_t>(1, std::min<size_t>(16, (160 * 1024) / std::max<size_t>(lds, 1)));
  if (const char* v = std::getenv("FGX_TRAJ_PERCU")) per_cu = std::max(1, std::min(per_cu, std::atoi(v)));
  return {GE, RC, nt, sep, threads, per_cu, lds};
}

// 0: launched; 1: not applicable (the caller runs k_traj_valu); 2: launch error
template <int NL>
inline int launch_traj_run(const DevCfg& c, const DevState& s, const float* params, float* dpos, float* dvel,
                           hipStream_t stream) {
  if (std::getenv("FGX_TRAJ_VALU")) return 1;   // A/B: the one-env-per-lane kernel
  if (c.nl != NL || c.T <= 0) return 1;
  const TrajRunShape sh = traj_run_shape(c);
  if (sh.lds > 160 * 1024) return 1;
  const bool v4 = ((c.T * NL) % 4) == 0 && ((sh.RC * NL) % 4) == 0 && (((uintptr_t)dpos | (uintptr_t)dvel) & 15) == 0;
  const int64_t groups = (c.N + sh.GE - 1) / sh.GE;
  const int nt = sh.nt;
  const int blocks = (int)std::min<int64_t>(groups, (int64_t)traj_run_cus() * sh.per_cu);
  const dim3 grid(blocks), block(sh.threads);
#define RUN(MPV, NBV, V4V)                                                                                      \
  launch_lds((const void*)k_traj_run<MPV, NL, NBV, V4V>, sh.lds, [&] {                                        \
    hipLaunchKernelGGL((k_traj_run<MPV, NL, NBV, V4V>), grid, block, sh.lds, stream, c, s, params, dpos, dvel, \
                       sh.GE, sh.RC, nt, sh.sep);                                                             \
  })
#define BY_V4(MPV, NBV) \
  if (v4) RUN(MPV, NBV, true); else RUN(MPV, NBV, false)
#define BY_NB(MPV) \
  if (c.nb == 5) { BY_V4(MPV, 5); } else { BY_V4(MPV, 0); }
  if (c.mp == MP_PROMP) { BY_NB(MP_PROMP) }
  else if (c.mp == MP_DMP) { BY_NB(MP_DMP) }
  else if (c.mp == MP_PRODMP) { BY_NB(MP_PRODMP) }
  else return 1;
#undef BY_NB
#undef BY_V4
#undef RUN
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

}  // namespace fgx
