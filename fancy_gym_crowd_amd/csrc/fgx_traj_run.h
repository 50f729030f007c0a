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
                                                              int GE, int RC, int nt) {
  constexpr bool SEQ = MP == MP_DMP;                   // per-joint lanes through every chunk
  using TrajT = Traj<MP, SEQ ? 1 : NL, NB>;
  extern __shared__ float4 lds_run[];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int64_t N = c.N;
  const int T = c.T;
  const int str = TrajT::KS ? TrajT::KS : c.stride;
  float* tab = (float*)lds_run;
  const int tab_f = c.rows * c.stride;
  for (int i = t; i < tab_f; i += kTrajRunThreads) tab[i] = s.tables[i];
  const int ESR = RC * NL + 4;                         // LDS floats per env and region (16-B aligned)
  float* rpos = tab + ((tab_f + 3) & ~3);
  float* rvel = rpos + GE * ESR;
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
  const int parts = kTrajRunThreads / GE;
  const bool role = SEQ ? je < GE : part < parts;

  // one region's pieces (rows [row0, row0 + rows) of the group's env runs) to out
  auto store_region = [&](const float* reg, float* out, int64_t e0, int ne, int row0, int rows) __attribute__((always_inline)) {
    const int nf = rows * NL;                          // floats per piece
    for (int j = wave; j < ne; j += kTrajRunThreads / 64) {
      gchar* base = uniform_ptr(out + ((e0 + j) * T + row0) * NL);
      const float* src = reg + j * ESR;
      if constexpr (V4) {
        if (nt) {   // (A/B: streaming stores)
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
      if (act) {
        float pos[SEQ ? 1 : NL], vel[SEQ ? 1 : NL];
        if constexpr (SEQ) {
          float* dp = rpos + je * ESR + dl;
          float* dv = rvel + je * ESR + dl;
          for (int k = row0; k < row0 + rows; ++k) {
            tg.template at_rows<false>(c, k, tab + (size_t)(s0 + k + 1) * str, pos, vel);
            dp[(k - row0) * NL] = pos[0];
            dv[(k - row0) * NL] = vel[0];
          }
        } else {
          const int rs = (rows + parts - 1) / parts;   // rows per lane
          const int kb = row0 + part * rs, kend = min(kb + rs, row0 + rows);
          if (kb < kend) {
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
            float* dp = rpos + je * ESR;
            float* dv = rvel + je * ESR;
            for (int k = ka; k < kend; ++k) {
              tg.template at_rows<false>(c, MP == MP_PROMP ? k - ka : k, tab + (size_t)(s0 + k + 1) * str, pos, vel);
              if (k >= kb) {
#pragma unroll
                for (int d = 0; d < NL; ++d) {
                  dp[(k - row0) * NL + d] = pos[d];
                  dv[(k - row0) * NL + d] = vel[d];
                }
              }
            }
          }
        }
      }
      lds_barrier();
      store_region(rpos, dpos, e0, ne, row0, rows);
      store_region(rvel, dvel, e0, ne, row0, rows);
      lds_barrier();   // every wave's region reads done before the next chunk overwrites it
    }
  }
}

// workgroup shape of k_traj_run: GE envs per group, RC rows per chunk (RC >= T: whole runs), nt:
// streaming stores.  Chosen from the A/B at 65536 envs, T = 200, 5 links
// (profiles/r05_s10_traj_hpinfo.jsonl, us per launch):
//   * ProMP (replanning): whole runs of 8 envs (two workgroups per CU) 102 us, 5.2 TB/s;
//   * ProDMP (replanning, a 402-row table in LDS): 16 envs x 64 rows with streaming stores 151 us
//     (whole runs of 8 envs 303-313 us: the table leaves room for one workgroup per CU);
//   * DMP: one wave of joint lanes (64 / dof envs) x 40 rows 167 us (12 x 32 / 64: 174 / 193;
//     17 / 25 envs: 175-185; streaming stores no better).
// FGX_TRAJ_GE / FGX_TRAJ_RC / FGX_TRAJ_NT=0|1 override (A/B).
struct TrajRunShape {
  int GE, RC, nt;
  size_t lds;
};
inline size_t traj_run_lds(const DevCfg& c, int GE, int RC) {
  return (((size_t)c.rows * c.stride + 3) & ~(size_t)3) * 4 + 2 * (size_t)GE * ((size_t)RC * c.nl + 4) * 4;
}
inline TrajRunShape traj_run_shape(const DevCfg& c) {
  const int nl = c.nl, T = c.T;
  const size_t budget = 80 * 1024;   // two workgroups per CU
  int GE, RC, nt = 0;
  // RC * nl a multiple of 4 (whole 16-B chunks per piece)
  auto rc_align = [&](int rc) { while (rc > 4 && (rc * nl) % 4) --rc; return rc; };
  if (c.mp == MP_DMP) {
    GE = 64 / nl;
    RC = rc_align(std::min(T, 40));
  } else if (c.mp == MP_PRODMP) {
    GE = 16;
    RC = rc_align(std::min(T, 64));
    nt = 1;
  } else {
    GE = 32;
    while (GE > 1 && traj_run_lds(c, GE, T) > budget) GE >>= 1;
    RC = T;
    if (traj_run_lds(c, GE, T) > budget) {   // a run too long for the region: chunks
      const size_t per = budget > traj_run_lds(c, GE, 0) ? (budget - traj_run_lds(c, GE, 0)) / (2 * (size_t)GE * 4) : 0;
      RC = rc_align(std::max(4, (int)std::min<size_t>((size_t)T, per / nl)));
    }
  }
  if (const char* v = std::getenv("FGX_TRAJ_GE")) GE = std::max(1, std::min(kTrajRunThreads, std::atoi(v)));
  if (c.mp == MP_DMP) GE = std::min(GE, kTrajRunThreads / nl);
  if (const char* v = std::getenv("FGX_TRAJ_RC")) RC = std::max(1, std::min(T, std::atoi(v)));
  if (const char* v = std::getenv("FGX_TRAJ_NT")) nt = v[0] == '1';
  RC = std::min(RC, T);
  return {GE, RC, nt, traj_run_lds(c, GE, RC)};
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
  const int per_cu = (int)std::max<size_t>(1, std::min<size_t>(8, (160 * 1024) / std::max<size_t>(sh.lds, 1)));
  const int blocks = (int)std::min<int64_t>(groups, (int64_t)traj_run_cus() * per_cu);
  const dim3 grid(blocks), block(kTrajRunThreads);
#define RUN(MPV, NBV, V4V)                                                                                      \
  launch_lds((const void*)k_traj_run<MPV, NL, NBV, V4V>, sh.lds, [&] {                                        \
    hipLaunchKernelGGL((k_traj_run<MPV, NL, NBV, V4V>), grid, block, sh.lds, stream, c, s, params, dpos, dvel, \
                       sh.GE, sh.RC, nt);                                                                     \
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
