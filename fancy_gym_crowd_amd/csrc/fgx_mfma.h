// fgx_mfma.h — desired trajectories as an f32 MFMA GEMM (v_mfma_f32_32x32x2_f32).
//
// For plans that all start at the same step (no replanning) the ProMP / ProDMP trajectory
// of every env is   Y[k, (e, d)] = sum_j H[k + 1][j] * C[e][d][j]   — a [T x K] basis table
// times a [K x (N*dof)] coefficient matrix with K = 8 (ProMP: 5 weights + 3 zero pads;
// ProDMP: 5 weights, goal, c1, c2).  One wave owns 32 envs (the MFMA's 32 columns) and walks
// the T rows in 32-row tiles; per dof the K = 8 contraction is 4 chained
// v_mfma_f32_32x32x2_f32, whose numerics are bit-for-bit the k-ordered fmaf chain of the
// VALU path (cdna_hip_programming.md §3), so k_traj_mfma == k_traj_valu == k_episode.
//
// Operand maps (32x32x2 f32): lane l holds A[i = l&31][k = l>>5] and B[k = l>>5][j = l&31];
// C/D: col = l&31, row = (r&3) + 8*(r>>2) + 4*(l>>5) for accumulator register r.
// The kernel is bound by writing the [N, T, dof] f32 outputs (arithmetic intensity
// 2*K flop per 8 output bytes = 2 flop/B), not by the matrix pipe.
#pragma once
#include <cstdlib>
#include <cstring>
#include <algorithm>

#include "fgx_kernels.h"

namespace fgx {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kTrajWaves = 2;   // k_traj_mfma_r3: waves per workgroup (LDS tile 20.5 KB per wave: 3 groups per CU)

template <int MP, int NL>
__global__ __launch_bounds__(64 * kTrajWaves) void k_traj_mfma_r3(DevCfg c, DevState s, const float* __restrict__ params,
                                                               float* __restrict__ dpos, float* __restrict__ dvel) {
  constexpr int NB = 5, K = 8;
  constexpr int kEnvStride = 32 * NL + 4;      // dwords per env in the LDS tile (bank-spread)
  __shared__ __attribute__((aligned(16))) float lds_stage[kTrajWaves * 32 * kEnvStride];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int j = lane & 31, h = lane >> 5;
  const int64_t N = c.N;
  const int64_t e = ((int64_t)blockIdx.x * (blockDim.x >> 6) + wave) * 32 + j;
  const bool valid = e < N;
  const int64_t ec = valid ? e : (N - 1);
  const float* tab = s.tables;
  const int stride = c.stride;

  // ---- per-env coefficients C[d][k] (only the k = 2s + h this lane feeds are kept)
  float bco[NL][4];
  if (MP == MP_PROMP) {
    const float* p = params + ec * c.n_params;
#pragma unroll
    for (int d = 0; d < NL; ++d)
#pragma unroll
      for (int sidx = 0; sidx < 4; ++sidx) {
        const int kk = 2 * sidx + h;
        bco[d][sidx] = (kk < NB) ? p[d * NB + kk] : 0.0f;
      }
  } else {   // ProDMP, bc at step 0 (oracle/mp.py)
    const float* p = params + ec * c.n_params;
    const float* rb = tab;   // row 0
    const float y1 = rb[2 * NB + 2], y2 = rb[2 * NB + 3], dy1 = rb[2 * NB + 4], dy2 = rb[2 * NB + 5];
    const float det = y1 * dy2 - y2 * dy1;
#pragma unroll
    for (int d = 0; d < NL; ++d) {
      float w[K];
#pragma unroll
      for (int kk = 0; kk < NB; ++kk) w[kk] = p[d * (NB + 1) + kk] * c.ws32;
      w[NB] = p[d * (NB + 1) + NB] * c.gs32;
      float P = 0.0f, V = 0.0f;
#pragma unroll
      for (int kk = 0; kk <= NB; ++kk) {
        P = __builtin_fmaf(rb[kk], w[kk], P);
        V = __builtin_fmaf(rb[NB + 1 + kk], w[kk], V);
      }
      const double q0 = s.q[d * N + ec], qd0 = s.qd[d * N + ec];
      const float A = (float)q0 - P;
      const float B = (float)qd0 * c.tau32 - V;
      w[NB + 1] = (dy2 * A - y2 * B) / det;
      w[NB + 2] = (y1 * B - dy1 * A) / det;
#pragma unroll
      for (int sidx = 0; sidx < 4; ++sidx) bco[d][sidx] = w[2 * sidx + h];
    }
  }

  const int T = c.T;
  for (int tb = 0; tb < T; tb += 32) {
    // ---- A operands: this lane feeds time row i = j of the tile, k = 2s + h
    const int kt = tb + j;                       // plan sample index of the row this lane feeds
    const int ktc = kt < T ? kt : T - 1;
    const int row = ktc + 1;                     // table row (s0 = 0)
    float a1[4], a2[4];
    if (MP == MP_PROMP) {
      const int row2 = (ktc < T - 1) ? row + 1 : row - 1;
#pragma unroll
      for (int sidx = 0; sidx < 4; ++sidx) {
        const int kk = 2 * sidx + h;
        a1[sidx] = (kk < NB) ? tab[(size_t)row * stride + kk] : 0.0f;
        a2[sidx] = (kk < NB) ? tab[(size_t)row2 * stride + kk] : 0.0f;
      }
    } else {
      const float* r = tab + (size_t)row * stride;
#pragma unroll
      for (int sidx = 0; sidx < 4; ++sidx) {
        const int kk = 2 * sidx + h;
        a1[sidx] = (kk <= NB) ? r[kk] : r[2 * NB + 2 + (kk - NB - 1)];
        a2[sidx] = (kk <= NB) ? r[NB + 1 + kk] : r[2 * NB + 4 + (kk - NB - 1)];
      }
    }
    f32x16 cp[NL], cq[NL];
#pragma unroll
    for (int d = 0; d < NL; ++d) {
      f32x16 z = {0.0f};
      cp[d] = z;
      cq[d] = z;
#pragma unroll
      for (int sidx = 0; sidx < 4; ++sidx) {
        cp[d] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[sidx], bco[d][sidx], cp[d], 0, 0, 0);
        cq[d] = __builtin_amdgcn_mfma_f32_32x32x2f32(a2[sidx], bco[d][sidx], cq[d], 0, 0, 0);
      }
    }
    // ---- epilogue: lane (j, h) owns env e, rows 8g + 4h + {0..3}, g = 0..3.  The tile is
    // staged in LDS in the output layout ([env][row][dof], env stride padded to 4 mod 32
    // dwords) and then written with coalesced 16-B stores: each env's rows of the tile are one
    // contiguous run of rows*NL floats in [N, T, dof].
    float* stage = lds_stage + wave * (32 * kEnvStride);
    float vbuf[4][4 * NL];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int k0 = tb + 8 * g + 4 * h;
      float pv[4 * NL];
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        const int reg = 4 * g + r4;
        const int k = k0 + r4;
#pragma unroll
        for (int d = 0; d < NL; ++d) {
          const float P = cp[d][reg], Q = cq[d][reg];
          float vel;
          if (MP == MP_PROMP) {
            const int kc = k < T ? k : T - 1;
            const float* dr = tab + (size_t)((kc < T - 1) ? kc + 1 : kc) * stride + NB;
            vel = (kc < T - 1) ? div_rcp(Q - P, dr[0], dr[1]) : div_rcp(P - Q, dr[0], dr[1]);
          } else {
            vel = div_rcp(Q, c.tau32, c.rcp_tau32);
          }
          pv[r4 * NL + d] = P;
          vbuf[g][r4 * NL + d] = vel;
        }
      }
      float* dst = stage + j * kEnvStride + (8 * g + 4 * h) * NL;
#pragma unroll
      for (int q4 = 0; q4 < NL; ++q4)
        *reinterpret_cast<f32x4*>(dst + 4 * q4) = f32x4{pv[4 * q4], pv[4 * q4 + 1], pv[4 * q4 + 2], pv[4 * q4 + 3]};
    }
    const int rows = (T - tb) < 32 ? (T - tb) : 32;     // multiple of 4 (T % 4 == 0)
    const int chunks = rows * NL / 4;                   // 16-B chunks per env in this tile
    const int64_t e0 = e - j;                           // first env of this wave
    // Each wave owns its LDS tile, so a wave-local barrier suffices (LDS ops of one wave complete
    // in order; wait for them, not for the outstanding global stores as __syncthreads would).
    auto wave_sync = [] {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
    };
    for (int pass = 0; pass < 2; ++pass) {
      wave_sync();
      if (pass == 1) {   // restage with the velocities
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          float* dst = stage + j * kEnvStride + (8 * g + 4 * h) * NL;
#pragma unroll
          for (int q4 = 0; q4 < NL; ++q4)
            *reinterpret_cast<f32x4*>(dst + 4 * q4) =
                f32x4{vbuf[g][4 * q4], vbuf[g][4 * q4 + 1], vbuf[g][4 * q4 + 2], vbuf[g][4 * q4 + 3]};
        }
        wave_sync();
      }
      float* out = pass == 0 ? dpos : dvel;
      constexpr int kFull = 32 * NL / 4;   // chunks per env of a full tile (division by a constant)
      for (int idx = lane; idx < 32 * chunks; idx += 64) {
        const int je = (chunks == kFull) ? idx / kFull : idx / chunks;
        const int ch = idx - je * chunks;
        const int64_t ee = e0 + je;
        if (ee < N) {
          const f32x4 x = *reinterpret_cast<const f32x4*>(stage + je * kEnvStride + 4 * ch);
          *reinterpret_cast<f32x4*>(out + (ee * T + tb) * NL + 4 * ch) = x;
        }
      }
    }
    wave_sync();
  }
}

// ---------------------------------------------------------------------------------------------------
// k_traj_mfma (round 4): the same GEMM, laid out for the output write it is bound by.
//
// k_traj_mfma_r3 (above; FGX_TRAJ_R3=1 selects it for A/B) wrote 537 MB in 179 us at 65536 envs
// (3.0 TB/s, 0.37 of HBM peak).  The write pattern sets that ceiling, not the GEMM: a store-only
// kernel writing every env's 4000-B [T, dof] run as 160..2000-B pieces (a tile loop's order) reaches
// 3.2-4.3 TB/s on the box, the same runs written whole 5.2 TB/s, the 128-KB region of 32 envs
// linearly 5.4-5.6 TB/s (tools/wbench.hip, profiles/r04_wbench.jsonl).  So here a workgroup owns GE
// envs and writes their runs whole (ProMP 184 -> 112.5 us = 4.7 TB/s, ProDMP 145 -> 139.6 us at
// 65536 envs, profiles/r04_traj_ab_s2.txt):
//   * one 8-wave workgroup per CU walks 32-env groups; per group its waves compute one 32-row tile
//     each (a segment of 8 tiles covers T = 200) into an LDS region [env][row][dof] (32 x T x dof
//     floats, 128 KB), one workgroup barrier (an LDS-only one: s_barrier after lgkmcnt(0), not
//     __syncthreads, whose fence would wait for the outstanding global stores), then waves 0..6
//     stream whole env runs out with 16-B stores (consecutive lanes on consecutive chunks) —
//     positions, then velocities;
//   * wave 7 stores nothing: it loads the next group's weights (and ProDMP's q0 / qd0) into LDS, so
//     no load waits behind the stores (vmcnt counts loads and stores in one queue); the basis table
//     sits in LDS for the same reason;
//   * ProMP computes each position once: the forward difference takes row k + 1 from the next
//     register of the lane, or for the last row of a lane's 4-row group from the other half-wave
//     (v_permlane32_swap: rows 8g + 4 .. 8g + 7 live in lanes 32..63); a tile outputs its first 28
//     rows (the 28th's successor is in the tile), the plan's last tile all its remaining rows
//     (velocity of the last = the previous one, as Traj::at).  ProDMP's velocities are their own
//     contraction (the second basis, vb), computed into the position accumulators once the
//     positions left; its tiles step 32 rows.
// (Tried and slower: 16-env groups at two workgroups per CU, 123 us; 4 compute + 4 store waves
// with double-buffered 16-env halves, 171 us; velocities held in registers across the position
// stores, ProDMP 141.6 us.)
constexpr int kTrajGWaves = 8;   // waves (tiles of a segment) per workgroup
constexpr int kTrajGE = 32;      // envs per group (the MFMA's columns)

// rows of one segment (8 tiles; ProMP's last tile may output 32 rows)
__host__ __device__ inline int traj_seg_rows(int T, int mp) {
  const int r = kTrajGWaves * (mp == MP_PROMP ? 28 : 32) + 4;
  return T < r ? T : r;
}
// per-env coefficient inputs staged by the loader wave: the weights (ProMP NL NB; ProDMP NL (NB + 1))
// and for ProDMP (float) q0, (float) qd0; odd stride
__host__ __device__ constexpr int traj_coef_stride(int mp, int nl) {
  return (mp == MP_PROMP ? nl * 5 : nl * 6 + 2 * nl) | 1;
}
inline size_t traj_mfma_lds_bytes(int rows, int stride, int T, int mp, int nl) {
  return (((size_t)rows * stride + 3) & ~(size_t)3) * sizeof(float) +
         (size_t)kTrajGE * ((size_t)traj_seg_rows(T, mp) * nl + 4) * sizeof(float) +
         2 * (size_t)kTrajGE * traj_coef_stride(mp, nl) * sizeof(float);
}

template <int MP, int NL>
__global__ __launch_bounds__(64 * kTrajGWaves) void k_traj_mfma(DevCfg c, DevState s, const float* __restrict__ params,
                                                            float* __restrict__ dpos, float* __restrict__ dvel) {
  constexpr int NB = 5, K = 8, GE = kTrajGE;
  constexpr bool PRO = MP == MP_PROMP;
  constexpr int RSTEP = PRO ? 28 : 32;           // output rows per (non-final) tile
  extern __shared__ float4 lds_traj[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;             // the wave's tile within a segment
  const int j = lane & 31, h = lane >> 5;
  const int64_t N = c.N;
  const int T = c.T;
  const int nt = PRO ? (T <= 32 ? 1 : (T - 32 + RSTEP - 1) / RSTEP + 1) : (T + 31) / 32;   // tiles per plan
  const int SR = traj_seg_rows(T, MP);           // (a multiple of 4: T % 4 == 0)
  const int ESR = SR * NL + 4;                   // LDS floats per env of the region
  const int64_t groups = (N + GE - 1) / GE;
  float* tab = (float*)lds_traj;
  const int tab_f = c.rows * c.stride;
  for (int i = threadIdx.x; i < tab_f; i += blockDim.x) tab[i] = s.tables[i];
  const int stride = c.stride;
  float* reg = (float*)(lds_traj + (tab_f + 3) / 4);   // [GE][ESR]
  constexpr int CW = PRO ? NL * NB : NL * (NB + 1);   // weights per env
  constexpr int CS = traj_coef_stride(MP, NL);
  float* coefs = reg + GE * ESR;                       // [2][GE][CS]
  // the loader wave (the last; it stores nothing, so its loads never wait behind global stores:
  // vmcnt counts loads and stores in one queue) stages group grp's inputs into buffer b
  constexpr int kLoader = kTrajGWaves - 1;
  auto load_coefs = [&](int64_t grp, int b) __attribute__((always_inline)) {
    const int64_t ge0 = grp * GE;
    const int ne = (int)min((int64_t)GE, N - ge0);
    float* cb = coefs + b * GE * CS;
    for (int idx = lane; idx < ne * CW; idx += 64) {
      const int jj = idx / CW, m = idx - jj * CW;
      cb[jj * CS + m] = params[(ge0 + jj) * c.n_params + m];
    }
    if constexpr (!PRO) {
      for (int idx = lane; idx < ne * NL; idx += 64) {
        const int d = idx / ne, jj = idx - d * ne;
        cb[jj * CS + CW + d] = (float)s.q[d * N + ge0 + jj];
        cb[jj * CS + CW + NL + d] = (float)s.qd[d * N + ge0 + jj];
      }
    }
  };
  if (wave == kLoader && (int64_t)blockIdx.x < groups) load_coefs(blockIdx.x, 0);
  __syncthreads();   // table and the first group's inputs staged

  // the other half-wave's value of x (lane l <-> l ^ 32)
  auto partner = [&](float x) __attribute__((always_inline)) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(h ? r[0] : r[1]);
  };
  auto lds_barrier = [] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  // workgroups walk the env groups (a grid smaller than the group count keeps its CU busy: the
  // next group's GEMM runs while the previous group's stores drain)
  int it = 0;
  for (int64_t grp = blockIdx.x; grp < groups; grp += gridDim.x, ++it) {
    const int64_t e0 = grp * GE;
    const int nenv = (int)min((int64_t)GE, N - e0);
    const bool stager = j < nenv;                // lanes whose column is one of the group's envs
    const int jc = min(j, nenv - 1);
    const float* cin = coefs + (it & 1) * GE * CS + jc * CS;   // this group's inputs (LDS)
    // the next group's inputs into the other buffer (read by nobody until the next iteration's
    // first barrier; its previous contents were read in the previous iteration)
    if (wave == kLoader && grp + gridDim.x < groups) load_coefs(grp + gridDim.x, (it + 1) & 1);
    // ---- per-env coefficients C[d][k] (only the k = 2 sidx + h this lane feeds are kept)
    float bco[NL][4];
    if (PRO) {
      const float* p = cin;
  #pragma unroll
      for (int d = 0; d < NL; ++d)
  #pragma unroll
        for (int sidx = 0; sidx < 4; ++sidx) {
          const int kk = 2 * sidx + h;
          bco[d][sidx] = (kk < NB) ? p[d * NB + kk] : 0.0f;
        }
    } else {   // ProDMP, bc at step 0 (oracle/mp.py)
      const float* p = cin;
      const float* rb = tab;   // row 0
      const float y1 = rb[2 * NB + 2], y2 = rb[2 * NB + 3], dy1 = rb[2 * NB + 4], dy2 = rb[2 * NB + 5];
      const float det = y1 * dy2 - y2 * dy1;
  #pragma unroll
      for (int d = 0; d < NL; ++d) {
        float w[K];
  #pragma unroll
        for (int kk = 0; kk < NB; ++kk) w[kk] = p[d * (NB + 1) + kk] * c.ws32;
        w[NB] = p[d * (NB + 1) + NB] * c.gs32;
        float P = 0.0f, V = 0.0f;
  #pragma unroll
        for (int kk = 0; kk <= NB; ++kk) {
          P = __builtin_fmaf(rb[kk], w[kk], P);
          V = __builtin_fmaf(rb[NB + 1 + kk], w[kk], V);
        }
        const float A = p[CW + d] - P;            // (float) q0 - P
        const float B = p[CW + NL + d] * c.tau32 - V;   // (float) qd0 * tau - V
        w[NB + 1] = (dy2 * A - y2 * B) / det;
        w[NB + 2] = (y1 * B - dy1 * A) / det;
  #pragma unroll
        for (int sidx = 0; sidx < 4; ++sidx) bco[d][sidx] = w[2 * sidx + h];
      }
    }
    // the region's env runs (rows [row0, row0 + rows)) to out: wave w < 7 streams envs w, w + 7, ...,
    // the run's 16-B chunks over consecutive lanes; the env's base in SGPRs, the lane's offset in a VGPR
    auto store_region = [&](float* out, int row0, int rows) __attribute__((always_inline)) {
      const int cpe = rows * NL / 4;   // 16-B chunks per env run
      if (wave == kLoader) return;
      for (int je = wave; je < nenv; je += kTrajGWaves - 1) {
        gchar* base = uniform_ptr(out + ((e0 + je) * T + row0) * NL);
        const float* src = reg + je * ESR;
        for (int ch = lane; ch < cpe; ch += 64) {
          const f32x4 x = *reinterpret_cast<const f32x4*>(src + 4 * ch);
          *(__attribute__((address_space(1))) f32x4*)(base + 16u * (uint32_t)ch) = x;
        }
      }
    };

    for (int seg = 0; seg < nt; seg += kTrajGWaves) {
      const int row0 = seg * RSTEP;
      const int rows = (seg + kTrajGWaves >= nt) ? T - row0 : kTrajGWaves * RSTEP;   // (<= SR)
      const int t = seg + wave;
      const bool has_tile = t < nt;
      const int tb = t * RSTEP;
      const int rows_out = (t == nt - 1) ? T - tb : RSTEP;   // multiple of 4
      // lane (j, h) holds rows 8g + 4h + {0..3} of the tile (registers 4g + {0..3}); its LDS rows
      float* dst0 = reg + j * ESR + (tb - row0 + 4 * h) * NL;
      f32x16 cp[NL], cv[PRO ? NL : 1];   // positions, ProMP velocities
      float a1[4], a2[4];
      if (has_tile) {
        // ---- A operands: this lane feeds time row i = j of the tile, k = 2 sidx + h
        const int ktc = min(tb + j, T - 1);
        const float* ar = tab + (size_t)(ktc + 1) * stride;   // table row (s0 = 0)
#pragma unroll
        for (int sidx = 0; sidx < 4; ++sidx) {
          const int kk = 2 * sidx + h;
          if (PRO) {
            a1[sidx] = (kk < NB) ? ar[kk] : 0.0f;
            a2[sidx] = 0.0f;
          } else {
            a1[sidx] = (kk <= NB) ? ar[kk] : ar[2 * NB + 2 + (kk - NB - 1)];
            a2[sidx] = (kk <= NB) ? ar[NB + 1 + kk] : ar[2 * NB + 4 + (kk - NB - 1)];
          }
        }
#pragma unroll
        for (int d = 0; d < NL; ++d) {
          f32x16 z = {0.0f};
          cp[d] = z;
#pragma unroll
          for (int sidx = 0; sidx < 4; ++sidx) cp[d] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[sidx], bco[d][sidx], cp[d], 0, 0, 0);
        }
        if constexpr (PRO) {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            float dv0[4], dv1[4];
#pragma unroll
            for (int r4 = 0; r4 < 4; ++r4) {
              const int k = min(tb + 8 * g + 4 * h + r4, T - 1);
              // vel_k = (pos_{k+1} - pos_k) / dt32 of row k + 1; the last sample repeats vel_{T-2}
              const float* dr = tab + (size_t)(k + 1 - (k == T - 1 ? 1 : 0)) * stride + NB;
              dv0[r4] = dr[0];
              dv1[r4] = dr[1];
            }
#pragma unroll
            for (int d = 0; d < NL; ++d) {
              // the position after the lane's 4th row (row 8g + 4h + 4) is register 4g of the upper
              // half-wave for h = 0 and register 4g + 4 of the lower half for h = 1 (row 32: never
              // output): each half provides what the other needs
              const float nxt = partner(h ? cp[d][4 * g] : cp[d][min(4 * g + 4, 15)]);
#pragma unroll
              for (int r4 = 0; r4 < 4; ++r4) {
                const int rg = 4 * g + r4;
                const int k = tb + 8 * g + 4 * h + r4;   // plan sample of this row
                const float P = cp[d][rg];
                const float Q = (r4 < 3) ? cp[d][rg + 1] : nxt;
                const float Pp = (r4 > 0) ? cp[d][rg - 1] : 0.0f;
                cv[d][rg] = (k < T - 1) ? div_rcp(Q - P, dv0[r4], dv1[r4]) : div_rcp(P - Pp, dv0[r4], dv1[r4]);
              }
            }
          }
        }
      }
      // rows 8g + 4h .. + 3 of the lane's env: 4 NL consecutive floats (16-B aligned)
      auto stage = [&](const f32x16* v) __attribute__((always_inline)) {
        if (!has_tile || !stager) return;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          if (8 * g + 4 * h >= rows_out) break;
          f32x4* dst = reinterpret_cast<f32x4*>(dst0 + 8 * g * NL);
#pragma unroll
          for (int q = 0; q < NL; ++q) {
            f32x4 x;
#pragma unroll
            for (int u = 0; u < 4; ++u) x[u] = v[(4 * q + u) % NL][4 * g + (4 * q + u) / NL];
            dst[q] = x;
          }
        }
      };
      stage(cp);
      lds_barrier();
      store_region(dpos, row0, rows);
      lds_barrier();   // (every wave's region reads done before the velocities overwrite it)
      if constexpr (PRO) {
        stage(cv);
      } else {   // ProDMP velocities: the second contraction, into the position accumulators
        if (has_tile) {
#pragma unroll
          for (int d = 0; d < NL; ++d) {
            f32x16 z = {0.0f};
            cp[d] = z;
#pragma unroll
            for (int sidx = 0; sidx < 4; ++sidx) cp[d] = __builtin_amdgcn_mfma_f32_32x32x2f32(a2[sidx], bco[d][sidx], cp[d], 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 16; ++r) cp[d][r] = div_rcp(cp[d][r], c.tau32, c.rcp_tau32);
          }
        }
        stage(cp);
      }
      lds_barrier();
      store_region(dvel, row0, rows);
      lds_barrier();
    }
  }
}

// a launch with more than 64 KB of dynamic LDS needs the kernel's limit raised first
template <typename F>
inline void launch_lds(const void* kernel, size_t lds, F&& launch) {
  (void)raise_lds_limit(kernel, lds);
  launch();
}

inline int launch_traj_mfma(const DevCfg& c, const DevState& s, const float* params, float* dpos, float* dvel,
                            hipStream_t stream) {
  if (c.replan != 0 || c.nb != 5 || c.cond_desired || (c.T % 4) != 0) return 1;   // per-env plan starts: VALU kernel
  if (((uintptr_t)dpos | (uintptr_t)dvel) & 15) return 1;
  if ((int64_t)c.T * c.nl * 4 * 32 >= (int64_t)1 << 31) return 1;   // (32-bit run offsets)
  const bool r3 = std::getenv("FGX_TRAJ_R3") != nullptr;   // A/B: the round-3 kernel
  if (r3) {
    const int64_t groups = (c.N + 31) / 32;
    const int blocks = (int)((groups + kTrajWaves - 1) / kTrajWaves);
#define X(NL)                                                                                                  \
    if (c.nl == NL) {                                                                                          \
      if (c.mp == MP_PROMP) hipLaunchKernelGGL((k_traj_mfma_r3<MP_PROMP, NL>), dim3(blocks), dim3(64 * kTrajWaves), 0, stream, c, s, params, dpos, dvel); \
      else hipLaunchKernelGGL((k_traj_mfma_r3<MP_PRODMP, NL>), dim3(blocks), dim3(64 * kTrajWaves), 0, stream, c, s, params, dpos, dvel); \
      return hipGetLastError() == hipSuccess ? 0 : 2;                                                          \
    }
    X(2) X(5)
#undef X
    return 1;
  }
  const size_t lds = traj_mfma_lds_bytes(c.rows, c.stride, c.T, c.mp, c.nl);
  if (lds > 160 * 1024) return 1;   // (a table this long: the VALU kernel)
  // one workgroup per CU (its LDS), each walking groups; FGX_TRAJ_GRID (A/B) overrides the grid
  const int64_t groups = (c.N + kTrajGE - 1) / kTrajGE;
  int blocks = (int)std::min<int64_t>(groups, 256);
  if (const char* gv = std::getenv("FGX_TRAJ_GRID")) blocks = (int)std::max<int64_t>(1, std::min<int64_t>(groups, std::atoll(gv)));
#define X(NL)                                                                                                  \
  if (c.nl == NL) {                                                                                            \
    if (c.mp == MP_PROMP)                                                                                      \
      launch_lds((const void*)k_traj_mfma<MP_PROMP, NL>, lds, [&] { hipLaunchKernelGGL((k_traj_mfma<MP_PROMP, NL>), dim3(blocks), dim3(64 * kTrajGWaves), lds, stream, c, s, params, dpos, dvel); }); \
    else                                                                                                       \
      launch_lds((const void*)k_traj_mfma<MP_PRODMP, NL>, lds, [&] { hipLaunchKernelGGL((k_traj_mfma<MP_PRODMP, NL>), dim3(blocks), dim3(64 * kTrajGWaves), lds, stream, c, s, params, dpos, dvel); }); \
    return hipGetLastError() == hipSuccess ? 0 : 2;                                                            \
  }
  X(2) X(5)
#undef X
  return 1;
}

}  // namespace fgx
