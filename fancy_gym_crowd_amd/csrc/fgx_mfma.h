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
// (3.0 TB/s, 0.37 of HBM peak): it evaluated ProMP positions twice (rows k and k + 1, a second MFMA
// set) for the forward difference, held ~400 registers and a 20.5 KB LDS tile per wave (about one
// wave per SIMD), and alternated compute and store phases.  Here:
//   * ProMP computes each position once.  The forward difference takes row k + 1 from the next
//     register of the lane, or for the last row of a lane's 4-row group from the other half-wave
//     (v_permlane32_swap: rows 8g + 4 .. 8g + 7 live in lanes 32..63); a tile outputs its first 28
//     rows (the 28th's successor is in the tile, and 28-row steps keep every env's run 16-B aligned),
//     the plan's last tile all its remaining rows (velocity of the last = the previous one, as
//     Traj::at).  ProDMP's velocities are their own contraction (the second basis, vb) and keep their
//     MFMA set; its tiles step 32 rows.
//   * The output leaves through LDS one 8-row group (g) at a time: pos and vel of the group,
//     [env][row][dof] (row stride 8 NL + 4 floats), then 16-B stores where consecutive lanes write
//     consecutive chunks of each env's contiguous run (8 NL floats).  11 KB of LDS per wave instead of
//     20.5 KB: three 4-wave workgroups per CU.
template <int MP, int NL>
__global__ __launch_bounds__(256) void k_traj_mfma(DevCfg c, DevState s, const float* __restrict__ params,
                                                   float* __restrict__ dpos, float* __restrict__ dvel) {
  constexpr int NB = 5, K = 8;
  constexpr bool PRO = MP == MP_PROMP;
  constexpr int RSTEP = PRO ? 28 : 32;           // output rows per (non-final) tile
  constexpr int ES = 8 * NL + 4;                  // LDS floats per env of one staged group
  constexpr int WSTAGE = 2 * 32 * ES;             // pos + vel of 32 envs
  __shared__ __attribute__((aligned(16))) float lds_tr[4 * WSTAGE];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int j = lane & 31, h = lane >> 5;
  const int64_t N = c.N;
  const int64_t e0 = ((int64_t)blockIdx.x * 4 + wave) * 32;   // first env of this wave
  const int64_t e = e0 + j;
  const int64_t ec = e < N ? e : (N - 1);
  const float* tab = s.tables;
  const int stride = c.stride;
  float* sp = lds_tr + wave * WSTAGE;   // [env][8 rows][NL] positions
  float* sv = sp + 32 * ES;             // velocities

  // ---- per-env coefficients C[d][k] (only the k = 2 sidx + h this lane feeds are kept)
  float bco[NL][4];
  if (PRO) {
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
  // the other half-wave's value of x (lane l <-> l ^ 32)
  auto partner = [&](float x) __attribute__((always_inline)) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(h ? r[0] : r[1]);
  };
  auto wave_sync = [] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  };

  const int T = c.T;
  for (int tb = 0; tb < T;) {
    const bool last_tile = T - tb <= 32;
    const int rows_out = last_tile ? T - tb : RSTEP;   // multiple of 4 (T % 4 == 0)
    // ---- A operands: this lane feeds time row i = j of the tile, k = 2 sidx + h
    const int ktc = min(tb + j, T - 1);
    const int row = ktc + 1;                     // table row (s0 = 0)
    float a1[4], a2[4];
#pragma unroll
    for (int sidx = 0; sidx < 4; ++sidx) {
      const int kk = 2 * sidx + h;
      const float* r = tab + (size_t)row * stride;
      if (PRO) {
        a1[sidx] = (kk < NB) ? r[kk] : 0.0f;
        a2[sidx] = 0.0f;
      } else {
        a1[sidx] = (kk <= NB) ? r[kk] : r[2 * NB + 2 + (kk - NB - 1)];
        a2[sidx] = (kk <= NB) ? r[NB + 1 + kk] : r[2 * NB + 4 + (kk - NB - 1)];
      }
    }
    f32x16 cp[NL], cq[PRO ? 1 : NL];
#pragma unroll
    for (int d = 0; d < NL; ++d) {
      f32x16 z = {0.0f};
      cp[d] = z;
#pragma unroll
      for (int sidx = 0; sidx < 4; ++sidx) cp[d] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[sidx], bco[d][sidx], cp[d], 0, 0, 0);
      if constexpr (!PRO) {
        cq[d] = z;
#pragma unroll
        for (int sidx = 0; sidx < 4; ++sidx)
          cq[d] = __builtin_amdgcn_mfma_f32_32x32x2f32(a2[sidx], bco[d][sidx], cq[d], 0, 0, 0);
      }
    }
    // ---- per 8-row group g: lane (j, h) holds rows 8g + 4h + {0..3} (registers 4g + {0..3})
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int rg = min(max(rows_out - 8 * g, 0), 8);   // rows of the group this tile outputs (0, 4 or 8)
      if (rg == 0) break;
      float pv[4 * NL], vv[4 * NL];
#pragma unroll
      for (int d = 0; d < NL; ++d) {
        // ProMP: the position after the lane's 4th row (row 8g + 4h + 4) is register 4g of the upper
        // half-wave for h = 0 and register 4g + 4 of the lower half for h = 1 (row 32: never output):
        // each half provides what the other needs
        float nxt = 0.0f;
        if constexpr (PRO) nxt = partner(h ? cp[d][4 * g] : cp[d][min(4 * g + 4, 15)]);
#pragma unroll
        for (int r4 = 0; r4 < 4; ++r4) {
          const int reg = 4 * g + r4;
          const int k = tb + 8 * g + 4 * h + r4;   // plan sample of this row
          const float P = cp[d][reg];
          float vel;
          if constexpr (PRO) {
            const float Q = (r4 < 3) ? cp[d][reg + 1] : nxt;
            const int kc = k < T ? k : T - 1;
            // vel_k = (pos_{k+1} - pos_k) / dt32 of row k + 1; the last sample repeats vel_{T-2}
            const float* dr = tab + (size_t)(kc + 1 - (kc == T - 1 ? 1 : 0)) * stride + NB;
            const float Pp = (r4 > 0) ? cp[d][reg - 1] : 0.0f;
            vel = (kc < T - 1) ? div_rcp(Q - P, dr[0], dr[1]) : div_rcp(P - Pp, dr[0], dr[1]);
          } else {
            vel = div_rcp(cq[d][reg], c.tau32, c.rcp_tau32);
          }
          pv[r4 * NL + d] = P;
          vv[r4 * NL + d] = vel;
        }
      }
      float* dp_ = sp + j * ES + 4 * h * NL;
      float* dv_ = sv + j * ES + 4 * h * NL;
#pragma unroll
      for (int q4 = 0; q4 < NL; ++q4) {
        *reinterpret_cast<f32x4*>(dp_ + 4 * q4) = f32x4{pv[4 * q4], pv[4 * q4 + 1], pv[4 * q4 + 2], pv[4 * q4 + 3]};
        *reinterpret_cast<f32x4*>(dv_ + 4 * q4) = f32x4{vv[4 * q4], vv[4 * q4 + 1], vv[4 * q4 + 2], vv[4 * q4 + 3]};
      }
      wave_sync();
      // each env's run of this group: rg rows x NL floats, contiguous in [N, T, dof] at row tb + 8 g
      const int chunks = rg * NL / 4;   // 16-B chunks per env
      const int64_t obase = (int64_t)(tb + 8 * g) * NL;
      for (int idx = lane; idx < 32 * chunks; idx += 64) {
        const int je = idx / chunks, ch = idx - je * chunks;
        const int64_t ee = e0 + je;
        if (ee < N) {
          const int64_t off = ee * T * NL + obase + 4 * ch;
          *reinterpret_cast<f32x4*>(dpos + off) = *reinterpret_cast<const f32x4*>(sp + je * ES + 4 * ch);
          *reinterpret_cast<f32x4*>(dvel + off) = *reinterpret_cast<const f32x4*>(sv + je * ES + 4 * ch);
        }
      }
      wave_sync();
    }
    tb += rows_out;
  }
}

inline int launch_traj_mfma(const DevCfg& c, const DevState& s, const float* params, float* dpos, float* dvel,
                            hipStream_t stream) {
  if (c.replan != 0 || c.nb != 5 || c.cond_desired || (c.T % 4) != 0) return 1;   // per-env plan starts: VALU kernel
  if (((uintptr_t)dpos | (uintptr_t)dvel) & 15) return 1;
  const bool r3 = std::getenv("FGX_TRAJ_R3") != nullptr;   // A/B: the round-3 kernel
  const int threads = r3 ? 64 * kTrajWaves : 256;
  const int64_t groups = (c.N + 31) / 32;
  const int blocks = (int)((groups + (threads / 64) - 1) / (threads / 64));
#define X(NL)                                                                                                  \
  if (c.nl == NL) {                                                                                            \
    if (c.mp == MP_PROMP) {                                                                                    \
      if (r3) hipLaunchKernelGGL((k_traj_mfma_r3<MP_PROMP, NL>), dim3(blocks), dim3(threads), 0, stream, c, s, params, dpos, dvel); \
      else hipLaunchKernelGGL((k_traj_mfma<MP_PROMP, NL>), dim3(blocks), dim3(threads), 0, stream, c, s, params, dpos, dvel); \
    } else {                                                                                                   \
      if (r3) hipLaunchKernelGGL((k_traj_mfma_r3<MP_PRODMP, NL>), dim3(blocks), dim3(threads), 0, stream, c, s, params, dpos, dvel); \
      else hipLaunchKernelGGL((k_traj_mfma<MP_PRODMP, NL>), dim3(blocks), dim3(threads), 0, stream, c, s, params, dpos, dvel); \
    }                                                                                                          \
    return hipGetLastError() == hipSuccess ? 0 : 2;                                                            \
  }
  X(2) X(5)
#undef X
  return 1;
}

}  // namespace fgx
