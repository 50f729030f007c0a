// fgx_ws.h — k_episode_ws: the wave-specialised black-box step for SimpleReacher + PD (the metric
// path at N = 65536 envs per GPU).
//
// k_episode keeps one env per lane with the whole BlackBoxWrapper.step (black_box_wrapper.py:
// 170-253) in one instruction stream: MP trajectory (f32 basis contraction + velocity division),
// PD controller, clip, torque Euler step, reward and the numpy pairwise return.  At N = 65536 that
// is one wave per SIMD, and a lone wave issues a VALU instruction only every ~6-9 cycles however
// independent its instructions are (profiles/r01_valu_rates.jsonl: 2 waves reach ~5, the SIMD
// ~4.5 for f64).  Here a workgroup of 8 waves owns 256 envs and splits every env's stream in two:
//   waves 4..7 (producers) evaluate the desired trajectory of their 64 envs (Traj, exactly the
//              operations of k_episode) a chunk of kWsChunk samples ahead and store pos / vel in LDS;
//   waves 0..3 (consumers) read them and run PD, clip, dynamics, reward, return, TimeLimit,
//              replanning, the FK at env step 199 and the epilogue, one env per lane as k_episode.
// Wave w and wave w + 4 of a workgroup always share a SIMD (tools/wave_placement.hip: 4096 of 4096
// pairs), so every SIMD interleaves one producer and one consumer: two issuing waves with no
// duplicated instruction.  The chunk buffers are double-buffered: one workgroup barrier per chunk.
//
// Every expression rounds exactly as in k_episode (same operations, same order), so results are
// bit-identical (tests/test_gpu_ws.py).  Served: ENV_SIMPLE + PD + shared tables + info_level < 2
// + static replanning schedules + T <= 256 (fgx_dispatch.h picks among k_episode / _jp / _ws).
#pragma once
#include "fgx_jp.h"

namespace fgx {

constexpr int kWsChunk = 4;   // samples per LDS chunk (fast 8-blocks are two chunks)
constexpr int kWsPairs = 4;   // consumer / producer wave pairs per workgroup
#ifndef FGX_WS_WAVES
#define FGX_WS_WAVES 2
#endif

// pos / vel of one sample for 64 lanes: 2 NL floats per lane, padded to float4 groups
template <int NL>
__host__ __device__ constexpr int ws_quads() { return (2 * NL + 3) / 4; }
template <int NL>
inline size_t ws_lds_bytes(int rows, int stride) {
  return (((size_t)rows * stride + 3) & ~(size_t)3) * sizeof(float) +
         (size_t)kWsPairs * 2 * kWsChunk * ws_quads<NL>() * 64 * sizeof(float4) + 16 * sizeof(int);
}

template <int MP, int NL, int NB>
__global__ __launch_bounds__(512, FGX_WS_WAVES) void k_episode_ws(DevCfg c, DevState s, const float* __restrict__ params,
                                                       Outputs o) {
  constexpr int Q = ws_quads<NL>();
  extern __shared__ float4 lds_ws[];
  float* tab = (float*)lds_ws;
  const int tab_f = c.rows * c.stride;
  float4* buf = lds_ws + (tab_f + 3) / 4;                // [pair][2][kWsChunk][Q][64]
  int* red = (int*)(buf + kWsPairs * 2 * kWsChunk * Q * 64);
  for (int i = threadIdx.x; i < tab_f; i += blockDim.x) tab[i] = s.tables[i];

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool producer = w >= kWsPairs;
  const int pair = w & (kWsPairs - 1);
  const int64_t N = c.N;
  const int64_t e0 = (int64_t)blockIdx.x * (64 * kWsPairs) + pair * 64 + lane;
  const bool valid = e0 < N;
  const int64_t e = valid ? e0 : N - 1;   // clamped index: loads stay in bounds, nothing is stored
  float4* mybuf = buf + (size_t)pair * 2 * kWsChunk * Q * 64;
  auto slot = [&](int b, int i, int qd) -> float4& { return mybuf[((b * kWsChunk + i) * Q + qd) * 64 + lane]; };

  // segment length of every env (the same in both waves of a pair); workgroup-wide chunk count
  JpSeg sg;
  sg.init(c, s, e, valid);
  const int Lw = wave_max(sg.L);   // (all lanes take part in the shuffles)
  if (lane == 0) red[w] = Lw;
  __syncthreads();   // table staged, red[] written
  int Lwg = 0;
#pragma unroll
  for (int i = 0; i < 2 * kWsPairs; ++i) Lwg = max(Lwg, red[i]);
  const int nch = (Lwg + kWsChunk - 1) / kWsChunk;

  if (producer) {
    // ------------------------------------------------------------------ producer waves
    Traj<MP, NL, NB> tg;
    {
      double ic_q[NL], ic_qd[NL];
      const bool has_cond = c.cond_desired && (sg.flags & 2u);
#pragma unroll
      for (int k = 0; k < NL; ++k) {
        ic_q[k] = has_cond ? (double)s.cond[k * N + e] : s.q[k * N + e];
        ic_qd[k] = has_cond ? (double)s.cond[(NL + k) * N + e] : s.qd[k * N + e];
      }
      const int s0 = c.replan ? sg.steps : 0;
      tg.init(c, params + e * c.n_params, tab, s0, ic_q, ic_qd);
    }
    auto produce = [&](int ch) {
      const int b = ch & 1;
#pragma unroll
      for (int i = 0; i < kWsChunk; ++i) {
        float f[4 * Q];
        tg.at(c, ch * kWsChunk + i, f, f + NL);
#pragma unroll
        for (int j = 2 * NL; j < 4 * Q; ++j) f[j] = 0.0f;
#pragma unroll
        for (int qd = 0; qd < Q; ++qd) slot(b, i, qd) = make_float4(f[4 * qd], f[4 * qd + 1], f[4 * qd + 2], f[4 * qd + 3]);
      }
    };
    if (nch > 0) produce(0);
    __syncthreads();
    for (int ch = 0; ch < nch; ++ch) {
      if (ch + 1 < nch) produce(ch + 1);
      __syncthreads();
    }
    return;
  }

  // -------------------------------------------------------------------- consumer waves
  Env<NL> v;
  load_env(c, s, e, v, false);   // SimpleReacher: no hole / reward state
  const int k_replan = sg.k_replan;
  const int Te = c.T;
  // numpy pairwise split of the return sum (SimpleReacher never terminates: L is known now)
  const int split = (sg.L > 128) ? ((sg.L / 2) & ~7) : 0;
  PairwiseSum ps;
  ps.init();
  bool stop = false, trunc = false;
  float pos[NL], vel[NL];
  const double act_lo = __builtin_canonicalize(c.act_lo), act_hi = __builtin_canonicalize(c.act_hi);

  // fast 8-blocks as in k_episode: no lane reaches env step 199 (FK), the TimeLimit or the
  // replanning sample inside them; a wave-uniform count, one split per wave
  int nfast;
  {
    int lim = min(199, c.max_steps - 1) - v.steps;
    if (k_replan >= 0) lim = min(lim, k_replan);
    nfast = min(Te, max(0, lim)) / 8;
    if (!valid) nfast = 0;
    if (__ballot(1) != ~0ull) nfast = 0;
    if (__ballot(split != __builtin_amdgcn_readfirstlane(split)) != 0) nfast = 0;
    nfast = wave_min(nfast);
  }
  const int usplit = __builtin_amdgcn_readfirstlane(split);

  // one sample: PD (black_box_wrapper.py:201-205) on the staged desired state, env.step
  auto controls = [&](double* a, bool exact_nan) {
    bool nan_in = false;
#pragma unroll
    for (int d = 0; d < NL; ++d) {
      const double u = fadd(c.pg[d] * fsub((double)pos[d], v.q[d]), c.dg[d] * fsub((double)vel[d], v.qd[d]));
      a[d] = __builtin_fmin(__builtin_fmax(u, act_lo), act_hi);
      nan_in |= (u != u);
      if (exact_nan) a[d] = (u != u) ? u : a[d];
    }
    // np.clip propagates NaN; max/min do not: fix up (rare, wave-uniform branch)
    if (!exact_nan && __builtin_expect(__ballot(nan_in) != 0, 0)) {
#pragma unroll
      for (int d = 0; d < NL; ++d) {
        const double u = fadd(c.pg[d] * fsub((double)pos[d], v.q[d]), c.dg[d] * fsub((double)vel[d], v.qd[d]));
        if (u != u) a[d] = u;
      }
    }
  };
  auto load_sample = [&](int b, int i) {
    float f[4 * Q];
#pragma unroll
    for (int qd = 0; qd < Q; ++qd) {
      const float4 x = slot(b, i, qd);
      f[4 * qd] = x.x; f[4 * qd + 1] = x.y; f[4 * qd + 2] = x.z; f[4 * qd + 3] = x.w;
    }
#pragma unroll
    for (int d = 0; d < NL; ++d) { pos[d] = f[d]; vel[d] = f[NL + d]; }
  };
  // fast sample with compile-time slot J and phase PH (PairwiseSum::add_fast)
  auto fast_sample = [&](int b, int i, auto Jtag, auto PHtag) {
    constexpr int J = decltype(Jtag)::value, PH = decltype(PHtag)::value;
    load_sample(b, i);
    double a[NL];
    float a32[NL];
    controls(a, false);
    const StepOut r = substep<ENV_SIMPLE, false, NL, false>(c, v, a, a32, false);
    ps.template add_fast<J, PH>(r.reward);
  };
  // generic sample k (per lane): FK at step 199, TimeLimit, replanning, condition_on_desired
  int k_next = 0;
  auto generic_sample = [&](int b, int i, int k) {
    load_sample(b, i);
    double a[NL];
    float a32[NL];
    controls(a, true);
    const StepOut r = substep<ENV_SIMPLE, false, NL, true>(c, v, a, a32, false);
    trunc = v.steps >= c.max_steps;
    ps.add(k, r.reward, split);
    k_next = k + 1;
    if (trunc || k == k_replan) {
      if (c.cond_desired) {   // black_box_wrapper.py:234-236
#pragma unroll
        for (int d = 0; d < NL; ++d) { s.cond[d * N + e] = pos[d]; s.cond[(NL + d) * N + e] = vel[d]; }
        v.flags |= 2u;
      }
      stop = true;
    }
  };

  __syncthreads();   // chunk 0 staged
  bool synced = false;   // PairwiseSum tails combined after the fast blocks
  for (int ch = 0; ch < nch; ++ch) {
    const int b = ch & 1, k0 = ch * kWsChunk;
    if (k0 + kWsChunk <= 8 * nfast) {
      if (usplit > 0 && k0 == usplit) ps.first = PairwiseSum::comb(ps.a);   // blocks [0, split)
      const int ph = (k0 < 128 ? 1 : 0) | ((usplit > 0 && k0 >= usplit) ? 2 : 0);
      const bool hi = (k0 & 7) != 0;   // second half of an 8-block: slots 4..7
#define FGX_WS_CHUNK(PH, J0)                                                                             \
      fast_sample(b, 0, std::integral_constant<int, J0>{}, std::integral_constant<int, PH>{});     \
      fast_sample(b, 1, std::integral_constant<int, J0 + 1>{}, std::integral_constant<int, PH>{}); \
      fast_sample(b, 2, std::integral_constant<int, J0 + 2>{}, std::integral_constant<int, PH>{}); \
      fast_sample(b, 3, std::integral_constant<int, J0 + 3>{}, std::integral_constant<int, PH>{});
      static_assert(kWsChunk == 4, "fast chunk unrolled for 4 samples");
      if (ph == 1) { if (hi) { FGX_WS_CHUNK(1, 4) } else { FGX_WS_CHUNK(1, 0) } }
      else if (ph == 3) { if (hi) { FGX_WS_CHUNK(3, 4) } else { FGX_WS_CHUNK(3, 0) } }
      else { if (hi) { FGX_WS_CHUNK(2, 4) } else { FGX_WS_CHUNK(2, 0) } }
#undef FGX_WS_CHUNK
      k_next = k0 + kWsChunk;
    } else {
      if (!synced) { ps.sync_tails(); synced = true; }
#pragma unroll
      for (int i = 0; i < kWsChunk; ++i) {
        const int k = k0 + i;
        if (valid && !stop && k < Te) generic_sample(b, i, k);
      }
    }
    __syncthreads();   // chunk consumed; the producers' next chunk is staged
  }
  if (!synced) ps.sync_tails();
  if (!valid) return;
  const int L = k_next;   // samples executed (trajectory_length)
  v.fk();
  episode_epilogue(c, s, o, e, v, sg.plans, L, ps.result(L, split), false, trunc);
}

}  // namespace fgx
