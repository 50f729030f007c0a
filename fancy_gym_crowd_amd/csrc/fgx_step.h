// fgx_step.h — k_step_raw: one step-based env.step for all envs (the per-substep kernel of the
// step-based ids 'fancy/{Simple,LongSimple,Hole,ViaPoint}Reacher-v0'; base_reacher.py:98-119,
// base_reacher_torque.py:20-37, base_reacher_direct.py).  Own header: only fgx_api.hip
// instantiates it, so the episode units do not recompile for it.
#pragma once
#include "fgx_kernels.h"

namespace fgx {

// One env.step (base_reacher_torque.py:20-37 / base_reacher_direct.py) for all envs, one thread
// per env, state in the SoA arrays.  Actions [N, NL] and observations [N, obs_dim] are per-env
// rows (AoS): the workgroup moves its contiguous slice of them through LDS, so every
// wave-instruction of the HBM side reads / writes 64 consecutive floats (256 B) instead of one
// float per lane at a NL·4 / obs_dim·4-byte stride.  LDS rows use an odd stride (no bank
// conflicts for the per-thread row accesses).  Dynamic LDS: kStepRawBlock · (NL + 1 | od + 1)
// floats, twice with final_obs (fgx_step_raw sizes it).
constexpr int kStepRawBlock = 256;
__host__ __device__ constexpr int step_raw_stride(int w) { return w | 1; }

template <int ENV, int NL>
__global__ __launch_bounds__(kStepRawBlock) void k_step_raw(DevCfg c, DevState s, const float* __restrict__ act,
                                                            float* obs, double* rew, uint8_t* term, uint8_t* trunc,
                                                            float* final_obs, int autoreset) {
  constexpr int B = kStepRawBlock;
  extern __shared__ float lds_raw[];
  const int od = c.obs_dim, so = step_raw_stride(od);
  constexpr int sa = step_raw_stride(NL);
  const int64_t e0 = (int64_t)blockIdx.x * B;
  const int t = threadIdx.x;
  const int nb = (int)((c.N - e0) < B ? (c.N - e0) : B);   // envs of this workgroup (grid = ceil(N / B))
  const int64_t e = e0 + t;
  const bool live = t < nb;
  float* lo = lds_raw;                                       // actions, then observations
  float* lf = lds_raw + B * (so > sa ? so : sa);             // final observations
  float a32[NL];
  double a[NL];
#ifndef FGX_STEP_RAW_DIRECT
  const float* ag = act + e0 * NL;
  for (int i = t; i < nb * NL; i += B) lo[(i / NL) * sa + i % NL] = ag[i];
  __syncthreads();
#pragma unroll
  for (int d = 0; d < NL; ++d) { a32[d] = live ? lo[t * sa + d] : 0.f; a[d] = (double)a32[d]; }
  __syncthreads();   // the action rows are read: lo now takes the observations
#else   // A/B diagnostics build (tools/bench_kernels.py raw): round 1's per-lane AoS rows
#pragma unroll
  for (int d = 0; d < NL; ++d) { a32[d] = live ? act[e * NL + d] : 0.f; a[d] = (double)a32[d]; }
#endif
  if (live) {
    Env<NL> v;
    load_env(c, s, e, v, ENV != ENV_SIMPLE);
    const StepOut r = substep<ENV, true, NL>(c, v, a, a32, true);
    const bool te = (ENV != ENV_SIMPLE) && r.coll, tr = v.steps >= c.max_steps;
    rew[e] = r.reward;
    term[e] = te;
    trunc[e] = tr;
#ifndef FGX_STEP_RAW_DIRECT
    float* ob = lo + t * so;
    float* fo = final_obs ? lf + t * so : nullptr;
#else
    float* ob = obs + e * od;
    float* fo = final_obs ? final_obs + e * od : nullptr;
#endif
    if (autoreset && (te || tr)) {
      if (fo) emit_obs(c, v, false, fo, nullptr);
      autoreset_env(c, s, e, v);
      v.flags = 0;
      emit_obs(c, v, false, ob, nullptr);
    } else {
      emit_obs(c, v, false, ob, fo);
    }
    store_env(c, s, e, v, ENV != ENV_SIMPLE);
  }
#ifndef FGX_STEP_RAW_DIRECT
  __syncthreads();
  float* og = obs + e0 * od;
  for (int i = t; i < nb * od; i += B) og[i] = lo[(i / od) * so + i % od];
  if (final_obs) {
    float* fg = final_obs + e0 * od;
    for (int i = t; i < nb * od; i += B) fg[i] = lf[(i / od) * so + i % od];
  }
#endif
}

}  // namespace fgx
