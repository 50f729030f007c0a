// fgx_ep_nl.h — every kernel family of one link count FGX_NL outside the registered 2 and 5
// (include/fgx.h n_links 1..8; the reference env takes any n_links, base_reacher.py:17-39, and
// bb_env_constructor forwards env kwargs, envs/registry.py:280-281).  Included once by each
// fgx_ep_nl<n>.hip, which defines FGX_NL, so that the counts compile in parallel.  The episode is the
// logging k_episode (fgx_dispatch.h LOG_ONLY: it serves every info level and the validity checks) on
// the generic basis count (NB = 0, any n_basis <= 12); reset, step-based step, trajectories and the
// learned-phase plans are the same templates the registered counts use.  Sums over the joints follow
// numpy's order at every count (np_sum, fgx_device.h: the pairwise tree at 8).
#pragma once
#include "fgx_dispatch.h"
#include "fgx_learned.h"
#include "fgx_step.h"
#include "fgx_traj_run.h"

#define FGX_NL_CAT2(a, b) a##b
#define FGX_NL_CAT(a, b) FGX_NL_CAT2(a, b)

namespace {
using namespace fgx;
constexpr int NLV = FGX_NL;

int hip_status(const char* what, std::string& err) {
  const hipError_t e = hipGetLastError();
  if (e == hipSuccess) return 0;
  err = std::string(what) + ": " + hipGetErrorString(e);
  return -2;
}

int nl_episode(const DevCfg& c, const DevState& s, int mp, const float* params, const float* dpos, const float* dvel,
               const Outputs& o, hipStream_t stream, std::string& err) {
  switch (c.env) {
    case ENV_SIMPLE: return launch_episode_env<ENV_SIMPLE, 0, NLV>(c, s, mp, params, dpos, dvel, o, stream, err);
    case ENV_HOLE: return launch_episode_env<ENV_HOLE, 0, NLV>(c, s, mp, params, dpos, dvel, o, stream, err);
    case ENV_VIA: return launch_episode_env<ENV_VIA, 0, NLV>(c, s, mp, params, dpos, dvel, o, stream, err);
  }
  err = "bad env kind";
  return -1;
}

int nl_reset(const DevCfg& c, const DevState& s, const uint64_t* seeds, const uint8_t* mask, int rs_mode, float* obs,
             hipStream_t stream, std::string& err) {
  const int threads = 256;
  hipLaunchKernelGGL((k_reset<NLV>), dim3((unsigned)((c.N + threads - 1) / threads)), dim3(threads), 0, stream, c, s,
                     seeds, mask, rs_mode, obs);
  return hip_status("k_reset", err);
}

int nl_step_raw(const DevCfg& c, const DevState& s, const float* act, float* obs, double* rew, uint8_t* term,
                uint8_t* trunc, float* final_obs, int autoreset, size_t lds, hipStream_t stream, std::string& err) {
  const dim3 grid((unsigned)((c.N + kStepRawBlock - 1) / kStepRawBlock)), block(kStepRawBlock);
  if (c.env == ENV_SIMPLE)
    hipLaunchKernelGGL((k_step_raw<ENV_SIMPLE, NLV>), grid, block, lds, stream, c, s, act, obs, rew, term, trunc,
                       final_obs, autoreset);
  else if (c.env == ENV_HOLE)
    hipLaunchKernelGGL((k_step_raw<ENV_HOLE, NLV>), grid, block, lds, stream, c, s, act, obs, rew, term, trunc,
                       final_obs, autoreset);
  else
    hipLaunchKernelGGL((k_step_raw<ENV_VIA, NLV>), grid, block, lds, stream, c, s, act, obs, rew, term, trunc,
                       final_obs, autoreset);
  return hip_status("k_step_raw", err);
}

int nl_traj(const DevCfg& c, const DevState& s, const float* params, float* dpos, float* dvel, hipStream_t stream,
            std::string& err) {
  const int rr = launch_traj_run<NLV>(c, s, params, dpos, dvel, stream);
  if (rr == 0) return 0;
  if (rr == 2) return hip_status("k_traj_run", err);
  const int threads = 256;
  const dim3 grid((unsigned)((c.N + threads - 1) / threads)), block(threads);
  if (c.mp == MP_PROMP) hipLaunchKernelGGL((k_traj_valu<MP_PROMP, NLV, 0>), grid, block, 0, stream, c, s, params, dpos, dvel);
  else if (c.mp == MP_DMP) hipLaunchKernelGGL((k_traj_valu<MP_DMP, NLV, 0>), grid, block, 0, stream, c, s, params, dpos, dvel);
  else if (c.mp == MP_PRODMP) hipLaunchKernelGGL((k_traj_valu<MP_PRODMP, NLV, 0>), grid, block, 0, stream, c, s, params, dpos, dvel);
  else { err = "step-based handle has no trajectory generator"; return -1; }
  return hip_status("k_traj_valu", err);
}

int nl_traj_env(const DevCfg& c, const DevState& s, const float* params, float* env_tab, float* dpos, float* dvel,
                int32_t* plan_len, float* info_pos, float* info_vel, hipStream_t stream, std::string& err) {
  const int threads = 256;
  const dim3 grid((unsigned)((c.N + threads - 1) / threads)), block(threads);
#define FGX_NL_TRAJ_ENV(MPV)                                                                                  \
  hipLaunchKernelGGL((k_traj_env<MPV, NLV, 0>), grid, block, 0, stream, c, s, params, env_tab, dpos, dvel, plan_len, \
                     info_pos, info_vel)
  if (c.mp == MP_PROMP) FGX_NL_TRAJ_ENV(MP_PROMP);
  else if (c.mp == MP_DMP) FGX_NL_TRAJ_ENV(MP_DMP);
  else if (c.mp == MP_PRODMP) FGX_NL_TRAJ_ENV(MP_PRODMP);
  else { err = "learned phase parameters need a movement primitive"; return -1; }
#undef FGX_NL_TRAJ_ENV
  return hip_status("k_traj_env", err);
}
}  // namespace

const fgx::NlOps* FGX_NL_CAT(fgx_nl_ops_, FGX_NL)() {
  static const fgx::NlOps ops = {nl_episode, nl_reset, nl_step_raw, nl_traj, nl_traj_env};
  return &ops;
}
