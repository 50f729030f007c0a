// fgx_dispatch.h — template dispatch of the episode kernel.  One translation unit per env kind
// and basis specialisation (fgx_ep_<env>.hip: NB = 5, the registered configs; fgx_ep_<env>_gen.hip:
// NB = 0, the generic runtime basis count), so that the build compiles them in parallel.
#pragma once
#include <string>

#include "fgx_kernels.h"

// returns 0 / FGX_E_* code, message in err
#define FGX_DECLARE_LAUNCH(NAME)                                                                             \
  int NAME(const fgx::DevCfg& c, const fgx::DevState& s, int mp, const float* params, const float* dpos,     \
           const float* dvel, const fgx::Outputs& o, hipStream_t stream, std::string& err);
FGX_DECLARE_LAUNCH(fgx_launch_episode_simple)
FGX_DECLARE_LAUNCH(fgx_launch_episode_hole)
FGX_DECLARE_LAUNCH(fgx_launch_episode_via)
FGX_DECLARE_LAUNCH(fgx_launch_episode_simple_gen)
FGX_DECLARE_LAUNCH(fgx_launch_episode_hole_gen)
FGX_DECLARE_LAUNCH(fgx_launch_episode_via_gen)
#undef FGX_DECLARE_LAUNCH

namespace fgx {

template <int ENV, int MP, int CTRL, int NL, int NB>
static int launch_episode_nl(const DevCfg& c, const DevState& s, const float* params, const float* dpos,
                             const float* dvel, const Outputs& o, hipStream_t stream, std::string& err) {
  const int threads = 256;
  const int blocks = (int)((c.N + threads - 1) / threads);
  const size_t lds = (MP == MP_GIVEN) ? 0 : (size_t)c.rows * c.stride * sizeof(float);
  const bool log = o.positions || o.step_actions || o.step_obs || o.step_rewards || o.is_collided ||
                   o.end_effector || o.reward_dist;
  if (log)
    hipLaunchKernelGGL((k_episode<ENV, MP, CTRL, NL, NB, true>), dim3(blocks), dim3(threads), lds, stream, c, s,
                       params, dpos, dvel, o);
  else
    hipLaunchKernelGGL((k_episode<ENV, MP, CTRL, NL, NB, false>), dim3(blocks), dim3(threads), lds, stream, c, s,
                       params, dpos, dvel, o);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) { err = std::string("k_episode launch: ") + hipGetErrorString(e); return -2; }
  return 0;
}

template <int ENV, int MP, int CTRL, int NB>
static int launch_episode_ctrl(const DevCfg& c, const DevState& s, const float* params, const float* dpos,
                               const float* dvel, const Outputs& o, hipStream_t stream, std::string& err) {
  if (c.nl == 2) return launch_episode_nl<ENV, MP, CTRL, 2, NB>(c, s, params, dpos, dvel, o, stream, err);
  if (c.nl == 5) return launch_episode_nl<ENV, MP, CTRL, 5, NB>(c, s, params, dpos, dvel, o, stream, err);
  err = "n_links not instantiated (supported: 2, 5)";
  return -4;
}

template <int ENV, int MP, int NB>
static int launch_episode_mp(const DevCfg& c, const DevState& s, const float* params, const float* dpos,
                             const float* dvel, const Outputs& o, hipStream_t stream, std::string& err) {
  switch (c.ctrl) {
    case CTRL_PD: return launch_episode_ctrl<ENV, MP, CTRL_PD, NB>(c, s, params, dpos, dvel, o, stream, err);
    case CTRL_VEL: return launch_episode_ctrl<ENV, MP, CTRL_VEL, NB>(c, s, params, dpos, dvel, o, stream, err);
    case CTRL_POS: return launch_episode_ctrl<ENV, MP, CTRL_POS, NB>(c, s, params, dpos, dvel, o, stream, err);
  }
  err = "bad ctrl_kind";
  return -1;
}

// NB = 5: every MP kind and the caller-given trajectory; NB = 0: the MP kinds with c.nb != 5
template <int ENV, int NB>
static int launch_episode_env(const DevCfg& c, const DevState& s, int mp, const float* params, const float* dpos,
                              const float* dvel, const Outputs& o, hipStream_t stream, std::string& err) {
  switch (mp) {
    case MP_PROMP: return launch_episode_mp<ENV, MP_PROMP, NB>(c, s, params, dpos, dvel, o, stream, err);
    case MP_DMP: return launch_episode_mp<ENV, MP_DMP, NB>(c, s, params, dpos, dvel, o, stream, err);
    case MP_PRODMP: return launch_episode_mp<ENV, MP_PRODMP, NB>(c, s, params, dpos, dvel, o, stream, err);
    case MP_GIVEN:
      if (NB == 5) return launch_episode_mp<ENV, MP_GIVEN, 5>(c, s, params, dpos, dvel, o, stream, err);
      break;
  }
  err = "bad mp kind";
  return -1;
}

}  // namespace fgx
