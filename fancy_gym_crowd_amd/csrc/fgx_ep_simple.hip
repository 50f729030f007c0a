// SimpleReacher (torque) instantiations of k_episode, NB = 5 (the registered basis count).
#include "fgx_dispatch.h"

int fgx_launch_episode_simple(const fgx::DevCfg& c, const fgx::DevState& s, int mp, const float* params,
                              const float* dpos, const float* dvel, const fgx::Outputs& o, hipStream_t stream,
                              std::string& err) {
  return fgx::launch_episode_env<fgx::ENV_SIMPLE, 5>(c, s, mp, params, dpos, dvel, o, stream, err);
}
