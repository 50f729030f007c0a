// ViaPointReacher (direct velocity) instantiations of k_episode, NB = 0 (generic runtime basis count).
#include "fgx_dispatch.h"

int fgx_launch_episode_via_gen(const fgx::DevCfg& c, const fgx::DevState& s, int mp, const float* params,
                                  const float* dpos, const float* dvel, const fgx::Outputs& o, hipStream_t stream,
                                  std::string& err) {
  return fgx::launch_episode_env<fgx::ENV_VIA, 0>(c, s, mp, params, dpos, dvel, o, stream, err);
}
