// k_episode_hp instantiations (fgx_hp.h): HoleReacher, 5 links, 5 basis functions, every MP kind and
// controller, one group per workgroup (small batches: spread over the CUs) or four (one per SIMD).
#include "fgx_hp.h"

namespace fgx {

template <int MP, int CTRL, int G, bool INFO>
static int launch_hp(const DevCfg& c, const DevState& s, const float* params, const Outputs& o, hipStream_t stream,
                     std::string& err) {
  if (c.stride != Traj<MP, 1, 5>::KS) {
    err = "k_episode_hp: basis table stride does not match the compiled layout";
    return -1;
  }
  const size_t lds = hp_lds_bytes(5, G);
  if (raise_lds_limit((const void*)k_episode_hp<MP, CTRL, 5, 5, G, INFO>, lds) != hipSuccess) {
    err = "k_episode_hp: cannot raise the dynamic LDS limit";
    return -2;
  }
  const int64_t per = 64 * G;
  hipLaunchKernelGGL((k_episode_hp<MP, CTRL, 5, 5, G, INFO>), dim3((unsigned)((c.N + per - 1) / per)), dim3(192 * G), lds,
                     stream, c, s, params, o);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) { err = std::string("k_episode_hp launch: ") + hipGetErrorString(e); return -2; }
  hipLaunchKernelGGL((k_hp_finish<5, CTRL != CTRL_PD>), dim3((unsigned)((c.N + 255) / 256)), dim3(256), 0, stream, c, s,
                     o);
  e = hipGetLastError();
  if (e != hipSuccess) { err = std::string("k_hp_finish launch: ") + hipGetErrorString(e); return -2; }
  return 0;
}

template <int MP, int G>
static int launch_hp_ctrl(const DevCfg& c, const DevState& s, const float* params, const Outputs& o, hipStream_t stream,
                          std::string& err) {
  // per-step arrays: the INFO instantiation
  const bool info = o.positions || o.step_actions || o.step_obs || o.step_rewards || o.is_collided || o.end_effector;
#ifdef FGX_HP_ONLY_CFG3   // diagnostics builds (tools/unit_variant.py): config 3's instantiation only
  if (MP == MP_PRODMP && c.ctrl == CTRL_PD && !info) return launch_hp<MP_PRODMP, CTRL_PD, G, false>(c, s, params, o, stream, err);
  err = "FGX_HP_ONLY_CFG3 build";
  return -1;
#endif
  switch (c.ctrl) {
    case CTRL_PD: return info ? launch_hp<MP, CTRL_PD, G, true>(c, s, params, o, stream, err)
                              : launch_hp<MP, CTRL_PD, G, false>(c, s, params, o, stream, err);
    case CTRL_VEL: return info ? launch_hp<MP, CTRL_VEL, G, true>(c, s, params, o, stream, err)
                               : launch_hp<MP, CTRL_VEL, G, false>(c, s, params, o, stream, err);
    case CTRL_POS: return info ? launch_hp<MP, CTRL_POS, G, true>(c, s, params, o, stream, err)
                               : launch_hp<MP, CTRL_POS, G, false>(c, s, params, o, stream, err);
  }
  err = "bad ctrl_kind";
  return -1;
}

template <int G>
static int launch_hp_mp(const DevCfg& c, const DevState& s, int mp, const float* params, const Outputs& o,
                        hipStream_t stream, std::string& err) {
  switch (mp) {
    case MP_PROMP: return launch_hp_ctrl<MP_PROMP, G>(c, s, params, o, stream, err);
    case MP_DMP: return launch_hp_ctrl<MP_DMP, G>(c, s, params, o, stream, err);
    case MP_PRODMP: return launch_hp_ctrl<MP_PRODMP, G>(c, s, params, o, stream, err);
  }
  err = "k_episode_hp: bad mp kind";
  return -1;
}

// envs of one full round of this kernel with G = 4: one workgroup of 256 envs per CU
static int64_t hp_round_envs() {
  static const int64_t r = [] {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
    return (int64_t)cus * 256;
  }();
  return r;
}

}  // namespace fgx

// four groups per workgroup (one per SIMD, one workgroup per CU) once the batch fills every CU that
// way; one group per workgroup below (FGX_HP_G=1 / 4 forces)
int fgx_launch_episode_hp(const fgx::DevCfg& c, const fgx::DevState& s, int mp, const float* params,
                          const fgx::Outputs& o, hipStream_t stream, std::string& err) {
  if (c.nl != 5 || c.nb != 5) {
    err = "k_episode_hp: 5 links and 5 basis functions only";
    return -4;
  }
  int G = (c.N >= fgx::hp_round_envs()) ? 4 : 1;
  if (const char* v = std::getenv("FGX_HP_G")) G = std::atoi(v) == 4 ? 4 : 1;
  return G == 4 ? fgx::launch_hp_mp<4>(c, s, mp, params, o, stream, err)
                : fgx::launch_hp_mp<1>(c, s, mp, params, o, stream, err);
}
