// fgx_dispatch.h — template dispatch of the episode kernel.  One translation unit per env kind
// and basis specialisation (fgx_ep_<env>.hip: NB = 5, the registered configs; fgx_ep_<env>_gen.hip:
// NB = 0, the generic runtime basis count), so that the build compiles them in parallel.
#pragma once
#include <cstdlib>
#include <cstring>
#include <string>

#include "fgx_jp.h"

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

// k_episode_jp (fgx_jp.h) covers SimpleReacher + PD over the shared basis tables with static
// replanning schedules, max_episode_steps <= 200 and no per-step info.  FGX_EPISODE_KERNEL=classic
// forces k_episode, =jp forces k_episode_jp wherever it applies (A/B benchmarks and the
// kernel-equivalence tests).
inline bool jp_enabled() {
  const char* v = std::getenv("FGX_EPISODE_KERNEL");
  return !(v && std::strcmp(v, "classic") == 0);
}

// Where k_episode_jp beats k_episode (both kernels timed over envs per GPU x MP kind x links,
// profiles/r01_jp_vs_classic.jsonl).  k_episode holds one wave (64 envs) per SIMD, so it runs in
// ceil(N / (64 x 4 x CUs)) rounds of a fixed ~75-93 us; k_episode_jp's time grows ~linearly
// (5 links: ~1.65 us per 1k envs).  Hence for 5 links: jp while k_episode's one round is at most 3/4
// full or its last round at most half full, and DMP at every size (its per-joint Euler plan splits
// cheaply).  Two links (2 waves per 64 envs) and short replanning segments (per-chunk exchange
// overhead) stay on k_episode except DMP up to one full round.
inline bool jp_preferred(const DevCfg& c, int mp) {
  const char* v = std::getenv("FGX_EPISODE_KERNEL");
  if (v && std::strcmp(v, "jp") == 0) return true;
  if (c.replan) return false;
  static const int64_t round_envs = [] {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
    return (int64_t)cus * 4 * 64;
  }();
  const int64_t tail = c.N % round_envs;
  if (c.nl == 5)
    return mp == MP_DMP || 4 * c.N <= 3 * round_envs || (c.N > round_envs && tail != 0 && 2 * tail <= round_envs);
  return mp == MP_DMP && c.N <= round_envs;
}

template <int MP, int NL, int NB>
static int launch_jp(const DevCfg& c, const DevState& s, const float* params, const Outputs& o, hipStream_t stream,
                     std::string& err) {
  const size_t lj = jp_lds_bytes<NL>(c.rows, c.stride);
  if (lj > 160 * 1024) {
    err = "k_episode_jp: basis table too large for LDS";
    return -4;
  }
  if (lj > 64 * 1024 &&
      hipFuncSetAttribute((const void*)k_episode_jp<MP, NL, NB>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)lj) != hipSuccess) {
    err = "k_episode_jp: cannot raise the dynamic LDS limit";
    return -2;
  }
  hipLaunchKernelGGL((k_episode_jp<MP, NL, NB>), dim3((unsigned)((c.N + 63) / 64)), dim3(NL * 64), lj, stream, c, s,
                     params, o);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) { err = std::string("k_episode_jp launch: ") + hipGetErrorString(e); return -2; }
  return 0;
}

template <int ENV, int MP, int CTRL, int NL, int NB>
static int launch_episode_nl(const DevCfg& c, const DevState& s, const float* params, const float* dpos,
                             const float* dvel, const Outputs& o, hipStream_t stream, std::string& err) {
  const int threads = 256;
  const int blocks = (int)((c.N + threads - 1) / threads);
  const size_t lds = (MP == MP_GIVEN) ? 0 : (size_t)c.rows * c.stride * sizeof(float);
  const bool log = o.positions || o.step_actions || o.step_obs || o.step_rewards || o.is_collided ||
                   o.end_effector || o.reward_dist;
  if constexpr (MP != MP_GIVEN && NB != 0) {
    if (c.stride != Traj<MP, 1, NB>::KS) {
      err = "basis table stride does not match the compiled layout";
      return -1;
    }
  }
  if constexpr (ENV == ENV_SIMPLE && MP != MP_GIVEN && CTRL == CTRL_PD) {
    if (!log && !c.sched_state && c.T <= 256 && c.max_steps <= 200 && !s.plan_len && !c.learn_tau && !c.learn_delay &&
        jp_enabled() && jp_preferred(c, MP))
      return launch_jp<MP, NL, NB>(c, s, params, o, stream, err);
  }
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
