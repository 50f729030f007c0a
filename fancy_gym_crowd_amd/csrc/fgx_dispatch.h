// fgx_dispatch.h — template dispatch of the episode kernel.  One translation unit per env kind
// and basis specialisation (fgx_ep_<env>.hip: NB = 5, the registered configs; fgx_ep_<env>_gen.hip:
// NB = 0, the generic runtime basis count), so that the build compiles them in parallel.
#pragma once
#include <cstdlib>
#include <cstring>
#include <string>

#include "fgx_ws.h"
#include "fgx_v2.h"

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
// k_episode_jl instantiations (fgx_ep_jl.hip): nbs = the compiled basis count (5, or 0 = generic)
int fgx_launch_episode_jl(const fgx::DevCfg& c, const fgx::DevState& s, int mp, int nbs, const float* params,
                          const fgx::Outputs& o, hipStream_t stream, std::string& err);

namespace fgx {
// Link counts other than the registered 2 and 5 (include/fgx.h: n_links 1..8; base_reacher.py:17-39
// takes any count and bb_env_constructor forwards env kwargs, envs/registry.py:280-281): one
// translation unit per count (fgx_ep_nl<n>.hip -> fgx_ep_nl.h) with the logging k_episode for every
// env kind / MP kind / controller plus the reset, step-based, trajectory and learned-phase kernels.
struct NlOps {
  int (*episode)(const DevCfg& c, const DevState& s, int mp, const float* params, const float* dpos, const float* dvel,
                 const Outputs& o, hipStream_t stream, std::string& err);
  int (*reset)(const DevCfg& c, const DevState& s, const uint64_t* seeds, const uint8_t* mask, int rs_mode, float* obs,
               hipStream_t stream, std::string& err);
  int (*step_raw)(const DevCfg& c, const DevState& s, const float* act, float* obs, double* rew, uint8_t* term,
                  uint8_t* trunc, float* final_obs, int autoreset, size_t lds, hipStream_t stream, std::string& err);
  int (*traj)(const DevCfg& c, const DevState& s, const float* params, float* dpos, float* dvel, hipStream_t stream,
              std::string& err);
  int (*traj_env)(const DevCfg& c, const DevState& s, const float* params, float* env_tab, float* dpos, float* dvel,
                  int32_t* plan_len, float* info_pos, float* info_vel, hipStream_t stream, std::string& err);
};
}  // namespace fgx
const fgx::NlOps* fgx_nl_ops_1();
const fgx::NlOps* fgx_nl_ops_3();
const fgx::NlOps* fgx_nl_ops_4();
const fgx::NlOps* fgx_nl_ops_6();
const fgx::NlOps* fgx_nl_ops_7();
const fgx::NlOps* fgx_nl_ops_8();

namespace fgx {

// Episode kernels: k_episode (fgx_kernels.h, one env per lane, every case), k_episode_jl (fgx_jl.h,
// one lane per env x joint), k_episode_jp (fgx_jp.h, one wave per joint) and k_episode_ws
// (fgx_ws.h, trajectory-producer / dynamics-consumer wave pairs).  The last three serve
// SimpleReacher + PD over the shared basis tables with static replanning schedules,
// max_episode_steps <= 200 and no per-step info, bit-identically to k_episode (tests/test_gpu_jl.py,
// test_gpu_jp.py, test_gpu_ws.py).  Which one runs follows the measured table
// profiles/r02_kernel_scan_all.jsonl (every kernel forced over envs per GPU x MP kind x links on one
// MI355X, tools/scan_all.sh):
//  * k_episode holds one wave (64 envs) per SIMD: a near-fixed ~73-105 us (5 links) up to one full
//    round of 65536 envs, where its 5 independent joint chains per lane keep the lone wave busy;
//  * k_episode_jl puts 5x the lanes to work below that (8192 envs: 26 us vs 41 us k_episode_jp and
//    61 us k_episode, ProMP 5 links) and wins at every size for 2 links (the 2-link k_episode is a
//    short-chain lone wave too), replanning included;
//  * past one round whose last round is at most half full (5 links), k_episode_jl again (98304 envs:
//    112 us vs 127 us k_episode, profiles/r02_jl_scan.jsonl; it took k_episode_jp's place there once
//    its exchange rows stopped conflicting on LDS banks).
// k_episode_jp and k_episode_ws stay selectable: FGX_EPISODE_KERNEL=classic|jp|ws|jl forces a kernel
// wherever it applies (A/B benchmarks, tests).
enum : int { EK_CLASSIC = 0, EK_JP = 1, EK_WS = 2, EK_JL = 3, EK_CLASSIC_W2 = 4, EK_PAIR = 5, EK_V2 = 6, EK_V2H = 7 };

inline int64_t round_envs() {   // envs of one k_episode round: one 64-lane wave per SIMD
  static const int64_t r = [] {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
    return (int64_t)cus * 4 * 64;
  }();
  return r;
}

// k_episode or k_episode_w2: 5-link SimpleReacher without per-step info past one k_episode round
// (two resident waves per SIMD, profiles/r02_w2_ab.jsonl); FGX_EPISODE_KERNEL=classic keeps k_episode
inline bool w2_applies(const DevCfg& c, bool log) { return c.env == ENV_SIMPLE && c.nl == 5 && !log; }
// k_episode_pair: 5-link HoleReacher without per-step info (two lanes per env, fgx_kernels.h) while
// its 2N lanes fit one wave per SIMD (N <= 32768 on 256 CUs): each lane issues 15% fewer VALU
// instructions than k_episode's (16384 / 32768 envs: 487 / 493 vs 517 / 525 us).  Past that the
// pairs' second wave per SIMD does not pay for the duplicated plan / controller / dynamics work
// (65536: 648 vs 530 us; profiles/r03_pair_scan.jsonl).  FGX_EPISODE_KERNEL=classic / =pair force.
inline bool pair_applies(const DevCfg& c, bool log) { return c.env == ENV_HOLE && c.nl == 5 && !log; }
// k_episode_v2h (fgx_kernels.h): the per-step info rows of the direct envs (HoleReacher,
// ViaPointReacher) stored by a partner wave per SIMD; whole 256-env workgroups only.  FGX_V2=0 (or
// FGX_EPISODE_KERNEL=classic) keeps the logging k_episode (A/B, tests)
inline bool v2h_applies(const DevCfg& c, bool log) {
  if (const char* v = std::getenv("FGX_V2"))
    if (std::strcmp(v, "0") == 0) return false;
  if (const char* v = std::getenv("FGX_EPISODE_KERNEL"))
    if (std::strcmp(v, "classic") == 0) return false;
  return log && c.env != ENV_SIMPLE && c.N % 256 == 0 && (c.nl == 2 || c.nl == 5) &&
         v2h_lds_bytes(c.mp, c.rows, c.stride, c.nl, c.full_dim) <= 160 * 1024;
}

inline int classic_choice(const DevCfg& c, bool log) {
  if (v2h_applies(c, log)) return EK_V2H;
  if (pair_applies(c, log)) {
    if (const char* v = std::getenv("FGX_EPISODE_KERNEL")) {
      if (std::strcmp(v, "classic") == 0) return EK_CLASSIC;
      if (std::strcmp(v, "pair") == 0) return EK_PAIR;
    }
    return 2 * c.N <= round_envs() ? EK_PAIR : EK_CLASSIC;
  }
  if (!w2_applies(c, log)) return EK_CLASSIC;
  if (const char* v = std::getenv("FGX_EPISODE_KERNEL")) {
    if (std::strcmp(v, "classic") == 0) return EK_CLASSIC;
    if (std::strcmp(v, "w2") == 0) return EK_CLASSIC_W2;
  }
  return c.N > round_envs() ? EK_CLASSIC_W2 : EK_CLASSIC;
}

// k_episode_v2 (fgx_v2.h): the per-step info arrays of SimpleReacher + PD (info_level >= 1, the
// reference's verbose-2 default) with the observation's trigonometry on a second wave of each SIMD;
// FGX_V2=0 (or FGX_EPISODE_KERNEL=classic) keeps the logging k_episode (A/B, tests)
inline bool v2_applies(const DevCfg& c, int mp, bool log, bool per_env_plans) {
  if (const char* v = std::getenv("FGX_V2"))
    if (std::strcmp(v, "0") == 0) return false;
  if (const char* v = std::getenv("FGX_EPISODE_KERNEL"))   // a forced kernel wins
    if (std::strcmp(v, "classic") == 0) return false;
  return log && c.env == ENV_SIMPLE && c.ctrl == CTRL_PD && mp != MP_GIVEN && mp != MP_NONE && !per_env_plans &&
         !c.learn_tau && !c.learn_delay && !c.sched_state && c.valid_flags == 0 && c.T <= 256 && c.max_steps <= 200 &&
         (c.nl == 2 || c.nl == 5) && v2_lds_bytes(c.rows, c.stride, c.nl) <= 160 * 1024;
}

inline int episode_kernel_choice(const DevCfg& c, int mp, bool log, bool per_env_plans) {
  if (v2_applies(c, mp, log, per_env_plans)) return EK_V2;
  const bool eligible = c.env == ENV_SIMPLE && mp != MP_GIVEN && mp != MP_NONE && c.ctrl == CTRL_PD && !log &&
                        !c.sched_state && c.T <= 256 && c.max_steps <= 200 && !per_env_plans && !c.learn_tau &&
                        !c.learn_delay && (c.nl == 2 || c.nl == 5);
  if (!eligible) return classic_choice(c, log);
  if (const char* v = std::getenv("FGX_EPISODE_KERNEL")) {
    if (std::strcmp(v, "classic") == 0 || std::strcmp(v, "w2") == 0) return classic_choice(c, log);
    if (std::strcmp(v, "jp") == 0) return EK_JP;
    if (std::strcmp(v, "ws") == 0) return EK_WS;
    if (std::strcmp(v, "jl") == 0) return EK_JL;
  }
  const int64_t R = round_envs(), tail = c.N % R;
  if (c.nl == 2) return EK_JL;
  if (4 * c.N <= 3 * R) return EK_JL;
  if (!c.replan && c.N > R && tail != 0 && 2 * tail <= R) return EK_JL;
  return classic_choice(c, log);
}

template <int MP, int NL, int NB>
static int launch_jp(const DevCfg& c, const DevState& s, const float* params, const Outputs& o, hipStream_t stream,
                     std::string& err) {
  const size_t lj = jp_lds_bytes<NL>(c.rows, c.stride);
  if (lj > 160 * 1024) {
    err = "k_episode_jp: basis table too large for LDS";
    return -4;
  }
  if (raise_lds_limit((const void*)k_episode_jp<MP, NL, NB>, lj) != hipSuccess) {
    err = "k_episode_jp: cannot raise the dynamic LDS limit";
    return -2;
  }
  hipLaunchKernelGGL((k_episode_jp<MP, NL, NB>), dim3((unsigned)((c.N + 63) / 64)), dim3(NL * 64), lj, stream, c, s,
                     params, o);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) { err = std::string("k_episode_jp launch: ") + hipGetErrorString(e); return -2; }
  return 0;
}

template <int MP, int NL, int NB>
static int launch_ws(const DevCfg& c, const DevState& s, const float* params, const Outputs& o, hipStream_t stream,
                     std::string& err) {
  const size_t lw = ws_lds_bytes<NL>(c.rows, c.stride);
  if (lw > 160 * 1024) {
    err = "k_episode_ws: basis table too large for LDS";
    return -4;
  }
  if (raise_lds_limit((const void*)k_episode_ws<MP, NL, NB>, lw) != hipSuccess) {
    err = "k_episode_ws: cannot raise the dynamic LDS limit";
    return -2;
  }
  const int64_t per_block = 64 * kWsPairs;
  hipLaunchKernelGGL((k_episode_ws<MP, NL, NB>), dim3((unsigned)((c.N + per_block - 1) / per_block)), dim3(512), lw,
                     stream, c, s, params, o);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) { err = std::string("k_episode_ws launch: ") + hipGetErrorString(e); return -2; }
  return 0;
}

// LOG_ONLY (n_links outside {2, 5}, fgx_ep_nl.h): only the logging k_episode is instantiated; it
// serves every info level (no per-step array given: nothing is staged or stored) and the validity
// checks, so each further link count costs one kernel per (env, MP, controller), not a family.
template <int ENV, int MP, int CTRL, int NL, int NB, bool LOG_ONLY = false>
static int launch_episode_nl(const DevCfg& c, const DevState& s, const float* params, const float* dpos,
                             const float* dvel, const Outputs& o, hipStream_t stream, std::string& err) {
  const int threads = 256;
  const int blocks = (int)((c.N + threads - 1) / threads);
  const size_t lds = (MP == MP_GIVEN) ? 0 : (size_t)c.rows * c.stride * sizeof(float);
  // the logging instantiation also runs the trajectory-validity checks (c.valid_flags)
  const bool log = LOG_ONLY || o.positions || o.step_actions || o.step_obs || o.step_rewards || o.is_collided ||
                   o.end_effector || o.reward_dist || c.valid_flags != 0;
  if constexpr (MP != MP_GIVEN && NB != 0) {
    if (c.stride != Traj<MP, 1, NB>::KS) {
      err = "basis table stride does not match the compiled layout";
      return -1;
    }
  }
  if constexpr (!LOG_ONLY && ENV == ENV_SIMPLE && MP != MP_GIVEN && CTRL == CTRL_PD) {
    const int k = episode_kernel_choice(c, MP, log, s.plan_len != nullptr);
    if (k == EK_V2) {
      const size_t lv = v2_lds_bytes(c.rows, c.stride, NL);
      if (raise_lds_limit((const void*)k_episode_v2<MP, NL, NB>, lv) != hipSuccess) {
        err = "k_episode_v2: cannot raise the dynamic LDS limit";
        return -2;
      }
      hipLaunchKernelGGL((k_episode_v2<MP, NL, NB>), dim3((unsigned)((c.N + 64 * kV2Pairs - 1) / (64 * kV2Pairs))),
                         dim3(kV2Threads), lv, stream, c, s, params, o);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) { err = std::string("k_episode_v2 launch: ") + hipGetErrorString(e); return -2; }
      return 0;
    }
    if (k == EK_JP) return launch_jp<MP, NL, NB>(c, s, params, o, stream, err);
    if (k == EK_WS) return launch_ws<MP, NL, NB>(c, s, params, o, stream, err);
    if (k == EK_JL) return fgx_launch_episode_jl(c, s, MP, NB, params, o, stream, err);
  }
  if constexpr (!LOG_ONLY && ENV == ENV_HOLE && NL == 5) {
    if (classic_choice(c, log) == EK_PAIR) {
      const int pblocks = (int)((2 * c.N + threads - 1) / threads);
      hipLaunchKernelGGL((k_episode_pair<ENV, MP, CTRL, NL, NB>), dim3(pblocks), dim3(threads), lds, stream, c, s,
                         params, dpos, dvel, o);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) { err = std::string("k_episode_pair launch: ") + hipGetErrorString(e); return -2; }
      return 0;
    }
  }
  if constexpr (!LOG_ONLY && ENV == ENV_SIMPLE && NL == 5) {
    if (classic_choice(c, log) == EK_CLASSIC_W2 &&
        (MP == MP_GIVEN || CTRL != CTRL_PD || episode_kernel_choice(c, MP, log, s.plan_len != nullptr) == EK_CLASSIC_W2)) {
      hipLaunchKernelGGL((k_episode_w2<ENV, MP, CTRL, NL, NB, false>), dim3(blocks), dim3(threads), lds, stream, c,
                         s, params, dpos, dvel, o);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) { err = std::string("k_episode_w2 launch: ") + hipGetErrorString(e); return -2; }
      return 0;
    }
  }
  if constexpr (!LOG_ONLY && ENV != ENV_SIMPLE) {
    if (v2h_applies(c, log)) {
      const size_t lh = v2h_lds_bytes(MP, c.rows, c.stride, NL, c.full_dim);
      if (raise_lds_limit((const void*)k_episode_v2h<ENV, MP, CTRL, NL, NB>, lh) != hipSuccess) {
        err = "k_episode_v2h: cannot raise the dynamic LDS limit";
        return -2;
      }
      hipLaunchKernelGGL((k_episode_v2h<ENV, MP, CTRL, NL, NB>), dim3((unsigned)(c.N / 256)), dim3(512), lh, stream,
                         c, s, params, dpos, dvel, o);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) { err = std::string("k_episode_v2h launch: ") + hipGetErrorString(e); return -2; }
      return 0;
    }
  }
  if (log) {
    if (ENV == ENV_SIMPLE && o.step_obs && !o.qlog) {
      err = "SimpleReacher per-step observations need the qlog scratch (fgx_step attaches it)";
      return -1;
    }
    // + the four waves' info staging regions (InfoStage, fgx_device.h)
    const size_t ll = stage_tab_offset(lds / sizeof(float)) + (threads / 64) * stage_wave_bytes(NL, c.full_dim);
    if (raise_lds_limit((const void*)k_episode<ENV, MP, CTRL, NL, NB, true>, ll) != hipSuccess) {
      err = "k_episode (info rows): cannot raise the dynamic LDS limit";
      return -2;
    }
    hipLaunchKernelGGL((k_episode<ENV, MP, CTRL, NL, NB, true>), dim3(blocks), dim3(threads), ll, stream, c, s,
                       params, dpos, dvel, o);
    if constexpr (ENV == ENV_SIMPLE) {
      if (o.qlog && o.step_obs) {   // the observation trigonometry of the logged rows (k_info_obs)
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) { err = std::string("k_episode launch: ") + hipGetErrorString(e); return -2; }
        hipLaunchKernelGGL((k_info_obs<NL>), dim3(blocks, c.T), dim3(threads), 0, stream, c, o);
      }
    }
  }
  else if constexpr (!LOG_ONLY)
    hipLaunchKernelGGL((k_episode<ENV, MP, CTRL, NL, NB, false>), dim3(blocks), dim3(threads), lds, stream, c, s,
                       params, dpos, dvel, o);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) { err = std::string("k_episode launch: ") + hipGetErrorString(e); return -2; }
  return 0;
}

// NLV > 0: that link count only (the per-link-count units of fgx_ep_nl.h, logging kernel only);
// NLV = 0: the registered 2 and 5
template <int ENV, int MP, int CTRL, int NB, int NLV = 0>
static int launch_episode_ctrl(const DevCfg& c, const DevState& s, const float* params, const float* dpos,
                               const float* dvel, const Outputs& o, hipStream_t stream, std::string& err) {
  if constexpr (NLV > 0) {
    if (c.nl == NLV) return launch_episode_nl<ENV, MP, CTRL, NLV, NB, true>(c, s, params, dpos, dvel, o, stream, err);
  } else {
    if (c.nl == 2) return launch_episode_nl<ENV, MP, CTRL, 2, NB>(c, s, params, dpos, dvel, o, stream, err);
    if (c.nl == 5) return launch_episode_nl<ENV, MP, CTRL, 5, NB>(c, s, params, dpos, dvel, o, stream, err);
  }
  err = "n_links not instantiated in this unit";
  return -4;
}

template <int ENV, int MP, int NB, int NLV = 0>
static int launch_episode_mp(const DevCfg& c, const DevState& s, const float* params, const float* dpos,
                             const float* dvel, const Outputs& o, hipStream_t stream, std::string& err) {
  switch (c.ctrl) {
    case CTRL_PD: return launch_episode_ctrl<ENV, MP, CTRL_PD, NB, NLV>(c, s, params, dpos, dvel, o, stream, err);
    case CTRL_VEL: return launch_episode_ctrl<ENV, MP, CTRL_VEL, NB, NLV>(c, s, params, dpos, dvel, o, stream, err);
    case CTRL_POS: return launch_episode_ctrl<ENV, MP, CTRL_POS, NB, NLV>(c, s, params, dpos, dvel, o, stream, err);
  }
  err = "bad ctrl_kind";
  return -1;
}

// NB = 5: every MP kind and the caller-given trajectory; NB = 0: the MP kinds with c.nb != 5 (and,
// in the per-link-count units NLV > 0, every basis count and the caller-given trajectory)
template <int ENV, int NB, int NLV = 0>
static int launch_episode_env(const DevCfg& c, const DevState& s, int mp, const float* params, const float* dpos,
                              const float* dvel, const Outputs& o, hipStream_t stream, std::string& err) {
  switch (mp) {
    case MP_PROMP: return launch_episode_mp<ENV, MP_PROMP, NB, NLV>(c, s, params, dpos, dvel, o, stream, err);
    case MP_DMP: return launch_episode_mp<ENV, MP_DMP, NB, NLV>(c, s, params, dpos, dvel, o, stream, err);
    case MP_PRODMP: return launch_episode_mp<ENV, MP_PRODMP, NB, NLV>(c, s, params, dpos, dvel, o, stream, err);
    case MP_GIVEN:
      // (if constexpr: the NB = 0 units of 2 / 5 links do not compile a second caller-given family)
      if constexpr (NB == 5 || NLV > 0)
        return launch_episode_mp<ENV, MP_GIVEN, NB, NLV>(c, s, params, dpos, dvel, o, stream, err);
      break;
  }
  err = "bad mp kind";
  return -1;
}

}  // namespace fgx
