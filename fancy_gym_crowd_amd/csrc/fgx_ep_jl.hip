// k_episode_jl instantiations (fgx_jl.h): SimpleReacher + PD, every MP kind, 2 / 5 links, the
// registered basis count (NB = 5) and the generic one (NB = 0).  A translation unit of its own so
// that the build compiles it in parallel with the k_episode units.
#include "fgx_dispatch.h"
#include "fgx_jl.h"

#include <algorithm>
#include <cstdlib>

namespace {
int jl_cus() {
  static const int n = [] {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
    return cus;
  }();
  return n;
}

template <int MP, int NL, int NB, int HLP = 0>
int launch_jl(const fgx::DevCfg& c, const fgx::DevState& s, const float* params, const fgx::Outputs& o,
              hipStream_t stream, std::string& err) {
  using S = fgx::JlShape<NL, HLP>;
  if constexpr (NB != 0) {
    if (c.stride != fgx::Traj<MP, 1, NB>::KS) {
      err = "basis table stride does not match the compiled layout";
      return -1;
    }
  }
  int gw = S::G;   // (fewer envs per wave measured slower at every N: profiles/r02_jl_scan.jsonl)
  if (const char* v = std::getenv("FGX_JL_GW")) gw = std::max(1, std::min(S::G, std::atoi(v)));   // experiments
  const int64_t per_block = (int64_t)S::WAVES * gw;
  const unsigned blocks = (unsigned)((c.N + per_block - 1) / per_block);
  // the reset wave (fgx_jl.h) while every workgroup has a CU of its own (the 8-GPU shard: 8192 envs
  // 23.8-24.0 -> 21.9-22.2 us, config 2 22.4 -> 20.1 us); past that its fifth wave costs a workgroup
  // slot per CU (32768 envs 45.2 -> 48.2 us, profiles/r06_jl_resetwave_ab.log).  FGX_JL_RW=0 / 1: A/B
  int rw = (!HLP && blocks <= (unsigned)jl_cus()) ? 1 : 0;
  if (const char* v = std::getenv("FGX_JL_RW")) rw = (!HLP && v[0] == '1') ? 1 : 0;
  hipLaunchKernelGGL((fgx::k_episode_jl<MP, NL, NB, HLP>), dim3(blocks), dim3(S::THREADS + 64 * rw), S::lds_bytes(),
                     stream, c, s, params, o, gw, rw);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) { err = std::string("k_episode_jl launch: ") + hipGetErrorString(e); return -2; }
  return 0;
}

// the helper form (fgx_jl.h, HLP 1 / 2): ProMP on the column table, measured slower than the plain
// form and compiled only into diagnostics builds (-DFGX_JL_HELPER_FORM,
// _build.build_variant); FGX_JL_HELPER=1 / 2 selects it there and is refused by the release build
inline int jl_helper(const fgx::DevCfg& c) {
  if (const char* v = std::getenv("FGX_JL_HELPER")) return v[0] == '1' ? 1 : v[0] == '2' ? 2 : 0;
  (void)c;
  return 0;
}

template <int MP, int NB>
int launch_jl_nl(const fgx::DevCfg& c, const fgx::DevState& s, const float* params, const fgx::Outputs& o,
                 hipStream_t stream, std::string& err) {
  if (const int h = jl_helper(c)) {
#ifdef FGX_JL_HELPER_FORM
    if constexpr (MP == fgx::MP_PROMP && NB == 5) {
      if (h == 1) {
        if (c.nl == 2) return launch_jl<MP, 2, NB, 1>(c, s, params, o, stream, err);
        if (c.nl == 5) return launch_jl<MP, 5, NB, 1>(c, s, params, o, stream, err);
      } else {
        if (c.nl == 2) return launch_jl<MP, 2, NB, 2>(c, s, params, o, stream, err);
        if (c.nl == 5) return launch_jl<MP, 5, NB, 2>(c, s, params, o, stream, err);
      }
    }
#else
    (void)h;
    err = "k_episode_jl: FGX_JL_HELPER asks for the helper form, which this build does not contain "
          "(a diagnostics build with -DFGX_JL_HELPER_FORM does)";
    return -4;
#endif
  }
  if (c.nl == 2) return launch_jl<MP, 2, NB>(c, s, params, o, stream, err);
  if (c.nl == 5) return launch_jl<MP, 5, NB>(c, s, params, o, stream, err);
  err = "k_episode_jl: n_links not instantiated (supported: 2, 5)";
  return -4;
}

template <int NB>
int launch_jl_mp(const fgx::DevCfg& c, const fgx::DevState& s, int mp, const float* params, const fgx::Outputs& o,
                 hipStream_t stream, std::string& err) {
  switch (mp) {
    case fgx::MP_PROMP: return launch_jl_nl<fgx::MP_PROMP, NB>(c, s, params, o, stream, err);
    case fgx::MP_DMP: return launch_jl_nl<fgx::MP_DMP, NB>(c, s, params, o, stream, err);
    case fgx::MP_PRODMP: return launch_jl_nl<fgx::MP_PRODMP, NB>(c, s, params, o, stream, err);
  }
  err = "k_episode_jl: bad mp kind";
  return -1;
}
}  // namespace

int fgx_launch_episode_jl(const fgx::DevCfg& c, const fgx::DevState& s, int mp, int nbs, const float* params,
                          const fgx::Outputs& o, hipStream_t stream, std::string& err) {
  if (nbs == 5) return launch_jl_mp<5>(c, s, mp, params, o, stream, err);
  if (nbs == 0) return launch_jl_mp<0>(c, s, mp, params, o, stream, err);
  err = "k_episode_jl: basis count not instantiated";
  return -4;
}
