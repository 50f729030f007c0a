// fgx_aux.h — trajectory-only launches and state (de)serialisation kernels.
#pragma once
#include <string>

#include "fgx_kernels.h"
#include "fgx_mfma.h"
#include "fgx_traj_run.h"

namespace fgx {

// SoA [k][N] <-> row-major [N, k]
__global__ void k_get_state(DevCfg c, DevState s, double* q, double* qd, double* goal, double* hole, int32_t* steps) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= c.N) return;
  const int64_t N = c.N;
  for (int k = 0; k < c.nl; ++k) {
    if (q) q[e * c.nl + k] = s.q[k * N + e];
    if (qd) qd[e * c.nl + k] = s.qd[k * N + e];
  }
  if (goal) { goal[2 * e] = s.goal[e]; goal[2 * e + 1] = s.goal[N + e]; }
  if (hole) for (int k = 0; k < 3; ++k) hole[3 * e + k] = s.hole[k * N + e];
  if (steps) steps[e] = s.steps[e];
}

__global__ void k_set_state(DevCfg c, DevState s, const double* q, const double* qd, const double* goal,
                            const double* hole, const int32_t* steps) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= c.N) return;
  const int64_t N = c.N;
  for (int k = 0; k < c.nl; ++k) {
    if (q) s.q[k * N + e] = q[e * c.nl + k];
    if (qd) s.qd[k * N + e] = qd[e * c.nl + k];
  }
  if (goal) { s.goal[e] = goal[2 * e]; s.goal[N + e] = goal[2 * e + 1]; }
  if (hole) for (int k = 0; k < 3; ++k) s.hole[k * N + e] = hole[3 * e + k];
  if (steps) s.steps[e] = steps[e];
}

inline int launch_trajectory(const DevCfg& c, const DevState& s, const float* params, float* dpos, float* dvel,
                             hipStream_t stream, std::string& err) {
  const int threads = 256;
  const int blocks = (int)((c.N + threads - 1) / threads);
  if (c.mp == MP_NONE) { err = "step-based handle has no trajectory generator"; return -1; }
  if (c.mp == MP_PROMP || c.mp == MP_PRODMP) {
    if (launch_traj_mfma(c, s, params, dpos, dvel, stream) == 0) return 0;
  }
#define LAUNCH(MPV, NLV, NBV) \
  hipLaunchKernelGGL((k_traj_valu<MPV, NLV, NBV>), dim3(blocks), dim3(threads), 0, stream, c, s, params, dpos, dvel)
#define X(NL)                                                                                 \
  if (c.nl == NL) {                                                                           \
    const int rr = launch_traj_run<NL>(c, s, params, dpos, dvel, stream);                      \
    if (rr == 0) return 0;                                                                    \
    if (rr == 2) { err = hipGetErrorString(hipGetLastError()); return -2; }                   \
    const bool nb5 = c.nb == 5;                                                               \
    if (c.mp == MP_PROMP) { if (nb5) LAUNCH(MP_PROMP, NL, 5); else LAUNCH(MP_PROMP, NL, 0); } \
    else if (c.mp == MP_DMP) { if (nb5) LAUNCH(MP_DMP, NL, 5); else LAUNCH(MP_DMP, NL, 0); } \
    else { if (nb5) LAUNCH(MP_PRODMP, NL, 5); else LAUNCH(MP_PRODMP, NL, 0); }              \
    hipError_t e = hipGetLastError();                                                         \
    if (e != hipSuccess) { err = hipGetErrorString(e); return -2; }                           \
    return 0;                                                                                 \
  }
  X(2) X(5)
#undef X
#undef LAUNCH
  err = "n_links not instantiated (supported: 2, 5)";
  return -4;
}

}  // namespace fgx

inline int fgx_transpose_state(const fgx::DevCfg& c, const fgx::DevState& s, double* q, double* qd, double* goal,
                               double* hole, int32_t* steps, hipStream_t stream, std::string& err) {
  const int threads = 256;
  const int blocks = (int)((c.N + threads - 1) / threads);
  hipLaunchKernelGGL(fgx::k_get_state, dim3(blocks), dim3(threads), 0, stream, c, s, q, qd, goal, hole, steps);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) { err = hipGetErrorString(e); return -2; }
  return 0;
}

inline int fgx_untranspose_state(const fgx::DevCfg& c, const fgx::DevState& s, const double* q, const double* qd,
                                 const double* goal, const double* hole, const int32_t* steps, hipStream_t stream,
                                 std::string& err) {
  const int threads = 256;
  const int blocks = (int)((c.N + threads - 1) / threads);
  hipLaunchKernelGGL(fgx::k_set_state, dim3(blocks), dim3(threads), 0, stream, c, s, q, qd, goal, hole, steps);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) { err = hipGetErrorString(e); return -2; }
  return 0;
}
