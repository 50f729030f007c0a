// fgx_tables_k.h — the basis-table kernels, run once per handle by fgx_create (included by
// fgx_api.hip only; the device functions they call are in fgx_tables.h).
//   k_tables_rbf        ProMP / DMP rows, one thread per row
//   k_tables_prodmp     ProDMP precompute on the fine grid, then the rows at j(i)
//   k_tables_transpose  column-major copy for k_episode_jl's scalar loads
#pragma once
#include "fgx_tables.h"

namespace fgx {

__global__ void k_tables_rbf(DevCfg c, double tau, double delay, double alpha_x, double bw, float* tab) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= c.rows) return;
  rbf_row(c, i, tau, delay, alpha_x, bw, tab + (size_t)i * c.stride);
}

// ProDMP precompute (oracle/mp.py:prodmp_fine64).  Single block; scratch dp: [Rf][2*nb] f64 over the
// fine grid s_j = j * bdt / tau, Rf = prodmp_fine_rows(...) (= rows without a delay or own basis dt).
__global__ void k_tables_prodmp(DevCfg c, double tau, double delay, double alpha_x, double bw, int Rf, double* dp,
                                float* tab) {
  const int nb = c.nb, W = 2 * nb;
  const double h = c.bdt / tau;
  for (int i = threadIdx.x; i < Rf; i += blockDim.x)
    prodmp_integrands(c, (double)i * h, alpha_x, bw, dp + (size_t)i * W, dp + (size_t)i * W + nb);
  __syncthreads();
  // cumulative trapezoid, one thread per column, sequential (same order as the oracle)
  if ((int)threadIdx.x < W) {
    const int j = threadIdx.x;
    double p = 0.0, prev = dp[j];
    dp[j] = 0.0;
    for (int i = 1; i < Rf; ++i) {
      const double cur = dp[(size_t)i * W + j];
      p = p + h * (prev + cur) / 2;
      dp[(size_t)i * W + j] = p;
      prev = cur;
    }
  }
  __syncthreads();
  const bool ident = prodmp_identity(delay, c.dt, c.bdt);
  for (int i = threadIdx.x; i < c.rows; i += blockDim.x) {   // row i = fine-grid row j(i)
    const int j = ident ? i : prodmp_delay_index(c.dt, c.bdt, i, tau, delay, Rf - 1);
    prodmp_row(c, (double)j * h, dp + (size_t)j * W, dp + (size_t)j * W + nb, tab + (size_t)i * c.stride);
  }
}

// column-major copy of the shared table (DevState::tables_t)
__global__ void k_tables_transpose(int rows, int stride, int nb, const float* tab, float* tt) {
  const int RT = tables_t_rows(rows);
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= stride * RT) return;
  const int col = i / RT, r = i - col * RT - tables_t_pad(col, nb);
  tt[i] = (r >= 0 && r < rows) ? tab[(size_t)r * stride + col] : 0.0f;
}

}  // namespace fgx
