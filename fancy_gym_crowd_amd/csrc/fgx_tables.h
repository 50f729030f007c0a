// fgx_tables.h — basis-table kernels (included by fgx_api.hip only).
//   k_tables_rbf     ProMP / DMP rows: normalized-RBF basis on the phase of t_i = i*dt
//   k_tables_prodmp  ProDMP precompute: cumulative-trapezoid integrals + homogeneous solutions
// All values are computed in f64 and rounded once to f32 (oracle/mp.py:build_tables).
#pragma once
#include "fgx_device.h"

namespace fgx {

// ============================================================================ tables
__device__ inline double phase64(const DevCfg& c, double t, double tau, double delay, double alpha_x) {
  double lin = (t - delay) / tau;
  lin = lin > 0.0 ? lin : 0.0;   // np.maximum(x, 0.0)
  if (c.phase == 0) return lin < 1.0 ? lin : 1.0;
  return exp((-alpha_x) * lin);
}

// normalized RBF at phase x, f64, all n = nb + zs + zg columns (oracle/mp.py:rbf64); centres at the
// unbounded phase of linspace(delay - o d, delay + tau + o d, n), d = tau / (n - 2o - 1), i.e. linear
// phase u_j = (j - o) / (n - 2o - 1) (o = num_basis_outside; 0: j / (n - 1))
__device__ inline void rbf64(const DevCfg& c, double alpha_x, double bw, double x, double* phi) {
  const int n = c.nb + c.zs + c.zg;
  double cen[kMaxBasis + 4], e[kMaxBasis + 4];
  for (int j = 0; j < n; ++j) {
    const double u = (n > 1) ? (double)(j - c.nbo) / (double)(n - 2 * c.nbo - 1) : 0.0;
    cen[j] = (c.phase == 0) ? u : exp((-alpha_x) * u);
  }
  for (int j = 0; j < n; ++j) {
    double d = (n > 1) ? ((j < n - 1) ? cen[j + 1] - cen[j] : cen[n - 1] - cen[n - 2]) : 1.0;
    const double h = bw / (d * d);
    const double dd = x - cen[j];
    e[j] = exp((-h) * (dd * dd) / 2);
  }
  double s;
  if (n < 8) {
    s = e[0] + 0.0;
    for (int j = 1; j < n; ++j) s = s + e[j];
  } else {   // numpy pairwise (8 accumulators, n <= 128)
    double r[8];
    for (int j = 0; j < 8; ++j) r[j] = e[j];
    int i = 8;
    for (; i < n - (n % 8); i += 8)
      for (int j = 0; j < 8; ++j) r[j] = r[j] + e[i + j];
    s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) s = s + e[i];
  }
  for (int j = 0; j < n; ++j) phi[j] = e[j] / s;
}

// One ProMP / DMP table row i (t_i = i*dt) for the phase (tau, delay).
__device__ inline void rbf_row(const DevCfg& c, int i, double tau, double delay, double alpha_x, double bw,
                               float* row) {
  double phi[kMaxBasis + 4];
  const double t = (double)i * c.dt;
  const double x = phase64(c, t, tau, delay, alpha_x);
  rbf64(c, alpha_x, bw, x, phi);
  if (c.mp == MP_PROMP) {
    for (int j = 0; j < c.nb; ++j) row[j] = (float)(c.weights_scale * phi[c.zs + j]);
    const float t0 = (float)t, t1 = (float)((double)(i + 1) * c.dt);
    const float dt32 = t1 - t0;
    row[c.nb] = dt32;
    row[c.nb + 1] = 1.0f / dt32;     // RN(1/dt32) for div_rcp
  } else {   // DMP: psi = x * phi ; sdt = f32(s_{i+1}) - f32(s_i)
    for (int j = 0; j < c.nb; ++j) row[j] = (float)(x * phi[c.zs + j]);
    double s0 = (t - delay) / tau, s1 = ((double)(i + 1) * c.dt - delay) / tau;
    s0 = s0 > 0.0 ? s0 : 0.0;
    s1 = s1 > 0.0 ? s1 : 0.0;
    row[c.nb] = (float)s1 - (float)s0;
  }
}

// ProMP / DMP tables: one thread per row.
__global__ void k_tables_rbf(DevCfg c, double tau, double delay, double alpha_x, double bw, float* tab) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= c.rows) return;
  rbf_row(c, i, tau, delay, alpha_x, bw, tab + (size_t)i * c.stride);
}

// ProDMP fine-grid pieces at s = i*h (oracle/mp.py:prodmp_fine64): the variation-of-parameters
// integrands k1*phi, k2*phi and the homogeneous solutions.
__device__ inline void prodmp_integrands(const DevCfg& c, double s, double alpha_x, double bw, double* d1,
                                         double* d2) {
  const double x = exp((-alpha_x) * s);
  double phi[kMaxBasis + 4];
  rbf64(c, alpha_x, bw, x, phi);
  const double e = exp(c.alpha * s / 2);
  const double k1 = s * e * x, k2 = e * x;
  for (int j = 0; j < c.nb; ++j) {
    d1[j] = k1 * phi[c.zs + j];
    d2[j] = k2 * phi[c.zs + j];
  }
}

// ProDMP table row from the cumulative integrals p1, p2 at s.
__device__ inline void prodmp_row(const DevCfg& c, double s, const double* p1, const double* p2, float* row) {
  const int nb = c.nb;
  const double a = c.alpha;
  const double e = exp(a * s / 2);
  const double y1 = exp((-a) * s / 2);
  const double y2 = s * y1;
  const double dy1 = -a / 2 * y1;
  const double dy2 = -a / 2 * y2 + y1;
  const double q1 = (a * s / 2 - 1) * e + 1;
  const double q2 = a / 2 * (e - 1);
  for (int j = 0; j < nb; ++j) {
    row[j] = (float)(p2[j] * y2 - p1[j] * y1);
    row[nb + 1 + j] = (float)(p2[j] * dy2 - p1[j] * dy1);
  }
  row[nb] = (float)(q2 * y2 - q1 * y1);
  row[2 * nb + 1] = (float)(q2 * dy2 - q1 * dy1);
  row[2 * nb + 2] = (float)y1;
  row[2 * nb + 3] = (float)y2;
  row[2 * nb + 4] = (float)dy1;
  row[2 * nb + 5] = (float)dy2;
}

// ProDMP with a delay: the basis is looked up on the left-bounded linear phase, fine-grid index
// j(i) = rint(max((t_i - delay) / tau, 0) / (dt / tau)) for t_i = i dt (oracle/mp.py:
// prodmp_delay_index): rows before the delay all equal the s = 0 row, so the plan holds its
// initial position and velocity there (test_black_box.py:267-307).  j(i) <= i, non-decreasing.
__device__ inline int prodmp_delay_index(const DevCfg& c, int i, double tau, double delay) {
  double u = ((double)i * c.dt - delay) / tau;
  u = u > 0.0 ? u : 0.0;                       // (NaN -> 0)
  // j <= i holds for every delay >= 0 (fgx_create refuses a negative or non-finite static delay,
  // learned delays are clipped to delay_bound, lo >= 0); the clamp keeps any other value inside
  // the rows already computed
  const double j = rint(u / (c.dt / tau));
  return j < (double)i ? (int)j : i;
}

// One env's ProDMP rows 0..R-1 for its own tau, sequentially in one thread (the cumulative
// trapezoid in the same order as k_tables_prodmp / the oracle), then the delay remap in place
// (descending i: row j(i) <= i is still the fine-grid row when row i is written).
__device__ inline void prodmp_rows_seq(const DevCfg& c, double tau, double delay, double alpha_x, double bw, int R,
                                       float* tab) {
  const int nb = c.nb;
  const double h = c.dt / tau;
  double p1[kMaxBasis], p2[kMaxBasis], prev1[kMaxBasis], prev2[kMaxBasis], cur1[kMaxBasis], cur2[kMaxBasis];
  prodmp_integrands(c, 0.0, alpha_x, bw, prev1, prev2);
  for (int j = 0; j < nb; ++j) { p1[j] = 0.0; p2[j] = 0.0; }
  prodmp_row(c, 0.0, p1, p2, tab);
  for (int i = 1; i < R; ++i) {
    const double s = (double)i * h;
    prodmp_integrands(c, s, alpha_x, bw, cur1, cur2);
    for (int j = 0; j < nb; ++j) {
      p1[j] = p1[j] + h * (prev1[j] + cur1[j]) / 2;
      p2[j] = p2[j] + h * (prev2[j] + cur2[j]) / 2;
      prev1[j] = cur1[j];
      prev2[j] = cur2[j];
    }
    prodmp_row(c, s, p1, p2, tab + (size_t)i * c.stride);
  }
  if (delay != 0.0)
    for (int i = R - 1; i > 0; --i) {
      const int j = prodmp_delay_index(c, i, tau, delay);
      if (j != i)
        for (int k = 0; k < c.stride; ++k) tab[(size_t)i * c.stride + k] = tab[(size_t)j * c.stride + k];
    }
}

// ProDMP precompute (oracle/mp.py:prodmp_fine64).  Single block; scratch: [rows][2*nb] f64.
__global__ void k_tables_prodmp(DevCfg c, double tau, double delay, double alpha_x, double bw, double* dp,
                                float* tab) {
  const int nb = c.nb, R = c.rows, W = 2 * nb;
  const double h = c.dt / tau;
  for (int i = threadIdx.x; i < R; i += blockDim.x)
    prodmp_integrands(c, (double)i * h, alpha_x, bw, dp + (size_t)i * W, dp + (size_t)i * W + nb);
  __syncthreads();
  // cumulative trapezoid, one thread per column, sequential (same order as the oracle)
  if ((int)threadIdx.x < W) {
    const int j = threadIdx.x;
    double p = 0.0, prev = dp[j];
    dp[j] = 0.0;
    for (int i = 1; i < R; ++i) {
      const double cur = dp[(size_t)i * W + j];
      p = p + h * (prev + cur) / 2;
      dp[(size_t)i * W + j] = p;
      prev = cur;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < R; i += blockDim.x) {   // row i = fine-grid row j(i) (delay)
    const int j = delay != 0.0 ? prodmp_delay_index(c, i, tau, delay) : i;
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
