// fgx_tables.h — basis-table device functions (the kernels that run them once per handle are in
// fgx_tables_k.h; k_traj_env builds per-env rows with the same functions, fgx_learned.h):
//   rbf_row          ProMP / DMP rows: normalized-RBF basis on the phase of t_i = i*dt
//   prodmp_*         ProDMP precompute: cumulative-trapezoid integrals + homogeneous solutions
// All values are computed in f64 and rounded once to f32 (oracle/mp.py:build_tables); every exp is
// fgx_exp (fgx_exp.h), which oracle/mp.py:exp64 restates operation for operation, so the tables
// equal the oracle's bit for bit.
#pragma once
#include "fgx_device.h"
#include "fgx_exp.h"

namespace fgx {

// ============================================================================ tables
__device__ inline double phase64(const DevCfg& c, double t, double tau, double delay, double alpha_x) {
  double lin = (t - delay) / tau;
  lin = lin > 0.0 ? lin : 0.0;   // np.maximum(x, 0.0)
  if (c.phase == 0) return lin < 1.0 ? lin : 1.0;
  return fgx_exp((-alpha_x) * lin);
}

// normalized RBF at phase x, f64, all n = nb + zs + zg columns (oracle/mp.py:rbf64); centres at the
// unbounded phase of linspace(delay - o d, delay + tau + o d, n), d = tau / (n - 2o - 1), i.e. linear
// phase u_j = (j - o) / (n - 2o - 1) (o = num_basis_outside; 0: j / (n - 1))
__device__ inline void rbf64(const DevCfg& c, double alpha_x, double bw, double x, double* phi) {
  const int n = c.nb + c.zs + c.zg;
  double cen[kMaxBasis + 4], e[kMaxBasis + 4];
  for (int j = 0; j < n; ++j) {
    const double u = (n > 1) ? (double)(j - c.nbo) / (double)(n - 2 * c.nbo - 1) : 0.0;
    cen[j] = (c.phase == 0) ? u : fgx_exp((-alpha_x) * u);
  }
  for (int j = 0; j < n; ++j) {
    double d = (n > 1) ? ((j < n - 1) ? cen[j + 1] - cen[j] : cen[n - 1] - cen[n - 2]) : 1.0;
    const double h = bw / (d * d);
    const double dd = x - cen[j];
    e[j] = fgx_exp((-h) * (dd * dd) / 2);
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

// ProDMP fine-grid pieces at s = i*h (oracle/mp.py:prodmp_fine64): the variation-of-parameters
// integrands k1*phi, k2*phi and the homogeneous solutions.
__device__ inline void prodmp_integrands(const DevCfg& c, double s, double alpha_x, double bw, double* d1,
                                         double* d2) {
  const double x = fgx_exp((-alpha_x) * s);
  double phi[kMaxBasis + 4];
  rbf64(c, alpha_x, bw, x, phi);
  const double e = fgx_exp(c.alpha * s / 2);
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
  const double e = fgx_exp(a * s / 2);
  const double y1 = fgx_exp((-a) * s / 2);
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

// ProDMP with a delay or a basis dt of its own (basis_generator_kwargs dt,
// basis_generator_factory.py:8-23): the basis is looked up on the left-bounded linear phase, fine-grid
// index j(i) = rint(max((t_i - delay) / tau, 0) / (bdt / tau)) for t_i = i dt (oracle/mp.py:
// prodmp_delay_index): rows before the delay all equal the s = 0 row, so the plan holds its initial
// position and velocity there (test_black_box.py:267-307).  j(i) is non-decreasing in i; without a
// delay and with bdt = dt it is i (prodmp_identity: no lookup).  jmax clamps a non-finite value.
__host__ __device__ inline bool prodmp_identity(double delay, double dt, double bdt) { return delay == 0.0 && bdt == dt; }
__host__ __device__ inline int prodmp_delay_index(double dt, double bdt, int i, double tau, double delay, int jmax) {
  double u = ((double)i * dt - delay) / tau;
  u = u > 0.0 ? u : 0.0;                       // (NaN -> 0)
  const double j = __builtin_rint(u / (bdt / tau));
  return j < (double)jmax ? (j > 0.0 ? (int)j : 0) : jmax;
}
// fine-grid rows the shared table needs: j(rows - 1) + 1 (host: scratch size; device: the grid)
__host__ __device__ inline int prodmp_fine_rows(double dt, double bdt, int rows, double tau, double delay) {
  if (prodmp_identity(delay, dt, bdt)) return rows;
  return prodmp_delay_index(dt, bdt, rows - 1, tau, delay, 1 << 24) + 1;
}

// One env's ProDMP rows 0..R-1 for its own tau, sequentially in one thread: the cumulative
// trapezoid walks the fine grid in the same order as k_tables_prodmp / the oracle, and row i is
// emitted when the walk reaches fine-grid row j(i) (non-decreasing in i).  jmax: the walk's bound.
__device__ inline void prodmp_rows_seq(const DevCfg& c, double tau, double delay, double alpha_x, double bw, int R,
                                       float* tab) {
  const int nb = c.nb;
  const double h = c.bdt / tau;
  const bool ident = prodmp_identity(delay, c.dt, c.bdt);
  const int jmax = ident ? R - 1 : prodmp_delay_index(c.dt, c.bdt, R - 1, tau, delay, 1 << 20);
  double p1[kMaxBasis], p2[kMaxBasis], prev1[kMaxBasis], prev2[kMaxBasis], cur1[kMaxBasis], cur2[kMaxBasis];
  prodmp_integrands(c, 0.0, alpha_x, bw, prev1, prev2);
  for (int j = 0; j < nb; ++j) { p1[j] = 0.0; p2[j] = 0.0; }
  int f = 0;   // fine-grid row of p1 / p2
  for (int i = 0; i < R; ++i) {
    const int ji = ident ? i : prodmp_delay_index(c.dt, c.bdt, i, tau, delay, jmax);
    for (; f < ji; ++f) {
      const double s = (double)(f + 1) * h;
      prodmp_integrands(c, s, alpha_x, bw, cur1, cur2);
      for (int j = 0; j < nb; ++j) {
        p1[j] = p1[j] + h * (prev1[j] + cur1[j]) / 2;
        p2[j] = p2[j] + h * (prev2[j] + cur2[j]) / 2;
        prev1[j] = cur1[j];
        prev2[j] = cur2[j];
      }
    }
    prodmp_row(c, (double)f * h, p1, p2, tab + (size_t)i * c.stride);
  }
}

}  // namespace fgx
