// Host-side property check of csrc/fgx_trig.h's observation fast path (obs_trig_fast,
// fgx_sincos_fast, f32_checked), run on the CPU by tests/test_host_trig.py: for random joint angles
// and goals, every f32 the fast path accepts must equal the exact path's f32 — libm cos / sin of the
// joint angles and of numpy's rounded cumulative angles, the end effector as Env::fk's sequential
// sums (fgx_device.h) — and fallbacks must stay rare.  Prints one JSON line.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>

#include "../../fancy_gym_crowd_amd/csrc/fgx_trig.h"

template <int NL>
static void exact(const double* q, double gx, double gy, float* out) {
  double ang = 0.0, x = 0.0, y = 0.0;
  for (int k = 0; k < NL; ++k) {
    ang = (k == 0) ? q[0] : ang + q[k];
    const double c = std::cos(ang), s = std::sin(ang);
    x = (k == 0) ? c : x + c;
    y = (k == 0) ? s : y + s;
    if (k == 0) { out[0] = (float)c; out[NL] = (float)s; }
  }
  for (int d = 1; d < NL; ++d) { out[d] = (float)std::cos(q[d]); out[NL + d] = (float)std::sin(q[d]); }
  out[2 * NL] = (float)((0.0 + x) - gx);
  out[2 * NL + 1] = (float)((0.0 + y) - gy);
}

template <int NL>
static void run(long n, unsigned seed, long& bad, long& fb, long& vals) {
  std::mt19937_64 g(seed);
  std::uniform_real_distribution<double> u(-1.0, 1.0);
  for (long t = 0; t < n; ++t) {
    double q[NL];
    const int kind = (int)(t % 8);
    const double scale = kind < 4 ? 3.2 : (kind < 6 ? 40.0 : 1e4);
    for (int d = 0; d < NL; ++d) q[d] = u(g) * scale;
    if (kind == 7) q[t % NL] = u(g) * 1e-9;             // sin / cos below the margin's f32 resolution
    if (kind == 6 && (t & 1)) q[0] = M_PI / 2;
    const double gx = u(g) * 2.0, gy = u(g) * 2.0;
    float f[2 * NL + 2], e[2 * NL + 2];
    const bool ok = fgx::obs_trig_fast<NL>(q, gx, gy, f);
    exact<NL>(q, gx, gy, e);
    vals += 2 * NL + 2;
    if (!ok) { ++fb; continue; }
    for (int i = 0; i < 2 * NL + 2; ++i)
      if (f[i] != e[i] && !(std::isnan(f[i]) && std::isnan(e[i]))) ++bad;
  }
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 1000000;
  long bad = 0, fb = 0, vals = 0;
  run<5>(n, 1, bad, fb, vals);
  run<2>(n / 2, 2, bad, fb, vals);
  run<8>(n / 4, 3, bad, fb, vals);
  // range / NaN guards: the fast path must refuse them
  long guard_fail = 0;
  const double odd[] = {1048576.0, -1048576.0, 1e300, NAN, INFINITY};
  for (double v : odd) {
    double q[5] = {0.3, v, -0.2, 0.1, 0.0};
    float f[12];
    if (fgx::obs_trig_fast<5>(q, 0.0, 0.0, f)) ++guard_fail;
  }
  // fgx_sincos_fast's absolute error against long double
  double maxerr = 0.0;
  std::mt19937_64 g(9);
  std::uniform_real_distribution<double> u(-1e4, 1e4);
  for (long t = 0; t < n; ++t) {
    const double x = u(g);
    double s, c;
    fgx::fgx_sincos_fast(x, &s, &c);
    maxerr = std::fmax(maxerr, (double)std::fabs((long double)s - sinl((long double)x)));
    maxerr = std::fmax(maxerr, (double)std::fabs((long double)c - cosl((long double)x)));
  }
  printf("{\"values\": %ld, \"checked_but_different\": %ld, \"fallback_samples\": %ld, \"guard_failures\": %ld, "
         "\"sincos_fast_max_abs_err\": %.3g}\n", vals, bad, fb, guard_fail, maxerr);
  return 0;
}
