// fgx_trig.h — f64 sin / cos for the kernels: the ocml algorithm (ROCm device libs,
// __ocml_sincos_f64) restated operation for operation, so every result is bit-identical to
// sincos(); only the argument reduction differs in *how* it is reached.  ocml reduces |x| < 2^30
// with a three-part Cody-Waite step and larger |x| with a Payne-Hanek step (v_trig_preop_f64), and
// the compiler, both being side-effect free, if-converts the two into straight-line code: every
// sincos() call then executes the large-argument reduction as well (~100 of its ~155 VALU
// instructions, tools: isa_blocks.py on a one-call kernel).  Here the small path runs inline and
// |x| >= 2^30, inf and NaN take a real branch to ocml.
#pragma once
#include <hip/hip_runtime.h>

namespace fgx {

static __device__ __attribute__((noinline)) void sincos_ocml(double x, double* s, double* c) { ::sincos(x, s, c); }

__device__ __forceinline__ double bits_f64(unsigned long long u) { return __longlong_as_double((long long)u); }

__device__ __forceinline__ void fgx_sincos(double x, double* sp, double* cp) {
#ifdef FGX_OCML_SINCOS   // A/B builds only: the library call
  ::sincos(x, sp, cp);
  return;
#endif
  const double ax = __builtin_fabs(x);
  if (__builtin_expect(!(ax < 0x1p30), 0)) {   // (and inf / NaN)
    sincos_ocml(x, sp, cp);
    return;
  }
  // __ocmlpriv_trigredsmall_f64(ax): r = hi + lo, quadrant i
  const double k = __builtin_rint(ax * bits_f64(0x3FE45F306DC9C883ull));
  const double r4 = __builtin_fma(k, bits_f64(0xBFF921FB54442D18ull), ax);
  const double r5 = __builtin_fma(k, bits_f64(0xBC91A62633145C00ull), r4);
  const double r6 = k * bits_f64(0x3C91A62633145C00ull);
  const double r8 = __builtin_fma(k, bits_f64(0x3C91A62633145C00ull), -r6);
  const double r9 = r4 - r6;
  const double r10 = r4 - r9;
  const double r11 = r10 - r6;
  const double r12 = r9 - r5;
  const double r13 = r12 + r11;
  const double r14 = r13 - r8;
  const double r15 = __builtin_fma(k, bits_f64(0xB97B839A252049C0ull), r14);
  const double hi = r5 + r15;
  const double r17 = hi - r5;
  const double lo = r15 - r17;
  const int i = ((int)k) & 3;
  // __ocmlpriv_sincosred2_f64(hi, lo)
  const double x2 = hi * hi;
  const double h = x2 * 0.5;
  const double c5 = 1.0 - h;
  const double c6 = 1.0 - c5;
  const double c7 = c6 - h;
  const double x4 = x2 * x2;
  double pc = __builtin_fma(x2, bits_f64(0xBDA907DB46CC5E42ull), bits_f64(0x3E21EEB69037AB78ull));
  pc = __builtin_fma(x2, pc, bits_f64(0xBE927E4FA17F65F6ull));
  pc = __builtin_fma(x2, pc, bits_f64(0x3EFA01A019F4EC90ull));
  pc = __builtin_fma(x2, pc, bits_f64(0xBF56C16C16C16967ull));
  pc = __builtin_fma(x2, pc, bits_f64(0x3FA5555555555555ull));
  const double c15 = __builtin_fma(hi, -lo, c7);
  const double c16 = __builtin_fma(x4, pc, c15);
  const double cr = c5 + c16;
  double ps = __builtin_fma(x2, bits_f64(0x3DE5E0B2F9A43BB8ull), bits_f64(0xBE5AE600B42FDFA7ull));
  ps = __builtin_fma(x2, ps, bits_f64(0x3EC71DE3796CDE01ull));
  ps = __builtin_fma(x2, ps, bits_f64(0xBF2A01A019E83E5Cull));
  ps = __builtin_fma(x2, ps, bits_f64(0x3F81111111110BB3ull));
  const double s23 = hi * -x2;
  const double s25 = __builtin_fma(s23, ps, lo * 0.5);
  const double s26 = __builtin_fma(x2, s25, -lo);
  const double s27 = __builtin_fma(s23, bits_f64(0xBFC5555555555555ull), s26);
  const double sr = hi - s27;
  // __ocml_sincos_f64: quadrant selection and signs
  const unsigned flip = i > 1 ? 0x80000000u : 0u;
  const bool even = (i & 1) == 0;
  const double sm = even ? sr : cr;
  const double cm = even ? cr : -sr;
  const unsigned xs = (unsigned)((unsigned long long)__double_as_longlong(x) >> 32) & 0x80000000u;
  const unsigned long long sb = (unsigned long long)__double_as_longlong(sm);
  const unsigned long long cb = (unsigned long long)__double_as_longlong(cm);
  *sp = __longlong_as_double((long long)(sb ^ ((unsigned long long)(xs ^ flip) << 32)));
  *cp = __longlong_as_double((long long)(cb ^ ((unsigned long long)flip << 32)));
}

// sin / cos for |x| < 2^20 to ~5e-16 absolute (not bit-identical to fgx_sincos): a two-part
// Cody-Waite reduction by pi/2 (each step one rounding: |r| error <= 1.2e-16) and Taylor polynomials
// through r^15 / r^16 on |r| <= pi/4 (truncation < 5e-17), ~30 VALU instead of ~50.  For results
// that are then rounded to f32 and checked against that error (f32_checked below): equal to the
// exact path's f32 whenever the check passes.
__host__ __device__ __forceinline__ void fgx_sincos_fast(double x, double* sp, double* cp) {
  const double k = __builtin_rint(x * 0x1.45f306dc9c883p-1);                 // x * 2 / pi
  double r = __builtin_fma(-k, 0x1.921fb54442d18p+0, x);                     // pi / 2 (hi)
  r = __builtin_fma(-k, 0x1.1a62633145c07p-54, r);                           // pi / 2 (lo)
  const double r2 = r * r;
  double ps = __builtin_fma(r2, -0x1.ae7f3e733b81fp-41, 0x1.6124613a86d09p-33);
  ps = __builtin_fma(r2, ps, -0x1.ae64567f544e4p-26);
  ps = __builtin_fma(r2, ps, 0x1.71de3a556c734p-19);
  ps = __builtin_fma(r2, ps, -0x1.a01a01a01a01ap-13);
  ps = __builtin_fma(r2, ps, 0x1.1111111111111p-7);
  ps = __builtin_fma(r2, ps, -0x1.5555555555555p-3);
  const double sr = __builtin_fma(r * r2, ps, r);
  double pc = __builtin_fma(r2, 0x1.ae7f3e733b81fp-45, -0x1.93974a8c07c9dp-37);
  pc = __builtin_fma(r2, pc, 0x1.1eed8eff8d898p-29);
  pc = __builtin_fma(r2, pc, -0x1.27e4fb7789f5cp-22);
  pc = __builtin_fma(r2, pc, 0x1.a01a01a01a01ap-16);
  pc = __builtin_fma(r2, pc, -0x1.6c16c16c16c17p-10);
  pc = __builtin_fma(r2, pc, 0x1.5555555555555p-5);
  pc = __builtin_fma(r2, pc, -0.5);
  const double cr = __builtin_fma(r2, pc, 1.0);
  const int i = ((int)k) & 3;   // quadrant: sin x = [s, c, -s, -c][i], cos x = [c, -s, -c, s][i]
  const bool odd = (i & 1) != 0;
  const double sm = odd ? cr : sr, cm = odd ? sr : cr;
  *sp = (i & 2) ? -sm : sm;
  *cp = ((i + 1) & 2) ? -cm : cm;
}

// (float) v where v is within m of the exact value whose (float) is wanted: both ends of [v - m, v + m]
// round alike, or ok is cleared (the caller recomputes exactly)
__host__ __device__ __forceinline__ float f32_checked(double v, double m, bool& ok) {
  const float lo = (float)(v - m), hi = (float)(v + m);
  ok = ok && (lo == hi);
  return lo;
}

// The observation's trigonometric components of one sample (emit_obs / k_info_obs order: cos q[0..NL),
// sin q[0..NL), end effector x - gx, y - gy) as f32, from the fast path: fgx_sincos_fast of every
// joint angle, the cumulative angles' cos / sin by angle addition, the end effector as the same
// sequential sums, every f32 through f32_checked.  Returns false if any value could round otherwise
// than the exact path's (Env::fk + fgx_sincos) — or |q| >= 2^20, or NaN: the caller recomputes then.
//   cos / sin of q: |fast - exact| <= 1.5e-16 + the exact path's own <= 1 ulp: margin 1e-15;
//   end effector: link d's cos / sin carry d angle additions' product roundings (~3e-16 each) and
//   the exact path's roundings of the cumulative angles (<= 1.1e-16 A each, A = sum |q| >= every
//   |angle|); summed over the links with the sums' own roundings, < NL^2 / 2 (1.1e-16 A + 3e-16) +
//   4.4e-16 NL: the margin doubles that.
template <int NL>
__host__ __device__ __forceinline__ bool obs_trig_fast(const double* q, double gx, double gy, float* out) {
  double cq[NL], sq[NL];
  bool ok = true;
  double A = 0.0;
#pragma unroll
  for (int d = 0; d < NL; ++d) {
    ok = ok && __builtin_fabs(q[d]) < 0x1p20;   // (and not NaN)
    fgx_sincos_fast(q[d], &sq[d], &cq[d]);
    A += __builtin_fabs(q[d]);
  }
  constexpr double kTrigM = 1e-15;
  const double kEeM = NL * NL * (2e-16 * A + 1e-15) + 1e-14;
  double ca = cq[0], sa = sq[0], x = cq[0], y = sq[0];   // cos / sin of the cumulative angle
#pragma unroll
  for (int d = 1; d < NL; ++d) {
    const double c2 = __builtin_fma(ca, cq[d], -(sa * sq[d]));
    const double s2 = __builtin_fma(sa, cq[d], ca * sq[d]);
    ca = c2;
    sa = s2;
    x = x + ca;
    y = y + sa;
  }
#pragma unroll
  for (int d = 0; d < NL; ++d) {
    out[d] = f32_checked(cq[d], kTrigM, ok);
    out[NL + d] = f32_checked(sq[d], kTrigM, ok);
  }
  out[2 * NL] = f32_checked((0.0 + x) - gx, kEeM, ok);
  out[2 * NL + 1] = f32_checked((0.0 + y) - gy, kEeM, ok);
  return ok;
}

}  // namespace fgx
