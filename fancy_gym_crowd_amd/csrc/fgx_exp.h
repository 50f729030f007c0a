// fgx_exp.h — the exp of the basis tables (fgx_tables.h), restated operation for operation by
// oracle/mp.py:exp64 so that the device tables equal the oracle's bit for bit.
//
// The tables are computed in f64 and rounded once to f32 (oracle/mp.py module docstring).  With a
// library exp on each side (ocml on the device, numpy's SIMD exp on the host) the two f64 values
// differ by an ulp now and then, and ProDMP's cancellations (p2 y2 - p1 y1) carry that into ~1% of
// the f32 entries.  This exp uses only IEEE-exact-rounded f64 operations in a fixed order: the
// Cody-Waite reduction x = k ln2 + r (fdlibm's two-part ln2, k ln2_hi exact), a degree-13 Taylor
// polynomial of exp(r), |r| <= 0.35, in Horner form (plain mul / add: no fma, the unit is built
// with -ffp-contract=off), and the scaling by 2^k as an exact ldexp, or for a subnormal result an
// exact ldexp followed by one multiplication by 2^-600 (one rounding on either side).  Accuracy:
// a few ulp of f64, far below the f32 rounding the tables apply.
// Plain header (no HIP types): tests/test_host_cpu.py compiles it with g++ and compares it with
// exp64 bit for bit; __host__ / __device__ come from the HIP headers in the device units.
#pragma once

namespace fgx {

constexpr double kExpL2E = 1.4426950408889634;            // RN(1 / ln 2)
constexpr double kExpLn2Hi = 6.93147180369123816490e-01;  // 0x3fe62e42fee00000 (32 significant bits)
constexpr double kExpLn2Lo = 1.90821492927058770002e-10;  // ln 2 - kExpLn2Hi
// 1 / n!, n = 13 .. 2 (Python repr of 1 / math.factorial(n): the same doubles in oracle/mp.py)
constexpr double kExpC[12] = {1.6059043836821613e-10, 2.08767569878681e-09, 2.505210838544172e-08,
                              2.755731922398589e-07,  2.7557319223985893e-06, 2.48015873015873e-05,
                              0.0001984126984126984,  0.001388888888888889,  0.008333333333333333,
                              0.041666666666666664,   0.16666666666666666,   0.5};

__host__ __device__ inline double fgx_exp(double x) {
  if (x != x) return x;
  if (x > 709.8) return __builtin_inf();
  if (x < -746.0) return 0.0;
  const double k = __builtin_rint(x * kExpL2E);
  const double r = (x - k * kExpLn2Hi) - k * kExpLn2Lo;
  double p = kExpC[0];
#pragma unroll
  for (int i = 1; i < 12; ++i) p = p * r + kExpC[i];
  p = p * r + 1.0;
  p = p * r + 1.0;
  const int ki = (int)k;
  if (ki < -1000) return __builtin_ldexp(p, ki + 600) * 0x1p-600;
  return __builtin_ldexp(p, ki);
}

}  // namespace fgx
