// Does a lone wave hide independent VALU work in the dependency stalls of a serial f64 chain?
// k_episode_jl's fast chunk runs, per sample and lane, a 9-deep dependent f64 recurrence (PD, clip,
// semi-implicit Euler: fsub, mul, add, max, min, mul, add, mul, add) plus ~12 independent VALU
// instructions (f32 trajectory look-ahead, conversions, the velocity branch, a^2).  The compiler
// emits the chain back to back and the independent work as a separate run.  This benchmark times,
// for one wave per SIMD (1024 single-wave workgroups) and 200 x 8 samples, the same instruction
// mix written in inline asm (volatile: issued in exactly this order) as
//   mode 0: chain only                     mode 1: independent ops only
//   mode 2: chain, then the independent ops (the compiler's order)
//   mode 3: one independent op after each chain op (interleaved)
//   mode 4: two independent ops after each chain op
// and prints cycles per sample (at the measured kernel time and 2.4 GHz) as one JSON line per mode.
//   hipcc --offload-arch=gfx950 -O3 tools/chainbench.hip -o tools/chainbench && tools/chainbench
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("hip error %s\n", hipGetErrorString(e_)); return 1; } } while (0)

typedef float f32x2 __attribute__((ext_vector_type(2)));
constexpr int SAMPLES = 1600;

// one step of the recurrence for one joint: q, qd carried; p, v the sample's desired state (f64)
#define CH_SUB(dst, a, b) asm volatile("v_fma_f64 %0, -%1, %2, %3" : "=v"(dst) : "v"(b), "s"(one), "v"(a))
#define CH_MUL(dst, a, b) asm volatile("v_mul_f64 %0, %1, %2" : "=v"(dst) : "v"(a), "v"(b))
#define CH_ADD(dst, a, b) asm volatile("v_fma_f64 %0, %1, %2, %3" : "=v"(dst) : "v"(a), "s"(one), "v"(b))
#define CH_MAX(dst, a, b) asm volatile("v_max_f64 %0, %1, %2" : "=v"(dst) : "v"(a), "v"(b))
#define CH_MIN(dst, a, b) asm volatile("v_min_f64 %0, %1, %2" : "=v"(dst) : "v"(a), "v"(b))
#define IND(i) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(ind[(i) & 7]) : "v"(wa), "v"(wb))
// a 64-bit scalar address advance (what the fast chunk does per scalar table load)
#define SAL(i) asm volatile("s_add_u32 %0, %0, 32\n\ts_addc_u32 %1, %1, 0" : "+s"(sa[(i) & 3]), "+s"(sb[(i) & 3]) :: "scc")

template <int MODE>
__global__ __launch_bounds__(512) void k_chain(double* out, double pg, double dg, double dt, double lo, double hi,
                                               float wseed) {
  const int e = blockIdx.x * 64 + threadIdx.x;
  double one = 1.0;
  asm volatile("" : "+s"(one));
  double q = 1e-3 * e, qd = 0.0, p = 0.5, v = 0.25;
  f32x2 ind[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) ind[i] = f32x2{wseed + i, wseed - i};
  const f32x2 wa = {0.999f, 0.998f}, wb = {1e-3f, 2e-3f};
  unsigned sa[4] = {1, 2, 3, 4}, sb[4] = {5, 6, 7, 8};
  for (int k = 0; k < SAMPLES; ++k) {
    double e1, e2, u1, u2, u, a, t1, t2;
    if constexpr (MODE == 1) {
#pragma unroll
      for (int i = 0; i < 12; ++i) IND(i);
      continue;
    } else {
      // after f64 op i (0..12): mode 3 one independent op (i < 12), mode 4 two (i < 6)
#define SLOT(i)                                  \
  if (MODE == 3 && (i) < 12) IND(i);             \
  if (MODE == 4 && (i) < 6) { IND(2 * (i)); IND(2 * (i) + 1); }
      // the velocity branch's two independent f64 ops (as in the kernel), then the chain:
      // q -> sub -> mul -> add -> max -> min -> mul -> add (qd) -> mul -> add (q)
      CH_SUB(e2, v, qd); SLOT(0)
      CH_MUL(u2, e2, dg); SLOT(1)
      CH_SUB(e1, p, q); SLOT(2)
      CH_MUL(u1, e1, pg); SLOT(3)
      CH_ADD(u, u1, u2); SLOT(4)
      CH_MAX(a, u, lo); SLOT(5)
      CH_MIN(a, a, hi); SLOT(6)
      CH_MUL(t1, a, dt); SLOT(7)
      CH_ADD(qd, t1, qd); SLOT(8)
      CH_MUL(t2, qd, dt); SLOT(9)
      CH_ADD(q, t2, q); SLOT(10)
      if (MODE == 3) IND(11);
      if (MODE == 2) {
#pragma unroll
        for (int i = 0; i < 12; ++i) IND(i);
      }
      if (MODE == 5) {   // chain + 4 scalar 64-bit address advances (8 SALU)
#pragma unroll
        for (int i = 0; i < 4; ++i) SAL(i);
      }
    }
  }
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += ind[i].x + ind[i].y;
  out[e] = q + qd + s + (double)(sa[0] + sa[1] + sa[2] + sa[3] + sb[0] + sb[1] + sb[2] + sb[3]);
}

template <int MODE>
static int run(double* out, int waves, int threads = 64) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  for (int rep = 0; rep < 2; ++rep) {   // warm-up launch, then the timed one
    CHK(hipEventRecord(a));
    hipLaunchKernelGGL(k_chain<MODE>, dim3(waves * 64 / threads), dim3(threads), 0, 0, out, 0.6, 0.075, 0.01, -1.0, 1.0,
                       0.5f);
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
  }
  float ms = 0.0f;
  CHK(hipEventElapsedTime(&ms, a, b));
  const char* names[] = {"chain only (13 f64, 9 dependent)", "12 independent pk_fma only", "chain then 12 independent",
                         "chain with 1 independent after each of its ops (12 total)",
                         "chain with 2 independent after each of its first 6 ops (12 total)",
                         "chain then 8 SALU (4 s_add_u32 / s_addc_u32 pairs)"};
  printf("{\"mode\": %d, \"what\": \"%s\", \"waves\": %d, \"threads\": %d, \"us\": %.2f, "
         "\"cycles_per_sample_at_2.4GHz\": %.1f}\n", MODE, names[MODE], waves, threads, ms * 1e3,
         ms * 1e-3 * 2.4e9 / SAMPLES);
  return 0;
}

int main() {
  double* out;
  const int waves = 1024;   // one wave per SIMD on 256 CUs
  CHK(hipMalloc(&out, sizeof(double) * 64 * waves));
  CHK(hipFree(out));
  CHK(hipMalloc(&out, sizeof(double) * 64 * waves * 2));
  if (run<0>(out, waves) || run<1>(out, waves) || run<2>(out, waves) || run<3>(out, waves) || run<4>(out, waves) ||
      run<5>(out, waves))
    return 1;
  // two waves per SIMD (2048 waves in 512-thread workgroups: waves w, w + 4 share a SIMD)
  if (run<0>(out, 2 * waves, 512) || run<1>(out, 2 * waves, 512) || run<2>(out, 2 * waves, 512)) return 1;
  // one wave per SIMD through 256-thread workgroups (4 waves per CU, one per SIMD)
  if (run<2>(out, waves, 256)) return 1;
  CHK(hipFree(out));
  return 0;
}
