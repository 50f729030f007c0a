// Measures sustained VALU issue rates on the GPU for the instruction classes the episode kernel
// is made of (f64 add/mul/fma/max, f32 fma, packed f32 fma, f32->f64 convert).  Each lane runs
// 8 independent dependency chains; the grid puts `waves` waves on every SIMD.  Prints one JSON
// line per op: wave-instructions per SIMD per cycle at the measured clock-free rate
// (instr/s per SIMD) and the implied cycles/instruction at 2.4 GHz.
//   hipcc --offload-arch=gfx950 -O3 tools/valu_rates.hip -o /tmp/valu_rates && /tmp/valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("hip error %s\n", hipGetErrorString(e_)); return 1; } } while (0)

constexpr int ITERS = 4096;

template <int OP>
__global__ __launch_bounds__(256) void k_rate(double* out, double s) {
  double a[8];
  float f[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { a[j] = threadIdx.x * 1e-3 + j; f[j] = (float)a[j]; }
  const double m = s * 0.5, c = s * 1e-9;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (OP == 0) asm volatile("v_add_f64 %0, %0, %1" : "+v"(a[j]) : "v"(c));
      if (OP == 1) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(a[j]) : "v"(m));
      if (OP == 2) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a[j]) : "v"(m), "v"(c));
      if (OP == 3) asm volatile("v_max_f64 %0, %0, %1" : "+v"(a[j]) : "v"(c));
      if (OP == 4) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f[j]) : "v"((float)m), "v"((float)c));
      if (OP == 5) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(m), "v"(c));
      if (OP == 6) asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(a[j]) : "v"(f[j]));
      if (OP == 7) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(f[j]) : "v"((float)c));
      if (OP == 8) asm volatile("v_mov_b64 %0, %1" : "=v"(a[j]) : "v"(a[(j + 1) & 7]));
      if (OP == 9) asm volatile("v_fma_f64 %0, %0, 1.0, %1" : "+v"(a[j]) : "v"(c));
      if (OP == 10) asm volatile("v_min_f64 %0, %0, %1" : "+v"(a[j]) : "v"(c));
      if (OP == 11) asm volatile("v_add_f32 %0, %0, %1" : "+v"(f[j]) : "v"((float)c));
      // single dependency chain (latency): the 8 instructions all update a[0]
      if (OP == 12) asm volatile("v_add_f64 %0, %0, %1" : "+v"(a[0]) : "v"(c));
      if (OP == 13) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a[0]) : "v"(m), "v"(c));
      if (OP == 15) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a[j]) : "v"(s), "v"(c));
      if (OP == 16) asm volatile("v_add_f64 %0, %0, %1" : "+v"(a[j]) : "v"(m));
      if (OP == 17) asm volatile("v_add_f64 %0, %0, %1" : "+v"(a[j]) : "s"(c));
      if (OP == 18) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(a[j]) : "v"(s));
      if (OP == 14) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f[0]) : "v"((float)m), "v"((float)c));
    }
  }
  double r = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) r += a[j] + f[j];
  if (r == 12345.678) out[0] = r;
}

template <int OP>
static int run(const char* name, int waves_per_simd, double* d) {
  int dev = 0, cus = 0;
  CHK(hipGetDevice(&dev));
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int blocks = cus * waves_per_simd;   // 256 threads = 4 waves = one per SIMD
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  k_rate<OP><<<blocks, 256>>>(d, 1.0);
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(a));
  const int reps = 5;
  for (int r = 0; r < reps; ++r) k_rate<OP><<<blocks, 256>>>(d, 1.0);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  const double instr_per_simd = (double)reps * waves_per_simd * ITERS * 8;
  const double rate = instr_per_simd / (ms * 1e-3);   // wave-instructions per second per SIMD
  printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"us\": %.1f, \"winstr_per_s_per_simd\": %.4g, "
         "\"cycles_per_winstr_at_2.4GHz\": %.2f}\n", name, waves_per_simd, ms * 1e3 / reps, rate, 2.4e9 / rate);
  return 0;
}

int main() {
  double* d;
  CHK(hipMalloc(&d, 64));
  for (int w : {1, 4}) {
    if (run<0>("v_add_f64", w, d) || run<1>("v_mul_f64", w, d) || run<2>("v_fma_f64", w, d) ||
        run<3>("v_max_f64", w, d) || run<4>("v_fma_f32", w, d) || run<5>("v_pk_fma_f32", w, d) ||
        run<6>("v_cvt_f64_f32", w, d) || run<7>("v_cndmask_b32", w, d) || run<8>("v_mov_b64", w, d) ||
        run<9>("v_fma_f64(x,1.0,c) as add", w, d) || run<10>("v_min_f64", w, d) || run<11>("v_add_f32", w, d) ||
        run<12>("v_add_f64 1-chain", w, d) || run<13>("v_fma_f64 1-chain", w, d) || run<14>("v_fma_f32 1-chain", w, d) ||
        run<15>("v_fma_f64(x,one_vgpr,c)", w, d) || run<16>("v_add_f64 +0.5", w, d) ||
        run<17>("v_add_f64 sgpr", w, d) || run<18>("v_mul_f64 x1.0", w, d))
      return 1;
  }
  CHK(hipFree(d));
  return 0;
}
