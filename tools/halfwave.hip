// Does a wave with half its lanes active issue faster on gfx950's SIMD-32 (one pass instead of
// two)?  The body is the metric kernel's per-sample f64 work (PD, clip, semi-implicit Euler,
// sum of squared actions for 5 joints, f32 -> f64 converts of a synthetic desired state), run by
// `lanes` active lanes per wave over a fixed total of 65536 lanes: 64 lanes -> 1024 waves (one
// per SIMD), 32 -> 2048 (two per SIMD), 16 -> 4096.  Prints one JSON line per configuration.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/halfwave.hip -o /tmp/halfwave && /tmp/halfwave
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("hip error %s\n", hipGetErrorString(e_)); return 1; } } while (0)

constexpr int NL = 5, SAMPLES = 200;

__global__ __launch_bounds__(256) void k_body(double* out, int lanes, long long total, float w0, double pg, double dg, double dt) {
  const int lane = threadIdx.x & 63, wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (lane >= lanes) return;
  const long long e = (long long)wave * lanes + lane;
  if (e >= total) return;
  double q[NL], qd[NL], acc = 0.0;
  float cur[NL];
#pragma unroll
  for (int d = 0; d < NL; ++d) { q[d] = 1e-3 * e + d; qd[d] = 0.0; cur[d] = w0 * (d + 1); }
  for (int k = 0; k < SAMPLES; ++k) {
    double ctrl = 0.0;
#pragma unroll
    for (int d = 0; d < NL; ++d) {
      const float nx = __builtin_fmaf(cur[d], 0.999f, 1e-3f * (float)k);
      const float vel = (nx - cur[d]) * 100.0f;
      const double u = pg * ((double)cur[d] - q[d]) + dg * ((double)vel - qd[d]);
      const double a = __builtin_fmin(__builtin_fmax(u, -1000.0), 1000.0);
      qd[d] = qd[d] + dt * a;
      q[d] = q[d] + dt * qd[d];
      ctrl = (d == 0) ? a * a : ctrl + a * a;
      cur[d] = nx;
    }
    acc = acc - ctrl;
  }
  double r = acc;
#pragma unroll
  for (int d = 0; d < NL; ++d) r += q[d];
  out[e] = r;
}

int main() {
  const long long total = 65536;
  double* d;
  CHK(hipMalloc(&d, total * sizeof(double)));
  for (int lanes : {64, 32, 16, 64, 32}) {
    const long long waves = (total + lanes - 1) / lanes;
    const int blocks = (int)((waves * 64 + 255) / 256);
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    k_body<<<blocks, 256>>>(d, lanes, total, 0.5f, 0.6, 0.075, 0.01);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(a));
    const int reps = 20;
    for (int r = 0; r < reps; ++r) k_body<<<blocks, 256>>>(d, lanes, total, 0.5f, 0.6, 0.075, 0.01);
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, a, b));
    printf("{\"lanes_per_wave\": %d, \"waves\": %lld, \"us\": %.2f}\n", lanes, waves, ms * 1e3 / reps);
  }
  CHK(hipFree(d));
  return 0;
}
