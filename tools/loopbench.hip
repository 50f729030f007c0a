// What makes k_episode's sample loop slower than a plain f64 PD / Euler loop?  The same per-sample
// work as the metric kernel's fast blocks (5 joints, ProMP basis contraction on joint pairs, PD,
// clip, semi-implicit Euler, sum of squared actions, reward pushed into 8 pairwise slots), built
// up feature by feature; 65536 lanes = one wave per SIMD, 200 samples.  One JSON line per variant.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/loopbench.hip -o tools/loopbench
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("hip error %s\n", hipGetErrorString(e_)); return 1; } } while (0)

typedef float f32x2 __attribute__((ext_vector_type(2)));
constexpr int NL = 5, NB = 5, NLP = 3, SAMPLES = 200, KS = 8;

__device__ __forceinline__ double one64() {
  double o = 1.0;
  asm("" : "+s"(o));
  return o;
}

// V bit 0: adds as fma with an opaque SGPR 1.0; bit 1: desired state from the ProMP pair chain over
// an LDS table (else a cheap synthetic f32 recurrence); bit 2: reward into 8 pairwise slots (else
// one accumulator); bit 3: table rows through the constant address space (scalar loads)
template <int V>
__global__ __launch_bounds__(256) void k_loop(double* out, const float* tab_g, const float* wts, double pg, double dg,
                                              double dt) {
  __shared__ float tab[(SAMPLES + 4) * KS];
  for (int i = threadIdx.x; i < (SAMPLES + 4) * KS; i += blockDim.x) tab[i] = tab_g[i];
  __syncthreads();
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  auto add = [](double x, double y) { return (V & 1) ? __builtin_fma(x, one64(), y) : x + y; };
  auto sub = [](double x, double y) { return (V & 1) ? __builtin_fma(-y, one64(), x) : x - y; };
  double q[NL], qd[NL], acc[8];
  f32x2 w[NLP][NB], cur[NLP];
  float syn[NL];
#pragma unroll
  for (int d = 0; d < NL; ++d) { q[d] = 1e-3 * e + d; qd[d] = 0.0; syn[d] = 0.5f * (d + 1); }
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.0;
#pragma unroll
  for (int p = 0; p < NLP; ++p) {
#pragma unroll
    for (int j = 0; j < NB; ++j) w[p][j] = f32x2{wts[(2 * p) * NB + j], 2 * p + 1 < NL ? wts[(2 * p + 1) * NB + j] : 0.0f};
    cur[p] = f32x2{0.0f, 0.0f};
  }
  typedef const float __attribute__((address_space(4)))* cptr;
  const cptr ctab = (cptr)(uintptr_t)tab_g;
  for (int kb = 0; kb < SAMPLES; kb += 8) {
#pragma unroll
    for (int J = 0; J < 8; ++J) {
      const int k = kb + J;
      float pos[NL], vel[NL];
      if (V & 2) {
        float row[NB + 2], nrow[NB];
#pragma unroll
        for (int j = 0; j < NB + 2; ++j) row[j] = (V & 8) ? ctab[(k + 1) * KS + j] : tab[(k + 1) * KS + j];
#pragma unroll
        for (int j = 0; j < NB; ++j) nrow[j] = (V & 8) ? ctab[(k + 2) * KS + j] : tab[(k + 2) * KS + j];
#pragma unroll
        for (int p = 0; p < NLP; ++p) {
          f32x2 nx = {0.0f, 0.0f};
#pragma unroll
          for (int j = 0; j < NB; ++j) nx = __builtin_elementwise_fma((f32x2)nrow[j], w[p][j], nx);
          const f32x2 x = nx - cur[p];
          const f32x2 qq = x * row[NB + 1];
          const f32x2 er = __builtin_elementwise_fma(-qq, (f32x2)row[NB], x);
          const f32x2 vl = __builtin_elementwise_fma(er, (f32x2)row[NB + 1], qq);
          pos[2 * p] = cur[p].x;
          vel[2 * p] = vl.x;
          if (2 * p + 1 < NL) { pos[2 * p + 1] = cur[p].y; vel[2 * p + 1] = vl.y; }
          cur[p] = nx;
        }
      } else {
#pragma unroll
        for (int d = 0; d < NL; ++d) {
          const float nx = __builtin_fmaf(syn[d], 0.999f, 1e-3f * (float)k);
          pos[d] = syn[d];
          vel[d] = (nx - syn[d]) * 100.0f;
          syn[d] = nx;
        }
      }
      double ctrl = 0.0;
#pragma unroll
      for (int d = 0; d < NL; ++d) {
        const double u = add(pg * sub((double)pos[d], q[d]), dg * sub((double)vel[d], qd[d]));
        const double a = __builtin_fmin(__builtin_fmax(u, -1000.0), 1000.0);
        qd[d] = add(qd[d], dt * a);
        q[d] = add(q[d], dt * qd[d]);
        ctrl = (d == 0) ? a * a : add(ctrl, a * a);
      }
      if (V & 4) acc[J] = sub(acc[J], ctrl);
      else acc[0] = sub(acc[0], ctrl);
    }
  }
  double r = 0.0;
#pragma unroll
  for (int j = 0; j < 8; ++j) r += acc[j];
#pragma unroll
  for (int d = 0; d < NL; ++d) r += q[d];
  out[e] = r;
}

template <int V>
static int run(double* d, const float* tab, const float* w) {
  const int total = 65536, blocks = total / 256;
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  k_loop<V><<<blocks, 256>>>(d, tab, w, 0.6, 0.075, 0.01);
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(a));
  const int reps = 20;
  for (int r = 0; r < reps; ++r) k_loop<V><<<blocks, 256>>>(d, tab, w, 0.6, 0.075, 0.01);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  printf("{\"variant\": %d, \"fma_adds\": %d, \"promp_pairs\": %d, \"pairwise_slots\": %d, \"scalar_table\": %d, "
         "\"us\": %.2f}\n", V, V & 1, (V >> 1) & 1, (V >> 2) & 1, (V >> 3) & 1, ms * 1e3 / reps);
  return 0;
}

int main() {
  double* d;
  float *tab, *w;
  CHK(hipMalloc(&d, 65536 * sizeof(double)));
  CHK(hipMalloc(&tab, (SAMPLES + 4) * KS * sizeof(float)));
  CHK(hipMalloc(&w, NL * NB * sizeof(float)));
  float ht[(SAMPLES + 4) * KS], hw[NL * NB];
  for (int r = 0; r < SAMPLES + 4; ++r)
    for (int j = 0; j < KS; ++j) ht[r * KS + j] = j < NB ? 0.2f + 0.01f * ((r + j) % 7) : (j == NB ? 0.01f : 100.0f);
  for (int i = 0; i < NL * NB; ++i) hw[i] = 0.3f * ((i % 5) - 2);
  CHK(hipMemcpy(tab, ht, sizeof(ht), hipMemcpyHostToDevice));
  CHK(hipMemcpy(w, hw, sizeof(hw), hipMemcpyHostToDevice));
  for (int rep = 0; rep < 2; ++rep)
    if (run<0>(d, tab, w) || run<1>(d, tab, w) || run<2>(d, tab, w) || run<3>(d, tab, w) || run<4>(d, tab, w) ||
        run<6>(d, tab, w) || run<7>(d, tab, w) || run<15>(d, tab, w) || run<14>(d, tab, w))
      return 1;
  return 0;
}
