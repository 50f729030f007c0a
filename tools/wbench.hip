// Write-pattern microbenchmark for the [N, T, dof] f32 trajectory layout (k_traj_mfma's output):
// each env owns a contiguous run of RUN bytes; a wave serves a group of 32 envs and writes
// PIECE-byte pieces of every env's run (piece-major, as a tile loop does) or the group's region
// linearly (env-major).  Prints GB/s per pattern.  Standalone: hipcc -O3 --offload-arch=gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void k_piece(float* out, long long nenv, int run, int piece, int waves_per_group) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wpb = blockDim.x >> 6;
  const long long gw = (long long)blockIdx.x * wpb + w;
  const long long grp = gw / waves_per_group;
  const int sub = gw % waves_per_group;
  const long long e0 = grp * 32;
  if (e0 >= nenv) return;
  const int chunks = piece / 16, npieces = run / piece;
  const f32x4 v = {1.0f, 2.0f, 3.0f, 4.0f};
  for (int k = sub; k < npieces; k += waves_per_group)
    for (int idx = lane; idx < 32 * chunks; idx += 64) {
      const int je = idx / chunks, ch = idx - je * chunks;
      char* p = (char*)out + (e0 + je) * (long long)run + (long long)k * piece + 16 * ch;
      *(f32x4*)p = v;
    }
}

// the same pieces with their boundaries moved to 128-B lines of the output (the run's ends excepted):
// every line but a run's first / last is written whole by one piece
template <int ALIGN>
__global__ void k_piece_aligned(float* out, long long nenv, int run, int piece, int waves_per_group) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wpb = blockDim.x >> 6;
  const long long gw = (long long)blockIdx.x * wpb + w;
  const long long grp = gw / waves_per_group;
  const int sub = gw % waves_per_group;
  const long long e0 = grp * 32;
  if (e0 >= nenv) return;
  const int npieces = run / piece;
  const f32x4 v = {1.0f, 2.0f, 3.0f, 4.0f};
  for (int k = sub; k < npieces; k += waves_per_group)
    for (int je = 0; je < 32; ++je) {
      const long long S = (e0 + je) * (long long)run;
      auto bound = [&](int kk) -> long long {
        if (kk <= 0) return S;
        if (kk >= npieces) return S + run;
        return ALIGN ? (S + (long long)kk * piece + 127) & ~127LL : S + (long long)kk * piece;
      };
      const long long b0 = bound(k), b1 = bound(k + 1);
      for (long long off = b0 + 16 * lane; off < b1; off += 16 * 64) *(f32x4*)((char*)out + off) = v;
    }
}

template <int NT>
__global__ void k_linear(float* out, long long nenv, int run, int waves_per_group) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wpb = blockDim.x >> 6;
  const long long gw = (long long)blockIdx.x * wpb + w;
  const long long grp = gw / waves_per_group;
  const int sub = gw % waves_per_group;
  const long long e0 = grp * 32;
  if (e0 >= nenv) return;
  const long long bytes = 32LL * run;
  const f32x4 v = {1.0f, 2.0f, 3.0f, 4.0f};
  char* base = (char*)out + e0 * (long long)run;
  for (long long off = (long long)(sub * 64 + lane) * 16; off < bytes; off += 64LL * 16 * waves_per_group) {
    if (NT) __builtin_nontemporal_store(v, (f32x4*)(base + off));
    else *(f32x4*)(base + off) = v;
  }
}

// grid-stride fill: the whole buffer, consecutive lanes on consecutive 16-B chunks
__global__ void k_fill(float* out, long long chunks) {
  const f32x4 v = {1.0f, 2.0f, 3.0f, 4.0f};
  for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < chunks; q += (long long)gridDim.x * blockDim.x)
    ((f32x4*)out)[q] = v;
}

int main() {
  const long long nenv = 65536;
  const int run = 4000;   // T 200 x 5 dof x 4 B
  float* buf[2];
  for (int i = 0; i < 2; ++i) hipMalloc(&buf[i], nenv * run);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto timeit = [&](const char* name, int piece, int wpg, int wpb, int linear) {
    const long long groups = nenv / 32;
    const long long waves = groups * wpg;
    const int blocks = (int)((waves + wpb - 1) / wpb);
    float best = 1e30f;
    for (int rep = 0; rep < 6; ++rep) {
      hipEventRecord(a);
      for (int i = 0; i < 2; ++i) {
        if (linear == 1) hipLaunchKernelGGL(k_linear<0>, dim3(blocks), dim3(64 * wpb), 0, 0, buf[i], nenv, run, wpg);
        else if (linear == 2) hipLaunchKernelGGL(k_linear<1>, dim3(blocks), dim3(64 * wpb), 0, 0, buf[i], nenv, run, wpg);
        else if (linear == 3) hipLaunchKernelGGL(k_fill, dim3(blocks), dim3(64 * wpb), 0, 0, buf[i], nenv * run / 16);
        else if (linear == 4) hipLaunchKernelGGL(k_piece_aligned<1>, dim3(blocks), dim3(64 * wpb), 0, 0, buf[i], nenv, run, piece, wpg);
        else if (linear == 5) hipLaunchKernelGGL(k_piece_aligned<0>, dim3(blocks), dim3(64 * wpb), 0, 0, buf[i], nenv, run, piece, wpg);
        else hipLaunchKernelGGL(k_piece, dim3(blocks), dim3(64 * wpb), 0, 0, buf[i], nenv, run, piece, wpg);
      }
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (rep > 0 && ms < best) best = ms;
    }
    printf("{\"pattern\": \"%s\", \"piece\": %d, \"waves_per_group\": %d, \"waves_per_block\": %d, \"us\": %.1f, \"GBps\": %.0f}\n",
           name, piece, wpg, wpb, best * 1e3, 2.0 * nenv * run / (best * 1e-3) / 1e9);
  };
  timeit("linear", 0, 1, 4, 1);
  timeit("linear", 0, 8, 8, 1);
  timeit("linear_nt", 0, 1, 4, 2);
  timeit("linear_nt", 0, 8, 8, 2);
  timeit("fill_gridstride", 0, 1, 4, 3);   // blocks = groups / 4 = 512 x 256 threads
  timeit("fill_gridstride", 0, 8, 8, 3);   // 2048 x 512 threads
  timeit("fill_gridstride", 0, 1, 16, 3);  // 128 x 1024
  timeit("piece", 4000, 1, 4, 0);
  timeit("piece", 4000, 8, 8, 0);
  for (int pc : {400, 800}) {   // (whole 16-B chunks per piece)
    timeit("piece_per_env", pc, 8, 8, 5);
    timeit("piece_aligned", pc, 8, 8, 4);
    timeit("piece_per_env", pc, 1, 4, 5);
    timeit("piece_aligned", pc, 1, 4, 4);
  }
  return 0;
}
