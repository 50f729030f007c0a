// Which SIMD / CU / XCD does each wave of a workgroup land on (HW_ID / XCC_ID hardware registers)?
// Prints a histogram: for workgroups of W waves, the SIMD of wave w (w = 0..W-1).
//   hipcc --offload-arch=gfx950 -O3 tools/wave_placement.hip -o /tmp/wave_placement && /tmp/wave_placement
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_where(unsigned* out, int spin) {
  // spin so that the workgroups of the grid are co-resident when sampled
  long long t0 = clock64();
  while (clock64() - t0 < spin) {}
  if ((threadIdx.x & 63) == 0) {
    unsigned hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));   // HW_REG_HW_ID (id 4), bits 0..31
    out[(blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64)] = hw;
  }
}

int main() {
  for (int W : {2, 4, 5, 8}) {
    const int blocks = 1024;
    unsigned* d;
    hipMalloc(&d, blocks * W * 4);
    hipLaunchKernelGGL(k_where, dim3(blocks), dim3(64 * W), 0, 0, d, 200000);
    std::vector<unsigned> h(blocks * W);
    hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    // gfx9 HW_ID: wave_id [3:0], simd_id [5:4], pipe_id [7:6], cu_id [11:8], sh_id [12], se_id [15:13]
    int hist[8][4] = {};
    int same_simd_pairs = 0;
    for (int b = 0; b < blocks; ++b)
      for (int w = 0; w < W; ++w) {
        const int simd = (h[b * W + w] >> 4) & 3;
        hist[w][simd]++;
        if (w >= 4 && simd == ((h[b * W + w - 4] >> 4) & 3)) same_simd_pairs++;
      }
    printf("W=%d\n", W);
    for (int w = 0; w < W; ++w) printf("  wave %d -> simd histogram %d %d %d %d\n", w, hist[w][0], hist[w][1], hist[w][2], hist[w][3]);
    if (W == 8) printf("  waves w and w+4 on the same SIMD: %d of %d\n", same_simd_pairs, blocks * 4);
    // first 6 blocks raw
    for (int b = 0; b < 6; ++b) {
      printf("  block %d:", b);
      for (int w = 0; w < W; ++w) { unsigned x = h[b * W + w]; printf(" [se%u cu%u simd%u wv%u]", (x >> 13) & 7, (x >> 8) & 15, (x >> 4) & 3, x & 15); }
      printf("\n");
    }
    hipFree(d);
  }
  return 0;
}
