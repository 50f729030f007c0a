// fgx_rng.h — numpy-exact reset randomness, on the device.
//
// The reference seeds each env with gymnasium seeding.np_random(seed) =
// np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed))) [EXT-H] and draws with
// Generator.uniform / Generator.choice (base_reacher.py:82, simple_reacher.py:87-92,
// hole_reacher.py:79-112).  This header restates those numpy algorithms bit-exactly:
//   SeedSequence(seed).generate_state(4, uint64)   (numpy/random/bit_generator.pyx)
//   PCG64 XSL-RR 128/64, set_seed, next64, buffered next32 (numpy/random/src/pcg64)
//   next_double = (next64 >> 11) * 2^-53; uniform(lo, hi) = lo + (hi - lo) * next_double
//   integers(0, 2) (choice of 2) = buffered_bounded_lemire_uint32(rng=1) = next32 >> 31
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fgx {

struct Pcg64 {
  unsigned __int128 state;
  unsigned __int128 inc;
  uint32_t has_u32;
  uint32_t u32;
};

__host__ __device__ inline uint32_t ss_hashmix(uint32_t value, uint32_t& hash_const) {
  value ^= hash_const;
  hash_const *= 0x931e8875u;   // MULT_A
  value *= hash_const;
  value ^= value >> 16;
  return value;
}

__host__ __device__ inline uint32_t ss_mix(uint32_t x, uint32_t y) {
  uint32_t r = 0xca01f9ddu * x - 0x4973f715u * y;   // MIX_MULT_L, MIX_MULT_R
  r ^= r >> 16;
  return r;
}

// SeedSequence(seed) with a non-negative integer seed (entropy words = little-endian u32
// limbs of the seed, at least one), pool_size 4; then generate_state(4, uint64).
__host__ __device__ inline void seedseq_state4(uint64_t seed, uint64_t out[4]) {
  uint32_t ent[2];
  int n_ent = 1;
  ent[0] = (uint32_t)seed;
  ent[1] = (uint32_t)(seed >> 32);
  if (ent[1] != 0u) n_ent = 2;
  uint32_t pool[4];
  uint32_t hc = 0x43b0d7e5u;   // INIT_A
  for (int i = 0; i < 4; ++i) pool[i] = ss_hashmix(i < n_ent ? ent[i] : 0u, hc);
  for (int s = 0; s < 4; ++s)
    for (int d = 0; d < 4; ++d)
      if (s != d) pool[d] = ss_mix(pool[d], ss_hashmix(pool[s], hc));
  uint32_t w[8];
  uint32_t hb = 0x8b51f9ddu;   // INIT_B
  for (int i = 0; i < 8; ++i) {
    uint32_t v = pool[i & 3];
    v ^= hb;
    hb *= 0x58f38dedu;         // MULT_B
    v *= hb;
    v ^= v >> 16;
    w[i] = v;
  }
  for (int k = 0; k < 4; ++k) out[k] = (uint64_t)w[2 * k] | ((uint64_t)w[2 * k + 1] << 32);
}

__host__ __device__ inline unsigned __int128 pcg_mult() {
  return ((unsigned __int128)2549297995355413924ULL << 64) | (unsigned __int128)4865540595714422341ULL;
}

__host__ __device__ inline void pcg_step(Pcg64& r) { r.state = r.state * pcg_mult() + r.inc; }

__host__ __device__ inline void pcg_seed(Pcg64& r, uint64_t seed) {
  uint64_t v[4];
  seedseq_state4(seed, v);
  unsigned __int128 initstate = ((unsigned __int128)v[0] << 64) | v[1];
  unsigned __int128 initseq = ((unsigned __int128)v[2] << 64) | v[3];
  r.state = 0;
  r.inc = (initseq << 1) | 1u;
  pcg_step(r);
  r.state += initstate;
  pcg_step(r);
  r.has_u32 = 0;
  r.u32 = 0;
}

__host__ __device__ inline uint64_t pcg_next64(Pcg64& r) {
  pcg_step(r);
  uint64_t hi = (uint64_t)(r.state >> 64), lo = (uint64_t)r.state;
  uint32_t rot = (uint32_t)(r.state >> 122);
  uint64_t x = hi ^ lo;
  return (x >> rot) | (x << ((64u - rot) & 63u));
}

__host__ __device__ inline uint32_t pcg_next32(Pcg64& r) {
  if (r.has_u32) {
    r.has_u32 = 0;
    return r.u32;
  }
  uint64_t n = pcg_next64(r);
  r.has_u32 = 1;
  r.u32 = (uint32_t)(n >> 32);
  return (uint32_t)(n & 0xffffffffu);
}

__host__ __device__ inline double pcg_next_double(Pcg64& r) {
  return (double)(pcg_next64(r) >> 11) * (1.0 / 9007199254740992.0);
}

// Generator.uniform(low, high): low + (high - low) * next_double
__host__ __device__ inline double rng_uniform(Pcg64& r, double low, double high) {
  double range = high - low;
  return low + range * pcg_next_double(r);
}

// Generator.choice([-1, 1]) -> integers(0, 2) -> Lemire on a buffered u32 with rng_excl = 2
__host__ __device__ inline int rng_choice_pm1(Pcg64& r) {
  uint32_t u = pcg_next32(r);
  return (u >> 31) ? 1 : -1;
}

}  // namespace fgx
