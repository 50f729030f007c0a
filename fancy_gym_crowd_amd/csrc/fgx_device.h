// fgx_device.h — device-side building blocks of the rollout engine (gfx950).
//
// Everything here is compiled with -ffp-contract=off: every f64/f32 expression rounds exactly
// like the reference's numpy expression it restates; fused multiply-adds appear only where
// they are written explicitly (__builtin_fma / __builtin_fmaf), i.e. the basis contraction
// (k-ordered f32 fma chain == f32-input MFMA numerics) and the OpenBLAS ddot orderings of
// np.linalg.norm / np.dot (verified against the reference's goldens).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>
#include <unordered_map>

#include "fgx_rng.h"
#include "fgx_trig.h"

namespace fgx {

// two f32 lanes per register pair: v_pk_{fma,mul,add}_f32 operands
typedef float f32x2 __attribute__((ext_vector_type(2)));
// read-only table memory in the constant address space: a wave-uniform address is loaded with
// s_load into SGPRs (the scalar cache), not per lane through LDS / VMEM
typedef const float __attribute__((address_space(4)))* cfloat_ptr;

// Host: a launch with more than 64 KB of dynamic LDS needs the kernel's limit raised first.  The
// limit is raised once per kernel (to the largest size asked for so far) and cached, so the
// per-step launches do not pay a hipFuncSetAttribute each.
inline hipError_t raise_lds_limit(const void* kernel, size_t lds) {
  if (lds <= 64 * 1024) return hipSuccess;
  int dev = 0;
  (void)hipGetDevice(&dev);
  static std::mutex mu;
  static std::unordered_map<const void*, size_t> raised[64];   // per device ordinal
  if (dev < 0 || dev >= 64) return hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  std::lock_guard<std::mutex> lock(mu);
  size_t& have = raised[dev][kernel];
  if (have >= lds) return hipSuccess;
  const hipError_t e = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e == hipSuccess) have = lds;
  return e;
}

constexpr int kMaxLinks = 8;
constexpr int kMaxObs = 3 * kMaxLinks + 5;
constexpr int kMaxBasis = 16;

enum : int { ENV_SIMPLE = 0, ENV_HOLE = 1, ENV_VIA = 2 };
enum : int { REW_SIMPLE = 0, REW_VEL_ACC = 1, REW_UNBOUNDED = 2 };
enum : int { SCHED_EVERY = 0, SCHED_AT = 1, SCHED_NORM_PERIOD = 2 };
enum : int { MP_NONE = 0, MP_PROMP = 1, MP_DMP = 2, MP_PRODMP = 3, MP_GIVEN = 4 };
enum : int { CTRL_PD = 0, CTRL_VEL = 1, CTRL_POS = 2 };
enum : int { VALID_TAU = 1, VALID_DELAY = 2, VALID_POS = 4, INVALID_OBS_ZEROS = 0, INVALID_OBS_CURRENT = 1 };

// Table layouts (row = absolute env step index i, see oracle/mp.py):
//   ProMP : [phi_0 .. phi_{nb-1}, dt32]                      stride nb + 1
//   DMP   : [psi_0 .. psi_{nb-1}, sdt]                       stride nb + 1
//   ProDMP: [pb_0 .. pb_nb, vb_0 .. vb_nb, y1, y2, dy1, dy2] stride 2 (nb + 1) + 4

// Flat POD copy of the resolved configuration, passed by value to every kernel.
struct DevCfg {
  int64_t N;
  int env, nl, random_start, allow_self, allow_wall;
  int mp, phase, nb, zs, zg, nbo /* num_basis_outside */, ctrl, T, max_steps, replan /* do_replanning */, max_plans, cond_desired, time_aware,
      return_context;
  int obs_dim;      // full env observation (3n+3 simple, 3n+4 hole)
  int full_dim;     // obs_dim + time_aware
  int out_dim;      // BB observation width (ctx_dim if return_context else full_dim)
  int n_params, rows, stride;
  int rand_width, rand_x, rand_depth;
  int rew_fct;      // HoleReacher reward function (REW_*)
  int learn_tau, learn_delay, sub_traj;   // per-env phase parameters at the front of params
  // replanning schedule: OR of sched_n clauses (replan != 0 iff sched_n > 0); sched_state: some
  // clause reads the observation (evaluated after every env step, no fast path)
  int sched_n, sched_state;
  int sched_kind[4], sched_k[4], sched_i0[4], sched_i1[4];
  double sched_mul[4], sched_div[4];
  int rand_via, rand_target;   // ViaPointReacher: via point / target sampled at reset
  int ctx_idx[kMaxObs + 1];
  double dt, rcp_dt, tau, act_lo, act_hi;
  double pg[kMaxLinks], dg[kMaxLinks];   // PD gains per joint (scalars broadcast)
  float act_lo32, act_hi32, dt32, rcp_dt32, tau32, rcp_tau32;
  double hole_w0, hole_d0, hole_x0, penalty, weights_scale, goal_scale, alpha;
  double via_x0, via_y0, tgt_x0, tgt_y0;
  double delay, alpha_phase, bandwidth;   // phase / basis generator (per-env tables)
  double bdt;                             // ProDMP basis generator dt (its precompute grid; = dt by default)
  float tau_lo32, tau_hi32, delay_lo32, delay_hi32;   // action-space bounds of tau / delay
  float ws32, gs32, alpha32, beta32;
  // trajectory validity (include/fgx.h FGX_VALID_*; only the logging k_episode reads these)
  int valid_flags, invalid_obs, invalid_term, invalid_trunc;
  float vtau_lo32, vtau_hi32, vdelay_lo32, vdelay_hi32;
  double invalid_reward;
  double vpos_lo[kMaxLinks], vpos_hi[kMaxLinks];
  // ProMP NaN-free wave guard (k_episode / k_episode_jl fast blocks): every |w| < wbound32 bounds
  // |pos| <= max_i sum_j |table_ij| |w_j| < 1e30 (the table carries weights_scale); set by fgx_create
  float wbound32;
};

// SoA env state, owned by the handle ([k][N] for per-link arrays).
struct DevState {
  double* q;       // [nl][N]
  double* qd;      // [nl][N]
  double* goal;    // [2][N]
  double* hole;    // [3][N]  HoleReacher x, width, depth | ViaPointReacher via x, via y, -
  double* aux;     // [3][N]  HoleReacher reward state: saved end effector x, y (unbounded),
                   //         collision distance (vel_acc)
  int32_t* steps;  // [N] env steps since reset (== TimeLimit elapsed == current_traj_steps)
  int32_t* plans;  // [N] plan_steps (black_box_wrapper.py:88,199)
  uint32_t* flags; // [N] bit0: qd holds an f32 array (velocity controller), bit1: has condition,
                   //     bit2: vel_acc reward function's sticky collision flag
  uint64_t* rng;   // [5][N]  state hi, state lo, inc hi, inc lo, (has_u32 << 32 | u32)
  float* cond;     // [2][nl][N] condition_on_desired pos / vel
  double* start;   // [N] _start_pos[0] (Env::sp)
  double* rew;     // [T][N] step rewards of the current BB step (direct envs with T > 128 only):
                   //        the exact numpy pairwise return for lengths 128 < L <= T
  const int32_t* plan_len;   // [N] per-env plan length (learned tau / sub-trajectories) or null
  const float* tables;
  // the same table column-major, [stride][tables_t_rows(rows)]: column j, row r at
  // j * RT + r + tables_t_pad(j, nb) (k_episode_jl's ProMP chunks load 8 consecutive rows of one
  // column with one 32-byte-aligned scalar load)
  const float* tables_t;
};

__host__ __device__ inline int tables_t_rows(int rows) { return (rows + 32 + 7) & ~7; }
// basis columns start their rows at offset 6 (a chunk reads rows k0 + 2 ..), the dt columns at 7
// (rows k0 + 1 ..): both land on multiples of 8 for k0 % 8 == 0
__host__ __device__ inline int tables_t_pad(int col, int nb) { return col < nb ? 6 : 7; }

struct Outputs {
  float* obs;        // [N, out_dim]
  double* ret;       // [N]
  uint8_t* term;     // [N]
  uint8_t* trunc;    // [N]
  int32_t* tlen;     // [N]
  float* final_obs;  // [N, out_dim]
  // info (black_box_wrapper.py:220-249), [N, T, ...]
  float* positions;
  float* velocities;
  double* step_actions;
  float* step_obs;
  double* step_rewards;
  uint8_t* is_collided;
  uint8_t* is_success;
  double* end_effector;
  double* reward_dist;
  double* reward_ctrl;
  long long* inner_steps;
  // info_level 2, SimpleReacher: the logging k_episode leaves the trigonometric and end-effector
  // components of the per-step observations to k_info_obs; it logs q per sample ([T][NL][N] f64) and
  // the episode's goal ([2][N] f64, before the auto-reset) for it (handle scratch, fgx_api.hip)
  double* qlog;
  double* gsave;
  int autoreset;
#ifdef FGX_STAMPS
  unsigned long long* stamps;   // diagnostics build only: per-wave section clocks (tools/stamps.py)
#endif
};

// Section clocks of one wave (diagnostics build, -DFGX_STAMPS): lane 0 of wave w stores the shader
// clock (s_memtime) at point i to stamps[w * 16 + i] with an ordinary vector store; points 6 and 7
// store s_memrealtime (kernel entry / exit), points 8..15 are further shader-clock sections.
#ifdef FGX_STAMPS
#define FGX_STAMP(o, e, i)                                                                \
  do {                                                                                    \
    const unsigned long long t_ = ((i) == 6 || (i) == 7) ? __builtin_amdgcn_s_memrealtime() \
                                                         : __builtin_readcyclecounter();  \
    if ((threadIdx.x & 63) == 0 && (o).stamps && ((e) >> 6) < 16384)                      \
      (o).stamps[((e) >> 6) * 16 + (i)] = t_;                                             \
  } while (0)
#else
#define FGX_STAMP(o, e, i) do { } while (0)
#endif

// The device inner-step counter (fgx_info.inner_steps, include/fgx.h): `sum` (the trajectory
// lengths of this wave's envs, already reduced) goes to the wave's line of FGX_INNER_SLOTS partial
// counters by one lane -- one device-scope atomic per wave, spread over the lines.
constexpr int kInnerSlots = 128, kInnerStride = 16;   // = FGX_INNER_SLOTS / FGX_INNER_STRIDE (fgx_api.hip)
__device__ __forceinline__ void count_inner(long long* base, long long sum, bool leader) {
  const unsigned w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (leader && sum != 0)
    atomicAdd((unsigned long long*)(base + (size_t)(w % kInnerSlots) * kInnerStride), (unsigned long long)sum);
}

// orders this wave's LDS writes before its later reads (and reads before later writes): LDS
// operations of one wave execute in order, so the compiler's ordering is all that is needed
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// workgroup barrier for an LDS handover between waves: this wave's LDS operations complete, then
// s_barrier; unlike __syncthreads no fence on global memory, so outstanding global stores are not
// waited for (vmcnt) — the storing waves keep their stores in flight across it
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ------------------------------------------------------------------ wave write-combining of info rows
// The logging k_episode writes the verbose-2 per-step arrays ([T, N] / [T, X, N], up to GBs per BB
// step).  InfoStage collects the wave's values of one sample (every row of every array) in the wave's
// LDS region, one slot of 64 lanes per row, and writes them back transposed: each lane stores 16
// contiguous bytes (4 f32 / 2 f64 envs), so one store instruction covers 4 f32 rows (or 2 f64 rows)
// of the wave's 64 envs = 1 KiB.  Slots: f32 [positions NL | velocities NL | step_obs full_dim],
// f64 [step_actions NL | step_rewards | end_effector x, y | reward_dist | reward_ctrl | q NL (qlog)],
// u8 [is_collided | is_success].  Each array's row block of the sample is a wave-uniform (SGPR)
// address and a lane's piece a 32-bit offset in it (global_store saddr form; fgx_step rejects
// per-step arrays for N >= 2^24).  With qlog (defer) the step_obs components k_info_obs writes (cos /
// sin of q, end effector - goal) are not stored here.
__host__ __device__ inline int stage_n32(int nl, int full_dim) { return 2 * nl + full_dim; }
__host__ __device__ inline int stage_n64(int nl) { return 2 * nl + 5; }
__host__ __device__ inline size_t stage_wave_bytes(int nl, int full_dim) {
  return (size_t)stage_n64(nl) * 512 + (size_t)stage_n32(nl, full_dim) * 256 + 128;
}
__host__ __device__ inline size_t stage_tab_offset(size_t tab_floats) { return (tab_floats * 4 + 15) & ~(size_t)15; }

// a wave-uniform global address as SGPRs, typed in the global address space: a generic pointer
// rebuilt from integers would make every store through it a FLAT store, which also counts in
// lgkmcnt, so that the next LDS wait of the wave would wait for the global stores as well
typedef __attribute__((address_space(1))) char gchar;
template <typename T>
__device__ __forceinline__ gchar* uniform_ptr(T* p) {
  const uint64_t a = (uint64_t)p;
  return (gchar*)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32)) << 32) |
                  (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a));
}

template <int NL>
struct InfoStage {
  static constexpr int N64 = 2 * NL + 5;
  double* d;       // [N64][64]
  float* f;        // [n32][64]
  uint8_t* b;      // [2][64]
  int64_t N, e0;
  int lane, n32, nval, full_dim;
  bool any;        // some info array is written
  bool full;       // 64 envs, rows 16-B aligned (N % 4 == 0): transposed 16-B pieces
  bool defer;      // SimpleReacher observation trigonometry left to k_info_obs (o.qlog)
  bool plan_rows;  // positions / velocities are this kernel's (not a given plan)

  // region: the block's staging area (after the basis table); e: the lane's env (< N)
  __device__ __forceinline__ void init(const DevCfg& c, const Outputs& o, char* region, int64_t e, bool plan) {
    init_at(c, o, region + (size_t)(threadIdx.x >> 6) * stage_wave_bytes(NL, c.full_dim), e, plan);
  }
  // the staging slot at w (k_episode_v2h: two slots per dynamics wave, flushed by a partner wave)
  __device__ __forceinline__ void rebase(char* w) {
    d = (double*)w;
    f = (float*)(w + N64 * 512);
    b = (uint8_t*)(w + N64 * 512 + n32 * 256);
  }
  __device__ __forceinline__ void init_at(const DevCfg& c, const Outputs& o, char* w, int64_t e, bool plan) {
    lane = (int)(threadIdx.x & 63);
    full_dim = c.full_dim;
    n32 = stage_n32(NL, c.full_dim);
    rebase(w);
    N = c.N;
    e0 = e - lane;
    nval = (int)min((int64_t)64, N - e0);
    full = nval == 64 && (N & 3) == 0;
    any = o.positions || o.step_actions || o.step_obs || o.step_rewards || o.is_collided || o.end_effector ||
          o.reward_dist;
    defer = o.qlog != nullptr;
    plan_rows = plan;
  }
  // the lane's value of slot s of the current sample
  __device__ __forceinline__ void pos(int dd, float x) { f[dd * 64 + lane] = x; }
  __device__ __forceinline__ void vel(int dd, float x) { f[(NL + dd) * 64 + lane] = x; }
  __device__ __forceinline__ float* obs_row() { return f + 2 * NL * 64 + lane; }   // element stride 64
  __device__ __forceinline__ void act(int dd, double x) { d[dd * 64 + lane] = x; }
  __device__ __forceinline__ void rew(double x) { d[NL * 64 + lane] = x; }
  __device__ __forceinline__ void ee(double x, double y) { d[(NL + 1) * 64 + lane] = x; d[(NL + 2) * 64 + lane] = y; }
  __device__ __forceinline__ void rdc(double x, double y) { d[(NL + 3) * 64 + lane] = x; d[(NL + 4) * 64 + lane] = y; }
  __device__ __forceinline__ void flags(uint8_t x, uint8_t y) { b[lane] = x; b[64 + lane] = y; }
  __device__ __forceinline__ void ql(int dd, double x) { d[(NL + 5 + dd) * 64 + lane] = x; }

  // components c0..X-1 (at most MAXX) of sample k of the [T, X, N] array A from the staging slots
  // st[comp * 64 ..]; skip(comp): not this kernel's
  template <typename T, int MAXX, typename Skip>
  __device__ __forceinline__ void rows(T* A, int X, int c0, const T* st, uint32_t k, Skip skip) const {
    constexpr int PER = 16 / (int)sizeof(T);   // envs per lane piece
    constexpr int LPR = 64 / PER;              // lanes per row piece
    constexpr int RPI = 64 / LPR;              // rows per store instruction
    gchar* rb = uniform_ptr(A + (uint64_t)k * (uint64_t)X * (uint64_t)N);   // the sample's row block
    if (full) {
      typedef T V __attribute__((ext_vector_type(PER)));
      const int q = lane % LPR, r = lane / LPR;
#pragma unroll
      for (int c = 0; c < MAXX; c += RPI) {
        if (c + c0 >= X) break;
        const int comp = c0 + c + r;
        const V x = *(const V*)(st + comp * 64 + PER * q);
        if (comp < X && !skip(comp))
          *(__attribute__((address_space(1))) V*)(rb + (uint32_t)(((uint32_t)comp * (uint32_t)N +
                                                                   (uint32_t)(e0 + PER * q)) * sizeof(T))) = x;
      }
    } else {   // partial last wave (its lanes past N have left the kernel) or N % 4 != 0: own element
      for (int comp = c0; comp < X; ++comp)
        if (!skip(comp))
          *(__attribute__((address_space(1))) T*)(rb + (uint32_t)(((uint32_t)comp * (uint32_t)N +
                                                                   (uint32_t)(e0 + lane)) * sizeof(T))) =
              st[comp * 64 + lane];
    }
  }

  // write the staged rows of sample kk (wave-uniform); every lane of the wave's envs active
  __device__ __forceinline__ void flush(int kk, const Outputs& o) {
    if (!any) return;
    wave_lds_sync();
    const uint32_t k = (uint32_t)kk;
    auto none = [](int) { return false; };
    if (o.positions && plan_rows) {
      rows<float, NL>(o.positions, NL, 0, f, k, none);
      rows<float, NL>(o.velocities, NL, 0, f + NL * 64, k, none);
    }
    if (o.step_obs) {
      const float* so = f + 2 * NL * 64;
      if (defer)   // qd, steps, time: components 2 NL .. (cos / sin of q and the end effector: k_info_obs)
        rows<float, kMaxObs + 1 - (2 * NL & ~3)>(o.step_obs, full_dim, 2 * NL & ~3, so, k,
                                                 [](int p) { return p < 2 * NL || p == 3 * NL || p == 3 * NL + 1; });
      else
        rows<float, kMaxObs + 1>(o.step_obs, full_dim, 0, so, k, none);
    }
    if (o.step_actions) rows<double, NL>(o.step_actions, NL, 0, d, k, none);
    if (o.step_rewards) rows<double, 1>(o.step_rewards, 1, 0, d + NL * 64, k, none);
    if (o.end_effector) rows<double, 2>(o.end_effector, 2, 0, d + (NL + 1) * 64, k, none);
    if (o.reward_dist) {
      rows<double, 1>(o.reward_dist, 1, 0, d + (NL + 3) * 64, k, none);
      rows<double, 1>(o.reward_ctrl, 1, 0, d + (NL + 4) * 64, k, none);
    }
    if (o.qlog) rows<double, NL>(o.qlog, NL, 0, d + (NL + 5) * 64, k, none);
    if (o.is_collided) {   // [T, N] u8 rows: lanes 0-15 is_collided, 16-31 is_success, 4 envs each
      gchar* rc = uniform_ptr(o.is_collided + (uint64_t)k * (uint64_t)N);
      gchar* rs = uniform_ptr(o.is_success + (uint64_t)k * (uint64_t)N);
      typedef __attribute__((address_space(1))) uint32_t gu32;
      if (full) {
        if (lane < 16) *(gu32*)(rc + (uint32_t)(e0 + 4 * lane)) = *(const uint32_t*)(b + 4 * lane);
        else if (lane < 32) *(gu32*)(rs + (uint32_t)(e0 + 4 * (lane - 16))) = *(const uint32_t*)(b + 64 + 4 * (lane - 16));
      } else {
        rc[(uint32_t)(e0 + lane)] = (char)b[lane];
        rs[(uint32_t)(e0 + lane)] = (char)b[64 + lane];
      }
    }
    wave_lds_sync();
  }
};

// ------------------------------------------------------------------ wave reductions (all 64 lanes active)
__device__ __forceinline__ int wave_min(int x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x = min(x, __shfl_xor(x, off, 64));
  return __builtin_amdgcn_readfirstlane(x);
}
__device__ __forceinline__ int wave_max(int x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x = max(x, __shfl_xor(x, off, 64));
  return __builtin_amdgcn_readfirstlane(x);
}
// The same on the joint-lane kernels' prologue (all 64 lanes active there, lone waves at the shard
// sizes): within each row of 16 lanes by DPP (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror,
// row_mirror: VALU, no LDS round trip), then the four rows' values by readlane on the scalar unit;
// __shfl_xor lowers to a chain of six ds_bpermute round trips, ~0.6 k cycles for a lone wave
// (A/B, profiles/r03_shard_ab_s16.jsonl: jl 8192 envs 24.1 -> 23.8 us; k_episode keeps the shuffles,
// whose one reduction measured 0.7% faster there).
template <typename Op>
__device__ __forceinline__ int wave_reduce_dpp(int x, Op op) {
  x = op(x, __builtin_amdgcn_update_dpp(x, x, 0xB1, 0xF, 0xF, false));
  x = op(x, __builtin_amdgcn_update_dpp(x, x, 0x4E, 0xF, 0xF, false));
  x = op(x, __builtin_amdgcn_update_dpp(x, x, 0x141, 0xF, 0xF, false));
  x = op(x, __builtin_amdgcn_update_dpp(x, x, 0x140, 0xF, 0xF, false));
  return op(op(__builtin_amdgcn_readlane(x, 0), __builtin_amdgcn_readlane(x, 16)),
            op(__builtin_amdgcn_readlane(x, 32), __builtin_amdgcn_readlane(x, 48)));
}
__device__ __forceinline__ int wave_min_dpp(int x) { return wave_reduce_dpp(x, [](int a, int b) { return min(a, b); }); }
__device__ __forceinline__ int wave_max_dpp(int x) { return wave_reduce_dpp(x, [](int a, int b) { return max(a, b); }); }
// the partner lane's value in lane pairs (2i, 2i + 1): DPP quad_perm [1, 0, 3, 2]; both lanes of a
// pair are always active together (k_episode_pair)
__device__ __forceinline__ int pair_swap32(int x) { return __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false); }
__device__ __forceinline__ double pair_swap(double x) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(x);
  const unsigned lo = (unsigned)pair_swap32((int)(unsigned)b), hi = (unsigned)pair_swap32((int)(unsigned)(b >> 32));
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ bool pair_or(bool x) { return ((int)x | pair_swap32((int)x)) != 0; }
// min of x in [0, 65535] over the ACTIVE lanes (divergent code allowed): 16 ballots fix the bits from
// the top, m keeps the minimum's bits above b; wave-uniform result
__device__ __forceinline__ int wave_min_active(int x) {
  int m = 0;
#pragma unroll
  for (int b = 15; b >= 0; --b)
    if (__ballot(((x ^ m) >> b) == 0) == 0) m |= 1 << b;
  return m;
}

// ------------------------------------------------------------------ exact small helpers
__device__ __forceinline__ double np_max(double x, double lo) { return (x != x) ? x : (x > lo ? x : lo); }
__device__ __forceinline__ double np_min(double x, double hi) { return (x != x) ? x : (x < hi ? x : hi); }
__device__ __forceinline__ float np_maxf(float x, float lo) { return (x != x) ? x : (x > lo ? x : lo); }
__device__ __forceinline__ float np_minf(float x, float hi) { return (x != x) ? x : (x < hi ? x : hi); }

// np.clip(x, lo, hi) = minimum(maximum(x, lo), hi) with NaN propagation (umath clip)
__device__ __forceinline__ double np_clip(double x, double lo, double hi) {
  const double y = __builtin_fmin(__builtin_fmax(x, lo), hi);
  return (x != x) ? x : y;
}
__device__ __forceinline__ float np_clipf(float x, float lo, float hi) {
  const float y = __builtin_fminf(__builtin_fmaxf(x, lo), hi);
  return (x != x) ? x : y;
}

// Correctly rounded f32 x / d given r = RN(1/d) (Markstein: q = RN(x r), e = x - q d exact by
// fma, RN(q + e r) == RN(x / d)); three instructions instead of the IEEE division sequence.
// Exactness for the divisors the engine uses (the dt32 / tau32 table values) is checked by
// tests/test_mp_structure.py::test_division_by_reciprocal_is_exact.
__device__ __forceinline__ float div_rcp(float x, float d, float r) {
  const float q = x * r;
  const float e = __builtin_fmaf(-q, d, x);
  return __builtin_fmaf(e, r, q);
}

// f64 x + y and x - y issued as v_fma_f64 with a multiplier of 1.0 the compiler cannot see
// through: bit-identical to the add (x * 1 is exact, one rounding; signed zeros, infinities and
// NaN-ness as the add), but a lone wave issues v_fma_f64 every ~6 cycles against ~9 for v_add_f64
// (profiles/r01_valu_rates_operands.jsonl: "v_fma_f64(x,one_vgpr,c)" vs "v_add_f64").
__device__ __forceinline__ double one64() {
  double o = 1.0;
  asm("" : "+s"(o));
  return o;
}
__device__ __forceinline__ double fadd(double x, double y) { return __builtin_fma(x, one64(), y); }
__device__ __forceinline__ double fsub(double x, double y) { return __builtin_fma(-y, one64(), x); }

__device__ __forceinline__ double div_rcp64(double x, double d, double r) {
  const double q = x * r;
  const double e = __builtin_fma(-q, d, x);
  return __builtin_fma(e, r, q);
}

// np.sum of NL values v(0), ..., v(NL - 1) in numpy's pairwise_sum order (umath loops_utils.h):
// a left-to-right loop for NL < 8 (its leading 0 + v(0) is v(0) for the engine's summands, squares
// that are never -0), for NL = 8 eight accumulators combined as ((r0 + r1) + (r2 + r3)) +
// ((r4 + r5) + (r6 + r7)).  add: the two-operand add (fadd for the f64 issue-rate form).
template <int NL, typename T, typename V, typename Add>
__device__ __forceinline__ T np_sum(V v, Add add) {
  static_assert(NL >= 1 && NL <= 8, "n_links in 1..8");
  if constexpr (NL < 8) {
    T s = v(0);
#pragma unroll
    for (int d = 1; d < NL; ++d) s = add(s, v(d));
    return s;
  } else {
    return add(add(add(v(0), v(1)), add(v(2), v(3))), add(add(v(4), v(5)), add(v(6), v(7))));
  }
}

// np.linalg.norm of a 2-vector == sqrt(ddot) == sqrt(fma(y, y, x*x)) (OpenBLAS order)
__device__ __forceinline__ double norm2(double x, double y) { return __builtin_sqrt(__builtin_fma(y, y, x * x)); }

__device__ __forceinline__ bool ccw(double ax, double ay, double bx, double by, double cx, double cy) {
  return (cy - ay) * (bx - ax) - (by - ay) * (cx - ax) > 1e-12;   // classic_control/utils.py:1-2
}

// numpy pairwise summation (np.sum of a length-L f64 vector, L <= 256) done online: exact for
// L <= 128, and for 128 < L <= 256 when split == (L/2) & ~7 (the caller knows L in advance).
struct PairwiseSum {
  double a[8], t;       // single-level state (valid for L <= 128)
  double b[8], u;       // second-half state (t >= split)
  double first;
  __device__ __forceinline__ static double comb(const double* r) {
    return ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  }
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int j = 0; j < 8; ++j) { a[j] = 0.0; b[j] = 0.0; }
    t = 0.0; u = 0.0; first = 0.0;
  }
  __device__ __forceinline__ static void push(double* r, double& tail, int pos, double v) {
    const int j = pos & 7;
    const int ju = __builtin_amdgcn_readfirstlane(j);
    if (__ballot(j != ju) == 0) {
      // the sample index is the same in every active lane (k_episode's generic loop): a scalar
      // branch picks the slot, no per-lane select chain over the 8 accumulators
      switch (ju) {
#define FGX_PUSH_SLOT(Q) case Q: r[Q] = (pos < 8) ? v : r[Q] + v; break;
        FGX_PUSH_SLOT(0) FGX_PUSH_SLOT(1) FGX_PUSH_SLOT(2) FGX_PUSH_SLOT(3)
        FGX_PUSH_SLOT(4) FGX_PUSH_SLOT(5) FGX_PUSH_SLOT(6) FGX_PUSH_SLOT(7)
#undef FGX_PUSH_SLOT
      }
      if (ju == 7) tail = comb(r);
      else tail = tail + v;
    } else {
      // runtime j: select-chain keeps r[] in registers
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (q == j) r[q] = (pos < 8) ? v : r[q] + v;
      if (j == 7) tail = comb(r);
      else tail = tail + v;
    }
  }
  // Unrolled fast loop: compile-time slot J == k & 7 and a block-uniform phase PH (bit 0: the
  // sample is in [0, 128), bit 1: in [split, T)).  The accumulators start at 0, so 0 + v == v
  // replaces numpy's first-block copy (only the sign of an all-zero partial sum can differ).
  // Fast blocks are always complete, so the running tails are not needed inside them: the
  // caller sets t = comb(a), u = comb(b) after the fast loop (sync_tails).
  template <int J, int PH>
  __device__ __forceinline__ void add_fast(double v) {
    if (PH & 1) a[J] = fadd(a[J], v);
    if (PH & 2) b[J] = fadd(b[J], v);
  }
  // The same with the value given as its negation c (SimpleReacher fast blocks push the reward
  // 0 - ctrl as acc - ctrl, one instruction less: equal because no accumulator is ever -0 — they
  // start at +0 and 0 - ctrl is never -0 — so acc + (0 - ctrl) and acc - ctrl round the same sum)
  template <int J, int PH>
  __device__ __forceinline__ void sub_fast(double c) {
    if (PH & 1) a[J] = fsub(a[J], c);
    if (PH & 2) b[J] = fsub(b[J], c);
  }
  template <int J, int PH>
  __device__ __forceinline__ void sub_partial(double c) {
    if (PH & 1) { a[J] = fsub(a[J], c); t = fsub(t, c); }
    if (PH & 2) { b[J] = fsub(b[J], c); u = fsub(u, c); }
  }
  // A partial block (fewer than 8 samples, slots J < 7, after sync_tails): the running tail
  // follows each push as numpy's sequential remainder would (push() with j != 7).
  template <int J, int PH>
  __device__ __forceinline__ void add_partial(double v) {
    if (PH & 1) { a[J] = fadd(a[J], v); t = fadd(t, v); }
    if (PH & 2) { b[J] = fadd(b[J], v); u = fadd(u, v); }
  }
  __device__ __forceinline__ void sync_tails() {
    t = comb(a);
    u = comb(b);
  }
  __device__ __forceinline__ void add(int k, double v, int split) {
    if (split > 0 && k == split) first = comb(a);   // blocks [0, split) only
    if (k < 128) push(a, t, k, v);
    if (split > 0 && k >= split) push(b, u, k - split, v);
  }
  __device__ __forceinline__ double result(int L, int split) const {
    if (L <= 128 || split == 0) return t;
    return first + u;
  }
};

// numpy pairwise_sum (umath loops_utils.h) over a[0], a[st], ..., a[(n-1) st], n <= 256
__device__ inline double pairwise_strided(const double* a, int64_t st, int n) {
  auto block = [&](int lo, int m) -> double {
    if (m < 8) {
      double r = 0.0;
      for (int i = 0; i < m; ++i) r = r + a[(lo + i) * st];
      return r;
    }
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = a[(lo + j) * st];
    int i = 8;
    for (; i < m - (m % 8); i += 8)
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = r[j] + a[(lo + i + j) * st];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < m; ++i) res = res + a[(lo + i) * st];
    return res;
  };
  if (n <= 128) return block(0, n);
  int n2 = n / 2;
  n2 -= n2 % 8;
  return block(0, n2) + block(n2, n - n2);
}

// ------------------------------------------------------------------ RNG state load/store
__device__ __forceinline__ Pcg64 load_rng(const uint64_t* rng, int64_t N, int64_t e) {
  Pcg64 r;
  r.state = ((unsigned __int128)rng[e] << 64) | rng[N + e];
  r.inc = ((unsigned __int128)rng[2 * N + e] << 64) | rng[3 * N + e];
  const uint64_t b = rng[4 * N + e];
  r.has_u32 = (uint32_t)(b >> 32);
  r.u32 = (uint32_t)b;
  return r;
}

__device__ __forceinline__ void store_rng(uint64_t* rng, int64_t N, int64_t e, const Pcg64& r) {
  rng[e] = (uint64_t)(r.state >> 64);
  rng[N + e] = (uint64_t)r.state;
  rng[2 * N + e] = (uint64_t)(r.inc >> 64);
  rng[3 * N + e] = (uint64_t)r.inc;
  rng[4 * N + e] = ((uint64_t)r.has_u32 << 32) | r.u32;
}

// ------------------------------------------------------------------ one env in registers
template <int NL>
struct Env {
  double q[NL], qd[NL];
  double gx, gy;
  double hx, hw, hd;     // HoleReacher hole | ViaPointReacher via point (hx, hw)
  double ex, ey, cd;     // HoleReacher reward-function state (aux)
  double sp;             // _start_pos[0] (base_reacher.py:81-86): the first joint a non-random reset
                         // restores; a random reset draws it and keeps it
  int steps;
  uint32_t flags;
  // forward kinematics (base_reacher.py:95-103): joints[k+1] = cumsum of (cos, sin)(cumsum q)
  double jx[NL + 1], jy[NL + 1];
  double c[NL], s[NL];   // cos/sin of the cumulative angles

  __device__ __forceinline__ void fk() {
    double ang = 0.0, x = 0.0, y = 0.0;
    jx[0] = 0.0; jy[0] = 0.0;
#pragma unroll
    for (int k = 0; k < NL; ++k) {
      ang = (k == 0) ? q[0] : ang + q[k];
      double sn, cs;
      fgx_sincos(ang, &sn, &cs);
      c[k] = cs; s[k] = sn;
      x = (k == 0) ? cs : x + cs;
      y = (k == 0) ? sn : y + sn;
      jx[k + 1] = 0.0 + x;
      jy[k + 1] = 0.0 + y;
    }
  }
  // the same FK given cos / sin of the cumulative angles (computed elsewhere with the same sincos of
  // the same angles, e.g. one joint per lane in k_episode_jl)
  __device__ __forceinline__ void fk_given(const double* cs, const double* sn) {
    double x = 0.0, y = 0.0;
    jx[0] = 0.0; jy[0] = 0.0;
#pragma unroll
    for (int k = 0; k < NL; ++k) {
      c[k] = cs[k]; s[k] = sn[k];
      x = (k == 0) ? cs[k] : x + cs[k];
      y = (k == 0) ? sn[k] : y + sn[k];
      jx[k + 1] = 0.0 + x;
      jy[k + 1] = 0.0 + y;
    }
  }

  // reset draws (simple_reacher.py:46-54,85-96; hole_reacher.py:60-112; base_reacher.py:73-93)
  // rs: random_start of this reset (the constructor's, or reset(options={'random_start': ...}),
  // base_reacher.py:77-80)
  __device__ __forceinline__ void first_joint(Pcg64& r, bool rs) {
    if (rs) {
      const double lo = M_PI / 4, hi = 3 * M_PI / 4;
      q[0] = rng_uniform(r, lo, hi);
      sp = q[0];
    } else {
      q[0] = sp;
    }
#pragma unroll
    for (int k = 1; k < NL; ++k) q[k] = 0.0;
#pragma unroll
    for (int k = 0; k < NL; ++k) qd[k] = 0.0;
    steps = 0;
    flags = 0;
  }

  __device__ __forceinline__ void goal_sample(const DevCfg& cf, Pcg64& r) {
    if (!cf.rand_target) {   // SimpleReacherEnv(target=...) (simple_reacher.py:93-94): no draws
      gx = cf.tgt_x0; gy = cf.tgt_y0;
      return;
    }
    const double total = (double)NL;    // np.sum(link_lengths), unit links
    double g0 = total, g1 = total;
    while (norm2(g0, g1) >= total) {
      g0 = rng_uniform(r, -total, total);
      g1 = rng_uniform(r, -total, total);
    }
    gx = g0; gy = g1;
  }

  __device__ __forceinline__ void hole_sample(const DevCfg& cf, Pcg64& r) {
    const double w = cf.rand_width ? rng_uniform(r, 0.15, 0.5) : cf.hole_w0;
    double x;
    if (cf.rand_x) {
      const int side = rng_choice_pm1(r);
      x = (double)side * rng_uniform(r, w / 2, 3.5);
    } else {
      x = cf.hole_x0;
    }
    const double d = cf.rand_depth ? rng_uniform(r, 1.0, 1.0) : cf.hole_d0;
    hx = x; hw = w; hd = d;
    gx = x; gy = -d;
  }

  // viapoint_reacher.py:56-77: via point in the disk of radius L/2, target in the annulus
  // (L/2, L) by rejection (L = n_links, unit links); fixed values when configured
  __device__ __forceinline__ void via_sample(const DevCfg& cf, Pcg64& r) {
    const double total = (double)NL;
    if (cf.rand_via) {
      double v0 = total, v1 = total;
      while (norm2(v0, v1) >= 0.5 * total) {
        v0 = rng_uniform(r, -0.5 * total, 0.5 * total);
        v1 = rng_uniform(r, -0.5 * total, 0.5 * total);
      }
      hx = v0; hw = v1;
    } else {
      hx = cf.via_x0; hw = cf.via_y0;
    }
    if (cf.rand_target) {
      double g0 = total, g1 = total;
      while (norm2(g0, g1) >= total || norm2(g0, g1) <= 0.5 * total) {
        g0 = rng_uniform(r, -total, total);
        g1 = rng_uniform(r, -total, total);
      }
      gx = g0; gy = g1;
    } else {
      gx = cf.tgt_x0; gy = cf.tgt_y0;
    }
    hd = 0.0;
  }

  // seeded: reseed-only semantics (the discarded pre-seed goal draw has no effect);
  // unseeded: continue the stream exactly as the reference's reset() does.
  // SimpleReacher and ViaPointReacher sample their goal(s), reset, sample again, reset again
  // (simple_reacher.py:46-54, viapoint_reacher.py:46-54).
  __device__ __forceinline__ void reset(const DevCfg& cf, Pcg64& r, bool seeded, uint64_t seed) {
    reset(cf, r, seeded, seed, cf.random_start != 0);
  }
  __device__ __forceinline__ void reset(const DevCfg& cf, Pcg64& r, bool seeded, uint64_t seed, bool rs) {
    if (cf.env != ENV_HOLE) {
      const bool via = (cf.env == ENV_VIA);
      if (!via) { hx = 0.0; hw = 0.0; hd = 0.0; }   // unused by SimpleReacher: keep the state defined
      if (seeded) {
        pcg_seed(r, seed);
        first_joint(r, rs);
        if (via) via_sample(cf, r); else goal_sample(cf, r);
        pcg_seed(r, seed);
        first_joint(r, rs);
      } else {
        if (via) via_sample(cf, r); else goal_sample(cf, r);
        first_joint(r, rs);
        if (via) via_sample(cf, r); else goal_sample(cf, r);
        first_joint(r, rs);
      }
      ex = ey = cd = 0.0;
    } else {
      if (seeded) pcg_seed(r, seed);
      hole_sample(cf, r);
      first_joint(r, rs);
      cd = 0.0;   // reward_function.reset() (the saved end effector is rewritten before use)
      ex = ey = 0.0;
    }
    fk_fresh();
  }
  // fk() of a freshly reset arm: q = [q0, +0, ..., +0] makes every cumulative angle q0 exactly
  // (q0 + 0.0 == q0: q0 is never -0), so one sincos serves all links; the running sums are fk()'s
  __device__ __forceinline__ void fk_fresh() {
    double sn, cs;
    fgx_sincos(q[0], &sn, &cs);
    double x = 0.0, y = 0.0;
    jx[0] = 0.0; jy[0] = 0.0;
#pragma unroll
    for (int k = 0; k < NL; ++k) {
      c[k] = cs; s[k] = sn;
      x = (k == 0) ? cs : x + cs;
      y = (k == 0) ? sn : y + sn;
      jx[k + 1] = 0.0 + x;
      jy[k + 1] = 0.0 + y;
    }
  }

  // ---------------------------------------------------------------- collisions (HoleReacher)
  __device__ __forceinline__ bool self_collision() const {
#pragma unroll
    for (int k = 0; k < NL; ++k)
      if (q[k] > M_PI || q[k] < -M_PI) return true;   // base_reacher.py:38-39,111
    bool hit = false;
#pragma unroll
    for (int i = 0; i < NL; ++i)
#pragma unroll
      for (int j = i + 2; j < NL; ++j) {
        const double ax = jx[i], ay = jy[i], bx = jx[i + 1], by = jy[i + 1];
        const double cx = jx[j], cy = jy[j], dx = jx[j + 1], dy = jy[j + 1];
        hit |= (ccw(ax, ay, cx, cy, dx, dy) != ccw(bx, by, cx, cy, dx, dy)) &&
               (ccw(ax, ay, bx, by, cx, cy) != ccw(ax, ay, bx, by, dx, dy));
      }
    return hit;
  }

  // hole_reacher.py:126-179 (_get_line_points, check_wall_collision).  Points of link k:
  // p_j = (c_k*lin_j + jx_k, s_k*lin_j + jy_k), j = 0..99, with p_0 = joint k and p_99 = joint k+1
  // exactly.  Both coordinates are monotone in j (lin_j increases and rounding is monotone), so every
  // atomic test (px < left, py < 0, ...) holds on a prefix or a suffix of 0..99: its boundary is the
  // real-valued crossing, confirmed by evaluating the very same point expressions on both sides of it
  // (a 7-step binary search where that check fails), and the three wall conditions become interval
  // intersections.  A link whose two end joints have y >= 0 cannot reach below the ground and is
  // skipped.
  __device__ __forceinline__ bool wall_collision(const DevCfg& cf) const {
    const double left = hx - hw / 2, right = hx + hw / 2, nd = -hd;
    bool hit = false;
#pragma unroll
    for (int k = 0; k < NL; ++k) {
      const double y0 = jy[k], y1 = jy[k + 1];
      if (y0 >= 0.0 && y1 >= 0.0 && nd <= 0.0) continue;
      hit |= link_wall(left, right, nd, jx[k], jy[k], c[k], s[k]);
    }
    return hit;
  }
  // the wall test of one submerged link starting at (bx, by) with direction (ck, sk)
  static __device__ __forceinline__ bool link_wall(double left, double right, double nd, double bx, double by,
                                                   double ck, double sk) {
    {
      // lin_j = np.linspace(0, 1, 100)[j] = j * RN(1/99), last = 1 (computed, not loaded: the
      // binary searches would otherwise chain dependent memory loads)
      auto lin = [](int j) { return j == 99 ? 1.0 : (double)j * (1.0 / 99.0); };
      auto px = [&](int j) { return ck * lin(j) + bx; };
      auto py = [&](int j) { return sk * lin(j) + by; };
      // a link that crosses no hole edge (x = left / right): px is monotone in j, so its points all lie
      // on the side of both edges its end points p_0, p_99 lie on, and each condition reduces to the end
      // points' y (py monotone too): c1 / c2 to "some py < 0", c3 to "some py < -depth" -- exact, no
      // crossing search (needs left <= right; NaN end points fall through)
      {
        const double x0 = px(0), x1 = px(99), y0 = py(0), y1 = py(99);
        if (left <= right) {
          if ((x0 < left && x1 < left) || (x0 > right && x1 > right)) return y0 < 0.0 || y1 < 0.0;
          if (x0 > left && x0 < right && x1 > left && x1 < right) return y0 < nd || y1 < nd;
        }
      }
      // first j in [0, 100) with pred(j) (pred monotone false -> true), 100 if none.  The estimate je
      // (the real-valued crossing, rounded up) is exact without evaluating a point when the crossing
      // is far from every index (`clear`, below); otherwise it is checked with two evaluations of the
      // very same point expressions -- pred(je - 1) false and pred(je) true -- and only a lane whose
      // estimate misses (a crossing within rounding of a point, NaN / inf state) runs the 7-step
      // binary search.
      // Why `clear` is exact: the evaluated point f(j) = fl(fl(k lin_j) + b) differs from the real
      // F(j) = k j / 99 + b by at most E = 4u (|k| + |b|) (u = 2^-53; lin_j within 2u of j / 99), so
      // the comparison of f(j) with t is decided by the side of j against the real crossing
      // j* = 99 (t - b) / k whenever |j - j*| > 99 E / |k| <= 5e-8 (|k| >= 1e-3, |b|, |t| <= 1e3:
      // `sane`).  est = fl32(fl32(t - b) * fl32(rcp32(fl32(k)) * 99)) is within 6 f32 roundings of j*
      // (relative 5e-7, rcp32 1 ulp): |est - j*| < 6e-5 for |est| <= 101.  So when est lies more than
      // 1e-4 from every integer, or beyond [-1, 101], ceil(est) clamped to [0, 100] is the index the
      // binary search would find.
      auto first = [&](auto pred, float est, bool sane) {
        const int je = (est > 0.0f) ? ((est < 100.0f) ? (int)__builtin_ceilf(est) : 100) : 0;
        const float fr = est - __builtin_floorf(est);
        const bool clear = sane && (est < -1.0f || est > 101.0f || (fr > 1e-4f && fr < 1.0f - 1e-4f));
        if (__builtin_expect(clear, 1)) return je;
        const bool ok = (je == 0 || !pred(je - 1)) && (je == 100 || pred(je));
        if (__builtin_expect(ok, 1)) return je;
        int lo = 0, hi = 100;
#pragma unroll
        for (int it = 0; it < 7; ++it) {
          const int mid = (lo + hi) >> 1;
          const bool p = lo < hi && pred(mid);
          if (lo < hi) { if (p) hi = mid; else lo = mid + 1; }
        }
        return lo;
      };
      // real-valued index where f(j) = b + k j / 99 crosses t (an estimate only)
      const float rck = __builtin_amdgcn_rcpf((float)ck) * 99.0f, rsk = __builtin_amdgcn_rcpf((float)sk) * 99.0f;
      auto cross = [](double t, double b, float r) { return (float)(t - b) * r; };
      // the bounds under which an estimate far from every index is exact (`first`)
      const bool tsane = __builtin_fabs(left) <= 1e3 && __builtin_fabs(right) <= 1e3 && __builtin_fabs(nd) <= 1e3;
      const bool xsane = tsane && __builtin_fabs(ck) >= 1e-3 && __builtin_fabs(bx) <= 1e3;
      const bool ysane = tsane && __builtin_fabs(sk) >= 1e-3 && __builtin_fabs(by) <= 1e3;
      // {j : f(j) < t} / {j : f(j) > t} as [lo, hi) for f monotone with slope sign of `dir`
      auto below = [&](auto f, double dir, double t, float est, bool sane, int& lo, int& hi) {
        if (dir > 0.0) { lo = 0; hi = first([&](int j) { return !(f(j) < t); }, est, sane); }
        else if (dir < 0.0) { lo = first([&](int j) { return f(j) < t; }, est, sane); hi = 100; }
        else { lo = 0; hi = (f(0) < t) ? 100 : 0; }   // constant (or NaN) along the link
      };
      auto above = [&](auto f, double dir, double t, float est, bool sane, int& lo, int& hi) {
        if (dir > 0.0) { lo = first([&](int j) { return f(j) > t; }, est, sane); hi = 100; }
        else if (dir < 0.0) { lo = 0; hi = first([&](int j) { return !(f(j) > t); }, est, sane); }
        else { lo = 0; hi = (f(0) > t) ? 100 : 0; }
      };
      int xl0, xl1, xr0, xr1, xL0, xL1, xR0, xR1, yg0, yg1, yd0, yd1;
      const float el = cross(left, bx, rck), er = cross(right, bx, rck);
      below(px, ck, left, el, xsane, xl0, xl1);    // px < left
      above(px, ck, right, er, xsane, xr0, xr1);   // px > right
      above(px, ck, left, el, xsane, xL0, xL1);    // px > left
      below(px, ck, right, er, xsane, xR0, xR1);   // px < right
      below(py, sk, 0.0, cross(0.0, by, rsk), ysane, yg0, yg1);   // py < 0
      below(py, sk, nd, cross(nd, by, rsk), ysane, yd0, yd1);     // py < -depth
      const bool c1 = max(xl0, yg0) < min(xl1, yg1);
      const bool c2 = max(xr0, yg0) < min(xr1, yg1);
      const bool c3 = max(max(xL0, xR0), yd0) < min(min(xL1, xR1), yd1);
      return c1 || c2 || c3;
    }
  }

  // ---------------------------------------------------------------- lane pairs (k_episode_pair)
  // Both lanes of a pair (2i, 2i + 1) hold the same env and run the same step; p = this lane's
  // parity.  The costly parts of a HoleReacher step are divided between them: lane p evaluates the
  // sincos of the cumulative angles p, p + 2, ..., every other segment pair of the self-collision
  // test and every other link of the wall test, and takes the partner's results over a DPP lane
  // swap.  Each lane ends with exactly the values fk() / self_collision() / wall_collision()
  // compute: the same expressions on the same operands, only evaluated in the other lane.  The
  // selections below use the lane parity as data (v_cndmask), never as a branch, so both lanes'
  // shares issue as one instruction stream.
  __device__ __forceinline__ void fk_pair(int p) {
    constexpr int H = (NL + 1) / 2;
    double ang[NL];
#pragma unroll
    for (int k = 0; k < NL; ++k) ang[k] = (k == 0) ? q[0] : ang[k - 1] + q[k];
    double ms[H], mc[H], os[H], oc[H];
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const double a = p ? ang[min(2 * h + 1, NL - 1)] : ang[2 * h];
      fgx_sincos(a, &ms[h], &mc[h]);
      os[h] = pair_swap(ms[h]);
      oc[h] = pair_swap(mc[h]);
    }
    double x = 0.0, y = 0.0;
    jx[0] = 0.0; jy[0] = 0.0;
#pragma unroll
    for (int k = 0; k < NL; ++k) {
      const int h = k >> 1;
      // angle k is lane (k & 1)'s (both lanes evaluate the last one when NL is odd)
      const bool own = (2 * h + 1 >= NL) || ((k & 1) == p);
      const double cs = own ? mc[h] : oc[h], sn = own ? ms[h] : os[h];
      c[k] = cs; s[k] = sn;
      x = (k == 0) ? cs : x + cs;
      y = (k == 0) ? sn : y + sn;
      jx[k + 1] = 0.0 + x;
      jy[k + 1] = 0.0 + y;
    }
  }
  // segment pair n of the self-collision test in index order: (i, j), j >= i + 2
  static constexpr int seg_pair(int n, int which) {
    int m = 0;
    for (int i = 0; i < NL; ++i)
      for (int j = i + 2; j < NL; ++j) {
        if (m == n) return which ? j : i;
        ++m;
      }
    return 0;
  }
  __device__ __forceinline__ bool self_collision_pair(int p) const {
#pragma unroll
    for (int k = 0; k < NL; ++k)
      if (q[k] > M_PI || q[k] < -M_PI) return true;   // base_reacher.py:38-39,111
    constexpr int NP = (NL - 1) * (NL - 2) / 2;
    bool hit = false;
#pragma unroll
    for (int t = 0; 2 * t < NP; ++t) {   // lane p: pair 2t + p (lane 1 repeats pair 2t past the end)
      const int n0 = 2 * t, n1 = (2 * t + 1 < NP) ? 2 * t + 1 : 2 * t;
      const int i0 = seg_pair(n0, 0), j0 = seg_pair(n0, 1), i1 = seg_pair(n1, 0), j1 = seg_pair(n1, 1);
      const double ax = p ? jx[i1] : jx[i0], ay = p ? jy[i1] : jy[i0];
      const double bx = p ? jx[i1 + 1] : jx[i0 + 1], by = p ? jy[i1 + 1] : jy[i0 + 1];
      const double cx = p ? jx[j1] : jx[j0], cy = p ? jy[j1] : jy[j0];
      const double dx = p ? jx[j1 + 1] : jx[j0 + 1], dy = p ? jy[j1 + 1] : jy[j0 + 1];
      hit |= (ccw(ax, ay, cx, cy, dx, dy) != ccw(bx, by, cx, cy, dx, dy)) &&
             (ccw(ax, ay, bx, by, cx, cy) != ccw(ax, ay, bx, by, dx, dy));
    }
    return pair_or(hit);
  }
  __device__ __forceinline__ bool wall_collision_pair(const DevCfg& cf, int p) const {
    const double left = hx - hw / 2, right = hx + hw / 2, nd = -hd;
    bool hit = false;
#pragma unroll
    for (int t = 0; 2 * t < NL; ++t) {   // lane p: link 2t + p (none for lane 1 past the end)
      const int k0 = 2 * t, k1 = (2 * t + 1 < NL) ? 2 * t + 1 : 2 * t;
      const bool none = (2 * t + 1 >= NL) && p;
      const double y0 = p ? jy[k1] : jy[k0], y1 = p ? jy[k1 + 1] : jy[k0 + 1];
      if (none || (y0 >= 0.0 && y1 >= 0.0 && nd <= 0.0)) continue;
      hit |= link_wall(left, right, nd, p ? jx[k1] : jx[k0], y0, p ? c[k1] : c[k0], p ? s[k1] : s[k0]);
    }
    return pair_or(hit);
  }
};

}  // namespace fgx
