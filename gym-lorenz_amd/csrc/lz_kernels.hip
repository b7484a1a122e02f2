// Batched env kernels for gfx950 (MI355X, CDNA4): reset, step, fused K-step rollout.
//
// One env per lane, 256 envs (4 waves) per workgroup.  The hot path is HBM-bound
// byte streaming (<1 FLOP/B, three to eight coupled scalar ODEs, no contraction):
//   - state lives in SoA planes -> every per-plane load/store is a coalesced
//     64 x 4 B (or 8 B) wave access;
//   - the row-major [N, A] action and [N, O] observation tensors that SB3 / torch
//     hand over are staged through LDS so that global traffic moves as 16-B-per-lane
//     contiguous vectors (1 KiB per wave instruction) instead of A- or O-strided
//     scalar accesses;
//   - done envs are compacted with a 64-lane ballot + prefix popcount and ONE
//     atomic per wave (not per env) into the terminal-observation list;
//   - auto-reset happens in the same lane (counter-based Philox, no RNG state).
// See lz_systems.h for the per-system arithmetic and its reference citations.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

#include "lz_body.h"
#include "lz_internal.h"
#include "lz_rms_math.h"
#include "lz_systems.h"

namespace lz {

// ------------------------------------------------------------------ LDS staging
// Copy the block's [nb, W] slice of a row-major T tensor into LDS (row = env).
template <bool NT, typename T, int W, int B = kBlock>
__device__ __forceinline__ void stage_in(T* __restrict__ lds, const T* __restrict__ g, int nb,
                                         int tid, bool vec) {
  constexpr int kElems = B * W;
  if (vec && nb == B) {
    constexpr int kVec = kElems * (int)sizeof(T) / 16;
    const f4v* __restrict__ gv = reinterpret_cast<const f4v*>(g);
    f4v* lv = reinterpret_cast<f4v*>(lds);
#pragma unroll
    for (int v = tid; v < kVec; v += B) lv[v] = gload<NT>(gv + v);
  } else {
    for (int e = tid; e < nb * W; e += B) lds[e] = gload<NT>(g + e);
  }
}

template <bool NT, typename T, int W, int B = kBlock>
__device__ __forceinline__ void stage_out(T* __restrict__ g, const T* __restrict__ lds, int nb,
                                          int tid, bool vec) {
  constexpr int kElems = B * W;
  if (vec && nb == B) {
    constexpr int kVec = kElems * (int)sizeof(T) / 16;
    f4v* __restrict__ gv = reinterpret_cast<f4v*>(g);
    const f4v* lv = reinterpret_cast<const f4v*>(lds);
#pragma unroll
    for (int v = tid; v < kVec; v += B) gstore<NT>(gv + v, lv[v]);
  } else {
    for (int e = tid; e < nb * W; e += B) gstore<NT>(g + e, lds[e]);
  }
}

// Workgroup barrier for LDS hand-offs only.  __syncthreads() also drains vmcnt, i.e.
// waits until every global STORE of the wave has been acknowledged; the staging here
// only needs this wave's LDS ops complete (lgkmcnt(0)) before the s_barrier, so the
// obs / reward / state stores stay in flight across it.
template <bool kFull>
__device__ __forceinline__ void wg_barrier() {
  if constexpr (kFull) {
    __syncthreads();
  } else {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
}

// ------------------------------------------------------------------ reset
template <class Sys, typename T>
__global__ __launch_bounds__(kBlock) void k_reset(KArgs a) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint64_t tick = *a.tick_in;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    *a.tick_out = tick + a.tick_adv;
    // the next launch's compact-list cursor (lz_reset flips the parity like a step):
    // without this a step after step(dones) -> reset would start at the old count
    *a.counter_next = 0;
  }
  if (i >= a.n) return;
  if (a.mask && a.mask[i] == 0) return;
  Sys sys;
  sys.setup(a);
  T v[Sys::NI];
  if (a.init) {
#pragma unroll
    for (int j = 0; j < Sys::NI; ++j) v[j] = static_cast<const T*>(a.init)[i * Sys::NI + j];
  } else {
    Sys::draw(a, (uint64_t)(a.gid0 + i), tick, v);
  }
  sys.init(v, a);
  sys.store_reset(a, i);
  static_cast<int32_t*>(a.pl[Sys::kStepPlane])[i] = 0;
  if (a.obs) {
    T o[Sys::O];
    sys.reset_obs(o);
#pragma unroll
    for (int j = 0; j < Sys::O; ++j) static_cast<T*>(a.obs)[i * Sys::O + j] = o[j];
  }
}

// ------------------------------------------------------------------ step
#ifndef LZ_F64_PROLOGUE  // float64 steps keep round 3's prologue (step_tile)
#define LZ_F64_PROLOGUE 1
#endif
// V (tuning variant, lz_config.reserved[0], default 0): bit 0 = plain (temporal)
// act/obs/rew/done accesses instead of non-temporal, bit 1 = lanes access their own
// act/obs rows directly instead of LDS staging, bit 2 = __syncthreads() instead of the
// LDS-only barrier.  Measured at 1M envs (profiles/r01): non-temporal I/O is 13%
// faster than plain, LDS staging 7-11% faster than direct.
template <int V>
constexpr int step_block() {  // bits 3-4 of V: workgroup size
  return ((V >> 3) & 3) == 1 ? 512 : ((V >> 3) & 3) == 2 ? 128 : ((V >> 3) & 3) == 3 ? 1024 : 256;
}

// ------------------------------------------------------------------ VecNormalize epilogue
// (lz_step_vecnorm, lz_internal.h VArgs).  Per-workgroup float64 moments of the obs
// columns (read back from the LDS obs tile as the float32 values SB3 sees) and of the
// updated returns: Q groups of 32 lanes per column (Q = 1 for 256-env, 4 for 1024-env
// workgroups), lane j of group q summing rows j + 32 k of the q-th row quarter in order,
// then the lane sums in a fixed order; one plain store per column into the column-major
// partials.  Every normalise workgroup of lz_vecnorm_apply reduces them in one fixed
// order (no cross-workgroup synchronisation inside the step: an in-kernel last-arriver
// reduction needs every workgroup to wait for its stores' acknowledgements before
// taking a ticket, which measured 4x the step time at 1M envs).
template <int O, int SB, typename T>
__device__ __forceinline__ void vn_epilogue(const T* s_obs, const double* s_ret, int nb, int tid,
                                            const VArgs& v) {
  constexpr int C = O + 1;
  constexpr int G = SB / 32;                   // 32-lane groups
  constexpr int CP = C <= 8 ? 8 : 16;          // column slots
  constexpr int Q = G / CP >= 1 ? G / CP : 1;  // groups per column
  constexpr int KR = SB / 32 / Q;              // rows per lane
  __shared__ double red[2 * C][Q * 32 + 1];    // [column sums | sums of squares][lane]
  const int j = tid & 31;
  for (int it = tid >> 5; it < C * Q; it += G) {
    const int c = it / Q, q = it % Q;
    double s = 0.0, sq = 0.0;
#pragma unroll
    for (int k = 0; k < KR; ++k) {  // rows j + 32 (q KR + k), in order
      const int r = j + 32 * (q * KR + k);
      if (r < nb) {
        const double x = c < O ? (double)(float)s_obs[r * O + c] : s_ret[r];
        s += x;
        sq += x * x;
      }
    }
    red[c][q * 32 + j] = s;
    red[C + c][q * 32 + j] = sq;
  }
  __syncthreads();
  if constexpr (Q == 1) {
    if (tid < 2 * C) {
      double t = 0.0;
#pragma unroll
      for (int k = 0; k < 32; ++k) t += red[tid][k];
      v.part[(int64_t)tid * v.n_wg + blockIdx.x] = t;
    }
  } else {
    __shared__ double red2[2 * C][Q];
    if (tid < 2 * C * Q) {
      const int c = tid / Q, q = tid % Q;
      double t = 0.0;
#pragma unroll
      for (int k = 0; k < 32; ++k) t += red[c][q * 32 + k];
      red2[c][q] = t;
    }
    __syncthreads();
    if (tid < 2 * C) {
      double t = red2[tid][0];
#pragma unroll
      for (int q = 1; q < Q; ++q) t += red2[tid][q];
      v.part[(int64_t)tid * v.n_wg + blockIdx.x] = t;
    }
  }
}

// The step's second launch, with LZ_VN_DEFER or when there are too many partials for
// every normalise workgroup to reduce them (VArgs::fused == 0).  It publishes the
// step's done count and, in training, reduces the partial columns (vn_col_totals, the
// order the normalise pass uses) into the moments vector for the caller's all-reduce
// (DEFER; lz_vecnorm_apply then updates from the moments) or into the totals the
// normalise pass reads.  (Otherwise there is no second launch: the normalise pass
// reduces the partials and publishes the done count.)
constexpr int kVnColBlock = 256;
template <int O>
__global__ __launch_bounds__(kVnColBlock) void k_vn_colsum(VArgs v, int64_t n,
                                                          const int32_t* counter,
                                                          int32_t* n_done_out) {
  constexpr int C = O + 1;
  const int tid = (int)threadIdx.x;
  if (blockIdx.x == 0 && tid == 0) *n_done_out = *counter;
  if (!(v.flags & LZ_VN_TRAINING)) return;
  const bool defer = (v.flags & LZ_VN_DEFER) != 0;
  // (count, sums[O], sumsq[O]) for obs, then (count, sum, sumsq) for returns
  auto put = [&](int c, double t) {
    if (!defer) {
      v.tot[c] = t;
      return;
    }
    const int slot = c < O ? 1 + c : c == O ? 2 * O + 2 : c < C + O ? 1 + O + (c - C) : 2 * O + 3;
    v.moments[slot] = t;
    if (c == 0) {
      v.moments[0] = (double)n;
      v.moments[2 * O + 1] = (double)n;
    }
  };
  if (v.fused) {  // one workgroup, the normalise pass's order (DEFER at fused sizes)
    __shared__ double red[LZ_VN_RED(2 * C)];
    __shared__ double tot[2 * C];
    vn_col_totals<2 * C>(v.part, v.n_wg, red, tot);
    if (tid < 2 * C) put(tid, tot[tid]);
    return;
  }
  // many partials: one workgroup per column (2 (O + 1) of them), lane t adds rows t,
  // t + 1024, ... into accumulator u of rows t + 256 u, the 4 accumulators in order,
  // then a fixed LDS pairing tree
  __shared__ double red[kVnColBlock];
  const int c = (int)blockIdx.x;
  const double* col = v.part + (int64_t)c * v.n_wg;
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  for (int r = tid; r < v.n_wg; r += 4 * kVnColBlock) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int ru = r + u * kVnColBlock;
      if (ru < v.n_wg) acc[u] += col[ru];
    }
  }
  red[tid] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  __syncthreads();
#pragma unroll
  for (int half = kVnColBlock / 2; half > 0; half >>= 1) {
    if (tid < half) red[tid] += red[tid + half];
    __syncthreads();
  }
  if (tid == 0) put(c, red[0]);
}

// One 256-env tile of lz_step (k_step) or lz_step_vecnorm (k_step_vn, kVN).
template <class Sys, typename T, int V, bool kVN>
__device__ __forceinline__ void step_tile(const KArgs& a, const VArgs& v) {
  constexpr int SB = step_block<V>();
  constexpr bool NT = (V & 1) == 0;
  constexpr bool kLds = (V & 2) == 0;
  constexpr bool kFullBar = (V & 4) != 0;
  constexpr bool kDoneT = (V & 32) != 0;  // A/B: temporal done-byte stores
  __shared__ __attribute__((aligned(16))) float s_act[kLds ? SB * Sys::A : 4];
  __shared__ __attribute__((aligned(16))) T s_obs[kLds ? SB * Sys::O : 2];
  const int tid = (int)threadIdx.x;
  const int64_t base = (int64_t)blockIdx.x * SB;
  const int64_t i = base + tid;
  const int nb = (int)((a.n - base) < SB ? (a.n - base) : SB);
  const bool live = tid < nb;
  const bool vec = a.vec_ok != 0;
  // the pointers the step dereferences, with the first batch of kernel-argument loads:
  // otherwise the compiler issues their s_loads late and waits for each (the action
  // pointer's after the first lgkmcnt wait, the terminal-obs pointer's right after the
  // action barrier) -- serial kernel-argument round trips on the step's critical path
  // (float64 keeps round 3's prologue -- the tick as a scalar load at entry, no forced
  // argument batch: with the float32 prologue the float64 LORENZ3 step measured 18.34 ->
  // 19.84 us at 1M, profiles/r04/tick/ab_f64_1M.json; LZ_F64_PROLOGUE=0 for the A/B)
  constexpr bool kOldProlog = LZ_F64_PROLOGUE && sizeof(T) == 8;
  const float* ga_early = static_cast<const float*>(a.act);
  uint64_t tick0 = 0;
  if constexpr (kOldProlog) {
    tick0 = *a.tick_in;
    if (blockIdx.x == 0 && tid == 0) {
      *a.counter_next = 0;
      *a.tick_out = tick0 + a.tick_adv;
    }
  } else {
    asm volatile("" ::"s"(a.term_obs), "s"(a.obs), "s"(a.rew), "s"(a.done));
    if constexpr (Sys::kUsesAction) asm volatile("" ::"s"(ga_early));
    if (blockIdx.x == 0 && tid == 0) *a.counter_next = 0;
  }
  if constexpr (kVN) {  // the statistics before this step, for the normalise pass
    if (blockIdx.x == 0 && (v.flags & LZ_VN_TRAINING) && !(v.flags & LZ_VN_DEFER)) {
      if (tid < 2 * Sys::O + 1) v.old[tid] = v.obs_state[tid];
      if (tid < 3) v.old[2 * Sys::O + 1 + tid] = v.ret_state[tid];
    }
  }
  Sys sys;
  sys.setup(a);
  int32_t steps = 0;
  double ret_in = 0.0;  // kVN: VecNormalize.returns[i], loaded with the state
  if (live) {  // state loads first: in flight together with the action staging
    sys.load(a, i);
    if (a.count_steps) steps = static_cast<const int32_t*>(a.pl[Sys::kStepPlane])[i];
    if constexpr (kVN) ret_in = v.returns[i];
  }
  uint64_t tick = kOldProlog ? tick0 : load_tick(a.tick_in);  // in flight with the state and action loads
  float act[Sys::A];
  if constexpr (Sys::kUsesAction) {
    const float* ga = ga_early;
    if constexpr (kLds) {
      stage_in<NT, float, Sys::A, SB>(s_act, ga + base * Sys::A, nb, tid, vec);
      wg_barrier<kFullBar>();
      if (live) {
#pragma unroll
        for (int j = 0; j < Sys::A; ++j) act[j] = s_act[tid * Sys::A + j];
      }
    } else if (live) {
#pragma unroll
      for (int j = 0; j < Sys::A; ++j) act[j] = gload<NT>(ga + i * Sys::A + j);
    }
  }
  if constexpr (!kOldProlog) tick = tick_ready(tick);
  T o[Sys::O];
  T rew = (T)0;
  bool did_reset;
  double rn = 0.0;  // kVN: the updated VecNormalize.returns[i] (before the done reset)
  const uint8_t dflag =
      step_body<Sys, T, false>(sys, steps, a, i, live, act, tick, 0, o, rew, did_reset);
  if constexpr (!kOldProlog)
    if (blockIdx.x == 0 && tid == 0) *a.tick_out = tick + a.tick_adv;  // tick waited for here
  __shared__ double s_ret[kVN ? SB : 1];
  if constexpr (kVN) {  // VecNormalize.returns: r*gamma + reward, moments, then [done] = 0
    if (live) {
      double r0 = ret_in;
      if (v.flags & LZ_VN_TRAINING) r0 = r0 * v.gamma + (double)(float)rew;
      rn = r0;
      v.returns[i] = dflag ? 0.0 : r0;
    }
    s_ret[tid] = rn;
  }
  if (live) {
    sys.store(a, i);
    if (did_reset) sys.store_autoreset_extra(a, i);
    if (a.count_steps) static_cast<int32_t*>(a.pl[Sys::kStepPlane])[i] = steps;
    if constexpr (kLds) {
#pragma unroll
      for (int j = 0; j < Sys::O; ++j) s_obs[tid * Sys::O + j] = o[j];
    } else {
#pragma unroll
      for (int j = 0; j < Sys::O; ++j) gstore<NT>(static_cast<T*>(a.obs) + i * Sys::O + j, o[j]);
    }
    gstore<NT>(static_cast<T*>(a.rew) + i, rew);
    gstore<NT && !kDoneT>(a.done + i, dflag);
  }
  if constexpr (kLds) {
    wg_barrier<kFullBar>();
    stage_out<NT, T, Sys::O, SB>(static_cast<T*>(a.obs) + base * Sys::O, s_obs, nb, tid, vec);
  }
  if constexpr (kVN) {
    static_assert(kLds, "the VecNormalize epilogue reads the LDS obs tile");
    if (v.flags & LZ_VN_TRAINING) vn_epilogue<Sys::O, SB, T>(s_obs, s_ret, nb, tid, v);
  }
}

// Occupancy hint per system (Sys::kStepWaves, default none): a register-heavy step body
// compiled for more resident waves, so that the 4096 workgroups of a 1M-env step need
// fewer rounds over the CUs (HR f32: 82 VGPRs = 5 waves/SIMD unconstrained).
template <class Sys, class = void>
struct step_waves {
  static constexpr int value = 1;
};
template <class Sys>
struct step_waves<Sys, std::void_t<decltype(Sys::kStepWaves)>> {
  static constexpr int value = Sys::kStepWaves;
};

template <class Sys, typename T, int V>
__global__ __launch_bounds__(step_block<V>())
__attribute__((amdgpu_waves_per_eu(step_waves<Sys>::value))) void k_step(KArgs a) {
  step_tile<Sys, T, V, false>(a, VArgs{});
}

// VB: the step variant carrying the workgroup size (0: 256, 24: 1024 envs)
template <class Sys, typename T, int VB>
__global__ __launch_bounds__(step_block<VB>()) void k_step_vn(KArgs a, VArgs v) {
  step_tile<Sys, T, VB, true>(a, v);
}

// ------------------------------------------------------------------ multi-tile step
// E consecutive 256-env tiles per workgroup, each lane one env of every tile (PMSM and
// HR float32, A = 2).  k_step gives every wave ONE tile: its state loads, ~300-400
// dependent instructions, its stores -- and at PMSM 262,144 envs all 4,096 waves are
// resident at once, so the chip reads everything, then computes, then writes (the time
// is the sum of the three, profiles/r03/step).  Here every tile's loads are issued at
// entry, tile e steps as soon as its own loads have landed (the compiler waits with
// vmcnt(#later loads)), while tiles e+1.. are still arriving and tile e-1's stores
// drain.  Actions come straight from the row-major [N, 2] tensor, one 8-B load per lane
// (a wave instruction reads 512 contiguous bytes); the obs tile leaves through LDS as
// in k_step, one LDS buffer per tile (no reuse hazard between tiles).  Same step_body,
// same per-env arithmetic: bit-identical to k_step.
typedef float f2m __attribute__((ext_vector_type(2)));
// Load layout of k_step_multi per system (measured, profiles/r04/kargs/): "flat" issues
// every tile's loads straight-line -- each lane loads (index clamped to the last env; a
// dead lane's values are never stored), the step counter unconditionally (plane 0 stands
// in when there is none, the value then unused), a scheduling barrier between tiles -- so
// the compiler's wait at tile 0's step covers tile 0's loads only, and the tick is a
// scalar load (HR f32 1M: 18.19 -> 17.35 us).  PMSM keeps round 3's layout (loads under
// the lane condition, the vector tick of k_step): flat measured 23.66 -> 26.14 us there.
template <class Sys>
struct multi_flat_loads {
  static constexpr bool value = false;
};
template <>
struct multi_flat_loads<SysHR<float>> {
  static constexpr bool value = true;
};
template <>
struct multi_flat_loads<SysL3<float>> {
  static constexpr bool value = true;
};

template <class Sys, typename T, int E, bool kDoneT = false>
__global__ __launch_bounds__(kBlock) void k_step_multi(KArgs a) {
  static_assert(Sys::kUsesAction && (Sys::A == 2 || multi_flat_loads<Sys>::value),
                "k_step_multi: systems with actions (round 3's loads: two actions)");
  constexpr int SB = kBlock;
  constexpr bool kFlat = multi_flat_loads<Sys>::value;
  __shared__ __attribute__((aligned(16))) T s_obs[E][SB * Sys::O];
  const int tid = (int)threadIdx.x;
  const bool vec = a.vec_ok != 0;
  Sys sys[E];
  int32_t steps[E];
  float act[E][Sys::A];
  const float* ga = static_cast<const float*>(a.act);
  uint64_t tick;
  if constexpr (kFlat) {
    tick = *a.tick_in;
    if (blockIdx.x == 0 && tid == 0) {
      *a.counter_next = 0;
      *a.tick_out = tick + a.tick_adv;
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int64_t i = ((int64_t)blockIdx.x * E + e) * SB + tid;
      const int64_t ic = i < a.n ? i : a.n - 1;
      sys[e].setup(a);
      sys[e].load(a, ic);
      const int32_t* sp = static_cast<const int32_t*>(a.count_steps ? a.pl[Sys::kStepPlane] : a.pl[0]);
      steps[e] = sp[ic];
#pragma unroll
      for (int j = 0; j < Sys::A; ++j)  // (merged into one 8-B / 12-B load)
        act[e][j] = __builtin_nontemporal_load(ga + Sys::A * ic + j);
      __builtin_amdgcn_sched_barrier(0);  // tile e's loads stay ahead of tile e+1's
    }
  } else if constexpr (Sys::A == 2) {
    tick = load_tick(a.tick_in);
    if (blockIdx.x == 0 && tid == 0) *a.counter_next = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {  // every tile's loads, in tile order
      const int64_t i = ((int64_t)blockIdx.x * E + e) * SB + tid;
      sys[e].setup(a);
      steps[e] = 0;
      act[e][0] = act[e][1] = 0.0f;
      if (i < a.n) {
        sys[e].load(a, i);
        if (a.count_steps) steps[e] = static_cast<const int32_t*>(a.pl[Sys::kStepPlane])[i];
        if (vec) {
          const f2m v2 = __builtin_nontemporal_load(reinterpret_cast<const f2m*>(ga) + i);
          act[e][0] = v2[0];
          act[e][1] = v2[1];
        } else {
          act[e][0] = __builtin_nontemporal_load(ga + 2 * i);
          act[e][1] = __builtin_nontemporal_load(ga + 2 * i + 1);
        }
      }
    }
    tick = tick_ready(tick);
  }
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int64_t base = ((int64_t)blockIdx.x * E + e) * SB;
    if (base >= a.n) break;  // workgroup-uniform: the trailing tiles of the last group
    const int64_t i = base + tid;
    const int nb = (int)((a.n - base) < SB ? (a.n - base) : SB);
    const bool live = tid < nb;
    T o[Sys::O];
    T rew = (T)0;
    bool did_reset;
    // noise is never injected here (step_tiles sends injected-noise launches to k_step)
    const uint8_t dflag = step_body<Sys, T, false, false, false, !kFlat>(sys[e], steps[e], a, i, live, act[e],
                                                                         tick, 0, o, rew, did_reset);
    if (live) {
      sys[e].store(a, i);
      if (did_reset) sys[e].store_autoreset_extra(a, i);
      if (a.count_steps) static_cast<int32_t*>(a.pl[Sys::kStepPlane])[i] = steps[e];
#pragma unroll
      for (int j = 0; j < Sys::O; ++j) s_obs[e][tid * Sys::O + j] = o[j];
      gstore<true>(static_cast<T*>(a.rew) + i, rew);
      gstore<!kDoneT>(a.done + i, dflag);
    }
    wg_barrier<false>();
    stage_out<true, T, Sys::O, SB>(static_cast<T*>(a.obs) + base * Sys::O, s_obs[e], nb, tid, vec);
  }
  if constexpr (!kFlat) {
    if (blockIdx.x == 0 && tid == 0) *a.tick_out = tick + a.tick_adv;
  }
}

// Tiles per workgroup of k_step_multi: variant bits 14-15 (16384 x {1, 2, 3}) force 1
// (k_step), 2 or 4; 0 = the measured default, step_tiles_balanced.
template <class Sys>
struct multi_step_ok {
  static constexpr bool value = false;
};
template <>
struct multi_step_ok<SysPMSM> {
  static constexpr bool value = true;
};
template <>
struct multi_step_ok<SysHR<float>> {
  static constexpr bool value = true;
};
// LORENZ3 f32 (straight-line loads, 3 actions as one 12-B load): at 1,048,576 envs E = 4
// (one chip generation, 4 waves per SIMD) 11.31-11.41 -> 11.09-11.12 us per step; E = 2
// 12.8 us; at 131,072 / 2M / 4M k_step wins (profiles/r04/l3multi/); only on balanced
// grids (step_tiles_balanced)
template <>
struct multi_step_ok<SysL3<float>> {
  static constexpr bool value = true;
};
// Round 3: four tiles per workgroup only where that grid is ONE full generation of the chip (4
// waves per SIMD, 109 VGPRs: 4 workgroups of 1,024 envs per CU, more than 3/4 of them
// used): then k_step's 2-3 generations (HR 1M: 4,096 workgroups at 6 waves per SIMD =
// 2.67) and their partial last one go away.  Elsewhere one wave running its tiles in
// sequence is slower than k_step's waves running theirs in parallel (each tile is a
// ~1.6 us dependent chain of ~400 instructions): PMSM 262,144 6.9 -> 11.3 us, HR 2M
// 32 -> 35.6 us.  Measured (profiles/r03/multi_step/): HR 1M 17.0 -> 15.8 us, PMSM 1M
// 24.6 -> 23.5, PMSM 786,432 19.0 -> 18.1; 917,504 a tie.
// Round 4: four tiles only on a balanced grid -- exactly 4 (or, LORENZ3 / PMSM, 3)
// workgroups of 1,024 envs on every CU; elsewhere the CUs holding one more workgroup set
// the time.  Measured (profiles/r04/l3window/, profiles/r04/hrflat/ window runs), k_step
// -> E = 4 in us: LORENZ3 1,048,576 11.36 -> 11.11, 786,432 8.93 -> 8.58, 851,968 9.29 ->
// 11.26, 917,504 9.54 -> 11.69; PMSM 786,432 19.46 -> 18.16, 851,968 21.20 -> 21.49,
// 917,504 22.83 -> 22.61; HR 786,432 14.89 -> 15.38, 851,968 15.75 -> 16.90, 917,504
// 16.73 -> 17.39 (HR 1M: +3.5-4.8%, above).
// Round 6: TWO tiles for LORENZ3 where that grid is exactly 2 workgroups of 512 envs per CU
// (262,144 envs on 256 CUs, the 4-GPU strong shard) measured 3.74 vs 3.96 us per step on
// the first boxes (profiles/r06/tiles/), then proved bimodal: per HANDLE (buffer placement,
// profiles/r06/tile_probe/), 3.76 - 3.90 or 4.22 - 4.25 us, about half of 22 handles slow,
// while one tile holds 3.94 - 4.03.  A 4-GPU line is the max over its ranks, so the default
// stays one tile; variant 32768 still forces two.
inline int step_tiles_balanced(int64_t n, int num_cus, bool three) {
  const int64_t groups = (n + 4 * kBlock - 1) / (4 * kBlock);
  return groups == 4 * (int64_t)num_cus || (three && groups == 3 * (int64_t)num_cus) ? 4 : 1;
}
template <class Sys>
inline int step_tiles(const KArgs& a) {
  if (a.noise) return 1;  // injected noise: k_step (k_step_multi draws its noise on device)
  switch ((a.variant >> 14) & 3) {
    case 1: return 1;
    case 2: return 2;
    case 3: return 4;
    default:
      return step_tiles_balanced(a.n, a.num_cus > 0 ? a.num_cus : 256, !std::is_same<Sys, SysHR<float>>::value);
  }
}


// ------------------------------------------------------------------ fused rollout
// K steps in one launch, state in VGPRs.  B = envs per workgroup: 256, or 64 (one
// wave) when N is too small to give every CU several 256-lane workgroups (cfg5:
// 32,768 envs per GPU -> 512 one-wave groups).
//
// Full workgroups take a branch-free path: every lane moves exactly its row's bytes
// of the act / obs slices in fixed-size chunks (chunk c = j*B + lane: each wave
// instruction stays contiguous), and the next step's actions are prefetched into
// registers.  With no exec-masked stores the compiler can count the vector-memory
// ops issued after the prefetch and wait for the prefetch alone (vmcnt(N)) instead
// of for every outstanding store (vmcnt(0)) -- a store-ack round trip per step.
typedef float f2v __attribute__((ext_vector_type(2)));
template <int RB>
struct Chunk {  // widest power-of-two chunk (<= 16 B) that tiles a RB-byte row
  using t = typename std::conditional<RB % 16 == 0, f4v,
                                      typename std::conditional<RB % 8 == 0, f2v, float>::type>::type;
  static constexpr int N = RB / (int)sizeof(t);
};

// Action prefetch by LDS-DMA (global_load_lds_dword, non-temporal), issued from inline
// asm: the data lands in LDS without a VGPR destination and hipcc does not see the
// DMA at all -- so it neither drains vmcnt(0) before later LDS reads (its LDS-DMA
// alias rule) nor before reusing the address VGPRs, both of which it does for the
// builtin.  The loop waits explicitly with vmcnt(N), N = the vector-memory
// instructions it knows were issued after the DMA; older stores stay in flight.
// Destination = M0 (wave-uniform LDS byte offset) + lane * 4.
typedef __attribute__((address_space(3))) void* las_t;
__device__ __forceinline__ uint32_t lds_off(const float* p) {
  return (uint32_t)(uintptr_t)(las_t)(const_cast<float*>(p));
}
__device__ __forceinline__ void dma4_nt(const float* g, uint32_t m0) {
  uint32_t saved;  // M0 is a reserved register hipcc may hold a value in: save/restore
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\tglobal_load_lds_dword %1, off nt\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(saved)
               : "v"(g), "s"(m0)
               : "memory");
}
// 16-B LDS-DMA (global_load_lds_dwordx4); the s_nop separates the M0 write from the
// DMA that reads it.
__device__ __forceinline__ void dma16_nt(const float* g, uint32_t m0) {
  uint32_t saved;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(saved)
               : "v"(g), "s"(m0)
               : "memory");
}
// Row DMA of the fused rollout: ONE 16-B LDS-DMA per wave and step moves the wave's
// contiguous [envs, A] action slice (envs = 64, or 32 in the split-lane kernel) into the
// wave's own 1-KiB LDS region, row-major: lane l loads 16-B chunk l mod C of the slice
// (C = envs * A / 4 chunks; the remaining lanes repeat chunks, so no lane reads past
// the slice), landing at region + 16 l.  Needs the slice 16-B aligned (the launch's
// vec_ok: actions 16-B aligned, N a multiple of 4) and envs * A a multiple of 4.
template <int A, int E>
constexpr bool row_dma() { return (A == 2 || A == 3) && (E * A) % 4 == 0; }
constexpr int kRowRegionF = 256;  // floats per wave region and slot (64 lanes x 16 B)
// LDS floats of the DMA ring per slot for a B-lane workgroup
template <int A, int B>
constexpr int act_slot_floats() { return row_dma<A, 64>() ? (B / 64) * kRowRegionF : B * A; }
// LDS reads of the DMA'd slot, also from asm (with their own lgkmcnt wait), so that
// no compiler-visible LDS access depends on the hidden DMA.
template <int A>
__device__ __forceinline__ void lds_read_act(float* act, const float* p0, int stride) {
  if constexpr (A == 3) {
    asm volatile("ds_read_b32 %0, %3\n\tds_read_b32 %1, %4\n\tds_read_b32 %2, %5\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(act[0]), "=&v"(act[1]), "=&v"(act[2])
                 : "v"(lds_off(p0)), "v"(lds_off(p0 + stride)), "v"(lds_off(p0 + 2 * stride))
                 : "memory");
  } else {
    static_assert(A == 2, "action dim");
    asm volatile("ds_read_b32 %0, %2\n\tds_read_b32 %1, %3\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(act[0]), "=&v"(act[1])
                 : "v"(lds_off(p0)), "v"(lds_off(p0 + stride))
                 : "memory");
  }
}
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N <= 63, "vmcnt immediate (6 bits on gfx9)");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Prefetch distance D of the fused rollout's action DMA (steps in flight; D + 1 LDS
// slots, a power of two).  vmcnt counts stores as well as loads, so D also bounds how
// many steps of stores stay in flight behind the wait at the top of a step.
// D = 7 measured against 3 (tools/ab_rollout.py, K = 2048): LORENZ3 f32 +5% at 32,768
// envs (split lanes), +1.5% at 262,144; PMSM +4% at 32,768, even at 262,144.
constexpr int kDmaDist = 7;
template <int D>
constexpr int dma_slots() { return D + 1; }

// vmcnt wait at the top of step k < D: the vector-memory ops issued after step k's
// DMA are the prologue's later DMAs ((D-1-k) * kA) and k earlier steps' DMA + stores
template <int D, int kA, int kSt, int J = 0>
__device__ __forceinline__ void ladder_wait(int k) {
  if constexpr (J < D) {
    if (k == J) {
      wait_vmcnt<(D - 1 - J) * kA + J * (kA + kSt)>();
      return;
    }
    ladder_wait<D, kA, kSt, J + 1>(k);
  }
}

constexpr int kZSlots = 4;  // steps of normals a producer wave may draw ahead (k_rollout kNP)
constexpr uint32_t kZSpinCap = 1u << 24;  // polls of one flag before a wave gives up (~1 s)
// LZ_RAG: which systems' ragged last group takes the full path (kRag): 2 (default) the
// noise-free systems (LORENZ3 / LORENZ4 / T1 / T2), 1 every system, 0 none (A/B builds,
// tools/build_ab.sh).  Compiled into the noisy systems' rollout kernels (PMSM, HR, whose
// loops are ~3x larger) the second copy of the loop slowed their WHOLE groups by 5-6 %
// (PMSM lane pair 1,929 -> 2,038 us, HR 1,352 -> 1,419 at 32,768 x 2048; LORENZ3 unchanged,
// profiles/r06/rag_ab/), so their ragged group keeps the staged path (its action row
// prefetched one step ahead).
#ifndef LZ_RAG
#define LZ_RAG 2
#endif
template <class Sys>
constexpr bool rag_full() {
  return LZ_RAG == 1 || (LZ_RAG == 2 && !Sys::kNoise);
}
// kRag (FULL one-wave groups only): the launch's ragged LAST group (nb < 64, N a multiple
// of 4 -- vec_ok) runs the full path too: its DMA sources are clamped to the group's own
// rows (nb * A floats, whole 16-B chunks since nb % 4 == 0), and the lanes past nb compute
// on stale LDS but store nothing (their stores exec-masked: still issued, so the vmcnt
// counts hold -- lane 0 is always live).  The staged path's per-step action load made that
// one group the launch's straggler (LORENZ3 16,400 x 2048: 1,860 vs 465 us).
template <class Sys, typename T, int B, bool FULL, int D, bool kNoDone, bool kDoneT, bool kNP = false,
          bool kZN = false, bool kRag = false>
__device__ __forceinline__ void rollout_loop(Sys& sys, int32_t& steps, bool& any_reset,
                                             const KArgs& a, int64_t base, int tid, int nb,
                                             uint64_t tick, float* s_act, T* s_obs,
                                             const float* s_z = nullptr, int* zflag = nullptr) {
  static_assert(!kNP || (FULL && B == 64), "the noise producer pairs with full one-wave groups");
  using CO = Chunk<Sys::O * (int)sizeof(T)>;
  using co_t = typename CO::t;
  const int64_t i = base + tid;
  static_assert(!kRag || (FULL && B == 64), "kRag: full-path one-wave groups");
  const bool live = (FULL && !kRag) || tid < nb;
  const float* gact = static_cast<const float*>(a.act);
  const int wave = tid >> 6;
  // One-wave workgroups (small N, latency-bound): no LDS obs staging and no barriers --
  // each lane writes its own obs row (the L2 merges the partial lines of the row's
  // stores before they leave for HBM) and reads its actions from a [A][64] LDS slot.
  constexpr bool kDirect = FULL && B == 64;
  // Lower bound on the vector-memory instructions every full-path step issues after
  // its DMA, whatever the branch: the reward store, the done store and the obs stores
  // -- CO::N chunk stores B*chunk bytes apart (never merged), or a lane's contiguous
  // row, which hipcc may merge into ceil(row/16) stores.  A LOWER bound is safe.
  constexpr int kRowB = Sys::O * (int)sizeof(T);
  constexpr int kSt = 2 + (kDirect ? (kRowB + 15) / 16 : CO::N);
  constexpr bool kRow = row_dma<Sys::A, 64>();
  constexpr int kA = kRow ? 1 : Sys::A;  // DMA instructions per step
  constexpr int kSlotF = act_slot_floats<Sys::A, B>();
  const int lane = tid & 63;
  // steady-state wait: step k's DMA has one step's stores plus D-1 steps' (DMA +
  // stores) issued after it (lower bounds, see kSt)
  constexpr int kSteady = kSt + (D - 1) * (kA + kSt);
  static_assert(D >= 1 && kSteady <= 63, "vmcnt immediate (6 bits on gfx9)");
  constexpr int kDmaSlots = dma_slots<D>();
  // DMA step kk's action slice into LDS slot `slot` (B*A floats):
  // direct: component-major [A][B]; staged: a verbatim copy of the row-major slice.
  // src = this lane's first source float of step kk (component j is j, resp. j*B, on).
  // M0 = LDS byte address of this wave's 64 destination floats: computed once,
  // wave-uniform, then constant offsets per slot / component (no per-DMA address-space
  // cast or readfirstlane)
  const uint32_t m0_wave = __builtin_amdgcn_readfirstlane(
      lds_off(s_act) + (uint32_t)wave * (kRow ? kRowRegionF * 4u : 256u));
  auto issue = [&](const float* src, int slot) __attribute__((always_inline)) {
    if constexpr (kRow) {
      dma16_nt(src, m0_wave + (uint32_t)(slot * kSlotF) * 4u);
    } else {
#pragma unroll
      for (int j = 0; j < Sys::A; ++j)
        dma4_nt(src + (kDirect ? j : j * B), m0_wave + (uint32_t)((slot * Sys::A + j) * B) * 4u);
    }
  };
  // this lane's DMA source pointer for step kk, and the per-step advance
  const int64_t wave_row0 = (base + 64 * (int64_t)wave) * Sys::A;  // the wave's slice
  const int lane_src = kRag ? (kRow ? min(lane % (64 * Sys::A / 4), nb * Sys::A / 4 - 1) : min(tid, nb - 1))
                            : (kRow ? lane % (64 * Sys::A / 4) : tid);
  const int64_t lane0 = kRow ? wave_row0 + 4 * lane_src
                             : kDirect ? (base + lane_src) * Sys::A : base * Sys::A + tid;
  const int64_t dstride = a.n * Sys::A;
  auto dma_src = [&](int kk) __attribute__((always_inline)) {
    return gact + ((int64_t)kk * dstride + lane0);
  };
  // settle every compiler-visible load of the prologue (state planes) here, so that
  // hipcc's wait bookkeeping enters the loop with nothing pending and emits no drain
  // inside it (vmcnt(0) alone: 0x0F70 = expcnt 7, lgkmcnt 15, vmcnt 0)
  if constexpr (FULL) __builtin_amdgcn_s_waitcnt(0x0F70);
  if constexpr (FULL && Sys::kUsesAction) {
#pragma unroll
    for (int d = 0; d < D; ++d) issue(dma_src(d < a.K ? d : a.K - 1), d);
  }
  // running source of the DMA issued at step k (step min(k + D, K - 1)): advanced by
  // one step per step until it reaches the last (no per-step 64-bit multiply)
  const float* dsrc = dma_src(D < a.K ? D : a.K - 1);
  uint32_t zcap = 0;  // kNP: the producer timed out once -- stop waiting for it (sticky)
  // kZN: step k's normals, drawn during step k - 1 (step 0's here); see step_body kZMode 2
  float zn[3] = {0.0f, 0.0f, 0.0f};
  if constexpr (kZN) {
    if (live && (a.flags & LZ_FLAG_ADD_NOISE)) normal3(a.seed, (uint64_t)(a.gid0 + i), tick, zn);
  }
  float anext[Sys::A > 0 ? Sys::A : 1];  // !FULL: the next step's action row (prefetched)
  // kLadder: one of the first D steps (its wait count depends on k); later steps all
  // wait with the steady-state count -- peeled so the hot loop carries no ladder
  auto run_step = [&](int k, auto ladder) __attribute__((always_inline)) {
    const int64_t off = (int64_t)k * a.n;
    float act[Sys::A];
    if constexpr (Sys::kUsesAction) {
      if constexpr (FULL) {
        if constexpr (decltype(ladder)::value) ladder_wait<D, kA, kSt>(k);
        else wait_vmcnt<kSteady>();
        // staged path: every wave is past the previous step's reads of s_obs (and, without
        // row DMA, every wave's DMA of this slot has landed)
        if constexpr (!kDirect) wg_barrier<false>();
        const float* slot = s_act + (k % kDmaSlots) * kSlotF;
        if constexpr (kRow) {  // ordinary LDS loads: ordered after the wait by its clobber
#pragma unroll
          for (int j = 0; j < Sys::A; ++j)
            act[j] = slot[wave * kRowRegionF + lane * Sys::A + j];
        } else if constexpr (kDirect) {
          lds_read_act<Sys::A>(act, slot + tid, B);
        } else {
          lds_read_act<Sys::A>(act, slot + tid * Sys::A, 1);
        }
        // prefetch step k+D into the slot step k-1 used (every reader is past this
        // point); near the end re-read step K-1: no branch, same op count
        issue(dsrc, (k + D) % kDmaSlots);
        if (k + D + 1 < a.K) dsrc += dstride;
      } else {
        // a ragged last group / unaligned actions: each lane loads its own row, ONE STEP
        // AHEAD into registers (a load issued and waited for in the same step put a memory
        // round trip into every step of the group's chain: PMSM 24,608 x 2048, one ragged
        // group of 32 envs, 3,421 us against 2,094 at 24,576, profiles/r06/pair/); the
        // barrier keeps the obs tile's reuse rule of the staged full path
        wg_barrier<false>();
        if (live) {
          if (k == 0) {
#pragma unroll
            for (int j = 0; j < Sys::A; ++j) anext[j] = gload<true>(gact + i * Sys::A + j);
          }
#pragma unroll
          for (int j = 0; j < Sys::A; ++j) act[j] = anext[j];
          if (k + 1 < a.K) {
#pragma unroll
            for (int j = 0; j < Sys::A; ++j) anext[j] = gload<true>(gact + (off + a.n + i) * Sys::A + j);
          }
        }
      }
    }
    T o[Sys::O];
    T rew = (T)0;
    bool did_reset;
    const float* zp = nullptr;
    if constexpr (kNP) {  // step k's normals: wait for the producer wave (LDS flag, relaxed:
      // LDS operations of a wave execute in order, the signal fences keep the compiler's)
      uint32_t spin = zcap;
      while (spin < kZSpinCap &&  // (a cap: every wave leaves, whatever happens)
             __hip_atomic_load(&zflag[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) <= k) {
        __builtin_amdgcn_s_sleep(1);
        ++spin;
      }
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      const float* zs = s_z + (k % kZSlots) * 3 * B + tid;  // (LDS ring)
      // the producer never delivered: this step's normals and every later step's are NaN
      // (NaN obs / reward: a wrong result is visible, never silently stale), poisoned in
      // the stepping wave's own registers (zp = nullptr: step_body kZMode 1) -- the ring
      // slot is left alone, so a producer that is only slow cannot mix valid normals into
      // a poisoned step; it leaves on its own cap and is not waited for again
      if (spin >= kZSpinCap) zcap = kZSpinCap;
      zp = spin >= kZSpinCap ? nullptr : zs;
    }
    if constexpr (kZN) zp = zn;
    const uint8_t dflag = step_body<Sys, T, true, false, kNoDone, false, kNP ? 1 : kZN ? 2 : 0>(
        sys, steps, a, i, live, act, tick + (uint64_t)k, k, o, rew, did_reset, nullptr, true, zp);
    if constexpr (kNP) {  // slot k % kZSlots is free again
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      if (tid == 0) __hip_atomic_store(&zflag[1], k + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    any_reset = any_reset || did_reset;
    T* gobs = static_cast<T*>(a.obs) + (off + base) * Sys::O;
    if constexpr (kDirect) {
      if (!kRag || live) {
        gstore<true>(static_cast<T*>(a.rew) + off + i, rew);
        gstore<!kDoneT>(a.done + off + i, dflag);
        const co_t* src = reinterpret_cast<const co_t*>(o);
#pragma unroll
        for (int j = 0; j < CO::N; ++j) gstore<false>(reinterpret_cast<co_t*>(gobs) + tid * CO::N + j, src[j]);
      }
      return;
    }
    // the obs tile of this step: systems with actions pass a workgroup barrier at the top
    // of every step (after the previous step's reads of the tile); systems without (LORENZ4,
    // SC) alternate two tiles, so a wave's writes for step k+1 never meet a slower wave's
    // reads of step k's tile, and step k+2's writes follow step k+1's barrier
    T* so = s_obs + ((Sys::kUsesAction || (k & 1) == 0) ? 0 : B * Sys::O);
    if (live) {
#pragma unroll
      for (int j = 0; j < Sys::O; ++j) so[tid * Sys::O + j] = o[j];
      gstore<true>(static_cast<T*>(a.rew) + off + i, rew);
      gstore<!kDoneT>(a.done + off + i, dflag);
    }
    wg_barrier<false>();
    if constexpr (FULL) {
#pragma unroll
      for (int j = 0; j < CO::N; ++j)
        gstore<true>(reinterpret_cast<co_t*>(gobs) + j * B + tid,
                     reinterpret_cast<const co_t*>(so)[j * B + tid]);
    } else {
      stage_out<true, T, Sys::O, B>(gobs, so, nb, tid, false);
    }
  };
  int k = 0;
  if constexpr (FULL && Sys::kUsesAction) {
    const int kp = D < a.K ? D : a.K;
    for (; k < kp; ++k) run_step(k, std::true_type{});
  }
  for (; k < a.K; ++k) run_step(k, std::false_type{});
}

// kDoneT: temporal done-byte stores (the default: a wave's 64 done bytes are half a
// 128-B line, merged in the L2 with the other wave's half; +5.6% mean over three
// allocations at 262,144 envs, K = 2048, profiles/r03/done_stores/); variant bit 21 keeps
// the non-temporal stores (A/B)
// kNP (one-wave groups of a system with process noise, noise on; opt-in, variant bit
// 1<<25): a second wave per group draws the normals -- Philox + Box-Muller, ~1/5 of a
// PMSM / HR step (noise off: HR 32,768 x 2048 1,829 -> 1,461 us), and independent of the
// state -- up to kZSlots steps ahead into an LDS ring; the stepping wave reads them
// instead of drawing (bit-identical: the same normal3(seed, gid, tick) values).  The
// intent was a shorter dependent chain per stepping wave and work for the idle SIMDs of
// a small-N launch; measured, the pair is SLOWER (HR +42% at 32,768, +74% at 65,536; PMSM
// +4%, profiles/r04/np/), so the one-wave kernel draws its own by default.  Flags in LDS: zflag[0] = steps drawn, zflag[1] = steps consumed.  Only full
// groups pair (the last, ragged group's producer leaves at once and its stepping wave
// draws itself; a finished wave no longer holds up s_barrier).
template <class Sys>
__device__ __forceinline__ void noise_producer(const KArgs& a, int64_t base, int lane, uint64_t tick,
                                               float* s_z, int* zflag) {
  const uint64_t gid = (uint64_t)(a.gid0 + base + lane);
  for (int k = 0; k < a.K; ++k) {
    if (k >= kZSlots) {  // the stepping wave is done with step k - kZSlots's slot
      uint32_t spin = 0;
      while (spin < kZSpinCap &&
             __hip_atomic_load(&zflag[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) <= k - kZSlots) {
        __builtin_amdgcn_s_sleep(1);
        ++spin;
      }
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      if (spin >= kZSpinCap) return;  // never overwrite a slot still in use: stop drawing
    }
    float z[3];
    normal3(a.seed, gid, tick + (uint64_t)k, z);
    float* slot = s_z + (k % kZSlots) * 3 * 64 + lane;
    slot[0] = z[0];
    slot[64] = z[1];
    slot[128] = z[2];
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    if (lane == 0) __hip_atomic_store(&zflag[0], k + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}

template <class Sys, typename T, int B, int D, bool kNoDone = false, bool kDoneT = true, bool kZN = false>
__global__ __launch_bounds__(B) void k_rollout(KArgs a) {
  // DMA ring (a placeholder for systems that take no action)
  __shared__ __attribute__((aligned(16))) float s_act[Sys::kUsesAction ? dma_slots<D>() * act_slot_floats<Sys::A, B>() : 4];
  __shared__ __attribute__((aligned(16))) T s_obs[(Sys::kUsesAction ? 1 : 2) * B * Sys::O];
  const int tid = (int)threadIdx.x;
  const int64_t base = (int64_t)blockIdx.x * B;
  const int64_t i = base + tid;
  const int nb = (int)((a.n - base) < B ? (a.n - base) : B);
  const bool live = tid < nb;
  const uint64_t tick = *a.tick_in;
  if (blockIdx.x == 0 && tid == 0) {
    *a.counter_next = 0;
    *a.tick_out = tick + a.tick_adv;
  }
  Sys sys;
  sys.setup(a);
  int32_t steps = 0;
  bool any_reset = false;
  if (live) {
    sys.load(a, i);
    if (a.count_steps) steps = static_cast<const int32_t*>(a.pl[Sys::kStepPlane])[i];
  }
  if (nb == B && a.vec_ok)
    rollout_loop<Sys, T, B, true, D, kNoDone, kDoneT, false, kZN>(sys, steps, any_reset, a, base, tid, nb, tick,
                                                                  s_act, s_obs);
  else if (rag_full<Sys>() && B == 64 && a.vec_ok)  // the ragged last one-wave group: the full path, kRag
    rollout_loop<Sys, T, B, B == 64, D, kNoDone, kDoneT, false, kZN, B == 64>(sys, steps, any_reset, a, base, tid,
                                                                              nb, tick, s_act, s_obs);
  else
    rollout_loop<Sys, T, B, false, D, kNoDone, kDoneT, false, kZN>(sys, steps, any_reset, a, base, tid, nb, tick,
                                                                   s_act, s_obs);
  if (live) {
    sys.store(a, i);
    if (any_reset) sys.store_autoreset_extra(a, i);
    if (a.count_steps) static_cast<int32_t*>(a.pl[Sys::kStepPlane])[i] = steps;
  }
}

// one-wave groups + a noise-producer wave (kNP above): 128 threads per 64 envs, wave 1
// the producer; wave 0 is k_rollout<Sys, T, 64, D>'s wave with the normals read from LDS
template <class Sys, typename T, int D>
__global__ __launch_bounds__(128) void k_rollout_np(KArgs a) {
  constexpr int B = 64;
  __shared__ __attribute__((aligned(16))) float s_act[dma_slots<D>() * act_slot_floats<Sys::A, B>()];
  __shared__ __attribute__((aligned(16))) T s_obs[B * Sys::O];
  __shared__ float s_z[kZSlots * 3 * B];
  __shared__ int zflag[2];
  static_assert(Sys::kUsesAction && Sys::kNoise, "k_rollout_np: noisy systems with actions");
  const int tid = (int)threadIdx.x;
  if (tid == 0) zflag[0] = zflag[1] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * B;
  const int nb = (int)((a.n - base) < B ? (a.n - base) : B);
  const bool full = nb == B && a.vec_ok;
  if (tid >= B) {  // the producer wave (none for the last, ragged group)
    if (full) noise_producer<Sys>(a, base, tid - B, *a.tick_in, s_z, zflag);
    return;
  }
  const int64_t i = base + tid;
  const bool live = tid < nb;
  const uint64_t tick = *a.tick_in;
  if (blockIdx.x == 0 && tid == 0) {
    *a.counter_next = 0;
    *a.tick_out = tick + a.tick_adv;
  }
  Sys sys;
  sys.setup(a);
  int32_t steps = 0;
  bool any_reset = false;
  if (live) {
    sys.load(a, i);
    if (a.count_steps) steps = static_cast<const int32_t*>(a.pl[Sys::kStepPlane])[i];
  }
  if (full)
    rollout_loop<Sys, T, B, true, D, false, true, true>(sys, steps, any_reset, a, base, tid, nb, tick, s_act, s_obs,
                                                        s_z, zflag);
  else
    rollout_loop<Sys, T, B, false, D, false, true>(sys, steps, any_reset, a, base, tid, nb, tick, s_act, s_obs);
  if (live) {
    sys.store(a, i);
    if (any_reset) sys.store_autoreset_extra(a, i);
    if (a.count_steps) static_cast<int32_t*>(a.pl[Sys::kStepPlane])[i] = steps;
  }
}

// ------------------------------------------------------------------ split-lane rollout
// Small N (cfg5: 32,768 envs per GPU): one env per lane gives 512 one-wave groups for
// 1,024 SIMDs -- half the chip idles and every wave runs its step chain alone.  Here
// R = 2 adjacent lanes carry the same env (lane 2e + q, q = 0/1): both run the whole
// step (bit-identical arithmetic, same Philox draws), and the step's OUTPUT is split
// between them -- lane q stores half of the obs row (the wave's obs store stays one
// contiguous 64 x O/2-element instruction), q = 0 the reward, q = 1 the done byte, and
// only q = 0 enters the compact done list and writes the state back.  Twice the waves
// for the same per-wave instruction stream: pays where the step is cheap and the SIMDs
// otherwise idle (rollout_split).
typedef float f3v __attribute__((ext_vector_type(3)));
typedef f3v f3v_a4 __attribute__((aligned(4)));

// store W contiguous T's of v[] at p (p aligned to the row-half, W * sizeof(T) bytes)
template <typename T, int W>
__device__ __forceinline__ void store_half(T* p, const T* v) {
  constexpr int RB = W * (int)sizeof(T);
  if constexpr (RB == 12) {
    const f3v x = {(float)v[0], (float)v[1], (float)v[2]};
    __builtin_nontemporal_store(x, reinterpret_cast<f3v_a4*>(p));
  } else {
    using C = Chunk<RB>;
    using ct = typename C::t;
    const ct* src = reinterpret_cast<const ct*>(v);
#pragma unroll
    for (int j = 0; j < C::N; ++j) gstore<true>(reinterpret_cast<ct*>(p) + j, src[j]);
  }
}

// kNoDone: no done can occur in this launch (never-terminating system, no step
// counter; LORENZ3 with the reference's constants): step_body's done bookkeeping --
// compact list, auto-reset, step counter -- is compiled out (~25 of ~130 instructions
// per step), and the done byte stored is a constant 0.
// Actions (A = 2, 3): ONE 16-B row DMA per step (row_dma) moves the wave's 32 action
// rows into a row-major LDS slot (the launch needs vec_ok; otherwise every workgroup
// takes the gload path); the step reads its row with ordinary LDS loads after the
// vmcnt wait (the wait asm's
// memory clobber orders them after it, and the slot's address escapes into the DMA
// asm, so the compiler assumes the DMA writes it) -- the compiler then places the
// lgkmcnt wait where the action is first used, and the state-only part of the step
// (the RHS of the old state) overlaps the LDS latency.
// kPair (PMSM, k_rollout_pair): the lane pair SPLITS the step instead
// of repeating it (SysPMSM::step_pair: lane q integrates system q, one division and two
// square roots per lane, exchanged by DPP), and draws the slave's process noise two steps
// at a time: at an even step k lane 1 draws normal3(tick + k) -- its own, for step k --
// while lane 0 draws normal3(tick + k + 1) and hands it over (pair_swap) for step k + 1,
// so each lane runs one Philox + Box-Muller per two steps.  The same values as
// normal3(seed, gid, tick + k) at every step: bit-identical to k_rollout.
template <class Sys, typename T, int R, bool FULL, int D, bool kNoDone, int SV, bool kPair = false,
          bool kRag = false>  // kRag: the ragged last group on the full path (rollout_loop's)
__device__ __forceinline__ void split_loop(Sys& sys, int32_t& steps, bool& any_reset,
                                           const KArgs& a, int64_t base, int tid, int nb,
                                           uint64_t tick, float* s_act) {
  static_assert(R == 2 && Sys::O % 2 == 0, "split-lane rollout: two lanes per env");
  constexpr int H = Sys::O / R;  // obs elements stored per lane
  constexpr bool kRow = row_dma<Sys::A, 32>();  // one 16-B DMA per step (else 4-B per component)
  const int el = tid / R, q = tid % R;
  const bool lead = q == 0;
  const int64_t i = base + el;
  const bool live = (FULL && !kRag) || el < nb;
  const float* gact = static_cast<const float*>(a.act);
  // vector-memory ops every step issues after its DMA (lower bound): reward or done
  // (two exec-masked stores) + at least one obs store
  constexpr int kSt = 3;
  constexpr int kA = kRow ? 1 : Sys::A;
  constexpr int kSteady = kSt + (D - 1) * (kA + kSt);
  static_assert(D >= 1 && kSteady <= 63, "vmcnt immediate (6 bits on gfx9)");
  constexpr int kDmaSlots = dma_slots<D>();
  constexpr int kSlotF = kRow ? kRowRegionF : 64 * Sys::A;  // floats per slot
  const uint32_t m0_wave = __builtin_amdgcn_readfirstlane(lds_off(s_act));
  auto issue = [&](const float* src, int slot) __attribute__((always_inline)) {
    if constexpr (kRow) {
      dma16_nt(src, m0_wave + (uint32_t)(slot * kSlotF) * 4u);
    } else {
#pragma unroll
      for (int j = 0; j < Sys::A; ++j) dma4_nt(src + j, m0_wave + (uint32_t)((slot * Sys::A + j) * 64) * 4u);
    }
  };
  const int64_t dstride = a.n * Sys::A;
  // kRow: lane tid loads chunk tid mod C of the wave's 32-env slice; else: lane tid
  // loads its own env's components
  const int64_t src_el = kRag ? min(el, nb - 1) : el;
  const int src_chunk = kRag ? min(tid % (32 * Sys::A / 4), nb * Sys::A / 4 - 1) : tid % (32 * Sys::A / 4);
  const float* dsrc = kRow ? gact + base * Sys::A + 4 * src_chunk : gact + (base + src_el) * Sys::A;
  if constexpr (FULL) __builtin_amdgcn_s_waitcnt(0x0F70);
  if constexpr (FULL && Sys::kUsesAction) {
#pragma unroll
    for (int d = 0; d < D; ++d) issue(dsrc + (int64_t)(d < a.K ? d : a.K - 1) * dstride, d);
    dsrc += (int64_t)(D < a.K ? D : a.K - 1) * dstride;
  }
  float znext[3] = {0.0f, 0.0f, 0.0f};  // kPair: lane 0's normals for the next (odd) step
  float anext[Sys::A > 0 ? Sys::A : 1];  // !FULL: the next step's action row (prefetched)
  auto run_step = [&](int k, auto ladder) __attribute__((always_inline)) {
    const int64_t off = (int64_t)k * a.n;
    float act[Sys::A];
    if constexpr (Sys::kUsesAction) {
      if constexpr (FULL) {
        if constexpr (decltype(ladder)::value) ladder_wait<D, kA, kSt>(k);
        else wait_vmcnt<kSteady>();
        const float* slot = s_act + (k % kDmaSlots) * kSlotF;
        if constexpr (kRow) {
#pragma unroll
          for (int j = 0; j < Sys::A; ++j) act[j] = slot[el * Sys::A + j];
        } else {
          lds_read_act<Sys::A>(act, slot + tid, 64);
        }
        issue(dsrc, (k + D) % kDmaSlots);
        if (k + D + 1 < a.K) dsrc += dstride;
      } else if (live) {  // ragged / unaligned: the lane's row, one step ahead (rollout_loop)
        if (k == 0) {
#pragma unroll
          for (int j = 0; j < Sys::A; ++j) anext[j] = gload<true>(gact + i * Sys::A + j);
        }
#pragma unroll
        for (int j = 0; j < Sys::A; ++j) act[j] = anext[j];
        if (k + 1 < a.K) {
#pragma unroll
          for (int j = 0; j < Sys::A; ++j) anext[j] = gload<true>(gact + (off + a.n + i) * Sys::A + j);
        }
      }
    }
    T o[Sys::O];
    T rew = (T)0;
    bool did_reset;
    float zcur[3] = {0.0f, 0.0f, 0.0f};
    if constexpr (kPair) {
      if (live && (a.flags & LZ_FLAG_ADD_NOISE)) {  // (both lanes of a pair: the same `live`)
        if ((k & 1) == 0) {
          normal3(a.seed, (uint64_t)(a.gid0 + i), tick + (uint64_t)k + (lead ? 1u : 0u), zcur);
#pragma unroll
          for (int j = 0; j < 3; ++j) znext[j] = pair_swap(zcur[j]);
        } else {
#pragma unroll
          for (int j = 0; j < 3; ++j) zcur[j] = znext[j];
        }
      }
    }
    const uint8_t dflag = step_body<Sys, T, true, false, kNoDone, false, kPair ? 3 : 0>(
        sys, steps, a, i, live, act, tick + (uint64_t)k, k, o, rew, did_reset, nullptr, lead, zcur);
    any_reset = any_reset || did_reset;
    if (!live) return;
    if (lead) gstore<(SV & 2) == 0>(static_cast<T*>(a.rew) + off + i, rew);
    else gstore<(SV & 1) == 0>(a.done + off + i, kNoDone ? (uint8_t)0 : dflag);
    // this lane's half row: elements [q*H, q*H + H) of env i = elements tid*H of the
    // block's contiguous obs slice
    T* p = static_cast<T*>(a.obs) + (off + base) * Sys::O + (int64_t)tid * H;
    T h[H];
#pragma unroll
    for (int j = 0; j < H; ++j) h[j] = q ? o[H + j] : o[j];
    if constexpr ((SV & 4) != 0) {  // A/B: plain (temporal) obs stores
#pragma unroll
      for (int j = 0; j < H; ++j) p[j] = h[j];
    } else {
      store_half<T, H>(p, h);
    }
  };
  int k = 0;
  if constexpr (FULL && Sys::kUsesAction) {
    const int kp = D < a.K ? D : a.K;
    for (; k < kp; ++k) run_step(k, std::true_type{});
  }
  for (; k < a.K; ++k) run_step(k, std::false_type{});
}

// SV: temporal instead of non-temporal stores -- bit 0 the done bytes (the default: a
// wave's 32 done bytes are a quarter of a 128-B line; temporal stores let the L2 merge
// the four waves' quarters before the line leaves, +7.8% at 32,768 envs, K = 2048,
// profiles/r03/done_stores/), bit 1 the rewards, bit 2 the obs half rows (A/B only,
// variant bits 18-20 = 1, 3, 4, 7 select SV = 0, 3, 5, 7)
template <class Sys, typename T, int R, int D, bool kNoDone = false, int SV = 1, bool kPair = false>
__device__ __forceinline__ void rollout_split_body(KArgs a) {
  constexpr int E = 64 / R;  // envs per one-wave workgroup
  __shared__ __attribute__((aligned(16))) float s_act[dma_slots<D>() * (row_dma<Sys::A, 32>() ? kRowRegionF : 64 * Sys::A)];
  const int tid = (int)threadIdx.x;
  const int64_t base = (int64_t)blockIdx.x * E;
  const int el = tid / R;
  const int64_t i = base + el;
  const int nb = (int)((a.n - base) < E ? (a.n - base) : E);
  const bool live = el < nb;
  const bool lead = (tid % R) == 0;
  const uint64_t tick = *a.tick_in;
  if (blockIdx.x == 0 && tid == 0) {
    *a.counter_next = 0;
    *a.tick_out = tick + a.tick_adv;
  }
  Sys sys;
  sys.setup(a);
  int32_t steps = 0;
  bool any_reset = false;
  if (live) {
    sys.load(a, i);
    if (a.count_steps) steps = static_cast<const int32_t*>(a.pl[Sys::kStepPlane])[i];
  }
  if (nb == E && a.vec_ok)
    split_loop<Sys, T, R, true, D, kNoDone, SV, kPair>(sys, steps, any_reset, a, base, tid, nb, tick, s_act);
  else if (rag_full<Sys>() && a.vec_ok)  // the ragged last group: the full path, kRag
    split_loop<Sys, T, R, true, D, kNoDone, SV, kPair, true>(sys, steps, any_reset, a, base, tid, nb, tick, s_act);
  else
    split_loop<Sys, T, R, false, D, kNoDone, SV, kPair>(sys, steps, any_reset, a, base, tid, nb, tick, s_act);
  if (live && lead) {
    sys.store(a, i);
    if (any_reset) sys.store_autoreset_extra(a, i);
    if (a.count_steps) static_cast<int32_t*>(a.pl[Sys::kStepPlane])[i] = steps;
  }
}
template <class Sys, typename T, int R, int D, bool kNoDone = false, int SV = 1>
__global__ __launch_bounds__(64) void k_rollout_split(KArgs a) {
  rollout_split_body<Sys, T, R, D, kNoDone, SV>(a);
}
// The lane-pair rollout (split_loop kPair; PMSM): the split-lane kernel's layout and I/O,
// the step itself divided between the two lanes (SysPMSM::step_pair).
template <class Sys, typename T, int D>
__global__ __launch_bounds__(64) void k_rollout_pair(KArgs a) {
  rollout_split_body<Sys, T, 2, D, false, 1, true>(a);
}

// ------------------------------------------------------------------ launchers
static inline int64_t grid_for(int64_t n) { return (n + kBlock - 1) / kBlock; }

// Two lanes per env in the small-N rollout (variant bit 256 forces one, 512 forces two):
// by default for LORENZ3 f32 from 32,768 envs (below 256 x CUs = 65,536 the one-wave
// path runs, launch_rollout_d).
// Measured (profiles/r01/ab_rollout_*.json, K = 2048): +11% at 32,768 and +13% at
// 65,536 envs; slower at 16,384 (the wave's step chain, not the SIMD count, bounds it
// there) and for PMSM at any N (its step is 3-4x the instructions: doubling them costs
// more than the extra waves recover).
// The lane-pair PMSM rollout (k_rollout_pair, SysPMSM::step_pair): by default where its
// 32-env waves number more than 2 and at most 4 per CU (16,384 < N <= 32,768 on 256 CUs),
// measured: PMSM 32,768 x 2048 2,088 -> 1,890 us, 28,672 2,087 -> 1,950.  At 2 waves per
// CU the one-env-per-lane waves (one per CU) win (16,384: 1,934 vs 2,045 us), and with
// more, two 32-env waves per SIMD lose to one 64-env wave (49,152: 1,956 vs 2,577;
// 65,536: 1,958 vs 2,534; 131,072: 3,009 vs 4,359; 262,144: 5,982 vs 8,092;
// profiles/r06/pair/).  Variant bit 1<<27 forces it at any N, 1<<28 disables it; the
// other kernels' force bits (256 / 512 split choice, 1<<23 / 1<<24 group shape, 1<<25
// producer wave, 1<<26 kZN) select theirs.
template <class Sys>
static inline bool rollout_pair(const KArgs& a) {
  if constexpr (!std::is_same<Sys, SysPMSM>::value) {
    return false;
  } else {
    if (a.variant & (1 << 28)) return false;
    if (a.variant & (1 << 27)) return true;
    if (a.variant & (256 | 512 | (1 << 23) | (1 << 24) | (1 << 25) | (1 << 26))) return false;
    const int64_t cus = a.num_cus > 0 ? a.num_cus : 256, waves = (a.n + 31) / 32;
    return waves > 2 * cus && waves <= 4 * cus;
  }
}

template <class Sys>
static inline bool rollout_split(const KArgs& a) {
  if constexpr (Sys::O % 2 != 0) return false;
  if (a.variant & 256) return false;
  if (a.variant & 512) return true;
  return std::is_same<Sys, SysL3<float>>::value && a.n >= 32768;
}

// Which rollout kernel launch_rollout_d picks (lz_get_launch_shape reports it): 0 the
// 256-lane k_rollout, 1 one-wave k_rollout, 2 the split-lane kernel; no_done = the
// done-free instantiation.
struct RolloutPlan {
  int kind;  // 0 256-lane, 1 one-wave, 2 split lanes, 3 lane pair (PMSM)
  bool no_done;
  bool np;  // one-wave groups with a noise-producer wave (k_rollout kNP)
};
template <class Sys>
static RolloutPlan rollout_plan(const KArgs& a) {
  const int64_t cus = a.num_cus > 0 ? a.num_cus : 256;
  const int64_t one_wave_below =
      std::is_same<Sys, SysL3<float>>::value   ? (int64_t)kBlock * cus
      : std::is_same<Sys, SysL4<float>>::value ? (int64_t)kBlock * cus * 3 / 4
                                               : 2 * 256 * (int64_t)kBlock;
  bool nd = false;
  if constexpr (never_terminates<Sys>::value && !Sys::kNoise) nd = no_done<Sys>(a) && !(a.variant & 2048);
  if (rollout_pair<Sys>(a)) return {3, false, false};
  if ((a.n < one_wave_below || (a.variant & (1 << 24))) && !(a.variant & (1 << 23))) {
    if (rollout_split<Sys>(a)) return {2, nd, false};
    // variant bit 1<<25: with a noise-producer wave (k_rollout_np; A/B, measured slower:
    // HR f32 32,768 x 2048 1,840 -> 2,610 us, 65,536 1,823 -> 3,175; PMSM 2,190 -> 2,274 /
    // 2,111 -> 2,191, profiles/r04/np/)
    const bool np = Sys::kNoise && Sys::kUsesAction && (a.flags & LZ_FLAG_ADD_NOISE) && (a.variant & (1 << 25));
    return {1, false, np};
  }
  return {0, nd, false};
}

template <class Sys, typename T, int D, int DS = D>  // DS: the split-lane kernel's distance
static void launch_rollout_d(const KArgs& a, hipStream_t s) {
  // fewer 256-env workgroups than CUs: one-wave groups (variant bit 1<<23: the 256-lane
  // kernel at any N, A/B).  At 65,536 envs on 256 CUs the 256-lane kernel (one wave per
  // SIMD, 64 envs each) beats the split-lane one (two per SIMD, 32 envs each, every step
  // computed twice) by 15% (profiles/r03/done_stores/, three allocations per variant);
  // at 32,768 half the CUs would idle and it loses by 27%.  LORENZ4 float32 the same
  // way (profiles/r03/rollout_xover/, two allocations per variant): 65,536 envs 1,412 ->
  // 908 us per 2048-step launch, 98,304 1,808 -> 1,476; 32,768 615 vs 820 (one-wave
  // kept).  PMSM and HR (3-4x the instructions per step) are faster with one-wave groups
  // at 32,768-98,304 (2,209 vs 2,493 / 1,823 vs 2,038 us at 65,536): the round-2 bound.
  // LORENZ4's crossover lies lower, between 160 and 192 workgroups per 256 CUs (40,960
  // envs: 658 vs 918 us; 49,152: 870 vs 925-1,096; 57,344: 908 vs 1,007): from 3/4 x 256 x CUs.
  // (rollout_plan: variant bit 1<<24 forces one-wave groups at any N, 1<<23 the 256-lane
  // kernel, 2048 keeps the done path -- A/B)
  const RolloutPlan plan = rollout_plan<Sys>(a);
  if constexpr (std::is_same<Sys, SysPMSM>::value) {
    if (plan.kind == 3) {
      hipLaunchKernelGGL((k_rollout_pair<Sys, T, DS>), dim3((unsigned)((a.n + 31) / 32)), dim3(64), 0, s, a);
      return;
    }
  }
  if (plan.kind != 0) {
    if (plan.kind == 2) {
      const dim3 g((unsigned)((a.n + 31) / 32));
      if constexpr (never_terminates<Sys>::value && !Sys::kNoise) {
        if (plan.no_done) {
          switch ((a.variant >> 18) & 7) {  // A/B: store policy (SV; 1 = the default)
            case 1: hipLaunchKernelGGL((k_rollout_split<Sys, T, 2, DS, true, 0>), g, dim3(64), 0, s, a); return;
            case 3: hipLaunchKernelGGL((k_rollout_split<Sys, T, 2, DS, true, 3>), g, dim3(64), 0, s, a); return;
            case 4: hipLaunchKernelGGL((k_rollout_split<Sys, T, 2, DS, true, 5>), g, dim3(64), 0, s, a); return;
            case 7: hipLaunchKernelGGL((k_rollout_split<Sys, T, 2, DS, true, 7>), g, dim3(64), 0, s, a); return;
            default: break;
          }
          hipLaunchKernelGGL((k_rollout_split<Sys, T, 2, DS, true>), g, dim3(64), 0, s, a);
          return;
        }
      }
      hipLaunchKernelGGL((k_rollout_split<Sys, T, 2, DS>), g, dim3(64), 0, s, a);
    } else if constexpr (Sys::kNoise && Sys::kUsesAction) {
      if (plan.np)
        hipLaunchKernelGGL((k_rollout_np<Sys, T, D>), dim3((unsigned)((a.n + 63) / 64)), dim3(128), 0, s, a);
      else if (a.variant & (1 << 26))  // A/B: the next step's normals drawn during this step (kZN)
        hipLaunchKernelGGL((k_rollout<Sys, T, 64, D, false, true, true>), dim3((unsigned)((a.n + 63) / 64)),
                           dim3(64), 0, s, a);
      else
        hipLaunchKernelGGL((k_rollout<Sys, T, 64, D>), dim3((unsigned)((a.n + 63) / 64)), dim3(64), 0, s, a);
    } else {
      hipLaunchKernelGGL((k_rollout<Sys, T, 64, D>), dim3((unsigned)((a.n + 63) / 64)), dim3(64),
                         0, s, a);
    }
  } else {
    if constexpr (never_terminates<Sys>::value && !Sys::kNoise) {
      if (plan.no_done) {
        if (a.variant & (1 << 21))  // A/B: non-temporal done stores
          hipLaunchKernelGGL((k_rollout<Sys, T, kBlock, D, true, false>), dim3((unsigned)grid_for(a.n)),
                             dim3(kBlock), 0, s, a);
        else
          hipLaunchKernelGGL((k_rollout<Sys, T, kBlock, D, true>), dim3((unsigned)grid_for(a.n)),
                             dim3(kBlock), 0, s, a);
        return;
      }
    }
    if constexpr (Sys::kNoise && Sys::kUsesAction) {
      if (a.variant & (1 << 26)) {  // A/B: kZN, as above
        hipLaunchKernelGGL((k_rollout<Sys, T, kBlock, D, false, true, true>), dim3((unsigned)grid_for(a.n)),
                           dim3(kBlock), 0, s, a);
        return;
      }
    }
    if (a.variant & (1 << 21))  // A/B: non-temporal done stores
      hipLaunchKernelGGL((k_rollout<Sys, T, kBlock, D, false, false>), dim3((unsigned)grid_for(a.n)),
                         dim3(kBlock), 0, s, a);
    else
      hipLaunchKernelGGL((k_rollout<Sys, T, kBlock, D>), dim3((unsigned)grid_for(a.n)), dim3(kBlock),
                         0, s, a);
  }
}

// kVariants: instantiate the step-kernel tuning variants (A/B tools use LORENZ3 and
// PMSM; the other systems always run the default variant)
template <class Sys, typename T, bool kVariants = false>
static int launch_all(int which, const KArgs& a, hipStream_t s) {
  const dim3 grid((unsigned)grid_for(a.n)), block(kBlock);
  const int tiles = which == 1 && multi_step_ok<Sys>::value ? step_tiles<Sys>(a) : 1;
  if (which == 0)
    hipLaunchKernelGGL((k_reset<Sys, T>), grid, block, 0, s, a);
  else if (tiles > 1) {
    if constexpr (multi_step_ok<Sys>::value) {
      const int64_t per = (int64_t)kBlock * tiles;
      const dim3 g((unsigned)((a.n + per - 1) / per));
      if (tiles == 2) hipLaunchKernelGGL((k_step_multi<Sys, T, 2>), g, block, 0, s, a);
      else if (a.variant & (1 << 22))  // A/B: temporal done stores
        hipLaunchKernelGGL((k_step_multi<Sys, T, 4, true>), g, block, 0, s, a);
      else hipLaunchKernelGGL((k_step_multi<Sys, T, 4>), g, block, 0, s, a);
    }
  } else if (which == 1 && !kVariants) {
    hipLaunchKernelGGL((k_step<Sys, T, 0>), grid, block, 0, s, a);
  } else if (which == 1) {
    switch (a.variant & 63) {
#define LZ_STEP_V(VV)                                                                   \
  case VV:                                                                              \
    hipLaunchKernelGGL((k_step<Sys, T, VV>),                                            \
                       dim3((unsigned)((a.n + step_block<VV>() - 1) / step_block<VV>())), \
                       dim3(step_block<VV>()), 0, s, a);                                \
    break;
      LZ_STEP_V(1) LZ_STEP_V(2) LZ_STEP_V(3) LZ_STEP_V(4) LZ_STEP_V(5)
      LZ_STEP_V(8) LZ_STEP_V(16) LZ_STEP_V(24) LZ_STEP_V(32)
#undef LZ_STEP_V
      default: hipLaunchKernelGGL((k_step<Sys, T, 0>), grid, block, 0, s, a); break;
    }
  } else if constexpr (kVariants) {
    if (a.variant & 1024) launch_rollout_d<Sys, T, 3>(a, s);  // A/B: prefetch distance 3
    // A/B: split-lane distance 15 (vmcnt allows 59 ops in flight): no change at 32,768 -
    // 131,071 envs (profiles/r03/rollout/ab_split_dma_distance_15_rejected.json)
    else if (a.variant & 4096) launch_rollout_d<Sys, T, kDmaDist, 15>(a, s);
    else launch_rollout_d<Sys, T, kDmaDist>(a, s);
  } else {
    launch_rollout_d<Sys, T, kDmaDist>(a, s);
  }
  return (int)hipGetLastError();
}

static int dispatch(int which, int system, int f64, const KArgs& a, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (system) {
    case LZ_SYS_LORENZ3:
      return f64 ? launch_all<SysL3<double>, double>(which, a, s)
                 : launch_all<SysL3<float>, float, true>(which, a, s);
    case LZ_SYS_LORENZ4:
      return f64 ? launch_all<SysL4<double>, double>(which, a, s)
                 : launch_all<SysL4<float>, float>(which, a, s);
    case LZ_SYS_LORENZ3 + kSysRK4:
      return f64 ? launch_all<SysL3RK4<double>, double>(which, a, s)
                 : launch_all<SysL3RK4<float>, float>(which, a, s);
    case LZ_SYS_LORENZ4 + kSysRK4:
      return f64 ? launch_all<SysL4RK4<double>, double>(which, a, s)
                 : launch_all<SysL4RK4<float>, float>(which, a, s);
    case LZ_SYS_PMSM:
      return launch_all<SysPMSM, float, true>(which, a, s);
    case LZ_SYS_HR:
      return f64 ? launch_all<SysHR<double>, double>(which, a, s)
                 : launch_all<SysHR<float>, float>(which, a, s);
    case LZ_SYS_T1:
      return f64 ? launch_all<SysT1<double>, double>(which, a, s)
                 : launch_all<SysT1<float>, float>(which, a, s);
    case LZ_SYS_T2:
      return f64 ? launch_all<SysT2<double>, double>(which, a, s)
                 : launch_all<SysT2<float>, float>(which, a, s);
    case LZ_SYS_TP:
      return f64 ? launch_all<SysTP<double>, double>(which, a, s)
                 : launch_all<SysTP<float>, float>(which, a, s);
    case LZ_SYS_SC:
      return f64 ? launch_all<SysSC<double>, double>(which, a, s)
                 : launch_all<SysSC<float>, float>(which, a, s);
  }
  return (int)hipErrorInvalidValue;
}

// ------------------------------------------------------------------ launch shapes
// What lz_step / lz_rollout launch for these arguments (lz_get_launch_shape): kernel code,
// envs per wave, waves per workgroup, workgroups, flags (lorenz_env.h LZ_KERNEL_* /
// LZ_SHAPE_*) -- the same decisions launch_all / launch_rollout_d take.
template <class Sys, typename T>
static int env_shape_t(int which, const KArgs& a, int32_t* o) {
  if (which == 1) {
    const int tiles = multi_step_ok<Sys>::value ? step_tiles<Sys>(a) : 1;
    const int64_t per = (int64_t)kBlock * tiles;
    o[0] = tiles > 1 ? LZ_KERNEL_STEP_MULTI : LZ_KERNEL_STEP;
    o[1] = 64;
    o[2] = kBlock / 64;
    o[3] = (int32_t)((a.n + per - 1) / per);
    o[4] = 0;
    return 0;
  }
  const RolloutPlan p = rollout_plan<Sys>(a);
  o[0] = p.kind == 0   ? LZ_KERNEL_ROLLOUT
         : p.kind == 1 ? LZ_KERNEL_ROLLOUT_WAVE
         : p.kind == 2 ? LZ_KERNEL_ROLLOUT_SPLIT
                       : LZ_KERNEL_ROLLOUT_PAIR;
  o[1] = p.kind >= 2 ? 32 : 64;
  o[2] = p.kind == 0 ? kBlock / 64 : p.np ? 2 : 1;
  const int64_t per = p.kind == 0 ? kBlock : p.kind == 1 ? 64 : 32;
  o[3] = (int32_t)((a.n + per - 1) / per);
  o[4] = p.no_done ? LZ_SHAPE_NO_DONE : 0;
  return 0;
}

int env_launch_shape(int which, int system, int f64, const KArgs& a, int32_t* o) {
  switch (system) {
    case LZ_SYS_LORENZ3: return f64 ? env_shape_t<SysL3<double>, double>(which, a, o) : env_shape_t<SysL3<float>, float>(which, a, o);
    case LZ_SYS_LORENZ4: return f64 ? env_shape_t<SysL4<double>, double>(which, a, o) : env_shape_t<SysL4<float>, float>(which, a, o);
    case LZ_SYS_LORENZ3 + kSysRK4:
      return f64 ? env_shape_t<SysL3RK4<double>, double>(which, a, o) : env_shape_t<SysL3RK4<float>, float>(which, a, o);
    case LZ_SYS_LORENZ4 + kSysRK4:
      return f64 ? env_shape_t<SysL4RK4<double>, double>(which, a, o) : env_shape_t<SysL4RK4<float>, float>(which, a, o);
    case LZ_SYS_PMSM: return env_shape_t<SysPMSM, float>(which, a, o);
    case LZ_SYS_HR: return f64 ? env_shape_t<SysHR<double>, double>(which, a, o) : env_shape_t<SysHR<float>, float>(which, a, o);
    case LZ_SYS_T1: return f64 ? env_shape_t<SysT1<double>, double>(which, a, o) : env_shape_t<SysT1<float>, float>(which, a, o);
    case LZ_SYS_T2: return f64 ? env_shape_t<SysT2<double>, double>(which, a, o) : env_shape_t<SysT2<float>, float>(which, a, o);
    case LZ_SYS_TP: return f64 ? env_shape_t<SysTP<double>, double>(which, a, o) : env_shape_t<SysTP<float>, float>(which, a, o);
    case LZ_SYS_SC: return f64 ? env_shape_t<SysSC<double>, double>(which, a, o) : env_shape_t<SysSC<float>, float>(which, a, o);
  }
  return (int)hipErrorInvalidValue;
}

// ------------------------------------------------------------------ resident step server
// lz_resident_step (lz_internal.h ResBox / ResMember, the request lines): the per-env
// drop-in classes step ONE env per env.step() call, and a launch + stream synchronisation
// per call costs 20-27 us (profiles/r01/dropin).  This kernel stays on the GPU between
// calls: one wave per registered handle serves that handle's requests with the same
// step_body as k_step (state in registers, tick += 1 per request, injected noise staged
// through LDS), the reply going straight into host memory; one poller wave reads every
// member's request line and hands new requests (tag + inline inputs) to the member waves
// through LDS.  Bounded: every wave leaves on a stop granule or after idle_ticks without
// a new request (the shared flag in LDS), so the launch ends as a whole and a relaunch
// includes every handle.
struct ResShared {
  int exit_;
  unsigned long long last;                  // wall_clock64() of the latest new request / reply
  uint32_t req[kRsMaxHandles];              // the newest request tag handed to each member
  uint32_t pay[kRsMaxHandles][kRsLineWords];  // its inline input words
  uint64_t rep[kRsMaxHandles][kRsReplyWords / 2];  // a one-env member's reply words (as 2 x 32 b)
};

__device__ __forceinline__ uint32_t rs_tag(int64_t seq) { return (uint32_t)seq & kRsTagMask; }

template <class Sys, typename T>
__device__ __forceinline__ void resident_serve(const ResMember& m, int wave, ResShared* sh, double* s_nz) {
  const KArgs& a = m.a;
  const ResBox& box = m.box;
  const int lane = (int)(threadIdx.x & 63u);
  const bool live = lane < a.n;
  const bool inl = box.inline_words >= 0;  // wave-uniform
  Sys sys;
  sys.setup(a);
  int32_t steps = 0;
  if (live) {
    sys.load(a, lane);
    if (a.count_steps) steps = static_cast<const int32_t*>(a.pl[Sys::kStepPlane])[lane];
    // the published copy starts as the planes (every plane, byte for byte)
    for (int p = 0; p < kMaxPlanes; ++p) {
      const int es = box.pub_es[p];
      if (es == 8) static_cast<uint64_t*>(box.pub[p])[lane] = static_cast<const uint64_t*>(a.pl[p])[lane];
      else if (es == 4) static_cast<uint32_t*>(box.pub[p])[lane] = static_cast<const uint32_t*>(a.pl[p])[lane];
      if (box.reply && es) {  // and the reply's plane words (planes a step does not store)
        uint32_t* w = reinterpret_cast<uint32_t*>(sh->rep[wave]) + box.rep_pub[p];
        w[0] = static_cast<const uint32_t*>(a.pl[p])[0];
        if (es == 8) w[1] = static_cast<const uint32_t*>(a.pl[p])[1];
      }
    }
  }
  uint64_t tick = *a.tick_in;
  if (lane == 0) *a.counter_next = 0;  // as k_step leaves it for the launch that follows
  KArgs b = a;
  b.noise = box.use_noise ? s_nz : nullptr;
  b.term_obs = nullptr;
  KArgs pubk = a;  // sys.store into the published planes
#pragma unroll
  for (int p = 0; p < kMaxPlanes; ++p) pubk.pl[p] = box.pub[p];
  KArgs pubr = a;  // ... or into the reply's words in LDS (one env, index 0)
#pragma unroll
  for (int p = 0; p < kMaxPlanes; ++p)
    pubr.pl[p] = box.rep_pub[p] >= 0 ? reinterpret_cast<uint32_t*>(sh->rep[wave]) + box.rep_pub[p] : nullptr;
  int64_t next = box.next;
  for (;;) {
    int c = 0;
    if (lane == 0) {  // LDS only: the poller reads host memory
      const uint32_t want = rs_tag(next);
      for (;;) {
        if (__hip_atomic_load(&sh->req[wave], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == want) {
          c = 1;
          break;
        }
        if (__hip_atomic_load(&sh->exit_, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
          c = -1;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    c = __shfl(c, 0, 64);
    if (c < 0) break;
    float act[Sys::A > 0 ? Sys::A : 1];
    if (live) {
      if (inl) {  // one env (lane 0): the inputs came in the request line, now in LDS
        const uint32_t* w = sh->pay[wave];
#pragma unroll
        for (int j = 0; j < Sys::A; ++j) act[j] = j < box.act_words ? __uint_as_float(w[j]) : 0.0f;
        if (box.use_noise) {
#pragma unroll
          for (int j = 0; j < 3; ++j)
            s_nz[j] = __hiloint2double((int)w[box.act_words + 2 * j + 1], (int)w[box.act_words + 2 * j]);
        }
      } else {
#pragma unroll
        for (int j = 0; j < Sys::A; ++j)
          act[j] = __hip_atomic_load(box.act + lane * Sys::A + j, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_SYSTEM);
        if (box.use_noise) {  // the three loads in flight together, then into LDS
          double nzv[3];
#pragma unroll
          for (int j = 0; j < 3; ++j)
            nzv[j] = __hip_atomic_load(box.noise + lane * 3 + j, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
#pragma unroll
          for (int j = 0; j < 3; ++j) s_nz[lane * 3 + j] = nzv[j];
        }
      }
    }
    T o[Sys::O];
    T rew = (T)0;
    bool did_reset;
    const uint8_t d = step_body<Sys, T, false>(sys, steps, b, lane, live, act, tick, 0, o, rew,
                                               did_reset);
    if (box.reply) {  // one env: the reply as tagged granules (ResBox), one store per lane
      uint32_t* w = reinterpret_cast<uint32_t*>(sh->rep[wave]);
      if (live) {  // lane 0 lays the words out in LDS (the planes through the LDS copy)
#pragma unroll
        for (int j = 0; j < Sys::O; ++j) reinterpret_cast<T*>(w + box.rep_obs)[j] = o[j];
        *reinterpret_cast<T*>(w + box.rep_rew) = rew;
        w[box.rep_done] = d;
        sys.store(pubr, 0);
        if (a.count_steps) *static_cast<int32_t*>(pubr.pl[Sys::kStepPlane]) = steps;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (lane < box.rep_words)
        __hip_atomic_store(box.reply + lane, ((uint64_t)rs_tag(next) << 32) | w[lane], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    } else {
      if (live) {
#pragma unroll
        for (int j = 0; j < Sys::O; ++j) static_cast<T*>(box.obs)[lane * Sys::O + j] = o[j];
        static_cast<T*>(box.rew)[lane] = rew;
        box.done[lane] = d;
        sys.store(pubk, lane);
        if (a.count_steps) static_cast<int32_t*>(pubk.pl[Sys::kStepPlane])[lane] = steps;
      }
      // the outputs of the whole wave reach host memory before the reply (release)
      if (lane == 0) __hip_atomic_store(box.resp, next, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    tick += 1;
    if (lane == 0)
      __hip_atomic_fetch_max(&sh->last, (unsigned long long)wall_clock64(), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
    ++next;
  }
  if (live) {
    sys.store(a, lane);
    if (a.count_steps) static_cast<int32_t*>(a.pl[Sys::kStepPlane])[lane] = steps;
  }
  if (lane == 0) *a.tick_out = tick;
}

// The poller wave: member k's request line is granules 8k .. 8k+7 of `lines` (mapped host
// memory); lane 4k + q reads granules 8k + 2q and 8k + 2q + 1 (two 8-B loads issued
// together: one PCIe round trip per poll for every member).  Line k is accepted when
// granule 0's tag differs from the last one handed over and every granule the member
// uses (inline_words, at least 1) carries that tag; then the four lanes copy the data
// words into LDS and lane 4k hands the tag over (release, workgroup scope).  An all-ones
// granule 0 is the stop command.
__device__ void resident_poll(const ResMember* __restrict__ table, int n, const uint64_t* lines,
                              ResShared* sh, uint64_t idle_ticks) {
  const int lane = (int)(threadIdx.x & 63u);
  const int k = lane >> 2, q = lane & 3;
  const bool mine = k < n;
  int ng = 1;
  if (mine && table[k].box.inline_words > 1) ng = table[k].box.inline_words;
  // a member on the mailbox path (inline_words < 0) reads its inputs from host memory
  // after the LDS hand-off: the poller orders the host's mailbox stores before that hand-off
  // with one system-scope acquire per accepted request
  const bool mailbox = mine && table[k].box.inline_words < 0;
  const uint64_t* src = lines + (int64_t)k * kRsLineWords + 2 * q;
  uint32_t seen = 0xffffffffu;  // no tag: the first pass hands over every line (a request
                                // may predate the launch)
  for (;;) {
    uint64_t g0 = 0, g1 = 0;
    if (mine) {
      g0 = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      g1 = __hip_atomic_load(src + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    const uint32_t tag_a = (uint32_t)(g0 >> 32), tag_b = (uint32_t)(g1 >> 32);
    const uint32_t t0 = (uint32_t)__shfl((int)tag_a, lane & ~3, 64);  // the line's granule 0
    const bool stop = mine && q == 0 && g0 == ~0ull;
    if (__ballot(stop)) break;  // stop: every wave leaves
    const bool ok = mine && (2 * q >= ng || tag_a == t0) && (2 * q + 1 >= ng || tag_b == t0);
    const unsigned long long okm = __ballot(ok);
    const bool whole = ((okm >> (4 * k)) & 0xfull) == 0xfull;
    const bool fresh = mine && whole && t0 != seen;
    if (__ballot(fresh && mailbox)) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    if (fresh) {
      if (2 * q < ng) sh->pay[k][2 * q] = (uint32_t)g0;
      if (2 * q + 1 < ng) sh->pay[k][2 * q + 1] = (uint32_t)g1;
      seen = t0;
    }
    if (fresh && q == 0)
      __hip_atomic_store(&sh->req[k], t0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (__ballot(fresh)) {
      if (lane == 0)
        __hip_atomic_fetch_max(&sh->last, (unsigned long long)wall_clock64(), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
      continue;
    }
    bool idle = false;
    if (lane == 0) {
      const unsigned long long last =
          __hip_atomic_load(&sh->last, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      idle = wall_clock64() - last > idle_ticks;
    }
    if (__shfl((int)idle, 0, 64)) break;
    __builtin_amdgcn_s_sleep(1);
  }
  if (lane == 0) __hip_atomic_store(&sh->exit_, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// kWaves: the register budget -- up to 7 handles (8 waves, 2 per SIMD: 256 VGPRs, the
// float64 RK4 bodies do not spill) or up to 15 (16 waves: 128 VGPRs)
template <int kWaves>
__global__ __launch_bounds__(64 * kWaves) void k_resident_multi(
    const ResMember* __restrict__ table, int n, const uint64_t* lines, uint64_t idle_ticks) {
  __shared__ ResShared sh;
  __shared__ double s_nz[kRsMaxHandles][64 * 3];
  // wave-uniform to the compiler too: the member's fields are scalar loads, and the
  // PMSM bias table pointer can feed its scalar load (SysPMSM::sload2)
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  if (threadIdx.x == 0) {
    sh.exit_ = 0;
    sh.last = wall_clock64();
  }
  if ((int)threadIdx.x < n) sh.req[threadIdx.x] = rs_tag(table[threadIdx.x].box.next - 1);
  __syncthreads();
  if (wave == n) {
    resident_poll(table, n, lines, &sh, idle_ticks);
    return;
  }
  const ResMember& m = table[wave];
  const int key = m.system * 2 + m.f64;
  switch (key) {  // wave-uniform: each wave runs its own handle's system
    case LZ_SYS_LORENZ3 * 2: resident_serve<SysL3<float>, float>(m, wave, &sh, s_nz[wave]); break;
    case LZ_SYS_LORENZ3 * 2 + 1: resident_serve<SysL3<double>, double>(m, wave, &sh, s_nz[wave]); break;
    case LZ_SYS_LORENZ4 * 2: resident_serve<SysL4<float>, float>(m, wave, &sh, s_nz[wave]); break;
    case LZ_SYS_LORENZ4 * 2 + 1: resident_serve<SysL4<double>, double>(m, wave, &sh, s_nz[wave]); break;
    case (LZ_SYS_LORENZ3 + kSysRK4) * 2: resident_serve<SysL3RK4<float>, float>(m, wave, &sh, s_nz[wave]); break;
    case (LZ_SYS_LORENZ3 + kSysRK4) * 2 + 1:
      resident_serve<SysL3RK4<double>, double>(m, wave, &sh, s_nz[wave]);
      break;
    case (LZ_SYS_LORENZ4 + kSysRK4) * 2: resident_serve<SysL4RK4<float>, float>(m, wave, &sh, s_nz[wave]); break;
    case (LZ_SYS_LORENZ4 + kSysRK4) * 2 + 1:
      resident_serve<SysL4RK4<double>, double>(m, wave, &sh, s_nz[wave]);
      break;
    case LZ_SYS_PMSM * 2: resident_serve<SysPMSM, float>(m, wave, &sh, s_nz[wave]); break;
    case LZ_SYS_HR * 2: resident_serve<SysHR<float>, float>(m, wave, &sh, s_nz[wave]); break;
    case LZ_SYS_HR * 2 + 1: resident_serve<SysHR<double>, double>(m, wave, &sh, s_nz[wave]); break;
    case LZ_SYS_T1 * 2: resident_serve<SysT1<float>, float>(m, wave, &sh, s_nz[wave]); break;
    case LZ_SYS_T1 * 2 + 1: resident_serve<SysT1<double>, double>(m, wave, &sh, s_nz[wave]); break;
    case LZ_SYS_T2 * 2: resident_serve<SysT2<float>, float>(m, wave, &sh, s_nz[wave]); break;
    case LZ_SYS_T2 * 2 + 1: resident_serve<SysT2<double>, double>(m, wave, &sh, s_nz[wave]); break;
    case LZ_SYS_TP * 2: resident_serve<SysTP<float>, float>(m, wave, &sh, s_nz[wave]); break;
    case LZ_SYS_TP * 2 + 1: resident_serve<SysTP<double>, double>(m, wave, &sh, s_nz[wave]); break;
    case LZ_SYS_SC * 2: resident_serve<SysSC<float>, float>(m, wave, &sh, s_nz[wave]); break;
    case LZ_SYS_SC * 2 + 1: resident_serve<SysSC<double>, double>(m, wave, &sh, s_nz[wave]); break;
    default: break;
  }
}

int launch_resident_multi(const ResMember* table, int n, const uint64_t* lines, uint64_t idle_ticks,
                          void* stream) {
  if (n < 1 || n > kRsMaxHandles) return (int)hipErrorInvalidValue;
  if (n + 1 <= 8)
    hipLaunchKernelGGL(k_resident_multi<8>, dim3(1), dim3(64 * (n + 1)), 0, static_cast<hipStream_t>(stream),
                       table, n, lines, idle_ticks);
  else
    hipLaunchKernelGGL(k_resident_multi<kRsMaxHandles + 1>, dim3(1), dim3(64 * (n + 1)), 0,
                       static_cast<hipStream_t>(stream), table, n, lines, idle_ticks);
  return (int)hipGetLastError();
}

// lz_step_vecnorm's envs per workgroup: kVnBlock on the fused path, kBlock on the split
// path (the round-1 shape, faster there), or LZ_VN_BLOCK (A/B knob)
int vn_fuse_max_wg() {
  static const int m = [] {
    const char* e = std::getenv("LZ_VN_FUSE_MAX_WG");
    return e ? std::atoi(e) : 256;
  }();
  return m;
}

bool vn_fused(int64_t n) { return (n + kVnBlock - 1) / kVnBlock <= vn_fuse_max_wg(); }

int vn_block(int64_t n) {
  static const int forced = [] {
    const char* e = std::getenv("LZ_VN_BLOCK");
    const int b = e ? std::atoi(e) : 0;
    return b == 256 || b == 512 || b == 1024 ? b : 0;
  }();
  if (forced) return forced;
  return vn_fused(n) ? kVnBlock : kBlock;
}

template <class Sys, typename T>
static int launch_vn(const KArgs& a, const VArgs& v, hipStream_t s) {
  static_assert(Sys::O <= kVnMaxObs, "obs too wide for the VecNormalize epilogue");
  const int vb = vn_block(a.n);
  const unsigned grid = (unsigned)((a.n + vb - 1) / vb);
  if (vb == 1024)
    hipLaunchKernelGGL((k_step_vn<Sys, T, 24>), dim3(grid), dim3(1024), 0, s, a, v);
  else if (vb == 512)
    hipLaunchKernelGGL((k_step_vn<Sys, T, 8>), dim3(grid), dim3(512), 0, s, a, v);
  else
    hipLaunchKernelGGL((k_step_vn<Sys, T, 0>), dim3(grid), dim3(256), 0, s, a, v);
  if ((v.flags & LZ_VN_DEFER) || ((v.flags & LZ_VN_TRAINING) && !v.fused))
    hipLaunchKernelGGL((k_vn_colsum<Sys::O>), dim3(v.fused ? 1 : 2 * (Sys::O + 1)),
                       dim3(kVnColBlock), 0, s, v, a.n, a.counter, v.n_done_out);
  return (int)hipGetLastError();
}

int launch_step_vecnorm(int system, int f64, const KArgs& a, const VArgs& v, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (system) {
    case LZ_SYS_LORENZ3:
      return f64 ? launch_vn<SysL3<double>, double>(a, v, s) : launch_vn<SysL3<float>, float>(a, v, s);
    case LZ_SYS_LORENZ4:
      return f64 ? launch_vn<SysL4<double>, double>(a, v, s) : launch_vn<SysL4<float>, float>(a, v, s);
    case LZ_SYS_LORENZ3 + kSysRK4:
      return f64 ? launch_vn<SysL3RK4<double>, double>(a, v, s) : launch_vn<SysL3RK4<float>, float>(a, v, s);
    case LZ_SYS_LORENZ4 + kSysRK4:
      return f64 ? launch_vn<SysL4RK4<double>, double>(a, v, s) : launch_vn<SysL4RK4<float>, float>(a, v, s);
    case LZ_SYS_PMSM:
      return launch_vn<SysPMSM, float>(a, v, s);
    case LZ_SYS_HR:
      return f64 ? launch_vn<SysHR<double>, double>(a, v, s) : launch_vn<SysHR<float>, float>(a, v, s);
    case LZ_SYS_T1:
      return f64 ? launch_vn<SysT1<double>, double>(a, v, s) : launch_vn<SysT1<float>, float>(a, v, s);
    case LZ_SYS_T2:
      return f64 ? launch_vn<SysT2<double>, double>(a, v, s) : launch_vn<SysT2<float>, float>(a, v, s);
    case LZ_SYS_TP:
      return f64 ? launch_vn<SysTP<double>, double>(a, v, s) : launch_vn<SysTP<float>, float>(a, v, s);
    case LZ_SYS_SC:
      return f64 ? launch_vn<SysSC<double>, double>(a, v, s) : launch_vn<SysSC<float>, float>(a, v, s);
  }
  return (int)hipErrorInvalidValue;
}

int launch_reset(int system, int f64, const KArgs& a, void* stream) {
  return dispatch(0, system, f64, a, stream);
}
int launch_step(int system, int f64, const KArgs& a, void* stream) {
  return dispatch(1, system, f64, a, stream);
}
int launch_rollout(int system, int f64, const KArgs& a, void* stream) {
  return dispatch(2, system, f64, a, stream);
}

// Indexed plane access (lz_get_state / lz_set_state with indices): one lane per index,
// elements of E bytes.  Indices outside [0, n) are skipped by the scatter and read as
// zero bits by the gather -- no fault; the host wrappers validate before launching.
template <typename E>
__global__ __launch_bounds__(256) void k_plane_gather(const E* __restrict__ plane, int64_t n,
                                                      const int64_t* __restrict__ idx, int64_t count,
                                                      E* __restrict__ dst) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < count; i += (int64_t)gridDim.x * 256) {
    const int64_t j = idx[i];
    dst[i] = (j >= 0 && j < n) ? plane[j] : E(0);
  }
}

template <typename E>
__global__ __launch_bounds__(256) void k_plane_scatter(E* __restrict__ plane, int64_t n,
                                                       const int64_t* __restrict__ idx, int64_t count,
                                                       const E* __restrict__ src) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < count; i += (int64_t)gridDim.x * 256) {
    const int64_t j = idx[i];
    if (j >= 0 && j < n) plane[j] = src[i];
  }
}

int launch_plane_index(bool scatter, int es, void* plane, int64_t n, const int64_t* idx, int64_t count,
                       void* buf, void* stream) {
  if (count <= 0) return 0;
  const int64_t want = (count + 255) / 256;
  const dim3 g((unsigned)(want < 65536 ? want : 65536));  // grid-stride beyond 16M ids
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (es == 8) {
    if (scatter)
      hipLaunchKernelGGL(k_plane_scatter<uint64_t>, g, dim3(256), 0, s, static_cast<uint64_t*>(plane), n, idx,
                         count, static_cast<const uint64_t*>(buf));
    else
      hipLaunchKernelGGL(k_plane_gather<uint64_t>, g, dim3(256), 0, s, static_cast<const uint64_t*>(plane), n,
                         idx, count, static_cast<uint64_t*>(buf));
  } else {
    if (scatter)
      hipLaunchKernelGGL(k_plane_scatter<uint32_t>, g, dim3(256), 0, s, static_cast<uint32_t*>(plane), n, idx,
                         count, static_cast<const uint32_t*>(buf));
    else
      hipLaunchKernelGGL(k_plane_gather<uint32_t>, g, dim3(256), 0, s, static_cast<const uint32_t*>(plane), n,
                         idx, count, static_cast<uint32_t*>(buf));
  }
  return (int)hipGetLastError();
}

}  // namespace lz
