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

#include "lz_internal.h"
#include "lz_systems.h"

namespace lz {

// ------------------------------------------------------------------ global access
// NT = non-temporal (streaming) hint for buffers touched once per step (actions in,
// obs / reward / done out); the state planes are re-read next step and keep the
// default policy.
typedef float f4v __attribute__((ext_vector_type(4)));

template <bool NT, typename V>
__device__ __forceinline__ V gload(const V* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT, typename V>
__device__ __forceinline__ void gstore(V* p, V v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// ------------------------------------------------------------------ LDS staging
// Copy the block's [nb, W] slice of a row-major T tensor into LDS (row = env).
template <bool NT, typename T, int W>
__device__ __forceinline__ void stage_in(T* __restrict__ lds, const T* __restrict__ g, int nb,
                                         int tid, bool vec) {
  constexpr int kElems = kBlock * W;
  if (vec && nb == kBlock) {
    constexpr int kVec = kElems * (int)sizeof(T) / 16;
    const f4v* __restrict__ gv = reinterpret_cast<const f4v*>(g);
    f4v* lv = reinterpret_cast<f4v*>(lds);
#pragma unroll
    for (int v = tid; v < kVec; v += kBlock) lv[v] = gload<NT>(gv + v);
  } else {
    for (int e = tid; e < nb * W; e += kBlock) lds[e] = gload<NT>(g + e);
  }
}

template <bool NT, typename T, int W>
__device__ __forceinline__ void stage_out(T* __restrict__ g, const T* __restrict__ lds, int nb,
                                          int tid, bool vec) {
  constexpr int kElems = kBlock * W;
  if (vec && nb == kBlock) {
    constexpr int kVec = kElems * (int)sizeof(T) / 16;
    f4v* __restrict__ gv = reinterpret_cast<f4v*>(g);
    const f4v* lv = reinterpret_cast<const f4v*>(lds);
#pragma unroll
    for (int v = tid; v < kVec; v += kBlock) gstore<NT>(gv + v, lv[v]);
  } else {
    for (int e = tid; e < nb * W; e += kBlock) gstore<NT>(g + e, lds[e]);
  }
}

// 64-lane ballot compaction: returns this lane's slot in the compact list (or -1).
// Must be reached by every lane of the wave.
__device__ __forceinline__ int32_t wave_compact(bool flag, int32_t* counter) {
  const unsigned long long m = __ballot(flag);
  if (m == 0ull) return -1;
  const int lane = (int)(threadIdx.x & 63u);
  const int leader = __ffsll((long long)m) - 1;
  int32_t base = 0;
  if (lane == leader) base = atomicAdd(counter, (int32_t)__popcll(m));
  base = __shfl(base, leader, 64);
  const unsigned long long lt = (lane == 0) ? 0ull : (m & (~0ull >> (64 - lane)));
  return flag ? base + (int32_t)__popcll(lt) : -1;
}

template <class Sys, typename T>
__device__ __forceinline__ void make_noise(const Sys& sys, const KArgs& a, int64_t i, uint64_t tick,
                                           double* nz) {
  if (a.noise) {
#pragma unroll
    for (int j = 0; j < 3; ++j) nz[j] = a.noise[3 * i + j];
  } else {
    float z[3];
    normal3(a.seed, (uint64_t)(a.gid0 + i), tick, z);
    sys.noise_from_normals(z, nz);
  }
}

// ------------------------------------------------------------------ reset
template <class Sys, typename T>
__global__ __launch_bounds__(kBlock) void k_reset(KArgs a) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint64_t tick = *a.tick_in;
  if (blockIdx.x == 0 && threadIdx.x == 0) *a.tick_out = tick + a.tick_adv;
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

// ------------------------------------------------------------------ one step body
// Shared by k_step (K = 1, state in HBM) and k_rollout (state in VGPRs across K).
// Returns the done byte; o[] holds the observation to emit (post-reset if reset).
template <class Sys, typename T, bool kRollout>
__device__ __forceinline__ uint8_t step_body(Sys& sys, int32_t& steps, const KArgs& a, int64_t i,
                                             bool live, const float* act, uint64_t tick, int k,
                                             T* o, T& rew, bool& did_reset) {
  uint8_t dflag = 0;
  did_reset = false;
  if (live) {
    double nz[3] = {0.0, 0.0, 0.0};
    bool use_nz = false;
    if constexpr (Sys::kNoise) {
      if (a.flags & LZ_FLAG_ADD_NOISE) {
        make_noise<Sys, T>(sys, a, i, tick, nz);
        use_nz = true;
      }
    }
    bool term = sys.step(act, use_nz, nz, o, rew, a);
    bool trunc = false;
    if (a.count_steps) {
      steps += 1;
      if (steps == a.t_done_step) term = true;            // reference 't == T'
      if (a.max_steps > 0 && steps >= a.max_steps) trunc = true;
    }
    dflag = (uint8_t)((term ? LZ_DONE_TERMINATED : 0u) | (trunc ? LZ_DONE_TRUNCATED : 0u));
  }
  // compact list of done envs: ballot + one atomic per wave (all lanes reach this)
  if (a.term_obs) {
    const int32_t pos = wave_compact(dflag != 0, a.counter);
    if (pos >= 0) {
      if constexpr (kRollout) {
        if (pos < a.term_cap) {
          a.done_idx64[pos] = (int64_t)k * a.n + i;
#pragma unroll
          for (int j = 0; j < Sys::O; ++j) static_cast<T*>(a.term_obs)[(int64_t)pos * Sys::O + j] = o[j];
        }
      } else {
        a.done_idx32[pos] = (int32_t)i;
#pragma unroll
        for (int j = 0; j < Sys::O; ++j) static_cast<T*>(a.term_obs)[(int64_t)pos * Sys::O + j] = o[j];
      }
    }
  }
  if (live && dflag && (a.flags & LZ_FLAG_AUTORESET)) {  // SB3 DummyVecEnv auto-reset
    T v[Sys::NI];
    Sys::draw(a, (uint64_t)(a.gid0 + i), tick, v);
    sys.init(v, a);
    sys.reset_obs(o);
    steps = 0;
    did_reset = true;
  }
  return dflag;
}

// ------------------------------------------------------------------ step
// V (tuning variant, lz_config.reserved[0], default 0): bit 0 = plain (temporal)
// act/obs/rew/done accesses instead of non-temporal, bit 1 = lanes access their own
// act/obs rows directly instead of LDS staging.  Measured at 1M envs (profiles/r01):
// non-temporal I/O is 13% faster than plain, LDS staging 7-11% faster than direct.
template <class Sys, typename T, int V>
__global__ __launch_bounds__(kBlock) void k_step(KArgs a) {
  constexpr bool NT = (V & 1) == 0;
  constexpr bool kLds = (V & 2) == 0;
  __shared__ __attribute__((aligned(16))) float s_act[kLds ? kBlock * Sys::A : 4];
  __shared__ __attribute__((aligned(16))) T s_obs[kLds ? kBlock * Sys::O : 2];
  const int tid = (int)threadIdx.x;
  const int64_t base = (int64_t)blockIdx.x * kBlock;
  const int64_t i = base + tid;
  const int nb = (int)((a.n - base) < kBlock ? (a.n - base) : kBlock);
  const bool live = tid < nb;
  const bool vec = a.vec_ok != 0;
  const uint64_t tick = *a.tick_in;
  if (blockIdx.x == 0 && tid == 0) {
    *a.counter_next = 0;
    *a.tick_out = tick + a.tick_adv;
  }
  Sys sys;
  sys.setup(a);
  int32_t steps = 0;
  if (live) {  // state loads first: in flight together with the action staging
    sys.load(a, i);
    if (a.count_steps) steps = static_cast<const int32_t*>(a.pl[Sys::kStepPlane])[i];
  }
  float act[Sys::A];
  if constexpr (Sys::kUsesAction) {
    const float* ga = static_cast<const float*>(a.act);
    if constexpr (kLds) {
      stage_in<NT, float, Sys::A>(s_act, ga + base * Sys::A, nb, tid, vec);
      __syncthreads();
      if (live) {
#pragma unroll
        for (int j = 0; j < Sys::A; ++j) act[j] = s_act[tid * Sys::A + j];
      }
    } else if (live) {
#pragma unroll
      for (int j = 0; j < Sys::A; ++j) act[j] = gload<NT>(ga + i * Sys::A + j);
    }
  }
  T o[Sys::O];
  T rew = (T)0;
  bool did_reset;
  const uint8_t dflag =
      step_body<Sys, T, false>(sys, steps, a, i, live, act, tick, 0, o, rew, did_reset);
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
    gstore<NT>(a.done + i, dflag);
  }
  if constexpr (kLds) {
    __syncthreads();
    stage_out<NT, T, Sys::O>(static_cast<T*>(a.obs) + base * Sys::O, s_obs, nb, tid, vec);
  }
}

// ------------------------------------------------------------------ fused rollout
template <class Sys, typename T>
__global__ __launch_bounds__(kBlock) void k_rollout(KArgs a) {
  __shared__ __attribute__((aligned(16))) float s_act[kBlock * Sys::A];
  __shared__ __attribute__((aligned(16))) T s_obs[kBlock * Sys::O];
  const int tid = (int)threadIdx.x;
  const int64_t base = (int64_t)blockIdx.x * kBlock;
  const int64_t i = base + tid;
  const int nb = (int)((a.n - base) < kBlock ? (a.n - base) : kBlock);
  const bool live = tid < nb;
  const bool vec = a.vec_ok != 0;
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
  for (int k = 0; k < a.K; ++k) {
    const int64_t off = (int64_t)k * a.n;
    if constexpr (Sys::kUsesAction)
      stage_in<true, float, Sys::A>(s_act, static_cast<const float*>(a.act) + (off + base) * Sys::A, nb,
                                   tid, vec);
    __syncthreads();
    float act[Sys::A];
    if constexpr (Sys::kUsesAction) {
      if (live) {
#pragma unroll
        for (int j = 0; j < Sys::A; ++j) act[j] = s_act[tid * Sys::A + j];
      }
    }
    T o[Sys::O];
    T rew = (T)0;
    bool did_reset;
    const uint8_t dflag = step_body<Sys, T, true>(sys, steps, a, i, live, act, tick + (uint64_t)k,
                                                  k, o, rew, did_reset);
    any_reset = any_reset || did_reset;
    if (live) {
#pragma unroll
      for (int j = 0; j < Sys::O; ++j) s_obs[tid * Sys::O + j] = o[j];
      gstore<true>(static_cast<T*>(a.rew) + off + i, rew);
      gstore<true>(a.done + off + i, dflag);
    }
    __syncthreads();
    stage_out<true, T, Sys::O>(static_cast<T*>(a.obs) + (off + base) * Sys::O, s_obs, nb, tid, vec);
  }
  if (live) {
    sys.store(a, i);
    if (any_reset) sys.store_autoreset_extra(a, i);
    if (a.count_steps) static_cast<int32_t*>(a.pl[Sys::kStepPlane])[i] = steps;
  }
}

// ------------------------------------------------------------------ launchers
static inline int64_t grid_for(int64_t n) { return (n + kBlock - 1) / kBlock; }

template <class Sys, typename T>
static int launch_all(int which, const KArgs& a, hipStream_t s) {
  const dim3 grid((unsigned)grid_for(a.n)), block(kBlock);
  if (which == 0)
    hipLaunchKernelGGL((k_reset<Sys, T>), grid, block, 0, s, a);
  else if (which == 1) {
    switch (a.variant & 3) {
      case 1: hipLaunchKernelGGL((k_step<Sys, T, 1>), grid, block, 0, s, a); break;
      case 2: hipLaunchKernelGGL((k_step<Sys, T, 2>), grid, block, 0, s, a); break;
      case 3: hipLaunchKernelGGL((k_step<Sys, T, 3>), grid, block, 0, s, a); break;
      default: hipLaunchKernelGGL((k_step<Sys, T, 0>), grid, block, 0, s, a); break;
    }
  } else
    hipLaunchKernelGGL((k_rollout<Sys, T>), grid, block, 0, s, a);
  return (int)hipGetLastError();
}

static int dispatch(int which, int system, int f64, const KArgs& a, void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (system) {
    case LZ_SYS_LORENZ3:
      return f64 ? launch_all<SysL3<double>, double>(which, a, s)
                 : launch_all<SysL3<float>, float>(which, a, s);
    case LZ_SYS_LORENZ4:
      return f64 ? launch_all<SysL4<double>, double>(which, a, s)
                 : launch_all<SysL4<float>, float>(which, a, s);
    case LZ_SYS_PMSM:
      return launch_all<SysPMSM, float>(which, a, s);
    case LZ_SYS_HR:
      return f64 ? launch_all<SysHR<double>, double>(which, a, s)
                 : launch_all<SysHR<float>, float>(which, a, s);
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

}  // namespace lz
