// Device building blocks shared by the env kernels (lz_kernels.hip) and the
// policy rollout (lz_policy.hip): global access helpers, wave compaction of done
// envs, process noise and the one-step body (env step + done bits + compact list +
// auto-reset).  Internal, not part of the ABI.
#pragma once
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
// LZ_STEP_WT (A/B builds only, tools/build_ab.sh; default 0): the streaming (NT) stores
// as write-through `sc1` stores instead (the line leaves the XCD's L2 at once: nothing
// left dirty at the kernel boundary, MI355X_MICROARCH.md "stores of each flavour").
#ifndef LZ_STEP_WT
#define LZ_STEP_WT 0
#endif
template <bool NT, typename V>
__device__ __forceinline__ void gstore(V* p, V v) {
  if constexpr (NT && LZ_STEP_WT) {
    if constexpr (sizeof(V) == 16)
      asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    else
      __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else if constexpr (NT) {
    __builtin_nontemporal_store(v, p);
  } else {
    *p = v;
  }
}

// The launch's tick (KArgs::tick_in).  A plain load of the uniform pointer compiles to a
// scalar load, and the compiler's lgkmcnt(0) in front of the first use of a later
// kernel-argument load (the action pointer) then also waits for it: one serial memory
// round trip (the tick was written by the previous launch, possibly on another XCD)
// before the action tile is even requested.  As a vector (relaxed atomic) load it
// travels with the state and action loads.  tick_ready() marks the point of first use:
// the empty asm takes the value as a VGPR operand, so the compiler neither moves it to
// SGPRs (a v_readfirstlane, with its vmcnt wait, right behind the load) nor waits for
// it earlier.  LZ_TICK_SCALAR=1 (A/B builds, tools/build_ab.sh) restores the scalar load.
#ifndef LZ_TICK_SCALAR
#define LZ_TICK_SCALAR 0
#endif
__device__ __forceinline__ uint64_t load_tick(const uint64_t* p) {
  if constexpr (LZ_TICK_SCALAR) return *p;
  else return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t tick_ready(uint64_t t) {
  if constexpr (LZ_TICK_SCALAR) return t;
  uint32_t lo = (uint32_t)t, hi = (uint32_t)(t >> 32);
  asm volatile("" : "+v"(lo), "+v"(hi));
  return ((uint64_t)hi << 32) | lo;
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

template <class Sys, typename T, bool kInjectable>
__device__ __forceinline__ void make_noise(const Sys& sys, const KArgs& a, int64_t i, uint64_t tick,
                                           double* nz) {
  if (kInjectable && a.noise) {
#pragma unroll
    for (int j = 0; j < 3; ++j) nz[j] = a.noise[3 * i + j];
  } else {
    float z[3];
    normal3(a.seed, (uint64_t)(a.gid0 + i), tick, z);
    sys.noise_from_normals(z, nz);
  }
}

// ------------------------------------------------------------------ one step body
// Shared by k_step (K = 1, state in HBM), k_rollout and k_rollout_policy (state in
// VGPRs across K).  Returns the done byte; o[] holds the observation to emit
// (post-reset if reset); with kKeepTerm, o_term[] receives the pre-reset observation.
// lead = false: a lane that computes a copy of another lane's env (the split-lane
// rollout) -- same arithmetic, but it takes no slot in the compact done list.
// kNoDone: the launch can produce no done at all (a never-terminating system and no
// step counter, see no_done()): the step alone, no done bookkeeping.
// kZMode (noisy systems, device noise): 0 draws this step's normals here; 1 reads them
// from a producer wave's LDS ring (zpre[0], zpre[64], zpre[128]); 2 (software-pipelined,
// k_rollout kZN) reads them from the caller's registers zpre[0..2] and draws the NEXT
// step's normals (tick + 1) into the same registers here, in the basic block of sys.step,
// so the scheduler interleaves that independent Philox + Box-Muller chain with the
// integrator's; 3 (the lane-pair rollout, k_rollout_pair) runs sys.step_pair with
// lead = lane 0 of the pair and the slave lane's normals in zpre[0..2].  The normals are
// keyed by (seed, env id, tick) only: bit-identical.
template <class Sys, typename T, bool kRollout, bool kKeepTerm = false, bool kNoDone = false,
          bool kInject = !kRollout, int kZMode = 0>
__device__ __forceinline__ uint8_t step_body(Sys& sys, int32_t& steps, const KArgs& a, int64_t i,
                                             bool live, const float* act, uint64_t tick, int k,
                                             T* o, T& rew, bool& did_reset,
                                             T* o_term = nullptr, bool lead = true,
                                             const float* zpre = nullptr) {
  uint8_t dflag = 0;
  did_reset = false;
  if constexpr (kNoDone) {
    static_assert(never_terminates<Sys>::value && !Sys::kNoise && !kKeepTerm,
                  "kNoDone: a never-terminating, noise-free system");
    if (live) {
      double nz[3] = {0.0, 0.0, 0.0};
      (void)sys.step(act, false, nz, o, rew, a);
    }
    return 0;
  }
  if (live) {
    double nz[3] = {0.0, 0.0, 0.0};
    bool use_nz = false;
    if constexpr (Sys::kNoise) {
      if (a.flags & LZ_FLAG_ADD_NOISE) {
        if constexpr (kZMode == 1) {  // the normals drawn ahead by a producer wave (k_rollout kNP):
          // zpre[0], zpre[64], zpre[128] -- the same normal3(seed, gid, tick) values; zpre =
          // nullptr: the producer timed out, the step runs on NaN normals
          const float q = __builtin_nanf("");
          float z[3] = {q, q, q};
          if (zpre) {
            z[0] = zpre[0];
            z[1] = zpre[64];
            z[2] = zpre[128];
          }
          sys.noise_from_normals(z, nz);
        } else if constexpr (kZMode == 2) {  // this step's from registers; draw the next step's
          float z[3] = {zpre[0], zpre[1], zpre[2]};
          normal3(a.seed, (uint64_t)(a.gid0 + i), tick + 1, const_cast<float*>(zpre));
          sys.noise_from_normals(z, nz);
        } else if constexpr (kZMode == 3) {  // lane pair: the slave lane's normals, drawn by the
          // pair's schedule (split_loop kPair) -- normal3(seed, gid, tick)'s values
          float z[3] = {zpre[0], zpre[1], zpre[2]};
          sys.noise_from_normals(z, nz);
        } else {
          make_noise<Sys, T, kInject>(sys, a, i, tick, nz);
        }
        use_nz = true;
      }
    }
    bool term;
    if constexpr (kZMode == 3) term = sys.step_pair(!lead, act, use_nz, nz, o, rew, a);  // lane pair
    else term = sys.step(act, use_nz, nz, o, rew, a);
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
    const int32_t pos = wave_compact(dflag != 0 && lead, a.counter);
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
  if constexpr (kKeepTerm) {
#pragma unroll
    for (int j = 0; j < Sys::O; ++j) o_term[j] = o[j];
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

// The launch-wide condition for step_body's kNoDone (host side): no step counter and a
// system whose step never terminates
template <class Sys>
inline bool no_done(const KArgs& a) {
  return never_terminates<Sys>::value && !a.count_steps;
}

}  // namespace lz
