// Internal structures shared by the C-ABI (lz_api.cpp) and the kernels
// (lz_kernels.hip).  Not part of the public ABI.
#pragma once
#include <stdint.h>

#include "lorenz_env.h"

namespace lz {

constexpr int kBlock = 256;   // envs per workgroup (4 waves of 64 lanes)
constexpr int kMaxPlanes = 12;

// Everything a launch needs, passed by value as the kernel argument.
struct KArgs {
  void* pl[kMaxPlanes];      // SoA state planes (see lorenz_env.h plane enums)
  const void* act;           // T [N, A]   (rollout: [K, N, A])
  const double* noise;       // double [N, 3] injected noise or nullptr
  void* obs;                 // T [N, O]   (rollout: [K, N, O])
  void* rew;                 // T [N]      (rollout: [K, N])
  uint8_t* done;             // uint8 [N]  (rollout: [K, N])
  int32_t* done_idx32;       // step: compact env indices (nullable)
  int64_t* done_idx64;       // rollout: compact k*N+env (nullable)
  void* term_obs;            // compact terminal observations (nullable)
  int64_t term_cap;          // rollout capacity of the compact buffers
  int32_t* counter;          // compact-list cursor for this launch
  int32_t* counter_next;     // the other slot, zeroed by this launch for the next
  const float* bc1;          // PMSM: (float)(1 - beta1**k), k < bc_len
  const float* bc2;          // PMSM: (float)(1 - beta2**k)
  const uint8_t* mask;       // reset: env selection (nullable)
  const void* init;          // reset: injected initial states (nullable)
  int64_t n;                 // envs in this handle
  int64_t gid0;              // global id of env 0 (RNG key)
  uint64_t seed;
  // Call counter (the RNG counter): device-resident so that launches can be captured
  // in a hipGraph and replayed.  Launch reads *tick_in; block 0 lane 0 writes
  // *tick_out = tick + tick_adv (the other slot of a 2-slot ping-pong selected by the
  // host-side call parity).  Rollout step k uses tick + k.
  const uint64_t* tick_in;
  uint64_t* tick_out;
  uint64_t tick_adv;
  int32_t bc_len;
  int32_t max_steps;         // truncation limit (0 = none)
  int32_t t_done_step;       // reference 't == T' step (-1 = never)
  int32_t count_steps;       // maintain the STEP plane
  uint32_t flags;            // LZ_FLAG_*
  int32_t vec_ok;            // act/obs base pointers 16-B aligned
  int32_t K;                 // rollout length
  int32_t variant;           // step-kernel tuning variant (lz_config.reserved[0])
  float alpha;               // PMSM
  double prm[LZ_MAX_PARAMS];
};

// record the thread-local message lz_last_error() returns; returns s
lz_status set_error(lz_status s, const char* msg);

// host-side launchers (lz_kernels.hip)
int launch_reset(int system, int f64, const KArgs& a, void* stream);
int launch_step(int system, int f64, const KArgs& a, void* stream);
int launch_rollout(int system, int f64, const KArgs& a, void* stream);

}  // namespace lz
