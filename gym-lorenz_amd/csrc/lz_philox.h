// Counter-based RNG for on-device resets and process noise: Philox4x32-10
// (Salmon, Moraes, Dror, Shaw, SC'11).  Stateless: every draw is a pure function of
// (seed, global env id, purpose, call tick, word index), so a shard of the env axis
// on any GPU reproduces exactly the draws of the same envs on one GPU.
// Counter layout (mirrored by oracle/lz_oracle.c draw_word):
//   c0 = gid[31:0]
//   c1 = gid[39:32] | (word/4) << 8 | purpose << 24
//   c2 = tick[31:0], c3 = tick[63:32];   key = seed
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lz {

enum : uint32_t { kPurposeReset = 1, kPurposeNoise = 2, kPurposePolicy = 3 };

struct U4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // one 32x32->64 product per word (v_mad_u64_u32) instead of separate lo / hi
    // multiplies (both quarter-rate)
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
    const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
    c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// Four consecutive words [4*blk, 4*blk+4) of the stream (gid, purpose, tick).
__device__ __forceinline__ U4 philox_block(uint64_t seed, uint64_t gid, uint32_t purpose,
                                           uint64_t tick, uint32_t blk) {
  U4 c{(uint32_t)gid, (uint32_t)((gid >> 32) & 0xFFu) | (blk << 8) | (purpose << 24),
       (uint32_t)tick, (uint32_t)(tick >> 32)};
  return philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
}

// [0,1) with 24 / 53 random bits -- exact conversions, identical on the CPU oracle.
__device__ __forceinline__ float u01f(uint32_t x) {
  return (float)(x >> 8) * 5.9604644775390625e-08f;
}
__device__ __forceinline__ double u01d(uint32_t a, uint32_t b) {
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * 1.1102230246251565e-16;
}

// One Box-Muller pair from two 32-bit words: u1 in (0, 1], u2 in [0, 1);
// r = sqrt(-2 ln u1) = sqrt(-2 ln2 * log2 u1), (c, s) = r * (cos, sin)(2 pi u2).
// Hardware transcendentals (v_log_f32, v_sqrt_f32, v_sin_f32 / v_cos_f32, which take
// the angle in revolutions): a few ulp, far below what the N(0, sigma) draws are
// checked for, and ~10 instructions instead of the ~150 of libm-accurate logf /
// sincospif / sqrtf.  Tails are bounded by the 24-bit u1 (|z| <= 5.77) either way.
__device__ __forceinline__ void box_muller(uint32_t wa, uint32_t wb, float& c, float& s) {
  const float u1 = (float)((wa >> 8) + 1u) * 5.9604644775390625e-08f;
  const float u2 = u01f(wb);
  const float r = __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u1));
  c = r * __builtin_amdgcn_cosf(u2);
  s = r * __builtin_amdgcn_sinf(u2);
}

// Three standard normals (two Box-Muller pairs) for per-step process noise.
__device__ __forceinline__ void normal3(uint64_t seed, uint64_t gid, uint64_t tick, float z[3]) {
  const U4 w = philox_block(seed, gid, kPurposeNoise, tick, 0);
  float s1, s2;
  box_muller(w.x, w.y, z[0], s1);
  z[1] = s1;
  box_muller(w.z, w.w, z[2], s2);
  (void)s2;
}

// Two standard normals for the policy's Gaussian action sample (purpose 3): the first
// Box-Muller pair of normal4 (identical values), for action dims <= 2.
__device__ __forceinline__ void normal2(uint64_t seed, uint64_t gid, uint64_t tick, float z[4]) {
  const U4 w = philox_block(seed, gid, kPurposePolicy, tick, 0);
  box_muller(w.x, w.y, z[0], z[1]);
}

// Four standard normals for the policy's Gaussian action sample (purpose 3).
__device__ __forceinline__ void normal4(uint64_t seed, uint64_t gid, uint64_t tick, float z[4]) {
  const U4 w = philox_block(seed, gid, kPurposePolicy, tick, 0);
  box_muller(w.x, w.y, z[0], z[1]);
  box_muller(w.z, w.w, z[2], z[3]);
}

}  // namespace lz
