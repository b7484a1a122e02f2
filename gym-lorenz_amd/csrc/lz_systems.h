// Device models of the four reference env systems, one env per lane.
//
// Every arithmetic expression follows the reference's Python/NumPy evaluation
// ORDER and dtype PROMOTION (numpy 2, NEP 50); the file is compiled with
// -ffp-contract=off so no a*b+c is fused, and with HIP's default correctly rounded
// f32 division / sqrt.  In fp64 (LORENZ3/4, HR) this is the reference's own
// arithmetic, so LORENZ3/4 are bit-identical to dynamic.py / lorenz_env_transient.py.
// References are file:line in /root/reference/code/gym-lorenz/gym_lorenz/envs/.
#pragma once
#include <type_traits>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lz_internal.h"
#include "lz_philox.h"

namespace lz {

// np.clip: NaN-propagating (np.maximum / np.minimum propagate NaN; fmaxf would not)
template <typename T>
__device__ __forceinline__ T clip(T x, T lo, T hi) {
  return x < lo ? lo : (x > hi ? hi : x);
}
// np.clip with NONZERO bounds: float32 through IEEE 754-2019 maximum / minimum
// (v_maximum3_f32 / v_minimum3_f32 on gfx950, NaN-propagating): the value clip() gives
// (bounds away from 0, so no signed-zero case) except a NaN's payload, in 2 instructions
// instead of 2 compares + 2 selects; float64 keeps clip() (no native f64 maximum).
template <typename T>
__device__ __forceinline__ T clip_nz(T x, T lo, T hi) {
  if constexpr (std::is_same<T, float>::value)
    return __builtin_elementwise_minimum(__builtin_elementwise_maximum(x, lo), hi);
  else
    return clip(x, lo, hi);
}

// The partner lane's value in a lane pair (2e, 2e + 1): DPP quad_perm [1, 0, 3, 2], one
// full-rate v_mov_b32_dpp -- the exchange of the lane-pair rollout (k_rollout_split with
// kPair, SysPMSM::step_pair).
__device__ __forceinline__ float pair_swap(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
}

template <typename T>
__device__ __forceinline__ T ld(const void* p, int64_t i) {
  return static_cast<const T*>(p)[i];
}
// LZ_STATE_NT / LZ_STATE_WT (A/B builds only, tools/build_ab.sh; default 0): state-plane
// stores with the non-temporal hint / write-through (`sc1`, relaxed agent-scope atomic
// store).  The product stores them plain: the planes are re-read by the next launch.
#ifndef LZ_STATE_NT
#define LZ_STATE_NT 0
#endif
#ifndef LZ_STATE_WT
#define LZ_STATE_WT 0
#endif
template <typename T>
__device__ __forceinline__ void st(void* p, int64_t i, T v) {
  if constexpr (LZ_STATE_WT) __hip_atomic_store(static_cast<T*>(p) + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else if constexpr (LZ_STATE_NT) __builtin_nontemporal_store(v, static_cast<T*>(p) + i);
  else static_cast<T*>(p)[i] = v;
}

// Uniform initial-state draws (purpose RESET): value j of [lo, hi).
//   T=float : word j, 24 bits         T=double : words (2j, 2j+1), 53 bits
template <typename T>
struct Draw;
template <>
struct Draw<float> {
  __device__ static float u(uint64_t seed, uint64_t gid, uint64_t tick, int j) {
    const U4 w = philox_block(seed, gid, kPurposeReset, tick, (uint32_t)(j >> 2));
    const uint32_t x = (j & 3) == 0 ? w.x : (j & 3) == 1 ? w.y : (j & 3) == 2 ? w.z : w.w;
    return u01f(x);
  }
  __device__ static float uniform(uint64_t seed, uint64_t gid, uint64_t tick, int j, float lo,
                                  float hi) {
    return lo + (hi - lo) * u(seed, gid, tick, j);
  }
};
template <>
struct Draw<double> {
  __device__ static double u(uint64_t seed, uint64_t gid, uint64_t tick, int j) {
    const U4 w = philox_block(seed, gid, kPurposeReset, tick, (uint32_t)(j >> 1));
    return (j & 1) ? u01d(w.z, w.w) : u01d(w.x, w.y);
  }
  __device__ static double uniform(uint64_t seed, uint64_t gid, uint64_t tick, int j, double lo,
                                   double hi) {
    return lo + (hi - lo) * u(seed, gid, tick, j);
  }
};

// ===========================================================================
// LORENZ3 -- dynamic.py:5-93, lorenzEnv_transient (3-state Lorenz, Euler)
// params: sigma(self.u)=10, rho(self.i)=28, beta(self.o)=8/3, dt=0.01, clip=500
// planes: x, y, z [, step]
// ===========================================================================
// A system whose step() can never report termination (done then only comes from the
// step counter: truncation or the reference's 't == T')
template <class S, class = void>
struct never_terminates { static constexpr bool value = false; };
template <class S>
struct never_terminates<S, decltype((void)S::kNeverTerminates)> {
  static constexpr bool value = S::kNeverTerminates;
};

template <typename T>
struct SysL3 {
  static constexpr int A = 3, O = 6, NI = 3;
  static constexpr bool kUsesAction = true, kNoise = false;
  static constexpr bool kNeverTerminates = true;  // step() returns false: :85-89
  static constexpr int kStepPlane = LZ_L3_STEP;
  T x, y, z;
  T sg, rh, be, dt, cl;

  __device__ void setup(const KArgs& a) {
    sg = (T)a.prm[0]; rh = (T)a.prm[1]; be = (T)a.prm[2]; dt = (T)a.prm[3]; cl = (T)a.prm[4];
  }
  __device__ void load(const KArgs& a, int64_t i) {
    x = ld<T>(a.pl[0], i); y = ld<T>(a.pl[1], i); z = ld<T>(a.pl[2], i);
  }
  __device__ void store(const KArgs& a, int64_t i) const {
    st<T>(a.pl[0], i, x); st<T>(a.pl[1], i, y); st<T>(a.pl[2], i, z);
  }
  __device__ void store_reset(const KArgs& a, int64_t i) const { store(a, i); }
  __device__ void store_autoreset_extra(const KArgs&, int64_t) const {}
  // dynamic.py:39-41 (reset) / :70-72 / :77-79 (step)
  __device__ void rhs(T& fx, T& fy, T& fz) const {
    fx = sg * (y - x);
    fy = (rh * x - y) - x * z;
    fz = x * y - be * z;
  }
  __device__ static void draw(const KArgs& a, uint64_t gid, uint64_t tick, T* v) {
    for (int j = 0; j < 3; ++j) v[j] = Draw<T>::uniform(a.seed, gid, tick, j, (T)-30, (T)30);  // :37
  }
  __device__ void init(const T* v, const KArgs&) { x = v[0]; y = v[1]; z = v[2]; }
  // reset(): dynamic.py:35-50 -> state0 - state2 (zeros(6))
  __device__ void reset_obs(T* o) const {
    T fx, fy, fz;
    rhs(fx, fy, fz);
    o[0] = x - (T)0; o[1] = y - (T)0; o[2] = z - (T)0;
    o[3] = fx - (T)0; o[4] = fy - (T)0; o[5] = fz - (T)0;
  }
  // step(): dynamic.py:61-90
  // act: float32 (SB3 hands np.float32 actions; np.clip keeps f32, then promotes)
  __device__ bool step(const float* act, bool, const double*, T* o, T& rew, const KArgs&) {
    const T u1 = clip_nz((T)act[0], -cl, cl), u2 = clip_nz((T)act[1], -cl, cl),
            u3 = clip_nz((T)act[2], -cl, cl);
    T fx, fy, fz;
    rhs(fx, fy, fz);                 // :70-72, all from the old state
    x = (x + fx * dt) + u1;          // :73
    y = (y + fy * dt) + u2;          // :74
    z = (z + fz * dt) + u3;          // :75
    reset_obs(o);                    // :77-83 obs = [s', f(s')]
    // :84 -sum(abs(x) for x in now[0:3]); python's sum starts from int 0
    rew = -((((T)0 + fabs(o[0])) + fabs(o[1])) + fabs(o[2]));
    return false;                    // :85-89 't == 10' handled by t_done_step
  }
};

// ===========================================================================
// LORENZ4 -- lorenz_env_transient.py:247-376 (4-state master/slave, Euler)
// params: a=10, b=8/3, c=28, dt=0.001, clip=2; the action is never used (:316-318)
// planes: master x1..x4, slave x1..x4 [, step]
// ===========================================================================
template <typename T>
struct SysL4 {
  static constexpr int A = 3, O = 8, NI = 8;
  static constexpr bool kUsesAction = false, kNoise = false;
  static constexpr int kStepPlane = LZ_L4_STEP;
  T m[4], s[4];
  T pa, pb, pc, dt;

  __device__ void setup(const KArgs& a) {
    pa = (T)a.prm[0]; pb = (T)a.prm[1]; pc = (T)a.prm[2]; dt = (T)a.prm[3];
  }
  __device__ void load(const KArgs& a, int64_t i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) { m[j] = ld<T>(a.pl[j], i); s[j] = ld<T>(a.pl[4 + j], i); }
  }
  __device__ void store(const KArgs& a, int64_t i) const {
#pragma unroll
    for (int j = 0; j < 4; ++j) { st<T>(a.pl[j], i, m[j]); st<T>(a.pl[4 + j], i, s[j]); }
  }
  __device__ void store_reset(const KArgs& a, int64_t i) const { store(a, i); }
  __device__ void store_autoreset_extra(const KArgs&, int64_t) const {}
  // :323-326 (master) / :344-347 (slave); also :280-283, :333-336, :354-357
  __device__ void rhs(const T* v, T* f) const {
    f[0] = pa * (v[1] - v[0]) + v[3];
    f[1] = (pc * v[0] - v[1]) - v[0] * v[2];
    f[2] = v[0] * v[1] - pb * v[2];
    f[3] = (-v[0]) * v[1] - pb * v[2];
  }
  __device__ static void draw(const KArgs& a, uint64_t gid, uint64_t tick, T* v) {
    for (int j = 0; j < 8; ++j) v[j] = Draw<T>::uniform(a.seed, gid, tick, j, (T)0, (T)5);  // :277-278
  }
  __device__ void init(const T* v, const KArgs&) {
#pragma unroll
    for (int j = 0; j < 4; ++j) { m[j] = v[j]; s[j] = v[4 + j]; }
  }
  // :284-300 obs = [m - s, f(m) - f(s)]
  __device__ void reset_obs(T* o) const {
    T fm[4], fs[4];
    rhs(m, fm);
    rhs(s, fs);
#pragma unroll
    for (int j = 0; j < 4; ++j) { o[j] = m[j] - s[j]; o[4 + j] = fm[j] - fs[j]; }
  }
  // :314-373
  __device__ bool step(const float*, bool, const double*, T* o, T& rew, const KArgs&) {
    T f[4];
    rhs(m, f);                                              // :323-326
#pragma unroll
    for (int j = 0; j < 4; ++j) m[j] = m[j] + f[j] * dt;    // :327-330
    rhs(s, f);                                              // :344-347
#pragma unroll
    for (int j = 0; j < 4; ++j) s[j] = s[j] + f[j] * dt;    // :348-351
    reset_obs(o);                                           // :333-339, :354-362
    const T r = -(((((T)0 + fabs(o[0])) + fabs(o[1])) + fabs(o[2])) + fabs(o[3]));  // :363
    rew = r;
    return r < (T)-1e6;                                     // :369 (t == 5 never fires)
  }
};

// ===========================================================================
// LZ_INT_RK4 (lz_config.integrator): the classical RK4 step of HRSyncEnv
// (lorenz_env_try.py:100-113 -- k1 = f(s), k2 = f(s + dt/2 k1), k3 = f(s + dt/2 k2),
// k4 = f(s + dt k3), s += (dt/6.0) (((k1 + 2 k2) + 2 k3) + k4), python-float dt/2 and
// dt/6.0) on the LORENZ3 / LORENZ4 right-hand sides.  The four stages stay in
// registers, the stage sum accumulated as the stages complete (SysHR::rk4's order: the
// same operations, one stage live).  LORENZ3 keeps dynamic.py:73-75's additive action
// after the integration step: s' = (s + h6 sum) + u.  Everything else (reset, obs,
// reward, done) is the Euler system's.  No reference oracle exists (the reference's
// Lorenz envs are Euler only): oracle/lz_oracle.c orc_l3_step_rk4 / orc_l4_step_rk4
// restate this arithmetic.
// ===========================================================================
template <typename T>
struct SysL3RK4 : SysL3<T> {
  using B = SysL3<T>;
  T h2, h6;
  __device__ void setup(const KArgs& a) {
    B::setup(a);
    h2 = (T)(a.prm[3] / 2);    // python dt/2
    h6 = (T)(a.prm[3] / 6.0);  // python dt/6.0
  }
  __device__ void f(T x, T y, T z, T& fx, T& fy, T& fz) const {  // dynamic.py:70-72
    fx = B::sg * (y - x);
    fy = (B::rh * x - y) - x * z;
    fz = x * y - B::be * z;
  }
  __device__ bool step(const float* act, bool, const double*, T* o, T& rew, const KArgs&) {
    const T cl = B::cl;
    const T u1 = clip_nz((T)act[0], -cl, cl), u2 = clip_nz((T)act[1], -cl, cl),
            u3 = clip_nz((T)act[2], -cl, cl);
    const T x = B::x, y = B::y, z = B::z;
    T kx, ky, kz, ax, ay, az;
    f(x, y, z, kx, ky, kz);                                               // k1
    ax = kx; ay = ky; az = kz;
    f(x + h2 * kx, y + h2 * ky, z + h2 * kz, kx, ky, kz);                 // k2
    ax = ax + (T)2 * kx; ay = ay + (T)2 * ky; az = az + (T)2 * kz;
    f(x + h2 * kx, y + h2 * ky, z + h2 * kz, kx, ky, kz);                 // k3
    ax = ax + (T)2 * kx; ay = ay + (T)2 * ky; az = az + (T)2 * kz;
    f(x + B::dt * kx, y + B::dt * ky, z + B::dt * kz, kx, ky, kz);        // k4
    B::x = (x + h6 * (ax + kx)) + u1;                                     // + u: :73-75
    B::y = (y + h6 * (ay + ky)) + u2;
    B::z = (z + h6 * (az + kz)) + u3;
    B::reset_obs(o);                                                      // :77-83
    rew = -((((T)0 + fabs(o[0])) + fabs(o[1])) + fabs(o[2]));             // :84
    return false;
  }
};

template <typename T>
struct SysL4RK4 : SysL4<T> {
  using B = SysL4<T>;
  T h2, h6;
  __device__ void setup(const KArgs& a) {
    B::setup(a);
    h2 = (T)(a.prm[3] / 2);
    h6 = (T)(a.prm[3] / 6.0);
  }
  __device__ void rk4(T* x) const {
    T k[4], acc[4], y[4];
    B::rhs(x, k);
#pragma unroll
    for (int j = 0; j < 4; ++j) { acc[j] = k[j]; y[j] = x[j] + h2 * k[j]; }
    B::rhs(y, k);
#pragma unroll
    for (int j = 0; j < 4; ++j) { acc[j] = acc[j] + (T)2 * k[j]; y[j] = x[j] + h2 * k[j]; }
    B::rhs(y, k);
#pragma unroll
    for (int j = 0; j < 4; ++j) { acc[j] = acc[j] + (T)2 * k[j]; y[j] = x[j] + B::dt * k[j]; }
    B::rhs(y, k);
#pragma unroll
    for (int j = 0; j < 4; ++j) x[j] = x[j] + h6 * (acc[j] + k[j]);
  }
  __device__ bool step(const float*, bool, const double*, T* o, T& rew, const KArgs&) {
    rk4(B::m);                                                            // master
    rk4(B::s);                                                            // slave
    B::reset_obs(o);                                                      // :333-362
    const T r = -(((((T)0 + fabs(o[0])) + fabs(o[1])) + fabs(o[2])) + fabs(o[3]));  // :363
    rew = r;
    return r < (T)-1e6;                                                   // :369
  }
};

// ===========================================================================
// PMSM -- lorenz_env_try_pmsm.py:7-187 PMSM_Sync_Env (float32 throughout)
// params: sigma=5.46, gamma=20, dt=1e-3, f_max=50, lambda_lr=1e-3, beta1=.9,
//         beta2=.999, eps=1e-8, err_threshold=5, max_steps=2000, term=1000
// planes: state1(3), state2(3), lambda, m_t, v_t, adam_step(i32), step(i32)
// ===========================================================================
#ifndef LZ_PMSM_BIAS_FAST  // 2: early constant-space load; 1: in-place asm load; 0: waterfall alone (A/B)
#define LZ_PMSM_BIAS_FAST 2
#endif
#ifndef LZ_PMSM_NO_BIAS_LOAD
#define LZ_PMSM_NO_BIAS_LOAD 0
#endif
struct SysPMSM {
  using T = float;
  static constexpr int A = 2, O = 6, NI = 6;
  static constexpr bool kUsesAction = true, kNoise = true;
  static constexpr int kStepPlane = LZ_PMSM_STEP;
  float s1[3], s2[3], lam, mt, vt;
  int32_t adam;
  float sg, gm, dt, fmax, lr, b1, b2, eps, thr, tterm, c1, c2, alpha;

  __device__ void setup(const KArgs& a) {
    sg = (float)a.prm[0]; gm = (float)a.prm[1]; dt = (float)a.prm[2]; fmax = (float)a.prm[3];
    lr = (float)a.prm[4]; b1 = (float)a.prm[5]; b2 = (float)a.prm[6]; eps = (float)a.prm[7];
    thr = (float)a.prm[8]; tterm = (float)a.prm[10];
    c1 = (float)(1.0 - a.prm[5]); c2 = (float)(1.0 - a.prm[6]);   // (1 - beta) python floats
    alpha = a.alpha;
  }
  __device__ void load(const KArgs& a, int64_t i) {
#pragma unroll
    for (int j = 0; j < 3; ++j) { s1[j] = ld<float>(a.pl[j], i); s2[j] = ld<float>(a.pl[3 + j], i); }
    lam = ld<float>(a.pl[6], i); mt = ld<float>(a.pl[7], i); vt = ld<float>(a.pl[8], i);
    adam = ld<int32_t>(a.pl[9], i);
  }
  __device__ void store(const KArgs& a, int64_t i) const {
#pragma unroll
    for (int j = 0; j < 3; ++j) { st<float>(a.pl[j], i, s1[j]); st<float>(a.pl[3 + j], i, s2[j]); }
    st<float>(a.pl[6], i, lam); st<float>(a.pl[7], i, mt); st<float>(a.pl[8], i, vt);
    st<int32_t>(a.pl[9], i, adam);
  }
  // reset(): Adam m/v/step and lambda are NOT reset (:59-75)
  __device__ void store_reset(const KArgs& a, int64_t i) const {
#pragma unroll
    for (int j = 0; j < 3; ++j) { st<float>(a.pl[j], i, s1[j]); st<float>(a.pl[3 + j], i, s2[j]); }
  }
  __device__ void store_autoreset_extra(const KArgs&, int64_t) const {}
  // :51-58 _get_derivatives; python int 0 stays f32, a float64 noise promotes the sum
  // to f64 before np.array(..., float32) rounds it
  __device__ void rhs(const float* x, float a1, float a2, bool use_nz, const double* nz,
                      float* d) const {
    const float t1 = (-x[0] + x[1] * x[2]) + a1;
    const float t2 = ((-x[1] - x[0] * x[2]) + gm * x[2]) + a2;
    const float t3 = sg * (x[1] - x[2]);
    if (use_nz) {
      d[0] = (float)((double)t1 + nz[0]);
      d[1] = (float)((double)t2 + nz[1]);
      d[2] = (float)((double)t3 + nz[2]);
    } else {
      d[0] = t1 + 0.0f; d[1] = t2 + 0.0f; d[2] = t3 + 0.0f;
    }
  }
  __device__ static void draw(const KArgs& a, uint64_t gid, uint64_t tick, float* v) {
    // :64-65 np_random.uniform(-30,30,3) in float64, then astype(float32)
    for (int j = 0; j < 6; ++j) v[j] = (float)Draw<double>::uniform(a.seed, gid, tick, j, -30.0, 30.0);
  }
  __device__ void init(const float* v, const KArgs&) {
#pragma unroll
    for (int j = 0; j < 3; ++j) { s1[j] = v[j]; s2[j] = v[3 + j]; }
  }
  __device__ void reset_obs(float* o) const {  // :66-74
    float d1[3], d2[3];
    rhs(s1, 0.0f, 0.0f, false, nullptr, d1);
    rhs(s2, 0.0f, 0.0f, false, nullptr, d2);
#pragma unroll
    for (int j = 0; j < 3; ++j) { o[j] = s1[j] - s2[j]; o[3 + j] = d1[j] - d2[j]; }
  }
  // process noise N(0, 3) (:80), as np_random.normal(loc=0, scale=3) = 0 + 3*z
  __device__ void noise_from_normals(const float* z, double* nz) const {
#pragma unroll
    for (int j = 0; j < 3; ++j) nz[j] = 3.0 * (double)z[j];
  }
  // f32 x**alpha: (float)pow((double)x, alpha) -- correctly rounded except in rare
  // cases, reproducible by the CPU oracle; alpha = 0.5 (the reference default and
  // cfg4) is exactly sqrtf (double-rounding of a square root through double is
  // innocuous), which keeps the fp64 pow off the hot path.
  __device__ float fpow(float x) const {
    if (alpha == 0.5f) return sqrtf(x);
    return (float)pow((double)x, (double)alpha);
  }
  __device__ static float bias(const float* tab, int32_t len, int32_t k) {
    return k < len ? tab[k] : 1.0f;
  }
  // The two table values for this env's Adam step (one interleaved pair), by a SCALAR
  // load issued from asm (waited on with lgkmcnt): a vector load would be waited on with vmcnt, which in the
  // fused rollouts also drains every store still in flight from the previous step.  A
  // waterfall over the distinct steps in the wave -- normally one: all envs of a batch
  // step their (never reset) Adam counters together.  The loads are asm so that hipcc
  // cannot rewrite the uniform index back into the lane's own (a vector load).
  __device__ static void sload2(const float* p, float& x, float& y) {
    uint64_t v;
    asm volatile("s_load_dwordx2 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
    x = __uint_as_float((uint32_t)v);
    y = __uint_as_float((uint32_t)(v >> 32));
  }
  // LZ_PMSM_BIAS_FAST 2: the pair for the wave's first lane's next step, loaded at the top
  // of step() through a constant-address-space pointer -- a scalar load the compiler issues
  // there and waits for (lgkmcnt) only at the first use, after the two RHS evaluations, so
  // its latency overlaps them (the table is never written while a kernel runs).
  struct BiasPre {
    float m, v;
    int32_t k;
  };
  __device__ BiasPre bias_pre(const KArgs& a) const {
    BiasPre p{1.0f, 1.0f, 0};
#if LZ_PMSM_BIAS_FAST == 2 && !LZ_PMSM_NO_BIAS_LOAD
    typedef const __attribute__((address_space(4))) uint64_t cu64;
    p.k = __builtin_amdgcn_readfirstlane(adam) + 1;  // this step's Adam k (:121)
    const int32_t kc = p.k < a.bc_len ? p.k : a.bc_len - 1;
    const uint64_t t = ((cu64*)a.bc)[kc > 0 ? kc : 0];
    p.m = __uint_as_float((uint32_t)t);
    p.v = __uint_as_float((uint32_t)(t >> 32));
#endif
    return p;
  }
  __device__ void bias_pair(const KArgs& a, float& bm, float& bv, const BiasPre& pre) const {
#if LZ_PMSM_NO_BIAS_LOAD  // A/B only (tools/build_ab.sh): what the table load costs -- WRONG results
    bm = bv = 1.0f;
    return;
#endif
#if LZ_PMSM_BIAS_FAST == 2
    {  // the early pair (bias_pre); the waterfall below only when the wave's steps differ
      const bool in = pre.k < a.bc_len;
      bm = in ? pre.m : 1.0f;
      bv = in ? pre.v : 1.0f;
      if (__builtin_expect(__builtin_amdgcn_ballot_w64(adam != pre.k) == 0, 1)) return;
    }
#elif LZ_PMSM_BIAS_FAST
    {  // the wave's first lane's step, loaded without a branch (index clamped, 1.0 selected
       // past the table); the waterfall below only when the wave's steps differ
      const int32_t k0 = __builtin_amdgcn_readfirstlane(adam);
      const int32_t kc = __builtin_amdgcn_readfirstlane(k0 < a.bc_len ? k0 : a.bc_len - 1);
      float m, v;
      sload2(a.bc + 2 * (int64_t)(kc > 0 ? kc : 0), m, v);
      const bool in = k0 < a.bc_len;
      bm = in ? m : 1.0f;
      bv = in ? v : 1.0f;
      if (__builtin_expect(__builtin_amdgcn_ballot_w64(adam != k0) == 0, 1)) return;
    }
#endif
    for (;;) {
      const int32_t k0 = __builtin_amdgcn_readfirstlane(adam);
      float m = 1.0f, v = 1.0f;
      if (k0 < a.bc_len) sload2(a.bc + 2 * (int64_t)k0, m, v);
      if (adam == k0) {
        bm = m;
        bv = v;
        break;
      }
    }
  }
  // step(): :76-184
  __device__ bool step(const float* act, bool use_nz, const double* nz, float* o, float& rew,
                       const KArgs& a) {
    const BiasPre pre = bias_pre(a);
    const float a1 = clip_nz(act[0], -1.0f, 1.0f) * fmax;  // :81-82
    const float a2 = clip_nz(act[1], -1.0f, 1.0f) * fmax;
    float d1[3], d2[3];
    rhs(s1, 0.0f, 0.0f, false, nullptr, d1);                      // :88
    rhs(s2, a1, a2, use_nz, nz, d2);                               // :89-90
#pragma unroll
    for (int j = 0; j < 3; ++j) { s1[j] = s1[j] + d1[j] * dt; s2[j] = s2[j] + d2[j] * dt; }  // :92-93
    rhs(s1, 0.0f, 0.0f, false, nullptr, d1);                      // :95
    rhs(s2, a1, a2, use_nz, nz, d2);                               // :96-97
#pragma unroll
    for (int j = 0; j < 3; ++j) { o[j] = s1[j] - s2[j]; o[3 + j] = d1[j] - d2[j]; }  // :99-102
    const float e1 = fabsf(o[0]), e2 = fabsf(o[1]), e3 = fabsf(o[2]);             // :105-107
    const float es = (e1 + e2) + e3;                       // :108 np.sum (a0+a1)+a2
    const float grad = thr - es;                           // :118
    adam += 1;                                             // :121
    mt = b1 * mt + c1 * grad;                              // :124
    vt = b2 * vt + c2 * (grad * grad);                     // :127 (glibc powf(g,2) in ref)
    float bcm, bcv;
    bias_pair(a, bcm, bcv, pre);
    const float mh = mt / bcm;                             // :130 (1-b1**k) -> f32
    const float vh = vt / bcv;                             // :131
    lam = lam - (lr * mh) / (sqrtf(vh) + eps);             // :135
    lam = clip(lam, 0.0f, 0.5f);                           // :138
    const float tiny = 1e-6f;                              // :158-160 (x + 1e-6)**alpha
    const float fp = (fpow(fabsf(e1) + tiny) + fpow(fabsf(e2) + tiny)) + fpow(fabsf(e3) + tiny);
    const float ap = lam * (act[0] * act[0] + act[1] * act[1]);  // :165 raw action
    float r = ((-es) - fp) - ap;                           // :167
    bool te = false;
    if (es > tterm) { r = -1000.0f; te = true; }           // :174-176
    rew = r;
    return te;
  }
  // step() split over a LANE PAIR (k_rollout_pair: lanes 2e, 2e + 1 both carry env
  // e's full state; lane q = 1 is the "slave" lane).  Every value either lane ends with is
  // the one step() computes -- the same operations on the same operands -- but the work
  // that comes in independent halves runs once per pair instead of twice per lane:
  //  * lane q integrates system q only (q = 0 the master s1 with actions 0 and no noise,
  //    q = 1 the slave s2), then the pair swaps states and derivatives (pair_swap);
  //    the master's RHS runs the noisy form with noise 0.0: (float)((double)t + 0.0) is
  //    t + 0.0f for every float t (-0 -> +0 in both, NaN stays NaN);
  //  * nz_slave: the slave's process noise (lane 1's value is used; the caller's pair
  //    schedule draws the normals, see split_loop);
  //  * the two bias-corrected moments are ONE division per lane (lane 0 mt / bcm, lane 1
  //    vt / bcv) and, at alpha = 0.5, the four square roots TWO per lane (lane 0 sqrt(vh)
  //    and fpow(e1), lane 1 fpow(e2) and fpow(e3)), exchanged.
  __device__ bool step_pair(bool q, const float* act, bool use_nz, const double* nz_slave, float* o,
                            float& rew, const KArgs& a) {
    const BiasPre pre = bias_pre(a);
    const float a1 = clip_nz(act[0], -1.0f, 1.0f) * fmax;  // :81-82
    const float a2 = clip_nz(act[1], -1.0f, 1.0f) * fmax;
    const float u1 = q ? a1 : 0.0f, u2 = q ? a2 : 0.0f;
    double nz[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) nz[j] = q ? nz_slave[j] : 0.0;
    float x[3], d[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) x[j] = q ? s2[j] : s1[j];
    rhs(x, u1, u2, use_nz, nz, d);                                 // :88-90
#pragma unroll
    for (int j = 0; j < 3; ++j) x[j] = x[j] + d[j] * dt;           // :92-93
    rhs(x, u1, u2, use_nz, nz, d);                                 // :95-97
#pragma unroll
    for (int j = 0; j < 3; ++j) {                                  // :99-102
      const float px = pair_swap(x[j]), pd = pair_swap(d[j]);
      s1[j] = q ? px : x[j];
      s2[j] = q ? x[j] : px;
      const float d1 = q ? pd : d[j], d2 = q ? d[j] : pd;
      o[j] = s1[j] - s2[j];
      o[3 + j] = d1 - d2;
    }
    const float e1 = fabsf(o[0]), e2 = fabsf(o[1]), e3 = fabsf(o[2]);             // :105-107
    const float es = (e1 + e2) + e3;                       // :108
    const float grad = thr - es;                           // :118
    adam += 1;                                             // :121
    mt = b1 * mt + c1 * grad;                              // :124
    vt = b2 * vt + c2 * (grad * grad);                     // :127
    float bcm, bcv;
    bias_pair(a, bcm, bcv, pre);
    const float mv = (q ? vt : mt) / (q ? bcv : bcm);      // :130-131, one division per lane
    const float mvp = pair_swap(mv);
    const float mh = q ? mvp : mv, vh = q ? mv : mvp;
    const float tiny = 1e-6f;                              // :158-160 (x + 1e-6)**alpha
    float sv, fp;
    if (alpha == 0.5f) {  // fpow = sqrtf: the four roots two per lane
      const float ra = sqrtf(q ? fabsf(e2) + tiny : vh);
      const float rb = sqrtf(q ? fabsf(e3) + tiny : fabsf(e1) + tiny);
      const float pa = pair_swap(ra), pb = pair_swap(rb);
      sv = q ? pa : ra;
      const float f1 = q ? pb : rb, f2 = q ? ra : pa, f3 = q ? rb : pb;
      fp = (f1 + f2) + f3;
    } else {
      sv = sqrtf(vh);
      fp = (fpow(fabsf(e1) + tiny) + fpow(fabsf(e2) + tiny)) + fpow(fabsf(e3) + tiny);
    }
    lam = lam - (lr * mh) / (sv + eps);                    // :135
    lam = clip(lam, 0.0f, 0.5f);                           // :138
    const float ap = lam * (act[0] * act[0] + act[1] * act[1]);  // :165 raw action
    float r = ((-es) - fp) - ap;                           // :167
    bool te = false;
    if (es > tterm) { r = -1000.0f; te = true; }           // :174-176
    rew = r;
    return te;
  }
};

// ===========================================================================
// HR -- lorenz_env_try.py:7-179 HRSyncEnv (Hindmarsh-Rose, RK4 dt=0.001)
// params: a=1, b=3, c=1, d=5, r=0.006, s=4, I=3.2, x_rest=-1.6, dt=0.001,
//         scale=50, master_scale=20, action_alpha=0.95, term=70
// planes: master(3), slave(3), sigma (T), filtered_action(2) f32 [, step]
// x1**2 / x1**3: correctly rounded here; the reference's glibc pow() is not always
// (<= 1 ulp apart, see oracle/lz_oracle.c ORC_REF vs ORC_DEV).
// ===========================================================================
template <typename T>
__device__ __forceinline__ T cube_cr(T x) {
  const T p = x * x;
  const T e = fma(x, x, -p);
  const T h = p * x;
  const T l = fma(p, x, -h) + e * x;
  return h + l;
}

// x / c for the HR obs scalings, exactly IEEE: in float32, for the reference constants
// c = 50 and 20, as q = x*r, q' = fma(fma(-q, c, x), r, q) with r = RN(1/c) -- three
// instructions instead of the ~10 of a correctly rounded divide.
// tools/div_const_check.c verifies it bit-for-bit against x / c for all 2^32 floats
// with 2^-100 <= |x| <= 2^100; zeros, subnormal quotients and inf/NaN are not covered
// and take the divide (a wave-uniform branch, see SysHR::step).
__device__ __forceinline__ float div_fast(float x, float c, float r) {
  const float q = x * r;
  return fmaf(fmaf(-q, c, x), r, q);
}
__device__ __forceinline__ bool div_fast_ok(float x) {
  const float ax = fabsf(x);
  return ax >= 0x1p-100f && ax <= 0x1p100f;
}

template <typename T>
struct SysHR {
  static constexpr int A = 2, O = 6, NI = 7;
  static constexpr bool kUsesAction = true, kNoise = true;
  static constexpr int kStepPlane = LZ_HR_STEP;
#ifndef LZ_HR_PACKED
#define LZ_HR_PACKED 1
#endif
#ifndef LZ_HR_STEP_WAVES
#define LZ_HR_STEP_WAVES 6
#endif
  static constexpr int kStepWaves = sizeof(T) == 4 ? LZ_HR_STEP_WAVES : 1;  // k_step occupancy hint
  T m[3], s[3], sigma;
  float fa0, fa1;
  T pa, pb, pc, pd, pr, ps, pI, pxr, dt, h2, h6, sc, ms, tterm;
  float falpha, f1m;
  bool fastdiv;

  __device__ void setup(const KArgs& a) {
    pa = (T)a.prm[0]; pb = (T)a.prm[1]; pc = (T)a.prm[2]; pd = (T)a.prm[3];
    pr = (T)a.prm[4]; ps = (T)a.prm[5]; pI = (T)a.prm[6]; pxr = (T)a.prm[7];
    dt = (T)a.prm[8]; h2 = (T)(a.prm[8] / 2); h6 = (T)(a.prm[8] / 6.0);   // :102-105
    sc = (T)a.prm[9]; ms = (T)a.prm[10]; tterm = (T)a.prm[12];
    falpha = (float)a.prm[11]; f1m = (float)(1.0 - a.prm[11]);            // :86
    fastdiv = a.prm[9] == 50.0 && a.prm[10] == 20.0;  // the constants div_fast is verified for
  }
  __device__ void load(const KArgs& a, int64_t i) {
#pragma unroll
    for (int j = 0; j < 3; ++j) { m[j] = ld<T>(a.pl[j], i); s[j] = ld<T>(a.pl[3 + j], i); }
    // sigma / the filter planes are read unconditionally -- from plane 0's own element
    // (already being fetched: no extra traffic) when the flag is off, the value then
    // unused -- so the loads carry no branch: a branch between them makes the compiler's
    // wait counts conservative (k_step_multi's tiles waited for each other's loads)
    const bool nz = (a.flags & LZ_FLAG_ADD_NOISE) != 0, fl = (a.flags & LZ_FLAG_ADD_FILTER) != 0;
    constexpr int64_t kW = sizeof(T) / 4;  // float words per T: plane 0's element i as floats
    sigma = ld<T>(nz ? a.pl[6] : a.pl[0], i);
    fa0 = ld<float>(fl ? a.pl[7] : a.pl[0], fl ? i : i * kW);
    fa1 = ld<float>(fl ? a.pl[8] : a.pl[0], fl ? i : i * kW);
  }
  __device__ void store(const KArgs& a, int64_t i) const {
#pragma unroll
    for (int j = 0; j < 3; ++j) { st<T>(a.pl[j], i, m[j]); st<T>(a.pl[3 + j], i, s[j]); }
    if (a.flags & LZ_FLAG_ADD_FILTER) { st<float>(a.pl[7], i, fa0); st<float>(a.pl[8], i, fa1); }
  }
  __device__ void store_reset(const KArgs& a, int64_t i) const {  // :55-69
#pragma unroll
    for (int j = 0; j < 3; ++j) { st<T>(a.pl[j], i, m[j]); st<T>(a.pl[3 + j], i, s[j]); }
    st<T>(a.pl[6], i, sigma);
    st<float>(a.pl[7], i, 0.0f); st<float>(a.pl[8], i, 0.0f);
  }
  // fields init() sets that store() does not persist: the episode's sigma
  __device__ void store_autoreset_extra(const KArgs& a, int64_t i) const {
    st<T>(a.pl[6], i, sigma);
  }
  // :7-12 hr_derivatives
  __device__ void rhs(const T* x, T a1, T a2, T* d) const {
    const T x2 = x[0] * x[0], x3 = cube_cr(x[0]);
    d[0] = (((x[1] - pa * x3) + pb * x2) - x[2]) + pI;
    d[1] = ((pc - pd * x2) - x[1]) + a1;
    d[2] = pr * (ps * (x[0] - pxr) - x[2]) + a2;
  }
  // The stage sum ((k1 + 2 k2) + 2 k3) + k4 is accumulated as the stages complete --
  // the same operations in the same order, with one stage live instead of four.
  __device__ void rk4(T* x, T a1, T a2) const {  // :100-113
    T k[3], acc[3], y[3];
    rhs(x, a1, a2, k);
#pragma unroll
    for (int j = 0; j < 3; ++j) { acc[j] = k[j]; y[j] = x[j] + h2 * k[j]; }
    rhs(y, a1, a2, k);
#pragma unroll
    for (int j = 0; j < 3; ++j) { acc[j] = acc[j] + (T)2 * k[j]; y[j] = x[j] + h2 * k[j]; }
    rhs(y, a1, a2, k);
#pragma unroll
    for (int j = 0; j < 3; ++j) { acc[j] = acc[j] + (T)2 * k[j]; y[j] = x[j] + dt * k[j]; }
    rhs(y, a1, a2, k);
#pragma unroll
    for (int j = 0; j < 3; ++j) x[j] = x[j] + h6 * (acc[j] + k[j]);
  }
  // float32: master (actions 0, 0) and slave (a1, a2) RK4 steps as one packed
  // computation (lane pair = {master, slave}: v_pk_fma / v_pk_mul / v_pk_add), the
  // same IEEE operations in the same order per element as rhs() / rk4() -- bit-identical.
  typedef float f2 __attribute__((ext_vector_type(2)));
  __device__ static f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
  __device__ void rhs2(const f2* x, f2 act1, f2 act2, f2* d) const {
    const f2 p = x[0] * x[0];                               // cube_cr, elementwise
    const f2 e = fma2(x[0], x[0], -p);
    const f2 h = p * x[0];
    const f2 l = fma2(p, x[0], -h) + e * x[0];
    const f2 x3 = h + l;
    const f2 A = (f2)(float)pa, B = (f2)(float)pb, Cc = (f2)(float)pc, D = (f2)(float)pd;
    const f2 R = (f2)(float)pr, S = (f2)(float)ps, I = (f2)(float)pI, XR = (f2)(float)pxr;
    d[0] = (((x[1] - A * x3) + B * p) - x[2]) + I;
    d[1] = ((Cc - D * p) - x[1]) + act1;
    d[2] = R * (S * (x[0] - XR) - x[2]) + act2;
  }
  __device__ void rk4_pair(T* xm, T* xs, float a1, float a2) {
    f2 x[3], k[3], acc[3], y[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) x[j] = (f2){(float)xm[j], (float)xs[j]};
    const f2 u1 = {0.0f, a1}, u2 = {0.0f, a2};
    const f2 H2 = (f2)(float)h2, DT = (f2)(float)dt, H6 = (f2)(float)h6, TWO = (f2)2.0f;
    rhs2(x, u1, u2, k);
#pragma unroll
    for (int j = 0; j < 3; ++j) { acc[j] = k[j]; y[j] = x[j] + H2 * k[j]; }
    rhs2(y, u1, u2, k);
#pragma unroll
    for (int j = 0; j < 3; ++j) { acc[j] = acc[j] + TWO * k[j]; y[j] = x[j] + H2 * k[j]; }
    rhs2(y, u1, u2, k);
#pragma unroll
    for (int j = 0; j < 3; ++j) { acc[j] = acc[j] + TWO * k[j]; y[j] = x[j] + DT * k[j]; }
    rhs2(y, u1, u2, k);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      x[j] = x[j] + H6 * (acc[j] + k[j]);
      xm[j] = (T)x[j][0];
      xs[j] = (T)x[j][1];
    }
  }
  __device__ static void draw(const KArgs& a, uint64_t gid, uint64_t tick, T* v) {
    for (int j = 0; j < 6; ++j) v[j] = Draw<T>::uniform(a.seed, gid, tick, j, (T)-10, (T)20);  // :55-57
    T sgm = (T)0;                                                                                  // :60-69
    if (a.flags & LZ_FLAG_ADD_NOISE)
      sgm = (a.flags & LZ_FLAG_EVAL_MODE) ? (T)2 : Draw<T>::uniform(a.seed, gid, tick, 6, (T)0, (T)2);
    v[6] = sgm;
  }
  __device__ void init(const T* v, const KArgs&) {
#pragma unroll
    for (int j = 0; j < 3; ++j) { m[j] = v[j]; s[j] = v[3 + j]; }
    sigma = v[6];
    fa0 = 0.0f; fa1 = 0.0f;
  }
  __device__ void reset_obs(T* o) const {  // :71-78 (error clipped in reset only)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      o[j] = clip_nz((m[j] - s[j]) / sc, (T)-1, (T)1);
      o[3 + j] = clip_nz(m[j] / ms, (T)-1, (T)1);
    }
  }
  __device__ void noise_from_normals(const float* z, double* nz) const {  // :136 N(0, sigma)
#pragma unroll
    for (int j = 0; j < 3; ++j) nz[j] = (double)sigma * (double)z[j];
  }
  // step(): :80-179
  __device__ bool step(const float* act, bool use_nz, const double* nz, T* o, T& rew,
                       const KArgs& a) {
    float f0 = act[0], f1 = act[1];
    if (a.flags & LZ_FLAG_ADD_FILTER) {                    // :85-86
      fa0 = f1m * fa0 + falpha * f0;
      fa1 = f1m * fa1 + falpha * f1;
      f0 = fa0; f1 = fa1;
    }
    const float a1 = clip_nz(f0, -1.0f, 1.0f) * 100.0f;    // :92-93 np.float32 * 100.0
    const float a2 = clip_nz(f1, -1.0f, 1.0f) * 100.0f;
    if constexpr (std::is_same<T, float>::value && LZ_HR_PACKED) {
      rk4_pair(m, s, a1, a2);                              // both systems, packed f32
    } else {
      rk4(m, (T)0, (T)0);                                  // :100-105
      rk4(s, (T)a1, (T)a2);                                // :108-113
    }
    if (use_nz) {                                          // :135-137
#pragma unroll
      for (int j = 0; j < 3; ++j) m[j] = m[j] + (T)nz[j] * dt;
    }
    T e[3];
    bool te = false;
#pragma unroll
    for (int j = 0; j < 3; ++j) e[j] = m[j] - s[j];
    bool slow = true;
    if constexpr (std::is_same<T, float>::value) {  // div_fast: bit-identical to the divide
      bool ok = fastdiv;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        ok = ok && div_fast_ok(e[j]) && div_fast_ok(m[j]);
        o[j] = div_fast(e[j], 50.0f, 0x1.47ae14p-6f);      // RN(1/50)
        o[3 + j] = div_fast(m[j], 20.0f, 0x1.99999ap-5f);  // RN(1/20)
      }
      slow = !__all(ok);  // wave-uniform: the divides run only if some lane needs them
    }
    if (slow) {
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        o[j] = e[j] / sc;
        o[3 + j] = m[j] / ms;
      }
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {                          // :150-156
      o[3 + j] = clip_nz(o[3 + j], (T)-1, (T)1);
      te = te || (fabs(e[j]) > tterm);                     // :174
    }
    const float q = act[0] * act[0] + act[1] * act[1];     // np.square + np.sum (f32)
    const float pen = 0.05f * q;                           // 0.050 * f32 -> f32
    T r = (-((fabs(o[0]) + fabs(o[1])) + fabs(o[2]))) - (T)pen;  // :165
    if (te) r = (T)-2000.0;                                // :175-176
    rew = r;
    return te;
  }
};

// ===========================================================================
// Legacy, unregistered variants, fp64 in the reference.  Shared RHS
// of the PMSM-form 3-state system (a = 5.46, b = 20):
//   f = [(-x) + y*z, ((-y) - x*z) + b*z, a*(y - z)]   (python evaluation order)
// ===========================================================================
template <typename T>
__device__ __forceinline__ void pmsm3_rhs(T x, T y, T z, T pa, T pb, T* f) {
  f[0] = (-x) + y * z;
  f[1] = ((-y) - x * z) + pb * z;
  f[2] = pa * (y - z);
}

// T1 -- lorenz_env_transient1.py:18-104: one controlled system, additive actions
// (clip +-10, np.float32) on x and y, Euler dt=0.01; the N(0,1) draw of :77 is unused.
// params: a=5.46, b=20, -, dt=0.01, clip=10, T_end=10.  planes: x, y, z [, step]
template <typename T>
struct SysT1 {
  static constexpr int A = 2, O = 6, NI = 3;
  static constexpr bool kUsesAction = true, kNoise = false;
  static constexpr int kStepPlane = LZ_T1_STEP;
  T v[3];
  T pa, pb, dt;
  float cl;

  __device__ void setup(const KArgs& a) {
    pa = (T)a.prm[0]; pb = (T)a.prm[1]; dt = (T)a.prm[3]; cl = (float)a.prm[4];
  }
  __device__ void load(const KArgs& a, int64_t i) {
#pragma unroll
    for (int j = 0; j < 3; ++j) v[j] = ld<T>(a.pl[j], i);
  }
  __device__ void store(const KArgs& a, int64_t i) const {
#pragma unroll
    for (int j = 0; j < 3; ++j) st<T>(a.pl[j], i, v[j]);
  }
  __device__ void store_reset(const KArgs& a, int64_t i) const { store(a, i); }
  __device__ void store_autoreset_extra(const KArgs&, int64_t) const {}
  __device__ static void draw(const KArgs& a, uint64_t gid, uint64_t tick, T* w) {
    for (int j = 0; j < 3; ++j) w[j] = Draw<T>::uniform(a.seed, gid, tick, j, (T)-30, (T)30);  // :43
  }
  __device__ void init(const T* w, const KArgs&) { v[0] = w[0]; v[1] = w[1]; v[2] = w[2]; }
  __device__ void reset_obs(T* o) const {  // :44-57 [s, f(s)] - zeros(6)
    T f[3];
    pmsm3_rhs(v[0], v[1], v[2], pa, pb, f);
#pragma unroll
    for (int j = 0; j < 3; ++j) { o[j] = v[j] - (T)0; o[3 + j] = f[j] - (T)0; }
  }
  __device__ void noise_from_normals(const float*, double* nz) const { nz[0] = nz[1] = nz[2] = 0.0; }
  __device__ bool step(const float* act, bool, const double*, T* o, T& rew, const KArgs&) {
    const float u1 = clip_nz(act[0], -cl, cl), u2 = clip_nz(act[1], -cl, cl);  // :71-72
    T f[3];
    pmsm3_rhs(v[0], v[1], v[2], pa, pb, f);                              // :78-80
    v[0] = (v[0] + f[0] * dt) + (T)u1;                                   // :84
    v[1] = (v[1] + f[1] * dt) + (T)u2;                                   // :85
    v[2] = v[2] + f[2] * dt;                                             // :86
    reset_obs(o);                                                        // :88-97
    rew = -((((T)0 + fabs(o[0])) + fabs(o[1])) + fabs(o[2]));            // :98
    return false;                                                        // :100 never fires
  }
};

// T2 -- lorenz_env_transient2.py:115-240: 4-state master/slave, actions (clip +-2,
// np.float32, * 100 in float32) on slave x1, x2, x4, Euler dt=0.001; the N(0,0.5)
// draw of :209 is unused; reward -S - S**(1/3).
// params: a=30, b=1, c=36, dt=0.001, clip=2, T_end=5, d=0.5, h=0.003, gain=100, 0.01
// planes: master x1..x4, slave x1..x4 [, step]
template <typename T>
struct SysT2 {
  static constexpr int A = 3, O = 8, NI = 8;
  static constexpr bool kUsesAction = true, kNoise = false;
  static constexpr int kStepPlane = LZ_T2_STEP;
  T m[4], s[4];
  T pa, pb, pc, dt, pd, ph, dmp;
  float cl, gain;

  __device__ void setup(const KArgs& a) {
    pa = (T)a.prm[0]; pb = (T)a.prm[1]; pc = (T)a.prm[2]; dt = (T)a.prm[3];
    cl = (float)a.prm[4]; pd = (T)a.prm[6]; ph = (T)a.prm[7]; gain = (float)a.prm[8];
    dmp = (T)a.prm[9];
  }
  __device__ void load(const KArgs& a, int64_t i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) { m[j] = ld<T>(a.pl[j], i); s[j] = ld<T>(a.pl[4 + j], i); }
  }
  __device__ void store(const KArgs& a, int64_t i) const {
#pragma unroll
    for (int j = 0; j < 4; ++j) { st<T>(a.pl[j], i, m[j]); st<T>(a.pl[4 + j], i, s[j]); }
  }
  __device__ void store_reset(const KArgs& a, int64_t i) const { store(a, i); }
  __device__ void store_autoreset_extra(const KArgs&, int64_t) const {}
  // :145-148 / :189-192
  __device__ void rhs(const T* x, T* f) const {
    const T q = ((T)2 * x[3]) * x[3];
    f[0] = pa * (q * (x[1] - x[0]) + pd * x[0]);
    f[1] = pb * (q * (x[0] - x[1]) - x[2]);
    f[2] = pc * (x[1] - ph * x[2]);
    f[3] = (x[1] - x[0]) - dmp * x[3];
  }
  __device__ static void draw(const KArgs& a, uint64_t gid, uint64_t tick, T* w) {
    for (int j = 0; j < 8; ++j) w[j] = Draw<T>::uniform(a.seed, gid, tick, j, (T)0, (T)5);  // :141-142
  }
  __device__ void init(const T* w, const KArgs&) {
#pragma unroll
    for (int j = 0; j < 4; ++j) { m[j] = w[j]; s[j] = w[4 + j]; }
  }
  __device__ void reset_obs(T* o) const {  // :143-166 [m, f(m)] - [s, f(s)]
    T fm[4], fs[4];
    rhs(m, fm);
    rhs(s, fs);
#pragma unroll
    for (int j = 0; j < 4; ++j) { o[j] = m[j] - s[j]; o[4 + j] = fm[j] - fs[j]; }
  }
  __device__ void noise_from_normals(const float*, double* nz) const { nz[0] = nz[1] = nz[2] = 0.0; }
  __device__ bool step(const float* act, bool, const double*, T* o, T& rew, const KArgs&) {
    const float g1 = clip_nz(act[0], -cl, cl) * gain;   // :182-184, :210-213 u*100 in f32
    const float g2 = clip_nz(act[1], -cl, cl) * gain;
    const float g3 = clip_nz(act[2], -cl, cl) * gain;
    T f[4];
    rhs(m, f);                                       // :189-192
#pragma unroll
    for (int j = 0; j < 4; ++j) m[j] = m[j] + f[j] * dt;   // :193-196
    rhs(s, f);                                       // :210-213
    f[0] = f[0] + (T)g1;
    f[1] = f[1] + (T)g2;
    f[3] = f[3] + (T)g3;
#pragma unroll
    for (int j = 0; j < 4; ++j) s[j] = s[j] + f[j] * dt;   // :214-217
    reset_obs(o);                                    // :198-227
    const T S = ((((T)0 + fabs(o[0])) + fabs(o[1])) + fabs(o[2])) + fabs(o[3]);
    const T r = (-S) - (T)pow((double)S, 1.0 / 3.0);  // :229
    rew = r;
    return r < (T)-1e6;                              // :235 (t == 5 never fires)
  }
};

// TP -- lorenz_env_transient_pmsm.py:17-133: PMSM-form master/slave, actions (clip
// +-2, * 20 in float32) and process noise N(0,3) (:86) on the slave, Euler dt=0.01,
// reward -S - S**(1/10).  The reference always adds the noise (LZ_FLAG_ADD_NOISE is
// this system's default).
// params: a=5.46, b=20, gain=20, dt=0.01, clip=2, T_end=5, noise std=3
// planes: master(3), slave(3) [, step]
template <typename T>
struct SysTP {
  static constexpr int A = 2, O = 6, NI = 6;
  static constexpr bool kUsesAction = true, kNoise = true;
  static constexpr int kStepPlane = LZ_TP_STEP;
  T m[3], s[3];
  T pa, pb, dt;
  float cl, gain;
  double nstd;

  __device__ void setup(const KArgs& a) {
    pa = (T)a.prm[0]; pb = (T)a.prm[1]; gain = (float)a.prm[2]; dt = (T)a.prm[3];
    cl = (float)a.prm[4]; nstd = a.prm[6];
  }
  __device__ void load(const KArgs& a, int64_t i) {
#pragma unroll
    for (int j = 0; j < 3; ++j) { m[j] = ld<T>(a.pl[j], i); s[j] = ld<T>(a.pl[3 + j], i); }
  }
  __device__ void store(const KArgs& a, int64_t i) const {
#pragma unroll
    for (int j = 0; j < 3; ++j) { st<T>(a.pl[j], i, m[j]); st<T>(a.pl[3 + j], i, s[j]); }
  }
  __device__ void store_reset(const KArgs& a, int64_t i) const { store(a, i); }
  __device__ void store_autoreset_extra(const KArgs&, int64_t) const {}
  __device__ static void draw(const KArgs& a, uint64_t gid, uint64_t tick, T* w) {
    for (int j = 0; j < 6; ++j) w[j] = Draw<T>::uniform(a.seed, gid, tick, j, (T)-10, (T)10);  // :45-46
  }
  __device__ void init(const T* w, const KArgs&) {
#pragma unroll
    for (int j = 0; j < 3; ++j) { m[j] = w[j]; s[j] = w[3 + j]; }
  }
  __device__ void reset_obs(T* o) const {  // :47-65
    T fm[3], fs[3];
    pmsm3_rhs(m[0], m[1], m[2], pa, pb, fm);
    pmsm3_rhs(s[0], s[1], s[2], pa, pb, fs);
#pragma unroll
    for (int j = 0; j < 3; ++j) { o[j] = m[j] - s[j]; o[3 + j] = fm[j] - fs[j]; }
  }
  __device__ void noise_from_normals(const float* z, double* nz) const {
#pragma unroll
    for (int j = 0; j < 3; ++j) nz[j] = nstd * (double)z[j];
  }
  __device__ bool step(const float* act, bool use_nz, const double* nz, T* o, T& rew,
                       const KArgs&) {
    const float g1 = clip_nz(act[0], -cl, cl) * gain;   // :78-79, :91-92 u*20 in f32
    const float g2 = clip_nz(act[1], -cl, cl) * gain;
    T f[3];
    pmsm3_rhs(m[0], m[1], m[2], pa, pb, f);          // :87-89
#pragma unroll
    for (int j = 0; j < 3; ++j) m[j] = m[j] + f[j] * dt;   // :97-99
    pmsm3_rhs(s[0], s[1], s[2], pa, pb, f);          // :91-93
    f[0] = f[0] + (T)g1;
    f[1] = f[1] + (T)g2;
    if (use_nz) {
#pragma unroll
      for (int j = 0; j < 3; ++j) f[j] = f[j] + (T)nz[j];
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) s[j] = s[j] + f[j] * dt;   // :101-103
    reset_obs(o);                                    // :104-121
    const T S = (((T)0 + fabs(o[0])) + fabs(o[1])) + fabs(o[2]);
    const T r = (-S) - (T)pow((double)S, 0.1);       // :122
    rew = r;
    return r < (T)-1e6;                              // :129 (t == 5 never fires)
  }
};

// SC -- lorenz_singlecontrol.py:97-172: a fixed-start ([25, 1, -1], :121) PMSM-form
// system driven only by process noise N(0,3) on its derivatives (:147-153), no action
// (step() takes none), Euler dt=0.01.  Noise is always on in the reference.
// params: a=5.46, b=20, -, dt=0.01, clip=100, T_end=1000, noise std=3, x0, y0, z0
// planes: x, y, z [, step]
template <typename T>
struct SysSC {
  static constexpr int A = 2, O = 6, NI = 3;
  static constexpr bool kUsesAction = false, kNoise = true;
  static constexpr int kStepPlane = LZ_SC_STEP;
  T v[3];
  T pa, pb, dt;
  double nstd;

  __device__ void setup(const KArgs& a) {
    pa = (T)a.prm[0]; pb = (T)a.prm[1]; dt = (T)a.prm[3]; nstd = a.prm[6];
  }
  __device__ void load(const KArgs& a, int64_t i) {
#pragma unroll
    for (int j = 0; j < 3; ++j) v[j] = ld<T>(a.pl[j], i);
  }
  __device__ void store(const KArgs& a, int64_t i) const {
#pragma unroll
    for (int j = 0; j < 3; ++j) st<T>(a.pl[j], i, v[j]);
  }
  __device__ void store_reset(const KArgs& a, int64_t i) const { store(a, i); }
  __device__ void store_autoreset_extra(const KArgs&, int64_t) const {}
  __device__ static void draw(const KArgs& a, uint64_t, uint64_t, T* w) {
    w[0] = (T)a.prm[7]; w[1] = (T)a.prm[8]; w[2] = (T)a.prm[9];   // :121 fixed start
  }
  __device__ void init(const T* w, const KArgs&) { v[0] = w[0]; v[1] = w[1]; v[2] = w[2]; }
  __device__ void reset_obs(T* o) const {  // :122-131
    T f[3];
    pmsm3_rhs(v[0], v[1], v[2], pa, pb, f);
#pragma unroll
    for (int j = 0; j < 3; ++j) { o[j] = v[j] - (T)0; o[3 + j] = f[j] - (T)0; }
  }
  __device__ void noise_from_normals(const float* z, double* nz) const {
#pragma unroll
    for (int j = 0; j < 3; ++j) nz[j] = nstd * (double)z[j];
  }
  __device__ bool step(const float*, bool use_nz, const double* nz, T* o, T& rew, const KArgs&) {
    T f[3];
    pmsm3_rhs(v[0], v[1], v[2], pa, pb, f);          // :150-152
    if (use_nz) {
#pragma unroll
      for (int j = 0; j < 3; ++j) f[j] = f[j] + (T)nz[j];
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) v[j] = v[j] + f[j] * dt;   // :154-156
    reset_obs(o);                                    // :158-164
    rew = -((((T)0 + fabs(o[0])) + fabs(o[1])) + fabs(o[2]));   // :165
    return false;                                    // :169 't == 1000' never fires
  }
};

}  // namespace lz
