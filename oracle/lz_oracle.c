/*
 * lz_oracle.c -- CPU restatement of the reference's env hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (gym-lorenz_amd/) links,
 * loads or calls this file.  It is used by tests/ (the parity checker),
 * __graft_entry__.smoke() (checker) and bench.py's cpu_baseline leg.
 *
 * Each function is a scalar loop over a batch of independent envs that follows
 * the reference's Python/NumPy expression ORDER and DTYPE PROMOTION (numpy 2.2,
 * NEP 50) line by line; file:line citations are relative to
 * /root/reference/code/gym-lorenz/gym_lorenz/envs/.  Compiled with
 * -ffp-contract=off (no FMA contraction, like NumPy's scalar ops).
 *
 * Pinning: tests/test_oracle_golden.py checks the fp64 (LORENZ3, LORENZ4, HR) and
 * fp32 (PMSM) variants in mode ORC_REF BIT-EXACTLY against the tests/golden npz fixtures,
 * which were produced by running the reference env classes themselves
 * (tests/golden/make_golden.py).
 *
 * `mode` selects how x**k is evaluated, the only place where the reference's
 * result depends on a libm implementation (glibc pow/powf, which NumPy's scalar
 * power calls and which is not correctly rounded):
 *   ORC_REF: glibc pow()/powf() exactly as NumPy          -> bit-exact vs golden
 *   ORC_DEV: the device kernel's formulas (correctly rounded x*x, a double-double
 *            x^3, and (float)pow((double)x, a) for PMSM's fractional power)
 *            -> bit-exact vs the HIP kernel; differs from ORC_REF by <= 1 ulp in
 *            the rare cases where glibc's pow is not correctly rounded.
 * Layout: AoS batches, row i = env i.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#define ORC_REF 0
#define ORC_DEV 1

/* np.clip: NaN-propagating (maximum/minimum propagate NaN) */
static inline double clipd(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }
static inline float clipf(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }

/* correctly rounded x*x*x via an error-free double-double product (device formula) */
static inline double cube_dd(double x) {
  double p = x * x;
  double e = fma(x, x, -p);
  double h = p * x;
  double l = fma(p, x, -h) + e * x;
  return h + l;
}
static inline float cube_ddf(float x) {
  float p = x * x;
  float e = fmaf(x, x, -p);
  float h = p * x;
  float l = fmaf(p, x, -h) + e * x;
  return h + l;
}

/* =========================================================================
 * LORENZ3 -- dynamic.py:5-93 lorenzEnv_transient (3-state, Euler, dt=0.01)
 * p = {sigma(self.u)=10, rho(self.i)=28, beta(self.o)=8/3, dt=0.01, clip=500}
 * ========================================================================= */
#define L3_BODY(T, CLIP)                                                             \
  /* dynamic.py:39-41 / :70-72 / :77-79 */                                          \
  static inline void l3_rhs_##T(const T* s, T* f, const T* p) {                     \
    f[0] = p[0] * (s[1] - s[0]);                                                     \
    f[1] = (p[1] * s[0] - s[1]) - s[0] * s[2];                                       \
    f[2] = s[0] * s[1] - p[2] * s[2];                                                \
  }                                                                                  \
  /* reset obs: dynamic.py:35-50 (state0 - zeros) */                                 \
  void orc_l3_reset_obs_##T(int64_t n, const T* st, T* obs, const double* pd) {      \
    T p[5]; for (int j = 0; j < 5; ++j) p[j] = (T)pd[j];                             \
    for (int64_t i = 0; i < n; ++i) {                                                \
      T f[3]; l3_rhs_##T(st + 3 * i, f, p);                                          \
      for (int j = 0; j < 3; ++j) { obs[6 * i + j] = st[3 * i + j] - (T)0;           \
                                    obs[6 * i + 3 + j] = f[j] - (T)0; }              \
    }                                                                                \
  }                                                                                  \
  /* step: dynamic.py:61-90 */                                                       \
  void orc_l3_step_##T(int64_t n, T* st, const T* act, T* obs, T* rew,               \
                       const double* pd) {                                           \
    T p[5]; for (int j = 0; j < 5; ++j) p[j] = (T)pd[j];                             \
    for (int64_t i = 0; i < n; ++i) {                                                \
      T* s = st + 3 * i; T u[3], f[3];                                               \
      for (int j = 0; j < 3; ++j) u[j] = CLIP(act[3 * i + j], -p[4], p[4]); /*:63-65*/\
      l3_rhs_##T(s, f, p);                                          /* :70-72 */     \
      for (int j = 0; j < 3; ++j) s[j] = (s[j] + f[j] * p[3]) + u[j]; /* :73-75 */   \
      l3_rhs_##T(s, f, p);                                          /* :77-79 */     \
      T* o = obs + 6 * i;                                                            \
      for (int j = 0; j < 3; ++j) { o[j] = s[j] - (T)0; o[3 + j] = f[j] - (T)0; }    \
      /* :84  -sum(abs(x) for x in now[0:3]) : python sum starts from int 0 */       \
      rew[i] = -((((T)0 + (T)fabs(o[0])) + (T)fabs(o[1])) + (T)fabs(o[2]));          \
    }                                                                                \
  }
L3_BODY(double, clipd)
L3_BODY(float, clipf)

/* =========================================================================
 * LORENZ4 -- lorenz_env_transient.py:247-376 (4-state master/slave, dt=0.001)
 * p = {a=10, b=8/3, c=28, dt=0.001, clip=2}; the action is clipped but never used
 * ========================================================================= */
#define L4_BODY(T)                                                                   \
  /* :323-326 (master), :344-347 (slave) */                                          \
  static inline void l4_rhs_##T(const T* s, T* f, const T* p) {                     \
    f[0] = p[0] * (s[1] - s[0]) + s[3];                                              \
    f[1] = (p[2] * s[0] - s[1]) - s[0] * s[2];                                       \
    f[2] = s[0] * s[1] - p[1] * s[2];                                                \
    f[3] = (-s[0]) * s[1] - p[1] * s[2];                                             \
  }                                                                                  \
  /* reset obs :275-300 : [m - s, f(m) - f(s)] ; st row = [master(4), slave(4)] */   \
  void orc_l4_reset_obs_##T(int64_t n, const T* st, T* obs, const double* pd) {      \
    T p[5]; for (int j = 0; j < 5; ++j) p[j] = (T)pd[j];                             \
    for (int64_t i = 0; i < n; ++i) {                                                \
      const T* m = st + 8 * i; const T* s = m + 4; T fm[4], fs[4];                   \
      l4_rhs_##T(m, fm, p); l4_rhs_##T(s, fs, p);                                    \
      for (int j = 0; j < 4; ++j) { obs[8 * i + j] = m[j] - s[j];                    \
                                    obs[8 * i + 4 + j] = fm[j] - fs[j]; }            \
    }                                                                                \
  }                                                                                  \
  /* step :314-373 ; done = (t == 5) [host] or reward < -1e6 */                      \
  void orc_l4_step_##T(int64_t n, T* st, T* obs, T* rew, uint8_t* done,              \
                       const double* pd) {                                           \
    T p[5]; for (int j = 0; j < 5; ++j) p[j] = (T)pd[j];                             \
    for (int64_t i = 0; i < n; ++i) {                                                \
      T* m = st + 8 * i; T* s = m + 4; T f[4];                                       \
      l4_rhs_##T(m, f, p);                                          /* :323-326 */   \
      for (int j = 0; j < 4; ++j) m[j] = m[j] + f[j] * p[3];        /* :327-330 */   \
      T fm[4]; l4_rhs_##T(m, fm, p);                                /* :333-336 */   \
      l4_rhs_##T(s, f, p);                                          /* :344-347 */   \
      for (int j = 0; j < 4; ++j) s[j] = s[j] + f[j] * p[3];        /* :348-351 */   \
      T fs[4]; l4_rhs_##T(s, fs, p);                                /* :354-357 */   \
      T* o = obs + 8 * i;                                                            \
      for (int j = 0; j < 4; ++j) { o[j] = m[j] - s[j]; o[4 + j] = fm[j] - fs[j]; }  \
      T r = -(((((T)0 + (T)fabs(o[0])) + (T)fabs(o[1])) + (T)fabs(o[2])) +           \
              (T)fabs(o[3]));                                       /* :121 */       \
      rew[i] = r;                                                                    \
      done[i] = (r < (T)-1e6) ? 1 : 0;                              /* :127 */       \
    }                                                                                \
  }
L4_BODY(double)
L4_BODY(float)

/* =========================================================================
 * LZ_INT_RK4 (lz_config.integrator) -- an opt-in mode of LORENZ3 / LORENZ4 that the
 * reference does NOT have (its Lorenz envs are forward Euler, dynamic.py:70-75): the
 * classical RK4 step in HRSyncEnv's stage order (lorenz_env_try.py:100-113):
 *   k1 = f(s); k2 = f(s + dt/2*k1); k3 = f(s + dt/2*k2); k4 = f(s + dt*k3);
 *   s  = s + (dt/6.0)*(((k1 + 2*k2) + 2*k3) + k4)
 * with python-float dt/2 and dt/6.0, on the L3 / L4 right-hand sides above; LORENZ3
 * then adds the clipped action as dynamic.py:73-75 does: s' = (s + ...) + u.  Obs,
 * reward and done are the Euler steps'.  PARITY UNPINNED against the reference (no RK4
 * Lorenz exists there); tests/test_oracle_golden.py pins this C code to an independent
 * vectorised NumPy float64 RK4 of dynamic.py's RHS instead.
 * ========================================================================= */
#define RK4_BODY(T, CLIP)                                                            \
  static inline void l3_rk4_##T(T* s, const T* p, T h2, T h, T h6) {                 \
    T k1[3], k2[3], k3[3], k4[3], y[3];                                              \
    l3_rhs_##T(s, k1, p);                                                            \
    for (int j = 0; j < 3; ++j) y[j] = s[j] + h2 * k1[j];                            \
    l3_rhs_##T(y, k2, p);                                                            \
    for (int j = 0; j < 3; ++j) y[j] = s[j] + h2 * k2[j];                            \
    l3_rhs_##T(y, k3, p);                                                            \
    for (int j = 0; j < 3; ++j) y[j] = s[j] + h * k3[j];                             \
    l3_rhs_##T(y, k4, p);                                                            \
    for (int j = 0; j < 3; ++j)                                                      \
      s[j] = s[j] + h6 * (((k1[j] + (T)2 * k2[j]) + (T)2 * k3[j]) + k4[j]);           \
  }                                                                                  \
  void orc_l3_step_rk4_##T(int64_t n, T* st, const T* act, T* obs, T* rew,           \
                           const double* pd) {                                       \
    T p[5]; for (int j = 0; j < 5; ++j) p[j] = (T)pd[j];                             \
    const T h2 = (T)(pd[3] / 2), h = (T)pd[3], h6 = (T)(pd[3] / 6.0);                \
    for (int64_t i = 0; i < n; ++i) {                                                \
      T* s = st + 3 * i; T u[3], f[3];                                               \
      for (int j = 0; j < 3; ++j) u[j] = CLIP(act[3 * i + j], -p[4], p[4]);          \
      l3_rk4_##T(s, p, h2, h, h6);                                                   \
      for (int j = 0; j < 3; ++j) s[j] = s[j] + u[j];        /* :73-75's + u */      \
      l3_rhs_##T(s, f, p);                                                           \
      T* o = obs + 6 * i;                                                            \
      for (int j = 0; j < 3; ++j) { o[j] = s[j] - (T)0; o[3 + j] = f[j] - (T)0; }    \
      rew[i] = -((((T)0 + (T)fabs(o[0])) + (T)fabs(o[1])) + (T)fabs(o[2]));          \
    }                                                                                \
  }                                                                                  \
  static inline void l4_rk4_##T(T* s, const T* p, T h2, T h, T h6) {                 \
    T k1[4], k2[4], k3[4], k4[4], y[4];                                              \
    l4_rhs_##T(s, k1, p);                                                            \
    for (int j = 0; j < 4; ++j) y[j] = s[j] + h2 * k1[j];                            \
    l4_rhs_##T(y, k2, p);                                                            \
    for (int j = 0; j < 4; ++j) y[j] = s[j] + h2 * k2[j];                            \
    l4_rhs_##T(y, k3, p);                                                            \
    for (int j = 0; j < 4; ++j) y[j] = s[j] + h * k3[j];                             \
    l4_rhs_##T(y, k4, p);                                                            \
    for (int j = 0; j < 4; ++j)                                                      \
      s[j] = s[j] + h6 * (((k1[j] + (T)2 * k2[j]) + (T)2 * k3[j]) + k4[j]);           \
  }                                                                                  \
  void orc_l4_step_rk4_##T(int64_t n, T* st, T* obs, T* rew, uint8_t* done,          \
                           const double* pd) {                                       \
    T p[5]; for (int j = 0; j < 5; ++j) p[j] = (T)pd[j];                             \
    const T h2 = (T)(pd[3] / 2), h = (T)pd[3], h6 = (T)(pd[3] / 6.0);                \
    for (int64_t i = 0; i < n; ++i) {                                                \
      T* m = st + 8 * i; T* s = m + 4; T fm[4], fs[4];                               \
      l4_rk4_##T(m, p, h2, h, h6);                                                   \
      l4_rk4_##T(s, p, h2, h, h6);                                                   \
      l4_rhs_##T(m, fm, p); l4_rhs_##T(s, fs, p);                                    \
      T* o = obs + 8 * i;                                                            \
      for (int j = 0; j < 4; ++j) { o[j] = m[j] - s[j]; o[4 + j] = fm[j] - fs[j]; }  \
      T r = -(((((T)0 + (T)fabs(o[0])) + (T)fabs(o[1])) + (T)fabs(o[2])) +           \
              (T)fabs(o[3]));                                                        \
      rew[i] = r;                                                                    \
      done[i] = (r < (T)-1e6) ? 1 : 0;                                               \
    }                                                                                \
  }
RK4_BODY(double, clipd)
RK4_BODY(float, clipf)

/* =========================================================================
 * PMSM -- lorenz_env_try_pmsm.py:7-187 PMSM_Sync_Env (float32 throughout)
 * p = {sigma=5.46, gamma=20, dt=0.001, f_max=50, lambda_lr=1e-3, beta1=.9,
 *      beta2=.999, eps=1e-8, err_threshold=5, max_steps=2000, term=1000}
 * ========================================================================= */
/* :51-58 _get_derivatives. The action/noise adds follow NumPy promotion: python int
 * 0 is weak (stays f32), a float64 noise promotes the sum to f64 before the final
 * np.array(..., float32) rounding. */
static inline void pmsm_rhs(const float* x, float a1, float a2, const double* nz, float sig,
                            float gam, float* d) {
  float t1 = (-x[0] + x[1] * x[2]) + a1;
  float t2 = ((-x[1] - x[0] * x[2]) + gam * x[2]) + a2;
  float t3 = sig * (x[1] - x[2]);
  if (nz) {
    d[0] = (float)((double)t1 + nz[0]);
    d[1] = (float)((double)t2 + nz[1]);
    d[2] = (float)((double)t3 + nz[2]);
  } else {
    d[0] = t1 + 0.0f; d[1] = t2 + 0.0f; d[2] = t3 + 0.0f;
  }
}

/* reset obs :59-75 ; st row = [state1(3), state2(3)] */
void orc_pmsm_reset_obs(int64_t n, const float* st, float* obs, const double* pd) {
  float sig = (float)pd[0], gam = (float)pd[1];
  for (int64_t i = 0; i < n; ++i) {
    const float* s1 = st + 6 * i; const float* s2 = s1 + 3; float d1[3], d2[3];
    pmsm_rhs(s1, 0.0f, 0.0f, NULL, sig, gam, d1);
    pmsm_rhs(s2, 0.0f, 0.0f, NULL, sig, gam, d2);
    for (int j = 0; j < 3; ++j) { obs[6 * i + j] = s1[j] - s2[j]; obs[6 * i + 3 + j] = d1[j] - d2[j]; }
  }
}

/* f32 x**k as NumPy (glibc powf) or as the device */
static inline float pmsm_pow(float x, float a, int mode) {
  if (mode == ORC_REF) return powf(x, a);
  if (a == 0.5f) return sqrtf(x); /* device: exact (rounding sqrt via double is innocuous) */
  return (float)pow((double)x, (double)a);
}
static inline float pmsm_sq(float x, int mode) { return mode == ORC_REF ? powf(x, 2.0f) : x * x; }

/* (float)(1 - beta**k) : python float expression rounded to f32 when it meets an
 * np.float32 (:130-131).  Both modes use libm pow; the device reads a host-built
 * table of exactly these values. */
static inline float pmsm_bias(double beta, int32_t k) { return (float)(1.0 - pow(beta, (double)k)); }

/* step :76-184.  lam/m/v/adam_step persist across resets; cur_step is reset by the
 * caller.  noise: double [n,3] (the N(0,3) draw, always consumed by the reference;
 * used only when add_noise) or NULL. */
void orc_pmsm_step(int64_t n, float* st, float* lam, float* mt, float* vt, int32_t* adam_step,
                   int32_t* cur_step, const float* act, const double* noise, int add_noise,
                   float alpha, int mode, float* obs, float* rew, uint8_t* term, uint8_t* trunc,
                   const double* pd) {
  const float sig = (float)pd[0], gam = (float)pd[1], dt = (float)pd[2], fmax = (float)pd[3];
  const float lr = (float)pd[4], b1 = (float)pd[5], b2 = (float)pd[6], eps = (float)pd[7];
  const float thr = (float)pd[8], tterm = (float)pd[10];
  const float c1 = (float)(1.0 - pd[5]), c2 = (float)(1.0 - pd[6]);
  const int32_t max_steps = (int32_t)pd[9];
  const float tiny = (float)1e-6;
  for (int64_t i = 0; i < n; ++i) {
    float* s1 = st + 6 * i; float* s2 = s1 + 3;
    cur_step[i] += 1;                                                       /* :78 */
    const double* nz = (add_noise && noise) ? noise + 3 * i : NULL;        /* :80,90 */
    float a1 = clipf(act[2 * i], -1.0f, 1.0f) * fmax;                      /* :81-82 */
    float a2 = clipf(act[2 * i + 1], -1.0f, 1.0f) * fmax;
    float d1[3], d2[3];
    pmsm_rhs(s1, 0.0f, 0.0f, NULL, sig, gam, d1);                          /* :88 */
    pmsm_rhs(s2, a1, a2, nz, sig, gam, d2);                                /* :89-90 */
    for (int j = 0; j < 3; ++j) { s1[j] = s1[j] + d1[j] * dt; s2[j] = s2[j] + d2[j] * dt; } /* :92-93 */
    pmsm_rhs(s1, 0.0f, 0.0f, NULL, sig, gam, d1);                          /* :95 */
    pmsm_rhs(s2, a1, a2, nz, sig, gam, d2);                                /* :96-97 */
    float* o = obs + 6 * i;
    for (int j = 0; j < 3; ++j) { o[j] = s1[j] - s2[j]; o[3 + j] = d1[j] - d2[j]; } /* :99-102 */
    float e1 = fabsf(o[0]), e2 = fabsf(o[1]), e3 = fabsf(o[2]);            /* :105-107 */
    float es = (e1 + e2) + e3;                                             /* :108 np.sum */
    float grad = thr - es;                                                 /* :118 */
    adam_step[i] += 1;                                                     /* :121 */
    mt[i] = b1 * mt[i] + c1 * grad;                                        /* :124 */
    vt[i] = b2 * vt[i] + c2 * pmsm_sq(grad, mode);                         /* :127 */
    float mh = mt[i] / pmsm_bias(pd[5], adam_step[i]);                     /* :130 */
    float vh = vt[i] / pmsm_bias(pd[6], adam_step[i]);                     /* :131 */
    lam[i] = lam[i] - (lr * mh) / (sqrtf(vh) + eps);                      /* :135 */
    lam[i] = clipf(lam[i], 0.0f, 0.5f);                                    /* :138 */
    float fp = (pmsm_pow(fabsf(e1) + tiny, alpha, mode) +                  /* :158-160 */
                pmsm_pow(fabsf(e2) + tiny, alpha, mode)) +
               pmsm_pow(fabsf(e3) + tiny, alpha, mode);
    float ap = lam[i] * (pmsm_sq(act[2 * i], mode) + pmsm_sq(act[2 * i + 1], mode)); /* :165 */
    float r = ((-es) - fp) - ap;                                           /* :167 */
    uint8_t te = 0;
    if (es > tterm) { r = -1000.0f; te = 1; }                              /* :174-176 */
    rew[i] = r;
    term[i] = te;
    trunc[i] = cur_step[i] >= max_steps ? 1 : 0;                           /* :179-180 */
  }
}

/* =========================================================================
 * HR -- lorenz_env_try.py:7-179 HRSyncEnv (RK4, dt=0.001)
 * p = {a=1, b=3, c=1, d=5, r=0.006, s=4, I=3.2, x_rest=-1.6, dt=0.001,
 *      scale=50, master_scale=20, action_alpha=0.95, term=70}
 * ========================================================================= */
#define HR_BODY(T, ABS, CUBE_DEV)                                                    \
  static inline T hr_sq_##T(T x, int mode) {                                         \
    return mode == ORC_REF ? (T)pow((double)x, 2.0) : x * x;                         \
  }                                                                                  \
  static inline T hr_cube_##T(T x, int mode) {                                       \
    return mode == ORC_REF ? (T)pow((double)x, 3.0) : CUBE_DEV(x);                   \
  }                                                                                  \
  /* :7-12 hr_derivatives ; a1/a2 enter as f32 values promoted to T */               \
  static inline void hr_rhs_##T(const T* x, T a1, T a2, const T* p, int mode, T* d) {\
    T x2 = hr_sq_##T(x[0], mode), x3 = hr_cube_##T(x[0], mode);                      \
    d[0] = (((x[1] - p[0] * x3) + p[1] * x2) - x[2]) + p[6];                         \
    d[1] = ((p[2] - p[3] * x2) - x[1]) + a1;                                         \
    d[2] = p[4] * (p[5] * (x[0] - p[7]) - x[2]) + a2;                                \
  }                                                                                  \
  static inline void hr_rk4_##T(T* x, T a1, T a2, const T* p, int mode, T h2, T h,   \
                                T h6) {                                              \
    T k1[3], k2[3], k3[3], k4[3], y[3];                                              \
    hr_rhs_##T(x, a1, a2, p, mode, k1);                                /* :101 */    \
    for (int j = 0; j < 3; ++j) y[j] = x[j] + h2 * k1[j];                            \
    hr_rhs_##T(y, a1, a2, p, mode, k2);                                /* :102 */    \
    for (int j = 0; j < 3; ++j) y[j] = x[j] + h2 * k2[j];                            \
    hr_rhs_##T(y, a1, a2, p, mode, k3);                                /* :103 */    \
    for (int j = 0; j < 3; ++j) y[j] = x[j] + h * k3[j];                             \
    hr_rhs_##T(y, a1, a2, p, mode, k4);                                /* :104 */    \
    for (int j = 0; j < 3; ++j)                                        /* :105 */    \
      x[j] = x[j] + h6 * (((k1[j] + (T)2 * k2[j]) + (T)2 * k3[j]) + k4[j]);           \
  }                                                                                  \
  /* reset obs :70-78 (error clipped in reset, unlike step) ; row = [m(3), s(3)] */  \
  void orc_hr_reset_obs_##T(int64_t n, const T* st, T* obs, const double* pd) {      \
    const T sc = (T)pd[9], ms = (T)pd[10];                                           \
    for (int64_t i = 0; i < n; ++i) {                                                \
      const T* m = st + 6 * i; const T* s = m + 3;                                   \
      for (int j = 0; j < 3; ++j) {                                                  \
        obs[6 * i + j] = (T)clipd((double)((m[j] - s[j]) / sc), -1.0, 1.0);          \
        obs[6 * i + 3 + j] = (T)clipd((double)(m[j] / ms), -1.0, 1.0);               \
      }                                                                              \
    }                                                                                \
  }                                                                                  \
  /* step :80-179. fa: float [n,2] filter memory. noise: T [n,3] = N(0, sigma) draws \
   * (:136) or NULL. */                                                              \
  void orc_hr_step_##T(int64_t n, T* st, float* fa, const float* act, const T* noise,\
                       int add_noise, int add_filter, int mode, T* obs, T* rew,      \
                       uint8_t* term, const double* pd) {                            \
    T p[13]; for (int j = 0; j < 13; ++j) p[j] = (T)pd[j];                           \
    /* dt/2, dt, dt/6.0 are python-float expressions (:102-105) */                   \
    const T h2 = (T)(pd[8] / 2), h = (T)pd[8], h6 = (T)(pd[8] / 6.0);                \
    const float fal = (float)pd[11], fa1 = (float)(1.0 - pd[11]);                    \
    for (int64_t i = 0; i < n; ++i) {                                                \
      T* m = st + 6 * i; T* s = m + 3;                                               \
      float f0, f1;                                                                  \
      if (add_filter) {                                                /* :85-86 */  \
        f0 = fa1 * fa[2 * i] + fal * act[2 * i];                                     \
        f1 = fa1 * fa[2 * i + 1] + fal * act[2 * i + 1];                             \
        fa[2 * i] = f0; fa[2 * i + 1] = f1;                                          \
      } else { f0 = act[2 * i]; f1 = act[2 * i + 1]; }                 /* :88 */     \
      float a1 = clipf(f0, -1.0f, 1.0f) * 100.0f;                      /* :92-93 */  \
      float a2 = clipf(f1, -1.0f, 1.0f) * 100.0f;                                    \
      hr_rk4_##T(m, (T)0, (T)0, p, mode, h2, h, h6);                   /* :100-105 */\
      hr_rk4_##T(s, (T)a1, (T)a2, p, mode, h2, h, h6);                 /* :108-113 */\
      if (add_noise && noise)                                          /* :135-137 */\
        for (int j = 0; j < 3; ++j) m[j] = m[j] + noise[3 * i + j] * p[8];           \
      T e[3]; T* o = obs + 6 * i;                                                    \
      for (int j = 0; j < 3; ++j) {                                    /* :150-156 */\
        e[j] = m[j] - s[j];                                                          \
        o[j] = e[j] / p[9];                                                          \
        o[3 + j] = (T)clipd((double)(m[j] / p[10]), -1.0, 1.0);                      \
      }                                                                              \
      float q = act[2 * i] * act[2 * i] + act[2 * i + 1] * act[2 * i + 1];           \
      float pen = 0.05f * q;                                                         \
      T r = (-((ABS(o[0]) + ABS(o[1])) + ABS(o[2]))) - (T)pen;         /* :165 */    \
      uint8_t te = 0;                                                                \
      for (int j = 0; j < 3; ++j) if (ABS(e[j]) > p[12]) te = 1;       /* :174 */    \
      if (te) r = (T)-2000.0;                                                        \
      rew[i] = r; term[i] = te;                                                      \
    }                                                                                \
  }
HR_BODY(double, fabs, cube_dd)
HR_BODY(float, fabsf, cube_ddf)

/* =========================================================================
 * Philox4x32-10 + the device's draw conversions (for checking on-device resets)
 * ========================================================================= */
static inline void philox_round(uint32_t* c, const uint32_t* k) {
  uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
  uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
  uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
  uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
  uint32_t n0 = hi1 ^ c[1] ^ k[0], n2 = hi0 ^ c[3] ^ k[1];
  c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
}
void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  uint32_t c[4] = {ctr[0], ctr[1], ctr[2], ctr[3]}, k[2] = {key[0], key[1]};
  for (int r = 0; r < 10; ++r) {
    philox_round(c, k);
    k[0] += 0x9E3779B9u; k[1] += 0xBB67AE85u;
  }
  memcpy(out, c, sizeof(c));
}

/* word w of the Philox stream (gid, purpose, tick) -- same counter layout as
 * csrc/lz_philox.h */
static uint32_t draw_word(uint64_t seed, uint64_t gid, uint32_t purpose, uint64_t tick, int w) {
  uint32_t ctr[4] = {(uint32_t)gid,
                     (uint32_t)((gid >> 32) & 0xFFu) | ((uint32_t)(w >> 2) << 8) | (purpose << 24),
                     (uint32_t)tick, (uint32_t)(tick >> 32)};
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)}, out[4];
  orc_philox4x32_10(ctr, key, out);
  return out[w & 3];
}
static inline float u01f(uint32_t x) { return (float)(x >> 8) * 5.9604644775390625e-08f; }
static inline double u01d(uint32_t a, uint32_t b) {
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * 1.1102230246251565e-16;
}

/* The on-device reset draws (purpose 1), per system / dtype:
 * init rows as lz_reset's `init` layout.  f32: value j = lo + (hi-lo)*u24(word j);
 * f64 (and PMSM, which the reference draws in f64 then casts): words (2j, 2j+1). */
static void draw_row(int32_t system, int32_t f64, int64_t i, uint64_t g, uint64_t seed,
                     uint64_t tick, int32_t hr_flags, void* out) {
  const uint32_t RESET = 1;
  {
    int nv; double lo, hi;
    switch (system) {
      case 0: nv = 3; lo = -30; hi = 30; break;  /* dynamic.py:37 */
      case 1: nv = 8; lo = 0; hi = 5; break;     /* lorenz_env_transient.py:277-278 */
      case 2: nv = 6; lo = -30; hi = 30; break;  /* lorenz_env_try_pmsm.py:64-65 */
      case 3: nv = 7; lo = -10; hi = 20; break;  /* lorenz_env_try.py:55-57 (+sigma) */
      case 4: nv = 3; lo = -30; hi = 30; break;  /* lorenz_env_transient1.py:43 */
      case 5: nv = 8; lo = 0; hi = 5; break;     /* lorenz_env_transient2.py:141-142 */
      case 6: nv = 6; lo = -10; hi = 10; break;  /* lorenz_env_transient_pmsm.py:45-46 */
      default: {                                 /* lorenz_singlecontrol.py:121 fixed */
        const double x0[3] = {25.0, 1.0, -1.0};
        for (int j = 0; j < 3; ++j) {
          if (f64) ((double*)out)[i * 3 + j] = x0[j];
          else ((float*)out)[i * 3 + j] = (float)x0[j];
        }
        return;
      }
    }
    for (int j = 0; j < nv; ++j) {
      double l = lo, h = hi;
      int hr_sigma = (system == 3 && j == 6);
      if (hr_sigma) { l = 0; h = 2; }  /* :67 */
      if (system == 2) {
        double u = u01d(draw_word(seed, g, RESET, tick, 2 * j), draw_word(seed, g, RESET, tick, 2 * j + 1));
        ((float*)out)[i * nv + j] = (float)(l + (h - l) * u);
      } else if (f64) {
        double u = u01d(draw_word(seed, g, RESET, tick, 2 * j), draw_word(seed, g, RESET, tick, 2 * j + 1));
        double v = l + (h - l) * u;
        if (hr_sigma) v = (hr_flags & 2) ? ((hr_flags & 4) ? 2.0 : v) : 0.0;
        ((double*)out)[i * nv + j] = v;
      } else {
        float u = u01f(draw_word(seed, g, RESET, tick, j));
        float v = (float)l + ((float)h - (float)l) * u;
        if (hr_sigma) v = (hr_flags & 2) ? ((hr_flags & 4) ? 2.0f : v) : 0.0f;
        ((float*)out)[i * nv + j] = v;
      }
    }
  }
}

void orc_reset_draw(int32_t system, int32_t f64, int64_t n, int64_t gid0, uint64_t seed,
                    uint64_t tick, int32_t hr_flags, void* out) {
  for (int64_t i = 0; i < n; ++i) draw_row(system, f64, i, (uint64_t)(gid0 + i), seed, tick, hr_flags, out);
}

/* the same draws for a list of global ids (row r of out = env gids[r]): the auto-reset
 * draws of a step touch only the envs that finished in it */
void orc_reset_draw_idx(int32_t system, int32_t f64, int64_t m, const int64_t* gids, uint64_t seed,
                        uint64_t tick, int32_t hr_flags, void* out) {
  for (int64_t r = 0; r < m; ++r) draw_row(system, f64, r, (uint64_t)gids[r], seed, tick, hr_flags, out);
}

/* the reference's float accumulator done test 't == T' (dynamic.py:85-89,
 * lorenz_env_transient.py:364,369): first step k at which it fires, or -1 */
int32_t orc_t_done_step(double dt, double t_end, int32_t max_k) {
  double t = 0.0;
  for (int32_t k = 1; k <= max_k; ++k) {
    t = t + dt;
    if (t == t_end) return k;
    if (t > t_end) return -1;
  }
  return -1;
}

/* =========================================================================
 * Legacy, unregistered variants (fp64 in the reference).  PMSM-form RHS
 * f = [(-x) + y*z, ((-y) - x*z) + b*z, a*(y - z)]   (python evaluation order)
 * ========================================================================= */
#define LEGACY_BODY(T)                                                               \
  static inline void p3_rhs_##T(const T* v, T a, T b, T* f) {                       \
    f[0] = (-v[0]) + v[1] * v[2];                                                    \
    f[1] = ((-v[1]) - v[0] * v[2]) + b * v[2];                                       \
    f[2] = a * (v[1] - v[2]);                                                        \
  }                                                                                  \
  /* T1 -- lorenz_env_transient1.py:41-104; p = {a, b, -, dt, clip, T_end} */        \
  void orc_t1_reset_obs_##T(int64_t n, const T* st, T* obs, const double* pd) {      \
    for (int64_t i = 0; i < n; ++i) {                                                \
      T f[3]; p3_rhs_##T(st + 3 * i, (T)pd[0], (T)pd[1], f);        /* :44-52 */     \
      for (int j = 0; j < 3; ++j) { obs[6 * i + j] = st[3 * i + j] - (T)0;           \
                                    obs[6 * i + 3 + j] = f[j] - (T)0; }              \
    }                                                                                \
  }                                                                                  \
  void orc_t1_step_##T(int64_t n, T* st, const float* act, T* obs, T* rew,           \
                       const double* pd) {                                           \
    const T a = (T)pd[0], b = (T)pd[1], dt = (T)pd[3]; const float cl = (float)pd[4];\
    for (int64_t i = 0; i < n; ++i) {                                                \
      T* v = st + 3 * i; T f[3];                                                     \
      float u1 = clipf(act[2 * i], -cl, cl), u2 = clipf(act[2 * i + 1], -cl, cl); /* :71-72 */ \
      p3_rhs_##T(v, a, b, f);                                       /* :78-80 */     \
      v[0] = (v[0] + f[0] * dt) + (T)u1;                            /* :84 */        \
      v[1] = (v[1] + f[1] * dt) + (T)u2;                            /* :85 */        \
      v[2] = v[2] + f[2] * dt;                                      /* :86 */        \
      p3_rhs_##T(v, a, b, f);                                       /* :88-91 */     \
      T* o = obs + 6 * i;                                                            \
      for (int j = 0; j < 3; ++j) { o[j] = v[j] - (T)0; o[3 + j] = f[j] - (T)0; }    \
      rew[i] = -((((T)0 + (T)fabs(o[0])) + (T)fabs(o[1])) + (T)fabs(o[2])); /* :98 */\
    }                                                                                \
  }                                                                                  \
  /* T2 -- lorenz_env_transient2.py:139-240;                                        \
   * p = {a, b, c, dt, clip, T_end, d, h, gain, damping}; st row [m(4), s(4)] */     \
  static inline void t2_rhs_##T(const T* x, const double* pd, T* f) {                \
    const T q = ((T)2 * x[3]) * x[3];                                                \
    f[0] = (T)pd[0] * (q * (x[1] - x[0]) + (T)pd[6] * x[0]);                         \
    f[1] = (T)pd[1] * (q * (x[0] - x[1]) - x[2]);                                    \
    f[2] = (T)pd[2] * (x[1] - (T)pd[7] * x[2]);                                      \
    f[3] = (x[1] - x[0]) - (T)pd[9] * x[3];                                          \
  }                                                                                  \
  void orc_t2_reset_obs_##T(int64_t n, const T* st, T* obs, const double* pd) {      \
    for (int64_t i = 0; i < n; ++i) {                                                \
      const T* m = st + 8 * i; const T* s = m + 4; T fm[4], fs[4];                   \
      t2_rhs_##T(m, pd, fm); t2_rhs_##T(s, pd, fs);                 /* :143-160 */   \
      for (int j = 0; j < 4; ++j) { obs[8 * i + j] = m[j] - s[j];                    \
                                    obs[8 * i + 4 + j] = fm[j] - fs[j]; }            \
    }                                                                                \
  }                                                                                  \
  void orc_t2_step_##T(int64_t n, T* st, const float* act, T* obs, T* rew,           \
                       uint8_t* done, const double* pd) {                            \
    const T dt = (T)pd[3]; const float cl = (float)pd[4], g = (float)pd[8];         \
    for (int64_t i = 0; i < n; ++i) {                                                \
      T* m = st + 8 * i; T* s = m + 4; T f[4];                                       \
      float g1 = clipf(act[3 * i], -cl, cl) * g;                    /* :182-184 */   \
      float g2 = clipf(act[3 * i + 1], -cl, cl) * g;                /* u*100: f32 */ \
      float g3 = clipf(act[3 * i + 2], -cl, cl) * g;                                 \
      t2_rhs_##T(m, pd, f);                                         /* :189-192 */   \
      for (int j = 0; j < 4; ++j) m[j] = m[j] + f[j] * dt;          /* :193-196 */   \
      t2_rhs_##T(s, pd, f);                                         /* :210-213 */   \
      f[0] = f[0] + (T)g1; f[1] = f[1] + (T)g2; f[3] = f[3] + (T)g3;                 \
      for (int j = 0; j < 4; ++j) s[j] = s[j] + f[j] * dt;          /* :214-217 */   \
      T fm[4], fs[4]; t2_rhs_##T(m, pd, fm); t2_rhs_##T(s, pd, fs);  /* :198-224 */  \
      T* o = obs + 8 * i;                                                            \
      for (int j = 0; j < 4; ++j) { o[j] = m[j] - s[j]; o[4 + j] = fm[j] - fs[j]; }  \
      T S = (((((T)0 + (T)fabs(o[0])) + (T)fabs(o[1])) + (T)fabs(o[2])) +            \
             (T)fabs(o[3]));                                                         \
      /* :229 -S - S**(1/3): glibc pow as NumPy; the GPU's OCML pow may differ by */ \
      /* an ulp, so the device reward is checked within a relative tolerance */       \
      T r = (-S) - (T)pow((double)S, 1.0 / 3.0);                                     \
      rew[i] = r;                                                                    \
      done[i] = r < (T)-1e6 ? 1 : 0;                                /* :235 */       \
    }                                                                                \
  }                                                                                  \
  /* TP -- lorenz_env_transient_pmsm.py:43-133; p = {a, b, gain, dt, clip, T_end,   \
   * noise std}; st row [m(3), s(3)]; noise double [n,3] (the N(0,3) draw) or NULL */\
  void orc_tp_reset_obs_##T(int64_t n, const T* st, T* obs, const double* pd) {      \
    for (int64_t i = 0; i < n; ++i) {                                                \
      const T* m = st + 6 * i; const T* s = m + 3; T fm[3], fs[3];                   \
      p3_rhs_##T(m, (T)pd[0], (T)pd[1], fm); p3_rhs_##T(s, (T)pd[0], (T)pd[1], fs);  \
      for (int j = 0; j < 3; ++j) { obs[6 * i + j] = m[j] - s[j];    /* :47-65 */    \
                                    obs[6 * i + 3 + j] = fm[j] - fs[j]; }            \
    }                                                                                \
  }                                                                                  \
  void orc_tp_step_##T(int64_t n, T* st, const float* act, const double* noise,      \
                       T* obs, T* rew, uint8_t* done, const double* pd) {            \
    const T a = (T)pd[0], b = (T)pd[1], dt = (T)pd[3];                               \
    const float g = (float)pd[2], cl = (float)pd[4];                                 \
    for (int64_t i = 0; i < n; ++i) {                                                \
      T* m = st + 6 * i; T* s = m + 3; T f[3];                                       \
      float g1 = clipf(act[2 * i], -cl, cl) * g;                    /* :78-79 */     \
      float g2 = clipf(act[2 * i + 1], -cl, cl) * g;                /* u*20: f32 */  \
      p3_rhs_##T(m, a, b, f);                                       /* :87-89 */     \
      for (int j = 0; j < 3; ++j) m[j] = m[j] + f[j] * dt;          /* :97-99 */     \
      p3_rhs_##T(s, a, b, f);                                       /* :91-93 */     \
      f[0] = f[0] + (T)g1; f[1] = f[1] + (T)g2;                                      \
      if (noise) for (int j = 0; j < 3; ++j) f[j] = f[j] + (T)noise[3 * i + j];      \
      for (int j = 0; j < 3; ++j) s[j] = s[j] + f[j] * dt;          /* :101-103 */   \
      T fm[3], fs[3]; p3_rhs_##T(m, a, b, fm); p3_rhs_##T(s, a, b, fs); /* :108-120 */\
      T* o = obs + 6 * i;                                                            \
      for (int j = 0; j < 3; ++j) { o[j] = m[j] - s[j]; o[3 + j] = fm[j] - fs[j]; }  \
      T S = (((T)0 + (T)fabs(o[0])) + (T)fabs(o[1])) + (T)fabs(o[2]);                \
      T r = (-S) - (T)pow((double)S, 0.1);                          /* :122 */     \
      rew[i] = r;                                                                    \
      done[i] = r < (T)-1e6 ? 1 : 0;                                /* :129 */       \
    }                                                                                \
  }                                                                                  \
  /* SC -- lorenz_singlecontrol.py:120-172; p = {a, b, -, dt, clip, T_end, std, x0..}*/\
  void orc_sc_step_##T(int64_t n, T* st, const double* noise, T* obs, T* rew,        \
                       const double* pd) {                                           \
    const T a = (T)pd[0], b = (T)pd[1], dt = (T)pd[3];                               \
    for (int64_t i = 0; i < n; ++i) {                                                \
      T* v = st + 3 * i; T f[3];                                                     \
      p3_rhs_##T(v, a, b, f);                                       /* :150-152 */   \
      if (noise) for (int j = 0; j < 3; ++j) f[j] = f[j] + (T)noise[3 * i + j];      \
      for (int j = 0; j < 3; ++j) v[j] = v[j] + f[j] * dt;          /* :154-156 */   \
      p3_rhs_##T(v, a, b, f);                                       /* :158-161 */   \
      T* o = obs + 6 * i;                                                            \
      for (int j = 0; j < 3; ++j) { o[j] = v[j] - (T)0; o[3 + j] = f[j] - (T)0; }    \
      rew[i] = -((((T)0 + (T)fabs(o[0])) + (T)fabs(o[1])) + (T)fabs(o[2])); /* :165 */\
    }                                                                                \
  }
LEGACY_BODY(double)
LEGACY_BODY(float)

/* =========================================================================
 * f3 / f2: the float32 MlpPolicy -- stable-baselines3 2.7.1 ActorCriticPolicy
 * ("MlpPolicy", net_arch pi=[H,H] vf=[H,H], activation Tanh; code/lorenz_pmsm/
 * train.py:150-176, code/gym_try.py:106-116), whose forward SB3 runs in torch
 * float32:  latent = tanh(W2 tanh(W1 x + b1) + b2);  mean = action_net(latent_pi);
 * value = value_net(latent_vf).  Restated in the operation order of the fused
 * kernel's float32 variant (gym-lorenz_amd/csrc/lz_policy.hip mlp_f32 -- this is the
 * DEV-mode restatement the GPU is checked against bit for bit; its agreement with the
 * torch forward SB3 computes is checked separately, tests/test_policy_f32_host.py):
 *   hidden unit u: acc = b[u]; acc = fmaf(w[u][k], x[k], acc) over the inputs k in the
 *     order (k-step s, lane half h): layer 1 k = 2s + h, layer 2 k = 32 ti +
 *     row(g, h) for ti = 0..3, g = 0..15, h = 0, 1; then orc_tanh_tab(acc);
 *   head row r: per half h an fmaf chain from +0 over k = 32 t + row(g, h), t = 0..3,
 *     g = 0..15; out = (part0 + part1) + b[r].
 * Nets narrower than 128 are zero-padded (exactly what the packer does).
 * ========================================================================= */
/* lz_policy.hip tanh_tab: sign(x) p_k(|x| - k/8), k = floor(8|x|) (segments of width
 * 1/8 over [0, 9)), p_k of degree 5 by Horner in fmaf; 1 for |x| >= 9.  The coefficients
 * (tools/tanh_table.py) are the 72 x 8 floats the packer puts into the blob, scaled by
 * 8^-j there (the kernel's Horner runs in u = 8 t: the same bits, see lz_policy.hip). */
static const float orc_tanh_coef[72 * 8] = {
    0.0f, 0x1.0000000000000p+0f, 0x1.c0e2b20000000p-22f, -0x1.555bea0000000p-2f, 0x1.06810a0000000p-11f, 0x1.0a051c0000000p-3f, 0.0f, 0.0f,
    0x1.fd59920000000p-4f, 0x1.f815240000000p-1f, -0x1.f574200000000p-4f, -0x1.40a4860000000p-2f, 0x1.51c1e40000000p-4f, 0x1.8de4da0000000p-4f, 0.0f, 0.0f,
    0x1.f597ea0000000p-3f, 0x1.e1499e0000000p-1f, -0x1.d77de40000000p-3f, -0x1.075b220000000p-2f, 0x1.258ef60000000p-3f, 0x1.784c640000000p-5f, 0.0f, 0.0f,
    0x1.6ef53e0000000p-2f, 0x1.be3fb80000000p-1f, -0x1.3fd3c00000000p-2f, -0x1.6e322a0000000p-3f, 0x1.5f12440000000p-3f, -0x1.76ae540000000p-8f, 0.0f, 0.0f,
    0x1.d9353e0000000p-2f, 0x1.92a9460000000p-1f, -0x1.7426460000000p-2f, -0x1.8264340000000p-4f, 0x1.559cc60000000p-3f, -0x1.634c080000000p-5f, 0.0f, 0.0f,
    0x1.1bf47e0000000p-1f, 0x1.6284c20000000p-1f, -0x1.893b040000000p-2f, -0x1.24e9760000000p-6f, 0x1.1c00ce0000000p-3f, -0x1.f82a900000000p-5f, 0.0f, 0.0f,
    0x1.45323e0000000p-1f, 0x1.3173b20000000p-1f, -0x1.8403fc0000000p-2f, 0x1.56a9400000000p-5f, 0x1.977e660000000p-4f, -0x1.00bcee0000000p-4f, 0.0f, 0.0f,
    0x1.6866500000000p-1f, 0x1.02500a0000000p-1f, -0x1.6ba8380000000p-2f, 0x1.4f4f300000000p-4f, 0x1.eb1db60000000p-5f, -0x1.b2d63e0000000p-5f, 0.0f, 0.0f,
    0x1.85efac0000000p-1f, 0x1.ae0dc20000000p-2f, -0x1.4787420000000p-2f, 0x1.a8a1900000000p-4f, 0x1.b57c4e0000000p-6f, -0x1.407aea0000000p-5f, 0.0f, 0.0f,
    0x1.9e5cb60000000p-1f, 0x1.6150040000000p-2f, -0x1.1df01e0000000p-2f, 0x1.c6cada0000000p-4f, 0x1.336ae80000000p-9f, -0x1.9e7f2e0000000p-6f, 0.0f, 0.0f,
    0x1.b2523c0000000p-1f, 0x1.1f25140000000p-2f, -0x1.e729ca0000000p-3f, 0x1.bbd41a0000000p-4f, -0x1.b407840000000p-7f, -0x1.c879220000000p-7f, 0.0f, 0.0f,
    0x1.c278a60000000p-1f, 0x1.cea7460000000p-3f, -0x1.970e820000000p-3f, 0x1.97f8360000000p-4f, -0x1.6603360000000p-6f, -0x1.7519460000000p-8f, 0.0f, 0.0f,
    0x1.cf6f980000000p-1f, 0x1.7216540000000p-3f, -0x1.4efc260000000p-3f, 0x1.67c6940000000p-4f, -0x1.9e1e4a0000000p-6f, -0x1.603d9c0000000p-12f, 0.0f, 0.0f,
    0x1.d9c6fa0000000p-1f, 0x1.265e340000000p-3f, -0x1.1064960000000p-3f, 0x1.33e9b00000000p-4f, -0x1.9ff4a80000000p-6f, 0x1.6a701c0000000p-9f, 0.0f, 0.0f,
    0x1.e1fbfa0000000p-1f, 0x1.d22ca20000000p-4f, -0x1.b6d87e0000000p-4f, 0x1.01bee00000000p-4f, -0x1.8292880000000p-6f, 0x1.1880380000000p-8f, 0.0f, 0.0f,
    0x1.e8789e0000000p-1f, 0x1.6fcfa60000000p-4f, -0x1.5ee8980000000p-4f, 0x1.a85d6c0000000p-5f, -0x1.56176c0000000p-6f, 0x1.38ecea0000000p-8f, 0.0f, 0.0f,
    0x1.ed95060000000p-1f, 0x1.2162c20000000p-4f, -0x1.16f9c80000000p-4f, 0x1.58f26e0000000p-5f, -0x1.24d6160000000p-6f, 0x1.3214000000000p-8f, 0.0f, 0.0f,
    0x1.f1994e0000000p-1f, 0x1.c65b1c0000000p-5f, -0x1.b993580000000p-5f, 0x1.15af780000000p-5f, -0x1.e9aec00000000p-7f, 0x1.16bf740000000p-8f, 0.0f, 0.0f,
    0x1.f4bfd60000000p-1f, 0x1.64108a0000000p-5f, -0x1.5c3d680000000p-5f, 0x1.bbc1f20000000p-6f, -0x1.9277020000000p-7f, 0x1.e5ac020000000p-9f, 0.0f, 0.0f,
    0x1.f737760000000p-1f, 0x1.16a7fc0000000p-5f, -0x1.11e0100000000p-5f, 0x1.608ac80000000p-6f, -0x1.46997e0000000p-7f, 0x1.9ab50e0000000p-9f, 0.0f, 0.0f,
    0x1.f925820000000p-1f, 0x1.b3afe20000000p-6f, -0x1.adda9c0000000p-6f, 0x1.16d5660000000p-6f, -0x1.0683400000000p-7f, 0x1.54263a0000000p-9f, 0.0f, 0.0f,
    0x1.faa7940000000p-1f, 0x1.5452000000000p-6f, -0x1.50c42c0000000p-6f, 0x1.b78e260000000p-7f, -0x1.a2f4000000000p-8f, 0x1.1581420000000p-9f, 0.0f, 0.0f,
    0x1.fbd50a0000000p-1f, 0x1.09a7a60000000p-6f, -0x1.077dd60000000p-6f, 0x1.5988ec0000000p-7f, -0x1.4c77120000000p-8f, 0x1.bfccd00000000p-10f, 0.0f, 0.0f,
    0x1.fcc04c0000000p-1f, 0x1.9e87d00000000p-7f, -0x1.9be6180000000p-7f, 0x1.0f10080000000p-7f, -0x1.06b6a00000000p-8f, 0x1.6650e60000000p-10f, 0.0f, 0.0f,
    0x1.fd77d20000000p-1f, 0x1.434a500000000p-7f, -0x1.41b0c00000000p-7f, 0x1.a8990a0000000p-8f, -0x1.9dd60e0000000p-9f, 0x1.1cecac0000000p-10f, 0.0f, 0.0f,
    0x1.fe06ec0000000p-1f, 0x1.f81bd80000000p-8f, -0x1.f62a160000000p-8f, 0x1.4c220c0000000p-8f, -0x1.451fa40000000p-9f, 0x1.c2fa040000000p-11f, 0.0f, 0.0f,
    0x1.fe767a0000000p-1f, 0x1.88ef660000000p-8f, -0x1.87c1060000000p-8f, 0x1.038d260000000p-8f, -0x1.fddc240000000p-10f, 0x1.639ac00000000p-11f, 0.0f, 0.0f,
    0x1.fecd6c0000000p-1f, 0x1.3238b60000000p-8f, -0x1.3181100000000p-8f, 0x1.955ae60000000p-9f, -0x1.8f2d7a0000000p-10f, 0x1.179dc40000000p-11f, 0.0f, 0.0f,
    0x1.ff112c0000000p-1f, 0x1.dd37d00000000p-9f, -0x1.dc58c00000000p-9f, 0x1.3c587c0000000p-9f, -0x1.3828040000000p-10f, 0x1.b6c8d60000000p-12f, 0.0f, 0.0f,
    0x1.ff45f60000000p-1f, 0x1.73cec00000000p-9f, -0x1.73474a0000000p-9f, 0x1.ed89380000000p-10f, -0x1.e7c4640000000p-11f, 0x1.57b4ac0000000p-12f, 0.0f, 0.0f,
    0x1.ff6f180000000p-1f, 0x1.21a7ae0000000p-9f, -0x1.21556a0000000p-9f, 0x1.80d9700000000p-10f, -0x1.7cd1160000000p-11f, 0x1.0ce2680000000p-12f, 0.0f, 0.0f,
    0x1.ff8f220000000p-1f, 0x1.c347040000000p-10f, -0x1.c2e3180000000p-10f, 0x1.2c03a80000000p-10f, -0x1.2927280000000p-11f, 0x1.a4466a0000000p-13f, 0.0f, 0.0f,
    0x1.ffa8180000000p-1f, 0x1.5f85ac0000000p-10f, -0x1.5f48f80000000p-10f, 0x1.d3a8a20000000p-11f, -0x1.cf8a840000000p-12f, 0x1.4832700000000p-13f, 0.0f, 0.0f,
    0x1.ffbb880000000p-1f, 0x1.11ce6e0000000p-10f, -0x1.11a98a0000000p-10f, 0x1.6c6dd60000000p-11f, -0x1.696d9a0000000p-12f, 0x1.0023620000000p-13f, 0.0f, 0.0f,
    0x1.ffcaac0000000p-1f, 0x1.aa87ce0000000p-11f, -0x1.aa5af40000000p-11f, 0x1.1bf2e20000000p-11f, -0x1.19bcb40000000p-12f, 0x1.8f9f0c0000000p-14f, 0.0f, 0.0f,
    0x1.ffd6780000000p-1f, 0x1.4c36520000000p-11f, -0x1.4c1b0a0000000p-11f, 0x1.ba702e0000000p-12f, -0x1.b725680000000p-13f, 0x1.37a1340000000p-14f, 0.0f, 0.0f,
    0x1.ffdfa80000000p-1f, 0x1.02bec80000000p-11f, -0x1.02ae2c0000000p-11f, 0x1.58aaf00000000p-12f, -0x1.5632180000000p-13f, 0x1.e5df3a0000000p-15f, 0.0f, 0.0f,
    0x1.ffe6ce0000000p-1f, 0x1.930b440000000p-12f, -0x1.92f7060000000p-12f, 0x1.0c7c6a0000000p-12f, -0x1.0a9da60000000p-13f, 0x1.7aad8a0000000p-15f, 0.0f, 0.0f,
    0x1.ffec620000000p-1f, 0x1.39e7820000000p-12f, -0x1.39db2a0000000p-12f, 0x1.a243ee0000000p-13f, -0x1.9f6bf40000000p-14f, 0x1.271a400000000p-15f, 0.0f, 0.0f,
    0x1.fff0b80000000p-1f, 0x1.e8f43c0000000p-13f, -0x1.e8e5260000000p-13f, 0x1.45c9dc0000000p-13f, -0x1.439da40000000p-14f, 0x1.cbe1040000000p-16f, 0.0f, 0.0f,
    0x1.fff41a0000000p-1f, 0x1.7ccec00000000p-13f, -0x1.7cc5840000000p-13f, 0x1.fb80320000000p-14f, -0x1.f829880000000p-15f, 0x1.6640d60000000p-16f, 0.0f, 0.0f,
    0x1.fff6bc0000000p-1f, 0x1.2894480000000p-13f, -0x1.288e9e0000000p-13f, 0x1.8b46180000000p-14f, -0x1.88b4ba0000000p-15f, 0x1.171a0c0000000p-16f, 0.0f, 0.0f,
    0x1.fff8c80000000p-1f, 0x1.cdf5a20000000p-14f, -0x1.cdeea60000000p-14f, 0x1.33dbd40000000p-14f, -0x1.31e0360000000p-15f, 0x1.b2ce400000000p-17f, 0.0f, 0.0f,
    0x1.fffa600000000p-1f, 0x1.67c7600000000p-14f, -0x1.67c30e0000000p-14f, 0x1.df8b600000000p-15f, -0x1.dc79c40000000p-16f, 0x1.52aa580000000p-17f, 0.0f, 0.0f,
    0x1.fffba00000000p-1f, 0x1.1832dc0000000p-14f, -0x1.18302e0000000p-14f, 0x1.757be60000000p-15f, -0x1.731cf80000000p-16f, 0x1.07d4f00000000p-17f, 0.0f, 0.0f,
    0x1.fffc980000000p-1f, 0x1.b470ec0000000p-15f, -0x1.b46d940000000p-15f, 0x1.22e0e40000000p-15f, -0x1.210ba60000000p-16f, 0x1.9b105c0000000p-18f, 0.0f, 0.0f,
    0x1.fffd580000000p-1f, 0x1.53e7140000000p-15f, -0x1.53e4f80000000p-15f, 0x1.c5151c0000000p-16f, -0x1.c239000000000p-17f, 0x1.400d220000000p-18f, 0.0f, 0.0f,
    0x1.fffdee0000000p-1f, 0x1.08b7b60000000p-15f, -0x1.08b6600000000p-15f, 0x1.60de040000000p-16f, -0x1.5ea5540000000p-17f, 0x1.f28c3a0000000p-19f, 0.0f, 0.0f,
    0x1.fffe640000000p-1f, 0x1.9c53760000000p-16f, -0x1.9c51c00000000p-16f, 0x1.12d13a0000000p-16f, -0x1.1118080000000p-17f, 0x1.8454820000000p-19f, 0.0f, 0.0f,
    0x1.fffebe0000000p-1f, 0x1.411ee60000000p-16f, -0x1.411dca0000000p-16f, 0x1.ac0f620000000p-17f, -0x1.a95f840000000p-18f, 0x1.2e64980000000p-19f, 0.0f, 0.0f,
    0x1.ffff060000000p-1f, 0x1.f42dde0000000p-17f, -0x1.f42c680000000p-17f, 0x1.4d60680000000p-17f, -0x1.4b4a280000000p-18f, 0x1.d70dd80000000p-20f, 0.0f, 0.0f,
    0x1.ffff3e0000000p-1f, 0x1.858a640000000p-17f, -0x1.85896a0000000p-17f, 0x1.03a2b60000000p-17f, -0x1.02031a0000000p-18f, 0x1.6ee1380000000p-20f, 0.0f, 0.0f,
    0x1.ffff680000000p-1f, 0x1.2f5ffa0000000p-17f, -0x1.2f5f520000000p-17f, 0x1.9469a00000000p-18f, -0x1.91ea5c0000000p-19f, 0x1.1df0ce0000000p-20f, 0.0f, 0.0f,
    0x1.ffff8a0000000p-1f, 0x1.d889a60000000p-18f, -0x1.d888be0000000p-18f, 0x1.3af4e80000000p-18f, -0x1.38fc400000000p-19f, 0x1.bcf95a0000000p-21f, 0.0f, 0.0f,
    0x1.ffffa40000000p-1f, 0x1.7003540000000p-18f, -0x1.7002b40000000p-18f, 0x1.ea946c0000000p-19f, -0x1.e789c40000000p-20f, 0x1.5ac44a0000000p-21f, 0.0f, 0.0f,
    0x1.ffffb80000000p-1f, 0x1.1e9be60000000p-18f, -0x1.1e9b7c0000000p-18f, 0x1.7e11e00000000p-19f, -0x1.7bcc880000000p-20f, 0x1.0ec8be0000000p-21f, 0.0f, 0.0f,
    0x1.ffffc80000000p-1f, 0x1.be6c3e0000000p-19f, -0x1.be6b9c0000000p-19f, 0x1.298dc20000000p-19f, -0x1.27ba2a0000000p-20f, 0x1.a4eaee0000000p-22f, 0.0f, 0.0f,
    0x1.ffffd40000000p-1f, 0x1.5bacb00000000p-19f, -0x1.5bac320000000p-19f, 0x1.cf76bc0000000p-20f, -0x1.cc7ce60000000p-21f, 0x1.46e1680000000p-22f, 0.0f, 0.0f,
    0x1.ffffde0000000p-1f, 0x1.0ec4f20000000p-19f, -0x1.0ec4900000000p-19f, 0x1.68f1bc0000000p-20f, -0x1.6696900000000p-21f, 0x1.fc8a4a0000000p-23f, 0.0f, 0.0f,
    0x1.ffffe60000000p-1f, 0x1.a5c0340000000p-20f, -0x1.a5bfa80000000p-20f, 0x1.191ab80000000p-20f, -0x1.1742f20000000p-21f, 0x1.8bd10e0000000p-23f, 0.0f, 0.0f,
    0x1.ffffec0000000p-1f, 0x1.4875bc0000000p-20f, -0x1.48755e0000000p-20f, 0x1.b5dbf00000000p-21f, -0x1.b3351a0000000p-22f, 0x1.35f54e0000000p-23f, 0.0f, 0.0f,
    0x1.fffff00000000p-1f, 0x1.ff9c180000000p-21f, -0x1.ff9ba20000000p-21f, 0x1.5503ba0000000p-21f, -0x1.531eac0000000p-22f, 0x1.e539840000000p-24f, 0.0f, 0.0f,
    0x1.fffff40000000p-1f, 0x1.8e712c0000000p-21f, -0x1.8e70b00000000p-21f, 0x1.09921a0000000p-21f, -0x1.07e4e20000000p-22f, 0x1.771bba0000000p-24f, 0.0f, 0.0f,
    0x1.fffff60000000p-1f, 0x1.364e9a0000000p-21f, -0x1.364e0a0000000p-21f, 0x1.9d9b540000000p-22f, -0x1.99fd1a0000000p-23f, 0x1.1c3ce60000000p-24f, 0.0f, 0.0f,
    0x1.fffff80000000p-1f, 0x1.e355b40000000p-22f, -0x1.e3555a0000000p-22f, 0x1.422b420000000p-22f, -0x1.4059560000000p-23f, 0x1.c98be20000000p-25f, 0.0f, 0.0f,
    0x1.fffffa0000000p-1f, 0x1.786be80000000p-22f, -0x1.786bb40000000p-22f, 0x1.f5d4f60000000p-23f, -0x1.f3812a0000000p-24f, 0x1.6887700000000p-25f, 0.0f, 0.0f,
    0x1.fffffc0000000p-1f, 0x1.25284a0000000p-22f, -0x1.2528040000000p-22f, 0x1.86cd8c0000000p-23f, -0x1.8485200000000p-24f, 0x1.1556120000000p-25f, 0.0f, 0.0f,
    0x1.fffffc0000000p-1f, 0x1.c89f580000000p-23f, -0x1.c89f6a0000000p-23f, 0x1.306a580000000p-23f, -0x1.2fd5d00000000p-24f, 0x1.c2272c0000000p-26f, 0.0f, 0.0f,
    0x1.fffffe0000000p-1f, 0x1.639e2c0000000p-23f, -0x1.639d480000000p-23f, 0x1.d9f5440000000p-24f, -0x1.d516000000000p-25f, 0x1.40da540000000p-26f, 0.0f, 0.0f,
    0x1.fffffe0000000p-1f, 0x1.14f49e0000000p-23f, -0x1.14f4b20000000p-23f, 0x1.7144f40000000p-24f, -0x1.705de60000000p-25f, 0x1.0f59800000000p-26f, 0.0f, 0.0f,
    0x1.fffffe0000000p-1f, 0x1.af62e00000000p-24f, -0x1.af60b00000000p-24f, 0x1.1f5d940000000p-24f, -0x1.1a7e740000000p-25f, 0x1.69ea620000000p-27f, 0.0f, 0.0f,
    0x1.fffffe0000000p-1f, 0x1.4ff6c80000000p-24f, -0x1.4ff5fe0000000p-24f, 0x1.bfc5e20000000p-25f, -0x1.bb37d80000000p-26f, 0x1.2ea2320000000p-27f, 0.0f, 0.0f,
};

float orc_tanh_tab(float x) {
  const float ax = fabsf(x);
  int k = ax < 9.0f ? (int)(ax * 8.0f) : 71;  /* NaN / inf / >= 9: any segment, overridden */
  if (k > 71) k = 71;
  const float* c = orc_tanh_coef + 8 * k;
  const float t = fmaf((float)k, -0.125f, ax);
  float y = fmaf(c[5], t, c[4]);
  y = fmaf(y, t, c[3]);
  y = fmaf(y, t, c[2]);
  y = fmaf(y, t, c[1]);
  y = fmaf(y, t, c[0]);
  y = ax >= 9.0f ? 1.0f : y;  /* NaN: ax >= 9 is false and t (so y) is already NaN */
  return copysignf(y, x);
}

static inline int pol_row(int g, int h) { return (g & 3) + 8 * (g >> 2) + 4 * h; }

static void mlp_f32_one(int O, int H, int R, const float* x, const float* w1, const float* b1,
                        const float* w2, const float* b2, const float* w3, const float* b3,
                        float* out) {
  float a1[128], a2[128];
  for (int u = 0; u < 128; ++u) {
    float acc = u < H ? b1[u] : 0.0f;
    for (int s = 0; s < (O + 1) / 2; ++s)
      for (int h = 0; h < 2; ++h) {
        const int k = 2 * s + h;
        const float w = (u < H && k < O) ? w1[u * O + k] : 0.0f;
        acc = fmaf(w, k < O ? x[k] : 0.0f, acc);
      }
    a1[u] = orc_tanh_tab(acc);
  }
  for (int u = 0; u < 128; ++u) {
    float acc = u < H ? b2[u] : 0.0f;
    for (int ti = 0; ti < 4; ++ti)
      for (int g = 0; g < 16; ++g)
        for (int h = 0; h < 2; ++h) {
          const int k = 32 * ti + pol_row(g, h);
          acc = fmaf((u < H && k < H) ? w2[u * H + k] : 0.0f, a1[k], acc);
        }
    a2[u] = orc_tanh_tab(acc);
  }
  for (int r = 0; r < R; ++r) {
    float part[2];
    for (int h = 0; h < 2; ++h) {
      float acc = 0.0f;
      for (int t = 0; t < 4; ++t)
        for (int g = 0; g < 16; ++g) {
          const int k = 32 * t + pol_row(g, h);
          acc = fmaf(k < H ? w3[r * H + k] : 0.0f, a2[k], acc);
        }
      part[h] = acc;
    }
    out[r] = (part[0] + part[1]) + b3[r];
  }
}

/* x [n, O] (the normalised observation the policy sees) -> mean [n, A], value [n] */
void orc_mlp_f32(int64_t n, int O, int A, int H, const float* x, const float* pi_w1,
                 const float* pi_b1, const float* pi_w2, const float* pi_b2, const float* vf_w1,
                 const float* vf_b1, const float* vf_w2, const float* vf_b2, const float* act_w,
                 const float* act_b, const float* val_w, const float* val_b, float* mean,
                 float* value) {
  for (int64_t i = 0; i < n; ++i) {
    mlp_f32_one(O, H, A, x + i * O, pi_w1, pi_b1, pi_w2, pi_b2, act_w, act_b, mean + i * A);
    mlp_f32_one(O, H, 1, x + i * O, vf_w1, vf_b1, vf_w2, vf_b2, val_w, val_b, value + i);
  }
}

void orc_tanh_tab_v(int64_t n, const float* x, float* out) {
  for (int64_t i = 0; i < n; ++i) out[i] = orc_tanh_tab(x[i]);
}

/* ---- SB3-exact VecNormalize of the fused float32 rollout (lz_policy_step_f32).
 * The batch moments of x [n, O] float32 in the device's fixed order (gym-lorenz_amd/
 * csrc/lz_internal.h PStepArgs; k_policy_step_f32 / k_obs_tile_moments + k_vn_tile_update):
 * per tile of 32 envs (0.0 past n) a 32-lane butterfly v_l += v_(l ^ m), m = 16 .. 1, of
 * (double)x (sums) or (double)x * (double)x (squares); per column, accumulator t < 256
 * sums the partials of tiles t, t + 256, ... from 0.0 in order; then the tree
 * a[t] += a[t + m], m = 128 .. 1.  tot[2 O] = (sums[O], sums of squares[O]).
 * SB3 2.7.1 RunningMeanStd.update (common/running_mean_std.py) takes np.mean / np.var
 * of the float32 rows instead; the statistics built on these sums follow
 * update_from_moments (the caller, oracle/__init__.py vn_rms_update). */
void orc_vn_tile_totals(const float* x, int64_t n, int O, double* tot) {
  const int64_t ntiles = (n + 31) / 32;
  for (int c = 0; c < 2 * O; ++c) {
    const int j = c % O, sq = c >= O;
    double acc[256];
    for (int t = 0; t < 256; ++t) acc[t] = 0.0;
    for (int64_t tile = 0; tile < ntiles; ++tile) {
      double v[32], w[32];
      for (int l = 0; l < 32; ++l) {
        const int64_t i = tile * 32 + l;
        const double d = i < n ? (double)x[i * O + j] : 0.0;
        v[l] = sq ? d * d : d;
      }
      for (int m = 16; m >= 1; m >>= 1) {
        for (int l = 0; l < 32; ++l) w[l] = v[l] + v[l ^ m];
        for (int l = 0; l < 32; ++l) v[l] = w[l];
      }
      acc[tile % 256] += v[0];
    }
    for (int m = 128; m >= 1; m >>= 1)
      for (int t = 0; t < m; ++t) acc[t] += acc[t + m];
    tot[c] = acc[0];
  }
}

/* ---- f3: the attention actor-critics at SB3's precision (float32), in the fused
 * kernel's operation order (gym-lorenz_amd/csrc/lz_policy.hip attn16_extract /
 * attn16_net; every product-sum a k-ordered fmaf chain -- what v_mfma_f32_16x16x4_f32
 * computes: k-step s of a 16-unit tile takes input 4G + s from lane group G = 0..3, in
 * that order).  code/train.py:52-95 AttentionFeaturesExtractor: x = relu(fc1(obs))
 * viewed as 8 tokens of 16; nn.MultiheadAttention(16, 4 heads) self-attention (q scaled
 * by 1/sqrt(4)); post_attention_fc(128 -> 64) + ReLU; code/lorenz_filter/train.py:54-103
 * adds x_seq = layer_norm(x_seq + attn_output) before post_attention_fc.  Then the pi /
 * vf [128, 128] Tanh nets on the 64 features (tanh_tab) and the two heads. */

/* exp(x) for the softmax (x <= 0, or NaN): rint(x log2 e) range reduction, a degree-6
 * Taylor polynomial in fmaf, ldexp; 0 below -86 (the result stays a normal number). */
float orc_exp_f32(float x) {
  if (x != x) return x;
  if (x < -86.0f) return 0.0f;
  const float k = rintf(x * 1.44269504088896341f);
  float r = fmaf(k, -0.693145751953125f, x);
  r = fmaf(k, -1.42860682030941723e-6f, r);
  float p = fmaf(1.38888892e-3f, r, 8.33333377e-3f);
  p = fmaf(p, r, 4.16666679e-2f);
  p = fmaf(p, r, 1.66666672e-1f);
  p = fmaf(p, r, 0.5f);
  p = fmaf(p, r, 1.0f);
  p = fmaf(p, r, 1.0f);
  return ldexpf(p, (int)k);
}

typedef struct {
  const float *fc1_w, *fc1_b, *in_w, *in_b, *out_w, *out_b, *post_w, *post_b, *ln_w, *ln_b;
  const void* post8;  /* non-NULL: post_attention_fc as i8x4 products (orc_attn_i8x4) */
} orc_attn_ext;

/* post_attention_fc of the i8x4 extractor: the 128 attention outputs of all 8 tokens ->
 * the 64 features (defined with the i8x4 section below) */
static void i8x_post(const void* post8, const float* uall, const float* post_b, float* feat);

/* acc + sum_{s < 4} sum_{G < 4} w[4G + s] * v[4G + s]: one 16-dim k order (4 k-steps) */
static inline float dot16(float acc, const float* w, const float* v) {
  for (int s = 0; s < 4; ++s)
    for (int G = 0; G < 4; ++G) acc = fmaf(w[4 * G + s], v[4 * G + s], acc);
  return acc;
}

/* (p0 + p1) + (p2 + p3), p_G = ((v[4G] + v[4G+1]) + v[4G+2]) + v[4G+3] (sq: the squares,
 * v[4G]^2 then fmaf) -- the kernel's per-lane-group partials and two lane swaps */
static inline float sum16(const float* v, int sq) {
  float p[4];
  for (int G = 0; G < 4; ++G) {
    const float* z = v + 4 * G;
    if (sq) {
      p[G] = z[0] * z[0];
      for (int d = 1; d < 4; ++d) p[G] = fmaf(z[d], z[d], p[G]);
    } else {
      p[G] = ((z[0] + z[1]) + z[2]) + z[3];
    }
  }
  return (p[0] + p[1]) + (p[2] + p[3]);
}

/* x [in_dim] -> feat [64] */
static void attn_ext_one(const orc_attn_ext* e, int in_dim, const float* x, float* feat) {
  float tok[128], kk[8][16], vv[8][16];
  const int KS = (in_dim + 3) / 4;
  for (int u = 0; u < 128; ++u) {
    float acc = e->fc1_b[u];
    for (int s = 0; s < KS; ++s)
      for (int G = 0; G < 4; ++G) {
        const int k = 4 * s + G;
        acc = fmaf(k < in_dim ? e->fc1_w[u * in_dim + k] : 0.0f, k < in_dim ? x[k] : 0.0f, acc);
      }
    tok[u] = acc < 0.0f ? 0.0f : acc;
  }
  for (int T = 0; T < 8; ++T)
    for (int o = 0; o < 16; ++o) {
      kk[T][o] = dot16(e->in_b[16 + o], e->in_w + (16 + o) * 16, tok + 16 * T);
      vv[T][o] = dot16(e->in_b[32 + o], e->in_w + (32 + o) * 16, tok + 16 * T);
    }
  float post[64], uall[128];
  for (int f = 0; f < 64; ++f) post[f] = e->post_b[f];
  for (int i = 0; i < 8; ++i) {
    float q[16], att[16], y[16], u[16];
    for (int o = 0; o < 16; ++o) {  /* 1/sqrt(head dim) = 0.5 folded (exact) */
      float w[16];
      for (int d = 0; d < 16; ++d) w[d] = 0.5f * e->in_w[o * 16 + d];
      q[o] = dot16(0.5f * e->in_b[o], w, tok + 16 * i);
    }
    for (int hd = 0; hd < 4; ++hd) {
      float sc[8], ex[8], m, sum = 0.0f, r;
      for (int j = 0; j < 8; ++j) {
        float t = q[4 * hd] * kk[j][4 * hd];
        for (int c = 1; c < 4; ++c) t = fmaf(q[4 * hd + c], kk[j][4 * hd + c], t);
        sc[j] = t;
      }
      m = sc[0];
      for (int j = 1; j < 8; ++j) m = (m != m || m >= sc[j]) ? m : sc[j];
      for (int j = 0; j < 8; ++j) {
        ex[j] = orc_exp_f32(sc[j] - m);
        sum = j == 0 ? ex[0] : sum + ex[j];
      }
      r = 1.0f / sum;
      for (int c = 0; c < 4; ++c) {
        float acc = (ex[0] * r) * vv[0][4 * hd + c];
        for (int j = 1; j < 8; ++j) acc = fmaf(ex[j] * r, vv[j][4 * hd + c], acc);
        att[4 * hd + c] = acc;
      }
    }
    for (int o = 0; o < 16; ++o) y[o] = dot16(e->out_b[o], e->out_w + o * 16, att);
    if (e->ln_w) {  /* LayerNorm(16) of (token + attention), eps 1e-5, biased variance */
      float z[16], mean, rstd;
      for (int d = 0; d < 16; ++d) z[d] = y[d] + tok[16 * i + d];
      mean = sum16(z, 0) * 0.0625f;
      for (int d = 0; d < 16; ++d) z[d] = z[d] - mean;
      rstd = 1.0f / sqrtf(sum16(z, 1) * 0.0625f + 1e-5f);
      for (int d = 0; d < 16; ++d) u[d] = fmaf(z[d] * rstd, e->ln_w[d], e->ln_b[d]);
    } else {
      for (int d = 0; d < 16; ++d) u[d] = y[d];
    }
    for (int d = 0; d < 16; ++d) uall[16 * i + d] = u[d];
    if (!e->post8)
      for (int f = 0; f < 64; ++f) post[f] = dot16(post[f], e->post_w + f * 128 + 16 * i, u);
  }
  if (e->post8) {
    i8x_post(e->post8, uall, e->post_b, feat);
    return;
  }
  for (int f = 0; f < 64; ++f) feat[f] = post[f] < 0.0f ? 0.0f : post[f];
}

/* one [128, 128] Tanh net + head on the 64 features (the kernel's attn16_net order):
 * layer k orders 16-dim blocks f (then s, G) in turn; the head is a per-lane-group fmaf
 * chain over units 16t + 4G + r (t, then r) from +0, the groups combined as sum16 */
static void attn_net_one(int R, const float* feat, const float* w1, const float* b1, const float* w2,
                         const float* b2, const float* w3, const float* b3, float* out) {
  float a1[128], a2[128];
  for (int u = 0; u < 128; ++u) {
    float acc = b1[u];
    for (int f = 0; f < 4; ++f) acc = dot16(acc, w1 + u * 64 + 16 * f, feat + 16 * f);
    a1[u] = orc_tanh_tab(acc);
  }
  for (int u = 0; u < 128; ++u) {
    float acc = b2[u];
    for (int q = 0; q < 8; ++q) acc = dot16(acc, w2 + u * 128 + 16 * q, a1 + 16 * q);
    a2[u] = orc_tanh_tab(acc);
  }
  for (int r = 0; r < R; ++r) {
    float part[4];
    for (int G = 0; G < 4; ++G) {
      float acc = 0.0f;
      for (int t = 0; t < 8; ++t)
        for (int c = 0; c < 4; ++c) {
          const int k = 16 * t + 4 * G + c;
          acc = fmaf(w3[r * 128 + k], a2[k], acc);
        }
      part[G] = acc;
    }
    out[r] = ((part[0] + part[1]) + (part[2] + part[3])) + b3[r];
  }
}

/* x [n, in_dim] (the policy input: normalised obs, or the VecFrameStack) -> mean [n, A],
 * value [n], feat [n, 64] (nullable).  ln_w == NULL: code/train.py's extractor. */
void orc_attn_f32(int64_t n, int in_dim, int A, const float* x, const float* fc1_w, const float* fc1_b,
                  const float* in_w, const float* in_b, const float* out_w, const float* out_b,
                  const float* post_w, const float* post_b, const float* ln_w, const float* ln_b,
                  const float* pi_w1, const float* pi_b1, const float* pi_w2, const float* pi_b2,
                  const float* vf_w1, const float* vf_b1, const float* vf_w2, const float* vf_b2,
                  const float* act_w, const float* act_b, const float* val_w, const float* val_b,
                  float* mean, float* value, float* feat_out) {
  const orc_attn_ext e = {fc1_w, fc1_b, in_w, in_b, out_w, out_b, post_w, post_b, ln_w, ln_b, NULL};
  for (int64_t i = 0; i < n; ++i) {
    float feat[64];
    attn_ext_one(&e, in_dim, x + i * in_dim, feat);
    if (feat_out)
      for (int f = 0; f < 64; ++f) feat_out[i * 64 + f] = feat[f];
    attn_net_one(A, feat, pi_w1, pi_b1, pi_w2, pi_b2, act_w, act_b, mean + i * A);
    attn_net_one(1, feat, vf_w1, vf_b1, vf_w2, vf_b2, val_w, val_b, value + i);
  }
}

/* ---- f3 opt-in precision "i8x4" (lz_attn_policy_pack_i8x4 / lz_attn_ln_policy_pack_i8x4,
 * gym-lorenz_amd/csrc/lz_policy.hip attn16_net<kI8>): the two wide layers of each pi / vf
 * net (64 -> 128 and 128 -> 128) as EXACT fixed-point dot products on the int8 MFMA
 * (v_mfma_i32_16x16x64_i8, 16 x the f32 MFMA's multiply rate), everything else as in
 * orc_attn_f32.  Restated here, operation for operation:
 *   fixed point:  V = (int32)rintf(ldexpf(v, q)), |V| <= 2^28 -- q = 28 for the layer-2
 *                 inputs (tanh outputs, |v| <= 1); q = 28 - e, m = fract * 2^e (frexpf) of
 *                 the env's largest feature for the layer-1 inputs (ReLU outputs >= 0); per
 *                 weight row q_r = 28 - e_r of the row's largest |w|;
 *   digits:       U = V + 0x808080, d_k = (int8)(byte k of U ^ 0x80) for k < 3 and d_3 =
 *                 (int8)(U >> 24): V = sum_k d_k 2^(8k), |d_3| <= 16 (balanced digits);
 *   products:     the 10 digit pairs (i, j) with i + j >= 3 (weight digit i, input digit
 *                 j), summed per level s = i + j in int32 (exact: no order, no rounding):
 *                 L6 .. L3; the dropped levels (i + j <= 2) weigh < 2^-24 of the leading;
 *   recombine:    hi = L6 * 256 + L5 (< 2^24: exact in float), lo = L4 * 256 + L3 (int32),
 *                 y = ldexpf(fmaf((float)hi, 65536, (float)lo), 24 - q_r - q) + bias;
 *   non-finite:   a NaN / inf feature makes every output of the env NaN (the weights are
 *                 finite: the packer refuses others).
 * Precision: the products are exact and one rounding (plus lo's) ends each sum -- closer
 * to the exact dot product than float32's k-ordered fmaf chain. */
static inline int32_t i8x_fixed(float v, int q) { return (int32_t)rintf(ldexpf(v, q)); }

static inline void i8x_digits(int32_t V, int8_t d[4]) {
  const int32_t U = (int32_t)((uint32_t)V + 0x808080u);
  d[0] = (int8_t)((U & 0xff) ^ 0x80);
  d[1] = (int8_t)(((U >> 8) & 0xff) ^ 0x80);
  d[2] = (int8_t)(((U >> 16) & 0xff) ^ 0x80);
  d[3] = (int8_t)(U >> 24);
}

/* q of a weight row / of an input vector with largest magnitude m: 28 - e, m = f 2^e */
static inline int i8x_q(float m) {
  int e = 0;
  (void)frexpf(m, &e);
  return 28 - e;
}

int32_t orc_i8x_row_q(const float* w, int32_t K) {
  float m = 0.0f;
  for (int k = 0; k < K; ++k) m = fmaxf(m, fabsf(w[k]));
  return i8x_q(m);
}

/* digits of n values at one q: d [n][4] (for tests) */
void orc_i8x_digits(int64_t n, const float* v, int32_t q, int8_t* d) {
  for (int64_t i = 0; i < n; ++i) i8x_digits(i8x_fixed(v[i], q), d + 4 * i);
}

/* sum_k W_k V_k over K digit rows, recombined and scaled by 2^sh (no bias) */
float orc_i8x_dot(int32_t K, const int8_t* wd, const int8_t* vd, int32_t sh) {
  int32_t L[7] = {0, 0, 0, 0, 0, 0, 0};
  for (int k = 0; k < K; ++k)
    for (int i = 0; i < 4; ++i)
      for (int j = 3 - i; j < 4; ++j) L[i + j] += (int32_t)wd[4 * k + i] * (int32_t)vd[4 * k + j];
  const int32_t hi = L[6] * 256 + L[5];
  const int32_t lo = L[4] * 256 + L[3];
  return ldexpf(fmaf((float)hi, 65536.0f, (float)lo), sh);
}

/* a wide layer's weight digits and row q's, made once per call */
typedef struct {
  int8_t d1[128 * 64 * 4], d2[128 * 128 * 4];
  int32_t q1[128], q2[128];
} i8x_net;

static void i8x_prep(i8x_net* t, const float* w1, const float* w2) {
  for (int u = 0; u < 128; ++u) {
    t->q1[u] = orc_i8x_row_q(w1 + u * 64, 64);
    for (int k = 0; k < 64; ++k) i8x_digits(i8x_fixed(w1[u * 64 + k], t->q1[u]), t->d1 + 4 * (u * 64 + k));
    t->q2[u] = orc_i8x_row_q(w2 + u * 128, 128);
    for (int k = 0; k < 128; ++k)
      i8x_digits(i8x_fixed(w2[u * 128 + k], t->q2[u]), t->d2 + 4 * (u * 128 + k));
  }
}

static void attn_net_one_i8x(int R, const float* feat, const i8x_net* t, const float* b1, const float* b2,
                             const float* w3, const float* b3, float* out) {
  float m = 0.0f;
  for (int f = 0; f < 64; ++f) m = (m != m || feat[f] != feat[f]) ? NAN : fmaxf(m, feat[f]);
  if (!(m <= 3.40282347e38f)) {
    for (int r = 0; r < R; ++r) out[r] = NAN;
    return;
  }
  const int qa = i8x_q(m);
  int8_t fd[64 * 4], ad[128 * 4];
  for (int f = 0; f < 64; ++f) i8x_digits(i8x_fixed(feat[f], qa), fd + 4 * f);
  float a2[128];
  for (int u = 0; u < 128; ++u) {
    const float y = orc_i8x_dot(64, t->d1 + 4 * 64 * u, fd, 24 - t->q1[u] - qa) + b1[u];
    i8x_digits(i8x_fixed(orc_tanh_tab(y), 28), ad + 4 * u);
  }
  for (int u = 0; u < 128; ++u)
    a2[u] = orc_tanh_tab(orc_i8x_dot(128, t->d2 + 4 * 128 * u, ad, 24 - t->q2[u] - 28) + b2[u]);
  for (int r = 0; r < R; ++r) {
    float part[4];
    for (int G = 0; G < 4; ++G) {
      float acc = 0.0f;
      for (int tt = 0; tt < 8; ++tt)
        for (int c = 0; c < 4; ++c) {
          const int k = 16 * tt + 4 * G + c;
          acc = fmaf(w3[r * 128 + k], a2[k], acc);
        }
      part[G] = acc;
    }
    out[r] = ((part[0] + part[1]) + (part[2] + part[3])) + b3[r];
  }
}

/* post_attention_fc in i8x4: the env's 128 attention outputs (any sign) at the scale of
 * their largest magnitude, the 64 rows at theirs; a NaN / inf output -> NaN features */
typedef struct {
  int8_t d[64 * 128 * 4];
  int32_t q[64];
} i8x_postw;

static void i8x_post(const void* post8, const float* uall, const float* post_b, float* feat) {
  const i8x_postw* pw = (const i8x_postw*)post8;
  float m = 0.0f;
  for (int k = 0; k < 128; ++k)
    m = (m != m || uall[k] != uall[k]) ? NAN : fmaxf(m, fabsf(uall[k]));
  if (!(m <= 3.40282347e38f)) {
    for (int f = 0; f < 64; ++f) feat[f] = NAN;
    return;
  }
  const int qu = i8x_q(m);
  int8_t ud[128 * 4];
  for (int k = 0; k < 128; ++k) i8x_digits(i8x_fixed(uall[k], qu), ud + 4 * k);
  for (int f = 0; f < 64; ++f) {
    const float y = orc_i8x_dot(128, pw->d + 4 * 128 * f, ud, 24 - pw->q[f] - qu) + post_b[f];
    feat[f] = y < 0.0f ? 0.0f : y;
  }
}

/* orc_attn_f32 with the i8x4 nets and post_attention_fc */
void orc_attn_i8x4(int64_t n, int in_dim, int A, const float* x, const float* fc1_w, const float* fc1_b,
                   const float* in_w, const float* in_b, const float* out_w, const float* out_b,
                   const float* post_w, const float* post_b, const float* ln_w, const float* ln_b,
                   const float* pi_w1, const float* pi_b1, const float* pi_w2, const float* pi_b2,
                   const float* vf_w1, const float* vf_b1, const float* vf_w2, const float* vf_b2,
                   const float* act_w, const float* act_b, const float* val_w, const float* val_b,
                   float* mean, float* value, float* feat_out) {
  static i8x_net pi, vf;  /* (not reentrant: test infrastructure) */
  static i8x_postw pw;
  i8x_prep(&pi, pi_w1, pi_w2);
  i8x_prep(&vf, vf_w1, vf_w2);
  for (int f = 0; f < 64; ++f) {
    pw.q[f] = orc_i8x_row_q(post_w + f * 128, 128);
    for (int k = 0; k < 128; ++k) i8x_digits(i8x_fixed(post_w[f * 128 + k], pw.q[f]), pw.d + 4 * (f * 128 + k));
  }
  const orc_attn_ext e = {fc1_w, fc1_b, in_w, in_b, out_w, out_b, post_w, post_b, ln_w, ln_b, &pw};
  for (int64_t i = 0; i < n; ++i) {
    float feat[64];
    attn_ext_one(&e, in_dim, x + i * in_dim, feat);
    if (feat_out)
      for (int f = 0; f < 64; ++f) feat_out[i * 64 + f] = feat[f];
    attn_net_one_i8x(A, feat, &pi, pi_b1, pi_b2, act_w, act_b, mean + i * A);
    attn_net_one_i8x(1, feat, &vf, vf_b1, vf_b2, val_w, val_b, value + i);
  }
}

/* orc_mlp_f32 with layer 2 as exact i8x4 products (lz_policy_pack_i8x4, LZ_POLICY_I8X4;
 * lz_policy.hip mlp_i8_tail): layer 1, tanh_tab and the heads as mlp_f32_one; layer 2's
 * inputs (tanh outputs, |a| <= 1) at q = 28, its 128 (zero-padded) rows at their own q;
 * y[u] = orc_i8x_dot(row u, a, 24 - q2[u] - 28) + b2[u] -> tanh_tab.  A NaN among an env's
 * layer-1 outputs makes that env's outputs NaN. */
static void mlp_i8x_one(int O, int H, int R, const float* x, const float* w1, const float* b1,
                        const int8_t* d2, const int32_t* q2, const float* b2, const float* w3,
                        const float* b3, float* out) {
  float a1[128], a2[128];
  int nan = 0;
  for (int u = 0; u < 128; ++u) {
    float acc = u < H ? b1[u] : 0.0f;
    for (int s = 0; s < (O + 1) / 2; ++s)
      for (int h = 0; h < 2; ++h) {
        const int k = 2 * s + h;
        const float w = (u < H && k < O) ? w1[u * O + k] : 0.0f;
        acc = fmaf(w, k < O ? x[k] : 0.0f, acc);
      }
    a1[u] = orc_tanh_tab(acc);
    nan |= a1[u] != a1[u];
  }
  if (nan) {
    for (int r = 0; r < R; ++r) out[r] = NAN;
    return;
  }
  int8_t ad[128 * 4];
  for (int k = 0; k < 128; ++k) i8x_digits(i8x_fixed(a1[k], 28), ad + 4 * k);
  for (int u = 0; u < 128; ++u)
    a2[u] = orc_tanh_tab(orc_i8x_dot(128, d2 + 4 * 128 * u, ad, 24 - q2[u] - 28) + (u < H ? b2[u] : 0.0f));
  for (int r = 0; r < R; ++r) {
    float part[2];
    for (int h = 0; h < 2; ++h) {
      float acc = 0.0f;
      for (int t = 0; t < 4; ++t)
        for (int g = 0; g < 16; ++g) {
          const int k = 32 * t + pol_row(g, h);
          acc = fmaf(k < H ? w3[r * H + k] : 0.0f, a2[k], acc);
        }
      part[h] = acc;
    }
    out[r] = (part[0] + part[1]) + b3[r];
  }
}

/* the 128 x 128 zero-padded layer-2 digits and row q's of an [H, H] weight */
static void i8x_prep_w2(int H, const float* w2, int8_t* d2, int32_t* q2) {
  float row[128];
  for (int u = 0; u < 128; ++u) {
    for (int k = 0; k < 128; ++k) row[k] = (u < H && k < H) ? w2[u * H + k] : 0.0f;
    q2[u] = orc_i8x_row_q(row, 128);
    for (int k = 0; k < 128; ++k) i8x_digits(i8x_fixed(row[k], q2[u]), d2 + 4 * (u * 128 + k));
  }
}

void orc_mlp_i8x4(int64_t n, int O, int A, int H, const float* x, const float* pi_w1,
                  const float* pi_b1, const float* pi_w2, const float* pi_b2, const float* vf_w1,
                  const float* vf_b1, const float* vf_w2, const float* vf_b2, const float* act_w,
                  const float* act_b, const float* val_w, const float* val_b, float* mean,
                  float* value) {
  static int8_t pd[128 * 128 * 4], vd[128 * 128 * 4];  /* (not reentrant: test infrastructure) */
  int32_t pq[128], vq[128];
  i8x_prep_w2(H, pi_w2, pd, pq);
  i8x_prep_w2(H, vf_w2, vd, vq);
  for (int64_t i = 0; i < n; ++i) {
    mlp_i8x_one(O, H, A, x + i * O, pi_w1, pi_b1, pd, pq, pi_b2, act_w, act_b, mean + i * A);
    mlp_i8x_one(O, H, 1, x + i * O, vf_w1, vf_b1, vd, vq, vf_b2, val_w, val_b, value + i);
  }
}
