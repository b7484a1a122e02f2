/* Drives libgym_lorenz_amd.so through include/lorenz_env.h from plain C (no Python,
 * no torch): the way a non-Python host (cgo / JNI / N-API / a C++ trainer) binds the
 * drop-in boundary.  LORENZ3 fp32, N envs with on-device resets, K steps of random
 * actions; every step's observations / rewards / dones are checked bit for bit
 * against the CPU oracle (oracle/lz_oracle.c, test infrastructure) fed the same
 * initial states and actions.  Also PMSM via lz_rollout against K oracle steps.
 * Build: gcc -O2 -I include -I /opt/rocm/include -D__HIP_PLATFORM_AMD__ abi_smoke.c
 *        -L<lib dirs> -lgym_lorenz_amd -llz_oracle -lamdhip64 -lm
 * Exit status 0 = parity, 1 = mismatch, 2 = API error. */
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "lorenz_env.h"

/* oracle (liblz_oracle.so) */
void orc_l3_step_float(int64_t n, float* st, const float* act, float* obs, float* rew, const double* p);
void orc_pmsm_step(int64_t n, float* st, float* lam, float* mt, float* vt, int32_t* adam_step,
                   int32_t* cur_step, const float* act, const double* noise, int add_noise,
                   float alpha, int mode, float* obs, float* rew, uint8_t* term, uint8_t* trunc,
                   const double* pd);

#define CHECK(x)                                                                   \
  do {                                                                             \
    lz_status s_ = (x);                                                            \
    if (s_ != LZ_OK) {                                                             \
      fprintf(stderr, "%s failed: %d %s\n", #x, (int)s_, lz_last_error());         \
      return 2;                                                                    \
    }                                                                              \
  } while (0)
#define HCHECK(x)                                                                  \
  do {                                                                             \
    if ((x) != hipSuccess) { fprintf(stderr, "%s failed\n", #x); return 2; }       \
  } while (0)

static uint32_t rng = 12345u;
static float urand(void) { rng = rng * 1664525u + 1013904223u; return (float)(rng >> 8) / 16777216.0f * 2.0f - 1.0f; }

static int same_bits(const float* a, const float* b, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    if (isnan(a[i]) && isnan(b[i])) continue;
    if (memcmp(&a[i], &b[i], 4) != 0) return 0;
  }
  return 1;
}

static int run_l3(int64_t n, int K) {
  lz_config cfg;
  CHECK(lz_config_init(&cfg, LZ_SYS_LORENZ3));
  cfg.num_envs = n;
  cfg.seed = 42;
  cfg.flags = LZ_FLAG_AUTORESET;
  lz_handle* h = NULL;
  CHECK(lz_create(&cfg, &h));
  lz_info info;
  CHECK(lz_get_info(h, &info));
  if (info.obs_dim != 6 || info.action_dim != 3 || info.bytes_per_env_step != 65) return 1;
  float *d_obs, *d_rew, *d_act, *d_x;
  uint8_t* d_done;
  HCHECK(hipMalloc((void**)&d_obs, n * 6 * 4));
  HCHECK(hipMalloc((void**)&d_rew, n * 4));
  HCHECK(hipMalloc((void**)&d_act, n * 3 * 4));
  HCHECK(hipMalloc((void**)&d_x, n * 4));
  HCHECK(hipMalloc((void**)&d_done, n));
  CHECK(lz_reset(h, NULL, NULL, d_obs));
  float* st = malloc(n * 3 * 4);
  float* x = malloc(n * 4);
  for (int j = 0; j < 3; ++j) {  /* the device-drawn initial states, plane by plane */
    CHECK(lz_get_state(h, LZ_L3_X + j, d_x, NULL, 0));
    CHECK(lz_sync(h));
    HCHECK(hipMemcpy(x, d_x, n * 4, hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < n; ++i) st[i * 3 + j] = x[i];
  }
  float *act = malloc(n * 3 * 4), *obs = malloc(n * 6 * 4), *rew = malloc(n * 4);
  float *o_ref = malloc(n * 6 * 4), *r_ref = malloc(n * 4);
  uint8_t* done = malloc(n);
  for (int k = 0; k < K; ++k) {
    for (int64_t i = 0; i < n * 3; ++i) act[i] = urand();
    HCHECK(hipMemcpy(d_act, act, n * 3 * 4, hipMemcpyHostToDevice));
    CHECK(lz_step(h, d_act, NULL, d_obs, d_rew, d_done, NULL, NULL, NULL));
    CHECK(lz_sync(h));
    HCHECK(hipMemcpy(obs, d_obs, n * 6 * 4, hipMemcpyDeviceToHost));
    HCHECK(hipMemcpy(rew, d_rew, n * 4, hipMemcpyDeviceToHost));
    HCHECK(hipMemcpy(done, d_done, n, hipMemcpyDeviceToHost));
    orc_l3_step_float(n, st, act, o_ref, r_ref, cfg.params);
    if (!same_bits(obs, o_ref, n * 6) || !same_bits(rew, r_ref, n)) {
      fprintf(stderr, "LORENZ3 mismatch at step %d\n", k);
      return 1;
    }
    for (int64_t i = 0; i < n; ++i)
      if (done[i]) { fprintf(stderr, "unexpected done\n"); return 1; }
  }
  printf("LORENZ3 fp32: %lld envs x %d lz_step calls bit-exact vs the oracle\n", (long long)n, K);
  hipFree(d_obs); hipFree(d_rew); hipFree(d_act); hipFree(d_x); hipFree(d_done);
  free(st); free(x); free(act); free(obs); free(rew); free(o_ref); free(r_ref); free(done);
  return lz_destroy(h) == LZ_OK ? 0 : 2;
}

static int run_pmsm_rollout(int64_t n, int K) {
  lz_config cfg;
  CHECK(lz_config_init(&cfg, LZ_SYS_PMSM));
  cfg.num_envs = n;
  cfg.seed = 7;
  lz_handle* h = NULL;
  CHECK(lz_create(&cfg, &h));
  float* init = malloc(n * 6 * 4);
  for (int64_t i = 0; i < n * 6; ++i) init[i] = 30.0f * urand();
  float *d_init, *d_act, *d_obs, *d_rew;
  uint8_t* d_done;
  HCHECK(hipMalloc((void**)&d_init, n * 6 * 4));
  HCHECK(hipMalloc((void**)&d_act, (size_t)K * n * 2 * 4));
  HCHECK(hipMalloc((void**)&d_obs, (size_t)K * n * 6 * 4));
  HCHECK(hipMalloc((void**)&d_rew, (size_t)K * n * 4));
  HCHECK(hipMalloc((void**)&d_done, (size_t)K * n));
  HCHECK(hipMemcpy(d_init, init, n * 6 * 4, hipMemcpyHostToDevice));
  CHECK(lz_reset(h, NULL, d_init, NULL));
  float* act = malloc((size_t)K * n * 2 * 4);
  for (int64_t i = 0; i < (int64_t)K * n * 2; ++i) act[i] = 1.2f * urand();
  HCHECK(hipMemcpy(d_act, act, (size_t)K * n * 2 * 4, hipMemcpyHostToDevice));
  CHECK(lz_rollout(h, K, d_act, d_obs, d_rew, d_done, NULL, NULL, 0, NULL));
  CHECK(lz_sync(h));
  float *obs = malloc((size_t)K * n * 6 * 4), *rew = malloc((size_t)K * n * 4);
  HCHECK(hipMemcpy(obs, d_obs, (size_t)K * n * 6 * 4, hipMemcpyDeviceToHost));
  HCHECK(hipMemcpy(rew, d_rew, (size_t)K * n * 4, hipMemcpyDeviceToHost));
  float *lam = calloc(n, 4), *mt = calloc(n, 4), *vt = calloc(n, 4);
  int32_t *adam = calloc(n, 4), *cur = calloc(n, 4);
  float *o_ref = malloc(n * 6 * 4), *r_ref = malloc(n * 4);
  uint8_t *te = malloc(n), *tr = malloc(n);
  for (int k = 0; k < K; ++k) {
    orc_pmsm_step(n, init, lam, mt, vt, adam, cur, act + (size_t)k * n * 2, NULL, 0, cfg.alpha,
                  1 /* ORC_DEV */, o_ref, r_ref, te, tr, cfg.params);
    if (!same_bits(obs + (size_t)k * n * 6, o_ref, n * 6) || !same_bits(rew + (size_t)k * n, r_ref, n)) {
      fprintf(stderr, "PMSM rollout mismatch at step %d\n", k);
      return 1;
    }
  }
  printf("PMSM: %lld envs x %d-step lz_rollout bit-exact vs the oracle\n", (long long)n, K);
  hipFree(d_init); hipFree(d_act); hipFree(d_obs); hipFree(d_rew); hipFree(d_done);
  return lz_destroy(h) == LZ_OK ? 0 : 2;
}

int main(void) {
  if (lz_abi_version() != LZ_ABI_VERSION) return 2;
  int r = run_l3(5003, 40);
  if (r) return r;
  return run_pmsm_rollout(3001, 64);
}
