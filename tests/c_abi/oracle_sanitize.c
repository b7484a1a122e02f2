/* Runs every function of the CPU oracle (oracle/lz_oracle.c, test infrastructure) on
 * exactly-sized heap buffers under AddressSanitizer + UndefinedBehaviorSanitizer
 * ("host CPU reference built with -fsanitize=address,undefined in tests"):
 * any out-of-bounds index or UB in the restatement aborts with a report.
 * Built and run by tests/test_sanitizers.py:
 *   gcc -O1 -g -fsanitize=address,undefined -fno-sanitize-recover=all -ffp-contract=off
 *       oracle/lz_oracle.c tests/c_abi/oracle_sanitize.c -lm */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define P(name) extern void name
P(orc_l3_reset_obs_double)(int64_t, const double*, double*, const double*);
P(orc_l3_step_double)(int64_t, double*, const double*, double*, double*, const double*);
P(orc_l3_step_float)(int64_t, float*, const float*, float*, float*, const double*);
P(orc_l4_reset_obs_float)(int64_t, const float*, float*, const double*);
P(orc_l4_step_float)(int64_t, float*, float*, float*, uint8_t*, const double*);
P(orc_pmsm_reset_obs)(int64_t, const float*, float*, const double*);
P(orc_pmsm_step)(int64_t, float*, float*, float*, float*, int32_t*, int32_t*, const float*,
                 const double*, int, float, int, float*, float*, uint8_t*, uint8_t*, const double*);
P(orc_hr_reset_obs_double)(int64_t, const double*, double*, const double*);
P(orc_hr_step_double)(int64_t, double*, float*, const float*, const double*, int, int, int,
                      double*, double*, uint8_t*, const double*);
P(orc_philox4x32_10)(const uint32_t*, const uint32_t*, uint32_t*);
P(orc_reset_draw)(int32_t, int32_t, int64_t, int64_t, uint64_t, uint64_t, int32_t, void*);
extern int32_t orc_t_done_step(double, double, int32_t);
P(orc_t1_reset_obs_double)(int64_t, const double*, double*, const double*);
P(orc_t1_step_double)(int64_t, double*, const float*, double*, double*, const double*);
P(orc_t2_reset_obs_double)(int64_t, const double*, double*, const double*);
P(orc_t2_step_double)(int64_t, double*, const float*, double*, double*, uint8_t*, const double*);
P(orc_tp_reset_obs_float)(int64_t, const float*, float*, const double*);
P(orc_tp_step_float)(int64_t, float*, const float*, const double*, float*, float*, uint8_t*,
                     const double*);
P(orc_sc_step_double)(int64_t, double*, const double*, double*, double*, const double*);

static void* xa(size_t bytes) {  /* exact-size buffer: ASan flags any overrun */
  void* p = malloc(bytes);
  memset(p, 0, bytes);
  return p;
}
static double prm[16] = {10, 28, 8.0 / 3, 0.01, 500, 10};

int main(void) {
  const int64_t n = 37;
  const int K = 50;
  /* reset draws for every system and dtype into exact-size buffers */
  const int ni[8] = {3, 8, 6, 7, 3, 8, 6, 3};
  for (int sys = 0; sys < 8; ++sys)
    for (int f64 = 0; f64 < 2; ++f64) {
      void* out = xa((size_t)n * ni[sys] * (f64 && sys != 2 ? 8 : 4));
      orc_reset_draw(sys, f64, n, 5, 42, 3, 6, out);
      free(out);
    }
  uint32_t c[4] = {1, 2, 3, 4}, k[2] = {5, 6}, o[4];
  orc_philox4x32_10(c, k, o);
  if (orc_t_done_step(0.01, 10.0, 5000) != -1) return 1;

  double* st = xa(n * 8 * 8);
  double* obs = xa(n * 8 * 8);
  double* rew = xa(n * 8);
  float* act = xa(n * 3 * 4);
  float* fst = xa(n * 8 * 4);
  float* fobs = xa(n * 8 * 4);
  float* frew = xa(n * 4);
  uint8_t* done = xa(n);
  uint8_t* done2 = xa(n);
  double* noise = xa(n * 3 * 8);
  for (int64_t i = 0; i < n * 3; ++i) { act[i] = (float)((i % 7) - 3) * 0.3f; noise[i] = 0.1 * (double)(i % 5); }
  for (int64_t i = 0; i < n * 8; ++i) { st[i] = 1.0 + 0.01 * (double)i; fst[i] = (float)st[i]; }

  orc_l3_reset_obs_double(n, st, obs, prm);
  for (int s = 0; s < K; ++s) orc_l3_step_double(n, st, (const double*)noise, obs, rew, prm);
  for (int s = 0; s < K; ++s) orc_l3_step_float(n, fst, act, fobs, frew, prm);
  double p4[16] = {10, 8.0 / 3, 28, 0.001, 2, 5};
  orc_l4_reset_obs_float(n, fst, fobs, p4);
  for (int s = 0; s < K; ++s) orc_l4_step_float(n, fst, fobs, frew, done, p4);

  double pp[16] = {5.46, 20, 0.001, 50, 0.001, 0.9, 0.999, 1e-8, 5, 2000, 1000};
  float *lam = xa(n * 4), *mt = xa(n * 4), *vt = xa(n * 4);
  int32_t *adam = xa(n * 4), *cur = xa(n * 4);
  orc_pmsm_reset_obs(n, fst, fobs, pp);
  for (int s = 0; s < K; ++s)
    orc_pmsm_step(n, fst, lam, mt, vt, adam, cur, act, noise, s & 1, 0.25f, s & 1, fobs, frew, done,
                  done2, pp);

  double ph[16] = {1, 3, 1, 5, 0.006, 4, 3.2, -1.6, 0.001, 50, 20, 0.95, 70};
  float* fa = xa(n * 2 * 4);
  orc_hr_reset_obs_double(n, st, obs, ph);
  for (int s = 0; s < K; ++s)
    orc_hr_step_double(n, st, fa, act, noise, s & 1, 1, s & 1, obs, rew, done, ph);

  double pt1[16] = {5.46, 20, 0, 0.01, 10, 10};
  double pt2[16] = {30, 1, 36, 0.001, 2, 5, 0.5, 0.003, 100, 0.01};
  double ptp[16] = {5.46, 20, 20, 0.01, 2, 5, 3};
  double psc[16] = {5.46, 20, 0, 0.01, 100, 1000, 3, 25, 1, -1};
  orc_t1_reset_obs_double(n, st, obs, pt1);
  for (int s = 0; s < K; ++s) orc_t1_step_double(n, st, act, obs, rew, pt1);
  orc_t2_reset_obs_double(n, st, obs, pt2);
  for (int s = 0; s < K; ++s) orc_t2_step_double(n, st, act, obs, rew, done, pt2);
  orc_tp_reset_obs_float(n, fst, fobs, ptp);
  for (int s = 0; s < K; ++s) orc_tp_step_float(n, fst, act, noise, fobs, frew, done, ptp);
  for (int s = 0; s < K; ++s) orc_sc_step_double(n, st, noise, obs, rew, psc);

  free(st); free(obs); free(rew); free(act); free(fst); free(fobs); free(frew); free(done);
  free(done2); free(noise); free(lam); free(mt); free(vt); free(adam); free(cur); free(fa);
  printf("oracle: all functions clean under ASan + UBSan\n");
  return 0;
}
