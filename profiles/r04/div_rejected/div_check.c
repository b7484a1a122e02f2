/* Test infrastructure (not the product): an exhaustive check of the PMSM kernel's
 * reciprocal-based division (gym-lorenz_amd/csrc/lz_systems.h SysPMSM::div_cr) against
 * the IEEE float32 quotient, for the Adam bias-correction divisors of
 * lorenz_env_try_pmsm.py:130-131 (mt / (1 - beta1**k), vt / (1 - beta2**k)).
 *
 * For each divisor b = (float)(1 - beta**k) (the table lz_api.cpp builds: same libm pow)
 * and EVERY float32 significand of x in the binade [1, 2) -- and, by the sign symmetry,
 * its negative -- it checks  fma(fma(-q, b, x), y, q) == x / b  with q = RN(x y),
 * y = RN(1 / b).  Scaling x by a power of two scales q, the residual and the quotient
 * exactly while no intermediate leaves the normal range, which the device guard
 * (|x|, |q| in [2^-60, 2^100]) ensures; so one binade per divisor covers them all.
 *
 *   div_check <beta> <k_first> <k_last> <k_stride> <threads> [naive]
 * prints "checked <divisors> <pairs> mismatches <n>" and exits 1 on any mismatch.
 *   gcc -O3 -mfma -ffp-contract=off -pthread oracle/div_check.c -o oracle/div_check -lm  (oracle/Makefile)
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  const float* bs;
  int nb;
  int t, nt;
  uint64_t bad, pairs;
} Job;

static int naive;  /* 1: no fma correction (the checker's own sanity check: must mismatch) */

static float div_cr(float x, float b, float y) {
  const float q = x * y;
  if (naive) return q;
  const float r = fmaf(-q, b, x);
  return fmaf(r, y, q);
}

static void* run(void* p) {
  Job* j = (Job*)p;
  for (int i = j->t; i < j->nb; i += j->nt) {
    const float b = j->bs[i];
    const float y = 1.0f / b;
    for (uint32_t m = 0; m < (1u << 23); ++m) {
      uint32_t u = 0x3f800000u | m;
      float x;
      memcpy(&x, &u, 4);
      const float e = x / b, g = div_cr(x, b, y);
      const float en = (-x) / b, gn = div_cr(-x, b, y);
      uint32_t ue, ug, uen, ugn;
      memcpy(&ue, &e, 4);
      memcpy(&ug, &g, 4);
      memcpy(&uen, &en, 4);
      memcpy(&ugn, &gn, 4);
      j->bad += (ue != ug) + (uen != ugn);
    }
    j->pairs += 2ull << 23;
  }
  return NULL;
}

int main(int argc, char** argv) {
  if (argc < 6) {
    fprintf(stderr, "usage: div_check beta k_first k_last k_stride threads\n");
    return 2;
  }
  const double beta = atof(argv[1]);
  const long k0 = atol(argv[2]), k1 = atol(argv[3]), ks = atol(argv[4]);
  int nt = atoi(argv[5]);
  naive = argc > 6 && strcmp(argv[6], "naive") == 0;
  if (nt < 1) nt = 1;
  if (nt > 64) nt = 64;
  float* bs = malloc(sizeof(float) * (size_t)((k1 - k0) / ks + 2));
  int nb = 0;
  for (long k = k0; k <= k1; k += ks) {
    const float b = (float)(1.0 - pow(beta, (double)k));
    if (b != 0.0f) bs[nb++] = b;
  }
  Job jobs[64];
  pthread_t th[64];
  for (int t = 0; t < nt; ++t) {
    jobs[t] = (Job){bs, nb, t, nt, 0, 0};
    pthread_create(&th[t], NULL, run, &jobs[t]);
  }
  uint64_t bad = 0, pairs = 0;
  for (int t = 0; t < nt; ++t) {
    pthread_join(th[t], NULL);
    bad += jobs[t].bad;
    pairs += jobs[t].pairs;
  }
  printf("checked %d divisors %llu pairs mismatches %llu\n", nb, (unsigned long long)pairs,
         (unsigned long long)bad);
  free(bs);
  return bad ? 1 : 0;
}
