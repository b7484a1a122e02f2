/* Exhaustive check, over all 2^32 float32 bit patterns, that division by a constant c
 * done as   q = x * r;  e = fma(-q, c, x);  q' = fma(e, r, q)   (r = RN(1/c))
 * returns exactly IEEE x / c (round-to-nearest-even), NaN payload aside.  Used to
 * justify the 3-instruction division in SysHR<float> (lz_systems.h) in place of the
 * ~10-instruction v_div_scale / v_div_fmas / v_div_fixup sequence.
 *   gcc -O2 -fopenmp -ffp-contract=off tools/div_const_check.c -o /tmp/dcc -lm && /tmp/dcc 50 20
 * (output: profiles/r01/div_const_check.txt)
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* The kernel's form: the FMA path only for 2^-100 <= |x| <= 2^100, else the divide.
 * -DVARIANT='fmaf(e, r, q)' (unguarded) differs for -0, subnormal quotients and inf. */
#ifndef VARIANT
#define VARIANT ((fabsf(x) >= 0x1p-100f && fabsf(x) <= 0x1p100f) ? fmaf(e, r, q) : x / c)
#endif

static float f_of(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t u_of(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

int main(int argc, char** argv) {
  int bad_total = 0;
  for (int a = 1; a < argc; ++a) {
    const float c = (float)atof(argv[a]);
    const float r = 1.0f / c;
    uint64_t bad = 0, bad_sub = 0, bad_zero = 0, bad_big = 0;
    uint32_t first = 0;
#pragma omp parallel for reduction(+ : bad, bad_sub, bad_zero, bad_big) schedule(static)
    for (int64_t k = 0; k < (1LL << 32); ++k) {
      const float x = f_of((uint32_t)k);
      const float want = x / c;
      const float q = x * r;
      const float e = fmaf(-q, c, x);
      const float got = VARIANT;
      if (isnan(want) ? !isnan(got) : u_of(want) != u_of(got)) {
        bad += 1;
        if (x == 0.0f) bad_zero += 1;
        else if (fabsf(want) < 0x1p-126f) bad_sub += 1;
        else if (fabsf(x) > 0x1p120f) bad_big += 1;
        else first = (uint32_t)k;
      }
    }
    printf("c = %g (r = %a): %llu of 2^32 inputs differ from IEEE x / c (zero %llu, "
           "subnormal quotient %llu, |x| > 2^120 %llu, other %llu, e.g. x = %a)\n", c, r,
           (unsigned long long)bad, (unsigned long long)bad_zero, (unsigned long long)bad_sub,
           (unsigned long long)bad_big,
           (unsigned long long)(bad - bad_zero - bad_sub - bad_big), f_of(first));
    bad_total += bad != 0;
  }
  return bad_total;
}
