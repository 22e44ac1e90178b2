/* oracle/expf_glibc_check.c -- test infrastructure: pins bbm_amd/csrc/math.hpp's expf_glibc (a restatement of
 * glibc 2.35's expf, sysdeps/ieee754/flt-32/e_expf.c + e_exp2f_data.c, the Arm optimized-routines algorithm) to
 * this machine's libm, which is what the reference's bbm::exp(float) calls (std::exp -> expf).
 *
 *   expf_glibc_check [stride]   every stride-th float in [-110, 90] (default 1: all 2.24e9 of them)
 *
 * The same double-precision steps as the device function (FMA-contracted, the x86-64 ifunc variant for FMA
 * hosts); prints the mismatch count and exits 1 on any mismatch. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static const uint64_t T[32] = {
  0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
  0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
  0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
  0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
  0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
  0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
  0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
  0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull};

static float expf_restated(float x)
{
  const double InvLn2N = 0x1.71547652b82fep+0 * 32, Shift = 0x1.8p+52;
  const double C0 = 0x1.c6af84b912394p-5 / 32 / 32 / 32, C1 = 0x1.ebfce50fac4f3p-3 / 32 / 32, C2 = 0x1.62e42ff0c52d6p-1 / 32;
  if (x < -0x1.9fe368p6f) return 0.0f;
  if (x > 0x1.62e42ep6f) return INFINITY;
  if (x != x) return x + x;
  const double xd = x;
  double kb = fma(InvLn2N, xd, Shift);
  uint64_t ki;
  memcpy(&ki, &kb, 8);
  const double kd = kb - Shift;
  const double r = fma(InvLn2N, xd, -kd);
  uint64_t t = T[ki & 31u] + (ki << 47);
  double s;
  memcpy(&s, &t, 8);
  const double z = fma(C0, r, C1), r2 = r * r;
  double y = fma(C2, r, 1.0);
  y = fma(z, r2, y);
  return (float)(y * s);
}

int main(int argc, char** argv)
{
  const uint64_t stride = argc > 1 ? strtoull(argv[1], 0, 10) : 1;
  long total = 0, bad = 0;
  for (uint64_t u = 0; u < (1ull << 32); u += stride)
  {
    const uint32_t v = (uint32_t)u;
    float x;
    memcpy(&x, &v, 4);
    if (!(x >= -110.f && x <= 90.f)) continue;
    ++total;
    volatile float ref = expf(x);
    const float got = expf_restated(x);
    if (memcmp(&got, (const void*)&ref, 4) != 0)
    {
      if (bad < 5) printf("mismatch x=%a libm=%a restated=%a\n", x, (double)ref, (double)got);
      ++bad;
    }
  }
  printf("expf_glibc_check: %ld floats in [-110, 90], %ld mismatches\n", total, bad);
  return bad ? 1 : 0;
}
