/* oracle/sincosf_glibc_check.c -- test infrastructure: pins bbm_amd/csrc/math.hpp's sincosf_glibc
 * (restatements of glibc 2.35's sinf and cosf, sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c, sincosf.h and
 * sincosf_data.c -- the Arm optimized-routines algorithms) to this machine's libm, which is what the reference's
 * bbm::cossin / bbm::sin / bbm::cos of a float call (backbone/native/include/backbone/math.h:126: std::cos, std::sin).
 *
 *   sincosf_glibc_check [stride]   every stride-th float with |x| < 120 (default 1: all of them -- the device's domain,
 *                                  every sampler angle), both signs, both functions
 *
 * The steps are the x86-64 ifunc variant built with FMA contraction (__sinf_fma / __cosf_fma on any FMA-capable
 * host): |x| < 0.75 (abstop12 below pi/4's): the odd / even polynomial in x directly; |x| < 120: n = nearest
 * quadrant from x * (2/pi 2^24) truncated to int32 (+2^23, >> 24), r = x - n pi/2 (one FMA), the quadrant's sign
 * and, for quadrants 2 and 3, the second coefficient set; the odd polynomial for sin in even quadrants and for cos in
 * odd ones, the even one otherwise.  The coefficients are glibc's table (__sincosf_table, read from this machine's
 * libm.so.6: sign[4], 2/pi 2^24, pi/2, then c0, c1, s1, c2, s2, c3, s3, c4), not the reference's.  Prints the mismatch
 * counts and exits 1 on any mismatch. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct { double sign[4], hpi_inv, hpi, c0, c1, s1, c2, s2, c3, s3, c4; } sincos_t;
static const sincos_t TAB[2] = {
  {{1.0, -1.0, -1.0, 1.0}, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0, 0x1p+0, -0x1.ffffffd0c621cp-2,
   -0x1.555545995a603p-3, 0x1.55553e1068f19p-5, 0x1.1107605230bc4p-7, -0x1.6c087e89a359dp-10,
   -0x1.994eb3774cf24p-13, 0x1.99343027bf8c3p-16},
  {{1.0, -1.0, -1.0, 1.0}, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0, -0x1p+0, 0x1.ffffffd0c621cp-2,
   -0x1.555545995a603p-3, -0x1.55553e1068f19p-5, 0x1.1107605230bc4p-7, 0x1.6c087e89a359dp-10,
   -0x1.994eb3774cf24p-13, -0x1.99343027bf8c3p-16}};

static uint32_t abstop12(float x) { uint32_t u; memcpy(&u, &x, 4); return (u >> 20) & 0x7ff; }

static float poly(double x, double x2, const sincos_t* p, int n)
{
  if ((n & 1) == 0)
  {
    const double x3 = x * x2;
    const double s1 = fma(x2, p->s3, p->s2);
    const double x7 = x3 * x2;
    const double s = fma(x3, p->s1, x);
    return (float)fma(x7, s1, s);
  }
  const double x4 = x2 * x2;
  const double c2 = fma(x2, p->c4, p->c3);
  const double c1 = fma(x2, p->c1, p->c0);
  const double x6 = x4 * x2;
  const double c = fma(x4, p->c2, c1);
  return (float)fma(x6, c2, c);
}

/* cos = 0, sin = 1 */
static float sc(float y, int want_sin)
{
  double x = y;
  const sincos_t* p = &TAB[0];
  if (abstop12(y) < abstop12(0x1.921fb6p-1f))
  {
    if (abstop12(y) < abstop12(0x1p-12f)) return want_sin ? y : 1.0f;
    return poly(x, x * x, p, want_sin ? 0 : 1);
  }
  const double r = x * p->hpi_inv;
  const int n = ((int32_t)r + 0x800000) >> 24;
  x = fma(-(double)n, p->hpi, x);
  const double s = p->sign[n & 3];
  if (n & 2) p = &TAB[1];
  return poly(x * s, x * x, p, want_sin ? n : (n ^ 1));
}

int main(int argc, char** argv)
{
  const uint32_t stride = (argc > 1) ? (uint32_t)strtoul(argv[1], NULL, 10) : 1u;
  long bad[2] = {0, 0}, tested = 0;
  for (uint32_t u = 0; u < 0x42f00000u; u += stride)
    for (int sign = 0; sign < 2; ++sign)
    {
      const uint32_t b = u | (sign ? 0x80000000u : 0u);
      float x;
      memcpy(&x, &b, 4);
      for (int f = 0; f < 2; ++f)
      {
        const float got = sc(x, f), want = f ? sinf(x) : cosf(x);
        uint32_t g, w;
        memcpy(&g, &got, 4);
        memcpy(&w, &want, 4);
        if (g != w && bad[f]++ < 5) printf("%s(%a): restated %a, libm %a\n", f ? "sinf" : "cosf", x, got, want);
      }
      ++tested;
    }
  printf("sincosf_glibc_check: %ld floats, cosf mismatches %ld, sinf mismatches %ld\n", tested, bad[0], bad[1]);
  return (bad[0] || bad[1]) ? 1 : 0;
}
