/* oracle/erfcf_glibc_check.c -- test infrastructure: pins bbm_amd/csrc/math.hpp's erfcf_glibc (a restatement of
 * glibc 2.35's erfcf, sysdeps/ieee754/flt-32/s_erff.c -- the Sun fdlibm algorithm in float arithmetic, with
 * __ieee754_expf = the Arm expf of e_expf.c) to this machine's libm, which is what the reference's bbm::erfc(float)
 * calls (backbone/native/include/backbone/math.h: using std::erfc -> erfcf).
 *
 *   erfcf_glibc_check [stride]   every stride-th float (default 1: all 2^32 bit patterns), erfcf and erff
 *
 * glibc's erfcf is not correctly rounded; the He family's shadowing S1 (he.h:266-291) subtracts it from a
 * nearly equal quantity, so the device must return glibc's own float.  The constants are fdlibm's float
 * coefficients, as this machine's libm.so.6 holds them; plain float operations (s_erff.c has no FMA variant).
 * Prints the mismatch count and exits 1 on any mismatch. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* glibc's expf (oracle/expf_glibc_check.c, FMA variant) */
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

static const float erx = 8.4506291151e-01f,
  pp0 = 1.2837916613e-01f, pp1 = -3.2504209876e-01f, pp2 = -2.8481749818e-02f, pp3 = -5.7702702470e-03f,
  pp4 = -2.3763017452e-05f, qq1 = 3.9791721106e-01f, qq2 = 6.5022252500e-02f, qq3 = 5.0813062117e-03f,
  qq4 = 1.3249473704e-04f, qq5 = -3.9602282413e-06f,
  pa0 = -2.3621185683e-03f, pa1 = 4.1485610604e-01f, pa2 = -3.7220788002e-01f, pa3 = 3.1834661961e-01f,
  pa4 = -1.1089469492e-01f, pa5 = 3.5478305072e-02f, pa6 = -2.1663755178e-03f, qa1 = 1.0642088205e-01f,
  qa2 = 5.4039794207e-01f, qa3 = 7.1828655899e-02f, qa4 = 1.2617121637e-01f, qa5 = 1.3637083583e-02f,
  qa6 = 1.1984500103e-02f,
  ra0 = -9.8649440333e-03f, ra1 = -6.9385856390e-01f, ra2 = -1.0558626175e+01f, ra3 = -6.2375331879e+01f,
  ra4 = -1.6239666748e+02f, ra5 = -1.8460508728e+02f, ra6 = -8.1287437439e+01f, ra7 = -9.8143291473e+00f,
  sa1 = 1.9651271820e+01f, sa2 = 1.3765776062e+02f, sa3 = 4.3456588745e+02f, sa4 = 6.4538726807e+02f,
  sa5 = 4.2900814819e+02f, sa6 = 1.0863500214e+02f, sa7 = 6.5702495575e+00f, sa8 = -6.0424413532e-02f,
  rb0 = -9.8649431020e-03f, rb1 = -7.9928326607e-01f, rb2 = -1.7757955551e+01f, rb3 = -1.6063638306e+02f,
  rb4 = -6.3756646729e+02f, rb5 = -1.0250950928e+03f, rb6 = -4.8351919556e+02f, sb1 = 3.0338060379e+01f,
  sb2 = 3.2579251099e+02f, sb3 = 1.5367296143e+03f, sb4 = 3.1998581543e+03f, sb5 = 2.5530502930e+03f,
  sb6 = 4.7452853394e+02f, sb7 = -2.2440952301e+01f;


static float erfcf_restated(float x)
{
  const int32_t hx = (int32_t)f2u(x);
  const uint32_t ix = (uint32_t)hx & 0x7fffffffu;
  if (ix >= 0x7f800000u) return (float)(((uint32_t)hx >> 31) << 1) + 1.0f / x;
  if (ix < 0x3f580000u)
  {
    if (ix < 0x32800000u) return 1.0f - x;
    const float z = x * x;
    const float r = pp0 + z * (pp1 + z * (pp2 + z * (pp3 + z * pp4)));
    const float s = 1.0f + z * (qq1 + z * (qq2 + z * (qq3 + z * (qq4 + z * qq5))));
    const float y = r / s;
    if (hx < 0x3e800000) return 1.0f - (x + x * y);
    float rr = x * y;
    rr += (x - 0.5f);
    return 0.5f - rr;
  }
  if (ix < 0x3fa00000u)
  {
    const float s = fabsf(x) - 1.0f;
    const float P = pa0 + s * (pa1 + s * (pa2 + s * (pa3 + s * (pa4 + s * (pa5 + s * pa6)))));
    const float Q = 1.0f + s * (qa1 + s * (qa2 + s * (qa3 + s * (qa4 + s * (qa5 + s * qa6)))));
    if (hx >= 0) return (1.0f - erx) - P / Q;
    return 1.0f + (erx + P / Q);
  }
  if (ix < 0x41e00000u)
  {
    const float ax = fabsf(x);
    const float s = 1.0f / (ax * ax);
    float R, S;
    if (ix < 0x4036DB6Du)
    {
      R = ra0 + s * (ra1 + s * (ra2 + s * (ra3 + s * (ra4 + s * (ra5 + s * (ra6 + s * ra7))))));
      S = 1.0f + s * (sa1 + s * (sa2 + s * (sa3 + s * (sa4 + s * (sa5 + s * (sa6 + s * (sa7 + s * sa8)))))));
    }
    else
    {
      if (hx < 0 && ix >= 0x40c00000u) return 2.0f - 1e-30f;
      R = rb0 + s * (rb1 + s * (rb2 + s * (rb3 + s * (rb4 + s * (rb5 + s * rb6)))));
      S = 1.0f + s * (sb1 + s * (sb2 + s * (sb3 + s * (sb4 + s * (sb5 + s * (sb6 + s * sb7))))));
    }
    const float z = u2f(f2u(ax) & 0xffffe000u);
    const float r = expf_restated(-z * z - 0.5625f) * expf_restated((z - ax) * (z + ax) + R / S);
    if (hx > 0) return r / ax;
    return 2.0f - r / ax;
  }
  if (hx > 0) return 1e-30f * 1e-30f;
  return 2.0f - 1e-30f;
}

static uint32_t g_erf_split = 0x4036DB6Eu, g_erf_mask = 0xfffff000u;   /* erff truncates z to 12 bits, erfcf to 11 */
static float erff_restated(float x)
{
  const int32_t hx = (int32_t)f2u(x);
  const uint32_t ix = (uint32_t)hx & 0x7fffffffu;
  if (ix >= 0x7f800000u) return (float)(1 - (int)(((uint32_t)hx >> 31) << 1)) + 1.0f / x;
  if (ix < 0x3f580000u)
  {
    if (ix < 0x31800000u)
    {
      if (ix < 0x04000000u) return 0.0625f * (16.0f * x + u2f(0x400375d4u) * x);
      return x + pp0 * x;
    }
    const float z = x * x;
    const float r = pp0 + z * (pp1 + z * (pp2 + z * (pp3 + z * pp4)));
    const float s = 1.0f + z * (qq1 + z * (qq2 + z * (qq3 + z * (qq4 + z * qq5))));
    const float y = r / s;
    return x + x * y;
  }
  if (ix < 0x3fa00000u)
  {
    const float s = fabsf(x) - 1.0f;
    const float P = pa0 + s * (pa1 + s * (pa2 + s * (pa3 + s * (pa4 + s * (pa5 + s * pa6)))));
    const float Q = 1.0f + s * (qa1 + s * (qa2 + s * (qa3 + s * (qa4 + s * (qa5 + s * qa6)))));
    if (hx >= 0) return erx + P / Q;
    return -erx - P / Q;
  }
  if (ix >= 0x40c00000u) return (hx >= 0) ? 1.0f - 1e-30f : 1e-30f - 1.0f;
  const float ax = fabsf(x);
  const float s = 1.0f / (ax * ax);
  float R, S;
  if (ix < g_erf_split)
  {
    R = ra0 + s * (ra1 + s * (ra2 + s * (ra3 + s * (ra4 + s * (ra5 + s * (ra6 + s * ra7))))));
    S = 1.0f + s * (sa1 + s * (sa2 + s * (sa3 + s * (sa4 + s * (sa5 + s * (sa6 + s * (sa7 + s * sa8)))))));
  }
  else
  {
    R = rb0 + s * (rb1 + s * (rb2 + s * (rb3 + s * (rb4 + s * (rb5 + s * rb6)))));
    S = 1.0f + s * (sb1 + s * (sb2 + s * (sb3 + s * (sb4 + s * (sb5 + s * (sb6 + s * sb7))))));
  }
  const float z = u2f(f2u(ax) & g_erf_mask);
  const float r = expf_restated(-z * z - 0.5625f) * expf_restated((z - ax) * (z + ax) + R / S);
  if (hx >= 0) return 1.0f - r / ax;
  return r / ax - 1.0f;
}

int main(int argc, char** argv)
{
  const uint64_t stride = argc > 1 ? strtoull(argv[1], 0, 10) : 1;
  if (argc > 2) g_erf_mask = (uint32_t)strtoul(argv[2], 0, 16);
  long total = 0, bad = 0;
  for (uint64_t u = 0; u < (1ull << 32); u += stride)
  {
    const float x = u2f((uint32_t)u);
    ++total;
    volatile float ref = erfcf(x);
    const float got = erfcf_restated(x);
    if (f2u(got) != f2u(ref) && !(got != got && ref != ref))
    {
      if (bad < 8) printf("mismatch x=%a libm=%a restated=%a\n", x, (double)ref, (double)got);
      ++bad;
    }
  }
  long ebad = 0;
  for (uint64_t u = 0; u < (1ull << 32); u += stride)
  {
    const float x = u2f((uint32_t)u);
    volatile float ref = erff(x);
    const float got = erff_restated(x);
    if (f2u(got) != f2u(ref) && !(got != got && ref != ref))
    {
      if (ebad < 8) printf("erff mismatch x=%a libm=%a restated=%a\n", x, (double)ref, (double)got);
      ++ebad;
    }
  }
  printf("erfcf_glibc_check: %ld floats, erfcf %ld mismatches, erff %ld mismatches\n", total, bad, ebad);
  bad += ebad;
  return bad ? 1 : 0;
}
