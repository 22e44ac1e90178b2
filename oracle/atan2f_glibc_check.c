/* oracle/atan2f_glibc_check.c -- test infrastructure: pins bbm_amd/csrc/math.hpp's atan2f_glibc (a restatement of
 * glibc 2.35's atan2f: sysdeps/ieee754/flt-32/e_atan2f.c with s_atanf.c, Sun fdlibm's float algorithms, no FMA
 * variant) to this machine's libm, which is what the reference's spherical::phi calls (core/spherical.h:42-46:
 * atan2 of two floats -> backbone/native/include/backbone/math.h:87-88 std::atan2 -> atan2f).
 *
 *   atan2f_glibc_check [n]   n random (y, x) pairs per input class (default 2e8): unit-vector components (the
 *                            callers' domain), any finite floats, mixed magnitudes; plus zeros, infinities, NaN,
 *                            and x = 1 against every 13th y
 *
 * atan(y / x) by fdlibm's float atanf: four breakpoints (atan 0.5, 1, 1.5, inf as hi + lo), an 11-term odd
 * polynomial split in two Horner chains, all in float arithmetic; the quadrant fix-ups with pi_lo.  The constants are
 * fdlibm's (present in this machine's libm.so.6), not the reference's.  glibc's atan2f is not correctly rounded,
 * which is why the device restates it rather than rounding a double atan2.  Prints the mismatch counts, exits 1 on
 * any mismatch. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static const float atanhi[] = {4.6364760399e-01f, 7.8539812565e-01f, 9.8279368877e-01f, 1.5707962513e+00f};
static const float atanlo[] = {5.0121582440e-09f, 3.7748947079e-08f, 3.4473217170e-08f, 7.5497894159e-08f};
static const float aT[] = {3.3333334327e-01f, -2.0000000298e-01f, 1.4285714924e-01f, -1.1111110449e-01f,
                           9.0908870101e-02f, -7.6918758452e-02f, 6.6610731184e-02f, -5.8335702866e-02f,
                           4.9768779427e-02f, -3.6531571299e-02f, 1.6285819933e-02f};

static uint32_t bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float fromb(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* s_atanf.c for a finite x >= 0 below 2^25 (atan2f's only use: |y / x|) */
static float atanf_pos(float x)
{
  const uint32_t ix = bits(x);
  int id;
  if (ix < 0x3ee00000u) id = -1;                                   /* |x| < 0.4375 (tiny x: the polynomial gives x) */
  else if (ix < 0x3f980000u)
  {
    if (ix < 0x3f300000u) { id = 0; x = (2.0f * x - 1.0f) / (2.0f + x); }
    else { id = 1; x = (x - 1.0f) / (x + 1.0f); }
  }
  else if (ix < 0x401c0000u) { id = 2; x = (x - 1.5f) / (1.0f + 1.5f * x); }
  else { id = 3; x = -1.0f / x; }
  const float z = x * x;
  const float w = z * z;
  const float s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
  const float s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
  if (id < 0) return x - x * (s1 + s2);
  return atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
}

static float atan2f_r(float y, float x)
{
  const float pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f, pi = 3.1415927410e+00f,
              pi_lo = -8.7422776573e-08f;
  const uint32_t hx = bits(x), hy = bits(y), ix = hx & 0x7fffffffu, iy = hy & 0x7fffffffu;
  if (ix > 0x7f800000u || iy > 0x7f800000u) return x + y;
  const int m = (int)(((hy >> 31) & 1u) | ((hx >> 30) & 2u));
  /* glibc's x = 1 shortcut (atanf(y)) is not restated: the general path below gives the same float there
     (y / 1 = y; |y| >= 2^25: hi + lo = pi_o_2 + pi_lo / 2), which the x = 1 sweep in main checks */
  if (iy == 0) return (m < 2) ? y : ((m == 2) ? pi : -pi);
  if (ix == 0) return (hy >> 31) ? -pi_o_2 : pi_o_2;
  if (ix == 0x7f800000u)
  {
    if (iy == 0x7f800000u) return (m == 0) ? pi_o_4 : (m == 1) ? -pi_o_4 : (m == 2) ? 3.0f * pi_o_4 : -3.0f * pi_o_4;
    return (m == 0) ? 0.0f : (m == 1) ? -0.0f : (m == 2) ? pi : -pi;
  }
  if (iy == 0x7f800000u) return (hy >> 31) ? -pi_o_2 : pi_o_2;
  const int k = ((int)iy - (int)ix) >> 23;
  float z;
  if (k > 60) z = pi_o_2 + 0.5f * pi_lo;
  else if ((hx >> 31) && k < -60) z = 0.0f;
  else
  {
    const float q = fabsf(y / x);
    z = (bits(q) >= 0x4c000000u) ? atanhi[3] + atanlo[3] : atanf_pos(q);
  }
  switch (m)
  {
    case 0: return z;
    case 1: return -z;
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
  }
}

static uint64_t rng = 0x9e3779b97f4a7c15ull;
static uint64_t next(void) { rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17; return rng; }
static float unif(void) { return (float)((next() >> 40) * (1.0 / 16777216.0)) * 2.0f - 1.0f; }

int main(int argc, char** argv)
{
  const long n = (argc > 1) ? atol(argv[1]) : 200000000L;
  long bad = 0, tested = 0;
  const float sp[] = {0.0f, -0.0f, 1.0f, -1.0f, INFINITY, -INFINITY, NAN, 1e-45f, -1e-45f, 3e38f, -3e38f, 0.5f};
  for (int i = 0; i < 12; ++i)
    for (int j = 0; j < 12; ++j)
    {
      const float got = atan2f_r(sp[i], sp[j]), want = atan2f(sp[i], sp[j]);
      if (bits(got) != bits(want) && !(isnan(got) && isnan(want)) && bad++ < 8)
        printf("atan2f(%a, %a): restated %a, libm %a\n", sp[i], sp[j], got, want);
      ++tested;
    }
  for (uint32_t u = 0; u < 0x7f800000u; u += 13)                  /* x = 1, every 13th y of both signs */
    for (int sgn = 0; sgn < 2; ++sgn)
    {
      const float y = fromb(u | (sgn ? 0x80000000u : 0u));
      const float got = atan2f_r(y, 1.0f), want = atan2f(y, 1.0f);
      if (bits(got) != bits(want) && bad++ < 8) printf("atan2f(%a, 1): restated %a, libm %a\n", y, got, want);
      ++tested;
    }
  for (int cls = 0; cls < 3; ++cls)
    for (long i = 0; i < n; ++i)
    {
      float y, x;
      if (cls == 0) { y = unif(); x = unif(); }                               /* unit-vector components */
      else if (cls == 1) { y = fromb((uint32_t)next() & 0xff7fffffu); x = fromb((uint32_t)next() & 0xff7fffffu); }
      else { y = unif() * ldexpf(1.0f, (int)(next() % 80) - 40); x = unif() * ldexpf(1.0f, (int)(next() % 80) - 40); }
      const float got = atan2f_r(y, x), want = atan2f(y, x);
      if (bits(got) != bits(want) && !(isnan(got) && isnan(want)) && bad++ < 8)
        printf("atan2f(%a, %a): restated %a, libm %a\n", y, x, got, want);
      ++tested;
    }
  printf("atan2f_glibc_check: %ld (y, x) pairs, %ld mismatches\n", tested, bad);
  return bad ? 1 : 0;
}
