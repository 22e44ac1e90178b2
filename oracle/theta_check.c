/* oracle/theta_check.c -- test infrastructure: pins the algorithm of bbm_amd/csrc/spectral.hpp's theta_of (the
 * reference's spherical::theta, core/spherical.h:26-32: float(2 asin(|v - pole| / 2)) in double, pi - that below
 * the horizon) to this machine's glibc asin.  For every float chord length nrm in [0, 2] (every stride-th; default 1)
 * the restated double steps -- the degree-11 polynomial for asin, its upper-range reflection through sqrt((1 - y) / 2),
 * the 256-ulp midpoint guard that sends a lane to the library asin -- must give glibc's float for both hemispheres.
 * (The device's square root of w is an rsq seed and two Newton steps; here the IEEE sqrt, whose bits those steps
 * reach.)  Prints the counts (fallback lanes included) and exits 1 on any mismatch. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static const double kP[12] = {0x1.555555555554ep-3, 0x1.3333333337110p-4, 0x1.6db6db68067fep-5,
                              0x1.f1c71fb700f11p-6, 0x1.6e8b26f89d407p-6, 0x1.1c598c739143cp-6,
                              0x1.c86b17413a7b6p-7, 0x1.8559b6cfd3c89p-7, 0x1.fd4f1fa1ac91cp-8,
                              0x1.084522a849f25p-6, -0x1.65717d3785d18p-7, 0x1.cf6d7d2572a46p-6};

static long fallbacks = 0;

static float theta_r(float nrm, int below)
{
  const float pi_f = 3.14159274101257324f;
  const double y = 0.5 * (double)nrm;
  const int hi = y > 0.5;
  const double w = hi ? (1.0 - y) * 0.5 : y * y;
  const double s = hi ? sqrt(w) : y;
  double p = kP[11];
  for (int k = 10; k >= 0; --k) p = fma(p, w, kP[k]);
  const double r = fma(s * w, p, s);
  const double t = 2.0 * (hi ? 0x1.921fb54442d18p+0 - 2.0 * r : r);
  double u = below ? (double)pi_f - t : t;
  uint64_t b;
  memcpy(&b, &u, 8);
  const uint32_t lo = (uint32_t)b & 0x1fffffffu;
  if ((uint32_t)(lo - 0x0fffff00u) < 0x200u || u != u)
  {
    ++fallbacks;
    const double te = 2.0 * asin(y);
    u = below ? (double)pi_f - te : te;
  }
  return (float)u;
}

int main(int argc, char** argv)
{
  const uint32_t stride = (argc > 1) ? (uint32_t)strtoul(argv[1], NULL, 10) : 1u;
  const float pi_f = 3.14159274101257324f;
  long bad = 0, tested = 0;
  for (uint32_t u = 0; u <= 0x40000000u; u += stride)               /* nrm in [0, 2] */
  {
    float nrm;
    memcpy(&nrm, &u, 4);
    for (int below = 0; below < 2; ++below)
    {
      const double te = 2.0 * asin(0.5 * (double)nrm);
      const float want = (float)(below ? (double)pi_f - te : te);
      const float got = theta_r(nrm, below);
      if (memcmp(&got, &want, 4) != 0 && bad++ < 8) printf("nrm %a below %d: restated %a, glibc %a\n", nrm, below, got, want);
      ++tested;
    }
  }
  printf("theta_check: %ld (nrm, hemisphere) cases, %ld mismatches, %ld fallbacks\n", tested, bad, fallbacks);
  return bad ? 1 : 0;
}
