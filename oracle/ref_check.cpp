/* oracle/ref_check.cpp -- TEST INFRASTRUCTURE ONLY: the pieces of bin/checkBsdf.cpp that are not
 * bsdfmodel calls, evaluated with the reference's own headers (core/spherical.h, util/gamma.h, the
 * native backbone), so tests/ can recompute every checkBsdf statistic on the CPU from the same random
 * draws the GPU used.  checkBsdf.cpp is a program, not a header: its few lines of driver logic are
 * restated here, each citing the line it follows.
 */
#include "core/spherical.h"
#include "util/gamma.h"

namespace {
using C = bbm::floatRGB;
using Value = bbm::get_config<C>::Value;
using Vec2d = bbm::vec2d<Value>;
using Vec3d = bbm::vec3d<Value>;
using Constants = bbm::constants<Value>;
}

extern "C" {

/* sampleSphere (checkBsdf.cpp:28-35) / sampleHemisphere (:38-45) of n uniform pairs: direction + pdf */
void bbmref_sphere_dirs(size_t n, const float* xi0, const float* xi1, int hemisphere,
                        float* x, float* y, float* z, float* pdf)
{
  for(size_t i=0; i < n; ++i)
  {
    Vec2d coord;
    if(hemisphere)
    {
      bbm::spherical::theta(coord) = bbm::safe_acos(Value(xi0[i]));
      pdf[i] = 1.0 / Constants::Pi(2);
    }
    else
    {
      bbm::spherical::theta(coord) = bbm::safe_acos(1.0 - 2.0 * Value(xi0[i]));
      pdf[i] = 1.0 / Constants::Pi(4);
    }
    bbm::spherical::phi(coord) = Value(xi1[i]) * Constants::Pi(2);
    Vec3d d = bbm::spherical::convert(coord);
    x[i] = d[0]; y[i] = d[1]; z[i] = d[2];
  }
}

/* chi-square bin of n sampled directions (checkBsdf.cpp:374-377) */
void bbmref_chi2_bins(size_t n, const float* x, const float* y, const float* z, size_t theta, size_t phi,
                      uint64_t* idx)
{
  for(size_t i=0; i < n; ++i)
  {
    Vec2d sph_coord = bbm::spherical::convert(Vec3d(x[i], y[i], z[i]));
    size_t t = bbm::cast<size_t>(bbm::min( bbm::spherical::theta(sph_coord) / Constants::Pi() * theta, theta-1));
    size_t p = bbm::cast<size_t>(bbm::min( bbm::spherical::phi(sph_coord) / Constants::Pi(2) * phi, phi-1));
    idx[i] = t * phi + p;
  }
}

/* the pdf-integration point of bin (t, p) for a uniform pair (checkBsdf.cpp:351-356): direction and
 * solid-angle weight */
void bbmref_chi2_bin_points(size_t n, const uint32_t* t, const uint32_t* p, const float* rnd0, const float* rnd1,
                            size_t theta, size_t phi, float* x, float* y, float* z, float* w)
{
  for(size_t i=0; i < n; ++i)
  {
    Vec2d sph_coord;
    bbm::spherical::phi(sph_coord) = Constants::Pi(2) * (size_t(p[i]) + rnd0[i]) / phi;
    bbm::spherical::theta(sph_coord) = Constants::Pi() * (size_t(t[i]) + rnd1[i]) / theta;
    Vec3d dir = bbm::spherical::convert(sph_coord);
    Value wp = Constants::Pi2(2) * bbm::abs(bbm::spherical::sinTheta(sph_coord)) / (phi * theta);
    x[i] = dir[0]; y[i] = dir[1]; z[i] = dir[2]; w[i] = wp;
  }
}

/* P value of the chi-square statistic (checkBsdf.cpp:402-405) */
double bbmref_gamma_q(float a, float x) { return double(bbm::gamma_q(a, x)); }

} // extern "C"

extern "C" {
/* The reference's precomputed EPD shadowing table (include/precomputed/holzschuchpacanowski/G1.h), row-major
 * [p][t] -- compared entry by entry with the table libbbm_hip builds on the GPU. */
int bbmref_epd_g1(float* out, int cap)
{
  const auto& t = bbm::precomputed::holzschuchpacanowski::G1;
  for(size_t i=0; out && i < t.size() && int(i) < cap; ++i) out[i] = t[i];
  return int(t.size());
}
} // extern "C"
