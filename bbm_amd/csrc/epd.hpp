// bbm_amd/csrc/epd.hpp -- the Exponential Power Distribution microfacet model of Holzschuch and
// Pacanowski 2017 (include/bsdfmodel/holzschuchpacanowski.h:34-42):
//
//   microfacet< ndf::epd, maskingshadowing::vanginneken, fresnel::complex<Value>, Walter (4) >  (not scaled)
//
// Parameters (attribute declaration order): beta, p (ndf::epd, ndf/epd.h:180-182), eta = (n, k) (complex ior).
//
// The shadowing term G1 is a lookup into a 100 x 1000 table of precomputed values
// (include/precomputed/holzschuchpacanowski/G1.h, interpolated by core/precompute.h:126-198).  That
// table is not copied: the library computes it on the GPU the first time an EPD model is used,
// restating the reference's generator (precompute/HolzschuchPacanowski/G1.cpp:91-223: the P2 integral
// by a 10 000-interval midpoint rule, the incremental Delta recurrence over tan(theta), G1 = 1/(1+Delta))
// and rounding every entry to the 6 significant digits the generator printed into G1.h
// (bbm::toString(float) = ostream << float).  tests/test_gpu_parity.py compares the result with the
// reference's own table entry by entry.
#pragma once
#include <cmath>
#include "math.hpp"
#include "microfacet.hpp"
#include "fit.hpp"     // phi_of
#include "kernels.hpp"  // host_prepare

namespace bbmhip {

constexpr int kEpdRows = 100, kEpdCols = 1000;

// The table the EPD kernels read (set by epd_prepare() in inst_epd.hip, the only unit that launches
// EPD kernels; internal linkage, so other units carry an unused copy).
static __device__ const float* g_epd_g1 = nullptr;

// std::lerp(a, b, t) for doubles (libstdc++ <cmath>, C++20): exact at the ends, monotone.
__device__ __forceinline__ double std_lerp(double a, double b, double t)
{
  if ((a <= 0 && b >= 0) || (a >= 0 && b <= 0)) return t * b + (1 - t) * a;
  if (t == 1) return b;
  const double x = a + t * (b - a);
  return ((t > 1) == (b > a)) ? ((b < x) ? x : b) : ((x < b) ? x : b);
}

// tab<float, {100, 1000}, MAP0, MAP1>::interpolate<float>(p, t) (core/precompute.h:126-198, G1.h:14-16):
// mapped indices (double) m0 = 5.0 / p - 1.0, m1 = exp(-exp(log(1/t) * 0.05)) * 1000.0 - 1.0; bilinear
// lerp of the clamped floor/ceil entries, the inner lerp rounded to float (the RET type) before the outer.
__device__ __forceinline__ float epd_g1_lookup(const float* tab, float p, float t)
{
  const double m0 = 5.0 / double(p) - 1.0;
#ifdef BBM_HIP_EPD_OCML_EXP
  const double m1 = exp(-exp(double(logf_cr(div_nr(1.0f, t))) * 0.05)) * 1000.0 - 1.0;
#else
  // the two double exponentials on exp_dd (~2^-44, a 9-FMA polynomial) instead of the device library's (~40
  // instructions each): m1 only places the bilinear weights, which are continuous across a floor() flip, so an
  // m1 within 1e-12 of the reference's moves the interpolated G1 by ~1e-12 relative
  // (L = +-inf at t = 0 / inf: the reference's exp(-exp(L 0.05)) is 0 / 1, exp_dd's polynomial would give NaN)
#if defined(BBM_HIP_EPD_LOGF_CR)
  const double L = double(logf_cr(div_nr(1.0f, t)));
#elif defined(BBM_HIP_EPD_LOGF_GLIBC)
  const double L = double(logf_glibc(div_nr(1.0f, t)));      // A/B: glibc's logf, bit for bit
#else
  // ln(1 / t) from log2_acc (~2^-44 absolute) instead of the library's double log: like m1's exponentials it only
  // places the bilinear weights, continuously (dm1/dL <= ~18.4), so ~1e-13 in L moves G1 by ~1e-12 relative
  const float it = div_nr(1.0f, t);
  const double L = (it == 0.0f) ? -__builtin_inf() : ((it > 3.40282347e38f) ? __builtin_inf()
                   : ((it != it) ? double(it) : double(float(log2_acc(it) * 0.69314718055994530942))));
#endif
  const double e1 = __builtin_isfinite(L) ? exp_dd(-exp_dd(L * 0.05)) : ((L > 0.0) ? 0.0 : 1.0);
  const double m1 = (L != L) ? L : e1 * 1000.0 - 1.0;        // NaN stays NaN
#endif
  auto at = [&](double i0, double i1) {
    const int r = int(fmin(fmax(i0, 0.0), double(kEpdRows - 1)));
    const int c = int(fmin(fmax(i1, 0.0), double(kEpdCols - 1)));
    return tab[r * kEpdCols + c];
  };
  const double f0 = floor(m0), c0 = ceil(m0), w0 = m0 - floor(m0);
  const double f1 = floor(m1), c1 = ceil(m1), w1 = m1 - floor(m1);
  const float lo = float(std_lerp(at(f0, f1), at(f0, c1), w1));
  const float hi = float(std_lerp(at(c0, f1), at(c0, c1), w1));
  return float(std_lerp(lo, hi, w0));
}

// Regularised lower incomplete gamma P(a, x) in double (series for x < a + 1, Lentz continued fraction
// for Q otherwise; Numerical Recipes 6.2, the algorithm util/gamma.h:22-25 follows for a < 20).
__device__ __forceinline__ void gamma_pq_d(double a, double x, double& P, double& Q)
{
  if (x <= 0) { P = 0; Q = 1; return; }
  const double lead = exp(-x + a * log(x) - lgamma(a));
  if (x < a + 1)
  {
    double ap = a, sum = 1.0 / a, del = sum;
    for (int n = 0; n < 500; ++n)
    {
      ap += 1;
      del *= x / ap;
      sum += del;
      if (fabs(del) < fabs(sum) * 1e-16) break;
    }
    P = sum * lead;
    Q = 1 - P;
    return;
  }
  const double tiny = 1e-300;
  double b = x + 1 - a, c = 1 / tiny, d = 1 / b, h = d;
  for (int i = 1; i < 500; ++i)
  {
    const double an = -i * (i - a);
    b += 2;
    d = an * d + b;
    if (fabs(d) < tiny) d = tiny;
    c = b + an / c;
    if (fabs(c) < tiny) c = tiny;
    d = 1 / d;
    const double del = d * c;
    h *= del;
    if (fabs(del - 1) < 1e-16) break;
  }
  Q = lead * h;
  P = 1 - Q;
}

// gamma_q_inv(a, q): x with Q(a, x) = q (util/invgamma.h:446-452).  The reference refines DiDonato &
// Morris's initial estimate with three float Newton-Halley steps; here the same Halley update
// (invgamma.h:404-414: t = (P - p) / R, R = x^a e^-x / Gamma(a), x *= 1 - (t + w t^2)) runs in double
// until converged from a simple start (DiDonato-Morris Eq. 31/32 for a > 1, Eq. 21's power form
// otherwise), so the result is the float nearest the exact inverse -- what the reference's float
// iteration converges to.
__device__ __forceinline__ double gamma_q_inv_d(double a, double q)
{
  if (!(a > 0) || !(q > 0)) return 0.0;
  if (q >= 1) return 0.0;
  const double p = 1 - q;
  const double lg = lgamma(a);
  double x;
  if (a > 1)
  {
    // Eq. 32 (normal quantile) + Eq. 31 (Wilson-Hilferty-like expansion)
    const double pp = (p < 0.5) ? p : q;
    const double t = sqrt(-2 * log(pp));
    double s = t - (3.31125922108741 + t * (11.6616720288968 + t * (4.28342155967104 + t * 0.213623493715853))) /
                   (1 + t * (6.61053765625462 + t * (6.40691597760039 + t * (1.27364489782223 + t * 0.3611708101884203e-1))));
    if (p < 0.5) s = -s;
    const double sa = sqrt(a);
    x = a - 1.0 / 3.0 + 16 / (810 * a) + s * (sa - 7 / (36 * sa) - 433 / (38880 * a * sa)) +
        s * s * (1.0 / 3.0 - 7 / (810 * a)) + s * s * s * (1 / (36 * sa) + 256 / (38880 * a * sa)) +
        s * s * s * s * (-3 / (810 * a)) + s * s * s * s * s * (9 / (38880 * a * sa));
    if (!(x > 0)) x = a * 0.01;
  }
  else
  {
    x = pow(p * exp(lg) * a, 1 / a);          // P(a, x) ~ x^a / Gamma(a + 1) for small x
    if (!(x > 0) || x > 5 * (a + 1)) x = -log(q) + (a - 1) * log(fmax(-log(q), 1e-300));
    if (!(x > 0)) x = 1e-3;
  }
  for (int it = 0; it < 60; ++it)
  {
    double P, Q;
    gamma_pq_d(a, x, P, Q);
    const double r = exp(-x - lg + log(x) * a);
    if (!(r > 0)) break;
    const double t = ((p <= 0.5) ? (P - p) : (q - Q)) / r;
    const double w = 0.5 * (a - 1 - x);
    const double step = (fabs(t) <= 0.1 && fabs(w * t) <= 0.1) ? t + w * t * t : t;
    double xn = x * (1 - step);
    if (!(xn > 0)) xn = 0.5 * x;
    if (fabs(xn - x) <= 1e-14 * x) { x = xn; break; }
    x = xn;
  }
  return x;
}

// ndf::epd (ndf/epd.h:43-186)
struct EpdNdf
{
  static constexpr int kParams = 2;
  float beta, p, normalization, inv_p;
  // The slots after EPD's parameters (EpdM: 4, 5): glibc's tgammaf(1 / p) computed on the host (host_params<EpdM>)
  // and the p it belongs to.  glibc 2.35's tgammaf is not correctly rounded (it differs from the correctly rounded
  // float on 27 % of the floats in [0.19, 5.1]) and the device library's is a third function again: a normalization
  // an ulp off moved D, and with it eval and pdf, by an ulp on ~4 % of the lanes of a set (EPD[2] of the golden
  // sets).  Where no host value rides along (a probe of the fitting loss, whose parameters are made on the device)
  // the correctly rounded tgamma of the double.
  static constexpr int kGammaSlot = 4;
  __device__ explicit EpdNdf(const float* q) : beta(q[0]), p(q[1])
  {
    // compute_normalization (epd.h:160-178): p InvPi rcp(tgamma(rcp(p))) / beta^2, 0 if p <= eps
    uint32_t tag, pb;
    __builtin_memcpy(&tag, q + kGammaSlot + 1, 4);
    __builtin_memcpy(&pb, &p, 4);
    const float g = (tag == pb && pb != 0u) ? q[kGammaSlot] : float(tgamma(double(div_nr(1.0f, p))));
    const float n = (p > kEpsF) ? (p * kInvPiF) * div_nr(1.0f, g) : 0.0f;
    normalization = div_nr(n, beta * beta);
    inv_p = div_nr(1.0f, p);
  }

  // epd.h:56-73: normalization exp(-pow(tan^2 / beta^2, p)) / cos^4, masked z(h) > 0.  The power is glibc's powf to
  // its last bit (math.hpp): the exponential amplifies a 1-ulp power into x ulps of D (x = the power, up to ~100
  // where D is still normal), and powf_acc -- correctly rounded, where glibc's powf is not always -- left lanes up
  // to 109 ulp apart (7.7e-6 relative) on a rough, high-p parameter set
  __device__ __forceinline__ static float pw(float x, float y)
  {
#ifdef BBM_HIP_EPD_POWF_ACC
    return powf_acc(x, y);              // A/B: the correctly rounded power
#else
    return powf_glibc<true>(x, y);
#endif
  }
  __device__ __forceinline__ float eval(v3 h) const
  {
    const float c2 = h.z * h.z;
    const float t2 = div_nr(1 - c2, c2);
    const float D = div_nr(normalization * expf_lobe(-pw(div_nr(t2, beta * beta), p)), c2 * c2);
    return (h.z > 0) ? D : 0.0f;
  }

  // epd.h:140-152: G1 table at (p, tan(theta_v) beta), masked z(v) > 0 and v.m > 0
  __device__ __forceinline__ float G1(v3 v, v3 m) const
  {
    const bool mask = (v.z > 0) && (dot3(v, m) > 0);
    const float g = epd_g1_lookup(g_epd_g1, p, tan_theta(v) * beta);
    return mask ? g : 0.0f;
  }

  // epd.h:118-134: eval(m) cos(m), masked z(m) > 0 and pdf > 0
  __device__ __forceinline__ float pdf(v3, v3 m, float D) const
  {
    const float q = D * m.z;
    return ((m.z > 0) && (q > 0)) ? q : 0.0f;
  }

  // epd.h:84-106 (Eq. 49-50): phi = 2 pi xi0, tan^2 = beta^2 gamma_q_inv(1/p, xi1)^(1/p)
  __device__ __forceinline__ v3 sample(v3, float xi0, float xi1) const
  {
    if (!((xi0 >= 0) && (xi1 >= 0) && (xi0 <= 1) && (xi1 <= 1))) return mk3(0.0f, 0.0f, 0.0f);
    float sp, cp;
    cossin_cr(kPi2F * xi0, cp, sp);
    const float g = float(gamma_q_inv_d(double(inv_p), double(xi1)));
    const float tan2 = beta * beta * powf_glibc(g, inv_p);      // glibc powf (epd.h:100)
    const float cosT = float(1.0 / sqrt(1.0 + double(tan2)));          // rsqrt(1.0 + tan2) in double, stored as Value
    const float sinT = float(safe_sqrt(1.0 - double(cosT * cosT)));
    return mk3(cp * sinT, sp * sinT, cosT);
  }
};

// maskingshadowing::vanginneken (maskingshadowing/vanginneken.h:30-71), Heitz 2014 Eq. 101
struct VanGinneken
{
  template<class NDF>
  __device__ __forceinline__ static float eval(const NDF& ndf, v3 in, v3 out, v3 m, float inm, float outm)
  {
#ifdef BBM_HIP_EPD_PHI_GLIBC
    // spherical::phi of both directions as the reference's own floats (glibc's atan2f restated, math.hpp): measured
    // 0.234 -> 0.341 ms per 10 M pairs (profiles/r04_ab_models.txt) for bit-identical lanes 0.8345 -> 0.8358 --
    // the G1 table's index map and the NDF's exponentials leave the rest -- so not the default
    const float phi = fabsf(phi_of(in) - phi_of(out));
#else
    // spherical::phi is glibc's atan2f (not correctly rounded); here the device library's f32 atan2 instead: phi only
    // scales lambda (continuously), each phi within ~2 ulp, so G1 moves by <= ~2e-6 relative where the two azimuths
    // nearly cancel and far less elsewhere
    auto phif = [](v3 v) { const float r = atan2f(v.y, v.x); return (r < 0) ? r + kPi2F : r; };
    const float phi = fabsf(phif(in) - phif(out));
#endif
    const float lambda = float(4.41 * double(phi) / (4.41 * double(phi) + 1.0));
    const float gi = ndf.G1(in, m), go = ndf.G1(out, m);
    const float gio = gi * go;
    const float maxg = fmaxf(gi, go), ming = fminf(gi, go);
    const float denom = maxg + lambda * (ming - gio);
    const float g = div_nr(gio, denom);
    return ((inm > 0) && (outm > 0) && (denom > kEpsF)) ? g : 0.0f;
  }
};

// fresnel::complex<Value> (include/bbm/fresnel_complex.h:38-63), Shirley 1985 Eqs. 2.4-2.7: the float
// inputs promote to double at `0.5 * (...)`, so a, Rs, Rp are double; the result is rounded to float.
struct FresnelComplex
{
  static constexpr int kParams = 2;
  float n, k;
  __device__ explicit FresnelComplex(const float* q) : n(q[0]), k(q[1]) {}
  __device__ __forceinline__ float eval(float c) const
  {
    const float c2 = c * c;
    const float s2 = 1 - c2;
    const float n2 = n * n, k2 = k * k;
    const float temp = n2 - k2 - s2;
    const float a2b2 = safe_sqrtf(temp * temp + 4 * n2 * k2);
    const double a = safe_sqrt(0.5 * double(a2b2 + temp));          // float sum, then double
    const double a2c = 2 * a * double(c);
    // Rs and Rp are doubles in the reference (`auto` of double expressions, fresnel_complex.h:47-52), rounded to
    // float once, at the return (rounds 1-4 stored Rs as a float first: EPD's reflectance was then 1 ulp off on
    // ~22 % of the golden lanes); the double quotients by ddiv_nr (within an ulp of IEEE: the one float rounding
    // agrees except within ~2^-28 ulp of a midpoint)
    const double Rs = ddiv_nr(double(a2b2) - a2c + double(c2), double(a2b2) + a2c + double(c2));
    const double ca = double(c2 * a2b2);                               // float product
    const double Rp = ddiv_nr(Rs * (ca - (a2c - double(s2)) * double(s2)), ca + (a2c + double(s2)) * double(s2));
    return float(0.5 * (Rs + Rp));
  }
};

using EpdM = Microfacet<EpdNdf, VanGinneken, FresnelComplex, Norm::Walter, false>;   // holzschuchpacanowski.h:34-42

// Builds the G1 table on the current device once (inst_epd.hip) and points g_epd_g1 at it.
int epd_prepare(hipStream_t s);
template<> struct host_prepare<EpdM> { static int run(hipStream_t s) { return epd_prepare(s); } };
// the host's (glibc's) tgammaf(1 / p) for the normalization, and the p it was computed for (EpdNdf::kGammaSlot)
template<> struct host_params<EpdM>
{
  static_assert(EpdM::kParams == EpdNdf::kGammaSlot, "EPD's gamma slots follow its parameters");
  static int run(ParamBlock& q, uint32_t, hipStream_t, void**)
  {
    const float p = q.v[1];
    q.v[EpdNdf::kGammaSlot] = std::tgamma(1.0f / p);      // tgammaf: float argument, float result
    __builtin_memcpy(&q.v[EpdNdf::kGammaSlot + 1], &p, 4);
    return 0;
  }
  static void done(void*, hipStream_t) {}
};

}  // namespace bbmhip
