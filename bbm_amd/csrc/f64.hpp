// bbm_amd/csrc/f64.hpp -- the doubleRGB configuration on the device (backbone/native/include/backbone.h:41-42:
// Value = double, Spectrum = color<double>).
//
// In doubleRGB every Value of the reference is a double and every literal meets it as a double, so the
// float-semantics machinery of the floatRGB kernels (compensated f32 quotients, float(...) roundings of double
// intermediates, correctly rounded powf) has nothing to reproduce here: these policies restate the reference's
// expressions directly in f64 with the device's IEEE double division / square root and ocml's f64 exp / log /
// pow / tgamma (<= 2 ulp against glibc).  Constants::Epsilon() is the double epsilon (core/constants.h:18).
//
// Covered compositions: Lambertian, OrenNayar, every microfacet<NDF, G, F, N> composition of the floatRGB
// registry (Beckmann / GGX / Phong / Student-T / Low NDFs x v-groove / uncorrelated / height-correlated x Cook /
// Schlick Fresnel), the lobe models (Ward x 5, Phong, Lafortune x 2, Ashikhmin-Shirley x 4, LowSmooth), Bagher, EPD,
// the He family and the Aggregate(Lambertian, X) fits of those: every analytic model.  Layout: SoA f64 (8 B per coordinate), two pairs per
// thread with 16 B loads: 48 B in + 32 B out = 80 B per eval+pdf pair.
#pragma once
#include "math.hpp"
#include "epd.hpp"      // gamma_q_inv_d

// Round-3 defaults, each with an A/B switch back (tools/build_variant_units.sh), measured per 10 M pairs in
// tools/gpu_r03_u.sh (profiles/r03_f64_fdiv_ab.txt):
// * BBM_HIP_F64_FDIV / _MF: the quotients whose operands are provably in range on every lane that keeps its result
//   (Student-T's G1 rationals, 1 / (1 + lambda) and cotangent, the microfacet scale and pdf divisions, the Cook
//   Fresnel, Bagher's reciprocals) as div_fast / rsqrt_fast instead of the IEEE sequences -- Ribardiere 0.250 ->
//   0.220 ms, CookTorrance 0.148 -> 0.144; off with -DBBM_HIP_F64_IEEE_QUOTIENTS
// * BBM_HIP_F64_VPARAM: Bagher's 27 per-channel parameters pinned in VGPRs -- as kernel arguments they exceeded the
//   SGPR file and were spilled into VGPR lanes, one v_readlane per use (1 154 of the two-pairs kernel's 6 113 VALU
//   instructions); Bagher 0.259 -> 0.248 ms; off with -DBBM_HIP_F64_SGPR_PARAMS
#ifndef BBM_HIP_F64_IEEE_QUOTIENTS
#define BBM_HIP_F64_FDIV 1
#define BBM_HIP_F64_FDIV_MF 1
#endif
#ifndef BBM_HIP_F64_SGPR_PARAMS
#define BBM_HIP_F64_VPARAM 1
#endif

namespace bbmhip {
namespace f64 {

constexpr int kMaxParamsF64 = 64;      // parameter block size; the last slot carries the aggregate mode (Aggregate)

constexpr double kEps = 2.220446049250313080847263336181640625e-16;   // numeric_limits<double>::epsilon()
constexpr double kPi = 3.141592653589793115997963468544185161590576171875;          // std::numbers::pi (double)
constexpr double kInvPi = 0.31830988618379069121644420192751567810773849487304688;  // std::numbers::inv_pi

// models whose doubleRGB evaluation is a long f64 computation (the He family's prelude and series, Bagher): launched
// one pair per thread with an occupancy floor of kF64Waves waves per SIMD (f64.hip), where two pairs per thread took
// ~290 VGPRs for He (1 wave per SIMD).  0: the default launch (two pairs per thread, no floor).
template<class M> constexpr int heavy_f64()
{
  if constexpr (requires { M::kF64Waves; }) return M::kF64Waves;
  else return 0;
}
// an occupancy floor for the default two-pairs-per-thread launch (1: none)
template<class M> constexpr int floor_f64()
{
  if constexpr (requires { M::kF64Floor; }) return M::kF64Floor;
  else return 1;
}

struct d3 { double x, y, z; };
__device__ __forceinline__ d3 mk(double x, double y, double z) { return d3{x, y, z}; }
__device__ __forceinline__ double dot(d3 a, d3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
// horizontal.h:106-108: t * rsqrt(squared_norm(t)), rsqrt = 1 / sqrt (math.h:109-112)
__device__ __forceinline__ d3 normalize(d3 v)
{
  const double s = 1.0 / sqrt(dot(v, v));
  return mk(v.x * s, v.y * s, v.z * s);
}
__device__ __forceinline__ double sqnorm2(double x, double y) { return x * x + y * y; }
__device__ __forceinline__ double sin_theta2(d3 v) { return fmax(1.0 - v.z * v.z, 0.0); }   // spherical.h:80
__device__ __forceinline__ double tan_theta(d3 v) { return sqrt(sin_theta2(v)) / v.z; }      // spherical.h:180
__device__ __forceinline__ double tan_theta2(d3 v) { return sin_theta2(v) / (v.z * v.z); }   // spherical.h:186
__device__ __forceinline__ double safe_sqrt(double a) { return sqrt((a < 0.0) ? 0.0 : a); }

// exp / log / pow in double (exp2m1_poly, exp2_d, exp_d, log2_d, exp_lib, log_d, pow_d): math.hpp, shared with the
// floatRGB exact mode

// x^5 for the Schlick / Bagher / Ashikhmin-Shirley factors (1 - c)^5, as glibc's pow(x, 5.0) rounds it: the
// power carried as a double-double through three exact products (two FMA residuals each), rounded once -- the
// correctly rounded x^5 but within ~2^-45 ulp of a midpoint.  These factors feed the reflectance weights that
// pick an aggregate's child at xi0 = 1, where an ulp of a weight decides the pick (tests/test_gpu_f64.py).
__device__ __forceinline__ double pow5_d(double x)
{
#ifdef BBM_HIP_F64_OCML
  return pow(x, 5.0);
#endif
  const double x2 = x * x, e2 = __builtin_fma(x, x, -x2);                                   // x^2 = x2 + e2
  const double x4 = x2 * x2, e4 = __builtin_fma(x2, x2, -x4) + 2.0 * x2 * e2;              // x^4 ~ x4 + e4
  const double x5 = x4 * x, e5 = __builtin_fma(x4, x, -x5) + e4 * x;
  return x5 + e5;
}

__device__ __forceinline__ d3 cross(d3 a, d3 b) { return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
__device__ __forceinline__ bool xi_ok(double xi0, double xi1) { return (xi0 >= 0) && (xi1 >= 0) && (xi0 <= 1) && (xi1 <= 1); }
// spherical.h:156-161 cossinPhi: (1, 0) at the pole, else clamp(xy / sinTheta, -1, 1)
__device__ __forceinline__ void cossin_phi(d3 v, double& c, double& s)
{
  const double sT = sqrt(sin_theta2(v));
  const double r = 1.0 / sT;
  const bool pole = fabs(sT) < kEps;
  c = pole ? 1.0 : fmin(fmax(v.x * r, -1.0), 1.0);
  s = pole ? 0.0 : fmin(fmax(v.y * r, -1.0), 1.0);
}
// n / d for a finite d whose reciprocal is a finite normal double (no IEEE special-case handling): the v_rcp_f64 seed,
// two Newton steps and one remainder correction -- the IEEE quotient or its neighbour (8 instructions against the
// division sequence's 11).  Only where the operands are provably in range on every lane whose result is used.
__device__ __forceinline__ double div_fast(double n, double d)
{
  double r = __builtin_amdgcn_rcp(d);
  r = __builtin_fma(r, __builtin_fma(-d, r, 1.0), r);
  r = __builtin_fma(r, __builtin_fma(-d, r, 1.0), r);
  const double q = n * r;
  return __builtin_fma(__builtin_fma(-d, q, n), r, q);
}
// 1 / sqrt(x) for a finite normal x > 0: the v_rsq_f64 seed and two Goldschmidt steps (g -> sqrt x, h -> 1 / (2 sqrt x)),
// within a few ulp of 1.0 / sqrt(x) against ~23 instructions for the IEEE square root and division
__device__ __forceinline__ double rsqrt_fast(double x)
{
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = 0.5 * y;
  double r = __builtin_fma(-g, h, 0.5);
  g = __builtin_fma(g, r, g); h = __builtin_fma(h, r, h);
  r = __builtin_fma(-g, h, 0.5);
  h = __builtin_fma(h, r, h);
  return 2.0 * h;
}

// the native backbone's erfinv (backbone/native/include/backbone/math.h:115-120, Giles' polynomials) in double
__device__ __forceinline__ double erfinv(double a)
{
  const double w = -log_d((1.0 - a) * (1.0 + a));
  double p;
  if (w < 5)
  {
    const double x = w - 2.5;
    p = 2.81022636e-08;
    p = p * x + 3.43273939e-07; p = p * x + -3.5233877e-06; p = p * x + -4.39150654e-06;
    p = p * x + 0.00021858087; p = p * x + -0.00125372503; p = p * x + -0.00417768164;
    p = p * x + 0.246640727; p = p * x + 1.50140941;
  }
  else
  {
    const double x = sqrt(w) - 3.0;
    p = -0.000200214257;
    p = p * x + 0.000100950558; p = p * x + 0.00134934322; p = p * x + -0.00367342844;
    p = p * x + 0.00573950773; p = p * x + -0.0076224613; p = p * x + 0.00943887047;
    p = p * x + 1.00167406; p = p * x + 2.83297682;
  }
  return p * a;
}
constexpr double kInvSqrtPi = 0.56418958354775627928034964497783221304416656494140625;   // std::numbers::inv_sqrtpi

// Walter's rational approximation of the Smith G1 (beckmann.h:195, phong.h G1)
__device__ __forceinline__ double walter_g1(double a) { return (a < 1.6) ? (3.535 * a + 2.181 * a * a) / (1 + 2.276 * a + 2.577 * a * a) : 1.0; }

// ----------------------------------------------------------------------------------------------------- NDFs

// ndf::beckmann (include/ndf/beckmann.h:49-66 eval, :180-201 G1)
template<bool Aniso, bool Normalize>
struct Beckmann
{
  static constexpr int kParams = Aniso ? 2 : 1;
  double au, av, iau, iav;     // 1 / alpha: the per-pair quotients by the roughness as products (<= 1 ulp apart)
  __device__ explicit Beckmann(const double* p) : au(p[0]), av(Aniso ? p[1] : p[0]), iau(1.0 / au), iav(1.0 / av) {}
  __device__ __forceinline__ double eval(d3 h) const
  {
    const double c2 = h.z * h.z;
    double D = exp_d(-sqnorm2(h.x * iau, h.y * iav) / c2) / (au * av * c2 * c2);
    if (Normalize) D *= kInvPi;
    return (h.z > 0) ? D : 0.0;
  }
  __device__ __forceinline__ double G1(d3 v, d3 m) const
  {
    const bool mask = (v.z > 0) && (dot(v, m) > 0);
    const double a = Aniso ? 1.0 / sqrt(sqnorm2(v.x * au, v.y * av) / (v.z * v.z)) : 1.0 / (au * tan_theta(v));
    return mask ? walter_g1(a) : 0.0;
  }
  // beckmann.h:76-116: visible normals after [Jakob 2014] (stretch, three Newton steps on erfinv, rotate, unstretch)
  __device__ __forceinline__ d3 sample(d3 view, double xi0, double xi1) const
  {
    if (!xi_ok(xi0, xi1)) return mk(0.0, 0.0, 0.0);
    const d3 vs = normalize(mk(view.x * au, view.y * av, view.z));
    const double tanT = tan_theta(vs);
    const double maxval = erf(1.0 / tanT);
    double xc0 = fmin(fmax(xi0, 10e-6), 1.0 - 10e-6);
    const double xc1 = fmin(fmax(xi1, 10e-6), 1.0 - 10e-6);
    double x = maxval - (maxval + 1) * erf(sqrt(-log_d(xc0)));
    xc0 *= 1.0 + maxval + kInvSqrtPi * tanT * exp_d(-(vs.z * vs.z));
    for (int i = 0; i < 3; ++i)
    {
      const double slope = erfinv(x);
      const double val = 1.0 + x + kInvSqrtPi * tanT * exp_d(-slope * slope) - xc0;
      const double der = 1.0 - slope * tanT;
      x -= val / der;
    }
    double s0 = 0.0, s1 = 0.0;
    if (x > -1.0 && x < +1.0) { s0 = erfinv(x); s1 = erfinv(2.0 * xc1 - 1.0); }
    double c, s;
    cossin_phi(vs, c, s);
    const double u0 = (c * s0 + -s * s1) * au, u1 = (s * s0 + c * s1) * av;
    return normalize(mk(-u0, -u1, 1.0));
  }
};

// ndf::ggx (include/ndf/ggx.h:50-65 eval, :173-189 G1)
template<bool Aniso>
struct GGX
{
  static constexpr int kParams = Aniso ? 2 : 1;
  double au, av, iau, iav;     // 1 / alpha (as Beckmann)
  __device__ explicit GGX(const double* p) : au(p[0]), av(Aniso ? p[1] : p[0]), iau(1.0 / au), iav(1.0 / av) {}
  __device__ __forceinline__ double eval(d3 h) const
  {
    const double s = sqnorm2(h.x * iau, h.y * iav) + h.z * h.z;
    const double D = 1.0 / (kPi * (au * av) * (s * s));
    return (h.z > 0) ? D : 0.0;
  }
  __device__ __forceinline__ double G1(d3 v, d3 m) const
  {
    const bool mask = (v.z > 0) && (dot(v, m) > 0);
    const double denom = 1.0 + sqrt(1.0 + (au * av) * tan_theta2(v));
    return mask ? 2.0 / denom : 0.0;
  }
  // ggx.h:84-108: visible normals after [Heitz 2017]
  __device__ __forceinline__ d3 sample(d3 view, double xi0, double xi1) const
  {
    if (!xi_ok(xi0, xi1)) return mk(0.0, 0.0, 0.0);
    const d3 vs = normalize(mk(view.x * au, view.y * av, view.z));
    const d3 T1 = (vs.z < 1.0 - kEps) ? normalize(cross(vs, mk(0.0, 0.0, 1.0))) : mk(1.0, 0.0, 0.0);
    const d3 T2 = cross(T1, vs);
    const double a = 1.0 / (1.0 + vs.z);
    const double r = sqrt(xi0);
    const double phi = ((xi1 < a) ? xi1 / a : 1.0 + (xi1 - a) / (1.0 - a)) * kPi;
    double sp, cp;
    sincos(phi, &sp, &cp);
    const double P1 = r * cp;
    const double P2 = ((xi1 < a) ? 1.0 : vs.z) * r * sp;
    const double sq = safe_sqrt(1.0 - P1 * P1 - P2 * P2);
    const d3 n = mk((P1 * T1.x + P2 * T2.x) + sq * vs.x, (P1 * T1.y + P2 * T2.y) + sq * vs.y, (P1 * T1.z + P2 * T2.z) + sq * vs.z);
    return normalize(mk(n.x * au, n.y * av, fmax(0.0, n.z)));
  }
};

// ndf::phong (include/ndf/phong.h:31-140): D = (s + 2) / (2 pi) cos^s, pdf = D cos, Walter's G1 rational
struct PhongNdf
{
  static constexpr int kParams = 1;
  double sharpness;
  __device__ explicit PhongNdf(const double* p) : sharpness(p[0]) {}
  __device__ __forceinline__ double eval(d3 h) const
  {
    const double D = pow_d(h.z, sharpness) * ((sharpness + 2) / (2.0 * kPi));
    return (h.z > 0) ? D : 0.0;
  }
  __device__ __forceinline__ double G1(d3 v, d3 m) const
  {
    const bool mask = (v.z > 0) && (dot(v, m) > 0);
    return mask ? walter_g1(sqrt(0.5 * sharpness + 1) / tan_theta(v)) : 0.0;
  }
  __device__ __forceinline__ double pdf(d3, d3 m, double D) const { return (m.z > 0) ? D * fabs(m.z) : 0.0; }
  // phong.h:64-79
  __device__ __forceinline__ d3 sample(d3, double xi0, double xi1) const
  {
    if (!xi_ok(xi0, xi1)) return mk(0.0, 0.0, 0.0);
    const double cosT = pow_d(xi0, 1.0 / (sharpness + 2));
    const double sinT = safe_sqrt(1.0 - cosT * cosT);
    double sp, cp;
    sincos(xi1 * (2.0 * kPi), &sp, &cp);
    return mk(cp * sinT, sp * sinT, cosT);
  }
};

// ndf::studentt (include/ndf/studentt.h:34-195), Ribardiere et al. 2017
template<bool Aniso>
struct StudentT
{
  static constexpr int kParams = (Aniso ? 2 : 1) + 1;
  double au, av, gamma, lam_scale, s1_scale, sqrt_g1, f22, f23, iau, iav;
  __device__ explicit StudentT(const double* p) : au(p[0]), av(Aniso ? p[1] : p[0]), gamma(p[Aniso ? 2 : 1])
  {
    iau = 1.0 / au;
    iav = 1.0 / av;
    // parameter-only factors of G1 (studentt.h:152-156), once per thread
    lam_scale = tgamma(gamma - 0.5) / tgamma(gamma) * kInvSqrtPi;
    s1_scale = pow_d(gamma - 1, gamma) / (2 * gamma - 3);
    sqrt_g1 = sqrt(gamma - 1);
    f22 = F22(gamma);
    f23 = F23(gamma);
  }
  __device__ __forceinline__ double eval(d3 h) const
  {
    const double z2 = h.z * h.z;
#ifdef BBM_HIP_F64_FDIV
    // the roughness quotients as products with hoisted reciprocals (<= 1 ulp apart)
    const double den = pow_d(1.0 + sqnorm2(h.x * iau, h.y * iav) / ((gamma - 1) * z2), gamma);
#else
    const double den = pow_d(1.0 + sqnorm2(h.x / au, h.y / av) / ((gamma - 1) * z2), gamma);
#endif
    const double D = 1.0 / (kPi * (au * av) * (z2 * z2) * den);
    return (h.z > 0) ? D : 0.0;
  }
#ifdef BBM_HIP_F64_FDIV
  // F21 / F24 / 1 / (1 + lambda): denominators >= 0.5 on every lane whose G1 is used (z > 0, lambda > -1/2)
  __device__ __forceinline__ static double qdiv(double n, double d) { return div_fast(n, d); }
#else
  __device__ __forceinline__ static double qdiv(double n, double d) { return n / d; }
#endif
  __device__ __forceinline__ static double F21(double z)
  {
    const double z2 = z * z, z3 = z2 * z;
    return qdiv(1.066 * z + 2.655 * z2 + 4.892 * z3, 1.038 + 2.969 * z + 4.305 * z2 + 4.418 * z3);
  }
  __device__ __forceinline__ static double F22(double g)
  {
    const double g2 = g * g, g3 = g2 * g;
    return (14.402 - 27.145 * g + 20.574 * g2 - 2.745 * g3) / (-30.612 + 86.567 * g - 84.341 * g2 + 29.938 * g3);
  }
  __device__ __forceinline__ static double F23(double g)
  {
    const double g2 = g * g, g3 = g2 * g;
    return (-129.404 + 324.987 * g - 299.305 * g2 + 93.268 * g3) / (-92.609 + 256.006 * g - 245.663 * g2 + 86.064 * g3);
  }
  __device__ __forceinline__ static double F24(double z)
  {
    const double z2 = z * z, z3 = z2 * z;
    return qdiv(6.537 + 6.074 * z - 0.623 * z2 + 5.223 * z3, 6.538 + 6.103 * z - 3.218 * z2 + 6.347 * z3);
  }
  // studentt.h:128-156
  __device__ __forceinline__ double G1(d3 v, d3 m) const
  {
    const bool mask = (v.z > 0) && (dot(v, m) > 0);
    const bool normal_mask = v.z < 1.0 - kEps;
#ifdef BBM_HIP_F64_FDIV
    // |v.xy alpha|^2 >= alpha^2 (1 - (1 - eps)^2) > 0 where normal_mask holds (the only lanes whose lambda is used)
    const double z = v.z * rsqrt_fast(sqnorm2(v.x * au, v.y * av));
#else
    const double z = v.z * (1.0 / sqrt(sqnorm2(v.x * au, v.y * av)));
#endif
    const double S1 = pow_d((gamma - 1) + z * z, 1.5 - gamma) / z;
    const double S2 = F21(z) * (f22 + f23 * F24(z));
    const double lambda = normal_mask ? lam_scale * (s1_scale * S1 + sqrt_g1 * S2) - 0.5 : 0.0;
    return mask ? (normal_mask ? qdiv(1.0, 1.0 + lambda) : 1.0) : 0.0;
  }
  __device__ __forceinline__ double pdf(d3, d3 m, double D) const
  {
    const double p = D * m.z;
    return ((m.z > 0) && (p > 0)) ? p : 0.0;
  }
  // studentt.h:67-90
  __device__ __forceinline__ d3 sample(d3, double xi0, double xi1) const
  {
    if (!xi_ok(xi0, xi1)) return mk(0.0, 0.0, 0.0);
    double sp, cp;
    sincos((2.0 * kPi) * xi0, &sp, &cp);
    double normalization;
    if (Aniso)
    {
      normalization = 1.0 / sqnorm2(cp / au, sp / av);
      const double x = cp * au, y = sp * av, r = 1.0 / sqrt(x * x + y * y);
      cp = x * r; sp = y * r;
    }
    else normalization = au * au;
    const double tan2 = (pow_d(xi1, 1.0 / (1.0 - gamma)) - 1) * (gamma - 1) * normalization;
    const double cosT = 1.0 / sqrt(1.0 + tan2);
    const double sinT = safe_sqrt(1.0 - cosT * cosT);
    return mk(cp * sinT, sp * sinT, cosT);
  }
};

// ndf::low (include/ndf/low.h:32-141): the ABC "S" term as an NDF; G1 = 1
struct LowNdf
{
  static constexpr int kParams = 2;
  double B, C, norm_pdf;
  __device__ explicit LowNdf(const double* p) : B(p[0]), C(p[1])
  {
    const double normalization = (fabs(C - 1) < kEps) ? 1.0 / log_d(1.0 + B) : (C - 1.0) / (1.0 - pow_d(1.0 + B, 1.0 - C));
    norm_pdf = 0.5 * kInvPi * normalization;
  }
  // low.h:67-89: inverse of the marginal CDF of cos(theta)
  __device__ __forceinline__ d3 sample(d3, double xi0, double xi1) const
  {
    if (!xi_ok(xi0, xi1)) return mk(0.0, 0.0, 0.0);
    const double term = (fabs(C - 1) < kEps) ? exp_d(xi0 * log_d(1.0 + B)) : pow_d(1.0 + xi0 * (pow_d(1.0 + B, 1.0 - C) - 1.0), -1.0 / (C - 1.0));
    const double cosT = (1.0 + B - term) / B;
    const double sinT = safe_sqrt(1.0 - cosT * cosT);
    double sp, cp;
    sincos(xi1 * (2.0 * kPi), &sp, &cp);
    return mk(cp * sinT, sp * sinT, cosT);
  }
  __device__ __forceinline__ double eval(d3 h) const { return (h.z > 0) ? pow_d(1.0 + B * (1.0 - h.z), -C) : 0.0; }
  __device__ __forceinline__ double G1(d3, d3) const { return 1.0; }
  // low.h:96-112
  __device__ __forceinline__ double pdf(d3, d3, double D) const
  {
    const double p = D * B * norm_pdf;
    return (p > 0) ? p : 0.0;
  }
};

// visible-normal pdf of Beckmann / GGX (beckmann.h:149-170, ggx.h:142-163): D G1(view, m) |view.m| / cos(view)
template<class NDF>
__device__ __forceinline__ double vndf_pdf(const NDF& ndf, d3 view, d3 m, double D)
{
  const double p = D * (ndf.G1(view, m) * fabs(dot(view, m)) / view.z);
  return ((m.z > 0) && (p > 0)) ? p : 0.0;
}
template<class NDF> struct ndf_pdf { __device__ static double run(const NDF& n, d3 v, d3 m, double D) { return n.pdf(v, m, D); } };
template<bool A, bool N> struct ndf_pdf<Beckmann<A, N>>
{ __device__ static double run(const Beckmann<A, N>& n, d3 v, d3 m, double D) { return vndf_pdf(n, v, m, D); } };
template<bool A> struct ndf_pdf<GGX<A>>
{ __device__ static double run(const GGX<A>& n, d3 v, d3 m, double D) { return vndf_pdf(n, v, m, D); } };

// ---------------------------------------------------------------------------------------- masking-shadowing

// maskingshadowing::vgroove (vgroove.h:30-47)
struct VGroove
{
  template<class NDF>
  __device__ __forceinline__ static double eval(const NDF&, d3 in, d3 out, d3 m, double inm, double outm)
  {
    const double G = fmin(1.0, fmin(2.0 * m.z * in.z / inm, 2.0 * m.z * out.z / outm));
    return ((inm > 0) && (outm > 0)) ? G : 0.0;
  }
};

// maskingshadowing::uncorrelated (uncorrelated.h:30-42)
struct Uncorrelated
{
  template<class NDF>
  __device__ __forceinline__ static double eval(const NDF& ndf, d3 in, d3 out, d3 m, double inm, double outm)
  {
    const double g = ndf.G1(in, m) * ndf.G1(out, m);
    return ((inm > 0) && (outm > 0)) ? g : 0.0;
  }
};

// maskingshadowing::heightcorrelated (heightcorrelated.h:30-54)
struct HeightCorrelated
{
  template<class NDF>
  __device__ __forceinline__ static double eval(const NDF& ndf, d3 in, d3 out, d3 m, double inm, double outm)
  {
    const double gi = ndf.G1(in, m), go = ndf.G1(out, m);
    const double gio = gi * go;
    const double denom = gi + go - gio;
    return ((inm > 0) && (outm > 0) && (denom > kEps)) ? gio / denom : 0.0;
  }
};

// ------------------------------------------------------------------------------------------------- fresnel

// fresnel::cook (bbm/fresnel_cook.h:41-56)
struct FresnelCook
{
  static constexpr int kParams = 1;
  double eta;
  __device__ explicit FresnelCook(const double* p) : eta(p[0]) {}
  __device__ __forceinline__ double eval(double c) const
  {
    const double g = safe_sqrt(eta * eta + c * c - 1.0);
#ifdef BBM_HIP_F64_FDIV_MF
    // eta >= 1: g >= |c|, so g + c >= 0 and c (g - c) + 1 >= 1 - c^2 + c g > 0 for c in [0, 1] (0 / 0 -> NaN either way)
    const double a = div_fast(g - c, g + c);
    const double b = div_fast(c * (g + c) - 1.0, c * (g - c) + 1.0);
#else
    const double a = (g - c) / (g + c);
    const double b = (c * (g + c) - 1.0) / (c * (g - c) + 1.0);
#endif
    return fmax(0.5 * (a * a) * (1.0 + b * b), 0.0);
  }
};

// fresnel::schlick (bbm/fresnel_schlick.h:42-53): R0 + (1 - R0) pow(1 - cos, 5)
struct FresnelSchlick
{
  static constexpr int kParams = 1;
  double r0;
  __device__ explicit FresnelSchlick(const double* p) : r0(p[0]) {}
  __device__ __forceinline__ double eval(double c) const { return r0 + (1.0 - r0) * pow5_d(1.0 - c); }
};

// ----------------------------------------------------------------------------------------------- models

enum class Norm { One, Walter, Cook };
template<Norm N> struct norm_value;
template<> struct norm_value<Norm::One> { static constexpr double v = 1.0; };
template<> struct norm_value<Norm::Walter> { static constexpr double v = 4.0; };
template<> struct norm_value<Norm::Cook> { static constexpr double v = kPi; };

// microfacet<NDF, MS, F, N> (bsdfmodel/microfacet.h:74-196), x albedo when Scaled (scaledmodel.h:50-67)
template<class NDF, class MS, class FRESNEL, Norm N, bool Scaled>
struct Microfacet
{
  static constexpr int kParams = (Scaled ? 3 : 0) + NDF::kParams + FRESNEL::kParams;
  static constexpr uint32_t kComponent = kFlagSpecular;
  double albedo[3];
  NDF ndf;
  FRESNEL fresnel;
  __device__ explicit Microfacet(const double* p) : ndf(p + (Scaled ? 3 : 0)), fresnel(p + (Scaled ? 3 : 0) + NDF::kParams)
  {
    albedo[0] = Scaled ? p[0] : 1.0;
    albedo[1] = Scaled ? p[1] : 1.0;
    albedo[2] = Scaled ? p[2] : 1.0;
  }

  // eval :74-102 and pdf :154-174 share the halfway vector and D(h); both test Specular, z_in > 0, z_out > 0
  __device__ __forceinline__ void eval_pdf(d3 in, d3 out, uint32_t component, double* rgb, double& pdf) const
  {
    const bool active = (component & kFlagSpecular) && (in.z > 0) && (out.z > 0);
    // the halfway vector keeps the IEEE 1 / sqrt: a last-ulp h.z above 1 (in + out along z) would make 1 - z^2 < 0
    const d3 h = normalize(mk(in.x + out.x, in.y + out.y, in.z + out.z));
    const double D = ndf.eval(h);
    const double inh = dot(in, h), outh = dot(out, h);
    const double G = MS::eval(ndf, in, out, h, inh, outh);
    const double F = fresnel.eval(0.5 * (inh + outh));
#ifdef BBM_HIP_F64_FDIV_MF
    // z_in z_out > 0 and |out.h| > 0 on active lanes (the only ones whose results are kept); the pdf's 0 / 0 where
    // out.h = 0 stays NaN either way
    const double res = div_fast(D * G * F / norm_value<N>::v, in.z * out.z);
#pragma unroll
    for (int c = 0; c < 3; ++c) rgb[c] = active ? (Scaled ? res * albedo[c] : res) : 0.0;
    pdf = active ? div_fast(ndf_pdf<NDF>::run(ndf, out, h, D), 4.0 * fabs(outh)) : 0.0;
#else
    const double res = D * G * F / norm_value<N>::v / (in.z * out.z);
#pragma unroll
    for (int c = 0; c < 3; ++c) rgb[c] = active ? (Scaled ? res * albedo[c] : res) : 0.0;
    // the pdf's `h = z(h) < 0 ? -h : h` (:167) never fires on active lanes
    pdf = active ? ndf_pdf<NDF>::run(ndf, out, h, D) / (4.0 * fabs(outh)) : 0.0;
#endif
  }

  // :115-141: m ~ NDF sample(out), direction = reflect(out, m) = m (m.out) 2.0 - out (core/vec_transform.h:43-44),
  // pdf = pdf(direction, out), flag Specular
  __device__ __forceinline__ void sample(d3 out, double xi0, double xi1, uint32_t component, d3& dir, double& pdf,
                                         uint32_t& flag) const
  {
    dir = mk(0.0, 0.0, 0.0);
    pdf = 0.0;
    flag = kFlagNone;
    if (!(component & kFlagSpecular) || !xi_ok(xi0, xi1) || !(out.z > 0)) return;
    const d3 m = ndf.sample(out, xi0, xi1);
    const double d = dot(m, out);
    dir = mk(m.x * d * 2.0 - out.x, m.y * d * 2.0 - out.y, m.z * d * 2.0 - out.z);
    double rgb[3];
    eval_pdf(dir, out, component, rgb, pdf);
    flag = kFlagSpecular;
  }

  // :182-196 mirror approximation Fresnel(eta, z(out)) / N * 4.0, x albedo
  __device__ __forceinline__ void reflectance(d3 out, uint32_t component, double* rgb) const
  {
    const bool m = (component & kFlagSpecular) && (out.z > 0);
    const double f = fresnel.eval(out.z) / norm_value<N>::v * 4.0;
#pragma unroll
    for (int c = 0; c < 3; ++c) rgb[c] = m ? (Scaled ? f * albedo[c] : f) : 0.0;
  }
};

// bbm::lambertian (bsdfmodel/lambertian.h:45-59 eval, :115-125 pdf, :136-140 reflectance)
struct Lambertian
{
  static constexpr int kParams = 3;
  static constexpr uint32_t kComponent = kFlagDiffuse;
  double albedo[3];
  __device__ explicit Lambertian(const double* p) { albedo[0] = p[0]; albedo[1] = p[1]; albedo[2] = p[2]; }
  __device__ __forceinline__ void eval_pdf(d3 in, d3 out, uint32_t component, double* rgb, double& pdf) const
  {
    const bool m = (component & kFlagDiffuse) && (in.z >= 0) && (out.z >= 0);
#pragma unroll
    for (int c = 0; c < 3; ++c) rgb[c] = m ? albedo[c] * kInvPi : 0.0;
    pdf = m ? in.z * kInvPi : 0.0;
  }
  __device__ __forceinline__ void reflectance(d3, uint32_t component, double* rgb) const
  {
    const bool m = component & kFlagDiffuse;
#pragma unroll
    for (int c = 0; c < 3; ++c) rgb[c] = m ? albedo[c] : 0.0;
  }
  // lambertian.h:76-103: cosine-weighted directions
  __device__ __forceinline__ void sample(d3 out, double xi0, double xi1, uint32_t component, d3& dir, double& pdf,
                                         uint32_t& flag) const
  {
    dir = mk(0.0, 0.0, 0.0);
    pdf = 0.0;
    flag = kFlagNone;
    if (!(component & kFlagDiffuse) || !xi_ok(xi0, xi1)) return;
    double s, c;
    sincos(xi0 * (2.0 * kPi), &s, &c);
    const double sinT = safe_sqrt(1.0 - xi1);
    dir = mk(c * sinT, s * sinT, safe_sqrt(xi1));
    const bool m = (dir.z >= 0) && (out.z >= 0);
    pdf = m ? dir.z * kInvPi : 0.0;
    flag = kFlagDiffuse;
  }
};

// bbm::orennayar (bsdfmodel/orennayar.h:45-137); sample / pdf are Lambertian's
struct OrenNayar
{
  static constexpr int kParams = 4;
  static constexpr uint32_t kComponent = kFlagDiffuse;
  double albedo[3], A, B;
  __device__ explicit OrenNayar(const double* p)
  {
    albedo[0] = p[0]; albedo[1] = p[1]; albedo[2] = p[2];
    const double sigma2 = p[3] * p[3];
    A = 1 - 0.5 * sigma2 / (sigma2 + 0.33);
    B = 0.45 * sigma2 / (sigma2 + 0.09);
  }
  __device__ __forceinline__ void eval_pdf(d3 in, d3 out, uint32_t component, double* rgb, double& pdf) const
  {
    const bool diff = component & kFlagDiffuse;
    const bool m = diff && (in.z > 0) && (out.z > 0);
    const double factor = A + (B * fmax((in.x * out.x) + (in.y * out.y), 0.0) / fmax(in.z, out.z));
#pragma unroll
    for (int c = 0; c < 3; ++c) rgb[c] = m ? albedo[c] / kPi * factor : 0.0;
    pdf = (diff && (in.z >= 0) && (out.z >= 0)) ? in.z * kInvPi : 0.0;
  }
  __device__ __forceinline__ void reflectance(d3, uint32_t component, double* rgb) const
  {
    const bool m = component & kFlagDiffuse;
#pragma unroll
    for (int c = 0; c < 3; ++c) rgb[c] = m ? albedo[c] : 0.0;
  }
  __device__ __forceinline__ void sample(d3 out, double xi0, double xi1, uint32_t component, d3& dir, double& pdf,
                                         uint32_t& flag) const
  {
    const double one[3] = {1.0, 1.0, 1.0};
    Lambertian(one).sample(out, xi0, xi1, component, dir, pdf, flag);
  }
};

// aggregatemodel<A, B> (bsdfmodel/aggregatemodel.h:60-163): eval and reflectance sum (right folds of two
// children), pdf = (w_A pdf_A + w_B pdf_B) / (w_A + w_B) with w = hsum(reflectance(out)), 0 if the sum <= eps
template<class A, class B>
struct Aggregate
{
  static constexpr int kParams = A::kParams + B::kParams;
  static constexpr uint32_t kComponent = A::kComponent | B::kComponent;
  static constexpr int kF64Waves = heavy_f64<A>() > heavy_f64<B>() ? heavy_f64<A>() : heavy_f64<B>();
  A a;
  B b;
  bool runtime;            // aggregatebsdf semantics (bbm_amd/csrc/aggregate.hpp): the parameter block's last slot
  __device__ explicit Aggregate(const double* p) : a(p), b(p + A::kParams), runtime(p[kMaxParamsF64 - 1] != 0.0) {}
  __device__ __forceinline__ void eval_pdf(d3 in, d3 out, uint32_t component, double* rgb, double& pdf) const
  {
    double ra[3], rb[3], pa, pb;
    a.eval_pdf(in, out, component, ra, pa);
    b.eval_pdf(in, out, component, rb, pb);
#pragma unroll
    for (int c = 0; c < 3; ++c) rgb[c] = ra[c] + rb[c];
    double wa, wb;
    weights(out, component, wa, wb);
    pdf = component ? mix(pa, pb, wa, wb) : 0.0;
  }
  // hsum(reflectance(out)) per child (horizontal.h:64-67)
  __device__ __forceinline__ void weights(d3 out, uint32_t component, double& wa, double& wb) const
  {
    double ra[3], rb[3];
    a.reflectance(out, component, ra);
    b.reflectance(out, component, rb);
    wa = ((0.0 + ra[0]) + ra[1]) + ra[2];
    wb = ((0.0 + rb[0]) + rb[1]) + rb[2];
  }
  // inner_product(pdfs, weights, 0) / sum, masked sum > eps (:141-142); aggregatebsdf: w_k pdf_k / sum per term
  __device__ __forceinline__ double mix(double pa, double pb, double wa, double wb) const
  {
    const double sum = (0.0 + wa) + wb;
    if (!(sum > kEps)) return 0.0;
    if (runtime) return (0.0 + wa * pa / sum) + wb * pb / sum;
    return ((0.0 + pa * wa) + pb * wb) / sum;
  }
  // :81-113: the child claiming xi0 * sum (a later child that also claims it wins), pdf of the mixture
  __device__ __forceinline__ void sample(d3 out, double xi0, double xi1, uint32_t component, d3& dir, double& pdf,
                                         uint32_t& flag) const
  {
    dir = mk(0.0, 0.0, 0.0);
    pdf = 0.0;
    flag = kFlagNone;
    if (!component) return;
    double wa, wb, p;
    weights(out, component, wa, wb);
    if (runtime && !((0.0 + wa) + wb > kEps)) return;      // aggregatebsdf's bail-out (aggregatebsdf.h:115-116)
    double x = xi0 * ((0.0 + wa) + wb);
    if ((x >= 0) && (x <= wa)) a.sample(out, (wa > kEps) ? x / wa : 0.0, xi1, component, dir, p, flag);
    x -= wa;
    if ((x >= 0) && (x <= wb)) b.sample(out, (wb > kEps) ? x / wb : 0.0, xi1, component, dir, p, flag);
    double rgb[3], pa, pb;
    a.eval_pdf(dir, out, component, rgb, pa);
    b.eval_pdf(dir, out, component, rgb, pb);
    pdf = mix(pa, pb, wa, wb);
  }
  __device__ __forceinline__ void reflectance(d3 out, uint32_t component, double* rgb) const
  {
    double ra[3], rb[3];
    a.reflectance(out, component, ra);
    b.reflectance(out, component, rb);
#pragma unroll
    for (int c = 0; c < 3; ++c) rgb[c] = ra[c] + rb[c];
  }
};

// ------------------------------------------------------------------------------------------ lobe models

__device__ __forceinline__ d3 reflect(d3 out, d3 m)     // core/vec_transform.h:43-44
{
  const double d = dot(m, out);
  return mk(m.x * d * 2.0 - out.x, m.y * d * 2.0 - out.y, m.z * d * 2.0 - out.z);
}

// toGlobalShadingFrame(normal) * v (core/shading_frame.h:24-48, Duff et al. 2017)
__device__ __forceinline__ d3 to_global(d3 normal, d3 v)
{
  const d3 Z = normalize(normal);
  const double sign = copysign(1.0, Z.z);
  const double a = -1.0 / (sign + Z.z);
  const double b = Z.x * Z.y * a;
  const d3 X = mk(1.0 + sign * Z.x * Z.x * a, sign * b, -sign * Z.x);
  const d3 Y = mk(b, sign + Z.y * Z.y * a, -Z.y);
  return mk(((0.0 + X.x * v.x) + Y.x * v.y) + Z.x * v.z, ((0.0 + X.y * v.x) + Y.y * v.y) + Z.y * v.z,
            ((0.0 + X.z * v.x) + Y.z * v.y) + Z.z * v.z);
}

#define BBM_F64_SAMPLE_PROLOGUE                          \
  dir = mk(0.0, 0.0, 0.0); pdf = 0.0; flag = kFlagNone;  \
  if (!((component & kFlagSpecular) && xi_ok(xi0, xi1))) return;

// Ward (ward.h:26-168, KIND 0), Ward-Duer (wardduer.h:29-81, KIND 1), Ward-Duer-Geisler-Moroder
// (wardduergeislermoroder.h:29-81, KIND 2); isotropic: NganWard / NganWardDuer (ngan.h:30-38)
template<int KIND, bool Aniso>
struct Ward
{
  static constexpr int kParams = 3 + (Aniso ? 2 : 1);
  static constexpr uint32_t kComponent = kFlagSpecular;
  double albedo[3], rx, ry;
  __device__ explicit Ward(const double* p) : rx(p[3]), ry(Aniso ? p[4] : p[3]) { albedo[0] = p[0]; albedo[1] = p[1]; albedo[2] = p[2]; }
  __device__ __forceinline__ void eval_pdf(d3 in, d3 out, uint32_t component, double* rgb, double& pdf) const
  {
    const bool active = (component & kFlagSpecular) && (in.z >= 0) && (out.z >= 0);
    const d3 H = mk(in.x + out.x, in.y + out.y, in.z + out.z);
    const double zH2 = H.z * H.z;
    const double exponent = sqnorm2(H.x / rx, H.y / ry) / zH2;
    double nf;
    if (KIND == 0) nf = 4.0 * kPi * sqrt(in.z * out.z) * rx * ry;
    else if (KIND == 1) nf = 4.0 * kPi * rx * ry * (in.z * out.z);
    else nf = 4.0 * kPi * rx * ry * (zH2 * zH2) / dot(H, H);
    const double f = exp_d(-exponent) / nf;
#pragma unroll
    for (int c = 0; c < 3; ++c) rgb[c] = active ? albedo[c] * f : 0.0;
    // ward.h:126-140
    const d3 h = normalize(H);
    const double np = 4.0 * kPi * rx * ry * dot(in, h) * (h.z * h.z * h.z);
    pdf = active ? exp_d(-(sqnorm2(h.x / rx, h.y / ry) / (h.z * h.z))) / np : 0.0;
  }
  __device__ __forceinline__ void reflectance(d3, uint32_t component, double* rgb) const
  {
    const bool m = component & kFlagSpecular;
#pragma unroll
    for (int c = 0; c < 3; ++c) rgb[c] = m ? albedo[c] : 0.0;
  }
  // ward.h:90-110
  __device__ __forceinline__ void sample(d3 out, double xi0, double xi1, uint32_t component, d3& dir, double& pdf,
                                         uint32_t& flag) const
  {
    BBM_F64_SAMPLE_PROLOGUE
    double s, c;
    sincos(2.0 * kPi * xi0, &s, &c);
    const double cx = c * rx, cy = s * ry, r = 1.0 / sqrt(sqnorm2(cx, cy));
    const double csx = cx * r, csy = cy * r;
    const double cosT = 1.0 / sqrt(1.0 - (log_d(xi1) / sqnorm2(csx / rx, csy / ry)));
    const double sinT = safe_sqrt(1.0 - cosT * cosT);
    dir = reflect(out, mk(csx * sinT, csy * sinT, cosT));
    double rgb[3];
    eval_pdf(dir, out, component, rgb, pdf);
    flag = kFlagSpecular;
  }
};

// Phong lobe about reflect(in) (bsdfmodel/phong.h:25-163; NganBlinnPhong, ngan.h:43-44)
struct PhongLobe
{
  static constexpr int kParams = 4;
  static constexpr uint32_t kComponent = kFlagSpecular;
  double albedo[3], s;
  __device__ explicit PhongLobe(const double* p) : s(p[3]) { albedo[0] = p[0]; albedo[1] = p[1]; albedo[2] = p[2]; }
  __device__ __forceinline__ void eval_pdf(d3 in, d3 out, uint32_t component, double* rgb, double& pdf) const
  {
    const bool active = (component & kFlagSpecular) && (in.z >= 0) && (out.z >= 0);
    const double pw = pow_d(fmax(dot(mk(-in.x, -in.y, in.z), out), 0.0), s);
    const double f = (s + 2) * (0.5 * kInvPi) * pw;
#pragma unroll
    for (int c = 0; c < 3; ++c) rgb[c] = active ? albedo[c] * f : 0.0;
    pdf = active ? (s + 1) * (0.5 * kInvPi) * pw : 0.0;
  }
  __device__ __forceinline__ void reflectance(d3, uint32_t component, double* rgb) const
  {
    const bool m = component & kFlagSpecular;
#pragma unroll
    for (int c = 0; c < 3; ++c) rgb[c] = m ? albedo[c] : 0.0;
  }
  __device__ __forceinline__ void sample(d3 out, double xi0, double xi1, uint32_t component, d3& dir, double& pdf,
                                         uint32_t& flag) const
  {
    BBM_F64_SAMPLE_PROLOGUE
    double sp, cp;
    sincos(xi0 * (2.0 * kPi), &sp, &cp);
    const double cosT = pow_d(xi1, 1.0 / (s + 1));
    const double sinT = safe_sqrt(1.0 - cosT * cosT);
    dir = to_global(mk(-out.x, -out.y, out.z), mk(cp * sinT, sp * sinT, cosT));
    double rgb[3];
    eval_pdf(dir, out, component, rgb, pdf);
    flag = kFlagSpecular;
  }
};

// Lafortune (bsdfmodel/lafortune.h:28-172) and Ngan's normalised isotropic lobe (ngan.h:54-129)
template<bool Aniso, bool NGAN>
struct Lafortune
{
  static constexpr int kParams = 3 + (Aniso ? 2 : 1) + 2;
  static constexpr uint32_t kComponent = kFlagSpecular;
  double albedo[3], cx, cy, cz, s, ngan;
  __device__ explicit Lafortune(const double* p) : cx(p[3]), cy(Aniso ? p[4] : p[3]), cz(p[Aniso ? 5 : 4]), s(p[Aniso ? 6 : 5])
  {
    albedo[0] = p[0]; albedo[1] = p[1]; albedo[2] = p[2];
    ngan = NGAN ? (s + 2.0) * (0.5 * kInvPi) / pow_d(fmax(cz * cz, cx * cx), s * 0.5) : 1.0;
  }
  __device__ __forceinline__ void eval_pdf(d3 in, d3 out, uint32_t component, double* rgb, double& pdf) const
  {
    const bool ev = (component & kFlagSpecular) && (in.z > 0) && (out.z > 0);
    const double fr = pow_d(fmax(dot(mk(cx, cy, cz), mk(in.x * out.x, in.y * out.y, in.z * out.z)), 0.0), s);
#pragma unroll
    for (int c = 0; c < 3; ++c) rgb[c] = ev ? (NGAN ? albedo[c] * fr * ngan : albedo[c] * fr) : 0.0;
    const bool pd = (component & kFlagSpecular) && (in.z >= 0) && (out.z >= 0);
    const d3 co = normalize(mk(cx * out.x, cy * out.y, cz * out.z));
    pdf = pd ? (s + 1) / (2.0 * kPi) * pow_d(fmax(dot(co, in), 0.0), s) : 0.0;
  }
  __device__ __forceinline__ void reflectance(d3 out, uint32_t component, double* rgb) const
  {
    const bool m = component & kFlagSpecular;
    const d3 co = mk(cx * out.x, cy * out.y, cz * out.z);
    const double normalization = pow_d(sqrt(dot(co, co)), s) * (2.0 * kPi) / (s + 2);
#pragma unroll
    for (int c = 0; c < 3; ++c) rgb[c] = m ? (NGAN ? albedo[c] * normalization * ngan : albedo[c] * normalization) : 0.0;
  }
  __device__ __forceinline__ void sample(d3 out, double xi0, double xi1, uint32_t component, d3& dir, double& pdf,
                                         uint32_t& flag) const
  {
    BBM_F64_SAMPLE_PROLOGUE
    double sp, cp;
    sincos(xi0 * (2.0 * kPi), &sp, &cp);
    const double cosT = pow_d(xi1, 1.0 / (s + 1));
    const double sinT = safe_sqrt(1.0 - cosT * cosT);
    dir = to_global(mk(cx * out.x, cy * out.y, cz * out.z), mk(cp * sinT, sp * sinT, cosT));
    double rgb[3];
    eval_pdf(dir, out, component, rgb, pdf);
    flag = kFlagSpecular;
  }
};

// Schlick with a Spectrum reflectance (fresnel_schlick.h:42-53, per channel); ScalarFresnel3: a scalar Fresnel
// broadcast to the three channels
struct FresnelSchlickRGB
{
  static constexpr int kParams = 3;
  double r0[3];
  __device__ explicit FresnelSchlickRGB(const double* p) { r0[0] = p[0]; r0[1] = p[1]; r0[2] = p[2]; }
  __device__ __forceinline__ void eval3(double c, double* F) const
  {
    const double x5 = pow5_d(1.0 - c);
#pragma unroll
    for (int k = 0; k < 3; ++k) F[k] = r0[k] + (1.0 - r0[k]) * x5;
  }
  __device__ __forceinline__ double hsum() const { return ((0.0 + r0[0]) + r0[1]) + r0[2]; }
};
template<class F>
struct ScalarFresnel3 : F
{
  __device__ explicit ScalarFresnel3(const double* p) : F(p) {}
  __device__ __forceinline__ void eval3(double c, double* out) const { out[0] = out[1] = out[2] = F::eval(c); }
};

// Ashikhmin-Shirley (ashikhminshirley.h:29-221), the scaled Low / Ngan variants (low.h:24-25, ngan.h:157-158) and
// the full model with its coupled diffuse term (ashikhminshirleyfull.h:31-191)
template<class FRES, bool Aniso, bool SCALED, bool FULL>
struct AshikhminShirley
{
  static constexpr int kOff = (SCALED ? 3 : 0) + (FULL ? 3 : 0);
  static constexpr int kParams = kOff + FRES::kParams + (Aniso ? 2 : 1);
  static constexpr uint32_t kComponent = FULL ? kFlagAll : kFlagSpecular;
  double albedo[3], diffuse[3], su, sv;
  FRES fres;
  __device__ explicit AshikhminShirley(const double* p)
      : su(p[kOff + FRES::kParams]), sv(p[kOff + FRES::kParams + (Aniso ? 1 : 0)]), fres(p + kOff)
  {
#pragma unroll
    for (int k = 0; k < 3; ++k) { albedo[k] = SCALED ? p[k] : 1.0; diffuse[k] = FULL ? p[k] : 0.0; }
  }
  __device__ __forceinline__ double exponent(d3 h) const
  {
    if (!Aniso) return su;
    return (h.z < 1.0 - kEps) ? (su * (h.x * h.x) + sv * (h.y * h.y)) / (1.0 - h.z * h.z) : 0.0;
  }
  // ashikhminshirley.h:148-176
  __device__ __forceinline__ double spec_pdf(d3 in, d3 out, uint32_t component) const
  {
    const bool active = (component & kFlagSpecular) && (in.z >= 0) && (out.z >= 0);
    const d3 h = normalize(mk(in.x + out.x, in.y + out.y, in.z + out.z));
    const double normalization = Aniso ? sqrt((su + 1) * (sv + 1)) / (2.0 * kPi) : (su + 1.0) / (2.0 * kPi);
    return active ? normalization * pow_d(h.z, exponent(h)) / (4.0 * dot(h, in)) : 0.0;
  }
  __device__ __forceinline__ double diff_albedo() const
  {
    return (((0.0 + diffuse[0]) + diffuse[1]) + diffuse[2]) * (1.0 - fres.hsum());
  }
  __device__ __forceinline__ void eval_pdf(d3 in, d3 out, uint32_t component, double* rgb, double& pdf) const
  {
    const bool upper = (in.z > 0) && (out.z > 0);
    const bool spec = (component & kFlagSpecular) && upper;
    const d3 h = normalize(mk(in.x + out.x, in.y + out.y, in.z + out.z));
    const double hdi = dot(h, in);
    double F[3];
    fres.eval3(hdi, F);
    const double normalization = Aniso ? sqrt((su + 1) * (sv + 1)) / (8.0 * kPi) : (su + 1) / (8.0 * kPi);
    const double np = normalization * pow_d(h.z, exponent(h));
    const double denom = hdi * fmax(in.z, out.z);
    double diff_scale = 0.0;
    if constexpr (FULL)
      diff_scale = 28.0 / (23.0 * kPi) * ((1.0 * (1.0 - pow5_d(1.0 - 0.5 * in.z))) * (1.0 - pow5_d(1.0 - 0.5 * out.z)));
    const bool diff = FULL && (component & kFlagDiffuse) && upper;
#pragma unroll
    for (int c = 0; c < 3; ++c)
    {
      double v = np * F[c] / denom;
      if (SCALED) v *= albedo[c];
      v = spec ? v : 0.0;
      if constexpr (FULL) v = diff ? (diff_scale * diffuse[c] * (1.0 - fres.r0[c])) + v : v;
      rgb[c] = upper ? v : 0.0;
    }
    const double sp = spec_pdf(in, out, component);
    if constexpr (FULL)
    {
      // ashikhminshirleyfull.h:148-168
      const double dpdf = ((component & kFlagDiffuse) && (in.z >= 0) && (out.z >= 0)) ? in.z * kInvPi : 0.0;
      const double da = diff_albedo(), sa = fres.hsum();
      const double dw = (da > kEps) ? da / (da + sa) : 0.0;
      const double sw = 1.0 - dw;
      pdf = !(component & kFlagDiffuse) ? sp : (!(component & kFlagSpecular) ? dpdf : sw * sp + dw * dpdf);
    }
    else pdf = sp;
  }
  // ashikhminshirley.h:181-190 (+ ashikhminshirleyfull.h:170-185)
  __device__ __forceinline__ void reflectance(d3 out, uint32_t component, double* rgb) const
  {
    const bool up = out.z > 0;
    const bool ms = (component & kFlagSpecular) && up;
    double F[3];
    fres.eval3(out.z, F);
#pragma unroll
    for (int c = 0; c < 3; ++c)
    {
      double v = ms ? (SCALED ? F[c] * albedo[c] : F[c]) : 0.0;
      if constexpr (FULL) v = (up && (component & kFlagDiffuse)) ? diffuse[c] * (1.0 - fres.r0[c]) + v : v;
      rgb[c] = up ? v : 0.0;
    }
  }
  // ashikhminshirley.h:98-140
  __device__ __forceinline__ void spec_sample(d3 out, double xi0, double xi1, uint32_t component, d3& dir, double& pdf,
                                              uint32_t& flag) const
  {
    BBM_F64_SAMPLE_PROLOGUE
    double cp, sp, cosT;
    if (Aniso)
    {
      double phi = atan(sqrt((su + 1.0) / (sv + 1.0)) * tan(xi0 * (2.0 * kPi)));
      phi = ((xi0 > 0.25) && (xi0 < 0.75)) ? phi + kPi : phi;
      sincos(phi, &sp, &cp);
      cosT = pow_d(xi1, 1.0 / ((su * (cp * cp)) + (sv * (sp * sp)) + 1.0));
    }
    else
    {
      sincos(xi0 * (2.0 * kPi), &sp, &cp);
      cosT = pow_d(xi1, 1.0 / (su + 1.0));
    }
    const double sinT = safe_sqrt(1.0 - cosT * cosT);
    dir = reflect(out, mk(cp * sinT, sp * sinT, cosT));
    pdf = spec_pdf(dir, out, component);
    flag = kFlagSpecular;
  }
  __device__ __forceinline__ void sample(d3 out, double xi0, double xi1, uint32_t component, d3& dir, double& pdf,
                                         uint32_t& flag) const
  {
    if constexpr (!FULL) { spec_sample(out, xi0, xi1, component, dir, pdf, flag); return; }
    else {
    if (!(component & kFlagDiffuse)) { spec_sample(out, xi0, xi1, component, dir, pdf, flag); return; }
    const double one[3] = {1.0, 1.0, 1.0};
    const Lambertian lam(one);
    if (!(component & kFlagSpecular)) { lam.sample(out, xi0, xi1, component, dir, pdf, flag); return; }
    // ashikhminshirleyfull.h:96-124: one-sample mixture of the specular lobe and cosine sampling
    const double da = diff_albedo(), sa = fres.hsum();
    const double dw = da / (da + sa), sw = 1.0 - dw;
    d3 ds, dd; double ps, pd; uint32_t fs, fd;
    spec_sample(out, (sw > kEps) ? xi0 / sw : 0.0, xi1, component, ds, ps, fs);
    lam.sample(out, (dw > kEps) ? (xi0 - sw) / dw : 0.0, xi1, component, dd, pd, fd);
    const bool pick_s = xi0 <= sw;
    dir = pick_s ? ds : dd;
    flag = pick_s ? fs : fd;
    pdf = sw * ps + dw * pd;
    }
  }
};

// Low et al.'s smooth-surface model (bsdfmodel/lowsmooth.h:17-194): A (RGB), B, C, eta
struct LowSmooth
{
  static constexpr int kParams = 6;
  static constexpr uint32_t kComponent = kFlagSpecular;
  double A[3], B, C;
  FresnelCook fres;
  __device__ explicit LowSmooth(const double* p) : B(p[3]), C(p[4]), fres(p + 5) { A[0] = p[0]; A[1] = p[1]; A[2] = p[2]; }
  // B InvPi / temp (lowsmooth.h:130-135)
  __device__ __forceinline__ double md(d3 out) const
  {
    const double ro2 = sin_theta2(out);
    const double bb = B * (1.0 - ro2);
    const double t = 1.0 + (2 * B * (1.0 + ro2)) + bb * bb;
    const double temp = -0x1.62e42fefa39efp-1 + log_d(1 + B * (1 - ro2) + safe_sqrt(t));
    return B * kInvPi * (1.0 / temp);
  }
  __device__ __forceinline__ void eval_pdf(d3 in, d3 out, uint32_t component, double* rgb, double& pdf) const
  {
    const bool active = (component & kFlagSpecular) && (in.z >= 0) && (out.z >= 0);
    const double dp2 = sqnorm2(in.x + out.x, in.y + out.y);
    const double cosD = safe_sqrt(1 - 0.25 * sqnorm2(in.x - out.x, in.y - out.y));
    const double S = pow_d(1.0 + B * dp2, -C);
    const double Q = fres.eval(cosD);
#pragma unroll
    for (int c = 0; c < 3; ++c) rgb[c] = active ? A[c] * S * Q : 0.0;
    pdf = active ? md(out) / (1.0 + B * dp2) * in.z : 0.0;
  }
  // lowsmooth.h:166-176
  __device__ __forceinline__ void reflectance(d3 out, uint32_t component, double* rgb) const
  {
    const bool m = (component & kFlagSpecular) && (out.z > 0);
    const double factor = (fabs(C - 1) < kEps) ? log_d(B + 1) / (2 * B) : (1.0 - pow_d(B + 1, 1 - C)) / (2 * B * (C - 1));
    const double q = (fres.eta - 1) / (fres.eta + 1);
    const double R0 = q * q;
#pragma unroll
    for (int c = 0; c < 3; ++c) rgb[c] = m ? ((2.0 * kPi * A[c]) * factor) * R0 : 0.0;
  }
  // lowsmooth.h:75-111
  __device__ __forceinline__ void sample(d3 out, double xi0, double xi1, uint32_t component, d3& dir, double& pdf,
                                         uint32_t& flag) const
  {
    BBM_F64_SAMPLE_PROLOGUE
    const double ro2 = sin_theta2(out);
    const double bb = B * (1 - ro2);
    double temp = 1.0 + (2 * B * (1.0 + ro2)) + bb * bb;
    temp = -0x1.62e42fefa39efp-1 + log_d(1 + B * (1 - ro2) + safe_sqrt(temp));
    const double mdpi = B * (1.0 / temp);
    const double E = 2.0 * exp_d(xi0 * B * (1.0 / mdpi));
    const double ri = safe_sqrt((E - 2) * (E + 2 * B * ro2) / (2 * E * B));
    const double ro = sqrt(ro2);
    const double rp = ri + ro, rm = ri - ro;
    const double scale = sqrt((1.0 + B * (rp * rp)) / (1.0 + B * (rm * rm)));
    double phio = atan2(out.y, out.x);
    phio = (phio < 0) ? phio + 2.0 * kPi : phio;
    const double phi = 2.0 * atan(tan(xi1 * kPi) * scale) + phio;
    double sp, cp;
    sincos(phi, &sp, &cp);
    dir = mk(cp * ri, sp * ri, safe_sqrt(1.0 - ri * ri));
    double rgb[3];
    eval_pdf(dir, out, component, rgb, pdf);
    flag = kFlagSpecular;
  }
};
#undef BBM_F64_SAMPLE_PROLOGUE

// --------------------------------------------------------------------------------------------------- Bagher

// spherical::theta(v) (core/spherical.h:26-32): 2 asin(0.5 |v - (0, 0, sign z)|), Pi - that below the horizon
__device__ __forceinline__ double theta_of(d3 v)
{
  const double dz = v.z - copysign(1.0, v.z);
  const double t = 2.0 * asin(0.5 * sqrt(((0.0 + v.x * v.x) + v.y * v.y) + dz * dz));
  return (v.z >= 0) ? t : kPi - t;
}

// scaledmodel<microfacet<ndf::sgd, uncorrelated, fresnel::bagher, Cook>> (bsdfmodel/bagher.h:62-68; ndf/sgd.h:48-63,
// 143-193): Spectrum-valued NDF / G1 / Fresnel; sampled and pdf'd by GGX with the channel-averaged alpha
// (sgd.h:73-93).  Parameters as the floatRGB Bagher (spectral.hpp).
struct Bagher
{
  static constexpr int kParams = 30;
  static constexpr uint32_t kComponent = kFlagSpecular;
#ifdef BBM_HIP_F64_BAGHER_FLOOR
  static constexpr int kF64Floor = BBM_HIP_F64_BAGHER_FLOOR;   // A/B: two pairs per thread, an occupancy floor
#endif
  double albedo[3], K[3], Lambda[3], c[3], theta0[3], k[3], alpha[3], p[3], F0[3], F1[3], inv_alpha[3], hc0[3], hc_min;
  GGX<false> ggx;
  __device__ explicit Bagher(const double* q) : ggx(q + 18)
  {
    for (int j = 0; j < 3; ++j)
    {
      albedo[j] = q[j]; K[j] = q[3 + j]; Lambda[j] = q[6 + j]; c[j] = q[9 + j]; theta0[j] = q[12 + j];
      k[j] = q[15 + j]; alpha[j] = q[18 + j]; p[j] = q[21 + j]; F0[j] = q[24 + j]; F1[j] = q[27 + j];
      inv_alpha[j] = 1.0 / alpha[j];
      // theta > theta0 <=> 2 asin(c) > theta0 <=> c > sin(theta0 / 2) for the half chord c of theta_of (asin is
      // increasing; both sides round, so only lanes within an ulp of the boundary can decide differently, where
      // G1 = 1 + Lambda (1 - e^(c 0^k)) = 1 on either side)
      // compared as squared chords (4 hc^2 against the chord's squared length: no square root per pair)
      const double hc = (theta0[j] <= 0.0) ? -1.0 : ((theta0[j] >= kPi) ? 2.0 : sin(0.5 * theta0[j]));
      hc0[j] = (hc < 0.0) ? -1.0 : 4.0 * hc * hc;
    }
    hc_min = fmin(fmin(hc0[0], hc0[1]), hc0[2]);
    ggx.au = ggx.av = (((0.0 + alpha[0]) + alpha[1]) + alpha[2]) / 3;
    ggx.iau = ggx.iav = 1.0 / ggx.au;
#ifdef BBM_HIP_F64_VPARAM
    // an empty asm with a VGPR operand: the value stays in a VGPR (no SGPR copy to spill and read back per use)
    for (int j = 0; j < 3; ++j)
    {
      asm("" : "+v"(albedo[j])); asm("" : "+v"(K[j])); asm("" : "+v"(Lambda[j])); asm("" : "+v"(c[j]));
      asm("" : "+v"(theta0[j])); asm("" : "+v"(k[j])); asm("" : "+v"(F0[j])); asm("" : "+v"(F1[j]));
      asm("" : "+v"(p[j]));
    }
#endif
  }
  // sgd.h:185-190 G1 for an upper-hemisphere direction with squared chord hc (theta = 2 asin(sqrt(hc) / 2)): the
  // branch skips the shadowing term (a log and two exponentials) where theta <= theta0; th is theta_of(v),
  // evaluated only if some channel needs it
  __device__ __forceinline__ double G1h(int j, double hc, double th) const
  {
    double g = 1.0;
    if (hc > hc0[j]) g = 1.0 + Lambda[j] * (1.0 - exp_d(c[j] * pow_d(th - theta0[j], k[j])));
    return g;
  }
  __device__ __forceinline__ static double half_chord(d3 v)     // the squared chord |v - (0, 0, 1)|^2
  {
    const double dz = v.z - 1.0;
    return ((0.0 + v.x * v.x) + v.y * v.y) + dz * dz;
  }
  __device__ __forceinline__ void eval_pdf(d3 in, d3 out, uint32_t component, double* rgb, double& pdf) const
  {
    const bool active = (component & kFlagSpecular) && (in.z > 0) && (out.z > 0);
    const d3 h = normalize(mk(in.x + out.x, in.y + out.y, in.z + out.z));
    const double inh = dot(in, h), outh = dot(out, h);
    const double tan2 = tan_theta2(h);
    const double z2 = h.z * h.z;
    const double dnorm = kPi * (z2 * z2);
    const bool gmask = (inh > 0) && (outh > 0);
    // in.z, out.z > 0 wherever the result is used: theta_of = 2 asin(half chord)
    const double hc_in = half_chord(in), hc_out = half_chord(out);
    double th_in = 0.0, th_out = 0.0;
    if (hc_in > hc_min) th_in = theta_of(in);
    if (hc_out > hc_min) th_out = theta_of(out);
    const double cosF = 0.5 * (inh + outh);
    const double x5 = pow5_d(1.0 - cosF);
    // the quotients by per-channel constants and by the pair's common denominators as products with one
    // reciprocal each (<= 2 ulp apart from the reference's quotients), and sgd.h:58-59's
    // exp(-t) / pow(t, p) as one exponential e^(-t - p ln t) on log2_d (den > eps <=> p log2 t > -52)
#ifdef BBM_HIP_F64_FDIV_MF
    // dnorm > 0 where h.z > 0 and z_in z_out > 0 on active lanes; other lanes are selected away
    const double inv_dnorm = div_fast(1.0, dnorm), inv_cos = div_fast(1.0, kPi * (in.z * out.z));
#else
    const double inv_dnorm = 1.0 / dnorm, inv_cos = 1.0 / (kPi * (in.z * out.z));
#endif
#pragma unroll
    for (int j = 0; j < 3; ++j)
    {
      const double t = alpha[j] + tan2 * inv_alpha[j];
      const double lden = p[j] * log2_d(t);
#ifdef BBM_HIP_F64_BAGHER_EXPD
      const double P22 = (lden > -52.0) ? exp_d(-__builtin_fma(lden, 0x1.62e42fefa39efp-1, t)) : 0.0;
#else
      // a factor of D, not cancelled: exp_dd's ~2^-44 (9 FMAs) instead of exp_d's full double (15 FMAs)
      const double P22 = (lden > -52.0) ? exp_dd(fmax(-__builtin_fma(lden, 0x1.62e42fefa39efp-1, t), -1.0e4)) : 0.0;
#endif
      const double Dj = ((h.z > 0) ? P22 * inv_dnorm : 0.0) * K[j];
      const double Gj = gmask ? G1h(j, hc_in, th_in) * G1h(j, hc_out, th_out) : 0.0;
      const double Fj = (F0[j] + (1.0 - F0[j]) * x5) - F1[j] * cosF;
      const double res = Dj * Gj * Fj * inv_cos;
      rgb[j] = active ? res * albedo[j] : 0.0;
    }
#ifdef BBM_HIP_F64_FDIV_MF
    pdf = active ? div_fast(vndf_pdf(ggx, out, h, ggx.eval(h)), 4.0 * fabs(outh)) : 0.0;
#else
    pdf = active ? vndf_pdf(ggx, out, h, ggx.eval(h)) / (4.0 * fabs(outh)) : 0.0;
#endif
  }
  __device__ __forceinline__ void reflectance(d3 out, uint32_t component, double* rgb) const
  {
    const bool m = (component & kFlagSpecular) && (out.z > 0);
    const double x5 = pow5_d(1.0 - out.z);
#pragma unroll
    for (int j = 0; j < 3; ++j) rgb[j] = m ? ((F0[j] + (1.0 - F0[j]) * x5) - F1[j] * out.z) / kPi * 4.0 * albedo[j] : 0.0;
  }
  __device__ __forceinline__ void sample(d3 out, double xi0, double xi1, uint32_t component, d3& dir, double& pdf,
                                         uint32_t& flag) const
  {
    dir = mk(0.0, 0.0, 0.0);
    pdf = 0.0;
    flag = kFlagNone;
    if (!(component & kFlagSpecular) || !xi_ok(xi0, xi1) || !(out.z > 0)) return;
    dir = reflect(out, ggx.sample(out, xi0, xi1));
    double rgb[3];
    eval_pdf(dir, out, component, rgb, pdf);
    flag = kFlagSpecular;
  }
};

// ------------------------------------------------------------------------------------------------------ EPD

// std::lerp(a, b, t) for doubles (libstdc++ <cmath>, C++20): exact at the ends, monotone
__device__ __forceinline__ double lerp(double a, double b, double t)
{
  if ((a <= 0 && b >= 0) || (a >= 0 && b <= 0)) return t * b + (1 - t) * a;
  if (t == 1) return b;
  const double x = a + t * (b - a);
  return ((t > 1) == (b > a)) ? ((b < x) ? x : b) : ((x < b) ? x : b);
}

// ndf::epd (ndf/epd.h:43-186) in doubleRGB.  G1 is tab<float, {100, 1000}>::interpolate<double> (core/precompute.h:
// 126-198) of the shadowing table the library builds on the device (inst_epd.hip, epd.hpp): the float entries are
// read as they are and interpolated in double.  The table's device address travels in the parameter block's
// slot after the model's four parameters (bit pattern of a double), filled by the launcher.
struct EpdNdf
{
  static constexpr int kParams = 2;
  static constexpr int kTableSlot = 4;    // EpdM: ndf at offset 0, unscaled, 2 + 2 parameters
  double beta, p, normalization, inv_p;
  const float* tab;
  __device__ explicit EpdNdf(const double* q) : beta(q[0]), p(q[1])
  {
    // compute_normalization (epd.h:160-178)
    normalization = ((p > kEps) ? (p * kInvPi) * (1.0 / tgamma(1.0 / p)) : 0.0) / (beta * beta);
    inv_p = 1.0 / p;
    tab = reinterpret_cast<const float*>(__builtin_bit_cast(unsigned long long, q[kTableSlot]));
  }
  // epd.h:56-73
  __device__ __forceinline__ double eval(d3 h) const
  {
    const double c2 = h.z * h.z;
    const double D = normalization * exp_d(-pow_d(((1 - c2) / c2) / (beta * beta), p)) / (c2 * c2);
    return (h.z > 0) ? D : 0.0;
  }
  // G1.h:14-16 index maps, then the bilinear interpolation of the clamped floor / ceil entries
  __device__ __forceinline__ double lookup(double t) const
  {
    const double m0 = 5.0 / p - 1.0;
    const double m1 = exp_d(-exp_d(log_d(1.0 / t) * 0.05)) * 1000.0 - 1.0;
    auto at = [&](double i0, double i1) {
      const int r = int(fmin(fmax(i0, 0.0), 99.0)), c = int(fmin(fmax(i1, 0.0), 999.0));
      return double(tab[r * 1000 + c]);
    };
    const double f0 = floor(m0), c0 = ceil(m0), w0 = m0 - f0;
    const double f1 = floor(m1), c1 = ceil(m1), w1 = m1 - f1;
    return lerp(lerp(at(f0, f1), at(f0, c1), w1), lerp(at(c0, f1), at(c0, c1), w1), w0);
  }
  // epd.h:140-152
  __device__ __forceinline__ double G1(d3 v, d3 m) const
  {
    const bool mask = (v.z > 0) && (dot(v, m) > 0);
    return mask ? lookup(tan_theta(v) * beta) : 0.0;
  }
  // epd.h:118-134
  __device__ __forceinline__ double pdf(d3, d3 m, double D) const
  {
    const double q = D * m.z;
    return ((m.z > 0) && (q > 0)) ? q : 0.0;
  }
  // epd.h:84-106 (Eq. 49-50): tan^2 = beta^2 gamma_q_inv(1/p, xi1)^(1/p); gamma_q_inv_d (epd.hpp) converges the
  // Halley iteration of util/invgamma.h:404-414 in double
  __device__ __forceinline__ d3 sample(d3, double xi0, double xi1) const
  {
    if (!xi_ok(xi0, xi1)) return mk(0.0, 0.0, 0.0);
    double sp, cp;
    sincos(2.0 * kPi * xi0, &sp, &cp);
    // xi1 = 1: the reference's gamma_q_inv(a, q = 1) starts its Halley iteration at p = 0, x = 0, where
    // t = (P - p) / R(a, 0) = 0 / 0 (util/invgamma.h:404-414): its sampled normal is NaN, and so is this one
    const double g = (xi1 >= 1.0) ? __builtin_nan("") : gamma_q_inv_d(inv_p, xi1);
    const double tan2 = beta * beta * pow_d(g, inv_p);
    const double cosT = 1.0 / sqrt(1.0 + tan2);
    const double sinT = safe_sqrt(1.0 - cosT * cosT);
    return mk(cp * sinT, sp * sinT, cosT);
  }
};

// spherical::phi (core/spherical.h:42-46)
__device__ __forceinline__ double phi_of(d3 v)
{
  const double r = atan2(v.y, v.x);
  return (r < 0) ? r + 2.0 * kPi : r;
}

// maskingshadowing::vanginneken (vanginneken.h:30-71)
struct VanGinneken
{
  template<class NDF>
  __device__ __forceinline__ static double eval(const NDF& ndf, d3 in, d3 out, d3 m, double inm, double outm)
  {
    const double phi = fabs(phi_of(in) - phi_of(out));
    const double lambda = 4.41 * phi / (4.41 * phi + 1.0);
    const double gi = ndf.G1(in, m), go = ndf.G1(out, m);
    const double gio = gi * go;
    const double denom = fmax(gi, go) + lambda * (fmin(gi, go) - gio);
    return ((inm > 0) && (outm > 0) && (denom > kEps)) ? gio / denom : 0.0;
  }
};

// fresnel::complex<Value> (bbm/fresnel_complex.h:38-63), Shirley 1985 Eqs. 2.4-2.7
struct FresnelComplex
{
  static constexpr int kParams = 2;
  double n, k;
  __device__ explicit FresnelComplex(const double* q) : n(q[0]), k(q[1]) {}
  __device__ __forceinline__ double eval(double c) const
  {
    const double c2 = c * c, s2 = 1 - c2, n2 = n * n, k2 = k * k;
    const double temp = n2 - k2 - s2;
    const double a2b2 = safe_sqrt(temp * temp + 4 * n2 * k2);
    const double a = safe_sqrt(0.5 * (a2b2 + temp));
    const double a2c = 2 * a * c;
    const double Rs = (a2b2 - a2c + c2) / (a2b2 + a2c + c2);
    const double Rp = Rs * (c2 * a2b2 - (a2c - s2) * s2) / (c2 * a2b2 + (a2c + s2) * s2);
    return 0.5 * (Rs + Rp);
  }
};

// ------------------------------------------------------------------------------------------- the He family

// doubleRGB::wavelength() (backbone/native/include/backbone.h:36), micron
constexpr double kWavelength[3] = {0.645, 0.526, 0.444};

__device__ __forceinline__ d3 sph_to_vec(double phi, double theta)    // spherical::convert (core/spherical.h)
{
  double st, ct, sp, cp;
  sincos(theta, &st, &ct);
  sincos(phi, &sp, &cp);
  return mk(cp * st, sp * st, ct);
}

// ndf::sampler<NDF, 90, 1>::pdf (ndf/sampler.h:102-128) of the halfway vector m over a 90-entry double CDF
__device__ __forceinline__ double ndf_sampler_pdf(const double* __restrict__ cdf, d3 m)
{
  const double theta = theta_of(m);
  const double ti = sqrt(theta / (0.5 * kPi)) * 90 - 0.5;
  const double w = ti - floor(ti);
  const double fl = floor(ti), ce = ceil(ti);
  // clamp(cast<Size_t>(floor(ti)), 0, 89): a negative value cast to size_t wraps (-> 89)
  const int lidx = (fl < 0) ? 89 : int(fmin(fl, 89.0)), uidx = (ce < 0) ? 89 : int(fmin(ce, 89.0));
  auto cpdf = [&](int i) { return cdf[i] - ((i >= 1) ? cdf[i - 1] : 0.0); };
  const double p = cpdf(lidx) * (1 - w) + cpdf(uidx) * w;
  const double jac = (sqrt(theta) * (0.25 * kPi * kPi) / 90) * fabs(sin(theta)) * (2.0 * kPi);
  return ((m.z > 0) && (jac > kEps)) ? p / jac : 0.0;
}

// ndf::sampler::sample (ndf/sampler.h:63-92) with cdf::sample (util/cdf.h:73-83)
__device__ __forceinline__ d3 ndf_sampler_halfway(const double* __restrict__ cdf, double xi0, double xi1)
{
  int idx = 0;
  while (idx < 90 && cdf[idx] < xi0) ++idx;
  const bool valid = idx < 90;
  const double prev = (valid && idx >= 1) ? cdf[idx - 1] : 0.0;
  const double residual = valid ? (xi0 - prev) / (cdf[idx] - prev) : 0.0;
  const double off = 1 - safe_sqrt(1 - 2 * fabs(residual - 0.5));
  const double q = (double(idx) + 0.5 + copysign(1.0, residual - 0.5) * off) / 90;
  double theta = (q * q) * (0.5 * kPi);
  theta = (theta > 0.5 * kPi) ? kPi - theta : theta;
  return sph_to_vec(2.0 * kPi * xi1, theta);
}

// fresnel::complex<CONF, Spectrum> per channel (bbm/fresnel_complex.h:38-63); params n RGB, k RGB
struct FresnelComplexRGB
{
  static constexpr int kParams = 6;
  FresnelComplex f[3];
  __device__ explicit FresnelComplexRGB(const double* q) : f{FresnelComplex(q), FresnelComplex(q), FresnelComplex(q)}
  {
    for (int c = 0; c < 3; ++c) { f[c].n = q[c]; f[c].k = q[3 + c]; }
  }
  __device__ __forceinline__ void eval3(double cs, double* F) const { for (int c = 0; c < 3; ++c) F[c] = f[c].eval(cs); }
};
struct FresnelCookRGB
{
  static constexpr int kParams = 1;
  FresnelCook f;
  __device__ explicit FresnelCookRGB(const double* q) : f(q) {}
  __device__ __forceinline__ void eval3(double cs, double* F) const { F[0] = F[1] = F[2] = f.eval(cs); }
};

// he_base<...> (bsdfmodel/he.h:115-482) behind ndf_sampler (bbm/ndf_sampler.h:22-164), doubleRGB: every term in
// double, Constants::Epsilon() the double epsilon (the adaptive Taylor stop included).  The sampler's 90-entry CDF
// (double) is built per launch (k_he_cdf_f64) and its address and the component it was built for ride in the two
// parameter slots after the model's own (as the floatRGB He, he.hpp).
template<class FRES, bool ERRATA, bool WESTIN, int TAYLOR, bool ADAPTIVE, int APPROX, bool SCALED>
struct He
{
  static constexpr int kOff = SCALED ? 3 : 0;
  static constexpr int kParams = kOff + 2 + FRES::kParams;
  static constexpr uint32_t kComponent = kFlagSpecular;
#ifndef BBM_HIP_F64_HE_WAVES
#define BBM_HIP_F64_HE_WAVES 2     // one pair per thread, <= 256 VGPRs: He 2.22 -> 1.49 ms per 10 M pairs (3 / 4: slower)
#endif
  static constexpr int kF64Waves = BBM_HIP_F64_HE_WAVES;
  double albedo[3], sigma0, tau;
  FRES fres;
  const double* cdf;
  uint32_t launch_component;
  __device__ explicit He(const double* p) : sigma0(p[kOff]), tau(p[kOff + 1]), fres(p + kOff + 2)
  {
    for (int c = 0; c < 3; ++c) albedo[c] = SCALED ? p[c] : 1.0;
    cdf = reinterpret_cast<const double*>(__builtin_bit_cast(unsigned long long, p[kParams]));
    launch_component = uint32_t(p[kParams + 1]);
  }
  __device__ __forceinline__ bool masked(uint32_t component) const { return component != launch_component; }

  // he.h:266-291, Eqs. 24-25
  __device__ __forceinline__ double S1(d3 v) const
  {
    const double scot = tau * (1.0 / tan_theta(v)) / (2.0 * sigma0);
    const double ec = 0.5 * erfc(scot);
    double lambda = 0.5 * kInvSqrtPi / scot;
    if (ERRATA) lambda *= exp_lib(-(scot * scot));
    lambda -= ec;
    return (sigma0 < kEps) ? 1.0 : (1.0 - ec) / (lambda + 1.0);
  }
  // he.h:306-352, Eq. 76
  __device__ __forceinline__ double G(d3 in, d3 out) const
  {
    const d3 v = mk(in.x + out.x, in.y + out.y, in.z + out.z);
    const double vq = dot(v, v) / v.z;
    const double v_scale = vq * vq;
    const double kixn2 = 1 - in.z * in.z, krxn2 = 1 - out.z * out.z;
    const double kikr = dot(mk(-in.x, -in.y, -in.z), out);
    const double sikr = out.y * in.x - out.x * in.y, srki = in.y * out.x - in.x * out.y;
    const double pikr = out.z + kikr * in.z, prki = in.z + kikr * out.z;
    const double dd = 1.0 - kikr * kikr;
    const double denom = dd * dd;
    const double nom = (sikr * sikr + pikr * pikr) * (srki * srki + prki * prki) / (krxn2 * kixn2);
    return (denom > kEps) ? v_scale * nom / denom : 1.0;
  }
  // he.h:365-400, Eq. 80 by 4 Newton-Raphson steps
  __device__ __forceinline__ double sigma(d3 in, d3 out) const
  {
    const double ti = tan_theta(in), to = tan_theta(out);
    auto K = [&](double t) { return t * erfc(tau / (2 * sigma0 * t)); };
    const double Ki = (ti > kEps) ? K(ti) : 0.0, Ko = (to > kEps) ? K(to) : 0.0;
    const double f0 = (1.0 / sqrt(8.0 * kPi)) * (Ki + Ko);
    double x = (f0 <= 1.0) ? f0 : safe_sqrt(2.0 * log_d(f0));
    for (int s = 0; s < 4; ++s)
    {
      const double expn = exp_lib(0.5 * x * x);
      const double ev = x * expn - f0, grad = (1 + x * x) * expn;
      x -= (grad > kEps) ? ev / grad : 0.0;
    }
    return (sigma0 > kEps) ? sigma0 / safe_sqrt(1 + x * x) : 0.0;
  }
  // he.h:411-467, Eqs. 78-79
  __device__ __forceinline__ void D(d3 in, d3 out, double* Dout) const
  {
    const double vxy2 = sqnorm2(in.x + out.x, in.y + out.y);
    const double sg = sigma(in, out);
    const double tau2 = tau * tau;
    double g[3], eb[3], norm[3];
    for (int c = 0; c < 3; ++c)
    {
      const double gg = 2.0 * kPi * sg * (in.z + out.z) / kWavelength[c];
      g[c] = gg * gg;
      const double l2 = kWavelength[c] * kWavelength[c];
      norm[c] = 0.25 * kPi * kPi * tau2 / l2;
      eb[c] = vxy2 * tau2 / 4;
      if (WESTIN) eb[c] *= 4.0 * kPi * kPi / l2;
    }
    const double gmin = fmin(fmin(g[0], g[1]), g[2]);
    double rough[3] = {0.0, 0.0, 0.0}, weight = 0.0;
    if (APPROX >= 0 && gmin > double(APPROX))
    {
      for (int c = 0; c < 3; ++c) rough[c] = exp_lib(-eb[c] / g[c]) / g[c];
      weight = fmin(fmax(gmin - double(APPROX), 0.0), 1.0);
    }
    double sum[3] = {0.0, 0.0, 0.0}, gm[3] = {1.0, 1.0, 1.0}, term[3] = {0.0, 0.0, 0.0}, last[3];
    bool converged = (APPROX >= 0) && (gmin - 1.0 > double(APPROX));
#ifdef BBM_HIP_F64_HE_V1
    for (int m = 1; m <= TAYLOR && !converged; ++m)
    {
      for (int c = 0; c < 3; ++c)
      {
        last[c] = term[c];
        gm[c] *= g[c] / m;
        term[c] = exp_lib(-g[c] - eb[c] / m) * gm[c] / m;
        sum[c] += term[c];
      }
      if (ADAPTIVE)
      {
        const double t = fmin(fmin(term[0], term[1]), term[2]);
        converged = (t < kEps) && (t < fmin(fmin(last[0], last[1]), last[2]));
      }
    }
#else
    // term = exp(-g - eb/m) gm / m (he.h:452-454) as exp(-g) (once per channel) x exp(-eb/m) (per term) with exp_dd
    // (a 9-FMA polynomial, ~2^-44 relative) instead of the library's double exp (~40 instructions), and the
    // divisions by m as products with 1/m (a table): each term within ~1e-13 of the reference's, far inside the
    // 1e-9 the doubleRGB tests hold the He family to.
#ifdef BBM_HIP_HE_PROBE_NO_SERIES
    converged = true;       // timing probe only (tools/build_variant.sh): the prelude without the series
#endif
    double eg[3], cap[3];
#pragma unroll
    for (int c = 0; c < 3; ++c)
    {
      eg[c] = converged ? 0.0 : exp_dd(fmax(-g[c], -1.0e4));
      cap[c] = (ADAPTIVE && !converged) ? eg[c] * exp_dd(fmax(-eb[c] * (1.0 / 64.0), -1.0e4)) * (1.0 + 0x1p-30) : 0.0;
    }
    for (int m = 1; m <= TAYLOR && !converged; ++m)
    {
      const double rm = inv_small(m);
      double ex[3];
      if (WESTIN)
      {
#pragma unroll
        for (int c = 0; c < 3; ++c) ex[c] = exp_dd(fmax(-eb[c] * rm, -1.0e4));
      }
      else ex[0] = ex[1] = ex[2] = exp_dd(fmax(-eb[0] * rm, -1.0e4));   // eb is the same on every channel
#pragma unroll
      for (int c = 0; c < 3; ++c)
      {
        last[c] = term[c];
        gm[c] *= g[c] * rm;
        term[c] = eg[c] * ex[c] * gm[c] * rm;
        sum[c] += term[c];
      }
      if (ADAPTIVE)
      {
        const double t = fmin(fmin(term[0], term[1]), term[2]);
        converged = (t < kEps) && (t < fmin(fmin(last[0], last[1]), last[2]));
        // Exact early exit (as the floatRGB series, he.hpp): past the peak (m + 1 >= g) every later term is at most
        // e^(-g) e^(-eb/64) gm_m / m; once that is below half an ulp of every channel's sum (2^-1075 for a zero
        // sum), no later term changes any sum, so stopping here returns the sums the full loop would.  Lanes whose
        // early terms underflow (eb / m > 745) otherwise never meet the stop rule (0 < 0 is false).
        if ((m & 3) == 0)
        {
          bool settled = true;
#pragma unroll
          for (int c = 0; c < 3; ++c)
          {
            const double bound = cap[c] * gm[c] * rm;     // cap = e^(-g) e^(-eb/64) (1 + 2^-30), loop-invariant
            // 2 bound < ulp(sum): the ulp of a normal sum is 2^(ilogb - 52), of a zero or subnormal one 2^-1074
            const int e = (sum[c] > 0.0) ? max(__builtin_amdgcn_frexp_exp(sum[c]) - 53, -1074) : -1074;   // frexp exponent = ilogb + 1
            settled = settled && (double(m) + 1.0 >= g[c]) && (2.0 * bound < __builtin_ldexp(1.0, e));
          }
          converged = converged || settled;
        }
      }
    }
#endif
    for (int c = 0; c < 3; ++c) Dout[c] = norm[c] * lerp(sum[c], rough[c], weight);
  }
  // he_base::eval (he.h:142-166) [x albedo, scaledmodel.h:50-53; the sampler sees the unscaled he_base]
  template<bool SCALE = true>
  __device__ __forceinline__ void eval_rgb(d3 in, d3 out, uint32_t component, double* rgb) const
  {
    const bool active = (component & kFlagSpecular) && (in.z > 0) && (out.z > 0);
    double Dv[3], F[3];
    const double S = S1(in) * S1(out);
    const double Gv = G(in, out);
    D(in, out, Dv);
    fres.eval3(safe_sqrt((1 + dot(in, out)) / 2.0), F);
    const double nrm = 1.0 / (kPi * in.z * out.z);
    for (int c = 0; c < 3; ++c)
    {
      double v = nrm * F[c] * S * Gv * Dv[c];
      if (SCALED && SCALE) v *= albedo[c];
      rgb[c] = active ? v : 0.0;
    }
  }
  // ndf_sampler::pdf (bbm/ndf_sampler.h:128-156): sampler pdf of h / |4 out.h|
  __device__ __forceinline__ void eval_pdf(d3 in, d3 out, uint32_t component, double* rgb, double& pdf) const
  {
    eval_rgb(in, out, component, rgb);
    const d3 h = normalize(mk(in.x + out.x, in.y + out.y, in.z + out.z));
    const bool active = (out.z > 0) && (in.z > 0) && !masked(component);
    pdf = active ? ndf_sampler_pdf(cdf, h) / fabs(4.0 * dot(out, h)) : 0.0;
  }
  // he.h:230-244
  __device__ __forceinline__ void reflectance(d3 out, uint32_t component, double* rgb) const
  {
    const bool m = (component & kFlagSpecular) && (out.z > 0);
    double F[3];
    fres.eval3(out.z, F);
    for (int c = 0; c < 3; ++c) rgb[c] = m ? (SCALED ? F[c] / kPi * 4.0 * albedo[c] : F[c] / kPi * 4.0) : 0.0;
  }
  // ndf_sampler::sample (bbm/ndf_sampler.h:78-111)
  __device__ __forceinline__ void sample(d3 out, double xi0, double xi1, uint32_t component, d3& dir, double& pdf,
                                         uint32_t& flag) const
  {
    dir = mk(0.0, 0.0, 0.0); pdf = 0.0; flag = kFlagNone;
    if (!(xi_ok(xi0, xi1) && (out.z > 0)) || masked(component)) return;
    dir = reflect(out, ndf_sampler_halfway(cdf, xi0, xi1));
    double rgb[3];
    eval_pdf(dir, out, component, rgb, pdf);
    flag = component;
  }
};

// Compositions (the floatRGB registry's, models.hpp)
using CookTorranceM = Microfacet<Beckmann<false, false>, VGroove, FresnelCook, Norm::Cook, true>;
using GGXM = Microfacet<GGX<false>, Uncorrelated, FresnelCook, Norm::Walter, true>;
using CookTorranceWalterM = Microfacet<Beckmann<false, true>, Uncorrelated, FresnelCook, Norm::Walter, true>;
using CookTorranceHeitzM = Microfacet<Beckmann<true, true>, HeightCorrelated, FresnelCook, Norm::Walter, true>;
using GGXHeitzM = Microfacet<GGX<true>, HeightCorrelated, FresnelCook, Norm::Walter, true>;
using NganCookTorranceM = Microfacet<Beckmann<false, true>, VGroove, FresnelSchlick, Norm::Cook, true>;
using PhongWalterM = Microfacet<PhongNdf, Uncorrelated, FresnelCook, Norm::Walter, true>;
using RibardiereM = Microfacet<StudentT<false>, Uncorrelated, FresnelCook, Norm::Walter, true>;
using RibardiereAnisoM = Microfacet<StudentT<true>, Uncorrelated, FresnelCook, Norm::Walter, true>;
using LowMicrofacetM = Microfacet<LowNdf, VGroove, FresnelCook, Norm::Cook, true>;
using AggCookTorranceM = Aggregate<Lambertian, CookTorranceM>;
using AggGGXM = Aggregate<Lambertian, GGXM>;
using AggNganCookTorranceM = Aggregate<Lambertian, NganCookTorranceM>;
using AggLowMicrofacetM = Aggregate<Lambertian, LowMicrofacetM>;
using WardM = Ward<0, true>;
using WardDuerM = Ward<1, true>;
using WardDGMM = Ward<2, true>;
using NganWardM = Ward<0, false>;
using NganWardDuerM = Ward<1, false>;
using LafortuneM = Lafortune<true, false>;
using NganLafortuneM = Lafortune<false, true>;
using ASM = AshikhminShirley<FresnelSchlickRGB, true, false, false>;
using ASFullM = AshikhminShirley<FresnelSchlickRGB, true, false, true>;
using LowASM = AshikhminShirley<ScalarFresnel3<FresnelCook>, false, true, false>;
using NganASM = AshikhminShirley<ScalarFresnel3<FresnelSchlick>, false, true, false>;
using AggLowASM = Aggregate<Lambertian, LowASM>;
using AggLowSmoothM = Aggregate<Lambertian, LowSmooth>;
using AggNganASM = Aggregate<Lambertian, NganASM>;
using AggPhongM = Aggregate<Lambertian, PhongLobe>;
using AggNganLafortuneM = Aggregate<Lambertian, NganLafortuneM>;
using AggNganWardM = Aggregate<Lambertian, NganWardM>;
using AggNganWardDuerM = Aggregate<Lambertian, NganWardDuerM>;
using AggBagherM = Aggregate<Lambertian, Bagher>;
using EpdM = Microfacet<EpdNdf, VanGinneken, FresnelComplex, Norm::Walter, false>;   // holzschuchpacanowski.h:34-42
using HeM = He<FresnelComplexRGB, false, false, 64, true, 18, false>;      // he.h:489-496
using HeWestinM = He<FresnelComplexRGB, true, true, 64, true, 18, false>;
using HeHolzschuchM = He<FresnelComplexRGB, true, false, 10, false, -1, false>;
using NganHeM = He<FresnelCookRGB, true, true, 64, true, 18, true>;        // ngan.h:166-167
using AggNganHeM = Aggregate<Lambertian, NganHeM>;

// ------------------------------------------------------------------------------------------------- kernels

struct ParamBlockF64 { double v[kMaxParamsF64]; };

struct EvalArgsF64
{
  const double* ix; const double* iy; const double* iz;
  const double* ox; const double* oy; const double* oz;
  const uint8_t* mask;
  double* r; double* g; double* b; double* pdf;
  uint64_t n;
  uint32_t component;
  ParamBlockF64 p;
};

struct ReflArgsF64
{
  const double* ox; const double* oy; const double* oz;
  const uint8_t* mask;
  double* r; double* g; double* b;
  uint64_t n;
  uint32_t component;
  ParamBlockF64 p;
};

struct SampleArgsF64
{
  const double* ox; const double* oy; const double* oz;
  const double* xi0; const double* xi1;
  const uint8_t* mask;
  double* dx; double* dy; double* dz; double* pdf; uint32_t* flag;
  uint64_t n;
  uint32_t component;
  ParamBlockF64 p;
};

using EvalLauncherF64 = int (*)(const EvalArgsF64&, hipStream_t);
using ReflLauncherF64 = int (*)(const ReflArgsF64&, hipStream_t);
using SampleLauncherF64 = int (*)(const SampleArgsF64&, hipStream_t);

// A composition's f64 launchers (f64.hip), looked up by registry name; nullptr for a model without a doubleRGB
// kernel.
struct F64Launchers { EvalLauncherF64 eval_pdf; ReflLauncherF64 reflectance; SampleLauncherF64 sample; };

}  // namespace f64
// EPD's shadowing table on the current device, built on first use (inst_epd.hip); nullptr on failure
const float* epd_table_device(hipStream_t s);
namespace f64 {
const F64Launchers* f64_launchers(const char* name);

}  // namespace f64
}  // namespace bbmhip
