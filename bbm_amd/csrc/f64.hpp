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
// Schlick Fresnel) and Aggregate(Lambertian, X) of those.  Layout: SoA f64 (8 B per coordinate), two pairs per
// thread with 16 B loads: 48 B in + 32 B out = 80 B per eval+pdf pair.
#pragma once
#include "math.hpp"

namespace bbmhip {
namespace f64 {

constexpr double kEps = 2.220446049250313080847263336181640625e-16;   // numeric_limits<double>::epsilon()
constexpr double kPi = 3.141592653589793115997963468544185161590576171875;          // std::numbers::pi (double)
constexpr double kInvPi = 0.31830988618379069121644420192751567810773849487304688;  // std::numbers::inv_pi

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

// Walter's rational approximation of the Smith G1 (beckmann.h:195, phong.h G1)
__device__ __forceinline__ double walter_g1(double a) { return (a < 1.6) ? (3.535 * a + 2.181 * a * a) / (1 + 2.276 * a + 2.577 * a * a) : 1.0; }

// ----------------------------------------------------------------------------------------------------- NDFs

// ndf::beckmann (include/ndf/beckmann.h:49-66 eval, :180-201 G1)
template<bool Aniso, bool Normalize>
struct Beckmann
{
  static constexpr int kParams = Aniso ? 2 : 1;
  double au, av;
  __device__ explicit Beckmann(const double* p) : au(p[0]), av(Aniso ? p[1] : p[0]) {}
  __device__ __forceinline__ double eval(d3 h) const
  {
    const double c2 = h.z * h.z;
    double D = exp(-sqnorm2(h.x / au, h.y / av) / c2) / (au * av * c2 * c2);
    if (Normalize) D *= kInvPi;
    return (h.z > 0) ? D : 0.0;
  }
  __device__ __forceinline__ double G1(d3 v, d3 m) const
  {
    const bool mask = (v.z > 0) && (dot(v, m) > 0);
    const double a = Aniso ? 1.0 / sqrt(sqnorm2(v.x * au, v.y * av) / (v.z * v.z)) : 1.0 / (au * tan_theta(v));
    return mask ? walter_g1(a) : 0.0;
  }
};

// ndf::ggx (include/ndf/ggx.h:50-65 eval, :173-189 G1)
template<bool Aniso>
struct GGX
{
  static constexpr int kParams = Aniso ? 2 : 1;
  double au, av;
  __device__ explicit GGX(const double* p) : au(p[0]), av(Aniso ? p[1] : p[0]) {}
  __device__ __forceinline__ double eval(d3 h) const
  {
    const double s = sqnorm2(h.x / au, h.y / av) + h.z * h.z;
    const double D = 1.0 / (kPi * (au * av) * (s * s));
    return (h.z > 0) ? D : 0.0;
  }
  __device__ __forceinline__ double G1(d3 v, d3 m) const
  {
    const bool mask = (v.z > 0) && (dot(v, m) > 0);
    const double denom = 1.0 + sqrt(1.0 + (au * av) * tan_theta2(v));
    return mask ? 2.0 / denom : 0.0;
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
    const double D = pow(h.z, sharpness) * ((sharpness + 2) / (2.0 * kPi));
    return (h.z > 0) ? D : 0.0;
  }
  __device__ __forceinline__ double G1(d3 v, d3 m) const
  {
    const bool mask = (v.z > 0) && (dot(v, m) > 0);
    return mask ? walter_g1(sqrt(0.5 * sharpness + 1) / tan_theta(v)) : 0.0;
  }
  __device__ __forceinline__ double pdf(d3, d3 m, double D) const { return (m.z > 0) ? D * fabs(m.z) : 0.0; }
};

// ndf::studentt (include/ndf/studentt.h:34-195), Ribardiere et al. 2017
template<bool Aniso>
struct StudentT
{
  static constexpr int kParams = (Aniso ? 2 : 1) + 1;
  double au, av, gamma, lam_scale, s1_scale, sqrt_g1, f22, f23;
  __device__ explicit StudentT(const double* p) : au(p[0]), av(Aniso ? p[1] : p[0]), gamma(p[Aniso ? 2 : 1])
  {
    // parameter-only factors of G1 (studentt.h:152-156), once per thread
    lam_scale = tgamma(gamma - 0.5) / tgamma(gamma) * 0.56418958354775627928034964497783221304416656494140625;
    s1_scale = pow(gamma - 1, gamma) / (2 * gamma - 3);
    sqrt_g1 = sqrt(gamma - 1);
    f22 = F22(gamma);
    f23 = F23(gamma);
  }
  __device__ __forceinline__ double eval(d3 h) const
  {
    const double z2 = h.z * h.z;
    const double den = pow(1.0 + sqnorm2(h.x / au, h.y / av) / ((gamma - 1) * z2), gamma);
    const double D = 1.0 / (kPi * (au * av) * (z2 * z2) * den);
    return (h.z > 0) ? D : 0.0;
  }
  __device__ __forceinline__ static double F21(double z)
  {
    const double z2 = z * z, z3 = z2 * z;
    return (1.066 * z + 2.655 * z2 + 4.892 * z3) / (1.038 + 2.969 * z + 4.305 * z2 + 4.418 * z3);
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
    return (6.537 + 6.074 * z - 0.623 * z2 + 5.223 * z3) / (6.538 + 6.103 * z - 3.218 * z2 + 6.347 * z3);
  }
  // studentt.h:128-156
  __device__ __forceinline__ double G1(d3 v, d3 m) const
  {
    const bool mask = (v.z > 0) && (dot(v, m) > 0);
    const bool normal_mask = v.z < 1.0 - kEps;
    const double z = v.z * (1.0 / sqrt(sqnorm2(v.x * au, v.y * av)));
    const double S1 = pow((gamma - 1) + z * z, 1.5 - gamma) / z;
    const double S2 = F21(z) * (f22 + f23 * F24(z));
    const double lambda = normal_mask ? lam_scale * (s1_scale * S1 + sqrt_g1 * S2) - 0.5 : 0.0;
    return mask ? (normal_mask ? 1.0 / (1.0 + lambda) : 1.0) : 0.0;
  }
  __device__ __forceinline__ double pdf(d3, d3 m, double D) const
  {
    const double p = D * m.z;
    return ((m.z > 0) && (p > 0)) ? p : 0.0;
  }
};

// ndf::low (include/ndf/low.h:32-141): the ABC "S" term as an NDF; G1 = 1
struct LowNdf
{
  static constexpr int kParams = 2;
  double B, C, norm_pdf;
  __device__ explicit LowNdf(const double* p) : B(p[0]), C(p[1])
  {
    const double normalization = (fabs(C - 1) < kEps) ? 1.0 / log(1.0 + B) : (C - 1.0) / (1.0 - pow(1.0 + B, 1.0 - C));
    norm_pdf = 0.5 * kInvPi * normalization;
  }
  __device__ __forceinline__ double eval(d3 h) const { return (h.z > 0) ? pow(1.0 + B * (1.0 - h.z), -C) : 0.0; }
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
    const double a = (g - c) / (g + c);
    const double b = (c * (g + c) - 1.0) / (c * (g - c) + 1.0);
    return fmax(0.5 * (a * a) * (1.0 + b * b), 0.0);
  }
};

// fresnel::schlick (bbm/fresnel_schlick.h:42-53): R0 + (1 - R0) pow(1 - cos, 5)
struct FresnelSchlick
{
  static constexpr int kParams = 1;
  double r0;
  __device__ explicit FresnelSchlick(const double* p) : r0(p[0]) {}
  __device__ __forceinline__ double eval(double c) const { return r0 + (1.0 - r0) * pow(1.0 - c, 5.0); }
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
    const d3 h = normalize(mk(in.x + out.x, in.y + out.y, in.z + out.z));
    const double D = ndf.eval(h);
    const double inh = dot(in, h), outh = dot(out, h);
    const double G = MS::eval(ndf, in, out, h, inh, outh);
    const double F = fresnel.eval(0.5 * (inh + outh));
    const double res = D * G * F / norm_value<N>::v / (in.z * out.z);
#pragma unroll
    for (int c = 0; c < 3; ++c) rgb[c] = active ? (Scaled ? res * albedo[c] : res) : 0.0;
    // the pdf's `h = z(h) < 0 ? -h : h` (:167) never fires on active lanes
    pdf = active ? ndf_pdf<NDF>::run(ndf, out, h, D) / (4.0 * fabs(outh)) : 0.0;
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
};

// aggregatemodel<A, B> (bsdfmodel/aggregatemodel.h:60-163): eval and reflectance sum (right folds of two
// children), pdf = (w_A pdf_A + w_B pdf_B) / (w_A + w_B) with w = hsum(reflectance(out)), 0 if the sum <= eps
template<class A, class B>
struct Aggregate
{
  static constexpr int kParams = A::kParams + B::kParams;
  static constexpr uint32_t kComponent = A::kComponent | B::kComponent;
  A a;
  B b;
  __device__ explicit Aggregate(const double* p) : a(p), b(p + A::kParams) {}
  __device__ __forceinline__ void eval_pdf(d3 in, d3 out, uint32_t component, double* rgb, double& pdf) const
  {
    double ra[3], rb[3], pa, pb;
    a.eval_pdf(in, out, component, ra, pa);
    b.eval_pdf(in, out, component, rb, pb);
#pragma unroll
    for (int c = 0; c < 3; ++c) rgb[c] = ra[c] + rb[c];
    a.reflectance(out, component, ra);
    b.reflectance(out, component, rb);
    const double wa = ((0.0 + ra[0]) + ra[1]) + ra[2], wb = ((0.0 + rb[0]) + rb[1]) + rb[2];
    const double sum = (0.0 + wa) + wb;
    const double ip = (0.0 + pa * wa) + pb * wb;
    pdf = (component && sum > kEps) ? ip / sum : 0.0;
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

// ------------------------------------------------------------------------------------------------- kernels

constexpr int kMaxParamsF64 = 64;
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

using EvalLauncherF64 = int (*)(const EvalArgsF64&, hipStream_t);
using ReflLauncherF64 = int (*)(const ReflArgsF64&, hipStream_t);

// A composition's f64 launchers (f64.hip), looked up by registry name; nullptr for a model without a doubleRGB
// kernel.
struct F64Launchers { EvalLauncherF64 eval_pdf; ReflLauncherF64 reflectance; };
const F64Launchers* f64_launchers(const char* name);

}  // namespace f64
}  // namespace bbmhip
