// bbm_amd/csrc/microfacet.hpp -- the microfacet family as composable device policies.
//
// One fused kernel serves every microfacet<NDF, MaskingShadowing, Fresnel, Normalization>
// composition (include/bsdfmodel/microfacet.h:51-212), optionally wrapped in scaledmodel
// (include/bsdfmodel/scaledmodel.h:25-80).  A model is a C++ type assembled from the policies
// below; parameters arrive as the flat bbm::parameter_values() vector (attribute declaration
// order: albedo, NDF attributes, Fresnel parameter) and are uniform per launch (kernarg/SGPRs).
#pragma once
#include "math.hpp"

namespace bbmhip {

// ------------------------------------------------------------------------------------- NDFs

// ndf::beckmann<CONF, Symmetry, Normalize> (include/ndf/beckmann.h:40-213)
template<bool Aniso, bool Normalize>
struct Beckmann
{
  static constexpr int kParams = Aniso ? 2 : 1;
  float au, av;
  __device__ explicit Beckmann(const float* p) : au(p[0]), av(Aniso ? p[1] : p[0]) {}

  // beckmann.h:49-66: exp(-|h.xy/alpha|^2 / cos^2) / (au av cos^4) [x 1/pi if Normalize]
  __device__ __forceinline__ float eval(v3 h) const
  {
    if (!(h.z > 0)) return 0.0f;
    const float c2 = h.z * h.z;
    const float sn = sqnorm2(h.x / au, h.y / av);
    float D = expf(-sn / c2) / (au * av * c2 * c2);
    if (Normalize) D *= kInvPiF;
    return D;
  }

  // beckmann.h:180-201: Walter's rational approximation of the Smith G1 term
  __device__ __forceinline__ float G1(v3 v, v3 m) const
  {
    if (!((v.z > 0) && (dot3(v, m) > 0))) return 0.0f;
    float a;
    if (Aniso) a = 1 / sqrtf(sqnorm2(v.x * au, v.y * av) / pow2f(v.z));
    else a = 1 / (au * tan_theta(v));
    const double g = (a < 1.6) ? (3.535 * a + 2.181 * a * a) / (1 + 2.276 * a + 2.577 * a * a) : 1.0;
    return float(g);
  }
};

// ndf::ggx<CONF, Symmetry> (include/ndf/ggx.h:37-196)
template<bool Aniso>
struct GGX
{
  static constexpr int kParams = Aniso ? 2 : 1;
  float au, av;
  __device__ explicit GGX(const float* p) : au(p[0]), av(Aniso ? p[1] : p[0]) {}

  // ggx.h:50-65: rcp(Pi * alpha2 * pow(|h.xy/alpha|^2 + pow(z,2), 2.0)) -- the outer pow in double
  __device__ __forceinline__ float eval(v3 h) const
  {
    if (!(h.z > 0)) return 0.0f;
    const float alpha2 = (1.0f * au) * av;
    const float s = sqnorm2(h.x / au, h.y / av) + pow2f(h.z);
    const double sd = double(s);
    const double d = kPiF * alpha2 * (sd * sd);
    return float(1 / d);
  }

  // ggx.h:173-189: 2 / (1 + sqrt(1 + alpha^2 tan^2)) with `Value denom` rounding to float
  __device__ __forceinline__ float G1(v3 v, v3 m) const
  {
    if (!((v.z > 0) && (dot3(v, m) > 0))) return 0.0f;
    const float r2 = (1.0f * au) * av;
    const float denom = float(1.0 + sqrt(1.0 + r2 * tan_theta2(v)));
    return float(2.0 / denom);
  }
};

// ndf pdf shared by Beckmann/GGX VNDF sampling (beckmann.h:149-170, ggx.h:142-163):
// D(m) * G1(view, m) * |view.m| / cos(view), masked to pdf > 0.  D(m) is passed in (already
// computed by eval on the same halfway vector).
template<class NDF>
__device__ __forceinline__ float vndf_pdf(const NDF& ndf, v3 view, v3 m, float D)
{
  if (!(m.z > 0)) return 0.0f;
  float pdf = D;
  pdf *= ndf.G1(view, m) * fabsf(dot3(view, m)) / view.z;
  if (!(pdf > 0)) return 0.0f;
  return pdf;
}

// ---------------------------------------------------------------------- masking-shadowing

// maskingshadowing::vgroove (include/maskingshadowing/vgroove.h:30-47): the `2.0` literal makes
// both ratios double; bbm::min -> fmin(double); the result is cast back to the G1 return type.
struct VGroove
{
  template<class NDF>
  __device__ __forceinline__ static float eval(const NDF&, v3 in, v3 out, v3 m, float inm, float outm)
  {
    if (!((inm > 0) && (outm > 0))) return 0.0f;
    const double gi = 2.0 * m.z * in.z / inm;
    const double go = 2.0 * m.z * out.z / outm;
    return float(fmin(1.0, fmin(gi, go)));
  }
};

// maskingshadowing::uncorrelated (include/maskingshadowing/uncorrelated.h:30-42)
struct Uncorrelated
{
  template<class NDF>
  __device__ __forceinline__ static float eval(const NDF& ndf, v3 in, v3 out, v3 m, float inm, float outm)
  {
    if (!((inm > 0) && (outm > 0))) return 0.0f;
    return ndf.G1(in, m) * ndf.G1(out, m);
  }
};

// ---------------------------------------------------------------------------- fresnel

// fresnel::cook with a scalar ior (include/bbm/fresnel_cook.h:41-56)
struct FresnelCook
{
  static constexpr int kParams = 1;
  float eta;
  __device__ explicit FresnelCook(const float* p) : eta(p[0]) {}
  __device__ __forceinline__ float eval(float c) const
  {
    const float g = safe_sqrtf(eta * eta + c * c - 1.0f);
    const float a = (g - c) / (g + c);
    const float b = (c * (g + c) - 1.0f) / (c * (g - c) + 1.0f);
    return float(fmax(double(0.5f * (a * a) * (1.0f + b * b)), 0.0));   // bbm::max(x, 0.0)
  }
};

// ---------------------------------------------------------------------- microfacet model

// microfacet_n (include/bsdfmodel/microfacet.h:31-36), literal<double>
enum class Norm { One, Walter, Cook };
template<Norm N> struct norm_value;
template<> struct norm_value<Norm::One> { static constexpr double v = 1.0; };
template<> struct norm_value<Norm::Walter> { static constexpr double v = 4.0; };
template<> struct norm_value<Norm::Cook> { static constexpr double v = kPiD; };

enum : int { kModeEval = 1, kModePdf = 2, kModeEvalPdf = 3 };

template<class NDF, class MS, class FRESNEL, Norm N, bool Scaled>
struct Microfacet
{
  static constexpr int kParams = (Scaled ? 3 : 0) + NDF::kParams + FRESNEL::kParams;
  static constexpr uint32_t kComponent = kFlagSpecular;
  float albedo[3];
  NDF ndf;
  FRESNEL fresnel;

  __device__ explicit Microfacet(const float* p)
      : ndf(p + (Scaled ? 3 : 0)), fresnel(p + (Scaled ? 3 : 0) + NDF::kParams)
  {
    albedo[0] = Scaled ? p[0] : 1.0f;
    albedo[1] = Scaled ? p[1] : 1.0f;
    albedo[2] = Scaled ? p[2] : 1.0f;
  }

  // microfacet.h:74-102 (eval) + :154-174 (pdf), fused: both share the halfway vector and D(h).
  template<int MODE>
  __device__ __forceinline__ void eval_pdf(v3 in, v3 out, uint32_t component, float* rgb, float& pdf) const
  {
    rgb[0] = rgb[1] = rgb[2] = 0.0f;
    pdf = 0.0f;
    if (!(component & kFlagSpecular)) return;
    if (!((in.z > 0.0f) && (out.z > 0.0f))) return;   // eval :80 and pdf :163 use the same test
    const v3 h = halfway(in, out);
    const float D = ndf.eval(h);
    const float outh = dot3(out, h);
    if (MODE & kModeEval)
    {
      const float inh = dot3(in, h);
      const float G = MS::eval(ndf, in, out, h, inh, outh);
      const float F = fresnel.eval(0.5f * (inh + outh));
      // (D G F) / NormalizationFactor / (z_in z_out): literal<double> promotes to double
      const float res = float(D * G * F / norm_value<N>::v / (in.z * out.z));
      if (Scaled) { rgb[0] = res * albedo[0]; rgb[1] = res * albedo[1]; rgb[2] = res * albedo[2]; }
      else { rgb[0] = rgb[1] = rgb[2] = res; }
    }
    if (MODE & kModePdf)
    {
      if (h.z < 0)   // microfacet.h:167 -- unreachable for z_in, z_out > 0 but kept for NaN-free parity
      {
        const v3 hf = neg3(h);
        pdf = float(vndf_pdf(ndf, out, hf, ndf.eval(hf)) / (4.0 * fabsf(dot3(out, hf))));
      }
      else pdf = float(vndf_pdf(ndf, out, h, D) / (4.0 * fabsf(outh)));
    }
  }
};

}  // namespace bbmhip
