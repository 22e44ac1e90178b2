// bbm_amd/csrc/diffuse.hpp -- the diffuse family (Lambertian, Oren-Nayar).
#pragma once
#include "math.hpp"
#include "microfacet.hpp"   // kMode*

namespace bbmhip {

// bbm::lambertian (include/bsdfmodel/lambertian.h:22-153); params: albedo RGB.
struct Lambertian
{
  static constexpr bool kHasGeo = true;
  static constexpr int kParams = 3;
  static constexpr uint32_t kComponent = kFlagDiffuse;
  float albedo[3];
  __device__ explicit Lambertian(const float* p) { albedo[0] = p[0]; albedo[1] = p[1]; albedo[2] = p[2]; }

  // the loss kernel's per-pair prelude (kernels.hpp k_loss): nothing to share beyond the pair itself
  struct Geo { v3 in, out; };
  __device__ __forceinline__ static Geo geometry(v3 in, v3 out) { return Geo{in, out}; }
  __device__ __forceinline__ void eval_geo(const Geo& g, uint32_t component, float* rgb) const
  {
    float pdf;
    eval_pdf<kModeEval>(g.in, g.out, component, rgb, pdf);
  }

  // lambertian.h:45-59 eval (albedo * InvPi, non-strict z >= 0) and :115-125 pdf (z_in * InvPi)
  template<int MODE>
  __device__ __forceinline__ void eval_pdf(v3 in, v3 out, uint32_t component, float* rgb, float& pdf) const
  {
    const bool m = (component & kFlagDiffuse) && (in.z >= 0) && (out.z >= 0);
    rgb[0] = m ? albedo[0] * kInvPiF : 0.0f;
    rgb[1] = m ? albedo[1] * kInvPiF : 0.0f;
    rgb[2] = m ? albedo[2] * kInvPiF : 0.0f;
    pdf = m ? in.z * kInvPiF : 0.0f;
  }

  // lambertian.h:136-140: albedo for the Diffuse component (no horizon test)
  __device__ __forceinline__ void reflectance(v3, uint32_t component, float* rgb) const
  {
    const bool m = component & kFlagDiffuse;
    rgb[0] = m ? albedo[0] : 0.0f; rgb[1] = m ? albedo[1] : 0.0f; rgb[2] = m ? albedo[2] : 0.0f;
  }

  // lambertian.h:76-103 cosine-weighted sampling; sinTheta = safe_sqrt(1.0 - xi1) in double
  __device__ __forceinline__ void sample(v3 out, float xi0, float xi1, uint32_t component, v3& dir, float& pdf,
                                         uint32_t& flag) const
  {
    dir = mk3(0.0f, 0.0f, 0.0f);
    pdf = 0.0f;
    flag = kFlagNone;
    if (!(component & kFlagDiffuse)) return;
    if (!((xi0 >= 0) && (xi1 >= 0) && (xi0 <= 1) && (xi1 <= 1))) return;
    float s, c;
    sincosf_glibc(xi0 * float(2.0f * kPiD), &s, &c);
    const float sin_t = float(safe_sqrt(1.0 - xi1));
    dir = mk3(c * sin_t, s * sin_t, safe_sqrtf(xi1));
    float rgb[3];
    eval_pdf<kModePdf>(dir, out, component, rgb, pdf);
    flag = kFlagDiffuse;
  }
};

// bbm::orennayar (include/bsdfmodel/orennayar.h:22-137); params: albedo RGB, roughness.  A and B
// are double expressions of the roughness (rounded to float once per thread); sample and pdf are
// Lambertian's.
struct OrenNayar
{
  static constexpr int kParams = 4;
  static constexpr uint32_t kComponent = kFlagDiffuse;
  float albedo[3], alb_pi[3], A, B;
  __device__ explicit OrenNayar(const float* p)
  {
    albedo[0] = p[0]; albedo[1] = p[1]; albedo[2] = p[2];
    const float sigma2 = p[3] * p[3];
    A = float(1 - 0.5 * sigma2 / (sigma2 + 0.33));
    B = float(0.45 * sigma2 / (sigma2 + 0.09));
    // albedo / Constants::Pi(): once per thread, IEEE division
    alb_pi[0] = p[0] / kPiF; alb_pi[1] = p[1] / kPiF; alb_pi[2] = p[2] / kPiF;
  }

  // orennayar.h:50-72 eval: strict z > 0; factor = A + B max(dot_xy, 0) / max(z_in, z_out)
  template<int MODE>
  __device__ __forceinline__ void eval_pdf(v3 in, v3 out, uint32_t component, float* rgb, float& pdf) const
  {
    const bool diff = component & kFlagDiffuse;
    const bool m = diff && (in.z > 0) && (out.z > 0);
    const float cos_beta = fmaxf(in.z, out.z);
    const float dot_xy = (in.x * out.x) + (in.y * out.y);
    const float factor = A + div_nr(B * fmaxf(dot_xy, 0.0f), cos_beta);
    rgb[0] = m ? alb_pi[0] * factor : 0.0f;
    rgb[1] = m ? alb_pi[1] * factor : 0.0f;
    rgb[2] = m ? alb_pi[2] * factor : 0.0f;
    pdf = (diff && (in.z >= 0) && (out.z >= 0)) ? in.z * kInvPiF : 0.0f;
  }

  // orennayar.h:131-135: albedo for the Diffuse component
  __device__ __forceinline__ void reflectance(v3, uint32_t component, float* rgb) const
  {
    const bool m = component & kFlagDiffuse;
    rgb[0] = m ? albedo[0] : 0.0f; rgb[1] = m ? albedo[1] : 0.0f; rgb[2] = m ? albedo[2] : 0.0f;
  }

  __device__ __forceinline__ void sample(v3 out, float xi0, float xi1, uint32_t component, v3& dir, float& pdf,
                                         uint32_t& flag) const
  {
    const float unit_albedo[3] = {1.0f, 1.0f, 1.0f};
    Lambertian(unit_albedo).sample(out, xi0, xi1, component, dir, pdf, flag);
  }
};

}  // namespace bbmhip
