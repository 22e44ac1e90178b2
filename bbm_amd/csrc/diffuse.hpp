// bbm_amd/csrc/diffuse.hpp -- the diffuse family (Lambertian).
#pragma once
#include "math.hpp"
#include "microfacet.hpp"   // kMode*

namespace bbmhip {

// bbm::lambertian (include/bsdfmodel/lambertian.h:22-153); params: albedo RGB.
struct Lambertian
{
  static constexpr int kParams = 3;
  static constexpr uint32_t kComponent = kFlagDiffuse;
  float albedo[3];
  __device__ explicit Lambertian(const float* p) { albedo[0] = p[0]; albedo[1] = p[1]; albedo[2] = p[2]; }

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
    sincosf(xi0 * float(2.0f * kPiD), &s, &c);
    const float sin_t = float(safe_sqrt(1.0 - xi1));
    dir = mk3(c * sin_t, s * sin_t, safe_sqrtf(xi1));
    float rgb[3];
    eval_pdf<kModePdf>(dir, out, component, rgb, pdf);
    flag = kFlagDiffuse;
  }
};

}  // namespace bbmhip
