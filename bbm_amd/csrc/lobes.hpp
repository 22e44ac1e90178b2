// bbm_amd/csrc/lobes.hpp -- the non-microfacet specular families: Ward (Ward, Ward-Duer,
// Ward-Duer-Geisler-Moroder; anisotropic / isotropic), Phong (Blinn-style lobe about the mirror
// direction), Lafortune (+ Ngan's normalisation), Ashikhmin-Shirley (specular / full / Low / Ngan
// variants) and Low et al.'s smooth-surface model.  Same conventions as microfacet.hpp: the
// reference's expressions and literal types are kept (double where C++ promotes), masks are
// applied with selects, parameters are the flat parameter_values() vector.
#pragma once
#include "math.hpp"
#include "diffuse.hpp"
#include "microfacet.hpp"

namespace bbmhip {

// reflect(out, m) = m * dot(m, out) * 2.0 - out (core/vec_transform.h:43-44), float-exact form
__device__ __forceinline__ v3 reflect_about(v3 out, v3 m)
{
  const float d = dot3(m, out);
  return mk3(2.0f * (m.x * d) - out.x, 2.0f * (m.y * d) - out.y, 2.0f * (m.z * d) - out.z);
}

// toGlobalShadingFrame(normal) * v (core/shading_frame.h:24-48, Duff et al. 2017): columns X, Y, Z
__device__ __forceinline__ v3 to_global(v3 normal, v3 v)
{
  // the normal is a model parameter (any vector a caller sets): the IEEE-style quotient keeps the reference's
  // results at the edges (|n|^2 = inf -> 0 components, not NaN); directions use the fast normalize3
  const float rn = div_nr(1.0f, sqrtf(dot3(normal, normal)));
  const v3 Z = mk3(normal.x * rn, normal.y * rn, normal.z * rn);
  const float sign = copysignf(1.0f, Z.z);
  const float a = div_nr(-1.0f, sign + Z.z);          // -1.0 / (sign + z): one double op on floats
  const float b = Z.x * Z.y * a;
  const v3 X = mk3(1.0f + sign * Z.x * Z.x * a, sign * b, -sign * Z.x);   // 1.0 + f: idem
  const v3 Y = mk3(b, sign + Z.y * Z.y * a, -Z.y);
  // mat3d * vec: row r = (X[r], Y[r], Z[r]) dotted with v (core/mat.h:107-116)
  return mk3(((0.0f + X.x * v.x) + Y.x * v.y) + Z.x * v.z,
             ((0.0f + X.y * v.x) + Y.y * v.y) + Z.y * v.z,
             ((0.0f + X.z * v.x) + Y.z * v.y) + Z.z * v.z);
}

__device__ __forceinline__ bool xi_valid(float xi0, float xi1)
{
  return (xi0 >= 0) && (xi1 >= 0) && (xi0 <= 1) && (xi1 <= 1);
}

// ------------------------------------------------------------------------------------ Ward

// bsdfmodel/ward.h:26-168 (KIND 0), wardduer.h:29-81 (KIND 1), wardduergeislermoroder.h:29-81
// (KIND 2); isotropic instances are NganWard / NganWardDuer (ngan.h:30-38).  sample and pdf are
// Ward's for every kind.
template<int KIND, bool Aniso>
struct Ward
{
  static constexpr int kParams = 3 + (Aniso ? 2 : 1);
  static constexpr uint32_t kComponent = kFlagSpecular;
  float albedo[3], rx, ry;
  __device__ explicit Ward(const float* p) : rx(p[3]), ry(Aniso ? p[4] : p[3])
  {
    albedo[0] = p[0]; albedo[1] = p[1]; albedo[2] = p[2];
  }

  template<int MODE>
  __device__ __forceinline__ void eval_pdf(v3 in, v3 out, uint32_t component, float* rgb, float& pdf) const
  {
    const bool active = (component & kFlagSpecular) && (in.z >= 0) && (out.z >= 0);
    if (MODE & kModeEval)
    {
      const v3 H = mk3(in.x + out.x, in.y + out.y, in.z + out.z);
      const float zH2 = H.z * H.z;
      const float sn = sqnorm2(div_nr(H.x, rx), div_nr(H.y, ry));
      const float exponent = div_nr(sn, zH2);
      float nf;
      if (KIND == 0) nf = kPi4F * sqrtf(in.z * out.z) * rx * ry;
      else if (KIND == 1) nf = kPi4F * rx * ry * (in.z * out.z);
      else nf = f_div_d(double(kPi4F * rx * ry) * (double(zH2) * double(zH2)), double(dot3(H, H)));
      // the exponential is subnormal on the lobe's far tail while the quotient is normal (nf < 1): div_sub<true> keeps
      // that quotient the IEEE one, where div_nr's f32 remainder is rounded to the subnormal grid (3/4 of the lanes
      // that were an ulp off, profiles/r06_ward_bitexact.txt); Ward is HBM-bound, the f64 remainder step is free
      const float e = expf_lobe(-exponent);
      const float f = (nf > 0.0f) ? div_sub<true>(e, nf) : div_nr(e, nf);    // nf = 0: IEEE x / 0 (div_nr)
      rgb[0] = active ? albedo[0] * f : 0.0f;
      rgb[1] = active ? albedo[1] * f : 0.0f;
      rgb[2] = active ? albedo[2] * f : 0.0f;
    }
    else rgb[0] = rgb[1] = rgb[2] = 0.0f;
    if (MODE & kModePdf)
    {
      const v3 h = halfway(in, out);
      // pow(cosTheta(h), 3) is glibc's powf, which is not always the correctly rounded cube (cube_f)
      const float nf = kPi4F * rx * ry * dot3(in, h) * powf_glibc<true>(h.z, 3.0f);
      const float exponent = div_nr(sqnorm2(div_nr(h.x, rx), div_nr(h.y, ry)), h.z * h.z);
      const float e = expf_lobe(-exponent);
      const float p = (nf > 0.0f) ? div_sub<true>(e, nf) : div_nr(e, nf);    // cos^3 underflowed: IEEE x / 0
      pdf = active ? p : 0.0f;
    }
    else pdf = 0.0f;
  }

  // ward.h:67-93
  // ward.h:151-155 (inherited by Ward-Duer variants): albedo for the Specular component
  __device__ __forceinline__ void reflectance(v3, uint32_t component, float* rgb) const
  {
    const bool m = component & kFlagSpecular;
#pragma unroll
    for (int c = 0; c < 3; ++c) rgb[c] = m ? albedo[c] : 0.0f;
  }

  __device__ __forceinline__ void sample(v3 out, float xi0, float xi1, uint32_t component, v3& dir, float& pdf,
                                         uint32_t& flag) const
  {
    dir = mk3(0.0f, 0.0f, 0.0f); pdf = 0.0f; flag = kFlagNone;
    if (!((component & kFlagSpecular) && xi_valid(xi0, xi1))) return;
    float s, c;
    sincosf_glibc(kPi2F * xi0, &s, &c);
    const float cx = c * rx, cy = s * ry;
    const float r = div_nr(1.0f, sqrtf(sqnorm2(cx, cy)));
    const float csx = cx * r, csy = cy * r;
    const float cosT = float(1.0 / sqrt(1.0 - double(div_nr(logf_glibc(xi1), sqnorm2(div_nr(csx, rx), div_nr(csy, ry))))));
    const float sinT = float(safe_sqrt(1.0 - cosT * cosT));
    dir = reflect_about(out, mk3(csx * sinT, csy * sinT, cosT));
    float rgb[3];
    eval_pdf<kModePdf>(dir, out, component, rgb, pdf);
    flag = kFlagSpecular;
  }
};

// ------------------------------------------------------------------------------------ Phong

// bsdfmodel/phong.h:25-163 (also NganBlinnPhong, ngan.h:43-44): lobe about reflect(in) = (-x,-y,z)
struct PhongLobe
{
  static constexpr int kParams = 4;
  static constexpr uint32_t kComponent = kFlagSpecular;
  float albedo[3], s;
  __device__ explicit PhongLobe(const float* p) : s(p[3]) { albedo[0] = p[0]; albedo[1] = p[1]; albedo[2] = p[2]; }

  template<int MODE>
  __device__ __forceinline__ void eval_pdf(v3 in, v3 out, uint32_t component, float* rgb, float& pdf) const
  {
    const bool active = (component & kFlagSpecular) && (in.z >= 0) && (out.z >= 0);
    const float cosA = fmaxf(dot3(mk3(-in.x, -in.y, in.z), out), 0.0f);
    const float pw = powf_ref(cosA, s);
    const float f = (s + 2) * kInvPiHalfF * pw;
    rgb[0] = active ? albedo[0] * f : 0.0f;
    rgb[1] = active ? albedo[1] * f : 0.0f;
    rgb[2] = active ? albedo[2] * f : 0.0f;
    pdf = active ? (s + 1) * kInvPiHalfF * pw : 0.0f;
  }

  // phong.h:145-149: albedo for the Specular component
  __device__ __forceinline__ void reflectance(v3, uint32_t component, float* rgb) const
  {
    const bool m = component & kFlagSpecular;
#pragma unroll
    for (int c = 0; c < 3; ++c) rgb[c] = m ? albedo[c] : 0.0f;
  }

  __device__ __forceinline__ void sample(v3 out, float xi0, float xi1, uint32_t component, v3& dir, float& pdf,
                                         uint32_t& flag) const
  {
    dir = mk3(0.0f, 0.0f, 0.0f); pdf = 0.0f; flag = kFlagNone;
    if (!((component & kFlagSpecular) && xi_valid(xi0, xi1))) return;
    float sp, cp;
    sincosf_glibc(xi0 * kPi2F, &sp, &cp);
    const float cosT = float(pow(double(xi1), 1.0 / (s + 1)));
    const float sinT = float(safe_sqrt(1.0 - cosT * cosT));
    dir = to_global(mk3(-out.x, -out.y, out.z), mk3(cp * sinT, sp * sinT, cosT));
    float rgb[3];
    eval_pdf<kModePdf>(dir, out, component, rgb, pdf);
    flag = kFlagSpecular;
  }
};

// --------------------------------------------------------------------------------- Lafortune

// bsdfmodel/lafortune.h:28-172 (Aniso: Cxy is a Vec2d); NGAN = Ngan's normalised isotropic lobe
// (ngan.h:54-129): eval scaled by (n + 2) / (2 pi max(Cz^2, Cxy^2)^(n/2)) in double
template<bool Aniso, bool NGAN>
struct Lafortune
{
  static constexpr int kParams = 3 + (Aniso ? 2 : 1) + 2;
  static constexpr uint32_t kComponent = kFlagSpecular;
  float albedo[3], cx, cy, cz, s;
  double ngan;
  __device__ explicit Lafortune(const float* p)
      : cx(p[3]), cy(Aniso ? p[4] : p[3]), cz(p[Aniso ? 5 : 4]), s(p[Aniso ? 6 : 5])
  {
    albedo[0] = p[0]; albedo[1] = p[1]; albedo[2] = p[2];
    ngan = NGAN ? (s + 2.0) * kInvPiHalfF / double(powf_glibc(fmaxf(cz * cz, cx * cx), s * 0.5f)) : 1.0;   // glibc powf
  }

  template<int MODE>
  __device__ __forceinline__ void eval_pdf(v3 in, v3 out, uint32_t component, float* rgb, float& pdf) const
  {
    if (MODE & kModeEval)
    {
      const bool active = (component & kFlagSpecular) && (in.z > 0) && (out.z > 0);
      const float fr = powf_ref(fmaxf(dot3(mk3(cx, cy, cz), mk3(in.x * out.x, in.y * out.y, in.z * out.z)), 0.0f), s);
#pragma unroll
      for (int c = 0; c < 3; ++c)
      {
        float v = albedo[c] * fr;
        if (NGAN) v = float(double(v) * ngan);
        rgb[c] = active ? v : 0.0f;
      }
    }
    else rgb[0] = rgb[1] = rgb[2] = 0.0f;
    if (MODE & kModePdf)
    {
      const bool active = (component & kFlagSpecular) && (in.z >= 0) && (out.z >= 0);
      const v3 co = normalize3(mk3(cx * out.x, cy * out.y, cz * out.z));
      const float cosA = fmaxf(dot3(co, in), 0.0f);
      const float p = div_nr(s + 1, kPi2F) * powf_ref(cosA, s);
      pdf = active ? p : 0.0f;
    }
    else pdf = 0.0f;
  }

  // lafortune.h:151-156: albedo pow(|C out|, s) 2 pi / (s + 2) for the Specular component
  // (no horizon test); NganLafortune masks the same way (ngan.h:109-121)
  __device__ __forceinline__ void reflectance(v3 out, uint32_t component, float* rgb) const
  {
    const bool m = component & kFlagSpecular;
    const v3 co = mk3(cx * out.x, cy * out.y, cz * out.z);
    const float nrm = powf_glibc(sqrtf(dot3(co, co)), s) * kPi2F;
    const float normalization = div_nr(nrm, s + 2);
#pragma unroll
    for (int c = 0; c < 3; ++c)
    {
      float v = albedo[c] * normalization;
      if (NGAN) v = float(double(v) * ngan);      // ngan.h:123: result *= Ngan normalization (double)
      rgb[c] = m ? v : 0.0f;
    }
  }

  __device__ __forceinline__ void sample(v3 out, float xi0, float xi1, uint32_t component, v3& dir, float& pdf,
                                         uint32_t& flag) const
  {
    dir = mk3(0.0f, 0.0f, 0.0f); pdf = 0.0f; flag = kFlagNone;
    if (!((component & kFlagSpecular) && xi_valid(xi0, xi1))) return;
    float sp, cp;
    sincosf_glibc(xi0 * kPi2F, &sp, &cp);
    const float cosT = float(pow(double(xi1), 1.0 / (s + 1)));
    const float sinT = float(safe_sqrt(1.0 - cosT * cosT));
    dir = to_global(mk3(cx * out.x, cy * out.y, cz * out.z), mk3(cp * sinT, sp * sinT, cosT));
    float rgb[3];
    eval_pdf<kModePdf>(dir, out, component, rgb, pdf);
    flag = kFlagSpecular;
  }
};

// -------------------------------------------------------------------------- Ashikhmin-Shirley

// fresnel::schlick with a Spectrum reflectance (fresnel_schlick.h:42-53, per channel)
struct FresnelSchlickRGB
{
  static constexpr int kParams = 3;
  float r0[3];
  __device__ explicit FresnelSchlickRGB(const float* p) { r0[0] = p[0]; r0[1] = p[1]; r0[2] = p[2]; }
  __device__ __forceinline__ void eval3(float c, float* F) const
  {
    const double x = double(1.0f - c);
    const double x2 = x * x;
    const double x5 = x2 * x2 * x;
#pragma unroll
    for (int k = 0; k < 3; ++k) F[k] = float(r0[k] + double(1.0f - r0[k]) * x5);
  }
  __device__ __forceinline__ float hsum() const { return ((0.0f + r0[0]) + r0[1]) + r0[2]; }
};

template<class F>
struct ScalarFresnel3 : F
{
  __device__ explicit ScalarFresnel3(const float* p) : F(p) {}
  __device__ __forceinline__ void eval3(float c, float* out) const { out[0] = out[1] = out[2] = F::eval(c); }
};

// ashikhminshirley.h:29-221: FRES in {FresnelSchlickRGB, ScalarFresnel3<FresnelCook>,
// ScalarFresnel3<FresnelSchlick>}; SCALED wraps it in scaledmodel (Low / Ngan variants, low.h:24-25,
// ngan.h:157-158); FULL adds the coupled diffuse term of ashikhminshirleyfull.h:31-191.
template<class FRES, bool Aniso, bool SCALED, bool FULL>
struct AshikhminShirley
{
  static constexpr int kOff = (SCALED ? 3 : 0) + (FULL ? 3 : 0);
  static constexpr int kParams = kOff + FRES::kParams + (Aniso ? 2 : 1);
  static constexpr uint32_t kComponent = FULL ? kFlagAll : kFlagSpecular;
  float albedo[3], diffuse[3], su, sv;
  FRES fres;
  __device__ explicit AshikhminShirley(const float* p)
      : su(p[kOff + FRES::kParams]), sv(p[kOff + FRES::kParams + (Aniso ? 1 : 0)]), fres(p + kOff)
  {
#pragma unroll
    for (int k = 0; k < 3; ++k)
    {
      albedo[k] = SCALED ? p[k] : 1.0f;
      diffuse[k] = FULL ? p[k] : 0.0f;
    }
  }

  // specular pdf (ashikhminshirley.h:148-176)
  __device__ __forceinline__ float spec_pdf(v3 in, v3 out, uint32_t component) const
  {
    const bool active = (component & kFlagSpecular) && (in.z >= 0) && (out.z >= 0);
    const v3 h = halfway(in, out);
    const float hdi = dot3(h, in);
    float exponent, normalization;
    if (Aniso)
    {
      const double num = double(su) * (double(h.x) * double(h.x)) + double(sv) * (double(h.y) * double(h.y));
      const float e = f_div_d(num, 1.0 - double(h.z * h.z));
      exponent = (h.z < 1.0 - kEpsF) ? e : 0.0f;
      normalization = div_nr(sqrtf((su + 1) * (sv + 1)), kPi2F);
    }
    else
    {
      exponent = su;
      normalization = f_div_d(double(su) + 1.0, double(kPi2F));
    }
    const float p = div_nr(normalization * powf_ref(h.z, exponent), 4.0f * hdi);
    return active ? p : 0.0f;
  }

  template<int MODE>
  __device__ __forceinline__ void eval_pdf(v3 in, v3 out, uint32_t component, float* rgb, float& pdf) const
  {
    if (MODE & kModeEval)
    {
      const bool upper = (in.z > 0) && (out.z > 0);
      const bool spec = (component & kFlagSpecular) && upper;
      const v3 h = halfway(in, out);
      const float hdi = dot3(h, in);
      const float denom = hdi * fmaxf(in.z, out.z);
      float F[3];
      fres.eval3(hdi, F);
      float exponent, normalization;
      if (Aniso)
      {
        const float e = div_nr(su * (h.x * h.x) + sv * (h.y * h.y), 1 - h.z * h.z);
        exponent = (h.z < 1 - kEpsF) ? e : 0.0f;
        normalization = div_nr(sqrtf((su + 1) * (sv + 1)), kPi8F);
      }
      else
      {
        exponent = su;
        normalization = div_nr(su + 1, kPi8F);
      }
      const float np = normalization * powf_ref(h.z, exponent);
      float diff_scale = 0.0f;
      if constexpr (FULL)
      {
        // hprod(Scalar(1) - pow(Scalar(1) - 0.5 * Vec2d(z_in, z_out), 5.0)): `double * array<float>` is the
        // array's friend operator*(const float&, array) (backbone/native/include/backbone/array.h:95), so
        // 1 - 0.5 z is formed in float; pow(float, 5.0) and the rest are double; 28 / (23 pi) in double
        const double ai = 1.0f - 0.5f * in.z, ao = 1.0f - 0.5f * out.z;
        const double ai2 = ai * ai, ao2 = ao * ao;
        const float scale = float((1.0 * (1.0 - ai2 * ai2 * ai)) * (1.0 - ao2 * ao2 * ao));
        const float normd = float(28.0 / (23.0 * double(kPiF)));
        diff_scale = normd * scale;
      }
      const bool diff = FULL && (component & kFlagDiffuse) && upper;
#pragma unroll
      for (int c = 0; c < 3; ++c)
      {
        float v = div_nr(np * F[c], denom);
        if (SCALED) v *= albedo[c];
        v = spec ? v : 0.0f;
        if constexpr (FULL) v = diff ? (diff_scale * diffuse[c] * (1.0f - fres.r0[c])) + v : v;
        rgb[c] = upper ? v : 0.0f;
      }
    }
    else rgb[0] = rgb[1] = rgb[2] = 0.0f;
    if (MODE & kModePdf)
    {
      const float sp = spec_pdf(in, out, component);
      if constexpr (FULL)
      {
        // ashikhminshirleyfull.h:148-168
        const bool has_d = component & kFlagDiffuse, has_s = component & kFlagSpecular;
        const float dpdf = ((component & kFlagDiffuse) && (in.z >= 0) && (out.z >= 0)) ? in.z * kInvPiF : 0.0f;
        const float spec_albedo = fres.hsum();
        const float diff_albedo = float(double(((0.0f + diffuse[0]) + diffuse[1]) + diffuse[2]) * (1.0 - spec_albedo));
        const float dw = (diff_albedo > kEpsF) ? div_nr(diff_albedo, diff_albedo + spec_albedo) : 0.0f;
        const float sw = float(1.0 - dw);
        const float mix = sw * sp + dw * dpdf;
        pdf = !has_d ? sp : (!has_s ? dpdf : mix);
      }
      else pdf = sp;
    }
    else pdf = 0.0f;
  }

  // specular lobe sampling (ashikhminshirley.h:98-140)
  __device__ __forceinline__ void spec_sample(v3 out, float xi0, float xi1, uint32_t component, v3& dir, float& pdf,
                                              uint32_t& flag) const
  {
    dir = mk3(0.0f, 0.0f, 0.0f); pdf = 0.0f; flag = kFlagNone;
    if (!((component & kFlagSpecular) && xi_valid(xi0, xi1))) return;
    float cp, sp, cosT;
    if (Aniso)
    {
      float phi = float(atan(sqrt((su + 1.0) / (sv + 1.0)) * double(tanf(xi0 * kPi2F))));
      phi = ((xi0 > 0.25) && (xi0 < 0.75)) ? phi + kPiF : phi;
      sincosf_glibc(phi, &sp, &cp);
      cosT = float(pow(double(xi1), 1.0 / ((su * (cp * cp)) + (sv * (sp * sp)) + 1.0)));
    }
    else
    {
      sincosf_glibc(xi0 * kPi2F, &sp, &cp);
      cosT = float(pow(double(xi1), 1.0 / (su + 1.0)));
    }
    const float sinT = float(safe_sqrt(1.0 - cosT * cosT));
    dir = reflect_about(out, mk3(cp * sinT, sp * sinT, cosT));
    pdf = spec_pdf(dir, out, component);
    flag = kFlagSpecular;
  }

  // ashikhminshirley.h:181-190 (Fresnel at z(out), Specular, z(out) > 0) [x albedo, scaledmodel.h:64-67];
  // FULL: + diffuse (1 - fresnelReflectance) for the Diffuse component (ashikhminshirleyfull.h:170-185)
  __device__ __forceinline__ void reflectance(v3 out, uint32_t component, float* rgb) const
  {
    const bool up = out.z > 0;
    const bool ms = (component & kFlagSpecular) && up;
    float F[3];
    fres.eval3(out.z, F);
#pragma unroll
    for (int c = 0; c < 3; ++c)
    {
      float v = ms ? (SCALED ? F[c] * albedo[c] : F[c]) : 0.0f;
      if constexpr (FULL)
      {
        const float d = diffuse[c] * (1.0f - fres.r0[c]);
        v = (up && (component & kFlagDiffuse)) ? d + v : v;
      }
      rgb[c] = up ? v : 0.0f;
    }
  }

  __device__ __forceinline__ void sample(v3 out, float xi0, float xi1, uint32_t component, v3& dir, float& pdf,
                                         uint32_t& flag) const
  {
    if constexpr (!FULL) { spec_sample(out, xi0, xi1, component, dir, pdf, flag); return; }
    else {
    if (!(component & kFlagDiffuse)) { spec_sample(out, xi0, xi1, component, dir, pdf, flag); return; }
    const float unit_albedo[3] = {1.0f, 1.0f, 1.0f};   // lambertian<Config>(): only its sampler/pdf are used
    const Lambertian lam(unit_albedo);
    if (!(component & kFlagSpecular)) { lam.sample(out, xi0, xi1, component, dir, pdf, flag); return; }
    // ashikhminshirleyfull.h:96-124: one-sample mixture of the specular lobe and cosine sampling
    const float spec_albedo = fres.hsum();
    const float diff_albedo = (((0.0f + diffuse[0]) + diffuse[1]) + diffuse[2]) * (1.0f - spec_albedo);
    const float dw = div_nr(diff_albedo, diff_albedo + spec_albedo);
    const float sw = 1.0f - dw;
    const float xs = (sw > kEpsF) ? div_nr(xi0, sw) : 0.0f;
    const float xd = (dw > kEpsF) ? div_nr(xi0 - sw, dw) : 0.0f;
    v3 ds, dd; float ps, pd; uint32_t fs, fd;
    spec_sample(out, xs, xi1, component, ds, ps, fs);
    lam.sample(out, xd, xi1, component, dd, pd, fd);
    const bool pick_s = xi0 <= sw;
    dir = pick_s ? ds : dd;
    flag = pick_s ? fs : fd;
    pdf = sw * ps + dw * pd;
    }
  }
};

// ------------------------------------------------------------------------------- Low smooth

// bsdfmodel/lowsmooth.h:17-194; params A (RGB), B, C, eta
struct LowSmooth
{
  static constexpr int kParams = 6;
  static constexpr uint32_t kComponent = kFlagSpecular;
  float A[3], B, C;
  FresnelCook fres;
  __device__ explicit LowSmooth(const float* p) : B(p[3]), C(p[4]), fres(p + 5) { A[0] = p[0]; A[1] = p[1]; A[2] = p[2]; }

  __device__ __forceinline__ float md(v3 out) const    // B * InvPi * rcp(temp), lowsmooth.h:130-135
  {
    const float ro2 = sin_theta2(out);
    const double t = 1.0 + (2 * B * (1.0 + ro2)) + pow2d(B * (1.0 - ro2));
    const float temp_f = float(t);
    const float temp = -logf_glibc(2.0f) + logf_glibc(1 + B * (1 - ro2) + safe_sqrtf(temp_f));   // float logs (glibc)
    return B * kInvPiF * div_nr(1.0f, temp);
  }
  __device__ __forceinline__ static double pow2d(double x) { return x * x; }

  // S's double power computed in double (f64::pow_d), rounded to float, in every mode (exact mode: the same)
  static constexpr bool kHasExact = true;
  template<int MODE, bool EXACT = false>
  __device__ __forceinline__ void eval_pdf(v3 in, v3 out, uint32_t component, float* rgb, float& pdf) const
  {
    const bool active = (component & kFlagSpecular) && (in.z >= 0) && (out.z >= 0);
    if (MODE & kModeEval)
    {
      const float dp2 = sqnorm2(in.x + out.x, in.y + out.y);
      const float cosD = float(safe_sqrt(1 - 0.25 * sqnorm2(in.x - out.x, in.y - out.y)));
      // the reference's double pow; round 5: in every mode (+1.3 % kernel time, profiles/r05_ab_low_exact.txt)
      const float S = float(f64::pow_d(1.0 + double(B * dp2), -double(C)));   // B Dp2 is a float product
      const float Q = fres.eval(cosD);
#pragma unroll
      for (int c = 0; c < 3; ++c) rgb[c] = active ? A[c] * S * Q : 0.0f;
    }
    else rgb[0] = rgb[1] = rgb[2] = 0.0f;
    if (MODE & kModePdf)
    {
      const float p = f_div_d(double(md(out)), 1.0 + B * sqnorm2(in.x + out.x, in.y + out.y));
      pdf = active ? p * in.z : 0.0f;
    }
    else pdf = 0.0f;
  }

  // lowsmooth.h:75-111
  // lowsmooth.h:166-176: 2 pi A factor R0, Specular component and z(out) > 0.  factor's branches
  // (log(B+1) / 2B in float; (1.0 - pow(B+1, 1-C)) / (2B(C-1)) in double) both rounded to float
  __device__ __forceinline__ void reflectance(v3 out, uint32_t component, float* rgb) const
  {
    const bool m = (component & kFlagSpecular) && (out.z > 0);
    const float f1 = div_nr(logf_glibc(B + 1), 2 * B);
    const float f2 = float((1.0 - double(powf_glibc(B + 1, 1 - C))) / double(2 * B * (C - 1)));
    const float factor = (fabsf(C - 1) < kEpsF) ? f1 : f2;
    const float q = div_nr(fres.eta - 1, fres.eta + 1);
    const float R0 = q * q;
#pragma unroll
    for (int c = 0; c < 3; ++c) rgb[c] = m ? ((kPi2F * A[c]) * factor) * R0 : 0.0f;
  }

  __device__ __forceinline__ void sample(v3 out, float xi0, float xi1, uint32_t component, v3& dir, float& pdf,
                                         uint32_t& flag) const
  {
    dir = mk3(0.0f, 0.0f, 0.0f); pdf = 0.0f; flag = kFlagNone;
    if (!((component & kFlagSpecular) && xi_valid(xi0, xi1))) return;
    const float ro2 = sin_theta2(out);
    const float bb = B * (1 - ro2);
    float temp = float(1.0 + (2 * B * (1.0 + ro2)) + double(bb * bb));
    temp = float(-log(2.0) + double(logf_glibc(1 + B * (1 - ro2) + safe_sqrtf(temp))));
    const float mdpi = B * div_nr(1.0f, temp);
    const float E = float(2.0 * double(expf_glibc(xi0 * B * div_nr(1.0f, mdpi))));
    const float ri = safe_sqrtf(div_nr((E - 2) * (E + 2 * B * ro2), 2 * E * B));
    const float ro = sqrtf(ro2);
    const double rp = double(ri + ro), rm = double(ri - ro);
    const float scale = float(sqrt((1.0 + B * (rp * rp)) / (1.0 + B * (rm * rm))));
    float phio = atan2f_glibc(out.y, out.x);
    phio = (phio < 0) ? phio + kPi2F : phio;
    const float phi = float(2.0 * double(atanf(tanf(xi1 * kPiF) * scale)) + phio);
    float sp, cp;
    sincosf_glibc(phi, &sp, &cp);
    dir = mk3(cp * ri, sp * ri, float(safe_sqrt(1.0 - ri * ri)));
    float rgb[3];
    eval_pdf<kModePdf>(dir, out, component, rgb, pdf);
    flag = kFlagSpecular;
  }
};

}  // namespace bbmhip
