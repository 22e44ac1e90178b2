// bbm_amd/csrc/microfacet.hpp -- the microfacet family as composable device policies.
//
// One fused kernel serves every microfacet<NDF, MaskingShadowing, Fresnel, Normalization>
// composition (include/bsdfmodel/microfacet.h:51-212), optionally wrapped in scaledmodel
// (include/bsdfmodel/scaledmodel.h:25-80).  A model is a C++ type assembled from the policies
// below; parameters arrive as the flat bbm::parameter_values() vector (attribute declaration
// order: albedo, NDF attributes, Fresnel parameter) and are uniform per launch (kernarg/SGPRs).
#pragma once
#include "math.hpp"

// where the Beckmann NDF's expf reads its table (math.hpp expf_tab): 1 = the kernel's LDS copy, 0 = the constant segment
#ifndef BBM_HIP_BECKMANN_TABLE_LDS
#define BBM_HIP_BECKMANN_TABLE_LDS 1
#endif

namespace bbmhip {

// ------------------------------------------------------------------------------------- NDFs

template<class NDF>
__device__ __forceinline__ float vndf_pdf(const NDF& ndf, v3 view, v3 m, float D);

// the sampler's erfinv, stored into a float (ndf/beckmann.h:99-106); -DBBM_HIP_ERFINV_D: the double evaluation (A/B)
__device__ __forceinline__ float erfinv_s(float a)
{
#ifdef BBM_HIP_ERFINV_D
  return float(erfinv_d(a));
#else
  return erfinv_f(a);
#endif
}

// ndf::beckmann<CONF, Symmetry, Normalize> (include/ndf/beckmann.h:40-213).  ExactSample: the exact-mode twin
// (exact_sample_t below), whose sampler reproduces glibc's erff / logf
template<bool Aniso, bool Normalize, bool ExactSample = false>
struct Beckmann
{
  static constexpr int kParams = Aniso ? 2 : 1;
  float au, av;
  __device__ explicit Beckmann(const float* p) : au(p[0]), av(Aniso ? p[1] : p[0]) {}

  // beckmann.h:49-66: exp(-|h.xy/alpha|^2 / cos^2) / (au av cos^4) [x 1/pi if Normalize]; EXACT: the quotient
  // correctly rounded on the subnormal grid too (div_sub)
  template<bool EXACT = false>
  __device__ __forceinline__ float eval(v3 h) const
  {
    const float c2 = h.z * h.z;
    const float sn = sqnorm2(div_nr(h.x, au), div_nr(h.y, av));
#if defined(BBM_HIP_BECKMANN_EXP_DN)
    float D = div_nr(expf_dn(div_nr(-sn, c2)), au * av * c2 * c2);      // A/B: the 1.4-ulp exponential
#elif defined(BBM_HIP_BECKMANN_EXP_RN)
    float D = div_nr(expf_rn(div_nr(-sn, c2)), au * av * c2 * c2);      // A/B: correctly rounded
#else
    float D = div_sub<EXACT>(expf_glibc_neg<BBM_HIP_BECKMANN_TABLE_LDS != 0>(div_nr(-sn, c2)), au * av * c2 * c2);   // glibc's expf, to its last bit (x <= 0)
#endif
    if (Normalize) D *= kInvPiF;
    return (h.z > 0) ? D : 0.0f;
  }

  // beckmann.h:180-201: Walter's rational approximation of the Smith G1 term
  __device__ __forceinline__ float G1(v3 v, v3 m) const
  {
    const bool mask = (v.z > 0) && (dot3(v, m) > 0);
    float a;
    if (Aniso) a = div_nr(1.0f, sqrtf(div_nr(sqnorm2(v.x * au, v.y * av), pow2f(v.z))));
    else a = div_nr(1.0f, au * tan_theta(v));
    const double ad = a;
    const float g = f_div_d(3.535 * ad + 2.181 * ad * ad, 1 + 2.276 * ad + 2.577 * ad * ad);
    return mask ? ((a < 1.6) ? g : 1.0f) : 0.0f;
  }

  // beckmann.h:76-116: visible-normal sampling following [Jakob 2014] (stretch, invert the
  // slope CDF with three Newton steps on erfinv, rotate, unstretch)
  __device__ __forceinline__ v3 sample(v3 view, float xi0, float xi1) const
  {
    if (!((xi0 >= 0) && (xi1 >= 0) && (xi0 <= 1) && (xi1 <= 1))) return mk3(0.0f, 0.0f, 0.0f);
    const v3 vs = normalize3(mk3(view.x * au, view.y * av, view.z));
    const float tanT = tan_theta(vs);
    // erf and log of floats: in the exact twin glibc's erff / logf restated bit for bit (math.hpp), so the Newton
    // iteration starts from the reference's own float -- 28 % of a CookTorrance importance sample (three divergent
    // erff branches per wave, 2.19 vs 1.70 ms per 125 M samples, profiles/r04_ab_sample_vndf.txt); by default the
    // device library's erff / logf (<= 2 ulp), from which the three Newton steps land on the reference's direction
    // on all but ~1e-5 of the lanes (the rest within the input-ulps proof, tests/test_gpu_parity.py)
    const float tc = div_nr(1.0f, tanT);
    float xc0 = clampf(xi0, float(10e-6), float(1.0 - 10e-6));
    const float xc1 = clampf(xi1, float(10e-6), float(1.0 - 10e-6));
    float maxval, x;
    if constexpr (ExactSample)
    {
      maxval = erff_glibc(tc);
      x = maxval - (maxval + 1) * erff_glibc(sqrtf(-logf_glibc(xc0)));
    }
    else
    {
      maxval = erff(tc);
      x = maxval - (maxval + 1) * erff(sqrtf(-logf(xc0)));
    }
    // exp of a float: glibc's expf (x <= 0) in the twin, the 1.4-ulp expf_dn by default
    const auto expn = [](float v) { return ExactSample ? expf_glibc_neg(v) : expf_dn(v); };
    xc0 = float(xc0 * (1.0 + maxval + kInvSqrtPiF * tanT * expn(-(vs.z * vs.z))));
    for (int i = 0; i < 3; ++i)
    {
      const float slope = erfinv_s(x);
      const float val = float(1.0 + x + kInvSqrtPiF * tanT * expn(-slope * slope) - xc0);
      // float(1.0 - p) of a float p: one double op on float operands rounded to float is the float op itself
      // (53 >= 2 x 24 + 2), so the f32 subtraction -- likewise 2 xc1 - 1 below (2 xc1 exact in either type)
      const float der = 1.0f - slope * tanT;
      x -= div_nr(val, der);
    }
    float s0 = 0.0f, s1 = 0.0f;
    if (x > -1.0 && x < +1.0) { s0 = erfinv_s(x); s1 = erfinv_s(2.0f * xc1 - 1.0f); }
    float c, s;
    cossin_phi(vs, c, s);
    const float u0 = ((0.0f + c * s0) + -s * s1) * au;
    const float u1 = ((0.0f + s * s0) + c * s1) * av;
    return normalize3(mk3(-u0, -u1, 1.0f));
  }

  __device__ __forceinline__ float pdf(v3 view, v3 m, float D) const { return vndf_pdf(*this, view, m, D); }
};

// ndf::ggx<CONF, Symmetry> (include/ndf/ggx.h:37-196).  ExactSample: the exact-mode twin (exact_sample_t), whose
// sampler takes glibc's sinf / cosf of the azimuth (the default: the device library's sincosf, <= 1 ulp; 10 % of a
// GGX importance sample, profiles/r04_ab_sample_sincos.txt)
template<bool Aniso, bool ExactSample = false>
struct GGX
{
  static constexpr int kParams = Aniso ? 2 : 1;
  float au, av;
  __device__ explicit GGX(const float* p) : au(p[0]), av(Aniso ? p[1] : p[0]) {}

  // ggx.h:50-65: rcp(Pi * alpha2 * pow(|h.xy/alpha|^2 + pow(z,2), 2.0)) -- the outer pow in double
  __device__ __forceinline__ float eval(v3 h) const
  {
    const float alpha2 = (1.0f * au) * av;
    const float s = sqnorm2(div_nr(h.x, au), div_nr(h.y, av)) + pow2f(h.z);
    const double sd = double(s);
    const double d = double(kPiF * alpha2) * (sd * sd);
    return (h.z > 0) ? f_div_d(1.0, d) : 0.0f;
  }

  // ggx.h:173-189: 2 / (1 + sqrt(1 + alpha^2 tan^2)) with `Value denom` rounding to float
  __device__ __forceinline__ float G1(v3 v, v3 m) const
  {
    const bool mask = (v.z > 0) && (dot3(v, m) > 0);
    const float r2 = (1.0f * au) * av;
    const float denom = f_one_plus_sqrt(1.0 + r2 * tan_theta2(v));      // float(1.0 + sqrt(...)), math.hpp
    // 2.0 / denom rounded to float: one IEEE op on float operands evaluated in double and rounded
    // once more to float is the float op itself (53 >= 2*24+2: double rounding is innocuous)
    return mask ? div_nr(2.0f, denom) : 0.0f;
  }

  // ggx.h:84-108: visible-normal sampling following [Heitz 2017]
  __device__ __forceinline__ v3 sample(v3 view, float xi0, float xi1) const
  {
    if (!((xi0 >= 0) && (xi1 >= 0) && (xi0 <= 1) && (xi1 <= 1))) return mk3(0.0f, 0.0f, 0.0f);
    const v3 vs = normalize3(mk3(view.x * au, view.y * av, view.z));
    const v3 T1 = (vs.z < 1.0 - kEpsF) ? normalize3(cross3(vs, mk3(0.0f, 0.0f, 1.0f))) : mk3(1.0f, 0.0f, 0.0f);
    const v3 T2 = cross3(T1, vs);
    const float a = float(ddiv_nr(1.0, 1.0 + vs.z));
    const float r = sqrtf(xi0);
    const float phi = float(((xi1 < a) ? double(div_nr(xi1, a)) : 1.0 + ddiv_nr(double(xi1 - a), 1.0 - a)) * kPiF);
    float sp, cp;
    if constexpr (ExactSample) sincosf_glibc(phi, &sp, &cp);
    else sincosf(phi, &sp, &cp);
    const float P1 = r * cp;
    const float P2 = float(((xi1 < a) ? 1.0 : double(vs.z)) * r * sp);
    const float sq = float(safe_sqrt(1.0 - P1 * P1 - P2 * P2));
    const v3 n = mk3((T1.x * P1 + T2.x * P2) + vs.x * sq, (T1.y * P1 + T2.y * P2) + vs.y * sq,
                     (T1.z * P1 + T2.z * P2) + vs.z * sq);
    return normalize3(mk3(n.x * au, n.y * av, float(fmax(0.0, double(n.z)))));
  }

  __device__ __forceinline__ float pdf(v3 view, v3 m, float D) const { return vndf_pdf(*this, view, m, D); }
};

// ndf::phong (include/ndf/phong.h:31-140): D = (s + 2) / (2 pi) cos^s; pdf = D |cos|; Walter's
// G1 rational with a = sqrt(0.5 s + 1) / tan (double); sampling cos = xi0^(1/(s+2)) (double pow)
struct PhongNdf
{
  static constexpr int kParams = 1;
  float sharpness;
  __device__ explicit PhongNdf(const float* p) : sharpness(p[0]) {}

  __device__ __forceinline__ float eval(v3 h) const
  {
    const float normalization = div_nr(sharpness + 2, float(2.0f * kPiD));
    const float D = powf_ref(h.z, sharpness) * normalization;    // h.z <= 0 lanes are selected away
    return (h.z > 0) ? D : 0.0f;
  }
  __device__ __forceinline__ float G1(v3 v, v3 m) const
  {
    const bool mask = (v.z > 0) && (dot3(v, m) > 0);
#ifdef BBM_HIP_PHONG_G1_IEEE
    const float a = float(sqrt(0.5 * sharpness + 1) / double(tan_theta(v)));
#else
    // the double quotient rounded to float as f_div_d (f32 seed + one f64 remainder step: the same float but within
    // ~2^-21 ulp of a midpoint) instead of the IEEE double division sequence
    const float a = f_div_d(sqrt(0.5 * sharpness + 1), double(tan_theta(v)));
#endif
    const double ad = a;
    const float g = f_div_d(3.535 * ad + 2.181 * ad * ad, 1 + 2.276 * ad + 2.577 * ad * ad);
    return mask ? ((a < 1.6) ? g : 1.0f) : 0.0f;
  }
  __device__ __forceinline__ float pdf(v3, v3 m, float D) const { return (m.z > 0) ? D * fabsf(m.z) : 0.0f; }
  __device__ __forceinline__ v3 sample(v3, float xi0, float xi1) const
  {
    if (!((xi0 >= 0) && (xi1 >= 0) && (xi0 <= 1) && (xi1 <= 1))) return mk3(0.0f, 0.0f, 0.0f);
    const float cosT = float(pow(double(xi0), 1.0 / (sharpness + 2)));
    const float sinT = float(safe_sqrt(1.0 - cosT * cosT));
    float sp, cp;
    sincosf_glibc(xi1 * float(2.0f * kPiD), &sp, &cp);
    return mk3(cp * sinT, sp * sinT, cosT);
  }
};

// ndf::studentt (include/ndf/studentt.h:34-195), Ribardiere et al. 2017; G1 via the paper's
// rational fits F21..F24 (float results of double-promoted expressions) and tgamma.
template<bool Aniso>
struct StudentT
{
  static constexpr int kParams = (Aniso ? 2 : 1) + 1;
  float au, av, gamma;
  // parameter-only factors of G1 (studentt.h:152-156), hoisted out of the per-pair path: tgamma ratio
  // (double, as the reference's bbm::tgamma of a double), S1_scale, sqrt(gamma - 1), F22(gamma), F23(gamma)
  double lam_scale;
  float s1_scale, sqrt_g1, f22, f23;
  __device__ explicit StudentT(const float* p) : au(p[0]), av(Aniso ? p[1] : p[0]), gamma(p[Aniso ? 2 : 1])
  {
    lam_scale = tgamma(gamma - 0.5) / double(tgammaf(gamma)) * kInvSqrtPiF;
    s1_scale = div_nr(powf_glibc(gamma - 1, gamma), 2 * gamma - 3);
    sqrt_g1 = sqrtf(gamma - 1);
    f22 = F22(gamma);
    f23 = F23(gamma);
  }

  template<bool EXACT = false>
  __device__ __forceinline__ float eval(v3 h) const
  {
    const float alpha2 = (1.0f * au) * av;
    const float z2 = h.z * h.z;
    const float normalization = kPiF * alpha2 * (z2 * z2);       // pow(cos, 4): powf(x, 4) = (x^2)^2 exactly rounded here
    const float sn = sqnorm2(div_nr(h.x, au), div_nr(h.y, av));
    // pow(1 + tan^2 / ((gamma - 1) alpha^2), gamma): the reference rounds a double pow; powf_fast is within
    // ~1e-6 of it (the transcendental unit where |gamma log2 x| <= 8, a double exponent beyond) instead of 227
    // f64 instructions.  EXACT (exact mode): the double power itself (f64::pow_d, ~1e-13), rounded to float --
    // the reference's float but within ~2^-19 ulp of a rounding midpoint
    const float q = div_nr(sn, (gamma - 1) * pow2f(h.z));
    float den;
    if constexpr (EXACT) den = float(f64::pow_d(1.0 + double(q), double(gamma)));
    else den = powf_fast(float(1.0 + q), gamma);
    const float D = div_nr(1.0f, normalization * den);
    return (h.z > 0) ? D : 0.0f;
  }

#ifdef BBM_HIP_STUDENT_T_DOUBLE_FITS
  __device__ __forceinline__ static float F21(float z)
  {
    const float z2 = z * z, z3 = z2 * z;
    const float num = float(1.066 * z + 2.655 * z2 + 4.892 * z3);
    const float den = float(1.038 + 2.969 * z + 4.305 * z2 + 4.418 * z3);
    return div_nr(num, den);
  }
#else
  // the per-pair fits F21 / F24 (double-promoted cubics rounded to float in the reference) as f32 Horner FMAs:
  // each cubic within ~2 ulp of the reference's float, a factor of S2 (no cancellation downstream: lambda moves by
  // ~1e-7 relative), 12 f32 FMAs instead of ~20 f64 operations per fit
  __device__ __forceinline__ static float F21(float z)
  {
    const float num = z * __builtin_fmaf(__builtin_fmaf(4.892f, z, 2.655f), z, 1.066f);
    const float den = __builtin_fmaf(__builtin_fmaf(__builtin_fmaf(4.418f, z, 4.305f), z, 2.969f), z, 1.038f);
    return div_nr(num, den);
  }
#endif
  __device__ __forceinline__ static float F22(float g)
  {
    const float g2 = g * g, g3 = g2 * g;
    return div_nr(float(14.402 - 27.145 * g + 20.574 * g2 - 2.745 * g3), float(-30.612 + 86.567 * g - 84.341 * g2 + 29.938 * g3));
  }
  __device__ __forceinline__ static float F23(float g)
  {
    const float g2 = g * g, g3 = g2 * g;
    return div_nr(float(-129.404 + 324.987 * g - 299.305 * g2 + 93.268 * g3), float(-92.609 + 256.006 * g - 245.663 * g2 + 86.064 * g3));
  }
#ifdef BBM_HIP_STUDENT_T_DOUBLE_FITS
  __device__ __forceinline__ static float F24(float z)
  {
    const float z2 = z * z, z3 = z2 * z;
    return div_nr(float(6.537 + 6.074 * z - 0.623 * z2 + 5.223 * z3), float(6.538 + 6.103 * z - 3.218 * z2 + 6.347 * z3));
  }
#else
  __device__ __forceinline__ static float F24(float z)
  {
    const float num = __builtin_fmaf(__builtin_fmaf(__builtin_fmaf(5.223f, z, -0.623f), z, 6.074f), z, 6.537f);
    const float den = __builtin_fmaf(__builtin_fmaf(__builtin_fmaf(6.347f, z, -3.218f), z, 6.103f), z, 6.538f);
    return div_nr(num, den);
  }
#endif

  // studentt.h:128-156
  __device__ __forceinline__ float G1(v3 v, v3 m) const
  {
    const bool mask = (v.z > 0) && (dot3(v, m) > 0);
    const bool normal_mask = v.z < 1.0 - kEpsF;
    const float z = v.z * div_nr(1.0f, sqrtf(sqnorm2(v.x * au, v.y * av)));
    // S1 = pow((gamma - 1) + z^2, 3/2 - gamma) / z (double in the reference), ~1e-6 via powf_fast
    const float S1 = div_nr(powf_fast((gamma - 1) + z * z, float(3.0 / 2.0 - gamma)), z);
    const float S2 = F21(z) * (f22 + f23 * F24(z));
    const double lam = lam_scale * double(s1_scale * S1 + sqrt_g1 * S2) - 0.5;
    const float lambda = normal_mask ? float(lam) : 0.0f;
#ifdef BBM_HIP_STUDENT_T_DOUBLE_FITS
    const float g = float(1.0 / (1.0 + lambda));
#else
    const float g = f_div_d(1.0, 1.0 + double(lambda));     // float(1.0 / (1.0 + lambda)) but within 2^-21 ulp of a midpoint
#endif
    return mask ? (normal_mask ? g : 1.0f) : 0.0f;
  }

  __device__ __forceinline__ float pdf(v3, v3 m, float D) const
  {
    const float p = D * m.z;
    return ((m.z > 0) && (p > 0)) ? p : 0.0f;
  }

  // studentt.h:64-90
  __device__ __forceinline__ v3 sample(v3, float xi0, float xi1) const
  {
    if (!((xi0 >= 0) && (xi1 >= 0) && (xi0 <= 1) && (xi1 <= 1))) return mk3(0.0f, 0.0f, 0.0f);
    float sp, cp;
    sincosf_glibc(float(2.0f * kPiD) * xi0, &sp, &cp);
    float normalization;
    if (Aniso)
    {
      normalization = div_nr(1.0f, sqnorm2(div_nr(cp, au), div_nr(sp, av)));
      const v3 cs = normalize3(mk3(cp * au, sp * av, 0.0f));
      cp = cs.x; sp = cs.y;
    }
    else normalization = au * au;
    const float tan2 = float((pow(double(xi1), 1.0 / (1.0 - gamma)) - 1) * (gamma - 1) * normalization);
    const float cosT = float(1.0 / sqrt(1.0 + tan2));
    const float sinT = float(safe_sqrt(1.0 - cosT * cosT));
    return mk3(cp * sinT, sp * sinT, cosT);
  }
};

// ndf pdf shared by Beckmann/GGX VNDF sampling (declared before use by the NDF structs below) (beckmann.h:149-170, ggx.h:142-163):
// D(m) * G1(view, m) * |view.m| / cos(view), masked to pdf > 0.  D(m) is passed in (already
// computed by eval on the same halfway vector).
template<class NDF>
__device__ __forceinline__ float vndf_pdf(const NDF& ndf, v3 view, v3 m, float D)
{
  float pdf = D;
  pdf *= div_nr(ndf.G1(view, m) * fabsf(dot3(view, m)), view.z);
  return ((m.z > 0) && (pdf > 0)) ? pdf : 0.0f;
}

// ---------------------------------------------------------------------- masking-shadowing

// maskingshadowing::vgroove (include/maskingshadowing/vgroove.h:30-47): the `2.0` literal makes
// both ratios double; bbm::min -> fmin(double); the result is cast back to the G1 return type.
struct VGroove
{
  template<class NDF>
  __device__ __forceinline__ static float eval(const NDF&, v3 in, v3 out, v3 m, float inm, float outm)
  {
    // min(1, Pi/inm, Po/outm) with Pi = 2 z_m z_in, exact in double in the reference; here the exact
    // product is an f32 pair (2 z_m is exact), the comparisons with 1 are exact, and only the
    // smaller ratio is divided -- one compensated f32 division, no f64.
    const float tm = 2.0f * m.z;
    float pih, pil, poh, pol;
    two_prod(tm, in.z, pih, pil);
    two_prod(tm, out.z, poh, pol);
    const bool li = (pih < inm) || (pih == inm && pil < 0.0f);
    const bool lo = (poh < outm) || (poh == outm && pol < 0.0f);
    const bool use_i = li && (!lo || pih * outm <= poh * inm);
    const float g = div_ff(use_i ? pih : poh, use_i ? pil : pol, use_i ? inm : outm, 0.0f);
    return ((inm > 0) && (outm > 0)) ? ((li || lo) ? g : 1.0f) : 0.0f;
  }
};

// maskingshadowing::uncorrelated (include/maskingshadowing/uncorrelated.h:30-42)
struct Uncorrelated
{
  template<class NDF>
  __device__ __forceinline__ static float eval(const NDF& ndf, v3 in, v3 out, v3 m, float inm, float outm)
  {
    const float g = ndf.G1(in, m) * ndf.G1(out, m);
    return ((inm > 0) && (outm > 0)) ? g : 0.0f;
  }
};

// maskingshadowing::heightcorrelated (include/maskingshadowing/heightcorrelated.h:30-54), Heitz 2014 Eq. 99
struct HeightCorrelated
{
  template<class NDF>
  __device__ __forceinline__ static float eval(const NDF& ndf, v3 in, v3 out, v3 m, float inm, float outm)
  {
    const float gi = ndf.G1(in, m), go = ndf.G1(out, m);
    const float gio = gi * go;
    const float denom = gi + go - gio;
    const float g = div_nr(gio, denom);
    return ((inm > 0) && (outm > 0) && (denom > kEpsF)) ? g : 0.0f;
  }
};

// The Low NDF's double power in every mode (A/B: -DBBM_HIP_LOW_EXACT_DEFAULT); by default powf_fast (~1e-6) outside
// exact mode: the double power cost LowMicrofacet(Fit) +8.5 % per 10 M pairs (profiles/r05_ab_low_exact.txt)
#ifdef BBM_HIP_LOW_EXACT_DEFAULT
constexpr bool kLowExactDefault = true;
#else
constexpr bool kLowExactDefault = false;
#endif

// ndf::low (include/ndf/low.h:32-141): the unnormalised ABC "S" term of [Low 2012] as an NDF.
// eval pow(1 + B (1 - z), -C) in double; pdf = eval B (1/(2 pi)) normalization with the
// normalization a per-thread double constant; sample inverts the marginal CDF of cos(theta)
// (not a visible-normal sampler: the view is ignored); G1 = 1 (Low uses v-groove shadowing).
struct LowNdf
{
  static constexpr int kParams = 2;
  float B, C, norm_pdf;
  double lg1pB, pw1pB, inv_exp;
  bool c_is_one;
  __device__ explicit LowNdf(const float* p) : B(p[0]), C(p[1])
  {
    c_is_one = fabsf(C - 1) < kEpsF;
    lg1pB = log(1.0 + B);
    pw1pB = pow(1.0 + B, 1.0 - C);
    inv_exp = -1.0 / (C - 1.0);
    const float normalization = float(c_is_one ? 1.0f / lg1pB : (C - 1.0) / (1.0 - pw1pB));
    norm_pdf = kInvPiHalfF * normalization;
  }

  template<bool EXACT = false>
  __device__ __forceinline__ float eval(v3 h) const
  {
    // pow(1 + B (1 - z), -C) in double in the reference; powf_fast: within ~1e-6; EXACT (exact mode): the double
    // power (f64::pow_d) of the double base, rounded to float
    float S;
    if constexpr (EXACT || kLowExactDefault) S = float(f64::pow_d(1.0 + double(B) * (1.0 - double(h.z)), -double(C)));
    else S = powf_fast(float(1.0 + B * (1.0 - h.z)), -C);
    return (h.z > 0) ? S : 0.0f;
  }

  __device__ __forceinline__ float G1(v3, v3) const { return 1.0f; }

  // low.h:67-89
  __device__ __forceinline__ v3 sample(v3, float xi0, float xi1) const
  {
    if (!((xi0 >= 0) && (xi1 >= 0) && (xi0 <= 1) && (xi1 <= 1))) return mk3(0.0f, 0.0f, 0.0f);
    const float term = float(c_is_one ? exp(xi0 * lg1pB) : pow(1.0 + xi0 * (pw1pB - 1.0), inv_exp));
    const float cosT = float((1.0 + B - term) / B);
    const float sinT = float(safe_sqrt(1.0 - cosT * cosT));
    float sp, cp;
    sincosf_glibc(xi1 * float(2.0f * kPiD), &sp, &cp);
    return mk3(cp * sinT, sp * sinT, cosT);
  }

  // low.h:96-112: mask m.z > 0 (via eval) and pdf > 0
  __device__ __forceinline__ float pdf(v3, v3, float D) const
  {
    const float p = D * B * norm_pdf;
    return (p > 0) ? p : 0.0f;
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
    // c = (in.h + out.h) / 2 in (0, 1] where the result is used and g >= 0, for ANY eta (the attribute's bound
    // eta >= 1, bsdf_attribute.h:89, is metadata the reference does not enforce): g + c >= c is a positive normal
    // float, and c (g - c) + 1 is either 0 (only at eta = 0 with c = 1, where the numerator is 0 as well: NaN in
    // both) or >= 2^-24 (1 - c^2 near 1 is a multiple of float steps); both quotients are normal, 0 or that NaN,
    // where the Markstein step alone (div_nr_n) is the IEEE quotient
    const float a = div_nr_n(g - c, g + c);
    const float b = div_nr_n(c * (g + c) - 1.0f, c * (g - c) + 1.0f);
    return fmaxf(0.5f * (a * a) * (1.0f + b * b), 0.0f);   // bbm::max(x, 0.0): fmax in double == fmaxf here
  }
};

// fresnel::schlick with a reflectance parameter (include/bbm/fresnel_schlick.h:42-53):
// R0 + (1 - R0) * pow(1 - cos, 5.0) in double (pow(x, 5.0) of a float x: x^2 exact, then two
// rounded products -- within 1.5 double ulp, below the final float rounding)
struct FresnelSchlick
{
  static constexpr int kParams = 1;
  float r0;
  __device__ explicit FresnelSchlick(const float* p) : r0(p[0]) {}
  __device__ __forceinline__ float eval(float c) const
  {
    const double x = double(1.0f - c);
    const double x2 = x * x;
    return float(r0 + double(1.0f - r0) * (x2 * x2 * x));
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

// float((x / NormalizationFactor) / y) for float x, y (microfacet.h:100).  Walter (4.0) and
// Unnormalized divide exactly by a power of two, so the double expression is one float division.
// Cook (pi): the reference's two double quotients are within ~2^-52 of x / (pi y); here pi y is
// formed as an f32 pair (pi = kPiHi + kPiLo to ~2^-48) and divided with the compensated f32
// quotient, so the float result agrees except within ~2^-20 ulp of a rounding midpoint.
constexpr float kPiHi = 3.14159274101257324f;    // RN_f(pi)
constexpr float kPiLo = -8.74227766e-08f;        // RN_f(pi - kPiHi)

template<Norm N, bool EXACT = false>
__device__ __forceinline__ float eval_scale(float x, float y)
{
  if (N == Norm::Cook)
  {
    float dh, dl;
    two_prod(y, kPiHi, dh, dl);
    dl = __builtin_fmaf(y, kPiLo, dl);
    return div_ff_sub<EXACT>(x, dh, dl);
  }
  // Walter: (x / 4.0) / y in double = x / (4 y), 4 y exact in float (x * 0.25f would round a subnormal x)
  return div_sub<EXACT>(x, N == Norm::Walter ? 4.0f * y : y);
}

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

  // EXACT (bbm_hip_set_exact_subnormals): the quotients a subnormal intermediate can reach rounded on the subnormal
  // grid as the reference's IEEE divisions are (div_sub) -- for NDFs with such an evaluation (Beckmann)
  static constexpr bool kHasExact = requires(const NDF& d, v3 v) { d.template eval<true>(v); };

  // microfacet.h:74-102 (eval) + :154-174 (pdf), fused: both share the halfway vector and D(h).
  template<int MODE, bool EXACT = false>
  __device__ __forceinline__ void eval_pdf(v3 in, v3 out, uint32_t component, float* rgb, float& pdf) const
  {
    // Branch-free: every term is computed and the masks are applied with selects, so the four
    // pairs a thread owns share one basic block and the scheduler interleaves them (this hides
    // the VALU->mask and transcendental hazards that otherwise cost an s_nop per compare).
    // eval :77-83 and pdf :160-164 test the same lanes: Specular component, z_in > 0, z_out > 0.
    const bool active = (component & kFlagSpecular) && (in.z > 0.0f) && (out.z > 0.0f);
    const v3 h = halfway(in, out);
    // pdf's `h = z(h) < 0 ? -h : h` (:167) never fires on active lanes: z(in + out) > 0 and
    // normalize scales by a positive factor, so h is used as is.
    float D;
    if constexpr (EXACT && kHasExact) D = ndf.template eval<true>(h);
    else D = ndf.eval(h);
    const float outh = dot3(out, h);
    if (MODE & kModeEval)
    {
      const float inh = dot3(in, h);
      const float G = MS::eval(ndf, in, out, h, inh, outh);
      const float F = fresnel.eval(0.5f * (inh + outh));
      // (D G F) / NormalizationFactor / (z_in z_out): literal<double> promotes to double
      const float res = eval_scale<N, EXACT && kHasExact>(D * G * F, in.z * out.z);
      rgb[0] = active ? (Scaled ? res * albedo[0] : res) : 0.0f;
      rgb[1] = active ? (Scaled ? res * albedo[1] : res) : 0.0f;
      rgb[2] = active ? (Scaled ? res * albedo[2] : res) : 0.0f;
    }
    else rgb[0] = rgb[1] = rgb[2] = 0.0f;
    if (MODE & kModePdf)
    {
      // float(p / (4.0 * |o.h|)): float operands, one double op -> identical to the float division
      const float p = div_sub<EXACT && kHasExact>(ndf.pdf(out, h, D), 4.0f * fabsf(outh));
      pdf = active ? p : 0.0f;
    }
    else pdf = 0.0f;
  }

  // microfacet.h:182-196 reflectance: mirror approximation Fresnel(eta, z(out)) / N * 4.0 (double),
  // x albedo (scaledmodel.h:64-67); Specular component and z(out) > 0, else 0.
  __device__ __forceinline__ void reflectance(v3 out, uint32_t component, float* rgb) const
  {
    const bool m = (component & kFlagSpecular) && (out.z > 0);
    const float f = float(double(fresnel.eval(out.z)) / norm_value<N>::v * 4.0);
#pragma unroll
    for (int c = 0; c < 3; ++c) rgb[c] = m ? (Scaled ? f * albedo[c] : f) : 0.0f;
  }

  // microfacet.h:115-141 sample: m ~ VNDF(out), direction = reflect(out, m)
  // (core/vec_transform.h:43-44, `m * dot(m, out) * 2.0 - out`: the double subtraction of two float
  // values rounded to float is the float subtraction), pdf = microfacet pdf of that direction.
  __device__ __forceinline__ void sample(v3 out, float xi0, float xi1, uint32_t component, v3& dir, float& pdf,
                                         uint32_t& flag) const
  {
    dir = mk3(0.0f, 0.0f, 0.0f);
    pdf = 0.0f;
    flag = kFlagNone;
    if (!(component & kFlagSpecular)) return;
    if (!((xi0 >= 0) && (xi1 >= 0) && (xi0 <= 1) && (xi1 <= 1))) return;
    if (!(out.z > 0)) return;
    const v3 m = ndf.sample(out, xi0, xi1);
    const float d = dot3(m, out);
    dir = mk3(2.0f * (m.x * d) - out.x, 2.0f * (m.y * d) - out.y, 2.0f * (m.z * d) - out.z);
    float rgb[3];
    eval_pdf<kModePdf>(dir, out, component, rgb, pdf);
    flag = kFlagSpecular;
  }

  // sample() followed by eval(dir, out): the sample's pdf IS pdf(dir, out) (microfacet.h:135), so one fused
  // eval_pdf at the sampled direction returns both -- one halfway vector and one D instead of two, results
  // bit-identical to the separate calls (the fused kernel's contract, tests/test_gpu_parity.py).  checkBsdf's
  // importance-sampled reflectance (config 4) uses it.
  static constexpr bool kFusedSampleEval = true;
  __device__ __forceinline__ void sample_eval(v3 out, float xi0, float xi1, uint32_t component, v3& dir, float* rgb,
                                              float& pdf, uint32_t& flag) const
  {
    dir = mk3(0.0f, 0.0f, 0.0f);
    pdf = 0.0f;
    flag = kFlagNone;
    rgb[0] = rgb[1] = rgb[2] = 0.0f;
    if (!(component & kFlagSpecular)) return;
    if (!((xi0 >= 0) && (xi1 >= 0) && (xi0 <= 1) && (xi1 <= 1))) return;
    if (!(out.z > 0)) return;
    const v3 m = ndf.sample(out, xi0, xi1);
    const float d = dot3(m, out);
    dir = mk3(2.0f * (m.x * d) - out.x, 2.0f * (m.y * d) - out.y, 2.0f * (m.z * d) - out.z);
    eval_pdf<kModeEvalPdf>(dir, out, component, rgb, pdf);
    flag = kFlagSpecular;
  }
};

template<bool A, bool N> struct exact_sample<Beckmann<A, N>> { using type = Beckmann<A, N, true>; };
template<bool A> struct exact_sample<GGX<A>> { using type = GGX<A, true>; };
template<class NDF, class MS, class FRESNEL, Norm N, bool Scaled>
struct exact_sample<Microfacet<NDF, MS, FRESNEL, N, Scaled>>
{ using type = Microfacet<exact_sample_t<NDF>, MS, FRESNEL, N, Scaled>; };

}  // namespace bbmhip
