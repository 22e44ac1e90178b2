// bbm_amd/csrc/spectral.hpp -- microfacet models whose NDF, shadowing and Fresnel terms are
// Spectrum-valued (one value per RGB channel), i.e. Bagher et al.'s Shifted Gamma Distribution
// model (include/bsdfmodel/bagher.h:62-68):
//
//   scaledmodel< microfacet< ndf::sgd, maskingshadowing::uncorrelated, fresnel::bagher, Cook (pi) > >
//
// Parameters (attribute declaration order, bbm::parameter_values incl. Dependent, 30 floats):
//   albedo[3], K[3], Lambda[3], c[3], theta0[3], k[3]   (ndf::sgd, ndf/sgd.h:197-203)
//   alpha[3], p[3]                                     (ndf::sgd_base, ndf/sgd.h:107-111)
//   eta[2][3] = (F0 RGB, F1 RGB)                       (fresnel::bagher, bagher.h:27-57)
// Sampling and pdf use a GGX<Isotropic> lobe with the channel-averaged alpha (ndf/sgd.h:73-93).
//
// The per-pair geometry (halfway vector, its tan^2, theta(in), theta(out), cos(theta_h)^4) is
// channel-independent and computed once; only the channel terms run three times.
#pragma once
#include "microfacet.hpp"

namespace bbmhip {

// spherical::theta(v) (include/core/spherical.h:26-32): 2.0 * asin(0.5 * |v - (0,0,sign(z))|), evaluated
// by the reference in double and returned as float; for z < 0, Pi - that.  theta_of keeps that (the
// linearizers, checkBsdf binning and the Bagher shadowing term use it -- the latter is so ill-conditioned
// for published fits that a 1-ulp different theta moves G by 1e-2, so theta is rounded from f64 as there).
//
// The double asin as a short polynomial: y = |v - pole| / 2 lies in [0, sqrt2 / 2]; asin y = y + y z P(z), z = y^2,
// for y <= 1/2, and pi/2 - 2 asin s with s = sqrt((1 - y) / 2) <= 1/2 above (w = (1 - y) / 2 exact in double).  P is
// the asin series economised on Chebyshev nodes over z in [0, 1/4] to degree 11 (truncation 2^-49 of P, well below
// double rounding once scaled by z / 6; coefficients from exact rational arithmetic, tools/asin_poly.py): the result
// is within a few double ulps of glibc's asin.  Its float is the reference's unless the double lies within 256 ulps of
// a float rounding midpoint (~1e-6 of the lanes, and any NaN): those take the device library's double asin, as
// before.  ~20 f64 VALU against ~70 f64 + ~60 other for the library asin.
namespace asin_poly {
constexpr double kP[12] = {
    0x1.555555555554ep-3, 0x1.3333333337110p-4, 0x1.6db6db68067fep-5,
    0x1.f1c71fb700f11p-6, 0x1.6e8b26f89d407p-6, 0x1.1c598c739143cp-6,
    0x1.c86b17413a7b6p-7, 0x1.8559b6cfd3c89p-7, 0x1.fd4f1fa1ac91cp-8,
    0x1.084522a849f25p-6, -0x1.65717d3785d18p-7, 0x1.cf6d7d2572a46p-6};
__device__ __forceinline__ double eval(double z)
{
  double p = kP[11];
#pragma unroll
  for (int k = 10; k >= 0; --k) p = __builtin_fma(p, z, kP[k]);
  return p;
}
}  // namespace asin_poly

// the guard's fallback, out of line: the library asin's registers would otherwise count against every kernel
__device__ __attribute__((noinline, pure)) inline double theta_lib(double y, bool below)
{
  const double te = 2.0 * asin(y);
  return below ? double(kPiF) - te : te;
}

__device__ __forceinline__ float theta_of(v3 v)
{
  const float sz = (v.z < 0.0f) ? -1.0f : 1.0f;          // bbm::sign = copysign(1, z)
  const float dz = v.z - sz;
  const float nrm = sqrtf(((0.0f + v.x * v.x) + v.y * v.y) + dz * dz);
  const double y = 0.5 * double(nrm);
  const bool hi = y > 0.5;
  const double w = hi ? (1.0 - y) * 0.5 : y * y;
  // sqrt(w) for the upper range (w in [0.146, 0.25]): rsq seed, two Newton steps (~2^-90 before rounding)
  const double g = __builtin_amdgcn_rsq(w);
  double sq = w * g;
  sq = __builtin_fma(__builtin_fma(-sq, sq, w), 0.5 * g, sq);
  sq = __builtin_fma(__builtin_fma(-sq, sq, w), 0.5 * g, sq);
  const double s = hi ? sq : y;
  const double r = __builtin_fma(s * w, asin_poly::eval(w), s);
  const double t = 2.0 * (hi ? 0x1.921fb54442d18p+0 - 2.0 * r : r);
  double u = (v.z >= 0) ? t : double(kPiF) - t;
  const uint32_t lo = uint32_t(__builtin_bit_cast(uint64_t, u)) & 0x1fffffffu;
  if (__builtin_expect(((lo - 0x0fffff00u) < 0x200u) || (u != u), false)) u = theta_lib(y, !(v.z >= 0));
  return float(u);
}

// sgd_base::eval x K for a channel whose (alpha, p) lies outside the attributes' range: IEEE quotients, glibc's powf
// with its negative-base and special-operand rules, expf with overflow.  Out of line for the eval kernels: inlined into
// the channel block its code cost Bagher's eval 15 % although no valid launch runs it (profiles/r06_ab_bagher_range.txt).
static __device__ __attribute__((noinline)) float p22_general(float alpha, float p, float tan2)
{
  const float t = alpha + tan2 / alpha;
  const float den = powf_glibc_any(t, p);
  return (den > kEpsF) ? expf_glibc(-t) / den : 0.0f;
}

struct Bagher
{
  static constexpr bool kHasGeo = true;      // geometry() / eval_geo(): the loss kernel shares the prelude per pair
  static constexpr int kParams = 30;
  static constexpr uint32_t kComponent = kFlagSpecular;
  float albedo[3], K[3], Lambda[3], c[3], theta0[3], k[3], alpha[3], p[3], F0[3], F1[3];
  float qc0[3], qc_min;   // conservative squared-chord thresholds of theta > theta0 (see G1 below)
  GGX<false> ggx;   // sampling / pdf lobe (ndf/sgd.h:73-93)

  __device__ static float avg_alpha(const float* a) { return div_nr(((0.0f + a[0]) + a[1]) + a[2], 3.0f); }

  __device__ explicit Bagher(const float* q) : ggx(q + 18)
  {
    for (int j = 0; j < 3; ++j)
    {
      albedo[j] = q[j]; K[j] = q[3 + j]; Lambda[j] = q[6 + j]; c[j] = q[9 + j]; theta0[j] = q[12 + j];
      k[j] = q[15 + j]; alpha[j] = q[18 + j]; p[j] = q[21 + j]; F0[j] = q[24 + j]; F1[j] = q[27 + j];
      // theta = 2 asin(|v - (0, 0, 1)| / 2) > theta0 needs |v - (0, 0, 1)|^2 > 4 sin^2(theta0 / 2); the threshold is
      // lowered by 2^-10 relative, far beyond every rounding of either side, so a lane below it has theta <= theta0
      const float sh = sinf(0.5f * theta0[j]);
      qc0[j] = (theta0[j] <= 0.0f) ? -1.0f : ((theta0[j] >= kPiF) ? 5.0f : 4.0f * sh * sh * (1.0f - 0x1p-10f));
    }
    qc_min = fminf(fminf(qc0[0], qc0[1]), qc0[2]);
    ggx.au = ggx.av = avg_alpha(alpha);
  }
  __device__ __forceinline__ static float chord2(v3 v)       // |v - (0, 0, 1)|^2 for z(v) >= 0
  {
    const float dz = v.z - 1.0f;
    return ((0.0f + v.x * v.x) + v.y * v.y) + dz * dz;
  }

  // ndf::sgd::G1 per channel (ndf/sgd.h:157-193), for a direction with theta(v) = th
  __device__ __forceinline__ float G1(int j, float th) const
  {
    // 1 + Lambda (1 - exp(c pow(...))) cancels catastrophically for published fits (fits/bagher_sgd.fit:
    // k ~ 48, c ~ 1e-7 -> g ~ 5e-4 at grazing angles): theta, pow and exp must be the reference's own floats --
    // glibc's powf and expf restated bit for bit (math.hpp; the correctly rounded power differs from glibc's on ~0.1 %
    // of the lanes, and each such lane moved G by up to 1e-2 relative).  th - theta0 may be <= 0 on lanes the select
    // below discards.
    return (th > theta0[j]) ? g1_tail(th - theta0[j], c[j], k[j], Lambda[j]) : 1.0f;
  }
  // 1 + Lambda (1 - exp(c d^k)) out of line: the exact powf / expf hold ~40 VGPRs of f64 temporaries, and inlined
  // into each of the six (channel, direction) branches they set the register budget of every kernel around them
  // (the loss kernel spilled 124 VGPRs instead of 69) although at the default theta0 = pi/2 no lane takes them
  __device__ __attribute__((noinline, pure)) static float g1_tail(float d, float c, float k, float Lambda)
  {
    // the constant-segment tables here: this out-of-line tail reading the kernel's LDS copies cost the fitting loss
    // kernel (8 waves per SIMD, spilling) ~13 % per compass step
    return 1.0f + Lambda * (1.0f - expf_glibc<false>(c * powf_glibc<false>(d, k)));
  }
  // the same for an upper-hemisphere direction with squared chord q: lanes below the conservative threshold have
  // theta <= theta0 and G1 = 1; the others evaluate G1 exactly as above, on a branch (the shadowing term's double
  // pow and exp are skipped where no lane of the wave needs them -- at the default theta0 = pi/2, every lane)
  __device__ __forceinline__ float G1q(int j, float q, float th) const
  {
    float g = 1.0f;
    if (q > qc0[j]) g = G1(j, th);
    return g;
  }

  // The parameter-independent part of eval (the halfway vector, its tan^2, cos^4 pi, the masks, the chords and
  // the Schlick base), computed once per direction pair and shared by every parameter vector evaluated at it (the
  // fitting loss evaluates 2P probes per pair, kernels.hpp k_loss).  theta(in) / theta(out) are filled on first
  // need (th < 0: not yet), since only lanes beyond a probe's theta0 use them.
  struct Geo
  {
    v3 in, out, h;
    float outh, tan2, q_in, q_out, th_in, th_out, cosF, zz;
    double dnorm, x5;
    bool sdirs, gmask;
    // the fitting loss's per-pair cache of the NDF term P22 = e^-t / t^p per channel, with the (alpha, p) it was
    // computed for, filled by the pair's first probe: a compass step's probes each move one parameter off the current
    // point, so all but the probes on channel j's alpha or p reuse it (eval_geo<..., true>).  Measured on config 5, ms
    // per compass step (profiles/r05_ab_fit_p22_cache.txt): no cache 0.675, refilled on every miss 0.438, filled
    // once 0.425; the round-4 fast D 0.411
    float ca[3], cp[3], cP22[3];
  };

  __device__ __forceinline__ static Geo geometry(v3 in, v3 out)
  {
    Geo g;
    g.in = in;
    g.out = out;
    g.sdirs = (in.z > 0.0f) && (out.z > 0.0f);
    g.h = halfway(in, out);
    g.outh = dot3(out, g.h);
    const float inh = dot3(in, g.h);
    g.tan2 = tan_theta2(g.h);
    const double z2 = double(g.h.z) * double(g.h.z);
    g.dnorm = double(kPiF) * (z2 * z2);      // Constants::Pi() * pow(cos, 4.0) (sgd.h:62)
    // uncorrelated (uncorrelated.h:30-42) + sgd::G1 masks: z(v) > 0 and v.m > 0 for both
    g.gmask = (inh > 0) && (g.outh > 0);
    g.q_in = chord2(in);
    g.q_out = chord2(out);
    g.th_in = g.th_out = -1.0f;
    g.cosF = 0.5f * (inh + g.outh);
    const double x = double(1.0f - g.cosF);
    g.x5 = (x * x) * (x * x) * x;
    g.zz = in.z * out.z;
    for (int j = 0; j < 3; ++j) g.ca[j] = g.cp[j] = g.cP22[j] = __builtin_nanf("");   // no cached term yet
    return g;
  }

  // eval (Specular component) at a prepared pair.  The NDF's power and exponential are glibc's own powf / expf (round
  // 5: by default; round 4 only in exact mode), so D is the reference's float -- Bagher and Aggregate(Lambertian,
  // Bagher) bit-identical on nearly every lane (the rest below 1e-30); +13 % kernel time against round 4's fast D
  // (0.108 -> 0.122 ms per 10 M pairs on one box, profiles/r05_ab_bagher_exact_d.txt; round 4's exact form: +68 %):
  // the LDS tables, the positive-normal powf, and the three channels' D chains in one branch-free block.  EXACT (exact
  // mode) adds the subnormal quotients of eval_scale.
  // EXACT_D = false (A/B builds with -DBBM_HIP_BAGHER_FAST_D): the round-4 D by powf_fast / expf_dn (~1e-6 relative).
  // CACHE (the fitting loss kernels): reuse the pair's P22 of channel j where the probe's (alpha_j, p_j) equal the
  // ones it was computed for -- the same float, computed once instead of once per probe.
#ifdef BBM_HIP_BAGHER_FAST_D
  static constexpr bool kExactD = false;
#else
  static constexpr bool kExactD = true;
#endif
  template<bool EXACT = false, bool EXACT_D = kExactD, bool CACHE = false>
  __device__ __forceinline__ void eval_geo(Geo& g, uint32_t component, float* rgb) const
  {
    const bool active = (component & kFlagSpecular) && g.sdirs;
    // the three channels' NDF terms first, in one branch-free block (eval): their dependent f64 and LDS-table chains
    // interleave there, where the shadowing branches below would otherwise serialise them channel by channel
    float P22[3];
#pragma unroll
    for (int j = 0; j < 3; ++j)
    {
      bool hit = false;
      if constexpr (CACHE) hit = (alpha[j] == g.ca[j]) && (p[j] == g.cp[j]);
      if (hit) P22[j] = g.cP22[j];
      else
      {
        // sgd_base::eval (sgd.h:48-63) x K (sgd.h:143-154): exp(-t) / t^p with t = alpha + tan^2 / alpha
        if (!(alpha[j] >= 0x1p-126f && alpha[j] < __builtin_inff() && __builtin_isfinite(p[j]))) [[unlikely]]
        {
          // a parameter outside the attribute's range (the reference accepts any alpha / p): the general forms, out
          // of line in the eval kernels (p22_general) and inline in the loss kernels (CACHE), where the call cost the
          // config-5 step 19 %.  The parameters are uniform per launch (per probe in the loss), so this branch never
          // splits a wave.
          if constexpr (CACHE)
          {
            const float t = alpha[j] + g.tan2 / alpha[j];
            const float den = powf_glibc_any(t, p[j]);
            P22[j] = (den > kEpsF) ? expf_glibc(-t) / den : 0.0f;
          }
          else P22[j] = p22_general(alpha[j], p[j], g.tan2);
          continue;                                              // (never cached: only valid parameters fill it)
        }
        const float t = alpha[j] + div_nr(g.tan2, alpha[j]);
        if constexpr (EXACT || EXACT_D)
        {
          // glibc's powf and expf restated (math.hpp), so D is the reference's float.  t >= alpha >= the parameter's
          // lower bound (Epsilon, bsdf_attribute.h:77) is a normal float (or +inf where tan^2 is, which gives the
          // reference's P22 = 0 here as well), so the power takes glibc's path for normal positive bases
          const float den = powf_glibc_pos(t, p[j]);
          P22[j] = (den > kEpsF) ? div_nr(expf_glibc_neg(-t), den) : 0.0f;
        }
        else
        {
          const float den = powf_fast(t, p[j]);
          P22[j] = (den > kEpsF) ? div_nr(expf_dn(-t), den) : 0.0f;
        }
        if constexpr (CACHE)
        if (g.ca[j] != g.ca[j])   // filled by the pair's first probe only (see Geo)
        {
          g.ca[j] = alpha[j];
          g.cp[j] = p[j];
          g.cP22[j] = P22[j];
        }
      }
    }
    // in.z, out.z > 0 on every lane whose result is used: theta_of only where a channel may need it
    if (g.q_in > qc_min && g.th_in < 0.0f) g.th_in = theta_of(g.in);
    if (g.q_out > qc_min && g.th_out < 0.0f) g.th_out = theta_of(g.out);
#pragma unroll
    for (int j = 0; j < 3; ++j)
    {
      const float Dj = ((g.h.z > 0) ? f_div_d(double(P22[j]), g.dnorm) : 0.0f) * K[j];
      const float Gj = g.gmask ? G1q(j, g.q_in, g.th_in) * G1q(j, g.q_out, g.th_out) : 0.0f;
      // fresnel::bagher (bagher.h:46-49): schlick(F0) rounded to float, minus F1 cos
      const float S = float(double(F0[j]) + double(1.0f - F0[j]) * g.x5);
      const float Fj = S - F1[j] * g.cosF;
      const float res = eval_scale<Norm::Cook, EXACT>((Dj * Gj) * Fj, g.zz);
      rgb[j] = active ? res * albedo[j] : 0.0f;
    }
  }

  __device__ __forceinline__ void eval_geo_cached(Geo& g, uint32_t component, float* rgb) const
  {
#ifdef BBM_HIP_BAGHER_NO_P22_CACHE
    eval_geo<false, kExactD, false>(g, component, rgb);   // A/B
#else
    eval_geo<false, kExactD, true>(g, component, rgb);
#endif
  }

  static constexpr bool kHasExact = true;
  template<int MODE, bool EXACT = false>
  __device__ __forceinline__ void eval_pdf(v3 in, v3 out, uint32_t component, float* rgb, float& pdf) const
  {
    Geo g = geometry(in, out);
    // the pdf first: straight-line code that schedules with the geometry and eval_geo's NDF block
    if (MODE & kModePdf)
    {
      const bool active = (component & kFlagSpecular) && g.sdirs;
      const float Dg = ggx.eval(g.h);
      const float pp = div_nr(ggx.pdf(out, g.h, Dg), 4.0f * fabsf(g.outh));
      pdf = active ? pp : 0.0f;
    }
    else pdf = 0.0f;
    if (MODE & kModeEval) eval_geo<EXACT>(g, component, rgb);
    else rgb[0] = rgb[1] = rgb[2] = 0.0f;
  }

  // microfacet.h:182-196 with fresnel::bagher at cos = z(out), x albedo (scaledmodel.h:64-67)
  __device__ __forceinline__ void reflectance(v3 out, uint32_t component, float* rgb) const
  {
    const bool m = (component & kFlagSpecular) && (out.z > 0);
    const double x = double(1.0f - out.z);
    const double x5 = (x * x) * (x * x) * x;
#pragma unroll
    for (int j = 0; j < 3; ++j)
    {
      const float S = float(double(F0[j]) + double(1.0f - F0[j]) * x5);
      const float F = S - F1[j] * out.z;
      rgb[j] = m ? float(double(F) / kPiD * 4.0) * albedo[j] : 0.0f;
    }
  }

  // microfacet.h:115-141 with the GGX(avg alpha) visible-normal sampler
  __device__ __forceinline__ void sample(v3 out, float xi0, float xi1, uint32_t component, v3& dir, float& pdf,
                                         uint32_t& flag) const
  {
    dir = mk3(0.0f, 0.0f, 0.0f);
    pdf = 0.0f;
    flag = kFlagNone;
    if (!(component & kFlagSpecular)) return;
    if (!((xi0 >= 0) && (xi1 >= 0) && (xi0 <= 1) && (xi1 <= 1))) return;
    if (!(out.z > 0)) return;
    const v3 m = ggx.sample(out, xi0, xi1);
    const float d = dot3(m, out);
    dir = mk3(2.0f * (m.x * d) - out.x, 2.0f * (m.y * d) - out.y, 2.0f * (m.z * d) - out.z);
    float rgb[3];
    eval_pdf<kModePdf>(dir, out, component, rgb, pdf);
    flag = kFlagSpecular;
  }
};

}  // namespace bbmhip
