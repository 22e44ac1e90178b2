// bbm_amd/csrc/he.hpp -- He et al. 1991's physically based BSDF (include/bsdfmodel/he.h:115-482) with
// BBM's data-driven importance sampler (include/bbm/ndf_sampler.h, include/ndf/sampler.h):
//
//   He           = ndf_sampler< he_base< complex Fresnel (RGB), WithoutExp, Regular, 4 NR steps, 64 Taylor, adaptive, 18 > >
//   HeWestin     = ndf_sampler< he_base< complex Fresnel (RGB), Errata,     Westin,  4, 64, adaptive, 18 > >
//   HeHolzschuch = ndf_sampler< he_base< complex Fresnel (RGB), Errata,     Regular, 4, 10, fixed,   none > >
//   NganHe       = scaledmodel< ndf_sampler< he_base< cook Fresnel (scalar), Errata, Westin, 4, 64, adaptive, 18 > > >
//                  (include/bsdfmodel/he.h:489-496, ngan.h:166-167)
//
// eval = the He model term by term (shadowing S, geometry G, the Taylor-series distribution D, Fresnel);
// sample / pdf use a 90-bin CDF over theta_h of the model's own backscatter eval(h, h) (ndf/sampler.h:143-181).
// That CDF depends on the parameters and the sampled component, so it is built per launch on the GPU
// (k_he_cdf: 90 evaluations + the serial float prefix sum of util/cdf.h:39-47) into stream-ordered
// scratch memory (scratch_acquire) whose address travels in the parameter block after the model's parameters; the kernels
// read it from there (host_params<He<...>> below).  No host synchronisation.
#pragma once
#include "math.hpp"
#include "microfacet.hpp"
#include "fit.hpp"       // theta_of, sph_to_vec, cossin_cr
#include "kernels.hpp"   // host_params, ParamBlock

namespace bbmhip {

constexpr int kHeBins = 90;                                      // samplesTheta (he.h:490)
constexpr float kPiHalfF = float(0.5 * kPiD);                    // Constants::Pi(0.5)
constexpr float kPiSqQuarterF = (0.25f * kPiF) * kPiF;           // Constants::Pi2(0.25) = scale * Pi() * Pi() in float
constexpr float kPiSqFourF = (4.0f * kPiF) * kPiF;               // Constants::Pi2(4)
// floatRGB::wavelength() (backbone/native/include/backbone.h:36), in micron
constexpr float kWavelength[3] = {float(0.645), float(0.526), float(0.444)};

// the CDF pointer rides in two parameter slots (param_ptr / set_param_ptr, kernels.hpp)

// std::lerp for floats (libstdc++ <cmath>)
__device__ __forceinline__ float std_lerpf(float a, float b, float t)
{
  if ((a <= 0 && b >= 0) || (a >= 0 && b <= 0)) return t * b + (1 - t) * a;
  if (t == 1) return b;
  const float x = a + t * (b - a);
  return ((t > 1) == (b > a)) ? ((b < x) ? x : b) : ((x < b) ? x : b);
}

// ndf::sampler<NDF, 90, 1> (include/ndf/sampler.h), the data-driven importance sampler bbm::ndf_sampler
// wraps around the He family and Merl (bbm/ndf_sampler.h:22-164), over a per-launch 90-bin CDF:
// ndf::sampler::pdf (ndf/sampler.h:102-128) of the halfway vector m
// theta is the reference's (spherical::theta: a double asin rounded to float): the bin weight w is ~45 x more
// sensitive to it than the pdf is, and adjacent bins can differ severalfold, so a 2-ulp float asin moved pdfs by
// ~2e-5.  sin(theta) enters only the Jacobian, as a factor: |m.xy| (~2 ulp from the sine of the float theta, m
// unit) replaces the correctly rounded sincos.
__device__ __forceinline__ float ndf_sampler_pdf(const float* __restrict__ cdf, v3 m)
{
  const float theta = theta_of(m);
  const float ti = float(double(sqrtf(theta / kPiHalfF) * float(kHeBins)) - 0.5);
  const float w = ti - floorf(ti);
  const float fl = floorf(ti), ce = ceilf(ti);
  // clamp(cast<Size_t>(floor(ti)), 0, 89): a negative float cast to size_t wraps on x86-64 (-> 89)
  const int lidx = (fl < 0) ? kHeBins - 1 : min(int(fl), kHeBins - 1);
  const int uidx = (ce < 0) ? kHeBins - 1 : min(int(ce), kHeBins - 1);
  auto cpdf = [&](int i) { return cdf[i] - ((i >= 1) ? cdf[i - 1] : 0.0f); };
  const float p = cpdf(lidx) * (1 - w) + cpdf(uidx) * w;
  // |sin(theta)| of the float theta as the reference takes it (bbm::sin -> glibc's sinf, restated: math.hpp) -- the
  // direction's own sqrt(x^2 + y^2) (rounds 1-5) is the same quantity rounded differently, an ulp off on ~1/4 of the
  // lanes, which moved the pdf by an ulp there
  float sn, cs;
  sincosf_glibc(theta, &sn, &cs);
  const float st = __builtin_fabsf(sn);
  const float jac = (((sqrtf(theta) * kPiSqQuarterF) / float(kHeBins)) * st) * kPi2F;
  return ((m.z > 0) && (jac > kEpsF)) ? div_nr(p, jac) : 0.0f;
}

// ndf::sampler::sample (ndf/sampler.h:63-92): the sampled halfway vector for (xi0, xi1)
__device__ __forceinline__ v3 ndf_sampler_halfway(const float* __restrict__ cdf, float xi0, float xi1)
{
  // cdf::sample (util/cdf.h:73-83): lower_bound of xi0, residual within the bin
  int idx = 0;
  while (idx < kHeBins && cdf[idx] < xi0) ++idx;
  const bool valid = idx < kHeBins;
  const float ev = valid ? cdf[idx] : 0.0f;
  const float prev = (valid && idx >= 1) ? cdf[idx - 1] : 0.0f;
  const float cp = ev - prev;
  const float residual = valid ? (xi0 - prev) / cp : 0.0f;
  const double xr = fabs(double(residual) - 0.5);
  const double off = 1 - safe_sqrt(1 - 2 * xr);
  const double sgn = copysign(1.0, double(residual) - 0.5);
  const double q = (double(idx) + 0.5 + sgn * off) / double(kHeBins);
  float theta = float(q * q * double(kPiHalfF));
  const float phi = kPi2F * xi1;
  theta = (theta > kPiHalfF) ? kPiF - theta : theta;
  return sph_to_vec(phi, theta);
}

// ln x for the early-exit bound: exact exponent (frexp, subnormals included) + v_log_f32 of the mantissa, ~1e-7
// absolute; -inf for 0 (a zero gm or g makes every later term 0)
__device__ __forceinline__ float ln_bound(float x)
{
  const float l = (float(__builtin_amdgcn_frexp_expf(x)) + __builtin_amdgcn_logf(__builtin_amdgcn_frexp_mantf(x))) * kLn2F;
  return (x > 0.0f) ? l : -__builtin_inff();
}

// fresnel::complex<CONF, Spectrum> per channel (include/bbm/fresnel_complex.h:38-63); params = n RGB, k RGB
struct FresnelComplexRGB
{
  static constexpr int kParams = 6;
  float n[3], k[3];
  __device__ explicit FresnelComplexRGB(const float* q)
  {
    for (int c = 0; c < 3; ++c) { n[c] = q[c]; k[c] = q[3 + c]; }
  }
  // With VALUE = Spectrum (he.h:116, 490-496) every operation is the native backbone's array arithmetic in float:
  // a double scalar on the left of an array (0.5 * (a2b2 + temp), 0.5 * (Rs + Rp)) converts to float first
  // (array.h:95, friend operator*(const T&, array)), and Rs / Rp are Spectrum -- so the reference's float at every
  // step, IEEE float quotients (div_nr: the correctly rounded quotient, with the IEEE fallback off the normal range)
  // and correctly rounded square roots (safe_sqrtf).  (Rounds 1-4 evaluated the numerators and denominators in
  // double, as the scalar-VALUE instantiation does (EPD's FresnelComplex, epd.hpp): the He family's backscatter values
  // were then 1-10 ulp off on 80-100 % of the 90 sampler-CDF directions, profiles/r05_he_cdf_before.json.)
  __device__ __forceinline__ void eval3(float cs, float* F) const
  {
    const float c2 = cs * cs;
    const float s2 = 1 - c2;
#pragma unroll
    for (int c = 0; c < 3; ++c)
    {
      const float n2 = n[c] * n[c], k2 = k[c] * k[c];
      const float temp = (n2 - k2) - s2;
      const float a2b2 = safe_sqrtf(temp * temp + (n2 * 4.0f) * k2);
      const float a = safe_sqrtf((a2b2 + temp) * 0.5f);
      const float a2c = (a * 2.0f) * cs;
      const float Rs = div_nr((a2b2 - a2c) + c2, (a2b2 + a2c) + c2);
      const float ca = c2 * a2b2;
      const float Rp = div_nr(Rs * (ca - (a2c - s2) * s2), ca + (a2c + s2) * s2);
      F[c] = (Rs + Rp) * 0.5f;
    }
  }
};

// fresnel::cook with a scalar ior, broadcast to RGB (NganHe)
struct FresnelCookRGB
{
  static constexpr int kParams = 1;
  FresnelCook f;
  __device__ explicit FresnelCookRGB(const float* q) : f(q) {}
  __device__ __forceinline__ void eval3(float cs, float* F) const { F[0] = F[1] = F[2] = f.eval(cs); }
};

// EQ25 errata, EQ78 Westin, Taylor terms, adaptive stop, rough approximation threshold (< 0: none), scaled
template<class FRES, bool ERRATA, bool WESTIN, int TAYLOR, bool ADAPTIVE, int APPROX, bool SCALED>
struct He
{
  static constexpr int kOff = SCALED ? 3 : 0;
  static constexpr int kParams = kOff + 2 + FRES::kParams;
  static constexpr uint32_t kComponent = kFlagSpecular;
  float albedo[3];
  float sigma0, tau;
  FRES fres;
  const float* cdf;      // kHeBins floats (the launch's component); only valid where host_params ran
  uint32_t launch_component;   // the component the CDF was built for; lanes passing another one are masked

  __device__ explicit He(const float* p) : sigma0(p[kOff]), tau(p[kOff + 1]), fres(p + kOff + 2)
  {
    for (int c = 0; c < 3; ++c) albedo[c] = SCALED ? p[c] : 1.0f;
    cdf = param_ptr(p, kParams);
    __builtin_memcpy(&launch_component, p + kParams + 2, 4);
  }

  // The kernels mask a lane by passing component 0.  A sampler built for a component without the specular
  // lobe is 0/0 (NaN) in the reference, and so is this one, but a masked lane is select(mask, ., 0) there.
  __device__ __forceinline__ bool masked(uint32_t component) const { return component != launch_component; }

  // The four erfcf evaluations of a pair's prelude -- S1 of in and out, sigma's K of in and out -- are 40 % of the
  // prelude (0.16 of 0.36 ms per 10 M He pairs, profiles/r06_ab_he_erfc.txt): each one a three-range fdlibm
  // erfcf whose ranges diverge within every wave.  Their arguments (erfc_args) are therefore separable from the
  // rest: the compaction kernel (kernels.hpp) evaluates a block's arguments as one work list sorted by range, S1's
  // and K's argument of a direction evaluated once where they are the same float, and hands the values back
  // (Erfc); every other path passes none and evaluates them in place.  Same function, same operands: same floats.
  static constexpr bool kErfcList = true;
  struct Erfc { float x[2], v[4]; };          // x: S1's arguments (in, out); v: erfcf of the four arguments
  __device__ __forceinline__ float s1_arg(v3 v) const
  {
    const float cot = div_nr(1.0f, tan_theta(v));
    // the double quotient stored straight into a float: f_div_d rounds like the reference
    return f_div_d(double(tau * cot), 2.0 * double(sigma0));
  }
  __device__ __forceinline__ float k_arg(float t) const { return div_nr(tau, 2 * sigma0 * t); }
  __device__ __forceinline__ void erfc_args(v3 in, v3 out, float* x) const
  {
    x[0] = s1_arg(in); x[1] = s1_arg(out);
    x[2] = k_arg(tan_theta(in)); x[3] = k_arg(tan_theta(out));
  }
  // S1 (he.h:266-291), Eqs. 24-25, of a direction whose s1_arg is scot and erfcf(scot) = ec
  __device__ __forceinline__ float S1(float scot, float ec) const
  {
    const bool smooth = sigma0 < kEpsF;
    const float erfc_ = 0.5f * ec;                  // float(0.5 * double(e)): exact; glibc's erfcf, bit for bit
    // the double quotients below are stored straight into floats: f_div_d rounds like the reference
    float lambda = f_div_d(0.5 * double(kInvSqrtPiF), double(scot));
    // Lambda *= exp(-pow(scot, 2.0)): a float times the double exponential, rounded once (compound assignment of a
    // double to a float); exp_dd is within ~2^-44 of glibc's exp, so the product rounds like the reference's
    if (ERRATA) lambda = float(double(lambda) * exp_dd(fmax(-(double(scot) * double(scot)), -745.0)));
    lambda -= erfc_;
    const float S = f_div_d(1.0 - double(erfc_), double(lambda) + 1.0);
    return smooth ? 1.0f : S;
  }
  __device__ __forceinline__ float S1(v3 v) const { const float x = s1_arg(v); return S1(x, erfcf_glibc(x)); }

  // G (he.h:306-352), Eq. 76
  __device__ __forceinline__ float G(v3 in, v3 out) const
  {
    const v3 v = mk3(in.x + out.x, in.y + out.y, in.z + out.z);
    const float vq = div_nr(dot3(v, v), v.z);
    const float v_scale = float(double(vq) * double(vq));
    const float kixn2 = 1 - in.z * in.z;
    const float krxn2 = 1 - out.z * out.z;
    const float kikr = dot3(neg3(in), out);
    const float sikr = out.y * in.x - out.x * in.y;
    const float srki = in.y * out.x - in.x * out.y;
    const float pikr = out.z + kikr * in.z;
    const float prki = in.z + kikr * out.z;
    const double dd = 1.0 - double(kikr * kikr);
    const float denom = float(dd * dd);
    const float nom = f_div_d((double(sikr) * double(sikr) + double(pikr) * double(pikr)) *
                                  (double(srki) * double(srki) + double(prki) * double(prki)), double(krxn2 * kixn2));
    const float g = div_nr(v_scale * nom, denom);
    return (denom > kEpsF) ? g : 1.0f;
  }

  // sigma (he.h:365-400), Eq. 80 by 4 Newton-Raphson steps; K's erfcf from the work list (ef) or in place
  __device__ __forceinline__ float sigma(v3 in, v3 out, const Erfc* ef) const
  {
    const float ti = tan_theta(in), to = tan_theta(out);
    auto K = [&](float t, int k) { return t * (ef ? ef->v[k] : erfcf_glibc(k_arg(t))); };
    const float Ki = (ti > kEpsF) ? K(ti, 2) : 0.0f;
    const float Ko = (to > kEpsF) ? K(to, 3) : 0.0f;
    const float f0 = div_nr(1.0f, sqrtf(kPi8F)) * (Ki + Ko);
    // safe_sqrt(2.0 * log(f0)): 2 x a float is exact in float and double alike, and a correctly rounded double
    // sqrt rounded to float is the correctly rounded float sqrt (53 >= 2 x 24 + 2): identical, without the f64 sqrt
    float x = (f0 <= 1.0f) ? f0 : safe_sqrtf(2.0f * logf_glibc(f0));
#pragma unroll
    for (int s = 0; s < 4; ++s)
    {
      // Value expn = exp(0.5 * x * x): the double exponential rounded to float -- exp2_cr (correctly rounded but
      // within ~2^-18 ulp of a midpoint), as glibc's 0.51-ulp exp rounded to float; exp_d2f's 1.5 ulp moved the
      // Newton root by an ulp on ~10 % of the lanes
      const float expn = exp2_cr(0.5 * double(x) * double(x) * 1.4426950408889634074);
      const float ev = x * expn - f0;
      const float grad = (1 + x * x) * expn;
      x -= (grad > kEpsF) ? div_nr(ev, grad) : 0.0f;
    }
    const float r = div_nr(sigma0, safe_sqrtf(1 + x * x));
    return (sigma0 > kEpsF) ? r : 0.0f;
  }

  // D (he.h:411-467), Eqs. 78-79: Taylor series in g with Beckmann's rough approximation blended in.  Split in two
  // for the compaction kernel's two-phase evaluation (kernels.hpp, k_eval_pdf_compact): D_prep everything before
  // the series (sigma's Newton steps, g, the exponent bases, the rough approximation), D_series the series itself
  // and the blend; D = both, in order, so every path evaluates the same operations on the same operands.
  struct DPrep { float gg[3], eb[3], rough[3]; };

  __device__ __forceinline__ void D_prep(v3 in, v3 out, const Erfc* ef, DPrep& d) const
  {
    const float vxy2 = sqnorm2(in.x + out.x, in.y + out.y);
    const float sg = sigma(in, out, ef);
    const float tau2 = float(double(tau) * double(tau));
    const float base = (vxy2 * tau2) / 4.0f;
    double g[3];
#pragma unroll
    for (int c = 0; c < 3; ++c)
    {
      d.gg[c] = div_nr((kPi2F * sg) * (in.z + out.z), kWavelength[c]);
      g[c] = double(d.gg[c]) * double(d.gg[c]);
      const double l2 = double(kWavelength[c]) * double(kWavelength[c]);
      d.eb[c] = WESTIN ? float(double(base) * (double(kPiSqFourF) / l2)) : base;
    }
    const double gmin = fmin(fmin(g[0], g[1]), g[2]);
    d.rough[0] = d.rough[1] = d.rough[2] = 0.0f;
    if (APPROX >= 0 && gmin > double(APPROX))
    {
#pragma unroll
      for (int c = 0; c < 3; ++c)
      {
        const double rg = ddiv_nr(1.0, g[c]);    // g > APPROX here
        d.rough[c] = float(exp_dd(-double(d.eb[c]) * rg) * rg);   // exp(-eb / g) / g in double, one rounding
      }
    }
  }

  // series length key of the two-phase kernel: lanes with a similar peak position g run similar numbers of terms
  // (0: no series -- the rough approximation alone)
  // Westin: the terms carry e^(-eb/m), which moves the series' mass to m* ~ the maximum of the log-term
  // -eb/m + m ln g - ln m!, i.e. eb / m^2 = ln(m / g) (Stirling); the key is m* of the blue channel (the largest g
  // and eb) by three Newton steps in u = ln m from m = sqrt(eb).  Modelled on 1 M hemisphere pairs (tools/he_geb.py,
  // the series lengths read back from the GPU): wave-max terms 31.1 with the g key, 27.9 with this one (the true
  // lengths as key: 23.9).  Only the order of the jobs depends on the key.
  __device__ __forceinline__ int D_key(const DPrep& d) const
  {
    const double g1 = double(d.gg[1]) * double(d.gg[1]);
    const double gmin = fmin(fmin(double(d.gg[0]) * double(d.gg[0]), g1), double(d.gg[2]) * double(d.gg[2]));
    if ((APPROX >= 0) && (gmin - 1.0 > double(APPROX))) return 0;
#ifndef BBM_HIP_HE_WESTIN_GKEY
    if (WESTIN)
    {
      const float gb = d.gg[2] * d.gg[2], e = d.eb[2];
      const float lg = __logf(fmaxf(gb, 1e-30f));
      float u = fmaxf(0.5f * __logf(fmaxf(e, 1.0f)), __logf(fmaxf(gb, 1.0f)));
#pragma unroll
      for (int it = 0; it < 3; ++it)
      {
        const float ex = e * __expf(-2.0f * u);
        u -= (ex - u + lg) / (-2.0f * ex - 1.0f);
      }
      return 1 + min(30, int(__expf(fminf(fmaxf(u, 0.0f), 4.1588830f))));   // m* in [1, 64]
    }
#endif
    return 1 + min(30, int(float(g1) * 1.5f));
  }

  __device__ __forceinline__ void D_series(const DPrep& d, float* Dout) const
  {
    double g[3], norm[3];
    float eb[3];
    const float tau2 = float(double(tau) * double(tau));
#pragma unroll
    for (int c = 0; c < 3; ++c)
    {
      g[c] = double(d.gg[c]) * double(d.gg[c]);
      const double l2 = double(kWavelength[c]) * double(kWavelength[c]);
      norm[c] = double(kPiSqQuarterF * tau2) * (1.0 / l2);   // constant reciprocal: within an ulp of the quotient
      eb[c] = d.eb[c];
    }
    const double gmin = fmin(fmin(g[0], g[1]), g[2]);
    const float weight = (APPROX >= 0 && gmin > double(APPROX)) ? float(fmin(fmax(gmin - double(APPROX), 0.0), 1.0)) : 0.0f;
    float sum[3] = {0.0f, 0.0f, 0.0f}, gm[3] = {1.0f, 1.0f, 1.0f}, term[3] = {0.0f, 0.0f, 0.0f}, last[3];
    bool converged = (APPROX >= 0) && (gmin - 1.0 > double(APPROX));
    // term = float(exp(-g - eb/m) gm / m) in double (he.h:454), gm = float(gm * (g / m)) rounded per step
    // (Spectrum *= array<double>), eb/m a float quotient -- formed here exactly that way, with the one double
    // exponential split into exp(-g) (once per channel) x exp(-eb/m) (per term; exp_dd, a short f64 polynomial
    // instead of the library's 42-instruction exp): the product agrees with the reference's exponential to
    // ~2^-44, so every float term -- subnormal ones included -- is the reference's own rounding of it except
    // within ~2^-20 ulp of a rounding midpoint.  (A 64-entry 2^(j/64) table with a degree-5 polynomial -- half the
    // FMAs, one 8 B gather of an L1-resident table per exponential -- measured slower: HeWestin 1.15 -> 1.36 ms per
    // 10 M pairs, three dependent gathers per term in a VALU-bound loop.)  That matters beyond accuracy: the adaptive stop (he.h:460)
    // compares consecutive terms, and near the series' peak they are nearly equal, so terms that differed by
    // an ulp would truncate the series one term early or late where D is tiny.
    double eg[3], cap[3];
    float lng[3];
    // non-Westin: eb (<= v_xy^2 tau^2 / 4) is the same small number on every channel, e^(-eb/64) bounds e^(-q_m')
    // closely, and the cheap bound cap gm_m / m below is tested every 4th term instead
    const double eb64 = (ADAPTIVE && !WESTIN && !converged) ? exp_dd(-double(eb[0]) * (1.0 / 64.0)) * (1.0 + 0x1p-10) : 0.0;
#pragma unroll
    for (int c = 0; c < 3; ++c)
    {
      eg[c] = converged ? 0.0 : exp_dd(-g[c]);
      lng[c] = (ADAPTIVE && WESTIN) ? ln_bound(float(g[c])) : 0.0f;
      cap[c] = eg[c] * eb64;
    }
    // Exact early exit (adaptive series only).  Past the peak (m + 1 >= g, r = g / (m + 1) <= 1) a later term
    // m' in [m + 1, 64] is at most
    //   e^(-g) (gm_m / m) e^(h(m')),   h(m') = -eb / m' + (m' - m) ln r
    // (gm_m' <= gm_m r^(m' - m), 1/m' < 1/m, q_m' = float(eb / m') >= eb / m' up to float rounding).  h is concave
    // in m', so its maximum over the range is at m* = sqrt(eb / -ln r) clamped to [m + 1, 64] -- a closed form.
    // Once that bound (in the log domain, +0.01 for every rounding involved) is below half an ulp of a
    // channel's float sum (2^-150 while the sum is 0) on all three channels, no later term can change any sum:
    // the loop's only output is final, so it stops there with exactly the reference's result, wherever the
    // reference's own stop (he.h:459) lies.  Without it, lanes whose terms underflow to 0 for small m (large eb)
    // never meet the stop rule (0 < 0 is false) and run all 64 terms, and one such lane keeps its wave busy.
    // Modelled on uniform hemisphere pairs (HeWestin defaults): wave-max 64 terms without the exit, 36 with the
    // simpler bound e^(-g) e^(-eb/64) gm_m / m, 31.6 with this one tested every 8th term (31.1 every 4th, 30.8 with
    // the exact tail maximum); measured HeWestin 1.36 -> 1.28 ms per 10 M pairs.  For the non-Westin series eb is
    // small and the same on every channel, e^(-eb/64) is close, and that cheaper bound (every 4th term) stays:
    // the concave one measured 0.89 -> 0.95 (every 8th) / 1.10 ms (every 4th) there.
#ifdef BBM_HIP_HE_PROBE_NO_SERIES
    converged = true;       // timing probe only (tools/build_variant.sh): the prelude without the series
#endif
#ifdef BBM_HIP_HE_COUNT_TERMS
    int nterms = 0;         // diagnostics build only (tools/he_terms.py): D = (terms run, length key, 0)
#endif
    for (int m = 1; m <= TAYLOR && !converged; ++m)
    {
#ifdef BBM_HIP_HE_COUNT_TERMS
      nterms = m;
#endif
      const double rm = inv_small(m);
      const float mf = float(m), rmf = float(rm);
      double ex[3];
      if (WESTIN)
      {
#pragma unroll
        for (int c = 0; c < 3; ++c) ex[c] = exp_dd(-double(div_small(eb[c], mf, rmf)));
      }
      else ex[0] = ex[1] = ex[2] = exp_dd(-double(div_small(eb[0], mf, rmf)));   // eb is the same for every channel
#pragma unroll
      for (int c = 0; c < 3; ++c)
      {
        last[c] = term[c];
        gm[c] = float(double(gm[c]) * (g[c] * rm));
        term[c] = float(eg[c] * ex[c] * double(gm[c]) * rm);
        sum[c] += term[c];
      }
      // converged |= hmin(term) < eps && hmin(term) < hmin(last) (he.h:460)
      if (ADAPTIVE)
      {
        converged = (fminf(fminf(term[0], term[1]), term[2]) < kEpsF) &&
                    (fminf(fminf(term[0], term[1]), term[2]) < fminf(fminf(last[0], last[1]), last[2]));
        if (!WESTIN && (m & 3) == 0)
        {
          bool settled = true;
#pragma unroll
          for (int c = 0; c < 3; ++c)
          {
            const int e = (sum[c] > 0.0f) ? max(__builtin_amdgcn_frexp_expf(sum[c]) - 25, -150) : -150;
            settled = settled && (double(m) + 1.0 >= g[c]) && (cap[c] * double(gm[c]) * rm < __builtin_ldexp(1.0, e));
          }
          converged = converged || settled;
        }
        // Westin: the concave bound, tested every 8th term (a term ~100 VALU, the test ~70)
        if (WESTIN && (m & 7) == 0)
        {
          bool settled = true;
          const float ln_m = ln_bound(mf), ln_m1 = ln_bound(mf + 1.0f);
#pragma unroll
          for (int c = 0; c < 3; ++c)
          {
            const float lnr = lng[c] - ln_m1;                                // ln r <= 0 past the peak
            float ms = (lnr < 0.0f) ? sqrtf(eb[c] / -lnr) : 64.0f;
            ms = fminf(fmaxf(ms, mf + 1.0f), 64.0f);
            const float h = -eb[c] / ms + (ms - mf) * lnr;
            const float bound = ((-float(g[c]) + ln_bound(gm[c])) - ln_m) + h + 0.01f;
            // ln of half an ulp of sum[c] (2^-150 for 0 and subnormal sums)
            const int e = (sum[c] > 0.0f) ? max(__builtin_amdgcn_frexp_expf(sum[c]) - 25, -150) : -150;
            settled = settled && (double(m) + 1.0 >= g[c]) && (bound < float(e) * kLn2F);
          }
          converged = converged || settled;
        }
      }
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) Dout[c] = float(norm[c] * double(std_lerpf(sum[c], d.rough[c], weight)));
#ifdef BBM_HIP_HE_COUNT_TERMS
#if BBM_HIP_HE_COUNT_TERMS == 2
    Dout[0] = float(nterms); Dout[1] = float(g[1]); Dout[2] = eb[1];     // (terms, g, eb) of the green channel
#else
    Dout[0] = float(nterms); Dout[1] = float(D_key(d)); Dout[2] = 0.0f;
#endif
#endif
  }

  __device__ __forceinline__ void D(v3 in, v3 out, float* Dout) const
  {
    DPrep d;
    D_prep(in, out, nullptr, d);
    D_series(d, Dout);
  }


  // he_base::eval (he.h:142-166), x albedo when scaled (scaledmodel.h:50-53); the sampler's backscatter
  // evaluations (k_he_cdf) see the unscaled he_base, which scaledmodel wraps from outside.  Two stages, as D:
  // eval_prep the prefactor ((1 / (pi z_i z_o)) F) S G per channel and D_prep; eval_finish the series and the
  // product.
  struct EvalPrep { float pre[3]; bool active; DPrep d; };

  __device__ __forceinline__ void eval_prep(v3 in, v3 out, uint32_t component, const Erfc* ef, EvalPrep& e) const
  {
    e.active = (component & kFlagSpecular) && (in.z > 0) && (out.z > 0);
    float F[3];
    const float S = ef ? S1(ef->x[0], ef->v[0]) * S1(ef->x[1], ef->v[1]) : S1(in) * S1(out);
    const float Gv = G(in, out);
    D_prep(in, out, ef, e.d);
    // float(safe_sqrt(double(1 + dot) / 2.0)): halving the float sum is exact in float (1 + dot >= 2^-24 or 0),
    // and the double-then-float sqrt equals the float sqrt (53 >= 2 x 24 + 2)
    const float cth = safe_sqrtf((1 + dot3(in, out)) * 0.5f);
    fres.eval3(cth, F);
    const float nrm = div_nr(1.0f, (kPiF * in.z) * out.z);
#pragma unroll
    for (int c = 0; c < 3; ++c) e.pre[c] = ((nrm * F[c]) * S) * Gv;
#if defined(BBM_HIP_HE_DIAG) && BBM_HIP_HE_DIAG == 2
    e.pre[0] = sigma(in, out, ef); e.pre[1] = S; e.pre[2] = Gv;
#elif defined(BBM_HIP_HE_DIAG) && BBM_HIP_HE_DIAG == 3
    e.pre[0] = F[0]; e.pre[1] = F[1]; e.pre[2] = nrm;
#endif
  }

  template<bool SCALE = true>
  __device__ __forceinline__ void eval_finish(const EvalPrep& e, float* rgb) const
  {
    float Dv[3];
    D_series(e.d, Dv);
#pragma unroll
    for (int c = 0; c < 3; ++c)
    {
      float v = e.pre[c] * Dv[c];
      if (SCALED && SCALE) v *= albedo[c];
      rgb[c] = e.active ? v : 0.0f;
#ifdef BBM_HIP_HE_COUNT_TERMS
      rgb[c] = Dv[c];
#endif
#if defined(BBM_HIP_HE_DIAG) && BBM_HIP_HE_DIAG == 1
      rgb[c] = Dv[c];            // diagnostics build only (tools/dbg_he_parts.py): D per channel
#elif defined(BBM_HIP_HE_DIAG) && BBM_HIP_HE_DIAG >= 2
      rgb[c] = e.pre[c];         // diagnostics build only: (sigma, S, G) / (F red, F green, 1 / (pi z z)), eval_prep
#endif
    }
  }

  template<bool SCALE = true>
  __device__ __forceinline__ void eval_rgb(v3 in, v3 out, uint32_t component, float* rgb) const
  {
    EvalPrep e;
    eval_prep(in, out, component, nullptr, e);
    eval_finish<SCALE>(e, rgb);
  }

  // ndf::sampler::pdf (ndf/sampler.h:102-128) of the halfway vector m
  __device__ __forceinline__ float sampler_pdf(v3 m) const { return ndf_sampler_pdf(cdf, m); }

  // ndf_sampler::pdf (bbm/ndf_sampler.h:128-156): sampler pdf of h / |4 out.h|, z(in), z(out) > 0
  __device__ __forceinline__ float pdf_of(v3 in, v3 out, uint32_t component) const
  {
    const bool active = (out.z > 0) && (in.z > 0) && !masked(component);
    const v3 h = halfway(in, out);
    const float p = float(double(sampler_pdf(h)) / fabs(4.0 * double(dot3(out, h))));
    return active ? p : 0.0f;
  }

  template<int MODE>
  __device__ __forceinline__ void eval_pdf(v3 in, v3 out, uint32_t component, float* rgb, float& pdf) const
  {
    if (MODE & kModeEval) eval_rgb(in, out, component, rgb);
    else rgb[0] = rgb[1] = rgb[2] = 0.0f;
    pdf = (MODE & kModePdf) ? pdf_of(in, out, component) : 0.0f;
  }

  // the compaction kernel's two-phase evaluation (kernels.hpp): stage 1 everything but the series, with its
  // length key; stage 2 the series and the product -- the same operations as eval_pdf, split at the series
  // measured per model (tools/gpu_r03_e.sh, config 3, ms per 10 M pairs, one-phase -> two-phase): He 0.737 ->
  // 0.671, HeWestin 1.153 -> 1.152, NganHe 1.089 -> 1.088, HeHolzschuch (10 fixed terms: nothing to sort)
  // 0.390 -> 0.406; on for the adaptive series only
#ifndef BBM_HIP_HE_ONEPHASE
  static constexpr bool kTwoPhase = ADAPTIVE;
#else
  static constexpr bool kTwoPhase = false;
#endif
  struct Stage { EvalPrep e; float pdf; };
  static constexpr int kStageWords = 14;
  __device__ __forceinline__ static void stage_store(const Stage& st, float* base, int stride)
  {
    for (int c = 0; c < 3; ++c)
    {
      base[c * stride] = st.e.pre[c];
      base[(3 + c) * stride] = st.e.d.gg[c];
      base[(6 + c) * stride] = st.e.d.eb[c];
      base[(9 + c) * stride] = st.e.d.rough[c];
    }
    base[12 * stride] = st.e.active ? 1.0f : 0.0f;
    base[13 * stride] = st.pdf;
  }
  __device__ __forceinline__ static void stage_load(Stage& st, const float* base, int stride)
  {
    for (int c = 0; c < 3; ++c)
    {
      st.e.pre[c] = base[c * stride];
      st.e.d.gg[c] = base[(3 + c) * stride];
      st.e.d.eb[c] = base[(6 + c) * stride];
      st.e.d.rough[c] = base[(9 + c) * stride];
    }
    st.e.active = base[12 * stride] != 0.0f;
    st.pdf = base[13 * stride];
  }
  template<int MODE>
  __device__ __forceinline__ int stage1(v3 in, v3 out, uint32_t component, const Erfc* ef, Stage& st) const
  {
    eval_prep(in, out, component, ef, st.e);
    st.pdf = (MODE & kModePdf) ? pdf_of(in, out, component) : 0.0f;
    return D_key(st.e.d);
  }
  __device__ __forceinline__ void stage2(const Stage& st, float* rgb) const { eval_finish(st.e, rgb); }

  // he_base::reflectance (he.h:230-244): Fresnel at z(out) / Pi * 4.0, x albedo when scaled
  __device__ __forceinline__ void reflectance(v3 out, uint32_t component, float* rgb) const
  {
    const bool m = (component & kFlagSpecular) && (out.z > 0);
    float F[3];
    fres.eval3(out.z, F);
#pragma unroll
    for (int c = 0; c < 3; ++c)
    {
      float v = float(double(F[c] / kPiF) * 4.0);
      if (SCALED) v *= albedo[c];
      rgb[c] = m ? v : 0.0f;
    }
  }

  // ndf_sampler::sample (bbm/ndf_sampler.h:78-111) with ndf::sampler::sample (ndf/sampler.h:63-92)
  __device__ __forceinline__ void sample(v3 out, float xi0, float xi1, uint32_t component, v3& dir, float& pdf,
                                         uint32_t& flag) const
  {
    dir = mk3(0.0f, 0.0f, 0.0f); pdf = 0.0f; flag = kFlagNone;
    if (!((xi0 >= 0) && (xi1 >= 0) && (xi0 <= 1) && (xi1 <= 1) && (out.z > 0)) || masked(component)) return;
    const v3 h = ndf_sampler_halfway(cdf, xi0, xi1);
    // reflect(out, h) = h dot(h, out) 2.0 - out (core/vec_transform.h:43-44)
    const float d = dot3(h, out);
    dir = mk3(2.0f * (h.x * d) - out.x, 2.0f * (h.y * d) - out.y, 2.0f * (h.z * d) - out.z);
    float rgb[3];
    eval_pdf<kModePdf>(dir, out, component, rgb, pdf);
    flag = component;
  }
};

// ndf::sampler::initialize (ndf/sampler.h:143-181) for one component: 90 backscatter evaluations
// hsum(eval(h, h)) at theta = (i / 90)^2 Pi/2, weighted by sin(theta1) sqrt(theta1), theta1 = ((i+1)/90)^2 Pi/2,
// then cdf(samples) (util/cdf.h:39-47): serial float prefix sum, normalised by the last entry.
template<class Model>
__global__ __launch_bounds__(128) void k_he_cdf(ParamBlock p, uint32_t component, float* __restrict__ cdf)
{
  math_tables_init();
  __shared__ float s[kHeBins];
  const Model m(p.v);
  const int i = threadIdx.x;
  if (i < kHeBins)
  {
    const float q = float(i) / float(kHeBins);
    const float theta = float(double(q) * double(q) * double(kPiHalfF));
    const v3 h = sph_to_vec(0.0f, theta);
    float rgb[3];
    m.template eval_rgb<false>(h, h, component, rgb);
    float v = ((0.0f + rgb[0]) + rgb[1]) + rgb[2];
    const float q1 = float(i + 1) / float(kHeBins);
    const float theta1 = float(double(q1) * double(q1) * double(kPiHalfF));
    float st, ct;
    cossin_cr(theta1, ct, st);
    v *= st * sqrtf(theta1);
    s[i] = v;
  }
  __syncthreads();
  if (i == 0)
  {
    float acc = 0.0f;
    for (int k = 0; k < kHeBins; ++k) { acc += s[k]; s[k] = acc; }
    for (int k = 0; k < kHeBins; ++k) cdf[k] = s[k] / acc;
  }
}

// Builds the launch's CDF into stream-ordered scratch and stores its address (two slots) and the component
// it was built for after the model's kParams parameters (M::kParams + 0..2).
template<class M>
int ndf_sampler_cdf_run(ParamBlock& p, uint32_t component, hipStream_t s, void** scratch, const char* who)
{
  float* cdf = static_cast<float*>(scratch_acquire(kHeBins * sizeof(float), s));
  if (!cdf) return fail(BBM_HIP_ERR_HIP, std::string(who) + " sampler CDF: scratch allocation failed: " + scratch_failure());
  hipError_t e;
  hipLaunchKernelGGL((k_he_cdf<M>), dim3(1), dim3(128), 0, s, p, component, cdf);
  if ((e = hipGetLastError()) != hipSuccess)
    return fail(BBM_HIP_ERR_HIP, std::string(who) + " sampler CDF: launch: " + hipGetErrorString(e));
  set_param_ptr(p.v, M::kParams, cdf);
  __builtin_memcpy(p.v + M::kParams + 2, &component, 4);
  *scratch = cdf;
  return BBM_HIP_OK;
}

template<class FRES, bool ERRATA, bool WESTIN, int TAYLOR, bool ADAPTIVE, int APPROX, bool SCALED>
struct host_params<He<FRES, ERRATA, WESTIN, TAYLOR, ADAPTIVE, APPROX, SCALED>>
{
  using M = He<FRES, ERRATA, WESTIN, TAYLOR, ADAPTIVE, APPROX, SCALED>;
  static int run(ParamBlock& p, uint32_t component, hipStream_t s, void** scratch)
  {
    return ndf_sampler_cdf_run<M>(p, component, s, scratch, "He");
  }
  static void done(void* scratch, hipStream_t s) { if (scratch) scratch_release(scratch, s); }
};

// The He evaluation is VALU-bound (the Taylor series, ~10^3 instructions per pair) and zero outside the upper
// hemisphere and on masked lanes (eval_rgb / eval_pdf above): evaluate live pairs only, packed densely
template<class FRES, bool ERRATA, bool WESTIN, int TAYLOR, bool ADAPTIVE, int APPROX, bool SCALED>
struct compact_eval<He<FRES, ERRATA, WESTIN, TAYLOR, ADAPTIVE, APPROX, SCALED>> { static constexpr bool value = true; };

// he.h:489-496, ngan.h:166-167
using HeM = He<FresnelComplexRGB, false, false, 64, true, 18, false>;
using HeWestinM = He<FresnelComplexRGB, true, true, 64, true, 18, false>;
using HeHolzschuchM = He<FresnelComplexRGB, true, false, 10, false, -1, false>;
using NganHeM = He<FresnelCookRGB, true, true, 64, true, 18, true>;

}  // namespace bbmhip
