// bbm_amd/csrc/math.hpp -- device math layer of the HIP backbone.
//
// The BBM native backbone (backbone/native/include/backbone/{math,horizontal,array}.h) fixes the
// rounding of every intermediate: Value = float, but C++'s usual arithmetic conversions promote
// a handful of intermediates to double (`2.0 * x`, `x / literal<double>`, `bbm::max(x, 0.0)`,
// `bbm::pow(x, 2.0)`).  HIP device code obeys the same conversions, so the model code in this
// directory keeps the reference's literal types and lets the compiler do the same promotions;
// the few helpers here pin down the ones that are library behaviour rather than language rules.
// The whole TU is compiled with -ffp-contract=off: every float op rounds on its own, exactly as
// the reference's x86-64 build does, so results match the CPU backbone to ~1 ulp (transcendentals
// are the only non-correctly-rounded ops on either side).
//
// Third-party notices (THIRD_PARTY_NOTICES.md has the full texts).  The float libm restatements below follow glibc 2.35
// (GNU C Library, LGPL-2.1-or-later), whose expf / logf / powf / sinf / cosf come from Arm's optimized-routines
// (Copyright (c) 2017-2018 Arm Ltd; MIT OR Apache-2.0 WITH LLVM-exception upstream) and whose erff / erfcf / atan2f come
// from Sun's fdlibm:
//   Copyright (C) 1993 by Sun Microsystems, Inc. All rights reserved.
//   Developed at SunPro, a Sun Microsystems, Inc. business.
//   Permission to use, copy, modify, and distribute this software is freely granted, provided that this notice
//   is preserved.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bbmhip {

// bsdf_flag (include/bbm/bsdf_flag.h:21-27), unit_t (include/bbm/unit.h:20-24)
enum : uint32_t { kFlagNone = 0, kFlagDiffuse = 1, kFlagSpecular = 2, kFlagAll = 3 };

constexpr double kPiD = 3.141592653589793238462643383279502884;
constexpr double kInvPiD = 0.318309886183790671537767526745028724;
constexpr double kInvSqrtPiD = 0.564189583547756286948079451560772586;
// constants<float>::Pi()/InvPi() (include/core/constants.h:17-19) = T(scale * std::numbers::pi)
constexpr float kPiF = float(1.0f * kPiD);
constexpr float kInvPiF = float(1.0f * kInvPiD);
constexpr float kInvSqrtPiF = float(1.0f * kInvSqrtPiD);
constexpr float kPi2F = float(2.0f * kPiD);          // Constants::Pi(2)
constexpr float kPi4F = float(4.0f * kPiD);          // Constants::Pi(4)
constexpr float kPi8F = float(8.0f * kPiD);          // Constants::Pi(8)
constexpr float kInvPiHalfF = float(0.5f * kInvPiD); // Constants::InvPi(0.5)
constexpr float kEpsF = 1.1920928955078125e-07f;   // numeric_limits<float>::epsilon()

// splitmix64 finaliser: the counter-based generators (synthetic directions, checkBsdf draws) hash
// (key + golden-ratio * index), so element i of a stream is a pure function of its global index.
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z)
{
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

struct v3 { float x, y, z; };
struct v2 { float x, y; };

// a model policy with a parameter-independent per-pair prelude: geometry(in, out) / eval_geo(geo, ...) (Bagher,
// Lambertian, their aggregates), which the fitting-loss kernel shares across the probes it evaluates at a pair
template<class M> constexpr bool has_geo()
{
  if constexpr (requires { M::kHasGeo; }) return M::kHasGeo;
  else return false;
}

// Models with an exact-mode evaluation (bbm_hip_set_exact_subnormals: Microfacet over Beckmann's subnormal quotients,
// Bagher's NDF by glibc's powf / expf, aggregates of such children -- Model::kHasExact) get a second instantiation
// of the eval kernels, launched while the mode is on (kernels.hpp).
template<class Model> constexpr bool model_has_exact()
{
  if constexpr (requires { Model::kHasExact; }) return Model::kHasExact;
  else return false;
}
// The samplers' exact-mode twin: a model type whose sampler reproduces glibc's float erff / logf where the default
// uses the device library's (Beckmann's visible-normal sampler, microfacet.hpp), launched by the sample and
// checkBsdf kernels while the mode is on.  Same parameters and layout; identity for every other model.
template<class M> struct exact_sample { using type = M; };
template<class M> using exact_sample_t = typename exact_sample<M>::type;
template<class M> constexpr bool has_exact_sample() { return !__is_same(exact_sample_t<M>, M); }

// eval at a prepared pair (has_geo models): CACHE = true where the model can keep per-pair terms across the parameter
// vectors evaluated at the pair (the fitting loss's probes: Bagher's NDF term)
template<bool CACHE, class Model, class G>
__device__ __forceinline__ void geo_eval(const Model& m, G& g, uint32_t component, float* rgb)
{
  if constexpr (CACHE && requires { m.eval_geo_cached(g, component, rgb); }) m.eval_geo_cached(g, component, rgb);
  else m.eval_geo(g, component, rgb);
}

template<int MODE, bool EXACT, class Model>
__device__ __forceinline__ void model_eval_pdf(const Model& m, v3 in, v3 out, uint32_t comp, float* rgb, float& pdf)
{
  if constexpr (EXACT && model_has_exact<Model>()) m.template eval_pdf<MODE, true>(in, out, comp, rgb, pdf);
  else m.template eval_pdf<MODE>(in, out, comp, rgb, pdf);
}

__device__ __forceinline__ v3 mk3(float x, float y, float z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }
__device__ __forceinline__ v3 neg3(v3 a) { return mk3(-a.x, -a.y, -a.z); }

// ---------------------------------------------------------------- division (VALU budget)
//
// IEEE division is the dominant VALU cost on this path (hipcc's correctly-rounded f32 divide is
// ~10 instructions with denormal-mode switches; f64 divide ~11 f64 instructions).  Both are
// replaced by the hardware reciprocal + Newton/Markstein correction:
//   q0 = n * rcp(d);  e = fma(-d, q0, n) (exact remainder);  q = fma(e, rcp(d), q0)
// which returns the correctly rounded quotient except when n/d lies within ~2^-22 ulp of a
// rounding midpoint (f32; ~2^-100 for the f64 form after two reciprocal refinements), i.e. a
// 1-ulp difference in roughly one division in four million.  IEEE special cases (d = 0, d = inf,
// n = inf, NaN) and subnormal quotients fall back to the uncorrected quotient, which is the IEEE result there.
// Denormal divisors (|d| < 2^-126) are outside the domain of this path (directions are unit
// vectors, parameters are >= their documented lower bounds).
__device__ __forceinline__ float div_nr(float n, float d)
{
  const float r = __builtin_amdgcn_rcpf(d);
  const float q = n * r;
  const float e = __builtin_fmaf(-d, q, n);
  const float q1 = __builtin_fmaf(e, r, q);
#ifdef BBM_HIP_DIV_SUB
  // q1 is the correctly rounded quotient where numerator and quotient are normal floats (or n = 0).  A subnormal
  // numerator or quotient rounds the remainder e to the subnormal grid, so the correction can be off by an ulp
  // there: those lanes (a wave-uniform branch, taken only when some lane needs it) divide in double with one f64
  // remainder step (f_div_d), rounded once to float -- the IEEE quotient on the subnormal grid as well.
  const bool fast = (__builtin_isnormal(q1) && __builtin_isnormal(n)) || n == 0.0f;
  float res = q1;
  if (__builtin_amdgcn_ballot_w64(!fast) != 0)
  {
    const double dd = double(d), nd = double(n);
    const double q0 = double(q);
    const double qd = __builtin_fma(__builtin_fma(-dd, q0, nd), double(r), q0);
    const float s = __builtin_isfinite(qd) ? float(qd) : q;      // d = 0 / inf, n = inf, NaN: IEEE result q
    res = fast ? q1 : s;
  }
  return res;
#else
  // q1 is the corrected quotient only where it is a normal float: for a subnormal quotient the remainder e is
  // itself rounded to the subnormal grid and the "correction" can move a correctly rounded q (n * rcp(d), within
  // ~1e-7 relative) off by an ulp; q is kept there, and for the IEEE special cases (inf, NaN, 0) as before.
  return __builtin_isnormal(q1) ? q1 : q;
#endif
}

// n / d correctly rounded on the subnormal grid as well (EXACT), for a finite normal d and any float n: the f32
// reciprocal seed q = n rcp(d) (~2^-22 relative), one remainder step in double (n - d q is exact in double: a 48-bit
// product and a cancelling difference), rounded once to float -- the IEEE float quotient (a subnormal or zero quotient
// from the IEEE double quotient, below), subnormal numerators included, where div_nr's f32 remainder is itself rounded
// to the subnormal grid.  For the sites where a subnormal intermediate can flow into a normal output (the Beckmann D
// of a far-tail halfway vector and the two quotients downstream of it); EXACT = false is div_nr.  Selected per
// launch (bbm_hip_set_exact_subnormals): measured +3.6-4.3 % on the headline kernel (0.703 -> 0.734, 0.726 -> 0.752 ms per 100 M pairs),
// CookTorrance eval+pdf then bit-identical to the reference on every lane of the 1 M-pair batches.  d = 0 / inf /
// NaN give inf / NaN, which those sites select away (or guard: Ward's pdf).  (Widening the fallback below to NaN
// and infinite quotients was tried in round 6: the fused Aggregate(Lambertian, NganHe) kernel then faulted on the
// GPU -- an illegal address, results permuted -- so the IEEE special cases stay with the callers.)
template<bool EXACT>
__device__ __forceinline__ float div_sub(float n, float d)
{
  if constexpr (EXACT)
  {
    const float r = __builtin_amdgcn_rcpf(d);
    const double q0 = double(n * r);
    float q = float(__builtin_fma(__builtin_fma(-double(d), q0, double(n)), double(r), q0));
    // A quotient that is not a normal float can lie exactly on (or within the step's error of) a midpoint of the
    // subnormal grid -- a normal one cannot: n = d m with m of 25 significant bits would need more than 24 bits in n
    // -- so those lanes (a wave-uniform branch, rarely taken) take the IEEE double quotient instead, which rounds to
    // the float grid exactly as the float division (53 >= 2 x 24 + 2, and a tie is exact in double).  Found by the
    // exhaustive device sweep of erfcf (tests/test_gpu_libm.py: erfcf(10) = 1.5 x 2^-149 rounded to even).
    const bool sub = __builtin_fabsf(q) < 0x1p-126f;
    if (__builtin_amdgcn_ballot_w64(sub) != 0)
      if (sub) q = float(double(n) / double(d));
    return q;
  }
  else return div_nr(n, d);
}

// a / d for the quotients that are a normal float or exactly 0 on every lane whose result is used (a finite
// nonzero divisor bounded away from the subnormal range, e.g. 1 / |h| with |h|^2 in (0, 4], or Fresnel's
// (g - c) / (g + c) with c > 0): the Markstein step alone, no special-case select.  Same result as div_nr there.
__device__ __forceinline__ float div_nr_n(float n, float d)
{
  const float r = __builtin_amdgcn_rcpf(d);
  const float q = n * r;
  return __builtin_fmaf(__builtin_fmaf(-d, q, n), r, q);
}

// sqrtf (IEEE, correctly rounded) as v_rsq_f32 and one Newton/Markstein step: s = x rsq(x), h = rsq(x) / 2,
// s' = s + (x - s^2) h with the residual x - s^2 exact (FMA) -- the correctly rounded root except within ~2^-22 ulp
// of a rounding midpoint (a root is never exactly one), ~7 VALU against the compiler's ~14-instruction sequence
// with its denormal scaling.  Zero, subnormal, infinite and NaN arguments take the hardware root (0, inf and NaN
// exact; a subnormal argument to ~1 ulp).
__device__ __forceinline__ float sqrt_nr(float x)
{
#ifdef BBM_HIP_SQRT_IEEE
  return sqrtf(x);
#else
  const float y = __builtin_amdgcn_rsqf(x);
  const float s = x * y;
  const float s1 = __builtin_fmaf(__builtin_fmaf(-s, s, x), 0.5f * y, s);
  return __builtin_isnormal(x) ? s1 : __builtin_amdgcn_sqrtf(x);
#endif
}

// ---------------------------------------------------------------- exponentials and powers
//
// Measured on gfx950 (tools/hwmath_probe.hip, every float in range): v_log_f32 is within 2.0 * 2^-24 relative of
// log2(x) for all normal x (incl. x -> 1), v_exp_f32 within 1.42 * 2^-24 relative on [-1, 1].  Neither returns
// subnormal results, and the device library's expf flushes below x = -103.28 although e^x still rounds to
// 2^-149 down to x = -103.97.  The reference (glibc) rounds every result into the subnormal range, and a BSDF
// value like D / (z_in z_out) carries such a subnormal into the normal range, so every exponential here
// scales by 2^n with v_ldexp_f32 (one rounding, subnormals kept; the kernels run with f32 denormals enabled).
constexpr float kLn2F = 0.693147180559945309f;

// 2^f for |f| <= 0.5 in double: 1 + f q(f), q a degree-8 polynomial fitted to (2^f - 1) / f on Chebyshev nodes
// of [-0.5, 0.5] (weighted for relative error): max relative error 2^-45.7 with double Horner, measured over 4e5
// points -- 9 f64 FMAs where the degree-11 Taylor series of e^(f ln2) took 12 and a multiply.  2^0 = 1 exactly.
__device__ __forceinline__ double exp2_poly(double f)
{
  double p = 1.013635714986865e-07;
  p = __builtin_fma(p, f, 1.3258369625240471e-06);
  p = __builtin_fma(p, f, 1.5253063845032086e-05);
  p = __builtin_fma(p, f, 0.00015403440667862952);
  p = __builtin_fma(p, f, 0.0013333557468222406);
  p = __builtin_fma(p, f, 0.009618129181589533);
  p = __builtin_fma(p, f, 0.055504108669737956);
  p = __builtin_fma(p, f, 0.24022650695720274);
  p = __builtin_fma(p, f, 0.6931471805598511);
  return __builtin_fma(p, f, 1.0);
}

// e^a in double for a in [-700, 700], to ~2^-44 relative (exp2_poly and an exact scaling)
__device__ __forceinline__ double exp_dd(double a)
{
  const double t = a * 1.4426950408889634074;
  const double n = __builtin_rint(t);
  return __builtin_ldexp(exp2_poly(t - n), int(n));
}

// The float nearest 2^t for a double t: correctly rounded except within ~2^-18 ulp of a rounding midpoint
// (2^-40 relative before the one rounding), over the whole range: overflow to inf, subnormal results rounded
// once by the f64 -> f32 conversion (f32 denormals are enabled), 0 below 2^-150.
__device__ __forceinline__ float exp2_cr(double t)
{
  const double n = __builtin_rint(t);
  const double p = exp2_poly(t - n);
  const float r = float(__builtin_ldexp(p, int(__builtin_fmin(__builtin_fmax(n, -400.0), 400.0))));
  return (t < -400.0) ? 0.0f : ((t > 400.0) ? __builtin_inff() : r);   // +-inf; NaN propagates through r
}

// expf over the whole float range, subnormal results included, to ~1.5 ulp (x log2(e) split into a head and a
// tail, v_exp_f32 of the fraction, v_ldexp_f32 by the integer part -- the library's scheme, whose only flaw here
// is its underflow cutoff: it returns 0 below x = -103.28 where e^x still rounds to 2^-149 down to -103.97).  A
// subnormal result is rounded once by v_ldexp_f32 from the 24-bit fraction: its error is <= 0.5 ulp of the
// subnormal grid + 1.4 2^-24 relative, so it differs from the correctly rounded value only where that lies
// within ~1e-7 relative of a midpoint of the grid (rare; the parity tests prove such lanes one by one).  The
// exact alternative (exp2_cr below the normal range) cost the headline CookTorrance kernel 9 %: with roughness
// 0.1 a few percent of all halfway vectors have their Beckmann exponent in [-104, -87].
__device__ __forceinline__ float expf_dn(float x)
{
  constexpr float kLog2eHi = 1.44269502162933349609375f;          // float(log2 e)
  constexpr float kLog2eLo = 1.925963033500011079e-08f;          // log2 e - kLog2eHi
  const float t = x * kLog2eHi;
  const float e = __builtin_fmaf(x, kLog2eLo, __builtin_fmaf(x, kLog2eHi, -t));
  const float n = __builtin_rintf(t);
  const float r = __builtin_ldexpf(__builtin_amdgcn_exp2f((t - n) + e), int(__builtin_fmaxf(n, -400.0f)));
  // x = -inf: t - n is NaN; e^x < 2^-150 rounds to 0 below x = -104; overflow to inf above 88.72
  return (x < -104.0f) ? 0.0f : ((x > 88.7228394f) ? __builtin_inff() : r);
}

// expf, branch-free, over the whole float range: the float nearest e^x (what glibc's expf returns, <= 0.502 ulp)
// except within ~2^-20 ulp of a rounding midpoint, subnormal results rounded once.  t = x log2(e) in double
// (|t| <= 150 on the finite domain: absolute error <= 2^-45.8) and exp2_cr: ~15 f64 VALU per call against ~10 f32
// for expf_dn, whose 1.4-ulp results differ from glibc's by an ulp on a few percent of all lanes and by a
// subnormal ulp -- up to 1e-4 relative once a quotient lifts the value back into the normal range -- below
// x = -87.3.  Every lane takes the same path, so no divergence (the earlier exact-below-the-normal-range branch
// cost the headline kernel 9 %).
__device__ __forceinline__ float expf_rn(float x) { return exp2_cr(double(x) * 1.4426950408889634074); }

// glibc's expf itself (glibc 2.35, sysdeps/ieee754/flt-32/e_expf.c with e_exp2f_data.c -- the Arm
// optimized-routines algorithm the reference's bbm::exp(float) -> std::exp -> expf runs on x86-64), restated in
// IEEE double ops: x N / ln2 = k + r (N = 32), 2^(k/N) from a 32-entry table of doubles plus an exponent shift,
// 2^(r/N) by a cubic, one final rounding to float.  The x86-64 library is the ifunc variant built with FMA
// contraction (__expf_fma on any FMA-capable host): r = fma(InvLn2N, x, -kd) and the cubic's three FMAs.  This
// restatement's steps, transcribed to host C (oracle/expf_glibc_check.c), return the same float as the container's
// libm for EVERY float in [-110, 90] (2.24e9 inputs); the device code itself is pinned by strided GPU sweeps of the
// bit patterns against the host libm (tests/test_gpu_libm.py).  Outside that range glibc's special cases (0, inf,
// NaN) are mirrored by selects.
// ~10 f64 VALU + a 64-bit table gather, branch-free: cheaper than exp2_cr's polynomial and exact to the bit.
__device__ __constant__ const uint64_t kExpfTab[32] = {
    0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
    0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
    0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
    0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
    0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
    0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
    0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
    0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull};
// The tables of the glibc restatements below (expf's 2^(j/32), logf's and powf's (1/c, log c)) are read per lane with a
// data-dependent index.  From the constant segment each lookup is a divergent 8-16 B gather through the vector memory
// pipeline, queued behind the kernel's streaming loads; so every kernel of the library copies them into LDS first
// (math_tables_init()) and looks them up with ds_read_b64 -- conflict-free, as each table spans the 64 banks once.
// Every wave writes the whole table itself (lanes 0..31; all waves of a workgroup write the same values to the same
// addresses) and reads it back in program order: no workgroup barrier delays the first streaming loads (with wave 0
// filling the table for all behind one s_barrier, the memory-bound headline kernel lost 1.7 %; with a private copy per
// wave, indexed by the wave id, Bagher and the He family lost 10-40 % to the extra addressing).  Measured against the
// constant-segment gathers (profiles/r05_ab_lds_tables.txt, ms per 10 M pairs): the powf / logf lobes
// (AshikhminShirley, Phong, Lafortune and their Ngan / Low forms) -5 to -12 %, PhongWalter -3.5 %, HeHolzschuch -4 %,
// the Beckmann models -1 to -2 %; the models that read no table pay the prologue: GGX / GGXHeitz / LowSmooth +3-4 %.
// -DBBM_HIP_EXPF_BPERM: every lane holds entry (lane & 31) in two VGPRs and the lookup is two ds_bpermute_b32.
// -DBBM_HIP_CONST_TABLES (A/B): the constant-segment gathers.
#ifndef BBM_HIP_CONST_TABLES
static __shared__ uint64_t g_lds_exptab[32];
static __shared__ double g_lds_logftab[16][2];
static __shared__ double g_lds_log2tab[16][2];
#endif
// LDS = false: the constant-segment table (for code that runs out of line, where a gather is cheaper than keeping the
// kernel's LDS copy reachable -- Bagher's shadowing tail)
template<bool LDS = true>
__device__ __forceinline__ uint64_t expf_tab(uint32_t j)
{
#ifndef BBM_HIP_CONST_TABLES
  if constexpr (LDS) return g_lds_exptab[j];
#endif
#ifdef BBM_HIP_EXPF_BPERM
  const uint64_t mine = kExpfTab[__lane_id() & 31u];
  const int lo = __builtin_amdgcn_ds_bpermute(int(j << 2), int(uint32_t(mine)));
  const int hi = __builtin_amdgcn_ds_bpermute(int(j << 2), int(uint32_t(mine >> 32)));
  return (uint64_t(uint32_t(hi)) << 32) | uint32_t(lo);
#else
  return kExpfTab[j];
#endif
}

template<bool LDS = true>
__device__ __forceinline__ float expf_glibc(float x)
{
  constexpr double kInvLn2N = 0x1.71547652b82fep+0 * 32;
  constexpr double kShift = 0x1.8p+52;
  constexpr double kC0 = 0x1.c6af84b912394p-5 / 32 / 32 / 32, kC1 = 0x1.ebfce50fac4f3p-3 / 32 / 32,
                   kC2 = 0x1.62e42ff0c52d6p-1 / 32;
  const double xd = double(x);
  const double kb = __builtin_fma(kInvLn2N, xd, kShift);          // k in the low bits (ties to even)
  const uint64_t ki = uint64_t(__builtin_bit_cast(int64_t, kb));
  const double kd = kb - kShift;
  const double r = __builtin_fma(kInvLn2N, xd, -kd);             // x N / ln2 - k, |r| <= 1/2
#ifdef BBM_HIP_EXPF_NOGATHER_TIMING
  // timing probe only (tools/build_variant.sh): the table gather replaced by arithmetic of the same shape (wrong values)
  const double s = __builtin_bit_cast(double, (0x3fef000000000000ull | ((ki & 31u) << 40)) + (ki << 47));
#else
  const double s = __builtin_bit_cast(double, expf_tab<LDS>(ki & 31u) + (ki << 47));   // 2^(k/N)
#endif
  const double z = __builtin_fma(kC0, r, kC1);
  const double r2 = r * r;
  double y = __builtin_fma(kC2, r, 1.0);
  y = __builtin_fma(z, r2, y);
  const float res = float(y * s);
  // |x| >= 88 or NaN in glibc: -inf and x < log(2^-150) -> 0, x > log(2^128) -> inf, NaN -> NaN (via res)
  return (x < -0x1.9fe368p6f) ? 0.0f : ((x > 0x1.62e42ep6f) ? __builtin_inff() : res);
}
// the exponential of the eval kernels' Gaussian-like lobes (Ward, EPD; -DBBM_HIP_LOBES_EXP_DN: the 1.4-ulp
// expf_dn, A/B).  Measured against expf_dn (tools/gpu_r03_e.sh, ms per 10 M pairs / bit-exact lanes): Ward
// 0.060 -> 0.060 ms, 97.0 -> 99.7 %; EPD 0.270 -> 0.285 ms, 80.1 -> 83.5 %
template<bool LDS = true> __device__ __forceinline__ float expf_glibc_neg(float x);
__device__ __forceinline__ float expf_lobe(float x)
{
#ifdef BBM_HIP_LOBES_EXP_DN
  return expf_dn(x);
#else
  return expf_glibc_neg(x);
#endif
}

// the same for x <= 0 or NaN (an exponent that is minus a square or a quotient of squares): no overflow select
template<bool LDS>
__device__ __forceinline__ float expf_glibc_neg(float x)
{
  constexpr double kInvLn2N = 0x1.71547652b82fep+0 * 32;
  constexpr double kShift = 0x1.8p+52;
  constexpr double kC0 = 0x1.c6af84b912394p-5 / 32 / 32 / 32, kC1 = 0x1.ebfce50fac4f3p-3 / 32 / 32,
                   kC2 = 0x1.62e42ff0c52d6p-1 / 32;
  const double xd = double(x);
  const double kb = __builtin_fma(kInvLn2N, xd, kShift);
  const uint64_t ki = uint64_t(__builtin_bit_cast(int64_t, kb));
  const double kd = kb - kShift;
  const double r = __builtin_fma(kInvLn2N, xd, -kd);
  const double s = __builtin_bit_cast(double, expf_tab<LDS>(ki & 31u) + (ki << 47));
  const double z = __builtin_fma(kC0, r, kC1);
  const double r2 = r * r;
  double y = __builtin_fma(kC2, r, 1.0);
  y = __builtin_fma(z, r2, y);
  const float res = float(y * s);
  return (x < -0x1.9fe368p6f) ? 0.0f : res;
}

// glibc 2.35's logf and powf (sysdeps/ieee754/flt-32/e_logf.c, e_powf.c with e_logf_data.c, e_powf_log2_data.c and
// e_exp2f_data.c -- the Arm optimized-routines algorithms behind the reference's bbm::log(float) / bbm::pow(float,
// float) -> std::log / std::pow -> logf / powf on x86-64), restated in IEEE double ops as the FMA-contracted ifunc
// variant the host runs.  Neither is correctly rounded (logf 0.82 ulp; powf carries up to 1.27 2^-26 relative error
// into its one rounding, so ~0.1 % of its results are not the nearest float), and where the reference cancels
// right after (Bagher's 1 - e^(c theta^k)) only glibc's own float reproduces its result.  The tables and polynomials
// are glibc's data (as in this machine's libm.so.6), not the reference's.  A host C transcription of the same steps
// (oracle/glibcf_check.c) matches the host libm for logf on every positive float and powf on 1e9 random pairs (0
// mismatches); the device code is pinned by strided GPU sweeps against the host libm (tests/test_gpu_libm.py).
__device__ __constant__ const double kLogfTab[16][2] = {    // {1/c, log c}
    {0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2}, {0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2},
    {0x1.49539f0f010b0p+0, -0x1.01eae7f513a67p-2}, {0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3},
    {0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3}, {0x1.25e227b0b8ea0p+0, -0x1.1aa2bc79c8100p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4}, {0x1.12358f08ae5bap+0, -0x1.1973c5a611cccp-4},
    {0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5}, {0x1p+0, 0x0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5}, {0x1.ca4b31f026aa0p-1, 0x1.c5e53aa362eb4p-4},
    {0x1.b2036576afce6p-1, 0x1.526e57720db08p-3}, {0x1.9c2d163a1aa2dp-1, 0x1.bc2860d224770p-3},
    {0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2}, {0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2}};
__device__ __constant__ const double kPowfLog2Tab[16][2] = {    // {1/c, log2 c}
    {0x1.661ec79f8f3bep+0, -0x1.efec65b963019p-2}, {0x1.571ed4aaf883dp+0, -0x1.b0b6832d4fca4p-2},
    {0x1.49539f0f010b0p+0, -0x1.7418b0a1fb77bp-2}, {0x1.3c995b0b80385p+0, -0x1.39de91a6dcf7bp-2},
    {0x1.30d190c8864a5p+0, -0x1.01d9bf3f2b631p-2}, {0x1.25e227b0b8ea0p+0, -0x1.97c1d1b3b7af0p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.2f9e393af3c9fp-3}, {0x1.12358f08ae5bap+0, -0x1.960cbbf788d5cp-4},
    {0x1.0953f419900a7p+0, -0x1.a6f9db6475fcep-5}, {0x1p+0, 0x0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.338ca9f24f53dp-4}, {0x1.ca4b31f026aa0p-1, 0x1.476a9543891bap-3},
    {0x1.b2036576afce6p-1, 0x1.e840b4ac4e4d2p-3}, {0x1.9c2d163a1aa2dp-1, 0x1.40645f0c6651cp-2},
    {0x1.886e6037841edp-1, 0x1.88e9c2c1b9ff8p-2}, {0x1.767dcf5534862p-1, 0x1.ce0a44eb17bccp-2}};

template<bool LDS = true>
__device__ __forceinline__ double powf_log2tab(uint32_t i, int c)
{
#ifndef BBM_HIP_CONST_TABLES
  if constexpr (LDS) return g_lds_log2tab[i][c];
#endif
  return kPowfLog2Tab[i][c];
}
template<bool LDS = true>
__device__ __forceinline__ double logf_tab(uint32_t i, int c)
{
#ifndef BBM_HIP_CONST_TABLES
  if constexpr (LDS) return g_lds_logftab[i][c];
#endif
  return kLogfTab[i][c];
}
// Every kernel's first statement (tests/test_kernel_prologue.py checks that every kernel of the library starts with
// it): every wave fills the tables with its active lanes (below); the wave's later reads of them follow in program
// order (a wavefront-scope fence keeps the compiler from moving them above the stores)
// Validation builds only (-DBBM_HIP_TABLES_POISON): what a kernel whose model is declared table-free
// (uses_math_tables, kernels.hpp) writes instead of the tables -- NaN everywhere, so any lookup shows in the parity
// tests.
__device__ __forceinline__ void math_tables_poison()
{
#ifndef BBM_HIP_CONST_TABLES
  const unsigned nl = unsigned(__builtin_popcountll(__builtin_amdgcn_read_exec()));
  for (unsigned t = __lane_id(); t < 32; t += nl)
  {
    g_lds_exptab[t] = 0x7ff8000000000000ull;
    g_lds_logftab[t >> 1][t & 1] = __builtin_nan("");
    g_lds_log2tab[t >> 1][t & 1] = __builtin_nan("");
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
#endif
}

__device__ __forceinline__ void math_tables_init()
{
#ifndef BBM_HIP_CONST_TABLES
  // each wave writes the 32 entries it will read itself (no workgroup barrier): the wave's active lanes -- all 64, or
  // the low lanes of a partial wave (a block smaller than a wave, a ragged last wave, any block shape) -- stride over
  // the entries, so every entry is written whatever the wave's population
  const unsigned nl = unsigned(__builtin_popcountll(__builtin_amdgcn_read_exec()));
  for (unsigned t = __lane_id(); t < 32; t += nl)
  {
    g_lds_exptab[t] = kExpfTab[t];
    g_lds_logftab[t >> 1][t & 1] = kLogfTab[t >> 1][t & 1];
    g_lds_log2tab[t >> 1][t & 1] = kPowfLog2Tab[t >> 1][t & 1];
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
#endif
}

// x = 2^k z with z in [0x3f330000, 2 x 0x3f330000): the bits of z, k, and the table row (subnormal x normalised)
__device__ __forceinline__ uint32_t glibcf_reduce(float x, uint32_t& i, int& k)
{
  const uint32_t ix0 = __float_as_uint(x);
  const uint32_t ix = (ix0 < 0x00800000u) ? ((__float_as_uint(x * 0x1p23f) & 0x7fffffffu) - (23u << 23)) : ix0;
  const uint32_t tmp = ix - 0x3f330000u;
  i = (tmp >> 19) & 15u;
  k = int32_t(tmp) >> 23;
  return ix - (tmp & 0xff800000u);
}

template<bool LDS = true>
__device__ __forceinline__ float logf_glibc(float x)
{
  uint32_t i;
  int k;
  const double z = double(__uint_as_float(glibcf_reduce(x, i, k)));
  const double r = __builtin_fma(z, logf_tab<LDS>(i, 0), -1.0);
  const double y0 = __builtin_fma(double(k), 0x1.62e42fefa39efp-1, logf_tab<LDS>(i, 1));
  const double r2 = r * r;
  double y = __builtin_fma(0x1.5575b0be00b6ap-2, r, -0x1.ffffef20a4123p-2);
  y = __builtin_fma(-0x1.00ea348b88334p-2, r2, y);
  y = __builtin_fma(y, r2, y0 + r);
  float res = float(y);                                           // x = 1: exactly +0
  res = (x == __builtin_inff()) ? x : res;
  res = (x == 0.0f) ? -__builtin_inff() : res;
  return (x < 0.0f || x != x) ? __builtin_nanf("") : res;
}

// powf for x >= 0 (or NaN), any y (the reference's uses: a distance or a sum of squares to a parameter power)
template<bool LDS = true>
__device__ __forceinline__ float powf_glibc(float x, float y)
{
  uint32_t i;
  int k;
  const double z = double(__uint_as_float(glibcf_reduce(x, i, k)));
  const double r = __builtin_fma(z, powf_log2tab<LDS>(i, 0), -1.0);
  const double y0 = powf_log2tab<LDS>(i, 1) + double(k);
  const double r2 = r * r;
  double q0 = __builtin_fma(0x1.27616c9496e0bp-2, r, -0x1.71969a075c67ap-2);
  const double p = __builtin_fma(0x1.ec70a6ca7baddp-2, r, -0x1.7154748bef6c8p-1);
  const double r4 = r2 * r2;
  double q = __builtin_fma(0x1.71547652ab82bp+0, r, y0);
  q = __builtin_fma(p, r2, q);
  const double ylogx = double(y) * __builtin_fma(q0, r4, q);      // log2(x) y
  // 2^ylogx: k/32 + rr, 2^(k/32) from expf's table, a cubic in rr
  constexpr double kShift = 0x1.8p+52 / 32;
  const double kb = ylogx + kShift;
  const uint64_t ki = uint64_t(__builtin_bit_cast(int64_t, kb));
  const double rr = ylogx - (kb - kShift);
  const double s = __builtin_bit_cast(double, expf_tab<LDS>(uint32_t(ki) & 31u) + (ki << 47));
  const double zz = __builtin_fma(0x1.c6af84b912394p-5, rr, 0x1.ebfce50fac4f3p-3);
  double e = __builtin_fma(0x1.62e42ff0c52d6p-1, rr, 1.0);
  e = __builtin_fma(zz, rr * rr, e);
  float res = float(e * s);
  res = (ylogx > 0x1.fffffffd1d571p+6) ? __builtin_inff() : res;
  res = (ylogx <= -150.0) ? 0.0f : res;
  // special operands: pow(0, y) = 0 / inf, pow(inf, y) = inf / 0, NaN, pow(x, 0) = pow(1, y) = 1
  res = (x == 0.0f) ? ((y < 0.0f) ? __builtin_inff() : 0.0f) : res;
  res = (x == __builtin_inff()) ? ((y < 0.0f) ? 0.0f : __builtin_inff()) : res;
  res = (x != x || y != y || x < 0.0f) ? __builtin_nanf("") : res;
  return (y == 0.0f || x == 1.0f) ? 1.0f : res;
}

// powf_glibc for a finite normal x > 0 and a finite y: the same steps without the special-operand selects and the
// subnormal normalisation (pow(1, y) and pow(x, 0) come out as exactly 1 from the table row {1, 0} and r = 0), for the
// sites whose base is provably a positive normal float (Bagher's t = alpha + tan^2 / alpha, alpha >= its lower bound)
template<bool LDS = true>
__device__ __forceinline__ float powf_glibc_pos(float x, float y)
{
  const uint32_t ix = __float_as_uint(x);
  const uint32_t tmp = ix - 0x3f330000u;
  const uint32_t i = (tmp >> 19) & 15u;
  const int k = int32_t(tmp) >> 23;
  const double z = double(__uint_as_float(ix - (tmp & 0xff800000u)));
  const double r = __builtin_fma(z, powf_log2tab<LDS>(i, 0), -1.0);
  const double y0 = powf_log2tab<LDS>(i, 1) + double(k);
  const double r2 = r * r;
  const double q0 = __builtin_fma(0x1.27616c9496e0bp-2, r, -0x1.71969a075c67ap-2);
  const double p = __builtin_fma(0x1.ec70a6ca7baddp-2, r, -0x1.7154748bef6c8p-1);
  const double r4 = r2 * r2;
  double q = __builtin_fma(0x1.71547652ab82bp+0, r, y0);
  q = __builtin_fma(p, r2, q);
  const double ylogx = double(y) * __builtin_fma(q0, r4, q);
  constexpr double kShift = 0x1.8p+52 / 32;
  const double kb = ylogx + kShift;
  const uint64_t ki = uint64_t(__builtin_bit_cast(int64_t, kb));
  const double rr = ylogx - (kb - kShift);
  const double s = __builtin_bit_cast(double, expf_tab<LDS>(uint32_t(ki) & 31u) + (ki << 47));
  const double zz = __builtin_fma(0x1.c6af84b912394p-5, rr, 0x1.ebfce50fac4f3p-3);
  double e = __builtin_fma(0x1.62e42ff0c52d6p-1, rr, 1.0);
  e = __builtin_fma(zz, rr * rr, e);
  float res = float(e * s);
  res = (ylogx > 0x1.fffffffd1d571p+6) ? __builtin_inff() : res;
  return (ylogx <= -150.0) ? 0.0f : res;
}

// glibc's powf over every operand, negative bases included (e_powf.c: checkint -- an integer y gives |x|^y with the
// sign of x for odd y, a non-integer y NaN; -0 and -inf as +0 / +inf except for odd integers; pow(-1, +-inf) = 1):
// for parameters outside an attribute's range (Bagher's D with alpha <= 0, spectral.hpp), never on a hot path
template<bool LDS = true>
__device__ __forceinline__ float powf_glibc_any(float x, float y)
{
  if (!__builtin_signbit(x) || x != x) return powf_glibc<LDS>(x, y);
  const float ax = __builtin_fabsf(x);
  if (y == 0.0f) return 1.0f;
  if (y != y) return y;
  if (__builtin_isinf(y)) return (ax == 1.0f) ? 1.0f : powf_glibc<LDS>(ax, y);
  const bool integer = __builtin_truncf(y) == y;
  if (!integer) return (ax == 0.0f || __builtin_isinf(ax)) ? powf_glibc<LDS>(ax, y) : __builtin_nanf("");
  const bool odd = __builtin_fabsf(y) < 0x1p24f && (int32_t(y) & 1) != 0;
  const float r = powf_glibc<LDS>(ax, y);
  return odd ? -r : r;
}

// glibc 2.35's erff / erfcf (sysdeps/ieee754/flt-32/s_erff.c: Sun fdlibm's rational approximations in float
// arithmetic, no FMA variant, __ieee754_expf = the expf above), restated op for op -- what the reference's
// bbm::erf / bbm::erfc of a float return (std::erf / std::erfc -> erff / erfcf).  Neither is correctly rounded; the
// He family's shadowing term S1 subtracts erfc from a nearly equal quantity and the Beckmann VNDF sampler inverts
// erf by Newton steps, so only glibc's own floats reproduce the reference there.  Coefficients: fdlibm's floats as
// this machine's libm.so.6 holds them.  A host C transcription (oracle/erfcf_glibc_check.c) matches the host libm on
// all 2^32 inputs (0 mismatches); the device code is pinned by strided GPU sweeps (tests/test_gpu_libm.py).
namespace fdlibm_erf {
constexpr float erx = 8.4506291151e-01f, pp0 = 1.2837916613e-01f, pp1 = -3.2504209876e-01f,
                pp2 = -2.8481749818e-02f, pp3 = -5.7702702470e-03f, pp4 = -2.3763017452e-05f, qq1 = 3.9791721106e-01f,
                qq2 = 6.5022252500e-02f, qq3 = 5.0813062117e-03f, qq4 = 1.3249473704e-04f, qq5 = -3.9602282413e-06f,
                pa0 = -2.3621185683e-03f, pa1 = 4.1485610604e-01f, pa2 = -3.7220788002e-01f, pa3 = 3.1834661961e-01f,
                pa4 = -1.1089469492e-01f, pa5 = 3.5478305072e-02f, pa6 = -2.1663755178e-03f, qa1 = 1.0642088205e-01f,
                qa2 = 5.4039794207e-01f, qa3 = 7.1828655899e-02f, qa4 = 1.2617121637e-01f, qa5 = 1.3637083583e-02f,
                qa6 = 1.1984500103e-02f, ra0 = -9.8649440333e-03f, ra1 = -6.9385856390e-01f, ra2 = -1.0558626175e+01f,
                ra3 = -6.2375331879e+01f, ra4 = -1.6239666748e+02f, ra5 = -1.8460508728e+02f, ra6 = -8.1287437439e+01f,
                ra7 = -9.8143291473e+00f, sa1 = 1.9651271820e+01f, sa2 = 1.3765776062e+02f, sa3 = 4.3456588745e+02f,
                sa4 = 6.4538726807e+02f, sa5 = 4.2900814819e+02f, sa6 = 1.0863500214e+02f, sa7 = 6.5702495575e+00f,
                sa8 = -6.0424413532e-02f, rb0 = -9.8649431020e-03f, rb1 = -7.9928326607e-01f, rb2 = -1.7757955551e+01f,
                rb3 = -1.6063638306e+02f, rb4 = -6.3756646729e+02f, rb5 = -1.0250950928e+03f, rb6 = -4.8351919556e+02f,
                sb1 = 3.0338060379e+01f, sb2 = 3.2579251099e+02f, sb3 = 1.5367296143e+03f, sb4 = 3.1998581543e+03f,
                sb5 = 2.5530502930e+03f, sb6 = 4.7452853394e+02f, sb7 = -2.2440952301e+01f;

// |x| < 0.84375: y = r / s of the erf expansion in z = x^2
__device__ __forceinline__ float small_y(float x)
{
  const float z = x * x;
  const float r = pp0 + z * (pp1 + z * (pp2 + z * (pp3 + z * pp4)));
  const float s = 1.0f + z * (qq1 + z * (qq2 + z * (qq3 + z * (qq4 + z * qq5))));
  return div_nr(r, s);
}
// 0.84375 <= |x| < 1.25: P / Q in s = |x| - 1
__device__ __forceinline__ float mid_pq(float ax)
{
  const float s = ax - 1.0f;
  const float P = pa0 + s * (pa1 + s * (pa2 + s * (pa3 + s * (pa4 + s * (pa5 + s * pa6)))));
  const float Q = 1.0f + s * (qa1 + s * (qa2 + s * (qa3 + s * (qa4 + s * (qa5 + s * qa6)))));
  return div_nr(P, Q);
}
// 1.25 <= |x| < 28: erfc(|x|) |x| = exp(-z^2 - 0.5625) exp((z - |x|)(z + |x|) + R/S), z = |x| with the low mantissa
// bits cleared (`mask`), R/S in s = 1/x^2 on [1.25, 1/0.35) or beyond (`split`).  The second branch's polynomials
// have one coefficient fewer: a zero top coefficient leaves every rounding unchanged (c + s 0 = c), so one Horner
// chain with selected coefficients serves both.
__device__ __forceinline__ float tail_r(float ax, uint32_t split, uint32_t mask)
{
  const bool a = __float_as_uint(ax) < split;
  const float s = div_nr(1.0f, ax * ax);
  const float R = (a ? ra0 : rb0) + s * ((a ? ra1 : rb1) + s * ((a ? ra2 : rb2) + s * ((a ? ra3 : rb3) +
                  s * ((a ? ra4 : rb4) + s * ((a ? ra5 : rb5) + s * ((a ? ra6 : rb6) + s * (a ? ra7 : 0.0f)))))));
  const float S = 1.0f + s * ((a ? sa1 : sb1) + s * ((a ? sa2 : sb2) + s * ((a ? sa3 : sb3) + s * ((a ? sa4 : sb4) +
                  s * ((a ? sa5 : sb5) + s * ((a ? sa6 : sb6) + s * ((a ? sa7 : sb7) + s * (a ? sa8 : 0.0f))))))));
  const float z = __uint_as_float(__float_as_uint(ax) & mask);
  return expf_glibc(-z * z - 0.5625f) * expf_glibc((z - ax) * (z + ax) + div_nr(R, S));
}
}  // namespace fdlibm_erf

// erfcf's three argument ranges as separate pieces (erfcf_glibc below is their composition; the He family's
// compaction kernel sorts the arguments of a block by range and evaluates each range densely, he.hpp):
// range of x: 0 = |x| >= 28, NaN (no arithmetic), 1 = |x| < 0.84375, 2 = [0.84375, 1.25), 3 = [1.25, 28)
__device__ __forceinline__ int erfcf_range(float x)
{
  const uint32_t ix = __float_as_uint(x) & 0x7fffffffu;
  return (ix < 0x3f580000u) ? 1 : ((ix < 0x3fa00000u) ? 2 : ((ix < 0x41e00000u) ? 3 : 0));
}
__device__ __forceinline__ float erfcf_r0(float x) { return (x != x) ? x : ((__float_as_uint(x) >> 31) ? 2.0f : 0.0f); }
__device__ __forceinline__ float erfcf_r1(float x)
{
  using namespace fdlibm_erf;
  const uint32_t hx = __float_as_uint(x), ix = hx & 0x7fffffffu;
  const float y = small_y(x);
  float r = x * y;
  r += (x - 0.5f);
  const float res = (int32_t(hx) < 0x3e800000) ? 1.0f - (x + x * y) : 0.5f - r;
  return (ix < 0x32800000u) ? 1.0f - x : res;
}
__device__ __forceinline__ float erfcf_r2(float x)
{
  using namespace fdlibm_erf;
  const float pq = mid_pq(__builtin_fabsf(x));
  return (__float_as_uint(x) >> 31) ? 1.0f + (erx + pq) : (1.0f - erx) - pq;
}
__device__ __forceinline__ float erfcf_r3(float x)
{
  using namespace fdlibm_erf;
  const uint32_t ix = __float_as_uint(x) & 0x7fffffffu;
  const float ax = __builtin_fabsf(x);
  // r / x can fall to ~1e-37 (x ~ 9): the f64 remainder step (div_sub<true>) keeps that quotient exact where
  // div_nr's f32 remainder would be subnormal
  const float q = div_sub<true>(tail_r(ax, 0x4036DB6Du, 0xffffe000u), ax);
  return (__float_as_uint(x) >> 31) ? ((ix >= 0x40c00000u) ? 2.0f : 2.0f - q) : q;    // x < -6: 2 - tiny = 2
}

__device__ __forceinline__ float erfcf_glibc(float x)
{
  const uint32_t ix = __float_as_uint(x) & 0x7fffffffu;
  float res;
  if (ix < 0x3f580000u) res = erfcf_r1(x);
  else if (ix < 0x3fa00000u) res = erfcf_r2(x);
  else if (ix < 0x41e00000u) res = erfcf_r3(x);
  else res = erfcf_r0(x);                                      // |x| >= 28 (inf included): 2 - tiny, tiny^2
  return (x != x) ? x : res;
}

__device__ __forceinline__ float erff_glibc(float x)
{
  using namespace fdlibm_erf;
  const uint32_t hx = __float_as_uint(x), ix = hx & 0x7fffffffu;
  const bool neg = (hx >> 31) != 0;
  const float ax = __builtin_fabsf(x);
  float res;
  if (ix < 0x3f580000u)
  {
    res = x + x * small_y(x);
    res = (ix < 0x31800000u) ? ((ix < 0x04000000u) ? 0.0625f * (16.0f * x + (16.0f * pp0) * x) : x + pp0 * x) : res;
  }
  else if (ix < 0x3fa00000u)
  {
    const float pq = mid_pq(ax);
    res = neg ? -erx - pq : erx + pq;
  }
  else if (ix < 0x40c00000u)
  {
    const float q = div_sub<true>(tail_r(ax, 0x4036DB6Eu, 0xfffff000u), ax);
    res = neg ? q - 1.0f : 1.0f - q;
  }
  else res = neg ? -1.0f : 1.0f;                               // |x| >= 6 (inf included): +-(1 - tiny)
  return (x != x) ? x : res;
}

// glibc 2.35's atan2f (sysdeps/ieee754/flt-32/e_atan2f.c with s_atanf.c: Sun fdlibm's float algorithms, no FMA
// variant) -- what the reference's spherical::phi (core/spherical.h:42-46) and every float atan2 call -- restated op
// for op in float arithmetic: q = |y / x| (IEEE division), atan(q) by fdlibm's reduction to one of four breakpoints
// (atan 0.5, 1, 1.5, inf as hi + lo; one more IEEE division) and its 11-term odd polynomial, then the quadrant
// fix-ups with pi_lo.  Not correctly rounded, hence restated rather than rounded from a double atan2.  Same float as
// this machine's libm on 6e7 random pairs (unit-vector components, any finite floats, mixed magnitudes) and on every
// combination of zeros, infinities and NaN, and at x = 1 (glibc's atanf shortcut, the same float) for every 13th y --
// measured on a host C transcription (oracle/atan2f_glibc_check.c); the device code by GPU sweeps against the host
// libm (tests/test_gpu_libm.py).  Selects around two IEEE divisions.
namespace fdlibm_atan {
constexpr float kHi[4] = {4.6364760399e-01f, 7.8539812565e-01f, 9.8279368877e-01f, 1.5707962513e+00f};
constexpr float kLo[4] = {5.0121582440e-09f, 3.7748947079e-08f, 3.4473217170e-08f, 7.5497894159e-08f};
constexpr float kT[11] = {3.3333334327e-01f, -2.0000000298e-01f, 1.4285714924e-01f, -1.1111110449e-01f,
                          9.0908870101e-02f, -7.6918758452e-02f, 6.6610731184e-02f, -5.8335702866e-02f,
                          4.9768779427e-02f, -3.6531571299e-02f, 1.6285819933e-02f};
// atanf (s_atanf.c) of a float x >= 0 below 2^25
__device__ __forceinline__ float atan_pos(float x)
{
  const uint32_t ix = __float_as_uint(x);
  const int id = (ix < 0x3f300000u) ? 0 : ((ix < 0x3f980000u) ? 1 : ((ix < 0x401c0000u) ? 2 : 3));
  // num = a x + b, den = c x + d with the reference's roundings (a x exact for a in {0, 1, 2}; 1.5 x rounded, then
  // + 1): constant selects and two products, no per-lane branches
  const float a = (id == 0) ? 2.0f : ((id == 3) ? 0.0f : 1.0f);
  const float b = (id == 0) ? -1.0f : ((id == 2) ? -1.5f : -1.0f);
  const float c = (id == 2) ? 1.5f : 1.0f;
  const float d = (id == 0) ? 2.0f : ((id == 3) ? 0.0f : 1.0f);
  const float num = a * x + b;
  const float den = c * x + d;
  const bool small = ix < 0x3ee00000u;                           // |x| < 0.4375: no reduction
  const float t = small ? x : __fdiv_rn(num, den);
  const float z = t * t;
  const float w = z * z;
  const float s1 = z * (kT[0] + w * (kT[2] + w * (kT[4] + w * (kT[6] + w * (kT[8] + w * kT[10])))));
  const float s2 = w * (kT[1] + w * (kT[3] + w * (kT[5] + w * (kT[7] + w * kT[9]))));
  const float hi = (id == 0) ? kHi[0] : ((id == 1) ? kHi[1] : ((id == 2) ? kHi[2] : kHi[3]));
  const float lo = (id == 0) ? kLo[0] : ((id == 1) ? kLo[1] : ((id == 2) ? kLo[2] : kLo[3]));
  return small ? t - t * (s1 + s2) : hi - ((t * (s1 + s2) - lo) - t);
}
}  // namespace fdlibm_atan

__device__ __forceinline__ float atan2f_glibc(float y, float x)
{
  using namespace fdlibm_atan;
  constexpr float pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f, pi = 3.1415927410e+00f,
                  pi_lo = -8.7422776573e-08f;
  const uint32_t hx = __float_as_uint(x), hy = __float_as_uint(y), ix = hx & 0x7fffffffu, iy = hy & 0x7fffffffu;
  const bool yneg = (hy >> 31) != 0, xneg = (hx >> 31) != 0;
  const int m = int(yneg) | (int(xneg) << 1);
  const float big = kHi[3] + kLo[3];
  // the general case (finite, nonzero x != 1 and y): atan |y / x|, then the quadrant
  const int k = (int(iy) - int(ix)) >> 23;
  const float q = __builtin_fabsf(__fdiv_rn(y, x));
  float z = (__float_as_uint(q) >= 0x4c000000u) ? big : atan_pos(q);
  z = (k > 60) ? pi_o_2 + 0.5f * pi_lo : ((xneg && k < -60) ? 0.0f : z);
  float r = (m == 0) ? z : ((m == 1) ? -z : ((m == 2) ? pi - (z - pi_lo) : (z - pi_lo) - pi));
  // (glibc's x = 1 shortcut, atanf(y), is this same float: y / 1 = y, |y| >= 2^25 -> hi + lo = pi_o_2 + pi_lo / 2)
  // infinities, zeros and NaN on a wave-uniform branch: a direction's components are finite and almost never 0
  const bool special = (ix - 1u >= 0x7f7fffffu) || (iy - 1u >= 0x7f7fffffu);
  if (__builtin_expect(__builtin_amdgcn_ballot_w64(special) == 0, true)) return r;
  r = (iy == 0x7f800000u) ? (yneg ? -pi_o_2 : pi_o_2) : r;
  const float xinf = (iy == 0x7f800000u) ? ((m == 0) ? pi_o_4 : (m == 1) ? -pi_o_4 : (m == 2) ? 3.0f * pi_o_4 : -3.0f * pi_o_4)
                                         : ((m == 0) ? 0.0f : (m == 1) ? -0.0f : (m == 2) ? pi : -pi);
  r = (ix == 0x7f800000u) ? xinf : r;
  r = (ix == 0) ? (yneg ? -pi_o_2 : pi_o_2) : r;
  r = (iy == 0) ? ((m < 2) ? y : ((m == 2) ? pi : -pi)) : r;
  return (ix > 0x7f800000u || iy > 0x7f800000u) ? x + y : r;
}

// glibc 2.35's sinf and cosf (sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c, sincosf.h, sincosf_data.c -- the Arm
// optimized-routines algorithms behind the reference's bbm::cossin(float) = (std::cos, std::sin), backbone/native/
// include/backbone/math.h:126, on every sampler's angle), restated in IEEE double ops as the FMA-contracted ifunc
// variant, both from one shared reduction.  |y| below 0.75 (pi/4's abstop12): the polynomials in y directly (y itself
// / 1 below 2^-12); |y| < 120: the quadrant n from y (2/pi) 2^24 truncated (+2^23, >> 24), r = y - n pi/2 by one
// FMA, sin(r) by the odd and cos(r) by the even polynomial, swapped in odd quadrants and signed per quadrant.  The
// coefficients are glibc's table (__sincosf_table[0]; table [1] is its even half negated, which the sign select
// reproduces exactly).  A host C transcription of these steps (oracle/sincosf_glibc_check.c) gives glibc's sinf and
// cosf bit for bit for every float |y| < 120 (all 2.2e9); the device code is pinned by a strided GPU sweep of that
// domain (tests/test_gpu_libm.py).  Larger |y|, inf and NaN (no sampler angle) take the device library's sincosf.
__device__ __forceinline__ void sincosf_glibc(float y, float* sp, float* cp)
{
  constexpr double kC0 = 1.0, kC1 = -0x1.ffffffd0c621cp-2, kC2 = 0x1.55553e1068f19p-5, kC3 = -0x1.6c087e89a359dp-10,
                   kC4 = 0x1.99343027bf8c3p-16;
  constexpr double kS1 = -0x1.555545995a603p-3, kS2 = 0x1.1107605230bc4p-7, kS3 = -0x1.994eb3774cf24p-13;
  const uint32_t top = (__float_as_uint(y) >> 20) & 0x7ffu;
  if (__builtin_expect(top >= 0x42fu, false))
  {
    sincosf(y, sp, cp);
    return;
  }
  double x = double(y);
  int n = 0;
  if (top >= 0x3f4u)
  {
    n = (int32_t(x * 0x1.45f306dc9c883p+23) + 0x800000) >> 24;
    x = __builtin_fma(-double(n), 0x1.921fb54442d18p+0, x);
  }
  const double x2 = x * x;
  const double xs = ((n ^ (n >> 1)) & 1) ? -x : x;               // sign[n & 3] = {1, -1, -1, 1}
  const double x3 = xs * x2;
  const double s = __builtin_fma(__builtin_fma(x2, kS3, kS2), x3 * x2, __builtin_fma(x3, kS1, xs));
  const double x4 = x2 * x2;
  double c = __builtin_fma(x4 * x2, __builtin_fma(x2, kC4, kC3), __builtin_fma(x4, kC2, __builtin_fma(x2, kC1, kC0)));
  c = (n & 2) ? -c : c;                                          // __sincosf_table[1]
  const bool tiny = top < 0x398u;
  const float so = tiny ? y : float(s), co = tiny ? 1.0f : float(c);
  *sp = (n & 1) ? co : so;
  *cp = (n & 1) ? so : co;
}

// a / m for a normal float a >= 0 and a small integer m (a loop counter) with its reciprocal rm = RN(1/m) known:
// q = a rm corrected once by the exact remainder -- the correctly rounded quotient (as div_nr) without v_rcp_f32
__device__ __forceinline__ float div_small(float a, float m, float rm)
{
  const float q = a * rm;
  return __builtin_fmaf(__builtin_fmaf(-m, q, a), rm, q);
}

// expf to ~0.5 ulp (correctly rounded but within ~2^-18 ulp of a midpoint): for the few places where the
// result is cancelled against a constant right after (Bagher's 1 - e^(c theta^k)), so the reference's
// correctly rounded glibc expf must be reproduced, not approximated
__device__ __forceinline__ float expf_acc(float x)
{
  if (__builtin_fabsf(x) < 1.49011612e-08f) return 1.0f;     // |x| < 2^-26: e^x rounds to 1
  return exp2_cr(double(x) * 1.4426950408889634074);
}

// float(exp(a)) for a double argument, to ~1.5 ulp of the float result: a log2(e) in double, split into an
// integer, a float head and a float tail, v_exp_f32 of the head, first-order fix-up by the tail, ldexp by the
// integer (a handful of f64 ops instead of a full double exp).  +-inf and overflow give inf / 0 like the
// reference; results in the subnormal range come from exp2_cr (one rounding).
__device__ __forceinline__ float exp_d2f(double a)
{
  const double t = a * 1.4426950408889634074;
  if (t < -126.0) return exp2_cr(t);
  const double n = __builtin_rint(t);
  const double f = t - n;
  const float fh = float(f);
  const float fl = float(f - double(fh));
  const float r0 = __builtin_amdgcn_exp2f(fh);
  const float r = __builtin_ldexpf(__builtin_fmaf(r0, fl * kLn2F, r0), int(__builtin_fmin(n, 400.0)));
  return (t > 200.0) ? __builtin_inff() : r;   // NaN propagates through r
}

// log2(x) for a normal or subnormal float x > 0 to ~2^-44 absolute (+ 2^-52 relative), in double:
// l0 = v_log_f32(x) (2 * 2^-24 relative), then one Newton step on 2^L = x with 2^-l0 from exp2_poly:
// q = x 2^-l0 = 1 + e (|e| < 2^-16), L = l0 + log2(1 + e) with e - e^2/2 + e^3/3.
__device__ __forceinline__ double log2_acc(float x)
{
  const bool sub = x < 1.17549435e-38f;
  const float xs = sub ? x * 4294967296.0f : x;                 // 2^32: v_log_f32 needs a normal input
  const float l0 = __builtin_amdgcn_logf(xs);
  const float n = __builtin_rintf(l0);
  const double p = exp2_poly(-double(l0 - n));                   // 2^-(l0 - n), l0 - n exact
  const double e = __builtin_fma(double(xs), __builtin_ldexp(p, -int(n)), -1.0);
  const double l1p = e * __builtin_fma(e, __builtin_fma(e, 1.0 / 3.0, -0.5), 1.0);
  return (double(l0) + l1p * 1.4426950408889634074) - (sub ? 32.0 : 0.0);
}

// x^y where the result is used as a factor (not amplified by an exponential or a cancellation): on the
// transcendental unit, exp2(y v_log_f32(x)), where |y log2 x| <= 8 -- relative error <= ln2 8 3.6e-7 / 2 + 1.4 ulp
// = 1.1e-6, results in [2^-8, 2^8] -- and powf_acc elsewhere.
__device__ __forceinline__ float powf_acc(float x, float y);
__device__ __forceinline__ float powf_fast(float x, float y)
{
  const float t0 = y * __builtin_amdgcn_logf(x);
  if (__builtin_fabsf(t0) <= 8.0f && x >= 1.17549435e-38f) return __builtin_amdgcn_exp2f(t0);
  return powf_acc(x, y);
}

// bbm::pow of two floats where the result is a model's value factor (Phong / Lafortune / Ashikhmin-Shirley lobes,
// the Phong NDF): glibc's powf to its last bit by default; -DBBM_HIP_POWF_FAST (A/B): the ~1e-6 powf_fast
__device__ __forceinline__ float powf_fast(float x, float y);
template<bool LDS> __device__ __forceinline__ float powf_glibc(float x, float y);
__device__ __forceinline__ float powf_ref(float x, float y)
{
#ifdef BBM_HIP_POWF_FAST
  return powf_fast(x, y);
#else
  return powf_glibc(x, y);
#endif
}

// x^y for x >= 0 (or NaN), y finite: the float nearest exp2(y log2 x) with y log2 x formed in double to ~2^-40,
// i.e. the correctly rounded power except within ~2^-18 ulp of a midpoint, over the whole float range
// (subnormal results included) -- what the reference's glibc powf / double pow rounded to float return.
// ~40 VALU (v_log_f32 + two short f64 polynomials) against 173 for the device library's powf.
__device__ __forceinline__ float powf_acc(float x, float y)
{
  float r = exp2_cr(double(y) * log2_acc(x));
  // pow(x, 0) = 1 (x NaN included); pow(0, y) = 0 / inf; x < 0 is outside the domain (NaN)
  r = (x == 0.0f) ? ((y > 0.0f) ? 0.0f : __builtin_inff()) : r;
  r = (x < 0.0f) ? __builtin_nanf("") : r;
  return (y == 0.0f) ? 1.0f : r;
}

// 1 / m for the loop counters of the series kernels (m <= 64), a uniform scalar load instead of a division
__device__ __forceinline__ double inv_small(int m)
{
  static constexpr double kInv[65] = {
      0.0,      1.0 / 1,  1.0 / 2,  1.0 / 3,  1.0 / 4,  1.0 / 5,  1.0 / 6,  1.0 / 7,  1.0 / 8,  1.0 / 9,  1.0 / 10,
      1.0 / 11, 1.0 / 12, 1.0 / 13, 1.0 / 14, 1.0 / 15, 1.0 / 16, 1.0 / 17, 1.0 / 18, 1.0 / 19, 1.0 / 20, 1.0 / 21,
      1.0 / 22, 1.0 / 23, 1.0 / 24, 1.0 / 25, 1.0 / 26, 1.0 / 27, 1.0 / 28, 1.0 / 29, 1.0 / 30, 1.0 / 31, 1.0 / 32,
      1.0 / 33, 1.0 / 34, 1.0 / 35, 1.0 / 36, 1.0 / 37, 1.0 / 38, 1.0 / 39, 1.0 / 40, 1.0 / 41, 1.0 / 42, 1.0 / 43,
      1.0 / 44, 1.0 / 45, 1.0 / 46, 1.0 / 47, 1.0 / 48, 1.0 / 49, 1.0 / 50, 1.0 / 51, 1.0 / 52, 1.0 / 53, 1.0 / 54,
      1.0 / 55, 1.0 / 56, 1.0 / 57, 1.0 / 58, 1.0 / 59, 1.0 / 60, 1.0 / 61, 1.0 / 62, 1.0 / 63, 1.0 / 64};
  return kInv[m];
}

__device__ __forceinline__ double ddiv_nr(double n, double d)
{
  double r = __builtin_amdgcn_rcp(d);
  double e = __builtin_fma(-d, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-d, r, 1.0);
  r = __builtin_fma(r, e, r);
  const double q = n * r;
  const double rem = __builtin_fma(-d, q, n);
  const double q1 = __builtin_fma(rem, r, q);
  return __builtin_isfinite(q1) ? q1 : n * __builtin_amdgcn_rcp(d);
}

// float(1.0 + sqrt(x)) for a double x >= 1, every step IEEE double as in the reference (ggx.h:180-185's
// 1 + sqrt(1 + alpha^2 tan^2) stored into a float `Value denom`), without the ~11 f64 VALU of the IEEE double
// square root: a float rsq seed (|rel. error| <= 2^-22.2 with the rounding of x to float) and one double Newton step
// give y = sqrt(x) within 2^-43.4 y, so 1 + y lands within ~800 double ulps of the reference's double.  Its float
// rounding can only differ where that double is that close to a float rounding midpoint (the low 29 bits near
// 2^28): those lanes (~1 in 2^16), and any x outside [1, 2^100], run the exact sequence instead -- the float is
// always the reference's.  Pinned against IEEE double on the host by tests/test_gpu_libm.py.
__device__ __forceinline__ float f_one_plus_sqrt(double x)
{
  const float xf = float(x);
  const float g = __builtin_amdgcn_rsqf(xf);
  const double s = double(xf * g);
  const double y = __builtin_fma(__builtin_fma(-s, s, x), double(0.5f * g), s);
  const double z = 1.0 + y;
  const uint32_t lo = uint32_t(__builtin_bit_cast(uint64_t, z)) & 0x1fffffffu;
  float res = float(z);
  if (__builtin_expect(((lo - 0x0ffff000u) < 0x2000u) || !(x >= 1.0 && x <= 0x1p100), false))
    res = float(1.0 + __builtin_sqrt(x));
  return res;
}

// float(n / d) for double n, d -- the reference's double-promoted quotients that are immediately
// stored into a float (e.g. maskingshadowing/vgroove.h:41-44, ndf/beckmann.h:196).  An f32
// reciprocal estimate (rel. error ~2^-22) plus one f64 remainder correction gives the quotient to
// ~2^-45, so the float rounding agrees with the reference except within ~2^-21 ulp of a midpoint;
// two f64 FMAs instead of a full f64 division.
__device__ __forceinline__ float f_div_d(double n, double d)
{
  const float r = __builtin_amdgcn_rcpf(float(d));
  const double q0 = double(float(n) * r);
  const double rem = __builtin_fma(-d, q0, n);
  const double q = __builtin_fma(rem, double(r), q0);
  return __builtin_isfinite(q) ? float(q) : float(n) * r;   // d = 0 / inf, n = inf: IEEE result
}

// ---------------------------------------------------------------- compensated f32 (double-float)
//
// Where the reference promotes to double only to form a product of two floats and divide it
// (e.g. vgroove's `2.0 * z_m * z_in / dot`), the exact product is carried as an unevaluated f32
// pair (hi + lo, Dekker/FMA two-product) and the quotient is corrected with the low part: the
// result is the float nearest the exact quotient (to ~2^-45), which is what rounding the
// reference's double quotient to float gives -- all in full-rate f32 instead of half-rate f64.
__device__ __forceinline__ void two_prod(float a, float b, float& hi, float& lo)
{
  hi = a * b;
  lo = __builtin_fmaf(a, b, -hi);
}

// float nearest (nh + nl) / (dh + dl), |nl| <= ulp(nh)/2, |dl| <= ulp(dh)/2
__device__ __forceinline__ float div_ff(float nh, float nl, float dh, float dl)
{
  const float r = __builtin_amdgcn_rcpf(dh);
  float q = nh * r;
  q = __builtin_fmaf(__builtin_fmaf(-dh, q, nh), r, q);           // ~correctly rounded nh / dh
  const float rem = __builtin_fmaf(-dh, q, nh) + __builtin_fmaf(-q, dl, nl);
  const float q1 = __builtin_fmaf(rem, r, q);
#ifdef BBM_HIP_DIV_SUB
  // subnormal numerator or quotient (see div_nr): the pair quotient in double (both pair sums are exact doubles),
  // rounded once to float, on a wave-uniform branch
  const bool fast = (__builtin_isnormal(q1) && __builtin_isnormal(nh)) || (nh == 0.0f && nl == 0.0f);
  float res = q1;
  if (__builtin_amdgcn_ballot_w64(!fast) != 0)
  {
    const float s = float((double(nh) + double(nl)) / (double(dh) + double(dl)));
    res = fast ? q1 : s;
  }
  return res;
#else
  return __builtin_isnormal(q1) ? q1 : nh * r;     // subnormal / special results: see div_nr
#endif
}

// nh / (dh + dl) as div_sub: the f32 seed and one remainder step in double (dh + dl exact in double), rounded
// once -- for a subnormal numerator too (the Cook-normalised eval of a far-tail halfway vector); EXACT = false is
// div_ff
template<bool EXACT>
__device__ __forceinline__ float div_ff_sub(float nh, float dh, float dl)
{
  if constexpr (EXACT)
  {
    const float r = __builtin_amdgcn_rcpf(dh);
    const double q0 = double(nh * r);
    const double dd = double(dh) + double(dl);
    return float(__builtin_fma(__builtin_fma(-dd, q0, double(nh)), double(r), q0));
  }
  else return div_ff(nh, 0.0f, dh, dl);
}

// horizontal.h:78-82: dot = inner_product(a, b, T(0)) -> ((0 + a0 b0) + a1 b1) + a2 b2
__device__ __forceinline__ float dot3(v3 a, v3 b) { return ((0.0f + a.x * b.x) + a.y * b.y) + a.z * b.z; }
__device__ __forceinline__ float sqnorm2(float a, float b) { return (0.0f + a * a) + b * b; }

// horizontal.h:96-100 normalize = t * rsqrt(|t|^2); math.h:109-112 rsqrt = rcp(sqrt) = 1 / sqrt
__device__ __forceinline__ v3 normalize3(v3 t)
{
  const float r = div_nr_n(1.0f, sqrt_nr(dot3(t, t)));   // |t|^2 of a sum of two unit vectors: 1 / |t| normal
  return mk3(t.x * r, t.y * r, t.z * r);
}

// core/vec_transform.h:76-80
__device__ __forceinline__ v3 halfway(v3 a, v3 b) { return normalize3(mk3(a.x + b.x, a.y + b.y, a.z + b.z)); }

// core/vec_transform.h:58-64 cross
__device__ __forceinline__ v3 cross3(v3 a, v3 b)
{
  return mk3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}

// math.h:129 safe_sqrt = sqrt(std::max(a, T(0))): std::max keeps a NaN argument (a < 0 is false)
__device__ __forceinline__ float safe_sqrtf(float a) { return sqrt_nr((a < 0.0f) ? 0.0f : a); }
__device__ __forceinline__ double safe_sqrt(double a) { return sqrt((a < 0.0) ? 0.0 : a); }

// core/spherical.h:79-80 sinTheta2 = bbm::max(1 - z*z, 0) -> fmaxf (result_t<float,int> = float)
__device__ __forceinline__ float sin_theta2(v3 v) { return fmaxf(1 - v.z * v.z, 0.0f); }
// spherical.h:179-180 tanTheta = sinTheta / cosTheta; :185-186 tanTheta2 = sinTheta2 / cosTheta2
__device__ __forceinline__ float tan_theta(v3 v) { return div_nr(sqrt_nr(sin_theta2(v)), v.z); }
__device__ __forceinline__ float tan_theta2(v3 v) { return div_nr(sin_theta2(v), v.z * v.z); }

// std::clamp(a, T(lo), T(hi)) (backbone/native/include/backbone/math.h:106-107)
__device__ __forceinline__ float clampf(float a, float lo, float hi) { return (a < lo) ? lo : ((hi < a) ? hi : a); }

// core/spherical.h:155-160 cossinPhi: (1, 0) at the pole, else clamp(xy / sinTheta, -1, 1)
__device__ __forceinline__ void cossin_phi(v3 v, float& c, float& s)
{
  const float sT = sqrtf(sin_theta2(v));
  const float rsT = div_nr(1.0f, sT);
  if (fabsf(sT) < kEpsF) { c = 1.0f; s = 0.0f; return; }
  c = clampf(v.x * rsT, -1.0f, 1.0f);
  s = clampf(v.y * rsT, -1.0f, 1.0f);
}

// backbone/native/include/backbone/math.h:115-126: Giles' single-precision erfinv polynomial.
// For T = float the native backbone computes w = -log((1.0 - a)(1.0 + a)) in double and stores it
// as float, then evaluates the Horner polynomial (util/poly.h:34-38) in double: the result is double,
// and its callers (ndf/beckmann.h:92-110) store it into a float.  erfinv_f returns that float with the
// polynomial -- Giles' coefficients are floats, fitted for single precision -- evaluated by f32 FMAs:
// within ~2 ulp of the double evaluation's rounding (the f32 w already differs by ~2 ulp) at a quarter of
// the issue cycles (9 f32 FMAs against 18 f64 mul/add).  Sampled directions move by ~1e-7 relative.
// w = float(-log((1 - a)(1 + a))): the reference's log is f64; here -log1p(-a^2) in f32 (a^2 as an exact
// two-product, log1p by the u = 1 + x correction on the device logf, ~2 ulp) -- ~20 VALU instead of ~100 f64
// instructions; the five erfinv calls of a Beckmann sample were its whole cost.
#ifdef BBM_HIP_ERFINV_V1
__device__ __forceinline__ float erfinv_w(float a)
{
  const float a2 = a * a;
  const float a2e = __builtin_fmaf(a, a, -a2);          // a^2 = a2 + a2e exactly
  const float u = 1.0f - a2;                            // log1p(-a2 - a2e) = log1p(-a2) - a2e / (1 - a2)
  const float l1p = (u == 1.0f) ? -a2 : logf(u) * div_nr(-a2, u - 1.0f);
  return (u == 0.0f) ? __builtin_inff() : -(l1p - div_nr(a2e, u));   // a = +-1: -log(0) = inf
}
#else
// The same w on the transcendental unit: u = 1 - a^2 is a normal float in [2^-24, 1] (or 0, or 1), so v_log_f32
// (2 2^-24 relative in log2 u, x -> 1 included) times ln 2 replaces the library logf, and the two correction
// factors -a2 / (u - 1) (= 1 + O(2^-24)) and a2e / u (a rounding residue) need no Newton step: w moves by <= 2 ulp
// against the library form, inside the ~2-ulp spread the f32 w already has against the reference's double w.
__device__ __forceinline__ float erfinv_w(float a)
{
  const float a2 = a * a;
  const float a2e = __builtin_fmaf(a, a, -a2);          // a^2 = a2 + a2e exactly
  const float u = 1.0f - a2;
  const float lu = (__builtin_amdgcn_logf(u) * kLn2F) * (-a2 * __builtin_amdgcn_rcpf(u - 1.0f));
  const float l1p = (u == 1.0f) ? -a2 : lu;
  return (u == 0.0f) ? __builtin_inff() : -(l1p - a2e * __builtin_amdgcn_rcpf(u));   // a = +-1: -log(0) = inf
}
#endif
__device__ __forceinline__ float erfinv_f(float a)
{
  const float w = erfinv_w(a);
  float p;
#ifdef BBM_HIP_ERFINV_V1
  if (w < 5)
#endif
  {
    const float x = w - 2.5f;
    p = 2.81022636e-08f;
    p = __builtin_fmaf(p, x, 3.43273939e-07f); p = __builtin_fmaf(p, x, -3.5233877e-06f);
    p = __builtin_fmaf(p, x, -4.39150654e-06f); p = __builtin_fmaf(p, x, 0.00021858087f);
    p = __builtin_fmaf(p, x, -0.00125372503f); p = __builtin_fmaf(p, x, -0.00417768164f);
    p = __builtin_fmaf(p, x, 0.246640727f); p = __builtin_fmaf(p, x, 1.50140941f);
  }
#ifdef BBM_HIP_ERFINV_V1
  else
#else
  // the tail (w >= 5: |a| > 0.9966) only where some lane of the wave needs it (a wave-uniform branch; the sampler
  // reaches it at grazing stretched views and for xi near 0 or 1): the central polynomial is not evaluated twice
  if (__builtin_amdgcn_ballot_w64(!(w < 5)) != 0)
#endif
  {
    const float x = sqrtf(w) - 3.0f;
    float q = -0.000200214257f;
    q = __builtin_fmaf(q, x, 0.000100950558f); q = __builtin_fmaf(q, x, 0.00134934322f);
    q = __builtin_fmaf(q, x, -0.00367342844f); q = __builtin_fmaf(q, x, 0.00573950773f);
    q = __builtin_fmaf(q, x, -0.0076224613f); q = __builtin_fmaf(q, x, 0.00943887047f);
    q = __builtin_fmaf(q, x, 1.00167406f); q = __builtin_fmaf(q, x, 2.83297682f);
#ifdef BBM_HIP_ERFINV_V1
    p = q;
#else
    p = (w < 5) ? p : q;
#endif
  }
  return p * a;
}
__device__ __forceinline__ double erfinv_d(float a)
{
  const float w = erfinv_w(a);
  if (w < 5)
  {
    const double x = w - 2.5;
    double p = 2.81022636e-08;
    p = p * x + 3.43273939e-07; p = p * x + -3.5233877e-06; p = p * x + -4.39150654e-06;
    p = p * x + 0.00021858087; p = p * x + -0.00125372503; p = p * x + -0.00417768164;
    p = p * x + 0.246640727; p = p * x + 1.50140941;
    return p * a;
  }
  const double x = sqrtf(w) - 3.0;
  double p = -0.000200214257;
  p = p * x + 0.000100950558; p = p * x + 0.00134934322; p = p * x + -0.00367342844;
  p = p * x + 0.00573950773; p = p * x + -0.0076224613; p = p * x + 0.00943887047;
  p = p * x + 1.00167406; p = p * x + 2.83297682;
  return p * a;
}

// bbm::pow(float, int) -> std::pow(float, float); for the exponent 2 used on this path the
// correctly rounded square is what glibc's powf returns.
__device__ __forceinline__ float pow2f(float x) { return x * x; }

// expf rounded from the f64 exponential: the float nearest e^x except within ~2^-29 ulp of a
// midpoint, i.e. what the reference's (glibc, ~0.5 ulp) expf returns.  Used where the result is
// cancelled against a constant right after (Low smooth sampling's E - 2 as xi0 -> 0), so that a
// 1-ulp expf difference is not amplified; the eval kernels keep the full-rate f32 expf.
__device__ __forceinline__ float expf_cr(float x) { return float(exp(double(x))); }
__device__ __forceinline__ float logf_cr(float x) { return float(log(double(x))); }
// x^y for x >= 0, y > 0, rounded from exp(y log x) in f64: the relative error of the f64 result
// (~|y log x| 2^-52) is far below float resolution, so this is the correctly rounded powf -- what glibc's
// powf returns -- except within ~2^-25 ulp of a midpoint; a double log + exp instead of the library powf's
// extended-precision log and special-case handling.  Only for the domain stated (Bagher's G1: x = theta -
// theta0 > 0, y = k > 0).
__device__ __forceinline__ float powf_xlog(float x, float y)
{
  return (x > 0.0f) ? float(exp(double(y) * log(double(x)))) : 0.0f;
}
// glibc powf (what std::pow(float, float) calls) is computed in double and rounded once; so is this
__device__ __forceinline__ float powf_cr(float x, float y) { return float(pow(double(x), double(y))); }

namespace f64 {

// ---------------------------------------------------------------- exp / log / pow in double
//
// The reference's doubleRGB exp / log / pow are glibc's (correctly rounded, or within ~0.52 ulp).  ocml's f64 pow
// carries its logarithm in double-double and is the bulk of the pow-heavy models' VALU per pair; these
// restatements stay within a few ulp of glibc at about half the cost (tools/f64math_probe.hip measures them
// against the host libm), far inside the doubleRGB bar (1e-10 relative, tests/test_gpu_f64.py).
//
// 2^f - 1 for |f| <= 1/2: f (c1 + f (c2 + ... c13)), the degree-13 Taylor polynomial of e^(f ln2) - 1
// (truncation <= 1e-17 relative); no 1 is added, so 2^f - 1 keeps its relative precision as f -> 0
__device__ __forceinline__ double exp2m1_poly(double f)
{
  double p = 0x1.816193166d0f9p-40;
  p = __builtin_fma(p, f, 0x1.c3bd650fc2986p-36);
  p = __builtin_fma(p, f, 0x1.e8cac7351bb25p-32);
  p = __builtin_fma(p, f, 0x1.e4cf5158b8ecap-28);
  p = __builtin_fma(p, f, 0x1.b5253d395e7c4p-24);
  p = __builtin_fma(p, f, 0x1.62c0223a5c824p-20);
  p = __builtin_fma(p, f, 0x1.ffcbfc588b0c7p-17);
  p = __builtin_fma(p, f, 0x1.430912f86c787p-13);
  p = __builtin_fma(p, f, 0x1.5d87fe78a6731p-10);
  p = __builtin_fma(p, f, 0x1.3b2ab6fba4e77p-7);
  p = __builtin_fma(p, f, 0x1.c6b08d704a0c0p-5);
  p = __builtin_fma(p, f, 0x1.ebfbdff82c58fp-3);
  p = __builtin_fma(p, f, 0x1.62e42fefa39efp-1);
  return p * f;
}

// 2^t over the whole double range: n = rint(t), 2^(t - n) (t - n exact) scaled by 2^n in one rounding, subnormal
// results included; overflow to inf, 0 far below 2^-1074, NaN propagates
__device__ __forceinline__ double exp2_d(double t)
{
  const double n = __builtin_rint(t);
  const double r = __builtin_ldexp(1.0 + exp2m1_poly(t - n), int(__builtin_fmin(__builtin_fmax(n, -1100.0), 1100.0)));
  return (t < -1100.0) ? 0.0 : ((t > 1100.0) ? __builtin_inf() : r);
}

// e^a: n = rint(a / ln2), r = a - n ln2 in two FMAs (Cody-Waite; n ln2_hi exact), e^r - 1 by its degree-13
// Taylor polynomial on |r| <= 0.35 (truncation 1e-17): ~1 ulp over the whole range, subnormal results included
__device__ __forceinline__ double exp_d(double a)
{
#ifdef BBM_HIP_F64_OCML
  return exp(a);   // A/B: the device library (tools/build_variant.sh)
#endif
  const double n = __builtin_rint(a * 0x1.71547652b82fep0);
  double r = __builtin_fma(-n, 0x1.62e42fefa3800p-1, a);
  r = __builtin_fma(-n, 0x1.ef35793c76730p-45, r);
  double p = 1.0 / 6227020800.0;                         // 1 / 13!
  p = __builtin_fma(p, r, 1.0 / 479001600.0);
  p = __builtin_fma(p, r, 1.0 / 39916800.0);
  p = __builtin_fma(p, r, 1.0 / 3628800.0);
  p = __builtin_fma(p, r, 1.0 / 362880.0);
  p = __builtin_fma(p, r, 1.0 / 40320.0);
  p = __builtin_fma(p, r, 1.0 / 5040.0);
  p = __builtin_fma(p, r, 1.0 / 720.0);
  p = __builtin_fma(p, r, 1.0 / 120.0);
  p = __builtin_fma(p, r, 1.0 / 24.0);
  p = __builtin_fma(p, r, 1.0 / 6.0);
  p = __builtin_fma(p, r, 0.5);
  p = __builtin_fma(p, r, 1.0);
  const double v = __builtin_ldexp(__builtin_fma(p, r, 1.0), int(__builtin_fmin(__builtin_fmax(n, -1100.0), 1100.0)));
  return (a < -746.0) ? 0.0 : ((a > 710.0) ? __builtin_inf() : v);
}

// log2(x) for finite x > 0 (subnormals included) to ~1 ulp + 2^-53 absolute: x = 2^k m with m in [1/sqrt2, sqrt2),
// l0 = v_log_f32(m) (|l0| <= 1/2, 2^-23 relative), one Newton step on 2^L = m: e = m 2^-l0 - 1
// = (m - 1)(1 + q) + q with q = 2^-l0 - 1 (|e| < 2^-21; m - 1 exact), L = l0 + log2(1 + e) by three terms.
// Near x = 1 (k = 0) the result keeps its relative precision.
__device__ __forceinline__ double log2_d(double x)
{
  double m = __builtin_amdgcn_frexp_mant(x);             // [1/2, 1)
  int k = __builtin_amdgcn_frexp_exp(x);
  const bool lo = m < 0.70710678118654752;
  m = lo ? m + m : m;
  k = lo ? k - 1 : k;
  const float l0 = __builtin_amdgcn_logf(float(m));
  const double q = exp2m1_poly(-double(l0));
  const double e = __builtin_fma(m - 1.0, 1.0 + q, q);
  const double l1p = e * __builtin_fma(e, __builtin_fma(e, 1.0 / 3.0, -0.5), 1.0);
  return double(k) + __builtin_fma(l1p, 0x1.71547652b82fep0, double(l0));
}

// the device library's f64 exp: measured faster than exp_d inside the He family's prelude (He 1.50 -> 1.47,
// HeHolzschuch 0.80 -> 0.75 ms per 10 M pairs; exp_d is faster in the microfacet models: CookTorrance 0.158 ->
// 0.150), where the kernel runs at its 256-VGPR cap
__device__ __forceinline__ double exp_lib(double a) { return exp(a); }

// glibc's log restated on log2_d (x < 0 -> NaN; x = 0 -> -inf; inf -> inf; NaN -> NaN)
__device__ __forceinline__ double log_d(double x)
{
#ifdef BBM_HIP_F64_OCML
  return log(x);
#endif
  const double v = log2_d(x) * 0x1.62e42fefa39efp-1;
  return (x == 0.0) ? -__builtin_inf() : ((x < 0.0) ? __builtin_nan("") : ((x == __builtin_inf()) ? x : v));
}
// x^y for x >= 0 (or NaN) and finite y: 2^(y log2 x), y log2 x to ~2^-52 relative + |y| 2^-53 absolute (~1e-13
// relative on every result above the subnormal range); pow(x, 0) = pow(1, y) = 1, pow(0, y) = 0 / inf,
// pow(inf, y) = inf / 0, x < 0 -> NaN (never reached: the reference's bases here are >= 0)
__device__ __forceinline__ double pow_d(double x, double y)
{
#ifdef BBM_HIP_F64_OCML
  return pow(x, y);
#endif
  double r = exp2_d(y * log2_d(x));
  const bool big = x == __builtin_inf();
  r = (x == 0.0 || big) ? (((y > 0.0) == big) ? __builtin_inf() : 0.0) : r;
  r = (x < 0.0) ? __builtin_nan("") : r;
  return (y == 0.0 || x == 1.0) ? 1.0 : r;
}
}  // namespace f64

}  // namespace bbmhip
