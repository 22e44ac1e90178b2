/* oracle/ref_ops.hpp -- TEST INFRASTRUCTURE ONLY: shared by the reference shim's translation units
 * (ref_harness.cpp: single models; ref_fit.cpp: aggregates, linearizers, losses, compass).
 * Includes the reference headers where they lie and wraps one model type M in the per-model
 * operations the ctypes shim exports (see ref_harness.cpp for the conventions).
 */
#pragma once
#include "bbm/bbm_core.h"
#include "bbm/bsdf_enumerate.h"
#include "bsdfmodel/scaledmodel.h"
#include "bsdfmodel/microfacet.h"
#include "bsdfmodel/aggregatemodel.h"
#include "bsdfmodel/lambertian.h"
#include "bsdfmodel/orennayar.h"
#include "bsdfmodel/cooktorrance.h"
#include "bsdfmodel/cooktorranceheitz.h"
#include "bsdfmodel/cooktorrancewalter.h"
#include "bsdfmodel/ggx.h"
#include "bsdfmodel/ggxheitz.h"
#include "bsdfmodel/phongwalter.h"
#include "bsdfmodel/ribardiere.h"
#include "bsdfmodel/bagher.h"
#include "bsdfmodel/lowmicrofacet.h"
#include "bsdfmodel/ward.h"
#include "bsdfmodel/wardduer.h"
#include "bsdfmodel/wardduergeislermoroder.h"
#include "bsdfmodel/phong.h"
#include "bsdfmodel/lafortune.h"
#include "bsdfmodel/ashikhminshirley.h"
#include "bsdfmodel/ashikhminshirleyfull.h"
#include "bsdfmodel/lowsmooth.h"
#include "bsdfmodel/he.h"
#include "bsdfmodel/low.h"
// ngan.h:169 concept-checks NganHe, whose ndf_sampler default NAME fails CTAD on g++ 11
// (include/ndf/sampler.h:34).  The check is a compile-time static_assert only; it is switched
// off for this one header so the six other Ngan models (which do compile) can be instantiated.
#pragma push_macro("BBM_CHECK_CONCEPT")
#undef BBM_CHECK_CONCEPT
#define BBM_CHECK_CONCEPT(...) static_assert(true, "")
#include "bsdfmodel/ngan.h"
#pragma pop_macro("BBM_CHECK_CONCEPT")
#include "ndf/epd.h"
#include "maskingshadowing/vanginneken.h"
#include "ref_he.hpp"
#include "bbm/bsdf_ptr.h"
#include "bbm/aggregatebsdf.h"

#include <cstdint>
#include <cstring>
#include <sstream>
#include <string>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace bbmref {


constexpr bbm::bsdf_attr kAllParams = bbm::bsdf_attr(0x1F);   // All | Dependent

// EPD: bsdfmodel/holzschuchpacanowski.h:34-42 composes it from ndf::epd, maskingshadowing::vanginneken,
// fresnel::complex and Walter's normalisation.  That header also #includes two precomputed blobs that
// are missing from the mount (.MISSING_LARGE_BLOBS: convolution.h, normalization.h) and that the EPD
// alias never uses, so the identical composition is written out here from the headers that exist
// (ndf/epd.h with its G1 and normalisation tables, maskingshadowing/vanginneken.h).
template<typename CONF>
using epd = bbm::microfacet<bbm::ndf::epd<CONF>, bbm::maskingshadowing::vanginneken<CONF>, bbm::fresnel::complex<CONF>,
                            bbm::microfacet_n::Walter, "EPD">;

// aggregatemodel_base<NAME, X...> and the ones with an aggregate child: the reference cannot reflect a nested
// aggregate as a whole (util/reflection.h:247 needs a reflection_base aggregatemodel_base does not declare), so its
// parameter vector is its children's, in base-class order -- the layout bbm_hip's composed aggregates use
template<typename M> struct is_agg : std::false_type {};
template<auto NM, typename... X>
struct is_agg<bbm::aggregatemodel_base<NM, X...>> : std::true_type { using kids = std::tuple<X...>; };
template<typename M> struct nested_agg : std::false_type {};
template<auto NM, typename... X>
struct nested_agg<bbm::aggregatemodel_base<NM, X...>> : std::bool_constant<(is_agg<X>::value || ...)> {};

template<typename M>
std::vector<typename M::Value*> flat_refs(M& m)
{
  std::vector<typename M::Value*> r;
  if constexpr (nested_agg<M>::value)
    [&]<typename... X>(const std::tuple<X...>*) {
      ([&] { auto c = flat_refs(static_cast<X&>(m)); r.insert(r.end(), c.begin(), c.end()); }(), ...);
    }(static_cast<const typename is_agg<M>::kids*>(nullptr));
  else
  {
    auto pv = bbm::parameter_values(m, kAllParams);
    for(size_t i = 0; i < pv.size(); ++i) { typename M::Value& v = pv[i]; r.push_back(&v); }
  }
  return r;
}

template<typename M>
std::vector<float> flat_bounds(const M& m, bool upper)
{
  std::vector<float> r;
  if constexpr (nested_agg<M>::value)
    [&]<typename... X>(const std::tuple<X...>*) {
      ([&] { auto c = flat_bounds(static_cast<const X&>(m), upper); r.insert(r.end(), c.begin(), c.end()); }(), ...);
    }(static_cast<const typename is_agg<M>::kids*>(nullptr));
  else
  {
    auto b = upper ? bbm::parameter_upper_bound(m, kAllParams) : bbm::parameter_lower_bound(m, kAllParams);
    for(auto& v : b) r.push_back(float(v));
  }
  return r;
}

template<typename M>
struct ops
{
  using Value = typename M::Value;
  using Vec3d = typename M::Vec3d;
  using Vec2d = typename M::Vec2d;

  static std::vector<float> defaults()
  {
    M m;
    std::vector<float> r;
    for(Value* v : flat_refs(m)) r.push_back(float(*v));
    return r;
  }

  static M make(const float* p, int np)
  {
    M m;
    auto pv = flat_refs(m);
    for(size_t i = 0; i < pv.size() && int(i) < np; ++i) *pv[i] = Value(p[i]);
    return m;
  }

  static std::vector<float> bounds(bool upper)
  {
    M m;
    return flat_bounds(m, upper);
  }

  // bbm::fromString<M> (include/bbm/bsdf_string_convert.h, aggregatemodel.h:193-218) -> the parameter vector
  static int from_string(const char* str, float* out, int cap)
  {
    try
    {
      M m = bbm::fromString<M>(std::string(str));
      int k = 0;
      for(Value* v : flat_refs(m)) { if(k < cap) out[k] = float(*v); ++k; }
      return k;
    }
    catch(const std::exception&) { return -1; }
  }

  static std::string to_string(const float* p, int np)
  {
    M m = make(p, np);
    std::ostringstream s;
    s << bbm::toString(m);
    return s.str();
  }

  // mode bit 1 = eval, bit 2 = pdf
  template<typename OUT, typename IN = float>
  static void evalpdf(const float* p, int np, size_t n,
                      const IN* ix, const IN* iy, const IN* iz,
                      const IN* ox, const IN* oy, const IN* oz,
                      uint32_t component, uint32_t unit, int mode,
                      OUT* r, OUT* g, OUT* b, OUT* pdf, int nthreads)
  {
    const M m0 = make(p, np);
    const auto comp = bbm::bsdf_flag(component);
    const auto u = bbm::unit_t(unit);
    // one model copy per thread: data-driven samplers (he_sampled) cache their CDFs in a mutable map
#ifdef _OPENMP
    #pragma omp parallel num_threads(nthreads > 0 ? nthreads : 1)
#endif
    {
    const M m = m0;
#ifdef _OPENMP
    #pragma omp for schedule(static)
#endif
    for(size_t i = 0; i < n; ++i)
    {
      Vec3d in(Value(ix[i]), Value(iy[i]), Value(iz[i]));
      Vec3d out(Value(ox[i]), Value(oy[i]), Value(oz[i]));
      if(mode & 1)
      {
        auto e = m.eval(in, out, comp, u);
        r[i] = OUT(e[0]); g[i] = OUT(e[1]); b[i] = OUT(e[2]);
      }
      if(mode & 2) pdf[i] = OUT(m.pdf(in, out, comp, u));
    }
    }
  }

  template<typename OUT>
  static void sample(const float* p, int np, size_t n,
                     const float* ox, const float* oy, const float* oz,
                     const float* xi0, const float* xi1,
                     uint32_t component, uint32_t unit,
                     OUT* dx, OUT* dy, OUT* dz, OUT* pdf, uint32_t* flag, int nthreads)
  {
    const M m0 = make(p, np);
    const auto comp = bbm::bsdf_flag(component);
    const auto u = bbm::unit_t(unit);
#ifdef _OPENMP
    #pragma omp parallel num_threads(nthreads > 0 ? nthreads : 1)
#endif
    {
    const M m = m0;
#ifdef _OPENMP
    #pragma omp for schedule(static)
#endif
    for(size_t i = 0; i < n; ++i)
    {
      Vec3d out(Value(ox[i]), Value(oy[i]), Value(oz[i]));
      Vec2d xi(Value(xi0[i]), Value(xi1[i]));
      auto s = m.sample(out, xi, comp, u);
      dx[i] = OUT(s.direction[0]); dy[i] = OUT(s.direction[1]); dz[i] = OUT(s.direction[2]);
      pdf[i] = OUT(s.pdf);
      flag[i] = uint32_t(s.flag);
    }
    }
  }

  // bbm::make_bsdf_ptr of the model at these parameters (bsdf_ptr.h:218-224): a leaf of the runtime aggregate
  // fromString<bsdf_ptr> builds (bsdf_string_convert.h:52-82); `out` is a bbm::bsdf_ptr<Config>*
  static void make_ptr(const float* p, int np, void* out)
  {
    *static_cast<bbm::bsdf_ptr<bbm::get_config<M>>*>(out) = bbm::make_bsdf_ptr(make(p, np));
  }

  template<typename OUT>
  static void reflectance(const float* p, int np, size_t n, const float* ox, const float* oy, const float* oz,
                          uint32_t component, uint32_t unit, OUT* r, OUT* g, OUT* b)
  {
    const M m = make(p, np);
    for(size_t i = 0; i < n; ++i)
    {
      Vec3d out(Value(ox[i]), Value(oy[i]), Value(oz[i]));
      auto e = m.reflectance(out, bbm::bsdf_flag(component), bbm::unit_t(unit));
      r[i] = OUT(e[0]); g[i] = OUT(e[1]); b[i] = OUT(e[2]);
    }
  }
};

struct entry
{
  const char* name;
  std::vector<float> (*defaults)();
  std::vector<float> (*bounds)(bool);
  std::string (*to_string)(const float*, int);
  void (*evalpdf_f)(const float*, int, size_t, const float*, const float*, const float*, const float*, const float*, const float*, uint32_t, uint32_t, int, float*, float*, float*, float*, int);
  void (*evalpdf_d)(const float*, int, size_t, const float*, const float*, const float*, const float*, const float*, const float*, uint32_t, uint32_t, int, double*, double*, double*, double*, int);
  void (*sample_f)(const float*, int, size_t, const float*, const float*, const float*, const float*, const float*, uint32_t, uint32_t, float*, float*, float*, float*, uint32_t*, int);
  void (*reflectance_f)(const float*, int, size_t, const float*, const float*, const float*, uint32_t, uint32_t, float*, float*, float*);
  int (*from_string)(const char*, float*, int) = nullptr;
  void (*reflectance_d)(const float*, int, size_t, const float*, const float*, const float*, uint32_t, uint32_t, double*, double*, double*) = nullptr;
  void (*sample_d)(const float*, int, size_t, const float*, const float*, const float*, const float*, const float*, uint32_t, uint32_t, double*, double*, double*, double*, uint32_t*, int) = nullptr;
  // doubleRGB eval / pdf at double directions (the per-lane proofs of the f64 kernels perturb directions in double)
  void (*evalpdf_dd)(const float*, int, size_t, const double*, const double*, const double*, const double*, const double*, const double*, uint32_t, uint32_t, int, double*, double*, double*, double*, int) = nullptr;
  // bsdf_ptr<floatRGB> / bsdf_ptr<doubleRGB> of the model (ref_runtime.cpp: runtime aggregates)
  void (*ptr_f)(const float*, int, void*) = nullptr;
  void (*ptr_d)(const float*, int, void*) = nullptr;
};

#define BBMREF_ENTRY(MODEL) BBMREF_ENTRY_NS(bbm, MODEL)
#define BBMREF_ENTRY_NS(NS, MODEL) \
  entry{ NS::MODEL<bbm::floatRGB>::name.value, \
         &ops<NS::MODEL<bbm::floatRGB>>::defaults, \
         &ops<NS::MODEL<bbm::floatRGB>>::bounds, \
         &ops<NS::MODEL<bbm::floatRGB>>::to_string, \
         &ops<NS::MODEL<bbm::floatRGB>>::template evalpdf<float>, \
         &ops<NS::MODEL<bbm::doubleRGB>>::template evalpdf<double>, \
         &ops<NS::MODEL<bbm::floatRGB>>::template sample<float>, \
         &ops<NS::MODEL<bbm::floatRGB>>::template reflectance<float>, \
         &ops<NS::MODEL<bbm::floatRGB>>::from_string, \
         &ops<NS::MODEL<bbm::doubleRGB>>::template reflectance<double>, \
         &ops<NS::MODEL<bbm::doubleRGB>>::template sample<double>, \
         &ops<NS::MODEL<bbm::doubleRGB>>::template evalpdf<double, double>, \
         &ops<NS::MODEL<bbm::floatRGB>>::make_ptr, \
         &ops<NS::MODEL<bbm::doubleRGB>>::make_ptr }


} // namespace bbmref
