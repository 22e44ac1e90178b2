/* oracle/ref_fit.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never measured as the product).
 *
 * Second translation unit of the reference shim (oracle/_ref/libbbm_ref.so): drives the reference's
 * own fitting machinery so the GPU fitting path can be checked against it:
 *   * Aggregate(Lambertian, X) models (include/bsdfmodel/aggregatemodel.h:22-233), the form of every
 *     published fit in /root/reference/fits/*.fit, registered like single models (ref_harness.cpp);
 *   * per-parameter bsdf_attr flags (include/bbm/bsdf_attr_flag.h:16-29) as seen through
 *     bbm::parameter_values(model, flag) (include/bbm/bsdf_enumerate.h:103-131);
 *   * the linearizers' index -> (in, out) maps (include/linearizer/spherical_linearizer.h:25-111,
 *     merl_linearizer.h:21-131);
 *   * sampledlossfunction (include/bbm/sampledlossfunction.h:34-97) with each of the six sample
 *     losses (include/loss/cosine_weighted_l2.h, cosine_weighted_log.h), per sample and as the
 *     reference's own serial float total;
 *   * compass search steps (include/optimizer/compass.h:40-183) on that loss;
 *   * bbm::batch (include/bbm/batch.h:27-92) over that loss: the indices its bbm::rng<Size_t> draws and the
 *     per-sample losses operator()(idx) returns (its whole-batch operator() reads an uninitialised loop index,
 *     batch.h:78, and is not called).
 * The reference model of a fit is a second instance of the same Aggregate type (a synthetic
 * "measured" material from a published fit): MERL .binary data does not exist in this container.
 */
#include "ref_ops.hpp"

#include "bbm/sampledlossfunction.h"
#include "loss/cosine_weighted_l2.h"
#include "loss/cosine_weighted_log.h"
#include "linearizer/spherical_linearizer.h"
#include "linearizer/merl_linearizer.h"
#include "optimizer/compass.h"
#include "bbm/batch.h"

namespace bbmref {

using C = bbm::floatRGB;
using CD = bbm::doubleRGB;

template<template<typename> class X>
using agg = bbm::aggregatemodel<bbm::lambertian<C>, X<C>>;
template<template<typename> class X>
using aggd = bbm::aggregatemodel<bbm::lambertian<CD>, X<CD>>;

// Aliases with a single template parameter for the models whose templates take defaulted extras.
template<typename T> using cooktorrance_t = bbm::cooktorrance<T>;
template<typename T> using lowcooktorrance_t = bbm::lowcooktorrance<T>;
template<typename T> using ggx_t = bbm::ggx<T>;
template<typename T> using bagher_t = bbm::bagher<T>;
template<typename T> using lowashikhminshirley_t = bbm::lowashikhminshirley<T>;
template<typename T> using lowmicrofacetfit_t = bbm::lowmicrofacetfit<T>;
template<typename T> using lowsmooth_t = bbm::lowsmooth<T>;
template<typename T> using nganashikhminshirley_t = bbm::nganashikhminshirley<T>;
template<typename T> using nganblinnphong_t = bbm::nganblinnphong<T>;
template<typename T> using ngancooktorrance_t = bbm::ngancooktorrance<T>;
template<typename T> using nganlafortune_t = bbm::nganlafortune<T>;
template<typename T> using nganward_t = bbm::nganward<T>;
template<typename T> using nganwardduer_t = bbm::nganwardduer<T>;
template<typename T> using nganhe_t = bbmref::nganhe<T>;
template<typename T> using lambertian_t = bbm::lambertian<T>;
template<typename T> using orennayar_t = bbm::orennayar<T>;
template<typename T> using ward_t = bbm::ward<T>;

// aggregatemodel<X...> of any models (aggregatemodel.h:222): the compositions the GPU evaluates by composing its
// children's kernels (bbm_hip_aggregate_*), a few of each kind: three children, no Lambertian, a data-driven
// sampler child (a child type may appear once: the children are the aggregate's base classes)
template<template<typename> class... X>
struct aggv
{
  using f = bbm::aggregatemodel<X<C>...>;
  using d = bbm::aggregatemodel<X<CD>...>;
};
#define BBMREF_AGGV(KEY, ...) \
  entry{ KEY, \
         &ops<typename aggv<__VA_ARGS__>::f>::defaults, &ops<typename aggv<__VA_ARGS__>::f>::bounds, \
         &ops<typename aggv<__VA_ARGS__>::f>::to_string, \
         &ops<typename aggv<__VA_ARGS__>::f>::template evalpdf<float>, \
         &ops<typename aggv<__VA_ARGS__>::d>::template evalpdf<double>, \
         &ops<typename aggv<__VA_ARGS__>::f>::template sample<float>, \
         &ops<typename aggv<__VA_ARGS__>::f>::template reflectance<float>, \
         &ops<typename aggv<__VA_ARGS__>::f>::from_string, &ops<typename aggv<__VA_ARGS__>::d>::template reflectance<double>, \
         &ops<typename aggv<__VA_ARGS__>::d>::template sample<double>, \
         &ops<typename aggv<__VA_ARGS__>::d>::template evalpdf<double, double> }

// an aggregate given by its floatRGB and doubleRGB types (nested aggregates: aggregatemodel_base takes any
// bsdfmodel child, aggregatemodel.h:22)
#define BBMREF_AGGT(KEY, TF, TD) \
  entry{ KEY, &ops<TF>::defaults, &ops<TF>::bounds, &ops<TF>::to_string, &ops<TF>::template evalpdf<float>, \
         &ops<TD>::template evalpdf<double>, &ops<TF>::template sample<float>, &ops<TF>::template reflectance<float>, \
         &ops<TF>::from_string, &ops<TD>::template reflectance<double>, &ops<TD>::template sample<double>, \
         &ops<TD>::template evalpdf<double, double> }

template<typename T> using nested1_t = bbm::aggregatemodel<bbm::aggregatemodel<bbm::lambertian<T>, bbm::ward<T>>, bbm::ggx<T>>;
template<typename T> using nested2_t = bbm::aggregatemodel<bbm::aggregatemodel<bbm::lambertian<T>, bbm::cooktorrance<T>>, bbm::ward<T>>;
template<typename T>
using nested3_t = bbm::aggregatemodel<bbm::ggx<T>, bbm::aggregatemodel<bbm::phong<T>, bbm::aggregatemodel<bbm::ward<T>, bbm::orennayar<T>>>>;

#define BBMREF_AGG(X, KEY) \
  entry{ KEY, \
         &ops<agg<X>>::defaults, &ops<agg<X>>::bounds, &ops<agg<X>>::to_string, \
         &ops<agg<X>>::template evalpdf<float>, &ops<aggd<X>>::template evalpdf<double>, \
         &ops<agg<X>>::template sample<float>, &ops<agg<X>>::template reflectance<float>, &ops<agg<X>>::from_string, \
         &ops<aggd<X>>::template reflectance<double>, &ops<aggd<X>>::template sample<double>, \
         &ops<aggd<X>>::template evalpdf<double, double> }

const std::vector<entry>& aggregate_registry()
{
  static const std::vector<entry> r = {
    BBMREF_AGG(bagher_t, "Aggregate<Lambertian,Bagher>"),                          // fits/bagher_sgd.fit
    BBMREF_AGG(cooktorrance_t, "Aggregate<Lambertian,CookTorrance>"),              // docs/source/fitting.rst:31-33
    BBMREF_AGG(ggx_t, "Aggregate<Lambertian,GGX>"),
    BBMREF_AGG(lowcooktorrance_t, "Aggregate<Lambertian,LowCookTorrance>"),        // fits/low_cooktorrance_E*.fit
    BBMREF_AGG(lowashikhminshirley_t, "Aggregate<Lambertian,LowAshikhminShirley>"),  // fits/low_ashikhminshirley_E*.fit
    BBMREF_AGG(lowmicrofacetfit_t, "Aggregate<Lambertian,LowMicrofacetFit>"),      // fits/low_lowmicrofacet_E2.fit
    BBMREF_AGG(lowsmooth_t, "Aggregate<Lambertian,LowSmooth>"),                    // fits/low_lowsmooth_E2.fit
    BBMREF_AGG(nganashikhminshirley_t, "Aggregate<Lambertian,NganAshikhminShirley>"),  // fits/ngan_ashikhminshirley.fit
    BBMREF_AGG(nganblinnphong_t, "Aggregate<Lambertian,NganBlinnPhong>"),          // fits/ngan_blinnphong.fit
    BBMREF_AGG(ngancooktorrance_t, "Aggregate<Lambertian,NganCookTorrance>"),      // fits/ngan_cooktorrance.fit
    BBMREF_AGG(nganlafortune_t, "Aggregate<Lambertian,NganLafortune>"),            // fits/ngan_lafortune.fit
    BBMREF_AGG(nganward_t, "Aggregate<Lambertian,NganWard>"),                      // fits/ngan_ward.fit
    BBMREF_AGG(nganwardduer_t, "Aggregate<Lambertian,NganWardDuer>"),              // fits/ngan_wardduer.fit
    BBMREF_AGG(nganhe_t, "Aggregate<Lambertian,NganHe>"),                          // fits/ngan_he.fit
    BBMREF_AGGV("Aggregate<Lambertian,CookTorrance,GGX>", lambertian_t, cooktorrance_t, ggx_t),
    BBMREF_AGGV("Aggregate<CookTorrance,GGX>", cooktorrance_t, ggx_t),
    BBMREF_AGGV("Aggregate<OrenNayar,NganHe,Ward>", orennayar_t, nganhe_t, ward_t),
    BBMREF_AGGT("Aggregate<Aggregate<Lambertian,Ward>,GGX>", nested1_t<C>, nested1_t<CD>),
    BBMREF_AGGT("Aggregate<Aggregate<Lambertian,CookTorrance>,Ward>", nested2_t<C>, nested2_t<CD>),
    BBMREF_AGGT("Aggregate<GGX,Aggregate<Phong,Aggregate<Ward,OrenNayar>>>", nested3_t<C>, nested3_t<CD>),
  };
  return r;
}

// ------------------------------------------------------------------ per-parameter attr flags

template<typename M>
std::vector<uint32_t> param_attrs()
{
  M m;
  auto all = bbm::parameter_values(m, kAllParams);
  std::vector<uint32_t> r(all.size(), 0u);
  for(size_t i = 0; i < all.size(); ++i) all[i] = float(i);
  for(uint32_t f : {0x01u, 0x02u, 0x04u, 0x08u, 0x10u})
    for(auto& v : bbm::parameter_values(m, bbm::bsdf_attr(f)))
      r[size_t(float(v))] |= f;
  return r;
}

// indices (into the full kAllParams vector) that parameter_values(model, flag) returns, in its order
template<typename M>
std::vector<uint32_t> param_select(uint32_t flag)
{
  M m;
  auto all = bbm::parameter_values(m, kAllParams);
  for(size_t i = 0; i < all.size(); ++i) all[i] = float(i);
  std::vector<uint32_t> r;
  for(auto& v : bbm::parameter_values(m, bbm::bsdf_attr(flag))) r.push_back(uint32_t(float(v)));
  return r;
}

// ------------------------------------------------------------------------- linearizers
//
// merl_linearizer's index -> direction map does not compile with the native backbone:
// convertFromHalfwayDifference (include/core/vec_transform.h:118-123) calls unqualified
// phi()/theta(), which exist only as bbm::spherical::phi/theta.  Only its inverse map
// (direction pair -> index, merl_linearizer.h:99-126) is instantiable; it pins our forward map by
// round trip.  Arbitrary direction sets (e.g. our MERL-grid directions) go through
// table_linearizer, a minimal concepts::inout_linearizer over caller-provided pairs.

struct lin_desc
{
  int kind;                 // 0 = spherical_linearizer, 1 = merl_linearizer (inverse map only), 2 = table
  uint64_t s_in[2], s_out[2];
  float start_in[2], end_in[2], start_out[2], end_out[2];
  size_t n;                 // table: number of pairs
  const float* dirs[6];     // table: in xyz, out xyz
};

struct table_linearizer
{
  BBM_IMPORT_CONFIG( C );
  lin_desc d;
  Size_t size(void) const { return d.n; }
  Vec3dPair operator()(Size_t idx, Mask mask=true) const
  {
    Vec3dPair r = {0, 0};
    if(!mask || idx >= d.n) return r;
    r.in = Vec3d(d.dirs[0][idx], d.dirs[1][idx], d.dirs[2][idx]);
    r.out = Vec3d(d.dirs[3][idx], d.dirs[4][idx], d.dirs[5][idx]);
    return r;
  }
  Size_t operator()(const Vec3d&, const Vec3d&, Mask = true) const { return d.n; }
};
static_assert(bbm::concepts::inout_linearizer<table_linearizer>);

bbm::spherical_linearizer<C> make_spherical(const lin_desc& d)
{
  using V2 = bbm::vec2d<float>;
  using S2 = bbm::vec2d<size_t>;
  return bbm::spherical_linearizer<C>(S2(d.s_in[0], d.s_in[1]), S2(d.s_out[0], d.s_out[1]),
                                      V2(d.start_in[0], d.start_in[1]), V2(d.end_in[0], d.end_in[1]),
                                      V2(d.start_out[0], d.start_out[1]), V2(d.end_out[0], d.end_out[1]));
}

bbm::merl_linearizer<C> make_merl(const lin_desc& d)
{
  using S2 = bbm::vec2d<size_t>;
  return bbm::merl_linearizer<C>(S2(d.s_in[0], d.s_in[1]), S2(d.s_out[0], d.s_out[1]));
}

template<typename LIN>
void linearize(const LIN& lin, uint64_t begin, size_t n, float* in[3], float* out[3])
{
  for(size_t i = 0; i < n; ++i)
  {
    auto p = lin(size_t(begin + i));
    for(int k = 0; k < 3; ++k) { in[k][i] = p.in[k]; out[k][i] = p.out[k]; }
  }
}

template<typename F>
auto with_lin(const lin_desc& d, F&& f)
{
  if(d.kind == 2) return f(table_linearizer{d});
  return f(make_spherical(d));
}

// ------------------------------------------------------------------------------ losses

template<typename LIN, typename F>
auto with_loss(int loss_kind, F&& f)
{
  switch(loss_kind)
  {
    case 0: return f(bbm::nganL2_error<C>());
    case 1: return f(bbm::lowL2_error<C>());
    case 2: return f(bbm::bieronL2_error<C>());
    case 3: return f(bbm::standardLog_error<C>());
    case 4: return f(bbm::lowLog_error<C>());
    default: return f(bbm::bieronLog_error<C>());
  }
}

// loss over [0, size) of the linearizer: per-sample values (OpenMP) and the reference's own serial
// float total sampledlossfunction::operator()() (sampledlossfunction.h:80-87)
template<typename M>
int loss(const float* fp, const float* rp, int np, const lin_desc& d, int loss_kind, float* per_sample,
         float* total, int nthreads)
{
  const M fitted = ops<M>::make(fp, np);
  const M reference = ops<M>::make(rp, np);
  return with_lin(d, [&](auto lin) {
    return with_loss<decltype(lin)>(loss_kind, [&](auto err) {
      bbm::sampledlossfunction<M, M, decltype(err), decltype(lin)> lf(fitted, reference, err, lin);
      const size_t n = lf.samples();
      if(per_sample)
      {
#ifdef _OPENMP
        #pragma omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : 1)
#endif
        for(size_t i = 0; i < n; ++i) per_sample[i] = lf(i);
      }
      if(total) *total = lf();
      return int(n);
    });
  });
}

// `steps` compass steps (compass.h:82-140) from `init` towards `reference`; records the optimised
// parameter vector (parameter_values(fitted), i.e. without Dependent attributes) and the loss after
// every step.  Returns the number of optimised parameters.
template<typename M>
int compass_run(const float* init, const float* rp, int np, const lin_desc& d, int loss_kind, int steps,
                float* params_out, float* loss_out, float* loss0)
{
  M fitted = ops<M>::make(init, np);
  const M reference = ops<M>::make(rp, np);
  return with_lin(d, [&](auto lin) {
    return with_loss<decltype(lin)>(loss_kind, [&](auto err) {
      bbm::sampledlossfunction<M, M, decltype(err), decltype(lin)> lf(fitted, reference, err, lin);
      auto param = bbm::parameter_values(fitted);
      auto low = bbm::parameter_lower_bound(fitted);
      auto up = bbm::parameter_upper_bound(fitted);
      bbm::compass opt(lf, param, low, up);
      if(loss0) *loss0 = lf();
      const int P = int(param.size());
      for(int t = 0; t < steps; ++t)
      {
        float e = opt.step();
        if(loss_out) loss_out[t] = e;
        if(params_out) for(int i = 0; i < P; ++i) params_out[size_t(t) * P + i] = float(param[i]);
      }
      return P;
    });
  });
}

// bbm::batch(batchsize, lf, seed) over the sampled loss, then `updates` more update() calls: per_sample receives
// operator()(idx) for idx in [0, batchsize) after construction and after every update ((updates + 1) x batchsize)
template<typename M>
int batch_run(const float* fp, const float* rp, int np, const lin_desc& d, int loss_kind, uint64_t seed,
              size_t batchsize, int updates, float* per_sample)
{
  const M fitted = ops<M>::make(fp, np);
  const M reference = ops<M>::make(rp, np);
  return with_lin(d, [&](auto lin) {
    return with_loss<decltype(lin)>(loss_kind, [&](auto err) {
      using LF = bbm::sampledlossfunction<M, M, decltype(err), decltype(lin)>;
      LF lf(fitted, reference, err, lin);
      bbm::batch<LF> b(batchsize, lf, seed);
      for(int u = 0; u <= updates; ++u)
      {
        if(u > 0) b.update();
        for(size_t i = 0; i < batchsize; ++i) per_sample[size_t(u) * batchsize + i] = b(i);
      }
      return int(lf.samples());
    });
  });
}

struct fit_entry
{
  const char* name;
  std::vector<uint32_t> (*attrs)();
  std::vector<uint32_t> (*select)(uint32_t);
  int (*loss)(const float*, const float*, int, const lin_desc&, int, float*, float*, int);
  int (*compass)(const float*, const float*, int, const lin_desc&, int, int, float*, float*, float*);
  int (*batch)(const float*, const float*, int, const lin_desc&, int, uint64_t, size_t, int, float*);
};

#define BBMREF_FIT(X, KEY) fit_entry{ KEY, &param_attrs<agg<X>>, &param_select<agg<X>>, &loss<agg<X>>, &compass_run<agg<X>>, \
                                      &batch_run<agg<X>> }

const std::vector<fit_entry>& fit_registry()
{
  static const std::vector<fit_entry> r = {
    BBMREF_FIT(bagher_t, "Aggregate<Lambertian,Bagher>"),
    BBMREF_FIT(cooktorrance_t, "Aggregate<Lambertian,CookTorrance>"),
    BBMREF_FIT(ggx_t, "Aggregate<Lambertian,GGX>"),
    BBMREF_FIT(lowcooktorrance_t, "Aggregate<Lambertian,LowCookTorrance>"),
    BBMREF_FIT(ngancooktorrance_t, "Aggregate<Lambertian,NganCookTorrance>"),
    BBMREF_FIT(nganward_t, "Aggregate<Lambertian,NganWard>"),
  };
  return r;
}

const fit_entry* find_fit(const char* name)
{
  for(auto& e : fit_registry()) if(std::strcmp(e.name, name) == 0) return &e;
  return nullptr;
}

// single models: per-parameter attr flags
#define BBMREF_ATTRS(MODEL) std::pair<const char*, std::vector<uint32_t> (*)()>{ \
  bbm::MODEL<C>::name.value, &param_attrs<bbm::MODEL<C>> }

const std::vector<std::pair<const char*, std::vector<uint32_t> (*)()>>& attr_registry()
{
  static const std::vector<std::pair<const char*, std::vector<uint32_t> (*)()>> r = {
    BBMREF_ATTRS(lambertian), BBMREF_ATTRS(orennayar), BBMREF_ATTRS(cooktorrance), BBMREF_ATTRS(cooktorranceheitz),
    BBMREF_ATTRS(cooktorrancewalter), BBMREF_ATTRS(ggx), BBMREF_ATTRS(ggxheitz), BBMREF_ATTRS(phongwalter),
    BBMREF_ATTRS(ribardiere), BBMREF_ATTRS(ribardiereanisotropic), BBMREF_ATTRS(bagher), BBMREF_ATTRS(lowcooktorrance),
    BBMREF_ATTRS(lowmicrofacet), BBMREF_ATTRS(lowmicrofacetfit), BBMREF_ATTRS(ngancooktorrance), BBMREF_ATTRS(ward),
    BBMREF_ATTRS(wardduer), BBMREF_ATTRS(wardduergeislermoroder), BBMREF_ATTRS(nganward), BBMREF_ATTRS(nganwardduer),
    BBMREF_ATTRS(phong), BBMREF_ATTRS(nganblinnphong), BBMREF_ATTRS(lafortune), BBMREF_ATTRS(nganlafortune),
    BBMREF_ATTRS(ashikhminshirley), BBMREF_ATTRS(ashikhminshirleyfull), BBMREF_ATTRS(lowashikhminshirley),
    BBMREF_ATTRS(nganashikhminshirley), BBMREF_ATTRS(lowsmooth),
    std::pair<const char*, std::vector<uint32_t> (*)()>{ "EPD", &param_attrs<bbmref::epd<C>> },
    std::pair<const char*, std::vector<uint32_t> (*)()>{ "He", &param_attrs<bbmref::he<C>> },
    std::pair<const char*, std::vector<uint32_t> (*)()>{ "HeWestin", &param_attrs<bbmref::hewestin<C>> },
    std::pair<const char*, std::vector<uint32_t> (*)()>{ "HeHolzschuch", &param_attrs<bbmref::heholzschuch<C>> },
    std::pair<const char*, std::vector<uint32_t> (*)()>{ "NganHe", &param_attrs<bbmref::nganhe<C>> },
  };
  return r;
}

#define BBMREF_AGG_ATTRS(X, KEY) std::pair<const char*, std::vector<uint32_t> (*)()>{ KEY, &param_attrs<agg<X>> }

const std::vector<std::pair<const char*, std::vector<uint32_t> (*)()>>& agg_attr_registry()
{
  static const std::vector<std::pair<const char*, std::vector<uint32_t> (*)()>> r = {
    BBMREF_AGG_ATTRS(bagher_t, "Aggregate<Lambertian,Bagher>"),
    BBMREF_AGG_ATTRS(cooktorrance_t, "Aggregate<Lambertian,CookTorrance>"),
    BBMREF_AGG_ATTRS(ggx_t, "Aggregate<Lambertian,GGX>"),
    BBMREF_AGG_ATTRS(lowcooktorrance_t, "Aggregate<Lambertian,LowCookTorrance>"),
    BBMREF_AGG_ATTRS(lowashikhminshirley_t, "Aggregate<Lambertian,LowAshikhminShirley>"),
    BBMREF_AGG_ATTRS(lowmicrofacetfit_t, "Aggregate<Lambertian,LowMicrofacetFit>"),
    BBMREF_AGG_ATTRS(lowsmooth_t, "Aggregate<Lambertian,LowSmooth>"),
    BBMREF_AGG_ATTRS(nganashikhminshirley_t, "Aggregate<Lambertian,NganAshikhminShirley>"),
    BBMREF_AGG_ATTRS(nganblinnphong_t, "Aggregate<Lambertian,NganBlinnPhong>"),
    BBMREF_AGG_ATTRS(ngancooktorrance_t, "Aggregate<Lambertian,NganCookTorrance>"),
    BBMREF_AGG_ATTRS(nganlafortune_t, "Aggregate<Lambertian,NganLafortune>"),
    BBMREF_AGG_ATTRS(nganward_t, "Aggregate<Lambertian,NganWard>"),
    BBMREF_AGG_ATTRS(nganwardduer_t, "Aggregate<Lambertian,NganWardDuer>"),
    BBMREF_AGG_ATTRS(nganhe_t, "Aggregate<Lambertian,NganHe>"),
    std::pair<const char*, std::vector<uint32_t> (*)()>{ "Aggregate<Lambertian,CookTorrance,GGX>", &param_attrs<aggv<lambertian_t, cooktorrance_t, ggx_t>::f> },
    std::pair<const char*, std::vector<uint32_t> (*)()>{ "Aggregate<CookTorrance,GGX>", &param_attrs<aggv<cooktorrance_t, ggx_t>::f> },
    std::pair<const char*, std::vector<uint32_t> (*)()>{ "Aggregate<OrenNayar,NganHe,Ward>", &param_attrs<aggv<orennayar_t, nganhe_t, ward_t>::f> },
  };
  return r;
}

// A sampled loss whose idx-th sample "loss" is idx itself (exact in float below 2^24): wrapped in the reference's
// bbm::batch, operator()(i) then returns the i-th index its bbm::rng<Size_t> drew (batch.h:64-70)
struct echo_loss
{
  BBM_IMPORT_CONFIG( C );
  Size_t n;
  void update(void) {}
  Size_t samples(void) const { return n; }
  Value operator()(Size_t idx, Mask = true) const { return Value(idx); }
  Value operator()(Mask = true) const { return 0; }
};
static_assert(bbm::concepts::sampledlossfunction<echo_loss>);

} // namespace bbmref

using namespace bbmref;

extern "C" {

int bbmref_param_attrs(const char* name, uint32_t* out, int cap)
{
  std::vector<uint32_t> v;
  bool found = false;
  for(auto& e : attr_registry()) if(std::strcmp(e.first, name) == 0) { v = e.second(); found = true; break; }
  if(!found)
    for(auto& e : agg_attr_registry()) if(std::strcmp(e.first, name) == 0) { v = e.second(); found = true; break; }
  if(!found) return -1;
  for(int i = 0; out && i < int(v.size()) && i < cap; ++i) out[i] = v[size_t(i)];
  return int(v.size());
}

int bbmref_param_select(const char* name, uint32_t flag, uint32_t* out, int cap)
{
  auto f = find_fit(name); if(!f) return -1;
  auto v = f->select(flag);
  for(int i = 0; out && i < int(v.size()) && i < cap; ++i) out[i] = v[size_t(i)];
  return int(v.size());
}

int bbmref_num_aggregates(void) { return int(aggregate_registry().size()); }
const char* bbmref_aggregate_name(int i)
{ return (i >= 0 && i < int(aggregate_registry().size())) ? aggregate_registry()[size_t(i)].name : nullptr; }

static lin_desc desc_of(int kind, const uint64_t* s_in, const uint64_t* s_out, const float* rng)
{
  lin_desc d{};
  d.kind = kind;
  if(kind == 2)
  {
    // table: s_in[0] = number of pairs, rng = 6 pointers (in xyz, out xyz) packed by the caller
    d.n = size_t(s_in[0]);
    const float* const* p = reinterpret_cast<const float* const*>(rng);
    for(int k = 0; k < 6; ++k) d.dirs[k] = p[k];
    return d;
  }
  for(int k = 0; k < 2; ++k)
  {
    d.s_in[k] = s_in[k]; d.s_out[k] = s_out[k];
    d.start_in[k] = rng[k]; d.end_in[k] = rng[2 + k]; d.start_out[k] = rng[4 + k]; d.end_out[k] = rng[6 + k];
  }
  return d;
}

// kind 0 (spherical): rng = {start_in[2], end_in[2], start_out[2], end_out[2]} as (phi, theta).
// kind 2 (table): s_in[0] = n, rng = address of 6 float* (in xyz, out xyz).  kind 1 (merl): size only.
int64_t bbmref_linearizer_size(int kind, const uint64_t* s_in, const uint64_t* s_out, const float* rng)
{
  const lin_desc d = desc_of(kind, s_in, s_out, rng);
  if(kind == 1) return int64_t(make_merl(d).size());
  return with_lin(d, [](auto lin) { return int64_t(lin.size()); });
}

// merl_linearizer's inverse map (merl_linearizer.h:99-126): direction pair -> linear index
int bbmref_merl_index(const uint64_t* s_h, const uint64_t* s_d, size_t n, const float* ix, const float* iy,
                      const float* iz, const float* ox, const float* oy, const float* oz, uint64_t* idx)
{
  lin_desc d{};
  d.kind = 1;
  for(int k = 0; k < 2; ++k) { d.s_in[k] = s_h[k]; d.s_out[k] = s_d[k]; }
  const auto lin = make_merl(d);
  using V3 = bbm::vec3d<float>;
  for(size_t i = 0; i < n; ++i) idx[i] = uint64_t(lin(V3(ix[i], iy[i], iz[i]), V3(ox[i], oy[i], oz[i])));
  return 0;
}

int bbmref_linearize(int kind, const uint64_t* s_in, const uint64_t* s_out, const float* rng, uint64_t begin, size_t n,
                     float* ix, float* iy, float* iz, float* ox, float* oy, float* oz)
{
  if(kind != 0) return -2;   // merl: forward map not instantiable (see above); table: nothing to do
  const lin_desc d = desc_of(kind, s_in, s_out, rng);
  float* in[3] = {ix, iy, iz};
  float* out[3] = {ox, oy, oz};
  with_lin(d, [&](auto lin) { linearize(lin, begin, n, in, out); return 0; });
  return 0;
}

int bbmref_loss(const char* name, const float* fitted, const float* reference, int np,
                int kind, const uint64_t* s_in, const uint64_t* s_out, const float* rng, int loss_kind,
                float* per_sample, float* total, int nthreads)
{
  auto e = find_fit(name); if(!e) return -1;
  if(kind == 1) return -2;
  return e->loss(fitted, reference, np, desc_of(kind, s_in, s_out, rng), loss_kind, per_sample, total, nthreads);
}

int bbmref_compass(const char* name, const float* init, const float* reference, int np,
                   int kind, const uint64_t* s_in, const uint64_t* s_out, const float* rng, int loss_kind,
                   int steps, float* params_out, float* loss_out, float* loss0)
{
  auto e = find_fit(name); if(!e) return -1;
  if(kind == 1) return -2;
  return e->compass(init, reference, np, desc_of(kind, s_in, s_out, rng), loss_kind, steps, params_out, loss_out, loss0);
}

// the indices of bbm::batch<...>(batchsize, loss with nsamples samples, seed) after construction and after each of
// `updates` update() calls: (updates + 1) x batchsize values in [0, nsamples] (nsamples < 2^24)
int bbmref_batch_indices(uint64_t seed, uint64_t nsamples, size_t batchsize, int updates, uint64_t* out)
{
  if(nsamples >= (uint64_t(1) << 24)) return -2;
  bbm::batch<echo_loss> b(batchsize, echo_loss{size_t(nsamples)}, seed);
  for(int u = 0; u <= updates; ++u)
  {
    if(u > 0) b.update();
    for(size_t i = 0; i < batchsize; ++i) out[size_t(u) * batchsize + i] = uint64_t(float(b(i)));
  }
  return 0;
}

int bbmref_batch_loss(const char* name, const float* fitted, const float* reference, int np,
                      int kind, const uint64_t* s_in, const uint64_t* s_out, const float* rng, int loss_kind,
                      uint64_t seed, size_t batchsize, int updates, float* per_sample)
{
  auto e = find_fit(name); if(!e) return -1;
  if(kind == 1) return -2;
  return e->batch(fitted, reference, np, desc_of(kind, s_in, s_out, rng), loss_kind, seed, batchsize, updates, per_sample);
}

} // extern "C"
