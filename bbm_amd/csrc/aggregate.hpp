// bbm_amd/csrc/aggregate.hpp -- aggregatemodel<A, B> (include/bsdfmodel/aggregatemodel.h:22-233):
// the sum of two models, the form of every published fit (fits/*.fit: Aggregate(Lambertian(...),
// X(...))).  Parameters are A's vector followed by B's (reflection order of the base classes).
//   eval        = A.eval + B.eval                                            (:61-64)
//   pdf         = (w_A pdf_A + w_B pdf_B) / (w_A + w_B), w = hsum(reflectance(out)), 0 if sum <= eps (:129-143)
//   sample      = pick A or B by xi0 * sum against w_A, rescale xi0, sample it; pdf as above (:81-113)
//   reflectance = A.reflectance + B.reflectance                              (:156-163)
//
// The same two children as the RUNTIME aggregate bsdf_import / fromString<bsdf_ptr> builds (aggregatebsdf,
// include/bbm/aggregatebsdf.h:40-190; bsdf_string_convert.h:59 maps "Aggregate" to it): eval and reflectance are
// left folds from 0 -- for two children the same floats -- but
//   pdf    = w_A pdf_A / sum + w_B pdf_B / sum, one quotient per term, 0 unless sum > eps (:173-187)
//   sample = no sample at all unless sum > eps (:113-116: the reference returns a default-constructed, i.e.
//            indeterminate, BsdfSample there; this returns {0, 0, None}); otherwise the same child selection, and
//            the pdf at the sampled direction term by term as above (:133-137)
// Selected per launch by the parameter block's last slot (kAggregateModeSlot, set by the C-ABI for model ids
// carrying BBM_HIP_RUNTIME_AGGREGATE); 0 (every other path) is aggregatemodel.
#pragma once
#include "math.hpp"
#include "microfacet.hpp"

namespace bbmhip {

constexpr int kAggregateModeSlot = 63;     // ParamBlock slot (kernels.hpp kMaxParams - 1): 1 = aggregatebsdf semantics

template<class A, class B>
struct Aggregate
{
  static constexpr int kParams = A::kParams + B::kParams;
  static constexpr uint32_t kComponent = A::kComponent | B::kComponent;
  static_assert(kParams + 3 <= kAggregateModeSlot, "the mode slot must lie beyond the children's parameter blocks");
  A a;
  B b;
  bool runtime;            // aggregatebsdf (fromString / bsdf_ptr) rather than aggregatemodel semantics
  __device__ explicit Aggregate(const float* p) : a(p), b(p + A::kParams), runtime(p[kAggregateModeSlot] != 0.0f) {}

  // both children's per-pair preludes (the loss kernel): eval_geo is eval's rgb = e_A + e_B from them
  static constexpr bool kHasGeo = has_geo<A>() && has_geo<B>();
  struct Geo { typename A::Geo a; typename B::Geo b; };
  __device__ __forceinline__ static Geo geometry(v3 in, v3 out) { return Geo{A::geometry(in, out), B::geometry(in, out)}; }
  __device__ __forceinline__ void eval_geo_cached(Geo& g, uint32_t component, float* rgb) const
  {
    eval_geo<true>(g, component, rgb);
  }
  template<bool CACHE = false>
  __device__ __forceinline__ void eval_geo(Geo& g, uint32_t component, float* rgb) const
  {
    float ra[3], rb[3];
    geo_eval<CACHE>(a, g.a, component, ra);
    geo_eval<CACHE>(b, g.b, component, rb);
    rgb[0] = ra[0] + rb[0];
    rgb[1] = ra[1] + rb[1];
    rgb[2] = ra[2] + rb[2];
  }

  // hsum(reflectance(out)) per child: std::accumulate from Value(0) (horizontal.h:64-67)
  __device__ __forceinline__ void weights(v3 out, uint32_t component, float& wa, float& wb) const
  {
    float ra[3], rb[3];
    a.reflectance(out, component, ra);
    b.reflectance(out, component, rb);
    wa = ((0.0f + ra[0]) + ra[1]) + ra[2];
    wb = ((0.0f + rb[0]) + rb[1]) + rb[2];
  }

  // aggregatemodel: inner_product(pdfs, weights, Value(0)) / sum, masked sum > eps (:141-142); aggregatebsdf:
  // pdf += weight * pdf_k / sum per child from 0 (aggregatebsdf.h:183-187)
  __device__ __forceinline__ float mix(float pa, float pb, float wa, float wb) const
  {
    const float sum = (0.0f + wa) + wb;
    const float ip = (0.0f + pa * wa) + pb * wb;
    const float tm = (0.0f + div_nr(wa * pa, sum)) + div_nr(wb * pb, sum);
    return (sum > kEpsF) ? (runtime ? tm : div_nr(ip, sum)) : 0.0f;
  }

  // exact mode (bbm_hip_set_exact_subnormals) for whichever child has one
  static constexpr bool kHasExact = model_has_exact<A>() || model_has_exact<B>();
  template<int MODE, bool EXACT = false>
  __device__ __forceinline__ void eval_pdf(v3 in, v3 out, uint32_t component, float* rgb, float& pdf) const
  {
    float ra[3], rb[3], pa, pb;
    model_eval_pdf<MODE, EXACT>(a, in, out, component, ra, pa);
    model_eval_pdf<MODE, EXACT>(b, in, out, component, rb, pb);
    rgb[0] = ra[0] + rb[0];
    rgb[1] = ra[1] + rb[1];
    rgb[2] = ra[2] + rb[2];
    if (MODE & kModePdf)
    {
      float wa, wb;
      weights(out, component, wa, wb);
      pdf = component ? mix(pa, pb, wa, wb) : 0.0f;
    }
    else pdf = 0.0f;
  }

  __device__ __forceinline__ void reflectance(v3 out, uint32_t component, float* rgb) const
  {
    float ra[3], rb[3];
    a.reflectance(out, component, ra);
    b.reflectance(out, component, rb);
    rgb[0] = ra[0] + rb[0];
    rgb[1] = ra[1] + rb[1];
    rgb[2] = ra[2] + rb[2];
  }

  __device__ __forceinline__ void sample(v3 out, float xi0, float xi1, uint32_t component, v3& dir, float& pdf,
                                         uint32_t& flag) const
  {
    dir = mk3(0.0f, 0.0f, 0.0f);
    pdf = 0.0f;
    flag = kFlagNone;
    if (!component) return;   // masked lane: the reference returns {0, 0, None}
    float wa, wb;
    weights(out, component, wa, wb);
    const float sum = (0.0f + wa) + wb;
    if (runtime && !(sum > kEpsF)) return;        // aggregatebsdf's bail-out (:115-116)
    float x = xi0 * sum;
    // CONSTFOREACH over the children in order; a later child that also claims x overrides (:95-108)
    const bool ma = (x >= 0) && (x <= wa);
    if (ma)
    {
      const float nx = (wa > kEpsF) ? div_nr(x, wa) : 0.0f;
      float p;
      a.sample(out, nx, xi1, component, dir, p, flag);
    }
    x -= wa;
    const bool mb = (x >= 0) && (x <= wb);
    if (mb)
    {
      const float nx = (wb > kEpsF) ? div_nr(x, wb) : 0.0f;
      float p;
      b.sample(out, nx, xi1, component, dir, p, flag);
    }
    float rgb[3], pa, pb;
    a.template eval_pdf<kModePdf>(dir, out, component, rgb, pa);
    b.template eval_pdf<kModePdf>(dir, out, component, rgb, pb);
    pdf = mix(pa, pb, wa, wb);
  }
};

template<class A, class B> struct exact_sample<Aggregate<A, B>> { using type = Aggregate<exact_sample_t<A>, exact_sample_t<B>>; };

}  // namespace bbmhip
