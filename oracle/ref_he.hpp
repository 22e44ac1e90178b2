/* oracle/ref_he.hpp -- TEST INFRASTRUCTURE ONLY: the He family for the reference shim.
 *
 * bsdfmodel/he.h:489-496 and ngan.h:166-167 wrap he_base in bbm::ndf_sampler, whose internal
 * ndf::sampler<backscatter, 90, 1> relies on the default template argument NAME = NDF::name + "_sampler"
 * (include/ndf/sampler.h:34) -- which g++ 11 cannot deduce (CTAD on a string_literal NTTP).  Nothing
 * else in the chain fails.  he_sampled below restates ndf_sampler (include/bbm/ndf_sampler.h:22-164:
 * the backscatter NDF pass-through, sample = reflect(out, sampler.sample), pdf = sampler.pdf / |4 out.h|)
 * with that one argument spelled out, so the reference's own he_base (eval, reflectance) and the
 * reference's own ndf::sampler (the 90-bin data-driven CDF, its sampling and pdf) are what runs.
 */
#pragma once
#include "bsdfmodel/he.h"
#include "bsdfmodel/scaledmodel.h"

namespace bbmref {

template<typename BSDFMODEL, bbm::string_literal NAME>
  class he_sampled : public BSDFMODEL
{
  BBM_BASETYPES( BSDFMODEL );

  struct backscatter          // bbm/ndf_sampler.h:33-53
  {
    BBM_BASETYPES(void);
    BBM_IMPORT_CONFIG( BSDFMODEL );
    static constexpr bbm::string_literal name = "backscatter_" + NAME;
    backscatter(void) {}
    backscatter(const BSDFMODEL* src, bbm::bsdf_flag c, bbm::unit_t u) : component(c), unit(u), model(src) {}
    Value eval(const Vec3d& halfway, Mask mask=true) const { return bbm::hsum(model->eval(halfway, halfway, component, unit, mask)); }
    Vec3d sample(const Vec3d& view, const Vec2d& xi, Mask mask=true) const;
    Value pdf(const Vec3d& view, const Vec3d& m, Mask mask=true) const;
    Value G1(const Vec3d& v, const Vec3d& m, Mask mask=true) const;
    bbm::bsdf_flag component;
    bbm::unit_t unit;
    const BSDFMODEL* model;
    BBM_ATTRIBUTES( bbm::reflection::attributes(*model) );
  };
  using sampler_t = bbm::ndf::sampler<backscatter, 90, 1, "backscatter_" + NAME + "_sampler">;

public:
  BBM_IMPORT_CONFIG( BSDFMODEL );
  static constexpr bbm::string_literal name = NAME;
  BBM_BSDF_FORWARD;

  template<typename... Ts> requires std::constructible_from<BSDFMODEL, Ts...>
    he_sampled(Ts&&... ts) : BSDFMODEL(std::forward<Ts>(ts)...), _samplers() {}

  using BSDFMODEL::eval;
  using BSDFMODEL::reflectance;

  BsdfSample sample(const Vec3d& out, const Vec2d& xi, BsdfFlag component=bbm::bsdf_flag::All, bbm::unit_t unit=bbm::unit_t::Radiance, Mask mask=true) const
  {
    BsdfSample sample = {0,0,bbm::bsdf_flag::None};
    mask &= (xi[0] >= 0) && (xi[1] >= 0) && (xi[0] <= 1) && (xi[1] <= 1);
    mask &= (bbm::vec::z(out) > 0);
    if(bbm::none(mask)) return sample;
    Vec3d halfway;
    for(auto u : bbm::reflection::enum_v<bbm::unit_t>)
      for(auto c : bbm::reflection::enum_v<bbm::bsdf_flag>)
      {
        auto sample_mask = mask && bbm::eq(component, c) && bbm::eq(unit, u);
        if(bbm::any(sample_mask))
        {
          auto [itr,init] = _samplers.try_emplace(std::pair(c,u), sampler_t(this, c, u));
          halfway = bbm::select(sample_mask, itr->second.sample(out, xi, sample_mask), halfway);
        }
      }
    sample.direction = bbm::select(mask, bbm::reflect(out, halfway), 0);
    sample.pdf = pdf(sample.direction, out, component, unit, mask);
    sample.flag = bbm::select(mask, component, BsdfFlag(bbm::bsdf_flag::None));
    return sample;
  }

  Value pdf(const Vec3d& in, const Vec3d& out, BsdfFlag component=bbm::bsdf_flag::All, bbm::unit_t unit=bbm::unit_t::Radiance, Mask mask=true) const
  {
    mask &= (bbm::vec::z(out) > 0) && (bbm::vec::z(in) > 0);
    if(bbm::none(mask)) return 0;
    Vec3d h = bbm::halfway(in, out);
    Value pdf(0);
    for(auto u : bbm::reflection::enum_v<bbm::unit_t>)
      for(auto c : bbm::reflection::enum_v<bbm::bsdf_flag>)
      {
        auto pdf_mask = mask && bbm::eq(component, c) && bbm::eq(unit, u);
        if(bbm::any(pdf_mask))
        {
          auto [itr,init] = _samplers.try_emplace(std::pair(c,u), sampler_t(this, c, u));
          pdf = bbm::select(pdf_mask, itr->second.pdf(out, h, pdf_mask), pdf);
        }
      }
    return bbm::select(mask, pdf / bbm::abs(4.0 * bbm::dot(out, h)), 0);
  }

private:
  mutable std::map< std::pair<bbm::bsdf_flag, bbm::unit_t>, sampler_t > _samplers;
};

// he.h:489-496, ngan.h:166-167 with he_sampled in place of ndf_sampler
template<typename CONF> using he = he_sampled<bbm::he_base<CONF, bbm::fresnel::complex<CONF, bbm::Spectrum_t<CONF>>, bbm::he_eq25::WithoutExp, bbm::he_eq78::Regular, 4, 64, true, 18>, "He">;
template<typename CONF> using hewestin = he_sampled<bbm::he_base<CONF, bbm::fresnel::complex<CONF, bbm::Spectrum_t<CONF>>, bbm::he_eq25::Errata, bbm::he_eq78::Westin, 4, 64, true, 18>, "HeWestin">;
template<typename CONF> using heholzschuch = he_sampled<bbm::he_base<CONF, bbm::fresnel::complex<CONF, bbm::Spectrum_t<CONF>>, bbm::he_eq25::Errata, bbm::he_eq78::Regular, 4, 10, false>, "HeHolzschuch">;
template<typename CONF> using nganhe = bbm::scaledmodel<he_sampled<bbm::he_base<CONF, bbm::fresnel::cook<CONF>, bbm::he_eq25::Errata, bbm::he_eq78::Westin, 4, 64, true, 18>, "NganHe">, bbm::bsdf_attr::SpecularScale>;

} // namespace bbmref
