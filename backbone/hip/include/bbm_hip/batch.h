/* backbone/hip/include/bbm_hip/batch.h -- C++20 host adapter: bbm::bsdfmodel<> -> libbbm_hip.
 *
 * Header-only, compiled by the BBM user's host compiler (g++/clang) together with the BBM headers;
 * it never includes HIP device code.  A model instance of the reference's template API, e.g.
 *
 *     bbm::cooktorrance<bbm::floatRGB> ct;             // include/bsdfmodel/cooktorrance.h:28-34
 *     bbm::hip::eval_pdf(ct, in, out, n, rgb, pdf);     // N pairs on the GPU
 *
 * is mapped to the HIP backbone in two steps:
 *   1. its *type* is matched against the compositions the kernels implement (cooktorrance<C>,
 *      ggx<C>, lambertian<C>, ...) -- a composition the GPU does not implement is a compile error,
 *      never a silent fallback;
 *   2. its attributes are packed with bbm::parameter_values(model, All | Dependent)
 *      (include/bbm/bsdf_enumerate.h), i.e. in declaration order, and passed by value.
 * Device buffers are caller-owned SoA float arrays; calls are asynchronous on `stream`.
 * Errors from the C-ABI are rethrown as bbm::hip::error (a std::runtime_error), matching the
 * reference's exception style (include/core/error.h:42-46).
 */
#ifndef BBM_HIP_BATCH_H
#define BBM_HIP_BATCH_H

#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

#include "bbm/bsdf_enumerate.h"
#include "bbm_hip.h"

namespace bbm {
  namespace hip {

    //! \brief SoA view of N directions in device memory (x[], y[], z[])
    struct soa3 { const float* x; const float* y; const float* z; };
    //! \brief SoA view of N writable 3-vectors / RGB spectra in device memory
    struct soa3_out { float* x; float* y; float* z; };

    //! \brief Error raised when the HIP backbone rejects a call
    struct error : public std::runtime_error
    {
      int code;
      error(int c, const std::string& what) : std::runtime_error("libbbm_hip: " + what), code(c) {}
    };

    inline void check(int rc)
    {
      if(rc < 0) throw error(rc, bbm_hip_last_error());
    }

    namespace detail {
      template<typename T> struct dependent_false : std::false_type {};

      //! \brief Registry name of the GPU kernel implementing MODEL's composition.
      template<typename MODEL>
        constexpr const char* gpu_name()
      {
        using C = get_config<MODEL>;
        using M = std::decay_t<MODEL>;
        static_assert(std::is_same_v<Value_t<C>, float>, "the HIP backbone evaluates floatRGB-style configs (Value = float)");
#ifdef _BBM_LAMBERTIAN_H_
        if constexpr (std::is_same_v<M, bbm::lambertian<C>>) return "Lambertian";
        else
#endif
#ifdef _BBM_COOKTORRANCE_H_
        if constexpr (std::is_same_v<M, bbm::cooktorrance<C>>) return "CookTorrance";
        else
#endif
#ifdef _BBM_LOW_FITMODELS_H_
        if constexpr (std::is_same_v<M, bbm::lowcooktorrance<C>>) return "LowCookTorrance";
        else
#endif
#ifdef _BBM_GGX_H_
        if constexpr (std::is_same_v<M, bbm::ggx<C>>) return "GGX";
        else
#endif
#ifdef _BBM_COOKTORRANCEWALTER_H_
        if constexpr (std::is_same_v<M, bbm::cooktorrancewalter<C>>) return "CookTorranceWalter";
        else
#endif
#ifdef _BBM_COOKTORRANCEHEITZ_H_
        if constexpr (std::is_same_v<M, bbm::cooktorranceheitz<C>>) return "CookTorranceHeitz";
        else
#endif
#ifdef _BBM_GGX_HEITZ_H_
        if constexpr (std::is_same_v<M, bbm::ggxheitz<C>>) return "GGXHeitz";
        else
#endif
#ifdef _BBM_PHONG_WALTER_H_
        if constexpr (std::is_same_v<M, bbm::phongwalter<C>>) return "PhongWalter";
        else
#endif
#ifdef _BBM_RIBARDIERE_H_
        if constexpr (std::is_same_v<M, bbm::ribardiere<C>>) return "Ribardiere";
        else if constexpr (std::is_same_v<M, bbm::ribardiereanisotropic<C>>) return "RibardiereAnisotropic";
        else
#endif
#ifdef _BBM_NGAN_H_
        if constexpr (std::is_same_v<M, bbm::ngancooktorrance<C>>) return "NganCookTorrance";
        else if constexpr (std::is_same_v<M, bbm::nganward<C>>) return "NganWard";
        else if constexpr (std::is_same_v<M, bbm::nganwardduer<C>>) return "NganWardDuer";
        else if constexpr (std::is_same_v<M, bbm::nganblinnphong<C>>) return "NganBlinnPhong";
        else if constexpr (std::is_same_v<M, bbm::nganlafortune<C>>) return "NganLafortune";
        else if constexpr (std::is_same_v<M, bbm::nganashikhminshirley<C>>) return "NganAshikhminShirley";
        else
#endif
#ifdef _BBM_ORENNAYAR_H_
        if constexpr (std::is_same_v<M, bbm::orennayar<C>>) return "OrenNayar";
        else
#endif
#ifdef _BBM_WARD_H_
        if constexpr (std::is_same_v<M, bbm::ward<C>>) return "Ward";
        else
#endif
#ifdef _BBM_WARD_DUER_H_
        if constexpr (std::is_same_v<M, bbm::wardduer<C>>) return "WardDuer";
        else
#endif
#ifdef _BBM_WARD_DUER_GEISLER_MORODER_H_
        if constexpr (std::is_same_v<M, bbm::wardduergeislermoroder<C>>) return "WardDuerGeislerMoroder";
        else
#endif
#ifdef _BBM_PHONG_H_
        if constexpr (std::is_same_v<M, bbm::phong<C>>) return "Phong";
        else
#endif
#ifdef _BBM_LAFORTUNE_H_
        if constexpr (std::is_same_v<M, bbm::lafortune<C>>) return "Lafortune";
        else
#endif
#ifdef _BBM_ASHIKHMIN_SHIRLEY_H_
        if constexpr (std::is_same_v<M, bbm::ashikhminshirley<C>>) return "AshikhminShirley";
        else
#endif
#ifdef _BBM_ASHIKHMIN_SHIRLEY_FULL_H_
        if constexpr (std::is_same_v<M, bbm::ashikhminshirleyfull<C>>) return "AshikhminShirleyFull";
        else
#endif
#ifdef _BBM_LOW_SMOOTH_H_
        if constexpr (std::is_same_v<M, bbm::lowsmooth<C>>) return "LowSmooth";
        else
#endif
#ifdef _BBM_LOW_MICROFACET_H_
        if constexpr (std::is_same_v<M, bbm::lowmicrofacet<C>>) return "LowMicrofacet";
        else
#endif
#ifdef _BBM_LOW_FITMODELS_H_
        if constexpr (std::is_same_v<M, bbm::lowmicrofacetfit<C>>) return "LowMicrofacetFit";
        else if constexpr (std::is_same_v<M, bbm::lowashikhminshirley<C>>) return "LowAshikhminShirley";
        else
#endif
#ifdef _BBM_BAGHER_H_
        if constexpr (std::is_same_v<M, bbm::bagher<C>>) return "Bagher";
        else
#endif
#ifdef _BBM_HOLZSCHUCHPACANOWSKI_H_
        if constexpr (std::is_same_v<M, bbm::epd<C>>) return "EPD";
        else
#endif
        static_assert(dependent_false<M>::value, "this bsdfmodel composition has no HIP kernel (see DESIGN.md)");
        return nullptr;
      }

#ifdef _BBM_AGGREGATEMODEL_H_
      //! \brief aggregatemodel<lambertian<C>, X> (include/bsdfmodel/aggregatemodel.h:222): the form of every
      //! published fit; the kernel is registered as "Aggregate<Lambertian,X>"
      template<typename M> struct lambertian_aggregate : std::false_type {};
      template<typename C, typename X>
        struct lambertian_aggregate<bbm::aggregatemodel<bbm::lambertian<C>, X>> : std::true_type { using child = X; };
#else
      template<typename M> struct lambertian_aggregate : std::false_type {};
#endif

      //! \brief Registry name of MODEL's kernel (single models and Aggregate(Lambertian, X))
      template<typename MODEL>
        inline std::string registry_name()
      {
        using M = std::decay_t<MODEL>;
        if constexpr (lambertian_aggregate<M>::value)
          return std::string("Aggregate<Lambertian,") + gpu_name<typename lambertian_aggregate<M>::child>() + ">";
        else return gpu_name<M>();
      }
    } // end detail namespace

    //! \brief libbbm_hip model id of MODEL (resolved once per type)
    template<typename MODEL>
      inline int model_id()
    {
      static const int id = [] { int i = bbm_hip_model_id(detail::registry_name<MODEL>().c_str()); check(i); return i; }();
      return id;
    }

    //! \brief Flat parameter vector of a model instance (attribute declaration order)
    template<typename MODEL>
      inline std::vector<float> parameters(const MODEL& model)
    {
      std::vector<float> p;
      for(auto& v : bbm::parameter_values(model, bsdf_attr(0x1F))) p.push_back(float(v));   // All | Dependent
      return p;
    }

    //! \brief eval + pdf of N (in, out) pairs (bsdfmodel::eval / ::pdf batched)
    template<typename MODEL>
      inline void eval_pdf(const MODEL& model, soa3 in, soa3 out, size_t n, soa3_out rgb, float* pdf,
                           bsdf_flag component=bsdf_flag::All, unit_t unit=unit_t::Radiance,
                           const uint8_t* mask=nullptr, void* stream=nullptr)
    {
      auto p = parameters(model);
      check(bbm_hip_eval_pdf(model_id<MODEL>(), p.data(), int(p.size()), in.x, in.y, in.z, out.x, out.y, out.z,
                             mask, n, uint32_t(component), uint32_t(unit), rgb.x, rgb.y, rgb.z, pdf, stream));
    }

    //! \brief eval of N (in, out) pairs -> RGB
    template<typename MODEL>
      inline void eval(const MODEL& model, soa3 in, soa3 out, size_t n, soa3_out rgb,
                       bsdf_flag component=bsdf_flag::All, unit_t unit=unit_t::Radiance,
                       const uint8_t* mask=nullptr, void* stream=nullptr)
    {
      auto p = parameters(model);
      check(bbm_hip_eval(model_id<MODEL>(), p.data(), int(p.size()), in.x, in.y, in.z, out.x, out.y, out.z,
                         mask, n, uint32_t(component), uint32_t(unit), rgb.x, rgb.y, rgb.z, stream));
    }

    //! \brief pdf of N (in, out) pairs
    template<typename MODEL>
      inline void pdf(const MODEL& model, soa3 in, soa3 out, size_t n, float* pdf,
                      bsdf_flag component=bsdf_flag::All, unit_t unit=unit_t::Radiance,
                      const uint8_t* mask=nullptr, void* stream=nullptr)
    {
      auto p = parameters(model);
      check(bbm_hip_pdf(model_id<MODEL>(), p.data(), int(p.size()), in.x, in.y, in.z, out.x, out.y, out.z,
                        mask, n, uint32_t(component), uint32_t(unit), pdf, stream));
    }

    //! \brief sample N (out, xi) -> BsdfSample{direction, pdf, flag} (bsdfmodel::sample batched)
    template<typename MODEL>
      inline void sample(const MODEL& model, soa3 out, const float* xi0, const float* xi1, size_t n,
                         soa3_out direction, float* pdf, uint32_t* flag,
                         bsdf_flag component=bsdf_flag::All, unit_t unit=unit_t::Radiance,
                         const uint8_t* mask=nullptr, void* stream=nullptr)
    {
      auto p = parameters(model);
      check(bbm_hip_sample(model_id<MODEL>(), p.data(), int(p.size()), out.x, out.y, out.z, xi0, xi1, mask, n,
                           uint32_t(component), uint32_t(unit), direction.x, direction.y, direction.z, pdf, flag,
                           stream));
    }

    //! \brief reflectance of N out directions -> RGB (bsdfmodel::reflectance batched)
    template<typename MODEL>
      inline void reflectance(const MODEL& model, soa3 out, size_t n, soa3_out rgb,
                              bsdf_flag component=bsdf_flag::All, unit_t unit=unit_t::Radiance,
                              const uint8_t* mask=nullptr, void* stream=nullptr)
    {
      auto p = parameters(model);
      check(bbm_hip_reflectance(model_id<MODEL>(), p.data(), int(p.size()), out.x, out.y, out.z, mask, n,
                                uint32_t(component), uint32_t(unit), rgb.x, rgb.y, rgb.z, stream));
    }

    //! \brief Sample losses of include/loss/*.h, for loss_sums
    enum class loss_t : int { nganL2 = BBM_LOSS_NGAN_L2, lowL2 = BBM_LOSS_LOW_L2, bieronL2 = BBM_LOSS_BIERON_L2,
                              standardLog = BBM_LOSS_STANDARD_LOG, lowLog = BBM_LOSS_LOW_LOG, bieronLog = BBM_LOSS_BIERON_LOG };

    //! \brief sampledlossfunction<MODEL, reference, loss, linearizer>::operator() (sampledlossfunction.h:62-87)
    //! for nprobes parameter vectors of MODEL's type at once (device array nprobes x parameters(model).size(),
    //! e.g. the 2P probes of a compass step), over n materialised pairs with reference values ref:
    //! sums[p] = sum_i loss(model(probes[p]).eval(in_i, out_i), ref_i) in double (device).  Divide by the
    //! linearizer size (after summing the shards of all GPUs) for the reference's loss value.
    template<typename MODEL>
      inline void loss_sums(const MODEL& model, const float* probes, int nprobes, soa3 in, soa3 out, size_t n,
                            soa3 ref, loss_t loss, double* sums, void* workspace, size_t workspace_bytes,
                            bsdf_flag component=bsdf_flag::All, void* stream=nullptr)
    {
      const int np = int(parameters(model).size());
      check(bbm_hip_loss_pairs(model_id<MODEL>(), probes, np, nprobes, n, in.x, in.y, in.z, out.x, out.y, out.z,
                               ref.x, ref.y, ref.z, int(loss), uint32_t(component), 0u, sums, workspace,
                               workspace_bytes, stream));
    }

  } // end hip namespace
} // end bbm namespace

#endif /* BBM_HIP_BATCH_H */
