/* backbone/hip/include/bbm_hip/batch.h -- C++20 host adapter: bbm::bsdfmodel<> / bsdf_ptr -> libbbm_hip.
 *
 * Header-only, compiled by the BBM user's host compiler (g++/clang) together with the BBM headers and the HIP
 * backbone (backbone/hip/include/backbone.h, selected by BBM_BACKBONE=hip); it never includes HIP device code.
 * A model instance of the reference's template API, e.g.
 *
 *     bbm::cooktorrance<bbm::floatRGB> ct;             // include/bsdfmodel/cooktorrance.h:28-34
 *     bbm::hip::eval_pdf(ct, in, out, n, rgb, pdf);     // N pairs on the GPU
 *
 * is mapped to the HIP backbone in two steps:
 *   1. its *type* is matched against the compositions the kernels implement (cooktorrance<C>, ggx<C>,
 *      lambertian<C>, the He family and Merl behind their data-driven sampler, aggregatemodel<...>) -- a
 *      composition the GPU does not implement is a compile error, never a silent fallback;
 *   2. its attributes are packed with bbm::parameter_values(model, All | Dependent)
 *      (include/bbm/bsdf_enumerate.h), i.e. in declaration order, and passed by value.
 * The runtime handle bsdf_ptr<C> (include/bbm/bsdf_ptr.h:21-165, what checkBsdf and the Mitsuba plugin hold)
 * is mapped through its toString() and the library's parser of the reference's model strings
 * (bbm_hip_parse_model_tree): a single model or fused aggregate runs its kernel, any other aggregate (including
 * the runtime aggregatebsdf, nested to any depth) runs composed from its children's kernels (bbm_hip_aggregate_*).
 * Device buffers are caller-owned SoA float arrays; calls are asynchronous on `stream`.  Errors from the C-ABI
 * are rethrown as bbm::hip::error (a std::runtime_error), matching the reference's exception style
 * (include/core/error.h:42-46).
 */
#ifndef BBM_HIP_BATCH_H
#define BBM_HIP_BATCH_H

#include <cstddef>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "bbm/bsdf_enumerate.h"
#include "bbm_hip.h"

namespace bbm {
  namespace hip {

    //! \brief SoA view of N directions in device memory (x[], y[], z[])
    struct soa3 { const float* x; const float* y; const float* z; };
    //! \brief SoA view of N writable 3-vectors / RGB spectra in device memory
    struct soa3_out { float* x; float* y; float* z; };

    //! \brief The same views over f64 arrays: the doubleRGB configuration (Value = double)
    struct soa3d { const double* x; const double* y; const double* z; };
    struct soa3d_out { double* x; double* y; double* z; };

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

    //! \brief Exact-subnormal mode (bbm_hip_set_exact_subnormals, process-wide): the Beckmann microfacet models'
    //!        eval / pdf bit for bit the reference's floats on every lane; returns the previous setting
    inline bool set_exact_subnormals(bool on)
    {
      const int prev = bbm_hip_set_exact_subnormals(on ? 1 : 0);
      check(prev);
      return prev != 0;
    }

    inline int id_of(const std::string& name)
    {
      const int i = bbm_hip_model_id(name.c_str());
      check(i);
      return i;
    }

    namespace detail {
      template<typename T> struct dependent_false : std::false_type {};

#ifdef _BBM_HE_H_
      //! \brief the he_base<...> (he.h:115-482) a type derives from, with its policy arguments
      template<typename T> struct he_params { static constexpr bool value = false; };
      template<typename C, typename F, bbm::he_eq25 A, bbm::he_eq78 B, size_t NR, size_t TT, bool AD, auto RA, auto NM>
        struct he_params<bbm::he_base<C, F, A, B, NR, TT, AD, RA, NM>>
      {
        static constexpr bool value = true;
        using base = bbm::he_base<C, F, A, B, NR, TT, AD, RA, NM>;
        static constexpr bool complex_fresnel = std::is_same_v<F, bbm::fresnel::complex<C, bbm::Spectrum_t<C>>>;
        static constexpr bool cook_fresnel = std::is_same_v<F, bbm::fresnel::cook<C>>;
        static constexpr bool errata = (A == bbm::he_eq25::Errata), westin = (B == bbm::he_eq78::Westin);
        static constexpr size_t newton = NR, taylor = TT;
        static constexpr bool adaptive = AD;
        static constexpr double approx = double(RA.value);
      };
      template<typename C, typename F, bbm::he_eq25 A, bbm::he_eq78 B, size_t NR, size_t TT, bool AD, auto RA, auto NM>
        he_params<bbm::he_base<C, F, A, B, NR, TT, AD, RA, NM>> he_base_of(const bbm::he_base<C, F, A, B, NR, TT, AD, RA, NM>*);
      he_params<void> he_base_of(...);

      //! \brief registry name of a He-family model: he_base with the policy arguments of he.h:489-496 (or ngan.h:166
      //! for "NganHe*", which the library exposes only with its specular scale), wrapped in the data-driven
      //! backscatter sampler (a bare he_base has no importance sampler of its own and is rejected); nullptr if
      //! W is none of them
      template<typename W>
        constexpr const char* he_name()
      {
        using P = decltype(he_base_of(static_cast<const W*>(nullptr)));
        if constexpr (!P::value) return nullptr;
        else if constexpr (std::is_same_v<W, typename P::base> || P::newton != 4) return nullptr;
        else if constexpr (P::complex_fresnel && !P::errata && !P::westin && P::taylor == 64 && P::adaptive && P::approx == 18.0) return "He";
        else if constexpr (P::complex_fresnel && P::errata && P::westin && P::taylor == 64 && P::adaptive && P::approx == 18.0) return "HeWestin";
        else if constexpr (P::complex_fresnel && P::errata && !P::westin && P::taylor == 10 && !P::adaptive) return "HeHolzschuch";
        else if constexpr (P::cook_fresnel && P::errata && P::westin && P::taylor == 64 && P::adaptive && P::approx == 18.0) return "NganHe*";
        else return nullptr;
      }
#endif

#ifdef _BBM_MERL_H_
      //! \brief merl_data<C, NAME> (staticmodel/merl.h:38-221) a type derives from
      template<typename C, auto NM> std::true_type merl_probe(const bbm::merl_data<C, NM>*);
      std::false_type merl_probe(...);
      template<typename C, auto NM> bbm::merl_data<C, NM> merl_base_of(const bbm::merl_data<C, NM>*);
#endif

#if defined(_BBM_NDF_EPD_H_) && defined(_BBM_MASKINGSHADOWING_VANGINNEKEN_H_)
      template<typename M> struct is_epd : std::false_type {};
      template<typename C, auto NM>
        struct is_epd<bbm::microfacet<bbm::ndf::epd<C>, bbm::maskingshadowing::vanginneken<C>, bbm::fresnel::complex<C>,
                                      bbm::microfacet_n::Walter, NM>> : std::true_type {};
#endif

      //! \brief Registry name of the GPU kernel implementing MODEL's composition.
      template<typename MODEL>
        constexpr const char* gpu_name()
      {
        using C = get_config<MODEL>;
        using M = std::decay_t<MODEL>;
        static_assert(std::is_same_v<Value_t<C>, float> || std::is_same_v<Value_t<C>, double>,
                      "the HIP backbone evaluates floatRGB- and doubleRGB-style configs (Value = float / double)");
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
#if defined(_BBM_NDF_EPD_H_) && defined(_BBM_MASKINGSHADOWING_VANGINNEKEN_H_)
        // EPD (holzschuchpacanowski.h:34-42) by its composition: the alias's normalisation argument is unused there
        if constexpr (is_epd<M>::value) return "EPD";
        else
#endif
#ifdef _BBM_HE_H_
        // He, HeWestin, HeHolzschuch: ndf_sampler<he_base<...>, 90, 1, NAME> (he.h:489-496)
        if constexpr (he_name<M>() != nullptr && he_name<M>()[0] == 'H') return he_name<M>();
        else
#endif
#ifdef _BBM_MERL_H_
        // Merl (merl.h:224-225): the registry entry; its parameters (the table) come from the file, see describe()
        if constexpr (decltype(merl_probe(static_cast<const M*>(nullptr)))::value) return "Merl";
        else
#endif
        static_assert(dependent_false<M>::value, "this bsdfmodel composition has no HIP kernel (see DESIGN.md)");
        return nullptr;
      }

#ifdef _BBM_SCALED_MODEL_H_
      //! \brief NganHe = scaledmodel<ndf_sampler<he_base<CONF, cook, Errata, Westin, 4, 64, true, 18>, 90, 1,
      //! "NganHe">, SpecularScale> (ngan.h:166-167)
      template<typename M> struct scaled_he { static constexpr bool value = false; };
#ifdef _BBM_HE_H_
      template<typename W>
        struct scaled_he<bbm::scaledmodel<W, bbm::bsdf_attr::SpecularScale>>
      {
        static constexpr bool value = he_name<W>() != nullptr && he_name<W>()[0] == 'N';
      };
#endif
#else
      template<typename M> struct scaled_he { static constexpr bool value = false; };
#endif

#ifdef _BBM_AGGREGATEMODEL_H_
      //! \brief aggregatemodel_base<NAME, MODELS...> (aggregatemodel.h:22-214): its children, in order
      template<typename M> struct aggregate_of { static constexpr bool value = false; };
      template<auto NM, typename... X>
        struct aggregate_of<bbm::aggregatemodel_base<NM, X...>> { static constexpr bool value = true; using children = std::tuple<X...>; };
#else
      template<typename M> struct aggregate_of { static constexpr bool value = false; };
#endif

      //! \brief an aggregate with an aggregate child: no fused kernel, and the reference cannot reflect its
      //! attributes as a whole (util/reflection.h:247), so it is described child by child
      template<typename M> struct nested_aggregate : std::false_type {};
#ifdef _BBM_AGGREGATEMODEL_H_
      template<auto NM, typename... X>
        struct nested_aggregate<bbm::aggregatemodel_base<NM, X...>> : std::bool_constant<(aggregate_of<X>::value || ...)> {};
#endif

      //! \brief calls f.template operator()<X>() for every type of a std::tuple<X...> (no instance is built)
      template<typename F, typename... X>
        inline void for_each_type(F&& f, const std::tuple<X...>*) { (f.template operator()<X>(), ...); }

      //! \brief single-kernel registry name of MODEL (single models; Aggregate<A,B,...> names the fused entry
      //! when the library has one, e.g. "Aggregate<Lambertian,NganHe>")
      template<typename MODEL>
        inline std::string single_name()
      {
        using M = std::decay_t<MODEL>;
        if constexpr (scaled_he<M>::value) return "NganHe";
        else if constexpr (aggregate_of<M>::value)
        {
          std::string key;
          for_each_type([&]<typename X>() { key += (key.empty() ? "Aggregate<" : ",") + single_name<X>(); },
                        static_cast<const typename aggregate_of<M>::children*>(nullptr));
          return key + ">";
        }
        else return gpu_name<M>();
      }
    } // end detail namespace

    //! \brief Flat parameter vector of a model instance (attribute declaration order, All | Dependent)
    template<typename MODEL>
      inline std::vector<float> parameters(const MODEL& model)
    {
      std::vector<float> p;
      for(auto& v : bbm::parameter_values(model, bsdf_attr(0x1F))) p.push_back(float(v));
      return p;
    }

    //! \brief The same vector in double (doubleRGB models: the attributes unrounded)
    template<typename MODEL>
      inline std::vector<double> parameters_f64(const MODEL& model)
    {
      std::vector<double> p;
      for(auto& v : bbm::parameter_values(model, bsdf_attr(0x1F))) p.push_back(double(v));
      return p;
    }

#ifdef _BBM_MERL_H_
    namespace detail {
      //! \brief device float4 table of a MERL file (bbm_hip_merl_table), built once per file and kept for the
      //! process's lifetime (the Merl model's parameters are its address)
      inline const float* merl_device_table(const std::string& filename)
      {
        static std::mutex mu;
        static std::map<std::string, void*> tables;
        std::lock_guard<std::mutex> lock(mu);
        auto it = tables.find(filename);
        if(it != tables.end()) return static_cast<const float*>(it->second);
        std::ifstream f(filename, std::ios::binary);
        if(!f) throw error(BBM_HIP_ERR_INVALID_ARG, "unable to open MERL BRDF: " + filename);
        uint32_t dims[3];
        f.read(reinterpret_cast<char*>(dims), sizeof(dims));
        const size_t n = size_t(dims[0]) * dims[1] * dims[2];
        if(!f || n != BBM_HIP_MERL_ENTRIES) throw error(BBM_HIP_ERR_INVALID_ARG, "not a recognized MERL BRDF: " + filename);
        std::vector<double> raw(3 * n);
        f.read(reinterpret_cast<char*>(raw.data()), std::streamsize(raw.size() * sizeof(double)));
        if(!f) throw error(BBM_HIP_ERR_INVALID_ARG, "truncated MERL BRDF: " + filename);
        void* draw = nullptr;
        void* table = nullptr;
        if(hipMalloc(&draw, raw.size() * sizeof(double)) != hipSuccess || hipMalloc(&table, n * 16) != hipSuccess)
          throw error(BBM_HIP_ERR_HIP, "hipMalloc failed for the MERL table");
        if(hipMemcpy(draw, raw.data(), raw.size() * sizeof(double), hipMemcpyHostToDevice) != hipSuccess)
          throw error(BBM_HIP_ERR_HIP, "hipMemcpy failed for the MERL table");
        check(bbm_hip_merl_table(static_cast<const double*>(draw), dims[0], dims[1], dims[2], static_cast<float*>(table), nullptr));
        if(hipDeviceSynchronize() != hipSuccess) throw error(BBM_HIP_ERR_HIP, "MERL table build failed");
        (void)hipFree(draw);
        tables[filename] = table;
        return static_cast<const float*>(table);
      }

      //! \brief filename of a merl_data model from its toString, Merl("...") (merl.h:161-164)
      inline std::string merl_filename(const std::string& s)
      {
        const size_t a = s.find('"'), b = s.rfind('"');
        if(a == std::string::npos || b <= a) throw error(BBM_HIP_ERR_INVALID_ARG, "not a Merl model string: " + s);
        return s.substr(a + 1, b - a - 1);
      }
    } // end detail namespace
#endif

    //! \brief A model as the library sees it: one registry entry (single model / fused aggregate) with its
    //! parameter vector, or a composed aggregate (id = BBM_HIP_AGGREGATE) whose children are model_descs again --
    //! aggregatemodel_base takes any bsdfmodel child (aggregatemodel.h:22), another aggregate included.  T: the
    //! configuration's Value (float: floatRGB, double: doubleRGB).
    template<typename T>
      struct basic_model_desc
    {
      int id = -1;
      std::vector<T> params;
      std::vector<basic_model_desc> kids;
      //! a composed aggregate: the template type's aggregatemodel (BBM_HIP_AGGREGATE) or, from a string / bsdf_ptr,
      //! the runtime aggregatebsdf (BBM_HIP_AGGREGATE_BSDF; a fused one carries BBM_HIP_RUNTIME_AGGREGATE in its id)
      bool composed(void) const { return id == BBM_HIP_AGGREGATE || id == BBM_HIP_AGGREGATE_BSDF; }
    };
    using model_desc = basic_model_desc<float>;
    using model_desc_f64 = basic_model_desc<double>;

    namespace detail {
      template<typename T> struct child_of { using type = bbm_hip_child; };
      template<> struct child_of<double> { using type = bbm_hip_child_f64; };

      //! \brief the C-ABI child arrays of a composed model_desc (nested arrays for nested aggregates), kept alive
      //! as long as this object
      template<typename T>
        struct child_tree
      {
        using child_t = typename child_of<T>::type;
        std::vector<std::vector<child_t>> store;
        const child_t* root = nullptr;
        int count = 0;
        explicit child_tree(const basic_model_desc<T>& m)
        {
          store.reserve(64);
          root = build(m);
          count = int(m.kids.size());
          if(m.id == BBM_HIP_AGGREGATE_BSDF)
          {
            // the runtime aggregate's own semantics at the top level: passed as its root node (include/bbm_hip.h)
            store.push_back(std::vector<child_t>{child_t{BBM_HIP_AGGREGATE_BSDF, nullptr, 0, root, count}});
            root = store.back().data();
            count = 1;
          }
        }
        const child_t* build(const basic_model_desc<T>& m)
        {
          std::vector<child_t> v(m.kids.size());
          for(size_t k = 0; k < m.kids.size(); ++k)
          {
            const auto& c = m.kids[k];
            if(c.composed()) v[k] = child_t{c.id, nullptr, 0, build(c), int(c.kids.size())};
            else v[k] = child_t{c.id, c.params.data(), int(c.params.size()), nullptr, 0};
          }
          if(store.size() == store.capacity()) throw error(BBM_HIP_ERR_INVALID_ARG, "aggregate tree too large");
          store.push_back(std::move(v));      // capacity reserved: earlier arrays never move
          return store.back().data();
        }
      };
    } // end detail namespace

    //! \brief model_desc of a model string (bsdf_ptr toString, a fits/ entry) via the library's parser
    inline model_desc from_string(const std::string& s)
    {
#ifdef _BBM_MERL_H_
      if(s.rfind("Merl(", 0) == 0)
      {
        const float* t = detail::merl_device_table(detail::merl_filename(s));
        const uint64_t v = reinterpret_cast<uint64_t>(t);
        const uint32_t lo = uint32_t(v), hi = uint32_t(v >> 32);
        std::vector<float> p(2);
        std::memcpy(&p[0], &lo, 4);
        std::memcpy(&p[1], &hi, 4);
        return model_desc{id_of("Merl"), p, {}};
      }
#endif
      std::vector<int> ids(256), nk(256), np(256);
      std::vector<float> buf(256 * 64);
      const int k = bbm_hip_parse_model_tree(s.c_str(), ids.data(), nk.data(), buf.data(), np.data(), 256, int(buf.size()));
      check(k);
      // preorder -> tree
      size_t node = 0, off = 0;
      auto take = [&](auto&& self) -> model_desc {
        model_desc d;
        d.id = ids[node];
        d.params.assign(buf.begin() + long(off), buf.begin() + long(off + size_t(np[node])));
        off += size_t(np[node]);
        const int nkids = nk[node++];
        for(int c = 0; c < nkids; ++c) d.kids.push_back(self(self));
        return d;
      };
      model_desc d = take(take);
      if(int(node) != k) throw error(BBM_HIP_ERR_INVALID_ARG, "malformed model tree from the parser");
      return d;
    }

    //! \brief model_desc of a model instance, resolved by type (compile-time dispatch); T = float for floatRGB
    //! models (float32 entry points), double for doubleRGB models (the *_f64 entry points)
    template<typename T, typename MODEL>
      inline basic_model_desc<T> describe_as(const MODEL& model)
    {
      using M = std::decay_t<MODEL>;
      static_assert(std::is_same_v<Value_t<get_config<M>>, T>, "the model's Value type must match the entry points");
#ifdef _BBM_MERL_H_
      // Merl: ndf_sampler<merl_data<C, "Merl">, 90, 1> (staticmodel/merl.h:224-225), identified by its file
      // (toString, merl.h:161-164); a bare merl_data (placeholder sampler, merl.h:108-115) is rejected
      if constexpr (!detail::scaled_he<M>::value && !detail::aggregate_of<M>::value &&
                    decltype(detail::merl_probe(static_cast<const M*>(nullptr)))::value)
      {
        static_assert(!std::is_same_v<M, decltype(detail::merl_base_of(static_cast<const M*>(nullptr)))>,
                      "merl_data without its data-driven sampler has no HIP kernel; use bbm::merl<CONF>");
        static_assert(std::is_same_v<T, float>, "Merl is a floatRGB model on the device (DESIGN.md §7)");
        return from_string(bbm::toString(model));
      }
      else
#endif
      if constexpr (detail::aggregate_of<M>::value)
      {
        if constexpr (!detail::nested_aggregate<M>::value)
        {
          const std::string key = detail::single_name<M>();
          const int fused = bbm_hip_model_id(key.c_str());
          if(fused >= 0)
          {
            if constexpr (std::is_same_v<T, float>) return basic_model_desc<T>{fused, parameters(model), {}};
            else return basic_model_desc<T>{fused, parameters_f64(model), {}};
          }
        }
        // composed: each child (a base class of the aggregate) with its own kernel(s) -- a nested aggregate stays
        // one child, composed in turn
        basic_model_desc<T> d;
        d.id = BBM_HIP_AGGREGATE;
        detail::for_each_type([&]<typename X>() { d.kids.push_back(describe_as<T>(static_cast<const X&>(model))); },
                              static_cast<const typename detail::aggregate_of<M>::children*>(nullptr));
        return d;
      }
      else
      {
        if constexpr (std::is_same_v<T, float>) return basic_model_desc<T>{id_of(detail::single_name<M>()), parameters(model), {}};
        else return basic_model_desc<T>{id_of(detail::single_name<M>()), parameters_f64(model), {}};
      }
    }

    template<typename MODEL>
      inline model_desc describe(const MODEL& model)
    {
      static_assert(std::is_same_v<Value_t<get_config<std::decay_t<MODEL>>>, float>,
                    "float32 entry points take floatRGB-style models; doubleRGB models use the soa3d overloads");
      return describe_as<float>(model);
    }

    namespace detail {
      //! the template type's semantics all the way down: aggregatemodel nodes and plain fused ids
      template<typename T>
        inline void as_template(basic_model_desc<T>& d)
      {
        if(d.id == BBM_HIP_AGGREGATE_BSDF) d.id = BBM_HIP_AGGREGATE;
        else if(d.id >= 0) d.id &= ~BBM_HIP_RUNTIME_AGGREGATE;
        for(auto& k : d.kids) as_template(k);
      }
    } // end detail namespace

#ifdef _BBM_BSDF_PTR_H_
    //! \brief bsdf_ptr<C> (include/bbm/bsdf_ptr.h:21-165): through its toString (bsdf.h:111-116 pipes the
    //! wrapped model's) and the library's parser.  The string of a bsdf<aggregatemodel<...>> and of the runtime
    //! aggregatebsdf (aggregatebsdf.h:40-190, what fromString<bsdf_ptr> builds) read alike, but they round the
    //! pdf differently and sample differently: the wrapped object decides -- an aggregatebsdf keeps the parser's
    //! runtime semantics (its children are the bsdf_ptrs its string describes), anything else is a template
    //! model, aggregatemodel at every level.
    //! Limitation: only the root is inspected.  Below a runtime root every aggregate child keeps runtime semantics,
    //! also one whose bsdf_ptr wraps a template bsdf<aggregatemodel<...>> (the string alone cannot tell them apart
    //! and aggregatebsdf exposes no accessor for its children); such a child's pdf rounding and its sum <= eps
    //! sampling rule then follow aggregatebsdf.  Build that child from its model type (describe(model)) where it
    //! matters.
    template<typename C>
      inline model_desc describe(const bbm::bsdf_ptr<C>& ptr)
    {
      model_desc d = from_string(ptr.toString());
#ifdef _BBM_AGGREGATEBSDF_H_
      const bool runtime = dynamic_cast<const bbm::aggregatebsdf<C>*>(ptr.ptr().get()) != nullptr;
#else
      const bool runtime = false;      // aggregatebsdf.h not included: no runtime aggregate can exist
#endif
      if(!runtime) detail::as_template(d);
      return d;
    }
#endif

    //! \brief libbbm_hip model id of MODEL's single kernel (resolved once per type)
    template<typename MODEL>
      inline int model_id()
    {
      static const int id = id_of(detail::single_name<MODEL>());
      return id;
    }

    //! \brief eval + pdf of N (in, out) pairs (bsdfmodel::eval / ::pdf batched)
    inline void eval_pdf(const model_desc& m, soa3 in, soa3 out, size_t n, soa3_out rgb, float* pdf,
                         bsdf_flag component=bsdf_flag::All, unit_t unit=unit_t::Radiance,
                         const uint8_t* mask=nullptr, void* stream=nullptr)
    {
      if(m.composed())
      {
        const detail::child_tree<float> c(m);
        check(bbm_hip_aggregate_eval_pdf(c.root, c.count, in.x, in.y, in.z, out.x, out.y, out.z, mask, n,
                                         uint32_t(component), uint32_t(unit), rgb.x, rgb.y, rgb.z, pdf, stream));
      }
      else
        check(bbm_hip_eval_pdf(m.id, m.params.data(), int(m.params.size()), in.x, in.y, in.z, out.x, out.y,
                               out.z, mask, n, uint32_t(component), uint32_t(unit), rgb.x, rgb.y, rgb.z, pdf, stream));
    }

    //! \brief eval of N (in, out) pairs -> RGB
    inline void eval(const model_desc& m, soa3 in, soa3 out, size_t n, soa3_out rgb,
                     bsdf_flag component=bsdf_flag::All, unit_t unit=unit_t::Radiance,
                     const uint8_t* mask=nullptr, void* stream=nullptr)
    {
      if(m.composed())
      {
        const detail::child_tree<float> c(m);
        check(bbm_hip_aggregate_eval_pdf(c.root, c.count, in.x, in.y, in.z, out.x, out.y, out.z, mask, n,
                                         uint32_t(component), uint32_t(unit), rgb.x, rgb.y, rgb.z, nullptr, stream));
      }
      else
        check(bbm_hip_eval(m.id, m.params.data(), int(m.params.size()), in.x, in.y, in.z, out.x, out.y,
                           out.z, mask, n, uint32_t(component), uint32_t(unit), rgb.x, rgb.y, rgb.z, stream));
    }

    //! \brief pdf of N (in, out) pairs
    inline void pdf(const model_desc& m, soa3 in, soa3 out, size_t n, float* pdf,
                    bsdf_flag component=bsdf_flag::All, unit_t unit=unit_t::Radiance,
                    const uint8_t* mask=nullptr, void* stream=nullptr)
    {
      if(m.composed())
      {
        const detail::child_tree<float> c(m);
        check(bbm_hip_aggregate_eval_pdf(c.root, c.count, in.x, in.y, in.z, out.x, out.y, out.z, mask, n,
                                         uint32_t(component), uint32_t(unit), nullptr, nullptr, nullptr, pdf, stream));
      }
      else
        check(bbm_hip_pdf(m.id, m.params.data(), int(m.params.size()), in.x, in.y, in.z, out.x, out.y,
                          out.z, mask, n, uint32_t(component), uint32_t(unit), pdf, stream));
    }

    //! \brief sample N (out, xi) -> BsdfSample{direction, pdf, flag} (bsdfmodel::sample batched)
    inline void sample(const model_desc& m, soa3 out, const float* xi0, const float* xi1, size_t n,
                       soa3_out direction, float* pdf, uint32_t* flag,
                       bsdf_flag component=bsdf_flag::All, unit_t unit=unit_t::Radiance,
                       const uint8_t* mask=nullptr, void* stream=nullptr)
    {
      if(m.composed())
      {
        const detail::child_tree<float> c(m);
        check(bbm_hip_aggregate_sample(c.root, c.count, out.x, out.y, out.z, xi0, xi1, mask, n,
                                       uint32_t(component), uint32_t(unit), direction.x, direction.y, direction.z, pdf,
                                       flag, stream));
      }
      else
        check(bbm_hip_sample(m.id, m.params.data(), int(m.params.size()), out.x, out.y, out.z, xi0, xi1, mask,
                             n, uint32_t(component), uint32_t(unit), direction.x, direction.y, direction.z, pdf, flag,
                             stream));
    }

    //! \brief reflectance of N out directions -> RGB (bsdfmodel::reflectance batched)
    inline void reflectance(const model_desc& m, soa3 out, size_t n, soa3_out rgb,
                            bsdf_flag component=bsdf_flag::All, unit_t unit=unit_t::Radiance,
                            const uint8_t* mask=nullptr, void* stream=nullptr)
    {
      if(m.composed())
      {
        const detail::child_tree<float> c(m);
        check(bbm_hip_aggregate_reflectance(c.root, c.count, out.x, out.y, out.z, mask, n, uint32_t(component),
                                            uint32_t(unit), rgb.x, rgb.y, rgb.z, stream));
      }
      else
        check(bbm_hip_reflectance(m.id, m.params.data(), int(m.params.size()), out.x, out.y, out.z, mask, n,
                                  uint32_t(component), uint32_t(unit), rgb.x, rgb.y, rgb.z, stream));
    }

    // The same entry points on a model instance (template API) or a bsdf_ptr: resolved, then dispatched.
    template<typename MODEL>
      inline void eval_pdf(const MODEL& model, soa3 in, soa3 out, size_t n, soa3_out rgb, float* p,
                           bsdf_flag component=bsdf_flag::All, unit_t unit=unit_t::Radiance,
                           const uint8_t* mask=nullptr, void* stream=nullptr)
    { eval_pdf(describe(model), in, out, n, rgb, p, component, unit, mask, stream); }

    template<typename MODEL>
      inline void eval(const MODEL& model, soa3 in, soa3 out, size_t n, soa3_out rgb,
                       bsdf_flag component=bsdf_flag::All, unit_t unit=unit_t::Radiance,
                       const uint8_t* mask=nullptr, void* stream=nullptr)
    { eval(describe(model), in, out, n, rgb, component, unit, mask, stream); }

    template<typename MODEL>
      inline void pdf(const MODEL& model, soa3 in, soa3 out, size_t n, float* p,
                      bsdf_flag component=bsdf_flag::All, unit_t unit=unit_t::Radiance,
                      const uint8_t* mask=nullptr, void* stream=nullptr)
    { pdf(describe(model), in, out, n, p, component, unit, mask, stream); }

    template<typename MODEL>
      inline void sample(const MODEL& model, soa3 out, const float* xi0, const float* xi1, size_t n,
                         soa3_out direction, float* p, uint32_t* flag,
                         bsdf_flag component=bsdf_flag::All, unit_t unit=unit_t::Radiance,
                         const uint8_t* mask=nullptr, void* stream=nullptr)
    { sample(describe(model), out, xi0, xi1, n, direction, p, flag, component, unit, mask, stream); }

    template<typename MODEL>
      inline void reflectance(const MODEL& model, soa3 out, size_t n, soa3_out rgb,
                              bsdf_flag component=bsdf_flag::All, unit_t unit=unit_t::Radiance,
                              const uint8_t* mask=nullptr, void* stream=nullptr)
    { reflectance(describe(model), out, n, rgb, component, unit, mask, stream); }

    //! \brief doubleRGB (Value = double) model_desc on f64 SoA arrays: eval + pdf evaluated in f64 on the device
    //! (bbm_hip_eval_pdf_f64, or bbm_hip_aggregate_eval_pdf_f64 for a composed aggregate).  Every leaf must have
    //! doubleRGB kernels (bbm_hip_model_has_f64: every analytic model and their Aggregate(Lambertian, X) fits);
    //! any other is rejected with BBM_HIP_ERR_UNSUPPORTED.
    inline void eval_pdf(const model_desc_f64& m, soa3d in, soa3d out, size_t n, soa3d_out rgb, double* p,
                         bsdf_flag component=bsdf_flag::All, unit_t unit=unit_t::Radiance,
                         const uint8_t* mask=nullptr, void* stream=nullptr)
    {
      if(m.composed())
      {
        const detail::child_tree<double> c(m);
        check(bbm_hip_aggregate_eval_pdf_f64(c.root, c.count, in.x, in.y, in.z, out.x, out.y, out.z, mask, n,
                                             uint32_t(component), uint32_t(unit), rgb.x, rgb.y, rgb.z, p, stream));
      }
      else
        check(bbm_hip_eval_pdf_f64(m.id, m.params.data(), int(m.params.size()), in.x, in.y, in.z, out.x, out.y, out.z,
                                   mask, n, uint32_t(component), uint32_t(unit), rgb.x, rgb.y, rgb.z, p, stream));
    }

    //! \brief doubleRGB sample of N (out, xi) -> direction, pdf, flag (bbm_hip_sample_f64 / _aggregate_sample_f64)
    inline void sample(const model_desc_f64& m, soa3d out, const double* xi0, const double* xi1, size_t n,
                       soa3d_out direction, double* p, uint32_t* flag,
                       bsdf_flag component=bsdf_flag::All, unit_t unit=unit_t::Radiance,
                       const uint8_t* mask=nullptr, void* stream=nullptr)
    {
      if(m.composed())
      {
        const detail::child_tree<double> c(m);
        check(bbm_hip_aggregate_sample_f64(c.root, c.count, out.x, out.y, out.z, xi0, xi1, mask, n, uint32_t(component),
                                           uint32_t(unit), direction.x, direction.y, direction.z, p, flag, stream));
      }
      else
        check(bbm_hip_sample_f64(m.id, m.params.data(), int(m.params.size()), out.x, out.y, out.z, xi0, xi1, mask, n,
                                 uint32_t(component), uint32_t(unit), direction.x, direction.y, direction.z, p, flag, stream));
    }

    //! \brief doubleRGB reflectance of N out directions (bbm_hip_reflectance_f64 / _aggregate_reflectance_f64)
    inline void reflectance(const model_desc_f64& m, soa3d out, size_t n, soa3d_out rgb,
                            bsdf_flag component=bsdf_flag::All, unit_t unit=unit_t::Radiance,
                            const uint8_t* mask=nullptr, void* stream=nullptr)
    {
      if(m.composed())
      {
        const detail::child_tree<double> c(m);
        check(bbm_hip_aggregate_reflectance_f64(c.root, c.count, out.x, out.y, out.z, mask, n, uint32_t(component),
                                                uint32_t(unit), rgb.x, rgb.y, rgb.z, stream));
      }
      else
        check(bbm_hip_reflectance_f64(m.id, m.params.data(), int(m.params.size()), out.x, out.y, out.z, mask, n,
                                      uint32_t(component), uint32_t(unit), rgb.x, rgb.y, rgb.z, stream));
    }

    // ... and on doubleRGB model instances (template API), single, fused or composed
    template<typename MODEL> requires std::is_same_v<Value_t<get_config<std::decay_t<MODEL>>>, double>
      inline void eval_pdf(const MODEL& model, soa3d in, soa3d out, size_t n, soa3d_out rgb, double* p,
                           bsdf_flag component=bsdf_flag::All, unit_t unit=unit_t::Radiance,
                           const uint8_t* mask=nullptr, void* stream=nullptr)
    { eval_pdf(describe_as<double>(model), in, out, n, rgb, p, component, unit, mask, stream); }

    template<typename MODEL> requires std::is_same_v<Value_t<get_config<std::decay_t<MODEL>>>, double>
      inline void sample(const MODEL& model, soa3d out, const double* xi0, const double* xi1, size_t n,
                         soa3d_out direction, double* p, uint32_t* flag,
                         bsdf_flag component=bsdf_flag::All, unit_t unit=unit_t::Radiance,
                         const uint8_t* mask=nullptr, void* stream=nullptr)
    { sample(describe_as<double>(model), out, xi0, xi1, n, direction, p, flag, component, unit, mask, stream); }

    template<typename MODEL> requires std::is_same_v<Value_t<get_config<std::decay_t<MODEL>>>, double>
      inline void reflectance(const MODEL& model, soa3d out, size_t n, soa3d_out rgb,
                              bsdf_flag component=bsdf_flag::All, unit_t unit=unit_t::Radiance,
                              const uint8_t* mask=nullptr, void* stream=nullptr)
    { reflectance(describe_as<double>(model), out, n, rgb, component, unit, mask, stream); }

    //! \brief Sample losses of include/loss/*.h, for loss_sums
    enum class loss_t : int { nganL2 = BBM_LOSS_NGAN_L2, lowL2 = BBM_LOSS_LOW_L2, bieronL2 = BBM_LOSS_BIERON_L2,
                              standardLog = BBM_LOSS_STANDARD_LOG, lowLog = BBM_LOSS_LOW_LOG, bieronLog = BBM_LOSS_BIERON_LOG };

    //! \brief sampledlossfunction<MODEL, reference, loss, linearizer>::operator() (sampledlossfunction.h:62-87)
    //! for nprobes parameter vectors of MODEL's type at once (device array nprobes x parameters(model).size(),
    //! e.g. the 2P probes of a compass step), over n materialised pairs with reference values ref:
    //! sums[p] = sum_i loss(model(probes[p]).eval(in_i, out_i), ref_i) in double (device).  Divide by the
    //! linearizer size (after summing the shards of all GPUs) for the reference's loss value.  MODEL must have a
    //! single kernel (single model or fused aggregate).
    //! COMPONENT and UNIT are sampledlossfunction's template arguments (sampledlossfunction.h:34, :70-71).
    template<typename MODEL>
      inline void loss_sums(const MODEL& model, const float* probes, int nprobes, soa3 in, soa3 out, size_t n,
                            soa3 ref, loss_t loss, double* sums, void* workspace, size_t workspace_bytes,
                            bsdf_flag component=bsdf_flag::All, unit_t unit=unit_t::Radiance, void* stream=nullptr)
    {
      const int np = int(parameters(model).size());
      check(bbm_hip_loss_pairs(model_id<MODEL>(), probes, np, nprobes, n, in.x, in.y, in.z, out.x, out.y, out.z,
                               ref.x, ref.y, ref.z, int(loss), uint32_t(component), uint32_t(unit), sums, workspace,
                               workspace_bytes, stream));
    }

  } // end hip namespace
} // end bbm namespace

#endif /* BBM_HIP_BATCH_H */
