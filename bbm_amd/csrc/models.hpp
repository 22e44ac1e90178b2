// bbm_amd/csrc/models.hpp -- the model compositions the library implements (one line per
// reference model, file:line of its definition), and the X-macro lists the instantiation units
// and the registry iterate over.
#pragma once
#include "diffuse.hpp"
#include "lobes.hpp"
#include "microfacet.hpp"
#include "spectral.hpp"
#include "aggregate.hpp"
#include "epd.hpp"
#include "he.hpp"
#include "merl.hpp"

#include <type_traits>

namespace bbmhip {

// Launch traits of the eval kernels (kernels.hpp), specialised here where every model type is complete.
// Aggregate(Lambertian, X) is zero outside the upper hemisphere and on masked lanes whenever X is (Lambertian's
// eval and pdf both need z(in), z(out) > 0), so it shares X's compaction and occupancy choices.
template<class B> struct compact_eval<Aggregate<Lambertian, B>> { static constexpr bool value = compact_eval<B>::value; };
template<class B> struct eval_waves<Aggregate<Lambertian, B>> { static constexpr int value = eval_waves<B>::value; };
template<class B> struct loss_waves<Aggregate<Lambertian, B>> { static constexpr int value = loss_waves<B>::value; };
template<class B> struct eval_grid_cap<Aggregate<Lambertian, B>> { static constexpr uint64_t value = eval_grid_cap<B>::value; };
template<class B> struct eval_prefetch<Aggregate<Lambertian, B>> { static constexpr bool value = eval_prefetch<B>::value; };
template<class FRES, bool ERRATA, bool WESTIN, int TAYLOR, bool ADAPTIVE, int APPROX, bool SCALED>
struct loss_waves<He<FRES, ERRATA, WESTIN, TAYLOR, ADAPTIVE, APPROX, SCALED>> { static constexpr int value = 1; };
template<class B> struct loss_pair_waves<Aggregate<Lambertian, B>> { static constexpr int value = loss_pair_waves<B>::value; };
template<class B> struct check_waves<Aggregate<Lambertian, B>> { static constexpr int value = check_waves<B>::value; };
template<class FRES, bool ERRATA, bool WESTIN, int TAYLOR, bool ADAPTIVE, int APPROX, bool SCALED>
struct check_waves<He<FRES, ERRATA, WESTIN, TAYLOR, ADAPTIVE, APPROX, SCALED>> { static constexpr int value = 1; };
template<> struct check_waves<EpdM> { static constexpr int value = 1; };
template<class FRES, bool ERRATA, bool WESTIN, int TAYLOR, bool ADAPTIVE, int APPROX, bool SCALED>
struct loss_pair_waves<He<FRES, ERRATA, WESTIN, TAYLOR, ADAPTIVE, APPROX, SCALED>> { static constexpr int value = 1; };
// Bagher's fitting loss (config 5) runs at 8 waves per SIMD: 64 VGPRs with ~55 of the per-sample decode state spilled
// to scratch (read back once per probe pair from L1), against 128 VGPRs and no spills at 4.  The kernel is
// latency-bound (issue 0.40), so the doubled occupancy outweighs the spill traffic.  Measured on config 5, ms per
// compass step, interleaved (profiles/r04_ab_fit_loss_waves*.txt): 4 waves 0.591, 5 0.618, 6 0.572, 7 0.588,
// 8 0.554; at 8 waves 3 or 4 probes per iteration 0.559 / 0.567, the probe models staged in LDS 0.566.
#ifndef BBM_HIP_BAGHER_LOSS_WAVES
#define BBM_HIP_BAGHER_LOSS_WAVES 8
#endif
template<> struct loss_pair_waves<Bagher> { static constexpr int value = BBM_HIP_BAGHER_LOSS_WAVES; };
// Bagher's evaluation holds ~180 VGPRs (two waves per SIMD) unconstrained.  Measured (10M pairs, eval+pdf,
// tools/gpu_ab_he.sh): Bagher 0.238 / 0.203 / 0.262 ms and Aggregate(Lambertian, Bagher) 0.266 / 0.231 / 0.324 ms
// at 2 / 3 / 4 waves per SIMD -- three it is.
#ifndef BBM_HIP_BAGHER_WAVES
#define BBM_HIP_BAGHER_WAVES 3
#endif
template<> struct eval_waves<Bagher> { static constexpr int value = BBM_HIP_BAGHER_WAVES; };
template<> struct eval_prefetch<Bagher> { static constexpr bool value = false; };
#ifdef BBM_HIP_BAGHER_COMPACT
template<> struct compact_eval<Bagher> { static constexpr bool value = true; };   // A/B
#endif
#ifdef BBM_HIP_MERL_WAVES
template<> struct eval_waves<Merl> { static constexpr int value = BBM_HIP_MERL_WAVES; };   // A/B
#endif
#ifdef BBM_HIP_EPD_WAVES
template<> struct eval_waves<EpdM> { static constexpr int value = BBM_HIP_EPD_WAVES; };   // A/B
#endif

// Ribardiere's per-thread Student-T setup (two tgamma, a pow): 2048 workgroups (8 per CU, each thread ~5 iterations
// over 10M pairs) measured 0.139 -> 0.121 ms per 10M-pair eval (1024 / 4096 / 8192: 0.125 / 0.128 / 0.134;
// tools/gpu_ab_blocks.sh); the HBM-bound models lose 5-15 % under the same cap and keep the full grid.

// Compositions (reference file:line):
using CookTorranceM = Microfacet<Beckmann<false, false>, VGroove, FresnelCook, Norm::Cook, true>;         // bsdfmodel/cooktorrance.h:28-34
#ifdef BBM_HIP_CT_WAVES
template<> struct eval_waves<CookTorranceM> { static constexpr int value = BBM_HIP_CT_WAVES; };   // A/B
#endif
using GGXM = Microfacet<GGX<false>, Uncorrelated, FresnelCook, Norm::Walter, true>;                        // bsdfmodel/ggx.h:27-33
using CookTorranceWalterM = Microfacet<Beckmann<false, true>, Uncorrelated, FresnelCook, Norm::Walter, true>;  // bsdfmodel/cooktorrancewalter.h:32-38

using CookTorranceHeitzM = Microfacet<Beckmann<true, true>, HeightCorrelated, FresnelCook, Norm::Walter, true>;   // bsdfmodel/cooktorranceheitz.h:33-39
using GGXHeitzM = Microfacet<GGX<true>, HeightCorrelated, FresnelCook, Norm::Walter, true>;                     // bsdfmodel/ggxheitz.h:28-34
// eval reads no glibc table (GGX's D, G1 and FresnelCook are rational / sqrt; Lambertian is a constant)
template<> struct uses_math_tables<Lambertian> { static constexpr bool value = false; };
template<> struct uses_math_tables<GGXM> { static constexpr bool value = false; };
template<> struct uses_math_tables<GGXHeitzM> { static constexpr bool value = false; };
using NganCookTorranceM = Microfacet<Beckmann<false, true>, VGroove, FresnelSchlick, Norm::Cook, true>;         // bsdfmodel/ngan.h:141-147
using PhongWalterM = Microfacet<PhongNdf, Uncorrelated, FresnelCook, Norm::Walter, true>;                         // bsdfmodel/phongwalter.h:27-33
#ifdef BBM_HIP_MIDTIER_WAVES   // A/B: the mid-tier microfacet variants' occupancy
template<> struct eval_waves<CookTorranceWalterM> { static constexpr int value = BBM_HIP_MIDTIER_WAVES; };
template<> struct eval_waves<CookTorranceHeitzM> { static constexpr int value = BBM_HIP_MIDTIER_WAVES; };
template<> struct eval_waves<PhongWalterM> { static constexpr int value = BBM_HIP_MIDTIER_WAVES; };
#endif
#ifdef BBM_HIP_MIDTIER_PIPE     // A/B: software-pipelined loop on a capped grid
template<> struct eval_pipeline<CookTorranceWalterM> { static constexpr bool value = true; };
template<> struct eval_pipeline<CookTorranceHeitzM> { static constexpr bool value = true; };
template<> struct eval_pipeline<PhongWalterM> { static constexpr bool value = true; };
template<> struct eval_grid_cap<CookTorranceWalterM> { static constexpr uint64_t value = BBM_HIP_MIDTIER_PIPE; };
template<> struct eval_grid_cap<CookTorranceHeitzM> { static constexpr uint64_t value = BBM_HIP_MIDTIER_PIPE; };
template<> struct eval_grid_cap<PhongWalterM> { static constexpr uint64_t value = BBM_HIP_MIDTIER_PIPE; };
#endif
#ifdef BBM_HIP_MIDTIER_NOPF     // A/B: their first-quad prefetch
template<> struct eval_prefetch<CookTorranceWalterM> { static constexpr bool value = false; };
template<> struct eval_prefetch<CookTorranceHeitzM> { static constexpr bool value = false; };
template<> struct eval_prefetch<PhongWalterM> { static constexpr bool value = false; };
#endif
using RibardiereM = Microfacet<StudentT<false>, Uncorrelated, FresnelCook, Norm::Walter, true>;                   // bsdfmodel/ribardiere.h:28-34
using RibardiereAnisoM = Microfacet<StudentT<true>, Uncorrelated, FresnelCook, Norm::Walter, true>;              // bsdfmodel/ribardiere.h:46-52

using LowMicrofacetM = Microfacet<LowNdf, VGroove, FresnelCook, Norm::Cook, true>;                             // bsdfmodel/lowmicrofacet.h:37-70, low.h:40-41
template<> struct eval_grid_cap<RibardiereM> { static constexpr uint64_t value = 2048; };
template<> struct eval_grid_cap<RibardiereAnisoM> { static constexpr uint64_t value = 2048; };
using WardM = Ward<0, true>;                  // bsdfmodel/ward.h:26-168
using WardDuerM = Ward<1, true>;              // bsdfmodel/wardduer.h:29-81
using WardDGMM = Ward<2, true>;               // bsdfmodel/wardduergeislermoroder.h:29-81
using NganWardM = Ward<0, false>;             // bsdfmodel/ngan.h:30-31
using NganWardDuerM = Ward<1, false>;         // bsdfmodel/ngan.h:37-38
using LafortuneM = Lafortune<true, false>;    // bsdfmodel/lafortune.h:28-172
using NganLafortuneM = Lafortune<false, true>;   // bsdfmodel/ngan.h:54-129
using ASM = AshikhminShirley<FresnelSchlickRGB, true, false, false>;                       // ashikhminshirley.h:29-221
using ASFullM = AshikhminShirley<FresnelSchlickRGB, true, false, true>;                    // ashikhminshirleyfull.h:31-191
using LowASM = AshikhminShirley<ScalarFresnel3<FresnelCook>, false, true, false>;          // bsdfmodel/low.h:24-25
using NganASM = AshikhminShirley<ScalarFresnel3<FresnelSchlick>, false, true, false>;      // bsdfmodel/ngan.h:157-158

// Aggregate(Lambertian, X): the form of every published fit (fits/*.fit), aggregatemodel.h:22-233
using AggBagherM = Aggregate<Lambertian, Bagher>;
using AggCookTorranceM = Aggregate<Lambertian, CookTorranceM>;
using AggGGXM = Aggregate<Lambertian, GGXM>;
template<> struct uses_math_tables<AggGGXM> { static constexpr bool value = false; };
using AggLowASM = Aggregate<Lambertian, LowASM>;
using AggLowMicrofacetM = Aggregate<Lambertian, LowMicrofacetM>;
using AggLowSmoothM = Aggregate<Lambertian, LowSmooth>;
using AggNganASM = Aggregate<Lambertian, NganASM>;
using AggPhongM = Aggregate<Lambertian, PhongLobe>;
using AggNganCookTorranceM = Aggregate<Lambertian, NganCookTorranceM>;
using AggNganLafortuneM = Aggregate<Lambertian, NganLafortuneM>;
using AggNganWardM = Aggregate<Lambertian, NganWardM>;
using AggNganWardDuerM = Aggregate<Lambertian, NganWardDuerM>;
using AggNganHeM = Aggregate<Lambertian, NganHeM>;    // fits/ngan_he.fit

// An aggregate's per-launch derived data is its children's (the He family's sampling CDF): B's block starts
// after A's parameters, and B's derived slots (B::kParams + ...) are then exactly the aggregate's own
// (A::kParams + B::kParams + ...), where B's device constructor (p + A::kParams) finds them.
template<class A, class B>
struct host_params<Aggregate<A, B>>
{
  static_assert(std::is_same_v<A, Lambertian>, "fused aggregates have a Lambertian first child");
  static int run(ParamBlock& p, uint32_t component, hipStream_t s, void** scratch)
  {
    ParamBlock q{};
    for (int k = A::kParams; k < kMaxParams; ++k) q.v[k - A::kParams] = p.v[k];
    if (const int rc = host_params<B>::run(q, component, s, scratch)) return rc;
    for (int k = A::kParams; k < kMaxParams; ++k) p.v[k] = q.v[k - A::kParams];
    return 0;
  }
  static void done(void* scratch, hipStream_t s) { host_params<B>::done(scratch, s); }
};

}  // namespace bbmhip

// X(composition) per instantiation unit
#define BBM_HIP_MICROFACET_MODELS(X) \
  X(CookTorranceM) X(GGXM) X(CookTorranceWalterM) X(CookTorranceHeitzM) X(GGXHeitzM) X(NganCookTorranceM) \
  X(PhongWalterM) X(RibardiereM) X(RibardiereAnisoM) X(LowMicrofacetM)
#define BBM_HIP_LOBE_MODELS(X) \
  X(WardM) X(WardDuerM) X(WardDGMM) X(NganWardM) X(NganWardDuerM) X(PhongLobe) X(LafortuneM) X(NganLafortuneM) \
  X(ASM) X(ASFullM) X(LowASM) X(NganASM) X(LowSmooth)
#define BBM_HIP_DIFFUSE_MODELS(X) X(Lambertian) X(OrenNayar)
#define BBM_HIP_SPECTRAL_MODELS(X) X(Bagher)
#define BBM_HIP_EPD_MODELS(X) X(EpdM)
#define BBM_HIP_HE_MODELS(X) X(HeM) X(HeWestinM) X(HeHolzschuchM) X(NganHeM)
#define BBM_HIP_MERL_MODELS(X) X(Merl)
#define BBM_HIP_AGGREGATE_MODELS(X) \
  X(AggBagherM) X(AggCookTorranceM) X(AggGGXM) X(AggLowASM) X(AggLowMicrofacetM) X(AggLowSmoothM) X(AggNganASM) \
  X(AggPhongM) X(AggNganCookTorranceM) X(AggNganLafortuneM) X(AggNganWardM) X(AggNganWardDuerM) X(AggNganHeM)

#define BBM_HIP_INSTANTIATE(M)                                                   \
  template int launch_eval_pdf<M>(const EvalArgs&, int, hipStream_t);           \
  template int launch_sample<M>(const SampleArgs&, hipStream_t);                \
  template int launch_reflectance<M>(const ReflArgs&, hipStream_t);            \
  template int launch_loss<M>(const LossArgs&, hipStream_t);                  \
  template int launch_check<M>(int, const CheckArgs&, double*, hipStream_t);
#define BBM_HIP_EXTERN(M)                                                        \
  extern template int launch_eval_pdf<M>(const EvalArgs&, int, hipStream_t);    \
  extern template int launch_sample<M>(const SampleArgs&, hipStream_t);         \
  extern template int launch_reflectance<M>(const ReflArgs&, hipStream_t);     \
  extern template int launch_loss<M>(const LossArgs&, hipStream_t);           \
  extern template int launch_check<M>(int, const CheckArgs&, double*, hipStream_t);
