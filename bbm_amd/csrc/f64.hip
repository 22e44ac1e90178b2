// bbm_amd/csrc/f64.hip -- doubleRGB kernels (f64.hpp) and their registry by model name.
#include <hip/hip_runtime.h>
#include <cstring>
#include <string>

#include "../../include/bbm_hip.h"
#include "f64.hpp"

namespace bbmhip {

int fail(int code, const std::string& msg);
std::string scratch_failure();

namespace f64 {
namespace {

constexpr int kBlock = 256;
constexpr uint64_t kMaxBlocks = 1u << 20;

typedef double dv2 __attribute__((ext_vector_type(2)));

// V pairs per thread-iteration: V = 2 loads / stores 16 B per array (every pointer 16 B aligned, checked on the
// host), V = 1 is the fallback for 8 B-aligned arrays.  A wave touches 64 x 8V contiguous bytes per array.
template<int V>
__device__ __forceinline__ void ld(const double* p, uint64_t t, double* v)
{
  if (V == 2)
  {
    const dv2 x = __builtin_nontemporal_load(reinterpret_cast<const dv2*>(p) + t);
    v[0] = x.x; v[1] = x.y;
  }
  else v[0] = __builtin_nontemporal_load(p + t);
}
template<int V>
__device__ __forceinline__ void st(double* p, uint64_t t, const double* v)
{
  if (V == 2) __builtin_nontemporal_store(dv2{v[0], v[1]}, reinterpret_cast<dv2*>(p) + t);
  else __builtin_nontemporal_store(v[0], p + t);
}

// W: minimum waves per SIMD (amdgpu_waves_per_eu; 1 = no constraint)
template<class Model, int V, bool MASK, int W = 1>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(W, 8))) void k_eval_pdf_f64(EvalArgsF64 a)
{
  math_tables_init();
  const Model m(a.p.v);
  const uint64_t nv = a.n / V;
  const uint64_t stride = uint64_t(gridDim.x) * kBlock;
  for (uint64_t t = uint64_t(blockIdx.x) * kBlock + threadIdx.x; t < nv; t += stride)
  {
    double ix[V], iy[V], iz[V], ox[V], oy[V], oz[V], r[V], g[V], b[V], p[V];
    ld<V>(a.ix, t, ix); ld<V>(a.iy, t, iy); ld<V>(a.iz, t, iz);
    ld<V>(a.ox, t, ox); ld<V>(a.oy, t, oy); ld<V>(a.oz, t, oz);
#pragma unroll
    for (int j = 0; j < V; ++j)
    {
      const uint32_t comp = (!MASK || a.mask[t * V + j]) ? a.component : 0u;
      double rgb[3];
      m.eval_pdf(mk(ix[j], iy[j], iz[j]), mk(ox[j], oy[j], oz[j]), comp, rgb, p[j]);
      r[j] = rgb[0]; g[j] = rgb[1]; b[j] = rgb[2];
    }
    st<V>(a.r, t, r); st<V>(a.g, t, g); st<V>(a.b, t, b); st<V>(a.pdf, t, p);
  }
  if (V == 2 && blockIdx.x == 0 && threadIdx.x == 0 && (a.n & 1))
  {
    const uint64_t i = a.n - 1;
    const uint32_t comp = (!MASK || a.mask[i]) ? a.component : 0u;
    double rgb[3], p;
    m.eval_pdf(mk(a.ix[i], a.iy[i], a.iz[i]), mk(a.ox[i], a.oy[i], a.oz[i]), comp, rgb, p);
    a.r[i] = rgb[0]; a.g[i] = rgb[1]; a.b[i] = rgb[2]; a.pdf[i] = p;
  }
}

template<class Model, bool MASK>
__global__ __launch_bounds__(kBlock) void k_reflectance_f64(ReflArgsF64 a)
{
  math_tables_init();
  const Model m(a.p.v);
  const uint64_t stride = uint64_t(gridDim.x) * kBlock;
  for (uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < a.n; i += stride)
  {
    double rgb[3];
    m.reflectance(mk(a.ox[i], a.oy[i], a.oz[i]), (!MASK || a.mask[i]) ? a.component : 0u, rgb);
    a.r[i] = rgb[0]; a.g[i] = rgb[1]; a.b[i] = rgb[2];
  }
}

template<class Model, bool MASK>
__global__ __launch_bounds__(kBlock) void k_sample_f64(SampleArgsF64 a)
{
  math_tables_init();
  const Model m(a.p.v);
  const uint64_t stride = uint64_t(gridDim.x) * kBlock;
  for (uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < a.n; i += stride)
  {
    d3 d;
    double pdf;
    uint32_t f;
    m.sample(mk(a.ox[i], a.oy[i], a.oz[i]), a.xi0[i], a.xi1[i], (!MASK || a.mask[i]) ? a.component : 0u, d, pdf, f);
    a.dx[i] = d.x; a.dy[i] = d.y; a.dz[i] = d.z; a.pdf[i] = pdf; a.flag[i] = f;
  }
}

unsigned grid(uint64_t units)
{
  const uint64_t b = (units + kBlock - 1) / kBlock;
  return unsigned(b < 1 ? 1 : (b > kMaxBlocks ? kMaxBlocks : b));
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

int launched(const char* what)
{
  const hipError_t e = hipGetLastError();
  return (e == hipSuccess) ? 0 : fail(BBM_HIP_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

// Grid cap (0 = full grid): the Student-T NDF's per-thread setup (two f64 tgamma and a pow) is amortised over
// several grid-stride iterations (the floatRGB kernels' eval_grid_cap, kernels.hpp)
template<class Model> struct grid_cap { static constexpr unsigned value = 0; };

template<> struct grid_cap<RibardiereM> { static constexpr unsigned value = 2048; };
template<> struct grid_cap<RibardiereAnisoM> { static constexpr unsigned value = 2048; };

// Per-model host work before a launch, stream-ordered: EPD's table address into its parameter slot
// (EpdNdf::kTableSlot); the He family's sampler CDF built into scratch, its address and component after the
// model's parameters; an aggregate forwards to its second child with the slots shifted past the first's.
template<class Model> struct host_params
{
  static int run(ParamBlockF64&, uint32_t, hipStream_t, void**) { return 0; }
  static void done(void*, hipStream_t) {}
};
template<> struct host_params<EpdM>
{
  static int run(ParamBlockF64& p, uint32_t, hipStream_t s, void**)
  {
    const float* t = epd_table_device(s);
    if (!t) return fail(BBM_HIP_ERR_HIP, "EPD: shadowing table unavailable");
    p.v[EpdNdf::kTableSlot] = __builtin_bit_cast(double, reinterpret_cast<unsigned long long>(t));
    return 0;
  }
  static void done(void*, hipStream_t) {}
};

// ndf::sampler::initialize (ndf/sampler.h:143-181) in double: 90 backscatter evaluations hsum(eval(h, h)) at
// theta = (i / 90)^2 Pi/2, weighted by sin(theta1) sqrt(theta1), then cdf(samples) (util/cdf.h:39-47)
template<class Model>
__global__ __launch_bounds__(128) void k_he_cdf_f64(ParamBlockF64 p, uint32_t component, double* __restrict__ cdf)
{
  math_tables_init();
  __shared__ double sm[90];
  const Model m(p.v);
  const int i = threadIdx.x;
  if (i < 90)
  {
    const double q = double(i) / 90.0, q1 = double(i + 1) / 90.0;
    const d3 h = sph_to_vec(0.0, (q * q) * (0.5 * kPi));
    double rgb[3];
    m.template eval_rgb<false>(h, h, component, rgb);
    const double theta1 = (q1 * q1) * (0.5 * kPi);
    sm[i] = (((0.0 + rgb[0]) + rgb[1]) + rgb[2]) / 1.0 * (sin(theta1) * sqrt(theta1));
  }
  __syncthreads();
  if (i == 0)
  {
    double acc = 0.0;
    for (int k = 0; k < 90; ++k) { acc += sm[k]; sm[k] = acc; }
    for (int k = 0; k < 90; ++k) cdf[k] = sm[k] / acc;
  }
}

template<class FRES, bool ERRATA, bool WESTIN, int TAYLOR, bool ADAPTIVE, int APPROX, bool SCALED>
struct host_params<He<FRES, ERRATA, WESTIN, TAYLOR, ADAPTIVE, APPROX, SCALED>>
{
  using M = He<FRES, ERRATA, WESTIN, TAYLOR, ADAPTIVE, APPROX, SCALED>;
  static int run(ParamBlockF64& p, uint32_t component, hipStream_t s, void** scratch)
  {
    double* cdf = static_cast<double*>(scratch_acquire(90 * sizeof(double), s));
    if (!cdf) return fail(BBM_HIP_ERR_HIP, "He (f64) sampler CDF: scratch allocation failed: " + scratch_failure());
    *scratch = cdf;
    hipLaunchKernelGGL((k_he_cdf_f64<M>), dim3(1), dim3(128), 0, s, p, component, cdf);
    if (const int rc = launched("k_he_cdf_f64")) return rc;
    p.v[M::kParams] = __builtin_bit_cast(double, reinterpret_cast<unsigned long long>(cdf));
    p.v[M::kParams + 1] = double(component);
    return 0;
  }
  static void done(void* scratch, hipStream_t s) { if (scratch) scratch_release(scratch, s); }
};

template<class A, class B>
struct host_params<Aggregate<A, B>>
{
  static int run(ParamBlockF64& p, uint32_t component, hipStream_t s, void** scratch)
  {
    ParamBlockF64 q{};
    for (int k = A::kParams; k < kMaxParamsF64; ++k) q.v[k - A::kParams] = p.v[k];
    if (const int rc = host_params<B>::run(q, component, s, scratch)) return rc;
    for (int k = A::kParams; k < kMaxParamsF64; ++k) p.v[k] = q.v[k - A::kParams];
    return 0;
  }
  static void done(void* scratch, hipStream_t s) { host_params<B>::done(scratch, s); }
};

// releases a launch's scratch (stream-ordered) when the launcher returns
template<class Model> struct Release
{
  void* p = nullptr;
  hipStream_t s;
  ~Release() { host_params<Model>::done(p, s); }
};

template<class Model>
int launch_eval_pdf(const EvalArgsF64& a0, hipStream_t s)
{
  EvalArgsF64 a = a0;
  Release<Model> rel{nullptr, s};
  if (const int rc = host_params<Model>::run(a.p, a.component, s, &rel.p)) return rc;
  const bool v2 = aligned16(a.ix) && aligned16(a.iy) && aligned16(a.iz) && aligned16(a.ox) && aligned16(a.oy) &&
                  aligned16(a.oz) && aligned16(a.r) && aligned16(a.g) && aligned16(a.b) && aligned16(a.pdf);
  unsigned blocks = grid(v2 ? (a.n + 1) / 2 : a.n);
  if (grid_cap<Model>::value && blocks > grid_cap<Model>::value) blocks = grid_cap<Model>::value;
  if constexpr (heavy_f64<Model>() > 0)
  {
    // one pair per thread with an occupancy floor: see heavy_f64 (f64.hpp)
    constexpr int W = heavy_f64<Model>();
    blocks = grid(a.n);
    if (grid_cap<Model>::value && blocks > grid_cap<Model>::value) blocks = grid_cap<Model>::value;
    if (a.mask) hipLaunchKernelGGL((k_eval_pdf_f64<Model, 1, true, W>), dim3(blocks), dim3(kBlock), 0, s, a);
    else hipLaunchKernelGGL((k_eval_pdf_f64<Model, 1, false, W>), dim3(blocks), dim3(kBlock), 0, s, a);
    return launched("k_eval_pdf_f64");
  }
  constexpr int F = floor_f64<Model>();
  if (v2 && a.mask) hipLaunchKernelGGL((k_eval_pdf_f64<Model, 2, true, F>), dim3(blocks), dim3(kBlock), 0, s, a);
  else if (v2) hipLaunchKernelGGL((k_eval_pdf_f64<Model, 2, false, F>), dim3(blocks), dim3(kBlock), 0, s, a);
  else if (a.mask) hipLaunchKernelGGL((k_eval_pdf_f64<Model, 1, true>), dim3(blocks), dim3(kBlock), 0, s, a);
  else hipLaunchKernelGGL((k_eval_pdf_f64<Model, 1, false>), dim3(blocks), dim3(kBlock), 0, s, a);
  return launched("k_eval_pdf_f64");
}

template<class Model>
int launch_reflectance(const ReflArgsF64& a0, hipStream_t s)
{
  ReflArgsF64 a = a0;     // reflectance reads no per-launch data (EPD: Fresnel only; He: Fresnel only)
  if (a.mask) hipLaunchKernelGGL((k_reflectance_f64<Model, true>), dim3(grid(a.n)), dim3(kBlock), 0, s, a);
  else hipLaunchKernelGGL((k_reflectance_f64<Model, false>), dim3(grid(a.n)), dim3(kBlock), 0, s, a);
  return launched("k_reflectance_f64");
}

template<class Model>
int launch_sample(const SampleArgsF64& a0, hipStream_t s)
{
  SampleArgsF64 a = a0;
  Release<Model> rel{nullptr, s};
  if (const int rc = host_params<Model>::run(a.p, a.component, s, &rel.p)) return rc;
  unsigned blocks = grid(a.n);
  if (grid_cap<Model>::value && blocks > grid_cap<Model>::value) blocks = grid_cap<Model>::value;
  if (a.mask) hipLaunchKernelGGL((k_sample_f64<Model, true>), dim3(blocks), dim3(kBlock), 0, s, a);
  else hipLaunchKernelGGL((k_sample_f64<Model, false>), dim3(blocks), dim3(kBlock), 0, s, a);
  return launched("k_sample_f64");
}

struct Entry { const char* name; F64Launchers l; };
#define BBM_HIP_F64(NAME, M) {NAME, {&launch_eval_pdf<M>, &launch_reflectance<M>, &launch_sample<M>}}
// names as in the floatRGB registry (bbm_hip.hip); aliases share a composition as they do there
const Entry kF64[] = {
  BBM_HIP_F64("Lambertian", Lambertian),
  BBM_HIP_F64("OrenNayar", OrenNayar),
  BBM_HIP_F64("CookTorrance", CookTorranceM),
  BBM_HIP_F64("LowCookTorrance", CookTorranceM),   // bsdfmodel/low.h:32-33
  BBM_HIP_F64("GGX", GGXM),
  BBM_HIP_F64("CookTorranceWalter", CookTorranceWalterM),
  BBM_HIP_F64("CookTorranceHeitz", CookTorranceHeitzM),
  BBM_HIP_F64("GGXHeitz", GGXHeitzM),
  BBM_HIP_F64("NganCookTorrance", NganCookTorranceM),
  BBM_HIP_F64("PhongWalter", PhongWalterM),
  BBM_HIP_F64("Ribardiere", RibardiereM),
  BBM_HIP_F64("RibardiereAnisotropic", RibardiereAnisoM),
  BBM_HIP_F64("LowMicrofacet", LowMicrofacetM),
  BBM_HIP_F64("LowMicrofacetFit", LowMicrofacetM),
  BBM_HIP_F64("Aggregate<Lambertian,CookTorrance>", AggCookTorranceM),
  BBM_HIP_F64("Aggregate<Lambertian,LowCookTorrance>", AggCookTorranceM),
  BBM_HIP_F64("Aggregate<Lambertian,GGX>", AggGGXM),
  BBM_HIP_F64("Aggregate<Lambertian,NganCookTorrance>", AggNganCookTorranceM),
  BBM_HIP_F64("Aggregate<Lambertian,LowMicrofacetFit>", AggLowMicrofacetM),
  BBM_HIP_F64("Ward", WardM),
  BBM_HIP_F64("WardDuer", WardDuerM),
  BBM_HIP_F64("WardDuerGeislerMoroder", WardDGMM),
  BBM_HIP_F64("NganWard", NganWardM),
  BBM_HIP_F64("NganWardDuer", NganWardDuerM),
  BBM_HIP_F64("Phong", PhongLobe),
  BBM_HIP_F64("NganBlinnPhong", PhongLobe),   // ngan.h:43-44
  BBM_HIP_F64("Lafortune", LafortuneM),
  BBM_HIP_F64("NganLafortune", NganLafortuneM),
  BBM_HIP_F64("AshikhminShirley", ASM),
  BBM_HIP_F64("AshikhminShirleyFull", ASFullM),
  BBM_HIP_F64("LowAshikhminShirley", LowASM),
  BBM_HIP_F64("NganAshikhminShirley", NganASM),
  BBM_HIP_F64("LowSmooth", LowSmooth),
  BBM_HIP_F64("Aggregate<Lambertian,LowAshikhminShirley>", AggLowASM),
  BBM_HIP_F64("Aggregate<Lambertian,LowSmooth>", AggLowSmoothM),
  BBM_HIP_F64("Aggregate<Lambertian,NganAshikhminShirley>", AggNganASM),
  BBM_HIP_F64("Aggregate<Lambertian,NganBlinnPhong>", AggPhongM),
  BBM_HIP_F64("Aggregate<Lambertian,NganLafortune>", AggNganLafortuneM),
  BBM_HIP_F64("Aggregate<Lambertian,NganWard>", AggNganWardM),
  BBM_HIP_F64("Aggregate<Lambertian,NganWardDuer>", AggNganWardDuerM),
  BBM_HIP_F64("Bagher", Bagher),
  BBM_HIP_F64("Aggregate<Lambertian,Bagher>", AggBagherM),
  BBM_HIP_F64("EPD", EpdM),
  BBM_HIP_F64("He", HeM),
  BBM_HIP_F64("HeWestin", HeWestinM),
  BBM_HIP_F64("HeHolzschuch", HeHolzschuchM),
  BBM_HIP_F64("NganHe", NganHeM),
  BBM_HIP_F64("Aggregate<Lambertian,NganHe>", AggNganHeM),
};
#undef BBM_HIP_F64

static_assert(Lambertian::kParams == 3 && OrenNayar::kParams == 4 && CookTorranceM::kParams == 5 && GGXM::kParams == 5 &&
              CookTorranceHeitzM::kParams == 6 && GGXHeitzM::kParams == 6 && NganCookTorranceM::kParams == 5 &&
              PhongWalterM::kParams == 5 && RibardiereM::kParams == 6 && RibardiereAnisoM::kParams == 7 &&
              LowMicrofacetM::kParams == 6 && AggCookTorranceM::kParams == 8 && WardM::kParams == 5 &&
              NganWardM::kParams == 4 && PhongLobe::kParams == 4 && LafortuneM::kParams == 7 &&
              NganLafortuneM::kParams == 6 && ASM::kParams == 5 && ASFullM::kParams == 8 && LowASM::kParams == 5 &&
              NganASM::kParams == 5 && LowSmooth::kParams == 6 && Bagher::kParams == 30 && EpdM::kParams == 4 && HeM::kParams == 8 && NganHeM::kParams == 6, "f64 nparams must match the floatRGB registry");

}  // namespace

const F64Launchers* f64_launchers(const char* name)
{
  if (!name) return nullptr;
  for (const auto& e : kF64)
    if (std::strcmp(e.name, name) == 0) return &e.l;
  return nullptr;
}

}  // namespace f64
}  // namespace bbmhip
