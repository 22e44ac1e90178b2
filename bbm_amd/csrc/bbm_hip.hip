// bbm_amd/csrc/bbm_hip.hip -- libbbm_hip.so: model registry, synthetic direction generator and
// the C-ABI declared in include/bbm_hip.h.  The kernels live in kernels.hpp and are instantiated
// per family in inst_*.hip.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/bbm_hip.h"
#include "kernels.hpp"
#include "models.hpp"

namespace bbmhip {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg)
{
  g_last_error = msg;
  return code;
}

BBM_HIP_MICROFACET_MODELS(BBM_HIP_EXTERN)
BBM_HIP_LOBE_MODELS(BBM_HIP_EXTERN)
BBM_HIP_DIFFUSE_MODELS(BBM_HIP_EXTERN)
BBM_HIP_SPECTRAL_MODELS(BBM_HIP_EXTERN)

namespace {

// ------------------------------------------------------------------------ model registry

struct ModelEntry
{
  const char* name;
  int nparams;
  uint32_t components;
  EvalLauncher eval_pdf;
  SampleLauncher sample;
  float defaults[kMaxParams];
  float lower[kMaxParams];
  float upper[kMaxParams];
};

constexpr float kFMax = 3.4028234663852886e+38f;
constexpr float kFMin = 1.1754943508222875e-38f;

// Defaults and bounds: bsdf_attribute.h:73-94 (scale 0.5 in [0,1], roughness 0.1 in [0,1] as
// reported by parameter_lower_bound/upper_bound, ior 1.3 in [1,5]); pinned against
// tests/golden/models.json by tests/test_abi.py.
const ModelEntry kModels[] = {
  {"Lambertian", 3, kFlagDiffuse, &launch_eval_pdf<Lambertian>, &launch_sample<Lambertian>,
   {0.5f, 0.5f, 0.5f}, {0, 0, 0}, {1, 1, 1}},
  {"CookTorrance", 5, kFlagSpecular, &launch_eval_pdf<CookTorranceM>, &launch_sample<CookTorranceM>,
   {0.5f, 0.5f, 0.5f, 0.1f, 1.3f}, {0, 0, 0, kEpsF, 1}, {1, 1, 1, 1, 5}},
  {"LowCookTorrance", 5, kFlagSpecular, &launch_eval_pdf<CookTorranceM>, &launch_sample<CookTorranceM>,   // bsdfmodel/low.h:32-33
   {0.5f, 0.5f, 0.5f, 0.1f, 1.3f}, {0, 0, 0, kEpsF, 1}, {1, 1, 1, 1, 5}},
  {"GGX", 5, kFlagSpecular, &launch_eval_pdf<GGXM>, &launch_sample<GGXM>,
   {0.5f, 0.5f, 0.5f, 0.1f, 1.3f}, {0, 0, 0, kEpsF, 1}, {1, 1, 1, 1, 5}},
  {"CookTorranceWalter", 5, kFlagSpecular, &launch_eval_pdf<CookTorranceWalterM>, &launch_sample<CookTorranceWalterM>,
   {0.5f, 0.5f, 0.5f, 0.1f, 1.3f}, {0, 0, 0, kEpsF, 1}, {1, 1, 1, 1, 5}},
  {"CookTorranceHeitz", 6, kFlagSpecular, &launch_eval_pdf<CookTorranceHeitzM>, &launch_sample<CookTorranceHeitzM>,
   {0.5f, 0.5f, 0.5f, 0.1f, 0.1f, 1.3f}, {0, 0, 0, kEpsF, kEpsF, 1}, {1, 1, 1, 1, 1, 5}},
  {"GGXHeitz", 6, kFlagSpecular, &launch_eval_pdf<GGXHeitzM>, &launch_sample<GGXHeitzM>,
   {0.5f, 0.5f, 0.5f, 0.1f, 0.1f, 1.3f}, {0, 0, 0, kEpsF, kEpsF, 1}, {1, 1, 1, 1, 1, 5}},
  {"NganCookTorrance", 5, kFlagSpecular, &launch_eval_pdf<NganCookTorranceM>, &launch_sample<NganCookTorranceM>,
   {0.5f, 0.5f, 0.5f, 0.1f, 0.1f}, {0, 0, 0, kEpsF, 0}, {1, 1, 1, 1, 1}},
  {"PhongWalter", 5, kFlagSpecular, &launch_eval_pdf<PhongWalterM>, &launch_sample<PhongWalterM>,
   {0.5f, 0.5f, 0.5f, 32.0f, 1.3f}, {0, 0, 0, 0, 1}, {1, 1, 1, kFMax, 5}},
  {"Ribardiere", 6, kFlagSpecular, &launch_eval_pdf<RibardiereM>, &launch_sample<RibardiereM>,
   {0.5f, 0.5f, 0.5f, 0.1f, 2.0f, 1.3f}, {0, 0, 0, kEpsF, 1.5f + kEpsF, 1}, {1, 1, 1, 1, 40, 5}},
  {"RibardiereAnisotropic", 7, kFlagSpecular, &launch_eval_pdf<RibardiereAnisoM>, &launch_sample<RibardiereAnisoM>,
   {0.5f, 0.5f, 0.5f, 0.1f, 0.1f, 2.0f, 1.3f}, {0, 0, 0, kEpsF, kEpsF, 1.5f + kEpsF, 1}, {1, 1, 1, 1, 1, 40, 5}},
  {"OrenNayar", 4, kFlagDiffuse, &launch_eval_pdf<OrenNayar>, &launch_sample<OrenNayar>,
   {0.5f, 0.5f, 0.5f, 0.1f}, {0, 0, 0, kEpsF}, {1, 1, 1, 1}},
  {"LowMicrofacet", 6, kFlagSpecular, &launch_eval_pdf<LowMicrofacetM>, &launch_sample<LowMicrofacetM>,
   {1, 1, 1, 1, 1, 1.3f}, {0, 0, 0, 0, 0, 1}, {kFMax, kFMax, kFMax, kFMax, kFMax, 5}},
  {"LowMicrofacetFit", 6, kFlagSpecular, &launch_eval_pdf<LowMicrofacetM>, &launch_sample<LowMicrofacetM>,
   {1, 1, 1, 1, 1, 1.3f}, {0, 0, 0, 0, 0, 1}, {kFMax, kFMax, kFMax, kFMax, kFMax, 5}},
  {"Ward", 5, kFlagSpecular, &launch_eval_pdf<WardM>, &launch_sample<WardM>,
   {0.5f, 0.5f, 0.5f, 0.1f, 0.1f}, {0, 0, 0, kEpsF, kEpsF}, {1, 1, 1, 1, 1}},
  {"WardDuer", 5, kFlagSpecular, &launch_eval_pdf<WardDuerM>, &launch_sample<WardDuerM>,
   {0.5f, 0.5f, 0.5f, 0.1f, 0.1f}, {0, 0, 0, kEpsF, kEpsF}, {1, 1, 1, 1, 1}},
  {"WardDuerGeislerMoroder", 5, kFlagSpecular, &launch_eval_pdf<WardDGMM>, &launch_sample<WardDGMM>,
   {0.5f, 0.5f, 0.5f, 0.1f, 0.1f}, {0, 0, 0, kEpsF, kEpsF}, {1, 1, 1, 1, 1}},
  {"NganWard", 4, kFlagSpecular, &launch_eval_pdf<NganWardM>, &launch_sample<NganWardM>,
   {0.5f, 0.5f, 0.5f, 0.1f}, {0, 0, 0, kEpsF}, {1, 1, 1, 1}},
  {"NganWardDuer", 4, kFlagSpecular, &launch_eval_pdf<NganWardDuerM>, &launch_sample<NganWardDuerM>,
   {0.5f, 0.5f, 0.5f, 0.1f}, {0, 0, 0, kEpsF}, {1, 1, 1, 1}},
  {"Phong", 4, kFlagSpecular, &launch_eval_pdf<PhongLobe>, &launch_sample<PhongLobe>,
   {0.5f, 0.5f, 0.5f, 32.0f}, {0, 0, 0, 0}, {1, 1, 1, kFMax}},
  {"NganBlinnPhong", 4, kFlagSpecular, &launch_eval_pdf<PhongLobe>, &launch_sample<PhongLobe>,   // ngan.h:43-44
   {0.5f, 0.5f, 0.5f, 32.0f}, {0, 0, 0, 0}, {1, 1, 1, kFMax}},
  {"Lafortune", 7, kFlagSpecular, &launch_eval_pdf<LafortuneM>, &launch_sample<LafortuneM>,
   {0.5f, 0.5f, 0.5f, -0.57735026919f, -0.57735026919f, 0.57735026919f, 32.0f},
   {0, 0, 0, kFMin, kFMin, kFMin, 0}, {1, 1, 1, kFMax, kFMax, kFMax, kFMax}},
  {"NganLafortune", 6, kFlagSpecular, &launch_eval_pdf<NganLafortuneM>, &launch_sample<NganLafortuneM>,
   {0.5f, 0.5f, 0.5f, -0.57735026919f, 0.57735026919f, 32.0f}, {0, 0, 0, kFMin, kFMin, 0}, {1, 1, 1, kFMax, kFMax, kFMax}},
  {"AshikhminShirley", 5, kFlagSpecular, &launch_eval_pdf<ASM>, &launch_sample<ASM>,
   {0.1f, 0.1f, 0.1f, 32.0f, 32.0f}, {0, 0, 0, 0, 0}, {1, 1, 1, kFMax, kFMax}},
  {"AshikhminShirleyFull", 8, kFlagAll, &launch_eval_pdf<ASFullM>, &launch_sample<ASFullM>,
   {0.5f, 0.5f, 0.5f, 0.1f, 0.1f, 0.1f, 32.0f, 32.0f}, {0, 0, 0, 0, 0, 0, 0, 0}, {1, 1, 1, 1, 1, 1, kFMax, kFMax}},
  {"LowAshikhminShirley", 5, kFlagSpecular, &launch_eval_pdf<LowASM>, &launch_sample<LowASM>,
   {0.5f, 0.5f, 0.5f, 1.3f, 32.0f}, {0, 0, 0, 1, 0}, {1, 1, 1, 5, kFMax}},
  {"NganAshikhminShirley", 5, kFlagSpecular, &launch_eval_pdf<NganASM>, &launch_sample<NganASM>,
   {0.5f, 0.5f, 0.5f, 0.1f, 32.0f}, {0, 0, 0, 0, 0}, {1, 1, 1, 1, kFMax}},
  {"LowSmooth", 6, kFlagSpecular, &launch_eval_pdf<LowSmooth>, &launch_sample<LowSmooth>,
   {1, 1, 1, 1, 1, 1.3f}, {0, 0, 0, 0, 0, 1}, {kFMax, kFMax, kFMax, kFMax, kFMax, 5}},
  // bsdfmodel/bagher.h:62-68: albedo, K, Lambda, c, theta0, k (ndf/sgd.h:197-203, Dependent),
  // alpha, p (sgd.h:107-111), eta = (F0, F1) RGB (bagher.h:31, default {1, 0}, lower {0, -1})
  {"Bagher", 30, kFlagSpecular, &launch_eval_pdf<Bagher>, &launch_sample<Bagher>,
   {0.5f, 0.5f, 0.5f, 7.5f, 7.5f, 7.5f, 1, 1, 1, 1, 1, 1, 1.5707963705062866f, 1.5707963705062866f, 1.5707963705062866f,
    1, 1, 1, 0.1f, 0.1f, 0.1f, 0.64f, 0.64f, 0.64f, 1, 1, 1, 0, 0, 0},
   {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, kEpsF, kEpsF, kEpsF, 0, 0, 0, 0, 0, 0, -1, -1, -1},
   {1, 1, 1, kFMax, kFMax, kFMax, kFMax, kFMax, kFMax, kFMax, kFMax, kFMax, kFMax, kFMax, kFMax, kFMax, kFMax, kFMax,
    1, 1, 1, kFMax, kFMax, kFMax, 1, 1, 1, 1, 1, 1}},
};
constexpr int kNumModels = int(sizeof(kModels) / sizeof(kModels[0]));
static_assert(Lambertian::kParams == 3 && OrenNayar::kParams == 4 && CookTorranceM::kParams == 5 && GGXM::kParams == 5 &&
              CookTorranceHeitzM::kParams == 6 && GGXHeitzM::kParams == 6 && NganCookTorranceM::kParams == 5 &&
              PhongWalterM::kParams == 5 && RibardiereM::kParams == 6 && RibardiereAnisoM::kParams == 7 &&
              LowMicrofacetM::kParams == 6 && WardM::kParams == 5 && NganWardM::kParams == 4 &&
              PhongLobe::kParams == 4 && LafortuneM::kParams == 7 && NganLafortuneM::kParams == 6 &&
              ASM::kParams == 5 && ASFullM::kParams == 8 && LowASM::kParams == 5 && NganASM::kParams == 5 &&
              LowSmooth::kParams == 6 && Bagher::kParams == 30, "registry nparams must match the compositions");

const ModelEntry* entry(int id) { return (id >= 0 && id < kNumModels) ? &kModels[id] : nullptr; }

int prepare(int model_id, const float* params, int nparams, size_t n, EvalArgs& a, const ModelEntry*& e)
{
  e = entry(model_id);
  if (!e) return fail(BBM_HIP_ERR_INVALID_MODEL, "unknown model id " + std::to_string(model_id));
  if (nparams != e->nparams)
    return fail(BBM_HIP_ERR_INVALID_ARG, std::string(e->name) + ": expected " + std::to_string(e->nparams) +
                                             " parameters, got " + std::to_string(nparams));
  if (nparams > 0 && !params) return fail(BBM_HIP_ERR_INVALID_ARG, "params is NULL");
  std::memset(&a, 0, sizeof(a));
  for (int i = 0; i < nparams; ++i) a.p.v[i] = params[i];
  a.n = n;
  return BBM_HIP_OK;
}

int check_dirs(const float* x, const float* y, const float* z, const char* what)
{
  if (!x || !y || !z) return fail(BBM_HIP_ERR_INVALID_ARG, std::string(what) + " direction pointer is NULL");
  return BBM_HIP_OK;
}

// ------------------------------------------------------------------- synthetic directions

// Counter-based generator: splitmix64 finaliser over (seed, stream, index).  Two 24-bit uniforms
// per direction.  Pure function of the global index -> shards regenerate identical slices.
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z)
{
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(kBlock) void k_fill_dirs(uint64_t key, uint64_t offset, uint64_t n, int mode,
                                                       float* __restrict__ x, float* __restrict__ y, float* __restrict__ z)
{
  const uint64_t stride = uint64_t(gridDim.x) * kBlock;
  for (uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride)
  {
    const uint64_t h = mix64(key + 0x9e3779b97f4a7c15ull * (offset + i));
    const float u1 = float(uint32_t(h >> 40)) * (1.0f / 16777216.0f);
    const float u2 = float(uint32_t(h >> 16) & 0xffffffu) * (1.0f / 16777216.0f);
    const float zz = (mode == 0) ? u1 : 2.0f * u1 - 1.0f;
    const float s = sqrtf(fmaxf(1.0f - zz * zz, 0.0f));
    float sp, cp;
    sincosf(2.0f * kPiF * u2, &sp, &cp);
    x[i] = s * cp;
    y[i] = s * sp;
    z[i] = zz;
  }
}

}  // namespace
}  // namespace bbmhip

using namespace bbmhip;

extern "C" {

int bbm_hip_abi_version(void) { return BBM_HIP_ABI_VERSION; }

const char* bbm_hip_last_error(void) { return g_last_error.c_str(); }

int bbm_hip_num_models(void) { return kNumModels; }

const char* bbm_hip_model_name(int model_id)
{
  const ModelEntry* e = entry(model_id);
  return e ? e->name : nullptr;
}

int bbm_hip_model_id(const char* name)
{
  if (!name) return fail(BBM_HIP_ERR_INVALID_ARG, "name is NULL");
  for (int i = 0; i < kNumModels; ++i)
    if (std::strcmp(kModels[i].name, name) == 0) return i;
  return fail(BBM_HIP_ERR_INVALID_MODEL, std::string("unknown BSDF model: ") + name);
}

int bbm_hip_model_nparams(int model_id)
{
  const ModelEntry* e = entry(model_id);
  return e ? e->nparams : fail(BBM_HIP_ERR_INVALID_MODEL, "unknown model id " + std::to_string(model_id));
}

int bbm_hip_model_params(int model_id, int which, float* out, int capacity)
{
  const ModelEntry* e = entry(model_id);
  if (!e) return fail(BBM_HIP_ERR_INVALID_MODEL, "unknown model id " + std::to_string(model_id));
  const float* src = (which == 0) ? e->defaults : (which == 1) ? e->lower : (which == 2) ? e->upper : nullptr;
  if (!src) return fail(BBM_HIP_ERR_INVALID_ARG, "which must be 0 (default), 1 (lower) or 2 (upper)");
  for (int i = 0; out && i < e->nparams && i < capacity; ++i) out[i] = src[i];
  return e->nparams;
}

int bbm_hip_model_components(int model_id)
{
  const ModelEntry* e = entry(model_id);
  return e ? int(e->components) : fail(BBM_HIP_ERR_INVALID_MODEL, "unknown model id " + std::to_string(model_id));
}

static int eval_common(int mode, int model_id, const float* params, int nparams,
                       const float* in_x, const float* in_y, const float* in_z,
                       const float* out_x, const float* out_y, const float* out_z,
                       const uint8_t* mask, size_t n, uint32_t component, uint32_t unit,
                       float* r, float* g, float* b, float* pdf, void* stream)
{
  (void)unit;   // no model on this path depends on unit_t (bsdfmodel/microfacet.h:74, lambertian.h:45)
  EvalArgs a;
  const ModelEntry* e;
  int rc = prepare(model_id, params, nparams, n, a, e);
  if (rc) return rc;
  if (n == 0) return BBM_HIP_OK;
  if ((rc = check_dirs(in_x, in_y, in_z, "in")) || (rc = check_dirs(out_x, out_y, out_z, "out"))) return rc;
  if ((mode & kModeEval) && (!r || !g || !b)) return fail(BBM_HIP_ERR_INVALID_ARG, "eval output pointer is NULL");
  if ((mode & kModePdf) && !pdf) return fail(BBM_HIP_ERR_INVALID_ARG, "pdf output pointer is NULL");
  a.ix = in_x; a.iy = in_y; a.iz = in_z; a.ox = out_x; a.oy = out_y; a.oz = out_z;
  a.mask = mask; a.r = r; a.g = g; a.b = b; a.pdf = pdf;
  a.component = component & kFlagAll;
  return e->eval_pdf(a, mode, static_cast<hipStream_t>(stream));
}

int bbm_hip_eval(int model_id, const float* params, int nparams,
                 const float* in_x, const float* in_y, const float* in_z,
                 const float* out_x, const float* out_y, const float* out_z,
                 const uint8_t* mask, size_t n, uint32_t component, uint32_t unit,
                 float* r, float* g, float* b, void* stream)
{
  return eval_common(kModeEval, model_id, params, nparams, in_x, in_y, in_z, out_x, out_y, out_z, mask, n,
                     component, unit, r, g, b, nullptr, stream);
}

int bbm_hip_pdf(int model_id, const float* params, int nparams,
                const float* in_x, const float* in_y, const float* in_z,
                const float* out_x, const float* out_y, const float* out_z,
                const uint8_t* mask, size_t n, uint32_t component, uint32_t unit,
                float* pdf, void* stream)
{
  return eval_common(kModePdf, model_id, params, nparams, in_x, in_y, in_z, out_x, out_y, out_z, mask, n,
                     component, unit, nullptr, nullptr, nullptr, pdf, stream);
}

int bbm_hip_eval_pdf(int model_id, const float* params, int nparams,
                     const float* in_x, const float* in_y, const float* in_z,
                     const float* out_x, const float* out_y, const float* out_z,
                     const uint8_t* mask, size_t n, uint32_t component, uint32_t unit,
                     float* r, float* g, float* b, float* pdf, void* stream)
{
  return eval_common(kModeEvalPdf, model_id, params, nparams, in_x, in_y, in_z, out_x, out_y, out_z, mask, n,
                     component, unit, r, g, b, pdf, stream);
}

int bbm_hip_sample(int model_id, const float* params, int nparams,
                   const float* out_x, const float* out_y, const float* out_z,
                   const float* xi0, const float* xi1,
                   const uint8_t* mask, size_t n, uint32_t component, uint32_t unit,
                   float* dir_x, float* dir_y, float* dir_z, float* pdf, uint32_t* flag,
                   void* stream)
{
  (void)unit;
  EvalArgs tmp;
  const ModelEntry* e;
  int rc = prepare(model_id, params, nparams, n, tmp, e);
  if (rc) return rc;
  if (n == 0) return BBM_HIP_OK;
  if ((rc = check_dirs(out_x, out_y, out_z, "out"))) return rc;
  if (!xi0 || !xi1) return fail(BBM_HIP_ERR_INVALID_ARG, "xi pointer is NULL");
  if (!dir_x || !dir_y || !dir_z || !pdf || !flag) return fail(BBM_HIP_ERR_INVALID_ARG, "sample output pointer is NULL");
  SampleArgs a;
  std::memset(&a, 0, sizeof(a));
  a.p = tmp.p;
  a.n = n;
  a.ox = out_x; a.oy = out_y; a.oz = out_z; a.xi0 = xi0; a.xi1 = xi1; a.mask = mask;
  a.dx = dir_x; a.dy = dir_y; a.dz = dir_z; a.pdf = pdf; a.flag = flag;
  a.component = component & kFlagAll;
  return e->sample(a, static_cast<hipStream_t>(stream));
}

int bbm_hip_fill_directions(uint64_t seed, uint32_t stream_id, uint64_t offset, size_t n, int mode,
                            float* x, float* y, float* z, void* stream)
{
  if (n == 0) return BBM_HIP_OK;
  if (!x || !y || !z) return fail(BBM_HIP_ERR_INVALID_ARG, "direction pointer is NULL");
  if (mode != 0 && mode != 1) return fail(BBM_HIP_ERR_INVALID_ARG, "mode must be 0 (hemisphere) or 1 (sphere)");
  uint64_t blocks = (n + kBlock - 1) / kBlock;
  if (blocks > kMaxBlocks) blocks = kMaxBlocks;
  const uint64_t key = mix64(seed) ^ (0xd1b54a32d192ed03ull * (uint64_t(stream_id) + 1));
  hipLaunchKernelGGL(k_fill_dirs, dim3(unsigned(blocks)), dim3(kBlock), 0, static_cast<hipStream_t>(stream), key,
                     offset, uint64_t(n), mode, x, y, z);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(BBM_HIP_ERR_HIP, std::string("kernel launch failed: ") + hipGetErrorString(e));
  return BBM_HIP_OK;
}

}  // extern "C"
