// bbm_amd/csrc/bbm_hip.hip -- libbbm_hip.so: model registry, synthetic direction generator and
// the C-ABI declared in include/bbm_hip.h.  The kernels live in kernels.hpp and are instantiated
// per family in inst_*.hip.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/bbm_hip.h"
#include "kernels.hpp"
#include "models.hpp"
#include "f64.hpp"

namespace bbmhip {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg)
{
  g_last_error = msg;
  return code;
}

// ------------------------------------------------------------------------ stream-ordered scratch

namespace {
struct ScratchBlock
{
  void* p;
  size_t bytes;
  int device;
  hipEvent_t released;     // recorded on `last` when the block was released
  hipStream_t last;
  bool busy, used;
  bool pinned;             // handed out while `last` was capturing a graph: the graph keeps the address, so the
                           // block is never handed out or freed again (bbm_hip_scratch_trim_captured aside)
};
std::mutex g_scratch_mu;
std::vector<ScratchBlock> g_scratch;
}  // namespace

namespace {
// idle bytes kept for reuse before released blocks are returned to the device (BBM_HIP_SCRATCH_RETAIN_MB)
size_t retain_limit()
{
  static const size_t v = [] {
    const char* e = std::getenv("BBM_HIP_SCRATCH_RETAIN_MB");
    return size_t(e ? std::strtoull(e, nullptr, 10) : 1024ull) << 20;
  }();
  return v;
}

// frees idle blocks (caller holds the lock): wait = false only those whose last use has completed on the GPU;
// wait = true all of them, after their release event.  `keep`: idle bytes that may stay.  Returns bytes freed.
size_t free_idle(bool wait, size_t keep)
{
  size_t idle = 0, freed = 0;
  for (const ScratchBlock& b : g_scratch) idle += b.busy ? 0 : b.bytes;
  for (size_t i = g_scratch.size(); i-- > 0 && idle > keep;)
  {
    ScratchBlock& b = g_scratch[i];
    if (b.busy || b.pinned) continue;
    if (b.used && (wait ? hipEventSynchronize(b.released) : hipEventQuery(b.released)) != hipSuccess) continue;
    (void)hipFree(b.p);
    (void)hipEventDestroy(b.released);
    idle -= b.bytes;
    freed += b.bytes;
    g_scratch.erase(g_scratch.begin() + long(i));
  }
  return freed;
}
}  // namespace

thread_local std::string g_scratch_why;

std::string scratch_failure() { return g_scratch_why.empty() ? std::string("out of device memory") : g_scratch_why; }

void* scratch_acquire(size_t bytes, hipStream_t s)
{
  g_scratch_why.clear();
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  bytes = (bytes + 255) & ~size_t(255);
  std::lock_guard<std::mutex> lock(g_scratch_mu);
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (const hipError_t e = hipStreamIsCapturing(s, &cap); e != hipSuccess)
  {
    // e.g. the legacy null stream while another stream is under a global-mode capture
    g_scratch_why = std::string("the stream's capture status cannot be read (hipStreamIsCapturing: ") +
                    hipGetErrorString(e) + "; a call on the null stream during a global-mode capture?)";
    return nullptr;
  }
  if (cap != hipStreamCaptureStatusNone)
  {
    // graph capture: a fresh block that belongs to the graph from now on.  No idle block is reused (its release
    // event was recorded outside the capture, and waiting on it would tie the graph to a pre-capture event), and
    // the allocation runs in relaxed capture mode (hipMalloc is not allowed under a global-mode capture).
    hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
    (void)hipThreadExchangeStreamCaptureMode(&mode);
    ScratchBlock b{nullptr, bytes, dev, nullptr, s, true, true, true};
    const bool ok = hipMalloc(&b.p, bytes) == hipSuccess;
    (void)hipThreadExchangeStreamCaptureMode(&mode);
    if (!ok) return nullptr;
    g_scratch.push_back(b);
    return b.p;
  }
  // best fit among idle blocks of this device, but not one much larger than the request (a 360-byte CDF must not
  // pin a block sized for 125M lanes)
  ScratchBlock* best = nullptr;
  for (ScratchBlock& b : g_scratch)
    if (!b.busy && !b.pinned && b.device == dev && b.bytes >= bytes && (b.bytes <= 4 * bytes || b.bytes - bytes <= (size_t(1) << 20)) &&
        (!best || b.bytes < best->bytes))
      best = &b;
  if (best)
  {
    // its last user's work must be done before this stream writes it: free on the same stream (stream
    // order), otherwise a GPU-side wait on the release event
    if (best->used && best->last != s && hipStreamWaitEvent(s, best->released, 0) != hipSuccess) return nullptr;
    best->busy = true;
    return best->p;
  }
  ScratchBlock b{nullptr, bytes, dev, nullptr, s, true, false, false};
  if (hipMalloc(&b.p, bytes) != hipSuccess)
  {
    // out of device memory: return every idle block (after its last use) and try once more
    (void)hipGetLastError();
    free_idle(true, 0);
    if (hipMalloc(&b.p, bytes) != hipSuccess) return nullptr;
  }
  if (hipEventCreateWithFlags(&b.released, hipEventDisableTiming) != hipSuccess)
  {
    (void)hipFree(b.p);
    return nullptr;
  }
  g_scratch.push_back(b);
  return b.p;
}

void scratch_release(void* p, hipStream_t s)
{
  std::lock_guard<std::mutex> lock(g_scratch_mu);
  for (ScratchBlock& b : g_scratch)
    if (b.p == p)
    {
      if (b.pinned) return;      // the captured graph owns it: no event, no reuse, and no freeing inside a capture
      (void)hipEventRecord(b.released, s);
      b.last = s;
      b.busy = false;
      b.used = true;
      break;
    }
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cap) == hipSuccess && cap == hipStreamCaptureStatusNone) free_idle(false, retain_limit());
}

size_t scratch_trim()
{
  std::lock_guard<std::mutex> lock(g_scratch_mu);
  return free_idle(true, 0);
}

size_t scratch_trim_captured()
{
  std::lock_guard<std::mutex> lock(g_scratch_mu);
  size_t freed = 0;
  bool synced = false;
  for (size_t i = g_scratch.size(); i-- > 0;)
  {
    ScratchBlock& b = g_scratch[i];
    if (!b.pinned) continue;
    if (!synced)
    {
      (void)hipDeviceSynchronize();
      synced = true;
    }
    (void)hipFree(b.p);
    if (b.released) (void)hipEventDestroy(b.released);
    freed += b.bytes;
    g_scratch.erase(g_scratch.begin() + long(i));
  }
  return freed + free_idle(true, 0);
}

size_t scratch_bytes()
{
  std::lock_guard<std::mutex> lock(g_scratch_mu);
  size_t t = 0;
  for (const ScratchBlock& b : g_scratch) t += b.bytes;
  return t;
}

BBM_HIP_MICROFACET_MODELS(BBM_HIP_EXTERN)
BBM_HIP_LOBE_MODELS(BBM_HIP_EXTERN)
BBM_HIP_DIFFUSE_MODELS(BBM_HIP_EXTERN)
BBM_HIP_SPECTRAL_MODELS(BBM_HIP_EXTERN)
BBM_HIP_AGGREGATE_MODELS(BBM_HIP_EXTERN)
BBM_HIP_EPD_MODELS(BBM_HIP_EXTERN)
BBM_HIP_HE_MODELS(BBM_HIP_EXTERN)
BBM_HIP_MERL_MODELS(BBM_HIP_EXTERN)
int epd_table_host(float* out, int capacity);

namespace {

// ------------------------------------------------------------------------ model registry

struct ModelEntry
{
  const char* name;
  int nparams;
  uint32_t components;
  EvalLauncher eval_pdf;
  SampleLauncher sample;
  ReflLauncher reflectance;
  LossLauncher loss;
  CheckLauncher check;
  float defaults[kMaxParams];
  float lower[kMaxParams];
  float upper[kMaxParams];
  // per-parameter bsdf_attr flags (include/bbm/bsdf_attr_flag.h:16-29), one letter per parameter:
  // d DiffuseScale, D DiffuseParameter, s SpecularScale, p SpecularParameter, x Dependent
  const char* attrs;
};

constexpr float kFMax = 3.4028234663852886e+38f;
constexpr float kFMin = 1.1754943508222875e-38f;

// Defaults and bounds: bsdf_attribute.h:73-94 (scale 0.5 in [0,1], roughness 0.1 in [0,1] as
// reported by parameter_lower_bound/upper_bound, ior 1.3 in [1,5]); pinned against
// tests/golden/models.json by tests/test_abi.py.
const ModelEntry kSingle[] = {
  {"Lambertian", 3, kFlagDiffuse, &launch_eval_pdf<Lambertian>, &launch_sample<Lambertian>, &launch_reflectance<Lambertian>, &launch_loss<Lambertian>, &launch_check<Lambertian>,
   {0.5f, 0.5f, 0.5f}, {0, 0, 0}, {1, 1, 1}, "ddd"},
  {"CookTorrance", 5, kFlagSpecular, &launch_eval_pdf<CookTorranceM>, &launch_sample<CookTorranceM>, &launch_reflectance<CookTorranceM>, &launch_loss<CookTorranceM>, &launch_check<CookTorranceM>,
   {0.5f, 0.5f, 0.5f, 0.1f, 1.3f}, {0, 0, 0, kEpsF, 1}, {1, 1, 1, 1, 5}, "ssspp"},
  {"LowCookTorrance", 5, kFlagSpecular, &launch_eval_pdf<CookTorranceM>, &launch_sample<CookTorranceM>, &launch_reflectance<CookTorranceM>, &launch_loss<CookTorranceM>, &launch_check<CookTorranceM>,   // bsdfmodel/low.h:32-33
   {0.5f, 0.5f, 0.5f, 0.1f, 1.3f}, {0, 0, 0, kEpsF, 1}, {1, 1, 1, 1, 5}, "ssspp"},
  {"GGX", 5, kFlagSpecular, &launch_eval_pdf<GGXM>, &launch_sample<GGXM>, &launch_reflectance<GGXM>, &launch_loss<GGXM>, &launch_check<GGXM>,
   {0.5f, 0.5f, 0.5f, 0.1f, 1.3f}, {0, 0, 0, kEpsF, 1}, {1, 1, 1, 1, 5}, "ssspp"},
  {"CookTorranceWalter", 5, kFlagSpecular, &launch_eval_pdf<CookTorranceWalterM>, &launch_sample<CookTorranceWalterM>, &launch_reflectance<CookTorranceWalterM>, &launch_loss<CookTorranceWalterM>, &launch_check<CookTorranceWalterM>,
   {0.5f, 0.5f, 0.5f, 0.1f, 1.3f}, {0, 0, 0, kEpsF, 1}, {1, 1, 1, 1, 5}, "ssspp"},
  {"CookTorranceHeitz", 6, kFlagSpecular, &launch_eval_pdf<CookTorranceHeitzM>, &launch_sample<CookTorranceHeitzM>, &launch_reflectance<CookTorranceHeitzM>, &launch_loss<CookTorranceHeitzM>, &launch_check<CookTorranceHeitzM>,
   {0.5f, 0.5f, 0.5f, 0.1f, 0.1f, 1.3f}, {0, 0, 0, kEpsF, kEpsF, 1}, {1, 1, 1, 1, 1, 5}, "sssppp"},
  {"GGXHeitz", 6, kFlagSpecular, &launch_eval_pdf<GGXHeitzM>, &launch_sample<GGXHeitzM>, &launch_reflectance<GGXHeitzM>, &launch_loss<GGXHeitzM>, &launch_check<GGXHeitzM>,
   {0.5f, 0.5f, 0.5f, 0.1f, 0.1f, 1.3f}, {0, 0, 0, kEpsF, kEpsF, 1}, {1, 1, 1, 1, 1, 5}, "sssppp"},
  {"NganCookTorrance", 5, kFlagSpecular, &launch_eval_pdf<NganCookTorranceM>, &launch_sample<NganCookTorranceM>, &launch_reflectance<NganCookTorranceM>, &launch_loss<NganCookTorranceM>, &launch_check<NganCookTorranceM>,
   {0.5f, 0.5f, 0.5f, 0.1f, 0.1f}, {0, 0, 0, kEpsF, 0}, {1, 1, 1, 1, 1}, "ssspp"},
  {"PhongWalter", 5, kFlagSpecular, &launch_eval_pdf<PhongWalterM>, &launch_sample<PhongWalterM>, &launch_reflectance<PhongWalterM>, &launch_loss<PhongWalterM>, &launch_check<PhongWalterM>,
   {0.5f, 0.5f, 0.5f, 32.0f, 1.3f}, {0, 0, 0, 0, 1}, {1, 1, 1, kFMax, 5}, "ssspp"},
  {"Ribardiere", 6, kFlagSpecular, &launch_eval_pdf<RibardiereM>, &launch_sample<RibardiereM>, &launch_reflectance<RibardiereM>, &launch_loss<RibardiereM>, &launch_check<RibardiereM>,
   {0.5f, 0.5f, 0.5f, 0.1f, 2.0f, 1.3f}, {0, 0, 0, kEpsF, 1.5f + kEpsF, 1}, {1, 1, 1, 1, 40, 5}, "sssppp"},
  {"RibardiereAnisotropic", 7, kFlagSpecular, &launch_eval_pdf<RibardiereAnisoM>, &launch_sample<RibardiereAnisoM>, &launch_reflectance<RibardiereAnisoM>, &launch_loss<RibardiereAnisoM>, &launch_check<RibardiereAnisoM>,
   {0.5f, 0.5f, 0.5f, 0.1f, 0.1f, 2.0f, 1.3f}, {0, 0, 0, kEpsF, kEpsF, 1.5f + kEpsF, 1}, {1, 1, 1, 1, 1, 40, 5}, "ssspppp"},
  {"OrenNayar", 4, kFlagDiffuse, &launch_eval_pdf<OrenNayar>, &launch_sample<OrenNayar>, &launch_reflectance<OrenNayar>, &launch_loss<OrenNayar>, &launch_check<OrenNayar>,
   {0.5f, 0.5f, 0.5f, 0.1f}, {0, 0, 0, kEpsF}, {1, 1, 1, 1}, "dddD"},
  {"LowMicrofacet", 6, kFlagSpecular, &launch_eval_pdf<LowMicrofacetM>, &launch_sample<LowMicrofacetM>, &launch_reflectance<LowMicrofacetM>, &launch_loss<LowMicrofacetM>, &launch_check<LowMicrofacetM>,
   {1, 1, 1, 1, 1, 1.3f}, {0, 0, 0, 0, 0, 1}, {kFMax, kFMax, kFMax, kFMax, kFMax, 5}, "pppppp"},
  {"LowMicrofacetFit", 6, kFlagSpecular, &launch_eval_pdf<LowMicrofacetM>, &launch_sample<LowMicrofacetM>, &launch_reflectance<LowMicrofacetM>, &launch_loss<LowMicrofacetM>, &launch_check<LowMicrofacetM>,
   {1, 1, 1, 1, 1, 1.3f}, {0, 0, 0, 0, 0, 1}, {kFMax, kFMax, kFMax, kFMax, kFMax, 5}, "pppppp"},
  {"Ward", 5, kFlagSpecular, &launch_eval_pdf<WardM>, &launch_sample<WardM>, &launch_reflectance<WardM>, &launch_loss<WardM>, &launch_check<WardM>,
   {0.5f, 0.5f, 0.5f, 0.1f, 0.1f}, {0, 0, 0, kEpsF, kEpsF}, {1, 1, 1, 1, 1}, "ssspp"},
  {"WardDuer", 5, kFlagSpecular, &launch_eval_pdf<WardDuerM>, &launch_sample<WardDuerM>, &launch_reflectance<WardDuerM>, &launch_loss<WardDuerM>, &launch_check<WardDuerM>,
   {0.5f, 0.5f, 0.5f, 0.1f, 0.1f}, {0, 0, 0, kEpsF, kEpsF}, {1, 1, 1, 1, 1}, "ssspp"},
  {"WardDuerGeislerMoroder", 5, kFlagSpecular, &launch_eval_pdf<WardDGMM>, &launch_sample<WardDGMM>, &launch_reflectance<WardDGMM>, &launch_loss<WardDGMM>, &launch_check<WardDGMM>,
   {0.5f, 0.5f, 0.5f, 0.1f, 0.1f}, {0, 0, 0, kEpsF, kEpsF}, {1, 1, 1, 1, 1}, "ssspp"},
  {"NganWard", 4, kFlagSpecular, &launch_eval_pdf<NganWardM>, &launch_sample<NganWardM>, &launch_reflectance<NganWardM>, &launch_loss<NganWardM>, &launch_check<NganWardM>,
   {0.5f, 0.5f, 0.5f, 0.1f}, {0, 0, 0, kEpsF}, {1, 1, 1, 1}, "sssp"},
  {"NganWardDuer", 4, kFlagSpecular, &launch_eval_pdf<NganWardDuerM>, &launch_sample<NganWardDuerM>, &launch_reflectance<NganWardDuerM>, &launch_loss<NganWardDuerM>, &launch_check<NganWardDuerM>,
   {0.5f, 0.5f, 0.5f, 0.1f}, {0, 0, 0, kEpsF}, {1, 1, 1, 1}, "sssp"},
  {"Phong", 4, kFlagSpecular, &launch_eval_pdf<PhongLobe>, &launch_sample<PhongLobe>, &launch_reflectance<PhongLobe>, &launch_loss<PhongLobe>, &launch_check<PhongLobe>,
   {0.5f, 0.5f, 0.5f, 32.0f}, {0, 0, 0, 0}, {1, 1, 1, kFMax}, "sssp"},
  {"NganBlinnPhong", 4, kFlagSpecular, &launch_eval_pdf<PhongLobe>, &launch_sample<PhongLobe>, &launch_reflectance<PhongLobe>, &launch_loss<PhongLobe>, &launch_check<PhongLobe>,   // ngan.h:43-44
   {0.5f, 0.5f, 0.5f, 32.0f}, {0, 0, 0, 0}, {1, 1, 1, kFMax}, "sssp"},
  {"Lafortune", 7, kFlagSpecular, &launch_eval_pdf<LafortuneM>, &launch_sample<LafortuneM>, &launch_reflectance<LafortuneM>, &launch_loss<LafortuneM>, &launch_check<LafortuneM>,
   {0.5f, 0.5f, 0.5f, -0.57735026919f, -0.57735026919f, 0.57735026919f, 32.0f},
   {0, 0, 0, kFMin, kFMin, kFMin, 0}, {1, 1, 1, kFMax, kFMax, kFMax, kFMax}, "ssspppp"},
  {"NganLafortune", 6, kFlagSpecular, &launch_eval_pdf<NganLafortuneM>, &launch_sample<NganLafortuneM>, &launch_reflectance<NganLafortuneM>, &launch_loss<NganLafortuneM>, &launch_check<NganLafortuneM>,
   {0.5f, 0.5f, 0.5f, -0.57735026919f, 0.57735026919f, 32.0f}, {0, 0, 0, kFMin, kFMin, 0}, {1, 1, 1, kFMax, kFMax, kFMax}, "sssppp"},
  {"AshikhminShirley", 5, kFlagSpecular, &launch_eval_pdf<ASM>, &launch_sample<ASM>, &launch_reflectance<ASM>, &launch_loss<ASM>, &launch_check<ASM>,
   {0.1f, 0.1f, 0.1f, 32.0f, 32.0f}, {0, 0, 0, 0, 0}, {1, 1, 1, kFMax, kFMax}, "ppppp"},
  {"AshikhminShirleyFull", 8, kFlagAll, &launch_eval_pdf<ASFullM>, &launch_sample<ASFullM>, &launch_reflectance<ASFullM>, &launch_loss<ASFullM>, &launch_check<ASFullM>,
   {0.5f, 0.5f, 0.5f, 0.1f, 0.1f, 0.1f, 32.0f, 32.0f}, {0, 0, 0, 0, 0, 0, 0, 0}, {1, 1, 1, 1, 1, 1, kFMax, kFMax}, "dddppppp"},
  {"LowAshikhminShirley", 5, kFlagSpecular, &launch_eval_pdf<LowASM>, &launch_sample<LowASM>, &launch_reflectance<LowASM>, &launch_loss<LowASM>, &launch_check<LowASM>,
   {0.5f, 0.5f, 0.5f, 1.3f, 32.0f}, {0, 0, 0, 1, 0}, {1, 1, 1, 5, kFMax}, "ssspp"},
  {"NganAshikhminShirley", 5, kFlagSpecular, &launch_eval_pdf<NganASM>, &launch_sample<NganASM>, &launch_reflectance<NganASM>, &launch_loss<NganASM>, &launch_check<NganASM>,
   {0.5f, 0.5f, 0.5f, 0.1f, 32.0f}, {0, 0, 0, 0, 0}, {1, 1, 1, 1, kFMax}, "ssspp"},
  {"LowSmooth", 6, kFlagSpecular, &launch_eval_pdf<LowSmooth>, &launch_sample<LowSmooth>, &launch_reflectance<LowSmooth>, &launch_loss<LowSmooth>, &launch_check<LowSmooth>,
   {1, 1, 1, 1, 1, 1.3f}, {0, 0, 0, 0, 0, 1}, {kFMax, kFMax, kFMax, kFMax, kFMax, 5}, "pppppp"},
  // bsdfmodel/bagher.h:62-68: albedo, K, Lambda, c, theta0, k (ndf/sgd.h:197-203, Dependent),
  // alpha, p (sgd.h:107-111), eta = (F0, F1) RGB (bagher.h:31, default {1, 0}, lower {0, -1})
  {"Bagher", 30, kFlagSpecular, &launch_eval_pdf<Bagher>, &launch_sample<Bagher>, &launch_reflectance<Bagher>, &launch_loss<Bagher>, &launch_check<Bagher>,
   {0.5f, 0.5f, 0.5f, 7.5f, 7.5f, 7.5f, 1, 1, 1, 1, 1, 1, 1.5707963705062866f, 1.5707963705062866f, 1.5707963705062866f,
    1, 1, 1, 0.1f, 0.1f, 0.1f, 0.64f, 0.64f, 0.64f, 1, 1, 1, 0, 0, 0},
   {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, kEpsF, kEpsF, kEpsF, 0, 0, 0, 0, 0, 0, -1, -1, -1},
   {1, 1, 1, kFMax, kFMax, kFMax, kFMax, kFMax, kFMax, kFMax, kFMax, kFMax, kFMax, kFMax, kFMax, kFMax, kFMax, kFMax,
    1, 1, 1, kFMax, kFMax, kFMax, 1, 1, 1, 1, 1, 1}, "sssxxxxxxxxxxxxxxxpppppppppppp"},
  // EPD (bsdfmodel/holzschuchpacanowski.h:34-42): beta, p (ndf/epd.h:180-182), eta = complex ior (n, k)
  {"EPD", 4, kFlagSpecular, &launch_eval_pdf<EpdM>, &launch_sample<EpdM>, &launch_reflectance<EpdM>, &launch_loss<EpdM>, &launch_check<EpdM>,
   {0.003f, 0.2f, 1.3f, 0.0f}, {0.0f, 0.0f, 0.1f, 0.0f}, {0.5f, 5.0f, 5.0f, 10.0f}, "pppp"},
  // He family (bsdfmodel/he.h:473-477, :489-496; ngan.h:166-167): roughness, autocorrelation, eta (complex RGB:
  // n RGB, k RGB; NganHe: albedo first and a scalar ior)
#define BBM_HIP_HE_ENTRY(NAME, M)                                                                             \
  {NAME, 8, kFlagSpecular, &launch_eval_pdf<M>, &launch_sample<M>, &launch_reflectance<M>, &launch_loss<M>, &launch_check<M>, \
   {0.18f, 3.0f, 1.3f, 1.3f, 1.3f, 0, 0, 0}, {0, 0, 0.1f, 0.1f, 0.1f, 0, 0, 0},                                 \
   {kFMax, kFMax, 5, 5, 5, 10, 10, 10}, "pppppppp"}
  BBM_HIP_HE_ENTRY("He", HeM),
  BBM_HIP_HE_ENTRY("HeWestin", HeWestinM),
  BBM_HIP_HE_ENTRY("HeHolzschuch", HeHolzschuchM),
  {"NganHe", 6, kFlagSpecular, &launch_eval_pdf<NganHeM>, &launch_sample<NganHeM>, &launch_reflectance<NganHeM>, &launch_loss<NganHeM>, &launch_check<NganHeM>,
   {0.5f, 0.5f, 0.5f, 0.18f, 3.0f, 1.3f}, {0, 0, 0, 0, 0, 1}, {1, 1, 1, kFMax, kFMax, 5}, "sssppp"},
  // Merl (staticmodel/merl.h:224-225): no attributes in the reference (the data comes from a file); the two
  // slots hold the device address of a table built by bbm_hip_merl_table, flagged Dependent so no fit moves them
  {"Merl", 2, kFlagAll, &launch_eval_pdf<Merl>, &launch_sample<Merl>, &launch_reflectance<Merl>, &launch_loss<Merl>, &launch_check<Merl>,
   {0, 0}, {0, 0}, {0, 0}, "xx"},
};
constexpr int kNumSingle = int(sizeof(kSingle) / sizeof(kSingle[0]));
static_assert(Lambertian::kParams == 3 && OrenNayar::kParams == 4 && CookTorranceM::kParams == 5 && GGXM::kParams == 5 &&
              CookTorranceHeitzM::kParams == 6 && GGXHeitzM::kParams == 6 && NganCookTorranceM::kParams == 5 &&
              PhongWalterM::kParams == 5 && RibardiereM::kParams == 6 && RibardiereAnisoM::kParams == 7 &&
              LowMicrofacetM::kParams == 6 && WardM::kParams == 5 && NganWardM::kParams == 4 &&
              PhongLobe::kParams == 4 && LafortuneM::kParams == 7 && NganLafortuneM::kParams == 6 &&
              ASM::kParams == 5 && ASFullM::kParams == 8 && LowASM::kParams == 5 && NganASM::kParams == 5 &&
              LowSmooth::kParams == 6 && Bagher::kParams == 30 && EpdM::kParams == 4 && HeM::kParams == 8 && NganHeM::kParams == 6, "registry nparams must match the compositions");

// Aggregate(Lambertian, X) (aggregatemodel.h:22-233): parameters, defaults, bounds and attribute
// flags are Lambertian's followed by X's; `child` names the registry entry X.
struct AggregateSpec
{
  const char* name;
  const char* child;
  uint32_t components;
  EvalLauncher eval_pdf;
  SampleLauncher sample;
  ReflLauncher reflectance;
  LossLauncher loss;
  CheckLauncher check;
};
#define BBM_HIP_AGG(KEY, CHILD, M) \
  {KEY, CHILD, kFlagDiffuse | M::kComponent, &launch_eval_pdf<M>, &launch_sample<M>, &launch_reflectance<M>, &launch_loss<M>, \
   &launch_check<M>}
const AggregateSpec kAggregates[] = {
  BBM_HIP_AGG("Aggregate<Lambertian,Bagher>", "Bagher", AggBagherM),                      // fits/bagher_sgd.fit
  BBM_HIP_AGG("Aggregate<Lambertian,CookTorrance>", "CookTorrance", AggCookTorranceM),    // docs/source/fitting.rst:31-33
  BBM_HIP_AGG("Aggregate<Lambertian,GGX>", "GGX", AggGGXM),
  BBM_HIP_AGG("Aggregate<Lambertian,LowCookTorrance>", "LowCookTorrance", AggCookTorranceM),   // fits/low_cooktorrance_E*.fit
  BBM_HIP_AGG("Aggregate<Lambertian,LowAshikhminShirley>", "LowAshikhminShirley", AggLowASM),  // fits/low_ashikhminshirley_E*.fit
  BBM_HIP_AGG("Aggregate<Lambertian,LowMicrofacetFit>", "LowMicrofacetFit", AggLowMicrofacetM),  // fits/low_lowmicrofacet_E2.fit
  BBM_HIP_AGG("Aggregate<Lambertian,LowSmooth>", "LowSmooth", AggLowSmoothM),             // fits/low_lowsmooth_E2.fit
  BBM_HIP_AGG("Aggregate<Lambertian,NganAshikhminShirley>", "NganAshikhminShirley", AggNganASM),  // fits/ngan_ashikhminshirley.fit
  BBM_HIP_AGG("Aggregate<Lambertian,NganBlinnPhong>", "NganBlinnPhong", AggPhongM),       // fits/ngan_blinnphong.fit
  BBM_HIP_AGG("Aggregate<Lambertian,NganCookTorrance>", "NganCookTorrance", AggNganCookTorranceM),  // fits/ngan_cooktorrance.fit
  BBM_HIP_AGG("Aggregate<Lambertian,NganLafortune>", "NganLafortune", AggNganLafortuneM),  // fits/ngan_lafortune.fit
  BBM_HIP_AGG("Aggregate<Lambertian,NganWard>", "NganWard", AggNganWardM),                 // fits/ngan_ward.fit
  BBM_HIP_AGG("Aggregate<Lambertian,NganWardDuer>", "NganWardDuer", AggNganWardDuerM),     // fits/ngan_wardduer.fit
  BBM_HIP_AGG("Aggregate<Lambertian,NganHe>", "NganHe", AggNganHeM),                       // fits/ngan_he.fit
};

const ModelEntry* single(const char* name)
{
  for (const auto& e : kSingle)
    if (std::strcmp(e.name, name) == 0) return &e;
  return nullptr;
}

struct Registry
{
  std::vector<ModelEntry> models;
  std::vector<std::string> attrs;   // storage for the aggregates' attribute strings
  Registry()
  {
    models.assign(kSingle, kSingle + kNumSingle);
    const ModelEntry* lam = single("Lambertian");
    attrs.reserve(sizeof(kAggregates) / sizeof(kAggregates[0]));
    for (const auto& g : kAggregates)
    {
      const ModelEntry* c = single(g.child);
      ModelEntry e{};
      e.name = g.name;
      e.nparams = lam->nparams + c->nparams;
      e.components = g.components;
      e.eval_pdf = g.eval_pdf; e.sample = g.sample; e.reflectance = g.reflectance; e.loss = g.loss; e.check = g.check;
      for (int i = 0; i < lam->nparams; ++i)
      {
        e.defaults[i] = lam->defaults[i]; e.lower[i] = lam->lower[i]; e.upper[i] = lam->upper[i];
      }
      for (int i = 0; i < c->nparams; ++i)
      {
        e.defaults[lam->nparams + i] = c->defaults[i];
        e.lower[lam->nparams + i] = c->lower[i];
        e.upper[lam->nparams + i] = c->upper[i];
      }
      attrs.push_back(std::string(lam->attrs) + c->attrs);
      e.attrs = attrs.back().c_str();
      models.push_back(e);
    }
  }
};

const Registry& registry()
{
  static const Registry r;
  return r;
}

int num_models() { return int(registry().models.size()); }
// a registry id, or a fused aggregate's id with BBM_HIP_RUNTIME_AGGREGATE (its aggregatebsdf semantics)
bool runtime_id(int id) { return id >= 0 && (id & BBM_HIP_RUNTIME_AGGREGATE) != 0; }
const ModelEntry* entry(int id)
{
  const int base = (id >= 0) ? (id & ~(BBM_HIP_RUNTIME_AGGREGATE | BBM_HIP_CALL_EXACT | BBM_HIP_CALL_DEFAULT)) : id;
  if (base < 0 || base >= num_models()) return nullptr;
  const ModelEntry* e = &registry().models[size_t(base)];
  if (runtime_id(id) && base < kNumSingle) return nullptr;    // the flag applies to fused aggregates only
  return e;
}
static_assert(kAggregateModeSlot == kMaxParams - 1, "the aggregate mode travels in the parameter block's last slot");

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
  a.p.v[kAggregateModeSlot] = runtime_id(model_id) ? 1.0f : 0.0f;
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
__global__ __launch_bounds__(kBlock) void k_fill_dirs(uint64_t key, uint64_t offset, uint64_t n, int mode,
                                                       float* __restrict__ x, float* __restrict__ y, float* __restrict__ z)
{
  math_tables_init();
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

__global__ __launch_bounds__(kBlock) void k_linearize(LinDesc d, uint64_t begin, uint64_t n, float* __restrict__ ix,
                                                      float* __restrict__ iy, float* __restrict__ iz, float* __restrict__ ox,
                                                      float* __restrict__ oy, float* __restrict__ oz)
{
  math_tables_init();
  const uint64_t stride = uint64_t(gridDim.x) * kBlock;
  for (uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride)
  {
    v3 in, out;
    lin_pair(d, begin + i, in, out);
    ix[i] = in.x; iy[i] = in.y; iz[i] = in.z;
    ox[i] = out.x; oy[i] = out.y; oz[i] = out.z;
  }
}

int to_desc(const bbm_hip_linearizer* lin, LinDesc& d)
{
  if (!lin) return fail(BBM_HIP_ERR_INVALID_ARG, "linearizer is NULL");
  if (lin->kind != kLinSpherical && lin->kind != kLinMerl)
    return fail(BBM_HIP_ERR_INVALID_ARG, "linearizer kind must be BBM_LIN_SPHERICAL or BBM_LIN_MERL");
  std::memset(&d, 0, sizeof(d));
  d.kind = lin->kind;
  for (int k = 0; k < 2; ++k)
  {
    if (lin->samples_in[k] == 0 || lin->samples_out[k] == 0)
      return fail(BBM_HIP_ERR_INVALID_ARG, "linearizer sample counts must be positive");
    d.s_in[k] = lin->samples_in[k];
    d.s_out[k] = lin->samples_out[k];
    d.start_in[k] = lin->start_in[k];
    d.start_out[k] = lin->start_out[k];
    d.size_in[k] = lin->end_in[k] - lin->start_in[k];      // _sizeIn(endIn - startIn), float
    d.size_out[k] = lin->end_out[k] - lin->start_out[k];
  }
  return BBM_HIP_OK;
}

}  // namespace

__global__ __launch_bounds__(kBlock) void k_loss_final(const double* block_sums, int nblocks, int nprobes, double* sums)
{
  math_tables_init();
  __shared__ double part[kBlock];
  const int p = blockIdx.x;
  double t = 0.0;
  for (int b = threadIdx.x; b < nblocks; b += kBlock) t += block_sums[size_t(b) * nprobes + p];
  part[threadIdx.x] = t;
  __syncthreads();
  for (int w = kBlock / 2; w > 0; w >>= 1)
  {
    if (int(threadIdx.x) < w) part[threadIdx.x] += part[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) sums[p] = part[0];
}

// partials [slot][b][kCheckAcc] -> acc[slot][kCheckAcc]: one wave per slot, fixed order
__global__ __launch_bounds__(64) void k_check_final(const double* partial, int nblocks, double* acc)
{
  math_tables_init();
  const int slot = blockIdx.x;
  double r[kCheckAcc];
#pragma unroll
  for (int e = 0; e < kCheckAcc; ++e) r[e] = 0.0;
  r[kCheckSums] = r[kCheckSums + 2] = -1.0;
  r[kCheckSums + 1] = r[kCheckSums + 3] = 1.8e19;
  for (int b = threadIdx.x; b < nblocks; b += 64)
  {
    const double* p = partial + (size_t(slot) * nblocks + b) * kCheckAcc;
#pragma unroll
    for (int e = 0; e < kCheckSums; ++e) r[e] += p[e];
    max_pair(r[kCheckSums], r[kCheckSums + 1], p[kCheckSums], p[kCheckSums + 1]);
    max_pair(r[kCheckSums + 2], r[kCheckSums + 3], p[kCheckSums + 2], p[kCheckSums + 3]);
  }
  wave_reduce_check(r);
  if (threadIdx.x == 0)
  {
#pragma unroll
    for (int e = 0; e < kCheckAcc; ++e) acc[size_t(slot) * kCheckAcc + e] = r[e];
  }
}

namespace {

// draw k of a check test: base key of the stream (test, k); the slot is mixed in by check_key

__global__ __launch_bounds__(kBlock) void k_draws(uint64_t key, uint64_t offset, uint64_t n, float* u0, float* u1)
{
  math_tables_init();
  const uint64_t stride = uint64_t(gridDim.x) * kBlock;
  for (uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride)
    uniform2(key, offset + i, u0[i], u1[i]);
}

__global__ __launch_bounds__(kBlock) void k_trials(uint64_t base, int ntrials, int sphere, float* x, float* y, float* z)
{
  math_tables_init();
  const int t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= ntrials) return;
  float u0, u1;
  uniform2(check_key(base, t), 0, u0, u1);
  const v3 d = sphere_dir(u0, u1, sphere == 0);
  x[t] = d.x; y[t] = d.y; z[t] = d.z;
}

__global__ __launch_bounds__(kBlock) void k_sphere_dirs(const float* u0, const float* u1, uint64_t n, int hemisphere,
                                                        float* x, float* y, float* z)
{
  math_tables_init();
  const uint64_t stride = uint64_t(gridDim.x) * kBlock;
  for (uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride)
  {
    const v3 d = sphere_dir(u0[i], u1[i], hemisphere != 0);
    x[i] = d.x; y[i] = d.y; z[i] = d.z;
  }
}

// bbm_hip_libm_eval: the device's restated libm floats, elementwise
__global__ __launch_bounds__(kBlock) void k_libm(int func, const float* a, const float* b, float* out, uint64_t n)
{
  math_tables_init();
  const uint64_t stride = uint64_t(gridDim.x) * kBlock;
  for (uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride)
  {
    const float x = a[i];
    float r;
    switch (func)
    {
      case BBM_HIP_LIBM_EXPF: r = expf_glibc(x); break;
      case BBM_HIP_LIBM_LOGF: r = logf_glibc(x); break;
      case BBM_HIP_LIBM_POWF: r = powf_glibc(x, b[i]); break;
      case BBM_HIP_LIBM_ERFF: r = erff_glibc(x); break;
      case BBM_HIP_LIBM_ONE_PLUS_SQRT: r = f_one_plus_sqrt(1.0 + double(x) * double(b[i])); break;
      case BBM_HIP_LIBM_SINF: { float c; sincosf_glibc(x, &r, &c); } break;
      case BBM_HIP_LIBM_COSF: { float sn; sincosf_glibc(x, &sn, &r); } break;
      case BBM_HIP_LIBM_ATAN2F: r = atan2f_glibc(x, b[i]); break;
      case BBM_HIP_LIBM_THETA: r = theta_of(mk3(x, 0.0f, b[i])); break;
      default: r = erfcf_glibc(x); break;
    }
    out[i] = r;
  }
}

int launched()
{
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(BBM_HIP_ERR_HIP, std::string("kernel launch failed: ") + hipGetErrorString(e));
  return BBM_HIP_OK;
}

}  // namespace

}  // namespace bbmhip

using namespace bbmhip;

extern "C" {

int bbm_hip_abi_version(void) { return BBM_HIP_ABI_VERSION; }

int bbm_hip_set_exact_subnormals(int on) { return exact_subnormals().exchange(on != 0 ? 1 : 0); }

size_t bbm_hip_scratch_trim(void) { return scratch_trim(); }

size_t bbm_hip_scratch_trim_captured(void) { return scratch_trim_captured(); }

size_t bbm_hip_scratch_bytes(void) { return scratch_bytes(); }

const char* bbm_hip_last_error(void) { return g_last_error.c_str(); }

int bbm_hip_num_models(void) { return num_models(); }

const char* bbm_hip_model_name(int model_id)
{
  const ModelEntry* e = entry(model_id);
  return e ? e->name : nullptr;
}

int bbm_hip_model_id(const char* name)
{
  if (!name) return fail(BBM_HIP_ERR_INVALID_ARG, "name is NULL");
  for (int i = 0; i < num_models(); ++i)
    if (std::strcmp(registry().models[size_t(i)].name, name) == 0) return i;
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
  const CallExactScope mode_scope(model_id);
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
  const CallExactScope mode_scope(model_id);
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

int bbm_hip_reflectance(int model_id, const float* params, int nparams,
                        const float* out_x, const float* out_y, const float* out_z,
                        const uint8_t* mask, size_t n, uint32_t component, uint32_t unit,
                        float* r, float* g, float* b, void* stream)
{
  (void)unit;
  const CallExactScope mode_scope(model_id);
  EvalArgs tmp;
  const ModelEntry* e;
  int rc = prepare(model_id, params, nparams, n, tmp, e);
  if (rc) return rc;
  if (n == 0) return BBM_HIP_OK;
  if ((rc = check_dirs(out_x, out_y, out_z, "out"))) return rc;
  if (!r || !g || !b) return fail(BBM_HIP_ERR_INVALID_ARG, "reflectance output pointer is NULL");
  ReflArgs a;
  std::memset(&a, 0, sizeof(a));
  a.p = tmp.p;
  a.n = n;
  a.ox = out_x; a.oy = out_y; a.oz = out_z; a.mask = mask; a.r = r; a.g = g; a.b = b;
  a.component = component & kFlagAll;
  return e->reflectance(a, static_cast<hipStream_t>(stream));
}

// ------------------------------------------------------------------------------- doubleRGB (f64.hip)

static int prepare_f64(int model_id, const double* params, int nparams, const ModelEntry*& e,
                       const f64::F64Launchers*& l, f64::ParamBlockF64& p)
{
  e = entry(model_id);
  if (!e) return fail(BBM_HIP_ERR_INVALID_MODEL, "unknown model id " + std::to_string(model_id));
  l = f64::f64_launchers(e->name);
  if (!l) return fail(BBM_HIP_ERR_UNSUPPORTED, std::string(e->name) + ": no doubleRGB kernel");
  if (nparams != e->nparams)
    return fail(BBM_HIP_ERR_INVALID_ARG, std::string(e->name) + ": expected " + std::to_string(e->nparams) +
                                             " parameters, got " + std::to_string(nparams));
  if (nparams > 0 && !params) return fail(BBM_HIP_ERR_INVALID_ARG, "params is NULL");
  std::memset(&p, 0, sizeof(p));
  for (int i = 0; i < nparams; ++i) p.v[i] = params[i];
  p.v[f64::kMaxParamsF64 - 1] = runtime_id(model_id) ? 1.0 : 0.0;
  return BBM_HIP_OK;
}

int bbm_hip_model_has_f64(int model_id)
{
  const ModelEntry* e = entry(model_id);
  if (!e) return fail(BBM_HIP_ERR_INVALID_MODEL, "unknown model id " + std::to_string(model_id));
  return f64::f64_launchers(e->name) ? 1 : 0;
}

int bbm_hip_eval_pdf_f64(int model_id, const double* params, int nparams,
                         const double* in_x, const double* in_y, const double* in_z,
                         const double* out_x, const double* out_y, const double* out_z,
                         const uint8_t* mask, size_t n, uint32_t component, uint32_t unit,
                         double* r, double* g, double* b, double* pdf, void* stream)
{
  (void)unit;
  const ModelEntry* e;
  const f64::F64Launchers* l;
  f64::EvalArgsF64 a;
  std::memset(&a, 0, sizeof(a));
  int rc = prepare_f64(model_id, params, nparams, e, l, a.p);
  if (rc) return rc;
  if (n == 0) return BBM_HIP_OK;
  if (!in_x || !in_y || !in_z || !out_x || !out_y || !out_z) return fail(BBM_HIP_ERR_INVALID_ARG, "direction pointer is NULL");
  if (!r || !g || !b || !pdf) return fail(BBM_HIP_ERR_INVALID_ARG, "output pointer is NULL");
  a.ix = in_x; a.iy = in_y; a.iz = in_z; a.ox = out_x; a.oy = out_y; a.oz = out_z;
  a.mask = mask; a.r = r; a.g = g; a.b = b; a.pdf = pdf;
  a.n = n;
  a.component = component & kFlagAll;
  return l->eval_pdf(a, static_cast<hipStream_t>(stream));
}

int bbm_hip_sample_f64(int model_id, const double* params, int nparams,
                       const double* out_x, const double* out_y, const double* out_z,
                       const double* xi0, const double* xi1,
                       const uint8_t* mask, size_t n, uint32_t component, uint32_t unit,
                       double* dir_x, double* dir_y, double* dir_z, double* pdf, uint32_t* flag, void* stream)
{
  (void)unit;
  const ModelEntry* e;
  const f64::F64Launchers* l;
  f64::SampleArgsF64 a;
  std::memset(&a, 0, sizeof(a));
  int rc = prepare_f64(model_id, params, nparams, e, l, a.p);
  if (rc) return rc;
  if (n == 0) return BBM_HIP_OK;
  if (!out_x || !out_y || !out_z) return fail(BBM_HIP_ERR_INVALID_ARG, "out direction pointer is NULL");
  if (!xi0 || !xi1) return fail(BBM_HIP_ERR_INVALID_ARG, "xi pointer is NULL");
  if (!dir_x || !dir_y || !dir_z || !pdf || !flag) return fail(BBM_HIP_ERR_INVALID_ARG, "sample output pointer is NULL");
  a.ox = out_x; a.oy = out_y; a.oz = out_z; a.xi0 = xi0; a.xi1 = xi1; a.mask = mask;
  a.dx = dir_x; a.dy = dir_y; a.dz = dir_z; a.pdf = pdf; a.flag = flag;
  a.n = n;
  a.component = component & kFlagAll;
  return l->sample(a, static_cast<hipStream_t>(stream));
}

int bbm_hip_reflectance_f64(int model_id, const double* params, int nparams,
                            const double* out_x, const double* out_y, const double* out_z,
                            const uint8_t* mask, size_t n, uint32_t component, uint32_t unit,
                            double* r, double* g, double* b, void* stream)
{
  (void)unit;
  const ModelEntry* e;
  const f64::F64Launchers* l;
  f64::ReflArgsF64 a;
  std::memset(&a, 0, sizeof(a));
  int rc = prepare_f64(model_id, params, nparams, e, l, a.p);
  if (rc) return rc;
  if (n == 0) return BBM_HIP_OK;
  if (!out_x || !out_y || !out_z) return fail(BBM_HIP_ERR_INVALID_ARG, "out direction pointer is NULL");
  if (!r || !g || !b) return fail(BBM_HIP_ERR_INVALID_ARG, "reflectance output pointer is NULL");
  a.ox = out_x; a.oy = out_y; a.oz = out_z; a.mask = mask; a.r = r; a.g = g; a.b = b;
  a.n = n;
  a.component = component & kFlagAll;
  return l->reflectance(a, static_cast<hipStream_t>(stream));
}

int bbm_hip_model_param_attrs(int model_id, uint32_t* out, int capacity)
{
  const ModelEntry* e = entry(model_id);
  if (!e) return fail(BBM_HIP_ERR_INVALID_MODEL, "unknown model id " + std::to_string(model_id));
  for (int i = 0; out && i < e->nparams && i < capacity; ++i)
  {
    switch (e->attrs[i])
    {
      case 'd': out[i] = 0x01u; break;
      case 'D': out[i] = 0x02u; break;
      case 's': out[i] = 0x04u; break;
      case 'p': out[i] = 0x08u; break;
      default: out[i] = 0x10u; break;
    }
  }
  return e->nparams;
}

int bbm_hip_linearizer_size(const bbm_hip_linearizer* lin, uint64_t* size)
{
  LinDesc d;
  int rc = to_desc(lin, d);
  if (rc) return rc;
  if (!size) return fail(BBM_HIP_ERR_INVALID_ARG, "size is NULL");
  *size = lin_size(d);
  return BBM_HIP_OK;
}

int bbm_hip_linearize(const bbm_hip_linearizer* lin, uint64_t begin, size_t n,
                      float* in_x, float* in_y, float* in_z, float* out_x, float* out_y, float* out_z,
                      void* stream)
{
  LinDesc d;
  int rc = to_desc(lin, d);
  if (rc) return rc;
  if (n == 0) return BBM_HIP_OK;
  if (begin + n > lin_size(d)) return fail(BBM_HIP_ERR_INVALID_ARG, "linearizer range out of bounds");
  if (!in_x || !in_y || !in_z || !out_x || !out_y || !out_z)
    return fail(BBM_HIP_ERR_INVALID_ARG, "direction pointer is NULL");
  uint64_t blocks = (n + kBlock - 1) / kBlock;
  if (blocks > kMaxBlocks) blocks = kMaxBlocks;
  hipLaunchKernelGGL(k_linearize, dim3(unsigned(blocks)), dim3(kBlock), 0, static_cast<hipStream_t>(stream), d, begin,
                     uint64_t(n), in_x, in_y, in_z, out_x, out_y, out_z);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(BBM_HIP_ERR_HIP, std::string("kernel launch failed: ") + hipGetErrorString(e));
  return BBM_HIP_OK;
}

size_t bbm_hip_loss_workspace_size(int nprobes)
{
  // per-block partial sums, then the probes' constructed models (kLossModelBytes each, 256-byte aligned)
  return nprobes > 0 ? size_t(kLossMaxBlocks) * size_t(nprobes) * sizeof(double) + size_t(nprobes) * kLossModelBytes : 0;
}

namespace {
int loss_common(int model_id, const float* probes, int nparams, int nprobes, const float* ref_r, const float* ref_g,
                const float* ref_b, size_t n, int loss_kind, uint32_t component, double* sums, void* workspace,
                size_t workspace_bytes, LossArgs& a, const ModelEntry*& e)
{
  e = entry(model_id);
  if (!e) return fail(BBM_HIP_ERR_INVALID_MODEL, "unknown model id " + std::to_string(model_id));
  if (nparams != e->nparams)
    return fail(BBM_HIP_ERR_INVALID_ARG, std::string(e->name) + ": expected " + std::to_string(e->nparams) +
                                             " parameters, got " + std::to_string(nparams));
  if (nprobes <= 0) return fail(BBM_HIP_ERR_INVALID_ARG, "nprobes must be positive");
  if (loss_kind < BBM_LOSS_NGAN_L2 || loss_kind > BBM_LOSS_BIERON_LOG) return fail(BBM_HIP_ERR_INVALID_ARG, "unknown loss kind");
  if (!probes || !sums) return fail(BBM_HIP_ERR_INVALID_ARG, "probes / sums pointer is NULL");
  if (n > 0 && (!ref_r || !ref_g || !ref_b)) return fail(BBM_HIP_ERR_INVALID_ARG, "reference pointer is NULL");
  if (!workspace || workspace_bytes < bbm_hip_loss_workspace_size(nprobes))
    return fail(BBM_HIP_ERR_INVALID_ARG, "workspace too small (bbm_hip_loss_workspace_size)");
  std::memset(&a, 0, sizeof(a));
  a.n = n;
  a.ref_r = ref_r; a.ref_g = ref_g; a.ref_b = ref_b;
  a.probes = probes; a.nprobes = nprobes; a.stride = nparams; a.loss_kind = loss_kind;
  a.component = component & kFlagAll;
  a.block_sums = static_cast<double*>(workspace);
  a.models = static_cast<char*>(workspace) + size_t(kLossMaxBlocks) * size_t(nprobes) * sizeof(double);
  a.sums = sums;
  return BBM_HIP_OK;
}
}  // namespace

int bbm_hip_loss(int model_id, const float* probes, int nparams, int nprobes,
                 const bbm_hip_linearizer* lin, uint64_t begin, size_t n,
                 const float* ref_r, const float* ref_g, const float* ref_b,
                 int loss_kind, uint32_t component, uint32_t unit,
                 double* sums, void* workspace, size_t workspace_bytes, void* stream)
{
  (void)unit;
  LinDesc d;
  int rc = to_desc(lin, d);
  if (rc) return rc;
  if (begin + n > lin_size(d)) return fail(BBM_HIP_ERR_INVALID_ARG, "linearizer range out of bounds");
  LossArgs a;
  const ModelEntry* e = nullptr;
  rc = loss_common(model_id, probes, nparams, nprobes, ref_r, ref_g, ref_b, n, loss_kind, component, sums, workspace,
                   workspace_bytes, a, e);
  if (rc) return rc;
  a.lin = d;
  a.begin = begin;
  return e->loss(a, static_cast<hipStream_t>(stream));
}

int bbm_hip_loss_pairs(int model_id, const float* probes, int nparams, int nprobes, size_t n,
                       const float* in_x, const float* in_y, const float* in_z,
                       const float* out_x, const float* out_y, const float* out_z,
                       const float* ref_r, const float* ref_g, const float* ref_b,
                       int loss_kind, uint32_t component, uint32_t unit,
                       double* sums, void* workspace, size_t workspace_bytes, void* stream)
{
  (void)unit;
  LossArgs a;
  const ModelEntry* e = nullptr;
  int rc = loss_common(model_id, probes, nparams, nprobes, ref_r, ref_g, ref_b, n, loss_kind, component, sums, workspace,
                       workspace_bytes, a, e);
  if (rc) return rc;
  if (n > 0 && (!in_x || !in_y || !in_z || !out_x || !out_y || !out_z))
    return fail(BBM_HIP_ERR_INVALID_ARG, "direction pointer is NULL");
  a.lin.kind = kLinSpherical;    // unused: the pairs are given
  a.pairs[0] = in_x; a.pairs[1] = in_y; a.pairs[2] = in_z;
  a.pairs[3] = out_x; a.pairs[4] = out_y; a.pairs[5] = out_z;
  return e->loss(a, static_cast<hipStream_t>(stream));
}

int bbm_hip_epd_g1_table(float* out, int capacity)
{
  return epd_table_host(out, capacity);
}

int bbm_hip_merl_table(const double* raw, uint32_t theta_h, uint32_t theta_d, uint32_t phi_d, float* table,
                       void* stream)
{
  if (!raw || !table) return fail(BBM_HIP_ERR_INVALID_ARG, "bbm_hip_merl_table: null pointer");
  if (theta_h != uint32_t(kMerlThetaH) || theta_d != uint32_t(kMerlThetaD) || phi_d != uint32_t(kMerlPhiD))
    return fail(BBM_HIP_ERR_INVALID_ARG, "BBM: not a recognized MERL BRDF (dimensions " + std::to_string(theta_h) + " x " +
                                         std::to_string(theta_d) + " x " + std::to_string(phi_d) + ", expected 90 x 90 x 180)");
  return merl_table_launch(raw, table, static_cast<hipStream_t>(stream));
}

size_t bbm_hip_check_workspace_size(const bbm_hip_check_desc* d)
{
  if (!d || d->nslots <= 0) return 0;
  return size_t(d->nslots) * check_blocks(d->n, d->nslots) * kCheckAcc * sizeof(double);
}

int bbm_hip_check(int model_id, const float* params, int nparams, const bbm_hip_check_desc* d,
                  double* acc, uint64_t* counts, void* workspace, size_t workspace_bytes, void* stream)
{
  const CallExactScope mode_scope(model_id);
  const ModelEntry* e = entry(model_id);
  if (!e) return fail(BBM_HIP_ERR_INVALID_MODEL, "unknown model id " + std::to_string(model_id));
  if (nparams != e->nparams)
    return fail(BBM_HIP_ERR_INVALID_ARG, std::string(e->name) + ": expected " + std::to_string(e->nparams) +
                                             " parameters, got " + std::to_string(nparams));
  if (nparams > 0 && !params) return fail(BBM_HIP_ERR_INVALID_ARG, "params is NULL");
  if (!d) return fail(BBM_HIP_ERR_INVALID_ARG, "check descriptor is NULL");
  if (d->test < 0 || d->test >= kCheckNumTests) return fail(BBM_HIP_ERR_INVALID_ARG, "unknown check test");
  if (d->nslots <= 0 || d->nslots > 65535) return fail(BBM_HIP_ERR_INVALID_ARG, "nslots must be in [1, 65535]");
  const bool chi2 = d->test == kCheckSamplePdf || d->test == kCheckSampleCount;
  const uint64_t bins = uint64_t(d->theta_bins) * d->phi_bins;
  if (chi2 && (d->theta_bins == 0 || d->phi_bins == 0 || bins > (1u << 20)))
    return fail(BBM_HIP_ERR_INVALID_ARG, "theta_bins / phi_bins must be positive (at most 2^20 bins)");
  if (d->test == kCheckSamplePdf && d->nslots % bins != 0)
    return fail(BBM_HIP_ERR_INVALID_ARG, "SAMPLE_PDF: nslots must be trials x theta_bins x phi_bins");
  const bool needs_dirs = d->test == kCheckReflectance || d->test == kCheckPdfInt || chi2;
  if (needs_dirs && (!d->slot_x || !d->slot_y || !d->slot_z))
    return fail(BBM_HIP_ERR_INVALID_ARG, "this test needs slot directions");
  if (d->test == kCheckSampleCount ? !counts : !acc) return fail(BBM_HIP_ERR_INVALID_ARG, "acc / counts pointer is NULL");
  if (d->test != kCheckSampleCount && (!workspace || workspace_bytes < bbm_hip_check_workspace_size(d)))
    return fail(BBM_HIP_ERR_INVALID_ARG, "workspace too small (bbm_hip_check_workspace_size)");
  CheckArgs a;
  std::memset(&a, 0, sizeof(a));
  for (int k = 0; k < 3; ++k) a.key[k] = check_base_key(d->seed, d->test, k);
  a.begin = d->begin; a.n = d->n; a.nslots = d->nslots;
  a.sx = d->slot_x; a.sy = d->slot_y; a.sz = d->slot_z;
  a.sphere = d->sphere; a.importance = d->importance; a.include_zero = d->include_zero_pdf;
  a.nth = d->theta_bins; a.nph = d->phi_bins;
  a.partial = static_cast<double*>(workspace);
  a.counts = reinterpret_cast<unsigned long long*>(counts);
  for (int i = 0; i < nparams; ++i) a.p.v[i] = params[i];
  a.p.v[kAggregateModeSlot] = runtime_id(model_id) ? 1.0f : 0.0f;
  const hipStream_t s = static_cast<hipStream_t>(stream);
  if (d->test == kCheckSampleCount)
  {
    const hipError_t me = hipMemsetAsync(counts, 0, size_t(d->nslots) * bins * sizeof(uint64_t), s);
    if (me != hipSuccess) return fail(BBM_HIP_ERR_HIP, std::string("hipMemsetAsync: ") + hipGetErrorString(me));
  }
  if (d->n == 0 && d->test != kCheckSampleCount)
  {
    const hipError_t me = hipMemsetAsync(acc, 0, size_t(d->nslots) * kCheckAcc * sizeof(double), s);
    return me == hipSuccess ? BBM_HIP_OK : fail(BBM_HIP_ERR_HIP, std::string("hipMemsetAsync: ") + hipGetErrorString(me));
  }
  if (d->n == 0) return BBM_HIP_OK;
  return e->check(d->test, a, acc, s);
}

int bbm_hip_check_draws(int test, uint64_t seed, int slot, int draw, uint64_t offset, size_t n,
                        float* xi0, float* xi1, void* stream)
{
  if (n == 0) return BBM_HIP_OK;
  if (!xi0 || !xi1) return fail(BBM_HIP_ERR_INVALID_ARG, "xi pointer is NULL");
  if (test < 0 || test >= kCheckNumTests || draw < 0 || draw > 2 || slot < 0)
    return fail(BBM_HIP_ERR_INVALID_ARG, "test / draw / slot out of range");
  uint64_t blocks = (n + kBlock - 1) / kBlock;
  if (blocks > kMaxBlocks) blocks = kMaxBlocks;
  hipLaunchKernelGGL(k_draws, dim3(unsigned(blocks)), dim3(kBlock), 0, static_cast<hipStream_t>(stream),
                     check_key(check_base_key(seed, test, draw), slot), offset, uint64_t(n), xi0, xi1);
  return launched();
}

int bbm_hip_check_trials(int test, uint64_t seed, int ntrials, int sphere, float* x, float* y, float* z, void* stream)
{
  if (ntrials <= 0) return ntrials == 0 ? BBM_HIP_OK : fail(BBM_HIP_ERR_INVALID_ARG, "ntrials < 0");
  if (!x || !y || !z) return fail(BBM_HIP_ERR_INVALID_ARG, "direction pointer is NULL");
  if (test < 0 || test >= kCheckNumTests) return fail(BBM_HIP_ERR_INVALID_ARG, "unknown check test");
  // the trial direction is its own stream (draw index 3), sample 0
  hipLaunchKernelGGL(k_trials, dim3(unsigned((ntrials + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), check_base_key(seed, test, 3), ntrials, sphere, x, y, z);
  return launched();
}

int bbm_hip_sphere_dirs(const float* xi0, const float* xi1, size_t n, int hemisphere, float* x, float* y, float* z,
                        void* stream)
{
  if (n == 0) return BBM_HIP_OK;
  if (!xi0 || !xi1 || !x || !y || !z) return fail(BBM_HIP_ERR_INVALID_ARG, "pointer is NULL");
  uint64_t blocks = (n + kBlock - 1) / kBlock;
  if (blocks > kMaxBlocks) blocks = kMaxBlocks;
  hipLaunchKernelGGL(k_sphere_dirs, dim3(unsigned(blocks)), dim3(kBlock), 0, static_cast<hipStream_t>(stream), xi0, xi1,
                     uint64_t(n), hemisphere, x, y, z);
  return launched();
}

int bbm_hip_libm_eval(int func, const float* a, const float* b, float* out, size_t n, void* stream)
{
  if (n == 0) return BBM_HIP_OK;
  if (func < BBM_HIP_LIBM_EXPF || func > BBM_HIP_LIBM_THETA)
    return fail(BBM_HIP_ERR_INVALID_ARG, "unknown libm function");
  if (!a || !out || ((func == BBM_HIP_LIBM_POWF || func == BBM_HIP_LIBM_ONE_PLUS_SQRT || func == BBM_HIP_LIBM_ATAN2F || func == BBM_HIP_LIBM_THETA) && !b)) return fail(BBM_HIP_ERR_INVALID_ARG, "pointer is NULL");
  uint64_t blocks = (n + kBlock - 1) / kBlock;
  if (blocks > kMaxBlocks) blocks = kMaxBlocks;
  hipLaunchKernelGGL(k_libm, dim3(unsigned(blocks)), dim3(kBlock), 0, static_cast<hipStream_t>(stream), func, a, b, out,
                     uint64_t(n));
  return launched();
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
