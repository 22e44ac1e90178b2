/* oracle/ref_harness.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never measured as the product).
 *
 * A thin extern "C" shim around the *reference's own headers* (/root/reference/include,
 * /root/reference/backbone/native/include) so that the real BBM native-backbone implementation
 * can be driven from ctypes to (a) generate the golden vectors under tests/golden/ and
 * (b) serve as the "reference" CPU baseline in bench.py (cpu_baseline.kind = "reference").
 *
 * Nothing from the reference is copied here: this file only #includes the reference headers where
 * they lie and instantiates them with the native backbone's floatRGB / doubleRGB configs
 * (backbone/native/include/backbone.h:41-42).  Built by oracle/Makefile into oracle/_ref/.
 *
 * Per-model calls follow the bsdfmodel concept (include/concepts/bsdfmodel.h:33-146):
 *   eval(in, out, component, unit) -> Spectrum, pdf(in, out, component, unit) -> Value,
 *   sample(out, xi, component, unit) -> {direction, pdf, flag}.
 * Parameters are exchanged as the flat vector bbm::parameter_values(model, flag)
 * (include/bbm/bsdf_enumerate.h), in attribute declaration order.
 *
 * Not instantiated (documented in DESIGN.md): He/HeWestin/HeHolzschuch/NganHe (ndf_sampler's
 * default NTTP name fails CTAD on g++ 11, include/ndf/sampler.h:34), EPD (needs the missing
 * precomputed/holzschuchpacanowski/{convolution,normalization}.h blobs), Merl (needs MERL data).
 */
#include "ref_ops.hpp"

namespace bbmref {
// aggregates of two models, defined in ref_fit.cpp
const std::vector<entry>& aggregate_registry();
}

namespace {
using namespace bbmref;

const std::vector<entry>& registry()
{
  static const std::vector<entry> r = {
    BBMREF_ENTRY(lambertian),
    BBMREF_ENTRY(orennayar),
    BBMREF_ENTRY(cooktorrance),
    BBMREF_ENTRY(cooktorranceheitz),
    BBMREF_ENTRY(cooktorrancewalter),
    BBMREF_ENTRY(ggx),
    BBMREF_ENTRY(ggxheitz),
    BBMREF_ENTRY(phongwalter),
    BBMREF_ENTRY(ribardiere),
    BBMREF_ENTRY(ribardiereanisotropic),
    BBMREF_ENTRY(bagher),
    BBMREF_ENTRY(lowcooktorrance),
    BBMREF_ENTRY(lowmicrofacet),
    BBMREF_ENTRY(lowmicrofacetfit),
    BBMREF_ENTRY(ngancooktorrance),
    BBMREF_ENTRY(ward),
    BBMREF_ENTRY(wardduer),
    BBMREF_ENTRY(wardduergeislermoroder),
    BBMREF_ENTRY(nganward),
    BBMREF_ENTRY(nganwardduer),
    BBMREF_ENTRY(phong),
    BBMREF_ENTRY(nganblinnphong),
    BBMREF_ENTRY(lafortune),
    BBMREF_ENTRY(nganlafortune),
    BBMREF_ENTRY(ashikhminshirley),
    BBMREF_ENTRY(ashikhminshirleyfull),
    BBMREF_ENTRY(lowashikhminshirley),
    BBMREF_ENTRY(nganashikhminshirley),
    BBMREF_ENTRY(lowsmooth),
    BBMREF_ENTRY_NS(bbmref, epd),
    BBMREF_ENTRY_NS(bbmref, he),
    BBMREF_ENTRY_NS(bbmref, hewestin),
    BBMREF_ENTRY_NS(bbmref, heholzschuch),
    BBMREF_ENTRY_NS(bbmref, nganhe),
  };
  return r;
}

const entry* find(const char* name)
{
  for(auto& e : registry()) if(std::strcmp(e.name, name) == 0) return &e;
  for(auto& e : aggregate_registry()) if(std::strcmp(e.name, name) == 0) return &e;
  return nullptr;
}

int copy_vec(const std::vector<float>& v, float* out, int cap)
{
  if(out) for(int i = 0; i < int(v.size()) && i < cap; ++i) out[i] = v[i];
  return int(v.size());
}

} // namespace

extern "C" {

// single models first, then the Aggregate(Lambertian, X) entries of ref_fit.cpp
int bbmref_num_models(void) { return int(registry().size() + aggregate_registry().size()); }
const char* bbmref_model_name(int i)
{
  const int a = int(registry().size()), b = int(aggregate_registry().size());
  if(i >= 0 && i < a) return registry()[size_t(i)].name;
  if(i >= a && i < a + b) return aggregate_registry()[size_t(i - a)].name;
  return nullptr;
}

int bbmref_default_params(const char* name, float* out, int cap)
{ auto e = find(name); return e ? copy_vec(e->defaults(), out, cap) : -1; }

int bbmref_param_bounds(const char* name, int upper, float* out, int cap)
{ auto e = find(name); return e ? copy_vec(e->bounds(upper != 0), out, cap) : -1; }

int bbmref_to_string(const char* name, const float* p, int np, char* buf, int cap)
{
  auto e = find(name); if(!e) return -1;
  std::string s = e->to_string(p, np);
  if(buf && cap > 0) { std::strncpy(buf, s.c_str(), size_t(cap - 1)); buf[cap - 1] = 0; }
  return int(s.size());
}

int bbmref_eval_pdf(const char* name, const float* p, int np, size_t n,
                    const float* ix, const float* iy, const float* iz,
                    const float* ox, const float* oy, const float* oz,
                    uint32_t component, uint32_t unit, int mode,
                    float* r, float* g, float* b, float* pdf, int nthreads)
{
  auto e = find(name); if(!e) return -1;
  e->evalpdf_f(p, np, n, ix, iy, iz, ox, oy, oz, component, unit, mode, r, g, b, pdf, nthreads);
  return 0;
}

int bbmref_eval_pdf_double(const char* name, const float* p, int np, size_t n,
                           const float* ix, const float* iy, const float* iz,
                           const float* ox, const float* oy, const float* oz,
                           uint32_t component, uint32_t unit, int mode,
                           double* r, double* g, double* b, double* pdf, int nthreads)
{
  auto e = find(name); if(!e) return -1;
  e->evalpdf_d(p, np, n, ix, iy, iz, ox, oy, oz, component, unit, mode, r, g, b, pdf, nthreads);
  return 0;
}

int bbmref_sample(const char* name, const float* p, int np, size_t n,
                  const float* ox, const float* oy, const float* oz, const float* xi0, const float* xi1,
                  uint32_t component, uint32_t unit,
                  float* dx, float* dy, float* dz, float* pdf, uint32_t* flag, int nthreads)
{
  auto e = find(name); if(!e) return -1;
  e->sample_f(p, np, n, ox, oy, oz, xi0, xi1, component, unit, dx, dy, dz, pdf, flag, nthreads);
  return 0;
}

int bbmref_reflectance(const char* name, const float* p, int np, size_t n,
                       const float* ox, const float* oy, const float* oz,
                       uint32_t component, uint32_t unit, float* r, float* g, float* b)
{
  auto e = find(name); if(!e) return -1;
  e->reflectance_f(p, np, n, ox, oy, oz, component, unit, r, g, b);
  return 0;
}

int bbmref_eval_pdf_dd(const char* name, const float* p, int np, size_t n,
                       const double* ix, const double* iy, const double* iz,
                       const double* ox, const double* oy, const double* oz,
                       uint32_t component, uint32_t unit, int mode,
                       double* r, double* g, double* b, double* pdf, int nthreads)
{
  auto e = find(name); if(!e || !e->evalpdf_dd) return -1;
  e->evalpdf_dd(p, np, n, ix, iy, iz, ox, oy, oz, component, unit, mode, r, g, b, pdf, nthreads);
  return 0;
}

int bbmref_sample_double(const char* name, const float* p, int np, size_t n,
                         const float* ox, const float* oy, const float* oz, const float* xi0, const float* xi1,
                         uint32_t component, uint32_t unit,
                         double* dx, double* dy, double* dz, double* pdf, uint32_t* flag, int nthreads)
{
  auto e = find(name); if(!e || !e->sample_d) return -1;
  e->sample_d(p, np, n, ox, oy, oz, xi0, xi1, component, unit, dx, dy, dz, pdf, flag, nthreads);
  return 0;
}

int bbmref_reflectance_double(const char* name, const float* p, int np, size_t n,
                              const float* ox, const float* oy, const float* oz,
                              uint32_t component, uint32_t unit, double* r, double* g, double* b)
{
  auto e = find(name); if(!e || !e->reflectance_d) return -1;
  e->reflectance_d(p, np, n, ox, oy, oz, component, unit, r, g, b);
  return 0;
}

// bbm::fromString of the model `name` (a model string as printed by toString / stored in fits/*.fit) -> its
// parameter vector (All | Dependent, declaration order); <0 if the reference rejects the string
int bbmref_from_string(const char* name, const char* str, float* out, int cap)
{
  auto e = find(name); if(!e || !e->from_string) return -2;
  return e->from_string(str, out, cap);
}

int bbmref_max_threads(void)
{
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

} // extern "C"
