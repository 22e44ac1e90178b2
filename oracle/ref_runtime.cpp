/* oracle/ref_runtime.cpp -- TEST INFRASTRUCTURE ONLY: the reference's RUNTIME aggregate, bbm::aggregatebsdf
 * (include/bbm/aggregatebsdf.h:40-190), which fromString<bsdf_ptr> / bsdf_import builds from "Aggregate(...)"
 * (include/bbm/bsdf_string_convert.h:52-82: every leaf a make_bsdf_ptr of its model, every "Aggregate" an
 * aggregatebsdf of those bsdf_ptrs).  That fromString itself needs the CMake-generated bbm_bsdfmodels.h
 * (cmake/bbm_helpers.cmake:45-60), which this plain-g++ build does not make; the same objects are built here from
 * the parsed tree instead -- the reference's own bsdf_ptr, bsdf<MODEL> and aggregatebsdf classes, evaluated through
 * their virtual interface.
 *
 * A tree is given in preorder: names[k] a model name or "Aggregate", nkids[k] its child count (0 for a model),
 * np[k] its parameter count, the leaves' parameters back to back in params. */
#include <memory>

namespace {
using namespace bbmref;

template<typename C>
bbm::bsdf_ptr<C> build_runtime(const char* const* names, const int* nkids, const float* params, const int* np,
                               int& node, int& off, bool& ok)
{
  const std::string nm = names[node];
  const int k = nkids[node], npar = np[node];
  ++node;
  if(nm == "Aggregate")
  {
    std::vector<bbm::bsdf_ptr<C>> kids;
    for(int j = 0; j < k; ++j) kids.push_back(build_runtime<C>(names, nkids, params, np, node, off, ok));
    return bbm::make_bsdf_ptr(bbm::aggregatebsdf<C>(kids.begin(), kids.end()));
  }
  bbm::bsdf_ptr<C> ptr;
  const entry* e = find(nm.c_str());
  auto make = e ? (std::is_same_v<C, bbm::floatRGB> ? e->ptr_f : e->ptr_d) : nullptr;
  if(!make) { ok = false; return ptr; }
  make(params + off, npar, &ptr);
  off += npar;
  return ptr;
}

template<typename C>
bool build_tree(int nnodes, const char* const* names, const int* nkids, const float* params, const int* np,
                bbm::bsdf_ptr<C>& out)
{
  int node = 0, off = 0;
  bool ok = true;
  out = build_runtime<C>(names, nkids, params, np, node, off, ok);
  return ok && node == nnodes;
}

template<typename C, typename IN, typename OUT>
int runtime_evalpdf(int nnodes, const char* const* names, const int* nkids, const float* params, const int* np,
                    size_t n, const IN* ix, const IN* iy, const IN* iz, const IN* ox, const IN* oy, const IN* oz,
                    uint32_t component, uint32_t unit, int mode, OUT* r, OUT* g, OUT* b, OUT* pdf, int nthreads)
{
  using Value = bbm::Value_t<C>;
  using Vec3d = bbm::Vec3d_t<C>;
  bool bad = false;
  // one tree per thread: the tabulated samplers cache their CDFs in mutable members
#ifdef _OPENMP
  #pragma omp parallel num_threads(nthreads > 0 ? nthreads : 1)
#endif
  {
    bbm::bsdf_ptr<C> m;
    const bool ok = build_tree<C>(nnodes, names, nkids, params, np, m);
    if(!ok) bad = true;
#ifdef _OPENMP
    #pragma omp for schedule(static)
#endif
    for(size_t i = 0; i < n; ++i)
    {
      if(!ok) continue;
      const Vec3d in(Value(ix[i]), Value(iy[i]), Value(iz[i]));
      const Vec3d out(Value(ox[i]), Value(oy[i]), Value(oz[i]));
      if(mode & 1)
      {
        auto e = m.eval(in, out, bbm::bsdf_flag(component), bbm::unit_t(unit));
        r[i] = OUT(e[0]); g[i] = OUT(e[1]); b[i] = OUT(e[2]);
      }
      if(mode & 2) pdf[i] = OUT(m.pdf(in, out, bbm::bsdf_flag(component), bbm::unit_t(unit)));
    }
  }
  return bad ? -1 : 0;
}

template<typename C, typename IN, typename OUT>
int runtime_sample(int nnodes, const char* const* names, const int* nkids, const float* params, const int* np,
                   size_t n, const IN* ox, const IN* oy, const IN* oz, const IN* xi0, const IN* xi1,
                   uint32_t component, uint32_t unit, OUT* dx, OUT* dy, OUT* dz, OUT* pdf, uint32_t* flag,
                   int nthreads)
{
  using Value = bbm::Value_t<C>;
  using Vec3d = bbm::Vec3d_t<C>;
  using Vec2d = bbm::Vec2d_t<C>;
  bool bad = false;
#ifdef _OPENMP
  #pragma omp parallel num_threads(nthreads > 0 ? nthreads : 1)
#endif
  {
    bbm::bsdf_ptr<C> m;
    const bool ok = build_tree<C>(nnodes, names, nkids, params, np, m);
    if(!ok) bad = true;
#ifdef _OPENMP
    #pragma omp for schedule(static)
#endif
    for(size_t i = 0; i < n; ++i)
    {
      if(!ok) continue;
      // (aggregatebsdf::sample returns a default-constructed, indeterminate sample where its weights sum to <= eps,
      // aggregatebsdf.h:113-116; the tests do not compare those lanes)
      const Vec3d out(Value(ox[i]), Value(oy[i]), Value(oz[i]));
      auto s = m.sample(out, Vec2d(Value(xi0[i]), Value(xi1[i])), bbm::bsdf_flag(component), bbm::unit_t(unit));
      dx[i] = OUT(s.direction[0]); dy[i] = OUT(s.direction[1]); dz[i] = OUT(s.direction[2]);
      pdf[i] = OUT(s.pdf);
      flag[i] = uint32_t(s.flag);
    }
  }
  return bad ? -1 : 0;
}

template<typename C, typename IN, typename OUT>
int runtime_reflectance(int nnodes, const char* const* names, const int* nkids, const float* params, const int* np,
                        size_t n, const IN* ox, const IN* oy, const IN* oz, uint32_t component, uint32_t unit,
                        OUT* r, OUT* g, OUT* b)
{
  using Value = bbm::Value_t<C>;
  using Vec3d = bbm::Vec3d_t<C>;
  bbm::bsdf_ptr<C> m;
  if(!build_tree<C>(nnodes, names, nkids, params, np, m)) return -1;
  for(size_t i = 0; i < n; ++i)
  {
    const Vec3d out(Value(ox[i]), Value(oy[i]), Value(oz[i]));
    auto e = m.reflectance(out, bbm::bsdf_flag(component), bbm::unit_t(unit));
    r[i] = OUT(e[0]); g[i] = OUT(e[1]); b[i] = OUT(e[2]);
  }
  return 0;
}

} // namespace

extern "C" {

int bbmref_runtime_eval_pdf(int nnodes, const char* const* names, const int* nkids, const float* params, const int* np,
                            size_t n, const float* ix, const float* iy, const float* iz,
                            const float* ox, const float* oy, const float* oz, uint32_t component, uint32_t unit,
                            int mode, float* r, float* g, float* b, float* pdf, int nthreads)
{
  return runtime_evalpdf<bbm::floatRGB>(nnodes, names, nkids, params, np, n, ix, iy, iz, ox, oy, oz, component, unit,
                                        mode, r, g, b, pdf, nthreads);
}

int bbmref_runtime_eval_pdf_dd(int nnodes, const char* const* names, const int* nkids, const float* params,
                               const int* np, size_t n, const double* ix, const double* iy, const double* iz,
                               const double* ox, const double* oy, const double* oz, uint32_t component,
                               uint32_t unit, int mode, double* r, double* g, double* b, double* pdf, int nthreads)
{
  return runtime_evalpdf<bbm::doubleRGB>(nnodes, names, nkids, params, np, n, ix, iy, iz, ox, oy, oz, component, unit,
                                         mode, r, g, b, pdf, nthreads);
}

int bbmref_runtime_sample(int nnodes, const char* const* names, const int* nkids, const float* params, const int* np,
                          size_t n, const float* ox, const float* oy, const float* oz, const float* xi0,
                          const float* xi1, uint32_t component, uint32_t unit, float* dx, float* dy, float* dz,
                          float* pdf, uint32_t* flag, int nthreads)
{
  return runtime_sample<bbm::floatRGB>(nnodes, names, nkids, params, np, n, ox, oy, oz, xi0, xi1, component, unit,
                                       dx, dy, dz, pdf, flag, nthreads);
}

int bbmref_runtime_sample_dd(int nnodes, const char* const* names, const int* nkids, const float* params,
                             const int* np, size_t n, const double* ox, const double* oy, const double* oz,
                             const double* xi0, const double* xi1, uint32_t component, uint32_t unit, double* dx,
                             double* dy, double* dz, double* pdf, uint32_t* flag, int nthreads)
{
  return runtime_sample<bbm::doubleRGB>(nnodes, names, nkids, params, np, n, ox, oy, oz, xi0, xi1, component, unit,
                                        dx, dy, dz, pdf, flag, nthreads);
}

int bbmref_runtime_reflectance(int nnodes, const char* const* names, const int* nkids, const float* params,
                               const int* np, size_t n, const float* ox, const float* oy, const float* oz,
                               uint32_t component, uint32_t unit, float* r, float* g, float* b)
{
  return runtime_reflectance<bbm::floatRGB>(nnodes, names, nkids, params, np, n, ox, oy, oz, component, unit, r, g, b);
}

int bbmref_runtime_reflectance_dd(int nnodes, const char* const* names, const int* nkids, const float* params,
                                  const int* np, size_t n, const double* ox, const double* oy, const double* oz,
                                  uint32_t component, uint32_t unit, double* r, double* g, double* b)
{
  return runtime_reflectance<bbm::doubleRGB>(nnodes, names, nkids, params, np, n, ox, oy, oz, component, unit, r, g, b);
}

} // extern "C"
