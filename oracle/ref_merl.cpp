/* oracle/ref_merl.cpp -- TEST INFRASTRUCTURE ONLY: Merl for the reference shim.
 *
 * staticmodel/merl.h:224-225 defines merl = ndf_sampler<merl_data<CONF, "Merl">, 90, 1>, whose inner
 * ndf::sampler needs the default NAME that g++ 11 cannot deduce (include/ndf/sampler.h:34; see
 * ref_he.hpp).  The header's concept check of that alias (merl.h:227) is switched off, and the model is
 * instantiated as he_sampled<merl_data<floatRGB, "Merl">, "Merl">: the reference's own merl_data (file
 * import, merl_linearizer lookup, reflectance placeholder) under the reference's own ndf::sampler.
 * Models are constructed from a MERL .binary file name, so these entry points take one instead of a
 * parameter vector.
 */
#pragma push_macro("BBM_CHECK_CONCEPT")
#undef BBM_CHECK_CONCEPT
#define BBM_CHECK_CONCEPT(...) static_assert(true, "")
#include "staticmodel/merl.h"
#pragma pop_macro("BBM_CHECK_CONCEPT")

namespace {
using merl_ref = bbmref::he_sampled<bbm::merl_data<bbm::floatRGB, "Merl">, "Merl">;
}

extern "C" {

// eval (mode bit 1) and pdf (bit 2) of the Merl model read from `filename`; returns -1 if the reference
// rejects the file (its exception text is dropped: the GPU side's errors are tested on their own)
int bbmref_merl_eval_pdf(const char* filename, size_t n,
                         const float* ix, const float* iy, const float* iz,
                         const float* ox, const float* oy, const float* oz,
                         uint32_t component, uint32_t unit, int mode,
                         float* r, float* g, float* b, float* pdf, int nthreads)
{
  try
  {
    const merl_ref m0{std::string(filename)};
    const auto comp = bbm::bsdf_flag(component);
    const auto u = bbm::unit_t(unit);
#ifdef _OPENMP
    #pragma omp parallel num_threads(nthreads > 0 ? nthreads : 1)
#endif
    {
    const merl_ref m = m0;      // one copy per thread: the sampler cache is mutable
#ifdef _OPENMP
    #pragma omp for schedule(static)
#endif
    for(size_t i = 0; i < n; ++i)
    {
      merl_ref::Vec3d in(ix[i], iy[i], iz[i]), out(ox[i], oy[i], oz[i]);
      if(mode & 1) { auto e = m.eval(in, out, comp, u); r[i] = e[0]; g[i] = e[1]; b[i] = e[2]; }
      if(mode & 2) pdf[i] = m.pdf(in, out, comp, u);
    }
    }
  }
  catch(const std::exception&) { return -1; }
  return 0;
}

int bbmref_merl_sample(const char* filename, size_t n,
                       const float* ox, const float* oy, const float* oz, const float* xi0, const float* xi1,
                       uint32_t component, uint32_t unit,
                       float* dx, float* dy, float* dz, float* pdf, uint32_t* flag)
{
  try
  {
    const merl_ref m{std::string(filename)};
    for(size_t i = 0; i < n; ++i)
    {
      merl_ref::Vec3d out(ox[i], oy[i], oz[i]);
      merl_ref::Vec2d xi(xi0[i], xi1[i]);
      auto s = m.sample(out, xi, bbm::bsdf_flag(component), bbm::unit_t(unit));
      dx[i] = s.direction[0]; dy[i] = s.direction[1]; dz[i] = s.direction[2];
      pdf[i] = s.pdf;
      flag[i] = uint32_t(s.flag);
    }
  }
  catch(const std::exception&) { return -1; }
  return 0;
}

int bbmref_merl_to_string(const char* filename, char* buf, int cap)
{
  try
  {
    const std::string s = bbm::toString(merl_ref{std::string(filename)});
    if(buf && cap > 0) { std::strncpy(buf, s.c_str(), size_t(cap - 1)); buf[cap - 1] = 0; }
    return int(s.size());
  }
  catch(const std::exception&) { return -1; }
}

} // extern "C"
