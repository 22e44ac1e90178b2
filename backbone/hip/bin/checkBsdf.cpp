/* backbone/hip/bin/checkBsdf.cpp -- the reference's checkBsdf command line (bin/checkBsdf.cpp:420-479) on the HIP
 * backbone: the same `key=value` options (include/util/option.h), the same tests and printed lines, every statistic
 * computed on the GPU by bbm_hip/check.h.
 *
 *   checkBsdf bsdfmodel="CookTorrance(roughness=0.3)" test=reflectance samples=1000000 theta=4
 *
 * Extra option: seed=<n> (the counter-based draws' seed, default 5489).  Differences from the reference, by design:
 * counter-based random numbers instead of one std::mt19937 (statistically equivalent), double accumulators, and the
 * pdf test counts every failure instead of stopping at maxError and printing each.
 * Built by tests/cpp/Makefile against the reference's headers (BBM_BACKBONE=hip) and libbbm_hip.so.
 */
#include <iostream>
#include <set>
#include <string>
#include <vector>

#include "bbm/bbm_core.h"
#include "bbm/vec3dpair.h"
#include "util/option.h"
#include "util/vector_util.h"
#include "bbm_hip/check.h"

using namespace bbm;
BBM_IMPORT_CONFIG( floatRGB );

static Vec3d to_vec(const hip::rgb_t& v) { return Vec3d(v[0], v[1], v[2]); }
static Spectrum spec(const hip::rgb_t& v) { return Spectrum(v[0], v[1], v[2]); }

static bool valid(const option_parser& opt, const std::set<std::string>& keys)
{
  std::set<std::string> k = keys;
  k.insert("seed");
  auto invalid = opt.validate(k);
  if(!invalid.empty())
  {
    std::cout << "ERROR: invalid keywords: " << invalid << "." << std::endl;
    return false;
  }
  return true;
}

static void testReflectance(const hip::model_desc& m, const option_parser& opt, uint64_t seed)
{
  size_t samples = opt.get<size_t>("samples", 100000);
  size_t numtheta = opt.get<size_t>("theta", 1);
  bool importance = opt.get<bool>("importanceSampling", false);
  if(!valid(opt, {"bsdfmodel", "test", "samples", "theta", "importanceSampling"})) return;
  std::cout << "Reflectance test with " << numtheta << " directions and " << samples << " samples." << std::endl;
  const auto r = hip::check_reflectance(m, samples, numtheta, importance, seed);
  for(size_t t = 0; t < numtheta; ++t)
    std::cout << " out = " << to_vec(r.out[t]) << " => Estimate: " << spec(r.estimate[t]) << " vs. " << spec(r.reflectance[t]) << std::endl;
}

static void testReciprocity(const hip::model_desc& m, const option_parser& opt, uint64_t seed)
{
  size_t samples = opt.get<size_t>("samples", 1000000);
  if(!valid(opt, {"bsdfmodel", "test", "samples"})) return;
  std::cout << "Reciprocity test with " << samples << " samples." << std::endl;
  const auto r = hip::check_reciprocity(m, samples, seed);
  const Vec3dPair pr{to_vec(r[0].in), to_vec(r[0].out)}, pi{to_vec(r[1].in), to_vec(r[1].out)};
  std::cout << "Radiance   average = " << spec(r[0].average) << ", max = " << spec(r[0].max) << " at " << pr << std::endl;
  std::cout << "Importance average = " << spec(r[1].average) << ", max = " << spec(r[1].max) << " at " << pi << std::endl;
}

static void testAdjoint(const hip::model_desc& m, const option_parser& opt, uint64_t seed)
{
  size_t samples = opt.get<size_t>("samples", 100000);
  if(!valid(opt, {"bsdfmodel", "test", "samples"})) return;
  std::cout << "Adjoint test with " << samples << " samples." << std::endl;
  const auto r = hip::check_adjoint(m, samples, seed);
  const Vec3dPair pa{to_vec(r.in), to_vec(r.out)};
  std::cout << "Adjoint difference average = " << spec(r.average) << ", max = " << spec(r.max) << " at " << pa << std::endl;
}

static void testPdf(const hip::model_desc& m, const option_parser& opt, uint64_t seed)
{
  size_t samples = opt.get<size_t>("samples", 100000);
  (void)opt.get<size_t>("maxError", 10);                    // accepted: every failure is counted here
  bool checkBelowHorizon = opt.get<bool>("checkBelowHorizon", false);
  bool samplesphere = opt.get<bool>("sampleSphere", false);
  if(!valid(opt, {"bsdfmodel", "test", "samples", "maxError", "checkBelowHorizon", "sampleSphere"})) return;
  std::cout << "Tesing PDF properties test with " << samples << " samples." << std::endl;
  const auto r = hip::check_pdf(m, samples, samplesphere, seed);
  std::cout << "PDF has " << r.negative[0] << "/" << r.negative[1] << " negative PDF values, ";
  if(checkBelowHorizon) std::cout << r.below_horizon[0] << "/" << r.below_horizon[1] << " sampled directions below the horizon, ";
  std::cout << "and " << Value(r.mismatch[0]) << "/" << Value(r.mismatch[1])
            << " average difference between the PDF from the sample method and the corresponding PDF from the pdf-method." << std::endl;
}

static void testPdfInt(const hip::model_desc& m, const option_parser& opt, uint64_t seed)
{
  size_t samples = opt.get<size_t>("samples", 1000000);
  size_t trials = opt.get<size_t>("trials", 10);
  bool samplesphere = opt.get<bool>("sampleSphere", false);
  if(!valid(opt, {"bsdfmodel", "test", "samples", "trials", "sampleSphere"})) return;
  std::cout << "Tesing PDF Integral with " << samples << " samples, for " << trials << " random directions sampled over the "
            << ((samplesphere) ? "sphere" : "hemisphere") << std::endl;
  const auto r = hip::check_pdf_int(m, samples, trials, samplesphere, seed);
  for(size_t t = 0; t < trials; ++t)
    std::cout << " Integral = " << Value(r.integral[t][0]) << "/" << Value(r.integral[t][1]) << " (radiance/importance) for "
              << to_vec(r.direction[t]) << std::endl;
}

static void testSample(const hip::model_desc& m, const option_parser& opt, uint64_t seed)
{
  size_t pdfSamples = opt.get<size_t>("pdfSamples", 4096);
  size_t samples = opt.get<size_t>("samples", 100000);
  size_t theta = opt.get<size_t>("theta", 10);
  size_t phi = opt.get<size_t>("phi", 20);
  size_t trials = opt.get<size_t>("trials", 10);
  bool samplesphere = opt.get<bool>("sampleSphere", false);
  bool includeZeroPdfSamples = opt.get<bool>("includeZeroPdfSamples", false);
  if(!valid(opt, {"bsdfmodel", "test", "pdfSamples", "samples", "theta", "phi", "trials", "sampleSphere", "includeZeroPdfSamples"})) return;
  std::cout << "Testing if sample and pdf match: " << pdfSamples << " PDF samples per bin, and " << samples
            << " direction samples, with (" << phi << " x " << theta << ") bins over " << trials << " trials";
  if(includeZeroPdfSamples) std::cout << ", including zero pdf samples";
  std::cout << "." << std::endl;
  const auto r = hip::check_sample(m, pdfSamples, samples, theta, phi, trials, samplesphere, includeZeroPdfSamples, seed);
  for(const auto& t : r)
  {
    std::cout << " Chi2 for " << to_vec(t.direction) << " = " << Value(t.chi2) << " (with " << Value(t.df) << " degrees of freedom)." << std::endl;
    if(t.df > 1) std::cout << "  P = " << Value(t.P) << " (reject if lower than confidence)." << std::endl;
    else std::cout << " No degrees of freedom; need at least 1 to compute P." << std::endl;
  }
}

int main(int argc, char** argv)
{
  if(argc == 1)
  {
    std::cout << "Usage: " << argv[0] << " [bsdfmodel=<bsdf string>] [test=<test name> [test options] [seed=<n>]" << std::endl;
    std::cout << "  + test=reflectance [samples=100000] [theta=1] [importanceSampling]: compare the approximated reflectance method with a MC integration of the BSDF." << std::endl;
    std::cout << "  + test=reciprocity [samples=100000]: checks if the BSDF is symmetric for 'samples' random dirctions." << std::endl;
    std::cout << "  + test=adjoint [samples=100000]: checks if the adjoint BSDF is equal to the BSDF with in/out swapped." << std::endl;
    std::cout << "  + test=pdf [samples=100000] [maxError=10] [checkBelowHorizon] [sampleSphere]: checks if the PDF >= 0, and the PDF returned by the sampling method matches the pdf from the pdf-method." << std::endl;
    std::cout << "  + test=pdfInt [samples=100000] [trials=10] [sampleSphere]: checks the integral (MC with 'samples' samples) of the PDF for 'trials' different directions." << std::endl;
    std::cout << "  + test=sample [pdfSamples=4069] [samples=100000] [theta=10] [phi=20] [trials=10] [sampleSphere] [includeZeroPdfSamples]: perform Chi2 test on the sample vs the pdf method." << std::endl;
    return -1;
  }
  try
  {
    option_parser opt(argc, argv);
    auto bsdfmodel = opt.get<std::string>("bsdfmodel");
    auto testname = opt.get<std::string>("test");
    const uint64_t seed = opt.get<size_t>("seed", size_t(hip::check_default_seed));
    if(testname == "")
    {
      std::cout << "ERROR: no test specified." << std::endl;
      return -1;
    }
    // the model string through the library's parser (the runtime fromString / bsdf_import, bsdf_string_convert.h:52-85)
    const hip::model_desc m = hip::from_string(bsdfmodel);
    if(testname == "reflectance") testReflectance(m, opt, seed);
    else if(testname == "reciprocity") testReciprocity(m, opt, seed);
    else if(testname == "adjoint") testAdjoint(m, opt, seed);
    else if(testname == "pdf") testPdf(m, opt, seed);
    else if(testname == "pdfInt") testPdfInt(m, opt, seed);
    else if(testname == "sample") testSample(m, opt, seed);
    else std::cout << "Unrecognized test: '" << testname << "'" << std::endl;
  }
  catch(const std::exception& e)
  {
    std::cout << "ERROR: " << e.what() << std::endl;
    return 1;
  }
  return 0;
}
