/* oracle/ref_cli.cpp -- TEST INFRASTRUCTURE ONLY: bin/checkBsdf.cpp's reflectance and pdf tests run on the reference's
 * own bsdf_ptr (built from a parsed model tree as in ref_runtime.cpp: bsdf_import needs the CMake-generated
 * bbm_bsdfmodels.h, so the program itself is not buildable here) with the program's random numbers -- one std::mt19937
 * seeded with `seed`, rndVec2d() = Vec2d(U(rnd), U(rnd)) compiled by this g++ like the reference binary -- and its
 * printed text captured.  The loops restate checkBsdf.cpp:51-97 (testReflectance) and :190-245 (testPdf) line for
 * line (option parsing aside); tests/test_gpu_cpp_cli.py diffs the HIP backbone's CLI (rng=mt19937) against them. */
#include <random>
#include <sstream>

namespace {

struct cli_rng
{
  std::mt19937 rnd;
  explicit cli_rng(uint64_t seed) : rnd(uint32_t(seed)) {}
  bbm::Vec2d_t<bbm::floatRGB> rndVec2d(void)          // checkBsdf.cpp:21-26
  {
    using Vec2d = bbm::Vec2d_t<bbm::floatRGB>;
    std::uniform_real_distribution<float> U(0,1);
    return Vec2d(U(rnd), U(rnd));
  }
};

template<typename C>
bbm::BsdfSample_t<C> cli_sample_dir(const bbm::Vec2d_t<C>& xi, bool sphere)      // checkBsdf.cpp:28-45
{
  using Constants = bbm::constants<bbm::Value_t<C>>;
  bbm::Vec2d_t<C> coord;
  bbm::spherical::theta(coord) = sphere ? bbm::safe_acos(1.0 - 2.0 * xi[0]) : bbm::safe_acos(xi[0]);
  bbm::spherical::phi(coord) = xi[1] * Constants::Pi(2);
  return bbm::BsdfSample_t<C>{ bbm::spherical::convert(coord), sphere ? 1.0 / Constants::Pi(4) : 1.0 / Constants::Pi(2),
                               bbm::bsdf_flag::None };
}

}  // namespace

extern "C" {

/* test 0 = reflectance (a = theta count, flag0 = importanceSampling), 1 = pdf (a = maxError, flag0 = checkBelowHorizon,
 * flag1 = sampleSphere); returns the text length, or < 0 if the tree cannot be built */
int bbmref_cli_test(int nnodes, const char* const* names, const int* nkids, const float* params, const int* np, int test,
                    size_t samples, size_t a, int flag0, int flag1, uint64_t seed, char* out, int cap)
{
  using C = bbm::floatRGB;
  using Value = bbm::Value_t<C>;
  using Vec2d = bbm::Vec2d_t<C>;
  using Vec3d = bbm::Vec3d_t<C>;
  using Spectrum = bbm::Spectrum_t<C>;
  using Constants = bbm::constants<Value>;
  bbm::bsdf_ptr<C> bsdf;
  if(!build_tree<C>(nnodes, names, nkids, params, np, bsdf)) return -1;
  cli_rng r(seed);
  std::ostringstream os;
  if(test == 0)
  {
    const size_t numtheta = a;
    const bool importance = flag0 != 0;
    os << "Reflectance test with " << numtheta << " directions and " << samples << " samples." << std::endl;
    Vec2d out_sp(0);
    for(size_t theta_idx = 0; theta_idx < numtheta; ++theta_idx)
    {
      bbm::spherical::theta(out_sp) = theta_idx * Constants::Pi(0.5) / numtheta;
      Vec3d dir_out = bbm::spherical::convert(out_sp);
      Spectrum estimate(0);
      for(size_t s = 0; s < samples; ++s)
      {
        auto sample = (importance) ? bsdf.sample(dir_out, r.rndVec2d()) : cli_sample_dir<C>(r.rndVec2d(), true);
        if(bbm::any(sample.pdf > Constants::Epsilon()))
          estimate += bsdf.eval(sample.direction, dir_out) * bbm::vec::z(sample.direction) / sample.pdf;
      }
      estimate /= samples;
      os << " out = " << dir_out << " => Estimate: " << estimate << " vs. " << bsdf->reflectance(dir_out) << std::endl;
    }
  }
  else
  {
    const size_t maxError = a;
    const bool checkBelowHorizon = flag0 != 0, samplesphere = flag1 != 0;
    os << "Tesing PDF properties test with " << samples << " samples." << std::endl;
    size_t count_negative_r = 0, count_negative_i = 0, count_zr = 0, count_zi = 0;
    Value mismatch_r = 0, mismatch_i = 0;
    for(size_t s = 0; s < samples && count_negative_r < maxError && count_negative_i < maxError && count_zr < maxError && count_zi < maxError; ++s)
    {
      auto sample = cli_sample_dir<C>(r.rndVec2d(), samplesphere);
      auto sample_r = bsdf.sample(sample.direction, r.rndVec2d(), bbm::bsdf_flag::All, bbm::unit_t::Radiance);
      auto sample_i = bsdf.sample(sample.direction, r.rndVec2d(), bbm::bsdf_flag::All, bbm::unit_t::Importance);
      if(checkBelowHorizon && bbm::any(bbm::vec::z(sample_r.direction) < 0)) { count_zr++; os << " Sampled direction " << sample_r.direction << " below horizon for " << sample.direction << std::endl; }
      if(checkBelowHorizon && bbm::any(bbm::vec::z(sample_i.direction) < 0)) { count_zi++; os << " Sampled direction " << sample_i.direction << " below horizon for " << sample.direction << std::endl; }
      auto pr = bsdf.pdf(sample_r.direction, sample.direction, bbm::bsdf_flag::All, bbm::unit_t::Radiance);
      auto pi = bsdf.pdf(sample_i.direction, sample.direction, bbm::bsdf_flag::All, bbm::unit_t::Importance);
      if(bbm::any(pr < 0)) { count_negative_r++; os << " Negative PDF (" << pr << ") for (" << sample_r.direction << ", " << sample.direction << ")" << std::endl; }
      if(bbm::any(pi < 0)) { count_negative_i++; os << " Negative PDF (" << pi << ") for (" << sample_i.direction << ", " << sample.direction << ")" << std::endl; }
      mismatch_r += bbm::abs(sample_r.pdf - pr);
      mismatch_i += bbm::abs(sample_i.pdf - pi);
    }
    mismatch_r /= samples;
    mismatch_i /= samples;
    os << "PDF has " << count_negative_r << "/" << count_negative_i << " negative PDF values, ";
    if(checkBelowHorizon) os << count_zr << "/" << count_zi << " sampled directions below the horizon, ";
    os << "and " << mismatch_r << "/" << mismatch_i << " average difference between the PDF from the sample method and the corresponding PDF from the pdf-method." << std::endl;
  }
  const std::string t = os.str();
  if(out && cap > 0) { std::strncpy(out, t.c_str(), size_t(cap - 1)); out[cap - 1] = 0; }
  return int(t.size());
}

}  // extern "C"
