/* oracle/ref_cli.cpp -- TEST INFRASTRUCTURE ONLY: bin/checkBsdf.cpp's reflectance and pdf tests run on the reference's
 * own bsdf_ptr (built from a parsed model tree as in ref_runtime.cpp: bsdf_import needs the CMake-generated
 * bbm_bsdfmodels.h, so the program itself is not buildable here) with the program's random numbers -- one std::mt19937
 * seeded with `seed`, rndVec2d() = Vec2d(U(rnd), U(rnd)) compiled by this g++ like the reference binary -- and its
 * printed text captured.  The loops restate checkBsdf.cpp:51-97 (testReflectance), :102-140 (testReciprocity), :145-185
 * (testAdjoint), :190-245 (testPdf), :250-290 (testPdfInt) and :300-418 (testSample) line for line (option parsing
 * aside); tests/test_gpu_cpp_cli.py diffs the HIP backbone's CLI (rng=mt19937) against them. */
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

/* test 0 = reflectance (o = samples, theta, importanceSampling), 1 = pdf (samples, maxError, checkBelowHorizon,
 * sampleSphere), 2 = reciprocity (samples), 3 = adjoint (samples), 4 = pdfInt (samples, trials, sampleSphere),
 * 5 = sample (pdfSamples, samples, theta, phi, trials, sampleSphere, includeZeroPdfSamples); returns the text length, or
 * < 0 if the tree cannot be built */
int bbmref_cli_test(int nnodes, const char* const* names, const int* nkids, const float* params, const int* np, int test,
                    const uint64_t* o, uint64_t seed, char* out, int cap)
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
  using namespace bbm;          // as the program (checkBsdf.cpp:13): unqualified calls resolve as there
  using Vec3dPair = bbm::Vec3dPair_t<C>;
  if(test == 0)
  {
    const size_t samples = o[0], numtheta = o[1];
    const bool importance = o[2] != 0;
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
  else if(test == 1)
  {
    const size_t samples = o[0], maxError = o[1];
    const bool checkBelowHorizon = o[2] != 0, samplesphere = o[3] != 0;
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
  else if(test == 2 || test == 3)
  {
    const size_t samples = o[0];
    const bool adjoint = test == 3;
    os << (adjoint ? "Adjoint" : "Reciprocity") << " test with " << samples << " samples." << std::endl;
    Spectrum sum_r = 0, max_r = 0, sum_i = 0, max_i = 0;
    Vec3dPair maxpair_i = {0,0}, maxpair_r = {0,0};
    for(size_t s = 0; s < samples; ++s)
    {
      auto sample1 = cli_sample_dir<C>(r.rndVec2d(), true);
      auto sample2 = cli_sample_dir<C>(r.rndVec2d(), true);
      Vec3dPair dir = {sample1.direction, sample2.direction};
      if(adjoint)
      {
        Spectrum diff_a = bbm::abs( bsdf.eval(dir.in, dir.out, bsdf_flag::All, unit_t::Radiance) - bsdf.eval(dir.out, dir.in, bsdf_flag::All, unit_t::Importance) );
        sum_r += diff_a;
        if( bbm::any(bbm::hsum(diff_a) > bbm::hsum(max_r)) ) { maxpair_r = dir; max_r = diff_a; }
        continue;
      }
      Spectrum diff_r = bbm::abs( bsdf.eval(dir.in, dir.out, bsdf_flag::All, unit_t::Radiance) - bsdf.eval(dir.out, dir.in, bsdf_flag::All, unit_t::Radiance) );
      Spectrum diff_i = bbm::abs( bsdf.eval(dir.in, dir.out, bsdf_flag::All, unit_t::Importance) - bsdf.eval(dir.out, dir.in, bsdf_flag::All, unit_t::Importance) );
      sum_r += diff_r;
      sum_i += diff_i;
      if( bbm::any(bbm::hsum(diff_r) > bbm::hsum(max_r)) ) { maxpair_r = dir; max_r = diff_r; }
      if( bbm::any(bbm::hsum(diff_i) > bbm::hsum(max_i)) ) { maxpair_i = dir; max_i = diff_i; }
    }
    sum_r /= samples;
    if(adjoint) os << "Adjoint difference average = " << sum_r << ", max = " << max_r << " at " << maxpair_r << std::endl;
    else
    {
      sum_i /= samples;
      os << "Radiance   average = " << sum_r << ", max = " << max_r << " at " << maxpair_r << std::endl;
      os << "Importance average = " << sum_i << ", max = " << max_i << " at " << maxpair_i << std::endl;
    }
  }
  else if(test == 4)
  {
    const size_t samples = o[0], trials = o[1];
    const bool samplesphere = o[2] != 0;
    os << "Tesing PDF Integral with " << samples << " samples, for " << trials << " random directions sampled over the " << ((samplesphere) ? "sphere" : "hemisphere") << std::endl;
    for(size_t t=0; t < trials; ++t)
    {
      Value pdf_r = 0, pdf_i = 0;
      auto sample_t = cli_sample_dir<C>(r.rndVec2d(), samplesphere);
      for(size_t s=0; s < samples; ++s)
      {
        auto sample_s = cli_sample_dir<C>(r.rndVec2d(), true);
        if(bbm::any(sample_s.pdf > Constants::Epsilon()))
        {
          pdf_r += bsdf.pdf(sample_s.direction, sample_t.direction, bsdf_flag::All, unit_t::Radiance) / sample_s.pdf;
          pdf_i += bsdf.pdf(sample_s.direction, sample_t.direction, bsdf_flag::All, unit_t::Importance) / sample_s.pdf;
        }
      }
      pdf_r /= samples;
      pdf_i /= samples;
      os << " Integral = " << pdf_r << "/" << pdf_i << " (radiance/importance) for " << sample_t.direction << std::endl;
    }
  }
  else
  {
    const size_t pdfSamples = o[0], samples = o[1], theta = o[2], phi = o[3], trials = o[4];
    const bool samplesphere = o[5] != 0, includeZeroPdfSamples = o[6] != 0;
    os << "Testing if sample and pdf match: " << pdfSamples << " PDF samples per bin, and " << samples << " direction samples, with (" << phi << " x " << theta << ") bins over " << trials << " trials";
    if(includeZeroPdfSamples) os << ", including zero pdf samples";
    os << "." << std::endl;
    for(size_t tr=0; tr < trials; ++tr)
    {
      auto sample_t = cli_sample_dir<C>(r.rndVec2d(), samplesphere);
      std::vector<Value> pdf(theta * phi, 0);
      std::vector<Value> count(theta * phi, 0);
      Vec2d sph_coord;
      size_t idx=0;
      for(size_t t=0; t < theta; ++t)
        for(size_t p=0; p < phi; ++p, ++idx)
        {
          for(size_t s=0; s < pdfSamples; ++s)
          {
            auto rnd = r.rndVec2d();
            spherical::phi(sph_coord) = Constants::Pi(2) * (p + rnd[0]) / phi;
            spherical::theta(sph_coord) = Constants::Pi() * (t + rnd[1]) / theta;
            Vec3d dir = spherical::convert(sph_coord);
            Value w = Constants::Pi2(2) * bbm::abs(spherical::sinTheta(sph_coord)) / (phi * theta);
            pdf[idx] += bsdf.pdf(dir, sample_t.direction ) * w;
          }
          pdf[idx] /= pdfSamples;
        }
      for(size_t s=0; s < samples; ++s)
      {
        auto sample = bsdf.sample(sample_t.direction, r.rndVec2d());
        if(includeZeroPdfSamples || bbm::any(sample.pdf > Constants::Epsilon()))
        {
          sph_coord = spherical::convert(sample.direction);
          size_t t = bbm::cast<size_t>(bbm::min( spherical::theta(sph_coord) / Constants::Pi() * theta, theta-1));
          size_t p = bbm::cast<size_t>(bbm::min( spherical::phi(sph_coord) / Constants::Pi(2) * phi, phi-1));
          count[t * phi + p]++;
        }
      }
      Value chi2 = 0, df = -1; idx=0;
      for(size_t t=0; t < theta; ++t)
        for(size_t p=0; p < phi; ++p, idx++)
        {
          Value m = pdf[idx] * samples;
          if(bbm::any(m > Constants::Epsilon() && count[idx] > 5))
          {
            chi2 += pow( count[idx] - m, 2) / m;
            df++;
          }
        }
      os << " Chi2 for " << sample_t.direction << " = " << chi2 << " (with " << df << " degrees of freedom)." << std::endl;
      if(bbm::any(df > 1))
      {
        Value P = bbm::gamma_q((df-1) / 2, chi2 / 2);
        os << "  P = " << P << " (reject if lower than confidence)." << std::endl;
      }
      else os << " No degrees of freedom; need at least 1 to compute P." << std::endl;
    }
  }
  const std::string t = os.str();
  if(out && cap > 0) { std::strncpy(out, t.c_str(), size_t(cap - 1)); out[cap - 1] = 0; }
  return int(t.size());
}

}  // extern "C"
