/* backbone/hip/bin/checkBsdf.cpp -- the reference's checkBsdf command line (bin/checkBsdf.cpp:420-479) on the HIP
 * backbone: the same `key=value` options (include/util/option.h), the same tests and printed lines, every BSDF
 * evaluation on the GPU.
 *
 *   checkBsdf bsdfmodel="CookTorrance(roughness=0.3)" test=reflectance samples=1000000 theta=4
 *
 * Extra options:
 *   seed=<n>      the draws' seed (default 5489, the default seed of the reference's std::mt19937 `rnd`, :18)
 *   rng=counter   (default) the library's counter-based draws, one stream per (test, slot, draw): the statistics are
 *                 batched reductions on the GPU (bbm_hip/check.h, double accumulators)
 *   rng=mt19937   the reference's own draw sequence -- one std::mt19937 seeded with `seed` and
 *                 uniform_real_distribution<float>(0, 1) per rndVec2d() (:21-26), consumed in the reference binary's
 *                 order -- with the per-sample BSDF calls batched on the GPU and every accumulation, check and printed
 *                 line on the host in the reference's loop order and float precision: every test prints what the
 *                 reference prints for the same seed wherever the GPU's per-sample values are the reference's floats
 *                 (tests/test_gpu_cpp_cli.py diffs the two; oracle/ref_cli.cpp runs the reference).
 * test=pdf runs the reference's loop in both modes (:219-243): it stops once `maxError` failures of one kind are
 * seen and prints each negative pdf and each sampled direction below the horizon as the reference does.
 * Built by tests/cpp/Makefile against the reference's headers (BBM_BACKBONE=hip) and libbbm_hip.so.
 */
#include <iostream>
#include <random>
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
  k.insert("rng");
  auto invalid = opt.validate(k);
  if(!invalid.empty())
  {
    std::cout << "ERROR: invalid keywords: " << invalid << "." << std::endl;
    return false;
  }
  return true;
}

// ------------------------------------------------------------------------------------------------ draws

/* rndVec2d() (checkBsdf.cpp:21-26).  mt19937: the program's single std::mt19937 (:18) and a
 * uniform_real_distribution<float>(0, 1) per call, as the reference binary consumes them -- GCC, which builds it,
 * evaluates the arguments of Vec2d(U(rnd), U(rnd)) right to left, so xi[1] is the first draw and xi[0] the second
 * (checked against the reference compiled here: oracle/ref_cli.cpp).  counter: draw `draw` of sample `s` of the test's
 * counter streams (bbm_hip_check_draws), what the GPU statistics draw. */
struct draw_source
{
  bool mt;
  uint64_t seed;
  int test;
  std::mt19937 rnd;
  draw_source(bool mt_, uint64_t seed_, int test_) : mt(mt_), seed(seed_), test(test_), rnd(uint32_t(seed_)) {}

  // k samples from `offset` on, `ndraws` rndVec2d() per sample in the loop's call order: xi[d] = (x0[d][j], x1[d][j])
  void fill(size_t offset, size_t k, int ndraws, std::vector<float>* x0, std::vector<float>* x1)
  {
    for(int d = 0; d < ndraws; ++d) { x0[d].resize(k); x1[d].resize(k); }
    if(mt)
    {
      std::uniform_real_distribution<float> U(0, 1);
      for(size_t j = 0; j < k; ++j)
        for(int d = 0; d < ndraws; ++d)
        {
          const float second = U(rnd);        // Vec2d(U(rnd), U(rnd)): the right argument first (GCC)
          const float first = U(rnd);
          x0[d][j] = first;
          x1[d][j] = second;
        }
      return;
    }
    hip::device_vector<float> a(k), b(k);
    for(int d = 0; d < ndraws; ++d)
    {
      hip::check(bbm_hip_check_draws(test, seed, 0, d, offset, k, a.data(), b.data(), nullptr));
      hip::hip_check(hipMemcpy(x0[d].data(), a.data(), k * 4, hipMemcpyDeviceToHost), "hipMemcpy");
      hip::hip_check(hipMemcpy(x1[d].data(), b.data(), k * 4, hipMemcpyDeviceToHost), "hipMemcpy");
    }
  }
};

// sampleSphere / sampleHemisphere (checkBsdf.cpp:28-45), on the host as the reference computes them
static BsdfSample uniformDirection(const Vec2d& xi, bool sphere)
{
  Vec2d coord;
  spherical::theta(coord) = sphere ? bbm::safe_acos(1.0 - 2.0 * xi[0]) : bbm::safe_acos(xi[0]);
  spherical::phi(coord) = xi[1] * Constants::Pi(2);
  return BsdfSample{ spherical::convert(coord), sphere ? 1.0 / Constants::Pi(4) : 1.0 / Constants::Pi(2), bsdf_flag::None };
}

// host <-> device SoA rows of k directions
struct dev3
{
  hip::device_vector<float> x, y, z;
  explicit dev3(size_t k) : x(k), y(k), z(k) {}
  hip::soa3 in(void) const { return hip::soa3{x.data(), y.data(), z.data()}; }
  hip::soa3_out out(void) { return hip::soa3_out{x.data(), y.data(), z.data()}; }
  void upload(const std::vector<Vec3d>& v)
  {
    std::vector<float> h[3];
    for(int c = 0; c < 3; ++c) { h[c].resize(v.size()); for(size_t j = 0; j < v.size(); ++j) h[c][j] = v[j][c]; }
    hip::hip_check(hipMemcpy(x.data(), h[0].data(), v.size() * 4, hipMemcpyHostToDevice), "hipMemcpy");
    hip::hip_check(hipMemcpy(y.data(), h[1].data(), v.size() * 4, hipMemcpyHostToDevice), "hipMemcpy");
    hip::hip_check(hipMemcpy(z.data(), h[2].data(), v.size() * 4, hipMemcpyHostToDevice), "hipMemcpy");
  }
  std::vector<Vec3d> download(size_t k) const
  {
    std::vector<float> h[3] = {std::vector<float>(k), std::vector<float>(k), std::vector<float>(k)};
    hip::hip_check(hipMemcpy(h[0].data(), x.data(), k * 4, hipMemcpyDeviceToHost), "hipMemcpy");
    hip::hip_check(hipMemcpy(h[1].data(), y.data(), k * 4, hipMemcpyDeviceToHost), "hipMemcpy");
    hip::hip_check(hipMemcpy(h[2].data(), z.data(), k * 4, hipMemcpyDeviceToHost), "hipMemcpy");
    std::vector<Vec3d> v(k);
    for(size_t j = 0; j < k; ++j) v[j] = Vec3d(h[0][j], h[1][j], h[2][j]);
    return v;
  }
};

static std::vector<float> download(const hip::device_vector<float>& d, size_t k)
{
  std::vector<float> h(k);
  hip::hip_check(hipMemcpy(h.data(), d.data(), k * 4, hipMemcpyDeviceToHost), "hipMemcpy");
  return h;
}

static std::vector<float> upload_of(hip::device_vector<float>& d, const std::vector<float>& h)
{
  hip::hip_check(hipMemcpy(d.data(), h.data(), h.size() * 4, hipMemcpyHostToDevice), "hipMemcpy");
  return h;
}

constexpr size_t kChunk = size_t(1) << 18;   // samples per batch of GPU calls in the reference-ordered loops

// ------------------------------------------------------------------------------------------------ tests

// checkBsdf.cpp:51-97 in the reference's order (rng=mt19937): per theta, per sample, sample (or sampleSphere) then eval,
// the estimate accumulated in float
static void reflectanceOrdered(const hip::model_desc& m, size_t samples, size_t numtheta, bool importance, draw_source& rng)
{
  Vec2d out_sp(0);
  std::vector<float> x0[1], x1[1];
  for(size_t theta_idx = 0; theta_idx < numtheta; ++theta_idx)
  {
    spherical::theta(out_sp) = theta_idx * Constants::Pi(0.5) / numtheta;
    Vec3d out = spherical::convert(out_sp);
    Spectrum estimate(0);
    for(size_t s0 = 0; s0 < samples; s0 += kChunk)
    {
      const size_t k = std::min(kChunk, samples - s0);
      rng.fill(s0, k, 1, x0, x1);
      std::vector<Vec3d> outs(k, out), dirs(k);
      std::vector<float> pdfs(k);
      dev3 dout(k), ddir(k), f(k);
      dout.upload(outs);
      if(importance)
      {
        hip::device_vector<float> a(k), b(k), p(k);
        hip::device_vector<uint32_t> fl(k);
        upload_of(a, x0[0]); upload_of(b, x1[0]);
        hip::sample(m, dout.in(), a.data(), b.data(), k, ddir.out(), p.data(), fl.data());
        dirs = ddir.download(k);
        pdfs = download(p, k);
      }
      else
      {
        for(size_t j = 0; j < k; ++j)
        {
          const BsdfSample u = uniformDirection(Vec2d(x0[0][j], x1[0][j]), true);
          dirs[j] = u.direction;
          pdfs[j] = u.pdf;
        }
        ddir.upload(dirs);
      }
      hip::eval(m, ddir.in(), dout.in(), k, f.out());
      const std::vector<Vec3d> fv = f.download(k);
      for(size_t j = 0; j < k; ++j)
        if(bbm::any(pdfs[j] > Constants::Epsilon()))
          estimate += Spectrum(fv[j][0], fv[j][1], fv[j][2]) * vec::z(dirs[j]) / pdfs[j];
    }
    estimate /= samples;
    dev3 o(1), r(1);
    o.upload({out});
    hip::reflectance(m, o.in(), 1, r.out());
    const Vec3d rv = r.download(1)[0];
    std::cout << " out = " << out << " => Estimate: " << estimate << " vs. " << Spectrum(rv[0], rv[1], rv[2]) << std::endl;
  }
}

// batched BSDF calls on host direction lists (one chunk), results back on the host
static std::vector<Spectrum> evalBatch(const hip::model_desc& m, const std::vector<Vec3d>& in, const std::vector<Vec3d>& out,
                                       unit_t unit)
{
  const size_t k = in.size();
  dev3 di(k), dout(k), f(k);
  di.upload(in);
  dout.upload(out);
  hip::eval(m, di.in(), dout.in(), k, f.out(), bsdf_flag::All, unit);
  const auto v = f.download(k);
  std::vector<Spectrum> r(k);
  for(size_t j = 0; j < k; ++j) r[j] = Spectrum(v[j][0], v[j][1], v[j][2]);
  return r;
}

static std::vector<float> pdfBatch(const hip::model_desc& m, const std::vector<Vec3d>& in, const std::vector<Vec3d>& out,
                                   unit_t unit)
{
  const size_t k = in.size();
  dev3 di(k), dout(k);
  di.upload(in);
  dout.upload(out);
  hip::device_vector<float> p(k);
  hip::pdf(m, di.in(), dout.in(), k, p.data(), bsdf_flag::All, unit);
  return download(p, k);
}

// checkBsdf.cpp:102-140 / :145-185 in the reference's order (rng=mt19937): two sampleSphere directions per sample, the
// evaluations batched, the float sums and the running maximum (first maximum kept on ties) on the host
static void symmetryOrdered(const hip::model_desc& m, size_t samples, bool adjoint, draw_source& rng)
{
  Spectrum sum_r = 0, max_r = 0, sum_i = 0, max_i = 0;
  Vec3dPair maxpair_r = {0, 0}, maxpair_i = {0, 0};
  std::vector<float> x0[2], x1[2];
  for(size_t s0 = 0; s0 < samples; s0 += kChunk)
  {
    const size_t k = std::min(kChunk, samples - s0);
    rng.fill(s0, k, 2, x0, x1);
    std::vector<Vec3d> a(k), b(k);
    for(size_t j = 0; j < k; ++j)
    {
      a[j] = uniformDirection(Vec2d(x0[0][j], x1[0][j]), true).direction;
      b[j] = uniformDirection(Vec2d(x0[1][j], x1[1][j]), true).direction;
    }
    const auto fr = evalBatch(m, a, b, unit_t::Radiance);
    const auto br = evalBatch(m, b, a, adjoint ? unit_t::Importance : unit_t::Radiance);
    std::vector<Spectrum> fi, bi;
    if(!adjoint) { fi = evalBatch(m, a, b, unit_t::Importance); bi = evalBatch(m, b, a, unit_t::Importance); }
    for(size_t j = 0; j < k; ++j)
    {
      const Vec3dPair dir = {a[j], b[j]};
      Spectrum diff_r = bbm::abs(fr[j] - br[j]);
      sum_r += diff_r;
      if(bbm::any(bbm::hsum(diff_r) > bbm::hsum(max_r))) { maxpair_r = dir; max_r = diff_r; }
      if(!adjoint)
      {
        Spectrum diff_i = bbm::abs(fi[j] - bi[j]);
        sum_i += diff_i;
        if(bbm::any(bbm::hsum(diff_i) > bbm::hsum(max_i))) { maxpair_i = dir; max_i = diff_i; }
      }
    }
  }
  sum_r /= samples;
  if(adjoint)
  {
    std::cout << "Adjoint difference average = " << sum_r << ", max = " << max_r << " at " << maxpair_r << std::endl;
    return;
  }
  sum_i /= samples;
  std::cout << "Radiance   average = " << sum_r << ", max = " << max_r << " at " << maxpair_r << std::endl;
  std::cout << "Importance average = " << sum_i << ", max = " << max_i << " at " << maxpair_i << std::endl;
}

// checkBsdf.cpp:250-290 in the reference's order (rng=mt19937): per trial its direction, then the sampleSphere draws
static void pdfIntOrdered(const hip::model_desc& m, size_t samples, size_t trials, bool samplesphere, draw_source& rng)
{
  std::vector<float> x0[1], x1[1];
  size_t off = 0;
  for(size_t t = 0; t < trials; ++t)
  {
    Value pdf_r = 0, pdf_i = 0;
    rng.fill(off++, 1, 1, x0, x1);
    const BsdfSample sample_t = uniformDirection(Vec2d(x0[0][0], x1[0][0]), samplesphere);
    for(size_t s0 = 0; s0 < samples; s0 += kChunk)
    {
      const size_t k = std::min(kChunk, samples - s0);
      rng.fill(off, k, 1, x0, x1);
      off += k;
      std::vector<Vec3d> dirs(k), ts(k, sample_t.direction);
      std::vector<Value> spdf(k);
      for(size_t j = 0; j < k; ++j)
      {
        const BsdfSample u = uniformDirection(Vec2d(x0[0][j], x1[0][j]), true);
        dirs[j] = u.direction;
        spdf[j] = u.pdf;
      }
      const auto pr = pdfBatch(m, dirs, ts, unit_t::Radiance), pi = pdfBatch(m, dirs, ts, unit_t::Importance);
      for(size_t j = 0; j < k; ++j)
        if(bbm::any(spdf[j] > Constants::Epsilon()))
        {
          pdf_r += pr[j] / spdf[j];
          pdf_i += pi[j] / spdf[j];
        }
    }
    pdf_r /= samples;
    pdf_i /= samples;
    std::cout << " Integral = " << pdf_r << "/" << pdf_i << " (radiance/importance) for " << sample_t.direction << std::endl;
  }
}

// checkBsdf.cpp:300-418 in the reference's order (rng=mt19937): per trial its direction, the per-bin pdf integrals
// (bin by bin, pdfSamples draws each), then the sample counts, the chi-square and P as the reference forms them
static void sampleOrdered(const hip::model_desc& m, size_t pdfSamples, size_t samples, size_t theta, size_t phi,
                          size_t trials, bool samplesphere, bool includeZeroPdfSamples, draw_source& rng)
{
  std::vector<float> x0[1], x1[1];
  size_t off = 0;
  for(size_t tr = 0; tr < trials; ++tr)
  {
    rng.fill(off++, 1, 1, x0, x1);
    const BsdfSample sample_t = uniformDirection(Vec2d(x0[0][0], x1[0][0]), samplesphere);
    std::vector<Value> pdf(theta * phi, 0), count(theta * phi, 0);
    // the pdf integrals: all bins' draws in order, evaluated in chunks
    const size_t total = theta * phi * pdfSamples;
    Vec2d sph_coord;
    for(size_t s0 = 0; s0 < total; s0 += kChunk)
    {
      const size_t k = std::min(kChunk, total - s0);
      rng.fill(off, k, 1, x0, x1);
      off += k;
      std::vector<Vec3d> dirs(k), ts(k, sample_t.direction);
      std::vector<Value> w(k);
      for(size_t j = 0; j < k; ++j)
      {
        const size_t idx = (s0 + j) / pdfSamples, t = idx / phi, p = idx % phi;
        const Vec2d rnd(x0[0][j], x1[0][j]);
        spherical::phi(sph_coord) = Constants::Pi(2) * (p + rnd[0]) / phi;
        spherical::theta(sph_coord) = Constants::Pi() * (t + rnd[1]) / theta;
        dirs[j] = spherical::convert(sph_coord);
        w[j] = Constants::Pi2(2) * bbm::abs(spherical::sinTheta(sph_coord)) / (phi * theta);
      }
      const auto pv = pdfBatch(m, dirs, ts, unit_t::Radiance);
      for(size_t j = 0; j < k; ++j)
      {
        const size_t idx = (s0 + j) / pdfSamples;
        pdf[idx] += pv[j] * w[j];
        if((s0 + j) % pdfSamples == pdfSamples - 1) pdf[idx] /= pdfSamples;
      }
    }
    // the sample counts
    for(size_t s0 = 0; s0 < samples; s0 += kChunk)
    {
      const size_t k = std::min(kChunk, samples - s0);
      rng.fill(off, k, 1, x0, x1);
      off += k;
      dev3 dt(k), dd(k);
      dt.upload(std::vector<Vec3d>(k, sample_t.direction));
      hip::device_vector<float> a(k), b(k), sp(k);
      hip::device_vector<uint32_t> fl(k);
      upload_of(a, x0[0]); upload_of(b, x1[0]);
      hip::sample(m, dt.in(), a.data(), b.data(), k, dd.out(), sp.data(), fl.data());
      const auto dirs = dd.download(k);
      const auto hp = download(sp, k);
      for(size_t j = 0; j < k; ++j)
        if(includeZeroPdfSamples || bbm::any(hp[j] > Constants::Epsilon()))
        {
          sph_coord = spherical::convert(dirs[j]);
          size_t t = bbm::cast<size_t>(bbm::min(spherical::theta(sph_coord) / Constants::Pi() * theta, theta - 1));
          size_t p = bbm::cast<size_t>(bbm::min(spherical::phi(sph_coord) / Constants::Pi(2) * phi, phi - 1));
          count[t * phi + p]++;
        }
    }
    Value chi2 = 0, df = -1;
    for(size_t idx = 0; idx < theta * phi; ++idx)
    {
      Value mm = pdf[idx] * samples;
      if(bbm::any(mm > Constants::Epsilon() && count[idx] > 5))
      {
        chi2 += pow(count[idx] - mm, 2) / mm;
        df++;
      }
    }
    std::cout << " Chi2 for " << sample_t.direction << " = " << chi2 << " (with " << df << " degrees of freedom)." << std::endl;
    if(bbm::any(df > 1))
    {
      Value P = bbm::gamma_q((df - 1) / 2, chi2 / 2);
      std::cout << "  P = " << P << " (reject if lower than confidence)." << std::endl;
    }
    else std::cout << " No degrees of freedom; need at least 1 to compute P." << std::endl;
  }
}

static void testReflectance(const hip::model_desc& m, const option_parser& opt, uint64_t seed)
{
  size_t samples = opt.get<size_t>("samples", 100000);
  size_t numtheta = opt.get<size_t>("theta", 1);
  bool importance = opt.get<bool>("importanceSampling", false);
  if(!valid(opt, {"bsdfmodel", "test", "samples", "theta", "importanceSampling"})) return;
  std::cout << "Reflectance test with " << numtheta << " directions and " << samples << " samples." << std::endl;
  if(opt.get<std::string>("rng", "counter") == "mt19937")
  {
    draw_source rng(true, seed, BBM_CHECK_REFLECTANCE);
    reflectanceOrdered(m, samples, numtheta, importance, rng);
    return;
  }
  const auto r = hip::check_reflectance(m, samples, numtheta, importance, seed);
  for(size_t t = 0; t < numtheta; ++t)
    std::cout << " out = " << to_vec(r.out[t]) << " => Estimate: " << spec(r.estimate[t]) << " vs. " << spec(r.reflectance[t]) << std::endl;
}

static void testReciprocity(const hip::model_desc& m, const option_parser& opt, uint64_t seed)
{
  size_t samples = opt.get<size_t>("samples", 1000000);
  if(!valid(opt, {"bsdfmodel", "test", "samples"})) return;
  std::cout << "Reciprocity test with " << samples << " samples." << std::endl;
  if(opt.get<std::string>("rng", "counter") == "mt19937")
  {
    draw_source rng(true, seed, BBM_CHECK_RECIPROCITY);
    symmetryOrdered(m, samples, false, rng);
    return;
  }
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
  if(opt.get<std::string>("rng", "counter") == "mt19937")
  {
    draw_source rng(true, seed, BBM_CHECK_ADJOINT);
    symmetryOrdered(m, samples, true, rng);
    return;
  }
  const auto r = hip::check_adjoint(m, samples, seed);
  const Vec3dPair pa{to_vec(r.in), to_vec(r.out)};
  std::cout << "Adjoint difference average = " << spec(r.average) << ", max = " << spec(r.max) << " at " << pa << std::endl;
}

static void testPdf(const hip::model_desc& m, const option_parser& opt, uint64_t seed)
{
  size_t samples = opt.get<size_t>("samples", 100000);
  size_t maxError = opt.get<size_t>("maxError", 10);
  bool checkBelowHorizon = opt.get<bool>("checkBelowHorizon", false);
  bool samplesphere = opt.get<bool>("sampleSphere", false);
  if(!valid(opt, {"bsdfmodel", "test", "samples", "maxError", "checkBelowHorizon", "sampleSphere"})) return;
  std::cout << "Tesing PDF properties test with " << samples << " samples." << std::endl;
  draw_source rng(opt.get<std::string>("rng", "counter") == "mt19937", seed, BBM_CHECK_PDF);

  // checkBsdf.cpp:219-243: the reference's loop, its three rndVec2d() per sample (the uniform direction, the radiance
  // and the importance sample), the four BSDF calls batched on the GPU per chunk, the checks, prints and the float
  // mismatch sums on the host in sample order, stopping as the reference does once maxError failures of one kind
  size_t count_negative_r = 0, count_negative_i = 0;
  size_t count_zr = 0, count_zi = 0;
  Value mismatch_r = 0, mismatch_i = 0;
  std::vector<float> x0[3], x1[3];
  auto running = [&]() { return count_negative_r < maxError && count_negative_i < maxError && count_zr < maxError && count_zi < maxError; };
  for(size_t s0 = 0; s0 < samples && running(); s0 += kChunk)
  {
    const size_t k = std::min(kChunk, samples - s0);
    rng.fill(s0, k, 3, x0, x1);
    std::vector<Vec3d> dirs(k);
    for(size_t j = 0; j < k; ++j) dirs[j] = uniformDirection(Vec2d(x0[0][j], x1[0][j]), samplesphere).direction;
    dev3 dd(k), dr(k), di(k);
    dd.upload(dirs);
    hip::device_vector<float> w0(k), w1(k), z0(k), z1(k), sr(k), si(k), pr(k), pi(k);
    hip::device_vector<uint32_t> fr(k), fi(k);
    upload_of(w0, x0[1]); upload_of(w1, x1[1]); upload_of(z0, x0[2]); upload_of(z1, x1[2]);
    hip::sample(m, dd.in(), w0.data(), w1.data(), k, dr.out(), sr.data(), fr.data(), bsdf_flag::All, unit_t::Radiance);
    hip::sample(m, dd.in(), z0.data(), z1.data(), k, di.out(), si.data(), fi.data(), bsdf_flag::All, unit_t::Importance);
    hip::pdf(m, dr.in(), dd.in(), k, pr.data(), bsdf_flag::All, unit_t::Radiance);
    hip::pdf(m, di.in(), dd.in(), k, pi.data(), bsdf_flag::All, unit_t::Importance);
    const auto hr = dr.download(k), hi = di.download(k);
    const auto hsr = download(sr, k), hsi = download(si, k), hpr = download(pr, k), hpi = download(pi, k);
    for(size_t j = 0; j < k && running(); ++j)
    {
      if(checkBelowHorizon && vec::z(hr[j]) < 0) { count_zr++; std::cout << " Sampled direction " << hr[j] << " below horizon for " << dirs[j] << std::endl; }
      if(checkBelowHorizon && vec::z(hi[j]) < 0) { count_zi++; std::cout << " Sampled direction " << hi[j] << " below horizon for " << dirs[j] << std::endl; }
      if(hpr[j] < 0) { count_negative_r++; std::cout << " Negative PDF (" << hpr[j] << ") for (" << hr[j] << ", " << dirs[j] << ")" << std::endl; }
      if(hpi[j] < 0) { count_negative_i++; std::cout << " Negative PDF (" << hpi[j] << ") for (" << hi[j] << ", " << dirs[j] << ")" << std::endl; }
      mismatch_r += bbm::abs(hsr[j] - hpr[j]);
      mismatch_i += bbm::abs(hsi[j] - hpi[j]);
    }
  }
  mismatch_r /= samples;
  mismatch_i /= samples;
  std::cout << "PDF has " << count_negative_r << "/" << count_negative_i << " negative PDF values, ";
  if(checkBelowHorizon) std::cout << count_zr << "/" << count_zi << " sampled directions below the horizon, ";
  std::cout << "and " << mismatch_r << "/" << mismatch_i
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
  if(opt.get<std::string>("rng", "counter") == "mt19937")
  {
    draw_source rng(true, seed, BBM_CHECK_PDFINT);
    pdfIntOrdered(m, samples, trials, samplesphere, rng);
    return;
  }
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
  if(opt.get<std::string>("rng", "counter") == "mt19937")
  {
    draw_source rng(true, seed, BBM_CHECK_SAMPLE_PDF);
    sampleOrdered(m, pdfSamples, samples, theta, phi, trials, samplesphere, includeZeroPdfSamples, rng);
    return;
  }
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
    std::cout << "Usage: " << argv[0] << " [bsdfmodel=<bsdf string>] [test=<test name> [test options]" << std::endl;
    std::cout << "  + test=reflectance [samples=100000] [theta=1] [importanceSampling]: compare the approximated reflectance method with a MC integration of the BSDF." << std::endl;
    std::cout << "  + test=reciprocity [samples=100000]: checks if the BSDF is symmetric for 'samples' random dirctions." << std::endl;
    std::cout << "  + test=adjoint [samples=100000]: checks if the adjoint BSDF is equal to the BSDF with in/out swapped." << std::endl;
    std::cout << "  + test=pdf [samples=100000] [maxError=10] [checkBelowHorizon] [sampleSphere]: checks if the PDF >= 0, and the PDF returned by the sampling method matches the pdf from the pdf-method. Abort if the number of fails exceeds 'maxError'" << std::endl;
    std::cout << "  + test=pdfInt [samples=100000] [trials=10] [sampleSphere]: checks the integral (MC with 'samples' samples) of the PDF for 'trials' different directions." << std::endl;
    std::cout << "  + test=sample [pdfSamples=4069] [samples=100000] [theta=10] [phi=20] [trials=10] [sampleSphere] [includeZeroPdfSamples]: perform Chi2 test on the sample vs the pdf method.  The domain is subdivided in [theta x phi] bins, and for each bin we integrate the PDF using MC.  A higher sampling rate might be needed for sharp BSDFs." << std::endl;
    std::cout << "  (HIP backbone) [seed=5489] [rng=counter|mt19937]: the draws' seed; the library's counter draws (GPU reductions) or the reference's std::mt19937 sequence and loop order." << std::endl;
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
