// tests/cpp/adapter_check.cpp -- drop-in check of the C++ host adapter (backbone/hip).
//
// The SAME bbm::bsdfmodel<> instances (reference template API, native floatRGB backbone for the
// per-pair CPU calls) are evaluated twice: once per pair on the CPU through the reference's own
// eval/pdf/sample, once in batch on the GPU through bbm::hip::{eval_pdf, sample}.  Prints one JSON
// line per model; exit code 1 if any model misses the parity bar.
//
// Built in the build container by tests/cpp/Makefile (needs /root/reference headers at compile
// time only); the binary runs on the GPU box.
#include "bbm/bbm_core.h"
#include "bsdfmodel/scaledmodel.h"
#include "bsdfmodel/microfacet.h"
#include "bsdfmodel/lambertian.h"
#include "bsdfmodel/cooktorrance.h"
#include "bsdfmodel/cooktorrancewalter.h"
#include "bsdfmodel/ggx.h"
#include "bsdfmodel/ashikhminshirley.h"
#include "bsdfmodel/lowmicrofacet.h"
#include "bsdfmodel/low.h"
#include "bsdfmodel/orennayar.h"
#include "bsdfmodel/ward.h"
#include "bsdfmodel/wardduer.h"
#include "bsdfmodel/wardduergeislermoroder.h"
#include "bsdfmodel/phong.h"
#include "bsdfmodel/lafortune.h"
#include "bsdfmodel/ashikhminshirleyfull.h"
#include "bsdfmodel/lowsmooth.h"
#include "bsdfmodel/cooktorranceheitz.h"
#include "bsdfmodel/ggxheitz.h"
#include "bsdfmodel/phongwalter.h"
#include "bsdfmodel/ribardiere.h"
#include "bsdfmodel/bagher.h"
#include "bsdfmodel/aggregatemodel.h"
#include "loss/cosine_weighted_log.h"
#include "bbm_hip/batch.h"

#include <hip/hip_runtime_api.h>

#include <cmath>
#include <cstdio>
#include <random>
#include <limits>
#include <string>
#include <type_traits>
#include <vector>

#define HIPCHECK(x) do { hipError_t e_ = (x); if(e_ != hipSuccess) { std::fprintf(stderr, "HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); std::exit(2); } } while(0)

struct dev_buf
{
  float* p = nullptr;
  explicit dev_buf(size_t n) { HIPCHECK(hipMalloc(&p, n * sizeof(float))); }
  dev_buf(const dev_buf&) = delete;
  dev_buf& operator=(const dev_buf&) = delete;
  dev_buf(dev_buf&& o) noexcept : p(o.p) { o.p = nullptr; }
  ~dev_buf() { if(p) (void)hipFree(p); }
};

static void upload(dev_buf& d, const std::vector<float>& h) { HIPCHECK(hipMemcpy(d.p, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice)); }
static std::vector<float> download(const dev_buf& d, size_t n) { std::vector<float> h(n); HIPCHECK(hipMemcpy(h.data(), d.p, n * sizeof(float), hipMemcpyDeviceToHost)); return h; }

static double relerr(double a, double b)
{
  if(a == b || (std::isnan(a) && std::isnan(b))) return 0;
  return std::fabs(a - b) / std::max(std::fabs(b), 1e-30);
}

template<typename MODEL>
static bool check_model(const MODEL& model, size_t n, unsigned seed)
{
  using Vec3d = typename MODEL::Vec3d;
  using Vec2d = typename MODEL::Vec2d;
  std::mt19937 rng(seed);
  std::uniform_real_distribution<float> u(0.0f, 1.0f);
  std::vector<float> h[8];
  for(auto& v : h) v.resize(n);
  for(size_t i = 0; i < n; ++i)
    for(int k = 0; k < 2; ++k)
    {
      float z = 2.0f * u(rng) - 1.0f, phi = 6.2831853f * u(rng), s = std::sqrt(std::max(1.0f - z * z, 0.0f));
      h[3 * k + 0][i] = s * std::cos(phi); h[3 * k + 1][i] = s * std::sin(phi); h[3 * k + 2][i] = z;
    }
  for(size_t i = 0; i < n; ++i) { h[6][i] = u(rng); h[7][i] = u(rng); }
  std::vector<dev_buf> d;
  d.reserve(8);
  for(int k = 0; k < 8; ++k) { d.emplace_back(n); upload(d.back(), h[k]); }
  dev_buf r(n), g(n), b(n), pdf(n), sx(n), sy(n), sz(n), spdf(n), sflag(n);
  bbm::hip::soa3 in{d[0].p, d[1].p, d[2].p}, out{d[3].p, d[4].p, d[5].p};
  bbm::hip::eval_pdf(model, in, out, n, {r.p, g.p, b.p}, pdf.p);
  bbm::hip::sample(model, out, d[6].p, d[7].p, n, {sx.p, sy.p, sz.p}, spdf.p, reinterpret_cast<uint32_t*>(sflag.p));
  HIPCHECK(hipDeviceSynchronize());
  auto R = download(r, n), G = download(g, n), B = download(b, n), P = download(pdf, n);
  auto SX = download(sx, n), SY = download(sy, n), SZ = download(sz, n), SP = download(spdf, n);
  std::vector<uint32_t> SF(n);
  HIPCHECK(hipMemcpy(SF.data(), sflag.p, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
  // reflectance(out) through the adapter vs the reference's own
  bbm::hip::reflectance(model, out, n, {r.p, g.p, b.p});
  HIPCHECK(hipDeviceSynchronize());
  auto RR = download(r, n), RG = download(g, n), RB = download(b, n);
  size_t bad_refl = 0;
  for(size_t i = 0; i < n; ++i)
  {
    auto rf = model.reflectance(Vec3d(h[3][i], h[4][i], h[5][i]));
    const float got[3] = {RR[i], RG[i], RB[i]};
    for(int k = 0; k < 3; ++k)
      if(!(got[k] == rf[k] || std::fabs(double(got[k]) - double(rf[k])) <= 1e-5 * std::fabs(double(rf[k])) + 1e-7)) ++bad_refl;
  }

  double peak = 0, ppeak = 0;
  std::vector<float> ce(3 * n), cp(n);
  for(size_t i = 0; i < n; ++i)
  {
    Vec3d vin(h[0][i], h[1][i], h[2][i]), vout(h[3][i], h[4][i], h[5][i]);
    auto e = model.eval(vin, vout);
    ce[3 * i] = e[0]; ce[3 * i + 1] = e[1]; ce[3 * i + 2] = e[2];
    cp[i] = model.pdf(vin, vout);
    if(std::isfinite(e[0])) peak = std::max(peak, std::fabs(double(e[0])));
    if(std::isfinite(cp[i])) ppeak = std::max(ppeak, std::fabs(double(cp[i])));
  }
  size_t bad = 0, bad_flag = 0;
  double worst = 0;
  for(size_t i = 0; i < n; ++i)
  {
    const float got[4] = {R[i], G[i], B[i], P[i]};
    const float ref[4] = {ce[3 * i], ce[3 * i + 1], ce[3 * i + 2], cp[i]};
    for(int k = 0; k < 4; ++k)
    {
      const double floor = 1e-6 * (k < 3 ? peak : ppeak);
      const double d = std::fabs(double(got[k]) - double(ref[k]));
      if(!(got[k] == ref[k] || (std::isnan(got[k]) && std::isnan(ref[k])) || d <= 1e-5 * std::fabs(double(ref[k])) + floor)) ++bad;
      if(std::fabs(ref[k]) > floor) worst = std::max(worst, relerr(got[k], ref[k]));
    }
    // sample: same flag; pdf of the GPU direction equals the CPU model's pdf at that direction
    Vec3d vout(h[3][i], h[4][i], h[5][i]);
    auto s = model.sample(vout, Vec2d(h[6][i], h[7][i]));
    if(uint32_t(s.flag) != SF[i]) ++bad_flag;
    Vec3d sd(SX[i], SY[i], SZ[i]);
    // the GPU sample's pdf equals the CPU sample's own pdf, or (a sharp lobe amplifies a 1-ulp
    // direction difference) the pdf the CPU sampler reports for the GPU direction.  Rejected lanes
    // (flag None) return the all-zero sample, whose pdf(0-vector) is undefined.
    auto close = [&](float a, float r) { return a == r || std::fabs(double(a) - double(r)) <= 1e-5 * std::fabs(double(r)) + 1e-6 * ppeak; };
    float at_dir = (uint32_t(s.flag) != 0) ? float(model.pdf(sd, vout)) : float(s.pdf);
    if constexpr (std::is_same_v<MODEL, bbm::ashikhminshirleyfull<bbm::floatRGB>>)
    {
      // w_s pdf_s(specular candidate) + w_d pdf_d(diffuse candidate): the chosen candidate at the
      // GPU direction, the other one drawn on the CPU (ashikhminshirleyfull.h:103-121)
      using V = float;
      const V sa = bbm::hsum(model.fresnelReflectance.value());
      const V da = bbm::hsum(model.diffuseReflectance.value()) * (V(1) - sa);
      const V dw = da / (da + sa), sw = V(1) - dw, eps = std::numeric_limits<V>::epsilon();
      const V xs = sw > eps ? V(h[6][i] / sw) : V(0), xd = dw > eps ? V((h[6][i] - sw) / dw) : V(0);
      const bool spec = uint32_t(s.flag) == uint32_t(bbm::bsdf_flag::Specular);
      const V ps = spec ? V(model.pdf(sd, vout, bbm::bsdf_flag::Specular)) : V(model.sample(vout, Vec2d(xs, h[7][i]), bbm::bsdf_flag::Specular).pdf);
      const V pd = !spec ? V(model.pdf(sd, vout, bbm::bsdf_flag::Diffuse)) : V(model.sample(vout, Vec2d(xd, h[7][i]), bbm::bsdf_flag::Diffuse).pdf);
      at_dir = (uint32_t(s.flag) != 0) ? sw * ps + dw * pd : float(s.pdf);
    }
    if(!(close(SP[i], float(s.pdf)) || close(SP[i], at_dir))) ++bad;
  }
  const bool ok = bad == 0 && bad_flag == 0 && bad_refl == 0;
  std::printf("{\"model\": \"%s\", \"n\": %zu, \"violations\": %zu, \"flag_mismatch\": %zu, \"reflectance_violations\": %zu, \"max_rel_err\": %.3e, \"ok\": %s}\n",
              bbm::toString(model).c_str(), n, bad, bad_flag, bad_refl, worst, ok ? "true" : "false");
  return ok;
}

// sampledlossfunction through the adapter (bbm::hip::loss_sums: 3 probes in one launch) vs the
// reference's own standardLog_error summed over the same pairs (double sums, 1e-5)
template<typename MODEL>
static bool check_loss(const MODEL& fitted, const MODEL& reference, size_t n, unsigned seed)
{
  using Vec3d = typename MODEL::Vec3d;
  std::mt19937 rng(seed);
  std::uniform_real_distribution<float> u(0.0f, 1.0f);
  std::vector<float> h[6];
  for(auto& v : h) v.resize(n);
  for(size_t i = 0; i < n; ++i)
    for(int k = 0; k < 2; ++k)
    {
      float z = u(rng), phi = 6.2831853f * u(rng), s = std::sqrt(std::max(1.0f - z * z, 0.0f));
      h[3 * k + 0][i] = s * std::cos(phi); h[3 * k + 1][i] = s * std::sin(phi); h[3 * k + 2][i] = z;
    }
  std::vector<dev_buf> d;
  d.reserve(6);
  for(int k = 0; k < 6; ++k) { d.emplace_back(n); upload(d.back(), h[k]); }
  bbm::hip::soa3 in{d[0].p, d[1].p, d[2].p}, out{d[3].p, d[4].p, d[5].p};
  dev_buf rr(n), rg(n), rb(n);
  bbm::hip::eval(reference, in, out, n, {rr.p, rg.p, rb.p});
  // probes: the fitted parameters, the reference's, and the fitted ones scaled by 1.01
  std::vector<std::vector<float>> pv = {bbm::hip::parameters(fitted), bbm::hip::parameters(reference), bbm::hip::parameters(fitted)};
  for(auto& x : pv[2]) x *= 1.01f;
  const size_t np = pv[0].size();
  std::vector<float> flat;
  for(auto& v : pv) flat.insert(flat.end(), v.begin(), v.end());
  dev_buf probes(flat.size());
  upload(probes, flat);
  const size_t wsb = bbm_hip_loss_workspace_size(3);
  void* ws = nullptr;
  double* sums = nullptr;
  HIPCHECK(hipMalloc(&ws, wsb));
  HIPCHECK(hipMalloc(reinterpret_cast<void**>(&sums), 3 * sizeof(double)));
  bbm::hip::loss_sums(fitted, probes.p, 3, in, out, n, {rr.p, rg.p, rb.p}, bbm::hip::loss_t::standardLog, sums, ws, wsb);
  double got[3];
  HIPCHECK(hipMemcpy(got, sums, sizeof(got), hipMemcpyDeviceToHost));
  (void)hipFree(ws);
  (void)hipFree(sums);
  bbm::standardLog_error<bbm::floatRGB> err;
  bool ok = true;
  double worst = 0;
  for(int p = 0; p < 3; ++p)
  {
    MODEL m = fitted;
    auto pvals = bbm::parameter_values(m, bbm::bsdf_attr(0x1F));
    for(size_t j = 0; j < np; ++j) pvals[j] = pv[p][j];
    double want = 0;
    for(size_t i = 0; i < n; ++i)
    {
      Vec3d vin(h[0][i], h[1][i], h[2][i]), vout(h[3][i], h[4][i], h[5][i]);
      want += double(err(vin, vout, m.eval(vin, vout), reference.eval(vin, vout)));
    }
    const double e = std::fabs(got[p] - want);
    worst = std::max(worst, e / std::max(std::fabs(want), 1e-30));
    ok &= (p == 1) ? (got[p] == 0.0 && want == 0.0) : (e <= 1e-5 * std::fabs(want));
  }
  std::printf("{\"loss\": \"standardLog\", \"model\": \"%s\", \"n\": %zu, \"max_rel_err\": %.3e, \"ok\": %s}\n",
              bbm::toString(fitted).c_str(), n, worst, ok ? "true" : "false");
  return ok;
}

int main()
{
  const size_t n = 1 << 18;
  bool ok = true;
  bbm::cooktorrance<bbm::floatRGB> ct;
  ok &= check_model(ct, n, 1);
  bbm::cooktorrance<bbm::floatRGB> ct2;
  {
    auto p = bbm::parameter_values(ct2);
    p[0] = 0.2f; p[1] = 0.4f; p[2] = 0.6f; p[3] = 0.35f; p[4] = 2.1f;
  }
  ok &= check_model(ct2, n, 2);
  ok &= check_model(bbm::ggx<bbm::floatRGB>(), n, 3);
  ok &= check_model(bbm::lambertian<bbm::floatRGB>(), n, 4);
  ok &= check_model(bbm::cooktorrancewalter<bbm::floatRGB>(), n, 5);
  ok &= check_model(bbm::lowcooktorrance<bbm::floatRGB>(), n, 6);
  ok &= check_model(bbm::orennayar<bbm::floatRGB>(), n, 7);
  ok &= check_model(bbm::ward<bbm::floatRGB>(), n, 8);
  ok &= check_model(bbm::wardduer<bbm::floatRGB>(), n, 9);
  ok &= check_model(bbm::wardduergeislermoroder<bbm::floatRGB>(), n, 10);
  ok &= check_model(bbm::phong<bbm::floatRGB>(), n, 11);
  ok &= check_model(bbm::lafortune<bbm::floatRGB>(), n, 12);
  ok &= check_model(bbm::ashikhminshirley<bbm::floatRGB>(), n, 13);
  ok &= check_model(bbm::ashikhminshirleyfull<bbm::floatRGB>(), n, 14);
  ok &= check_model(bbm::lowsmooth<bbm::floatRGB>(), n, 15);
  ok &= check_model(bbm::lowmicrofacet<bbm::floatRGB>(), n, 16);
  ok &= check_model(bbm::lowashikhminshirley<bbm::floatRGB>(), n, 17);
  ok &= check_model(bbm::cooktorranceheitz<bbm::floatRGB>(), n, 18);
  ok &= check_model(bbm::ggxheitz<bbm::floatRGB>(), n, 19);
  ok &= check_model(bbm::phongwalter<bbm::floatRGB>(), n, 20);
  ok &= check_model(bbm::ribardiere<bbm::floatRGB>(), n, 21);
  ok &= check_model(bbm::ribardiereanisotropic<bbm::floatRGB>(), n, 22);
  ok &= check_model(bbm::bagher<bbm::floatRGB>(), n, 23);
  using agg_bagher = bbm::aggregatemodel<bbm::lambertian<bbm::floatRGB>, bbm::bagher<bbm::floatRGB>>;
  using agg_ct = bbm::aggregatemodel<bbm::lambertian<bbm::floatRGB>, bbm::cooktorrance<bbm::floatRGB>>;
  ok &= check_model(agg_bagher(), n, 24);
  ok &= check_model(agg_ct(), n, 25);
  {
    // a fit: Aggregate(Lambertian, CookTorrance) against a perturbed reference of the same type
    agg_ct fitted, reference;
    auto p = bbm::parameter_values(reference, bbm::bsdf_attr(0x1F));
    for(auto& x : p) x = float(x) * 1.1f;
    ok &= check_loss(fitted, reference, 1 << 16, 26);
    agg_bagher bf, br;
    auto q = bbm::parameter_values(br, bbm::bsdf_attr(0x1F));
    for(auto& x : q) x = float(x) * 0.9f;
    ok &= check_loss(bf, br, 1 << 16, 27);
  }
  return ok ? 0 : 1;
}
