/* backbone/hip/include/bbm_hip/check.h -- C++20 host adapter: checkBsdf's statistics on the GPU.
 *
 * bin/checkBsdf.cpp (:51-418) validates a BSDF with six Monte-Carlo tests, one serial loop each.  Here every test is
 * one or two batched reductions of libbbm_hip (bbm_hip_check for a single-kernel floatRGB model, bbm_hip_check_tree /
 * _f64 for any other model tree), with the same per-sample terms in the reference's float semantics, double
 * accumulators and a fixed-order final reduction; the host divides by the sample counts and forms the printed numbers
 * (reflectance estimate, average / max differences, mismatch, integral, chi-square and its P value through the
 * reference's own bbm::gamma_q, include/util/gamma.h:564).
 *
 * Random numbers: counter-based, one stream per (test, slot, draw) (bbm_hip_check_draws) instead of the reference's one
 * std::mt19937 -- statistically equivalent; what a GPU computes for a sample is fixed by (seed, sample index), so the
 * samples can be split over GPUs.  The pdf test does not stop at maxError failures (it counts them all).
 *
 *   auto m = bbm::hip::from_string("CookTorrance(roughness=0.3)");
 *   auto r = bbm::hip::check_reflectance(m, 1000000, 4, false);    // r.estimate[t] vs r.reflectance[t]
 *
 * backbone/hip/bin/checkBsdf.cpp is the reference's command line on top of these functions.
 */
#ifndef BBM_HIP_CHECK_H
#define BBM_HIP_CHECK_H

#include <array>
#include <cmath>
#include <limits>
#include <vector>

#include "bbm_hip/fit.h"
#include "util/gamma.h"

namespace bbm {
  namespace hip {

    //! \brief checkBsdf's default random seed here: std::mt19937's default (the reference never seeds its `rnd`)
    constexpr uint64_t check_default_seed = 5489;

    using rgb_t = std::array<float, 3>;

    namespace detail {
      //! \brief one statistic of model m: (nslots x BBM_CHECK_ACC) accumulators, or for SAMPLE_COUNT the counts
      template<typename T>
        inline void check_run(const basic_model_desc<T>& m, bbm_hip_check_desc d, const T* sx, const T* sy, const T* sz,
                              std::vector<double>* acc, std::vector<uint64_t>* counts, void* stream)
      {
        const bool tree = m.composed() || !std::is_same_v<T, float>;
        const size_t nb = size_t(d.theta_bins) * d.phi_bins;
        device_vector<double> dacc;
        device_vector<uint64_t> dcnt;
        device_vector<char> ws;
        size_t wsb = 0;
        if(d.test == BBM_CHECK_SAMPLE_COUNT) dcnt.resize(size_t(d.nslots) * nb);
        else
        {
          dacc.resize(size_t(d.nslots) * BBM_CHECK_ACC);
          wsb = tree ? bbm_hip_check_tree_workspace_size(&d) : bbm_hip_check_workspace_size(&d);
          ws.resize(wsb);
        }
        if constexpr (std::is_same_v<T, float>)
        {
          d.slot_x = sx; d.slot_y = sy; d.slot_z = sz;
          if(tree)
          {
            // (the child arrays point into m: built from m itself, never from a temporary copy)
            const child_tree<float> c(m);
            const bbm_hip_child leaf{m.id, m.params.data(), int(m.params.size()), nullptr, 0};
            check(bbm_hip_check_tree(m.composed() ? c.root : &leaf, m.composed() ? c.count : 1, &d, dacc.data(),
                                     dcnt.data(), ws.data(), wsb, stream));
          }
          else
            check(bbm_hip_check(m.id, m.params.data(), int(m.params.size()), &d, dacc.data(), dcnt.data(), ws.data(), wsb,
                                stream));
        }
        else
        {
          const child_tree<double> c(m);
          const bbm_hip_child_f64 leaf{m.id, m.params.data(), int(m.params.size()), nullptr, 0};
          check(bbm_hip_check_tree_f64(m.composed() ? c.root : &leaf, m.composed() ? c.count : 1, &d, sx, sy, sz,
                                       dacc.data(), dcnt.data(), ws.data(), wsb, stream));
        }
        hip_check(hipStreamSynchronize(static_cast<hipStream_t>(stream)), "hipStreamSynchronize");
        if(acc)
        {
          acc->resize(size_t(d.nslots) * BBM_CHECK_ACC);
          hip_check(hipMemcpy(acc->data(), dacc.data(), acc->size() * sizeof(double), hipMemcpyDeviceToHost), "hipMemcpy");
        }
        if(counts)
        {
          counts->resize(size_t(d.nslots) * nb);
          hip_check(hipMemcpy(counts->data(), dcnt.data(), counts->size() * sizeof(uint64_t), hipMemcpyDeviceToHost), "hipMemcpy");
        }
      }

      inline bbm_hip_check_desc check_desc(int test, int nslots, uint64_t seed, uint64_t n)
      {
        bbm_hip_check_desc d{};
        d.test = test; d.nslots = nslots; d.seed = seed; d.begin = 0; d.n = n;
        return d;
      }

      //! \brief trial directions of pdfInt / sample (checkBsdf.cpp:294, :347), host copy and device arrays
      struct trials
      {
        device_vector<float> x, y, z;
        std::vector<rgb_t> host;
        trials(int test, uint64_t seed, size_t n, bool sphere, void* stream) : x(n), y(n), z(n), host(n)
        {
          check(bbm_hip_check_trials(test, seed, int(n), sphere ? 1 : 0, x.data(), y.data(), z.data(), stream));
          hip_check(hipStreamSynchronize(static_cast<hipStream_t>(stream)), "hipStreamSynchronize");
          std::vector<float> h[3] = {std::vector<float>(n), std::vector<float>(n), std::vector<float>(n)};
          hip_check(hipMemcpy(h[0].data(), x.data(), n * 4, hipMemcpyDeviceToHost), "hipMemcpy");
          hip_check(hipMemcpy(h[1].data(), y.data(), n * 4, hipMemcpyDeviceToHost), "hipMemcpy");
          hip_check(hipMemcpy(h[2].data(), z.data(), n * 4, hipMemcpyDeviceToHost), "hipMemcpy");
          for(size_t i = 0; i < n; ++i) host[i] = {h[0][i], h[1][i], h[2][i]};
        }
      };
    } // end detail namespace

    //! \brief reflectance test (checkBsdf.cpp:51-97)
    struct reflectance_stats
    {
      std::vector<rgb_t> out, estimate, reflectance;
      std::vector<double> accepted;           //!< samples with pdf > Epsilon per direction
    };

    inline reflectance_stats check_reflectance(const model_desc& m, size_t samples, size_t numtheta, bool importance,
                                               uint64_t seed = check_default_seed, void* stream = nullptr)
    {
      reflectance_stats r;
      // out = spherical::convert((theta_idx Pi(0.5) / numtheta, 0)) (checkBsdf.cpp:73-75)
      std::vector<float> ox(numtheta), oy(numtheta), oz(numtheta);
      for(size_t t = 0; t < numtheta; ++t)
      {
        const float theta = float(t) * float(0.5 * 3.14159265358979323846) / float(numtheta);
        const float st = float(std::sin(double(theta))), ct = float(std::cos(double(theta)));
        ox[t] = 1.0f * st; oy[t] = 0.0f * st; oz[t] = ct;
        r.out.push_back({ox[t], oy[t], oz[t]});
      }
      device_vector<float> dx(numtheta), dy(numtheta), dz(numtheta), rr(numtheta), rg(numtheta), rb(numtheta);
      hip_check(hipMemcpy(dx.data(), ox.data(), numtheta * 4, hipMemcpyHostToDevice), "hipMemcpy");
      hip_check(hipMemcpy(dy.data(), oy.data(), numtheta * 4, hipMemcpyHostToDevice), "hipMemcpy");
      hip_check(hipMemcpy(dz.data(), oz.data(), numtheta * 4, hipMemcpyHostToDevice), "hipMemcpy");
      auto d = detail::check_desc(BBM_CHECK_REFLECTANCE, int(numtheta), seed, samples);
      d.importance = importance ? 1 : 0;
      std::vector<double> acc;
      detail::check_run<float>(m, d, dx.data(), dy.data(), dz.data(), &acc, nullptr, stream);
      reflectance(m, soa3{dx.data(), dy.data(), dz.data()}, numtheta, soa3_out{rr.data(), rg.data(), rb.data()},
                  bsdf_flag::All, unit_t::Radiance, nullptr, stream);
      hip_check(hipStreamSynchronize(static_cast<hipStream_t>(stream)), "hipStreamSynchronize");
      std::vector<float> h[3] = {std::vector<float>(numtheta), std::vector<float>(numtheta), std::vector<float>(numtheta)};
      hip_check(hipMemcpy(h[0].data(), rr.data(), numtheta * 4, hipMemcpyDeviceToHost), "hipMemcpy");
      hip_check(hipMemcpy(h[1].data(), rg.data(), numtheta * 4, hipMemcpyDeviceToHost), "hipMemcpy");
      hip_check(hipMemcpy(h[2].data(), rb.data(), numtheta * 4, hipMemcpyDeviceToHost), "hipMemcpy");
      for(size_t t = 0; t < numtheta; ++t)
      {
        const double* a = acc.data() + t * BBM_CHECK_ACC;
        r.estimate.push_back({float(a[0] / double(samples)), float(a[1] / double(samples)), float(a[2] / double(samples))});
        r.reflectance.push_back({h[0][t], h[1][t], h[2][t]});
        r.accepted.push_back(a[3]);
      }
      return r;
    }

    //! \brief reciprocity (checkBsdf.cpp:102-152) and adjoint (:157-201) tests: per-channel average difference, and
    //! the largest difference (by its channel sum, first strict maximum) with the sample index it came from
    struct symmetry_stats
    {
      rgb_t average{}, max{};
      double max_hsum = 0;
      int64_t sample = -1;
      rgb_t in{}, out{};                      //!< the direction pair of that sample
    };

    namespace detail {
      //! \brief the (in, out) sphere pair of sample `index` of a symmetry test (draws 0 and 1 of slot 0)
      inline void check_pair_at(int test, uint64_t seed, int64_t index, rgb_t& in, rgb_t& out, void* stream)
      {
        device_vector<float> u(2), d(3);
        rgb_t* dst[2] = {&in, &out};
        for(int draw = 0; draw < 2; ++draw)
        {
          check(bbm_hip_check_draws(test, seed, 0, draw, uint64_t(index), 1, u.data(), u.data() + 1, stream));
          check(bbm_hip_sphere_dirs(u.data(), u.data() + 1, 1, 0, d.data(), d.data() + 1, d.data() + 2, stream));
          hip_check(hipStreamSynchronize(static_cast<hipStream_t>(stream)), "hipStreamSynchronize");
          float h[3];
          hip_check(hipMemcpy(h, d.data(), sizeof(h), hipMemcpyDeviceToHost), "hipMemcpy");
          *dst[draw] = {h[0], h[1], h[2]};
        }
      }

      inline rgb_t eval_at(const model_desc& m, const rgb_t& in, const rgb_t& out, unit_t unit, void* stream)
      {
        device_vector<float> v(12);
        const float h[6] = {in[0], in[1], in[2], out[0], out[1], out[2]};
        hip_check(hipMemcpy(v.data(), h, sizeof(h), hipMemcpyHostToDevice), "hipMemcpy");
        float* p = v.data();
        eval(m, soa3{p, p + 1, p + 2}, soa3{p + 3, p + 4, p + 5}, 1, soa3_out{p + 6, p + 7, p + 8}, bsdf_flag::All, unit,
             nullptr, stream);
        hip_check(hipStreamSynchronize(static_cast<hipStream_t>(stream)), "hipStreamSynchronize");
        float r[3];
        hip_check(hipMemcpy(r, p + 6, sizeof(r), hipMemcpyDeviceToHost), "hipMemcpy");
        return {r[0], r[1], r[2]};
      }

      inline symmetry_stats symmetry(const model_desc& m, int test, size_t samples, uint64_t seed, int which,
                                     const std::vector<double>& acc, void* stream)
      {
        symmetry_stats s;
        const int off = which ? 3 : 0, mx = which ? 10 : 8;
        for(int c = 0; c < 3; ++c) s.average[size_t(c)] = float(acc[size_t(off + c)] / double(samples));
        s.max_hsum = acc[size_t(mx)];
        if(samples > 0 && acc[size_t(mx)] > 0)
        {
          s.sample = int64_t(acc[size_t(mx) + 1]);
          check_pair_at(test, seed, s.sample, s.in, s.out, stream);
          // the differences at that pair, recomputed with the model (checkBsdf.cpp:131-132, :185)
          const unit_t u1 = unit_t::Radiance;
          const unit_t u2 = (test == BBM_CHECK_ADJOINT) ? unit_t::Importance : (which ? unit_t::Importance : unit_t::Radiance);
          const unit_t ua = (test == BBM_CHECK_ADJOINT) ? u1 : u2;
          const rgb_t f1 = eval_at(m, s.in, s.out, ua, stream), f2 = eval_at(m, s.out, s.in, u2, stream);
          for(size_t c = 0; c < 3; ++c) s.max[c] = std::fabs(f1[c] - f2[c]);
        }
        return s;
      }
    } // end detail namespace

    inline std::array<symmetry_stats, 2> check_reciprocity(const model_desc& m, size_t samples,
                                                           uint64_t seed = check_default_seed, void* stream = nullptr)
    {
      std::vector<double> acc;
      detail::check_run<float>(m, detail::check_desc(BBM_CHECK_RECIPROCITY, 1, seed, samples), nullptr, nullptr, nullptr,
                               &acc, nullptr, stream);
      return {detail::symmetry(m, BBM_CHECK_RECIPROCITY, samples, seed, 0, acc, stream),
              detail::symmetry(m, BBM_CHECK_RECIPROCITY, samples, seed, 1, acc, stream)};
    }

    inline symmetry_stats check_adjoint(const model_desc& m, size_t samples, uint64_t seed = check_default_seed,
                                        void* stream = nullptr)
    {
      std::vector<double> acc;
      detail::check_run<float>(m, detail::check_desc(BBM_CHECK_ADJOINT, 1, seed, samples), nullptr, nullptr, nullptr,
                               &acc, nullptr, stream);
      return detail::symmetry(m, BBM_CHECK_ADJOINT, samples, seed, 0, acc, stream);
    }

    //! \brief pdf test (checkBsdf.cpp:206-267): [0] Radiance, [1] Importance
    struct pdf_stats
    {
      std::array<size_t, 2> negative{}, below_horizon{};
      std::array<float, 2> mismatch{};        //!< average |sample.pdf - pdf(sample.direction, out)|
    };

    inline pdf_stats check_pdf(const model_desc& m, size_t samples, bool sphere = false,
                               uint64_t seed = check_default_seed, void* stream = nullptr)
    {
      auto d = detail::check_desc(BBM_CHECK_PDF, 1, seed, samples);
      d.sphere = sphere ? 1 : 0;
      std::vector<double> acc;
      detail::check_run<float>(m, d, nullptr, nullptr, nullptr, &acc, nullptr, stream);
      pdf_stats s;
      for(size_t k = 0; k < 2; ++k)
      {
        s.negative[k] = size_t(acc[k]);
        s.below_horizon[k] = size_t(acc[2 + k]);
        s.mismatch[k] = float(acc[4 + k] / double(samples));
      }
      return s;
    }

    //! \brief pdf integral test (checkBsdf.cpp:272-316): per trial direction, the MC integral of the pdf over the sphere
    struct pdfint_stats
    {
      std::vector<rgb_t> direction;
      std::vector<std::array<float, 2>> integral;      //!< (Radiance, Importance)
    };

    inline pdfint_stats check_pdf_int(const model_desc& m, size_t samples, size_t trials, bool sphere = false,
                                      uint64_t seed = check_default_seed, void* stream = nullptr)
    {
      detail::trials t(BBM_CHECK_PDFINT, seed, trials, sphere, stream);
      std::vector<double> acc;
      detail::check_run<float>(m, detail::check_desc(BBM_CHECK_PDFINT, int(trials), seed, samples), t.x.data(), t.y.data(),
                               t.z.data(), &acc, nullptr, stream);
      pdfint_stats s;
      s.direction = t.host;
      for(size_t k = 0; k < trials; ++k)
        s.integral.push_back({float(acc[k * BBM_CHECK_ACC] / double(samples)), float(acc[k * BBM_CHECK_ACC + 1] / double(samples))});
      return s;
    }

    //! \brief sample / pdf chi-square test (checkBsdf.cpp:321-418), per trial direction
    struct sample_trial
    {
      rgb_t direction{};
      double chi2 = 0;
      int df = -1;
      double P = std::numeric_limits<double>::quiet_NaN();     //!< NaN: fewer than 2 degrees of freedom
      std::vector<double> pdf;                                   //!< integrated pdf per (theta, phi) bin
      std::vector<uint64_t> count;                               //!< sampled directions per bin
    };

    inline std::vector<sample_trial> check_sample(const model_desc& m, size_t pdfSamples, size_t samples, size_t theta,
                                                  size_t phi, size_t trials, bool sphere = false,
                                                  bool includeZeroPdfSamples = false,
                                                  uint64_t seed = check_default_seed, void* stream = nullptr)
    {
      const size_t bins = theta * phi;
      detail::trials t(BBM_CHECK_SAMPLE_COUNT, seed, trials, sphere, stream);
      auto dp = detail::check_desc(BBM_CHECK_SAMPLE_PDF, int(trials * bins), seed, pdfSamples);
      dp.theta_bins = uint32_t(theta); dp.phi_bins = uint32_t(phi);
      std::vector<double> acc;
      detail::check_run<float>(m, dp, t.x.data(), t.y.data(), t.z.data(), &acc, nullptr, stream);
      auto dc = detail::check_desc(BBM_CHECK_SAMPLE_COUNT, int(trials), seed, samples);
      dc.theta_bins = uint32_t(theta); dc.phi_bins = uint32_t(phi);
      dc.include_zero_pdf = includeZeroPdfSamples ? 1 : 0;
      std::vector<uint64_t> counts;
      detail::check_run<float>(m, dc, t.x.data(), t.y.data(), t.z.data(), nullptr, &counts, stream);
      std::vector<sample_trial> out(trials);
      const double eps = double(std::numeric_limits<float>::epsilon());
      for(size_t k = 0; k < trials; ++k)
      {
        sample_trial& s = out[k];
        s.direction = t.host[k];
        for(size_t b = 0; b < bins; ++b)
        {
          s.pdf.push_back(acc[(k * bins + b) * BBM_CHECK_ACC] / double(pdfSamples));
          s.count.push_back(counts[k * bins + b]);
        }
        // checkBsdf.cpp:391-403: bins with an expected count > Epsilon and more than 5 samples
        for(size_t b = 0; b < bins; ++b)
        {
          const double e = s.pdf[b] * double(samples);
          if(e > eps && s.count[b] > 5)
          {
            s.chi2 += (double(s.count[b]) - e) * (double(s.count[b]) - e) / e;
            s.df++;
          }
        }
        if(s.df > 1) s.P = double(bbm::gamma_q(float(s.df - 1) / 2.0f, float(s.chi2) / 2.0f));
      }
      return out;
    }

  } // end hip namespace
} // end bbm namespace

#endif /* BBM_HIP_CHECK_H */
