/* backbone/hip/include/bbm_hip/fit.h -- C++20 host adapter: BBM's fitting layer on the HIP backbone.
 *
 * The reference fits a model with three pieces: a sampled loss (include/bbm/sampledlossfunction.h:
 * 34-97) -- the mean of a per-sample loss (include/loss/*.h) between the fitted model and a reference over the (in, out)
 * pairs of a linearizer --, optionally bbm::batch (include/bbm/batch.h:27-92) over a random subset of those samples,
 * and the compass search (include/optimizer/compass.h:40-183) that probes 2P parameter vectors per step.  Here:
 *
 *   bbm::hip::sampledlossfunction<BSDF, COMPONENT, UNIT>   concepts::sampledlossfunction, built like the reference's
 *       (bsdf, reference, samplelossfunc, linearizer): the linearizer's pairs of this rank's shard are materialised once
 *       in device memory, the reference model is evaluated on them once on the GPU, and every loss evaluation is one
 *       launch of the fitted model's kernels (bbm_hip_loss_pairs for a single-kernel floatRGB model, bbm_hip_loss_tree
 *       / _f64 for any composed / nested aggregate and for doubleRGB).  probe_losses() scores many parameter vectors
 *       in that one launch.  With a bbm::hip::comm the samples are sharded over the ranks (one process per GPU) and the
 *       per-probe sums are all-reduced over RCCL (bbm_hip_allreduce_sums);
 *   bbm::hip::batch<SAMPLEDLOSSFUNC>                       concepts::sampledlossfunction: the reference's batch --
 *       indices from the restated bbm::rng<Size_t> (bbm_hip_rng_*), the same for the same seed -- whose samples are
 *       gathered on the device (bbm_hip_gather_samples) and scored in one launch;
 *   bbm::hip::compass<LOSSFUNC, PARAM, BOX>                the reference's compass step with the 2P probes of a step
 *       evaluated in one batched call: the parameter updates (probe, box test, restore by the opposite update) are the
 *       reference's own float arithmetic on the same PARAM references, the sequential "strictly better" rule picks the
 *       same probe.  The reference's bbm::compass also runs unchanged on these loss types (one launch per probe).
 *
 * Every type owns its device memory (RAII); calls are synchronous with respect to the host (a loss value is a host
 * number) and run on the stream given at construction.  Errors are bbm::hip::error (std::runtime_error).
 */
#ifndef BBM_HIP_FIT_H
#define BBM_HIP_FIT_H

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <iterator>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "bbm_hip/batch.h"
#include "concepts/lossfunction.h"
#include "concepts/sampledlossfunction.h"
#include "concepts/inout_linearizer.h"
#include "loss/cosine_weighted_l2.h"
#include "loss/cosine_weighted_log.h"

namespace bbm {
  namespace hip {

    //! \brief device memory of N values of T (hipMalloc / hipFree), move-only
    template<typename T>
      class device_vector
    {
    public:
      device_vector(void) = default;
      explicit device_vector(size_t n) { resize(n); }
      device_vector(const device_vector&) = delete;
      device_vector& operator=(const device_vector&) = delete;
      device_vector(device_vector&& o) noexcept : _p(o._p), _n(o._n) { o._p = nullptr; o._n = 0; }
      ~device_vector(void) { if(_p) (void)hipFree(_p); }
      //! \brief (re)allocate for n values; contents are not kept
      void resize(size_t n)
      {
        if(n <= _n && _p) return;
        if(_p) (void)hipFree(_p);
        _p = nullptr;
        _n = 0;
        if(hipMalloc(reinterpret_cast<void**>(&_p), std::max<size_t>(n, 1) * sizeof(T)) != hipSuccess)
          throw error(BBM_HIP_ERR_HIP, "hipMalloc of " + std::to_string(n * sizeof(T)) + " bytes failed");
        _n = n;
      }
      T* data(void) { return _p; }
      const T* data(void) const { return _p; }
      size_t size(void) const { return _n; }
    private:
      T* _p = nullptr;
      size_t _n = 0;
    };

    inline void hip_check(hipError_t e, const char* what)
    {
      if(e != hipSuccess) throw error(BBM_HIP_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
    }

    /*******************************************************************/
    /*! \brief An RCCL communicator for the loss reduction (bbm_hip_comm_*): one per process, on its current device.

      Rank 0 makes the id (unique_id()) and hands its bytes to the other ranks by any means; from_env() reads them
      from BBM_HIP_COMM_ID (hex) with RANK / WORLD_SIZE (torchrun's variables).
    ********************************************************************/
    class comm
    {
    public:
      static std::vector<uint8_t> unique_id(void)
      {
        std::vector<uint8_t> id(BBM_HIP_COMM_ID_BYTES);
        check(bbm_hip_comm_unique_id(id.data(), id.size()));
        return id;
      }
      static std::string to_hex(const std::vector<uint8_t>& id)
      {
        static const char* d = "0123456789abcdef";
        std::string s;
        for(uint8_t b : id) { s += d[b >> 4]; s += d[b & 15]; }
        return s;
      }
      static std::vector<uint8_t> from_hex(const std::string& s)
      {
        if(s.size() != 2 * BBM_HIP_COMM_ID_BYTES) throw error(BBM_HIP_ERR_INVALID_ARG, "comm id: expected 256 hex digits");
        std::vector<uint8_t> id(BBM_HIP_COMM_ID_BYTES);
        for(size_t i = 0; i < id.size(); ++i) id[i] = uint8_t(std::stoi(s.substr(2 * i, 2), nullptr, 16));
        return id;
      }
      comm(const std::vector<uint8_t>& id, int rank, int world)
      {
        check(bbm_hip_comm_init(id.data(), id.size(), rank, world, &_h));
      }
      static comm from_env(void)
      {
        const char* id = std::getenv("BBM_HIP_COMM_ID");
        const char* r = std::getenv("RANK");
        const char* w = std::getenv("WORLD_SIZE");
        if(!id || !r || !w) throw error(BBM_HIP_ERR_INVALID_ARG, "BBM_HIP_COMM_ID / RANK / WORLD_SIZE not set");
        return comm(from_hex(id), std::atoi(r), std::atoi(w));
      }
      comm(const comm&) = delete;
      comm& operator=(const comm&) = delete;
      comm(comm&& o) noexcept : _h(o._h) { o._h = nullptr; }
      ~comm(void) { if(_h) (void)bbm_hip_comm_destroy(_h); }
      int rank(void) const { return bbm_hip_comm_rank(_h); }
      int size(void) const { return bbm_hip_comm_size(_h); }
      //! \brief sums[0 .. n-1] (device doubles) <- their sum over all ranks (stream-ordered)
      void allreduce(double* sums, size_t n, void* stream = nullptr) { check(bbm_hip_allreduce_sums(_h, sums, n, stream)); }
    private:
      bbm_hip_comm* _h = nullptr;
    };

    namespace detail {
      //! \brief the C-ABI loss kind of a reference sample loss type (include/loss/cosine_weighted_{l2,log}.h)
      template<typename C> constexpr loss_t loss_kind(const bbm::nganL2_error<C>*) { return loss_t::nganL2; }
      template<typename C> constexpr loss_t loss_kind(const bbm::lowL2_error<C>*) { return loss_t::lowL2; }
      template<typename C> constexpr loss_t loss_kind(const bbm::bieronL2_error<C>*) { return loss_t::bieronL2; }
      template<typename C> constexpr loss_t loss_kind(const bbm::standardLog_error<C>*) { return loss_t::standardLog; }
      template<typename C> constexpr loss_t loss_kind(const bbm::lowLog_error<C>*) { return loss_t::lowLog; }
      template<typename C> constexpr loss_t loss_kind(const bbm::bieronLog_error<C>*) { return loss_t::bieronLog; }

      //! \brief the leaves' parameter vectors of a model_desc back to back in preorder (a probe of bbm_hip_loss_tree)
      template<typename T>
        inline void flatten(const basic_model_desc<T>& d, std::vector<T>& out)
      {
        if(d.composed()) for(auto& k : d.kids) flatten(k, out);
        else out.insert(out.end(), d.params.begin(), d.params.end());
      }

      //! \brief model_desc of a template model or a bsdf_ptr, in the configuration's Value
      template<typename T, typename MODEL>
        inline basic_model_desc<T> describe_model(const MODEL& m)
      {
#ifdef _BBM_BSDF_PTR_H_
        if constexpr (requires { m.ptr(); }) { static_assert(std::is_same_v<T, float>, "bsdf_ptr: floatRGB"); return describe(m); }
        else
#endif
        return describe_as<T>(m);
      }

      //! \brief contiguous shard [begin, end) of `total` samples for `rank` of `world` (balanced, as bbm_amd.fit)
      inline std::pair<uint64_t, uint64_t> shard(uint64_t total, int rank, int world)
      {
        const uint64_t q = total / uint64_t(world), r = total % uint64_t(world), k = uint64_t(rank);
        const uint64_t b = k * q + std::min(k, r);
        return {b, b + q + (k < r ? 1 : 0)};
      }
    } // end detail namespace

    /*******************************************************************/
    /*! \brief sampledlossfunction<BSDF, REFERENCE, SAMPLELOSSFUNC, LINEARIZER, COMPONENT, UNIT> on the GPU
        (include/bbm/sampledlossfunction.h:34-97).  Satisfies concepts::sampledlossfunction.

      The fitted model is held by reference (as in the reference): a loss evaluation uses its parameters at call
      time.  The reference model and the linearizer are consumed at construction (reference values on the shard,
      materialised pairs); the per-sample loss kind comes from SAMPLELOSSFUNC's type.
    ********************************************************************/
    template<typename BSDF, bsdf_flag COMPONENT = bsdf_flag::All, unit_t UNIT = unit_t::Radiance>
      class sampledlossfunction
    {
    public:
      BBM_IMPORT_CONFIG( BSDF );
      using probe_t = std::vector<Value>;

      //! \brief from a reference model and any inout_linearizer: this rank's pairs come from the linearizer itself
      //! (its own float / double arithmetic), uploaded once
      template<typename REFERENCE, typename SAMPLELOSSFUNC, typename LINEARIZER> requires concepts::inout_linearizer<LINEARIZER>
        sampledlossfunction(const BSDF& bsdf, const REFERENCE& reference, const SAMPLELOSSFUNC&, const LINEARIZER& lin,
                            comm* c = nullptr, void* stream = nullptr)
        : _bsdf(bsdf), _s(std::make_shared<state>())
      {
        init(lin.size(), detail::loss_kind(static_cast<const SAMPLELOSSFUNC*>(nullptr)), c, stream);
        std::vector<Value> h[6];
        for(auto& v : h) v.resize(_s->n);
        for(size_t i = 0; i < _s->n; ++i)
        {
          const auto p = lin(Size_t(_s->begin + i));
          for(int k = 0; k < 3; ++k) { h[k][i] = Value(p.in[k]); h[3 + k][i] = Value(p.out[k]); }
        }
        for(int k = 0; k < 6; ++k)
          hip_check(hipMemcpy(_s->dirs[k].data(), h[k].data(), _s->n * sizeof(Value), hipMemcpyHostToDevice), "hipMemcpy");
        reference_table(reference);
      }

      //! \brief from the C-ABI linearizer descriptor (spherical / MERL grid generated on the device, floatRGB)
      template<typename REFERENCE, typename SAMPLELOSSFUNC>
        sampledlossfunction(const BSDF& bsdf, const REFERENCE& reference, const SAMPLELOSSFUNC&, const bbm_hip_linearizer& lin,
                            comm* c = nullptr, void* stream = nullptr)
        : _bsdf(bsdf), _s(std::make_shared<state>())
      {
        static_assert(std::is_same_v<Value, float>, "the device linearizer writes float directions (floatRGB)");
        uint64_t total = 0;
        check(bbm_hip_linearizer_size(&lin, &total));
        init(total, detail::loss_kind(static_cast<const SAMPLELOSSFUNC*>(nullptr)), c, stream);
        if(_s->n)
          check(bbm_hip_linearize(&lin, _s->begin, _s->n, _s->dirs[0].data(), _s->dirs[1].data(), _s->dirs[2].data(),
                                  _s->dirs[3].data(), _s->dirs[4].data(), _s->dirs[5].data(), _s->stream));
        reference_table(reference);
      }

      //! \brief sampledlossfunction::update(): nothing to refresh
      void update(void) {}

      //! \brief number of samples of the whole loss (all ranks)
      Size_t samples(void) const { return Size_t(_s->total); }

      //! \brief the loss of sample idx alone at the fitted model's current parameters (0 past the last sample)
      Value operator()(Size_t idx, Mask mask = true) const
      {
        if(!mask || idx >= samples()) return 0;
        const std::vector<uint64_t> one(1, uint64_t(idx));
        return Value(probe_sums({current_probe()}, &one)[0]);
      }

      //! \brief the loss over all samples: the mean of the per-sample losses (sampledlossfunction.h:78-87)
      Value operator()(Mask mask = true) const
      {
        if(!mask) return 0;
        return probe_losses({current_probe()})[0];
      }

      //! \brief the fitted model's current parameters as a probe (its leaves' parameter vectors back to back)
      probe_t current_probe(void) const
      {
        probe_t p;
        detail::flatten(detail::describe_model<Value>(_bsdf), p);
        return p;
      }

      //! \brief per-probe loss sums over all samples (or over the samples `subset` lists, global indices; an index
      //! past the last sample adds 0), all probes in one launch, reduced over the ranks
      std::vector<double> probe_sums(const std::vector<probe_t>& probes, const std::vector<uint64_t>* subset = nullptr) const
      {
        state& s = *_s;
        const size_t P = probes.size();
        if(P == 0) return {};
        const Value* dirs[6];
        const Value* ref[3];
        size_t n = s.n;
        for(int k = 0; k < 6; ++k) dirs[k] = s.dirs[k].data();
        for(int k = 0; k < 3; ++k) ref[k] = s.ref[k].data();
        if(subset)
        {
          // this rank's samples among the subset, gathered densely (draw order)
          std::vector<uint64_t> mine;
          for(uint64_t i : *subset) if(i >= s.begin && i < s.begin + s.n) mine.push_back(i - s.begin);
          for(auto& g : s.gathered) g.resize(std::max<size_t>(mine.size(), 1));
          const Value* src[9];
          Value* dst[9];
          for(int k = 0; k < 9; ++k) { src[k] = (k < 6) ? s.dirs[k].data() : s.ref[k - 6].data(); dst[k] = s.gathered[k].data(); }
          int got = 0;
          if constexpr (std::is_same_v<Value, float>) got = bbm_hip_gather_samples(mine.data(), mine.size(), s.n, src, dst, 9, s.stream);
          else got = bbm_hip_gather_samples_f64(mine.data(), mine.size(), s.n, src, dst, 9, s.stream);
          check(got);
          n = size_t(got);
          for(int k = 0; k < 6; ++k) dirs[k] = s.gathered[k].data();
          for(int k = 0; k < 3; ++k) ref[k] = s.gathered[6 + k].data();
        }
        s.sums.resize(P);
        if(n == 0) hip_check(hipMemsetAsync(s.sums.data(), 0, P * sizeof(double), static_cast<hipStream_t>(s.stream)), "hipMemsetAsync");
        else if(s.fused)
        {
          if constexpr (std::is_same_v<Value, float>)
          {
            std::vector<float> flat;
            for(auto& p : probes) flat.insert(flat.end(), p.begin(), p.end());
            const int np = int(probes[0].size());
            s.probes.resize(flat.size());
            hip_check(hipMemcpyAsync(s.probes.data(), flat.data(), flat.size() * sizeof(float), hipMemcpyHostToDevice,
                                     static_cast<hipStream_t>(s.stream)), "hipMemcpyAsync");
            const size_t wsb = bbm_hip_loss_workspace_size(int(P));
            s.workspace.resize(wsb);
            check(bbm_hip_loss_pairs(s.desc.id, s.probes.data(), np, int(P), n, dirs[0], dirs[1], dirs[2], dirs[3], dirs[4],
                                     dirs[5], ref[0], ref[1], ref[2], int(s.kind), uint32_t(COMPONENT), uint32_t(UNIT),
                                     s.sums.data(), s.workspace.data(), wsb, s.stream));
            hip_check(hipStreamSynchronize(static_cast<hipStream_t>(s.stream)), "hipStreamSynchronize");  // `flat` staged
          }
        }
        else
        {
          std::vector<Value> flat;
          for(auto& p : probes) flat.insert(flat.end(), p.begin(), p.end());
          const int np = int(probes[0].size());
          // a composed aggregate: its child arrays; any other model: one leaf node (include/bbm_hip.h)
          const detail::child_tree<Value> tree(s.desc);
          using child_t = typename detail::child_of<Value>::type;
          const child_t leaf{s.desc.id, s.desc.params.data(), int(s.desc.params.size()), nullptr, 0};
          const child_t* root = s.desc.composed() ? tree.root : &leaf;
          const int count = s.desc.composed() ? tree.count : 1;
          const size_t wsb = bbm_hip_loss_tree_workspace_size(int(P), n);
          s.workspace.resize(wsb);
          if constexpr (std::is_same_v<Value, float>)
            check(bbm_hip_loss_tree(root, count, flat.data(), np, int(P), n, dirs[0], dirs[1], dirs[2], dirs[3],
                                    dirs[4], dirs[5], ref[0], ref[1], ref[2], int(s.kind), uint32_t(COMPONENT),
                                    uint32_t(UNIT), s.sums.data(), s.workspace.data(), wsb, s.stream));
          else
            check(bbm_hip_loss_tree_f64(root, count, flat.data(), np, int(P), n, dirs[0], dirs[1], dirs[2],
                                        dirs[3], dirs[4], dirs[5], ref[0], ref[1], ref[2], int(s.kind), uint32_t(COMPONENT),
                                        uint32_t(UNIT), s.sums.data(), s.workspace.data(), wsb, s.stream));
        }
        if(s.cm) s.cm->allreduce(s.sums.data(), P, s.stream);
        std::vector<double> out(P);
        hip_check(hipMemcpyAsync(out.data(), s.sums.data(), P * sizeof(double), hipMemcpyDeviceToHost,
                                 static_cast<hipStream_t>(s.stream)), "hipMemcpyAsync");
        hip_check(hipStreamSynchronize(static_cast<hipStream_t>(s.stream)), "hipStreamSynchronize");
        return out;
      }

      //! \brief per-probe mean loss over all samples, as Value (err / numsamples, sampledlossfunction.h:86)
      std::vector<Value> probe_losses(const std::vector<probe_t>& probes) const
      {
        std::vector<double> s = probe_sums(probes);
        std::vector<Value> out(s.size());
        for(size_t k = 0; k < s.size(); ++k) out[k] = Value(s[k] / double(_s->total));
        return out;
      }

      //! \brief this rank's shard [begin, begin + n) of the samples
      std::pair<uint64_t, uint64_t> shard(void) const { return {_s->begin, _s->begin + _s->n}; }

    private:
      struct state
      {
        uint64_t total = 0, begin = 0;
        size_t n = 0;
        loss_t kind = loss_t::standardLog;
        comm* cm = nullptr;
        void* stream = nullptr;
        basic_model_desc<Value> desc;
        bool fused = false;
        device_vector<Value> dirs[6], ref[3], gathered[9];
        device_vector<double> sums;
        device_vector<float> probes;
        device_vector<char> workspace;
      };

      void init(uint64_t total, loss_t kind, comm* c, void* stream)
      {
        state& s = *_s;
        s.total = total;
        s.kind = kind;
        s.cm = c;
        s.stream = stream;
        const auto sh = c ? detail::shard(total, c->rank(), c->size()) : std::pair<uint64_t, uint64_t>{0, total};
        s.begin = sh.first;
        s.n = size_t(sh.second - sh.first);
        for(auto& d : s.dirs) d.resize(s.n);
        for(auto& r : s.ref) r.resize(s.n);
        s.desc = detail::describe_model<Value>(_bsdf);
        // one fused multi-probe kernel for a single-kernel floatRGB model; the materialised tree path otherwise
        s.fused = std::is_same_v<Value, float> && !s.desc.composed() && s.desc.id >= 0;
      }

      template<typename REFERENCE>
        void reference_table(const REFERENCE& reference)
      {
        state& s = *_s;
        if(s.n == 0) return;
        const auto rd = detail::describe_model<Value>(reference);
        if constexpr (std::is_same_v<Value, float>)
          eval(rd, soa3{s.dirs[0].data(), s.dirs[1].data(), s.dirs[2].data()},
               soa3{s.dirs[3].data(), s.dirs[4].data(), s.dirs[5].data()}, s.n,
               soa3_out{s.ref[0].data(), s.ref[1].data(), s.ref[2].data()}, bsdf_flag(COMPONENT), UNIT, nullptr, s.stream);
        else
        {
          device_vector<double> pdf(s.n);
          eval_pdf(rd, soa3d{s.dirs[0].data(), s.dirs[1].data(), s.dirs[2].data()},
                   soa3d{s.dirs[3].data(), s.dirs[4].data(), s.dirs[5].data()}, s.n,
                   soa3d_out{s.ref[0].data(), s.ref[1].data(), s.ref[2].data()}, pdf.data(), bsdf_flag(COMPONENT), UNIT,
                   nullptr, s.stream);
          hip_check(hipStreamSynchronize(static_cast<hipStream_t>(s.stream)), "hipStreamSynchronize");
        }
        hip_check(hipStreamSynchronize(static_cast<hipStream_t>(s.stream)), "hipStreamSynchronize");
      }

      const BSDF& _bsdf;
      std::shared_ptr<state> _s;      // shared by copies (bbm::batch copies its sampled loss, batch.h:40, :91)
    };

    /*******************************************************************/
    /*! \brief bbm::batch<SAMPLEDLOSSFUNC> (include/bbm/batch.h:27-92) over a GPU sampled loss.  Satisfies
        concepts::sampledlossfunction.

      Indices: bbm::rng<Size_t>(seed, 0, samples()) restated (bbm_hip_rng_*), drawn in the constructor and by every
      update() -- the reference's indices for the same seed.  operator()(idx) is batch.h:64-70; operator()(mask) is the
      mean over the batch, which batch.h:75-82 was written to compute (its loop index is never initialised, `for(size_t
      i; ...)`, so the reference's own value is undefined).
    ********************************************************************/
    template<typename SAMPLEDLOSSFUNC>
      class batch
    {
    public:
      BBM_IMPORT_CONFIG( SAMPLEDLOSSFUNC );
      using probe_t = typename SAMPLEDLOSSFUNC::probe_t;

      batch(size_t batchsize, const SAMPLEDLOSSFUNC& sampledlossfunc, seed_t seed = default_seed)
        : _sampledlossfunc(sampledlossfunc), _index(batchsize)
      {
        check(bbm_hip_rng_init(&_rng, uint64_t(seed), 0, uint64_t(sampledlossfunc.samples())));
        update();
      }

      //! \brief the wrapped loss's update(), then batchsize fresh indices (batch.h:48-54)
      void update(void)
      {
        _sampledlossfunc.update();
        check(bbm_hip_rng_draw(&_rng, _index.data(), _index.size()));
      }

      Size_t samples(void) const { return Size_t(_index.size()); }

      //! \brief the loss of the idx-th drawn sample
      Value operator()(Size_t idx, Mask mask = true) const
      {
        if(!mask || idx >= samples()) return 0;
        return _sampledlossfunc(Size_t(_index[idx]), mask);
      }

      //! \brief the mean loss over the batch at the fitted model's current parameters
      Value operator()(Mask mask = true) const
      {
        if(!mask) return 0;
        return probe_losses({current_probe()})[0];
      }

      probe_t current_probe(void) const { return _sampledlossfunc.current_probe(); }

      //! \brief per-probe loss sums over the batch (all probes in one launch, all ranks)
      std::vector<double> probe_sums(const std::vector<probe_t>& probes) const { return _sampledlossfunc.probe_sums(probes, &_index); }

      std::vector<Value> probe_losses(const std::vector<probe_t>& probes) const
      {
        std::vector<double> s = probe_sums(probes);
        std::vector<Value> out(s.size());
        for(size_t k = 0; k < s.size(); ++k) out[k] = Value(s[k] / double(_index.size()));
        return out;
      }

      //! \brief the indices drawn by the last update()
      const std::vector<uint64_t>& index(void) const { return _index; }

    private:
      SAMPLEDLOSSFUNC _sampledlossfunc;
      std::vector<uint64_t> _index;
      bbm_hip_rng _rng;
    };

    /*******************************************************************/
    /*! \brief compass<LOSSFUNC, PARAM, BOX> (include/optimizer/compass.h:40-183) with the probes of a step scored in
        one batched call (LOSSFUNC: a bbm::hip loss with current_probe() / probe_losses()).

      Same constructor, state and semantics as the reference: per step update() the loss, move PARAM by +-step along
      each cardinal direction (the reference's Value arithmetic, restored by the opposite move, compass.h:88-93,
      :128), test the box, keep the first strictly better in-box probe, then expand or contract the step.
    ********************************************************************/
    template<typename LOSSFUNC, typename PARAM, typename BOX = PARAM>
      class compass
    {
    public:
      BBM_IMPORT_CONFIG( LOSSFUNC );

      compass(LOSSFUNC& lossfunc, PARAM& param, const BOX& lower = BOX(), const BOX& upper = BOX(),
              Scalar tolerance = Constants::Epsilon(), Scalar stepSize = 1.0, Scalar contraction = 0.5,
              Scalar expansion = 1.0, Mask mask = true)
        : _lossfunc(lossfunc), _param(param), _lower(lower), _upper(upper), _initialStep(stepSize),
          _tolerance(tolerance), _contraction(contraction), _expansion(expansion), _mask(mask)
      {
        for(Scalar i = 1; i <= std::size(param); ++i)
        {
          _directions.push_back(+i);
          _directions.push_back(-i);
        }
        reset();
      }

      Value step(void)
      {
        if(!_mask || is_converged()) return 0;
        _lossfunc.update();
        // the 2P probes: each the PARAM references moved along one cardinal direction, then moved back
        std::vector<typename LOSSFUNC::probe_t> probes;
        std::vector<size_t> which;
        for(size_t k = 0; k < _directions.size(); ++k)
        {
          move(_directions[k]);
          if(in_box()) { probes.push_back(_lossfunc.current_probe()); which.push_back(k); }
          move(-_directions[k]);
        }
        std::vector<Value> err = probes.empty() ? std::vector<Value>() : _lossfunc.probe_losses(probes);
        // the first strictly better in-box probe, in cardinal order (compass.h:124-126)
        Value best = 0, loss = _lossValue;
        for(size_t j = 0; j < which.size(); ++j)
          if(err[j] < loss) { best = _directions[which[j]]; loss = err[j]; }
        const bool optimize = loss < _lossValue;
        if(optimize) move(best);
        _step = optimize ? Value(_expansion * _step) : Value(_contraction * _step);
        if(optimize) _lossValue = loss;
        return _lossValue;
      }

      //! \brief compass.h:145-153
      void reset(void)
      {
        _step = _initialStep;
        _lossfunc.update();
        _lossValue = _lossfunc(_mask);
      }

      Mask is_converged(void) const { return (_step < _tolerance) || (_mask == false); }

      Value loss(void) const { return _lossValue; }

    private:
      //! \brief PARAM[|cardinal| - 1] += (cardinal < 0 ? -step : step), in Value arithmetic (compass.h:88-93)
      void move(Value cardinal)
      {
        if(cardinal == 0) return;
        const size_t index = size_t(std::abs(cardinal) - 1);
        Value value = bbm::lookup<Value>(_param, index) + ((cardinal < 0) ? -_step : _step);
        bbm::set(_param, index, value);
      }

      bool in_box(void) const
      {
        if(!(_lower != BOX()) && !(_upper != BOX())) return true;     // no box (compass.h:114)
        const size_t n = std::size(_param);
        for(size_t i = 0; i < n; ++i)
        {
          const Value v = bbm::lookup<Value>(_param, i);
          if(!((v >= Value(bbm::lookup<Value>(_lower, i))) && (v <= Value(bbm::lookup<Value>(_upper, i))))) return false;
        }
        return true;
      }

      LOSSFUNC& _lossfunc;
      PARAM& _param;
      BOX _lower, _upper;
      Value _step;
      Value _lossValue;
      std::vector<Scalar> _directions;
      Scalar _initialStep;
      Scalar _tolerance;
      Scalar _contraction;
      Scalar _expansion;
      Mask _mask;
    };

  } // end hip namespace
} // end bbm namespace

#endif /* BBM_HIP_FIT_H */
