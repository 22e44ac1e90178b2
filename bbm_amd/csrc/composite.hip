// bbm_amd/csrc/composite.hip -- aggregatemodel<MODELS...> of ANY models (include/bsdfmodel/aggregatemodel.h:22-222),
// evaluated by composing the children's own kernels, in floatRGB and doubleRGB.
//
// The fused Aggregate<Lambertian, X> entries of the registry (aggregate.hpp) evaluate the published fits' form in
// one kernel; this unit covers every other composition -- any number of children, any registered single models,
// fused aggregates or further composed aggregates (aggregatemodel_base takes any bsdfmodel child, :22) as children
// -- at the price of one pass per child over the batch:
//   eval        = MODELS::eval(...) + ...   a right fold: e0 + (e1 + (e2 + ...))                    (:61-64)
//   pdf         = inner_product(pdfs, weights, 0) / accumulate(weights, 0), 0 unless sum > eps,
//                 weight_k = hsum(reflectance_k(out)) = ((0 + r) + g) + b                           (:129-150)
//   sample      = child k chosen where xi0 * sum falls in [0, w_k] after subtracting w_0..w_{k-1} (a later
//                 child claiming the lane wins), sampled with xi0' = that offset / w_k (0 unless w_k > eps);
//                 pdf as above at the sampled direction                                              (:81-121)
//   reflectance = MODELS::reflectance(...) + ...  (right fold)                                       (:165-172)
// A nested aggregate child is evaluated by the same functions, recursively, so each level keeps the reference's
// own order: the outer eval is inner_eval + (next + ...), the outer pdf mixes the inner aggregate's mixture pdf
// with the inner aggregate's reflectance as its weight, and the outer sample hands the chosen inner aggregate the
// rescaled xi0 (its own child selection then runs on that).  Each leaf runs through the public entry points (its
// registry kernel, its own host-side preparation such as the He family's CDF); the small kernels below only combine
// per-lane results in the reference's order and rounding (float or double: Value of the configuration).  Scratch
// is stream-ordered (scratch_acquire / scratch_release): no host synchronisation.
//
// A BBM_HIP_AGGREGATE_BSDF node is the reference's runtime aggregatebsdf (include/bbm/aggregatebsdf.h:40-190, what
// fromString<bsdf_ptr> builds): eval / reflectance as left folds from 0 ((0 + e0) + e1) + ..., pdf as the sum of
// w_k pdf_k / sum term by term (masked sum > eps), sample masked by sum > eps before the same child selection.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/bbm_hip.h"
#include "math.hpp"
#include "kernels.hpp"     // ParamBlock, k_loss_final, k_check_final, check.hpp (checkBsdf's per-sample terms)

namespace bbmhip {

namespace {

constexpr int kB = 256;
constexpr int kMaxDepth = 16;

unsigned grid(size_t n)
{
  const size_t b = (n + kB - 1) / kB;
  return unsigned(b < 1 ? 1 : (b > (1u << 20) ? (1u << 20) : b));
}

#define BBM_GRID_LOOP(i, n) \
  for (uint64_t i = uint64_t(blockIdx.x) * kB + threadIdx.x; i < (n); i += uint64_t(gridDim.x) * kB)

// Constants::Epsilon() of the configuration's Value (include/core/constants.h)
template<class T> __device__ __forceinline__ T eps_of();
template<> __device__ __forceinline__ float eps_of<float>() { return kEpsF; }
template<> __device__ __forceinline__ double eps_of<double>() { return 2.220446049250313e-16; }

// acc = t + acc (the fold's next term on the left)
template<class T>
__global__ __launch_bounds__(kB) void k_fold3(const T* tr, const T* tg, const T* tb, T* r, T* g, T* b, uint64_t n)
{
  math_tables_init();
  BBM_GRID_LOOP(i, n) { r[i] = tr[i] + r[i]; g[i] = tg[i] + g[i]; b[i] = tb[i] + b[i]; }
}

// aggregatebsdf's left fold (aggregatebsdf.h:79-83, :209-212): acc = (first ? 0 + acc : acc) + t, forward
template<class T>
__global__ __launch_bounds__(kB) void k_lfold3(const T* tr, const T* tg, const T* tb, T* r, T* g, T* b, uint64_t n,
                                               int first)
{
  math_tables_init();
  BBM_GRID_LOOP(i, n)
  {
    // the accumulation starts from Spectrum(0): 0 + e0 first (-0 becomes +0), then + e_k
    r[i] = (first ? T(0) + r[i] : r[i]) + tr[i];
    g[i] = (first ? T(0) + g[i] : g[i]) + tg[i];
    b[i] = (first ? T(0) + b[i] : b[i]) + tb[i];
  }
}

// aggregatebsdf::pdf (aggregatebsdf.h:173-187): pdf = 0; pdf += w_k pdf_k / sum, the lanes with sum <= eps masked
template<class T>
__global__ __launch_bounds__(kB) void k_inner_bsdf(const T* p, const T* w, const T* sum, T* ip, uint64_t n, int first)
{
  math_tables_init();
  BBM_GRID_LOOP(i, n) ip[i] = (first ? T(0) : ip[i]) + (w[i] * p[i]) / sum[i];
}

template<class T>
__global__ __launch_bounds__(kB) void k_mask_sum(const T* ip, const T* sum, T* pdf, uint64_t n)
{
  math_tables_init();
  BBM_GRID_LOOP(i, n) pdf[i] = (sum[i] > eps_of<T>()) ? ip[i] : T(0);
}

// w_k = hsum(reflectance_k) and sum = sum + w_k (forward, from 0)
template<class T>
__global__ __launch_bounds__(kB) void k_weight(const T* r, const T* g, const T* b, T* w, T* sum, uint64_t n, int first)
{
  math_tables_init();
  BBM_GRID_LOOP(i, n)
  {
    const T wk = ((T(0) + r[i]) + g[i]) + b[i];
    w[i] = wk;
    sum[i] = (first ? T(0) : sum[i]) + wk;
  }
}

// ip = ip + p_k w_k (forward, from 0)
template<class T>
__global__ __launch_bounds__(kB) void k_inner(const T* p, const T* w, T* ip, uint64_t n, int first)
{
  math_tables_init();
  BBM_GRID_LOOP(i, n) ip[i] = (first ? T(0) : ip[i]) + p[i] * w[i];
}

// pdf = select(sum > eps, ip / sum, 0) -- the IEEE division of Value operands
template<class T>
__global__ __launch_bounds__(kB) void k_mix(const T* ip, const T* sum, T* pdf, uint64_t n)
{
  math_tables_init();
  BBM_GRID_LOOP(i, n) pdf[i] = (sum[i] > eps_of<T>()) ? ip[i] / sum[i] : T(0);
}

// child selection of aggregatemodel::sample (:92-113): chosen = the last child claiming the lane (-1: none),
// xs = its rescaled xi0
template<class T>
__global__ __launch_bounds__(kB) void k_select(const T* w, int nchild, const T* sum, const T* xi0, const uint8_t* mask,
                                               int8_t* chosen, T* xs, uint64_t n, int bsdf)
{
  math_tables_init();
  BBM_GRID_LOOP(i, n)
  {
    // aggregatebsdf: mask &= (sum > eps) before the selection (aggregatebsdf.h:115)
    const bool m0 = (mask ? (mask[i] != 0) : true) && (!bsdf || sum[i] > eps_of<T>());
    T x = xi0[i] * sum[i];
    int c = -1;
    T nx = T(0);
    for (int k = 0; k < nchild; ++k)
    {
      const T wk = w[size_t(k) * n + i];
      const bool m = m0 && (x >= 0) && (x <= wk);
      if (m) { c = k; nx = (wk > eps_of<T>()) ? x / wk : T(0); }
      x -= wk;
    }
    chosen[i] = int8_t(c);
    xs[i] = nx;
  }
}

__global__ __launch_bounds__(kB) void k_child_mask(const int8_t* chosen, int k, uint8_t* m, uint64_t n)
{
  math_tables_init();
  BBM_GRID_LOOP(i, n) m[i] = (chosen[i] == k) ? 1 : 0;
}

template<class T>
__global__ __launch_bounds__(kB) void k_zero_sample(T* x, T* y, T* z, uint32_t* flag, uint64_t n)
{
  math_tables_init();
  BBM_GRID_LOOP(i, n) { x[i] = T(0); y[i] = T(0); z[i] = T(0); flag[i] = kFlagNone; }
}

template<class T>
__global__ __launch_bounds__(kB) void k_take(const int8_t* chosen, int k, const T* tx, const T* ty, const T* tz,
                                             const uint32_t* tf, T* x, T* y, T* z, uint32_t* flag, uint64_t n)
{
  math_tables_init();
  BBM_GRID_LOOP(i, n)
    if (chosen[i] == k) { x[i] = tx[i]; y[i] = ty[i]; z[i] = tz[i]; flag[i] = tf[i]; }
}

// stream-ordered scratch, released on the same stream when the call returns
struct Scratch
{
  hipStream_t s;
  std::vector<void*> ptrs;
  explicit Scratch(hipStream_t st) : s(st) {}
  ~Scratch() { for (void* p : ptrs) scratch_release(p, s); }
  template<class T> T* get(size_t count)
  {
    void* p = scratch_acquire((count ? count : 1) * sizeof(T), s);
    if (p) ptrs.push_back(p);
    return static_cast<T*>(p);
  }
};

int launched()
{
  const hipError_t e = hipGetLastError();
  return (e == hipSuccess) ? BBM_HIP_OK : fail(BBM_HIP_ERR_HIP, std::string("kernel launch failed: ") + hipGetErrorString(e));
}

// ------------------------------------------------------------------ leaves: the single-model entry points
template<class T> struct Leaf;

template<> struct Leaf<float>
{
  using Child = bbm_hip_child;
  static int eval(const Child& c, const float* ix, const float* iy, const float* iz, const float* ox, const float* oy,
                  const float* oz, const uint8_t* mask, size_t n, uint32_t comp, uint32_t unit, float* r, float* g,
                  float* b, hipStream_t s)
  {
    return bbm_hip_eval(c.model_id, c.params, c.nparams, ix, iy, iz, ox, oy, oz, mask, n, comp, unit, r, g, b, s);
  }
  static int pdf(const Child& c, const float* ix, const float* iy, const float* iz, const float* ox, const float* oy,
                 const float* oz, const uint8_t* mask, size_t n, uint32_t comp, uint32_t unit, float* p, hipStream_t s)
  {
    return bbm_hip_pdf(c.model_id, c.params, c.nparams, ix, iy, iz, ox, oy, oz, mask, n, comp, unit, p, s);
  }
  static int reflectance(const Child& c, const float* ox, const float* oy, const float* oz, const uint8_t* mask,
                         size_t n, uint32_t comp, uint32_t unit, float* r, float* g, float* b, hipStream_t s)
  {
    return bbm_hip_reflectance(c.model_id, c.params, c.nparams, ox, oy, oz, mask, n, comp, unit, r, g, b, s);
  }
  static int sample(const Child& c, const float* ox, const float* oy, const float* oz, const float* xi0,
                    const float* xi1, const uint8_t* mask, size_t n, uint32_t comp, uint32_t unit, float* dx,
                    float* dy, float* dz, float* p, uint32_t* f, hipStream_t s)
  {
    return bbm_hip_sample(c.model_id, c.params, c.nparams, ox, oy, oz, xi0, xi1, mask, n, comp, unit, dx, dy, dz, p, f, s);
  }
  static int eval_pdf(const Child& c, const float* ix, const float* iy, const float* iz, const float* ox, const float* oy,
                      const float* oz, const uint8_t* mask, size_t n, uint32_t comp, uint32_t unit, float* r, float* g,
                      float* b, float* p, hipStream_t s)
  {
    return bbm_hip_eval_pdf(c.model_id, c.params, c.nparams, ix, iy, iz, ox, oy, oz, mask, n, comp, unit, r, g, b, p, s);
  }
  static int nparams(int id) { return bbm_hip_model_nparams(id); }
  static bool supported(int) { return true; }
};

// doubleRGB: the f64 entry point evaluates eval and pdf together; the output a caller did not ask for goes to scratch
template<> struct Leaf<double>
{
  using Child = bbm_hip_child_f64;
  static int eval(const Child& c, const double* ix, const double* iy, const double* iz, const double* ox,
                  const double* oy, const double* oz, const uint8_t* mask, size_t n, uint32_t comp, uint32_t unit,
                  double* r, double* g, double* b, hipStream_t s)
  {
    Scratch sc(s);
    double* p = sc.get<double>(n);
    if (!p) return fail(BBM_HIP_ERR_HIP, "aggregate: scratch allocation failed: " + scratch_failure());
    return bbm_hip_eval_pdf_f64(c.model_id, c.params, c.nparams, ix, iy, iz, ox, oy, oz, mask, n, comp, unit, r, g, b,
                                p, s);
  }
  static int pdf(const Child& c, const double* ix, const double* iy, const double* iz, const double* ox,
                 const double* oy, const double* oz, const uint8_t* mask, size_t n, uint32_t comp, uint32_t unit,
                 double* p, hipStream_t s)
  {
    Scratch sc(s);
    double* r = sc.get<double>(n);
    double* g = sc.get<double>(n);
    double* b = sc.get<double>(n);
    if (!r || !g || !b) return fail(BBM_HIP_ERR_HIP, "aggregate: scratch allocation failed: " + scratch_failure());
    return bbm_hip_eval_pdf_f64(c.model_id, c.params, c.nparams, ix, iy, iz, ox, oy, oz, mask, n, comp, unit, r, g, b,
                                p, s);
  }
  static int reflectance(const Child& c, const double* ox, const double* oy, const double* oz, const uint8_t* mask,
                         size_t n, uint32_t comp, uint32_t unit, double* r, double* g, double* b, hipStream_t s)
  {
    return bbm_hip_reflectance_f64(c.model_id, c.params, c.nparams, ox, oy, oz, mask, n, comp, unit, r, g, b, s);
  }
  static int sample(const Child& c, const double* ox, const double* oy, const double* oz, const double* xi0,
                    const double* xi1, const uint8_t* mask, size_t n, uint32_t comp, uint32_t unit, double* dx,
                    double* dy, double* dz, double* p, uint32_t* f, hipStream_t s)
  {
    return bbm_hip_sample_f64(c.model_id, c.params, c.nparams, ox, oy, oz, xi0, xi1, mask, n, comp, unit, dx, dy, dz, p,
                              f, s);
  }
  static int eval_pdf(const Child& c, const double* ix, const double* iy, const double* iz, const double* ox,
                      const double* oy, const double* oz, const uint8_t* mask, size_t n, uint32_t comp, uint32_t unit,
                      double* r, double* g, double* b, double* p, hipStream_t s)
  {
    return bbm_hip_eval_pdf_f64(c.model_id, c.params, c.nparams, ix, iy, iz, ox, oy, oz, mask, n, comp, unit, r, g, b,
                                p, s);
  }
  static int nparams(int id) { return bbm_hip_model_nparams(id); }
  static bool supported(int id) { return bbm_hip_model_has_f64(id) == 1; }
};

// ------------------------------------------------------------------ the composition, recursive in the children
template<class T>
struct Composite
{
  using L = Leaf<T>;
  using Child = typename L::Child;

  static bool is_agg(int id) { return id == BBM_HIP_AGGREGATE || id == BBM_HIP_AGGREGATE_BSDF; }

  // the top level: `children` of an aggregatemodel, or (nchild = 1) the root node itself
  static void root(const Child*& c, int& nchild, bool& bsdf)
  {
    bsdf = false;
    if (c && nchild == 1 && is_agg(c[0].model_id))
    {
      bsdf = c[0].model_id == BBM_HIP_AGGREGATE_BSDF;
      nchild = c[0].nchildren;
      c = c[0].children;
    }
  }

  static int check(const Child* c, int nchild, int depth = 0)
  {
    if (depth > kMaxDepth) return fail(BBM_HIP_ERR_INVALID_ARG, "aggregates nested deeper than 16 levels");
    if (!c || nchild < 2) return fail(BBM_HIP_ERR_INVALID_ARG, "an aggregate needs at least two children");
    if (nchild > 127) return fail(BBM_HIP_ERR_INVALID_ARG, "at most 127 children");
    for (int k = 0; k < nchild; ++k)
    {
      if (is_agg(c[k].model_id))
      {
        const int rc = check(c[k].children, c[k].nchildren, depth + 1);
        if (rc) return rc;
        continue;
      }
      const int np = L::nparams(c[k].model_id);
      if (np < 0) return np;
      if (c[k].nparams != np || (np > 0 && !c[k].params))
        return fail(BBM_HIP_ERR_INVALID_ARG, "child " + std::to_string(k) + ": expected " + std::to_string(np) + " parameters");
      if (!L::supported(c[k].model_id))
        return fail(BBM_HIP_ERR_UNSUPPORTED, std::string(bbm_hip_model_name(c[k].model_id)) + ": no doubleRGB kernel");
    }
    return BBM_HIP_OK;
  }

  // --- one child, leaf or nested aggregate (of either kind)
  static int child_eval(const Child& c, const T* ix, const T* iy, const T* iz, const T* ox, const T* oy, const T* oz,
                        const uint8_t* mask, size_t n, uint32_t comp, uint32_t unit, T* r, T* g, T* b, hipStream_t s)
  {
    if (is_agg(c.model_id))
      return eval_pdf(c.children, c.nchildren, c.model_id == BBM_HIP_AGGREGATE_BSDF, ix, iy, iz, ox, oy, oz, mask, n,
                      comp, unit, r, g, b, nullptr, s);
    return L::eval(c, ix, iy, iz, ox, oy, oz, mask, n, comp, unit, r, g, b, s);
  }
  static int child_pdf(const Child& c, const T* ix, const T* iy, const T* iz, const T* ox, const T* oy, const T* oz,
                       const uint8_t* mask, size_t n, uint32_t comp, uint32_t unit, T* p, hipStream_t s)
  {
    if (is_agg(c.model_id))
      return eval_pdf(c.children, c.nchildren, c.model_id == BBM_HIP_AGGREGATE_BSDF, ix, iy, iz, ox, oy, oz, mask, n,
                      comp, unit, nullptr, nullptr, nullptr, p, s);
    return L::pdf(c, ix, iy, iz, ox, oy, oz, mask, n, comp, unit, p, s);
  }
  static int child_reflectance(const Child& c, const T* ox, const T* oy, const T* oz, const uint8_t* mask, size_t n,
                               uint32_t comp, uint32_t unit, T* r, T* g, T* b, hipStream_t s)
  {
    if (is_agg(c.model_id))
      return reflectance(c.children, c.nchildren, c.model_id == BBM_HIP_AGGREGATE_BSDF, ox, oy, oz, mask, n, comp, unit,
                         r, g, b, s);
    return L::reflectance(c, ox, oy, oz, mask, n, comp, unit, r, g, b, s);
  }
  static int child_sample(const Child& c, const T* ox, const T* oy, const T* oz, const T* xi0, const T* xi1,
                          const uint8_t* mask, size_t n, uint32_t comp, uint32_t unit, T* dx, T* dy, T* dz, T* p,
                          uint32_t* f, hipStream_t s)
  {
    if (is_agg(c.model_id))
      return sample(c.children, c.nchildren, c.model_id == BBM_HIP_AGGREGATE_BSDF, ox, oy, oz, xi0, xi1, mask, n, comp,
                    unit, dx, dy, dz, p, f, s);
    return L::sample(c, ox, oy, oz, xi0, xi1, mask, n, comp, unit, dx, dy, dz, p, f, s);
  }

  // weights w (nchild x n) and their sum for directions `out`
  static int weights(const Child* c, int nchild, const T* ox, const T* oy, const T* oz, const uint8_t* mask, size_t n,
                     uint32_t comp, uint32_t unit, T* w, T* sum, T* tr, T* tg, T* tb, hipStream_t s)
  {
    for (int k = 0; k < nchild; ++k)
    {
      int rc = child_reflectance(c[k], ox, oy, oz, mask, n, comp, unit, tr, tg, tb, s);
      if (rc) return rc;
      hipLaunchKernelGGL(k_weight<T>, dim3(grid(n)), dim3(kB), 0, s, tr, tg, tb, w + size_t(k) * n, sum, uint64_t(n),
                         int(k == 0));
      if ((rc = launched())) return rc;
    }
    return BBM_HIP_OK;
  }

  // pdf = mixture of the children's pdfs at (in, out) with weights w / sum: aggregatemodel's inner product over the
  // sum, or (bsdf) aggregatebsdf's per-term quotients
  static int mixture_pdf(const Child* c, int nchild, bool bsdf, const T* ix, const T* iy, const T* iz, const T* ox,
                         const T* oy, const T* oz, const uint8_t* mask, size_t n, uint32_t comp, uint32_t unit,
                         const T* w, const T* sum, T* tp, T* ip, T* pdf, hipStream_t s)
  {
    for (int k = 0; k < nchild; ++k)
    {
      int rc = child_pdf(c[k], ix, iy, iz, ox, oy, oz, mask, n, comp, unit, tp, s);
      if (rc) return rc;
      if (bsdf)
        hipLaunchKernelGGL(k_inner_bsdf<T>, dim3(grid(n)), dim3(kB), 0, s, tp, w + size_t(k) * n, sum, ip, uint64_t(n),
                           int(k == 0));
      else
        hipLaunchKernelGGL(k_inner<T>, dim3(grid(n)), dim3(kB), 0, s, tp, w + size_t(k) * n, ip, uint64_t(n), int(k == 0));
      if ((rc = launched())) return rc;
    }
    if (bsdf) hipLaunchKernelGGL(k_mask_sum<T>, dim3(grid(n)), dim3(kB), 0, s, ip, sum, pdf, uint64_t(n));
    else hipLaunchKernelGGL(k_mix<T>, dim3(grid(n)), dim3(kB), 0, s, ip, sum, pdf, uint64_t(n));
    return launched();
  }

  // the children's sum: aggregatemodel's right fold e0 + (e1 + (... + eK)), or (bsdf) aggregatebsdf's left fold
  // ((0 + e0) + e1) + ... ; `part` evaluates child k into the given outputs
  template<class F>
  static int fold(int nchild, bool bsdf, size_t n, T* r, T* g, T* b, T* tr, T* tg, T* tb, hipStream_t s, F&& part)
  {
    int rc;
    const int last = nchild - 1;
    if ((rc = part(bsdf ? 0 : last, r, g, b))) return rc;
    for (int j = 1; j <= last; ++j)
    {
      const int k = bsdf ? j : last - j;
      if ((rc = part(k, tr, tg, tb))) return rc;
      if (bsdf) hipLaunchKernelGGL(k_lfold3<T>, dim3(grid(n)), dim3(kB), 0, s, tr, tg, tb, r, g, b, uint64_t(n), int(j == 1));
      else hipLaunchKernelGGL(k_fold3<T>, dim3(grid(n)), dim3(kB), 0, s, tr, tg, tb, r, g, b, uint64_t(n));
      if ((rc = launched())) return rc;
    }
    return BBM_HIP_OK;
  }

  static int eval_pdf(const Child* c, int nchild, bool bsdf, const T* ix, const T* iy, const T* iz, const T* ox,
                      const T* oy, const T* oz, const uint8_t* mask, size_t n, uint32_t comp, uint32_t unit, T* r, T* g,
                      T* b, T* pdf, hipStream_t s)
  {
    Scratch sc(s);
    T* tr = sc.get<T>(n);
    T* tg = sc.get<T>(n);
    T* tb = sc.get<T>(n);
    if (!tr || !tg || !tb) return fail(BBM_HIP_ERR_HIP, "aggregate: scratch allocation failed: " + scratch_failure());
    int rc;
    if (r && (rc = fold(nchild, bsdf, n, r, g, b, tr, tg, tb, s, [&](int k, T* rr, T* gg, T* bb) {
          return child_eval(c[k], ix, iy, iz, ox, oy, oz, mask, n, comp, unit, rr, gg, bb, s);
        })))
      return rc;
    if (pdf)
    {
      T* w = sc.get<T>(size_t(nchild) * n);
      T* sum = sc.get<T>(n);
      T* ip = sc.get<T>(n);
      if (!w || !sum || !ip) return fail(BBM_HIP_ERR_HIP, "aggregate: scratch allocation failed: " + scratch_failure());
      if ((rc = weights(c, nchild, ox, oy, oz, mask, n, comp, unit, w, sum, tr, tg, tb, s))) return rc;
      if ((rc = mixture_pdf(c, nchild, bsdf, ix, iy, iz, ox, oy, oz, mask, n, comp, unit, w, sum, tr, ip, pdf, s)))
        return rc;
    }
    return BBM_HIP_OK;
  }

  static int reflectance(const Child* c, int nchild, bool bsdf, const T* ox, const T* oy, const T* oz,
                         const uint8_t* mask, size_t n, uint32_t comp, uint32_t unit, T* r, T* g, T* b, hipStream_t s)
  {
    Scratch sc(s);
    T* tr = sc.get<T>(n);
    T* tg = sc.get<T>(n);
    T* tb = sc.get<T>(n);
    if (!tr || !tg || !tb) return fail(BBM_HIP_ERR_HIP, "aggregate: scratch allocation failed: " + scratch_failure());
    return fold(nchild, bsdf, n, r, g, b, tr, tg, tb, s, [&](int k, T* rr, T* gg, T* bb) {
      return child_reflectance(c[k], ox, oy, oz, mask, n, comp, unit, rr, gg, bb, s);
    });
  }

  static int sample(const Child* c, int nchild, bool bsdf, const T* ox, const T* oy, const T* oz, const T* xi0,
                    const T* xi1, const uint8_t* mask, size_t n, uint32_t comp, uint32_t unit, T* dx, T* dy, T* dz,
                    T* pdf, uint32_t* flag, hipStream_t s)
  {
    Scratch sc(s);
    T* w = sc.get<T>(size_t(nchild) * n);
    T* sum = sc.get<T>(n);
    T* ip = sc.get<T>(n);
    T* t0 = sc.get<T>(n);
    T* t1 = sc.get<T>(n);
    T* t2 = sc.get<T>(n);
    T* t3 = sc.get<T>(n);
    uint32_t* tf = sc.get<uint32_t>(n);
    int8_t* chosen = sc.get<int8_t>(n);
    uint8_t* cm = sc.get<uint8_t>(n);
    T* xs = sc.get<T>(n);
    if (!w || !sum || !ip || !t0 || !t1 || !t2 || !t3 || !tf || !chosen || !cm || !xs)
      return fail(BBM_HIP_ERR_HIP, "aggregate: scratch allocation failed: " + scratch_failure());
    int rc;
    if ((rc = weights(c, nchild, ox, oy, oz, mask, n, comp, unit, w, sum, t0, t1, t2, s))) return rc;
    hipLaunchKernelGGL(k_select<T>, dim3(grid(n)), dim3(kB), 0, s, w, nchild, sum, xi0, mask, chosen, xs, uint64_t(n),
                       int(bsdf));
    hipLaunchKernelGGL(k_zero_sample<T>, dim3(grid(n)), dim3(kB), 0, s, dx, dy, dz, flag, uint64_t(n));
    if ((rc = launched())) return rc;
    for (int k = 0; k < nchild; ++k)
    {
      hipLaunchKernelGGL(k_child_mask, dim3(grid(n)), dim3(kB), 0, s, chosen, k, cm, uint64_t(n));
      if ((rc = launched())) return rc;
      if ((rc = child_sample(c[k], ox, oy, oz, xs, xi1, cm, n, comp, unit, t0, t1, t2, t3, tf, s))) return rc;
      hipLaunchKernelGGL(k_take<T>, dim3(grid(n)), dim3(kB), 0, s, chosen, k, t0, t1, t2, tf, dx, dy, dz, flag,
                         uint64_t(n));
      if ((rc = launched())) return rc;
    }
    // pdf of the sampled direction: the weighted mixture of every child's pdf (:116-117; aggregatebsdf.h:133-137,
    // where a lane without a sample keeps pdf 0: sum <= eps there, which the mixture masks)
    return mixture_pdf(c, nchild, bsdf, dx, dy, dz, ox, oy, oz, mask, n, comp, unit, w, sum, t3, ip, pdf, s);
  }
};


// ============================================================================ any model as a tree
// (a single registry model = one leaf node; an aggregatemodel's children; an aggregate root node)

template<class T>
struct Model
{
  using L = Leaf<T>;
  using Child = typename L::Child;
  using C = Composite<T>;
  const Child* c;
  int n;
  bool bsdf = false, leaf = false;
  Model(const Child* c0, int n0) : c(c0), n(n0)
  {
    leaf = c && n == 1 && !C::is_agg(c[0].model_id);
    if (!leaf) C::root(c, n, bsdf);
  }
  int check() const
  {
    if (!leaf) return C::check(c, n);
    const int np = L::nparams(c[0].model_id);
    if (np < 0) return np;
    if (c[0].nparams != np || (np > 0 && !c[0].params))
      return fail(BBM_HIP_ERR_INVALID_ARG, "model: expected " + std::to_string(np) + " parameters");
    if (!L::supported(c[0].model_id))
      return fail(BBM_HIP_ERR_UNSUPPORTED, std::string(bbm_hip_model_name(c[0].model_id)) + ": no doubleRGB kernel");
    return BBM_HIP_OK;
  }
  int eval_pdf(const T* ix, const T* iy, const T* iz, const T* ox, const T* oy, const T* oz, size_t m, uint32_t comp,
               uint32_t unit, T* r, T* g, T* b, T* p, hipStream_t s) const
  {
    if (!leaf) return C::eval_pdf(c, n, bsdf, ix, iy, iz, ox, oy, oz, nullptr, m, comp, unit, r, g, b, p, s);
    if (r && p) return L::eval_pdf(c[0], ix, iy, iz, ox, oy, oz, nullptr, m, comp, unit, r, g, b, p, s);
    if (r) return L::eval(c[0], ix, iy, iz, ox, oy, oz, nullptr, m, comp, unit, r, g, b, s);
    return L::pdf(c[0], ix, iy, iz, ox, oy, oz, nullptr, m, comp, unit, p, s);
  }
  int sample(const T* ox, const T* oy, const T* oz, const T* xi0, const T* xi1, size_t m, uint32_t comp, uint32_t unit,
             T* dx, T* dy, T* dz, T* p, uint32_t* f, hipStream_t s) const
  {
    if (!leaf) return C::sample(c, n, bsdf, ox, oy, oz, xi0, xi1, nullptr, m, comp, unit, dx, dy, dz, p, f, s);
    return L::sample(c[0], ox, oy, oz, xi0, xi1, nullptr, m, comp, unit, dx, dy, dz, p, f, s);
  }
};

// leaf parameter count of a tree (preorder), -1 on a malformed node
template<class Child>
int tree_params(const Child* c, int n, int depth = 0)
{
  if (!c || n < 1 || depth > kMaxDepth) return -1;
  int total = 0;
  for (int k = 0; k < n; ++k)
  {
    if (c[k].model_id == BBM_HIP_AGGREGATE || c[k].model_id == BBM_HIP_AGGREGATE_BSDF)
    {
      const int t = tree_params(c[k].children, c[k].nchildren, depth + 1);
      if (t < 0) return -1;
      total += t;
    }
    else
    {
      const int np = bbm_hip_model_nparams(c[k].model_id);
      if (np < 0) return -1;
      total += np;
    }
  }
  return total;
}

// a copy of the tree whose leaves read their parameters from `p` (preorder, back to back); kept alive by `store`
template<class Child, class P>
const Child* tree_with(const Child* c, int n, const P* p, int& off, std::vector<std::vector<Child>>& store)
{
  std::vector<Child> v(c, c + n);
  for (int k = 0; k < n; ++k)
  {
    if (v[k].model_id == BBM_HIP_AGGREGATE || v[k].model_id == BBM_HIP_AGGREGATE_BSDF)
      v[k].children = tree_with(c[k].children, c[k].nchildren, p, off, store);
    else
    {
      v[k].params = p + off;
      v[k].nparams = bbm_hip_model_nparams(c[k].model_id);
      off += v[k].nparams;
    }
  }
  store.push_back(std::move(v));       // the vector's buffer does not move with the outer vector
  return store.back().data();
}

// ---------------------------------------------------------------------------- materialised loss

constexpr unsigned kTreeLossBlocks = 1024;
unsigned loss_tree_blocks(size_t n)
{
  const size_t b = (n + kB - 1) / kB;
  return unsigned(b < 1 ? 1 : (b > kTreeLossBlocks ? kTreeLossBlocks : b));
}

__device__ __forceinline__ double tree_loss_term(int kind, float iz, float oz, const float* ref, const float* v)
{
  return double(sample_loss(kind, loss_prepare(kind, mk3(0.0f, 0.0f, iz), mk3(0.0f, 0.0f, oz), ref), v));
}
__device__ __forceinline__ double tree_loss_term(int kind, double iz, double oz, const double* ref, const double* v)
{
  return sample_loss_d(kind, loss_prepare_d(kind, iz, oz, ref), v);
}

// per-sample losses of one probe's evaluation -> one partial per workgroup (block_sums[b][p])
template<class T>
__global__ __launch_bounds__(kB) void k_loss_terms(const T* r, const T* g, const T* b, const T* iz, const T* oz,
                                                   const T* rr, const T* rg, const T* rb, int kind, uint64_t n,
                                                   double* block_sums, int p, int nprobes)
{
  math_tables_init();
  __shared__ double part[kB / 64];
  double acc = 0.0;
  BBM_GRID_LOOP(i, n)
  {
    const T v[3] = {r[i], g[i], b[i]};
    const T ref[3] = {rr[i], rg[i], rb[i]};
    acc += tree_loss_term(kind, iz[i], oz[i], ref, v);
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0)
  {
    double t = 0.0;
    for (int w = 0; w < kB / 64; ++w) t += part[w];
    block_sums[size_t(blockIdx.x) * size_t(nprobes) + size_t(p)] = t;
  }
}

template<class T>
int loss_tree(const typename Leaf<T>::Child* tree, int ntree, const T* probes, int nparams, int nprobes, size_t n,
              const T* const* in, const T* const* out, const T* const* ref, int kind, uint32_t comp, uint32_t unit,
              double* sums, void* ws, size_t wsb, hipStream_t s)
{
  using Child = typename Leaf<T>::Child;
  const int np = tree_params(tree, ntree);
  if (np < 0) return fail(BBM_HIP_ERR_INVALID_ARG, "malformed model tree");
  if (np != nparams)
    return fail(BBM_HIP_ERR_INVALID_ARG, "the tree's leaves take " + std::to_string(np) + " parameters, not " +
                                             std::to_string(nparams));
  if (nprobes < 1 || !probes || !sums) return fail(BBM_HIP_ERR_INVALID_ARG, "probes / sums");
  if (kind < kLossNganL2 || kind > kLossBieronLog) return fail(BBM_HIP_ERR_INVALID_ARG, "unknown loss");
  for (int k = 0; k < 3; ++k)
    if (n > 0 && (!in[k] || !out[k] || !ref[k])) return fail(BBM_HIP_ERR_INVALID_ARG, "direction / reference pointer is NULL");
  const unsigned blocks = loss_tree_blocks(n);
  if (!ws || wsb < size_t(blocks) * size_t(nprobes) * sizeof(double))
    return fail(BBM_HIP_ERR_INVALID_ARG, "workspace too small (bbm_hip_loss_tree_workspace_size)");
  double* block_sums = static_cast<double*>(ws);
  if (n == 0)
  {
    const hipError_t e = hipMemsetAsync(sums, 0, size_t(nprobes) * sizeof(double), s);
    return e == hipSuccess ? BBM_HIP_OK : fail(BBM_HIP_ERR_HIP, "hipMemsetAsync failed");
  }
  Scratch sc(s);
  T* rgb = sc.get<T>(3 * n);
  if (!rgb) return fail(BBM_HIP_ERR_HIP, "loss: scratch allocation failed: " + scratch_failure());
  for (int p = 0; p < nprobes; ++p)
  {
    std::vector<std::vector<Child>> store;
    store.reserve(64);
    int off = 0;
    const Child* t = tree_with(tree, ntree, probes + size_t(p) * size_t(nparams), off, store);
    const Model<T> m(t, ntree);
    int rc = m.check();
    if (rc) return rc;
    if ((rc = m.eval_pdf(in[0], in[1], in[2], out[0], out[1], out[2], n, comp, unit, rgb, rgb + n, rgb + 2 * n, nullptr, s)))
      return rc;
    hipLaunchKernelGGL(k_loss_terms<T>, dim3(blocks), dim3(kB), 0, s, rgb, rgb + n, rgb + 2 * n, in[2], out[2], ref[0],
                       ref[1], ref[2], kind, uint64_t(n), block_sums, p, nprobes);
    if ((rc = launched())) return rc;
  }
  hipLaunchKernelGGL(k_loss_final, dim3(unsigned(nprobes)), dim3(kBlock), 0, s, block_sums, int(blocks), nprobes, sums);
  return launched();
}

// ------------------------------------------------------------------------ materialised checkBsdf

// sampleSphere / sampleHemisphere (checkBsdf.cpp:28-45) in the configuration's Value: float as k_check
// (check.hpp sphere_dir), double all the way (theta = safe_acos(1 - 2 xi0), phi = xi1 Pi(2), double cos / sin)
__device__ __forceinline__ void sphere_dir_t(float u0, float u1, bool hemi, float& x, float& y, float& z)
{
  const v3 d = sphere_dir(u0, u1, hemi);
  x = d.x; y = d.y; z = d.z;
}
__device__ __forceinline__ void sphere_dir_t(float u0, float u1, bool hemi, double& x, double& y, double& z)
{
  const double theta = hemi ? acos(fmin(1.0, fmax(-1.0, double(u0)))) : acos(fmin(1.0, fmax(-1.0, 1.0 - 2.0 * double(u0))));
  const double phi = double(u1) * (2.0 * kPiD);
  double st, ct, sp, cp;
  sincos(theta, &st, &ct);
  sincos(phi, &sp, &cp);
  x = cp * st; y = sp * st; z = ct;
}
template<class T> __device__ __forceinline__ T inv_sphere_pdf();
template<> __device__ __forceinline__ float inv_sphere_pdf<float>() { return kInv4PiF; }
template<> __device__ __forceinline__ double inv_sphere_pdf<double>() { return 1.0 / (4.0 * kPiD); }
__device__ __forceinline__ float tdiv(float a, float b) { return div_nr(a, b); }
__device__ __forceinline__ double tdiv(double a, double b) { return a / b; }

// spherical::theta / phi of a direction in the Value type (chi-square binning, checkBsdf.cpp:374-377)
__device__ __forceinline__ float theta_t(float x, float y, float z) { return theta_of(mk3(x, y, z)); }
__device__ __forceinline__ float phi_t(float x, float y, float z) { return phi_of(mk3(x, y, z)); }
__device__ __forceinline__ double theta_t(double x, double y, double z)
{
  const double dz = z - ((z < 0) ? -1.0 : 1.0);
  const double t = 2.0 * asin(0.5 * sqrt(((0.0 + x * x) + y * y) + dz * dz));
  return (z >= 0) ? t : kPiD - t;
}
__device__ __forceinline__ double phi_t(double x, double y, double)
{
  const double r = atan2(y, x);
  return (r < 0) ? r + 2.0 * kPiD : r;
}

struct TreeCheckDims
{
  uint64_t begin, n;        // samples [begin, begin + n) of every slot
  uint64_t len;             // samples per slot in this chunk
  uint64_t i0;              // first sample of the chunk within its slot(s)
  int s0, nsl;              // first slot and number of slots in the chunk
  int nparts, part;         // partials per slot = nparts x bx; this chunk's part
  uint32_t nth, nph;
};

// per-lane inputs of one chunk: lane j <-> slot s0 + j / len, sample i0 + j % len
template<class T, int TEST>
__global__ __launch_bounds__(kB) void k_tree_gen(TreeCheckDims dm, uint64_t k0base, uint64_t k1base, uint64_t k2base,
                                                 const T* sx, const T* sy, const T* sz, int sphere, int importance,
                                                 T* ax, T* ay, T* az, T* bx, T* by, T* bz, T* x0, T* x1, T* y0,
                                                 T* y1, T* aux)
{
  math_tables_init();
  const uint64_t lanes = dm.len * uint64_t(dm.nsl);
  BBM_GRID_LOOP(j, lanes)
  {
    const int slot = dm.s0 + int(j / dm.len);
    const uint64_t smp = dm.begin + dm.i0 + j % dm.len;
    float u0, u1;
    uniform2(check_key(k0base, slot), smp, u0, u1);
    if constexpr (TEST == kCheckReflectance)
    {
      bx[j] = sx[slot]; by[j] = sy[slot]; bz[j] = sz[slot];
      if (importance) { x0[j] = T(u0); x1[j] = T(u1); }
      else { sphere_dir_t(u0, u1, false, ax[j], ay[j], az[j]); aux[j] = inv_sphere_pdf<T>(); }
    }
    else if constexpr (TEST == kCheckReciprocity || TEST == kCheckAdjoint)
    {
      float w0, w1;
      uniform2(check_key(k1base, slot), smp, w0, w1);
      sphere_dir_t(u0, u1, false, ax[j], ay[j], az[j]);
      sphere_dir_t(w0, w1, false, bx[j], by[j], bz[j]);
    }
    else if constexpr (TEST == kCheckPdf)
    {
      float w0, w1, z0, z1;
      uniform2(check_key(k1base, slot), smp, w0, w1);
      uniform2(check_key(k2base, slot), smp, z0, z1);
      sphere_dir_t(u0, u1, !sphere, bx[j], by[j], bz[j]);
      x0[j] = T(w0); x1[j] = T(w1); y0[j] = T(z0); y1[j] = T(z1);
    }
    else if constexpr (TEST == kCheckPdfInt)
    {
      sphere_dir_t(u0, u1, false, ax[j], ay[j], az[j]);
      bx[j] = sx[slot]; by[j] = sy[slot]; bz[j] = sz[slot];
    }
    else if constexpr (TEST == kCheckSamplePdf)
    {
      // checkBsdf.cpp:347-356: a uniform point in the (theta, phi) bin of this slot, weighted by its solid angle
      const uint32_t bins = dm.nth * dm.nph;
      const uint32_t bin = uint32_t(slot) % bins;
      const int trial = slot / int(bins);
      const uint32_t t = bin / dm.nph, pb = bin % dm.nph;
      if constexpr (sizeof(T) == 4)
      {
        const float phi = div_nr(kPi2F * (float(pb) + u0), float(dm.nph));
        const float theta = div_nr(kPiF * (float(t) + u1), float(dm.nth));
        const v3 d = sph_to_vec(phi, theta);
        float st, ct;
        cossin_cr(theta, ct, st);
        constexpr float kPiSq2 = (2.0f * kPiF) * kPiF;
        ax[j] = d.x; ay[j] = d.y; az[j] = d.z;
        aux[j] = div_nr(kPiSq2 * fabsf(st), float(dm.nph * dm.nth));
      }
      else
      {
        const double phi = (2.0 * kPiD) * (double(pb) + double(u0)) / double(dm.nph);
        const double theta = kPiD * (double(t) + double(u1)) / double(dm.nth);
        double st, ct, sp, cp;
        sincos(theta, &st, &ct);
        sincos(phi, &sp, &cp);
        ax[j] = cp * st; ay[j] = sp * st; az[j] = ct;
        aux[j] = ((2.0 * kPiD) * kPiD) * fabs(st) / (double(dm.nph) * double(dm.nth));
      }
      bx[j] = sx[trial]; by[j] = sy[trial]; bz[j] = sz[trial];
    }
    else   // kCheckSampleCount
    {
      bx[j] = sx[slot]; by[j] = sy[slot]; bz[j] = sz[slot];
      x0[j] = T(u0); x1[j] = T(u1);
    }
  }
}

// per-sample terms of one chunk -> partials[slot][part * gridDim.x + block] (or the histogram)
template<class T, int TEST>
__global__ __launch_bounds__(kB) void k_tree_acc(TreeCheckDims dm, const T* ax, const T* ay, const T* az, const T* bz,
                                                 const T* r, const T* g, const T* b, const T* r2, const T* g2,
                                                 const T* b2, const T* pa, const T* pb, const T* qa, const T* qb,
                                                 const T* a2z, const T* aux, int include_zero, double* partial,
                                                 unsigned long long* counts)
{
  math_tables_init();
  __shared__ double part[kB / 64][kCheckAcc];
  const int sl = blockIdx.y;                     // slot within the chunk
  const int slot = dm.s0 + sl;
  double acc[kCheckAcc];
#pragma unroll
  for (int e = 0; e < kCheckAcc; ++e) acc[e] = 0.0;
  acc[kCheckSums] = acc[kCheckSums + 2] = -1.0;
  acc[kCheckSums + 1] = acc[kCheckSums + 3] = 1.8e19;
  const T eps = eps_of<T>();
  for (uint64_t i = uint64_t(blockIdx.x) * kB + threadIdx.x; i < dm.len; i += uint64_t(gridDim.x) * kB)
  {
    const uint64_t j = uint64_t(sl) * dm.len + i;
    const uint64_t smp = dm.begin + dm.i0 + i;
    if constexpr (TEST == kCheckReflectance)
    {
      if (pa[j] > T(eps))
      {
        acc[0] += double(tdiv(r[j] * az[j], pa[j]));
        acc[1] += double(tdiv(g[j] * az[j], pa[j]));
        acc[2] += double(tdiv(b[j] * az[j], pa[j]));
        acc[3] += 1.0;
      }
    }
    else if constexpr (TEST == kCheckReciprocity || TEST == kCheckAdjoint)
    {
      const T d0 = fabs(r[j] - r2[j]), d1 = fabs(g[j] - g2[j]), d2 = fabs(b[j] - b2[j]);
      const double h = double(((T(0) + d0) + d1) + d2);
      acc[0] += double(d0); acc[1] += double(d1); acc[2] += double(d2);
      if (TEST == kCheckReciprocity) { acc[3] += double(d0); acc[4] += double(d1); acc[5] += double(d2); }
      max_pair(acc[kCheckSums], acc[kCheckSums + 1], h, double(smp));
      if (TEST == kCheckReciprocity) max_pair(acc[kCheckSums + 2], acc[kCheckSums + 3], h, double(smp));
    }
    else if constexpr (TEST == kCheckPdf)
    {
      acc[0] += (qa[j] < 0) ? 1.0 : 0.0;
      acc[1] += (qb[j] < 0) ? 1.0 : 0.0;
      acc[2] += (az[j] < 0) ? 1.0 : 0.0;
      acc[3] += (a2z[j] < 0) ? 1.0 : 0.0;
      acc[4] += double(fabs(pa[j] - qa[j]));
      acc[5] += double(fabs(pb[j] - qb[j]));
    }
    else if constexpr (TEST == kCheckPdfInt)
    {
      const double q = double(tdiv(qa[j], inv_sphere_pdf<T>()));
      acc[0] += q;
      acc[1] += q;
    }
    else if constexpr (TEST == kCheckSamplePdf)
    {
      acc[0] += double(qa[j] * aux[j]);
    }
    else   // kCheckSampleCount
    {
      if (include_zero || pa[j] > T(eps))
      {
        const uint32_t bins = dm.nth * dm.nph;
        const T th = fmin(theta_t(ax[j], ay[j], az[j]) / T(sizeof(T) == 4 ? double(kPiF) : kPiD) * T(dm.nth), T(dm.nth - 1));
        const T ph = fmin(phi_t(ax[j], ay[j], az[j]) / T(sizeof(T) == 4 ? double(kPi2F) : 2.0 * kPiD) * T(dm.nph),
                          T(dm.nph - 1));
        const uint32_t idx = uint32_t(th) * dm.nph + uint32_t(ph);
        atomicAdd(counts + size_t(slot) * bins + idx, 1ull);
      }
    }
  }
  if constexpr (TEST != kCheckSampleCount)
  {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    wave_reduce_check(acc);
    if (lane == 0)
    {
#pragma unroll
      for (int e = 0; e < kCheckAcc; ++e) part[wave][e] = acc[e];
    }
    __syncthreads();
    if (threadIdx.x == 0)
    {
      double rr[kCheckAcc];
#pragma unroll
      for (int e = 0; e < kCheckAcc; ++e) rr[e] = part[0][e];
      for (int w = 1; w < kB / 64; ++w)
      {
#pragma unroll
        for (int e = 0; e < kCheckSums; ++e) rr[e] += part[w][e];
        max_pair(rr[kCheckSums], rr[kCheckSums + 1], part[w][kCheckSums], part[w][kCheckSums + 1]);
        max_pair(rr[kCheckSums + 2], rr[kCheckSums + 3], part[w][kCheckSums + 2], part[w][kCheckSums + 3]);
      }
      const size_t nb = size_t(dm.nparts) * gridDim.x;
      double* dst = partial + (size_t(slot) * nb + size_t(dm.part) * gridDim.x + blockIdx.x) * kCheckAcc;
#pragma unroll
      for (int e = 0; e < kCheckAcc; ++e) dst[e] = rr[e];
    }
  }
}

constexpr uint64_t kTreeChunk = uint64_t(1) << 19;     // lanes materialised per chunk (all tests, all slots)
constexpr unsigned kTreeCheckBx = 64;                  // partials per slot and chunk part

struct TreeCheckPlan
{
  uint64_t len;      // samples per slot per chunk
  int per;           // slots per chunk
  int nparts;        // chunk parts per slot
};
TreeCheckPlan tree_check_plan(uint64_t n, int nslots)
{
  TreeCheckPlan p;
  if (n >= kTreeChunk) { p.len = kTreeChunk; p.per = 1; p.nparts = int((n + kTreeChunk - 1) / kTreeChunk); }
  else
  {
    p.len = n > 0 ? n : 1;
    p.per = int(std::min<uint64_t>(uint64_t(nslots), kTreeChunk / p.len));
    if (p.per < 1) p.per = 1;
    p.nparts = 1;
  }
  return p;
}

template<class T, int TEST>
int check_tree_test(const Model<T>& m, const bbm_hip_check_desc* d, const T* sx, const T* sy, const T* sz,
                    double* acc, uint64_t* counts, double* partial, hipStream_t s)
{
  const TreeCheckPlan plan = tree_check_plan(d->n, d->nslots);
  const uint64_t lanes = plan.len * uint64_t(plan.per);
  Scratch sc(s);
  T* buf[22];
  for (T*& q : buf)
    if (!(q = sc.get<T>(lanes))) return fail(BBM_HIP_ERR_HIP, "check: scratch allocation failed: " + scratch_failure());
  uint32_t* fa = sc.get<uint32_t>(lanes);
  uint32_t* fb = sc.get<uint32_t>(lanes);
  if (!fa || !fb) return fail(BBM_HIP_ERR_HIP, "check: scratch allocation failed: " + scratch_failure());
  T *ax = buf[0], *ay = buf[1], *az = buf[2], *bx = buf[3], *by = buf[4], *bz = buf[5], *x0 = buf[6], *x1 = buf[7];
  T *y0 = buf[8], *y1 = buf[9], *aux = buf[10], *r = buf[11], *g = buf[12], *b = buf[13], *r2 = buf[14];
  T *g2 = buf[15], *b2 = buf[16], *pa = buf[17], *pb = buf[18], *qa = buf[19], *qb = buf[20], *cz = buf[21];
  T *cx = r2, *cy = g2;      // the PDF test's second sample direction (no second evaluation there)
  const uint64_t k0 = check_base_key(d->seed, d->test, 0), k1 = check_base_key(d->seed, d->test, 1),
                 k2 = check_base_key(d->seed, d->test, 2);
  const uint32_t comp = kFlagAll;
  int rc;
  for (int s0 = 0; s0 < d->nslots; s0 += plan.per)
  {
    const int nsl = std::min(plan.per, d->nslots - s0);
    for (int part = 0; part < plan.nparts; ++part)
    {
      TreeCheckDims dm;
      dm.begin = d->begin; dm.n = d->n; dm.i0 = uint64_t(part) * plan.len;
      dm.len = std::min<uint64_t>(plan.len, d->n - dm.i0);
      dm.s0 = s0; dm.nsl = nsl; dm.nparts = plan.nparts; dm.part = part; dm.nth = d->theta_bins; dm.nph = d->phi_bins;
      const size_t ml = size_t(dm.len) * size_t(nsl);
      hipLaunchKernelGGL((k_tree_gen<T, TEST>), dim3(grid(ml)), dim3(kB), 0, s, dm, k0, k1, k2, sx, sy, sz, d->sphere,
                         d->importance, ax, ay, az, bx, by, bz, x0, x1, y0, y1, aux);
      if ((rc = launched())) return rc;
      if constexpr (TEST == kCheckReflectance)
      {
        if (d->importance && (rc = m.sample(bx, by, bz, x0, x1, ml, comp, 0, ax, ay, az, pa, fa, s))) return rc;
        if (!d->importance)
        {
          const hipError_t e = hipMemcpyAsync(pa, aux, ml * sizeof(T), hipMemcpyDeviceToDevice, s);
          if (e != hipSuccess) return fail(BBM_HIP_ERR_HIP, "hipMemcpyAsync failed");
        }
        if ((rc = m.eval_pdf(ax, ay, az, bx, by, bz, ml, comp, 0, r, g, b, nullptr, s))) return rc;
      }
      else if constexpr (TEST == kCheckReciprocity || TEST == kCheckAdjoint)
      {
        if ((rc = m.eval_pdf(ax, ay, az, bx, by, bz, ml, comp, 0, r, g, b, nullptr, s))) return rc;
        if ((rc = m.eval_pdf(bx, by, bz, ax, ay, az, ml, comp, TEST == kCheckAdjoint ? 1u : 0u, r2, g2, b2, nullptr, s)))
          return rc;
      }
      else if constexpr (TEST == kCheckPdf)
      {
        if ((rc = m.sample(bx, by, bz, x0, x1, ml, comp, 0, ax, ay, az, pa, fa, s))) return rc;
        if ((rc = m.sample(bx, by, bz, y0, y1, ml, comp, 1, cx, cy, cz, pb, fb, s))) return rc;
        if ((rc = m.eval_pdf(ax, ay, az, bx, by, bz, ml, comp, 0, nullptr, nullptr, nullptr, qa, s))) return rc;
        if ((rc = m.eval_pdf(cx, cy, cz, bx, by, bz, ml, comp, 1, nullptr, nullptr, nullptr, qb, s))) return rc;
      }
      else if constexpr (TEST == kCheckPdfInt || TEST == kCheckSamplePdf)
      {
        if ((rc = m.eval_pdf(ax, ay, az, bx, by, bz, ml, comp, 0, nullptr, nullptr, nullptr, qa, s))) return rc;
      }
      else
      {
        if ((rc = m.sample(bx, by, bz, x0, x1, ml, comp, 0, ax, ay, az, pa, fa, s))) return rc;
      }
      hipLaunchKernelGGL((k_tree_acc<T, TEST>), dim3(kTreeCheckBx, unsigned(nsl)), dim3(kB), 0, s, dm, ax, ay, az, bz,
                         r, g, b, r2, g2, b2, pa, pb, qa, qb, cz, aux, d->include_zero_pdf, partial,
                         reinterpret_cast<unsigned long long*>(counts));
      if ((rc = launched())) return rc;
    }
  }
  if (TEST != kCheckSampleCount)
  {
    hipLaunchKernelGGL(k_check_final, dim3(unsigned(d->nslots)), dim3(64), 0, s, partial, int(plan.nparts * kTreeCheckBx), acc);
    return launched();
  }
  return BBM_HIP_OK;
}

size_t check_tree_ws(const bbm_hip_check_desc* d)
{
  if (!d || d->nslots <= 0) return 0;
  const TreeCheckPlan p = tree_check_plan(d->n, d->nslots);
  return size_t(d->nslots) * size_t(p.nparts) * kTreeCheckBx * kCheckAcc * sizeof(double);
}

template<class T>
int check_tree(const typename Leaf<T>::Child* tree, int ntree, const bbm_hip_check_desc* d, const T* sx, const T* sy,
               const T* sz, double* acc, uint64_t* counts, void* ws, size_t wsb, hipStream_t s)
{
  const Model<T> m(tree, ntree);
  int rc = m.check();
  if (rc) return rc;
  if (!d) return fail(BBM_HIP_ERR_INVALID_ARG, "check descriptor is NULL");
  if (d->test < 0 || d->test >= kCheckNumTests) return fail(BBM_HIP_ERR_INVALID_ARG, "unknown check test");
  if (d->nslots <= 0 || d->nslots > 65535) return fail(BBM_HIP_ERR_INVALID_ARG, "nslots must be in [1, 65535]");
  const bool chi2 = d->test == kCheckSamplePdf || d->test == kCheckSampleCount;
  const uint64_t bins = uint64_t(d->theta_bins) * d->phi_bins;
  if (chi2 && (d->theta_bins == 0 || d->phi_bins == 0 || bins > (1u << 20)))
    return fail(BBM_HIP_ERR_INVALID_ARG, "theta_bins / phi_bins must be positive (at most 2^20 bins)");
  if (d->test == kCheckSamplePdf && d->nslots % bins != 0)
    return fail(BBM_HIP_ERR_INVALID_ARG, "SAMPLE_PDF: nslots must be trials x theta_bins x phi_bins");
  const bool needs_dirs = d->test == kCheckReflectance || d->test == kCheckPdfInt || chi2;
  if (needs_dirs && (!sx || !sy || !sz)) return fail(BBM_HIP_ERR_INVALID_ARG, "this test needs slot directions");
  if (d->test == kCheckSampleCount ? !counts : !acc) return fail(BBM_HIP_ERR_INVALID_ARG, "acc / counts pointer is NULL");
  if (d->test != kCheckSampleCount && (!ws || wsb < check_tree_ws(d)))
    return fail(BBM_HIP_ERR_INVALID_ARG, "workspace too small (bbm_hip_check_tree_workspace_size)");
  if (d->test == kCheckSampleCount)
  {
    const hipError_t me = hipMemsetAsync(counts, 0, size_t(d->nslots) * bins * sizeof(uint64_t), s);
    if (me != hipSuccess) return fail(BBM_HIP_ERR_HIP, std::string("hipMemsetAsync: ") + hipGetErrorString(me));
  }
  if (d->n == 0)
  {
    if (d->test == kCheckSampleCount) return BBM_HIP_OK;
    const hipError_t me = hipMemsetAsync(acc, 0, size_t(d->nslots) * kCheckAcc * sizeof(double), s);
    return me == hipSuccess ? BBM_HIP_OK : fail(BBM_HIP_ERR_HIP, std::string("hipMemsetAsync: ") + hipGetErrorString(me));
  }
  double* partial = static_cast<double*>(ws);
  switch (d->test)
  {
    case kCheckReflectance: return check_tree_test<T, kCheckReflectance>(m, d, sx, sy, sz, acc, counts, partial, s);
    case kCheckReciprocity: return check_tree_test<T, kCheckReciprocity>(m, d, sx, sy, sz, acc, counts, partial, s);
    case kCheckAdjoint: return check_tree_test<T, kCheckAdjoint>(m, d, sx, sy, sz, acc, counts, partial, s);
    case kCheckPdf: return check_tree_test<T, kCheckPdf>(m, d, sx, sy, sz, acc, counts, partial, s);
    case kCheckPdfInt: return check_tree_test<T, kCheckPdfInt>(m, d, sx, sy, sz, acc, counts, partial, s);
    case kCheckSamplePdf: return check_tree_test<T, kCheckSamplePdf>(m, d, sx, sy, sz, acc, counts, partial, s);
    default: return check_tree_test<T, kCheckSampleCount>(m, d, sx, sy, sz, acc, counts, partial, s);
  }
}

}  // namespace
}  // namespace bbmhip

using namespace bbmhip;

extern "C" {

int bbm_hip_aggregate_eval_pdf(const bbm_hip_child* children, int nchildren, const float* in_x, const float* in_y,
                               const float* in_z, const float* out_x, const float* out_y, const float* out_z,
                               const uint8_t* mask, size_t n, uint32_t component, uint32_t unit, float* r, float* g,
                               float* b, float* pdf, void* stream)
{
  bool bsdf;
  Composite<float>::root(children, nchildren, bsdf);
  int rc = Composite<float>::check(children, nchildren);
  if (rc) return rc;
  if (!r && !pdf) return fail(BBM_HIP_ERR_INVALID_ARG, "no output requested (rgb and pdf are NULL)");
  if (r && (!g || !b)) return fail(BBM_HIP_ERR_INVALID_ARG, "eval output pointer is NULL");
  if (n == 0) return BBM_HIP_OK;
  return Composite<float>::eval_pdf(children, nchildren, bsdf, in_x, in_y, in_z, out_x, out_y, out_z, mask, n, component,
                                    unit, r, g, b, pdf, static_cast<hipStream_t>(stream));
}

int bbm_hip_aggregate_reflectance(const bbm_hip_child* children, int nchildren, const float* out_x,
                                  const float* out_y, const float* out_z, const uint8_t* mask, size_t n,
                                  uint32_t component, uint32_t unit, float* r, float* g, float* b, void* stream)
{
  bool bsdf;
  Composite<float>::root(children, nchildren, bsdf);
  int rc = Composite<float>::check(children, nchildren);
  if (rc) return rc;
  if (!r || !g || !b) return fail(BBM_HIP_ERR_INVALID_ARG, "output pointer is NULL");
  if (n == 0) return BBM_HIP_OK;
  return Composite<float>::reflectance(children, nchildren, bsdf, out_x, out_y, out_z, mask, n, component, unit, r, g, b,
                                       static_cast<hipStream_t>(stream));
}

int bbm_hip_aggregate_sample(const bbm_hip_child* children, int nchildren, const float* out_x, const float* out_y,
                             const float* out_z, const float* xi0, const float* xi1, const uint8_t* mask, size_t n,
                             uint32_t component, uint32_t unit, float* dir_x, float* dir_y, float* dir_z, float* pdf,
                             uint32_t* flag, void* stream)
{
  bool bsdf;
  Composite<float>::root(children, nchildren, bsdf);
  int rc = Composite<float>::check(children, nchildren);
  if (rc) return rc;
  if (!xi0 || !xi1 || !dir_x || !dir_y || !dir_z || !pdf || !flag)
    return fail(BBM_HIP_ERR_INVALID_ARG, "xi / output pointer is NULL");
  if (n == 0) return BBM_HIP_OK;
  return Composite<float>::sample(children, nchildren, bsdf, out_x, out_y, out_z, xi0, xi1, mask, n, component, unit, dir_x,
                                  dir_y, dir_z, pdf, flag, static_cast<hipStream_t>(stream));
}

int bbm_hip_aggregate_eval_pdf_f64(const bbm_hip_child_f64* children, int nchildren, const double* in_x,
                                   const double* in_y, const double* in_z, const double* out_x, const double* out_y,
                                   const double* out_z, const uint8_t* mask, size_t n, uint32_t component,
                                   uint32_t unit, double* r, double* g, double* b, double* pdf, void* stream)
{
  bool bsdf;
  Composite<double>::root(children, nchildren, bsdf);
  int rc = Composite<double>::check(children, nchildren);
  if (rc) return rc;
  if (!r && !pdf) return fail(BBM_HIP_ERR_INVALID_ARG, "no output requested (rgb and pdf are NULL)");
  if (r && (!g || !b)) return fail(BBM_HIP_ERR_INVALID_ARG, "eval output pointer is NULL");
  if (n == 0) return BBM_HIP_OK;
  return Composite<double>::eval_pdf(children, nchildren, bsdf, in_x, in_y, in_z, out_x, out_y, out_z, mask, n, component,
                                     unit, r, g, b, pdf, static_cast<hipStream_t>(stream));
}

int bbm_hip_aggregate_reflectance_f64(const bbm_hip_child_f64* children, int nchildren, const double* out_x,
                                      const double* out_y, const double* out_z, const uint8_t* mask, size_t n,
                                      uint32_t component, uint32_t unit, double* r, double* g, double* b, void* stream)
{
  bool bsdf;
  Composite<double>::root(children, nchildren, bsdf);
  int rc = Composite<double>::check(children, nchildren);
  if (rc) return rc;
  if (!r || !g || !b) return fail(BBM_HIP_ERR_INVALID_ARG, "output pointer is NULL");
  if (n == 0) return BBM_HIP_OK;
  return Composite<double>::reflectance(children, nchildren, bsdf, out_x, out_y, out_z, mask, n, component, unit, r, g, b,
                                        static_cast<hipStream_t>(stream));
}

int bbm_hip_aggregate_sample_f64(const bbm_hip_child_f64* children, int nchildren, const double* out_x,
                                 const double* out_y, const double* out_z, const double* xi0, const double* xi1,
                                 const uint8_t* mask, size_t n, uint32_t component, uint32_t unit, double* dir_x,
                                 double* dir_y, double* dir_z, double* pdf, uint32_t* flag, void* stream)
{
  bool bsdf;
  Composite<double>::root(children, nchildren, bsdf);
  int rc = Composite<double>::check(children, nchildren);
  if (rc) return rc;
  if (!xi0 || !xi1 || !dir_x || !dir_y || !dir_z || !pdf || !flag)
    return fail(BBM_HIP_ERR_INVALID_ARG, "xi / output pointer is NULL");
  if (n == 0) return BBM_HIP_OK;
  return Composite<double>::sample(children, nchildren, bsdf, out_x, out_y, out_z, xi0, xi1, mask, n, component, unit, dir_x,
                                   dir_y, dir_z, pdf, flag, static_cast<hipStream_t>(stream));
}

}  // extern "C"

extern "C" {

size_t bbm_hip_loss_tree_workspace_size(int nprobes, size_t n)
{
  return nprobes > 0 ? size_t(loss_tree_blocks(n)) * size_t(nprobes) * sizeof(double) : 0;
}

int bbm_hip_loss_tree(const bbm_hip_child* tree, int ntree, const float* probes, int nparams, int nprobes, size_t n,
                      const float* in_x, const float* in_y, const float* in_z, const float* out_x, const float* out_y,
                      const float* out_z, const float* ref_r, const float* ref_g, const float* ref_b, int loss_kind,
                      uint32_t component, uint32_t unit, double* sums, void* workspace, size_t workspace_bytes,
                      void* stream)
{
  const float* in[3] = {in_x, in_y, in_z};
  const float* out[3] = {out_x, out_y, out_z};
  const float* ref[3] = {ref_r, ref_g, ref_b};
  return loss_tree<float>(tree, ntree, probes, nparams, nprobes, n, in, out, ref, loss_kind, component & kFlagAll, unit,
                          sums, workspace, workspace_bytes, static_cast<hipStream_t>(stream));
}

int bbm_hip_loss_tree_f64(const bbm_hip_child_f64* tree, int ntree, const double* probes, int nparams, int nprobes,
                          size_t n, const double* in_x, const double* in_y, const double* in_z, const double* out_x,
                          const double* out_y, const double* out_z, const double* ref_r, const double* ref_g,
                          const double* ref_b, int loss_kind, uint32_t component, uint32_t unit, double* sums,
                          void* workspace, size_t workspace_bytes, void* stream)
{
  const double* in[3] = {in_x, in_y, in_z};
  const double* out[3] = {out_x, out_y, out_z};
  const double* ref[3] = {ref_r, ref_g, ref_b};
  return loss_tree<double>(tree, ntree, probes, nparams, nprobes, n, in, out, ref, loss_kind, component & kFlagAll, unit,
                           sums, workspace, workspace_bytes, static_cast<hipStream_t>(stream));
}

size_t bbm_hip_check_tree_workspace_size(const bbm_hip_check_desc* desc) { return check_tree_ws(desc); }

int bbm_hip_check_tree(const bbm_hip_child* tree, int ntree, const bbm_hip_check_desc* desc, double* acc,
                       uint64_t* counts, void* workspace, size_t workspace_bytes, void* stream)
{
  return check_tree<float>(tree, ntree, desc, desc ? desc->slot_x : nullptr, desc ? desc->slot_y : nullptr,
                           desc ? desc->slot_z : nullptr, acc, counts, workspace, workspace_bytes,
                           static_cast<hipStream_t>(stream));
}

int bbm_hip_check_tree_f64(const bbm_hip_child_f64* tree, int ntree, const bbm_hip_check_desc* desc,
                           const double* slot_x, const double* slot_y, const double* slot_z, double* acc,
                           uint64_t* counts, void* workspace, size_t workspace_bytes, void* stream)
{
  return check_tree<double>(tree, ntree, desc, slot_x, slot_y, slot_z, acc, counts, workspace, workspace_bytes,
                            static_cast<hipStream_t>(stream));
}

}  // extern "C"
