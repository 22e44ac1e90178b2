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

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/bbm_hip.h"
#include "math.hpp"

namespace bbmhip {
int fail(int code, const std::string& msg);
void* scratch_acquire(size_t bytes, hipStream_t s);
void scratch_release(void* p, hipStream_t s);

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
  BBM_GRID_LOOP(i, n) { r[i] = tr[i] + r[i]; g[i] = tg[i] + g[i]; b[i] = tb[i] + b[i]; }
}

// aggregatebsdf's left fold (aggregatebsdf.h:79-83, :209-212): acc = (first ? 0 + acc : acc) + t, forward
template<class T>
__global__ __launch_bounds__(kB) void k_lfold3(const T* tr, const T* tg, const T* tb, T* r, T* g, T* b, uint64_t n,
                                               int first)
{
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
  BBM_GRID_LOOP(i, n) ip[i] = (first ? T(0) : ip[i]) + (w[i] * p[i]) / sum[i];
}

template<class T>
__global__ __launch_bounds__(kB) void k_mask_sum(const T* ip, const T* sum, T* pdf, uint64_t n)
{
  BBM_GRID_LOOP(i, n) pdf[i] = (sum[i] > eps_of<T>()) ? ip[i] : T(0);
}

// w_k = hsum(reflectance_k) and sum = sum + w_k (forward, from 0)
template<class T>
__global__ __launch_bounds__(kB) void k_weight(const T* r, const T* g, const T* b, T* w, T* sum, uint64_t n, int first)
{
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
  BBM_GRID_LOOP(i, n) ip[i] = (first ? T(0) : ip[i]) + p[i] * w[i];
}

// pdf = select(sum > eps, ip / sum, 0) -- the IEEE division of Value operands
template<class T>
__global__ __launch_bounds__(kB) void k_mix(const T* ip, const T* sum, T* pdf, uint64_t n)
{
  BBM_GRID_LOOP(i, n) pdf[i] = (sum[i] > eps_of<T>()) ? ip[i] / sum[i] : T(0);
}

// child selection of aggregatemodel::sample (:92-113): chosen = the last child claiming the lane (-1: none),
// xs = its rescaled xi0
template<class T>
__global__ __launch_bounds__(kB) void k_select(const T* w, int nchild, const T* sum, const T* xi0, const uint8_t* mask,
                                               int8_t* chosen, T* xs, uint64_t n, int bsdf)
{
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
  BBM_GRID_LOOP(i, n) m[i] = (chosen[i] == k) ? 1 : 0;
}

template<class T>
__global__ __launch_bounds__(kB) void k_zero_sample(T* x, T* y, T* z, uint32_t* flag, uint64_t n)
{
  BBM_GRID_LOOP(i, n) { x[i] = T(0); y[i] = T(0); z[i] = T(0); flag[i] = kFlagNone; }
}

template<class T>
__global__ __launch_bounds__(kB) void k_take(const int8_t* chosen, int k, const T* tx, const T* ty, const T* tz,
                                             const uint32_t* tf, T* x, T* y, T* z, uint32_t* flag, uint64_t n)
{
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
    if (!p) return fail(BBM_HIP_ERR_HIP, "aggregate: scratch allocation failed");
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
    if (!r || !g || !b) return fail(BBM_HIP_ERR_HIP, "aggregate: scratch allocation failed");
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
    if (!tr || !tg || !tb) return fail(BBM_HIP_ERR_HIP, "aggregate: scratch allocation failed");
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
      if (!w || !sum || !ip) return fail(BBM_HIP_ERR_HIP, "aggregate: scratch allocation failed");
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
    if (!tr || !tg || !tb) return fail(BBM_HIP_ERR_HIP, "aggregate: scratch allocation failed");
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
      return fail(BBM_HIP_ERR_HIP, "aggregate: scratch allocation failed");
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
