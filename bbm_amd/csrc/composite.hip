// bbm_amd/csrc/composite.hip -- aggregatemodel<MODELS...> of ANY registered models (include/bsdfmodel/
// aggregatemodel.h:22-222), evaluated by composing the children's own kernels.
//
// The fused Aggregate<Lambertian, X> entries of the registry (aggregate.hpp) evaluate the published fits' form in
// one kernel; this unit covers every other composition -- any number of children, any registered single models
// (or fused aggregates) as children -- at the price of one pass per child over the batch:
//   eval        = MODELS::eval(...) + ...   a right fold: e0 + (e1 + (e2 + ...))                    (:61-64)
//   pdf         = inner_product(pdfs, weights, 0) / accumulate(weights, 0), 0 unless sum > eps,
//                 weight_k = hsum(reflectance_k(out)) = ((0 + r) + g) + b                           (:129-143)
//   sample      = child k chosen where xi0 * sum falls in [0, w_k] after subtracting w_0..w_{k-1} (a later
//                 child claiming the lane wins), sampled with xi0' = that offset / w_k (0 unless w_k > eps);
//                 pdf as above at the sampled direction                                              (:81-113)
//   reflectance = MODELS::reflectance(...) + ...  (right fold)                                       (:156-163)
// Each child runs through the public entry points (its registry kernel, its own host-side preparation such as
// the He family's CDF); the small kernels below only combine per-lane results in the reference's order and
// rounding.  Scratch is stream-ordered (scratch_acquire / scratch_release): no host synchronisation.
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

unsigned grid(size_t n)
{
  const size_t b = (n + kB - 1) / kB;
  return unsigned(b < 1 ? 1 : (b > (1u << 20) ? (1u << 20) : b));
}

#define BBM_GRID_LOOP(i, n) \
  for (uint64_t i = uint64_t(blockIdx.x) * kB + threadIdx.x; i < (n); i += uint64_t(gridDim.x) * kB)

// acc = t + acc (the fold's next term on the left)
__global__ __launch_bounds__(kB) void k_fold3(const float* tr, const float* tg, const float* tb, float* r, float* g,
                                              float* b, uint64_t n)
{
  BBM_GRID_LOOP(i, n) { r[i] = tr[i] + r[i]; g[i] = tg[i] + g[i]; b[i] = tb[i] + b[i]; }
}

// w_k = hsum(reflectance_k) and sum = sum + w_k (forward, from 0)
__global__ __launch_bounds__(kB) void k_weight(const float* r, const float* g, const float* b, float* w, float* sum,
                                               uint64_t n, int first)
{
  BBM_GRID_LOOP(i, n)
  {
    const float wk = ((0.0f + r[i]) + g[i]) + b[i];
    w[i] = wk;
    sum[i] = (first ? 0.0f : sum[i]) + wk;
  }
}

// ip = ip + p_k w_k (forward, from 0)
__global__ __launch_bounds__(kB) void k_inner(const float* p, const float* w, float* ip, uint64_t n, int first)
{
  BBM_GRID_LOOP(i, n) ip[i] = (first ? 0.0f : ip[i]) + p[i] * w[i];
}

// pdf = select(sum > eps, ip / sum, 0) -- the float division of Value operands
__global__ __launch_bounds__(kB) void k_mix(const float* ip, const float* sum, float* pdf, uint64_t n)
{
  BBM_GRID_LOOP(i, n) pdf[i] = (sum[i] > kEpsF) ? ip[i] / sum[i] : 0.0f;
}

// child selection of aggregatemodel::sample (:92-109): chosen = the last child claiming the lane (-1: none),
// xs = its rescaled xi0
__global__ __launch_bounds__(kB) void k_select(const float* w, int nchild, const float* sum, const float* xi0,
                                               const uint8_t* mask, int8_t* chosen, float* xs, uint64_t n)
{
  BBM_GRID_LOOP(i, n)
  {
    const bool m0 = mask ? (mask[i] != 0) : true;
    float x = xi0[i] * sum[i];
    int c = -1;
    float nx = 0.0f;
    for (int k = 0; k < nchild; ++k)
    {
      const float wk = w[size_t(k) * n + i];
      const bool m = m0 && (x >= 0) && (x <= wk);
      if (m) { c = k; nx = (wk > kEpsF) ? x / wk : 0.0f; }
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

__global__ __launch_bounds__(kB) void k_zero_sample(float* x, float* y, float* z, uint32_t* flag, uint64_t n)
{
  BBM_GRID_LOOP(i, n) { x[i] = 0.0f; y[i] = 0.0f; z[i] = 0.0f; flag[i] = kFlagNone; }
}

__global__ __launch_bounds__(kB) void k_take(const int8_t* chosen, int k, const float* tx, const float* ty,
                                             const float* tz, const uint32_t* tf, float* x, float* y, float* z,
                                             uint32_t* flag, uint64_t n)
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

int check_children(const bbm_hip_child* c, int nchild)
{
  if (!c || nchild < 2) return fail(BBM_HIP_ERR_INVALID_ARG, "an aggregate needs at least two children");
  if (nchild > 127) return fail(BBM_HIP_ERR_INVALID_ARG, "at most 127 children");
  for (int k = 0; k < nchild; ++k)
  {
    const int np = bbm_hip_model_nparams(c[k].model_id);
    if (np < 0) return np;
    if (c[k].nparams != np || !c[k].params)
      return fail(BBM_HIP_ERR_INVALID_ARG, "child " + std::to_string(k) + ": expected " + std::to_string(np) + " parameters");
  }
  return BBM_HIP_OK;
}

int launched()
{
  const hipError_t e = hipGetLastError();
  return (e == hipSuccess) ? BBM_HIP_OK : fail(BBM_HIP_ERR_HIP, std::string("kernel launch failed: ") + hipGetErrorString(e));
}

// weights w (nchild x n) and their sum for directions `out`
int weights(const bbm_hip_child* c, int nchild, const float* ox, const float* oy, const float* oz, const uint8_t* mask,
            size_t n, uint32_t component, uint32_t unit, float* w, float* sum, float* tr, float* tg, float* tb,
            hipStream_t s)
{
  for (int k = 0; k < nchild; ++k)
  {
    int rc = bbm_hip_reflectance(c[k].model_id, c[k].params, c[k].nparams, ox, oy, oz, mask, n, component, unit, tr, tg,
                                 tb, s);
    if (rc) return rc;
    hipLaunchKernelGGL(k_weight, dim3(grid(n)), dim3(kB), 0, s, tr, tg, tb, w + size_t(k) * n, sum, uint64_t(n),
                       int(k == 0));
    if ((rc = launched())) return rc;
  }
  return BBM_HIP_OK;
}

// pdf = mixture of the children's pdfs at (in, out) with weights w / sum
int mixture_pdf(const bbm_hip_child* c, int nchild, const float* ix, const float* iy, const float* iz, const float* ox,
                const float* oy, const float* oz, const uint8_t* mask, size_t n, uint32_t component, uint32_t unit,
                const float* w, const float* sum, float* tp, float* ip, float* pdf, hipStream_t s)
{
  for (int k = 0; k < nchild; ++k)
  {
    int rc = bbm_hip_pdf(c[k].model_id, c[k].params, c[k].nparams, ix, iy, iz, ox, oy, oz, mask, n, component, unit, tp, s);
    if (rc) return rc;
    hipLaunchKernelGGL(k_inner, dim3(grid(n)), dim3(kB), 0, s, tp, w + size_t(k) * n, ip, uint64_t(n), int(k == 0));
    if ((rc = launched())) return rc;
  }
  hipLaunchKernelGGL(k_mix, dim3(grid(n)), dim3(kB), 0, s, ip, sum, pdf, uint64_t(n));
  return launched();
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
  int rc = check_children(children, nchildren);
  if (rc) return rc;
  if (!r && !pdf) return fail(BBM_HIP_ERR_INVALID_ARG, "no output requested (rgb and pdf are NULL)");
  if (r && (!g || !b)) return fail(BBM_HIP_ERR_INVALID_ARG, "eval output pointer is NULL");
  if (n == 0) return BBM_HIP_OK;
  const hipStream_t s = static_cast<hipStream_t>(stream);
  Scratch sc(s);
  float* tr = sc.get<float>(n);
  float* tg = sc.get<float>(n);
  float* tb = sc.get<float>(n);
  if (!tr || !tg || !tb) return fail(BBM_HIP_ERR_HIP, "aggregate: scratch allocation failed");
  if (r)
  {
    // right fold: the last child straight into the output, then e_k + acc for k = K-2 .. 0
    const int last = nchildren - 1;
    if ((rc = bbm_hip_eval(children[last].model_id, children[last].params, children[last].nparams, in_x, in_y, in_z,
                           out_x, out_y, out_z, mask, n, component, unit, r, g, b, stream)))
      return rc;
    for (int k = last - 1; k >= 0; --k)
    {
      if ((rc = bbm_hip_eval(children[k].model_id, children[k].params, children[k].nparams, in_x, in_y, in_z, out_x,
                             out_y, out_z, mask, n, component, unit, tr, tg, tb, stream)))
        return rc;
      hipLaunchKernelGGL(k_fold3, dim3(grid(n)), dim3(kB), 0, s, tr, tg, tb, r, g, b, uint64_t(n));
      if ((rc = launched())) return rc;
    }
  }
  if (pdf)
  {
    float* w = sc.get<float>(size_t(nchildren) * n);
    float* sum = sc.get<float>(n);
    float* ip = sc.get<float>(n);
    if (!w || !sum || !ip) return fail(BBM_HIP_ERR_HIP, "aggregate: scratch allocation failed");
    if ((rc = weights(children, nchildren, out_x, out_y, out_z, mask, n, component, unit, w, sum, tr, tg, tb, s))) return rc;
    if ((rc = mixture_pdf(children, nchildren, in_x, in_y, in_z, out_x, out_y, out_z, mask, n, component, unit, w, sum, tr,
                          ip, pdf, s)))
      return rc;
  }
  return BBM_HIP_OK;
}

int bbm_hip_aggregate_reflectance(const bbm_hip_child* children, int nchildren, const float* out_x,
                                  const float* out_y, const float* out_z, const uint8_t* mask, size_t n,
                                  uint32_t component, uint32_t unit, float* r, float* g, float* b, void* stream)
{
  int rc = check_children(children, nchildren);
  if (rc) return rc;
  if (!r || !g || !b) return fail(BBM_HIP_ERR_INVALID_ARG, "output pointer is NULL");
  if (n == 0) return BBM_HIP_OK;
  const hipStream_t s = static_cast<hipStream_t>(stream);
  Scratch sc(s);
  float* tr = sc.get<float>(n);
  float* tg = sc.get<float>(n);
  float* tb = sc.get<float>(n);
  if (!tr || !tg || !tb) return fail(BBM_HIP_ERR_HIP, "aggregate: scratch allocation failed");
  const int last = nchildren - 1;
  if ((rc = bbm_hip_reflectance(children[last].model_id, children[last].params, children[last].nparams, out_x, out_y,
                                out_z, mask, n, component, unit, r, g, b, stream)))
    return rc;
  for (int k = last - 1; k >= 0; --k)
  {
    if ((rc = bbm_hip_reflectance(children[k].model_id, children[k].params, children[k].nparams, out_x, out_y, out_z,
                                  mask, n, component, unit, tr, tg, tb, stream)))
      return rc;
    hipLaunchKernelGGL(k_fold3, dim3(grid(n)), dim3(kB), 0, s, tr, tg, tb, r, g, b, uint64_t(n));
    if ((rc = launched())) return rc;
  }
  return BBM_HIP_OK;
}

int bbm_hip_aggregate_sample(const bbm_hip_child* children, int nchildren, const float* out_x, const float* out_y,
                             const float* out_z, const float* xi0, const float* xi1, const uint8_t* mask, size_t n,
                             uint32_t component, uint32_t unit, float* dir_x, float* dir_y, float* dir_z, float* pdf,
                             uint32_t* flag, void* stream)
{
  int rc = check_children(children, nchildren);
  if (rc) return rc;
  if (!xi0 || !xi1 || !dir_x || !dir_y || !dir_z || !pdf || !flag)
    return fail(BBM_HIP_ERR_INVALID_ARG, "xi / output pointer is NULL");
  if (n == 0) return BBM_HIP_OK;
  const hipStream_t s = static_cast<hipStream_t>(stream);
  Scratch sc(s);
  float* w = sc.get<float>(size_t(nchildren) * n);
  float* sum = sc.get<float>(n);
  float* ip = sc.get<float>(n);
  float* t0 = sc.get<float>(n);
  float* t1 = sc.get<float>(n);
  float* t2 = sc.get<float>(n);
  float* t3 = sc.get<float>(n);
  uint32_t* tf = sc.get<uint32_t>(n);
  int8_t* chosen = sc.get<int8_t>(n);
  uint8_t* cm = sc.get<uint8_t>(n);
  float* xs = sc.get<float>(n);
  if (!w || !sum || !ip || !t0 || !t1 || !t2 || !t3 || !tf || !chosen || !cm || !xs)
    return fail(BBM_HIP_ERR_HIP, "aggregate: scratch allocation failed");
  if ((rc = weights(children, nchildren, out_x, out_y, out_z, mask, n, component, unit, w, sum, t0, t1, t2, s))) return rc;
  hipLaunchKernelGGL(k_select, dim3(grid(n)), dim3(kB), 0, s, w, nchildren, sum, xi0, mask, chosen, xs, uint64_t(n));
  hipLaunchKernelGGL(k_zero_sample, dim3(grid(n)), dim3(kB), 0, s, dir_x, dir_y, dir_z, flag, uint64_t(n));
  if ((rc = launched())) return rc;
  for (int k = 0; k < nchildren; ++k)
  {
    hipLaunchKernelGGL(k_child_mask, dim3(grid(n)), dim3(kB), 0, s, chosen, k, cm, uint64_t(n));
    if ((rc = launched())) return rc;
    if ((rc = bbm_hip_sample(children[k].model_id, children[k].params, children[k].nparams, out_x, out_y, out_z, xs, xi1,
                             cm, n, component, unit, t0, t1, t2, t3, tf, stream)))
      return rc;
    hipLaunchKernelGGL(k_take, dim3(grid(n)), dim3(kB), 0, s, chosen, k, t0, t1, t2, tf, dir_x, dir_y, dir_z, flag,
                       uint64_t(n));
    if ((rc = launched())) return rc;
  }
  // pdf of the sampled direction: the weighted mixture of every child's pdf (:111-112)
  return mixture_pdf(children, nchildren, dir_x, dir_y, dir_z, out_x, out_y, out_z, mask, n, component, unit, w, sum,
                     t3, ip, pdf, s);
}

}  // extern "C"
