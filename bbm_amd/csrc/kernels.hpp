// bbm_amd/csrc/kernels.hpp -- the streaming kernels and their host-side launchers, templated on
// the model composition.  Included by the per-family instantiation units (inst_*.hip), which
// explicitly instantiate launch_eval_pdf<M> / launch_sample<M> for their models, and by the
// registry unit (bbm_hip.hip), which only takes their addresses (extern template).
//
// Layout and launch: directions are SoA float32 in HBM; one thread owns four
// consecutive pairs, so each lane issues one 16-byte load per input array and one 16-byte store
// per output array -- every wave instruction moves a full 1 KiB, coalesced.  The grid covers the
// batch (one 256-thread workgroup per 1024 pairs); work is per-pair independent, so no LDS, no
// atomics and no inter-workgroup traffic are needed.  Parameters are passed by value in the
// kernarg segment and stay in SGPRs.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <string>

#include "../../include/bbm_hip.h"
#include "math.hpp"
#include "microfacet.hpp"
#include "fit.hpp"

namespace bbmhip {

constexpr int kMaxParams = 64;
constexpr int kBlock = 256;
constexpr int kMaxBlocks = 1 << 22;   // effectively one workgroup per 1024 pairs (full grid)

// Record `msg` as the calling thread's last error (bbm_hip_last_error) and return `code`.
int fail(int code, const std::string& msg);

// Stream-ordered device scratch (bbm_hip.hip): per-launch derived data (the tabulated samplers' CDFs) and the
// composed aggregates' per-lane temporaries.  A released block keeps an event recorded on the releasing
// stream; re-acquiring it on the same stream needs nothing (stream order), on another stream that stream
// waits for the event on the GPU.  No host synchronisation; blocks are kept for reuse.  (Replaces
// hipMallocAsync / hipFreeAsync on the caller's stream, under which tests/cpp/adapter_check -- a plain C++
// host program on the null stream -- saw He CDFs and composed-aggregate outputs corrupted at random.)
void* scratch_acquire(size_t bytes, hipStream_t s);
std::string scratch_failure();   // why the calling thread's last scratch_acquire returned nullptr
void scratch_release(void* p, hipStream_t s);

struct ParamBlock { float v[kMaxParams]; };

// a device address riding in two parameter slots (bit pattern of a 64-bit pointer): per-launch derived data such as
// the He family's sampler CDF or EPD's shadowing-table row pair (host_params below)
__host__ __device__ __forceinline__ const float* param_ptr(const float* p, int slot)
{
  uint32_t lo, hi;
  __builtin_memcpy(&lo, p + slot, 4);
  __builtin_memcpy(&hi, p + slot + 1, 4);
  return reinterpret_cast<const float*>((uint64_t(hi) << 32) | lo);
}
inline void set_param_ptr(float* p, int slot, const void* ptr)
{
  const uint64_t v = reinterpret_cast<uint64_t>(ptr);
  const uint32_t lo = uint32_t(v), hi = uint32_t(v >> 32);
  __builtin_memcpy(p + slot, &lo, 4);
  __builtin_memcpy(p + slot + 1, &hi, 4);
}

// Per-model host work before a launch (e.g. building a lookup table on first use); no-op by default.
template<class Model> struct host_prepare { static int run(hipStream_t) { return 0; } };

// Per-launch check of a parameter block before anything is enqueued (e.g. a table address that must be set);
// no-op by default.
template<class Model> struct host_validate { static int run(const ParamBlock&) { return 0; } };

// Per-launch derived data a model's sample / pdf need (e.g. a data-driven sampling CDF), enqueued on the
// launch stream and passed in the parameter block after the model's own parameters; `done` releases the
// stream-ordered scratch after the launch.  No-op by default.
template<class Model> struct host_params
{
  static int run(ParamBlock&, uint32_t, hipStream_t, void**) { return 0; }
  static void done(void*, hipStream_t) {}
};

struct EvalArgs
{
  const float* ix; const float* iy; const float* iz;
  const float* ox; const float* oy; const float* oz;
  const uint8_t* mask;
  float* r; float* g; float* b; float* pdf;
  uint64_t n;
  uint32_t component;
  ParamBlock p;
};

// exact mode (model_has_exact / model_eval_pdf: math.hpp)

// process-wide switch (bbm_hip_set_exact_subnormals; initial value from BBM_HIP_EXACT_SUBNORMALS)
inline std::atomic<int>& exact_subnormals()
{
  static std::atomic<int> v{[] {
    const char* e = std::getenv("BBM_HIP_EXACT_SUBNORMALS");
    return (e && std::atoi(e) != 0) ? 1 : 0;
  }()};
  return v;
}

// per-call override (BBM_HIP_CALL_EXACT / BBM_HIP_CALL_DEFAULT OR-ed into a model id): -1 = follow the process-wide
// switch.  Thread-local and scoped to the entry point that decoded the id (CallExactScope), so concurrent calls
// from different threads never see each other's mode; the launches are enqueued on the calling thread.
inline thread_local int t_call_exact = -1;
inline bool exact_on() { return t_call_exact >= 0 ? t_call_exact != 0 : exact_subnormals().load() != 0; }
struct CallExactScope
{
  int prev;
  explicit CallExactScope(int id) : prev(t_call_exact)
  {
    if (id >= 0 && (id & BBM_HIP_CALL_EXACT)) t_call_exact = 1;
    else if (id >= 0 && (id & BBM_HIP_CALL_DEFAULT)) t_call_exact = 0;
  }
  ~CallExactScope() { t_call_exact = prev; }
  CallExactScope(const CallExactScope&) = delete;
  CallExactScope& operator=(const CallExactScope&) = delete;
};

template<class Model> inline bool exact_launch() { return model_has_exact<Model>() && exact_on(); }

template<class Model, int MODE, bool EXACT = false>
__device__ __forceinline__ void one_pair(const Model& m, const EvalArgs& a, uint64_t i, bool active)
{
  float rgb[3], pdf;
  const v3 in = mk3(a.ix[i], a.iy[i], a.iz[i]);
  const v3 out = mk3(a.ox[i], a.oy[i], a.oz[i]);
  model_eval_pdf<MODE, EXACT>(m, in, out, active ? a.component : 0u, rgb, pdf);
  if (MODE & kModeEval) { a.r[i] = rgb[0]; a.g[i] = rgb[1]; a.b[i] = rgb[2]; }
  if (MODE & kModePdf) a.pdf[i] = pdf;
}

// Vector path: 4 consecutive pairs per thread-iteration, 16-byte loads/stores per array.
// Requires every array 16-byte aligned (checked on the host); the n % 4 tail runs scalar.
typedef float f4 __attribute__((ext_vector_type(4)));

template<bool NT>
__device__ __forceinline__ float4 ld4(const float* p, uint64_t t)
{
  if (NT)
  {
    const f4 v = __builtin_nontemporal_load(reinterpret_cast<const f4*>(p) + t);
    return make_float4(v.x, v.y, v.z, v.w);
  }
  return reinterpret_cast<const float4*>(p)[t];
}

template<bool NT>
__device__ __forceinline__ void st4(float* p, uint64_t t, float a, float b, float c, float d)
{
  if (NT) __builtin_nontemporal_store(f4{a, b, c, d}, reinterpret_cast<f4*>(p) + t);
  else reinterpret_cast<float4*>(p)[t] = make_float4(a, b, c, d);
}

#ifndef BBM_HIP_SGPR_LIMIT
#define BBM_HIP_KERNEL_ATTR
#else
// Cap the SGPR budget: 256-thread workgroups are admitted per CU only up to
// floor(800 / (ceil(sgpr/16)*16 + 16)) (MI355X_MICROARCH.md, Residency) -- 98 SGPRs = 6 per CU.
#define BBM_HIP_KERNEL_ATTR __attribute__((amdgpu_num_sgpr(BBM_HIP_SGPR_LIMIT)))
#endif

// Minimum waves per SIMD the eval kernels are compiled for (amdgpu_waves_per_eu: caps the VGPRs at 512 / N); 1 =
// the compiler's choice.  Raised per model where a VALU-bound evaluation would otherwise hold two or three waves
// per SIMD (too few to hide the f64 / transcendental latencies).
template<class Model> struct eval_waves { static constexpr int value = 1; };

// Whether k_eval_pdf_v4 issues a thread's first quad of loads before the LDS table prologue and the model's
// construction (their latencies then overlap; the loaded registers stay live across both).  Measured (ms, 100 M /
// 10 M pairs, profiles/r05_ab_prefetch.txt): CookTorrance headline 0.727 -> 0.700, AshikhminShirley 0.0655 -> 0.0621;
// Bagher, whose constructor holds ~40 registers of channel setup, 0.125 -> 0.131 -- off for it.
#ifdef BBM_HIP_NO_PREFETCH
template<class Model> struct eval_prefetch { static constexpr bool value = false; };   // A/B
#else
template<class Model> struct eval_prefetch { static constexpr bool value = true; };
#endif

// Whether a model's evaluation reads the glibc tables (math.hpp expf / logf / powf and what is built on them): the
// eval kernel skips the LDS prologue for the models declared table-free (models.hpp: Lambertian, GGX, GGXHeitz and
// their aggregate), which paid 3-4 % for it (profiles/r05_ab_lds_tables.txt).  Checked by a poisoned build
// (-DBBM_HIP_TABLES_POISON: NaN tables instead of none) under the parity tests.
template<class Model> struct uses_math_tables { static constexpr bool value = true; };

// Software pipelining of k_eval_pdf_v4's grid-stride loop: the next quad's six loads are issued before the current
// quad is evaluated, so a thread's HBM latency hides under its own compute (with a capped grid, eval_grid_cap, every
// thread runs several iterations).  For the latency-bound models whose waves otherwise all wait on their loads at
// the same time.
template<class Model> struct eval_pipeline { static constexpr bool value = false; };

// Grid cap of the eval kernels (0 = a full grid, one workgroup per 1024 pairs).  The model is constructed once per
// thread from the kernarg parameters; where that constructor is expensive (the Student-T NDF's two tgamma and a pow
// per thread) a capped grid-stride launch amortises it over several iterations.
template<class Model> struct eval_grid_cap { static constexpr uint64_t value = 0; };

template<class Model, int MODE, bool MASK, bool NT, bool EXACT = false>
__global__ __launch_bounds__(kBlock) BBM_HIP_KERNEL_ATTR __attribute__((amdgpu_waves_per_eu(eval_waves<Model>::value, 8)))
void k_eval_pdf_v4(EvalArgs a)
{
  const uint64_t n4 = a.n >> 2;
  const uint64_t stride = uint64_t(gridDim.x) * kBlock;
  uint64_t t = uint64_t(blockIdx.x) * kBlock + threadIdx.x;
  // the first quad's loads go out before the table prologue and the model's construction, so their latencies hide
  // under the loads' (most threads of a full grid run exactly one iteration; eval_prefetch)
  float4 ix, iy, iz, ox, oy, oz;
  uint32_t mk = 0x01010101u;
  const auto load = [&](uint64_t q) {
    ix = ld4<NT>(a.ix, q); iy = ld4<NT>(a.iy, q); iz = ld4<NT>(a.iz, q);
    ox = ld4<NT>(a.ox, q); oy = ld4<NT>(a.oy, q); oz = ld4<NT>(a.oz, q);
    if (MASK) mk = reinterpret_cast<const uint32_t*>(a.mask)[q];
  };
  constexpr bool pipe = eval_pipeline<Model>::value;
  constexpr bool pf = eval_prefetch<Model>::value || pipe;
  if (pf && t < n4) load(t);
  if constexpr (uses_math_tables<Model>::value) math_tables_init();
#ifdef BBM_HIP_TABLES_POISON
  else math_tables_poison();
#endif
  const Model m(a.p.v);
  for (bool first = true; t < n4; t += stride, first = false)
  {
    float4 nix, niy, niz, nox, noy, noz;
    uint32_t nmk = 0x01010101u;
    if constexpr (pipe)
    {
      // the next iteration's quad (clamped: every lane loads, the last iteration's loads are discarded)
      const uint64_t q = (t + stride < n4) ? t + stride : t;
      nix = ld4<NT>(a.ix, q); niy = ld4<NT>(a.iy, q); niz = ld4<NT>(a.iz, q);
      nox = ld4<NT>(a.ox, q); noy = ld4<NT>(a.oy, q); noz = ld4<NT>(a.oz, q);
      if (MASK) nmk = reinterpret_cast<const uint32_t*>(a.mask)[q];
    }
    else if (!pf || !first) load(t);
    const float inx[4] = {ix.x, ix.y, ix.z, ix.w}, iny[4] = {iy.x, iy.y, iy.z, iy.w}, inz[4] = {iz.x, iz.y, iz.z, iz.w};
    const float onx[4] = {ox.x, ox.y, ox.z, ox.w}, ony[4] = {oy.x, oy.y, oy.z, oy.w}, onz[4] = {oz.x, oz.y, oz.z, oz.w};
    float r[4], g[4], b[4], p[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
    {
      float rgb[3];
      const uint32_t comp = ((mk >> (8 * j)) & 0xffu) ? a.component : 0u;
      model_eval_pdf<MODE, EXACT>(m, mk3(inx[j], iny[j], inz[j]), mk3(onx[j], ony[j], onz[j]), comp, rgb, p[j]);
      r[j] = rgb[0]; g[j] = rgb[1]; b[j] = rgb[2];
    }
    if (MODE & kModeEval)
    {
      st4<NT>(a.r, t, r[0], r[1], r[2], r[3]);
      st4<NT>(a.g, t, g[0], g[1], g[2], g[3]);
      st4<NT>(a.b, t, b[0], b[1], b[2], b[3]);
    }
    if (MODE & kModePdf) st4<NT>(a.pdf, t, p[0], p[1], p[2], p[3]);
    if constexpr (pipe)
    {
      ix = nix; iy = niy; iz = niz; ox = nox; oy = noy; oz = noz;
      mk = nmk;
    }
  }
  // tail
  if (blockIdx.x == 0 && threadIdx.x < (a.n & 3))
  {
    const uint64_t i = (n4 << 2) + threadIdx.x;
    one_pair<Model, MODE, EXACT>(m, a, i, MASK ? (a.mask[i] != 0) : true);
  }
}

// Eight pairs per thread: two quads, each a fully coalesced 1 KiB wave access (quad t and quad
// t + 64 within the wave's 128-quad tile).  More independent work per wave for the scheduler.
template<class Model, int MODE, bool MASK, bool NT>
__global__ __launch_bounds__(kBlock) BBM_HIP_KERNEL_ATTR void k_eval_pdf_v8(EvalArgs a)
{
  math_tables_init();
  const Model m(a.p.v);
  const uint64_t n4 = a.n >> 2;
  const uint64_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t stride = uint64_t(gridDim.x) * (2 * kBlock);
  for (uint64_t base = uint64_t(blockIdx.x) * (2 * kBlock) + wave * 128; base < n4; base += stride)
  {
    uint64_t tq[2] = {base + lane, base + 64 + lane};
    float4 c[2][6];
    uint32_t cm[2] = {0x01010101u, 0x01010101u};
#pragma unroll
    for (int u = 0; u < 2; ++u)
    {
      const uint64_t t = tq[u] < n4 ? tq[u] : n4 - 1;
      c[u][0] = ld4<NT>(a.ix, t); c[u][1] = ld4<NT>(a.iy, t); c[u][2] = ld4<NT>(a.iz, t);
      c[u][3] = ld4<NT>(a.ox, t); c[u][4] = ld4<NT>(a.oy, t); c[u][5] = ld4<NT>(a.oz, t);
      if (MASK) cm[u] = reinterpret_cast<const uint32_t*>(a.mask)[t];
    }
    float r[2][4], g[2][4], b[2][4], p[2][4];
#pragma unroll
    for (int u = 0; u < 2; ++u)
    {
      const float inx[4] = {c[u][0].x, c[u][0].y, c[u][0].z, c[u][0].w}, iny[4] = {c[u][1].x, c[u][1].y, c[u][1].z, c[u][1].w};
      const float inz[4] = {c[u][2].x, c[u][2].y, c[u][2].z, c[u][2].w}, onx[4] = {c[u][3].x, c[u][3].y, c[u][3].z, c[u][3].w};
      const float ony[4] = {c[u][4].x, c[u][4].y, c[u][4].z, c[u][4].w}, onz[4] = {c[u][5].x, c[u][5].y, c[u][5].z, c[u][5].w};
#pragma unroll
      for (int j = 0; j < 4; ++j)
      {
        float rgb[3];
        const uint32_t comp = ((cm[u] >> (8 * j)) & 0xffu) ? a.component : 0u;
        m.template eval_pdf<MODE>(mk3(inx[j], iny[j], inz[j]), mk3(onx[j], ony[j], onz[j]), comp, rgb, p[u][j]);
        r[u][j] = rgb[0]; g[u][j] = rgb[1]; b[u][j] = rgb[2];
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
    {
      if (tq[u] >= n4) continue;
      const uint64_t t = tq[u];
      if (MODE & kModeEval)
      {
        st4<NT>(a.r, t, r[u][0], r[u][1], r[u][2], r[u][3]);
        st4<NT>(a.g, t, g[u][0], g[u][1], g[u][2], g[u][3]);
        st4<NT>(a.b, t, b[u][0], b[u][1], b[u][2], b[u][3]);
      }
      if (MODE & kModePdf) st4<NT>(a.pdf, t, p[u][0], p[u][1], p[u][2], p[u][3]);
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < (a.n & 3))
  {
    const uint64_t i = (n4 << 2) + threadIdx.x;
    one_pair<Model, MODE>(m, a, i, MASK ? (a.mask[i] != 0) : true);
  }
}

// Software-pipelined grid-stride variant: the six 16-byte loads of the thread's NEXT quad are
// issued before the current quad is computed, so every wave keeps HBM reads in flight while its
// VALU work runs (the plain kernel only overlaps load and compute across different waves).
template<class Model, int MODE, bool MASK, bool NT>
__global__ __launch_bounds__(kBlock) void k_eval_pdf_pipe(EvalArgs a)
{
  math_tables_init();
  const Model m(a.p.v);
  const uint64_t n4 = a.n >> 2;
  const uint64_t stride = uint64_t(gridDim.x) * kBlock;
  uint64_t t = uint64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (t < n4)
  {
    float4 c[6];
    uint32_t cm = 0x01010101u;
    c[0] = ld4<NT>(a.ix, t); c[1] = ld4<NT>(a.iy, t); c[2] = ld4<NT>(a.iz, t);
    c[3] = ld4<NT>(a.ox, t); c[4] = ld4<NT>(a.oy, t); c[5] = ld4<NT>(a.oz, t);
    if (MASK) cm = reinterpret_cast<const uint32_t*>(a.mask)[t];
    for (; t < n4; t += stride)
    {
      const uint64_t tn = (t + stride < n4) ? t + stride : t;   // clamped: the last prefetch re-reads
      float4 nx[6];
      uint32_t nm = 0x01010101u;
      nx[0] = ld4<NT>(a.ix, tn); nx[1] = ld4<NT>(a.iy, tn); nx[2] = ld4<NT>(a.iz, tn);
      nx[3] = ld4<NT>(a.ox, tn); nx[4] = ld4<NT>(a.oy, tn); nx[5] = ld4<NT>(a.oz, tn);
      if (MASK) nm = reinterpret_cast<const uint32_t*>(a.mask)[tn];
      const float inx[4] = {c[0].x, c[0].y, c[0].z, c[0].w}, iny[4] = {c[1].x, c[1].y, c[1].z, c[1].w};
      const float inz[4] = {c[2].x, c[2].y, c[2].z, c[2].w}, onx[4] = {c[3].x, c[3].y, c[3].z, c[3].w};
      const float ony[4] = {c[4].x, c[4].y, c[4].z, c[4].w}, onz[4] = {c[5].x, c[5].y, c[5].z, c[5].w};
      float r[4], g[4], b[4], p[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
      {
        float rgb[3];
        const uint32_t comp = ((cm >> (8 * j)) & 0xffu) ? a.component : 0u;
        m.template eval_pdf<MODE>(mk3(inx[j], iny[j], inz[j]), mk3(onx[j], ony[j], onz[j]), comp, rgb, p[j]);
        r[j] = rgb[0]; g[j] = rgb[1]; b[j] = rgb[2];
      }
      if (MODE & kModeEval)
      {
        st4<NT>(a.r, t, r[0], r[1], r[2], r[3]);
        st4<NT>(a.g, t, g[0], g[1], g[2], g[3]);
        st4<NT>(a.b, t, b[0], b[1], b[2], b[3]);
      }
      if (MODE & kModePdf) st4<NT>(a.pdf, t, p[0], p[1], p[2], p[3]);
#pragma unroll
      for (int k = 0; k < 6; ++k) c[k] = nx[k];
      cm = nm;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < (a.n & 3))
  {
    const uint64_t i = (n4 << 2) + threadIdx.x;
    one_pair<Model, MODE>(m, a, i, MASK ? (a.mask[i] != 0) : true);
  }
}

// Scalar path for unaligned arrays.
template<class Model, int MODE, bool MASK, bool EXACT = false>
__global__ __launch_bounds__(kBlock) void k_eval_pdf_v1(EvalArgs a)
{
  math_tables_init();
  const Model m(a.p.v);
  const uint64_t stride = uint64_t(gridDim.x) * kBlock;
  for (uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < a.n; i += stride)
    one_pair<Model, MODE, EXACT>(m, a, i, MASK ? (a.mask[i] != 0) : true);
}

// Models whose per-pair eval is VALU-heavy AND returns exactly zero (rgb and pdf) for every pair outside the
// upper hemisphere (z(in) <= 0 or z(out) <= 0, NaN included) and for masked pairs: those run through
// k_eval_pdf_compact, which evaluates only the live pairs, packed densely into waves.
template<class Model> struct compact_eval { static constexpr bool value = false; };

// Compaction on/off.  The shipped library always compacts; only an experimental build (BBM_HIP_EXPERIMENTAL, A/B
// runs) reads BBM_HIP_COMPACT=0 from the environment, so a user's environment cannot change which kernel runs.
inline bool use_compact()
{
#ifdef BBM_HIP_EXPERIMENTAL
  static const bool v = [] {
    const char* e = std::getenv("BBM_HIP_COMPACT");
    return e ? std::atoi(e) != 0 : true;
  }();
  return v;
#else
  return true;
#endif
}

// Stream compaction of live pairs before evaluation.  A wave executes the slowest of its 64 lanes: for a
// VALU-bound model (the He series) a wave of uniformly random sphere pairs spends 3/4 of its lanes on pairs
// that only ever produce 0 (both directions must be in the upper hemisphere) yet pay for the full evaluation
// in lock step with the live ones.  Here each workgroup takes a tile of 1024 pairs (4 per thread, the same
// 16-byte loads as k_eval_pdf_v4), writes the live ones' directions densely into LDS (wave prefix sum +
// per-wave offsets), evaluates them one per lane -- every wave but the last fully occupied -- and writes the
// results back into the LDS slot they came from; the owner threads then store all four outputs (zeros for
// dead pairs) with 16-byte streaming stores.  The evaluation is the model's own eval_pdf on the same
// operands, so the results are bit-identical to the uncompacted kernels.  LDS: 24 KiB per workgroup.
// Occupancy of the compaction kernel: at least 4 waves per SIMD (<= 128 VGPRs; the He evaluation alone would take
// 165 -> 3 waves).  Measured on HeWestin / He / HeHolzschuch (10M pairs, tools/gpu_ab_he.sh): 3 waves 1.76 / 1.18 /
// 0.60 ms, 4 waves 1.48 / 0.97 / 0.58, 5 waves 1.50 / 1.00 / 0.67, 6 waves 1.52 / 1.01 / 0.68 -- the few spilled
// dwords cost less than the latency the fourth wave hides.
#ifndef BBM_HIP_COMPACT_WAVES
#define BBM_HIP_COMPACT_WAVES 4
#endif
#define BBM_HIP_COMPACT_ATTR __attribute__((amdgpu_waves_per_eu(BBM_HIP_COMPACT_WAVES, 8)))
// models whose evaluation splits into a prelude and a variable-length series (He): stage1 / stage2 / Stage
constexpr int kSortBuckets = 32;
template<class Model, int MODE> constexpr bool two_phase()
{
  if constexpr (requires { Model::kTwoPhase; }) return Model::kTwoPhase && (MODE & kModeEval) != 0;
  else return false;
}
template<class Model> constexpr int stage_words()
{
  if constexpr (requires { Model::kStageWords; }) return Model::kStageWords;
  else return 1;
}

// Models whose two-phase prelude hands a few libm evaluations to a block-wide work list (He: its four erfcf,
// he.hpp kErfcList): each thread's arguments go into LDS sorted by the function's argument range (fdlibm's erfcf
// runs one of three code paths per range, and a wave whose lanes span all three runs all three), then the block
// evaluates the list densely -- every wave but the ones at a range boundary runs a single path -- and each thread
// reads its values back.  S1's and K's argument of a direction are often the same float: evaluated once.  Same
// function on the same operands as the inline evaluation: the same floats.
template<class Model> constexpr bool erfc_list()
{
  if constexpr (requires { Model::kErfcList; }) return Model::kErfcList;
  else return false;
}

__device__ __forceinline__ int lanes_below(uint64_t mask)
{
  return int(__builtin_amdgcn_mbcnt_hi(uint32_t(mask >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(mask), 0u)));
}

// All kBlock threads call this (block barriers inside).  list: >= 4 * kBlock floats of LDS, free until the call
// returns; cnt: per-wave range counts.
template<class Model>
__device__ __forceinline__ void erfc_block(const Model& m, bool mine, v3 in, v3 out, typename Model::Erfc& ef,
                                           float* list, int (*cnt)[4])
{
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float x[4];
  m.erfc_args(in, out, x);
  ef.x[0] = x[0];
  ef.x[1] = x[1];
  // K's argument equal to S1's of the same direction: one evaluation serves both
  const bool dup2 = __float_as_uint(x[2]) == __float_as_uint(x[0]);
  const bool dup3 = __float_as_uint(x[3]) == __float_as_uint(x[1]);
  int r[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) r[k] = mine ? erfcf_range(x[k]) : 0;    // 0: no list entry (range 0 is inline)
  r[2] = dup2 ? 0 : r[2];
  r[3] = dup3 ? 0 : r[3];
  uint64_t bal[4][3];
  int wc[3] = {0, 0, 0};
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int c = 0; c < 3; ++c)
    {
      bal[k][c] = __builtin_amdgcn_ballot_w64(r[k] == c + 1);
      wc[c] += __builtin_popcountll(bal[k][c]);
    }
  if (lane == 0)
    for (int c = 0; c < 3; ++c) cnt[wave][c] = wc[c];
  __syncthreads();
  int start[3], before[3], end[3];
  int run = 0;
#pragma unroll
  for (int c = 0; c < 3; ++c)
  {
    start[c] = run;
    before[c] = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w)
    {
      const int v = cnt[w][c];
      before[c] += (w < wave) ? v : 0;
      run += v;
    }
    end[c] = run;
  }
  int pos[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
  {
    pos[k] = 0;
#pragma unroll
    for (int c = 0; c < 3; ++c)
    {
      if (r[k] == c + 1) pos[k] = start[c] + before[c] + lanes_below(bal[k][c]);
      before[c] += __builtin_popcountll(bal[k][c]);
    }
    if (r[k] != 0) list[pos[k]] = x[k];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < end[2]; e += kBlock)
  {
    const float xv = list[e];
    float v;
    if (e < end[0]) v = erfcf_r1(xv);
    else if (e < end[1]) v = erfcf_r2(xv);
    else v = erfcf_r3(xv);
    list[e] = v;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) ef.v[k] = (r[k] != 0) ? list[pos[k]] : erfcf_r0(x[k]);
  ef.v[2] = dup2 ? ef.v[0] : ef.v[2];
  ef.v[3] = dup3 ? ef.v[1] : ef.v[3];
}

template<class Model, int MODE, bool MASK>
__global__ __launch_bounds__(kBlock) BBM_HIP_COMPACT_ATTR void k_eval_pdf_compact(EvalArgs a)
{
  math_tables_init();
  constexpr int kTile = 4 * kBlock;
  __shared__ float job[6][kTile];      // live pairs' in.xyz, out.xyz; rows 0..3 then hold rgb, pdf
  __shared__ int wave_total[kBlock / 64];
  // two-phase models only (the arrays are unused, and removed by the compiler, otherwise): 14 KiB of stage state
  __shared__ float stage[two_phase<Model, MODE>() ? stage_words<Model>() : 1][kBlock];
  __shared__ short origin[kBlock];
  __shared__ int bucket[kSortBuckets], bucket_off[kSortBuckets];
  __shared__ int erfc_cnt[erfc_list<Model>() ? kBlock / 64 : 1][4];
  const Model m(a.p.v);
  const uint64_t n4 = a.n >> 2;
  const uint64_t tiles = (n4 + kBlock - 1) / kBlock;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (uint64_t tile = blockIdx.x; tile < tiles; tile += gridDim.x)
  {
    const uint64_t t = tile * kBlock + threadIdx.x;
    const bool have = t < n4;
    float4 ix{}, iy{}, iz{}, ox{}, oy{}, oz{};
    uint32_t mk = 0;
    if (have)
    {
      ix = ld4<true>(a.ix, t); iy = ld4<true>(a.iy, t); iz = ld4<true>(a.iz, t);
      ox = ld4<true>(a.ox, t); oy = ld4<true>(a.oy, t); oz = ld4<true>(a.oz, t);
      mk = MASK ? reinterpret_cast<const uint32_t*>(a.mask)[t] : 0x01010101u;
    }
    const float inx[4] = {ix.x, ix.y, ix.z, ix.w}, iny[4] = {iy.x, iy.y, iy.z, iy.w}, inz[4] = {iz.x, iz.y, iz.z, iz.w};
    const float onx[4] = {ox.x, ox.y, ox.z, ox.w}, ony[4] = {oy.x, oy.y, oy.z, oy.w}, onz[4] = {oz.x, oz.y, oz.z, oz.w};
    bool live[4];
    int cnt = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
    {
      live[j] = ((mk >> (8 * j)) & 0xffu) && (inz[j] > 0) && (onz[j] > 0);
      cnt += live[j];
    }
    // inclusive prefix sum of the live counts over the wave
    int incl = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1)
    {
      const int v = __shfl_up(incl, d, 64);
      if (lane >= d) incl += v;
    }
    if (lane == 63) wave_total[wave] = incl;
    __syncthreads();
    int base = incl - cnt, total = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w)
    {
      const int tw = wave_total[w];
      base += (w < wave) ? tw : 0;
      total += tw;
    }
    int slot[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
    {
      slot[j] = base;
      if (live[j])
      {
        job[0][base] = inx[j]; job[1][base] = iny[j]; job[2][base] = inz[j];
        job[3][base] = onx[j]; job[4][base] = ony[j]; job[5][base] = onz[j];
        ++base;
      }
    }
    __syncthreads();
    if constexpr (two_phase<Model, MODE>())
    {
      // Two-phase evaluation, 256 jobs at a time: stage 1 (everything but the He series) one job per thread,
      // then the jobs are counting-sorted by the series-length key (32 buckets, LDS) and stage 2 (the series)
      // runs in key order, so each wave takes jobs of similar length: a wave runs as many terms as its longest
      // job, and mixing short and long series had each wave pay the longest one (wave-max / mean 1.5).  Every
      // job is still the model's own eval on the same operands, split at the series: results are bit-identical.
      for (int q0 = 0; q0 < total; q0 += kBlock)
      {
        const int q = q0 + int(threadIdx.x);
        const bool mine = q < total;
        typename Model::Stage st;
        int key = 0;
        const v3 jin = mk3(job[0][q], job[1][q], job[2][q]), jout = mk3(job[3][q], job[4][q], job[5][q]);
        if constexpr (erfc_list<Model>())
        {
          // the stage rows are free until the bucket sort below: the erfc work list's LDS
          static_assert(stage_words<Model>() >= 4, "the erfc work list needs 4 floats per thread");
          typename Model::Erfc ef;
          erfc_block(m, mine, jin, jout, ef, &stage[0][0], erfc_cnt);
          if (mine) key = m.template stage1<MODE>(jin, jout, a.component, &ef, st);
        }
        else if (mine) key = m.template stage1<MODE>(jin, jout, a.component, nullptr, st);
        if (threadIdx.x < kSortBuckets) bucket[threadIdx.x] = 0;
        __syncthreads();
        const int rank = mine ? atomicAdd(&bucket[key], 1) : 0;
        __syncthreads();
        if (threadIdx.x < 64)
        {
          // exclusive prefix of the bucket counts (one wave, kSortBuckets <= 64)
          const int c = (threadIdx.x < kSortBuckets) ? bucket[threadIdx.x] : 0;
          int incl = c;
#pragma unroll
          for (int d = 1; d < 64; d <<= 1)
          {
            const int v = __shfl_up(incl, d, 64);
            if (int(threadIdx.x) >= d) incl += v;
          }
          if (threadIdx.x < kSortBuckets) bucket_off[threadIdx.x] = incl - c;
        }
        __syncthreads();
        if (mine)
        {
          const int pos = bucket_off[key] + rank;
          Model::stage_store(st, &stage[0][pos], kBlock);
          origin[pos] = short(q);
        }
        __syncthreads();
        if (q0 + int(threadIdx.x) < total)
        {
          typename Model::Stage s2;
          Model::stage_load(s2, &stage[0][threadIdx.x], kBlock);
          float rgb[3];
          m.stage2(s2, rgb);
          const int o = origin[threadIdx.x];
          job[0][o] = rgb[0]; job[1][o] = rgb[1]; job[2][o] = rgb[2]; job[3][o] = s2.pdf;
        }
        __syncthreads();
      }
    }
    else
    {
      for (int q = threadIdx.x; q < total; q += kBlock)
      {
        float rgb[3], pdf;
        m.template eval_pdf<MODE>(mk3(job[0][q], job[1][q], job[2][q]), mk3(job[3][q], job[4][q], job[5][q]),
                                  a.component, rgb, pdf);
        job[0][q] = rgb[0]; job[1][q] = rgb[1]; job[2][q] = rgb[2]; job[3][q] = pdf;
      }
      __syncthreads();
    }
    if (have)
    {
      float r[4], g[4], b[4], p[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
      {
        r[j] = live[j] ? job[0][slot[j]] : 0.0f;
        g[j] = live[j] ? job[1][slot[j]] : 0.0f;
        b[j] = live[j] ? job[2][slot[j]] : 0.0f;
        p[j] = live[j] ? job[3][slot[j]] : 0.0f;
      }
      if (MODE & kModeEval)
      {
        st4<true>(a.r, t, r[0], r[1], r[2], r[3]);
        st4<true>(a.g, t, g[0], g[1], g[2], g[3]);
        st4<true>(a.b, t, b[0], b[1], b[2], b[3]);
      }
      if (MODE & kModePdf) st4<true>(a.pdf, t, p[0], p[1], p[2], p[3]);
    }
    __syncthreads();     // the next tile reuses job[] and wave_total[]
  }
  if (blockIdx.x == 0 && threadIdx.x < (a.n & 3))
  {
    const uint64_t i = (n4 << 2) + threadIdx.x;
    one_pair<Model, MODE>(m, a, i, MASK ? (a.mask[i] != 0) : true);
  }
}

// Grid cap for the grid-stride kernels.  Launch-variant knobs (BBM_HIP_MAX_BLOCKS, BBM_HIP_PPT = 8 pairs per thread,
// BBM_HIP_PIPE = the software-pipelined kernel, BBM_HIP_NT = 0 temporal loads / stores) exist only in an
// experimental build (-DBBM_HIP_EXPERIMENTAL, tools/build_variant.sh): the shipped library reads no tuning knob.
#ifdef BBM_HIP_EXPERIMENTAL
inline uint64_t max_blocks()
{
  static const uint64_t v = [] {
    const char* e = std::getenv("BBM_HIP_MAX_BLOCKS");
    const long long x = e ? std::atoll(e) : 0;
    return x > 0 ? uint64_t(x) : uint64_t(kMaxBlocks);
  }();
  return v;
}

inline int pairs_per_thread()
{
  static const int v = [] {
    const char* e = std::getenv("BBM_HIP_PPT");
    return (e && std::atoi(e) == 8) ? 8 : 4;
  }();
  return v;
}

inline bool use_pipe()
{
  static const bool v = [] {
    const char* e = std::getenv("BBM_HIP_PIPE");
    return e ? std::atoi(e) != 0 : false;
  }();
  return v;
}

inline bool use_nt()
{
  static const bool v = [] {
    const char* e = std::getenv("BBM_HIP_NT");
    return e ? std::atoi(e) != 0 : true;
  }();
  return v;
}
#else
constexpr uint64_t max_blocks() { return uint64_t(kMaxBlocks); }
#endif

// ------------------------------------------------------------------------------- sample

struct SampleArgs
{
  const float* ox; const float* oy; const float* oz;
  const float* xi0; const float* xi1;
  const uint8_t* mask;
  float* dx; float* dy; float* dz; float* pdf; uint32_t* flag;
  uint64_t n;
  uint32_t component;
  ParamBlock p;
};

template<class Model>
__device__ __forceinline__ void one_sample(const Model& m, const SampleArgs& a, uint64_t i, bool active)
{
  v3 d; float pdf; uint32_t f;
  m.sample(mk3(a.ox[i], a.oy[i], a.oz[i]), a.xi0[i], a.xi1[i], active ? a.component : 0u, d, pdf, f);
  a.dx[i] = d.x; a.dy[i] = d.y; a.dz[i] = d.z; a.pdf[i] = pdf; a.flag[i] = f;
}

// 4 samples per thread-iteration: 5 x 16-byte loads (out xyz, xi0, xi1), 5 x 16-byte stores.
template<class Model, bool MASK>
__global__ __launch_bounds__(kBlock) void k_sample_v4(SampleArgs a)
{
  math_tables_init();
  const Model m(a.p.v);
  const uint64_t n4 = a.n >> 2;
  const uint64_t stride = uint64_t(gridDim.x) * kBlock;
  for (uint64_t t = uint64_t(blockIdx.x) * kBlock + threadIdx.x; t < n4; t += stride)
  {
    const float4 ox = reinterpret_cast<const float4*>(a.ox)[t];
    const float4 oy = reinterpret_cast<const float4*>(a.oy)[t];
    const float4 oz = reinterpret_cast<const float4*>(a.oz)[t];
    const float4 x0 = reinterpret_cast<const float4*>(a.xi0)[t];
    const float4 x1 = reinterpret_cast<const float4*>(a.xi1)[t];
    uint32_t mk = 0x01010101u;
    if (MASK) mk = reinterpret_cast<const uint32_t*>(a.mask)[t];
    const float onx[4] = {ox.x, ox.y, ox.z, ox.w}, ony[4] = {oy.x, oy.y, oy.z, oy.w}, onz[4] = {oz.x, oz.y, oz.z, oz.w};
    const float u0[4] = {x0.x, x0.y, x0.z, x0.w}, u1[4] = {x1.x, x1.y, x1.z, x1.w};
    float dx[4], dy[4], dz[4], pd[4];
    uint32_t fl[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
    {
      v3 d;
      const uint32_t comp = ((mk >> (8 * j)) & 0xffu) ? a.component : 0u;
      m.sample(mk3(onx[j], ony[j], onz[j]), u0[j], u1[j], comp, d, pd[j], fl[j]);
      dx[j] = d.x; dy[j] = d.y; dz[j] = d.z;
    }
    reinterpret_cast<float4*>(a.dx)[t] = make_float4(dx[0], dx[1], dx[2], dx[3]);
    reinterpret_cast<float4*>(a.dy)[t] = make_float4(dy[0], dy[1], dy[2], dy[3]);
    reinterpret_cast<float4*>(a.dz)[t] = make_float4(dz[0], dz[1], dz[2], dz[3]);
    reinterpret_cast<float4*>(a.pdf)[t] = make_float4(pd[0], pd[1], pd[2], pd[3]);
    reinterpret_cast<uint4*>(a.flag)[t] = make_uint4(fl[0], fl[1], fl[2], fl[3]);
  }
  if (blockIdx.x == 0 && threadIdx.x < (a.n & 3))
  {
    const uint64_t i = (n4 << 2) + threadIdx.x;
    one_sample<Model>(m, a, i, MASK ? (a.mask[i] != 0) : true);
  }
}

template<class Model, bool MASK>
__global__ __launch_bounds__(kBlock) void k_sample_v1(SampleArgs a)
{
  math_tables_init();
  const Model m(a.p.v);
  const uint64_t stride = uint64_t(gridDim.x) * kBlock;
  for (uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < a.n; i += stride)
    one_sample<Model>(m, a, i, MASK ? (a.mask[i] != 0) : true);
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

template<class Model, int MODE, bool MASK>
int launch_mode(const EvalArgs& a0, hipStream_t s)
{
  if (const int rc = host_prepare<Model>::run(s)) return rc;
  if (const int rc = host_validate<Model>::run(a0.p)) return rc;
  EvalArgs a = a0;
  void* scratch = nullptr;
  if (MODE & kModePdf)
    if (const int rc = host_params<Model>::run(a.p, a.component, s, &scratch)) return rc;
  struct Release { void* p; hipStream_t s; ~Release() { host_params<Model>::done(p, s); } } release{scratch, s};
  bool vec = aligned16(a.ix) && aligned16(a.iy) && aligned16(a.iz) && aligned16(a.ox) && aligned16(a.oy) &&
             aligned16(a.oz) && (!MASK || (reinterpret_cast<uintptr_t>(a.mask) & 3u) == 0);
  if (MODE & kModeEval) vec = vec && aligned16(a.r) && aligned16(a.g) && aligned16(a.b);
  if (MODE & kModePdf) vec = vec && aligned16(a.pdf);
  const uint64_t units = vec ? (a.n >> 2) : a.n;
#ifdef BBM_HIP_EXPERIMENTAL
  // A/B variants (tools/gpu_ab.sh): 8 pairs/thread, software pipelining, temporal loads/stores.
  const uint64_t per_block = (vec && pairs_per_thread() == 8) ? 2 * kBlock : kBlock;
#else
  const uint64_t per_block = kBlock;
#endif
  uint64_t blocks = (units + per_block - 1) / per_block;
  if (blocks < 1) blocks = 1;
  if (blocks > max_blocks()) blocks = max_blocks();
  if (eval_grid_cap<Model>::value && blocks > eval_grid_cap<Model>::value) blocks = eval_grid_cap<Model>::value;
#ifdef BBM_HIP_EXPERIMENTAL
  if (vec && pairs_per_thread() == 8)
    hipLaunchKernelGGL((k_eval_pdf_v8<Model, MODE, MASK, true>), dim3(unsigned(blocks)), dim3(kBlock), 0, s, a);
  else if (vec && use_pipe()) hipLaunchKernelGGL((k_eval_pdf_pipe<Model, MODE, MASK, true>), dim3(unsigned(blocks)), dim3(kBlock), 0, s, a);
  else if (vec && !use_nt()) hipLaunchKernelGGL((k_eval_pdf_v4<Model, MODE, MASK, false>), dim3(unsigned(blocks)), dim3(kBlock), 0, s, a);
  else
#endif
  if (vec && compact_eval<Model>::value && use_compact())
    hipLaunchKernelGGL((k_eval_pdf_compact<Model, MODE, MASK>), dim3(unsigned(blocks)), dim3(kBlock), 0, s, a);
  else if (exact_launch<Model>())
  {
    if constexpr (model_has_exact<Model>())
    {
      if (vec) hipLaunchKernelGGL((k_eval_pdf_v4<Model, MODE, MASK, true, true>), dim3(unsigned(blocks)), dim3(kBlock), 0, s, a);
      else hipLaunchKernelGGL((k_eval_pdf_v1<Model, MODE, MASK, true>), dim3(unsigned(blocks)), dim3(kBlock), 0, s, a);
    }
  }
  else if (vec) hipLaunchKernelGGL((k_eval_pdf_v4<Model, MODE, MASK, true>), dim3(unsigned(blocks)), dim3(kBlock), 0, s, a);
  else hipLaunchKernelGGL((k_eval_pdf_v1<Model, MODE, MASK>), dim3(unsigned(blocks)), dim3(kBlock), 0, s, a);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(BBM_HIP_ERR_HIP, std::string("kernel launch failed: ") + hipGetErrorString(e));
  return BBM_HIP_OK;
}

template<class Model, bool MASK>
int launch_sample_mask(const SampleArgs& a0, hipStream_t s)
{
  if (const int rc = host_prepare<Model>::run(s)) return rc;
  if (const int rc = host_validate<Model>::run(a0.p)) return rc;
  SampleArgs a = a0;
  void* scratch = nullptr;
  if (const int rc = host_params<Model>::run(a.p, a.component, s, &scratch)) return rc;
  struct Release { void* p; hipStream_t s; ~Release() { host_params<Model>::done(p, s); } } release{scratch, s};
  const bool vec = aligned16(a.ox) && aligned16(a.oy) && aligned16(a.oz) && aligned16(a.xi0) && aligned16(a.xi1) &&
                   aligned16(a.dx) && aligned16(a.dy) && aligned16(a.dz) && aligned16(a.pdf) && aligned16(a.flag) &&
                   (!MASK || (reinterpret_cast<uintptr_t>(a.mask) & 3u) == 0);
  const uint64_t units = vec ? (a.n >> 2) : a.n;
  uint64_t blocks = (units + kBlock - 1) / kBlock;
  if (blocks < 1) blocks = 1;
  if (blocks > max_blocks()) blocks = max_blocks();
  bool twin = false;
  if constexpr (has_exact_sample<Model>())       // exact mode: the sampler's twin with glibc's erff / logf (math.hpp)
    if (exact_on())
    {
      using T = exact_sample_t<Model>;
      if (vec) hipLaunchKernelGGL((k_sample_v4<T, MASK>), dim3(unsigned(blocks)), dim3(kBlock), 0, s, a);
      else hipLaunchKernelGGL((k_sample_v1<T, MASK>), dim3(unsigned(blocks)), dim3(kBlock), 0, s, a);
      twin = true;
    }
  if (twin) {}
  else if (vec) hipLaunchKernelGGL((k_sample_v4<Model, MASK>), dim3(unsigned(blocks)), dim3(kBlock), 0, s, a);
  else hipLaunchKernelGGL((k_sample_v1<Model, MASK>), dim3(unsigned(blocks)), dim3(kBlock), 0, s, a);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(BBM_HIP_ERR_HIP, std::string("kernel launch failed: ") + hipGetErrorString(e));
  return BBM_HIP_OK;
}

template<class Model>
int launch_sample(const SampleArgs& a, hipStream_t s)
{
  return a.mask ? launch_sample_mask<Model, true>(a, s) : launch_sample_mask<Model, false>(a, s);
}

template<class Model>
int launch_eval_pdf(const EvalArgs& a, int mode, hipStream_t s)
{
  const bool mk = a.mask != nullptr;
  switch (mode)
  {
    case kModeEval: return mk ? launch_mode<Model, kModeEval, true>(a, s) : launch_mode<Model, kModeEval, false>(a, s);
    case kModePdf: return mk ? launch_mode<Model, kModePdf, true>(a, s) : launch_mode<Model, kModePdf, false>(a, s);
    default: return mk ? launch_mode<Model, kModeEvalPdf, true>(a, s) : launch_mode<Model, kModeEvalPdf, false>(a, s);
  }
}

// ------------------------------------------------------------------------- reflectance

struct ReflArgs
{
  const float* ox; const float* oy; const float* oz;
  const uint8_t* mask;
  float* r; float* g; float* b;
  uint64_t n;
  uint32_t component;
  ParamBlock p;
};

// bsdfmodel::reflectance per direction (not on the headline path: one scalar lane per direction)
template<class Model>
__global__ __launch_bounds__(kBlock) void k_reflectance(ReflArgs a)
{
  math_tables_init();
  const Model m(a.p.v);
  const uint64_t stride = uint64_t(gridDim.x) * kBlock;
  for (uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < a.n; i += stride)
  {
    float rgb[3];
    const bool active = a.mask ? (a.mask[i] != 0) : true;
    m.reflectance(mk3(a.ox[i], a.oy[i], a.oz[i]), active ? a.component : 0u, rgb);
    a.r[i] = rgb[0]; a.g[i] = rgb[1]; a.b[i] = rgb[2];
  }
}

template<class Model>
int launch_reflectance(const ReflArgs& a, hipStream_t s)
{
  if (const int rc = host_prepare<Model>::run(s)) return rc;
  if (const int rc = host_validate<Model>::run(a.p)) return rc;
  uint64_t blocks = (a.n + kBlock - 1) / kBlock;
  if (blocks < 1) blocks = 1;
  if (blocks > max_blocks()) blocks = max_blocks();
  hipLaunchKernelGGL((k_reflectance<Model>), dim3(unsigned(blocks)), dim3(kBlock), 0, s, a);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(BBM_HIP_ERR_HIP, std::string("kernel launch failed: ") + hipGetErrorString(e));
  return BBM_HIP_OK;
}

// ------------------------------------------------------------------------- fitting loss

constexpr int kProbeBatch = 12;         // probes evaluated per pass over the samples (f64 accumulators)
constexpr int kLossMaxBlocks = 2048;    // workspace = kLossMaxBlocks x nprobes doubles + the probes' models
constexpr size_t kLossModelBytes = 512; // one constructed model per probe in the workspace

struct LossArgs
{
  LinDesc lin;
  uint64_t begin, n;                    // samples [begin, begin + n) of the linearizer
  const float* pairs[6];                // or: the pairs themselves (in xyz, out xyz; pairs[0] == NULL: use lin)
  const float* ref_r; const float* ref_g; const float* ref_b;   // reference value of sample begin + i
  const float* probes;                  // nprobes x stride parameter vectors (device)
  int nprobes, stride, loss_kind;
  uint32_t component;
  double* block_sums;                   // [gridDim.x][nprobes]
  char* models;                         // [nprobes][kLossModelBytes]: Model constructed once per probe
  double* sums;                         // [nprobes]
};

// One thread per probe: copy the probe's parameter vector into a zero-padded block (models that read slots
// beyond their kParams -- He's and Merl's table pointers -- see zeros, never the next probe or past the
// buffer), construct the Model once, and store it for k_loss, whose threads then read it with uniform loads
// instead of re-running the constructor (tgamma, sampler setup, Aggregate weights) per sample and probe.
template<class Model>
__global__ __launch_bounds__(64) void k_loss_models(LossArgs a)
{
  math_tables_init();
  const int p = blockIdx.x * 64 + threadIdx.x;
  if (p >= a.nprobes) return;
  ParamBlock q;
#pragma unroll
  for (int k = 0; k < kMaxParams; ++k) q.v[k] = (k < a.stride) ? a.probes[size_t(p) * size_t(a.stride) + k] : 0.0f;
  const Model m(q.v);
  __builtin_memcpy(a.models + size_t(p) * kLossModelBytes, &m, sizeof(Model));
}

// The wave's sum of a double, computed in registers: four DPP row shifts (v_mov_b32_dpp on both halves, zero
// outside the row) leave each 16-lane row's sum in its lane 15, and the four row sums are added in row order --
// a fixed tree, like wave_sum's butterfly, at VALU latency instead of six LDS-crossbar round trips (ds_bpermute)
template<int CTRL>
__device__ __forceinline__ double dpp_row(double v)
{
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xf, 0xf, true);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double readlane_d(double v, int lane)
{
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), lane), __builtin_amdgcn_readlane(__double2loint(v), lane));
}
__device__ __forceinline__ double wave_sum_dpp(double v)
{
  v += dpp_row<0x111>(v);     // row_shr:1
  v += dpp_row<0x112>(v);     // row_shr:2
  v += dpp_row<0x114>(v);     // row_shr:4
  v += dpp_row<0x118>(v);     // row_shr:8 -> lane 15 of each row holds the row's sum
  return ((readlane_d(v, 15) + readlane_d(v, 31)) + readlane_d(v, 47)) + readlane_d(v, 63);
}

__device__ __forceinline__ double wave_sum(double v)
{
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Minimum waves per SIMD of the loss kernel (the probe-batch loop holds ~230 VGPRs unconstrained: 2 waves).
// Measured on config 5 (Aggregate(Lambertian, Bagher), 36 probes x the MERL grid, tools/gpu_ab_work.sh):
// 0.87 / 0.73 / 0.62 / 0.61 / 1.09 ms per compass step at 2 / 3 / 4 / 5 / 6 waves.  The He family keeps the
// compiler's choice (its series would spill heavily at 128 VGPRs; see models.hpp).
#ifndef BBM_HIP_LOSS_WAVES
#define BBM_HIP_LOSS_WAVES 4
#endif
template<class Model> struct loss_waves { static constexpr int value = BBM_HIP_LOSS_WAVES; };
template<class Model>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(loss_waves<Model>::value, 8))) void k_loss(LossArgs a)
{
  math_tables_init();
  static_assert(sizeof(Model) <= kLossModelBytes, "model does not fit its loss workspace slot");
  __shared__ double part[kBlock / 64][kProbeBatch];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t stride = uint64_t(gridDim.x) * kBlock;
  for (int p0 = 0; p0 < a.nprobes; p0 += kProbeBatch)
  {
    double acc[kProbeBatch];
#pragma unroll
    for (int j = 0; j < kProbeBatch; ++j) acc[j] = 0.0;
    for (uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < a.n; i += stride)
    {
      v3 in, out;
      if (a.pairs[0] != nullptr)
      {
        in = mk3(a.pairs[0][i], a.pairs[1][i], a.pairs[2][i]);
        out = mk3(a.pairs[3][i], a.pairs[4][i], a.pairs[5][i]);
      }
      else lin_pair(a.lin, a.begin + i, in, out);
      const float ref[3] = {a.ref_r[i], a.ref_g[i], a.ref_b[i]};
      const LossSample s = loss_prepare(a.loss_kind, in, out, ref);
      if constexpr (has_geo<Model>())
      {
        // the parameter-independent prelude (halfway vector, masks, ...) once per pair for all the batch's probes
        typename Model::Geo geo = Model::geometry(in, out);
#pragma unroll
        for (int j = 0; j < kProbeBatch; ++j)
        {
          if (p0 + j >= a.nprobes) break;           // uniform
          const Model& m = *reinterpret_cast<const Model*>(a.models + size_t(p0 + j) * kLossModelBytes);
          float rgb[3];
          geo_eval<true>(m, geo, a.component, rgb);
          acc[j] += double(sample_loss(a.loss_kind, s, rgb));
        }
      }
      else
      {
#pragma unroll
        for (int j = 0; j < kProbeBatch; ++j)
        {
          if (p0 + j >= a.nprobes) break;           // uniform
          const Model& m = *reinterpret_cast<const Model*>(a.models + size_t(p0 + j) * kLossModelBytes);
          float rgb[3], pdf;
          m.template eval_pdf<kModeEval>(in, out, a.component, rgb, pdf);
          acc[j] += double(sample_loss(a.loss_kind, s, rgb));
        }
      }
    }
#pragma unroll
    for (int j = 0; j < kProbeBatch; ++j)
    {
      const double v = wave_sum(acc[j]);
      if (lane == 0) part[wave][j] = v;
    }
    __syncthreads();
    if (threadIdx.x < kProbeBatch && p0 + int(threadIdx.x) < a.nprobes)
    {
      double t = 0.0;
#pragma unroll
      for (int w = 0; w < kBlock / 64; ++w) t += part[w][threadIdx.x];
      a.block_sums[size_t(blockIdx.x) * a.nprobes + p0 + threadIdx.x] = t;
    }
    __syncthreads();
  }
}

// The pair's side of a probe evaluation: the model's parameter-independent prelude where it has one (geometry() /
// eval_geo()), else the pair itself and the full eval.
template<class Model, bool G = has_geo<Model>()> struct LossGeo
{
  typename Model::Geo g;
  __device__ __forceinline__ void init(v3 in, v3 out) { g = Model::geometry(in, out); }
  __device__ __forceinline__ void eval(const Model& m, uint32_t component, float* rgb) { geo_eval<true>(m, g, component, rgb); }
};
template<class Model> struct LossGeo<Model, false>
{
  v3 in, out;
  __device__ __forceinline__ void init(v3 i, v3 o) { in = i; out = o; }
  __device__ __forceinline__ void eval(const Model& m, uint32_t component, float* rgb)
  {
    float pdf;
    m.template eval_pdf<kModeEval>(in, out, component, rgb, pdf);
  }
};

// Pair-major loss (the default): each thread decodes kLossPairs pairs once per call -- linearizer, reference value,
// loss prelude, model geometry -- and runs every probe over them in a runtime loop whose model is read with uniform
// (scalar) loads, so no probe's parameters are held in VGPRs across pairs; per probe, its kLossPairs losses are
// summed in order (double), the wave adds them up (fixed butterfly) and lane 0 adds the wave's total into its LDS
// row; the block's rows are summed in wave order at the end.  Against the probe-batch kernel below (k_loss): the
// decode runs once per call instead of once per 12-probe batch, and register pressure no longer grows with the batch.
#ifndef BBM_HIP_LOSS_PAIRS
#define BBM_HIP_LOSS_PAIRS 1
#endif
#ifndef BBM_HIP_LOSS_PAIRS_WAVES
#define BBM_HIP_LOSS_PAIRS_WAVES 4
#endif
// where k_loss_pairs reads a probe's model: 0 by reference in global memory (scalar loads at each use), 1 a copy by
// value (bulk scalar loads, SGPR spills to VGPR lanes), 2 staged in LDS at kernel start (broadcast LDS reads)
#ifndef BBM_HIP_LOSS_MODEL
#define BBM_HIP_LOSS_MODEL 0
#endif
#ifndef BBM_HIP_LOSS_PROBE_UNROLL
#define BBM_HIP_LOSS_PROBE_UNROLL 2
#endif
constexpr int kLossPairs = BBM_HIP_LOSS_PAIRS;
constexpr int kLossProbeUnroll = BBM_HIP_LOSS_PROBE_UNROLL;   // probes evaluated per iteration of the probe loop
static_assert(kLossPairs >= 1, "pairs per thread of the pair-major loss kernel");
#ifdef BBM_HIP_LOSS_PROBE_BATCH
constexpr bool kLossPairMajor = false;       // A/B: the probe-batch kernel k_loss everywhere
#else
constexpr bool kLossPairMajor = true;
#endif
// minimum waves per SIMD of k_loss_pairs; measured on config 5 (profiles/r04_ab_fit_loss_kernel*.txt, ms per compass
// step, interleaved on one box): 1 pair x 2 probes per iteration at 4 waves 0.599-0.601, 1 x 4 at 4 waves 0.603-0.607,
// 1 x 4 / 1 x 2 / 2 x 2 / 2 x 1 at 3 waves 0.67-0.70 (0.607-0.610 for 2 x 1 on an earlier box), unconstrained (2 waves,
// 218 VGPRs) 0.79-0.81, the probe-batch kernel 0.654-0.656.  The He family keeps the compiler's choice (models.hpp).
template<class Model> struct loss_pair_waves { static constexpr int value = BBM_HIP_LOSS_PAIRS_WAVES; };
template<class Model>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(loss_pair_waves<Model>::value, 8))) void k_loss_pairs(LossArgs a)
{
  math_tables_init();
  static_assert(sizeof(Model) <= kLossModelBytes, "model does not fit its loss workspace slot");
  extern __shared__ double part[];                       // [kBlock / 64][nprobes] (+ the models, BBM_HIP_LOSS_MODEL 2)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int j = threadIdx.x; j < (kBlock / 64) * a.nprobes; j += kBlock) part[j] = 0.0;
#if BBM_HIP_LOSS_MODEL == 2
  constexpr int kLdsModelBytes = (int(sizeof(Model)) + 15) & ~15;
  char* mlds = reinterpret_cast<char*>(part + (kBlock / 64) * a.nprobes);
  for (int w = threadIdx.x; w < a.nprobes * (kLdsModelBytes / 4); w += kBlock)
  {
    const int j = w / (kLdsModelBytes / 4), o = w % (kLdsModelBytes / 4);
    reinterpret_cast<uint32_t*>(mlds)[w] = reinterpret_cast<const uint32_t*>(a.models + size_t(j) * kLossModelBytes)[o];
  }
#endif
  __syncthreads();
  // this workgroup's contiguous share of the samples: equal to one sample per thread and pass across the grid, so
  // no workgroup runs an extra pass the others do not (the grid is a multiple of the resident workgroups)
  constexpr uint64_t span = uint64_t(kBlock) * kLossPairs;
  const uint64_t lo = a.n * blockIdx.x / gridDim.x, hi = a.n * (blockIdx.x + 1) / gridDim.x;
  for (uint64_t base = lo; base < hi; base += span)
  {
    LossGeo<Model> geo[kLossPairs];
    LossSample smp[kLossPairs];
    bool live[kLossPairs];
#pragma unroll
    for (int k = 0; k < kLossPairs; ++k)
    {
      const uint64_t i = base + uint64_t(k) * kBlock + threadIdx.x;
      live[k] = i < hi;
      if (!live[k]) continue;
      v3 in, out;
      if (a.pairs[0] != nullptr)
      {
        in = mk3(a.pairs[0][i], a.pairs[1][i], a.pairs[2][i]);
        out = mk3(a.pairs[3][i], a.pairs[4][i], a.pairs[5][i]);
      }
      else lin_pair(a.lin, a.begin + i, in, out);
      const float ref[3] = {a.ref_r[i], a.ref_g[i], a.ref_b[i]};
      smp[k] = loss_prepare(a.loss_kind, in, out, ref);
      geo[k].init(in, out);
    }
    for (int j0 = 0; j0 < a.nprobes; j0 += kLossProbeUnroll)
    {
      double acc[kLossProbeUnroll];
#pragma unroll
      for (int u = 0; u < kLossProbeUnroll; ++u)
      {
        acc[u] = 0.0;
        if (j0 + u >= a.nprobes) break;             // uniform
#if BBM_HIP_LOSS_MODEL == 2
        const Model& m = *reinterpret_cast<const Model*>(mlds + size_t(j0 + u) * kLdsModelBytes);
#elif BBM_HIP_LOSS_MODEL == 1
        const Model m = *reinterpret_cast<const Model*>(a.models + size_t(j0 + u) * kLossModelBytes);
#else
        const Model& m = *reinterpret_cast<const Model*>(a.models + size_t(j0 + u) * kLossModelBytes);
#endif
#pragma unroll
        for (int k = 0; k < kLossPairs; ++k)
        {
          if (!live[k]) continue;
          float rgb[3];
          geo[k].eval(m, a.component, rgb);
          acc[u] += double(sample_loss(a.loss_kind, smp[k], rgb));
        }
      }
#pragma unroll
      for (int u = 0; u < kLossProbeUnroll; ++u)
      {
        if (j0 + u >= a.nprobes) break;
#ifdef BBM_HIP_LOSS_SHFL
        const double v = wave_sum(acc[u]);     // A/B: the ds_bpermute butterfly
#else
        const double v = wave_sum_dpp(acc[u]);
#endif
        if (lane == 0) part[wave * a.nprobes + j0 + u] += v;
      }
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < a.nprobes; j += kBlock)
  {
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) t += part[w * a.nprobes + j];
    a.block_sums[size_t(blockIdx.x) * a.nprobes + j] = t;
  }
}

// Workgroups of `kernel` (kBlock threads, `lds` bytes of dynamic LDS) resident on the current device at once (0 if
// the runtime cannot say)
template<class K>
inline uint64_t resident_blocks(K kernel, size_t lds)
{
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kBlock, lds) != hipSuccess) return 0;
  return uint64_t(cus) * uint64_t(per_cu > 0 ? per_cu : 0);
}

// sums[p] = sum over blocks of block_sums[b][p], in block order (one workgroup per probe; fixed tree)
__global__ __launch_bounds__(kBlock) void k_loss_final(const double* block_sums, int nblocks, int nprobes, double* sums);

template<class Model>
int launch_loss(const LossArgs& a0, hipStream_t s)
{
  if (const int rc = host_prepare<Model>::run(s)) return rc;
  LossArgs a = a0;
  hipLaunchKernelGGL((k_loss_models<Model>), dim3(unsigned((a.nprobes + 63) / 64)), dim3(64), 0, s, a);
  uint64_t blocks;
  size_t lds = size_t(kBlock / 64) * size_t(a.nprobes) * sizeof(double);
#if BBM_HIP_LOSS_MODEL == 2
  lds += size_t(a.nprobes) * ((sizeof(Model) + 15) & ~size_t(15));
#endif
  if (kLossPairMajor && lds <= 48 * 1024)       // up to 1536 probes; more take the probe-batch kernel
  {
    // as many workgroups as there are passes of kLossPairs samples per thread, up to kLossMaxBlocks; beyond one
    // device-full of resident workgroups, a whole number of device-fulls (each workgroup then takes an equal
    // contiguous share), so the last round is not a partial one (measured on config 5: 2 048 workgroups at 768
    // resident ran 2.67 rounds)
    const uint64_t need = (a.n + uint64_t(kBlock) * kLossPairs - 1) / (uint64_t(kBlock) * kLossPairs);
    blocks = need < uint64_t(kLossMaxBlocks) ? need : uint64_t(kLossMaxBlocks);
    const uint64_t res = resident_blocks(k_loss_pairs<Model>, lds);
    if (res > 0 && blocks > res) blocks = res * (blocks / res);
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL((k_loss_pairs<Model>), dim3(unsigned(blocks)), dim3(kBlock), lds, s, a);
  }
  else
  {
    blocks = (a.n + kBlock - 1) / kBlock;
    if (blocks < 1) blocks = 1;
    if (blocks > kLossMaxBlocks) blocks = kLossMaxBlocks;
    hipLaunchKernelGGL((k_loss<Model>), dim3(unsigned(blocks)), dim3(kBlock), 0, s, a);
  }
  hipLaunchKernelGGL(k_loss_final, dim3(unsigned(a.nprobes)), dim3(kBlock), 0, s, a.block_sums, int(blocks), a.nprobes,
                     a.sums);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(BBM_HIP_ERR_HIP, std::string("kernel launch failed: ") + hipGetErrorString(e));
  return BBM_HIP_OK;
}

}  // namespace bbmhip

#include "check.hpp"

namespace bbmhip {

using LossLauncher = int (*)(const LossArgs&, hipStream_t);
using CheckLauncher = int (*)(int, const CheckArgs&, double*, hipStream_t);
using EvalLauncher = int (*)(const EvalArgs&, int, hipStream_t);
using SampleLauncher = int (*)(const SampleArgs&, hipStream_t);
using ReflLauncher = int (*)(const ReflArgs&, hipStream_t);

}  // namespace bbmhip
