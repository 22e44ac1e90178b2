// bbm_amd/csrc/check.hpp -- bin/checkBsdf's statistical tests as batched GPU reductions.
//
// The reference driver (bin/checkBsdf.cpp:51-418) loops over random samples on one CPU thread and
// accumulates float sums / maxima / histograms.  Here one launch runs `n` samples of every "slot"
// (a theta_out of the reflectance test, a trial direction of pdfInt / sample, a (trial, bin) of the
// chi-square pdf integral) with one thread per sample:
//
//   * random numbers come from a counter-based generator (splitmix64 of (seed, stream, index),
//     two 24-bit uniforms per rndVec2d() draw, checkBsdf.cpp:21-26), so a shard [begin, begin+n) of
//     the samples regenerates exactly the numbers a single GPU would have drawn -- the reference's
//     single mt19937 stream is replaced by independent streams per (test, slot, draw);
//   * every per-sample quantity is computed with the reference's float semantics (same model
//     kernels as eval/pdf/sample), accumulated in f64 registers, reduced with wavefront shuffles and
//     LDS, and written as one partial per workgroup; k_check_final sums the partials in a fixed order
//     (deterministic), and takes maxima with the lowest sample index on ties (the serial loop keeps
//     the first strict maximum);
//   * the chi-square histogram counts are integer atomics (order-independent).
//
// Per-slot accumulator layout (kCheckAcc doubles; entries 8..11 are two (max, sample index) pairs):
//   reflectance (:51-97)    0-2 sum eval(dir,out) z(dir) / pdf per channel, 3 accepted samples
//   reciprocity (:102-140)  0-2 sum |f(i,o) - f(o,i)| (Radiance), 3-5 (Importance), 8/9 max hsum (R), 10/11 (I)
//   adjoint (:145-185)      0-2 sum |f_R(i,o) - f_I(o,i)|, 8/9 max hsum
//   pdf (:190-245)          0/1 negative pdf (R/I), 2/3 sampled below horizon (R/I), 4/5 sum |sample.pdf - pdf|
//   pdfInt (:250-290)       0/1 sum pdf(dir, t) / pdf_sphere (R/I)
//   sample pdf (:330-357)   0 sum over pdfSamples of pdf(dir, t) * p(bin) for slot = (trial, bin)
//   sample count (:360-380) counts[trial][bin] += 1 per sample (histogram, atomics)
// No model on this path depends on unit_t (see bbm_hip_eval), so the Radiance and Importance
// variants of a statistic are the same evaluation, accumulated into both entries as the reference does.
#pragma once
#include "math.hpp"
#include "fit.hpp"     // sph_to_vec, phi_of, theta_of

namespace bbmhip {

enum : int
{
  kCheckReflectance = 0, kCheckReciprocity = 1, kCheckAdjoint = 2, kCheckPdf = 3, kCheckPdfInt = 4,
  kCheckSamplePdf = 5, kCheckSampleCount = 6, kCheckNumTests = 7
};
constexpr int kCheckAcc = 12;
constexpr int kCheckSums = 8;
constexpr int kCheckMaxBlocks = 4096;   // partials per launch (all slots together)

struct CheckArgs
{
  uint64_t key[3];          // generator keys of the rndVec2d() draws of one sample (per slot: + slot stride)
  uint64_t begin, n;        // samples [begin, begin + n) of every slot
  int nslots;
  const float* sx; const float* sy; const float* sz;   // slot direction (reflectance: out; pdfInt / sample: trial)
  int sphere;               // pdf: out uniform on the sphere (else hemisphere)
  int importance;           // reflectance: importance-sample the BSDF (else sampleSphere)
  int include_zero;         // sample count: count zero-pdf samples too
  uint32_t nth, nph;        // chi-square bins (theta x phi)
  double* partial;          // [nslots][gridDim.x][kCheckAcc]
  unsigned long long* counts;   // sample count: [nslots][nth * nph]
  ParamBlock p;
};

// base key of draw `draw` (0..2 per sample, 3 = trial directions) of `test`
__host__ __device__ __forceinline__ uint64_t check_base_key(uint64_t seed, int test, int draw)
{
  return mix64(seed) ^ (0xd1b54a32d192ed03ull * (uint64_t(0x10000) * uint64_t(test + 1) + uint64_t(draw) + 1));
}

// the key of draw k of slot s: streams never collide across slots, draws or tests
__host__ __device__ __forceinline__ uint64_t check_key(uint64_t base, int slot) { return mix64(base + 0x2545f4914f6cdd1dull * uint64_t(slot)); }

// rndVec2d() (checkBsdf.cpp:21-26): two uniforms in [0, 1) from one 64-bit hash
__device__ __forceinline__ void uniform2(uint64_t key, uint64_t i, float& u0, float& u1)
{
  const uint64_t h = mix64(key + 0x9e3779b97f4a7c15ull * i);
  u0 = float(uint32_t(h >> 40)) * (1.0f / 16777216.0f);
  u1 = float(uint32_t(h >> 16) & 0xffffffu) * (1.0f / 16777216.0f);
}

// sampleSphere (checkBsdf.cpp:28-35): theta = safe_acos(1.0 - 2.0 xi0) in double, stored as float;
// phi = xi1 Pi(2); pdf = 1.0 / Pi(4).  sampleHemisphere (:38-45): theta = safe_acos(xi0) in float,
// pdf = 1.0 / Pi(2).  spherical::convert (core/spherical.h:58-65) with float cos/sin.
constexpr float kInv4PiF = float(1.0 / double(kPi4F));
constexpr float kInv2PiF = float(1.0 / double(kPi2F));

__device__ __forceinline__ v3 sphere_dir(float xi0, float xi1, bool hemisphere)
{
  float theta;
  if (hemisphere) theta = float(acos(double(fminf(1.0f, fmaxf(-1.0f, xi0)))));
  else theta = float(acos(fmin(1.0, fmax(-1.0, 1.0 - 2.0 * double(xi0)))));
  return sph_to_vec(xi1 * kPi2F, theta);
}

__device__ __forceinline__ float hsum3(const float* v) { return ((0.0f + v[0]) + v[1]) + v[2]; }

// (max value, sample index) pair reduction: larger value wins, lower index on ties
__device__ __forceinline__ void max_pair(double& v, double& idx, double v2, double idx2)
{
  if (v2 > v || (v2 == v && idx2 < idx)) { v = v2; idx = idx2; }
}

__device__ __forceinline__ void wave_reduce_check(double* acc)
{
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
  {
#pragma unroll
    for (int e = 0; e < kCheckSums; ++e) acc[e] += __shfl_xor(acc[e], o, 64);
#pragma unroll
    for (int m = 0; m < 2; ++m)
    {
      const double v2 = __shfl_xor(acc[kCheckSums + 2 * m], o, 64);
      const double i2 = __shfl_xor(acc[kCheckSums + 2 * m + 1], o, 64);
      max_pair(acc[kCheckSums + 2 * m], acc[kCheckSums + 2 * m + 1], v2, i2);
    }
  }
}

// minimum waves per SIMD of the checkBsdf kernels: 4 (<= 128 VGPRs) -- the glibc-exact erff / logf / expf of the
// Beckmann VNDF took the CookTorrance importance-sampling kernel to 161 VGPRs (3 waves) when left to the compiler,
// at 4 it needs no spills; the He family and EPD spill at 4 and keep the compiler's choice (models.hpp)
#ifndef BBM_HIP_CHECK_WAVES
#define BBM_HIP_CHECK_WAVES 4
#endif
template<class Model> struct check_waves { static constexpr int value = BBM_HIP_CHECK_WAVES; };
template<class Model, int TEST>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(check_waves<Model>::value, 8))) void k_check(CheckArgs a)
{
  math_tables_init();
  __shared__ double part[kBlock / 64][kCheckAcc];
  const Model m(a.p.v);
  const int slot = blockIdx.y;
  const uint64_t k0 = check_key(a.key[0], slot), k1 = check_key(a.key[1], slot), k2 = check_key(a.key[2], slot);
  const v3 sd = (a.sx != nullptr) ? mk3(a.sx[slot], a.sy[slot], a.sz[slot]) : mk3(0.0f, 0.0f, 1.0f);
  double acc[kCheckAcc];
#pragma unroll
  for (int e = 0; e < kCheckAcc; ++e) acc[e] = 0.0;
  acc[kCheckSums] = acc[kCheckSums + 2] = -1.0;          // no maximum yet (differences are >= 0)
  acc[kCheckSums + 1] = acc[kCheckSums + 3] = 1.8e19;    // index above any sample
  // chi-square pdf integral: slot = trial * bins + bin
  const uint32_t bins = a.nth * a.nph;
  const uint32_t bin = (TEST == kCheckSamplePdf) ? uint32_t(slot) % bins : 0u;
  const int trial = (TEST == kCheckSamplePdf) ? slot / int(bins) : slot;
  v3 td = sd;
  if (TEST == kCheckSamplePdf) td = mk3(a.sx[trial], a.sy[trial], a.sz[trial]);

  const uint64_t stride = uint64_t(gridDim.x) * kBlock;
  for (uint64_t i = uint64_t(blockIdx.x) * kBlock + threadIdx.x; i < a.n; i += stride)
  {
    const uint64_t s = a.begin + i;
    float u0, u1;
    uniform2(k0, s, u0, u1);
    if constexpr (TEST == kCheckReflectance)
    {
      v3 dir; float pdf; uint32_t flag;
      float f[3], unused;
      bool fused = false;
      if (a.importance)
      {
        if constexpr (requires { Model::kFusedSampleEval; })
        {
          m.sample_eval(sd, u0, u1, kFlagAll, dir, f, pdf, flag);    // eval(dir, sd) and pdf(dir, sd) at once
          fused = true;
        }
        else m.sample(sd, u0, u1, kFlagAll, dir, pdf, flag);
      }
      else { dir = sphere_dir(u0, u1, false); pdf = kInv4PiF; }
      if (pdf > kEpsF)
      {
        if (!fused) m.template eval_pdf<kModeEval>(dir, sd, kFlagAll, f, unused);
#pragma unroll
        for (int c = 0; c < 3; ++c) acc[c] += double(div_nr(f[c] * dir.z, pdf));
        acc[3] += 1.0;
      }
    }
    else if constexpr (TEST == kCheckReciprocity || TEST == kCheckAdjoint)
    {
      float w0, w1;
      uniform2(k1, s, w0, w1);
      const v3 din = sphere_dir(u0, u1, false), dout = sphere_dir(w0, w1, false);
      float f1[3], f2[3], d[3], unused;
      m.template eval_pdf<kModeEval>(din, dout, kFlagAll, f1, unused);
      m.template eval_pdf<kModeEval>(dout, din, kFlagAll, f2, unused);
#pragma unroll
      for (int c = 0; c < 3; ++c) d[c] = fabsf(f1[c] - f2[c]);
      const double h = double(hsum3(d));
#pragma unroll
      for (int c = 0; c < 3; ++c)
      {
        acc[c] += double(d[c]);
        if (TEST == kCheckReciprocity) acc[3 + c] += double(d[c]);
      }
      max_pair(acc[kCheckSums], acc[kCheckSums + 1], h, double(s));
      if (TEST == kCheckReciprocity) max_pair(acc[kCheckSums + 2], acc[kCheckSums + 3], h, double(s));
    }
    else if constexpr (TEST == kCheckPdf)
    {
      float w0, w1, z0, z1;
      uniform2(k1, s, w0, w1);
      uniform2(k2, s, z0, z1);
      const v3 out = sphere_dir(u0, u1, !a.sphere);
      v3 dr, di; float sr, si, pr, pi, rgb[3]; uint32_t fr, fi;
      m.sample(out, w0, w1, kFlagAll, dr, sr, fr);
      m.sample(out, z0, z1, kFlagAll, di, si, fi);
      m.template eval_pdf<kModePdf>(dr, out, kFlagAll, rgb, pr);
      m.template eval_pdf<kModePdf>(di, out, kFlagAll, rgb, pi);
      acc[0] += (pr < 0) ? 1.0 : 0.0;
      acc[1] += (pi < 0) ? 1.0 : 0.0;
      acc[2] += (dr.z < 0) ? 1.0 : 0.0;
      acc[3] += (di.z < 0) ? 1.0 : 0.0;
      acc[4] += double(fabsf(sr - pr));
      acc[5] += double(fabsf(si - pi));
    }
    else if constexpr (TEST == kCheckPdfInt)
    {
      const v3 dir = sphere_dir(u0, u1, false);
      float rgb[3], p;
      m.template eval_pdf<kModePdf>(dir, sd, kFlagAll, rgb, p);
      const double q = double(div_nr(p, kInv4PiF));
      acc[0] += q;
      acc[1] += q;
    }
    else if constexpr (TEST == kCheckSamplePdf)
    {
      // checkBsdf.cpp:347-356: a uniform point in the (theta, phi) bin, weighted by its solid angle
      const uint32_t t = bin / a.nph, pb = bin % a.nph;
      const float phi = div_nr(kPi2F * (float(pb) + u0), float(a.nph));
      const float theta = div_nr(kPiF * (float(t) + u1), float(a.nth));
      const v3 dir = sph_to_vec(phi, theta);
      float st, ct;
      cossin_cr(theta, ct, st);
      constexpr float kPiSq2 = (2.0f * kPiF) * kPiF;      // Constants::Pi2(2) = scale * Pi() * Pi() in float
      const float w = div_nr(kPiSq2 * fabsf(st), float(a.nph * a.nth));
      float rgb[3], p;
      m.template eval_pdf<kModePdf>(dir, td, kFlagAll, rgb, p);
      acc[0] += double(p * w);
    }
    else if constexpr (TEST == kCheckSampleCount)
    {
      v3 dir; float pdf; uint32_t flag;
      m.sample(sd, u0, u1, kFlagAll, dir, pdf, flag);
      if (a.include_zero || pdf > kEpsF)
      {
        // checkBsdf.cpp:374-377: bin of the sample's spherical coordinates, clamped to the last bin
        const float th = fminf(theta_of(dir) / kPiF * float(a.nth), float(a.nth - 1));
        const float ph = fminf(phi_of(dir) / kPi2F * float(a.nph), float(a.nph - 1));
        const uint32_t idx = uint32_t(th) * a.nph + uint32_t(ph);
        atomicAdd(a.counts + size_t(slot) * bins + idx, 1ull);
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
      double r[kCheckAcc];
#pragma unroll
      for (int e = 0; e < kCheckAcc; ++e) r[e] = part[0][e];
      for (int w = 1; w < kBlock / 64; ++w)
      {
#pragma unroll
        for (int e = 0; e < kCheckSums; ++e) r[e] += part[w][e];
        max_pair(r[kCheckSums], r[kCheckSums + 1], part[w][kCheckSums], part[w][kCheckSums + 1]);
        max_pair(r[kCheckSums + 2], r[kCheckSums + 3], part[w][kCheckSums + 2], part[w][kCheckSums + 3]);
      }
      double* dst = a.partial + (size_t(slot) * gridDim.x + blockIdx.x) * kCheckAcc;
#pragma unroll
      for (int e = 0; e < kCheckAcc; ++e) dst[e] = r[e];
    }
  }
}

// Workgroups per slot: enough to fill the chip with few slots, capped so the partials stay small.
inline uint32_t check_blocks(uint64_t n, int nslots)
{
  uint64_t b = (n + kBlock - 1) / kBlock;
  uint64_t cap = uint64_t(kCheckMaxBlocks) / uint64_t(nslots > 0 ? nslots : 1);
  if (cap < 1) cap = 1;
  if (b > cap) b = cap;
  return uint32_t(b < 1 ? 1 : b);
}

// partials [nslots][nblocks][kCheckAcc] -> acc [nslots][kCheckAcc] (fixed order; defined in bbm_hip.hip)
__global__ __launch_bounds__(kBlock) void k_check_final(const double* partial, int nblocks, double* acc);

// one test's kernel for model type K; SAMPLING: only the tests that call the model's sampler (importance-sampled
// reflectance, pdf, sample-pdf, sample count) -- the exact-sampling twin needs no other instantiation.  false: no such test.
template<class K, bool SAMPLING>
bool launch_check_kernel(int test, dim3 grid, const CheckArgs& a, hipStream_t s)
{
  switch (test)
  {
    case kCheckReflectance: hipLaunchKernelGGL((k_check<K, kCheckReflectance>), grid, dim3(kBlock), 0, s, a); return true;
    case kCheckPdf: hipLaunchKernelGGL((k_check<K, kCheckPdf>), grid, dim3(kBlock), 0, s, a); return true;
    case kCheckSamplePdf: hipLaunchKernelGGL((k_check<K, kCheckSamplePdf>), grid, dim3(kBlock), 0, s, a); return true;
    case kCheckSampleCount: hipLaunchKernelGGL((k_check<K, kCheckSampleCount>), grid, dim3(kBlock), 0, s, a); return true;
    default: break;
  }
  if constexpr (!SAMPLING)
    switch (test)
    {
      case kCheckReciprocity: hipLaunchKernelGGL((k_check<K, kCheckReciprocity>), grid, dim3(kBlock), 0, s, a); return true;
      case kCheckAdjoint: hipLaunchKernelGGL((k_check<K, kCheckAdjoint>), grid, dim3(kBlock), 0, s, a); return true;
      case kCheckPdfInt: hipLaunchKernelGGL((k_check<K, kCheckPdfInt>), grid, dim3(kBlock), 0, s, a); return true;
      default: break;
    }
  return false;
}

template<class Model>
int launch_check(int test, const CheckArgs& a0, double* acc, hipStream_t s)
{
  if (const int rc = host_prepare<Model>::run(s)) return rc;
  if (const int rc = host_validate<Model>::run(a0.p)) return rc;
  CheckArgs a = a0;
  void* scratch = nullptr;
  if (const int rc = host_params<Model>::run(a.p, kFlagAll, s, &scratch)) return rc;
  struct Release { void* p; hipStream_t s; ~Release() { host_params<Model>::done(p, s); } } release{scratch, s};
  const uint32_t bx = check_blocks(a.n, a.nslots);
  const dim3 grid(bx, unsigned(a.nslots));
  bool launched = false;
  if constexpr (has_exact_sample<Model>())       // exact mode: the sampler's twin with glibc's erff / logf (math.hpp)
    if (exact_on()) launched = launch_check_kernel<exact_sample_t<Model>, true>(test, grid, a, s);
  if (!launched && !launch_check_kernel<Model, false>(test, grid, a, s))
    return fail(BBM_HIP_ERR_INVALID_ARG, "unknown check test");
  if (test != kCheckSampleCount)
    hipLaunchKernelGGL(k_check_final, dim3(unsigned(a.nslots)), dim3(64), 0, s, a.partial, int(bx), acc);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(BBM_HIP_ERR_HIP, std::string("kernel launch failed: ") + hipGetErrorString(e));
  return BBM_HIP_OK;
}

}  // namespace bbmhip
