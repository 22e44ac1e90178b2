// bbm_amd/csrc/merl.hpp -- the MERL-MIT measured BRDF (include/staticmodel/merl.h) on the GPU:
//   Merl = ndf_sampler< merl_data<CONF, "Merl">, 90, 1 >                      (merl.h:224-225)
// eval is a table lookup: merl_linearizer's forward map (in, out) -> (theta_h, theta_d, phi_d) bin
// (linearizer/merl_linearizer.h:93-125) into the 90 x 90 x 180 table the reference reads from a MERL
// .binary file and white-balances (merl.h:173-206).  The table lives in HBM as float4 (r, g, b, 0) --
// the reference's color<double> entries rounded to float exactly as lookup<Spectrum> does (merl.h:95) --
// so one pair costs one 16 B gather; it is built on the GPU from the file's doubles by bbm_hip_merl_table
// and its device address travels in parameter slots 0-1.  sample / pdf are the data-driven ndf_sampler
// over the backscatter eval(h, h) (bbm/ndf_sampler.h:22-164), shared with the He family (he.hpp);
// reflectance is merl_data's placeholder, 1 for component All (merl.h:149-156).
#pragma once
#include "he.hpp"    // ndf_sampler_pdf / ndf_sampler_halfway / ndf_sampler_cdf_run, param_ptr

namespace bbmhip {

constexpr int kMerlThetaH = 90, kMerlThetaD = 90, kMerlPhiD = 180;   // merl.h:184, merl_linearizer.h:28
constexpr uint32_t kMerlSize = uint32_t(kMerlThetaH) * kMerlThetaD * kMerlPhiD;

// merl_linearizer::operator()(in, out, mask) (linearizer/merl_linearizer.h:93-125) for samplesH = (1, 90),
// samplesD = (180, 90); the caller has checked z(in) >= 0 && z(out) >= 0.
__device__ __forceinline__ uint32_t merl_index(v3 in, v3 out)
{
  // convertToHalfwayDifference (core/vec_transform.h:90-97): half = normalize(in + out),
  // diff = rotationY(-theta_h) * (rotationZ(-phi_h) * in); matrix rows from transform.h:47-81
  const v3 half = halfway(in, out);
  const float h_phi = phi_of(half), h_th = theta_of(half);
  float cz, sz, cy, sy;
  cossin_cr(-h_phi, cz, sz);
  cossin_cr(-h_th, cy, sy);
  const v3 t = mk3(((0.0f + cz * in.x) + -sz * in.y) + 0.0f * in.z,
                   ((0.0f + sz * in.x) + cz * in.y) + 0.0f * in.z,
                   ((0.0f + 0.0f * in.x) + 0.0f * in.y) + 1.0f * in.z);
  const v3 d = mk3(((0.0f + cy * t.x) + 0.0f * t.y) + sy * t.z,
                   ((0.0f + 0.0f * t.x) + 1.0f * t.y) + 0.0f * t.z,
                   ((0.0f + -sy * t.x) + 0.0f * t.y) + cy * t.z);
  float d_phi = phi_of(d);
  const float d_th = theta_of(d);
  // phi_d is unstable for in ~= out; reciprocity folds it into [0, pi)
  if (dot3(in, out) > 1.0f - kEpsF) d_phi = 0.0f;
  if (d_phi >= kPiF) d_phi = d_phi - kPiF;
  // idx = floor((coord / Sphere(0.5) + eps) * samples), theta_h through a sqrt; clamp to the table
  const float ip = floorf((__fdiv_rn(d_phi, kPiF) + kEpsF) * float(kMerlPhiD));
  const float it = floorf((__fdiv_rn(d_th, kPiHalfF) + kEpsF) * float(kMerlThetaD));
  const float ih = floorf(safe_sqrtf(__fdiv_rn(h_th, kPiHalfF) + kEpsF) * float(kMerlThetaH));
  const int ipc = int(clampf(ip, 0.0f, float(kMerlPhiD - 1)));
  const int itc = int(clampf(it, 0.0f, float(kMerlThetaD - 1)));
  const int ihc = int(clampf(ih, 0.0f, float(kMerlThetaH - 1)));
  return uint32_t((ihc * kMerlThetaD + itc) * kMerlPhiD + ipc);
}

// The same bin from a cheap evaluation, where it is provably the same.  The exact map above spends ~600 VALU per
// pair on the reference's own floats (two glibc atan2f, two double asin thetas, two correctly rounded sincos) although
// only the three floor()ed bin coordinates matter.  Here the half-vector frame comes from the halfway vector itself
// (cos / sin of phi_h = half.xy / |half.xy|, of theta_h = half.z and |half.xy|: no angles), the difference vector d
// from those, and the angles from the device library's asinf / atan2f (<= 2 ulp).  Every approximation differs from
// the reference's float by a bounded amount: d by <= kMerlDErr per component (the reference's own cos / sin of
// rounded angles against the geometric ones, ~3e-7, and the float rotations, with a margin), theta_d through
// 2 asin(|d - pole| / 2) (slope <= sqrt2 for d.z >= 0), phi_d through atan2 (slope 1 / |d.xy|), theta_h only by the
// asin (half and its chord are the reference's own floats).  A coordinate is decided where floor() takes the same
// value over its whole error interval (plus two ulp of the float ops that form it, as the reference forms them);
// phi_d also away from its fold points (raw atan2 at 0 and +-pi, where the reference's +2 pi / -pi moves the bin to
// the other end).  Lanes not decided -- and NaN / degenerate frames -- set sure = false and take merl_index.
constexpr float kMerlDErr = 4e-6f;

__device__ __forceinline__ bool merl_floor_sure(float q, float e, float& f)
{
  const float lo = floorf(q - e), hi = floorf(q + e);
  f = lo;
  return lo == hi;
}

__device__ __forceinline__ uint32_t merl_index_fast(v3 in, v3 out, bool& sure)
{
  const v3 half = halfway(in, out);
  const float rxy2 = (0.0f + half.x * half.x) + half.y * half.y;
  const float rxy = sqrtf(rxy2);
  // theta_h as theta_of(half) forms it (z >= 0): the chord is the reference's float, the asin the device's
  const float dzh = half.z - 1.0f;
  const float h_th = 2.0f * asinf(0.5f * sqrtf(rxy2 + dzh * dzh));
  const float rinv = __builtin_amdgcn_rcpf(rxy);
  const float cph = half.x * rinv, sph = half.y * rinv;        // cos / sin of phi_h
  const float cth = half.z, sth = rxy;                         // cos / sin of theta_h
  // t = Rz(-phi_h) in, d = Ry(-theta_h) t
  const float tx = cph * in.x + sph * in.y;
  const float ty = cph * in.y - sph * in.x;
  const float dx = cth * tx - sth * in.z;
  const float dy = ty;
  const float dz = sth * tx + cth * in.z;
  const float dxy = sqrtf(dx * dx + dy * dy);
  // theta_d = 2 asin(|d - (0, 0, 1)| / 2) for d.z >= 0 (d.z = cos theta_d = in.half >= 0)
  const float ddz = dz - 1.0f;
  const float d_th = 2.0f * asinf(0.5f * sqrtf(dx * dx + dy * dy + ddz * ddz));
  const float raw = atan2f(dy, dx);
  const float e_phi = (1.5f * kMerlDErr) / dxy + 1.5e-6f;
  const float e_th = 3.0f * kMerlDErr + 1e-6f;
  float d_phi = (raw < 0) ? raw + kPi2F : raw;
  const bool same = dot3(in, out) > 1.0f - kEpsF;              // the reference's phi_d = 0 (computed identically)
  bool ok = same || ((fabsf(raw) > e_phi) && (kPiF - fabsf(raw) > e_phi));
  if (same) d_phi = 0.0f;
  if (d_phi >= kPiF) d_phi = d_phi - kPiF;
  float ip, it, ih;
  // q = (coord / range + eps) * samples: the error interval in bin units, plus two ulp of q for the float ops
  const float qp = (__fdiv_rn(d_phi, kPiF) + kEpsF) * float(kMerlPhiD);
  const float qt = (__fdiv_rn(d_th, kPiHalfF) + kEpsF) * float(kMerlThetaD);
  const float xh = __fdiv_rn(h_th, kPiHalfF) + kEpsF;
  const float qh = safe_sqrtf(xh) * float(kMerlThetaH);
  ok = merl_floor_sure(qp, same ? 0.0f : e_phi * (float(kMerlPhiD) / kPiF) + 4e-5f, ip) && ok;
  ok = merl_floor_sure(qt, e_th * (float(kMerlThetaD) / kPiHalfF) + 4e-5f, it) && ok;
  // theta_h: only the asin differs (<= 3 ulp of h_th); d sqrt(x) = dx / (2 sqrt x)
  const float e_xh = 6e-7f * xh + 2.4e-7f;
  ok = merl_floor_sure(qh, (0.5f * float(kMerlThetaH)) * e_xh * __builtin_amdgcn_rsqf(fmaxf(xh, 1e-30f)) + 4e-5f, ih) && ok;
  sure = ok && (rxy > 1e-6f) && (dxy > 1e-6f);                  // false for NaN as well
  const int ipc = int(clampf(ip, 0.0f, float(kMerlPhiD - 1)));
  const int itc = int(clampf(it, 0.0f, float(kMerlThetaD - 1)));
  const int ihc = int(clampf(ih, 0.0f, float(kMerlThetaH - 1)));
  return uint32_t((ihc * kMerlThetaD + itc) * kMerlPhiD + ipc);
}

// the bin of merl_index, by merl_index_fast where it decides it; -DBBM_HIP_MERL_EXACT_INDEX (A/B): always exact.
// Measured (10 M random pairs, profiles/r05_ab_merl_index.txt): 0.1555 -> 0.138 ms; without the exact fallback (a
// timing probe) 0.135, so the undecided lanes cost ~4 %.  What remains is the table gather: every random pair reads
// a different line of the 23 MB table from the Infinity Cache.  0 lanes off the reference's bin on the 2 x 1 M
// parity pairs + edge cases (tests/test_gpu_merl.py, MAX_FLIP_FRAC = 0).
__device__ __forceinline__ uint32_t merl_bin(v3 in, v3 out)
{
#ifdef BBM_HIP_MERL_EXACT_INDEX
  return merl_index(in, out);
#else
  bool sure;
  uint32_t idx = merl_index_fast(in, out, sure);
#ifndef BBM_HIP_MERL_PROBE_NOFALLBACK     // timing probe only: the undecided lanes keep the cheap bin
  if (!sure) idx = merl_index(in, out);
#endif
  return idx;
#endif
}

struct Merl
{
  static constexpr int kParams = 2;                      // device address of the float4 table
  static constexpr uint32_t kComponent = kFlagAll;
  const float4* table;
  const float* cdf;             // kHeBins floats for the launch's component (ndf_sampler_cdf_run)
  uint32_t launch_component;

  __device__ explicit Merl(const float* p)
  {
    table = reinterpret_cast<const float4*>(param_ptr(p, 0));
    cdf = param_ptr(p, kParams);
    __builtin_memcpy(&launch_component, p + kParams + 2, 4);
  }

  __device__ __forceinline__ bool masked(uint32_t component) const { return component != launch_component; }

  // merl_data::eval (merl.h:78-96): mask is_set(component, All) -- every bit of All set (util/flags.h:100-103),
  // so only component All -- and z(in) >= 0 && z(out) >= 0 (not strict)
  template<bool SCALE = true>
  __device__ __forceinline__ void eval_rgb(v3 in, v3 out, uint32_t component, float* rgb) const
  {
    rgb[0] = rgb[1] = rgb[2] = 0.0f;
    // the table check is wave-uniform; it only matters for probe vectors the host cannot see (fit loss)
    if (((component & kFlagAll) == kFlagAll) && (in.z >= 0) && (out.z >= 0) && table)
    {
      const float4 v = table[merl_bin(in, out)];
      rgb[0] = v.x; rgb[1] = v.y; rgb[2] = v.z;
    }
  }

  template<int MODE>
  __device__ __forceinline__ void eval_pdf(v3 in, v3 out, uint32_t component, float* rgb, float& pdf) const
  {
    if (MODE & kModeEval) eval_rgb(in, out, component, rgb);
    else rgb[0] = rgb[1] = rgb[2] = 0.0f;
    if (MODE & kModePdf)
    {
      // ndf_sampler::pdf (bbm/ndf_sampler.h:128-156)
      const bool active = (out.z > 0) && (in.z > 0) && !masked(component);
      const v3 h = halfway(in, out);
      const float p = float(double(ndf_sampler_pdf(cdf, h)) / fabs(4.0 * double(dot3(out, h))));
      pdf = active ? p : 0.0f;
    }
    else pdf = 0.0f;
  }

  // merl_data::reflectance (merl.h:149-156): a placeholder, 1 where is_set(component, All)
  __device__ __forceinline__ void reflectance(v3, uint32_t component, float* rgb) const
  {
    const float v = ((component & kFlagAll) == kFlagAll) ? 1.0f : 0.0f;
    rgb[0] = rgb[1] = rgb[2] = v;
  }

  // ndf_sampler::sample (bbm/ndf_sampler.h:78-111)
  __device__ __forceinline__ void sample(v3 out, float xi0, float xi1, uint32_t component, v3& dir, float& pdf,
                                         uint32_t& flag) const
  {
    dir = mk3(0.0f, 0.0f, 0.0f); pdf = 0.0f; flag = kFlagNone;
    if (!((xi0 >= 0) && (xi1 >= 0) && (xi0 <= 1) && (xi1 <= 1) && (out.z > 0)) || masked(component)) return;
    const v3 h = ndf_sampler_halfway(cdf, xi0, xi1);
    const float d = dot3(h, out);
    dir = mk3(2.0f * (h.x * d) - out.x, 2.0f * (h.y * d) - out.y, 2.0f * (h.z * d) - out.z);
    float rgb[3];
    eval_pdf<kModePdf>(dir, out, component, rgb, pdf);
    flag = component;
  }
};

template<>
struct host_validate<Merl>
{
  static int run(const ParamBlock& p)
  {
    if (!param_ptr(p.v, 0))
      return fail(BBM_HIP_ERR_INVALID_ARG, "Merl: parameters hold no table (build one with bbm_hip_merl_table)");
    return BBM_HIP_OK;
  }
};

template<>
struct host_params<Merl>
{
  static int run(ParamBlock& p, uint32_t component, hipStream_t s, void** scratch)
  {
    return ndf_sampler_cdf_run<Merl>(p, component, s, scratch, "Merl");
  }
  static void done(void* scratch, hipStream_t s) { if (scratch) scratch_release(scratch, s); }
};

// merl_data::import (merl.h:173-206): channel c of entry i is max(0, raw[c * size + i] * w_c / 1500.0) in
// double, w = (1.0, 1.15, 1.66), rounded to float by lookup<Spectrum>.
int merl_table_launch(const double* raw, float* table, hipStream_t s);

}  // namespace bbmhip
