// bbm_amd/csrc/fit.hpp -- the fitting-loss path (BASELINE config 5): linearizers, per-sample loss
// functions and the batched multi-probe loss reduction kernel.
//
// Reference (per probe, serial): sampledlossfunction::operator()() (include/bbm/sampledlossfunction.h:80-87)
//   err = sum_i loss(in_i, out_i, fitted.eval(in_i, out_i), reference.eval(in_i, out_i)) / N
// with (in_i, out_i) = linearizer(i), evaluated once per compass probe (include/optimizer/compass.h:82-140:
// 2P probes per step, one parameter moved by +-step each).
//
// Here one launch evaluates ALL probes of a compass step over a range of samples: each thread
// decodes its sample index into a direction pair once per probe batch, reads the reference RGB
// from a table (12 B/sample; a measured material is a table), and evaluates the fitted model for
// kProbeBatch parameter vectors, accumulating each probe's loss in an f64 register.  Per-block sums
// are reduced with wavefront shuffles and LDS and written to a workspace; a second kernel sums the
// blocks in a fixed order (deterministic, order-independent of the launch).  The caller divides by
// the total sample count after the cross-GPU all-reduce (bbm_amd.fit / backbone/hip fit.h).
#pragma once
#include "math.hpp"
#include "spectral.hpp"   // theta_of

namespace bbmhip {

// ------------------------------------------------------------------------------ linearizers

enum : int { kLinSpherical = 0, kLinMerl = 1 };

struct LinDesc
{
  int kind;
  uint64_t s_in[2], s_out[2];     // spherical: (phi, theta) samples in / out; merl: samplesH, samplesD
  float start_in[2], size_in[2], start_out[2], size_out[2];   // spherical: start, end - start
};

__host__ __device__ __forceinline__ uint64_t lin_size(const LinDesc& d)
{
  return (d.kind == kLinMerl) ? d.s_out[0] * d.s_out[1] * d.s_in[1] : d.s_in[0] * d.s_in[1] * d.s_out[0] * d.s_out[1];
}

// std::cos / std::sin of a float: glibc's cosf / sinf bit for bit (math.hpp sincosf_glibc; formerly the double
// sincos rounded to float, which differs from glibc's 0.56-ulp results on a few lanes and costs ~3x the f64 work)
__device__ __forceinline__ void cossin_cr(float a, float& c, float& s) { sincosf_glibc(a, &s, &c); }

// spherical::convert(vec2d(phi, theta)) (core/spherical.h:58-65): (cos phi sin theta, sin phi sin theta, cos theta)
__device__ __forceinline__ v3 sph_to_vec(float phi, float theta)
{
  float ct, st, cp, sp;
  cossin_cr(theta, ct, st);
  cossin_cr(phi, cp, sp);
  return mk3(cp * st, sp * st, ct);
}

// spherical::phi(vec3d) (core/spherical.h:42-46): atan2(y, x) -- glibc's atan2f (math.hpp) -- + 2 pi if negative
__device__ __forceinline__ float phi_of(v3 v)
{
  const float r = atan2f_glibc(v.y, v.x);
  return (r < 0) ? r + kPi2F : r;
}

__device__ __forceinline__ float zero_small(float x) { return (fabsf(x) < kEpsF) ? 0.0f : x; }

// spherical_linearizer::operator()(idx) (include/linearizer/spherical_linearizer.h:63-101)
__device__ __forceinline__ void spherical_pair(const LinDesc& d, uint64_t idx, v3& in, v3& out)
{
  const uint64_t oc1 = idx % d.s_out[1]; idx /= d.s_out[1];
  const uint64_t oc0 = idx % d.s_out[0]; idx /= d.s_out[0];
  const uint64_t ic1 = idx % d.s_in[1]; idx /= d.s_in[1];
  const uint64_t ic0 = idx;
  // sIn = (samplesIn[0], max(samplesIn[1] - 1, 1)): bins include the end points in theta
  const float si0 = float(d.s_in[0]), si1 = float(d.s_in[1] > 2 ? d.s_in[1] - 1 : 1);
  const float so0 = float(d.s_out[0]), so1 = float(d.s_out[1] > 2 ? d.s_out[1] - 1 : 1);
  // cast<Vec2d>(coord * size / s) + start: size_t -> float, then float ops
  const float pin = __fdiv_rn(float(ic0) * d.size_in[0], si0) + d.start_in[0];
  const float tin = __fdiv_rn(float(ic1) * d.size_in[1], si1) + d.start_in[1];
  const float pout = __fdiv_rn(float(oc0) * d.size_out[0], so0) + d.start_out[0];
  const float tout = __fdiv_rn(float(oc1) * d.size_out[1], so1) + d.start_out[1];
  in = sph_to_vec(pin, tin);
  out = sph_to_vec(pout, tout);
  in = mk3(zero_small(in.x), zero_small(in.y), zero_small(in.z));
  out = mk3(zero_small(out.x), zero_small(out.y), zero_small(out.z));
}

// merl_linearizer::operator()(idx) (include/linearizer/merl_linearizer.h:49-83) with
// convertFromHalfwayDifference (core/vec_transform.h:118-123) read as intended, i.e. with
// spherical::phi / spherical::theta of the halfway vector (the reference's unqualified calls do not
// compile with the native backbone; its inverse map pins this one by round trip, tests/test_fit.py).
//   in  = rotZ(phi_h) (rotY(theta_h) diff),  out = rotZ(phi_h) (rotY(theta_h) (-dx, -dy, dz))
// mat3d columns (core/mat.h:38-40) from rotationY/Z (core/transform.h:47-81); mat * vec = dot(row, v).
__device__ __forceinline__ v3 rot_y_z(float cy, float sy, float cz, float sz, v3 v)
{
  // rotY rows: (c, 0, s), (0, 1, 0), (-s, 0, c)
  const v3 t = mk3(((0.0f + cy * v.x) + 0.0f * v.y) + sy * v.z,
                   ((0.0f + 0.0f * v.x) + 1.0f * v.y) + 0.0f * v.z,
                   ((0.0f + -sy * v.x) + 0.0f * v.y) + cy * v.z);
  // rotZ rows: (c, -s, 0), (s, c, 0), (0, 0, 1)
  return mk3(((0.0f + cz * t.x) + -sz * t.y) + 0.0f * t.z,
             ((0.0f + sz * t.x) + cz * t.y) + 0.0f * t.z,
             ((0.0f + 0.0f * t.x) + 0.0f * t.y) + 1.0f * t.z);
}

__device__ __forceinline__ void merl_pair(const LinDesc& d, uint64_t idx, v3& in, v3& out)
{
  const uint64_t pd = idx % d.s_out[0]; idx /= d.s_out[0];
  const uint64_t td = idx % d.s_out[1]; idx /= d.s_out[1];
  const uint64_t th = idx;
  // half_sph = pow(idxH / samplesH, 2.0) * (0.5 * Sphere()): float quotient, double power and product
  const float qh_phi = __fdiv_rn(0.0f, float(d.s_in[0]));
  const float qh_th = __fdiv_rn(float(th), float(d.s_in[1]));
  const float h_phi = float(double(qh_phi) * double(qh_phi) * (0.5 * double(kPi2F)));
  const float h_th = float(double(qh_th) * double(qh_th) * (0.5 * double(kPiF)));
  // diff_sph = (idxD / samplesD) * (0.5 * Sphere())
  const float d_phi = float(double(__fdiv_rn(float(pd), float(d.s_out[0]))) * (0.5 * double(kPi2F)));
  const float d_th = float(double(__fdiv_rn(float(td), float(d.s_out[1]))) * (0.5 * double(kPiF)));
  const v3 half = sph_to_vec(h_phi, h_th);
  const v3 diff = sph_to_vec(d_phi, d_th);
  float cy, sy, cz, sz;
  cossin_cr(theta_of(half), cy, sy);
  cossin_cr(phi_of(half), cz, sz);
  in = rot_y_z(cy, sy, cz, sz, diff);
  out = rot_y_z(cy, sy, cz, sz, mk3(-diff.x, -diff.y, diff.z));
  in.z = fmaxf(in.z, 0.0f);      // bbm::max(z, 0): round-off below the horizon
  out.z = fmaxf(out.z, 0.0f);
}

__device__ __forceinline__ void lin_pair(const LinDesc& d, uint64_t idx, v3& in, v3& out)
{
  if (d.kind == kLinMerl) merl_pair(d, idx, in, out);
  else spherical_pair(d, idx, in, out);
}

// --------------------------------------------------------------------------- sample losses

// include/loss/cosine_weighted_l2.h:24-34 (nganL2), :95-105 (lowL2), :165-176 (bieronL2);
// include/loss/cosine_weighted_log.h:31-43 (lowLog), :100-112 (bieronLog), :170-180 (standardLog).
enum : int { kLossNganL2 = 0, kLossLowL2 = 1, kLossBieronL2 = 2, kLossStandardLog = 3, kLossLowLog = 4, kLossBieronLog = 5 };

// Everything that depends on the sample but not on the fitted parameters, computed once per
// sample and shared by all probes: the angular factors and the reference side of the error.
struct LossSample
{
  float c;               // max(cos theta_in, 0)
  float sin_in, sin_out, cos_out;
  float r[3];            // reference value (L2 losses)
  float lr[3];           // log(1 + reference c) (log losses)
};

__device__ __forceinline__ LossSample loss_prepare(int kind, v3 in, v3 out, const float* ref)
{
  LossSample s;
  s.c = fmaxf(in.z, 0.0f);                                       // bbm::max(cosTheta(in), 0)
  s.sin_in = sqrtf(fmaxf(1 - in.z * in.z, 0.0f));               // spherical::sinTheta (spherical.h:80-83)
  s.sin_out = sqrtf(fmaxf(1 - out.z * out.z, 0.0f));
  s.cos_out = fmaxf(out.z, 0.0f);
#pragma unroll
  for (int k = 0; k < 3; ++k)
  {
    s.r[k] = ref[k];
    s.lr[k] = (kind >= kLossStandardLog) ? logf(1 + ref[k] * s.c) : 0.0f;   // same log as the fitted side
  }
  return s;
}

// per-sample loss of a fitted value v, rounded to Value (float) like the reference's operator():
// hsum(pow(e, 2.0)) is a double sum of exact squares of float errors, then multiplied left to right
// by the float angular factors in double.
__device__ __forceinline__ float sample_loss(int kind, const LossSample& s, const float* v)
{
  double h = 0.0;
  if (kind <= kLossBieronL2)
  {
#pragma unroll
    for (int k = 0; k < 3; ++k)
    {
      const double e = double((v[k] - s.r[k]) * s.c);
      h = h + e * e;
    }
  }
  else
  {
#pragma unroll
    for (int k = 0; k < 3; ++k)
    {
      // std::log(float): the device logf (v_log_f32 + extended-precision ln 2 scaling, ~1 ulp, 14 VALU,
      // vs ~100 for a log rounded from f64) on both sides, so fitted == reference gives exactly 0
      const double e = double(logf(1 + v[k] * s.c) - s.lr[k]);
      h = h + e * e;
    }
  }
  switch (kind)
  {
    case kLossLowL2: case kLossLowLog: return float(h * double(s.sin_in));
    case kLossBieronL2: case kLossBieronLog: return float(((h * double(s.cos_out)) * double(s.sin_in)) * double(s.sin_out));
    default: return float((h * double(s.sin_in)) * double(s.sin_out));
  }
}

// the same losses in doubleRGB (Value = double: every step of the reference's operator() in double; the log the
// device's IEEE-accurate double log), for the materialised loss over any model tree (composite.hip)
struct LossSampleD
{
  double c, sin_in, sin_out, cos_out;
  double r[3], lr[3];
};

__device__ __forceinline__ LossSampleD loss_prepare_d(int kind, double inz, double outz, const double* ref)
{
  LossSampleD s;
  s.c = fmax(inz, 0.0);
  s.sin_in = sqrt(fmax(1 - inz * inz, 0.0));
  s.sin_out = sqrt(fmax(1 - outz * outz, 0.0));
  s.cos_out = fmax(outz, 0.0);
#pragma unroll
  for (int k = 0; k < 3; ++k)
  {
    s.r[k] = ref[k];
    s.lr[k] = (kind >= kLossStandardLog) ? log(1 + ref[k] * s.c) : 0.0;
  }
  return s;
}

__device__ __forceinline__ double sample_loss_d(int kind, const LossSampleD& s, const double* v)
{
  double h = 0.0;
#pragma unroll
  for (int k = 0; k < 3; ++k)
  {
    const double e = (kind <= kLossBieronL2) ? (v[k] - s.r[k]) * s.c : log(1 + v[k] * s.c) - s.lr[k];
    h = h + e * e;
  }
  switch (kind)
  {
    case kLossLowL2: case kLossLowLog: return h * s.sin_in;
    case kLossBieronL2: case kLossBieronLog: return ((h * s.cos_out) * s.sin_in) * s.sin_out;
    default: return (h * s.sin_in) * s.sin_out;
  }
}

}  // namespace bbmhip
