/* oracle/port/bbm_port.c -- TEST INFRASTRUCTURE ONLY (see bbm_port.h).
 *
 * Plain-C restatement of the BBM native backbone (floatRGB) for the batched eval/pdf/sample path.
 * Every function cites the reference file:line it restates.  Precision follows the native
 * backbone exactly: Value = float, but C++ promotion makes some intermediates double -- e.g.
 * `2.0 * z * z / dot` (maskingshadowing/vgroove.h:41-43), `x / NormalizationFactor` with a
 * literal<double> (bsdfmodel/microfacet.h:100), `bbm::max(x, 0.0)` (backbone/native/include/
 * backbone/math.h:100-103 result_t promotion).  C has the same usual arithmetic conversions, so
 * each expression below keeps the reference's literal types; contraction is disabled at build
 * time (-ffp-contract=off) so every float op is rounded on its own, like the reference build.
 */
#include "bbm_port.h"

#include <math.h>
#include <string.h>
#include <stdio.h>
#include <stdlib.h>

#define PI_D 3.141592653589793238462643383279502884
#define INV_PI_D 0.318309886183790671537767526745028724

/* bsdf_flag (include/bbm/bsdf_flag.h:21-27) */
enum { FLAG_NONE = 0, FLAG_DIFFUSE = 1, FLAG_SPECULAR = 2, FLAG_ALL = 3 };

typedef struct { float x, y, z; } v3;

/* constants<float> (include/core/constants.h:17-23): T(scale * double constant) */
static const float kPiF = (float)(1.0f * PI_D);
static const float kInvPiF = (float)(1.0f * INV_PI_D);

/* backbone/native/include/backbone/horizontal.h:78-82 dot = inner_product(..., T(0)) */
static inline float dot3(v3 a, v3 b) { return ((0.0f + a.x * b.x) + a.y * b.y) + a.z * b.z; }

/* horizontal.h:96-100 normalize = t * rsqrt(squared_norm(t)); math.h:109-112 rsqrt = 1/sqrt */
static inline v3 normalize3(v3 t)
{
  float r = 1 / sqrtf(dot3(t, t));
  v3 o = { t.x * r, t.y * r, t.z * r };
  return o;
}

/* core/vec_transform.h:76-80 halfway = normalize(a + b) */
static inline v3 halfway(v3 a, v3 b)
{
  v3 t = { a.x + b.x, a.y + b.y, a.z + b.z };
  return normalize3(t);
}

/* std::max(a, T(0)) semantics (NaN passes through), math.h:129 safe_sqrt */
static inline float safe_sqrtf(float a) { return sqrtf((a < 0.0f) ? 0.0f : a); }
static inline double safe_sqrt(double a) { return sqrt((a < 0.0) ? 0.0 : a); }

/* core/spherical.h:79-80 sinTheta2 = max(1 - z*z, 0) (float fmax); :179-180 tanTheta = sinT / cosT */
static inline float sin_theta2(v3 v) { return fmaxf(1 - v.z * v.z, 0); }
static inline float tan_theta(v3 v) { return sqrtf(sin_theta2(v)) / v.z; }
static inline float tan_theta2(v3 v) { return sin_theta2(v) / (v.z * v.z); }

/* ---------------------------------------------------------------- NDFs */

/* ndf/beckmann.h:49-66 eval */
static float beckmann_eval(v3 h, float au, float av, int normalize)
{
  if (!(h.z > 0)) return 0;
  float c2 = h.z * h.z;
  float sx = h.x / au, sy = h.y / av;
  float sn = (0.0f + sx * sx) + sy * sy;
  float D = expf(-sn / c2) / (au * av * c2 * c2);
  if (normalize) D *= kInvPiF;
  return D;
}

/* ndf/beckmann.h:180-201 G1 (isotropic branch `rcp(roughness * tanTheta(v))`; the anisotropic
   branch `rsqrt(|xy*roughness|^2 / pow(z,2))`) */
static float beckmann_G1(v3 v, v3 m, float au, float av, int aniso)
{
  if (!((v.z > 0) && (dot3(v, m) > 0))) return 0;
  float a;
  if (aniso)
  {
    float px = v.x * au, py = v.y * av;
    float sn = (0.0f + px * px) + py * py;
    a = 1 / sqrtf(sn / powf(v.z, 2.0f));
  }
  else a = 1 / (au * tan_theta(v));
  double g = (a < 1.6) ? (3.535 * a + 2.181 * a * a) / (1 + 2.276 * a + 2.577 * a * a) : 1.0;
  return (float)g;
}

/* ndf/ggx.h:50-65 eval */
static float ggx_eval(v3 h, float au, float av)
{
  if (!(h.z > 0)) return 0;
  float alpha2 = (1.0f * au) * av;            /* hprod, horizontal.h:64-68 */
  float sx = h.x / au, sy = h.y / av;
  float sn = (0.0f + sx * sx) + sy * sy;
  double d = kPiF * alpha2 * pow((double)(sn + powf(h.z, 2.0f)), 2.0);
  return (float)(1 / d);
}

/* ndf/ggx.h:173-189 G1 */
static float ggx_G1(v3 v, v3 m, float au, float av)
{
  if (!((v.z > 0) && (dot3(v, m) > 0))) return 0;
  float r2 = (1.0f * au) * av;
  float t2 = tan_theta2(v);
  float denom = (float)(1.0 + sqrt(1.0 + r2 * t2));
  return (float)(2.0 / denom);
}

/* ndf/{beckmann,ggx}.h pdf (beckmann.h:149-170, ggx.h:142-163): VNDF pdf D*G1*|v.m|/cos(v) */
typedef enum { NDF_BECKMANN, NDF_BECKMANN_NORM, NDF_GGX } ndf_kind;

static float ndf_eval(ndf_kind k, v3 h, float au, float av)
{
  return (k == NDF_GGX) ? ggx_eval(h, au, av) : beckmann_eval(h, au, av, k == NDF_BECKMANN_NORM);
}

static float ndf_G1(ndf_kind k, v3 v, v3 m, float au, float av, int aniso)
{
  return (k == NDF_GGX) ? ggx_G1(v, m, au, av) : beckmann_G1(v, m, au, av, aniso);
}

static float ndf_pdf(ndf_kind k, v3 view, v3 m, float au, float av, int aniso)
{
  if (!(m.z > 0)) return 0;
  float pdf = ndf_eval(k, m, au, av);
  pdf *= ndf_G1(k, view, m, au, av, aniso) * fabsf(dot3(view, m)) / view.z;
  if (!(pdf > 0)) return 0;
  return pdf;
}

/* ---------------------------------------------------------------- masking-shadowing */

typedef enum { MS_VGROOVE, MS_UNCORRELATED } ms_kind;

/* maskingshadowing/vgroove.h:30-47 (double via 2.0 literal, fmin) and uncorrelated.h:30-42 */
static float ms_eval(ms_kind ms, ndf_kind k, v3 in, v3 out, v3 m, float au, float av, int aniso)
{
  if (!((dot3(in, m) > 0) && (dot3(out, m) > 0))) return 0;
  if (ms == MS_VGROOVE)
  {
    double gi = 2.0 * m.z * in.z / dot3(in, m);
    double go = 2.0 * m.z * out.z / dot3(out, m);
    return (float)fmin(1.0, fmin(gi, go));
  }
  return ndf_G1(k, in, m, au, av, aniso) * ndf_G1(k, out, m, au, av, aniso);
}

/* ---------------------------------------------------------------- fresnel */

/* bbm/fresnel_cook.h:41-56 (float math; final bbm::max(x, 0.0) in double -> NaN becomes 0) */
static float fresnel_cook(float eta, float c)
{
  float g = safe_sqrtf(eta * eta + c * c - 1.0f);
  float a = (g - c) / (g + c);
  float b = (c * (g + c) - 1.0f) / (c * (g - c) + 1.0f);
  return (float)fmax(0.5f * (a * a) * (1.0f + b * b), 0.0);
}

/* ---------------------------------------------------------------- models */

typedef struct {
  const char* name;
  ndf_kind ndf;
  ms_kind ms;
  double norm;       /* microfacet_n (bsdfmodel/microfacet.h:31-36) */
  int aniso;         /* roughness is a Vec2d */
} microfacet_desc;

/* composition table: bsdfmodel/cooktorrance.h:28-34, ggx.h:27-33, cooktorrancewalter.h:32-38,
   low.h:32-33 (LowCookTorrance == cooktorrance) */
static const microfacet_desc kMicrofacet[] = {
  { "CookTorrance",       NDF_BECKMANN,      MS_VGROOVE,      PI_D, 0 },
  { "LowCookTorrance",    NDF_BECKMANN,      MS_VGROOVE,      PI_D, 0 },
  { "GGX",                NDF_GGX,           MS_UNCORRELATED, 4.0,  0 },
  { "CookTorranceWalter", NDF_BECKMANN_NORM, MS_UNCORRELATED, 4.0,  0 },
};
#define N_MICROFACET (int)(sizeof(kMicrofacet) / sizeof(kMicrofacet[0]))

/* bsdfmodel/microfacet.h:74-102 eval (scaled by albedo in scaledmodel.h:50-53) */
static void microfacet_eval(const microfacet_desc* d, const float* p, v3 in, v3 out, uint32_t comp, float* rgb)
{
  rgb[0] = rgb[1] = rgb[2] = 0;
  if (!(comp & FLAG_SPECULAR)) return;
  if (!((in.z > 0.0f) && (out.z > 0.0f))) return;
  const float au = p[3], av = d->aniso ? p[4] : p[3], eta = d->aniso ? p[5] : p[4];
  v3 h = halfway(in, out);
  float inh = dot3(in, h), outh = dot3(out, h);
  float D = ndf_eval(d->ndf, h, au, av);
  float G = ms_eval(d->ms, d->ndf, in, out, h, au, av, d->aniso);
  float F = fresnel_cook(eta, 0.5f * (inh + outh));
  float res = (float)(D * G * F / d->norm / (in.z * out.z));
  rgb[0] = res * p[0]; rgb[1] = res * p[1]; rgb[2] = res * p[2];
}

/* bsdfmodel/microfacet.h:154-174 pdf */
static float microfacet_pdf(const microfacet_desc* d, const float* p, v3 in, v3 out, uint32_t comp)
{
  if (!(comp & FLAG_SPECULAR)) return 0;
  if (!((out.z > 0) && (in.z > 0))) return 0;
  const float au = p[3], av = d->aniso ? p[4] : p[3];
  v3 h = halfway(in, out);
  if (h.z < 0) { h.x = -h.x; h.y = -h.y; h.z = -h.z; }
  double pdf = ndf_pdf(d->ndf, out, h, au, av, d->aniso) / (4.0 * fabsf(dot3(out, h)));
  return (float)pdf;
}

/* bsdfmodel/lambertian.h:45-59 eval, 115-125 pdf (non-strict z >= 0) */
static void lambertian_eval(const float* p, v3 in, v3 out, uint32_t comp, float* rgb)
{
  rgb[0] = rgb[1] = rgb[2] = 0;
  if (!(comp & FLAG_DIFFUSE)) return;
  if (!((in.z >= 0) && (out.z >= 0))) return;
  rgb[0] = p[0] * kInvPiF; rgb[1] = p[1] * kInvPiF; rgb[2] = p[2] * kInvPiF;
}

static float lambertian_pdf(v3 in, v3 out, uint32_t comp)
{
  if (!(comp & FLAG_DIFFUSE)) return 0;
  if (!((in.z >= 0) && (out.z >= 0))) return 0;
  return in.z * kInvPiF;
}

/* bsdfmodel/lambertian.h:76-103 sample (cosine-weighted) */
static void lambertian_sample(v3 out, float xi0, float xi1, uint32_t comp, v3* dir, float* pdf, uint32_t* flag)
{
  dir->x = dir->y = dir->z = 0; *pdf = 0; *flag = FLAG_NONE;
  if (!(comp & FLAG_DIFFUSE)) return;
  if (!((xi0 >= 0) && (xi1 >= 0) && (xi0 <= 1) && (xi1 <= 1))) return;
  float phi = xi0 * (float)(2.0f * PI_D);                  /* Constants::Pi(2) */
  float c = cosf(phi), s = sinf(phi);
  float sin_t = (float)safe_sqrt(1.0 - xi1);
  dir->x = c * sin_t; dir->y = s * sin_t; dir->z = safe_sqrtf(xi1);
  *pdf = lambertian_pdf(*dir, out, comp);
  *flag = FLAG_DIFFUSE;
}


/* ---------------------------------------------------------------- sampling */

static const float kInvSqrtPiF = (float)(1.0f * 0.564189583547756286948079451560772586);
static const float kEpsF = 1.1920928955078125e-07f;

/* std::clamp(a, T(lo), T(hi)) (backbone/native/include/backbone/math.h:106-107) */
static inline float clampf(float a, float lo, float hi) { return (a < lo) ? lo : ((hi < a) ? hi : a); }

/* backbone/native/include/backbone/math.h:115-126: Giles' erfinv; w rounds to T, the Horner
   polynomial (util/poly.h:34-38) runs in double and the result stays double */
static double erfinv_d(float a)
{
  float w = (float)(-log((1.0 - a) * (1.0 + a)));
  if (w < 5)
  {
    double x = w - 2.5;
    double p = 2.81022636e-08;
    p = p * x + 3.43273939e-07; p = p * x + -3.5233877e-06; p = p * x + -4.39150654e-06;
    p = p * x + 0.00021858087; p = p * x + -0.00125372503; p = p * x + -0.00417768164;
    p = p * x + 0.246640727; p = p * x + 1.50140941;
    return p * a;
  }
  double x = sqrtf(w) - 3.0;
  double p = -0.000200214257;
  p = p * x + 0.000100950558; p = p * x + 0.00134934322; p = p * x + -0.00367342844;
  p = p * x + 0.00573950773; p = p * x + -0.0076224613; p = p * x + 0.00943887047;
  p = p * x + 1.00167406; p = p * x + 2.83297682;
  return p * a;
}

/* core/spherical.h:155-160 cossinPhi */
static inline void cossin_phi(v3 v, float* c, float* s)
{
  float sT = sqrtf(sin_theta2(v));
  float rsT = 1 / sT;
  if (fabsf(sT) < kEpsF) { *c = 1; *s = 0; return; }
  *c = clampf(v.x * rsT, -1.0f, 1.0f);
  *s = clampf(v.y * rsT, -1.0f, 1.0f);
}

static inline v3 cross3(v3 a, v3 b)
{
  v3 r = { a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x };
  return r;
}

/* ndf/beckmann.h:76-116 VNDF sampling following [Jakob 2014] */
static v3 beckmann_sample(v3 view, float xi0, float xi1, float au, float av)
{
  v3 zero = { 0, 0, 0 };
  if (!((xi0 >= 0) && (xi1 >= 0) && (xi0 <= 1) && (xi1 <= 1))) return zero;
  v3 st = { view.x * au, view.y * av, view.z };
  v3 vs = normalize3(st);
  float tanT = tan_theta(vs);
  float maxval = erff(1 / tanT);
  float xc0 = clampf(xi0, (float)10e-6, (float)(1.0 - 10e-6));
  float xc1 = clampf(xi1, (float)10e-6, (float)(1.0 - 10e-6));
  float x = maxval - (maxval + 1) * erff(sqrtf(-logf(xc0)));
  xc0 = (float)(xc0 * (1.0 + maxval + kInvSqrtPiF * tanT * expf(-(vs.z * vs.z))));
  for (int i = 0; i < 3; ++i)
  {
    float slope = (float)erfinv_d(x);
    float val = (float)(1.0 + x + kInvSqrtPiF * tanT * expf(-slope * slope) - xc0);
    float der = (float)(1.0 - slope * tanT);
    x -= val / der;
  }
  float s0 = 0, s1 = 0;
  float t1 = (float)(2.0 * xc1 - 1.0);
  double e0 = erfinv_d(x), e1 = erfinv_d(t1);
  if (x > -1.0 && x < +1.0) { s0 = (float)e0; s1 = (float)e1; }
  float c, s;
  cossin_phi(vs, &c, &s);
  float u0 = ((0.0f + c * s0) + -s * s1) * au;
  float u1 = ((0.0f + s * s0) + c * s1) * av;
  v3 m = { -u0, -u1, 1 };
  return normalize3(m);
}

/* ndf/ggx.h:84-108 VNDF sampling following [Heitz 2017] */
static v3 ggx_sample(v3 view, float xi0, float xi1, float au, float av)
{
  v3 zero = { 0, 0, 0 };
  if (!((xi0 >= 0) && (xi1 >= 0) && (xi0 <= 1) && (xi1 <= 1))) return zero;
  v3 st = { view.x * au, view.y * av, view.z };
  v3 vs = normalize3(st);
  v3 ez = { 0, 0, 1 }, ex = { 1, 0, 0 };
  v3 T1 = (vs.z < 1.0 - kEpsF) ? normalize3(cross3(vs, ez)) : ex;
  v3 T2 = cross3(T1, vs);
  float a = (float)(1 / (1.0 + vs.z));
  float r = sqrtf(xi0);
  float phi = (float)(((xi1 < a) ? (double)(xi1 / a) : 1.0 + (xi1 - a) / (1.0 - a)) * kPiF);
  float cp = cosf(phi), sp = sinf(phi);
  float P1 = r * cp;
  float P2 = (float)(((xi1 < a) ? 1.0 : (double)vs.z) * r * sp);
  float sq = (float)safe_sqrt(1.0 - P1 * P1 - P2 * P2);
  v3 nrm = { (T1.x * P1 + T2.x * P2) + vs.x * sq, (T1.y * P1 + T2.y * P2) + vs.y * sq,
             (T1.z * P1 + T2.z * P2) + vs.z * sq };
  v3 un = { nrm.x * au, nrm.y * av, (float)fmax(0.0, (double)nrm.z) };
  return normalize3(un);
}

/* bsdfmodel/microfacet.h:115-141 sample: reflect(out, m) (core/vec_transform.h:43-44), pdf */
static void microfacet_sample(const microfacet_desc* d, const float* p, v3 out, float xi0, float xi1, uint32_t comp,
                              v3* dir, float* pdf, uint32_t* flag)
{
  dir->x = dir->y = dir->z = 0; *pdf = 0; *flag = FLAG_NONE;
  if (!(comp & FLAG_SPECULAR)) return;
  if (!((xi0 >= 0) && (xi1 >= 0) && (xi0 <= 1) && (xi1 <= 1))) return;
  if (!(out.z > 0)) return;
  const float au = p[3], av = d->aniso ? p[4] : p[3];
  v3 m = (d->ndf == NDF_GGX) ? ggx_sample(out, xi0, xi1, au, av) : beckmann_sample(out, xi0, xi1, au, av);
  float dm = dot3(m, out);
  dir->x = (float)((double)(m.x * dm) * 2.0 - out.x);
  dir->y = (float)((double)(m.y * dm) * 2.0 - out.y);
  dir->z = (float)((double)(m.z * dm) * 2.0 - out.z);
  *pdf = microfacet_pdf(d, p, *dir, out, comp);
  *flag = FLAG_SPECULAR;
}

/* ---------------------------------------------------------------- dispatch */

enum { M_LAMBERTIAN = -1 };

static int find_model(const char* name)
{
  if (strcmp(name, "Lambertian") == 0) return M_LAMBERTIAN;
  for (int i = 0; i < N_MICROFACET; ++i)
    if (strcmp(name, kMicrofacet[i].name) == 0) return i;
  return -1000;
}

int bbmport_num_models(void) { return N_MICROFACET + 1; }

const char* bbmport_model_name(int i)
{
  if (i == 0) return "Lambertian";
  if (i >= 1 && i <= N_MICROFACET) return kMicrofacet[i - 1].name;
  return 0;
}

int bbmport_eval_pdf(const char* name, const float* params, int nparams, size_t n,
                     const float* ix, const float* iy, const float* iz,
                     const float* ox, const float* oy, const float* oz,
                     uint32_t component, uint32_t unit, int mode,
                     float* r, float* g, float* b, float* pdf, int nthreads)
{
  (void)unit; (void)nparams;   /* unit is ignored by every model on this path */
  int m = find_model(name);
  if (m == -1000) return -1;
  const microfacet_desc* d = (m >= 0) ? &kMicrofacet[m] : 0;
  #pragma omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : 1)
  for (long long i = 0; i < (long long)n; ++i)
  {
    v3 in = { ix[i], iy[i], iz[i] }, out = { ox[i], oy[i], oz[i] };
    if (mode & 1)
    {
      float rgb[3];
      if (d) microfacet_eval(d, params, in, out, component, rgb);
      else lambertian_eval(params, in, out, component, rgb);
      r[i] = rgb[0]; g[i] = rgb[1]; b[i] = rgb[2];
    }
    if (mode & 2) pdf[i] = d ? microfacet_pdf(d, params, in, out, component) : lambertian_pdf(in, out, component);
  }
  return 0;
}

int bbmport_sample(const char* name, const float* params, int nparams, size_t n,
                   const float* ox, const float* oy, const float* oz,
                   const float* xi0, const float* xi1, uint32_t component, uint32_t unit,
                   float* dx, float* dy, float* dz, float* pdf, uint32_t* flag, int nthreads)
{
  (void)unit; (void)nparams;
  int m = find_model(name);
  if (m == -1000) return -1;
  const microfacet_desc* d = (m >= 0) ? &kMicrofacet[m] : 0;
  #pragma omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : 1)
  for (long long i = 0; i < (long long)n; ++i)
  {
    v3 out = { ox[i], oy[i], oz[i] }, dir;
    if (d) microfacet_sample(d, params, out, xi0[i], xi1[i], component, &dir, &pdf[i], &flag[i]);
    else lambertian_sample(out, xi0[i], xi1[i], component, &dir, &pdf[i], &flag[i]);
    dx[i] = dir.x; dy[i] = dir.y; dz[i] = dir.z;
  }
  return 0;
}

int bbmport_libm(int func, const float* a, const float* b, float* out, size_t n)
{
  for (size_t i = 0; i < n; ++i)
  {
    switch (func)
    {
      case 0: out[i] = expf(a[i]); break;
      case 1: out[i] = logf(a[i]); break;
      case 2: out[i] = powf(a[i], b[i]); break;
      case 3: out[i] = erff(a[i]); break;
      case 4: out[i] = erfcf(a[i]); break;
      case 6: out[i] = sinf(a[i]); break;
      case 7: out[i] = cosf(a[i]); break;
      case 8: out[i] = atan2f(a[i], b[i]); break;
      default: return -1;
    }
  }
  return 0;
}

/* ---------------------------------------------------------------------------------------------------------------
 * EPD's shadowing table: the arithmetic of the reference's generator precompute/HolzschuchPacanowski/G1.cpp
 * (P2 :91-113, G1series :174-223, rows :280-300) in floatRGB, one row p = 5 / (row + 1) at a time.  contract != 0
 * evaluates the three products GCC contracts into FMAs when the generator is built with FMA available and the
 * default -ffp-contract=fast of gnu++20 (x86-64-v3; objdump of that build shows exactly these three vfmadd): P2's
 * `r2 + q*q` (:107) and `integral += delta_q * exp(...)` (:107), and the series' `integral[j] += (r*t - 1) * p2`
 * (:205).  With contract = 1 every entry of a row equals the shipped include/precomputed/holzschuchpacanowski/G1.h;
 * with contract = 0 (each op rounded on its own) 3.6 % of the table differs in the 6th printed digit
 * (tests/test_oracle.py::test_epd_g1_generator_recipe).  out: 1000 floats, each the "%g" (ostream << float,
 * precision 6) print of G1 read back as the header's literal is. */
static float g1_conv_f(float x) { return powf(logf(1.0f / x), 20.0f); }
static double g1_conv_d(double x) { return pow(log(1.0 / x), (double)20.0f); }

int bbmport_epd_g1_row(int row, int contract, float* out)
{
  if (row < 0 || row >= 100 || !out) return -1;
  const float p = (float)(5.0 / (double)(float)(row + 1));
  const float norm = (float)((double)p / ((double)kPiF * tgamma(1.0 / (double)p)));
  float integral[1000];
  integral[0] = 0.0f;
  float prev = 0.0f, Pj = 0.0f;
  const float delta_x = 1.0f / 1000.0f;
  for (int j = 1; j < 1000; ++j)
  {
    const float x = (float)(j + 1) / 1000.0f;
    const float t = 1.0f / g1_conv_f(x);
    if (isinf(t)) { integral[j] = t; continue; }
    const float dr = g1_conv_f(x - delta_x) - g1_conv_f(x);
    const float r = (float)g1_conv_d((double)x - 0.5 * (double)delta_x);
    /* P2(r, p) */
    const float r2 = r * r;
    const float deltax = 0.0001f;
    float s = 0.0f;
    for (float xx = 1.0f; xx > deltax; xx -= deltax)
    {
      const float dq = g1_conv_f(xx - deltax) - g1_conv_f(xx);
      const float q = (float)g1_conv_d((double)xx - 0.5 * (double)deltax);
      if (isnan(dq)) continue;
      const float base = contract ? fmaf(q, q, r2) : r2 + q * q;
      const float e = expf(-powf(base, p));
      s = contract ? fmaf(dq, e, s) : s + dq * e;
    }
    const float p2 = (float)(2.0 * (double)norm * (double)s) * dr;
    float v = 0.0f;
    if (prev > 0) v = (integral[j - 1] + Pj) * t / prev - Pj;
    if (r * t > 1) v = contract ? fmaf(r * t - 1, p2, v) : v + (r * t - 1) * p2;
    integral[j] = v;
    prev = t;
    Pj += p2;
  }
  for (int j = 0; j < 1000; ++j)
  {
    char buf[64];
    snprintf(buf, sizeof(buf), "%g", (double)(float)(1.0 / (1.0 + (double)integral[j])));
    out[j] = (float)strtod(buf, NULL);
  }
  return 0;
}

/* Exhaustive libm pins (tests/test_gpu_libm.py): the inputs are the float bit patterns start .. start + n - 1; got[i]
 * is the device's value for pattern start + i (bbm_hip_libm_eval).  Returns the number of patterns whose host libm
 * value differs bitwise (any NaN equals any NaN), and writes up to `cap` of them to bad[]. */
long long bbmport_libm_sweep(int func, uint32_t start, size_t n, const float* got, uint32_t* bad, int cap, int nthreads)
{
  long long nbad = 0;
  #pragma omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : 1)
  for (long long i = 0; i < (long long)n; ++i)
  {
    const uint32_t bits = start + (uint32_t)i;
    float x;
    memcpy(&x, &bits, 4);
    float r;
    switch (func)
    {
      case 0: r = expf(x); break;
      case 1: r = logf(x); break;
      case 3: r = erff(x); break;
      case 4: r = erfcf(x); break;
      case 6: r = sinf(x); break;
      case 7: r = cosf(x); break;
      default: r = x; break;
    }
    uint32_t a, b;
    memcpy(&a, &r, 4);
    memcpy(&b, &got[i], 4);
    if (a != b && !(isnan(r) && isnan(got[i])))
    {
      long long k;
      #pragma omp atomic capture
      k = nbad++;
      if (k < cap && bad) bad[k] = bits;
    }
  }
  return nbad;
}
