/* oracle/libm_ulp.c -- TEST INFRASTRUCTURE ONLY: linked into oracle/_ref/libbbm_ref.so.
 *
 * Wrappers around the glibc float functions the reference's native backbone calls (std::erf(float) -> erff,
 * std::exp(float) -> expf, ...: backbone/native/include/backbone/math.h:51-57 brings in the std:: overloads),
 * so that a parity test can ask the reference itself: "if one call of libm function F returned its
 * neighbouring float, would the reference produce the GPU's value?"  glibc's float functions are not correctly
 * rounded (erff and erfcf differ from the correctly rounded result on ~6 % of inputs, sinf on ~0.5 %), and the
 * GPU evaluates the same functions with other last-bit behaviour, so an ill-conditioned output (an inverse-CDF
 * sample at a clamped xi, a cancellation) can differ by more than 1e-5 for that reason alone.  The test proves
 * such a lane by finding the single call whose 1-ulp change reproduces the GPU value (tests/oracle_util.py).
 *
 * The library is linked with -Bsymbolic-functions, so the reference code inside it calls these definitions;
 * each forwards to glibc's own function (dlsym(RTLD_NEXT)) and, when the thread's perturbation selects it,
 * moves the result by `ulps` floats.  Default: no perturbation (results are glibc's, bit for bit).
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <math.h>
#include <string.h>

enum { F_ERFF, F_ERFCF, F_EXPF, F_LOGF, F_POWF, F_SINF, F_COSF, F_TANF, F_ATANF, F_ATAN2F, F_ACOSF, F_SINCOSF_S,
       F_SINCOSF_C, F_TGAMMAF, F_NFN };

static __thread int g_fn = -1, g_call = -1, g_ulps = 0;
static __thread int g_count[F_NFN];

static float bump(int fn, float r)
{
  const int c = g_count[fn]++;
  if (fn == g_fn && (g_call < 0 || c == g_call))
    for (int k = 0; k < (g_ulps < 0 ? -g_ulps : g_ulps); ++k) r = nextafterf(r, g_ulps > 0 ? INFINITY : -INFINITY);
  return r;
}

#define REAL(name, type) \
  static type real = 0; \
  if (!real) real = (type)dlsym(RTLD_NEXT, name)

typedef float (*f1)(float);
typedef float (*f2)(float, float);
typedef void (*fsc)(float, float*, float*);

float erff(float x) { REAL("erff", f1); return bump(F_ERFF, real(x)); }
float erfcf(float x) { REAL("erfcf", f1); return bump(F_ERFCF, real(x)); }
float expf(float x) { REAL("expf", f1); return bump(F_EXPF, real(x)); }
float logf(float x) { REAL("logf", f1); return bump(F_LOGF, real(x)); }
float powf(float x, float y) { REAL("powf", f2); return bump(F_POWF, real(x, y)); }
float sinf(float x) { REAL("sinf", f1); return bump(F_SINF, real(x)); }
float cosf(float x) { REAL("cosf", f1); return bump(F_COSF, real(x)); }
float tanf(float x) { REAL("tanf", f1); return bump(F_TANF, real(x)); }
float atanf(float x) { REAL("atanf", f1); return bump(F_ATANF, real(x)); }
float atan2f(float y, float x) { REAL("atan2f", f2); return bump(F_ATAN2F, real(y, x)); }
float acosf(float x) { REAL("acosf", f1); return bump(F_ACOSF, real(x)); }
float tgammaf(float x) { REAL("tgammaf", f1); return bump(F_TGAMMAF, real(x)); }
void sincosf(float x, float* s, float* c)
{
  REAL("sincosf", fsc);
  real(x, s, c);
  *s = bump(F_SINCOSF_S, *s);
  *c = bump(F_SINCOSF_C, *c);
}

/* Select the perturbation of this thread's following calls (fn < 0: none) and reset the call counters. */
void bbmref_libm_ulp(int fn, int call, int ulps)
{
  g_fn = fn;
  g_call = call;
  g_ulps = ulps;
  memset(g_count, 0, sizeof(g_count));
}

/* Calls of `fn` made by this thread since the last bbmref_libm_ulp (to enumerate single-call perturbations). */
int bbmref_libm_calls(int fn) { return (fn >= 0 && fn < F_NFN) ? g_count[fn] : -1; }
int bbmref_libm_nfn(void) { return F_NFN; }
