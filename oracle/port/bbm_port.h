/* oracle/port/bbm_port.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C11) of the BBM native-backbone floatRGB semantics for the batched
 * eval/pdf/sample path.  Used only by tests/ (as a checker) and by bench.py's cpu_baseline leg
 * when the prebuilt reference harness is absent.  Never linked into the product (bbm_amd/).
 *
 * Pinned against the reference's own outputs: tests/golden/ (npz) (generated from the compiled
 * reference headers by oracle/gen_golden.py) -- see tests/test_oracle.py.
 *
 * Entry points mirror oracle/ref_harness.cpp so the two libraries are interchangeable.
 */
#ifndef BBM_PORT_H
#define BBM_PORT_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

int bbmport_num_models(void);
const char* bbmport_model_name(int i);

/* mode bit0 = eval (RGB), bit1 = pdf; SoA float inputs; nthreads <= 0 -> 1 */
int bbmport_eval_pdf(const char* name, const float* params, int nparams, size_t n,
                     const float* ix, const float* iy, const float* iz,
                     const float* ox, const float* oy, const float* oz,
                     uint32_t component, uint32_t unit, int mode,
                     float* r, float* g, float* b, float* pdf, int nthreads);

int bbmport_sample(const char* name, const float* params, int nparams, size_t n,
                   const float* ox, const float* oy, const float* oz,
                   const float* xi0, const float* xi1, uint32_t component, uint32_t unit,
                   float* dx, float* dy, float* dz, float* pdf, uint32_t* flag, int nthreads);

/* the host libm float functions elementwise (0 expf, 1 logf, 2 powf(a, b), 3 erff, 4 erfcf): what the reference's
 * native backbone calls, for pinning the device restatements (bbm_hip_libm_eval) on the same machine */
int bbmport_libm(int func, const float* a, const float* b, float* out, size_t n);

/* one row (p = 5 / (row + 1)) of EPD's shadowing table as the reference's generator computes it
 * (precompute/HolzschuchPacanowski/G1.cpp), printed to 6 digits and read back; contract != 0: with the FMA
 * contractions of the build that produced the shipped G1.h (see bbm_port.c).  out: 1000 floats. */
int bbmport_epd_g1_row(int row, int contract, float* out);

/* exhaustive sweep: host libm (func as bbmport_libm) on the float bit patterns start .. start + n - 1 against got[];
 * returns the mismatch count, the first `cap` mismatching patterns in bad[] */
long long bbmport_libm_sweep(int func, uint32_t start, size_t n, const float* got, uint32_t* bad, int cap, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
