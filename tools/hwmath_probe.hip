// Accuracy of the gfx950 transcendental unit (v_log_f32, v_exp_f32, v_rcp_f32) against f64, over every
// float in a range: used to size the fast/slow split of powf_acc (bbm_amd/csrc/math.hpp).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <math.h>
#include <stdint.h>

__global__ void k_log(uint32_t lo, uint32_t n, double* err_abs, double* err_rel)
{
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  double ea = 0, er = 0;
  for (uint32_t k = i; k < n; k += gridDim.x * blockDim.x)
  {
    uint32_t bits = lo + k;
    float x = __uint_as_float(bits);
    float l = __builtin_amdgcn_logf(x);
    double ref = log2((double)x);
    double a = fabs((double)l - ref);
    ea = fmax(ea, a);
    if (ref != 0) er = fmax(er, a / fabs(ref));
  }
  err_abs[i] = ea; err_rel[i] = er;
}

__global__ void k_exp(float lo, float hi, uint32_t n, double* err_rel)
{
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  double er = 0;
  for (uint32_t k = i; k < n; k += gridDim.x * blockDim.x)
  {
    float x = lo + (hi - lo) * (float)k / (float)n;
    double ref = exp2((double)x);
    double a = fabs((double)__builtin_amdgcn_exp2f(x) - ref) / ref;
    er = fmax(er, a);
  }
  err_rel[i] = er;
}

int main()
{
  const int T = 256 * 1024;
  double *ea, *er;
  hipMalloc(&ea, T * 8); hipMalloc(&er, T * 8);
  double* h1 = (double*)malloc(T * 8); double* h2 = (double*)malloc(T * 8);
  struct { float a, b; } ranges[] = {{0.5f, 2.0f}, {0.99f, 1.01f}, {0.999999f, 1.000001f}, {1e-30f, 1e30f}};
  for (auto r : ranges)
  {
    uint32_t lo = *(uint32_t*)&r.a, hi = *(uint32_t*)&r.b;
    k_log<<<1024, 256>>>(lo, hi - lo, ea, er);
    hipMemcpy(h1, ea, T * 8, hipMemcpyDeviceToHost); hipMemcpy(h2, er, T * 8, hipMemcpyDeviceToHost);
    double ma = 0, mr = 0;
    for (int i = 0; i < T; ++i) { ma = fmax(ma, h1[i]); mr = fmax(mr, h2[i]); }
    printf("v_log_f32 x in [%g, %g]: max abs err %.3e (= %.2f * 2^-24), max rel err %.3e (= %.2f * 2^-24)\n", r.a, r.b,
           ma, ma * 16777216.0, mr, mr * 16777216.0);
  }
  k_exp<<<1024, 256>>>(-1.0f, 1.0f, 1u << 30, er);
  hipMemcpy(h2, er, T * 8, hipMemcpyDeviceToHost);
  double mr = 0;
  for (int i = 0; i < T; ++i) mr = fmax(mr, h2[i]);
  printf("v_exp_f32 x in [-1, 1]: max rel err %.3e (= %.2f * 2^-24)\n", mr, mr * 16777216.0);
  return 0;
}
