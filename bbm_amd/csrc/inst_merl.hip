// bbm_amd/csrc/inst_merl.hip -- kernel instantiations for Merl (merl.hpp) and the MERL table builder.
#include "kernels.hpp"
#include "models.hpp"

namespace bbmhip {
BBM_HIP_MERL_MODELS(BBM_HIP_INSTANTIATE)

// merl.h:199-203, one entry per thread: three f64 reads (one per channel plane), one 16 B f32 write
__global__ __launch_bounds__(256) void k_merl_table(const double* __restrict__ raw, float4* __restrict__ table)
{
  math_tables_init();
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= kMerlSize) return;
  const double r = fmax(0.0, raw[i] * 1.0 / 1500.0);
  const double g = fmax(0.0, raw[kMerlSize + i] * 1.15 / 1500.0);
  const double b = fmax(0.0, raw[2u * kMerlSize + i] * 1.66 / 1500.0);
  table[i] = make_float4(float(r), float(g), float(b), 0.0f);
}

int merl_table_launch(const double* raw, float* table, hipStream_t s)
{
  hipLaunchKernelGGL(k_merl_table, dim3((kMerlSize + 255u) / 256u), dim3(256), 0, s, raw, reinterpret_cast<float4*>(table));
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(BBM_HIP_ERR_HIP, std::string("Merl table: launch: ") + hipGetErrorString(e));
  return BBM_HIP_OK;
}
}  // namespace bbmhip
