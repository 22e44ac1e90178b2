// tools/roofprobe.hip -- calibration only (not part of the product): the HBM ceiling of the
// eval+pdf access pattern (6 SoA float streams in, 4 out, 16 B per lane) with trivial compute,
// so the CookTorrance kernel's achieved bandwidth can be read against what this pattern can
// reach on MI355X, not only against the 8 TB/s spec.
//   variant 0: plain loads/stores, 4 pairs per thread-iteration (the product kernel's shape)
//   variant 1: nontemporal loads and stores
//   variant 2: 8 pairs per thread-iteration (two float4 per stream in flight)
//   variant 3: read-only (6 streams), variant 4: write-only (4 streams)
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f4 __attribute__((ext_vector_type(4)));
struct Args { const f4* in[6]; f4* out[4]; uint64_t n4; };

template<int V>
__global__ __launch_bounds__(256) void k_probe(Args a)
{
  const uint64_t stride = uint64_t(gridDim.x) * 256;
  if (V == 2)
  {
    for (uint64_t t = (uint64_t(blockIdx.x) * 256 + threadIdx.x); t < a.n4 / 2; t += stride)
    {
      f4 v[6][2];
#pragma unroll
      for (int k = 0; k < 6; ++k) { v[k][0] = a.in[k][t]; v[k][1] = a.in[k][t + a.n4 / 2]; }
#pragma unroll
      for (int u = 0; u < 2; ++u)
      {
        const uint64_t i = t + u * (a.n4 / 2);
        f4 s = v[0][u];
        s.x += v[3][u].x; s.y += v[4][u].y; s.z += v[5][u].z; s.w += v[1][u].w + v[2][u].x;
        a.out[0][i] = s; a.out[1][i] = v[1][u]; a.out[2][i] = v[2][u]; a.out[3][i] = v[4][u];
      }
    }
    return;
  }
  for (uint64_t t = uint64_t(blockIdx.x) * 256 + threadIdx.x; t < a.n4; t += stride)
  {
    if (V == 4)
    {
      const float f = float(t);
      a.out[0][t] = f4{f, f, f, f}; a.out[1][t] = f4{f, f, f, f};
      a.out[2][t] = f4{f, f, f, f}; a.out[3][t] = f4{f, f, f, f};
      continue;
    }
    f4 v[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) v[k] = (V == 1) ? __builtin_nontemporal_load(&a.in[k][t]) : a.in[k][t];
    f4 s = v[0];
    s.x += v[3].x; s.y += v[4].y; s.z += v[5].z; s.w += v[1].w + v[2].x;
    if (V == 3)
    {
      if (s.x == 12345.678f) a.out[0][t] = s;   // keep loads live; never true for unit vectors
      continue;
    }
    if (V == 1)
    {
      __builtin_nontemporal_store(s, &a.out[0][t]); __builtin_nontemporal_store(v[1], &a.out[1][t]);
      __builtin_nontemporal_store(v[2], &a.out[2][t]); __builtin_nontemporal_store(v[4], &a.out[3][t]);
    }
    else { a.out[0][t] = s; a.out[1][t] = v[1]; a.out[2][t] = v[2]; a.out[3][t] = v[4]; }
  }
}

extern "C" int roofprobe(int variant, const float* const* in, float* const* out, uint64_t n, int blocks, void* stream)
{
  Args a;
  for (int k = 0; k < 6; ++k) a.in[k] = reinterpret_cast<const f4*>(in[k]);
  for (int k = 0; k < 4; ++k) a.out[k] = reinterpret_cast<f4*>(out[k]);
  a.n4 = n / 4;
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (variant)
  {
    case 0: hipLaunchKernelGGL(k_probe<0>, dim3(blocks), dim3(256), 0, s, a); break;
    case 1: hipLaunchKernelGGL(k_probe<1>, dim3(blocks), dim3(256), 0, s, a); break;
    case 2: hipLaunchKernelGGL(k_probe<2>, dim3(blocks), dim3(256), 0, s, a); break;
    case 3: hipLaunchKernelGGL(k_probe<3>, dim3(blocks), dim3(256), 0, s, a); break;
    case 4: hipLaunchKernelGGL(k_probe<4>, dim3(blocks), dim3(256), 0, s, a); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -4;
}
