// tools/roofprobe.hip -- calibration only (not part of the product): the HBM ceiling of the
// eval+pdf access pattern (6 SoA float streams in, 4 out, 16 B per lane) with trivial compute,
// so the CookTorrance kernel's achieved bandwidth can be read against what this pattern can
// reach on MI355X, not only against the 8 TB/s spec.
//   variant 0: plain loads/stores, 4 pairs per thread-iteration (the product kernel's shape)
//   variant 1: nontemporal loads and stores
//   variant 2: 8 pairs per thread-iteration (two float4 per stream in flight)
//   variant 3: read-only (6 streams), variant 4: write-only (4 streams)
//   variant 15: nontemporal loads, plain stores; variant 16: plain loads, nontemporal stores (the read-only and
//               write-only calibrations favour nt for reads and plain for writes)
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
      // keep every loaded float live (round 4's form tested s.x alone, so the compiler dropped 4 of the 6 streams'
      // loads and the variant reported 19.2 TB/s); never true for unit vectors
      float all = 0.0f;
#pragma unroll
      for (int k = 0; k < 6; ++k) all += (v[k].x + v[k].y) + (v[k].z + v[k].w);
      if (all == 12345.678f) a.out[0][t] = s;
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

// variant 5: float4 copy (1 stream in, 1 out), nontemporal -- the guide's copy calibration
// variant 6: 6in/4out nontemporal, two quads per lane interleaved per wave (quad t and t + 64 of the
//            wave's 128-quad tile), all 12 loads issued before any store
// variant 7: read-only nontemporal, variant 8: write-only nontemporal
template<int V>
__global__ __launch_bounds__(256) void k_probe2(Args a)
{
  const uint64_t stride = uint64_t(gridDim.x) * 256;
  if (V == 5)
  {
    for (uint64_t t = uint64_t(blockIdx.x) * 256 + threadIdx.x; t < a.n4; t += stride)
      __builtin_nontemporal_store(__builtin_nontemporal_load(&a.in[0][t]), &a.out[0][t]);
    return;
  }
  if (V == 6)
  {
    const uint64_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint64_t base = uint64_t(blockIdx.x) * 512 + wave * 128; base < a.n4; base += uint64_t(gridDim.x) * 512)
    {
      const uint64_t t0 = base + lane, t1 = base + 64 + lane;
      f4 v[6][2];
#pragma unroll
      for (int k = 0; k < 6; ++k)
      {
        v[k][0] = __builtin_nontemporal_load(&a.in[k][t0 < a.n4 ? t0 : a.n4 - 1]);
        v[k][1] = __builtin_nontemporal_load(&a.in[k][t1 < a.n4 ? t1 : a.n4 - 1]);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u)
      {
        const uint64_t i = u ? t1 : t0;
        if (i >= a.n4) continue;
        f4 s = v[0][u];
        s.x += v[3][u].x; s.y += v[4][u].y; s.z += v[5][u].z; s.w += v[1][u].w + v[2][u].x;
        __builtin_nontemporal_store(s, &a.out[0][i]); __builtin_nontemporal_store(v[1][u], &a.out[1][i]);
        __builtin_nontemporal_store(v[2][u], &a.out[2][i]); __builtin_nontemporal_store(v[4][u], &a.out[3][i]);
      }
    }
    return;
  }
  for (uint64_t t = uint64_t(blockIdx.x) * 256 + threadIdx.x; t < a.n4; t += stride)
  {
    if (V == 8)
    {
      const float f = float(t);
      __builtin_nontemporal_store(f4{f, f, f, f}, &a.out[0][t]); __builtin_nontemporal_store(f4{f, f, f, f}, &a.out[1][t]);
      __builtin_nontemporal_store(f4{f, f, f, f}, &a.out[2][t]); __builtin_nontemporal_store(f4{f, f, f, f}, &a.out[3][t]);
      continue;
    }
    f4 v[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) v[k] = __builtin_nontemporal_load(&a.in[k][t]);
    float all = 0.0f;
#pragma unroll
    for (int k = 0; k < 6; ++k) all += (v[k].x + v[k].y) + (v[k].z + v[k].w);
    if (all == 12345.678f) a.out[0][t] = v[0];     // every loaded float live (see variant 3)
  }
}

// variants 9 / 10: each workgroup streams a contiguous chunk of 16 / 64 consecutive 4 KiB tiles per
// stream (DRAM row locality), nontemporal; grid = n4 / (256 * tiles)
template<int TILES>
__global__ __launch_bounds__(256) void k_probe_chunk(Args a)
{
  const uint64_t first = uint64_t(blockIdx.x) * TILES * 256;
  for (int k2 = 0; k2 < TILES; ++k2)
  {
    const uint64_t t = first + uint64_t(k2) * 256 + threadIdx.x;
    if (t >= a.n4) return;
    f4 v[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) v[k] = __builtin_nontemporal_load(&a.in[k][t]);
    f4 s = v[0];
    s.x += v[3].x; s.y += v[4].y; s.z += v[5].z; s.w += v[1].w + v[2].x;
    __builtin_nontemporal_store(s, &a.out[0][t]); __builtin_nontemporal_store(v[1], &a.out[1][t]);
    __builtin_nontemporal_store(v[2], &a.out[2][t]); __builtin_nontemporal_store(v[4], &a.out[3][t]);
  }
}

// variants 12-14: the reference's own pair layout -- a Vec3dPair array (in xyz, out xyz: 24 B per pair, one
// stream) in, (r, g, b, pdf) float4 per pair (one stream) out; nontemporal.  a.in[0] / a.out[0] are the two
// arrays, n4 counts quads of pairs.
//   12: one pair per lane, lane-consecutive pairs (two 12 B loads, one 16 B store per lane)
//   13: four consecutive pairs per lane (six 16 B loads, four 16 B stores: lanes 96 B / 64 B apart)
//   14: four pairs per lane at wave stride 64 (pairs w*256 + k*64 + lane), 8 loads of 12 B in flight
struct P3 { float x, y, z; };
template<int V>
__global__ __launch_bounds__(256) void k_probe_aos(Args a)
{
  const float* in = reinterpret_cast<const float*>(a.in[0]);
  f4* out = a.out[0];
  const uint64_t npairs = a.n4 * 4;
  if (V == 12)
  {
    for (uint64_t p = uint64_t(blockIdx.x) * 256 + threadIdx.x; p < npairs; p += uint64_t(gridDim.x) * 256)
    {
      const float* q = in + p * 6;
      const float ix = __builtin_nontemporal_load(q + 0), iy = __builtin_nontemporal_load(q + 1), iz = __builtin_nontemporal_load(q + 2);
      const float ox = __builtin_nontemporal_load(q + 3), oy = __builtin_nontemporal_load(q + 4), oz = __builtin_nontemporal_load(q + 5);
      __builtin_nontemporal_store(f4{ix + ox, iy + oy, iz + oz, ix * oz}, &out[p]);
    }
    return;
  }
  if (V == 13)
  {
    const f4* in4 = a.in[0];
    for (uint64_t t = uint64_t(blockIdx.x) * 256 + threadIdx.x; t < a.n4; t += uint64_t(gridDim.x) * 256)
    {
      f4 v[6];
#pragma unroll
      for (int k = 0; k < 6; ++k) v[k] = __builtin_nontemporal_load(&in4[t * 6 + k]);
      __builtin_nontemporal_store(f4{v[0].x + v[0].w, v[0].y + v[1].x, v[0].z + v[1].y, v[0].x * v[1].z}, &out[t * 4 + 0]);
      __builtin_nontemporal_store(f4{v[1].w + v[2].z, v[2].x + v[2].w, v[2].y + v[3].x, v[1].w * v[3].x}, &out[t * 4 + 1]);
      __builtin_nontemporal_store(f4{v[3].y + v[4].y, v[3].z + v[4].z, v[3].w + v[4].w, v[3].y * v[4].w}, &out[t * 4 + 2]);
      __builtin_nontemporal_store(f4{v[5].x + v[5].w, v[5].y + v[5].x, v[5].z + v[5].y, v[5].x * v[5].z}, &out[t * 4 + 3]);
    }
    return;
  }
  if (V == 14)
  {
    const uint64_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint64_t base = (uint64_t(blockIdx.x) * 4 + wave) * 256; base < npairs; base += uint64_t(gridDim.x) * 1024)
    {
      float v[4][6];
#pragma unroll
      for (int k = 0; k < 4; ++k)
      {
        const uint64_t p = base + k * 64 + lane;
        const float* q = in + (p < npairs ? p : npairs - 1) * 6;
#pragma unroll
        for (int c = 0; c < 6; ++c) v[k][c] = __builtin_nontemporal_load(q + c);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k)
      {
        const uint64_t p = base + k * 64 + lane;
        if (p < npairs) __builtin_nontemporal_store(f4{v[k][0] + v[k][3], v[k][1] + v[k][4], v[k][2] + v[k][5], v[k][0] * v[k][5]}, &out[p]);
      }
    }
    return;
  }
}

template<bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_probe_mix(Args a)
{
  const uint64_t stride = uint64_t(gridDim.x) * 256;
  for (uint64_t t = uint64_t(blockIdx.x) * 256 + threadIdx.x; t < a.n4; t += stride)
  {
    f4 v[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) v[k] = NTL ? __builtin_nontemporal_load(&a.in[k][t]) : a.in[k][t];
    f4 s = v[0];
    s.x += v[3].x; s.y += v[4].y; s.z += v[5].z; s.w += v[1].w + v[2].x;
    if (NTS)
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
    case 5: hipLaunchKernelGGL(k_probe2<5>, dim3(blocks), dim3(256), 0, s, a); break;
    case 6: hipLaunchKernelGGL(k_probe2<6>, dim3(blocks), dim3(256), 0, s, a); break;
    case 7: hipLaunchKernelGGL(k_probe2<7>, dim3(blocks), dim3(256), 0, s, a); break;
    case 8: hipLaunchKernelGGL(k_probe2<8>, dim3(blocks), dim3(256), 0, s, a); break;
    case 9: hipLaunchKernelGGL(k_probe_chunk<16>, dim3((a.n4 + 16 * 256 - 1) / (16 * 256)), dim3(256), 0, s, a); break;
    case 10: hipLaunchKernelGGL(k_probe_chunk<64>, dim3((a.n4 + 64 * 256 - 1) / (64 * 256)), dim3(256), 0, s, a); break;
    case 11: hipLaunchKernelGGL(k_probe_chunk<4>, dim3((a.n4 + 4 * 256 - 1) / (4 * 256)), dim3(256), 0, s, a); break;
    case 12: hipLaunchKernelGGL(k_probe_aos<12>, dim3(blocks), dim3(256), 0, s, a); break;
    case 13: hipLaunchKernelGGL(k_probe_aos<13>, dim3(blocks), dim3(256), 0, s, a); break;
    case 14: hipLaunchKernelGGL(k_probe_aos<14>, dim3(blocks), dim3(256), 0, s, a); break;
    case 15: hipLaunchKernelGGL((k_probe_mix<true, false>), dim3(blocks), dim3(256), 0, s, a); break;
    case 16: hipLaunchKernelGGL((k_probe_mix<false, true>), dim3(blocks), dim3(256), 0, s, a); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -4;
}
