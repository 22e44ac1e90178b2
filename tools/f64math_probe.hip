// tools/f64math_probe.hip -- the doubleRGB exp / log / pow restatements (bbm_amd/csrc/f64.hpp: exp_d, log_d,
// pow_d, pow5_d) against the host's glibc exp / log / pow (what the reference's doubleRGB models call) on seeded
// random inputs over the ranges the models use: max error in ulps of the glibc result and the bit-exact fraction.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -ffp-contract=off -Ibbm_amd/csrc tools/f64math_probe.hip -o f64math_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
#include "f64.hpp"

using namespace bbmhip::f64;

__global__ void k_probe(int op, const double* x, const double* y, double* r, int n)
{
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  switch (op)
  {
  case 0: r[i] = exp_d(x[i]); break;
  case 1: r[i] = log_d(x[i]); break;
  case 2: r[i] = pow_d(x[i], y[i]); break;
  default: r[i] = pow5_d(x[i]); break;
  }
}

static double ulps(double got, double want)
{
  if (std::isnan(got) && std::isnan(want)) return 0;
  if (got == want) return 0;
  if (!std::isfinite(got) || !std::isfinite(want)) return 1e300;
  const double u = std::ldexp(1.0, std::max(std::ilogb(want), -1022) - 52);
  return std::fabs(got - want) / u;
}

int main()
{
  const int n = 1 << 22;
  std::mt19937_64 rng(0xBB5EED);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  const char* names[4] = {"exp_d", "log_d", "pow_d", "pow5_d"};
  double *dx, *dy, *dr;
  hipMalloc(&dx, n * 8); hipMalloc(&dy, n * 8); hipMalloc(&dr, n * 8);
  std::vector<double> x(n), y(n), r(n);
  int fail = 0;
  for (int op = 0; op < 4; ++op)
  {
    for (int i = 0; i < n; ++i)
    {
      const double u = U(rng), v = U(rng);
      switch (op)
      {
      case 0: x[i] = (i & 3) == 0 ? (u - 0.5) * 1e-3 : -745.0 + u * 1454.0; break;            // exp over the range
      case 1: x[i] = (i & 3) == 0 ? 1.0 + (u - 0.5) * std::ldexp(1.0, -int(v * 50)) : std::ldexp(0.5 + 0.5 * u, int(v * 2090) - 1070); break;
      case 2: {
        // bases in (0, 2] and near 1; exponents from -50 to 1e4, results kept inside the double range
        x[i] = (i & 3) == 0 ? 1.0 + (u - 0.5) * 1e-6 : std::ldexp(0.5 + 0.5 * u, -int(v * 30));
        const double ymax = std::min(1e4, 1000.0 / std::max(std::fabs(std::log2(x[i])), 1e-12));
        y[i] = -std::min(50.0, ymax) + U(rng) * (ymax + std::min(50.0, ymax));
        break; }
      default: x[i] = u; break;
      }
    }
    hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
    hipMemcpy(dy, y.data(), n * 8, hipMemcpyHostToDevice);
    k_probe<<<(n + 255) / 256, 256>>>(op, dx, dy, dr, n);
    if (hipDeviceSynchronize() != hipSuccess) { std::printf("kernel failed\n"); return 2; }
    hipMemcpy(r.data(), dr, n * 8, hipMemcpyDeviceToHost);
    double worst = 0, worst_x = 0, worst_y = 0;
    long exact = 0;
    for (int i = 0; i < n; ++i)
    {
      const double want = op == 0 ? std::exp(x[i]) : op == 1 ? std::log(x[i]) : op == 2 ? std::pow(x[i], y[i]) : std::pow(x[i], 5.0);
      if (std::fabs(want) < 2.2250738585072014e-308) continue;     // subnormal results: not ulp-comparable
      const double e = ulps(r[i], want);
      exact += e == 0;
      if (e > worst) { worst = e; worst_x = x[i]; worst_y = y[i]; }
    }
    std::printf("{\"fn\": \"%s\", \"n\": %d, \"max_ulps\": %.3f, \"bit_exact\": %.6f, \"worst_x\": %.17g, \"worst_y\": %.17g}\n",
                names[op], n, worst, double(exact) / n, worst_x, worst_y);
    if (worst > (op == 2 ? 1e4 : 8)) fail = 1;   // pow_d: |y log2 x| 2^-53 relative (~1e-13), ulps grow with |y|
  }
  // special values
  const double sx[] = {0.0, 0.0, 1.0, INFINITY, 2.0, 0.5, NAN};
  const double sy[] = {2.5, -2.5, 1e300, 2.0, 0.0, 2000.0, 0.0};
  hipMemcpy(dx, sx, sizeof sx, hipMemcpyHostToDevice);
  hipMemcpy(dy, sy, sizeof sy, hipMemcpyHostToDevice);
  k_probe<<<1, 64>>>(2, dx, dy, dr, 7);
  hipMemcpy(r.data(), dr, 7 * 8, hipMemcpyDeviceToHost);
  for (int i = 0; i < 7; ++i)
  {
    const double want = std::pow(sx[i], sy[i]);
    const bool ok = (r[i] == want) || (std::isnan(r[i]) && std::isnan(want));
    std::printf("pow_d(%g, %g) = %g (glibc %g)%s\n", sx[i], sy[i], r[i], want, ok ? "" : "  MISMATCH");
    fail |= !ok;
  }
  std::printf(fail ? "FAIL\n" : "PASS\n");
  return fail;
}
