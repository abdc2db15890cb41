// Accuracy of the hardware f64 reciprocal / reciprocal square root (gfx950)
// against correctly rounded host results, in ulps.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>
__global__ void k(const double* x, double* r, double* q, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    r[i] = __builtin_amdgcn_rcp(x[i]);
    q[i] = __builtin_amdgcn_rsq(x[i]);
  }
}
static double ulps(double a, double b) {
  int64_t ia, ib;
  memcpy(&ia, &a, 8);
  memcpy(&ib, &b, 8);
  return (double)llabs(ia - ib);
}
int main() {
  const int n = 1 << 20;
  std::vector<double> x(n), r(n), q(n);
  uint64_t s = 12345;
  for (int i = 0; i < n; ++i) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    double u = (double)(s >> 11) / 9007199254740992.0;
    x[i] = std::exp(std::log(1e-3) + u * (std::log(1e7) - std::log(1e-3)));
  }
  double *dx, *dr, *dq;
  (void)hipMalloc(&dx, n * 8);
  (void)hipMalloc(&dr, n * 8);
  (void)hipMalloc(&dq, n * 8);
  (void)hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, dx, dr, dq, n);
  (void)hipMemcpy(r.data(), dr, n * 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(q.data(), dq, n * 8, hipMemcpyDeviceToHost);
  double mr = 0, mq = 0, sr = 0, sq = 0;
  for (int i = 0; i < n; ++i) {
    double er = ulps(r[i], 1.0 / x[i]), eq = ulps(q[i], 1.0 / std::sqrt(x[i]));
    mr = er > mr ? er : mr;
    mq = eq > mq ? eq : mq;
    sr += er;
    sq += eq;
  }
  printf("v_rcp_f64: max %.0f ulp, mean %.3f ulp\n", mr, sr / n);
  printf("v_rsq_f64: max %.0f ulp, mean %.3f ulp\n", mq, sq / n);
  return 0;
}
