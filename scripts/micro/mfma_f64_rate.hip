// Microbenchmark: issue rate of v_mfma_f64_4x4x4_4b_f64 vs v_mfma_f64_16x16x4_f64
// on gfx950 (one wave per SIMD, 8 independent accumulators, s_memtime cycles).
// Also prints the 4x4x4 operand/result lane layout from a known-answer run.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int ITER = 4096;

template <int SHAPE>
__global__ void kern(double* out, long long* cyc, double x0) {
  double a = x0 + threadIdx.x * 1e-3, b = x0 - threadIdx.x * 1e-3;
  double c1[8];
  d4 c4[8];
  for (int i = 0; i < 8; ++i) {
    c1[i] = 0.0;
    c4[i] = d4{0.0, 0.0, 0.0, 0.0};
  }
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      if (SHAPE == 0) c4[m] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c4[m], 0, 0, 0);
      else c1[m] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c1[m], 0, 0, 0);
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  double r = 0.0;
  for (int i = 0; i < 8; ++i) r += c1[i] + c4[i][0] + c4[i][1] + c4[i][2] + c4[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void layout(double* out) {
  // A = lane id, B = 1: C[i][j] of block b = sum_k A-values feeding row i
  const int l = threadIdx.x;
  double c = 0.0;
  c = __builtin_amdgcn_mfma_f64_4x4x4f64((double)l, 1.0, c, 0, 0, 0);
  out[l] = c;
  // B = lane id, A = 1
  double c2 = 0.0;
  c2 = __builtin_amdgcn_mfma_f64_4x4x4f64(1.0, (double)l, c2, 0, 0, 0);
  out[64 + l] = c2;
  // A = (lane == t) for t = 5 : which lanes of C see lane 5's A value
  double c3 = 0.0;
  c3 = __builtin_amdgcn_mfma_f64_4x4x4f64(l == 5 ? 1.0 : 0.0, 1.0, c3, 0, 0, 0);
  out[128 + l] = c3;
  double c5 = 0.0;
  c5 = __builtin_amdgcn_mfma_f64_4x4x4f64(1.0, l == 5 ? 1.0 : 0.0, c5, 0, 0, 0);
  out[192 + l] = c5;
}

template <int SHAPE>
void run(const char* name, int waves_per_cu) {
  double* out;
  long long* cyc;
  const int nb = 256;
  hipMalloc(&out, nb * 64 * waves_per_cu * 8);
  hipMalloc(&cyc, nb * 8);
  hipLaunchKernelGGL(kern<SHAPE>, dim3(nb), dim3(64 * waves_per_cu), 0, 0, out, cyc, 1.0);
  hipLaunchKernelGGL(kern<SHAPE>, dim3(nb), dim3(64 * waves_per_cu), 0, 0, out, cyc, 1.0);
  hipDeviceSynchronize();
  long long h[nb];
  hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < nb; ++i) m += h[i];
  m /= nb;
  const double per = m / (ITER * 8.0);
  const double fma = SHAPE == 0 ? 1024.0 : 256.0;
  printf("%-22s waves/CU %d: %.1f cycles per MFMA per wave -> %.1f FMA/cycle/SIMD\n", name, waves_per_cu, per,
         fma * (waves_per_cu / 4.0) / per);
  hipFree(out);
  hipFree(cyc);
}

int main() {
  run<0>("f64 16x16x4", 4);
  run<1>("f64 4x4x4 (4 blocks)", 4);
  run<0>("f64 16x16x4", 8);
  run<1>("f64 4x4x4 (4 blocks)", 8);
  double* o;
  hipMalloc(&o, 256 * 8);
  hipLaunchKernelGGL(layout, dim3(1), dim3(64), 0, 0, o);
  double h[256];
  hipMemcpy(h, o, sizeof(h), hipMemcpyDeviceToHost);
  const char* nm[4] = {"C(A=lane,B=1)", "C(A=1,B=lane)", "C(A=[lane==5])", "C(B=[lane==5])"};
  for (int q = 0; q < 4; ++q) {
    printf("%s:", nm[q]);
    for (int l = 0; l < 64; ++l) printf(" %g", h[64 * q + l]);
    printf("\n");
  }
  return 0;
}
