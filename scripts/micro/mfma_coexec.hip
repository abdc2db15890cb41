// Microbenchmark: can VALU work overlap f64 MFMA on one SIMD (gfx950)?
// Each kernel: one block of `waves` waves per CU, loop of ITER iterations.
// Reports cycles per iteration (s_memtime) per variant.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int ITER = 4096;

template <int NMFMA, int NDP, int NI32, int ROLE, int NF32 = 0>
__global__ void kern(double* out, long long* cyc, double x0) {
  // ROLE 0: every wave does MFMA+VALU mix; ROLE 1: waves < 4 MFMA only, waves >= 4 VALU only
  const int w = threadIdx.x >> 6;
  d4 acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = d4{0, 0, 0, 0};
  double a = x0 + threadIdx.x, b = x0 * 2.0 + threadIdx.x;
  double f[8];
  for (int i = 0; i < 8; ++i) f[i] = a + i;
  int u[8];
  for (int i = 0; i < 8; ++i) u[i] = threadIdx.x + i;
  float g[8];
  for (int i = 0; i < 8; ++i) g[i] = (float)threadIdx.x + i;
  const float gb = (float)x0 * 0.5f;
  const bool do_m = ROLE == 0 || w < 4, do_v = ROLE == 0 || w >= 4;
  __syncthreads();
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITER; ++it) {
    if (do_m) {
#pragma unroll
      for (int m = 0; m < NMFMA; ++m) acc[m & 7] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[m & 7], 0, 0, 0);
    }
    if (do_v) {
#pragma unroll
      for (int d = 0; d < NDP; ++d) f[d & 7] = fma(f[d & 7], b, a);
#pragma unroll
      for (int d = 0; d < NI32; ++d) u[d & 7] = u[d & 7] * 3 + 1;
#pragma unroll
      for (int d = 0; d < NF32; ++d) g[d & 7] = fmaf(g[d & 7], gb, 1.0f);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3] + f[i] + u[i] + g[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int NMFMA, int NDP, int NI32, int ROLE, int NF32 = 0>
void run(const char* name, int waves) {
  double* out;
  long long* cyc;
  const int blocks = 256;
  hipMalloc(&out, sizeof(double) * blocks * 64 * waves);
  hipMalloc(&cyc, sizeof(long long) * blocks);
  hipLaunchKernelGGL((kern<NMFMA, NDP, NI32, ROLE, NF32>), dim3(blocks), dim3(64 * waves), 0, 0, out, cyc, 1.0);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL((kern<NMFMA, NDP, NI32, ROLE, NF32>), dim3(blocks), dim3(64 * waves), 0, 0, out, cyc, 1.0);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  long long h[256];
  hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  double avg = 0;
  for (int i = 0; i < blocks; ++i) avg += h[i];
  avg /= blocks;
  printf("%-34s waves/CU=%d  cyc/iter=%8.1f  wall=%.3f ms\n", name, waves, avg / ITER, ms);
  hipFree(out);
  hipFree(cyc);
}

int main() {
  run<8, 0, 0, 0>("8 mfma", 4);
  run<8, 0, 0, 0>("8 mfma", 8);
  run<0, 8, 0, 0>("8 dp-fma", 4);
  run<0, 16, 0, 0>("16 dp-fma", 4);
  run<0, 0, 16, 0>("16 i32", 4);
  run<8, 8, 0, 0>("8 mfma + 8 dp-fma", 4);
  run<8, 16, 0, 0>("8 mfma + 16 dp-fma", 4);
  run<8, 0, 16, 0>("8 mfma + 16 i32", 4);
  run<8, 0, 32, 0>("8 mfma + 32 i32", 4);
  run<8, 16, 0, 1>("split: 4w mfma / 4w 16 dp-fma", 8);
  run<8, 0, 32, 1>("split: 4w mfma / 4w 32 i32", 8);
  run<8, 64, 0, 1>("split: 4w mfma / 4w 64 dp-fma", 8);
  run<0, 0, 0, 0, 64>("64 f32-fma", 4);
  run<8, 0, 0, 0, 32>("8 mfma + 32 f32-fma", 4);
  run<8, 0, 0, 1, 64>("split: 4w mfma / 4w 64 f32-fma", 8);
  run<8, 0, 0, 1, 256>("split: 4w mfma / 4w 256 f32-fma", 8);
  return 0;
}
