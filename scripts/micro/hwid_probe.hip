// Which SIMD does each wave of a 768-thread (12-wave) workgroup land on?
// HW_REG_HW_ID (gfx9): wave_id [3:0], simd_id [5:4], cu_id [11:8].
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(768) void probe(unsigned* out) {
  __shared__ double pad[18000];  // ~141 KB: one workgroup per CU
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(v));
  pad[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 12 + (threadIdx.x >> 6)] = v + (unsigned)(pad[threadIdx.x] * 0);
}
int main() {
  unsigned* d; hipMalloc(&d, 512 * 12 * 4);
  hipLaunchKernelGGL(probe, dim3(512), dim3(768), 0, 0, d);
  unsigned h[512 * 12]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int mism = 0, cnt[4];
  for (int b = 0; b < 512; ++b) {
    cnt[0] = cnt[1] = cnt[2] = cnt[3] = 0;
    for (int w = 0; w < 12; ++w) { int s = (h[b * 12 + w] >> 4) & 3; cnt[s]++; if (s != w % 4) mism++; }
    if (b < 3 || cnt[0] != 3 || cnt[1] != 3 || cnt[2] != 3 || cnt[3] != 3) {
      printf("block %d:", b);
      for (int w = 0; w < 12; ++w) printf(" w%d->s%d", w, (h[b * 12 + w] >> 4) & 3);
      printf("\n");
    }
  }
  printf("waves with simd != w %% 4: %d of %d\n", mism, 512 * 12);
  return 0;
}
