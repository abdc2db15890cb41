// Store-pattern microbenchmark for the c5 score matrices: B = 256 rows x
// N = 100000 f32 written by (V1) a linear float4 stream, (V2) the MFMA C-layout
// pattern of hyb_scores_kernel (per instruction 16 rows x 64 B), (V3) the same
// tiles re-arranged so each instruction writes 8 rows x 128 B, (V4) V2 with
// wave-contiguous item ranges instead of block-interleaved slices.
#include <hip/hip_runtime.h>
#include <cstdio>
constexpr int B = 256;
constexpr long N = 100000;

__global__ void v1(float* out) {
  const long n4 = (long)B * N / 4;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x)
    reinterpret_cast<float4*>(out)[i] = make_float4(1.f, 2.f, 3.f, (float)i);
}

// mode 2: C layout, mode 3: 8 rows x 128 B per instruction; wave_contig: slices of a wave adjacent
template <int MODE, bool WAVE_CONTIG>
__global__ __launch_bounds__(512) void vtile(float* out, int G) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  const long per = ((N + G - 1) / G + 15) / 16 * 16;
  const long i0 = blockIdx.x * per, i1 = i0 + per < N ? i0 + per : N;
  const long nsl = (i1 - i0 + 31) / 32;  // 32-item slices in the block
  const long spw = (nsl + 7) / 8;
  for (long sidx = 0;; ++sidx) {
    long sl = WAVE_CONTIG ? w * spw + sidx : w + 8 * sidx;
    if (WAVE_CONTIG ? (sidx >= spw || sl >= nsl) : sl >= nsl) break;
    const long jb = i0 + 32 * sl;
    for (int ch = 0; ch < 4; ++ch) {
      for (int u = 0; u < 4; ++u) {
        if (MODE == 2) {
          for (int t = 0; t < 2; ++t) {
            const long j = jb + 16 * t + 4 * g;
            const int row = ch * 64 + 16 * u + c;
            if (j + 3 < i1) *reinterpret_cast<float4*>(out + row * N + j) = make_float4(1.f, 2.f, 3.f, (float)j);
          }
        } else {  // 16 rows x 32 items = 2 KB per (ch, u): two instructions of 8 rows x 128 B
          for (int h = 0; h < 2; ++h) {
            const int row = ch * 64 + 16 * u + 8 * h + (lane >> 3);
            const long j = jb + 4 * (lane & 7);
            if (j + 3 < i1) *reinterpret_cast<float4*>(out + row * N + j) = make_float4(1.f, 2.f, 3.f, (float)j);
          }
        }
      }
    }
  }
}

template <class F>
float timeit(F f) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  f();
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a);
  for (int r = 0; r < 20; ++r) f();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / 20;
}

int main() {
  float* out;
  (void)hipMalloc(&out, sizeof(float) * B * N);
  const double gb = 4.0 * B * N / 1e9;
  float ms = timeit([&] { hipLaunchKernelGGL(v1, dim3(2048), dim3(256), 0, 0, out); });
  printf("V1 linear       %.1f us  %.2f TB/s\n", ms * 1e3, gb / ms);
  for (int G : {128, 256, 512}) {
    ms = timeit([&] { hipLaunchKernelGGL((vtile<2, false>), dim3(G), dim3(512), 0, 0, out, G); });
    printf("V2 C-layout G=%d  %.1f us  %.2f TB/s\n", G, ms * 1e3, gb / ms);
    ms = timeit([&] { hipLaunchKernelGGL((vtile<3, false>), dim3(G), dim3(512), 0, 0, out, G); });
    printf("V3 8x128B   G=%d  %.1f us  %.2f TB/s\n", G, ms * 1e3, gb / ms);
    ms = timeit([&] { hipLaunchKernelGGL((vtile<2, true>), dim3(G), dim3(512), 0, 0, out, G); });
    printf("V4 C wave-contig G=%d %.1f us  %.2f TB/s\n", G, ms * 1e3, gb / ms);
  }
  return 0;
}
