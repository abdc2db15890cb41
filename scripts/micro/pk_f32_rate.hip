// Microbenchmark: issue cost of packed f32 mul/add (v_pk_mul_f32 /
// v_pk_add_f32) against scalar v_mul_f32 / v_add_f32 on gfx950, the ops of
// the JVM-exact ALS scoring loop (csrc/score.hip: rounded product, rounded sum,
// no FMA). One block of `waves` waves per CU, cycles per iteration by s_memtime.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2v __attribute__((ext_vector_type(2)));
constexpr int ITER = 2048;

template <int MODE>
__global__ void kern(float* out, long long* cyc, float x0) {
#pragma clang fp contract(off)
  // MODE 0: 16 chains acc += u*v packed (mul + add); MODE 1: same, scalar;
  // MODE 2: packed, a broadcast operand (op_sel) as in the scoring loop
  f2v acc[16], v[2];
  float s[32];
  for (int i = 0; i < 16; ++i) acc[i] = f2v{0.f, (float)i};
  for (int i = 0; i < 32; ++i) s[i] = (float)i;
  v[0] = f2v{x0 + threadIdx.x, x0 - threadIdx.x};
  v[1] = f2v{x0 * 0.5f, x0 * 0.25f + threadIdx.x};
  __syncthreads();
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITER; ++it) {
    // inline asm: the compiler can neither hoist the loop-invariant products
    // nor merge the instructions
    if (MODE == 0) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        f2v t;
        asm volatile("v_pk_mul_f32 %0, %1, %2" : "=v"(t) : "v"(v[i & 1]), "v"(v[(i >> 1) & 1]));
        asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(acc[i]) : "v"(t));
      }
    } else if (MODE == 1) {
#pragma unroll
      for (int i = 0; i < 32; ++i) {
        float t;
        asm volatile("v_mul_f32 %0, %1, %2" : "=v"(t) : "v"(v[i & 1].x), "v"(v[(i >> 1) & 1].y));
        asm volatile("v_add_f32 %0, %0, %1" : "+v"(s[i]) : "v"(t));
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        f2v t;
        asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t) : "v"(v[1]), "v"(v[i & 1]));
        asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(acc[i]) : "v"(t));
      }
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  float r = 0.f;
  for (int i = 0; i < 16; ++i) r += acc[i].x + acc[i].y;
  for (int i = 0; i < 32; ++i) r += s[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE>
void run(const char* name, int waves) {
  float* out;
  long long* cyc;
  const int nb = 256;
  hipMalloc(&out, nb * waves * 64 * 4);
  hipMalloc(&cyc, nb * 8);
  hipLaunchKernelGGL(kern<MODE>, dim3(nb), dim3(64 * waves), 0, 0, out, cyc, 1.5f);  // warm-up
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0, 0);
  hipLaunchKernelGGL(kern<MODE>, dim3(nb), dim3(64 * waves), 0, 0, out, cyc, 1.5f);
  hipEventRecord(e1, 0);
  hipDeviceSynchronize();
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  long long h[nb];
  hipMemcpy(h, cyc, nb * 8, hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < nb; ++i) m += h[i];
  m /= nb;
  // per lane per iteration: 32 multiplies + 32 adds = 32 packed or 64 scalar instructions
  const double per_iter = m / ITER;
  const double instr = (MODE == 1 ? 64.0 : 32.0) * (waves / 4.0);  // per SIMD per iteration
  // s_memtime ticks per ns of wall time (kernel launch ~ the timed loop)
  printf("%-28s waves/SIMD %d: %8.1f ticks/iter = %5.2f ticks per instruction per SIMD; kernel %.3f ms, %.2f ticks/ns\n",
         name, waves / 4, per_iter, per_iter / instr, ms, m / (ms * 1e6));
  hipFree(out);
  hipFree(cyc);
}

int main() {
  for (int w : {4, 8, 16}) {
    run<0>("packed mul+add", w);
    run<1>("scalar mul+add", w);
    run<2>("packed, broadcast operand", w);
  }
  return 0;
}
