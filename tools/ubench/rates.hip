// Microbenchmark: sustained rate of v_mfma_f64_16x16x4_f64 and v_fma_f64 per SIMD on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int CHAINS>
__global__ void mfma_loop(double* out, int iters) {
  d4 acc[CHAINS];
  for (int c = 0; c < CHAINS; ++c) acc[c] = {0, 0, 0, 0};
  double a = threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-4;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
  for (int c = 0; c < CHAINS; ++c) s += acc[c][0] + acc[c][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) out[1 << 20 | blockIdx.x] = (double)(t1 - t0);
}

__global__ void fma_loop(double* out, int iters) {
  double x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
  const double m = 0.999999, c = 1e-9;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    x0 = fma(x0, m, c); x1 = fma(x1, m, c); x2 = fma(x2, m, c); x3 = fma(x3, m, c);
    x4 = fma(x4, m, c); x5 = fma(x5, m, c); x6 = fma(x6, m, c); x7 = fma(x7, m, c);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
  if (threadIdx.x == 0) out[1 << 20 | blockIdx.x] = (double)(t1 - t0);
}

int main() {
  double* d;
  hipMalloc(&d, sizeof(double) * (2 << 20));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 20000;
  for (int wpb : {1, 4, 8, 16}) {
    for (int pass = 0; pass < 2; ++pass) {
      const int blocks = 256;
      hipEventRecord(e0);
      hipLaunchKernelGGL(mfma_loop<4>, dim3(blocks), dim3(64 * wpb), 0, 0, d, iters);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      double tcyc;
      hipMemcpy(&tcyc, d + (1 << 20), sizeof(double), hipMemcpyDeviceToHost);
      const double mfmas = (double)blocks * wpb * iters * 4;
      const double flops = mfmas * 2048;
      if (pass) printf("mfma_f64 16x16x4: %2d waves/CU: %.1f TFLOP/s, %.1f cycles/MFMA/SIMD (memtime), clock %.2f GHz\n", wpb,
                       flops / ms / 1e9, tcyc * 4.0 * (wpb < 4 ? 1.0 : 4.0 / wpb) / (iters * 4.0) * (wpb < 4 ? 4.0 / wpb / 4.0 : 1.0) ,
                       tcyc / (ms * 1e-3) / 1e9);
    }
  }
  for (int wpb : {4, 8, 16}) {
    for (int pass = 0; pass < 2; ++pass) {
      const int blocks = 256;
      hipEventRecord(e0);
      hipLaunchKernelGGL(fma_loop, dim3(blocks), dim3(64 * wpb), 0, 0, d, iters);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double flops = (double)blocks * wpb * 64 * iters * 8 * 2;
      if (pass) printf("v_fma_f64: %2d waves/CU: %.1f TFLOP/s\n", wpb, flops / ms / 1e9);
    }
  }
  return 0;
}
