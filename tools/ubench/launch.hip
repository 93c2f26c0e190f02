// Per-kernel cost floor: back-to-back launches of empty / tiny kernels on one stream.
#include <hip/hip_runtime.h>
#include <cstdio>
struct Big { double v[112]; };  // ~900-byte kernarg like the DKG kernels
__global__ void empty_k() {}
__global__ void big_arg_k(Big b, double* out) { if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = b.v[blockIdx.x % 100]; }
__global__ void big_static_k(Big b, double* out) { if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = b.v[7] + b.v[90]; }
struct Mid { double v[32]; };
__global__ void mid_static_k(Mid b, double* out) { if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = b.v[7] + b.v[30]; }
__global__ void ptr_arg_k(const Big* b, double* out) { if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = b->v[blockIdx.x % 100]; }
__global__ void store_k(double* out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = i;
}
int main() {
  double* d;
  (void)hipMalloc(&d, 64 << 20);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipStream_t s;
  (void)hipStreamCreate(&s);
  Big big{};
  const int reps = 2000;
  for (int grid : {256, 1024}) {
    for (int kind = 0; kind < 6; ++kind) {
      for (int pass = 0; pass < 2; ++pass) {
        (void)hipEventRecord(e0, s);
        for (int r = 0; r < reps; ++r) {
          if (kind == 0) hipLaunchKernelGGL(empty_k, dim3(grid), dim3(256), 0, s);
          else if (kind == 1) hipLaunchKernelGGL(big_arg_k, dim3(grid), dim3(256), 0, s, big, d);
          else if (kind == 2) hipLaunchKernelGGL(store_k, dim3(grid), dim3(256), 0, s, d, grid * 256);
          else if (kind == 3) hipLaunchKernelGGL(big_static_k, dim3(grid), dim3(256), 0, s, big, d);
          else if (kind == 4) hipLaunchKernelGGL(mid_static_k, dim3(grid), dim3(256), 0, s, Mid{}, d);
          else hipLaunchKernelGGL(ptr_arg_k, dim3(grid), dim3(256), 0, s, (const Big*)(d + 4096), d);
        }
        (void)hipEventRecord(e1, s);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (pass) printf("grid %5d %-10s %.2f us/launch\n", grid, kind == 0 ? "empty" : kind == 1 ? "big-dyn" : kind == 2 ? "store" : kind == 3 ? "big-static" : kind == 4 ? "256B-static" : "ptr-arg",
                         ms * 1e3 / reps);
      }
    }
  }
  // graph of 3 dependent launches
  hipGraph_t g;
  hipGraphExec_t ge;
  (void)hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  for (int k = 0; k < 3; ++k) hipLaunchKernelGGL(store_k, dim3(1024), dim3(256), 0, s, d, 1024 * 256);
  (void)hipStreamEndCapture(s, &g);
  (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  for (int pass = 0; pass < 2; ++pass) {
    (void)hipEventRecord(e0, s);
    for (int r = 0; r < 500; ++r) (void)hipGraphLaunch(ge, s);
    (void)hipEventRecord(e1, s);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (pass) printf("graph of 3 store kernels (1024 WGs): %.2f us/replay\n", ms * 1e3 / 500);
  }
  return 0;
}
