// The gfx950 row-swap permutes inside a dependent loop (DESIGN.md "v_permlane*_swap").
//
// v_permlane16_swap_b32 / v_permlane32_swap_b32 write BOTH operands: permlane16
// swaps the odd 16-lane rows of the first operand with the even rows of the
// second, permlane32 the upper 32 lanes of the first with the lower 32 of the
// second.  The builtins return the pair {new first, new second}; a lane's
// xor-16 (xor-32) partner value is in the first element for lanes in odd rows
// (upper half) and in the second element for the other lanes.
//
// Each kernel runs ITERS iterations of: v = f(v, i) (dependent fp64 VALU work),
// then a butterfly step xor 16 and xor 32 on v, and compares the partner value
// with ds_bpermute's (__shfl_xor).  Variants:
//   0  both result elements, selected by the lane's row / half (the correct use)
//   1  the first element only (what a "partner = swap(v, v).first" reading does:
//      lanes of even rows / the lower half get their OWN value back)
//   2  as 0 with the step's result fed to the next iteration (a loop-carried chain)
// Output: mismatching lanes per variant and step, over all waves and iterations.
#include <hip/hip_runtime.h>

#include <cstdio>

__device__ __forceinline__ double shfl_xor_f64(double v, int m) { return __shfl_xor(v, m); }

template <int VAR, int STEP>  // STEP 16 or 32
__device__ __forceinline__ double partner(double v, int lane) {
  const unsigned lo = __double2loint(v), hi = __double2hiint(v);
  unsigned plo, phi;
  if constexpr (STEP == 16) {
    const auto rl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto rh = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    const bool odd = (lane >> 4) & 1;
    plo = (VAR == 1 || odd) ? rl[0] : rl[1];
    phi = (VAR == 1 || odd) ? rh[0] : rh[1];
  } else {
    const auto rl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto rh = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    const bool upper = lane >= 32;
    plo = (VAR == 1 || upper) ? rl[0] : rl[1];
    phi = (VAR == 1 || upper) ? rh[0] : rh[1];
  }
  return __hiloint2double((int)phi, (int)plo);
}

template <int VAR>
__global__ void swap_loop(int iters, unsigned long long* bad) {
  const int lane = threadIdx.x & 63;
  double v = 1.0 + lane * 0.37 + blockIdx.x * 1e-3;
  unsigned long long b16 = 0, b32 = 0;
  for (int i = 0; i < iters; ++i) {
    v = fma(v, 1.0000001, sqrt(v) * 1e-3 + i * 1e-7);  // dependent VALU work before the permute
    const double p16 = partner<VAR, 16>(v, lane), r16 = shfl_xor_f64(v, 16);
    const double p32 = partner<VAR, 32>(v, lane), r32 = shfl_xor_f64(v, 32);
    b16 += (p16 != r16);
    b32 += (p32 != r32);
    if constexpr (VAR == 2) v = fmin(v, p16) + 1e-3 * fmax(v, p32);  // the swaps feed the next iteration
  }
  atomicAdd(&bad[0], b16);
  atomicAdd(&bad[1], b32);
}

int main() {
  unsigned long long* bad;
  if (hipMalloc(&bad, 2 * sizeof(unsigned long long)) != hipSuccess) return 1;
  const int iters = 4096, blocks = 512, threads = 256;
  const char* names[3] = {"both elements by row (correct)", "first element only", "correct, loop-carried"};
  for (int var = 0; var < 3; ++var) {
    (void)hipMemset(bad, 0, 2 * sizeof(unsigned long long));
    if (var == 0) hipLaunchKernelGGL(swap_loop<0>, dim3(blocks), dim3(threads), 0, 0, iters, bad);
    if (var == 1) hipLaunchKernelGGL(swap_loop<1>, dim3(blocks), dim3(threads), 0, 0, iters, bad);
    if (var == 2) hipLaunchKernelGGL(swap_loop<2>, dim3(blocks), dim3(threads), 0, 0, iters, bad);
    unsigned long long h[2];
    (void)hipMemcpy(h, bad, sizeof(h), hipMemcpyDeviceToHost);
    printf("variant %d (%s): xor16 mismatches %llu, xor32 mismatches %llu of %llu lane-steps\n", var, names[var],
           h[0], h[1], (unsigned long long)iters * blocks * threads);
  }
  (void)hipFree(bad);
  return 0;
}
