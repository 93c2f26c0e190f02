// Shared device helpers for the Discrete-KG kernels (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dkg.h"

namespace dkg {

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int WAVE = 64;

__host__ __device__ inline int pad16(int x) { return (x + 15) & ~15; }

// All output states by value (kernel argument, < 1 KiB).
struct Outputs {
  dkg_output o[DKG_MAX_OUTPUTS];
};

// One v_mfma_f64_16x16x4_f64.  Lane maps (CDNA4, f64 form):
//   A (16x4): lane l holds A[l & 15][l >> 4]
//   B (4x16): lane l holds B[l >> 4][l & 15]
//   D (16x16): lane l, register r holds D[(l >> 4) + 4 r][l & 15]
__device__ __forceinline__ d4 mfma_f64(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// Kernel profile of ScaleKernel(base) at squared scaled distance r2:
// gpytorch MaternKernel.forward / RBFKernel (factory.py:116 catalog).
__device__ __forceinline__ double kernel_profile(int kind, double r2) {
  if (kind == DKG_RBF) return exp(-0.5 * r2);
  const double r = sqrt(r2);
  if (kind == DKG_MATERN12) return exp(-r);
  if (kind == DKG_MATERN32) {
    const double t = 1.7320508075688772 * r;
    return (t + 1.0) * exp(-t);
  }
  const double t = 2.23606797749979 * r;  // sqrt(5) r
  return (t + 1.0 + (5.0 / 3.0) * r2) * exp(-t);
}

__device__ __forceinline__ double scaled_r2(const double* __restrict__ xa, const double* __restrict__ xb,
                                            const double* __restrict__ il, int d) {
  double acc = 0.0;
  for (int k = 0; k < d; ++k) {
    const double t = (xa[k] - xb[k]) * il[k];
    acc = fma(t, t, acc);
  }
  return acc;
}

// Same with the first point held in registers (d <= DKG_MAX_DIM, unrolled).
__device__ __forceinline__ double scaled_r2_reg(const double (&xa)[DKG_MAX_DIM], const double* __restrict__ xb,
                                                const double* __restrict__ il, int d) {
  double acc = 0.0;
#pragma unroll
  for (int k = 0; k < DKG_MAX_DIM; ++k) {
    if (k < d) {
      const double t = (xa[k] - xb[k]) * il[k];
      acc = fma(t, t, acc);
    }
  }
  return acc;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off));
  return v;
}

__device__ __forceinline__ int lanes_below(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
}

// E[(Z - c)_+] for Z ~ N(0,1): phi(c) - c * (1 - Phi(c)).  Non-negative; the
// per-edge term of the cancellation-free KG sum (DESIGN.md "Envelope").
__device__ __forceinline__ double psi(double c) {
  return 0.3989422804014327 * exp(-0.5 * c * c) - 0.5 * c * erfc(0.7071067811865476 * c);
}

}  // namespace dkg
