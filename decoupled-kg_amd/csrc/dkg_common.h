// Shared device helpers for the Discrete-KG kernels (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <map>
#include <mutex>
#include <utility>

#include "dkg.h"

namespace dkg {

// Dynamic LDS above the 64 KiB default needs the kernel's limit raised once per (kernel, device):
// remembered here, so a launch pays a map lookup, not a runtime call (B = 1 latency).
inline void raise_lds_limit(const void* kernel, size_t lds) {
  if (lds <= 65536) return;
  static std::mutex mu;
  static std::map<std::pair<const void*, int>, size_t> done;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lock(mu);
  size_t& cur = done[{kernel, dev}];
  if (cur >= lds) return;
  if (hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess) cur = lds;
}

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int WAVE = 64;

__host__ __device__ inline int pad16(int x) { return (x + 15) & ~15; }

// All output states by value (kernel argument, < 1 KiB).
struct Outputs {
  dkg_output o[DKG_MAX_OUTPUTS];
};

// One LDS-DMA piece hidden from hipcc (cdna_hip_programming.md "What hipcc does not do", LDS-DMA recipe): 16 bytes
// per lane from gsrc into LDS at lds_dst + 16 lane (lds_dst wave-uniform, the LDS byte address).  The staged
// big-block kernels issue their panels with it and read them with plain (compiler-counted) LDS loads: hipcc then
// places every lgkmcnt wait before the registers' first use itself, and since it does not see the DMA it does not
// drain every DMA in flight (vmcnt(0)) before those loads, as it does after __builtin_amdgcn_global_load_lds.  The
// caller counts the DMA (s_waitcnt vmcnt(N) in asm), then passes a barrier, before reading the bytes.  (ds_reads in
// inline asm with a separate wait had left the allocator free to copy the destination registers before the data
// landed: the NaNs of the first fp32 block kernels)  M0 is written and restored in the statement.
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds_dst))
               : "memory");
}

// One v_mfma_f64_16x16x4_f64.  Lane maps (CDNA4, f64 form):
//   A (16x4): lane l holds A[l & 15][l >> 4]
//   B (4x16): lane l holds B[l >> 4][l & 15]
//   D (16x16): lane l, register r holds D[(l >> 4) + 4 r][l & 15]
__device__ __forceinline__ d4 mfma_f64(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// Pair-packed fragment layout (include/dkg.h "Data layout"): element
// (row 16 t + (l & 15), column 4 kb + (l >> 4)) of a matrix with KB = n_pad/4
// k-blocks sits at ((t * KB/2 + kb/2) * 64 + l) * 2 + (kb & 1), so lane l's
// operands of k-blocks 2j and 2j+1 are one aligned 16-byte word.
__host__ __device__ inline size_t frag_index(int t, int kb, int l, int KB) {
  return (((size_t)t * (KB >> 1) + (kb >> 1)) * 64 + l) * 2 + (kb & 1);
}

// Lane's operands of k-blocks 2 j and 2 j + 1 of tile `tile` (base = matrix start).
__device__ __forceinline__ double2 frag_pair(const double* __restrict__ base, int tile, int j, int lane, int KB) {
  return reinterpret_cast<const double2*>(base)[((size_t)tile * (KB >> 1) + j) * 64 + lane];
}

// fp32 form (DKG_PLAN_F32): v_mfma_f32_16x16x4_f32 has the same A/B lane maps
// as the f64 instruction above, so the same fragment order serves, but its D
// map differs: lane l, register r holds D[4 (l >> 4) + r][l & 15].  Four
// consecutive k-blocks share one aligned 16-byte word ("quad-packed"):
// element (16 t + (l & 15), 4 kb + (l >> 4)) at ((t * KB/4 + kb/4) * 64 + l) * 4 + (kb & 3).
typedef float f4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f4 mfma_f32(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__host__ __device__ inline size_t frag32_index(int t, int kb, int l, int KB) {
  return (((size_t)t * (KB >> 2) + (kb >> 2)) * 64 + l) * 4 + (kb & 3);
}
// Lane's operands of k-blocks 4 j .. 4 j + 3 of tile `tile`.
__device__ __forceinline__ float4 frag_quad(const float* __restrict__ base, int tile, int j, int lane, int KB) {
  return reinterpret_cast<const float4*>(base)[((size_t)tile * (KB >> 2) + j) * 64 + lane];
}

// psi's coefficients in one constant table (offsets PSI_OFF_*): exp's Taylor
// terms 1/k! (k = 0..13), then PA, QA (x < 4) and PB, QB (x >= 4) from
// tools/fit_psi.py.
static __constant__ double PSI_TAB[46] = {
    // EXP_TAYLOR
    1.0, 1.0, 0.5, 0.16666666666666666, 0.041666666666666664, 0.008333333333333333, 0.001388888888888889, 0.0001984126984126984, 2.48015873015873e-05, 2.7557319223985893e-06, 2.755731922398589e-07, 2.505210838544172e-08, 2.08767569878681e-09, 1.6059043836821613e-10,
    // PSI_PA
    1.0, 2.796346091120482, 4.476998603222499, 4.347508891535361, 2.7165796377890157, 1.0037192400095971, 0.17325326370833247, -4.618396778934904e-05, 3.3360288569271207e-06,
    // PSI_QA
    1.0, 7.809602640382476, 27.628540187254945, 58.0088790797422, 79.3523289449324, 72.75170128287581, 43.91331216452371, 16.08152617590387, 2.7670522859865594,
    // PSI_PB
    0.9981308338834465, 3.6598787850514367, 4.641485909810474, 2.472764850018868, 0.5303020141112789, 0.034608494860324725, 0.00012399724831674248,
    // PSI_QB
    1.0, 3.8515503731650442, 5.30522462058383, 3.263540634985728, 0.913625609211908, 0.10482146071245484, 0.003532980749196329,
};
constexpr int PSI_OFF_EXP = 0;
constexpr int PSI_OFF_PA = 14;
constexpr int PSI_OFF_QA = 23;
constexpr int PSI_OFF_PB = 32;
constexpr int PSI_OFF_QB = 39;

// a * b + c with c an SGPR operand: one v_fma_f64.  Written out because the
// compiler otherwise picks v_fmac_f64 (addend tied to the destination) and
// copies every scalar coefficient into VGPRs first, two v_mov per FMA.
__device__ __forceinline__ double fma_scalar_addend(double a, double b, double c) {
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c));
  return r;
}

// Horner over N coefficients at c (c[0] the constant term), c in SGPRs.
template <int N, class Ptr>
__device__ __forceinline__ double horner(Ptr c, double v) {
  double r = fma_scalar_addend(c[N - 1], v, c[N - 2]);
#pragma unroll
  for (int i = N - 3; i >= 0; --i) r = fma_scalar_addend(r, v, c[i]);
  return r;
}

// The table through an opaque constant-address-space pointer: the
// coefficients are scalar loads (s_load, the scalar cache) at the use, SGPR
// operands of the FMAs, never constants the compiler materialises early in
// VGPRs (a generic pointer here compiled to per-lane flat loads).
typedef const __attribute__((address_space(4))) double* const_dptr;
__device__ __forceinline__ const_dptr psi_tab() {
  const_dptr c = (const_dptr)PSI_TAB;
  asm volatile("" : "+s"(c));
  return c;
}

// exp(y) for y <= 0 (0 below -760, where it underflows, branch-free): y = k ln2 + r with
// the reduction in two FMAs (ln2 to 2^-106), the Taylor polynomial (terms to
// k = 13: truncation ~4e-18 on |r| <= ln2 / 2) from the table, v_ldexp
// (gradual underflow).  Relative error ~1e-16.
__device__ __forceinline__ double exp_nonpos(double y, const_dptr tab) {
  y = (y < -760.0) ? -760.0 : y;  // 2^k underflows ldexp to 0; NaN passes
  const double k = rint(y * 1.4426950408889634);
  double r = fma(-k, 0.6931471805599453, y);
  r = fma(-k, 2.3190468138462996e-17, r);
  return ldexp(horner<14>(tab + PSI_OFF_EXP, r), (int)k);
}

// sqrt for x >= 0 (no denormal inputs; 0 -> 0): v_rsq_f64 and two
// Goldschmidt steps, ~1 ulp; libm's sqrt adds denormal scaling and special
// cases the kernel profiles never need.
__device__ __forceinline__ double sqrt_nonneg(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = 0.5 * y;
  const double r = fma(-g, h, 0.5);
  g = fma(g, r, g);
  h = fma(h, r, h);
  const double d = fma(-g, g, x);
  g = fma(d, h, g);
  return (x > 0.0) ? g : 0.0;
}

// Kernel profile of ScaleKernel(base) at squared scaled distance r2:
// gpytorch MaternKernel.forward / RBFKernel (factory.py:116 catalog).
// exp and sqrt as exp_nonpos / sqrt_nonneg (arguments are <= 0 / >= 0 here):
// about half the instructions of libm's, whose range and special-case
// handling these arguments never need (~1 ulp either way).
__device__ __forceinline__ double kernel_profile(int kind, double r2, const_dptr tab = psi_tab()) {
  if (kind == DKG_RBF) return exp_nonpos(-0.5 * r2, tab);
  const double r = sqrt_nonneg(r2);
  if (kind == DKG_MATERN12) return exp_nonpos(-r, tab);
  if (kind == DKG_MATERN32) {
    const double t = 1.7320508075688772 * r;
    return (t + 1.0) * exp_nonpos(-t, tab);
  }
  const double t = 2.23606797749979 * r;  // sqrt(5) r
  return (t + 1.0 + (5.0 / 3.0) * r2) * exp_nonpos(-t, tab);
}

// Same with the family fixed at compile time (branch-free in unrolled loops).
// Loops pass the table pointer from outside (one address computation).
template <int KIND>
__device__ __forceinline__ double kernel_profile_t(double r2, const_dptr tab = psi_tab()) {
  if constexpr (KIND == DKG_RBF) {
    return exp_nonpos(-0.5 * r2, tab);
  } else if constexpr (KIND == DKG_MATERN12) {
    return exp_nonpos(-sqrt_nonneg(r2), tab);
  } else if constexpr (KIND == DKG_MATERN32) {
    const double t = 1.7320508075688772 * sqrt_nonneg(r2);
    return (t + 1.0) * exp_nonpos(-t, tab);
  } else {
    const double t = 2.23606797749979 * sqrt_nonneg(r2);
    return (t + 1.0 + (5.0 / 3.0) * r2) * exp_nonpos(-t, tab);
  }
}

// The covariance stage's kernel terms: kernel_profile_t's expression compiled without FP contraction, every
// product rounded on its own, so a term has the same bits in every kernel and context that evaluates it (the
// covariance kernels' block shapes are bit-identical only if their terms are; left to the compiler, the same
// expression was fused differently in two kernels).  exp_nonpos and sqrt_nonneg take their products through
// explicit fma()s or contraction-free copies here.
__device__ __forceinline__ double exp_nonpos_nc(double y, const_dptr tab) {
#pragma clang fp contract(off)
  y = (y < -760.0) ? -760.0 : y;
  const double k = rint(y * 1.4426950408889634);
  double r = fma(-k, 0.6931471805599453, y);
  r = fma(-k, 2.3190468138462996e-17, r);
  return ldexp(horner<14>(tab + PSI_OFF_EXP, r), (int)k);
}
__device__ __forceinline__ double sqrt_nonneg_nc(double x) {
#pragma clang fp contract(off)
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = 0.5 * y;
  const double r = fma(-g, h, 0.5);
  g = fma(g, r, g);
  h = fma(h, r, h);
  const double d = fma(-g, g, x);
  g = fma(d, h, g);
  return (x > 0.0) ? g : 0.0;
}
template <int KIND>
__device__ __forceinline__ double kernel_term_nc(double r2, const_dptr tab) {
#pragma clang fp contract(off)
  if constexpr (KIND == DKG_RBF) {
    return exp_nonpos_nc(-0.5 * r2, tab);
  } else if constexpr (KIND == DKG_MATERN12) {
    return exp_nonpos_nc(-sqrt_nonneg_nc(r2), tab);
  } else if constexpr (KIND == DKG_MATERN32) {
    const double t = 1.7320508075688772 * sqrt_nonneg_nc(r2);
    return (t + 1.0) * exp_nonpos_nc(-t, tab);
  } else {
    const double t = 2.23606797749979 * sqrt_nonneg_nc(r2);
    return (t + 1.0 + (5.0 / 3.0) * r2) * exp_nonpos_nc(-t, tab);
  }
}
__device__ __forceinline__ double kernel_term_nc(int kind, double r2, const_dptr tab) {
  switch (kind) {
    case DKG_RBF: return kernel_term_nc<DKG_RBF>(r2, tab);
    case DKG_MATERN12: return kernel_term_nc<DKG_MATERN12>(r2, tab);
    case DKG_MATERN32: return kernel_term_nc<DKG_MATERN32>(r2, tab);
    default: return kernel_term_nc<DKG_MATERN52>(r2, tab);
  }
}

// h(r2) = kappa'(r) / r of the kernel profile, so that for the scaled
// difference t = (x - z) / l:  d[s kappa(|t|)]/dx_j = s h(|t|^2) t_j / l_j.
// Finite at r = 0 except Matern-1/2, whose gradient at a coincident point is
// taken as 0 (GPyTorch clamps the distance there, which zeroes its gradient).
template <int KIND>
__device__ __forceinline__ double kernel_dprofile_t(double r2) {
  if constexpr (KIND == DKG_RBF) {
    return -exp(-0.5 * r2);
  } else if constexpr (KIND == DKG_MATERN12) {
    const double r = sqrt(r2);
    return (r2 > 1e-30) ? -exp(-r) / r : 0.0;
  } else if constexpr (KIND == DKG_MATERN32) {
    return -3.0 * exp(-1.7320508075688772 * sqrt(r2));
  } else {
    const double t = 2.23606797749979 * sqrt(r2);
    return -(5.0 / 3.0) * (1.0 + t) * exp(-t);
  }
}

__device__ __forceinline__ double kernel_dprofile(int kind, double r2) {
  switch (kind) {
    case DKG_RBF: return kernel_dprofile_t<DKG_RBF>(r2);
    case DKG_MATERN12: return kernel_dprofile_t<DKG_MATERN12>(r2);
    case DKG_MATERN32: return kernel_dprofile_t<DKG_MATERN32>(r2);
    default: return kernel_dprofile_t<DKG_MATERN52>(r2);
  }
}

// Standard normal pdf and cdf (cdf via erfc: accurate in both tails).
__device__ __forceinline__ double norm_pdf(double c) { return 0.3989422804014327 * exp(-0.5 * c * c); }
__device__ __forceinline__ double norm_cdf(double c) { return 0.5 * erfc(-0.7071067811865476 * c); }

__device__ __forceinline__ double scaled_r2(const double* __restrict__ xa, const double* __restrict__ xb,
                                            const double* __restrict__ il, int d) {
  double acc = 0.0;
  for (int k = 0; k < d; ++k) {
    const double t = (xa[k] - xb[k]) * il[k];
    acc = fma(t, t, acc);
  }
  return acc;
}

// Compile-time bound DM >= d: unrolled, branch-free, every load issued up
// front (indices clamped to d - 1; terms k >= d contribute zero).
template <int DM>
__device__ __forceinline__ double scaled_r2_dm(const double* __restrict__ xa, const double* __restrict__ xb,
                                               const double* __restrict__ il, int d) {
  double acc = 0.0;
#pragma unroll
  for (int k = 0; k < DM; ++k) {
    const int kk = min(k, d - 1);
    const double t = (xa[kk] - xb[kk]) * il[kk];
    acc = fma(t, (k < d) ? t : 0.0, acc);
  }
  return acc;
}

// Dimension bucket used to instantiate the kernels: 2, 4, 8 or 16.
__host__ __device__ inline int dim_bucket(int d) { return d <= 2 ? 2 : d <= 4 ? 4 : d <= 8 ? 8 : 16; }

// ---------------------------------------------------------------------------
// Wave butterflies: DPP within 16-lane rows (xor 1, xor 2 via quad_perm;
// row_half_mirror; row_mirror), then two cross-row exchanges.  Each step
// hands every lane the value of a partner lane in the other half of its
// current group; with a commutative combine all lanes end with the same result.
// (mov_dpp: every lane is written by these full-row patterns, so no "old"
// value, and no v_mov to set one up, is needed.)
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

// Returns the partner value of `v` for butterfly step `s` (0..5).
// Cross-row steps (xor 16, xor 32) use ds_bpermute; the reductions combine
// the four rows by v_readlane instead (combine_rows).  (gfx950's
// v_permlane16_swap / v_permlane32_swap write both operands: a lane's partner
// is the first result element in odd rows / the upper half and the second
// element elsewhere -- reading only the first returns half the lanes their
// own value, the "stale partner" of round 1; tools/ubench/permlane.hip,
// DESIGN.md 4.7.)
template <int STEP>
__device__ __forceinline__ double partner_f64(double v) {
  if constexpr (STEP == 0) return dpp_f64<0xB1>(v);        // quad_perm [1,0,3,2]
  else if constexpr (STEP == 1) return dpp_f64<0x4E>(v);   // quad_perm [2,3,0,1]
  else if constexpr (STEP == 2) return dpp_f64<0x141>(v);  // row_half_mirror
  else if constexpr (STEP == 3) return dpp_f64<0x140>(v);  // row_mirror
  else return __shfl_xor(v, STEP == 4 ? 16 : 32);
}

#define DKG_BUTTERFLY(...)                         \
  {                                                \
    { constexpr int S_ = 0; __VA_ARGS__ }          \
    { constexpr int S_ = 1; __VA_ARGS__ }          \
    { constexpr int S_ = 2; __VA_ARGS__ }          \
    { constexpr int S_ = 3; __VA_ARGS__ }          \
    { constexpr int S_ = 4; __VA_ARGS__ }          \
    { constexpr int S_ = 5; __VA_ARGS__ }          \
  }

// The four in-row steps only: afterwards every lane of a 16-lane row holds its
// row's combine.
#define DKG_BUTTERFLY_ROW(...)                     \
  {                                                \
    { constexpr int S_ = 0; __VA_ARGS__ }          \
    { constexpr int S_ = 1; __VA_ARGS__ }          \
    { constexpr int S_ = 2; __VA_ARGS__ }          \
    { constexpr int S_ = 3; __VA_ARGS__ }          \
  }

// v_min_f64 / v_max_f64 without the operand canonicalisation LLVM puts in
// front of fmin/fmax (one extra VALU op per operand).  The kernels run in IEEE
// mode, where a quiet-NaN operand yields the other operand: exactly fmin/fmax
// for the values fed here (arithmetic results and quiet-NaN padding, never a
// signalling NaN).
__device__ __forceinline__ double fmin_raw(double a, double b) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ double fmax_raw(double a, double b) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// c ? v : a quiet NaN (only the high word is selected: a NaN exponent with the
// quiet bit set is a quiet NaN whatever the low word holds).
__device__ __forceinline__ double keep_or_qnan(bool c, double v) {
  return __hiloint2double(c ? __double2hiint(v) : 0x7FF80000, __double2loint(v));
}

__device__ __forceinline__ double readlane_f64(double v, int l);

// A wave-uniform double moved to SGPRs (v_readfirstlane of both halves), so
// it takes no VGPRs while it stays live.
// A wave-uniform pointer to global memory, held in SGPRs: loads from it take the scalar-base form
// (global_load ... v_offset, s[base]) with one VGPR offset, instead of a 64-bit VGPR address per load.
typedef const __attribute__((address_space(1))) double* gdptr;
__device__ __forceinline__ gdptr uniform_gptr(const double* p) {
  const uint64_t u = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u), hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  return reinterpret_cast<gdptr>(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ double sgpr_f64(double v) {
  return __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(v)),
                          __builtin_amdgcn_readfirstlane(__double2loint(v)));
}


// Cross-row combine after DKG_BUTTERFLY_ROW: the four row values by v_readlane
// (scalar registers, no LDS round trip as the ds_bpermute steps 16/32 take),
// combined in a fixed order, (r0 op r1) op (r2 op r3): wave-uniform and
// deterministic.
template <class Op>
__device__ __forceinline__ double combine_rows(double v, Op op) {
  const double r0 = readlane_f64(v, 0), r1 = readlane_f64(v, 16);
  const double r2 = readlane_f64(v, 32), r3 = readlane_f64(v, 48);
  return sgpr_f64(op(op(r0, r1), op(r2, r3)));  // wave-uniform: held in SGPRs, not VGPRs
}

// Wave minimum of an int: the four in-row DPP steps, then the four row values by v_readlane.
__device__ __forceinline__ int wave_min_i32(int v) {
  v = min(v, __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false));
  v = min(v, __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false));
  v = min(v, __builtin_amdgcn_mov_dpp(v, 0x141, 0xF, 0xF, false));
  v = min(v, __builtin_amdgcn_mov_dpp(v, 0x140, 0xF, 0xF, false));
  const int r0 = __builtin_amdgcn_readlane(v, 0), r1 = __builtin_amdgcn_readlane(v, 16);
  const int r2 = __builtin_amdgcn_readlane(v, 32), r3 = __builtin_amdgcn_readlane(v, 48);
  return min(min(r0, r1), min(r2, r3));
}

__device__ __forceinline__ double wave_sum(double v) {
  DKG_BUTTERFLY_ROW({ v = v + partner_f64<S_>(v); })
  return combine_rows(v, [](double a, double b) { return a + b; });
}

__device__ __forceinline__ double wave_max(double v) {
  DKG_BUTTERFLY_ROW({ v = fmax(v, partner_f64<S_>(v)); })
  return combine_rows(v, [](double a, double b) { return fmax(a, b); });
}

// Wave ballot of a compare: the compare's lane mask itself (HIP's __ballot
// goes through an int and costs a v_cndmask + v_cmp per use).
__device__ __forceinline__ uint64_t ballot(bool c) { return __builtin_amdgcn_ballot_w64(c); }

// A condition every lane agrees on, made visibly wave-uniform (scalar branch,
// full EXEC) so cross-lane operations inside the branch see every lane.
__device__ __forceinline__ bool uniform(bool c) { return __builtin_amdgcn_readfirstlane((int)c) != 0; }

// Lane `l`'s value of v (l wave-uniform), as a scalar operand.
__device__ __forceinline__ double readlane_f64(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ int lanes_below(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
}

// E[(Z - c)_+] for Z ~ N(0,1): phi(c) - c * (1 - Phi(c)).  Non-negative; the
// per-edge term of the cancellation-free KG sum (DESIGN.md "Envelope").
// psi(x) = phi(x) g(x) for x = |c| with g(x) = 1 - x (1 - Phi(x)) / phi(x) (no
// cancellation: g is a smooth positive factor decaying like 1 / x^2), and
// psi(-x) = psi(x) + x.  g by two rational approximations fitted at 60 digits
// (tools/fit_psi.py; worst relative error of the double evaluation ~5e-16):
// x < 4 in v = x / 4, x >= 4 as s h(u) with s = 1 / x^2 and u the position of s
// in [1/1600, 1/16] (x <= 40; beyond, phi(x) underflows and only c < 0 keeps
// the x term).  Sixteen-odd FMAs and one division per branch and few
// registers: libm's exp / erfc kept ~40 more VGPRs live at the kernels' peak
// (their coefficients materialised in VGPRs); these coefficients are read
// from constant memory through an opaque pointer (horner), one scalar operand
// per FMA.

__device__ __forceinline__ double psi(double c) {
  const const_dptr tab = psi_tab();
  const double x = fabs(c);
  const double x2 = x * x, x2l = fma(x, x, -x2);  // x^2 = x2 + x2l exactly
  const double e = 0.3989422804014327 * exp_nonpos(-0.5 * x2, tab) * fma(-0.5, x2l, 1.0);
  double g;
  if (x < 4.0) {
    const double v = 0.25 * x;
    g = horner<9>(tab + PSI_OFF_PA, v) / horner<9>(tab + PSI_OFF_QA, v);
  } else {
    const double s = 1.0 / (x * x);
    const double u = (s - 0.000625) * 16.161616161616163;  // (s - 1/1600) / (1/16 - 1/1600)
    g = s * (horner<7>(tab + PSI_OFF_PB, u) / horner<7>(tab + PSI_OFF_QB, u));
  }
  const double r = e * g;
  return (c < 0.0) ? r + x : r;
}

// ---------------------------------------------------------------------------
// XCD grouping of a launch (MI355X_MICROARCH.md "Workgroup dispatch, XCD placement": workgroups are dealt
// round-robin over the 8 XCDs, so ids L and L + 8 share one; a speed matter only, never correctness).  A
// 1-D launch of xcd_group_size(nblk, groups) workgroups gives the `groups` members of block blk the ids
// 8 (q groups + member) + blk % 8 (q = blk / 8): they are dispatched one after another to one XCD and
// share its L2 -- the outputs of one covariance block write the same line records (whole records leave L2
// instead of one component per write-back), the workgroups of one candidate's envelope read the same
// records (one HBM read instead of one per workgroup).  False for the padding ids (blk >= nblk).
// DKG_XCD_GROUP=0 (A/B only: profiles/r04/abv, 9.95 against 10.2 M KG-evals/s with four forwards in flight): the ids
// follow the 2-D order (member-major, blk = L % nblk), every block's members on different XCDs.
#ifndef DKG_XCD_GROUP
#define DKG_XCD_GROUP 1
#endif
__host__ __device__ inline int xcd_group_size(int nblk, int groups) {
  return DKG_XCD_GROUP ? 8 * groups * ((nblk + 7) / 8) : nblk * groups;
}
__device__ __forceinline__ bool xcd_group(int L, int nblk, int groups, int& blk, int& member) {
  if (!DKG_XCD_GROUP) {
    blk = L % nblk;
    member = L / nblk;
    return true;
  }
  const int r = L >> 3;
  member = r % groups;
  blk = (r / groups) * 8 + (L & 7);
  return blk < nblk;
}

// Block order of a launch over (column block bx < nbx, row block by < nby, output oi < m) whose workgroups
// each read a row panel (by, oi) and a column panel (bx, oi): order 0 is xcd_group's (the outputs of one block
// side by side, blocks dealt over the XCDs); orders 1 and 2 give every XCD a contiguous range of the task list
// [bx][by][oi] (1) or [oi][bx][by] (2), so the workgroups resident on one XCD at once share panels in its L2
// (the ids L and L + 8 share an XCD: XCD L % 8 takes tasks (L % 8) tpx + L / 8, tpx = ceil(tasks / 8)).
// Order 3: XCD x owns the column blocks [x cb, x cb + cb), cb = ceil(nbx / 8), in the order [oi][bx][by].
__host__ __device__ inline int block_order_size(int nbx, int nby, int m, int order) {
  if (order == 3) return 8 * ((nbx + 7) / 8) * nby * m;
  return order == 0 ? xcd_group_size(nbx * nby, m) : 8 * ((nbx * nby * m + 7) / 8);
}
__device__ __forceinline__ bool block_order(int L, int nbx, int nby, int m, int order, int& bx, int& by, int& oi) {
  if (order == 0) {
    int blk;
    if (!xcd_group(L, nbx * nby, m, blk, oi)) return false;
    bx = blk % nbx;
    by = blk / nbx;
    return true;
  }
  if (order == 3) {
    const int cb = (nbx + 7) / 8, r = L >> 3;
    by = r % nby;
    bx = (L & 7) * cb + (r / nby) % cb;
    oi = r / (nby * cb);
    return bx < nbx;
  }
  const int T = nbx * nby * m, tpx = (T + 7) / 8;
  const int t = (L & 7) * tpx + (L >> 3);
  if (t >= T) return false;
  if (order == 1) {
    oi = t % m;
    const int u = t / m;
    by = u % nby;
    bx = u / nby;
  } else {
    by = t % nby;
    const int u = t / nby;
    bx = u % nbx;
    oi = u / nbx;
  }
  return true;
}

// ---------------------------------------------------------------------------
// In-launch hand-offs (the fused one-launch forward, dkg_fused.h), MI355X_MICROARCH.md
// "inter-workgroup visibility" / cdna_hip_programming.md Guideline 16, counter form:
// producers store the handed-off bytes write-through (sc1: no release fence needed), every
// storing wave drains them (s_waitcnt vmcnt(0)), the workgroup meets, one lane adds to an
// arrival counter (agent-scope atomic); a consumer polls that counter from one lane
// (relaxed, agent scope, s_sleep between polls, bounded), takes ONE agent-scope acquire
// (invalidates its CU's L1), drains it, and the workgroup meets before any load of the
// bytes.  Counters are zeroed at plan init and re-zeroed by the launch's last workgroup.
struct Handoff {
  unsigned long long* cnt1;  // [m][rt]: cross workgroups done per (output, 16-candidate row tile)
  unsigned long long* cnt2;  // [nrb]: covariance workgroups done per 32-candidate row block
  unsigned long long* done;  // envelope workgroups done; the last one re-zeroes every counter
  int* err;                  // bits of the waits that gave up (bounded spins): 0 when all matched
  int rt, nrb;               // row tiles, row blocks
  int rb_rows;               // candidates per row block (the covariance stage's)
  unsigned long long quota1, quota2, quota_done;
};

// Polls per wait before it gives up (sets its err bit and goes on): each poll is one memory round trip
// plus an s_sleep, so a wait that never matches ends in well under a second.
constexpr unsigned HANDOFF_SPIN_LIMIT = 1u << 18;
// Counters sit one per 128-byte line (16 words apart): hundreds of workgroups poll them at once, and
// pollers of different counters must not queue on one line (MI355X_MICROARCH.md row "polling-cost").
constexpr int HANDOFF_STRIDE = 16;

template <bool WT, class T>
__device__ __forceinline__ void st_out(T* p, T v) {
  if constexpr (WT) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // global_store ... sc1
  } else {
    *p = v;
  }
}

// Every storing wave drains its write-through stores; the workgroup meets; one lane counts the arrival.
__device__ __forceinline__ void handoff_publish(unsigned long long* cnt) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(cnt, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Wait until the counters cnt[0], cnt[HANDOFF_STRIDE], ... (count of them) each reached `quota`, then one
// acquire; the workgroup meets after it.  Between polls the lane sleeps longer the longer it has waited
// (64 to ~1000 cycles), so early-dispatched consumers do not flood the counters' lines.
__device__ __forceinline__ void handoff_wait(unsigned long long* cnt, int count, unsigned long long quota, int* err,
                                             int code) {
  if (threadIdx.x == 0) {
    for (int i = 0; i < count; ++i) {
      unsigned spins = 0;
      while (__hip_atomic_load(cnt + (size_t)i * HANDOFF_STRIDE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
             quota) {
        if (++spins > HANDOFF_SPIN_LIMIT) {
          __hip_atomic_fetch_or(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        if (spins < 8) __builtin_amdgcn_s_sleep(1);
        else if (spins < 64) __builtin_amdgcn_s_sleep(4);
        else __builtin_amdgcn_s_sleep(16);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

}  // namespace dkg
