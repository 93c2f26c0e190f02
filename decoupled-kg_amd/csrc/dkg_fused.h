// The Discrete-KG forward as ONE launch (gfx950): the cross, covariance and envelope
// workgroups of a forward share one grid and hand their results on through arrival
// counters (Handoff, dkg_common.h) instead of two dependent kernel boundaries.
//
// Roles by blockIdx.x, in dependency order, so every workgroup a consumer waits for has
// a lower index (dispatched before it; every wait is bounded in any case):
//   [0, nC)            cross      (row tile, column-pair group, output), row tile slowest
//   [nC, nC + nV)      covariance (column block, output, row block), row block slowest
//   [nC + nV, ...)     envelope   (candidate, half of the scalarisations)
// Each role runs the body its own kernel runs (cross_root_impl, posterior_cov_body,
// envelope_body), with its hand-off points:
//   cross  -> stores Q_X and the means write-through, counts itself into cnt1[output][row tile];
//   cov    -> evaluates its kernel terms and loads its first Q_D batch, waits for the cross
//             workgroups of its two row tiles, then loads Q_X; stores the covariance rows and
//             variances write-through and counts itself into cnt2[row block];
//   env    -> stages mu_D, the weights and the per-output scalars, waits for its candidate's
//             row block, then stages the candidate's covariance rows; the last envelope workgroup
//             re-zeroes the counters for the next launch on the plan.
// What overlaps: the covariance stage's kernel terms and Q_D loads with the cross stage, the
// envelope's staging with the covariance stage, and each stage's tail with the next stage's
// start; the two launch boundaries (~1.5-1.9 us each, MI355X_MICROARCH.md row "boundary") go.
#pragma once

#include <algorithm>
#include <type_traits>

#include "dkg_stages.h"

namespace dkg {

struct FusedArgs {
  const Plan* P;
  const double* xnew;
  double* kg;
  int B, dst;
  int nC, nV;          // cross / covariance workgroups
  int cgroups;         // cross column-pair groups per (row tile, output)
  int vcols, vrows;    // covariance column blocks, row blocks
  int split;           // envelope workgroups per candidate
  const double* mu_all;
  const double* cov_all;
  const double* var_all;
  const double* mux_all;
  const double* wts;
  const int* dup;
  long long cov_stride;
  int bpad;
  Handoff ho;
};

// Stamp slot of a role-local workgroup index (kid 0 cross, 1 covariance, 2 envelope).
__device__ __forceinline__ unsigned long long* kst_slot_wg(int dst, const Plan* P, int kid, int wg) {
  if (dst != 1) return nullptr;
  return (threadIdx.x == 0 && wg < KST_WG) ? P->kstamps + ((size_t)kid * KST_WG + wg) * 8 : nullptr;
}

template <int DM, int MAXL, int M>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(env_waves_per_eu(MAXL, M, false, false)))) void
forward_fused_kernel(FusedArgs a) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const Plan* __restrict__ P = a.P;
  const int id = blockIdx.x;
  if (id < a.nC) {
    const int m = P->m;
    const int grp = id % a.cgroups, oi = (id / a.cgroups) % m, ti = id / (a.cgroups * m);
    unsigned long long* st = kst_slot_wg(a.dst, P, 0, id);
    KST_BEGIN(st);
    if (grp == 0 && oi == 0) {
      // the KG accumulators and arrival tickets of this row tile's candidates, which the envelope stage adds
      // into (write-through): zeroed inside the dependency chain (this workgroup's cnt1 arrival -> the
      // covariance workgroups of output 0 in this row block -> cnt2 -> the envelope's wait), so every
      // zero store is visible before any envelope workgroup of these candidates adds to it
      const int r1 = std::min(a.B, 16 * (ti + 1));
      const int nt = pair_groups(P->S) + 1;
      for (int i = 16 * ti * nt + (int)threadIdx.x; i < r1 * nt; i += blockDim.x) st_out<true>(&P->tickets[i], 0);
      for (int i = 16 * ti + (int)threadIdx.x; i < r1; i += blockDim.x) {
        st_out<true>(&a.kg[i], 0.0);
        // (the covariance workgroups of the other outputs do not wait for this one, but every output's
        // workgroups mark the same coincidences, output 0's after this store: the mark survives)
        st_out<true>(&P->dup[i], DUP_NONE);
      }
    }
    cross_root_impl<DM, false, double, true>(P->o[oi], P->d, a.xnew, a.B, P->q[oi], P->mux[oi], ti, grp, smem, st);
    handoff_publish(a.ho.cnt1 + ((size_t)oi * a.ho.rt + ti) * HANDOFF_STRIDE);
    return;
  }
  if (id < a.nC + a.nV) {
    const int v = id - a.nC;
    const int m = P->m;
    const int bx = v % a.vcols, oi = (v / a.vcols) % m, by = v / (a.vcols * m);
    double* part = smem;                                  // [(PC_KS - 1) * 2 PC_RB * 4 * 64]
    double* qpart = smem + (PC_KS - 1) * 2 * PC_RB * 4 * 64;
    posterior_cov_body<DM, double, true>(P, a.xnew, a.B, bx, by, oi, part, qpart, kst_slot_wg(a.dst, P, 1, v), &a.ho);
    return;
  }
  const int e = id - a.nC - a.nV;
  envelope_body<MAXL, M, false, false, true>(P, a.B, a.kg, nullptr, a.dst, nullptr, nullptr, a.mu_all, a.cov_all,
                                             a.var_all, a.mux_all, a.wts, a.dup, a.cov_stride, a.bpad, e / a.split,
                                             e % a.split, a.split, smem, kst_slot_wg(a.dst, P, 2, e), &a.ho);
}

// Dynamic LDS of the fused launch: the largest of its roles'.
inline size_t fused_lds_bytes(const Plan& h) {
  const size_t cov = ((size_t)(PC_KS - 1) * 2 * PC_RB * 4 * 64 + (size_t)(PC_KS - 1) * 2 * PC_RB * 16) * sizeof(double);
  return std::max({cross_root_lds_bytes(h.max_np, h.d), envelope_lds_bytes(h.m, h.N, 8, h.S, false), cov});
}

template <int DM, int MAXL, int M>
hipError_t launch_fused_t(const FusedArgs& a, size_t lds, hipStream_t s) {
  raise_lds_limit((const void*)forward_fused_kernel<DM, MAXL, M>, lds);
  hipLaunchKernelGGL((forward_fused_kernel<DM, MAXL, M>), dim3(a.nC + a.nV + a.B * a.split), dim3(512), lds, s, a);
  return hipGetLastError();
}

// One output bucket M: the (dimension bucket, line-slot bucket) instantiation.  Defined in
// dkg_env_m<M>.hip next to the envelope instantiations of the same bucket.
template <int M>
hipError_t launch_fused_bucket(int dim_b, int lines, const FusedArgs& a, size_t lds, hipStream_t s) {
  auto by_dim = [&](auto maxl_c) -> hipError_t {
    constexpr int MAXL = decltype(maxl_c)::value;
    switch (dim_b) {
      case 2: return launch_fused_t<2, MAXL, M>(a, lds, s);
      case 4: return launch_fused_t<4, MAXL, M>(a, lds, s);
      case 8: return launch_fused_t<8, MAXL, M>(a, lds, s);
      default: return launch_fused_t<16, MAXL, M>(a, lds, s);
    }
  };
  if (lines <= 64 * 2) return by_dim(std::integral_constant<int, 2>{});
  if (lines <= 64 * 8) return by_dim(std::integral_constant<int, 8>{});
  if (lines <= 64 * 17) return by_dim(std::integral_constant<int, 17>{});
  return hipErrorInvalidValue;
}

hipError_t launch_fused_m1(int dim_b, int lines, const FusedArgs& a, size_t lds, hipStream_t s);
hipError_t launch_fused_m2(int dim_b, int lines, const FusedArgs& a, size_t lds, hipStream_t s);
hipError_t launch_fused_m3(int dim_b, int lines, const FusedArgs& a, size_t lds, hipStream_t s);
hipError_t launch_fused_m4(int dim_b, int lines, const FusedArgs& a, size_t lds, hipStream_t s);
hipError_t launch_fused_m8(int dim_b, int lines, const FusedArgs& a, size_t lds, hipStream_t s);

}  // namespace dkg
