// HIP kernels of the Discrete-KG hot path for gfx950 (MI355X, CDNA4).
//
// Pipeline per forward (DESIGN.md "Kernels"):
//   cross_root_kernel   Q = K(x, X) R  (fp64 MFMA, R upper triangular), mean = c + K(x,X) alpha
//   posterior_cov_kernel cov[b][k] = s k(x_b, D_k) - Q_b . Q_D[k]   (fp64 MFMA GEMM, split-K)
//   envelope_kernel     lines a_k + b_k z per (candidate, scalarisation), upper
//                       envelope, closed-form Gaussian expectation, mean over S
#include "dkg_common.h"
#include "dkg_kernels.h"

#include <type_traits>

namespace dkg {

// ---------------------------------------------------------------------------
// Kernel matrix (state preparation): out = s k(x1, x2) + diag_add I.
__global__ void kernel_matrix_kernel(dkg_output o, int d, const double* __restrict__ x1, int n1,
                                     const double* __restrict__ x2, int n2, double diag_add,
                                     double* __restrict__ out) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const int i = blockIdx.y;
  if (i >= n1 || j >= n2) return;
  double v = o.outputscale * kernel_profile(o.kernel, scaled_r2(x1 + (size_t)i * d, x2 + (size_t)j * d,
                                                                 o.inv_lengthscale, d));
  if (i == j) v += diag_add;
  out[(size_t)i * n2 + j] = v;
}

// Pack dense row-major R (n x n) as root_frag[tj][kb][l] = R[4kb+(l>>4)][16tj+(l&15)].
__global__ void pack_root_kernel(const double* __restrict__ r, int n, double* __restrict__ rf) {
  const int np = pad16(n);
  const int KB = np / 4;
  const size_t total = (size_t)np * np;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    // e enumerates (tj, kb, l) of the R^T view; written at its pair-packed slot
    const int l = (int)(e & 63);
    const size_t blk = e >> 6;
    const int kb = (int)(blk % KB);
    const int tj = (int)(blk / KB);
    const int row = 4 * kb + (l >> 4);
    const int col = 16 * tj + (l & 15);
    rf[frag_index(tj, kb, l, KB)] = (row < n && col < n) ? r[(size_t)row * n + col] : 0.0;
  }
}

// ---------------------------------------------------------------------------
// cross_root_kernel: one workgroup per (16-row tile ti, tile pair p, output).
// The pair is (p, T-1-p) of 16-column tiles of Q = K_x R; R upper triangular
// means tile tj only needs k-blocks kb < 4(tj+1), so pairing the shortest
// with the longest tile balances the MFMA count across workgroups.  The
// training inputs are staged in LDS, the K(x, X) tile is evaluated once into
// LDS in B-operand order, and the k range is split over the 8 waves
// (split-K) with every operand of a wave's chunk loaded before its MFMAs;
// partials are reduced in LDS in fixed wave order (deterministic).
// Per-workgroup phase stamps (Plan.debug_stamp): slot 0 = s_memrealtime at
// start (100 MHz), 1..6 = s_memtime at phase boundaries, 7 = s_memrealtime at end.
__device__ unsigned long long g_kstamps[3 * KST_WG * 8];
__device__ __forceinline__ unsigned long long* kst_slot(int debug, int kid) {
  const int wg = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
  return (debug && threadIdx.x == 0 && wg < KST_WG) ? g_kstamps + ((size_t)kid * KST_WG + wg) * 8 : nullptr;
}
#define KST_BEGIN(st)                                                  \
  do {                                                                 \
    if (st) {                                                          \
      (st)[0] = __builtin_amdgcn_s_memrealtime();                      \
      (st)[1] = __builtin_amdgcn_s_memtime();                          \
    }                                                                  \
  } while (0)
#define KST(st, k)                                                     \
  do {                                                                 \
    if (st) (st)[k] = __builtin_amdgcn_s_memtime();                    \
  } while (0)
#define KST_END(st)                                                    \
  do {                                                                 \
    if (st) {                                                          \
      (st)[6] = __builtin_amdgcn_s_memtime();                          \
      (st)[7] = __builtin_amdgcn_s_memrealtime();                      \
    }                                                                  \
  } while (0)

constexpr int CR_WAVES = 8;
constexpr int CR_U = 8;  // k-blocks per load batch

// GRAD: the same contraction with the kernel replaced by its derivative in
// the candidate's coordinate `gdim` (J = dK(x, X)/dx_g R, dmean = dK/dx_g alpha).
template <int DM, bool GRAD = false>
__device__ __forceinline__ void cross_root_impl(const dkg_output& o, int d, const double* __restrict__ x, int rows,
                                                double* __restrict__ qout, double* __restrict__ mout, int ti, int p,
                                                double* smem, unsigned long long* st = nullptr, int gdim = 0) {
  const int n = o.n;
  const int np = pad16(n);
  const int T = np / 16;
  const int KB = np / 4;
  const int P = (T + 1) / 2;
  if (p >= P) return;
  const int tA = p, tB = T - 1 - p;                  // tA <= tB
  const int kbA = 4 * (tA + 1), kbB = 4 * (tB + 1);  // k-block extents (kbB >= kbA)
  const int ncol = min(n, 4 * kbB);                  // training columns this pair needs

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  double* kb_lds = smem;                         // [KB][64]
  double* part = kb_lds + (size_t)KB * 64;       // [CR_WAVES][8][64]
  double* mred = part + CR_WAVES * 8 * 64;       // [CR_WAVES][16]
  double* xs = mred + CR_WAVES * 16;             // [np][d] staged training inputs
  double* als = xs + (size_t)np * d;             // [np] alpha

  // R fragments of this wave's first k-block batch: loaded before anything
  // else so their latency overlaps the staging and the kernel evaluations.
  // (k-block ranges are even: kbA, kbB are multiples of 4 and chunk is even)
  const int chunk = 2 * ((kbB / 2 + CR_WAVES - 1) / CR_WAVES);
  const int k0 = wave * chunk;
  const int k1 = min(kbB, k0 + chunk);
  double ra[CR_U], rb[CR_U];
#pragma unroll
  for (int u = 0; u < CR_U; u += 2) {
    const int j = min(k0 + u, kbB - 2) >> 1;
    const double2 vb = frag_pair(o.root_frag, tB, j, lane, KB);
    const double2 va = frag_pair(o.root_frag, tA, min(j, kbA / 2 - 1), lane, KB);
    rb[u] = vb.x; rb[u + 1] = vb.y;
    ra[u] = va.x; ra[u + 1] = va.y;
  }

  KST(st, 2);
  const bool want_mean = (mout != nullptr) && (p == 0);  // p == 0 covers every column
  // training inputs staged pre-scaled by 1/lengthscale (GPyTorch divides both
  // inputs by the lengthscale before the distance)
  for (int e = tid; e < ncol * d; e += CR_WAVES * WAVE) xs[e] = o.train_x[e] * o.inv_lengthscale[e % d];
  if (want_mean)
    for (int e = tid; e < ncol; e += CR_WAVES * WAVE) als[e] = o.alpha[e];
  const int row = ti * 16 + (lane & 15);
  const bool rv = row < rows;
  const int rowc = min(row, rows - 1);
  double xr[DM];  // the candidate row, pre-scaled (clamped loads, no branches)
#pragma unroll
  for (int k = 0; k < DM; ++k) {
    const int kk = min(k, d - 1);
    xr[k] = x[(size_t)rowc * d + kk] * o.inv_lengthscale[kk];
  }
  __syncthreads();

  KST(st, 3);
  // ---- fill K(x_row, X_col), col < 4*kbB, in B-operand order (zero outside)
  double mpart = 0.0;
  const double os = o.outputscale;
  const double ilg = GRAD ? o.inv_lengthscale[gdim] : 1.0;
  double xg = 0.0;  // the candidate's pre-scaled coordinate gdim (GRAD)
#pragma unroll
  for (int k = 0; k < DM; ++k) xg = (k == gdim) ? xr[k] : xg;
  const int fill = kbB * 64;
  const int iters = (fill + CR_WAVES * WAVE - 1) / (CR_WAVES * WAVE);  // uniform trip count
  // one straight-line loop per covariance family (the switch stays outside)
  auto fill_loop = [&](auto kind_c) {
    constexpr int KIND = decltype(kind_c)::value;
#pragma unroll 4
    for (int it = 0; it < iters; ++it) {
      const int e = tid + it * CR_WAVES * WAVE;
      const int col = 4 * (e >> 6) + (lane >> 4);
      const int cc = min(col, n - 1);
      double r2 = 0.0;
#pragma unroll
      for (int k = 0; k < DM; ++k) {
        const double t = xr[k] - xs[(size_t)cc * d + min(k, d - 1)];
        r2 = fma(t, (k < d) ? t : 0.0, r2);
      }
      double kv;
      if constexpr (GRAD) {
        kv = os * kernel_dprofile_t<KIND>(r2) * (xg - xs[(size_t)cc * d + gdim]) * ilg;
      } else {
        kv = os * kernel_profile_t<KIND>(r2);
      }
      const double v = (rv && col < n) ? kv : 0.0;
      const double al = als[cc];  // staged only when want_mean; otherwise ignored
      mpart = fma(v, want_mean ? al : 0.0, mpart);
      if (e < fill) kb_lds[e] = v;
    }
  };
  switch (o.kernel) {
    case DKG_MATERN12: fill_loop(std::integral_constant<int, DKG_MATERN12>{}); break;
    case DKG_MATERN32: fill_loop(std::integral_constant<int, DKG_MATERN32>{}); break;
    case DKG_RBF: fill_loop(std::integral_constant<int, DKG_RBF>{}); break;
    default: fill_loop(std::integral_constant<int, DKG_MATERN52>{}); break;
  }
  __syncthreads();

  KST(st, 4);
  // ---- split-K MFMA over the pair, loads batched ahead of the MFMAs
  d4 accA2[2] = {{0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}};
  d4 accB2[2] = {{0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}};
  const bool pairA = tA != tB;
  for (int base = k0; base < k1; base += CR_U) {
    double bo[CR_U];
    if (base != k0) {
#pragma unroll
      for (int u = 0; u < CR_U; u += 2) {
        const int j = min(base + u, kbB - 2) >> 1;
        const double2 vb = frag_pair(o.root_frag, tB, j, lane, KB);
        const double2 va = frag_pair(o.root_frag, tA, min(j, kbA / 2 - 1), lane, KB);
        rb[u] = vb.x; rb[u + 1] = vb.y;
        ra[u] = va.x; ra[u + 1] = va.y;
      }
    }
#pragma unroll
    for (int u = 0; u < CR_U; ++u) {
      const int kb = min(base + u, kbB - 1);
      bo[u] = (base + u < k1) ? kb_lds[kb * 64 + lane] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < CR_U; ++u) {
      accB2[u & 1] = mfma_f64(rb[u], bo[u], accB2[u & 1]);
      if (pairA && base + u < kbA) accA2[u & 1] = mfma_f64(ra[u], bo[u], accA2[u & 1]);
    }
  }
  const d4 accA = accA2[0] + accA2[1];
  const d4 accB = accB2[0] + accB2[1];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    part[(wave * 8 + r) * 64 + lane] = accA[r];
    part[(wave * 8 + 4 + r) * 64 + lane] = accB[r];
  }
  // mean partials: lanes l, l^16, l^32, l^48 share a row.
  if (want_mean) {
    mpart += partner_f64<4>(mpart);
    mpart += partner_f64<5>(mpart);
    if (lane < 16) mred[wave * 16 + lane] = mpart;
  }
  __syncthreads();

  KST(st, 5);
  // ---- reduce partials in fixed wave order; wave w finalises (tile, reg) = w.
  {
    const int tsel = wave >> 2;  // 0 -> tA, 1 -> tB
    const int r = wave & 3;
    if (tsel == 1 || pairA) {
      double s = 0.0;
#pragma unroll
      for (int w = 0; w < CR_WAVES; ++w) s += part[(w * 8 + tsel * 4 + r) * 64 + lane];
      const int tj = tsel ? tB : tA;
      // D = R^T K^T: lane holds Q[16ti + (l&15)][16tj + 4r + (l>>4)] = q_frag[ti][4tj + r][l]
      qout[frag_index(ti, 4 * tj + r, lane, KB)] = s;
    }
  }
  if (want_mean && tid < 16) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < CR_WAVES; ++w) s += mred[w * 16 + tid];
    const int rr = ti * 16 + tid;
    mout[rr] = (rr < rows) ? (GRAD ? s : o.mean_constant + s) : 0.0;
  }
  KST_END(st);
}

template <int DM>
__global__ __launch_bounds__(CR_WAVES * WAVE) void cross_root_kernel(CrossArgs a) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  cross_root_impl<DM>(a.o, a.d, a.x, a.rows, a.q, a.mean, blockIdx.x, blockIdx.y, smem);
}

// Forward: grid (B tiles, pairs, outputs); workgroup (0,0,0) also clears the
// KG accumulators (and arrival tickets) the envelope stage adds into.
template <int DM>
__global__ __launch_bounds__(CR_WAVES * WAVE) void cross_root_plan_kernel(const Plan* __restrict__ P,
                                                                          const double* __restrict__ xnew, int B,
                                                                          double* __restrict__ kg, int dst) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  unsigned long long* st = kst_slot(dst, 0);
  KST_BEGIN(st);
  const int oi = blockIdx.z;
  if (blockIdx.x == 0 && blockIdx.y == 0 && oi == 0) {
    for (int i = threadIdx.x; i < B; i += blockDim.x) {
      kg[i] = 0.0;
      if (P->split > 2) P->tickets[i] = 0;
    }
  }
  cross_root_impl<DM>(P->o[oi], P->d, xnew, B, P->q[oi], P->mux[oi], blockIdx.x, blockIdx.y, smem, st);
}

// Gradient cross stage: grid (B tiles, pairs, outputs x d); z = oi * d + g
// writes J_g = dK(x, X)/dx_g R (fragment-packed) and dmean/dx_g for output oi.
// Workgroup (0,0,0) clears the gradient accumulator dkg[B x d].
template <int DM>
__global__ __launch_bounds__(CR_WAVES * WAVE) void cross_grad_plan_kernel(const Plan* __restrict__ P,
                                                                          const double* __restrict__ xnew, int B,
                                                                          double* __restrict__ dkg, int dst) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  unsigned long long* st = kst_slot(dst, 0);
  const int d = P->d;
  const int oi = blockIdx.z / d, gdim = blockIdx.z % d;
  if (blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0)
    for (int i = threadIdx.x; i < B * d; i += blockDim.x) dkg[i] = 0.0;
  const dkg_output& o = P->o[oi];
  const size_t mat = (size_t)P->bpad * pad16(o.n);
  cross_root_impl<DM, true>(o, d, xnew, B, P->jq[oi] + gdim * mat, P->gmu[oi] + (size_t)gdim * P->bpad, blockIdx.x,
                            blockIdx.y, smem, st, gdim);
}

size_t cross_root_lds_bytes(int np, int d) {
  return ((size_t)(np / 4) * 64 + CR_WAVES * 8 * 64 + CR_WAVES * 16 + (size_t)np * d + np) * sizeof(double);
}

// ---------------------------------------------------------------------------
// posterior_cov_kernel: cov[b][k] = s k(x_b, D_k) - sum_l Q[b][l] Q_D[k][l]
// One workgroup (8 waves) per 32 x 32 block = 2 x 2 output tiles of one
// output; wave w computes tile (w & 3) over K-half (w >> 2).  The two waves
// of a tile that share a K-half of an operand tile read it at the same time,
// so a CU fetches each operand byte about once (L1); every load is a 16-byte
// pair (two k-blocks).  K-halves meet in LDS; the K-half-0 wave evaluates
// the kernel epilogue and stores.  Tiles with tk == 0 also produce the
// candidates' own variances s - |Q_X[b]|^2.
constexpr int PC_WAVES = 8;
constexpr int PC_P = 8;  // 16-byte pairs per operand per load batch (16 k-blocks)

template <int DM>
__global__ __launch_bounds__(PC_WAVES * WAVE) void posterior_cov_kernel(const Plan* __restrict__ P,
                                                                         const double* __restrict__ xnew, int B,
                                                                         int dst) {
  __shared__ __attribute__((aligned(16))) double part[4 * 4 * 64];  // K-half 1 partial tiles
  __shared__ double qpart[4 * 16];
  unsigned long long* st = kst_slot(dst, 1);
  KST_BEGIN(st);
  const int oi = blockIdx.z;
  const dkg_output& o = P->o[oi];
  const int N = P->N;
  const int dbg = P->debug_cov;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tt = wave & 3, half = wave >> 2;
  const int ti = 2 * blockIdx.y + (tt >> 1);
  const int tk = 2 * blockIdx.x + (tt & 1);
  const int KB = pad16(o.n) / 4;
  const bool have_d = N > 0;
  // tiles that exist in the workspace / state buffers (wave-uniform)
  const bool live = ti * 16 < pad16(B) && (tk * 16 < pad16(N) || (tk == 0 && !have_d));
  const bool want_var = tk == 0;
  // K-half of this wave, in whole 16-byte pairs
  const int KP = KB / 2;
  const int p0 = half * ((KP + 1) / 2), p1 = half ? KP : (KP + 1) / 2;

  // epilogue operands first (row b = 16 ti + (l >> 4) + 4 r, column k = 16 tk + (l & 15))
  const int d = P->d;
  const int k = tk * 16 + (lane & 15);
  double r2[4] = {0.0, 0.0, 0.0, 0.0};
  if (half == 0) {  // wave-uniform; P->disc is valid even when N == 0 (plan init)
    const double* xk = P->disc + (size_t)min(k, max(N, 1) - 1) * d;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int b = ti * 16 + (lane >> 4) + 4 * r;
      r2[r] = scaled_r2_dm<DM>(xnew + (size_t)min(b, B - 1) * d, xk, o.inv_lengthscale, d);
    }
  }
  KST(st, 2);
  d4 acc[4] = {{0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}};
  double qsq = 0.0;  // lane l: sum over this wave's k of Q_X[16 ti + (l & 15)][k]^2
  if (live) {
    for (int pb = p0; pb < p1; pb += PC_P) {
      double2 va[PC_P], vd[PC_P];
      // disc_frag tile 0 exists only when N > 0: the N == 0 variance-only
      // wave reads its own Q_X tile as a stand-in (multiplied by 0 below)
      const double* dsrc = have_d ? o.disc_frag : P->q[oi];
      const int dt = have_d ? tk : ti;
#pragma unroll
      for (int u = 0; u < PC_P; ++u) {
        const int j = min(pb + u, p1 - 1);
        va[u] = frag_pair(P->q[oi], ti, j, lane, KB);
        vd[u] = frag_pair(dsrc, dt, j, lane, KB);
      }
      if (dbg & 1) {
#pragma unroll
        for (int u = 0; u < PC_P; ++u) { va[u] = double2{1.0, 1.0}; vd[u] = double2{0.5, 0.5}; }
      }
#pragma unroll
      for (int u = 0; u < PC_P; ++u) {
        const bool in = pb + u < p1 && have_d;
        const double a0 = va[u].x, a1 = va[u].y;
        const double d0 = in ? vd[u].x : 0.0, d1 = in ? vd[u].y : 0.0;
        acc[(2 * u) & 3] = mfma_f64(a0, d0, acc[(2 * u) & 3]);
        acc[(2 * u + 1) & 3] = mfma_f64(a1, d1, acc[(2 * u + 1) & 3]);
        if (want_var) qsq = (pb + u < p1) ? fma(a1, a1, fma(a0, a0, qsq)) : qsq;
      }
    }
  }
  const d4 accs = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  KST(st, 3);
  if (want_var) {
    qsq += __shfl_xor(qsq, 16);
    qsq += __shfl_xor(qsq, 32);
  }
  if (half == 1) {
#pragma unroll
    for (int r = 0; r < 4; ++r) part[(tt * 4 + r) * 64 + lane] = accs[r];
    if (want_var && lane < 16) qpart[tt * 16 + lane] = qsq;
  }
  __syncthreads();
  KST(st, 4);
  if (half == 0 && live) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const double sum = accs[r] + part[(tt * 4 + r) * 64 + lane];
      const int b = ti * 16 + (lane >> 4) + 4 * r;
      if (b < B && k < N)
        P->cov[oi][(size_t)b * N + k] =
            ((dbg & 4) ? r2[r] : o.outputscale * kernel_profile(o.kernel, r2[r])) - sum;
    }
    if (want_var && lane < 16) {
      const int bb = ti * 16 + lane;
      if (bb < B) P->var[oi][bb] = o.outputscale - (qsq + qpart[tt * 16 + lane]);
    }
  }
  KST_END(st);
}

// ---------------------------------------------------------------------------
// Envelope stage.
//
// Lines k = 0..N for candidate b and weight vector w_j (k = 0 is the candidate
// itself, discretekg.py:182-183):
//   a_k = sum_i w_i (sd_i mu_i(z_k) + ym_i)                   (scalarised mean)
//   b_k = sum_i beta_i sd_i^2 cov_i(x_b, z_k)                 (slope of the fantasy z)
// full:    beta_i = w_i^2 / sqrt(sum_i w_i^2 sd_i^2 (v_i + noise_i))   (:201-223)
// target t: beta_t = w_t / sqrt(sd_t^2 (v_t + noise_t)), others 0   (:300-321)
//
// KG_j = E[max_k (a_k + b_k Z)] - max_k a_k.  With T = argmax a on the upper
// hull of the points (b_k, a_k) and edges e = (P -> Q) of that hull, breakpoint
// c_e = (a_P - a_Q) / (b_Q - b_P):
//   KG_j = sum_{e left of T} (b_Q - b_P) psi(-c_e) + sum_{e right of T} (b_Q - b_P) psi(c_e)
// (every term >= 0: no cancellation, unlike E - max a of the reference :233).
//
// Per wave: extremes L (min b), R (max b), T (max a) by register butterflies;
// the lines strictly above the chords L-T / T-R survive into an LDS list;
// gift wrapping from L over the survivors (next vertex = argmin of the next
// intersection, the reference's walk :382-401, compared by cross
// multiplication); the hull edges are collected one per lane and psi is
// evaluated for all of them at once.
constexpr int ENV_CAP = 128;  // survivor list per wave (overflow -> walk all lines)

// Gift wrap over all register lines (fallback when the survivor list
// overflows ENV_CAP): next vertex = argmin of the next intersection, found by
// a wave butterfly per hull step.
template <int MAXL>
__device__ __forceinline__ double envelope_walk(const double (&la)[MAXL], const double (&lb)[MAXL], int nl, int lane,
                                             double bL, double aL, double bR, double bT, int* nhull) {
  double bc = bL, ac = aL, kg = 0.0;
  int h = 1;
  for (int guard = 0; guard <= nl && uniform(bc < bR); ++guard) {
    double bn = INFINITY, bd = 1.0, bbest = -INFINITY, abest = -INFINITY;
#pragma unroll
    for (int t = 0; t < MAXL; ++t) {
      const double bb = lb[t], a = la[t];
      if (lane + 64 * t < nl && bb > bc) {
        const double num = ac - a, den = bb - bc;
        const double lhs = num * bd, rhs = bn * den;
        if (bbest == -INFINITY || lhs < rhs || (lhs == rhs && bb > bbest)) { bn = num; bd = den; bbest = bb; abest = a; }
      }
    }
    DKG_BUTTERFLY({
      const double on = partner_f64<S_>(bn), od = partner_f64<S_>(bd);
      const double ob = partner_f64<S_>(bbest), oa = partner_f64<S_>(abest);
      bool take;
      if (ob == -INFINITY) take = false;
      else if (bbest == -INFINITY) take = true;
      else {
        const double lhs = on * bd, rhs = bn * od;
        take = lhs < rhs || (lhs == rhs && (ob > bbest || (ob == bbest && oa > abest)));
      }
      if (take) { bn = on; bd = od; bbest = ob; abest = oa; }
    })
    if (!uniform(bbest > bc)) break;
    const double c = bn / bd;
    kg += (bbest - bc) * psi((bbest <= bT) ? -c : c);
    bc = bbest;
    ac = abest;
    ++h;
  }
  if (nhull) *nhull = h;
  return kg;
}

// Result of the register passes over one set of lines.
struct EnvFilter {
  double bL, aL, bR, aR, bT, aT;
  int cnt;      // survivors written to the LDS list (the list then holds L, T, R at cnt..cnt+2)
  int status;   // 0: list ready, 1: KG = 0 (short-circuit), 2: list overflow (caller walks the lines)
  int kL, kT, kR;  // IDX: line indices of L, T, R (lowest index among exact duplicates)
  int cntT;        // IDX: number of lines attaining max a (torch.max splits its gradient among them)
};

// Lowest line index k over the wave for which `hit` holds in the lane's slot (or a large value).
template <int MAXL, class Pred>
__device__ __forceinline__ int wave_first_index(int lane, Pred hit) {
  int k = 1 << 30;
#pragma unroll
  for (int t = MAXL - 1; t >= 0; --t) k = hit(t) ? lane + 64 * t : k;
  DKG_BUTTERFLY({
    const int o = __shfl_xor(k, S_ == 0 ? 1 : S_ == 1 ? 2 : S_ == 2 ? 4 : S_ == 3 ? 8 : S_ == 4 ? 16 : 32);
    k = min(k, o);
  })
  return k;
}

// Register passes over one set of lines held MAXL per lane (line k in lane
// k % 64, slot k / 64): extremes, exact ties, and the survivors of the chord
// filter compacted into the wave's LDS list (sb, sa).
template <int MAXL, bool IDX = false>
__device__ __forceinline__ EnvFilter envelope_filter(const double (&la)[MAXL], const double (&lb)[MAXL], int lane,
                                                     double* sb, double* sa, int* si = nullptr) {
  EnvFilter f;
  // ---- extremes by value, then exact tie passes:
  // L = min b (tie: max a), R = max b (tie: max a), T = max a (tie: min b).
  // (slots beyond the line count hold padding lines: a = -inf, b = a real slope)
  double bmin = INFINITY, bmax = -INFINITY, amax = -INFINITY;
#pragma unroll
  for (int t = 0; t < MAXL; ++t) {
    bmin = fmin(bmin, lb[t]);
    bmax = fmax(bmax, lb[t]);
    amax = fmax(amax, la[t]);
  }
  DKG_BUTTERFLY({
    bmin = fmin(bmin, partner_f64<S_>(bmin));
    bmax = fmax(bmax, partner_f64<S_>(bmax));
    amax = fmax(amax, partner_f64<S_>(amax));
  })
  // short-circuit of discretekg.py:363-367 (all |b| < 1e-9), and the
  // single-slope case (one hull vertex, E = max a): KG = 0.
  if (!uniform(fmax(fabs(bmin), fabs(bmax)) >= 1e-9 && bmin < bmax)) {
    f.status = 1;
    return f;
  }
  double aL = -INFINITY, aR = -INFINITY, bT = INFINITY;
#pragma unroll
  for (int t = 0; t < MAXL; ++t) {
    aL = fmax(aL, (lb[t] == bmin) ? la[t] : -INFINITY);
    aR = fmax(aR, (lb[t] == bmax) ? la[t] : -INFINITY);
    bT = fmin(bT, (la[t] == amax) ? lb[t] : INFINITY);
  }
  DKG_BUTTERFLY({
    aL = fmax(aL, partner_f64<S_>(aL));
    aR = fmax(aR, partner_f64<S_>(aR));
    bT = fmin(bT, partner_f64<S_>(bT));
  })
  const double bL = bmin, bR = bmax, aT = amax;
  f.bL = bL; f.aL = aL; f.bR = bR; f.aR = aR; f.bT = bT; f.aT = aT;

  // ---- survivors: lines strictly above the chord L-T or the chord T-R.
  // No left/right select is needed: every line has a <= aT, so a line left of
  // T is never above the extension of T-R (its slope is <= 0) and a line right
  // of T never above the extension of L-T (slope >= 0); a degenerate chord
  // (db = 0) admits nothing.  h = (a - a0) db - (b - b0) da > 0, evaluated as
  // a*db - b*da > a0*db - b0*da.  Rounding can only admit extra lines (L, T
  // or R themselves), which the exact test in envelope_hull discards.
  const double db1 = bT - bL, da1 = aT - aL, k1 = aL * db1 - bL * da1;
  const double db2 = bR - bT, da2 = aR - aT, k2 = aT * db2 - bT * da2;
  int cnt = 0;
#pragma unroll
  for (int t = 0; t < MAXL; ++t) {
    const double a = la[t], bb = lb[t];
    const bool s = fma(a, db1, -bb * da1) > k1 || fma(a, db2, -bb * da2) > k2;
    const uint64_t mk = __ballot(s);
    if (mk != 0) {  // wave-uniform, rarely taken
      if (s) {
        const int pos = cnt + lanes_below(mk);
        if (pos < ENV_CAP) {
          sb[pos] = bb;
          sa[pos] = a;
          if constexpr (IDX) si[pos] = lane + 64 * t;
        }
      }
      cnt += __popcll(mk);
    }
  }
  f.cnt = cnt;
  f.status = (cnt + 3 > ENV_CAP) ? 2 : 0;
  if constexpr (IDX) {
    f.kL = wave_first_index<MAXL>(lane, [&](int t) { return lb[t] == bL && la[t] == aL; });
    f.kT = wave_first_index<MAXL>(lane, [&](int t) { return la[t] == aT && lb[t] == bT; });
    f.kR = wave_first_index<MAXL>(lane, [&](int t) { return lb[t] == bR && la[t] == aR; });
    int c = 0;
#pragma unroll
    for (int t = 0; t < MAXL; ++t) c += __popcll(__ballot(la[t] == aT));
    f.cntT = c;
  }
  return f;
}

// Exact upper envelope of the candidate list (survivors + L, T, R) and the
// cancellation-free expectation; needs no register lines.
__device__ __forceinline__ double envelope_hull(const EnvFilter& f, int lane, double* sb, double* sa, int* nhull,
                                                int dbg = 0) {
  const int cnt = f.cnt;
  const double bT = f.bT;
  if (lane == 0) {
    sb[cnt] = f.bL; sa[cnt] = f.aL;
    sb[cnt + 1] = f.bT; sa[cnt + 1] = f.aT;
    sb[cnt + 2] = f.bR; sa[cnt + 2] = f.aR;
  }
  const int nc = cnt + 3;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (dbg & 1024) return sb[lane & 7];  // ablation: list only
  // ---- right neighbour of every candidate P (one per lane, two chunks of 64
  // at most): the line that takes over from P as z grows, i.e. the reference
  // walk's step (discretekg.py:382-401): argmin over b_Q > b_P of the
  // intersection (a_P - a_Q)/(b_Q - b_P), ties -> larger slope.  Compared by
  // cross multiplication (both denominators > 0).  The list is read from LDS
  // once; candidate Q = j is broadcast from lane j's register (v_readlane),
  // and the selection is branch-free.
  double lb_[2], la_[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int e = min(c * 64 + lane, nc - 1);
    lb_[c] = sb[e];
    la_[c] = sa[e];
  }
  int nxt[2] = {-1, -1};
  double cn[2] = {0.0, 0.0}, cd[2] = {1.0, 1.0}, cb[2] = {0.0, 0.0}, pb[2] = {0.0, 0.0};
  const int nc0 = min(nc, 64);
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    if (c * 64 >= nc) break;
    const double bP = lb_[c], aP = la_[c];
    double rn = 0.0, rd = 1.0, rb = 0.0;
    int rj = -1;
    auto consider = [&](double bQ, double aQ, int j) {
      const double num = aP - aQ, den = bQ - bP;
      const double x = num * rd, y = rn * den;
      const bool take = (den > 0.0) & ((rj < 0) | (x < y) | ((x == y) & (bQ > rb)));
      rn = take ? num : rn;
      rd = take ? den : rd;
      rb = take ? bQ : rb;
      rj = take ? j : rj;
    };
#pragma unroll 4
    for (int j = 0; j < nc0; ++j) consider(readlane_f64(lb_[0], j), readlane_f64(la_[0], j), j);
    for (int j = 64; j < nc; ++j) consider(readlane_f64(lb_[1], j - 64), readlane_f64(la_[1], j - 64), j);
    nxt[c] = rj; cn[c] = rn; cd[c] = rd; cb[c] = rb; pb[c] = bP;
  }

  if (dbg & 2048) return cn[0] + cd[1] + (double)nxt[0];  // ablation: + right neighbours
  // ---- follow the chain from L (index cnt): its members are the envelope
  // lines in increasing slope, ending at R (no right neighbour).
  uint64_t on0 = 0, on1 = 0;
  int h = 0;
  for (int cur = cnt, guard = 0; cur >= 0 && guard < nc; ++guard) {
    if (cur < 64) on0 |= 1ull << cur; else on1 |= 1ull << (cur - 64);
    ++h;
    cur = (cur < 64) ? __builtin_amdgcn_readlane(nxt[0], cur) : __builtin_amdgcn_readlane(nxt[1], cur - 64);
  }
  if (dbg & 4096) return (double)(on0 + on1) + cn[0];  // ablation: + chain walk
  // ---- each envelope line other than R contributes its right edge P -> Q:
  //   (b_Q - b_P) psi(+-c), minus sign when the edge ends at or left of T.
  double v = 0.0;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    if (c * 64 >= nc) break;
    const bool on = (((c == 0) ? on0 : on1) >> lane) & 1;
    if (on && nxt[c] >= 0) {
      const double cc = cn[c] / cd[c];
      const double sc = (cb[c] <= bT) ? -cc : cc;
      v += (cb[c] - pb[c]) * ((dbg & 64) ? sc * sc : psi(sc));  // 64: ablation, psi -> c^2
    }
  }
  if (nhull) *nhull = h;
  return wave_sum(v);
}


// ---------------------------------------------------------------------------
// Vertex visitors for the gradient: the envelope lines in increasing slope,
// each with its breakpoints (cL, cR) (-inf / +inf at the ends), passed to
// visit(k, b, a, cL, cR); the return value is KG_w as in the forward.

// From the candidate list of an IDX filter (si holds the line indices).
template <class Visit>
__device__ __forceinline__ double envelope_hull_visit(const EnvFilter& f, int lane, double* sb, double* sa, int* si,
                                                      Visit&& visit) {
  const int cnt = f.cnt;
  const double bT = f.bT;
  if (lane == 0) {
    sb[cnt] = f.bL; sa[cnt] = f.aL; si[cnt] = f.kL;
    sb[cnt + 1] = f.bT; sa[cnt + 1] = f.aT; si[cnt + 1] = f.kT;
    sb[cnt + 2] = f.bR; sa[cnt + 2] = f.aR; si[cnt + 2] = f.kR;
  }
  const int nc = cnt + 3;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  double lb_[2], la_[2];
  int li_[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int e = min(c * 64 + lane, nc - 1);
    lb_[c] = sb[e];
    la_[c] = sa[e];
    li_[c] = si[e];
  }
  int nxt[2] = {-1, -1};
  double cn[2] = {0.0, 0.0}, cd[2] = {1.0, 1.0};
  const int nc0 = min(nc, 64);
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    if (c * 64 >= nc) break;
    const double bP = lb_[c], aP = la_[c];
    double rn = 0.0, rd = 1.0, rb = 0.0;
    int rj = -1;
    auto consider = [&](double bQ, double aQ, int j) {
      const double num = aP - aQ, den = bQ - bP;
      const double x = num * rd, y = rn * den;
      const bool take = (den > 0.0) & ((rj < 0) | (x < y) | ((x == y) & (bQ > rb)));
      rn = take ? num : rn;
      rd = take ? den : rd;
      rb = take ? bQ : rb;
      rj = take ? j : rj;
    };
#pragma unroll 4
    for (int j = 0; j < nc0; ++j) consider(readlane_f64(lb_[0], j), readlane_f64(la_[0], j), j);
    for (int j = 64; j < nc; ++j) consider(readlane_f64(lb_[1], j - 64), readlane_f64(la_[1], j - 64), j);
    nxt[c] = rj; cn[c] = rn; cd[c] = rd;
  }
  // chain from L (index cnt) to R, one vertex per step
  double kg = 0.0, cL = -INFINITY;
  int cur = cnt;
  for (int guard = 0; guard < nc; ++guard) {
    const bool hi = cur >= 64;
    const int ln = cur & 63;
    const double bP = readlane_f64(hi ? lb_[1] : lb_[0], ln);
    const double aP = readlane_f64(hi ? la_[1] : la_[0], ln);
    const int kP = __builtin_amdgcn_readlane(hi ? li_[1] : li_[0], ln);
    const int nx = __builtin_amdgcn_readlane(hi ? nxt[1] : nxt[0], ln);
    double cR = INFINITY;
    if (nx >= 0) {
      cR = readlane_f64(hi ? cn[1] : cn[0], ln) / readlane_f64(hi ? cd[1] : cd[0], ln);
      const double bQ = readlane_f64(nx >= 64 ? lb_[1] : lb_[0], nx & 63);
      kg += (bQ - bP) * psi((bQ <= bT) ? -cR : cR);
    }
    visit(kP, bP, aP, cL, cR);
    if (nx < 0) break;
    cL = cR;
    cur = nx;
  }
  return kg;
}

// Gift wrap over register lines with the line index carried (list overflow).
template <int MAXL, class Visit>
__device__ __forceinline__ double envelope_walk_visit(const double (&la)[MAXL], const double (&lb)[MAXL], int nl,
                                                      int lane, const EnvFilter& f, Visit&& visit) {
  double bc = f.bL, ac = f.aL, kg = 0.0, cL = -INFINITY;
  int kc = f.kL;
  for (int guard = 0; guard <= nl; ++guard) {
    if (!uniform(bc < f.bR)) break;
    double bn = INFINITY, bd = 1.0, bbest = -INFINITY, abest = -INFINITY;
    int kbest = 1 << 30;
#pragma unroll
    for (int t = 0; t < MAXL; ++t) {
      const double bb = lb[t], a = la[t];
      if (lane + 64 * t < nl && bb > bc) {
        const double num = ac - a, den = bb - bc;
        const double lhs = num * bd, rhs = bn * den;
        if (bbest == -INFINITY || lhs < rhs || (lhs == rhs && (bb > bbest || (bb == bbest && a > abest)))) {
          bn = num; bd = den; bbest = bb; abest = a; kbest = lane + 64 * t;
        }
      }
    }
    DKG_BUTTERFLY({
      const double on = partner_f64<S_>(bn), od = partner_f64<S_>(bd);
      const double ob = partner_f64<S_>(bbest), oa = partner_f64<S_>(abest);
      const int ok = __shfl_xor(kbest, S_ == 0 ? 1 : S_ == 1 ? 2 : S_ == 2 ? 4 : S_ == 3 ? 8 : S_ == 4 ? 16 : 32);
      bool take;
      if (ob == -INFINITY) take = false;
      else if (bbest == -INFINITY) take = true;
      else {
        const double lhs = on * bd, rhs = bn * od;
        take = lhs < rhs ||
               (lhs == rhs && (ob > bbest || (ob == bbest && (oa > abest || (oa == abest && ok < kbest)))));
      }
      if (take) { bn = on; bd = od; bbest = ob; abest = oa; kbest = ok; }
    })
    if (!uniform(bbest > bc)) break;
    const double c = bn / bd;
    kg += (bbest - bc) * psi((bbest <= f.bT) ? -c : c);
    visit(kc, bc, ac, cL, c);
    cL = c;
    bc = bbest;
    ac = abest;
    kc = __builtin_amdgcn_readfirstlane(kbest);
  }
  visit(kc, bc, ac, cL, INFINITY);
  return kg;
}

// Whole envelope stage for register-held lines (lines_kg_kernel).
template <int MAXL>
__device__ __forceinline__ double envelope_kg(const double (&la)[MAXL], const double (&lb)[MAXL], int nl, int lane,
                                              double* sb, double* sa, int* nhull) {
  const EnvFilter f = envelope_filter<MAXL>(la, lb, lane, sb, sa);
  if (f.status == 1) {
    if (nhull) *nhull = 1;
    return 0.0;
  }
  if (f.status == 2) return envelope_walk<MAXL>(la, lb, nl, lane, f.bL, f.aL, f.bR, f.bT, nhull);
  return envelope_hull(f, lane, sb, sa, nhull);
}

// Debug phase stamps (debug_flags & 4): [wave][8] s_memtime values.
constexpr int STAMP_WAVES = 4096;
__device__ unsigned long long g_stamps[STAMP_WAVES * 8];
#define DKG_STAMP(k)                                                                              \
  do {                                                                                            \
    if ((dbg & 4) && lane == 0) {                                                    \
      const int sw_ = ((blockIdx.y * gridDim.x + blockIdx.x) * (blockDim.x >> 6) + wave);         \
      if (sw_ < STAMP_WAVES) g_stamps[sw_ * 8 + (k)] = __builtin_amdgcn_s_memtime();              \
    }                                                                                             \
  } while (0)

// Padded length (doubles) of one LDS-staged line array: whole 1 KiB DMA pieces.
__host__ __device__ inline int stage_len(int N) { return ((N + 127) / 128) * 128; }

// Async global -> LDS copy of n doubles (16 B per lane per wave instruction,
// global_load_lds_dwordx4): the data never touches VGPRs and every piece of
// every wave is in flight at once.  `dst` has stage_len(n) doubles of room.
__device__ __forceinline__ void dma_to_lds(const double* __restrict__ src, double* dst, int n, int wave, int nwaves,
                                           int lane) {
  const int chunks = (n + 1) / 2;  // 16-byte pieces
  for (int c0 = wave * 64; c0 < chunks; c0 += nwaves * 64) {
    const int c = min(c0 + lane, chunks - 1);
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + 2 * c),
                                     reinterpret_cast<__attribute__((address_space(3))) void*>(
                                         reinterpret_cast<uintptr_t>(dst + 2 * c0)),
                                     16, 0, 0);
  }
}

// GRAD: also dKG/dx_b (envelope theorem; include/dkg.h dkg_plan_forward_grad),
// accumulated into dkg[b x d]; the extra LDS follows the survivor lists.
template <int MAXL, int M, bool GRAD>
__global__ __launch_bounds__(512) void envelope_kernel(const Plan* __restrict__ P, int B, double* __restrict__ kg,
                                                       double* __restrict__ pairs_out, int dst,
                                                       const double* __restrict__ xnew, double* __restrict__ dkg) {
  __shared__ double s_tail[16];
  __shared__ double s_sv[DKG_MAX_OUTPUTS];   // noiseless posterior variance at x_b, per output
  __shared__ double s_mx[DKG_MAX_OUTPUTS];   // posterior mean at x_b (model space), per output
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int b = blockIdx.x;
  const int g = blockIdx.y;
  const int SW = blockDim.x >> 6;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int m = P->m;  // <= M
  const int N = P->N;
  const int NL = N + 1;
  const int S = P->S;
  const int target = P->target;
  const int dbg = P->debug_env;
  const bool full = target < 0;
  const int SL = stage_len(N);
  DKG_STAMP(0);
  unsigned long long* st = kst_slot(dst, 2);
  KST_BEGIN(st);

  // Per-output scalars, hoisted once (static kernarg offsets).
  double ysd[M], ymu[M], nz[M], os[M];
#pragma unroll
  for (int i = 0; i < M; ++i) {
    ysd[i] = P->o[i].y_std;
    ymu[i] = P->o[i].y_mean;
    nz[i] = P->o[i].noise;
    os[i] = P->o[i].outputscale;
  }

  // LDS: [pad][mu_i over D] per output, [pad][cov_i over D] per output (line
  // k >= 1 reads index k - 1; the pad makes the lane-0 / slot-0 read legal),
  // the weights, then the per-wave survivor lists.
  const int SLp = SL + 2;
  double* lmu = smem + 2;
  double* lcv = lmu + (size_t)M * SLp;
  double* lw = lcv + (size_t)M * SLp;
  double* sbuf = lw + ((S * m + 1) & ~1);
  // GRAD regions: per-wave index lists, per-wave Q_D accumulators u_i[c], the
  // candidate's q_i and J_i rows, gv / gm / per-wave gradient scratch, x_b.
  const int d = P->d;
  const int NP = P->max_np;
  int* sidx = nullptr;
  double *uacc = nullptr, *qrow = nullptr, *jrow = nullptr, *sgv = nullptr, *sgm = nullptr, *sgw = nullptr,
         *sx = nullptr;
  if constexpr (GRAD) {
    double* gb = sbuf + (size_t)SW * 2 * ENV_CAP;
    sidx = reinterpret_cast<int*>(gb);
    uacc = gb + (SW * ENV_CAP + 1) / 2;
    qrow = uacc + (size_t)SW * M * NP;
    jrow = qrow + (size_t)M * NP;
    sgv = jrow + (size_t)M * d * NP;                // [M][16]  d v_i / dx
    sgm = sgv + M * DKG_MAX_DIM;                     // [M][16]  d mu_i / dx
    sgw = sgm + M * DKG_MAX_DIM;                     // [SW][64] per wave: gacc | ga0 | gvv | gtot
    sx = sgw + SW * 64;                              // [16]     x_b
  }

  // ---- one round of memory traffic: DMA the line data, plain loads for the rest
#pragma unroll
  for (int i = 0; i < M; ++i) {
    if (i < m && !(dbg & 8)) {
      dma_to_lds(P->o[i].disc_mean, lmu + (size_t)i * SLp, N, wave, SW, lane);
      if (full || i == target) dma_to_lds(P->cov[i] + (size_t)b * N, lcv + (size_t)i * SLp, N, wave, SW, lane);
    }
  }
  for (int e = threadIdx.x; e < S * m; e += blockDim.x) lw[e] = P->weights[e];
  // candidate's own posterior (variance from the covariance stage, mean from the cross stage)
  if (threadIdx.x < m) {
    s_sv[threadIdx.x] = P->var[threadIdx.x][b];
    s_mx[threadIdx.x] = P->mux[threadIdx.x][b];
  }
  if constexpr (GRAD) {
    // the candidate's q_i and J_i rows (fragment-packed in the workspace)
#pragma unroll
    for (int i = 0; i < M; ++i) {
      if (i < m) {
        const int npi = pad16(P->o[i].n), KBi = npi / 4;
        const size_t mat = (size_t)P->bpad * npi;
        for (int c = threadIdx.x; c < NP; c += blockDim.x) {
          const size_t fi = frag_index(b >> 4, c >> 2, ((c & 3) << 4) | (b & 15), KBi);
          qrow[(size_t)i * NP + c] = (c < npi) ? P->q[i][fi] : 0.0;
          for (int dd = 0; dd < d; ++dd) jrow[((size_t)i * d + dd) * NP + c] = (c < npi) ? P->jq[i][dd * mat + fi] : 0.0;
        }
      }
    }
    if (threadIdx.x < m * d) {
      const int i = threadIdx.x / d, dd = threadIdx.x % d;
      sgm[i * DKG_MAX_DIM + dd] = P->gmu[i][(size_t)dd * P->bpad + b];
    }
    if (threadIdx.x < d) sx[threadIdx.x] = xnew[(size_t)b * d + threadIdx.x];
  }
  KST(st, 2);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  DKG_STAMP(1);
  KST(st, 3);

  double* sb = sbuf + (size_t)wave * 2 * ENV_CAP;
  double* sa = sb + ENV_CAP;
  double wave_acc = 0.0;
  int* si = nullptr;
  double *uw = nullptr, *gw = nullptr;
  if constexpr (GRAD) {
    si = sidx + (size_t)wave * ENV_CAP;
    uw = uacc + (size_t)wave * M * NP;
    gw = sgw + wave * 64;
    // d v_i / dx = -2 J_i^T q_i (model space), one (output, coordinate) per wave
    for (int pidx = wave; pidx < m * d; pidx += SW) {
      const int i = pidx / d, dd = pidx % d;
      double acc = 0.0;
      for (int c = lane; c < NP; c += 64) acc = fma(jrow[((size_t)i * d + dd) * NP + c], qrow[(size_t)i * NP + c], acc);
      acc = wave_sum(acc);
      if (lane == 0) sgv[i * DKG_MAX_DIM + dd] = -2.0 * acc;
    }
    for (int e = lane; e < M * NP; e += 64) uw[e] = 0.0;
    for (int e = lane; e < 64; e += 64) gw[e] = 0.0;
    __syncthreads();
  }
  const int waves_total = SW * gridDim.y;
  double sv[M], mx0[M];
#pragma unroll
  for (int i = 0; i < M; ++i) {
    sv[i] = (i < m) ? s_sv[i] : 0.0;
    mx0[i] = (i < m) ? s_mx[i] : 0.0;
  }

  for (int j = g * SW + wave; j < S; j += waves_total) {
    // ---- line coefficients (wave uniform)
    double w[M], wa[M], wb[M];
    double a_off = 0.0, den = 0.0;
#pragma unroll
    for (int i = 0; i < M; ++i) {
      w[i] = (i < m) ? lw[j * m + i] : 0.0;
      wa[i] = w[i] * ysd[i];
      a_off = fma(w[i], ymu[i], a_off);
      den = fma(w[i] * w[i], ysd[i] * ysd[i] * (sv[i] + nz[i]), den);
    }
    if (full) {
      const double inv_den = 1.0 / sqrt(den);
#pragma unroll
      for (int i = 0; i < M; ++i) wb[i] = w[i] * w[i] * ysd[i] * ysd[i] * inv_den;
    } else {
#pragma unroll
      for (int i = 0; i < M; ++i) {
        const double sd2 = ysd[i] * ysd[i];
        wb[i] = (i == target) ? w[i] * sd2 / sqrt(sd2 * (sv[i] + nz[i])) : 0.0;
      }
    }
    // ---- lines: slot t of lane l is line k = l + 64 t (k = 0: the candidate).
    // Branch-free bodies (one LDS read stream per array, no per-slot waits):
    // unused output slots read output 0 with a zero weight.  Rebuilt from the
    // staged LDS data when the survivor list overflows, so the register copy
    // is dead once the filter has run.
    auto build_lines = [&](double (&la)[MAXL], double (&lb)[MAXL]) {
      const double* mup[M];
#pragma unroll
      for (int i = 0; i < M; ++i) mup[i] = lmu + (size_t)((i < m) ? i : 0) * SLp + lane - 1;
      if (full) {
        const double* cvp[M];
#pragma unroll
        for (int i = 0; i < M; ++i) cvp[i] = lcv + (size_t)((i < m) ? i : 0) * SLp + lane - 1;
#pragma unroll
        for (int t = 0; t < MAXL; ++t) {
          double a = a_off, bb = 0.0;
#pragma unroll
          for (int i = 0; i < M; ++i) {
            a = fma(wa[i], mup[i][64 * t], a);
            bb = fma(wb[i], cvp[i][64 * t], bb);
          }
          la[t] = a;
          lb[t] = bb;
        }
      } else {
        const double* cvt = lcv + (size_t)target * SLp + lane - 1;
        double wbt = 0.0;
#pragma unroll
        for (int i = 0; i < M; ++i) wbt = (i == target) ? wb[i] : wbt;
#pragma unroll
        for (int t = 0; t < MAXL; ++t) {
          double a = a_off;
#pragma unroll
          for (int i = 0; i < M; ++i) a = fma(wa[i], mup[i][64 * t], a);
          la[t] = a;
          lb[t] = wbt * cvt[64 * t];
        }
      }
      {
        double a = a_off, bb = 0.0;  // line 0: the candidate itself (discretekg.py:182-183)
#pragma unroll
        for (int i = 0; i < M; ++i) {
          a = fma(wa[i], mx0[i], a);
          bb = fma(wb[i], sv[i], bb);
        }
        la[0] = (lane == 0) ? a : la[0];
        lb[0] = (lane == 0) ? bb : lb[0];
      }
      // padding lines beyond N (only in the last slots): never maximal, never
      // change the min/max slope
      const double bfill = __shfl(lb[0], 0);
#pragma unroll
      for (int t = 0; t < MAXL; ++t) {
        if (64 * t + 63 > N) {  // wave-uniform
          const bool pad = lane + 64 * t > N;
          la[t] = pad ? -INFINITY : la[t];
          lb[t] = pad ? bfill : lb[t];
        }
      }
    };

    double kgj;
    EnvFilter f;
    if constexpr (GRAD) {
      {
        double la[MAXL], lb[MAXL];
        build_lines(la, lb);
        f = envelope_filter<MAXL, true>(la, lb, lane, sb, sa, si);
      }
      double Vden = den;  // the variance under the square root of the slopes
      if (!full) {
        const double sd2 = ysd[target] * ysd[target];
        Vden = sd2 * (sv[target] + nz[target]);
      }
      if (lane == 0) {
        for (int dd = 0; dd < d; ++dd) {
          double ga0 = 0.0, gvs = 0.0;
#pragma unroll
          for (int i = 0; i < M; ++i) {
            if (i < m) {
              ga0 = fma(wa[i], sgm[i * DKG_MAX_DIM + dd], ga0);
              const double cv = full ? w[i] * w[i] * ysd[i] * ysd[i] : ((i == target) ? ysd[i] * ysd[i] : 0.0);
              gvs = fma(cv, sgv[i * DKG_MAX_DIM + dd], gvs);
            }
          }
          gw[16 + dd] = ga0;
          gw[32 + dd] = gvs / (2.0 * Vden);
        }
      }
      double sumDb = 0.0;
      // one envelope line: d/dx of its slope (and of line 0's intercept), weighted
      // by dE/db = phi(cL) - phi(cR) and dE/da = Phi(cR) - Phi(cL)
      auto visit = [&](int k, double bP, double aP, double cL, double cR) {
        (void)aP;
        const double Pw = norm_cdf(cR) - norm_cdf(cL);
        const double Dw = norm_pdf(cL) - norm_pdf(cR);
        sumDb = fma(Dw, bP, sumDb);
        if (k == 0) {
          if (lane == 0) {
            for (int dd = 0; dd < d; ++dd) {
              double gvs = 0.0;
#pragma unroll
              for (int i = 0; i < M; ++i)
                if (i < m) gvs = fma(wb[i], sgv[i * DKG_MAX_DIM + dd], gvs);
              gw[dd] += Dw * gvs + Pw * gw[16 + dd];
            }
          }
        } else if (k <= N) {
          const double* z = P->disc + (size_t)(k - 1) * d;
#pragma unroll
          for (int i = 0; i < M; ++i) {
            if (i < m && wb[i] != 0.0) {
              const dkg_output& o = P->o[i];
              double r2 = 0.0;
              for (int dd = 0; dd < d; ++dd) {
                const double t = (sx[dd] - z[dd]) * o.inv_lengthscale[dd];
                r2 = fma(t, t, r2);
              }
              const double coef = Dw * wb[i];
              const double hc = coef * os[i] * kernel_dprofile(o.kernel, r2);
              if (lane == 0)
                for (int dd = 0; dd < d; ++dd) {
                  const double il = o.inv_lengthscale[dd];
                  gw[dd] += hc * (sx[dd] - z[dd]) * il * il;
                }
              const int npi = pad16(o.n), KBi = npi / 4, r = k - 1;
              for (int c = lane; c < npi; c += 64)
                uw[(size_t)i * NP + c] = fma(coef, o.disc_frag[frag_index(r >> 4, c >> 2, ((c & 3) << 4) | (r & 15), KBi)],
                                             uw[(size_t)i * NP + c]);
            }
          }
        }
      };
      if (f.status == 1) {
        kgj = 0.0;
      } else {
        if (f.status == 0) {
          kgj = envelope_hull_visit(f, lane, sb, sa, si, visit);
        } else {
          double la[MAXL], lb[MAXL];
          build_lines(la, lb);
          kgj = envelope_walk_visit<MAXL>(la, lb, NL, lane, f, visit);
        }
        // - sum_i J_i^T u_i, - sum_e Dw_e b_e * dV/(2V), - [line 0 attains max a] da_0/dx
        for (int pidx = 0; pidx < m * d; ++pidx) {
          const int i = pidx / d, dd = pidx % d;
          double acc = 0.0;
          for (int c = lane; c < NP; c += 64) acc = fma(jrow[((size_t)i * d + dd) * NP + c], uw[(size_t)i * NP + c], acc);
          acc = wave_sum(acc);
          if (lane == 0) gw[dd] -= acc;
        }
        double a0 = a_off;
#pragma unroll
        for (int i = 0; i < M; ++i) a0 = fma(wa[i], mx0[i], a0);
        const double tfac = (a0 == f.aT) ? 1.0 / (double)f.cntT : 0.0;
        if (lane == 0)
          for (int dd = 0; dd < d; ++dd) gw[48 + dd] += gw[dd] - sumDb * gw[32 + dd] - tfac * gw[16 + dd];
        for (int e = lane; e < M * NP; e += 64) uw[e] = 0.0;
      }
      if (lane == 0)
        for (int dd = 0; dd < d; ++dd) gw[dd] = 0.0;
    } else {
      double la[MAXL], lb[MAXL];
      build_lines(la, lb);
      DKG_STAMP(2);
      if (dbg & 1) {  // ablation: lines + one reduction only
        double mxv = -INFINITY;
#pragma unroll
        for (int t = 0; t < MAXL; ++t) mxv = fmax(mxv, la[t] + lb[t]);
        f.status = 3;
        f.aT = wave_max(mxv);
      } else {
        f = envelope_filter<MAXL>(la, lb, lane, sb, sa);
      }
    }
    if constexpr (GRAD) {
    } else if (f.status == 3) {
      kgj = f.aT;
    } else if (f.status == 1) {
      kgj = 0.0;
    } else if (dbg & 32) {  // debug: report the candidate count instead of KG
      kgj = (double)(f.cnt + 3);
    } else if (f.status == 0) {
      kgj = envelope_hull(f, lane, sb, sa, nullptr, dbg);
    } else {  // list overflow: gift wrap over the (rebuilt) register lines
      double la[MAXL], lb[MAXL];
      build_lines(la, lb);
      kgj = envelope_walk<MAXL>(la, lb, NL, lane, f.bL, f.aL, f.bR, f.bT, nullptr);
    }
    DKG_STAMP(3);
    if (pairs_out != nullptr && lane == 0) pairs_out[(size_t)b * S + j] = kgj;
    wave_acc += kgj;
  }

  // ---- mean over S: per-wave sums -> per-WG sum (fixed order) -> across WGs
  KST(st, 4);
  if (lane == 0) s_tail[wave] = wave_acc;
  __syncthreads();
  DKG_STAMP(4);
  KST(st, 5);
  if constexpr (GRAD) {
    if (threadIdx.x < d) {
      double gs = 0.0;
      for (int w2 = 0; w2 < SW; ++w2) gs += sgw[w2 * 64 + 48 + threadIdx.x];
      // at most two workgroups per candidate (S <= 16): commutative, deterministic
      atomicAdd(&dkg[(size_t)b * d + threadIdx.x], gs / (double)S);
    }
  }
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int w2 = 0; w2 < SW; ++w2) s += s_tail[w2];
    const int G = gridDim.y;
    if (G == 1) {
      kg[b] = s / (double)S;
    } else if (G == 2 || (dbg & 2)) {
      // two addends onto a zeroed cell: fp addition commutes, so the order
      // the two workgroups arrive in does not change the bits.
      atomicAdd(&kg[b], s / (double)S);
    } else {
      P->wg_part[(size_t)b * G + g] = s;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int prev = atomicAdd(&P->tickets[b], 1);
      if (prev == G - 1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        double tot = 0.0;
        for (int q = 0; q < G; ++q)
          tot += __hip_atomic_load(&P->wg_part[(size_t)b * G + q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        kg[b] = tot / (double)S;
      }
    }
  }
  __syncthreads();
  DKG_STAMP(5);
  KST_END(st);
}

static int outputs_bucket(int m) { return m <= 1 ? 1 : m <= 2 ? 2 : m <= 3 ? 3 : m <= 4 ? 4 : 8; }

size_t envelope_lds_bytes(int m, int N, int waves, int S) {
  const int M = outputs_bucket(m);
  return ((size_t)2 + 2 * (size_t)M * (stage_len(N) + 2) + ((S * m + 1) & ~1) + (size_t)waves * 2 * ENV_CAP) *
         sizeof(double);
}

size_t envelope_grad_lds_bytes(int m, int N, int waves, int S, int d, int max_np) {
  const int M = outputs_bucket(m);
  const size_t extra = (size_t)(waves * ENV_CAP + 1) / 2 + (size_t)waves * M * max_np + (size_t)M * max_np +
                       (size_t)M * d * max_np + 2 * (size_t)M * DKG_MAX_DIM + (size_t)waves * 64 + DKG_MAX_DIM;
  return envelope_lds_bytes(m, N, waves, S) + extra * sizeof(double);
}

// ---------------------------------------------------------------------------
// lines_kg_kernel: KG = E[max_k (a_k + b_k Z)] - max_k a_k for P independent
// sets of L lines (row-major [P][L]); one wave per set.  Exposes the envelope
// stage on its own (reference calculate_epigraph_indices +
// calculate_expected_value_of_piecewise_linear_function, discretekg.py:341-452).
template <int MAXL>
__global__ __launch_bounds__(256) void lines_kg_kernel(const double* __restrict__ a, const double* __restrict__ b,
                                                        int P, int L, double* __restrict__ kg, int* __restrict__ nhull) {
  extern __shared__ __attribute__((aligned(16))) double sbuf[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int p = blockIdx.x * (blockDim.x >> 6) + wave;
  if (p >= P) return;
  double la[MAXL], lb[MAXL];
#pragma unroll
  for (int t = 0; t < MAXL; ++t) {
    const int k = min(lane + 64 * t, L - 1);
    la[t] = a[(size_t)p * L + k];
    lb[t] = b[(size_t)p * L + k];
  }
  double* sb = sbuf + (size_t)wave * 2 * ENV_CAP;
  int h = 0;
  const double v = envelope_kg<MAXL>(la, lb, L, lane, sb, sb + ENV_CAP, &h);
  if (lane == 0) {
    kg[p] = v;
    if (nhull) nhull[p] = h;
  }
}

// ---------------------------------------------------------------------------
__global__ void debug_mfma_kernel(const double* __restrict__ a, const double* __restrict__ b, double* __restrict__ c) {
  const int l = threadIdx.x;
  d4 acc = {0.0, 0.0, 0.0, 0.0};
  acc = mfma_f64(a[(l & 15) * 4 + (l >> 4)], b[(l >> 4) * 16 + (l & 15)], acc);
#pragma unroll
  for (int r = 0; r < 4; ++r) c[((l >> 4) + 4 * r) * 16 + (l & 15)] = acc[r];
}

// Self-test of the register butterflies: out[64 s + l] = partner_f64<s>(in[l])
// for s = 0..5, out[384 + l] = wave_sum(in), out[448 + l] = wave_max(in).
__global__ void debug_wave_kernel(const double* __restrict__ in, double* __restrict__ out) {
  const int l = threadIdx.x;
  const double v = in[l];
  out[0 * 64 + l] = partner_f64<0>(v);
  out[1 * 64 + l] = partner_f64<1>(v);
  out[2 * 64 + l] = partner_f64<2>(v);
  out[3 * 64 + l] = partner_f64<3>(v);
  out[4 * 64 + l] = partner_f64<4>(v);
  out[5 * 64 + l] = partner_f64<5>(v);
  out[6 * 64 + l] = wave_sum(v);
  out[7 * 64 + l] = wave_max(v);
}

// ---------------------------------------------------------------------------
// Launch helpers (host).
hipError_t launch_kernel_matrix(const dkg_output& o, int d, const double* x1, int n1, const double* x2, int n2,
                                double diag_add, double* out, hipStream_t s) {
  dim3 grid((n2 + 255) / 256, n1);
  hipLaunchKernelGGL(kernel_matrix_kernel, grid, dim3(256), 0, s, o, d, x1, n1, x2, n2, diag_add, out);
  return hipGetLastError();
}

hipError_t launch_pack_root(const double* r, int n, double* rf, hipStream_t s) {
  const size_t total = (size_t)pad16(n) * pad16(n);
  const int blocks = (int)std::min<size_t>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(pack_root_kernel, dim3(blocks), dim3(256), 0, s, r, n, rf);
  return hipGetLastError();
}

template <int DM>
static hipError_t launch_cross_root_t(const CrossArgs& a, hipStream_t s) {
  const int np = pad16(a.o.n);
  dim3 grid(pad16(a.rows) / 16, (np / 16 + 1) / 2, 1);
  const size_t lds = cross_root_lds_bytes(np, a.d);
  if (lds > 65536)
    (void)hipFuncSetAttribute((const void*)cross_root_kernel<DM>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(cross_root_kernel<DM>, grid, dim3(CR_WAVES * WAVE), lds, s, a);
  return hipGetLastError();
}

hipError_t launch_cross_root(const CrossArgs& a, hipStream_t s) {
  switch (dim_bucket(a.d)) {
    case 2: return launch_cross_root_t<2>(a, s);
    case 4: return launch_cross_root_t<4>(a, s);
    case 8: return launch_cross_root_t<8>(a, s);
    default: return launch_cross_root_t<16>(a, s);
  }
}

template <int DM>
static hipError_t launch_cross_cov_t(const Plan& h, const Plan* dev, const double* xnew, int B, double* kg,
                                     hipStream_t s, int stage) {
  if (stage == 0) {
    dim3 grid(pad16(B) / 16, (h.max_np / 16 + 1) / 2, h.m);
    const size_t lds = cross_root_lds_bytes(h.max_np, h.d);
    if (lds > 65536)
      (void)hipFuncSetAttribute((const void*)cross_root_plan_kernel<DM>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds);
    hipLaunchKernelGGL(cross_root_plan_kernel<DM>, grid, dim3(CR_WAVES * WAVE), lds, s, dev, xnew, B, kg,
                       h.debug_stamp);
    return hipGetLastError();
  }
  dim3 grid(std::max(1, (h.N + 31) / 32), (B + 31) / 32, h.m);
  hipLaunchKernelGGL(posterior_cov_kernel<DM>, grid, dim3(PC_WAVES * WAVE), 0, s, dev, xnew, B, h.debug_stamp);
  return hipGetLastError();
}

void envelope_geometry(int B, int S, int* waves_per_wg, int* split) {
  // Up to 8 scalarisation waves of one candidate per workgroup; with S <= 16
  // at most two workgroups per candidate, whose partial sums meet in one
  // commutative atomic add (no inter-workgroup fences).
  (void)B;
  const int sw = std::max(1, std::min(8, S));
  *waves_per_wg = sw;
  *split = (S + sw - 1) / sw;
}

struct EnvLaunch {
  const Plan* dev;
  int B;
  double* kg;
  double* pairs;
  dim3 grid, block;
  size_t lds;
  hipStream_t s;
  int dst;
  const double* xnew;  // GRAD
  double* dkg;         // GRAD
};

template <int MAXL, int M, bool GRAD>
static hipError_t launch_env_t(const EnvLaunch& a) {
  if (a.lds > 65536)
    (void)hipFuncSetAttribute((const void*)envelope_kernel<MAXL, M, GRAD>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)a.lds);
  hipLaunchKernelGGL((envelope_kernel<MAXL, M, GRAD>), a.grid, a.block, a.lds, a.s, a.dev, a.B, a.kg, a.pairs, a.dst,
                     a.xnew, a.dkg);
  return hipGetLastError();
}

template <int M, bool GRAD>
static hipError_t launch_env_m(int lines, const EnvLaunch& a) {
  if (lines <= 64 * 2) return launch_env_t<2, M, GRAD>(a);
  if (lines <= 64 * 4) return launch_env_t<4, M, GRAD>(a);
  if (lines <= 64 * 8) return launch_env_t<8, M, GRAD>(a);
  if (lines <= 64 * 17) return launch_env_t<17, M, GRAD>(a);
  if (lines <= 64 * 33) return launch_env_t<33, M, GRAD>(a);
  return hipErrorInvalidValue;
}

template <bool GRAD>
static hipError_t launch_env(const Plan& h, const EnvLaunch& a) {
  switch (outputs_bucket(h.m)) {
    case 1: return launch_env_m<1, GRAD>(h.N + 1, a);
    case 2: return launch_env_m<2, GRAD>(h.N + 1, a);
    case 3: return launch_env_m<3, GRAD>(h.N + 1, a);
    case 4: return launch_env_m<4, GRAD>(h.N + 1, a);
    default: return launch_env_m<8, GRAD>(h.N + 1, a);
  }
}

// The three launches of one forward on `s`; ev (nullable) gets 4 events
// recorded around them (dkg_forward_timed).
hipError_t launch_stage(const Plan& h, const Plan* dev, const double* xnew, int B, double* kg, double* pairs,
                        hipStream_t s, int stage) {
  if (stage == 0 || stage == 1) {
    switch (dim_bucket(h.d)) {
      case 2: return launch_cross_cov_t<2>(h, dev, xnew, B, kg, s, stage);
      case 4: return launch_cross_cov_t<4>(h, dev, xnew, B, kg, s, stage);
      case 8: return launch_cross_cov_t<8>(h, dev, xnew, B, kg, s, stage);
      default: return launch_cross_cov_t<16>(h, dev, xnew, B, kg, s, stage);
    }
  }
  EnvLaunch a{dev, B, kg, pairs, dim3(B, h.split), dim3(h.sw * WAVE), envelope_lds_bytes(h.m, h.N, h.sw, h.S), s,
              h.debug_stamp, nullptr, nullptr};
  return launch_env<false>(h, a);
}

template <int DM>
static hipError_t launch_cross_grad_t(const Plan& h, const Plan* dev, const double* xnew, int B, double* dkg,
                                      hipStream_t s) {
  dim3 grid(pad16(B) / 16, (h.max_np / 16 + 1) / 2, h.m * h.d);
  const size_t lds = cross_root_lds_bytes(h.max_np, h.d);
  if (lds > 65536)
    (void)hipFuncSetAttribute((const void*)cross_grad_plan_kernel<DM>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
  hipLaunchKernelGGL(cross_grad_plan_kernel<DM>, grid, dim3(CR_WAVES * WAVE), lds, s, dev, xnew, B, dkg, 0);
  return hipGetLastError();
}

hipError_t launch_forward_grad(const Plan& h, const Plan* dev, const double* xnew, int B, double* kg, double* dkg,
                               hipStream_t s) {
  hipError_t e;
  if ((e = launch_stage(h, dev, xnew, B, kg, nullptr, s, 0)) != hipSuccess) return e;  // Q_X, means; kg = 0
  if ((e = launch_stage(h, dev, xnew, B, kg, nullptr, s, 1)) != hipSuccess) return e;  // cov rows, variances
  switch (dim_bucket(h.d)) {                                                            // J_g, dmean; dkg = 0
    case 2: e = launch_cross_grad_t<2>(h, dev, xnew, B, dkg, s); break;
    case 4: e = launch_cross_grad_t<4>(h, dev, xnew, B, dkg, s); break;
    case 8: e = launch_cross_grad_t<8>(h, dev, xnew, B, dkg, s); break;
    default: e = launch_cross_grad_t<16>(h, dev, xnew, B, dkg, s); break;
  }
  if (e != hipSuccess) return e;
  EnvLaunch a{dev, B, kg, nullptr, dim3(B, h.split), dim3(h.sw * WAVE),
              envelope_grad_lds_bytes(h.m, h.N, h.sw, h.S, h.d, h.max_np), s, 0, xnew, dkg};
  return launch_env<true>(h, a);
}

hipError_t launch_forward(const Plan& h, const Plan* dev, const double* xnew, int B, double* kg, double* pairs,
                          hipStream_t s, hipEvent_t* ev) {
  for (int stage = 0; stage < 3; ++stage) {
    if (ev) (void)hipEventRecord(ev[stage], s);
    const hipError_t e = launch_stage(h, dev, xnew, B, kg, pairs, s, stage);
    if (e != hipSuccess) return e;
  }
  if (ev) (void)hipEventRecord(ev[3], s);
  return hipSuccess;
}

hipError_t launch_lines_kg(const double* a, const double* b, int P, int L, double* kg, int* nhull, hipStream_t s) {
  const int wpb = 4;
  dim3 grid((P + wpb - 1) / wpb), block(wpb * WAVE);
  const size_t lds = (size_t)wpb * 2 * ENV_CAP * sizeof(double);
  if (L <= 64 * 2) hipLaunchKernelGGL(lines_kg_kernel<2>, grid, block, lds, s, a, b, P, L, kg, nhull);
  else if (L <= 64 * 4) hipLaunchKernelGGL(lines_kg_kernel<4>, grid, block, lds, s, a, b, P, L, kg, nhull);
  else if (L <= 64 * 8) hipLaunchKernelGGL(lines_kg_kernel<8>, grid, block, lds, s, a, b, P, L, kg, nhull);
  else if (L <= 64 * 17) hipLaunchKernelGGL(lines_kg_kernel<17>, grid, block, lds, s, a, b, P, L, kg, nhull);
  else if (L <= 64 * 33) hipLaunchKernelGGL(lines_kg_kernel<33>, grid, block, lds, s, a, b, P, L, kg, nhull);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t read_kstamps(unsigned long long* host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_kstamps), sizeof(unsigned long long) * std::min(n, 3 * KST_WG * 8));
}

hipError_t read_stamps(unsigned long long* host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * std::min(n, STAMP_WAVES * 8));
}

hipError_t launch_debug_wave(const double* in, double* out, hipStream_t s) {
  hipLaunchKernelGGL(debug_wave_kernel, dim3(1), dim3(64), 0, s, in, out);
  return hipGetLastError();
}

hipError_t launch_debug_mfma(const double* a, const double* b, double* c, hipStream_t s) {
  hipLaunchKernelGGL(debug_mfma_kernel, dim3(1), dim3(64), 0, s, a, b, c);
  return hipGetLastError();
}

}  // namespace dkg
