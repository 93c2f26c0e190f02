// Fitted-state preparation on the device (gfx950): the caches GPyTorch's exact
// prediction keeps behind model.posterior (discretekg.py:182-185, 275-284;
// gpytorch DefaultPredictionStrategy + linear_operator psd_safe_cholesky):
//   L = chol(K)          blocked right-looking Cholesky (panel + MFMA trailing update)
//   Linv = L^{-1}        blocked right-looking triangular inverse (panel + MFMA update)
//   alpha = Linv^T Linv (y - c)
// K, L and Linv are row-major n x n fp64 (lower triangles; the upper triangle
// of L / Linv is zeroed at the end).  n <= 1024.  One launch pair per 32-wide
// block column: a single-workgroup panel kernel (factor / invert the diagonal
// block and solve the column below it) and a trailing-update kernel with one
// workgroup per 32 x 32 tile (four v_mfma_f64_16x16x4 sub-tiles, K = 32).
#include <algorithm>

#include "dkg_kernels.h"

namespace dkg {

constexpr int LB = 32;  // block width
#ifndef DKG_CHOL_TIMING
#define DKG_CHOL_TIMING 0
#endif
#ifndef DKG_CHOL_LDS_BCAST
#define DKG_CHOL_LDS_BCAST 1
#endif
// The pivot's sqrt and the column's division correctly rounded, as LAPACK's potrf does.  v_rsq_f64 + one Newton
// step saved ~0.02 ms of the 0.45 ms preparation but rounds differently; on the SMOKE surrogates (noise 1e-8,
// conditioning ~1e10) that difference moved L-BFGS-B runs from the oracle's by 3e-5 (profiles/r04/exactpiv/).
#ifndef DKG_CHOL_EXACT_PIVOT
#define DKG_CHOL_EXACT_PIVOT 1
#endif

// Lower tile (ti, tj), tj <= ti, of the row-major enumeration t = ti (ti + 1) / 2 + tj.
__device__ __forceinline__ void lower_tile(int t, int& ti, int& tj) {
  ti = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
  while ((ti + 1) * (ti + 2) / 2 <= t) ++ti;
  while (ti * (ti + 1) / 2 > t) --ti;
  tj = t - ti * (ti + 1) / 2;
}

// ---------------------------------------------------------------------------
// The diagonal block kb of one output, updated and held in LDS (sC, lower triangle valid): factor it
// (L_kk), invert it (W_kk = L_kk^{-1}), store L_kk into A's lower block (the block's upper part zeroed)
// and W_kk into X's diagonal block (the final inverse's diagonal block).  info: LAPACK potrf convention
// (first failing column + 1; NaN and non-positive pivots fail).  Called by the whole workgroup.
__device__ __forceinline__ void factor_diag(double* __restrict__ A, double* __restrict__ X, int n, int kb,
                                            int* __restrict__ info, double (*sC)[LB + 1], double (*sL)[LB + 1]) {
  __shared__ int bad;
  __shared__ __attribute__((aligned(16))) double scol[2][LB];  // the factoring wave's current column (by parity)
  __shared__ __attribute__((aligned(16))) double sT[16][17];    // W = L^{-1}: L21 W11
  const int k0 = kb * LB, nb = min(LB, n - k0);
  const int tid = threadIdx.x;
#if DKG_CHOL_TIMING
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned long long t1 = 0;
#endif
  if (tid < 64) {
    // one wave, lane r holds row r (rows past nb are identity rows); column j's pivot and entries reach
    // the other lanes by v_readlane, so the 32 steps need no LDS round trip and no barrier
    const int lane = tid;
    double a[LB];
#pragma unroll
    for (int c = 0; c < LB; ++c)
      a[c] = (lane < nb) ? ((c <= lane) ? sC[lane][c] : 0.0) : ((c == lane) ? 1.0 : 0.0);
    int fail = 0;
#pragma unroll
    for (int j = 0; j < LB; ++j) {
      if (j < nb && fail == 0) {  // uniform
        const double piv = readlane_f64(a[j], j);
        if (!(piv > 0.0) || !isfinite(piv)) {  // NaN fails too
          fail = k0 + j + 1;
        } else {
          // 1/sqrt(piv) by v_rsq_f64 and one Newton step, then L[j][j] = piv / sqrt(piv) and L[c][j] = a / sqrt(piv)
          // as products (the correctly rounded sqrt and division sequences made the step's dependent chain)
#if DKG_CHOL_EXACT_PIVOT
          // LAPACK's operations: the correctly rounded sqrt, and the column divided by it
          const double dj = sqrt(piv);
          a[j] = (lane == j) ? dj : a[j] / dj;
#else
          double rq = __builtin_amdgcn_rsq(piv);
          rq = rq * fma(-0.5 * piv, rq * rq, 1.5);
          const double dj = piv * rq;
          // (entries above the diagonal take part unmasked: they are never read into the lower triangle, and the
          // rows are masked when the factor leaves the registers)
          a[j] = (lane == j) ? dj : a[j] * rq;
#endif
#if DKG_CHOL_LDS_BCAST
          // column j through LDS: one store, then every lane reads L[c][j] (c > j) back as broadcasts
          // (16-byte reads of two entries) instead of 31 v_readlane pairs.  Two buffers by column parity: a
          // wave's LDS operations complete in issue order, so neither the read-after-write of this column nor
          // the next column's store needs a fence
          double* sc = scol[j & 1];
          if (lane < LB) sc[lane] = a[j];
#pragma unroll
          for (int c = j + 1; c < LB; ++c) {
            if (c < nb) {
              const double lcj = sc[c];  // L[c][j]
              a[c] = fma(-a[j], lcj, a[c]);
            }
          }
#else
#pragma unroll
          for (int c = j + 1; c < LB; ++c) {
            if (c < nb) {
              const double lcj = readlane_f64(a[j], c);  // L[c][j]
              a[c] = (lane >= c) ? fma(-a[j], lcj, a[c]) : a[c];
            }
          }
#endif
        }
      }
    }
    if (lane < LB) {
#pragma unroll
      for (int c = 0; c < LB; ++c) sL[lane][c] = (c <= lane) ? a[c] : 0.0;
    }
    if (lane == 0) bad = fail;
#if DKG_CHOL_TIMING
    t1 = __builtin_amdgcn_s_memtime();
#endif
    if (fail == 0) {
      // W = L^{-1} as 2 x 2 blocks of 16: lanes 0-15 solve L11 w = e_c (W11's columns) while lanes 16-31 solve
      // L22 w = e_c (W22's), 16 steps each, the entries L[j][q] read from sL as broadcasts within each half;
      // then W21 = -W22 (L21 W11) by two 16 x 16 MFMA products (the single 32-step solve with v_readlane
      // broadcasts took ~35 K cycles)
      const int h = (lane >> 4) & 1, cc = lane & 15, base = 16 * h;
      double w[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        double acc = (cc == j) ? 1.0 : 0.0;
#pragma unroll
        for (int q = 0; q < j; ++q) acc = fma(-sL[base + j][base + q], w[q], acc);
        w[j] = acc / sL[base + j][base + j];
      }
      __shared__ double sW11[16][17];
      if (lane < 16) {
#pragma unroll
        for (int j = 0; j < 16; ++j) sW11[j][cc] = w[j];
      }
      // T = L21 W11 (A: L21 from sL rows 16..31, cols 0..15; B: W11), then W21 = -(W22 T) (A: W22, B: T)
      d4 t = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int kb2 = 0; kb2 < 4; ++kb2) {
        const int kk = 4 * kb2 + (lane >> 4);
        t = mfma_f64(sL[16 + (lane & 15)][kk], sW11[kk][lane & 15], t);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) sT[(lane >> 4) + 4 * r][lane & 15] = t[r];
      double w22[16];  // lanes 16..31 hold W22's column cc; broadcast through LDS for the MFMA A operand
#pragma unroll
      for (int j = 0; j < 16; ++j) w22[j] = w[j];
      __shared__ double sW22[16][17];
      if (h == 1 && lane < 32) {
#pragma unroll
        for (int j = 0; j < 16; ++j) sW22[j][cc] = w22[j];
      }
      d4 u = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int kb2 = 0; kb2 < 4; ++kb2) {
        const int kk = 4 * kb2 + (lane >> 4);
        u = mfma_f64(sW22[lane & 15][kk], sT[kk][lane & 15], u);
      }
      // X's diagonal block: W11 (top left), W21 (bottom left), W22 (bottom right), zeros at the top right (the
      // panel solves and the inverse's MFMAs read the whole block)
      if (lane < 32) {
        const int c = lane;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int r = base + j;
          if (r < nb && c < nb) X[(size_t)(k0 + r) * n + k0 + c] = (h == 0) ? w[j] : w22[j];
          if (h == 1 && j < nb && c < nb) X[(size_t)(k0 + j) * n + k0 + c] = 0.0;
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 + (lane >> 4) + 4 * r, col = lane & 15;
        if (row < nb && col < nb) X[(size_t)(k0 + row) * n + k0 + col] = -u[r];
      }
    }
  }
  __syncthreads();
#if DKG_CHOL_TIMING
  if (tid == 0) printf("chol kb %d factor %llu inverse %llu\n", kb, t1 - t0, __builtin_amdgcn_s_memtime() - t1);
#endif
  if (bad != 0) {
    if (tid == 0) *info = bad;
    return;
  }
  for (int e = tid; e < nb * nb; e += blockDim.x) {
    const int r = e / nb, c = e % nb;
    A[(size_t)(k0 + r) * n + k0 + c] = sL[r][c];  // zeros above the diagonal
  }
}

// ---------------------------------------------------------------------------
// Blocked right-looking Cholesky, one launch per block column kb (kb = -1: factor the first diagonal
// block), all outputs side by side (blockIdx.y = output).  Workgroup (i, j), i >= j > kb, of launch kb:
//   P = A_ik W_kk^T, Q = A_jk W_kk^T    (the solved panel tiles L_ik, L_jk: MFMA, K = 32)
//   A_ij -= P Q^T                       (MFMA, K = 32)
// The diagonal workgroup (i, i) also stores L_ik^T into A's upper block (kb, i) -- nobody reads the upper
// triangle during the factorisation, so the unsolved A_ik stays readable for the other workgroups of the
// launch -- and (i = kb + 1) factors and inverts the freshly updated diagonal block (factor_diag).  The
// panel solves are thereby spread over the update workgroups (the single-wave panel kernels they replace
// took ~27 us per block column), and one launch per block column remains.  dkg_chol_finalize_kernel moves
// the panels to the lower triangle at the end.
__global__ __launch_bounds__(256) void chol_step_kernel(PrepBatch bt, int kb) {
  __shared__ double sP[LB][LB + 1], sQ[LB][LB + 1], sW[LB][LB + 1];
#if DKG_CHOL_TIMING
  const unsigned long long tk0 = __builtin_amdgcn_s_memtime();
#endif
  const int o = blockIdx.y;
  const int n = bt.n[o];
  double* __restrict__ A = bt.A[o];
  double* __restrict__ X = bt.X[o];
  int* info = bt.info[o];
  if (n <= 0 || *info != 0) return;  // an earlier step failed: nothing more to do
  const int tid = threadIdx.x;
  const int nbk = (n + LB - 1) / LB;
  if (kb < 0) {
    if (blockIdx.x != 0) return;
    const int nb = min(LB, n);
    for (int e = tid; e < LB * LB; e += blockDim.x) {
      const int r = e / LB, c = e % LB;
      sP[r][c] = (r < nb && c < nb) ? A[(size_t)r * n + c] : 0.0;
    }
    __syncthreads();
    factor_diag(A, X, n, 0, info, sP, sQ);
    return;
  }
  const int T = nbk - kb - 1;
  if (T <= 0 || (int)blockIdx.x >= T * (T + 1) / 2) return;
  int ti, tj;
  lower_tile(blockIdx.x, ti, tj);
  const int bi = kb + 1 + ti, bj = kb + 1 + tj;
  const int k0 = kb * LB, i0 = bi * LB, j0 = bj * LB;
  const int lane = tid & 63, wave = tid >> 6;
  const int si = wave >> 1, sj = wave & 1;  // this wave's 16 x 16 sub-tile
  // every global operand of the workgroup in flight at once, before the first barrier: the panels' A_ik /
  // A_jk entries this lane feeds its MFMAs, the A_ij entries it updates, and W_kk into LDS
  double pa[LB / 4], qa[LB / 4], aij[4];
  {
    const int ra = i0 + 16 * si + (lane & 15), rb = j0 + 16 * si + (lane & 15);
#pragma unroll
    for (int q = 0; q < LB / 4; ++q) {
      const int kk = 4 * q + (lane >> 4);
      pa[q] = (ra < n && k0 + kk < n) ? A[(size_t)ra * n + k0 + kk] : 0.0;
      qa[q] = (bi != bj && rb < n && k0 + kk < n) ? A[(size_t)rb * n + k0 + kk] : 0.0;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * si + (lane >> 4) + 4 * r, col = 16 * sj + (lane & 15);
      aij[r] = (i0 + row < n && j0 + col < n) ? A[(size_t)(i0 + row) * n + j0 + col] : 0.0;
    }
  }
  for (int e = tid; e < LB * LB; e += blockDim.x) {
    const int r = e / LB, c = e % LB;
    sW[r][c] = (k0 + r < n && k0 + c < n) ? X[(size_t)(k0 + r) * n + k0 + c] : 0.0;
  }
  __syncthreads();
  // solved panel tile: dst[r][c] = sum_q A[r0 + r][k0 + q] W[c][q]
  auto panel = [&](const double (&av)[LB / 4], double (*dst)[LB + 1]) {
    d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < LB / 4; ++q) {
      const int kk = 4 * q + (lane >> 4);
      acc = mfma_f64(av[q], sW[16 * sj + (lane & 15)][kk], acc);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) dst[16 * si + (lane >> 4) + 4 * r][16 * sj + (lane & 15)] = acc[r];
  };
  panel(pa, sP);
  if (bi != bj) panel(qa, sQ);
  __syncthreads();
  double(*Q)[LB + 1] = (bi == bj) ? sP : sQ;
  d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int q = 0; q < LB / 4; ++q) {
    const int kk = 4 * q + (lane >> 4);
    acc = mfma_f64(sP[16 * si + (lane & 15)][kk], Q[16 * sj + (lane & 15)][kk], acc);
  }
  const bool diag_next = (bi == bj) && (bi == kb + 1);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = 16 * si + (lane >> 4) + 4 * r, col = 16 * sj + (lane & 15);
    const bool in = i0 + row < n && j0 + col < n;
    const double v = in ? aij[r] - acc[r] : 0.0;
    if (diag_next) sW[row][col] = v;  // sW is free (read before the barrier above)
    else if (in) A[(size_t)(i0 + row) * n + j0 + col] = v;
  }
  if (bi == bj) {
    // L_ik^T into the upper block (kb, bi): row k0 + c, column i0 + r (r fastest: coalesced)
    for (int e = tid; e < LB * LB; e += blockDim.x) {
      const int c = e / LB, r = e % LB;
      if (i0 + r < n && k0 + c < n) A[(size_t)(k0 + c) * n + i0 + r] = sP[r][c];
    }
  }
  if (diag_next) {
    __syncthreads();
#if DKG_CHOL_TIMING
    if (tid == 0) printf("chol kb %d update %llu\n", kb, __builtin_amdgcn_s_memtime() - tk0);
#endif
    factor_diag(A, X, n, bi, info, sW, sQ);
  }
}

// After the factorisation: every panel block L_ik (i > k), held transposed in A's upper block (k, i),
// moves to the lower block (i, k), and the upper block is zeroed.  Grid (strictly lower tiles, outputs).
__global__ __launch_bounds__(256) void chol_finalize_kernel(PrepBatch bt) {
  __shared__ double sT[LB][LB + 1];
  const int o = blockIdx.y;
  const int n = bt.n[o];
  double* __restrict__ A = bt.A[o];
  if (n <= 0 || *bt.info[o] != 0) return;
  const int nbk = (n + LB - 1) / LB;
  if ((int)blockIdx.x >= nbk * (nbk - 1) / 2) return;
  int ti, tj;
  lower_tile(blockIdx.x, ti, tj);  // ti >= tj over nbk - 1 rows: the strictly lower tile (ti + 1, tj)
  const int i0 = (ti + 1) * LB, k0 = tj * LB;
  const int tid = threadIdx.x;
  for (int e = tid; e < LB * LB; e += blockDim.x) {
    const int r = e / LB, c = e % LB;  // upper block row k0 + r, column i0 + c
    sT[r][c] = (k0 + r < n && i0 + c < n) ? A[(size_t)(k0 + r) * n + i0 + c] : 0.0;
  }
  __syncthreads();
  for (int e = tid; e < LB * LB; e += blockDim.x) {
    const int r = e / LB, c = e % LB;
    if (i0 + r < n && k0 + c < n) {
      A[(size_t)(i0 + r) * n + k0 + c] = sT[c][r];
      A[(size_t)(k0 + c) * n + i0 + r] = 0.0;
    }
  }
}

// ---------------------------------------------------------------------------
// X = L^{-1} by independent column tiles (16 columns per workgroup; the diagonal blocks X_jj = W_jj are
// already in place from the factorisation): walking down the block rows of the tile,
//   X_i = -W_ii sum_{k = j}^{i-1} L_ik X_k
// (L_ik from the finalised lower triangle; the tile's earlier X_k kept in LDS).  Four waves: wave w takes
// row half w & 1 and the k blocks of parity w >> 1 (the two parities meet in LDS in a fixed order), then
// two waves apply -W_ii.  The rows above the diagonal block are zeroed.  Grid (n_pad / 16, outputs),
// dynamic LDS (blocks + 3) * 32 * 16 doubles.
__global__ __launch_bounds__(256) void trinv_col_kernel(PrepBatch bt) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int o = blockIdx.y;
  const int n = bt.n[o];
  const double* __restrict__ L = bt.A[o];
  double* __restrict__ X = bt.X[o];
  if (n <= 0 || *bt.info[o] != 0) return;
  const int c0 = 16 * blockIdx.x;
  if (c0 >= n) return;
  const int nbk = (n + LB - 1) / LB;
  const int bj = c0 / LB;
  const int nblk = nbk - bj;
  double* sX = sm;                               // [nblk][LB][16]
  double* sY = sX + (size_t)nblk * LB * 16;      // [LB][16]
  double* red = sY + LB * 16;                    // [LB][16]
  const int tid = threadIdx.x;
  for (int e = tid; e < bj * LB * 16; e += blockDim.x) {
    const int r = e / 16, c = e % 16;
    if (c0 + c < n) X[(size_t)r * n + c0 + c] = 0.0;
  }
  for (int e = tid; e < LB * 16; e += blockDim.x) {
    const int r = e / 16, c = e % 16;
    sX[e] = (bj * LB + r < n && c0 + c < n) ? X[(size_t)(bj * LB + r) * n + c0 + c] : 0.0;
  }
  __syncthreads();
  const int lane = tid & 63, wave = tid >> 6;
  const int si = wave & 1, kp = wave >> 1;
  for (int bi = bj + 1; bi < nbk; ++bi) {
    const int i0 = bi * LB;
    d4 acc = {0.0, 0.0, 0.0, 0.0};
    const int ra = i0 + 16 * si + (lane & 15);
    for (int bk = bj + kp; bk < bi; bk += 2) {
      const double* sxk = sX + (size_t)(bk - bj) * LB * 16;
#pragma unroll
      for (int q = 0; q < LB / 4; ++q) {
        const int kk = 4 * q + (lane >> 4);
        const double a = (ra < n && bk * LB + kk < n) ? L[(size_t)ra * n + bk * LB + kk] : 0.0;
        acc = mfma_f64(a, sxk[kk * 16 + (lane & 15)], acc);
      }
    }
    if (kp == 1) {
#pragma unroll
      for (int r = 0; r < 4; ++r) red[(16 * si + (lane >> 4) + 4 * r) * 16 + (lane & 15)] = acc[r];
    }
    __syncthreads();
    if (kp == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int idx = (16 * si + (lane >> 4) + 4 * r) * 16 + (lane & 15);
        sY[idx] = acc[r] + red[idx];
      }
    }
    __syncthreads();
    if (wave < 2) {
      d4 acc2 = {0.0, 0.0, 0.0, 0.0};
      const int rw = 16 * si + (lane & 15);  // row of W_ii
#pragma unroll
      for (int q = 0; q < LB / 4; ++q) {
        const int kk = 4 * q + (lane >> 4);
        const double a = (i0 + rw < n && i0 + kk < n) ? X[(size_t)(i0 + rw) * n + i0 + kk] : 0.0;
        acc2 = mfma_f64(a, sY[kk * 16 + (lane & 15)], acc2);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * si + (lane >> 4) + 4 * r, col = lane & 15;
        const double v = -acc2[r];
        sX[(size_t)(bi - bj) * LB * 16 + row * 16 + col] = v;
        if (i0 + row < n && c0 + col < n) X[(size_t)(i0 + row) * n + c0 + col] = v;
      }
    }
    __syncthreads();
  }
}

// alpha = X^T (X r) with r = y - c (X = L^{-1}); one workgroup, t in LDS.
// Also writes the zero padding alpha[n .. n_pad).
__global__ __launch_bounds__(1024) void alpha_kernel(const double* __restrict__ X, const double* __restrict__ y,
                                                     double c, int n, double* __restrict__ alpha,
                                                     const int* __restrict__ info) {
  __shared__ double t[1024];
  __shared__ double r[1024];
  if (*info != 0) return;
  for (int i = threadIdx.x; i < n; i += blockDim.x) r[i] = y[i] - c;
  __syncthreads();
  // t = X r, one row per wave (lanes along the row: coalesced reads), lane partial sums in q order
  // then a fixed-order wave reduction
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int i = wave; i < n; i += nw) {
    double s = 0.0;
    for (int q = lane; q <= i; q += 64) s = fma(X[(size_t)i * n + q], r[q], s);
    s = wave_sum(s);
    if (lane == 0) t[i] = s;
  }
  __syncthreads();
  // alpha = X^T t by groups of 64 columns: wave w sums the rows i = w (mod 16) of its lane's column (its
  // loads independent of each other, all in flight), then the 16 wave partials meet in LDS in wave order
  __shared__ double part[16][64];
  for (int g0 = 0; g0 < pad16(n); g0 += 64) {
    const int q = g0 + lane;
    double s = 0.0;
    if (q < n) {
      const int i1 = q + ((wave - q) % nw + nw) % nw;  // first row >= q with i = wave (mod nw)
      for (int i = i1; i < n; i += nw) s = fma(X[(size_t)i * n + q], t[i], s);  // coalesced across lanes
    }
    part[wave][lane] = s;
    __syncthreads();
    if (wave == 0 && q < pad16(n)) {
      double a = 0.0;
      for (int w2 = 0; w2 < nw; ++w2) a += part[w2][lane];
      alpha[q] = a;
    }
    __syncthreads();
  }
}

// root_frag from X = L^{-1} = R^T: P = R^T, element (row 16 tj + (l & 15),
// column 4 kb + (l >> 4)) of P is X[16 tj + (l & 15)][4 kb + (l >> 4)].
__global__ void pack_linv_kernel(const double* __restrict__ X, int n, double* __restrict__ rf) {
  const int np = pad16(n);
  const int KB = np / 4;
  const size_t total = (size_t)np * np;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    const int l = (int)(e & 63);
    const size_t blk = e >> 6;
    const int kb = (int)(blk % KB);
    const int tj = (int)(blk / KB);
    const int row = 16 * tj + (l & 15);
    const int col = 4 * kb + (l >> 4);
    rf[frag_index(tj, kb, l, KB)] = (row < n && col < n) ? X[(size_t)row * n + col] : 0.0;
  }
}

static int grid_for(size_t total) { return (int)std::min<size_t>((total + 255) / 256, 4096); }

// Blocked Cholesky of every output (A lower: L; X diagonal blocks: W_kk = L_kk^{-1}): one launch for the
// first diagonal block, one per further block column, then the panels moved to the lower triangle.
hipError_t launch_cholesky_batch(const PrepBatch& b, int m, hipStream_t s) {
  int nmax = 0;
  for (int i = 0; i < m; ++i) nmax = std::max(nmax, b.n[i]);
  const int nbk = (nmax + LB - 1) / LB;
  hipLaunchKernelGGL(chol_step_kernel, dim3(1, m), dim3(256), 0, s, b, -1);
  for (int kb = 0; kb + 1 < nbk; ++kb) {
    const int T = nbk - kb - 1;
    hipLaunchKernelGGL(chol_step_kernel, dim3(T * (T + 1) / 2, m), dim3(256), 0, s, b, kb);
  }
  if (nbk > 1) hipLaunchKernelGGL(chol_finalize_kernel, dim3(nbk * (nbk - 1) / 2, m), dim3(256), 0, s, b);
  return hipGetLastError();
}

hipError_t launch_cholesky(double* A, double* X, int n, int* info, hipStream_t s) {
  PrepBatch b{};
  b.A[0] = A;
  b.X[0] = X;
  b.n[0] = n;
  b.info[0] = info;
  return launch_cholesky_batch(b, 1, s);
}

// X = L^{-1} of every output, after launch_cholesky_batch (one launch: independent 16-column tiles).
hipError_t launch_tri_inverse_batch(const PrepBatch& b, int m, hipStream_t s) {
  int nmax = 0;
  for (int i = 0; i < m; ++i) nmax = std::max(nmax, b.n[i]);
  const int nbk = (nmax + LB - 1) / LB;
  const size_t lds = (size_t)(nbk + 2) * LB * 16 * sizeof(double);
  raise_lds_limit((const void*)trinv_col_kernel, lds);
  hipLaunchKernelGGL(trinv_col_kernel, dim3((nmax + 15) / 16, m), dim3(256), lds, s, b);
  return hipGetLastError();
}

hipError_t launch_tri_inverse(double* L, double* X, int n, const int* info, hipStream_t s) {
  PrepBatch b{};
  b.A[0] = L;
  b.X[0] = X;
  b.n[0] = n;
  b.info[0] = const_cast<int*>(info);
  return launch_tri_inverse_batch(b, 1, s);
}

hipError_t launch_alpha(const double* X, const double* y, double c, int n, double* alpha, const int* info,
                        hipStream_t s) {
  hipLaunchKernelGGL(alpha_kernel, dim3(1), dim3(1024), 0, s, X, y, c, n, alpha, info);
  return hipGetLastError();
}

hipError_t launch_pack_linv(const double* X, int n, double* rf, hipStream_t s) {
  hipLaunchKernelGGL(pack_linv_kernel, dim3(grid_for((size_t)pad16(n) * pad16(n))), dim3(256), 0, s, X, n, rf);
  return hipGetLastError();
}

}  // namespace dkg
