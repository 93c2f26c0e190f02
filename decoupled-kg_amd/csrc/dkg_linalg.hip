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

// ---------------------------------------------------------------------------
// Cholesky panel at block column k0: factor A[k0:k0+nb, k0:k0+nb] in LDS and
// solve the rows below it, A[i, k0:k0+nb] <- A[i, k0:k0+nb] Lkk^{-T}.
// info (device): 0 = fine; j + 1 = the pivot of column j is not positive/finite
// (LAPACK potrf convention, what cholesky_ex reports).
__global__ __launch_bounds__(256) void chol_panel_kernel(double* __restrict__ A, int n, int k0, int* __restrict__ info) {
  __shared__ double Lk[LB][LB + 1];
  __shared__ int bad;
  if (*info != 0) return;  // an earlier panel failed: nothing more to do
  const int nb = min(LB, n - k0);
  const int tid = threadIdx.x;
  if (tid == 0) bad = 0;
  for (int e = tid; e < LB * LB; e += blockDim.x) {
    const int r = e / LB, c = e % LB;
    Lk[r][c] = (r < nb && c <= r) ? A[(size_t)(k0 + r) * n + k0 + c] : 0.0;
  }
  __syncthreads();
  // unblocked right-looking on the diagonal block
  for (int j = 0; j < nb; ++j) {
    const double piv = Lk[j][j];
    __syncthreads();
    if (!(piv > 0.0) || !isfinite(piv)) {  // NaN fails too
      if (tid == 0 && bad == 0) bad = k0 + j + 1;
      break;
    }
    const double dj = sqrt(piv);
    for (int r = j + 1 + tid; r < nb; r += blockDim.x) Lk[r][j] /= dj;
    if (tid == 0) Lk[j][j] = dj;
    __syncthreads();
    const int m = nb - j - 1;
    for (int e = tid; e < m * m; e += blockDim.x) {
      const int r = j + 1 + e / m, c = j + 1 + e % m;
      if (c <= r) Lk[r][c] -= Lk[r][j] * Lk[c][j];
    }
    __syncthreads();
  }
  __syncthreads();
  if (bad != 0) {
    if (tid == 0) *info = bad;
    return;
  }
  for (int e = tid; e < nb * nb; e += blockDim.x) {
    const int r = e / nb, c = e % nb;
    if (c <= r) A[(size_t)(k0 + r) * n + k0 + c] = Lk[r][c];
  }
  // rows below: x Lkk^T = a  (forward substitution over the nb columns)
  for (int i = k0 + nb + tid; i < n; i += blockDim.x) {
    double x[LB];
    double* row = A + (size_t)i * n + k0;
#pragma unroll
    for (int c = 0; c < LB; ++c) x[c] = (c < nb) ? row[c] : 0.0;
#pragma unroll
    for (int c = 0; c < LB; ++c) {
      if (c < nb) {
        double s = x[c];
#pragma unroll
        for (int q = 0; q < c; ++q) s -= x[q] * Lk[c][q];
        x[c] = s / Lk[c][c];
      }
    }
#pragma unroll
    for (int c = 0; c < LB; ++c)
      if (c < nb) row[c] = x[c];
  }
}

// 32 x 32 tile update C -= P Q^T with P = A[pi.., kc..kc+32), Q = A[qi.., kc..kc+32)
// (row-major, leading dimension n), rows beyond n skipped.  Four waves, one
// 16 x 16 sub-tile each, eight MFMAs (K = 32).
__device__ __forceinline__ void tile_update(double* __restrict__ A, const double* __restrict__ Pm,
                                            const double* __restrict__ Qm, int n, int ci, int cj, int pi, int qi,
                                            int kc, int kn) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int si = wave >> 1, sj = wave & 1;  // sub-tile
  const int ra = pi + 16 * si + (lane & 15);  // A operand row (P)
  const int rb = qi + 16 * sj + (lane & 15);  // B operand column (row of Q)
  d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int kb = 0; kb < LB / 4; ++kb) {
    const int kk = 4 * kb + (lane >> 4);
    const double a = (ra < n && kk < kn) ? Pm[(size_t)ra * n + kc + kk] : 0.0;
    const double b = (rb < n && kk < kn) ? Qm[(size_t)rb * n + kc + kk] : 0.0;
    acc = mfma_f64(a, b, acc);
  }
  // D lane map: row (l >> 4) + 4 r, column l & 15
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = ci + 16 * si + (lane >> 4) + 4 * r;
    const int col = cj + 16 * sj + (lane & 15);
    if (row < n && col < n) A[(size_t)row * n + col] -= acc[r];
  }
}

// Trailing update after panel k0: A[i][j] -= sum_c L[i][c] L[j][c] over the
// panel's columns, for the lower tiles (ti >= tj) of the trailing matrix.
__global__ __launch_bounds__(256) void chol_update_kernel(double* __restrict__ A, int n, int k0,
                                                          const int* __restrict__ info) {
  if (*info != 0) return;
  const int base = k0 + LB;
  // blockIdx.x enumerates lower tiles (ti, tj), tj <= ti, row-major over ti
  const int t = blockIdx.x;
  int ti = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
  while ((ti + 1) * (ti + 2) / 2 <= t) ++ti;
  while (ti * (ti + 1) / 2 > t) --ti;
  const int tj = t - ti * (ti + 1) / 2;
  const int ci = base + LB * ti, cj = base + LB * tj;
  tile_update(A, A, A, n, ci, cj, ci, cj, k0, min(LB, n - k0));
}

// ---------------------------------------------------------------------------
// Triangular inverse X = L^{-1} (lower), right-looking by block rows of the
// right-hand side I: at step k0 the block row X_k = Lkk^{-1} B_k (B_k holds
// I_k minus the updates so far, columns < k0 + nb), then
// B_i -= L_ik X_k for every later block row i.  X overwrites B in `X`.
__global__ __launch_bounds__(256) void trinv_panel_kernel(const double* __restrict__ L, double* __restrict__ X, int n,
                                                          int k0, const int* __restrict__ info) {
  __shared__ double Lk[LB][LB + 1];
  if (*info != 0) return;
  const int nb = min(LB, n - k0);
  const int tid = threadIdx.x;
  for (int e = tid; e < LB * LB; e += blockDim.x) {
    const int r = e / LB, c = e % LB;
    Lk[r][c] = (r < nb && c <= r) ? L[(size_t)(k0 + r) * n + k0 + c] : 0.0;
  }
  __syncthreads();
  // columns 0 .. k0 + nb - 1 of block row k: Lkk x = b (forward substitution)
  for (int c = tid; c < k0 + nb; c += blockDim.x) {
    double x[LB];
#pragma unroll
    for (int r = 0; r < LB; ++r) x[r] = (r < nb) ? X[(size_t)(k0 + r) * n + c] : 0.0;
#pragma unroll
    for (int r = 0; r < LB; ++r) {
      if (r < nb) {
        double s = x[r];
#pragma unroll
        for (int q = 0; q < r; ++q) s -= Lk[r][q] * x[q];
        x[r] = s / Lk[r][r];
      }
    }
#pragma unroll
    for (int r = 0; r < LB; ++r)
      if (r < nb) X[(size_t)(k0 + r) * n + c] = x[r];
  }
}

// B_i[:, 0 : k0 + nb) -= L[i-block, k-block] X_k for block rows i > k; grid
// (column tiles of the first k0 + nb columns, later block rows).
__global__ __launch_bounds__(256) void trinv_update_kernel(const double* __restrict__ L, double* __restrict__ X, int n,
                                                           int k0, const int* __restrict__ info) {
  if (*info != 0) return;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int si = wave >> 1, sj = wave & 1;
  const int nb = min(LB, n - k0);
  const int ci = k0 + LB * (1 + blockIdx.y);  // output rows
  const int cj = LB * blockIdx.x;             // output columns
  const int ra = ci + 16 * si + (lane & 15);  // row of L (A operand)
  const int cb = cj + 16 * sj + (lane & 15);  // column of X_k (B operand)
  d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int kb = 0; kb < LB / 4; ++kb) {
    const int kk = 4 * kb + (lane >> 4);
    const double a = (ra < n && kk < nb) ? L[(size_t)ra * n + k0 + kk] : 0.0;
    const double b = (cb < n && kk < nb) ? X[(size_t)(k0 + kk) * n + cb] : 0.0;
    acc = mfma_f64(a, b, acc);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = ci + 16 * si + (lane >> 4) + 4 * r;
    const int col = cj + 16 * sj + (lane & 15);
    if (row < n && col < k0 + nb) X[(size_t)row * n + col] -= acc[r];
  }
}

// X = I (row-major n x n) and the upper triangle of L zeroed.
__global__ void trinv_init_kernel(double* __restrict__ L, double* __restrict__ X, int n) {
  const size_t total = (size_t)n * n;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    const int r = (int)(e / n), c = (int)(e % n);
    X[e] = (r == c) ? 1.0 : 0.0;
    if (c > r) L[e] = 0.0;
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
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    double s = 0.0;
    for (int q = 0; q <= i; ++q) s = fma(X[(size_t)i * n + q], r[q], s);
    t[i] = s;
  }
  __syncthreads();
  for (int q = threadIdx.x; q < pad16(n); q += blockDim.x) {
    double s = 0.0;
    if (q < n)
      for (int i = q; i < n; ++i) s = fma(X[(size_t)i * n + q], t[i], s);  // coalesced across q
    alpha[q] = s;
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

hipError_t launch_cholesky(double* A, int n, int* info, hipStream_t s) {
  for (int k0 = 0; k0 < n; k0 += LB) {
    hipLaunchKernelGGL(chol_panel_kernel, dim3(1), dim3(256), 0, s, A, n, k0, info);
    const int T = (n - k0 - LB + LB - 1) / LB;  // trailing tiles per side
    if (T > 0) hipLaunchKernelGGL(chol_update_kernel, dim3(T * (T + 1) / 2), dim3(256), 0, s, A, n, k0, info);
  }
  return hipGetLastError();
}

hipError_t launch_tri_inverse(double* L, double* X, int n, const int* info, hipStream_t s) {
  hipLaunchKernelGGL(trinv_init_kernel, dim3(grid_for((size_t)n * n)), dim3(256), 0, s, L, X, n);
  for (int k0 = 0; k0 < n; k0 += LB) {
    hipLaunchKernelGGL(trinv_panel_kernel, dim3(1), dim3(256), 0, s, L, X, n, k0, info);
    const int rows = (n - k0 - LB + LB - 1) / LB;
    const int cols = (k0 + LB + LB - 1) / LB;
    if (rows > 0) hipLaunchKernelGGL(trinv_update_kernel, dim3(cols, rows), dim3(256), 0, s, L, X, n, k0, info);
  }
  return hipGetLastError();
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
