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
__device__ __forceinline__ void chol_panel_body(double* __restrict__ A, int n, int k0, int* __restrict__ info) {
  __shared__ double Lk[LB][LB + 1];
  __shared__ int bad;
  if (*info != 0) return;  // an earlier panel failed: nothing more to do
  const int nb = min(LB, n - k0);
  const int tid = threadIdx.x;
  if (tid < 64) {
    // the diagonal block on one wave, in registers: lane r holds row r (zero rows past nb); column j's
    // pivot and entries reach the other lanes by v_readlane, so the 32 steps need no LDS round trip
    // and no barrier (the LDS version spent ~0.7 us per step on three barriers)
    const int lane = tid;
    double a[LB];
#pragma unroll
    for (int c = 0; c < LB; ++c) a[c] = (lane < nb && c <= lane) ? A[(size_t)(k0 + lane) * n + k0 + c] : 0.0;
    int fail = 0;
#pragma unroll
    for (int j = 0; j < LB; ++j) {
      if (j < nb && fail == 0) {  // uniform
        const double piv = readlane_f64(a[j], j);
        if (!(piv > 0.0) || !isfinite(piv)) {  // NaN fails too
          fail = k0 + j + 1;
        } else {
          const double dj = sqrt(piv);
          a[j] = (lane == j) ? dj : ((lane > j) ? a[j] / dj : a[j]);
#pragma unroll
          for (int c = j + 1; c < LB; ++c) {
            if (c < nb) {
              const double lcj = readlane_f64(a[j], c);  // L[c][j]
              a[c] = (lane >= c) ? fma(-a[j], lcj, a[c]) : a[c];
            }
          }
        }
      }
    }
    if (lane < LB) {
#pragma unroll
      for (int c = 0; c < LB; ++c) Lk[lane][c] = a[c];
    }
    if (lane == 0) bad = fail;
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
      // no LDS read of a later row is hoisted above this one: the unrolled solve would otherwise keep
      // all 528 Lk values live at once (256 VGPRs and ~700 bytes of scratch per lane)
      asm volatile("" ::: "memory");
    }
#pragma unroll
    for (int c = 0; c < LB; ++c)
      if (c < nb) row[c] = x[c];
  }
}

__global__ __launch_bounds__(256) void chol_panel_kernel(double* __restrict__ A, int n, int k0, int* __restrict__ info) {
  chol_panel_body(A, n, k0, info);
}

// All outputs' panels at block column k0 in one launch (blockIdx.y = output; outputs with n <= k0 are done).
__global__ __launch_bounds__(256) void chol_panel_batch_kernel(PrepBatch b, int k0) {
  const int i = blockIdx.y;
  if (k0 < b.n[i]) chol_panel_body(b.A[i], b.n[i], k0, b.info[i]);
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
__device__ __forceinline__ void chol_update_body(double* __restrict__ A, int n, int k0, const int* __restrict__ info,
                                                 int t) {
  if (*info != 0) return;
  const int base = k0 + LB;
  // t enumerates lower tiles (ti, tj), tj <= ti, row-major over ti
  int ti = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
  while ((ti + 1) * (ti + 2) / 2 <= t) ++ti;
  while (ti * (ti + 1) / 2 > t) --ti;
  const int tj = t - ti * (ti + 1) / 2;
  const int ci = base + LB * ti, cj = base + LB * tj;
  tile_update(A, A, A, n, ci, cj, ci, cj, k0, min(LB, n - k0));
}

__global__ __launch_bounds__(256) void chol_update_kernel(double* __restrict__ A, int n, int k0,
                                                          const int* __restrict__ info) {
  chol_update_body(A, n, k0, info, blockIdx.x);
}

__global__ __launch_bounds__(256) void chol_update_batch_kernel(PrepBatch b, int k0) {
  const int i = blockIdx.y;
  const int T = (b.n[i] - k0 - LB + LB - 1) / LB;  // trailing tiles per side of output i
  if (T > 0 && (int)blockIdx.x < T * (T + 1) / 2) chol_update_body(b.A[i], b.n[i], k0, b.info[i], blockIdx.x);
}

// ---------------------------------------------------------------------------
// Triangular inverse X = L^{-1} (lower), right-looking by block rows of the
// right-hand side I: at step k0 the block row X_k = Lkk^{-1} B_k (B_k holds
// I_k minus the updates so far, columns < k0 + nb), then
// B_i -= L_ik X_k for every later block row i.  X overwrites B in `X`.
__device__ __forceinline__ void trinv_panel_body(const double* __restrict__ L, double* __restrict__ X, int n, int k0,
                                                 const int* __restrict__ info) {
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
      asm volatile("" ::: "memory");  // as in chol_panel_kernel: one row of Lk live at a time
    }
#pragma unroll
    for (int r = 0; r < LB; ++r)
      if (r < nb) X[(size_t)(k0 + r) * n + c] = x[r];
  }
}

__global__ __launch_bounds__(256) void trinv_panel_kernel(const double* __restrict__ L, double* __restrict__ X, int n,
                                                          int k0, const int* __restrict__ info) {
  trinv_panel_body(L, X, n, k0, info);
}

__global__ __launch_bounds__(256) void trinv_panel_batch_kernel(PrepBatch b, int k0) {
  const int i = blockIdx.y;
  if (k0 < b.n[i]) trinv_panel_body(b.A[i], b.X[i], b.n[i], k0, b.info[i]);
}

// B_i[:, 0 : k0 + nb) -= L[i-block, k-block] X_k for block rows i > k; grid
// (column tiles of the first k0 + nb columns, later block rows).
__device__ __forceinline__ void trinv_update_body(const double* __restrict__ L, double* __restrict__ X, int n, int k0,
                                                  const int* __restrict__ info, int bx, int by) {
  if (*info != 0) return;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int si = wave >> 1, sj = wave & 1;
  const int nb = min(LB, n - k0);
  const int ci = k0 + LB * (1 + by);  // output rows
  const int cj = LB * bx;             // output columns
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

__global__ __launch_bounds__(256) void trinv_update_kernel(const double* __restrict__ L, double* __restrict__ X, int n,
                                                           int k0, const int* __restrict__ info) {
  trinv_update_body(L, X, n, k0, info, blockIdx.x, blockIdx.y);
}

__global__ __launch_bounds__(256) void trinv_update_batch_kernel(PrepBatch b, int k0) {
  const int i = blockIdx.z;
  const int n = b.n[i];
  if (k0 >= n) return;
  const int rows = (n - k0 - LB + LB - 1) / LB, cols = (k0 + LB + LB - 1) / LB;
  if ((int)blockIdx.x < cols && (int)blockIdx.y < rows) trinv_update_body(b.A[i], b.X[i], n, k0, b.info[i], blockIdx.x, blockIdx.y);
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
  // alpha = X^T t, one column q per thread summed over i in ascending order; unrolled so that eight
  // rows' loads are in flight at once (they do not depend on the running sum)
  for (int q = threadIdx.x; q < pad16(n); q += blockDim.x) {
    double s = 0.0;
    if (q < n) {
#pragma unroll 8
      for (int i = q; i < n; ++i) s = fma(X[(size_t)i * n + q], t[i], s);  // coalesced across q
    }
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

hipError_t launch_cholesky_batch(const PrepBatch& b, int m, hipStream_t s) {
  int nmax = 0;
  for (int i = 0; i < m; ++i) nmax = std::max(nmax, b.n[i]);
  for (int k0 = 0; k0 < nmax; k0 += LB) {
    hipLaunchKernelGGL(chol_panel_batch_kernel, dim3(1, m), dim3(256), 0, s, b, k0);
    const int T = (nmax - k0 - LB + LB - 1) / LB;
    if (T > 0) hipLaunchKernelGGL(chol_update_batch_kernel, dim3(T * (T + 1) / 2, m), dim3(256), 0, s, b, k0);
  }
  return hipGetLastError();
}

hipError_t launch_tri_inverse_batch(const PrepBatch& b, int m, hipStream_t s) {
  int nmax = 0;
  for (int i = 0; i < m; ++i) {
    nmax = std::max(nmax, b.n[i]);
    hipLaunchKernelGGL(trinv_init_kernel, dim3(grid_for((size_t)b.n[i] * b.n[i])), dim3(256), 0, s, b.A[i], b.X[i],
                       b.n[i]);
  }
  for (int k0 = 0; k0 < nmax; k0 += LB) {
    hipLaunchKernelGGL(trinv_panel_batch_kernel, dim3(1, m), dim3(256), 0, s, b, k0);
    const int rows = (nmax - k0 - LB + LB - 1) / LB;
    const int cols = (k0 + LB + LB - 1) / LB;
    if (rows > 0) hipLaunchKernelGGL(trinv_update_batch_kernel, dim3(cols, rows, m), dim3(256), 0, s, b, k0);
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
