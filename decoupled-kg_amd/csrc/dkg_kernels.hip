// HIP kernels of the Discrete-KG hot path for gfx950 (MI355X, CDNA4).
//
// Pipeline per forward (DESIGN.md "Kernels"):
//   cross_root_kernel   Q = K(x, X) R  (fp64 MFMA, R upper triangular), mean = c + K(x,X) alpha
//   posterior_cov_kernel cov[b][k] = s k(x_b, D_k) - Q_b . Q_D[k]   (fp64 MFMA GEMM, split-K)
//   envelope_kernel     lines a_k + b_k z per (candidate, scalarisation), upper
//                       envelope, closed-form Gaussian expectation, mean over S
#include "dkg_fused.h"
#include <cstdlib>

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

// out[r][c] (row-major, n_pad columns) = element (r, c) of a fragment-packed
// (rows x n) matrix; one thread per output element, coalesced stores.
__global__ void unpack_rows_kernel(const double* __restrict__ frag, int rows, int np, double* __restrict__ out) {
  const int KB = np / 4;
  const size_t total = (size_t)rows * np;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    const int r = (int)(e / np), c = (int)(e % np);
    out[e] = frag[frag_index(r >> 4, c >> 2, ((c & 3) << 4) | (r & 15), KB)];
  }
}

// fp32 quad-packed copy of a pair-packed fp64 fragment matrix (rows_pad x np):
// one thread per fp32 element, coalesced stores (DKG_PLAN_F32 plan init).
__global__ void frag_to_f32_kernel(const double* __restrict__ frag, int rows_pad, int np, float* __restrict__ out) {
  const int KB = np / 4;
  const size_t total = (size_t)rows_pad * np;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    const int r = (int)(e & 3);
    const size_t rest = e >> 2;
    const int l = (int)(rest & 63);
    const size_t blk = rest >> 6;
    const int kb = 4 * (int)(blk % (KB / 4)) + r;
    const int t = (int)(blk / (KB / 4));
    out[e] = (float)frag[frag_index(t, kb, l, KB)];
  }
}


// Plan init (staged forward): every scalarisation's intercepts a_k, k >= 1, with the envelope's own
// arithmetic (pair_coefs' a_off and w_i sd_i, build_lines' record dot in output order: the same bits as the
// lines the envelope used to build), NaN in slot 0 and past N; then their maximum over k >= 1 and the first
// k attaining it with the number of lines that do.  One workgroup per scalarisation.
struct IcptArgs {
  const double* mu_all;
  const double* weights;
  double* icpt;
  double* itop;
  int* itopk;
  int m, N, stride;
  double ysd[DKG_MAX_OUTPUTS], ymu[DKG_MAX_OUTPUTS];
};

template <int M>
__global__ __launch_bounds__(256) void intercepts_kernel(IcptArgs a) {
  __shared__ double smax[256];
  __shared__ int sfirst[256], scount[256];
  constexpr int MP = cov_rec(M);
  const int j = blockIdx.x, m = a.m;
  double w[M], wa[M], a_off = 0.0;
#pragma unroll
  for (int i = 0; i < M; ++i) {
    const bool live = i < m;
    w[i] = live ? a.weights[(size_t)j * m + i] : 0.0;
    wa[i] = w[i] * (live ? a.ysd[i] : 1.0);
    a_off = fma(w[i], live ? a.ymu[i] : 0.0, a_off);
  }
  double* out = a.icpt + (size_t)j * a.stride;
  double mx = -INFINITY;
  for (int k = threadIdx.x; k < a.stride; k += blockDim.x) {
    double v = __builtin_nan("");
    if (k >= 1 && k <= a.N) {
      const double* r = a.mu_all + (size_t)(k - 1) * MP;
      double acc = a_off;
      if constexpr (MP == 1) {
        acc = fma(wa[0], r[0], acc);
      } else {
#pragma unroll
        for (int q = 0; 2 * q < M; ++q) {
          acc = fma(wa[2 * q], r[2 * q], acc);
          if (2 * q + 1 < M) acc = fma(wa[2 * q + 1], r[2 * q + 1], acc);
        }
      }
      v = acc;
      mx = fmax(mx, v);
    }
    out[k] = v;
  }
  smax[threadIdx.x] = mx;
  __syncthreads();
  for (int h = blockDim.x / 2; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) smax[threadIdx.x] = fmax(smax[threadIdx.x], smax[threadIdx.x + h]);
    __syncthreads();
  }
  const double top = smax[0];
  int first = 0x7fffffff, count = 0;
  for (int k = threadIdx.x; k < a.stride; k += blockDim.x) {
    if (k >= 1 && k <= a.N && out[k] == top) {
      first = min(first, k);
      ++count;
    }
  }
  sfirst[threadIdx.x] = first;
  scount[threadIdx.x] = count;
  __syncthreads();
  for (int h = blockDim.x / 2; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) {
      sfirst[threadIdx.x] = min(sfirst[threadIdx.x], sfirst[threadIdx.x + h]);
      scount[threadIdx.x] += scount[threadIdx.x + h];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    a.itop[j] = top;
    a.itopk[2 * j] = scount[0] > 0 ? sfirst[0] : 0;
    a.itopk[2 * j + 1] = scount[0];
  }
}

hipError_t launch_intercepts(const Plan& h, hipStream_t s) {
  IcptArgs a{};
  a.mu_all = h.mu_all;
  a.weights = h.weights;
  a.icpt = h.icpt;
  a.itop = h.itop;
  a.itopk = h.itopk;
  a.m = h.m;
  a.N = h.N;
  a.stride = h.icpt_stride;
  for (int i = 0; i < h.m; ++i) {
    a.ysd[i] = h.o[i].y_std;
    a.ymu[i] = h.o[i].y_mean;
  }
  const dim3 grid(h.S), block(256);
  switch (h.m <= 1 ? 1 : h.m <= 2 ? 2 : h.m <= 3 ? 3 : h.m <= 4 ? 4 : 8) {
    case 1: hipLaunchKernelGGL(intercepts_kernel<1>, grid, block, 0, s, a); break;
    case 2: hipLaunchKernelGGL(intercepts_kernel<2>, grid, block, 0, s, a); break;
    case 3: hipLaunchKernelGGL(intercepts_kernel<3>, grid, block, 0, s, a); break;
    case 4: hipLaunchKernelGGL(intercepts_kernel<4>, grid, block, 0, s, a); break;
    default: hipLaunchKernelGGL(intercepts_kernel<8>, grid, block, 0, s, a); break;
  }
  return hipGetLastError();
}

template <int DM>
__global__ __launch_bounds__(CR_WAVES * WAVE) void cross_root_kernel(CrossArgs a) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  cross_root_impl<DM>(a.o, a.d, a.x, a.rows, a.q, a.mean, blockIdx.x, blockIdx.y, smem);
}

// The KG accumulators (and arrival tickets) the envelope stage adds into and the coincidence marks
// (Plan::dup) the covariance stage sets, cleared for row tile ti's 16 candidates: each tile's first
// workgroup clears its own rows, so a launch over many batches (dkg_plan_forward_batches) spreads the
// clearing instead of one workgroup looping over every candidate.
__device__ inline void clear_tile_accumulators(const Plan* __restrict__ P, double* __restrict__ kg, int B, int ti) {
  const int b0 = ti * 16, b1 = min(B, b0 + 16), ng1 = pair_groups(P->S) + 1;
  for (int i = b0 + (int)threadIdx.x; i < b1; i += blockDim.x) {
    kg[i] = 0.0;
    P->dup[i] = DUP_NONE;
  }
  for (int i = b0 * ng1 + (int)threadIdx.x; i < b1 * ng1; i += blockDim.x) P->tickets[i] = 0;
}

// Forward: grid (B tiles, pairs, outputs); the first workgroup of every row tile also clears that
// tile's accumulators (clear_tile_accumulators).
template <int DM, class T = double>
__global__ __launch_bounds__(CR_WAVES * WAVE) void cross_root_plan_kernel(const Plan* __restrict__ P,
                                                                          const double* __restrict__ xnew, int B,
                                                                          double* __restrict__ kg, int dst,
                                                                          int use_kx) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  unsigned long long* st = kst_slot(dst, P, 0);
  KST_BEGIN(st);
  const int oi = blockIdx.z;
  if (blockIdx.y == 0 && oi == 0) clear_tile_accumulators(P, kg, B, blockIdx.x);
  if (DKG_ABLATIONS && (__builtin_amdgcn_readfirstlane(P->debug_cov) & 2)) return;  // ablation: empty cross stage
  if constexpr (sizeof(T) == 8) {
    cross_root_impl<DM>(P->o[oi], P->d, xnew, B, P->q[oi], P->mux[oi], blockIdx.x, blockIdx.y, smem, st, 0,
                        use_kx ? P->kx[oi] : nullptr);
  } else {
    cross_root_impl<DM, false, float>(P->o[oi], P->d, xnew, B, P->q32[oi], P->mux[oi], blockIdx.x, blockIdx.y, smem,
                                      st, 0, use_kx ? P->kx[oi] : nullptr, nullptr, P->root32[oi]);
  }
}

// K(x, X) for the cross stage of large n (cross_kfill): grid (B tiles, k-block groups of KF_KB, outputs).
template <int DM>
__global__ __launch_bounds__(KF_WAVES * WAVE) void cross_kfill_kernel(const Plan* __restrict__ P,
                                                                     const double* __restrict__ xnew, int B) {
  const int oi = blockIdx.z;
  if (P->kx[oi] == nullptr) return;
  cross_kfill_body<DM>(P->o[oi], P->d, xnew, B, P->kx[oi], blockIdx.x, blockIdx.y * KF_KB, P->kx32[oi]);
}

// The cross stage of a launch with the K(x, X) fill (cross_kfill_launch) in one launch: the 64 x 32 blocks of
// Q_X (cross_big_body, the longest first), then RT x m workgroups for the means K(x, X) alpha + c and the
// accumulator clears.  The means follow cross_root_impl's arithmetic element for element -- its fill loop's
// per-thread fma order over the 512 threads of a row tile (thread t here runs the chains of threads t, t + 64 W,
// ... for W waves), the lane-group adds, the 8 waves in order -- so they have the bits of the one-kernel cross
// stage.
__device__ __forceinline__ void cross_means_body(const Plan* __restrict__ P, int B, double* __restrict__ kg, int L);

__global__ __launch_bounds__(XB_WAVES * WAVE) __attribute__((amdgpu_waves_per_eu(2))) void cross_big_kernel(
    const Plan* __restrict__ P, int B, double* __restrict__ kg) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int nbig = cross_big_blocks(P->max_np, B, P->m);
  if ((int)blockIdx.x < nbig) {
    if (DKG_ABLATIONS && (P->debug_cov & 16)) return;  // probe: the means alone
    cross_big_body(P, B, blockIdx.x, smem);
    return;
  }
  if (DKG_ABLATIONS && (P->debug_cov & 32)) return;  // probe: the Q_X blocks alone
  cross_means_body(P, B, kg, blockIdx.x - nbig);
}

// The fp32 plan's cross stage with the K(x, X) fill (DKG_PLAN_F32, e.g. BASELINE configs[4]): the 64 x 32 blocks
// on fp32 MFMA (cross_big32_body), then the fp64 means and clears of cross_big_kernel.
__global__ __launch_bounds__(XB_WAVES * WAVE) __attribute__((amdgpu_waves_per_eu(2))) void cross_big32_kernel(
    const Plan* __restrict__ P, int B, double* __restrict__ kg) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int nbig = cross_big_blocks(P->max_np, B, P->m);
  if ((int)blockIdx.x < nbig) {
    cross_big32_body(P, B, blockIdx.x, smem);
    return;
  }
  cross_means_body(P, B, kg, blockIdx.x - nbig);
}

// Means workgroup L (RT x m of them) of the big cross launches: K(x, X) alpha + c of row tile ti for output oi,
// and the accumulator clears.
__device__ __forceinline__ void cross_means_body(const Plan* __restrict__ P, int B, double* __restrict__ kg, int L) {
  const int RT = pad16(B) / 16;
  const int ti = L % RT, oi = L / RT;
  if (oi == 0) clear_tile_accumulators(P, kg, B, ti);
  const dkg_output& o = P->o[oi];
  const int n = o.n, KB = pad16(n) / 4;
  const double* kx = P->kx[oi];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool rv = ti * 16 + (lane & 15) < B;
  constexpr int VT = CR_WAVES * WAVE;  // the threads of cross_root_impl's fill
  constexpr int CH = VT / (XB_WAVES * WAVE);  // fill chains per thread
  static_assert(CH * XB_WAVES * WAVE == VT, "whole chains per thread");
  const int iters = (KB * 64 + VT - 1) / VT;
  double mpart[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) mpart[c] = 0.0;
  constexpr int U = 8;  // loads issued ahead of their fmas
  for (int it0 = 0; it0 < iters; it0 += U) {
    double kv[CH][U], al[CH][U];
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = tid + c * XB_WAVES * WAVE + min(it0 + u, iters - 1) * VT;
        const int col = 4 * (e >> 6) + (lane >> 4);
        kv[c][u] = (rv && col < n) ? kx[frag_index(ti, min(e >> 6, KB - 1), lane, KB)] : 0.0;
        al[c][u] = o.alpha[min(col, n - 1)];
      }
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (it0 + u < iters) mpart[c] = fma(kv[c][u], al[c][u], mpart[c]);
  }
  __shared__ double mred[CR_WAVES * 16];
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    double v = mpart[c];
    v += partner_f64<4>(v);
    v += partner_f64<5>(v);
    if (lane < 16) mred[(wave + c * XB_WAVES) * 16 + lane] = v;
  }
  __syncthreads();
  if (tid < 16) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < CR_WAVES; ++w) s += mred[w * 16 + tid];
    const int rr = ti * 16 + tid;
    P->mux[oi][rr] = (rr < B) ? o.mean_constant + s : 0.0;
  }
}

// Value + gradient cross stage, one launch: grid (B tiles, pairs, m + m d).
// z < m: the forward cross stage of output z (Q_X fragment-packed and row-major, means; kg and the
// tickets cleared).  z >= m, z - m = oi d + g: J_g = dK(x, X)/dx_g R (row-major) and dmean/dx_g for
// output oi; the first of these workgroups clears the gradient accumulator dkg[B x d].  The two halves
// read only x and the state, so they run side by side in one launch (at B = 1 the value+gradient chain
// is latency-bound: one launch and one dependency gap fewer than two cross launches).
// xa.n > 0 (dkg_plan_forward_grad_hostx): the candidates come in the kernel arguments; every workgroup
// reads them there, and the first leaves them in xnew for the later kernels of the chain.
template <int DM>
__global__ __launch_bounds__(CR_WAVES * WAVE) void cross_fwd_grad_kernel(const Plan* __restrict__ P,
                                                                         double* __restrict__ xstage, int B,
                                                                         double* __restrict__ kg,
                                                                         double* __restrict__ dkg, int dst,
                                                                         const XArg xa) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  unsigned long long* st = kst_slot(dst, P, 0);
  const int m = P->m, d = P->d;
  const int z = blockIdx.z;
  const double* xnew = xstage;
  if (xa.n > 0) {
    xnew = xa.v;
    if (blockIdx.x == 0 && blockIdx.y == 0 && z == 0)
      for (int i = threadIdx.x; i < xa.n; i += blockDim.x) xstage[i] = xa.v[i];
  }
  if (z < m) {
    if (blockIdx.y == 0 && z == 0) clear_tile_accumulators(P, kg, B, blockIdx.x);
    cross_root_impl<DM>(P->o[z], d, xnew, B, P->q[z], P->mux[z], blockIdx.x, blockIdx.y, smem, st, 0, nullptr,
                        P->qxrm[z]);
    return;
  }
  const int oi = (z - m) / d, gdim = (z - m) % d;
  if (blockIdx.x == 0 && blockIdx.y == 0 && z == m)
    for (int i = threadIdx.x; i < B * d; i += blockDim.x) dkg[i] = 0.0;
  const dkg_output& o = P->o[oi];
  const size_t mat = (size_t)P->bpad * pad16(o.n);
  cross_root_impl<DM, true>(o, d, xnew, B, P->jq[oi] + gdim * mat, P->gmu[oi] + (size_t)gdim * P->bpad, blockIdx.x,
                            blockIdx.y, smem, st, gdim);
}

size_t cross_root_lds_bytes(int np, int d) { return cross_lds_doubles(np, d, cross_pairs(np, d) > 1) * sizeof(double); }


static int outputs_bucket(int m) { return m <= 1 ? 1 : m <= 2 ? 2 : m <= 3 ? 3 : m <= 4 ? 4 : 8; }

size_t envelope_lds_bytes(int m, int N, int waves, int S, bool stream, bool grad, bool mu) {
  const int M = outputs_bucket(m);
  const size_t staged = stream ? 0 : (mu ? 2 : 1) * (size_t)stage_stride(N, cov_rec(M));
  const bool refine = stream && !grad;  // streaming forward: long lists + quickhull vertex arrays
  const size_t lc = list_cap(refine);
  // per wave: the list (slopes, intercepts; forward: line indices) and the streaming vertex arrays
  // streaming forward: the quickhull vertex arrays, or (M = 2..4) the staged chunk buffers in their place
  const size_t vroom = !refine ? 0
                       : stream_staged(M) ? std::max((size_t)waves * VREG, (size_t)4 * staged_chunk_len(cov_rec(M)))
                                          : (size_t)waves * VREG;
  // the kernel's layout (envelope_body): STAGE_FRONT doubles, the staged arrays, weights, pair sums, lists
  return ((size_t)STAGE_FRONT + staged + ((S * m + 1) & ~1) + ((S + 1) & ~1) + (size_t)waves * 2 * lc + vroom +
          (grad ? 0 : ((size_t)waves * lc + 1) / 2)) * sizeof(double);
}

size_t envelope_grad_lds_bytes(int m, int N, int waves, int S, int d, int max_np, bool stream) {
  const int M = outputs_bucket(m);
  const size_t extra = (size_t)(waves * ENV_CAP + 1) / 2 + (size_t)M * stage_len(max_np) +
                       (size_t)M * d * stage_len(max_np) +
                       2 * (size_t)M * DKG_MAX_DIM + (size_t)waves * 64 + DKG_MAX_DIM +
                       (size_t)M * DKG_MAX_DIM + (size_t)waves * (HCAP + max_np + ENV_CAP) +
                       (size_t)(waves * HCAP + 1) / 2;
  return envelope_lds_bytes(m, N, waves, S, stream, true) + extra * sizeof(double);
}

// ---------------------------------------------------------------------------
// lines_kg_kernel: KG = E[max_k (a_k + b_k Z)] - max_k a_k for P independent
// sets of L lines (row-major [P][L]); one wave per set.  Exposes the envelope
// stage on its own: the reference walk (calculate_epigraph_indices,
// discretekg.py:341-412, exactly: dkg_walk.h) and the cancellation-free
// expectation (calculate_expected_value_of_piecewise_linear_function + the
// baseline, :225-233, 415-452).  idx / xs (nullable): the walk's line indices
// [P][cap] and intersections [P][cap - 1] (dkg_epigraph).
template <int MAXL>
__global__ __launch_bounds__(256) void lines_kg_kernel(const double* __restrict__ a, const double* __restrict__ b,
                                                        int P, int L, double* __restrict__ kg, int* __restrict__ nhull,
                                                        long long* __restrict__ idx, double* __restrict__ xs,
                                                        int cap) {
  extern __shared__ __attribute__((aligned(16))) double sbuf[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int p = blockIdx.x * (blockDim.x >> 6) + wave;
  if (p >= P) return;
  // line k >= L: NaN intercept and slope (never an extreme, a tie, a survivor or a successor)
  auto build = [&](double (&la)[MAXL], double (&lb)[MAXL]) {
#pragma unroll
    for (int t = 0; t < MAXL; ++t) {
      const int k = lane + 64 * t;
      const int kk = min(k, L - 1);
      la[t] = (k < L) ? a[(size_t)p * L + kk] : __builtin_nan("");
      lb[t] = (k < L) ? b[(size_t)p * L + kk] : __builtin_nan("");
    }
  };
  const int nw = blockDim.x >> 6;
  double* sb = sbuf + (size_t)wave * 2 * ENV_CAP;
  int* si = reinterpret_cast<int*>(sbuf + (size_t)nw * 2 * ENV_CAP) + (size_t)wave * ENV_CAP;
  WalkOut out{idx ? idx + (size_t)p * cap : nullptr, xs ? xs + (size_t)p * (cap > 1 ? cap - 1 : 1) : nullptr, cap};
  int h = 0;
  const double v = env_pair_regs<MAXL>(build, L, lane, sb, sb + ENV_CAP, si, false, &h, idx ? &out : nullptr);
  if (lane == 0) {
    if (kg) kg[p] = v;
    if (nhull) nhull[p] = h;
  }
  if (idx) pad_walk_out(out, h, lane);
}

// Epigraph of line sets too long for the register path (L > 64 * 33): the
// reference walk over all lines, streamed from global memory each step.
__global__ __launch_bounds__(256) void lines_walk_kernel(const double* __restrict__ a, const double* __restrict__ b,
                                                         int P, int L, double* __restrict__ kg,
                                                         int* __restrict__ nhull, long long* __restrict__ idx,
                                                         double* __restrict__ xs, int cap) {
  constexpr int MAXL = 16;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int p = blockIdx.x * (blockDim.x >> 6) + wave;
  if (p >= P) return;
  const double* ap = a + (size_t)p * L;
  const double* bp = b + (size_t)p * L;
  auto build = [&](int c, double (&la)[MAXL], double (&lb)[MAXL]) {
#pragma unroll
    for (int t = 0; t < MAXL; ++t) {
      const int k = min(c * 64 * MAXL + lane + 64 * t, L - 1);
      la[t] = ap[k];
      lb[t] = bp[k];
    }
  };
  const int nch = (L + 64 * MAXL - 1) / (64 * MAXL);
  const FwdEnv f = env_extremes_stream<MAXL>(nch, L, lane, build);
  WalkOut out{idx ? idx + (size_t)p * cap : nullptr, xs ? xs + (size_t)p * (cap > 1 ? cap - 1 : 1) : nullptr, cap};
  int h = 1;
  double v = 0.0;
  if (f.status == 1) {
    if (idx && cap > 0) {  // first line attaining max a
      int k = KEY_NONE;
      for (int c = nch - 1; c >= 0; --c) {
        double la[MAXL], lb[MAXL];
        build(c, la, lb);
#pragma unroll
        for (int t = MAXL - 1; t >= 0; --t) {
          const int kk = c * 64 * MAXL + lane + 64 * t;
          k = (kk < L && la[t] == f.aT) ? kk : k;
        }
      }
      k = wave_min_i32(k);
      if (lane == 0) out.idx[0] = k;
    }
  } else {
    v = finish_edges(walk_stream<MAXL>(nch, L, lane, f.bL, f.aL, f.bT, &h, build, idx ? &out : nullptr));
  }
  if (lane == 0) {
    if (kg) kg[p] = v;
    if (nhull) nhull[p] = h;
  }
  if (idx) pad_walk_out(out, h, lane);
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

hipError_t launch_unpack_rows(const double* frag, int rows, int n, double* out, hipStream_t s) {
  const size_t total = (size_t)rows * pad16(n);
  if (total == 0) return hipSuccess;
  const int blocks = (int)std::min<size_t>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(unpack_rows_kernel, dim3(blocks), dim3(256), 0, s, frag, rows, pad16(n), out);
  return hipGetLastError();
}

hipError_t launch_frag_to_f32(const double* frag, int rows, int n, float* out, hipStream_t s) {
  const size_t total = (size_t)pad16(rows) * pad16(n);
  if (total == 0) return hipSuccess;
  const int blocks = (int)std::min<size_t>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(frag_to_f32_kernel, dim3(blocks), dim3(256), 0, s, frag, pad16(rows), pad16(n), out);
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
  dim3 grid(pad16(a.rows) / 16, cross_groups(np, a.d), 1);
  const size_t lds = cross_root_lds_bytes(np, a.d);
  raise_lds_limit((const void*)cross_root_kernel<DM>, lds);
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

// The 64 x 64 covariance blocks (posterior_cov_wide_kernel) when they still give every CU two blocks
// (e.g. the stress shape: 768 blocks); smaller batches keep the 32 x 32 blocks, whose latency is what
// sets a short forward.  DKG_COV_WIDE=0 / 1 (A/B measurements) forces the choice.
static bool cov_wide(int N, int B, int m) {
  static const char* env = std::getenv("DKG_COV_WIDE");
  if (env) return std::atoi(env) != 0 && N >= 64 && B >= 64;
  return N >= 64 && B >= 64 && (size_t)((N + 63) / 64) * ((B + 63) / 64) * m >= 512;
}

// The LDS-staged 64 x 64 blocks (posterior_cov_big_kernel: posterior_cov_kernel's bits; the fp32 plan's
// posterior_cov_big32_kernel) once a launch has at
// least one block per CU; decided on the launch's whole candidate count (a launch of several forward batches
// takes them whatever one batch would).  DKG_COV_BIG=0 / 1 (A/B measurements) forces the choice.
static bool cov_big(int N, int B, int m) {
  static const char* env = std::getenv("DKG_COV_BIG");
  if (env) return std::atoi(env) != 0 && N >= 1;
  return N >= 128 && (size_t)((N + 16 * PB_CT - 1) / (16 * PB_CT)) * ((B + 16 * PB_RT - 1) / (16 * PB_RT)) * m >= 256;
}

// The 64 x 32 covariance blocks (posterior_cov_blk_kernel: posterior_cov_kernel's bits, three per CU) once a launch
// has at least one per CU: they take precedence over the 64 x 64 blocks.  DKG_COV_BLK=0 / 1 (A/B) forces the choice.
// The opt-in covariance block kernels (bits: DKG_COV_ENABLE_BLK / _REC2 / _REG), enabled by their environment
// variables (DKG_COV_BLK / DKG_COV_REC2 / DKG_COV_REG) or by dkg_debug_cov_kernels (tests: each gives the narrow
// kernel's bits, checked by tests/test_gpu_batches.py with it enabled).
static int g_cov_enable = -1;  // -1: from the environment at first use
static int cov_enabled() {
  if (g_cov_enable < 0) {
    auto on = [](const char* v) { const char* e = std::getenv(v); return e && std::atoi(e) != 0; };
    g_cov_enable = (on("DKG_COV_BLK") ? DKG_COV_ENABLE_BLK : 0) | (on("DKG_COV_REC2") ? DKG_COV_ENABLE_REC2 : 0) |
                   (on("DKG_COV_REG") ? DKG_COV_ENABLE_REG : 0);
  }
  return g_cov_enable;
}
int set_cov_enabled(int mask) {
  const int prev = cov_enabled();
  g_cov_enable = mask & (DKG_COV_ENABLE_BLK | DKG_COV_ENABLE_REC2 | DKG_COV_ENABLE_REG);
  return prev;
}

// Off unless enabled: alone a 5-batch headline launch takes 27.7 us against the 64 x 64 blocks' 31.4, but
// with the four launch streams of bench.py the 64 x 64 blocks give the higher rate (10.0-10.4 against
// 9.5-9.7 M KG-evals/s at --steps 20, profiles/r06/bench/covab.txt): with forwards in flight the rate is the
// stages' summed CU time, not one launch's latency.  (m >= 3 alone: 164 against 143.7 us at configs[4].)
static bool cov_blk(int N, int B, int m) {
  return (cov_enabled() & DKG_COV_ENABLE_BLK) && N >= 64 &&
         (size_t)((N + 16 * PK_CT - 1) / (16 * PK_CT)) * ((B + 16 * PK_RT - 1) / (16 * PK_RT)) * m >= 256;
}

// The register-operand blocks (posterior_cov_reg_kernel: posterior_cov_kernel's bits, one workgroup per CU) for
// launches of at least one block per CU: the block height RT (4 or 5 candidate tiles, 4 line tiles) whose
// launch takes the fewest block-heights of device rounds -- ceil(blocks / 256) x RT -- (a 5-batch headline launch:
// 256 blocks of 5 x 4 tiles, one round; 4 x 4 tiles would need two).  One 8-wave workgroup per CU.  0: not this kernel.  DKG_COV_REG=0 / 4 / 5
// (A/B) disables it or forces RT.
static int cov_reg_rt(int N, int B, int m) {
  // off unless enabled: the 64 x 64 blocks are faster at m = 3, and it takes a CU whole as rec2 does
  if (!(cov_enabled() & DKG_COV_ENABLE_REG) || N < 64) return 0;
  auto blocks = [&](int rt) { return (size_t)((N + 63) / 64) * ((B + 16 * rt - 1) / (16 * rt)) * m; };
  if (blocks(4) < 256) return 0;
  auto cost = [&](int rt) { return ((blocks(rt) + 255) / 256) * (size_t)rt; };
  return cost(5) < cost(4) ? 5 : 4;
}

// posterior_cov_rec2_kernel (m = 2): blocks of RT candidate tiles x 32 lines x both outputs, the same block-height
// choice (blocks = ceil(B / 16 RT) x ceil(N / 32)).  DKG_COV_REC2=0 / 4 / 5 (A/B) disables it or forces RT.
// Off unless DKG_COV_REC2=1 (or 4 / 5 to force RT): the fastest covariance launch alone (a 5-batch headline launch
// 23.0 us, 0.38 of the fp64 roof, against 31.4), but one 8-wave workgroup of 256 VGPRs and 121 KB of LDS takes a
// CU whole, so nothing of the other streams' forwards runs beside it: 8.9-9.1 against 10.0-10.4 M KG-evals/s in
// bench.py's --steps 20 line (profiles/r06/bench/covab.txt).
static int cov_rec2_rt(int N, int B) {
  if (!(cov_enabled() & DKG_COV_ENABLE_REC2) || N < 32) return 0;
  auto blocks = [&](int rt) { return (size_t)((N + 31) / 32) * ((B + 16 * rt - 1) / (16 * rt)); };
  // (on) one device round of blocks (one workgroup per CU): the shortest block that fits in it; launches of more
  // take the 64 x 32 blocks, whose three workgroups per CU measured faster there (profiles/r06/cov/h_*.txt)
  if (blocks(5) <= 256 && blocks(5) > 192) return blocks(4) <= 256 ? 4 : 5;
  if (blocks(4) <= 256 && blocks(4) > 192) return 4;
  return 0;
}

// The cross stage of a launch with the K(x, X) fill as 64 x 32 blocks (cross_big_kernel); DKG_CROSS_BIG=0 (A/B
// measurements) keeps cross_root_plan_kernel.
static bool cross_big() {
  static const char* env = std::getenv("DKG_CROSS_BIG");
  return !env || std::atoi(env) != 0;
}

// The big blocks' order (block_order).  Measured per launch (L2 fetch x2 / write MB, stage us; DESIGN.md 4.7,
// profiles/r05/cov_order): stress (nbx 64, nby 4, m 3): order 0 363 / 37, 1 263 / 36, 2 145 / 101, 3 152 / 101,
// all 143 us; headline x 10 (nbx 16, nby 20, m 2): 0 49 / 21, 1 72 / 21, 2 44 / 42, all 47 us.  Orders 2 / 3
// read each panel about once but write every output's record sectors separately (3x the records); order 1 keeps
// the outputs of a block side by side (whole records leave L2) and shares the line panels of a wide launch.
// DKG_COV_ORDER=0..3 (A/B measurements) forces it.
static int cov_big_order(int nbx, int nby, int m) {
  static const char* env = std::getenv("DKG_COV_ORDER");
  if (env) return std::atoi(env);
  (void)m;
  return nbx >= 4 * nby ? 1 : 0;
}

template <int DM, class T>
static hipError_t launch_cross_cov_tt(const Plan& h, const Plan* dev, const double* xnew, int B, double* kg,
                                      hipStream_t s, int stage, int geom_B) {
  if (stage == 0) {
    const int use_kx = (h.kx[0] != nullptr && cross_kfill_launch(h.max_np, B)) ? 1 : 0;
    if (use_kx) {
      dim3 kgrid(pad16(B) / 16, (h.max_np / 4 + KF_KB - 1) / KF_KB, h.m);
      hipLaunchKernelGGL((cross_kfill_kernel<DM>), kgrid, dim3(KF_WAVES * WAVE), 0, s, dev, xnew, B);
    }
    // K(x, X) in place: the 64 x 32 blocks, then the means and the clears.  The fp32 blocks sum in another order
    // than cross_root_plan_kernel<float>, so an F32 plan takes them only where one batch of the launch would
    // (geom_B): a launch of several batches keeps the per-batch bits (dkg_plan_forward_batches)
    if (use_kx && cross_big() && (sizeof(T) == 8 || cross_kfill_launch(h.max_np, geom_B))) {
      const dim3 grid(cross_big_blocks(h.max_np, B, h.m) + pad16(B) / 16 * h.m);
      if constexpr (sizeof(T) == 8) {
        raise_lds_limit((const void*)cross_big_kernel, XB_LDS);
        hipLaunchKernelGGL(cross_big_kernel, grid, dim3(XB_WAVES * WAVE), XB_LDS, s, dev, B, kg);
      } else {
        raise_lds_limit((const void*)cross_big32_kernel, XB32_LDS);
        hipLaunchKernelGGL(cross_big32_kernel, grid, dim3(XB_WAVES * WAVE), XB32_LDS, s, dev, B, kg);
      }
      return hipGetLastError();
    }
    dim3 grid(pad16(B) / 16, cross_groups(h.max_np, h.d), h.m);
    const size_t lds = cross_root_lds_bytes(h.max_np, h.d);
    raise_lds_limit((const void*)cross_root_plan_kernel<DM, T>, lds);
    hipLaunchKernelGGL((cross_root_plan_kernel<DM, T>), grid, dim3(CR_WAVES * WAVE), lds, s, dev, xnew, B, kg,
                       h.debug_stamp, use_kx);
    return hipGetLastError();
  }
  if constexpr (sizeof(T) == 8 && DM <= 8) {  // (d > 8: the big blocks' kernel terms spill)
    // both outputs' records from one workgroup (d <= 2: with the wider candidates the late kernel terms spill)
    if (const int rt = (DM <= 2 && h.m == 2) ? cov_rec2_rt(h.N, B) : 0) {
      const int nbx = (h.N + 31) / 32, nby = (B + 16 * rt - 1) / (16 * rt);
      const int order = cov_big_order(nbx, nby, 1);
      dim3 grid(block_order_size(nbx, nby, 1, order));
      if (rt == 5) {
        raise_lds_limit((const void*)posterior_cov_rec2_kernel<DM, 5>, cov_rec2_lds<5>());
        hipLaunchKernelGGL((posterior_cov_rec2_kernel<DM, 5>), grid, dim3(PR_WAVES * WAVE), cov_rec2_lds<5>(), s,
                           dev, xnew, B, h.debug_stamp, order);
      } else {
        raise_lds_limit((const void*)posterior_cov_rec2_kernel<DM, 4>, cov_rec2_lds<4>());
        hipLaunchKernelGGL((posterior_cov_rec2_kernel<DM, 4>), grid, dim3(PR_WAVES * WAVE), cov_rec2_lds<4>(), s,
                           dev, xnew, B, h.debug_stamp, order);
      }
      return hipGetLastError();
    }
    if (const int rt = cov_reg_rt(h.N, B, h.m)) {
      const int nbx = (h.N + 63) / 64, nby = (B + 16 * rt - 1) / (16 * rt);
      const int order = cov_big_order(nbx, nby, h.m);
      dim3 grid(block_order_size(nbx, nby, h.m, order));
      if (rt == 5) {
        raise_lds_limit((const void*)posterior_cov_reg_kernel<DM, 5>, cov_reg_lds<5>());
        hipLaunchKernelGGL((posterior_cov_reg_kernel<DM, 5>), grid, dim3(PR_WAVES * WAVE), cov_reg_lds<5>(), s, dev,
                           xnew, B, h.debug_stamp, order);
      } else {
        raise_lds_limit((const void*)posterior_cov_reg_kernel<DM, 4>, cov_reg_lds<4>());
        hipLaunchKernelGGL((posterior_cov_reg_kernel<DM, 4>), grid, dim3(PR_WAVES * WAVE), cov_reg_lds<4>(), s, dev,
                           xnew, B, h.debug_stamp, order);
      }
      return hipGetLastError();
    }
    if (cov_blk(h.N, B, h.m)) {
      const int nbx = (h.N + 16 * PK_CT - 1) / (16 * PK_CT), nby = (B + 16 * PK_RT - 1) / (16 * PK_RT);
      const int order = cov_big_order(nbx, nby, h.m);
      dim3 grid(block_order_size(nbx, nby, h.m, order));
      raise_lds_limit((const void*)posterior_cov_blk_kernel<DM>, PK_LDS);
      hipLaunchKernelGGL((posterior_cov_blk_kernel<DM>), grid, dim3(PB_WAVES * WAVE), PK_LDS, s, dev, xnew, B,
                         h.debug_stamp, order);
      return hipGetLastError();
    }
    if (cov_big(h.N, B, h.m)) {
      const int nbx = (h.N + 16 * PB_CT - 1) / (16 * PB_CT), nby = (B + 16 * PB_RT - 1) / (16 * PB_RT);
      const int order = cov_big_order(nbx, nby, h.m);
      dim3 grid(block_order_size(nbx, nby, h.m, order));
      raise_lds_limit((const void*)posterior_cov_big_kernel<DM>, PB_LDS);
      hipLaunchKernelGGL((posterior_cov_big_kernel<DM>), grid, dim3(PB_WAVES * WAVE), PB_LDS, s, dev, xnew, B,
                         h.debug_stamp, order);
      return hipGetLastError();
    }
  }
  if constexpr (sizeof(T) == 4 && DM <= 8) {  // the fp32 plan's 64 x 64 blocks (DKG_COV_BIG32=0: A/B only)
    static const char* env = std::getenv("DKG_COV_BIG32");
    if (cov_big(h.N, geom_B, h.m) && (!env || std::atoi(env) != 0)) {  // (geom_B: as the cross stage above)
      const int nbx = (h.N + 16 * PB_CT - 1) / (16 * PB_CT), nby = (B + 16 * PB_RT - 1) / (16 * PB_RT);
      const int order = cov_big_order(nbx, nby, h.m);
      dim3 grid(block_order_size(nbx, nby, h.m, order));
      raise_lds_limit((const void*)posterior_cov_big32_kernel<DM>, PB32_LDS);
      hipLaunchKernelGGL((posterior_cov_big32_kernel<DM>), grid, dim3(PB_WAVES * WAVE), PB32_LDS, s, dev, xnew, B,
                         h.debug_stamp, order);
      return hipGetLastError();
    }
  }
  if constexpr (sizeof(T) == 8 && DM <= 4) {
    if (cov_wide(h.N, geom_B, h.m)) {
      dim3 grid(xcd_group_size(((h.N + 63) / 64) * ((B + 63) / 64), h.m));
      hipLaunchKernelGGL((posterior_cov_wide_kernel<DM>), grid, dim3(PW_WAVES * WAVE), 0, s, dev, xnew, B,
                         h.debug_stamp);
      return hipGetLastError();
    }
  }
  dim3 grid(xcd_group_size(std::max(1, (h.N + 31) / 32) * ((B + 16 * PC_RB - 1) / (16 * PC_RB)), h.m));
  hipLaunchKernelGGL((posterior_cov_kernel<DM, T>), grid, dim3(PC_WAVES * WAVE), 0, s, dev, xnew, B, h.debug_stamp);
  return hipGetLastError();
}

template <int DM>
static hipError_t launch_cross_cov_t(const Plan& h, const Plan* dev, const double* xnew, int B, double* kg,
                                     hipStream_t s, int stage, int geom_B) {
  return h.f32 ? launch_cross_cov_tt<DM, float>(h, dev, xnew, B, kg, s, stage, geom_B)
               : launch_cross_cov_tt<DM, double>(h, dev, xnew, B, kg, s, stage, geom_B);
}

// Narrow small-batch geometry: off (DKG_ENV_NARROW=0).  At B = 1 its 16 one-wave workgroups staged the lines
// 16 times and met in per-group tickets: the value+gradient envelope took 16.6 us against 14.1 us for two
// 8-wave workgroups (profiles/r04/b1).
#ifndef DKG_ENV_NARROW
#define DKG_ENV_NARROW 0
#endif
void envelope_geometry(int B, int S, int* waves_per_wg, int* split, bool narrow) {
  // Up to 8 scalarisation waves of one candidate per workgroup, one pair per
  // wave; with S <= 16 at most two workgroups per candidate, whose group sums
  // meet in one commutative atomic add (no inter-workgroup fences).
  // Small batches (narrow): fewer waves per workgroup until the launch has at least ENV_MIN_WGS
  // workgroups, so a B = 1 value+gradient call (the reference's optimize_acqf shape, batch_limit 1)
  // spreads its S pairs over S CUs, one wave per SIMD, instead of two workgroups; the workgroups of
  // one group of 8 pairs meet in ordered per-pair values (envelope_body: the same bits as the wide launch).
  constexpr int ENV_MIN_WGS = 128;
  int sw = std::max(1, std::min(8, S));
  static const char* env = std::getenv("DKG_ENV_SW");  // A/B measurements: waves per workgroup
  if (env && std::atoi(env) >= 1) sw = std::max(1, std::min(std::atoi(env), sw));
  if (narrow && DKG_ENV_NARROW)
    while (sw > 1 && (long long)B * ((S + sw - 1) / sw) < ENV_MIN_WGS) sw = (sw + 1) / 2;
  *waves_per_wg = sw;
  *split = (S + sw - 1) / sw;
}

// The envelope launch for the plan's output bucket.
template <bool GRAD>
static hipError_t launch_env(const Plan& h, const EnvLaunch& a) {
  const bool stream = h.stream != 0;
  switch (outputs_bucket(h.m)) {
    case 1: return launch_env_m1(GRAD, h.N + 1, stream, a);
    case 2: return launch_env_m2(GRAD, h.N + 1, stream, a);
    case 3: return launch_env_m3(GRAD, h.N + 1, stream, a);
    case 4: return launch_env_m4(GRAD, h.N + 1, stream, a);
    default: return launch_env_m8(GRAD, h.N + 1, stream, a);
  }
}

hipError_t launch_stage(const Plan& h, const Plan* dev, const double* xnew, int B, double* kg, double* pairs,
                        hipStream_t s, int stage, int geom_B) {
  if (stage == 0 || stage == 1) {
    const int gb = geom_B > 0 ? geom_B : B;
    switch (dim_bucket(h.d)) {
      case 2: return launch_cross_cov_t<2>(h, dev, xnew, B, kg, s, stage, gb);
      case 4: return launch_cross_cov_t<4>(h, dev, xnew, B, kg, s, stage, gb);
      case 8: return launch_cross_cov_t<8>(h, dev, xnew, B, kg, s, stage, gb);
      default: return launch_cross_cov_t<16>(h, dev, xnew, B, kg, s, stage, gb);
    }
  }
  EnvLaunch a{&h, dev, B, kg, pairs, dim3(xcd_group_size(B, h.split)), dim3(h.sw * WAVE),
              envelope_lds_bytes(h.m, h.N, h.sw, h.S, h.stream != 0, false, !DKG_ICP), s, h.debug_stamp, nullptr,
              nullptr};
  return launch_env<false>(h, a);
}

template <int DM>
static hipError_t launch_cross_fwd_grad_t(const Plan& h, const Plan* dev, const double* xnew, int B, double* kg,
                                          double* dkg, hipStream_t s, const XArg& xa) {
  dim3 grid(pad16(B) / 16, cross_groups(h.max_np, h.d), h.m * (1 + h.d));
  const size_t lds = cross_root_lds_bytes(h.max_np, h.d);
  raise_lds_limit((const void*)cross_fwd_grad_kernel<DM>, lds);
  hipLaunchKernelGGL(cross_fwd_grad_kernel<DM>, grid, dim3(CR_WAVES * WAVE), lds, s, dev,
                     const_cast<double*>(xnew), B, kg, dkg, h.debug_stamp, xa);
  return hipGetLastError();
}

hipError_t launch_forward_grad(const Plan& h, const Plan* dev, const double* xnew, int B, double* kg, double* dkg,
                               hipStream_t s, const XArg* xa, double* hout) {
  hipError_t e;
  XArg none;
  none.n = 0;
  const XArg& x = xa ? *xa : none;
  switch (dim_bucket(h.d)) {  // Q_X (fragment + row-major), means, J_g, dmean; kg = dkg = 0
    case 2: e = launch_cross_fwd_grad_t<2>(h, dev, xnew, B, kg, dkg, s, x); break;
    case 4: e = launch_cross_fwd_grad_t<4>(h, dev, xnew, B, kg, dkg, s, x); break;
    case 8: e = launch_cross_fwd_grad_t<8>(h, dev, xnew, B, kg, dkg, s, x); break;
    default: e = launch_cross_fwd_grad_t<16>(h, dev, xnew, B, kg, dkg, s, x); break;
  }
  if (e != hipSuccess) return e;
  if ((e = launch_stage(h, dev, xnew, B, kg, nullptr, s, 1)) != hipSuccess) return e;  // cov rows, variances
  EnvLaunch a{&h, dev, B, kg, nullptr, dim3(xcd_group_size(B, h.split)), dim3(h.sw * WAVE),
              envelope_grad_lds_bytes(h.m, h.N, h.sw, h.S, h.d, h.max_np, h.stream != 0), s, h.debug_stamp, xnew, dkg,
              hout};
  return launch_env<true>(h, a);
}

hipError_t launch_forward(const Plan& h, const Plan* dev, const double* xnew, int B, double* kg, double* pairs,
                          hipStream_t s, hipEvent_t* ev, int geom_B) {
  for (int stage = 0; stage < 3; ++stage) {
    if (ev) (void)hipEventRecord(ev[stage], s);
    const hipError_t e = launch_stage(h, dev, xnew, B, kg, pairs, s, stage, geom_B);
    if (e != hipSuccess) return e;
  }
  if (ev) (void)hipEventRecord(ev[3], s);
  return hipSuccess;
}

size_t fused_lds_bytes_host(const Plan& h) { return fused_lds_bytes(h); }

hipError_t launch_forward_auto(const Plan& h, const Plan* dev, const double* xnew, int B, double* kg, double* pairs,
                               hipStream_t s) {
  if (!h.fused || pairs != nullptr || B < 1) return launch_forward(h, dev, xnew, B, kg, pairs, s, nullptr);
  FusedArgs a{};
  a.P = dev;
  a.xnew = xnew;
  a.kg = kg;
  a.B = B;
  a.dst = h.debug_stamp;
  const int rt = pad16(B) / 16;
  a.cgroups = cross_groups(h.max_np, h.d);
  a.nC = rt * a.cgroups * h.m;
  a.vcols = std::max(1, (h.N + 31) / 32);
  a.vrows = (B + 16 * PC_RB - 1) / (16 * PC_RB);
  a.nV = a.vcols * a.vrows * h.m;
  a.split = h.split;
  a.mu_all = h.mu_all;
  a.cov_all = h.cov_all;
  a.var_all = h.var_all;
  a.mux_all = h.mux_all;
  a.wts = h.weights;
  a.dup = h.dup;
  a.cov_stride = (long long)h.cov_stride;
  a.bpad = h.bpad;
  // counters laid out for this B (every launch re-zeroes the range it used)
  a.ho.cnt1 = h.sync;
  a.ho.cnt2 = h.sync + (size_t)h.m * rt * HANDOFF_STRIDE;
  a.ho.done = a.ho.cnt2 + (size_t)a.vrows * HANDOFF_STRIDE;
  a.ho.err = h.sync_err;
  a.ho.rt = rt;
  a.ho.nrb = a.vrows;
  a.ho.rb_rows = 16 * PC_RB;
  a.ho.quota1 = (unsigned long long)a.cgroups;
  a.ho.quota2 = (unsigned long long)a.vcols * h.m;
  a.ho.quota_done = (unsigned long long)B * a.split;
  const size_t lds = fused_lds_bytes(h);
  const int db = dim_bucket(h.d), lines = h.N + 1;
  switch (outputs_bucket(h.m)) {
    case 1: return launch_fused_m1(db, lines, a, lds, s);
    case 2: return launch_fused_m2(db, lines, a, lds, s);
    case 3: return launch_fused_m3(db, lines, a, lds, s);
    case 4: return launch_fused_m4(db, lines, a, lds, s);
    default: return launch_fused_m8(db, lines, a, lds, s);
  }
}

hipError_t launch_lines_kg(const double* a, const double* b, int P, int L, double* kg, int* nhull, long long* idx,
                           double* xs, int cap, hipStream_t s) {
  const int wpb = 4;
  dim3 grid((P + wpb - 1) / wpb), block(wpb * WAVE);
  const size_t lds = (size_t)wpb * 2 * ENV_CAP * sizeof(double) + (size_t)wpb * ENV_CAP * sizeof(int);
  if (L <= 64 * 2) hipLaunchKernelGGL(lines_kg_kernel<2>, grid, block, lds, s, a, b, P, L, kg, nhull, idx, xs, cap);
  else if (L <= 64 * 4) hipLaunchKernelGGL(lines_kg_kernel<4>, grid, block, lds, s, a, b, P, L, kg, nhull, idx, xs, cap);
  else if (L <= 64 * 8) hipLaunchKernelGGL(lines_kg_kernel<8>, grid, block, lds, s, a, b, P, L, kg, nhull, idx, xs, cap);
  else if (L <= 64 * 17) hipLaunchKernelGGL(lines_kg_kernel<17>, grid, block, lds, s, a, b, P, L, kg, nhull, idx, xs, cap);
  else if (L <= 64 * 33) hipLaunchKernelGGL(lines_kg_kernel<33>, grid, block, lds, s, a, b, P, L, kg, nhull, idx, xs, cap);
  else hipLaunchKernelGGL(lines_walk_kernel, grid, block, 0, s, a, b, P, L, kg, nhull, idx, xs, cap);
  return hipGetLastError();
}

hipError_t launch_lines_export(const Plan& h, const Plan* dev, int B, double* a_out, double* b_out, hipStream_t s) {
  const dim3 grid(B, h.S), block(256);
  switch (outputs_bucket(h.m)) {
    case 1: hipLaunchKernelGGL(lines_export_kernel<1>, grid, block, 0, s, dev, a_out, b_out); break;
    case 2: hipLaunchKernelGGL(lines_export_kernel<2>, grid, block, 0, s, dev, a_out, b_out); break;
    case 3: hipLaunchKernelGGL(lines_export_kernel<3>, grid, block, 0, s, dev, a_out, b_out); break;
    case 4: hipLaunchKernelGGL(lines_export_kernel<4>, grid, block, 0, s, dev, a_out, b_out); break;
    default: hipLaunchKernelGGL(lines_export_kernel<8>, grid, block, 0, s, dev, a_out, b_out); break;
  }
  return hipGetLastError();
}

// E[f(Z)] of a piecewise-linear f given its pieces and boundaries, the
// reference's formula (calculate_expected_value_of_piecewise_linear_function,
// discretekg.py:415-452): sum_j a_j (Phi(c_j+1) - Phi(c_j)) - b_j (phi(c_j+1) - phi(c_j)),
// c_0 = -inf, c_m = +inf, with torch's Normal: pdf = exp(log_prob), cdf = (1 + erf(z / sqrt 2)) / 2.
// One wave per set of m pieces.
__global__ __launch_bounds__(256) void pwl_expectation_kernel(const double* __restrict__ a, const double* __restrict__ b,
                                                              const double* __restrict__ c, int P, int m,
                                                              double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int p = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (p >= P) return;
  auto bound = [&](int j) {  // c_j, j = 0 .. m
    return j == 0 ? -INFINITY : j == m ? INFINITY : c[(size_t)p * (m - 1) + j - 1];
  };
  auto pdf = [](double z) { return exp(-0.5 * z * z - 0.91893853320467274178); };  // log(sqrt(2 pi))
  auto cdf = [](double z) { return 0.5 * (1.0 + erf(z * 0.70710678118654752440)); };
  double acc = 0.0;
  for (int j = lane; j < m; j += 64) {
    const double lo = bound(j), hi = bound(j + 1);
    acc += a[(size_t)p * m + j] * (cdf(hi) - cdf(lo)) - b[(size_t)p * m + j] * (pdf(hi) - pdf(lo));
  }
  acc = wave_sum(acc);
  if (lane == 0) out[p] = acc;
}

hipError_t launch_pwl_expectation(const double* a, const double* b, const double* c, int P, int m, double* out,
                                  hipStream_t s) {
  const int wpb = 4;
  hipLaunchKernelGGL(pwl_expectation_kernel, dim3((P + wpb - 1) / wpb), dim3(wpb * WAVE), 0, s, a, b, c, P, m, out);
  return hipGetLastError();
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
