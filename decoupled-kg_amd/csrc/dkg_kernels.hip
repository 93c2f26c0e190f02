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
    const int l = (int)(e & 63);
    const size_t blk = e >> 6;
    const int kb = (int)(blk % KB);
    const int tj = (int)(blk / KB);
    const int row = 4 * kb + (l >> 4);
    const int col = 16 * tj + (l & 15);
    rf[e] = (row < n && col < n) ? r[(size_t)row * n + col] : 0.0;
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

template <int DM>
__device__ __forceinline__ void cross_root_impl(const dkg_output& o, int d, const double* __restrict__ x, int rows,
                                                double* __restrict__ qout, double* __restrict__ mout, int ti, int p,
                                                double* smem, unsigned long long* st = nullptr) {
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
  const double* rfA = o.root_frag + (size_t)tA * KB * 64 + lane;
  const double* rfB = o.root_frag + (size_t)tB * KB * 64 + lane;
  const int chunk = (kbB + CR_WAVES - 1) / CR_WAVES;
  const int k0 = wave * chunk;
  const int k1 = min(kbB, k0 + chunk);
  double ra[CR_U], rb[CR_U];
#pragma unroll
  for (int u = 0; u < CR_U; ++u) {
    const int kb = min(k0 + u, kbB - 1);
    rb[u] = rfB[(size_t)kb * 64];
    ra[u] = rfA[(size_t)min(kb, kbA - 1) * 64];
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
      const double kv = os * kernel_profile_t<KIND>(r2);
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
      for (int u = 0; u < CR_U; ++u) {
        const int kb = min(base + u, kbB - 1);
        rb[u] = rfB[(size_t)kb * 64];
        ra[u] = rfA[(size_t)min(kb, kbA - 1) * 64];
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
      qout[((size_t)ti * KB + 4 * tj + r) * 64 + lane] = s;
    }
  }
  if (want_mean && tid < 16) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < CR_WAVES; ++w) s += mred[w * 16 + tid];
    const int rr = ti * 16 + tid;
    mout[rr] = (rr < rows) ? o.mean_constant + s : 0.0;
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
                                                                          double* __restrict__ kg) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  unsigned long long* st = kst_slot(P->debug_stamp, 0);
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

size_t cross_root_lds_bytes(int np, int d) {
  return ((size_t)(np / 4) * 64 + CR_WAVES * 8 * 64 + CR_WAVES * 16 + (size_t)np * d + np) * sizeof(double);
}

// ---------------------------------------------------------------------------
// posterior_cov_kernel: cov[b][k] = s k(x_b, D_k) - sum_l Q[b][l] Q_D[k][l]
// One workgroup per 16x16 output tile (ti candidates x tk points) per output;
// the 4 waves split the n_pad/4 k-blocks; each wave issues the loads of a
// whole batch of PC_U k-blocks (2 x 512-byte coalesced fragment loads per
// k-block) before its MFMAs, so the L2 latency is paid once per batch.
// Partials are reduced in LDS in fixed wave order.
constexpr int PC_WAVES = 4;
constexpr int PC_U = 16;

// 4 workgroups per CU (<= 128 VGPRs): the whole 1024-workgroup headline grid is resident at once.
template <int DM>
__global__ __launch_bounds__(PC_WAVES * WAVE, 4) void posterior_cov_kernel(const Plan* __restrict__ P,
                                                                         const double* __restrict__ xnew, int B) {
  __shared__ __attribute__((aligned(16))) double part[PC_WAVES * 4 * 64];
  __shared__ double qpart[PC_WAVES * 16];
  unsigned long long* st = kst_slot(P->debug_stamp, 1);
  KST_BEGIN(st);
  const int tk = blockIdx.x;
  const int ti = blockIdx.y;
  const int oi = blockIdx.z;
  const dkg_output& o = P->o[oi];
  const int N = P->N;
  const int dbg = P->debug_cov;
  if (tk > 0 && tk * 16 >= N) return;  // tile 0 always runs: it also produces the candidates' variances
  const bool have_d = N > 0;
  const int KB = pad16(o.n) / 4;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

  const int chunk = (KB + PC_WAVES - 1) / PC_WAVES;
  const int k0 = wave * chunk;
  const int k1 = min(KB, k0 + chunk);
  const double* qa = P->q[oi] + (size_t)ti * KB * 64 + lane;
  const double* qd = o.disc_frag + (size_t)tk * KB * 64 + lane;
  // four independent accumulation chains (k-block mod 4): the f64 MFMA
  // dependent-issue latency is hidden by the other chains
  // epilogue operands (row b, column k of register r = wave) first: their
  // latency overlaps the fragment loads
  const int b = ti * 16 + (lane >> 4) + 4 * wave;
  const int k = tk * 16 + (lane & 15);
  const int d = P->d;
  const double* xb = xnew + (size_t)min(b, B - 1) * d;
  const double* xk = have_d ? P->disc + (size_t)min(k, N - 1) * d : xb;
  const double r2 = scaled_r2_dm<DM>(xb, xk, o.inv_lengthscale, d);
  KST(st, 2);
  d4 acc[4] = {{0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}};
  double qsq = 0.0;  // lane l: sum over this wave's k of Q_X[16 ti + (l & 15)][k]^2 (k = 4 kb + (l >> 4))
  for (int base = k0; base < k1; base += PC_U) {
    double ra[PC_U], rb[PC_U];
#pragma unroll
    for (int u = 0; u < PC_U; ++u) {
      const int kb = min(base + u, KB - 1);
      if (dbg & 1) {
        ra[u] = 1.0 + kb;
        rb[u] = 0.5;
      } else {
        ra[u] = qa[(size_t)kb * 64];
        rb[u] = (have_d && base + u < k1) ? qd[(size_t)kb * 64] : 0.0;
      }
    }
    if (dbg & 2) {
#pragma unroll
      for (int u = 0; u < PC_U; ++u) acc[0][u & 3] += ra[u] * rb[u];
      continue;
    }
#pragma unroll
    for (int u = 0; u < PC_U; ++u) acc[u & 3] = mfma_f64(ra[u], rb[u], acc[u & 3]);
    if (tk == 0) {  // the candidates' own |Q_X[b]|^2 (padding k-blocks of the batch repeat the last one)
#pragma unroll
      for (int u = 0; u < PC_U; ++u) qsq = (base + u < k1) ? fma(ra[u], ra[u], qsq) : qsq;
    }
  }
  const d4 accs = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  KST(st, 3);
#pragma unroll
  for (int r = 0; r < 4; ++r) part[(wave * 4 + r) * 64 + lane] = accs[r];
  if (tk == 0) {
    qsq += __shfl_xor(qsq, 16);
    qsq += __shfl_xor(qsq, 32);
    if (lane < 16) qpart[wave * 16 + lane] = qsq;
  }
  __syncthreads();
  if (tk == 0 && threadIdx.x < 16) {
    const int bb = ti * 16 + threadIdx.x;
    double q2 = 0.0;
#pragma unroll
    for (int w = 0; w < PC_WAVES; ++w) q2 += qpart[w * 16 + threadIdx.x];
    if (bb < B) P->var[oi][bb] = o.outputscale - q2;
  }

  KST(st, 4);
  double s = 0.0;
#pragma unroll
  for (int w = 0; w < PC_WAVES; ++w) s += part[(w * 4 + wave) * 64 + lane];
  if (b < B && k < N)
    P->cov[oi][(size_t)b * N + k] = ((dbg & 4) ? r2 : o.outputscale * kernel_profile(o.kernel, r2)) - s;
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

// KG of one set of lines held MAXL per lane (line k in lane k % 64, slot k / 64).
template <int MAXL>
__device__ __forceinline__ double envelope_kg(const double (&la)[MAXL], const double (&lb)[MAXL], int nl, int lane,
                                              double* sb, double* sa, int* nhull) {
  // ---- extremes by value, then exact tie passes (exec-masked, rarely taken):
  // L = min b (tie: max a), R = max b (tie: max a), T = max a (tie: min b).
  // (slots beyond nl hold padding lines: a = -inf, b = a real slope)
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
    if (nhull) *nhull = 1;
    return 0.0;
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

  // ---- survivors: lines strictly above the chord L-T or the chord T-R.
  // No left/right select is needed: every line has a <= aT, so a line left of
  // T is never above the extension of T-R (its slope is <= 0) and a line right
  // of T never above the extension of L-T (slope >= 0); a degenerate chord
  // (db = 0) admits nothing.  h = (a - a0) db - (b - b0) da > 0, evaluated as
  // a*db - b*da > a0*db - b0*da.  Rounding can only admit extra lines (L, T
  // or R themselves), which the exact test below discards.
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
        if (pos < ENV_CAP) { sb[pos] = bb; sa[pos] = a; }
      }
      cnt += __popcll(mk);
    }
  }
  if (cnt + 3 > ENV_CAP) return envelope_walk<MAXL>(la, lb, nl, lane, bL, aL, bR, bT, nhull);
  if (lane == 0) {
    sb[cnt] = bL; sa[cnt] = aL;
    sb[cnt + 1] = bT; sa[cnt + 1] = aT;
    sb[cnt + 2] = bR; sa[cnt + 2] = aR;
  }
  const int nc = cnt + 3;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

  // ---- right neighbour of every candidate P (one per lane, two chunks of 64
  // at most): the line that takes over from P as z grows, i.e. the reference
  // walk's step (discretekg.py:382-401): argmin over b_Q > b_P of the
  // intersection (a_P - a_Q)/(b_Q - b_P), ties -> larger slope.  Compared by
  // cross multiplication (both denominators > 0).
  int nxt[2] = {-1, -1};
  double cn[2] = {0.0, 0.0}, cd[2] = {1.0, 1.0}, cb[2] = {0.0, 0.0}, pb[2] = {0.0, 0.0};
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    if (c * 64 >= nc) break;
    const int e = c * 64 + lane;
    const bool mine = e < nc;
    const double bP = mine ? sb[e] : 0.0, aP = mine ? sa[e] : 0.0;
    double rn = 0.0, rd = 1.0, rb = 0.0;
    int rj = -1;
#pragma unroll 4
    for (int j = 0; j < nc; ++j) {
      const double bQ = sb[j], aQ = sa[j];
      const double num = aP - aQ, den = bQ - bP;
      const double x = num * rd, y = rn * den;
      const bool take = den > 0.0 && (rj < 0 || x < y || (x == y && bQ > rb));
      rn = take ? num : rn;
      rd = take ? den : rd;
      rb = take ? bQ : rb;
      rj = take ? j : rj;
    }
    nxt[c] = rj; cn[c] = rn; cd[c] = rd; cb[c] = rb; pb[c] = bP;
  }

  // ---- follow the chain from L (index cnt): its members are the envelope
  // lines in increasing slope, ending at R (no right neighbour).
  uint64_t on0 = 0, on1 = 0;
  int h = 0;
  for (int cur = cnt, guard = 0; cur >= 0 && guard < nc; ++guard) {
    if (cur < 64) on0 |= 1ull << cur; else on1 |= 1ull << (cur - 64);
    ++h;
    cur = (cur < 64) ? __builtin_amdgcn_readlane(nxt[0], cur) : __builtin_amdgcn_readlane(nxt[1], cur - 64);
  }
  // ---- each envelope line other than R contributes its right edge P -> Q:
  //   (b_Q - b_P) psi(+-c), minus sign when the edge ends at or left of T.
  double v = 0.0;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    if (c * 64 >= nc) break;
    const bool on = (((c == 0) ? on0 : on1) >> lane) & 1;
    if (on && nxt[c] >= 0) {
      const double cc = cn[c] / cd[c];
      v += (cb[c] - pb[c]) * psi((cb[c] <= bT) ? -cc : cc);
    }
  }
  if (nhull) *nhull = h;
  return wave_sum(v);
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

template <int MAXL, int M>
__global__ __launch_bounds__(512) void envelope_kernel(const Plan* __restrict__ P, int B, double* __restrict__ kg,
                                                       double* __restrict__ pairs_out) {
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
  unsigned long long* st = kst_slot(P->debug_stamp, 2);
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
  KST(st, 2);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  DKG_STAMP(1);
  KST(st, 3);

  double* sb = sbuf + (size_t)wave * 2 * ENV_CAP;
  double* sa = sb + ENV_CAP;
  double wave_acc = 0.0;
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
    // unused output slots read output 0 with a zero weight.
    const double* mup[M];
#pragma unroll
    for (int i = 0; i < M; ++i) mup[i] = lmu + (size_t)((i < m) ? i : 0) * SLp + lane - 1;
    double la[MAXL], lb[MAXL];
    if (dbg & 16) {  // ablation: no line build (synthetic lines)
#pragma unroll
      for (int t = 0; t < MAXL; ++t) {
        la[t] = a_off * (double)(lane + t);
        lb[t] = wb[0] * (double)(lane - t);
      }
    } else if (full) {
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
    {  // padding lines beyond N: never maximal, never change min/max slope
      const double bfill = __shfl(lb[0], 0);
#pragma unroll
      for (int t = 0; t < MAXL; ++t) {
        const bool pad = lane + 64 * t > N;
        la[t] = pad ? -INFINITY : la[t];
        lb[t] = pad ? bfill : lb[t];
      }
    }
    DKG_STAMP(2);

    double kgj;
    if (dbg & 1) {  // ablation: lines + one reduction only
      double mxv = -INFINITY;
#pragma unroll
      for (int t = 0; t < MAXL; ++t) mxv = fmax(mxv, la[t] + lb[t]);
      kgj = wave_max(mxv);
    } else {
      kgj = envelope_kg<MAXL>(la, lb, NL, lane, sb, sa, nullptr);
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
    hipLaunchKernelGGL(cross_root_plan_kernel<DM>, grid, dim3(CR_WAVES * WAVE), lds, s, dev, xnew, B, kg);
    return hipGetLastError();
  }
  dim3 grid(std::max(1, pad16(h.N) / 16), pad16(B) / 16, h.m);
  hipLaunchKernelGGL(posterior_cov_kernel<DM>, grid, dim3(PC_WAVES * WAVE), 0, s, dev, xnew, B);
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

template <int MAXL, int M>
static hipError_t launch_env_t(const Plan* dev, int B, double* kg, double* pairs, dim3 grid, dim3 block, size_t lds,
                               hipStream_t s) {
  if (lds > 65536)
    (void)hipFuncSetAttribute((const void*)envelope_kernel<MAXL, M>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
  hipLaunchKernelGGL((envelope_kernel<MAXL, M>), grid, block, lds, s, dev, B, kg, pairs);
  return hipGetLastError();
}

template <int M>
static hipError_t launch_env_m(int lines, const Plan* dev, int B, double* kg, double* pairs, dim3 grid, dim3 block,
                               size_t lds, hipStream_t s) {
  if (lines <= 64 * 2) return launch_env_t<2, M>(dev, B, kg, pairs, grid, block, lds, s);
  if (lines <= 64 * 4) return launch_env_t<4, M>(dev, B, kg, pairs, grid, block, lds, s);
  if (lines <= 64 * 8) return launch_env_t<8, M>(dev, B, kg, pairs, grid, block, lds, s);
  if (lines <= 64 * 17) return launch_env_t<17, M>(dev, B, kg, pairs, grid, block, lds, s);
  if (lines <= 64 * 33) return launch_env_t<33, M>(dev, B, kg, pairs, grid, block, lds, s);
  return hipErrorInvalidValue;
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
  dim3 grid(B, h.split), block(h.sw * WAVE);
  const size_t lds = envelope_lds_bytes(h.m, h.N, h.sw, h.S);
  switch (outputs_bucket(h.m)) {
    case 1: return launch_env_m<1>(h.N + 1, dev, B, kg, pairs, grid, block, lds, s);
    case 2: return launch_env_m<2>(h.N + 1, dev, B, kg, pairs, grid, block, lds, s);
    case 3: return launch_env_m<3>(h.N + 1, dev, B, kg, pairs, grid, block, lds, s);
    case 4: return launch_env_m<4>(h.N + 1, dev, B, kg, pairs, grid, block, lds, s);
    default: return launch_env_m<8>(h.N + 1, dev, B, kg, pairs, grid, block, lds, s);
  }
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
