// HIP kernels of the Discrete-KG hot path for gfx950 (MI355X, CDNA4).
//
// Pipeline per forward (DESIGN.md "Kernels"):
//   cross_root_kernel   Q = K(x, X) R  (fp64 MFMA, R upper triangular), mean = c + K(x,X) alpha
//   posterior_cov_kernel cov[b][k] = s k(x_b, D_k) - Q_b . Q_D[k]   (fp64 MFMA GEMM, split-K)
//   envelope_kernel     lines a_k + b_k z per (candidate, scalarisation), upper
//                       envelope, closed-form Gaussian expectation, mean over S
#include "dkg_device.h"
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

// Element-type plumbing of the two contractions (T = double: the reference's
// fp64; T = float: DKG_PLAN_F32): accumulator vector, MFMA, fragment words.
template <class T> struct AccT;
template <> struct AccT<double> { typedef d4 type; };
template <> struct AccT<float> { typedef f4 type; };
__device__ __forceinline__ d4 mfma_t(double a, double b, d4 c) { return mfma_f64(a, b, c); }
__device__ __forceinline__ f4 mfma_t(float a, float b, f4 c) { return mfma_f32(a, b, c); }
// k-blocks per 16-byte fragment word
template <class T> constexpr int kpack() { return sizeof(T) == 8 ? 2 : 4; }
template <class T>
__host__ __device__ inline size_t fragT_index(int t, int kb, int l, int KB) {
  if constexpr (sizeof(T) == 8) return frag_index(t, kb, l, KB);
  else return frag32_index(t, kb, l, KB);
}
// Row of the 16x16 MFMA result held by lane l in accumulator register r.
template <class T>
__device__ __forceinline__ int mfma_drow(int l, int r) {
  if constexpr (sizeof(T) == 8) return (l >> 4) + 4 * r;
  else return 4 * (l >> 4) + r;
}
// lane's operands of the kpack<T>() k-blocks of word j of tile `tile` into out[0 ..)
template <class T>
__device__ __forceinline__ void frag_word(const T* __restrict__ base, int tile, int j, int lane, int KB, T* out) {
  if constexpr (sizeof(T) == 8) {
    const double2 v = frag_pair(base, tile, j, lane, KB);
    out[0] = v.x; out[1] = v.y;
  } else {
    const float4 v = frag_quad(base, tile, j, lane, KB);
    out[0] = v.x; out[1] = v.y; out[2] = v.z; out[3] = v.w;
  }
}

// ---------------------------------------------------------------------------
// cross_root_kernel: one workgroup per (16-row tile ti, group c of tile pairs,
// output).  A pair is (p, T-1-p) of 16-column tiles of Q = K_x R; R upper
// triangular means tile tj only needs k-blocks kb < 4(tj+1), so pairing the
// shortest with the longest tile balances the MFMA count.  Group c holds
// pairs CR_PAIRS c .. CR_PAIRS c + CR_PAIRS - 1: the training inputs are
// staged in LDS and the K(x, X) tile is evaluated once into LDS in B-operand
// order for the group's widest pair, then each pair's k range is split over
// the 8 waves (split-K) with every operand of a wave's chunk loaded before its
// MFMAs (the next pair's first batch is loaded while this pair's partials are
// reduced); partials are reduced in LDS in fixed wave order (deterministic).
// One pair per workgroup evaluates the kernel 6.25x over at n = 256 (the fill
// is half of a workgroup's lifetime), but four pairs per workgroup made the
// launch 11 us instead of 6 and lowered the forwards-in-flight throughput
// (10.46 M against 11.01 M KG-evals/s, profiles/r02/r02za): with a few
// forwards in flight the stage's latency, not its summed workgroup time,
// sets the rate.  CR_PAIRS stays a tuning constant.
#ifndef DKG_CR_WAVES
#define DKG_CR_WAVES 8
#endif
constexpr int CR_WAVES = DKG_CR_WAVES;
constexpr int CR_U = 8;      // k-blocks per load batch
constexpr int CR_PAIRS = 1;  // tile pairs per workgroup

// LDS (doubles): the K tile [KB][64], the pair partials (their own region when
// a workgroup reduces several pairs; else overlaying the K tile), the mean
// partials, the staged inputs and alpha.  Pairs per workgroup: CR_PAIRS when
// that fits the CU's 160 KiB, else 1 (large n with large d).
__host__ __device__ inline size_t cross_lds_doubles(int np, int d, bool sep) {
  const size_t kb = (size_t)(np / 4) * 64, pt = (size_t)CR_WAVES * 8 * 64;
  return (sep ? kb + pt : (kb > pt ? kb : pt)) + CR_WAVES * 16 + (size_t)np * d + np;
}
__host__ __device__ inline int cross_pairs(int np, int d) {
  return cross_lds_doubles(np, d, true) * sizeof(double) <= 160 * 1024 ? CR_PAIRS : 1;
}
__host__ __device__ inline int cross_groups(int np, int d) {
  return ((np / 16 + 1) / 2 + cross_pairs(np, d) - 1) / cross_pairs(np, d);
}

// GRAD: the same contraction with the kernel replaced by its derivative in
// the candidate's coordinate `gdim` (J = dK(x, X)/dx_g R, dmean = dK/dx_g alpha).
// T = float (DKG_PLAN_F32): R^T and Q in fp32 (quad-packed), fp32 MFMA; the
// kernel evaluations and the mean stay fp64.
// qx_rm (fp64 forward only): also write Q row-major [rows_pad][n_pad] (the gradient envelope's rows).
template <int DM, bool GRAD = false, class ET = double>
__device__ __forceinline__ void cross_root_impl(const dkg_output& o, int d, const double* __restrict__ x, int rows,
                                                ET* __restrict__ qout, double* __restrict__ mout, int ti, int grp,
                                                double* smem, unsigned long long* st = nullptr, int gdim = 0,
                                                const double* __restrict__ /*unused*/ = nullptr,
                                                double* __restrict__ qx_rm = nullptr,
                                                const ET* __restrict__ root = nullptr) {
  static_assert(!GRAD || sizeof(ET) == 8, "the gradient stage is fp64");
  constexpr int QW = kpack<ET>();
  if constexpr (sizeof(ET) == 8) root = o.root_frag;
  const int n = o.n;
  const int np = pad16(n);
  const int T = np / 16;
  const int KB = np / 4;
  const int P = (T + 1) / 2;
  const int ppg = cross_pairs(np, d);
  const int pb = grp * ppg, pe = min(P, pb + ppg);
  if (pb >= pe) return;
  const int kbW = 4 * (T - pb);           // k-block extent of the group's widest pair (its tile T-1-pb)
  const int ncol = min(n, 4 * kbW);       // training columns the group needs

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  ET* kb_lds = reinterpret_cast<ET*>(smem);     // [KB][64]
  const bool sep = ppg > 1;
  double* part = sep ? smem + KB * 64 : smem;   // [CR_WAVES][8][64] pair partials (cross_lds_doubles)
  double* mred = smem + (sep ? KB * 64 + CR_WAVES * 8 * 64 : max(KB * 64, CR_WAVES * 8 * 64));  // [CR_WAVES][16]
  double* xs = mred + CR_WAVES * 16;            // [np][d] staged training inputs
  double* als = xs + (size_t)np * d;            // [np] alpha

  // a pair's geometry for this wave: tiles, k-block extents, the wave's k chunk
  // (k-block ranges are even: kbA, kbB are multiples of 4 and chunk is even)
  struct PairK {
    int tA, tB, kbA, kbB, k0, k1;
  };
  auto pair_k = [&](int p) {
    PairK q;
    q.tA = p;
    q.tB = T - 1 - p;  // tA <= tB
    q.kbA = 4 * (q.tA + 1);
    q.kbB = 4 * (q.tB + 1);
    const int chunk = QW * ((q.kbB / QW + CR_WAVES - 1) / CR_WAVES);
    q.k0 = wave * chunk;
    q.k1 = min(q.kbB, q.k0 + chunk);
    return q;
  };
  ET ra[CR_U], rb[CR_U];
  auto load_batch = [&](const PairK& q, int base) {
#pragma unroll
    for (int u = 0; u < CR_U; u += QW) {
      const int j = min(base + u, q.kbB - QW) / QW;
      frag_word<ET>(root, q.tB, j, lane, KB, rb + u);
      frag_word<ET>(root, q.tA, min(j, q.kbA / QW - 1), lane, KB, ra + u);
    }
  };
  // R fragments of this wave's first k-block batch of the first pair: loaded
  // before anything else so their latency overlaps the staging and the fill.
  PairK cur = pair_k(pb);
  load_batch(cur, cur.k0);

  KST(st, 2);
  const bool want_mean = (mout != nullptr) && (pb == 0);  // pair 0 covers every column
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
  // ---- fill K(x_row, X_col), col < 4*kbW, in B-operand order (zero outside)
  double mpart = 0.0;
  const double os = o.outputscale;
  const double ilg = GRAD ? o.inv_lengthscale[gdim] : 1.0;
  double xg = 0.0;  // the candidate's pre-scaled coordinate gdim (GRAD)
#pragma unroll
  for (int k = 0; k < DM; ++k) xg = (k == gdim) ? xr[k] : xg;
  const int fill = kbW * 64;
  const int iters = (fill + CR_WAVES * WAVE - 1) / (CR_WAVES * WAVE);  // uniform trip count
  // one straight-line loop per covariance family (the switch stays outside)
  auto fill_loop = [&](auto kind_c) {
    constexpr int KIND = decltype(kind_c)::value;
    const const_dptr tab = psi_tab();
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
        kv = os * kernel_profile_t<KIND>(r2, tab);
      }
      const double v = (rv && col < n) ? kv : 0.0;
      const double al = als[cc];  // staged only when want_mean; otherwise ignored
      mpart = fma(v, want_mean ? al : 0.0, mpart);
      if (e < fill) kb_lds[e] = (ET)v;
    }
  };
  switch (o.kernel) {
    case DKG_MATERN12: fill_loop(std::integral_constant<int, DKG_MATERN12>{}); break;
    case DKG_MATERN32: fill_loop(std::integral_constant<int, DKG_MATERN32>{}); break;
    case DKG_RBF: fill_loop(std::integral_constant<int, DKG_RBF>{}); break;
    default: fill_loop(std::integral_constant<int, DKG_MATERN52>{}); break;
  }
  // mean partials: lanes l, l^16, l^32, l^48 share a row.
  if (want_mean) {
    mpart += partner_f64<4>(mpart);
    mpart += partner_f64<5>(mpart);
    if (lane < 16) mred[wave * 16 + lane] = mpart;
  }
  __syncthreads();

  KST(st, 4);
  typedef typename AccT<ET>::type acc_t;
  for (int p = pb; p < pe; ++p) {
    // ---- split-K MFMA over the pair, loads batched ahead of the MFMAs
    acc_t accA2[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
    acc_t accB2[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
    const bool pairA = cur.tA != cur.tB;
    for (int base = cur.k0; base < cur.k1; base += CR_U) {
      ET bo[CR_U];
      if (base != cur.k0) load_batch(cur, base);
#pragma unroll
      for (int u = 0; u < CR_U; ++u) {
        const int kb = min(base + u, cur.kbB - 1);
        bo[u] = (base + u < cur.k1) ? kb_lds[kb * 64 + lane] : (ET)0;
      }
#pragma unroll
      for (int u = 0; u < CR_U; ++u) {
        accB2[u & 1] = mfma_t(rb[u], bo[u], accB2[u & 1]);
        if (pairA && base + u < cur.kbA) accA2[u & 1] = mfma_t(ra[u], bo[u], accA2[u & 1]);
      }
    }
    const acc_t accA = accA2[0] + accA2[1];
    const acc_t accB = accB2[0] + accB2[1];
    const PairK done = cur;
    if (p + 1 < pe) {  // the next pair's first batch, in flight during this pair's reduction
      cur = pair_k(p + 1);
      load_batch(cur, cur.k0);
    }
    __syncthreads();  // every wave is done with the previous pair's partials (and, overlaid, with kb_lds)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      part[(wave * 8 + r) * 64 + lane] = (double)accA[r];
      part[(wave * 8 + 4 + r) * 64 + lane] = (double)accB[r];
    }
    __syncthreads();

    // ---- reduce partials in fixed wave order; wave w < 8 finalises (tile, reg) = w.
    const int tsel = wave >> 2;  // 0 -> tA, 1 -> tB
    const int r = wave & 3;
    if (wave < 8 && (tsel == 1 || pairA)) {
      double s = 0.0;
#pragma unroll
      for (int w = 0; w < CR_WAVES; ++w) s += part[(w * 8 + tsel * 4 + r) * 64 + lane];
      const int tj = tsel ? done.tB : done.tA;
      // D = R^T K^T: lane holds Q[16ti + (l&15)][16tj + 4r + (l>>4)] = q_frag[ti][4tj + r][l]
      if constexpr (GRAD) {
        // J row-major [bpad][np] for the envelope's per-candidate row loads;
        // the gdim == 0 workgroups also copy Q_X's matching entries row-major
        const size_t rm = (size_t)(16 * ti + (lane & 15)) * np + 16 * tj + 4 * r + (lane >> 4);
        qout[rm] = s;
      } else {
        // D row dr = column 16 tj + dr of Q: k-block 4 tj + dr/4, operand lane (l & 15) | (dr % 4) << 4
        const int dr = mfma_drow<ET>(lane, r);
        qout[fragT_index<ET>(ti, 4 * tj + (dr >> 2), (lane & 15) | ((dr & 3) << 4), KB)] = (ET)s;
        if constexpr (sizeof(ET) == 8)
          if (qx_rm) qx_rm[(size_t)(16 * ti + (lane & 15)) * np + 16 * tj + dr] = s;
      }
    }
  }
  KST(st, 5);
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
template <int DM, class T = double>
__global__ __launch_bounds__(CR_WAVES * WAVE) void cross_root_plan_kernel(const Plan* __restrict__ P,
                                                                          const double* __restrict__ xnew, int B,
                                                                          double* __restrict__ kg, int dst) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  unsigned long long* st = kst_slot(dst, P, 0);
  KST_BEGIN(st);
  const int oi = blockIdx.z;
  if (blockIdx.x == 0 && blockIdx.y == 0 && oi == 0) {
    for (int i = threadIdx.x; i < B; i += blockDim.x) {
      kg[i] = 0.0;
      P->tickets[i] = 0;
    }
  }
  if (DKG_ABLATIONS && (__builtin_amdgcn_readfirstlane(P->debug_cov) & 2)) return;  // ablation: empty cross stage
  if constexpr (sizeof(T) == 8) {
    cross_root_impl<DM>(P->o[oi], P->d, xnew, B, P->q[oi], P->mux[oi], blockIdx.x, blockIdx.y, smem, st);
  } else {
    cross_root_impl<DM, false, float>(P->o[oi], P->d, xnew, B, P->q32[oi], P->mux[oi], blockIdx.x, blockIdx.y, smem,
                                      st, 0, nullptr, nullptr, P->root32[oi]);
  }
}

// Value + gradient cross stage, one launch: grid (B tiles, pairs, m + m d).
// z < m: the forward cross stage of output z (Q_X fragment-packed and row-major, means; kg and the
// tickets cleared).  z >= m, z - m = oi d + g: J_g = dK(x, X)/dx_g R (row-major) and dmean/dx_g for
// output oi; the first of these workgroups clears the gradient accumulator dkg[B x d].  The two halves
// read only x and the state, so they run side by side in one launch (at B = 1 the value+gradient chain
// is latency-bound: one launch and one dependency gap fewer than two cross launches).
template <int DM>
__global__ __launch_bounds__(CR_WAVES * WAVE) void cross_fwd_grad_kernel(const Plan* __restrict__ P,
                                                                         const double* __restrict__ xnew, int B,
                                                                         double* __restrict__ kg,
                                                                         double* __restrict__ dkg, int dst) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  unsigned long long* st = kst_slot(dst, P, 0);
  const int m = P->m, d = P->d;
  const int z = blockIdx.z;
  if (z < m) {
    if (blockIdx.x == 0 && blockIdx.y == 0 && z == 0)
      for (int i = threadIdx.x; i < B; i += blockDim.x) {
        kg[i] = 0.0;
        P->tickets[i] = 0;
      }
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

// ---------------------------------------------------------------------------
// posterior_cov_kernel: cov[b][k] = s k(x_b, D_k) - sum_l Q[b][l] Q_D[k][l]
// One workgroup (8 waves, 2 per SIMD) per 32 x 32 block = 2 x 2 output
// tiles of one output; wave w computes tile (w % 4) over K part (w / 4) of
// PC_KS = 2.
// Waves that share an operand tile and a K-half read it at the same time, so
// a CU fetches each operand byte about once (L1); every load is a 16-byte
// pair (two k-blocks).  K parts meet in LDS in fixed order; the part-0
// wave evaluates the kernel epilogue and stores.  Tiles with tk == 0 also produce the
// candidates' own variances s - |Q_X[b]|^2.  At <= 128 VGPRs and 8 waves a
// block shares its CU with another block or an envelope workgroup (also 8
// waves at <= 128 VGPRs) of another forward in flight: 16 waves (K quarters,
// 4 per SIMD) kept the block's lifetime and took the CU alone, and lowered
// the forwards-in-flight throughput from 11.0 M to 9.0 M KG-evals/s
// (profiles/r02/r02zc); a 64 x 32 block of 16 waves likewise (r02x).
constexpr int PC_WAVES = 8;
constexpr int PC_RB = 2;  // 16-row tiles per workgroup (32 candidates); 2 column tiles (32 lines)
constexpr int PC_KS = PC_WAVES / (2 * PC_RB);  // K splits: the waves of one tile
constexpr int PC_P = 8;  // 16-byte words per operand per load batch (16 k-blocks)

// T = float (DKG_PLAN_F32): the contraction Q_X . Q_D in fp32 (quad-packed
// operands, v_mfma_f32_16x16x4_f32); the kernel term, the subtraction and the
// variance sums (of the fp32 Q_X entries) in fp64.
template <int DM, class T = double>
__global__ __launch_bounds__(PC_WAVES * WAVE) void posterior_cov_kernel(const Plan* __restrict__ P,
                                                                         const double* __restrict__ xnew, int B,
                                                                         int dst) {
  constexpr int QW = kpack<T>();
  typedef typename AccT<T>::type acc_t;
  constexpr int NT = 2 * PC_RB;  // output tiles per workgroup
  __shared__ __attribute__((aligned(16))) double part[(PC_KS - 1) * NT * 4 * 64];  // K-split 1.. partial tiles
  __shared__ double qpart[(PC_KS - 1) * NT * 16];
  unsigned long long* st = kst_slot(dst, P, 1);
  if (DKG_ABLATIONS && (__builtin_amdgcn_readfirstlane(P->debug_cov) & 1)) return;  // ablation: empty covariance stage
  KST_BEGIN(st);
  const int oi = blockIdx.z;
  const dkg_output& o = P->o[oi];
  const int N = P->N;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tt = wave % NT, ks = wave / NT;
  const int ti = PC_RB * blockIdx.y + (tt >> 1);
  const int tk = 2 * blockIdx.x + (tt & 1);
  const int KB = pad16(o.n) / 4;
  const bool have_d = N > 0;
  // tiles that exist in the workspace / state buffers (wave-uniform)
  const bool live = ti * 16 < pad16(B) && (tk * 16 < pad16(N) || (tk == 0 && !have_d));
  const bool want_var = tk == 0;
  // K part of this wave, in whole 16-byte words (QW k-blocks each)
  const int KP = KB / QW;
  const int KPs = (KP + PC_KS - 1) / PC_KS;
  const int p0 = min(KP, ks * KPs), p1 = min(KP, p0 + KPs);
  const T* qx;
  const T* qd;
  if constexpr (sizeof(T) == 8) {
    qx = P->q[oi];
    qd = o.disc_frag;
  } else {
    qx = P->q32[oi];
    qd = P->disc32[oi];
  }

  // The first batch of contraction operands is loaded first and the epilogue's
  // inputs after it, so both memory round trips overlap (row b = 16 ti + (l >> 4) + 4 r,
  // column k = 16 tk + (l & 15)).
  const int d = P->d;
  const int k = tk * 16 + (lane & 15);
  // disc_frag tile 0 exists only when N == 0: the N == 0 variance-only
  // wave reads its own Q_X tile as a stand-in (multiplied by 0 below)
  const T* dsrc = have_d ? qd : qx;
  const int dt = have_d ? tk : ti;
  T va[PC_P][QW], vd[PC_P][QW];
  auto load_batch = [&](int pb) {
#pragma unroll
    for (int u = 0; u < PC_P; ++u) {
      const int j = min(pb + u, p1 - 1);
      frag_word<T>(qx, ti, j, lane, KB, va[u]);
      frag_word<T>(dsrc, dt, j, lane, KB, vd[u]);
    }
  };
  // The epilogue's kernel terms s k(x_b, D_k), evaluated by the K-part-0 waves before the
  // contraction: their VALU work overlaps the K-part-1 waves' MFMAs on the same SIMDs (splitting
  // the terms over both parts overlapped nothing and lengthened the block: profiles/r02/r02zm).
  // At small d (EPI_FIRST) their inputs are loaded ahead of the first operand batch: loads
  // complete in order, so the terms' wait does not include the batch and their VALU work overlaps
  // its round trip.  At larger d the inputs would stay live beside the batch (over 128 VGPRs).
  constexpr bool EPI_FIRST = DM <= 2;
  constexpr int RV = 4;
  const bool epi = ks == 0;  // wave-uniform
  // line k's coordinates (P->disc is valid even when N == 0: plan init)
  auto disc_row = [&]() { return P->disc + (size_t)min(k, max(N, 1) - 1) * d; };
  double ek[EPI_FIRST ? DM : 1], eb[RV][EPI_FIRST ? DM : 1];
  if (EPI_FIRST && epi) {
    const double* xk = disc_row();
#pragma unroll
    for (int c = 0; c < DM; ++c) {
      ek[c] = xk[min(c, d - 1)];
#pragma unroll
      for (int rr = 0; rr < RV; ++rr)
        eb[rr][c] = xnew[(size_t)min(ti * 16 + mfma_drow<T>(lane, rr), B - 1) * d + min(c, d - 1)];
    }
  }
  if (live && p0 < p1) load_batch(p0);
  double kv[RV] = {};
  if (epi) {
    const double os = o.outputscale;
    const int kind = o.kernel;
    const const_dptr tab = psi_tab();
#pragma unroll
    for (int rr = 0; rr < RV; ++rr) {
      double r2;
      if constexpr (EPI_FIRST) {
        r2 = 0.0;  // scaled_r2_dm's arithmetic on the preloaded inputs
#pragma unroll
        for (int c = 0; c < DM; ++c) {
          const double t = (eb[rr][c] - ek[c]) * o.inv_lengthscale[min(c, d - 1)];
          r2 = fma(t, (c < d) ? t : 0.0, r2);
        }
      } else {
        const int b = ti * 16 + mfma_drow<T>(lane, rr);
        r2 = scaled_r2_dm<DM>(xnew + (size_t)min(b, B - 1) * d, disc_row(), o.inv_lengthscale, d);
      }
      kv[rr] = os * kernel_profile(kind, r2, EPI_FIRST ? tab : psi_tab());
    }
  }
  KST(st, 2);
  acc_t acc[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
  double qsq = 0.0;  // lane l: sum over this wave's k of Q_X[16 ti + (l & 15)][k]^2
  if (live) {
    for (int pb = p0; pb < p1; pb += PC_P) {
      if (pb != p0) load_batch(pb);
#pragma unroll
      for (int u = 0; u < PC_P; ++u) {
        const bool in = pb + u < p1 && have_d;
#pragma unroll
        for (int q = 0; q < QW; ++q) {
          const T a = va[u][q], dd = in ? vd[u][q] : (T)0;
          acc[(QW * u + q) & 3] = mfma_t(a, dd, acc[(QW * u + q) & 3]);
          if (want_var) qsq = (pb + u < p1) ? fma((double)a, (double)a, qsq) : qsq;
        }
      }
    }
  }
  const acc_t accs = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  KST(st, 3);
  if (want_var) {
    qsq += __shfl_xor(qsq, 16);
    qsq += __shfl_xor(qsq, 32);
  }
  if (ks > 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) part[(((ks - 1) * NT + tt) * 4 + r) * 64 + lane] = (double)accs[r];
    if (want_var && lane < 16) qpart[((ks - 1) * NT + tt) * 16 + lane] = qsq;
  }
  __syncthreads();
  KST(st, 4);
  if (ks == 0 && live) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      double sum = (double)accs[r];
#pragma unroll
      for (int q = 0; q < PC_KS - 1; ++q) sum += part[((q * NT + tt) * 4 + r) * 64 + lane];  // fixed order
      const int b = ti * 16 + mfma_drow<T>(lane, r);
      if (b < B && k < N)  // line record k of candidate b, component oi (dkg_device.h cov_rec)
        P->cov_all[(size_t)b * P->cov_stride + (size_t)k * cov_rec(P->m) + oi] = kv[r] - sum;
    }
    if (want_var && lane < 16) {
      const int bb = ti * 16 + lane;
      double qs = qsq;
#pragma unroll
      for (int q = 0; q < PC_KS - 1; ++q) qs += qpart[(q * NT + tt) * 16 + lane];
      if (bb < B) P->var[oi][bb] = o.outputscale - qs;
    }
  }
  KST_END(st);
}

static int outputs_bucket(int m) { return m <= 1 ? 1 : m <= 2 ? 2 : m <= 3 ? 3 : m <= 4 ? 4 : 8; }

size_t envelope_lds_bytes(int m, int N, int waves, int S, bool stream, bool grad) {
  const int M = outputs_bucket(m);
  const size_t staged = stream ? 0 : 2 * (size_t)stage_stride(N, cov_rec(M));
  const bool refine = stream && !grad;  // streaming forward: long lists + quickhull vertex arrays
  const size_t lc = list_cap(refine);
  // per wave: the list (slopes, intercepts; forward: line indices) and the streaming vertex arrays
  return ((size_t)2 + staged + ((S * m + 1) & ~1) + ((S + 1) & ~1) + (size_t)waves * 2 * lc + (refine ? (size_t)waves * VREG : 0) +
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

template <int DM, class T>
static hipError_t launch_cross_cov_tt(const Plan& h, const Plan* dev, const double* xnew, int B, double* kg,
                                      hipStream_t s, int stage) {
  if (stage == 0) {
    dim3 grid(pad16(B) / 16, cross_groups(h.max_np, h.d), h.m);
    const size_t lds = cross_root_lds_bytes(h.max_np, h.d);
    if (lds > 65536)
      (void)hipFuncSetAttribute((const void*)cross_root_plan_kernel<DM, T>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((cross_root_plan_kernel<DM, T>), grid, dim3(CR_WAVES * WAVE), lds, s, dev, xnew, B, kg,
                       h.debug_stamp);
    return hipGetLastError();
  }
  dim3 grid(std::max(1, (h.N + 31) / 32), (B + 16 * PC_RB - 1) / (16 * PC_RB), h.m);
  hipLaunchKernelGGL((posterior_cov_kernel<DM, T>), grid, dim3(PC_WAVES * WAVE), 0, s, dev, xnew, B, h.debug_stamp);
  return hipGetLastError();
}

template <int DM>
static hipError_t launch_cross_cov_t(const Plan& h, const Plan* dev, const double* xnew, int B, double* kg,
                                     hipStream_t s, int stage) {
  return h.f32 ? launch_cross_cov_tt<DM, float>(h, dev, xnew, B, kg, s, stage)
               : launch_cross_cov_tt<DM, double>(h, dev, xnew, B, kg, s, stage);
}

void envelope_geometry(int B, int S, int* waves_per_wg, int* split) {
  // Up to 8 scalarisation waves of one candidate per workgroup, one pair per
  // wave; with S <= 16 at most two workgroups per candidate, whose partial
  // sums meet in one commutative atomic add (no inter-workgroup fences).
  (void)B;
  const int sw = std::max(1, std::min(8, S));
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
                        hipStream_t s, int stage) {
  if (stage == 0 || stage == 1) {
    switch (dim_bucket(h.d)) {
      case 2: return launch_cross_cov_t<2>(h, dev, xnew, B, kg, s, stage);
      case 4: return launch_cross_cov_t<4>(h, dev, xnew, B, kg, s, stage);
      case 8: return launch_cross_cov_t<8>(h, dev, xnew, B, kg, s, stage);
      default: return launch_cross_cov_t<16>(h, dev, xnew, B, kg, s, stage);
    }
  }
  EnvLaunch a{&h, dev, B, kg, pairs, dim3(B, h.split), dim3(h.sw * WAVE),
              envelope_lds_bytes(h.m, h.N, h.sw, h.S, h.stream != 0), s, h.debug_stamp, nullptr, nullptr};
  return launch_env<false>(h, a);
}

template <int DM>
static hipError_t launch_cross_fwd_grad_t(const Plan& h, const Plan* dev, const double* xnew, int B, double* kg,
                                          double* dkg, hipStream_t s) {
  dim3 grid(pad16(B) / 16, cross_groups(h.max_np, h.d), h.m * (1 + h.d));
  const size_t lds = cross_root_lds_bytes(h.max_np, h.d);
  if (lds > 65536)
    (void)hipFuncSetAttribute((const void*)cross_fwd_grad_kernel<DM>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
  hipLaunchKernelGGL(cross_fwd_grad_kernel<DM>, grid, dim3(CR_WAVES * WAVE), lds, s, dev, xnew, B, kg, dkg,
                     h.debug_stamp);
  return hipGetLastError();
}

hipError_t launch_forward_grad(const Plan& h, const Plan* dev, const double* xnew, int B, double* kg, double* dkg,
                               hipStream_t s) {
  hipError_t e;
  switch (dim_bucket(h.d)) {  // Q_X (fragment + row-major), means, J_g, dmean; kg = dkg = 0
    case 2: e = launch_cross_fwd_grad_t<2>(h, dev, xnew, B, kg, dkg, s); break;
    case 4: e = launch_cross_fwd_grad_t<4>(h, dev, xnew, B, kg, dkg, s); break;
    case 8: e = launch_cross_fwd_grad_t<8>(h, dev, xnew, B, kg, dkg, s); break;
    default: e = launch_cross_fwd_grad_t<16>(h, dev, xnew, B, kg, dkg, s); break;
  }
  if (e != hipSuccess) return e;
  if ((e = launch_stage(h, dev, xnew, B, kg, nullptr, s, 1)) != hipSuccess) return e;  // cov rows, variances
  EnvLaunch a{&h, dev, B, kg, nullptr, dim3(B, h.split), dim3(h.sw * WAVE),
              envelope_grad_lds_bytes(h.m, h.N, h.sw, h.S, h.d, h.max_np, h.stream != 0), s, h.debug_stamp, xnew, dkg};
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
