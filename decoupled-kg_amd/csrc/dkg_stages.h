// The two contraction stages of the Discrete-KG forward as device functions (gfx950):
// cross_root_impl (Q_X = K(x, X) R, the means) and posterior_cov_body (the covariance
// rows), shared by their own kernels (dkg_kernels.hip) and by the fused one-launch
// forward (dkg_fused.h).
#pragma once

#include "dkg_device.h"

#ifndef DKG_DUP_MARK  // A/B only: 0 drops the coincidence marks of the staged covariance (Plan::dup)
#define DKG_DUP_MARK 1
#endif

namespace dkg {

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
constexpr int KF_WAVES = 4;
#ifndef DKG_KF_KB
#define DKG_KF_KB 16
#endif
constexpr int KF_KB = DKG_KF_KB;  // k-blocks (of 4 columns) per fill workgroup

// Pre-scaled r^2 and the kernel term exactly as cross_root_impl's fill evaluates them (same operations,
// same order), so a loaded entry is the bits the fill would have produced.  Compiled without FP contraction
// (kernel_term_nc): with contraction the compiler fused differently in the fill loop and in cross_kfill_body's
// unrolled terms, and the two gave different bits.
template <int DM, int KIND>
__device__ __forceinline__ double cross_kernel_term(const double (&xr)[DM], const double* __restrict__ xs_col, int d,
                                                    double os, const_dptr tab) {
#pragma clang fp contract(off)
  double r2 = 0.0;
#pragma unroll
  for (int k = 0; k < DM; ++k) {
    const double t = xr[k] - xs_col[min(k, d - 1)];
    r2 = fma(t, (k < d) ? t : 0.0, r2);
  }
  return os * kernel_term_nc<KIND>(r2, tab);
}

// K(x_b, X_j) of output o for a row tile ti and KF_KB k-blocks, in the cross stage's B-operand order, pair-packed
// (frag_index: row 16 ti + (l & 15), column 4 kb + (l >> 4); the k-blocks 2 j, 2 j + 1 of a lane in one 16-byte
// word, as R^T's fragments, so cross_big_kernel stages both operands alike); zero outside B x n.
// kx32 (nullable, F32 plans): the same entries rounded to fp32 and quad-packed (frag32_index), cross_big32's B operand.
template <int DM>
__device__ __forceinline__ void cross_kfill_body(const dkg_output& o, int d, const double* __restrict__ x, int rows,
                                                 double* __restrict__ kx, int ti, int kb0,
                                                 float* __restrict__ kx32 = nullptr) {
  const int n = o.n;
  const int KB = pad16(n) / 4;
  const int lane = threadIdx.x & 63;
  const int row = ti * 16 + (lane & 15);
  const bool rv = row < rows;
  const int rowc = min(row, rows - 1);
  double xr[DM];
#pragma unroll
  for (int k = 0; k < DM; ++k) {
    const int kk = min(k, d - 1);
    xr[k] = x[(size_t)rowc * d + kk] * o.inv_lengthscale[kk];
  }
  const double os = o.outputscale;
  // the plan's fields and every training input this thread needs, read before the first store: a store into
  // kx may alias the plan for the compiler, which then re-read the pointers and the inputs after every store
  // (one dependent round trip per k-block: 7 us for a launch of a few hundred thousand entries)
  const double* __restrict__ txp = o.train_x;
  double il[DM];
#pragma unroll
  for (int k = 0; k < DM; ++k) il[k] = o.inv_lengthscale[min(k, d - 1)];
  constexpr int KPT = KF_KB / KF_WAVES;  // k-blocks per thread
  const int kbw = kb0 + (int)(threadIdx.x >> 6);
  double xs[KPT][DM];
#pragma unroll
  for (int q = 0; q < KPT; ++q) {
    const int cc = min(4 * (kbw + KF_WAVES * q) + (lane >> 4), n - 1);
#pragma unroll
    for (int k = 0; k < DM; ++k) {
      xs[q][k] = txp[(size_t)cc * d + min(k, d - 1)] * il[k];
      asm volatile("" : "+v"(xs[q][k]));  // rounded, as cross_root_impl's LDS copy (no fma into the difference)
    }
  }
  auto fill = [&](auto kind_c) {
    constexpr int KIND = decltype(kind_c)::value;
    const const_dptr tab = psi_tab();
    double kv[KPT];
#pragma unroll
    for (int q = 0; q < KPT; ++q) kv[q] = cross_kernel_term<DM, KIND>(xr, xs[q], d, os, tab);
#pragma unroll
    for (int q = 0; q < KPT; ++q) {
      const int kb = kbw + KF_WAVES * q;
      const int col = 4 * kb + (lane >> 4);
      if (kb < min(KB, kb0 + KF_KB)) {
        const double v = (rv && col < n) ? kv[q] : 0.0;
        kx[frag_index(ti, kb, lane, KB)] = v;
        if (kx32) kx32[frag32_index(ti, kb, lane, KB)] = (float)v;
      }
    }
  };
  switch (o.kernel) {
    case DKG_MATERN12: fill(std::integral_constant<int, DKG_MATERN12>{}); break;
    case DKG_MATERN32: fill(std::integral_constant<int, DKG_MATERN32>{}); break;
    case DKG_RBF: fill(std::integral_constant<int, DKG_RBF>{}); break;
    default: fill(std::integral_constant<int, DKG_MATERN52>{}); break;
  }
}

// WT: the forward's Q_X / mean stores write-through (sc1), for the fused forward's hand-off (st_out).
// GRAD: the same contraction with the kernel replaced by its derivative in
// the candidate's coordinate `gdim` (J = dK(x, X)/dx_g R, dmean = dK/dx_g alpha).
// T = float (DKG_PLAN_F32): R^T and Q in fp32 (quad-packed), fp32 MFMA; the
// kernel evaluations and the mean stay fp64.
// qx_rm (fp64 forward only): also write Q row-major [rows_pad][n_pad] (the gradient envelope's rows).
template <int DM, bool GRAD = false, class ET = double, bool WT = false>
__device__ __forceinline__ void cross_root_impl(const dkg_output& o, int d, const double* __restrict__ x, int rows,
                                                ET* __restrict__ qout, double* __restrict__ mout, int ti, int grp,
                                                double* smem, unsigned long long* st = nullptr, int gdim = 0,
                                                const double* __restrict__ kx = nullptr,
                                                double* __restrict__ qx_rm = nullptr,
                                                const ET* __restrict__ root = nullptr) {
  // kx (forward, large n): K(x, X) of this output filled by cross_kfill_kernel, loaded instead of evaluated
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
  if (kx == nullptr)
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
      double kv;
      if constexpr (GRAD) {
        double r2 = 0.0;
#pragma unroll
        for (int k = 0; k < DM; ++k) {
          const double t = xr[k] - xs[(size_t)cc * d + min(k, d - 1)];
          r2 = fma(t, (k < d) ? t : 0.0, r2);
        }
        kv = os * kernel_dprofile_t<KIND>(r2) * (xg - xs[(size_t)cc * d + gdim]) * ilg;
      } else if constexpr (KIND < 0) {
        kv = kx[frag_index(ti, min(e >> 6, KB - 1), lane, KB)];  // zero outside B x n (e & 63 == lane)
      } else {
        kv = cross_kernel_term<DM, KIND>(xr, xs + (size_t)cc * d, d, os, tab);
      }
      const double v = (rv && col < n) ? kv : 0.0;
      const double al = als[cc];  // staged only when want_mean; otherwise ignored
      mpart = fma(v, want_mean ? al : 0.0, mpart);
      if (e < fill) kb_lds[e] = (ET)v;
    }
  };
  if (!GRAD && kx != nullptr) {
    fill_loop(std::integral_constant<int, -1>{});  // K(x, X) from cross_kfill_kernel
  } else {
    switch (o.kernel) {
      case DKG_MATERN12: fill_loop(std::integral_constant<int, DKG_MATERN12>{}); break;
      case DKG_MATERN32: fill_loop(std::integral_constant<int, DKG_MATERN32>{}); break;
      case DKG_RBF: fill_loop(std::integral_constant<int, DKG_RBF>{}); break;
      default: fill_loop(std::integral_constant<int, DKG_MATERN52>{}); break;
    }
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
        st_out<WT>(&qout[fragT_index<ET>(ti, 4 * tj + (dr >> 2), (lane & 15) | ((dr & 3) << 4), KB)], (ET)s);
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
    st_out<WT>(&mout[rr], (rr < rows) ? (GRAD ? s : o.mean_constant + s) : 0.0);
  }
  KST_END(st);
}

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
template <int DM, class T = double, bool HO = false>
__device__ __forceinline__ void posterior_cov_body(const Plan* __restrict__ P, const double* __restrict__ xnew, int B,
                                                   int bx, int by, int oi, double* part, double* qpart,
                                                   unsigned long long* st, const Handoff* ho = nullptr) {
  constexpr int QW = kpack<T>();
  typedef typename AccT<T>::type acc_t;
  constexpr int NT = 2 * PC_RB;  // output tiles per workgroup
  KST_BEGIN(st);
  const dkg_output& o = P->o[oi];
  const int N = P->N;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tt = wave % NT, ks = wave / NT;
  const int ti = PC_RB * by + (tt >> 1);
  const int tk = 2 * bx + (tt & 1);
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
  // column k = 16 tk + (l & 15)).  HO (fused forward): Q_X is handed off by the cross
  // workgroups of this launch, so only Q_D's first batch is loaded ahead; Q_X after the wait.
  const int d = P->d;
  const int k = tk * 16 + (lane & 15);
  // disc_frag tile 0 exists only when N == 0: the N == 0 variance-only
  // wave reads its own Q_X tile as a stand-in (multiplied by 0 below)
  const T* dsrc = have_d ? qd : qx;
  const int dt = have_d ? tk : ti;
  T va[PC_P][QW], vd[PC_P][QW];
  auto load_x = [&](int pb) {
#pragma unroll
    for (int u = 0; u < PC_P; ++u) frag_word<T>(qx, ti, min(pb + u, p1 - 1), lane, KB, va[u]);
  };
  auto load_d = [&](int pb) {
#pragma unroll
    for (int u = 0; u < PC_P; ++u) frag_word<T>(dsrc, dt, min(pb + u, p1 - 1), lane, KB, vd[u]);
  };
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
  if constexpr (HO) {
    if (live && p0 < p1) load_d(p0);
  } else {
    if (live && p0 < p1) load_batch(p0);
  }
  double kv[RV] = {};
  // r^2 = 0: discretisation point k coincides with candidate b (Plan::dup).  The wave's hits are held as
  // lane masks in SGPRs across the contraction (a per-lane mark took the kernel past 128 VGPRs) and
  // marked with the stores (the fused launch: after its wait for the cross workgroups, one of which clears
  // the marks of these candidates)
  uint64_t hm[RV] = {};
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
      kv[rr] = os * kernel_term_nc(kind, r2, EPI_FIRST ? tab : psi_tab());
      // rounded here, never fused into the epilogue's subtraction: posterior_cov_big_kernel gives the same bits
      asm("" : "+v"(kv[rr]));
      if (DKG_DUP_MARK) hm[rr] = ballot(r2 == 0.0);
    }
  }
  if constexpr (HO) {
    // Q_X of this block's row tiles (cross workgroups of this launch): both tiles' arrivals, then one acquire
    const int rt0 = PC_RB * by;
    const int nrt = min(PC_RB, pad16(B) / 16 - rt0);
    handoff_wait(ho->cnt1 + ((size_t)oi * ho->rt + rt0) * HANDOFF_STRIDE, nrt, ho->quota1, ho->err, 1);
    if (live && p0 < p1) load_x(p0);
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
      if (b < B && k < N) {  // line record k of candidate b, component oi (dkg_device.h cov_rec)
        st_out<HO>(&P->cov_all[(size_t)b * P->cov_stride + (size_t)k * cov_rec(P->m) + oi], kv[r] - sum);
        if (hm[r] != 0 && ((hm[r] >> lane) & 1)) atomicMin(&P->dup[b], k);  // rare (wave-uniform test first)
      }
    }
    if (want_var && lane < 16) {
      const int bb = ti * 16 + lane;
      double qs = qsq;
#pragma unroll
      for (int q = 0; q < PC_KS - 1; ++q) qs += qpart[(q * NT + tt) * 16 + lane];
      if (bb < B) st_out<HO>(&P->var[oi][bb], o.outputscale - qs);
    }
  }
  if constexpr (HO) handoff_publish(ho->cnt2 + (size_t)by * HANDOFF_STRIDE);  // this block's cov_all / var rows are out
  KST_END(st);
}

// ---------------------------------------------------------------------------
// posterior_cov_wide_kernel (fp64, d <= 4, large B x N, e.g. BASELINE configs[4]): the same covariance rows from
// 64 x 64 blocks.  At 32 x 32 every operand byte feeds 32 flops: the stress shape's 3072 blocks read
// 1.5 GB of Q_X / Q_D tiles through L2 and the MALL (Q_D 96 MB), about what the MFMAs take.  Here wave w
// computes a 2 x 2 group of 16 x 16 tiles (row half (w & 3) >> 1, column half w & 1) over K part w >> 2:
// every 16-byte operand load feeds four MFMAs instead of two, and a block reads half the bytes per flop.
// The parts meet in LDS, each finalising one row tile of its group (deterministic: a sum of two commutes);
// the kernel terms of the 8 outputs per lane are evaluated there and stored.  One
// accumulator per tile (posterior_cov_kernel keeps four per tile, by k-block mod 4), so the sums agree
// with it to rounding, not bit for bit.
constexpr int PW_WAVES = 8;
constexpr int PW_KS = 2;  // K parts
constexpr int PW_P = 4;   // 16-byte words per operand tile per load batch

template <int DM>
__global__ __launch_bounds__(PW_WAVES * WAVE) __attribute__((amdgpu_waves_per_eu(4))) void posterior_cov_wide_kernel(const Plan* __restrict__ P,
                                                                             const double* __restrict__ xnew,
                                                                             int B, int dst) {
  __shared__ __attribute__((aligned(16))) double part[2 * 4 * 2 * 4 * 64];  // [row tile][sub-block][col tile] sums
  __shared__ double qpart[2 * 4 * 16];                                      // [row tile][sub-block] |Q_X|^2 sums
  // 1-D grid, the outputs of one 64 x 64 block side by side on one XCD (xcd_group)
  const int N = P->N;
  const int nbx = (N + 63) / 64, nby = (B + 63) / 64;
  int blk, oi;
  if (!xcd_group(blockIdx.x, nbx * nby, P->m, blk, oi)) return;
  unsigned long long* st = kst_slot(dst, P, 1);
  KST_BEGIN(st);
  const int bx = blk % nbx, by = blk / nbx;
  const dkg_output& o = P->o[oi];
  const int d = P->d;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int sb = wave & 3, ks = wave >> 2;
  const int ti0 = 4 * by + 2 * (sb >> 1);  // row tiles ti0, ti0 + 1
  const int tk0 = 4 * bx + 2 * (sb & 1);   // column tiles tk0, tk0 + 1
  const int RT = pad16(B) / 16, CT = pad16(N) / 16;  // tiles that exist
  const int KB = pad16(o.n) / 4;
  const int KP = KB / 2;  // 16-byte words (two k-blocks each)
  const int KPs = (KP + PW_KS - 1) / PW_KS;
  const int p0 = min(KP, ks * KPs), p1 = min(KP, p0 + KPs);
  const double* qx = P->q[oi];
  const double* qd = o.disc_frag;
  // dead tiles read a live one (results discarded)
  const int tr[2] = {min(ti0, RT - 1), min(ti0 + 1, RT - 1)};
  const int tc[2] = {min(tk0, CT - 1), min(tk0 + 1, CT - 1)};
  const bool want_var = (tk0 == 0);  // this wave's column tiles include tile 0: the row tiles' variances
  double va[PW_P][2][2], vd[PW_P][2][2];
  auto load_batch = [&](int pb) {
#pragma unroll
    for (int u = 0; u < PW_P; ++u) {
      const int j = min(pb + u, p1 - 1);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        frag_word<double>(qx, tr[h], j, lane, KB, va[u][h]);
        frag_word<double>(qd, tc[h], j, lane, KB, vd[u][h]);
      }
    }
  };
  if (p0 < p1) load_batch(p0);
  KST(st, 2);
  d4 acc[2][2] = {{{0, 0, 0, 0}, {0, 0, 0, 0}}, {{0, 0, 0, 0}, {0, 0, 0, 0}}};
  double qsq[2] = {0.0, 0.0};  // lane l: this wave's sum of Q_X[16 tr[h] + (l & 15)][k]^2
  for (int pb = p0; pb < p1; pb += PW_P) {
    if (pb != p0) load_batch(pb);
#pragma unroll
    for (int u = 0; u < PW_P; ++u) {
      const bool in = pb + u < p1;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
#pragma unroll
        for (int hr = 0; hr < 2; ++hr) {
          const double a = va[u][hr][q];
#pragma unroll
          for (int hc = 0; hc < 2; ++hc) acc[hr][hc] = mfma_f64(a, in ? vd[u][hc][q] : 0.0, acc[hr][hc]);
          if (want_var) qsq[hr] = in ? fma(a, a, qsq[hr]) : qsq[hr];
        }
      }
    }
  }
  KST(st, 3);
  if (want_var) {
#pragma unroll
    for (int hr = 0; hr < 2; ++hr) {
      qsq[hr] += __shfl_xor(qsq[hr], 16);
      qsq[hr] += __shfl_xor(qsq[hr], 32);
    }
  }
  // The two K parts exchange halves: part ks finalises row tile hr = ks of its 2 x 2 group and hands the
  // other row tile's sums to the other part (LDS), so both halves of the workgroup share the epilogue.
  {
    const int ho = 1 - ks;  // the row tile handed over
#pragma unroll
    for (int hc = 0; hc < 2; ++hc)
#pragma unroll
      for (int r = 0; r < 4; ++r) part[(((ho * 4 + sb) * 2 + hc) * 4 + r) * 64 + lane] = acc[ho][hc][r];
    if (want_var && lane < 16) qpart[(ho * 4 + sb) * 16 + lane] = qsq[ho];
  }
  __syncthreads();
  KST(st, 4);
  {
    // the kernel terms s k(x_b, D_k) here, after the contraction: held across it they took the block
    // past 128 VGPRs (one block per CU instead of two)
    const int hr = ks;
    const int rec = cov_rec(P->m);
    const double os = o.outputscale;
    const int kind = o.kernel;
#pragma unroll
    for (int hc = 0; hc < 2; ++hc) {
      const int k = 16 * (tk0 + hc) + (lane & 15);
      const double* xk = P->disc + (size_t)min(k, max(N, 1) - 1) * d;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        // K part 0 + K part 1 (fp addition commutes: the same bits whichever part adds)
        const double sum = acc[hr][hc][r] + part[(((hr * 4 + sb) * 2 + hc) * 4 + r) * 64 + lane];
        const int b = 16 * (ti0 + hr) + mfma_drow<double>(lane, r);
        const double r2 = scaled_r2_dm<DM>(xnew + (size_t)min(b, B - 1) * d, xk, o.inv_lengthscale, d);
        const double kv = os * kernel_profile(kind, r2);
        if (b < B && k < N) {
          P->cov_all[(size_t)b * P->cov_stride + (size_t)k * rec + oi] = kv - sum;
          if (r2 == 0.0) atomicMin(&P->dup[b], k);  // Plan::dup
        }
      }
    }
    if (want_var && lane < 16) {
      const int bb = 16 * (ti0 + hr) + lane;
      if (bb < B) P->var[oi][bb] = o.outputscale - (qsq[hr] + qpart[(hr * 4 + sb) * 16 + lane]);
    }
  }
  KST_END(st);
}

// ---------------------------------------------------------------------------
// posterior_cov_big_kernel (fp64): the covariance rows of launches over many candidates (forward batches in
// one launch, dkg_plan_forward_batches; the stress shape) with posterior_cov_kernel's arithmetic element for
// element, so the two give the same bits and the choice between them is a speed matter only.
// posterior_cov_kernel sums each element as two K halves (words [0, KPs) and [KPs, KP)), each over four
// chains of k-blocks (k-block index from the half's start mod 4, in increasing order), combined
// (c0 + c1) + (c2 + c3), then half 0 + half 1; its variance sums likewise per half (lane-wise FMAs in k order,
// then the xor-16 / xor-32 exchange), half 0 + half 1.  At 32 x 32 blocks every 16-byte operand load feeds two
// MFMAs and the L1 path, not the MFMA, sets the rate once a launch fills the device (37 % of the fp64 roof
// at 20 headline batches).  Here a workgroup of 4 waves (one per SIMD; two workgroups per CU, so one's
// epilogue and chunk barriers overlap the other's MFMAs) owns a 64 x 64 block (4 candidate tiles x 4 line
// tiles of one output); the operand tiles are staged once per workgroup through LDS in
// chunks of PB_WC words by LDS-DMA (PB_NSTG = 2 buffers: the next chunk in flight during the current one's MFMAs),
// and each wave computes a 2 x 2 group of tiles over both halves in turn (16 accumulator chains),
// reading its fragments from LDS with one 16-byte read per two MFMAs per operand tile.
// 16 bytes from global memory by a global_load (address space 1), not a flat load.
__device__ __forceinline__ double2 gload_d2(const double* p) {
  typedef double v2 __attribute__((ext_vector_type(2)));
  const v2 v = *reinterpret_cast<const __attribute__((address_space(1))) v2*>(reinterpret_cast<uintptr_t>(p));
  return make_double2(v.x, v.y);
}

// The kernel terms s k(x_b, D_k) of a big-block wave's 2 x 2 tiles (row tiles tr, tr + 1; column tiles tc,
// tc + 1), 16 elements per lane, parked in LDS (kvs[e * 64 + lane], e = (g * 2 + h) * 4 + r for column tile
// tc + g, row tile tr + h and register r of the T-form MFMA's D map): evaluated while a block's first chunks
// are in flight, so the epilogue only stores (in registers they would stay live across the contraction).
// Returns the r^2 == 0 bits (Plan::dup), one per element.  scaled_r2_dm's and kernel_term_nc's arithmetic
// (compiled without FP contraction, dkg_common.h), so the terms are posterior_cov_body's bits.
template <int DM, class T, class Sink>
__device__ __forceinline__ uint32_t big_block_terms(const Plan* __restrict__ P, const dkg_output& o,
                                                    const double* __restrict__ xnew, int B, int tr, int tc, int lane,
                                                    Sink&& sink) {
  const int N = P->N, d = P->d;
  const double os = o.outputscale;
  const int kind = o.kernel;
  const double* __restrict__ il_p = o.inv_lengthscale;
  const double* __restrict__ disc = P->disc;
  uint32_t zero_r2 = 0;
  double il[DM], xkv[2][DM];
#pragma unroll
  for (int c = 0; c < DM; ++c) il[c] = il_p[min(c, d - 1)];
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int k = 16 * (tc + g) + (lane & 15);
#pragma unroll
    for (int c = 0; c < DM; ++c) xkv[g][c] = disc[(size_t)min(k, N - 1) * d + min(c, d - 1)];
  }
  // one covariance family per instantiation (the switch outside the 16 terms: straight-line code the
  // scheduler interleaves) and one coefficient-table pointer for all of them
  auto terms = [&](auto kind_c) __attribute__((always_inline)) {
    constexpr int KIND = decltype(kind_c)::value;
    const const_dptr tab = psi_tab();
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int b = 16 * (tr + h) + mfma_drow<T>(lane, r);
        double xb[DM];
#pragma unroll
        for (int c = 0; c < DM; ++c) xb[c] = xnew[(size_t)min(b, B - 1) * d + min(c, d - 1)];
#pragma unroll
        for (int g = 0; g < 2; ++g) {
          double r2 = 0.0;
#pragma unroll
          for (int c = 0; c < DM; ++c) {
            const double t = (xb[c] - xkv[g][c]) * il[c];
            r2 = fma(t, (c < d) ? t : 0.0, r2);
          }
          const double kv = os * kernel_term_nc<KIND>(r2, tab);  // rounded (stored), as posterior_cov_body
          const int e = (g * 2 + h) * 4 + r;
          sink(e, kv);
          zero_r2 |= (r2 == 0.0 ? 1u : 0u) << e;
        }
      }
  };
  switch (kind) {
    case DKG_MATERN12: terms(std::integral_constant<int, DKG_MATERN12>{}); break;
    case DKG_MATERN32: terms(std::integral_constant<int, DKG_MATERN32>{}); break;
    case DKG_RBF: terms(std::integral_constant<int, DKG_RBF>{}); break;
    default: terms(std::integral_constant<int, DKG_MATERN52>{}); break;
  }
  return zero_r2;
}

template <int DM, class T>
__device__ __forceinline__ uint32_t big_block_terms(const Plan* __restrict__ P, const dkg_output& o,
                                                    const double* __restrict__ xnew, int B, int tr, int tc, int lane,
                                                    double* __restrict__ kvs) {
  return big_block_terms<DM, T>(P, o, xnew, B, tr, tc, lane,
                                [&](int e, double kv) __attribute__((always_inline)) { kvs[e * 64 + lane] = kv; });
}

constexpr int PB_WAVES = 4;
constexpr int PB_RT = 4;  // candidate tiles per block
constexpr int PB_CT = 4;  // line tiles per block
#ifndef DKG_PB_WC
#define DKG_PB_WC 2
#endif
constexpr int PB_WC = DKG_PB_WC;  // words (two k-blocks each) per staged chunk (2 or 4); even, so chains restart in step
// the kernel terms in registers (16 per lane) instead of parked in LDS: the LDS then holds the stage buffers only
#ifndef DKG_PB_KVREG
#define DKG_PB_KVREG 0
#endif
constexpr bool PB_KVREG = DKG_PB_KVREG != 0;
constexpr int PB_STAGE = (PB_RT + PB_CT) * PB_WC * 64;  // 16-byte words per stage buffer
#ifndef DKG_PB_NSTG
#define DKG_PB_NSTG 2
#endif
constexpr int PB_NSTG = DKG_PB_NSTG;                               // stage buffers: chunks in flight + the one computed
// the stage buffers, then the kernel terms (16 per lane per wave): 64 KiB, two workgroups per CU
constexpr size_t PB_LDS = PB_NSTG * (size_t)PB_STAGE * 16 + (PB_KVREG ? 0 : (size_t)PB_WAVES * 16 * 64 * 8);

template <int DM>
__global__ __launch_bounds__(PB_WAVES * WAVE) __attribute__((amdgpu_waves_per_eu(2))) void posterior_cov_big_kernel(
    const Plan* __restrict__ P, const double* __restrict__ xnew, int B, int dst, int order) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double2* stg = reinterpret_cast<double2*>(smem);
  const int N = P->N;
  const int nbx = (N + 16 * PB_CT - 1) / (16 * PB_CT), nby = (B + 16 * PB_RT - 1) / (16 * PB_RT);
  int bx, by, oi;
  if (!block_order(blockIdx.x, nbx, nby, P->m, order, bx, by, oi)) return;
  unsigned long long* st = kst_slot(dst, P, 1);
  KST_BEGIN(st);
  const dkg_output& o = P->o[oi];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int rp = wave & 1, cp = wave >> 1;  // the wave's tiles: rows 2 rp, 2 rp + 1; columns 2 cp, 2 cp + 1
  const int RT = pad16(B) / 16, CT = pad16(N) / 16;
  const int KB = pad16(o.n) / 4, KP = KB / 2, KPs = (KP + 1) / 2;  // posterior_cov_body's halves (PC_KS = 2)
  const int ti0 = PB_RT * by, tk0 = PB_CT * bx;
  const double* qx = P->q[oi];
  const double* qd = o.disc_frag;
  // chunks: half 0's words [0, KPs), then half 1's [KPs, KP), PB_WC words each, starting at each half's start
  const int nc0 = (KPs + PB_WC - 1) / PB_WC, nc = nc0 + (KP - KPs + PB_WC - 1) / PB_WC;
  auto chunk_start = [&](int c) { return c < nc0 ? c * PB_WC : KPs + (c - nc0) * PB_WC; };
  auto chunk_words = [&](int c) { return c < nc0 ? min(PB_WC, KPs - c * PB_WC) : min(PB_WC, KP - chunk_start(c)); };
  // Chunk staging by LDS-DMA, PB_NSTG buffers deep: chunk c + PB_NSTG - 1 is in flight while chunk c is
  // computed.  The fragment reads are inline-asm ds_reads with their own lgkmcnt waits: a compiler-visible
  // LDS read after an LDS-DMA makes the compiler wait for every DMA in flight first (it cannot tell the
  // buffers apart).  Every wave issues PB_PIECES DMA instructions per chunk (words past a chunk's end repeat
  // a live word, unused), so the chunk-c wait is vmcnt <= PB_PIECES x (chunks issued after it).
  constexpr int PB_PIECES = (PB_RT + PB_CT) * PB_WC / PB_WAVES;
  static_assert((PB_RT + PB_CT) * PB_WC % PB_WAVES == 0 && (PB_PIECES == 4 || PB_PIECES == 8),
                "four or eight DMA pieces per wave per chunk");
  auto stage = [&](int c) {
    const int j0 = chunk_start(c), nw = chunk_words(c);
    double2* buf = stg + (size_t)(c % PB_NSTG) * PB_STAGE;
#pragma unroll
    for (int q = 0; q < PB_PIECES; ++q) {
      const int piece = wave + PB_WAVES * q;
      const int t = piece / PB_WC, w = min(piece % PB_WC, nw - 1);
      const double* src = t < PB_RT ? qx : qd;
      const int tile = t < PB_RT ? min(ti0 + t, RT - 1) : min(tk0 + t - PB_RT, CT - 1);
      __builtin_amdgcn_global_load_lds(
          reinterpret_cast<const void*>(src + (((size_t)tile * KP + j0 + w) * 64 + lane) * 2),
          reinterpret_cast<__attribute__((address_space(3))) void*>(reinterpret_cast<uintptr_t>(buf + piece * 64)),
          16, 0, 0);
    }
  };
  typedef double v2d __attribute__((ext_vector_type(2)));
  // per-lane LDS byte addresses of the wave's candidate tiles (2 rp, 2 rp + 1) and line tiles in buffer 0
  const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>(stg);
  const uint32_t addrA = lds0 + (uint32_t)(((2 * rp) * PB_WC) * 64 + lane) * 16;
  const uint32_t addrB = lds0 + (uint32_t)(((PB_RT + 2 * cp) * PB_WC) * 64 + lane) * 16;
  const bool want_var = bx == 0 && cp == 0;  // the wave's column tiles include tile 0: its row tiles' variances
  d4 acc[2][2][4];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[h][g][c] = d4{0.0, 0.0, 0.0, 0.0};
  d4 sum0[2][2];
  double qsq[2] = {0.0, 0.0}, qh0[2] = {0.0, 0.0};
#pragma unroll
  for (int c = 0; c < PB_NSTG - 1; ++c)
    if (c < nc) stage(c);
  // The kernel terms s k(x_b, D_k) of the wave's 16 elements per lane (scaled_r2_dm's and kernel_profile's
  // arithmetic), evaluated while the first chunks' DMAs are in flight and parked in LDS (16 x 8 bytes per
  // lane: in registers they would stay live across the contraction): the epilogue then only stores.
  // r^2 == 0 (Plan::dup) as one bit per element.
  const double os = o.outputscale;
  double* kvs = reinterpret_cast<double*>(stg + (size_t)PB_NSTG * PB_STAGE) + (size_t)wave * 16 * 64;
  double kvr[PB_KVREG ? 16 : 1];
  uint32_t zero_r2;
  if constexpr (PB_KVREG) {
    zero_r2 = big_block_terms<DM, double>(P, o, xnew, B, ti0 + 2 * rp, tk0 + 2 * cp, lane,
                                          [&](int e, double kv) __attribute__((always_inline)) {
                                            asm volatile("" : "+v"(kv));  // rounded here (never fused later)
                                            kvr[e] = kv;
                                          });
  } else {
    zero_r2 = big_block_terms<DM, double>(P, o, xnew, B, ti0 + 2 * rp, tk0 + 2 * cp, lane, kvs);
  }
  KST(st, 2);
  for (int c = 0; c < nc; ++c) {
    // chunk c landed (this wave's pieces), then every wave's: the later chunks' DMAs stay in flight
    const int later = min(nc - 1 - c, PB_NSTG - 2);  // chunks issued after c (wave-uniform)
    switch (later * PB_PIECES) {
      case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
      case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
      case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
      default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
    // a bare s_barrier: __syncthreads()'s workgroup fence would make the compiler drain every DMA in flight
    // (vmcnt(0)) first; LDS needs no fence within the workgroup once the DMA has landed (vmcnt above)
    asm volatile("s_barrier" ::: "memory");
    // buffer (c + PB_NSTG - 1) % PB_NSTG held chunk c - 1, which every wave finished before the barrier
    if (c + PB_NSTG - 1 < nc) stage(c + PB_NSTG - 1);
    if (c == nc0) {  // half 0 done: its sums, and the chains restart for half 1
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int g = 0; g < 2; ++g) {
          sum0[h][g] = (acc[h][g][0] + acc[h][g][1]) + (acc[h][g][2] + acc[h][g][3]);
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[h][g][q] = d4{0.0, 0.0, 0.0, 0.0};
        }
      if (want_var) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          double q = qsq[h];
          q += __shfl_xor(q, 16);
          q += __shfl_xor(q, 32);
          qh0[h] = q;
          qsq[h] = 0.0;
        }
      }
    }
    const uint32_t so = (uint32_t)(c % PB_NSTG) * (uint32_t)(PB_STAGE * 16);
    const uint32_t aA = addrA + so, aB = addrB + so;
    const int nw = chunk_words(c);
    // the chunk's words in pairs, each pair in two register sets X and Y (no copies between them: a VALU copy into
    // registers an MFMA group just read holds the next group until that group has read them): word 2p + 1's read
    // is issued before word 2p's MFMAs, and LDS reads complete in order, so lgkmcnt(4) means word 2p has landed.
    // Set Y is read and waited for on every pair, a chunk's words past nw included (their slots repeat a live
    // word, stage()): no branch between an asm read and its wait, where the register allocator would be free to
    // copy the destination registers before the data lands (tools/asm_audit.py checks the compiled kernel).
    static_assert(PB_WC % 2 == 0, "words in pairs: register sets X and Y");
    v2d xa0, xa1, xb0, xb1, ya0, ya1, yb0, yb1;
    auto word = [&](const v2d& a0, const v2d& a1, const v2d& b0, const v2d& b1, auto chc) __attribute__((always_inline)) {
      constexpr int chx = decltype(chc)::value;  // k-blocks 2 j, 2 j + 1 of the half: chains chx, chx + 1
      acc[0][0][chx] = mfma_f64(a0.x, b0.x, acc[0][0][chx]);
      acc[0][1][chx] = mfma_f64(a0.x, b1.x, acc[0][1][chx]);
      acc[1][0][chx] = mfma_f64(a1.x, b0.x, acc[1][0][chx]);
      acc[1][1][chx] = mfma_f64(a1.x, b1.x, acc[1][1][chx]);
      acc[0][0][chx + 1] = mfma_f64(a0.y, b0.y, acc[0][0][chx + 1]);
      acc[0][1][chx + 1] = mfma_f64(a0.y, b1.y, acc[0][1][chx + 1]);
      acc[1][0][chx + 1] = mfma_f64(a1.y, b0.y, acc[1][0][chx + 1]);
      acc[1][1][chx + 1] = mfma_f64(a1.y, b1.y, acc[1][1][chx + 1]);
      if (want_var) {
        qsq[0] = fma(a0.x, a0.x, qsq[0]);
        qsq[0] = fma(a0.y, a0.y, qsq[0]);
        qsq[1] = fma(a1.x, a1.x, qsq[1]);
        qsq[1] = fma(a1.y, a1.y, qsq[1]);
      }
    };
    // Word g of the chunk goes through set X (g even) or Y (g odd).  Words 0 and 1 are read at the chunk start;
    // word g + 2 is read right after word g's MFMAs have issued (into the same set, sixteen wait states later),
    // so its LDS latency runs under word g + 1's MFMAs.  Before word g's MFMAs at most words g and g + 1 are in
    // flight (LDS reads complete in order): lgkmcnt(4) has word g, lgkmcnt(0) the chunk's last word.
    constexpr int TS = PB_WC * 1024;  // bytes between a wave's two tiles of one operand in a stage buffer
    auto rd = [](v2d& a0, v2d& a1, v2d& b0, v2d& b1, uint32_t pA, uint32_t pB, auto gc) __attribute__((always_inline)) {
      constexpr int g = decltype(gc)::value;
      if constexpr (g < 2) {
        asm volatile("ds_read_b128 %0, %4 offset:%6\n\tds_read_b128 %1, %4 offset:%7\n\t"
                     "ds_read_b128 %2, %5 offset:%6\n\tds_read_b128 %3, %5 offset:%7"
                     : "=&v"(a0), "=&v"(a1), "=&v"(b0), "=&v"(b1)
                     : "v"(pA), "v"(pB), "i"(g * 1024), "i"(g * 1024 + TS)
                     : "memory");
      } else {
        asm volatile("s_nop 7\n\ts_nop 7\n\tds_read_b128 %0, %4 offset:%6\n\tds_read_b128 %1, %4 offset:%7\n\t"
                     "ds_read_b128 %2, %5 offset:%6\n\tds_read_b128 %3, %5 offset:%7"
                     : "=&v"(a0), "=&v"(a1), "=&v"(b0), "=&v"(b1)
                     : "v"(pA), "v"(pB), "i"(g * 1024), "i"(g * 1024 + TS)
                     : "memory");
      }
    };
    rd(xa0, xa1, xb0, xb1, aA, aB, std::integral_constant<int, 0>{});
    rd(ya0, ya1, yb0, yb1, aA, aB, std::integral_constant<int, 1>{});
    auto group = [&](auto gc) __attribute__((always_inline)) {
      constexpr int g = decltype(gc)::value;
      v2d& a0 = (g & 1) ? ya0 : xa0;
      v2d& a1 = (g & 1) ? ya1 : xa1;
      v2d& b0 = (g & 1) ? yb0 : xb0;
      v2d& b1 = (g & 1) ? yb1 : xb1;
      if constexpr (g + 1 < PB_WC) asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(a0), "+v"(a1), "+v"(b0), "+v"(b1));
      else asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a0), "+v"(a1), "+v"(b0), "+v"(b1));
      if (g < nw) word(a0, a1, b0, b1, std::integral_constant<int, (g & 1) ? 2 : 0>{});  // wave-uniform
      __builtin_amdgcn_sched_barrier(0);  // the MFMAs issue before the next wait or rewrite
      if constexpr (g + 2 < PB_WC) rd(a0, a1, b0, b1, aA, aB, std::integral_constant<int, g + 2>{});
    };
    group(std::integral_constant<int, 0>{});
    group(std::integral_constant<int, 1>{});
    if constexpr (PB_WC > 2) {
      group(std::integral_constant<int, 2>{});
      group(std::integral_constant<int, 3>{});
    }
    static_assert(PB_WC == 2 || PB_WC == 4, "two or four words per chunk");
    // Both sets' MFMAs issue here, before the next chunk's wait, barrier and fragment reads: the rewrites of
    // sets X and Y are inline asm, which the scheduler may otherwise move the (memory-free) MFMA builtins
    // across, and which the hazard recognizer does not see.  A scheduling barrier holds the order.
    __builtin_amdgcn_sched_barrier(0);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  KST(st, 3);
  // epilogue: s k(x_b, D_k) - (half 0 + half 1), the coincidence marks and the variances
  const int rec = cov_rec(P->m);
  d4 tot[2][2];  // half 0 + half 1 (the chains are dead from here: registers for the kernel terms)
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      tot[h][g] = sum0[h][g] + ((acc[h][g][0] + acc[h][g][1]) + (acc[h][g][2] + acc[h][g][3]));
      asm volatile("" : "+v"(tot[h][g]));  // formed here: the chains are dead before the epilogue's loads
    }
  // the stores: the kernel terms from LDS (evaluated before the contraction), minus the contraction.  The
  // lane index through an opaque copy: the store addresses are formed here, not hoisted across the loop
  // (16 live 64-bit addresses spilled)
  int le = lane;
  asm volatile("" : "+v"(le));
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int k = 16 * (tk0 + 2 * cp + g) + (le & 15);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int b = 16 * (ti0 + 2 * rp + h) + mfma_drow<double>(le, r);
        const int e = (g * 2 + h) * 4 + r;
        if (b < B && k < N) {
          P->cov_all[(size_t)b * P->cov_stride + (size_t)k * rec + oi] =
              (PB_KVREG ? kvr[PB_KVREG ? e : 0] : kvs[e * 64 + le]) - tot[h][g][r];
          if (DKG_DUP_MARK && ((zero_r2 >> e) & 1)) atomicMin(&P->dup[b], k);  // Plan::dup
        }
      }
  }
  if (want_var) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      double q = qsq[h];
      q += __shfl_xor(q, 16);
      q += __shfl_xor(q, 32);
      const int bb = 16 * (ti0 + 2 * rp + h) + lane;
      if (lane < 16 && bb < B) P->var[oi][bb] = os - (qh0[h] + q);
    }
  }
  KST_END(st);
}

// ---------------------------------------------------------------------------
// posterior_cov_reg_kernel<DM, RT> (fp64): the covariance rows of launches over many candidates in blocks of RT
// candidate tiles x 4 line tiles of one output, one workgroup of 8 waves per CU, with posterior_cov_kernel's
// arithmetic element for element (two K halves, four k-block chains each, (c0 + c1) + (c2 + c3), half 0 + half 1;
// the variance per half, xor-16 / xor-32, half 0 + half 1).  Wave w owns line tile w & 3 and K half w >> 2 (the
// two waves of a SIMD run the two halves of one line tile): its Q_D fragments are its own, the RT candidate tiles'
// Q_X fragments are read by the four waves of its half at about the same time (one L2 read per CU, the rest from
// L1).  No LDS staging and no barrier in the contraction: every operand goes global -> registers one word ahead,
// 4 RT independent chains per wave and the partner wave on the SIMD hide the latencies.  The halves meet in LDS
// at the end, each wave finalising part of the block (a sum of two addends commutes: the same bits whichever
// adds).  RT picks the block height that fills the device in whole rounds (cov_reg_rt): a 5-batch headline
// launch (40 candidate tiles, 64 line tiles, 2 outputs) is exactly 256 blocks of 5 x 4 tiles, where 64 x 64
// blocks left 64 CUs with two.
constexpr int PR_WAVES = 8;
// row tiles finalised by half 0 (and whose kernel terms it evaluates, after its contraction in rec2): the
// smaller share, since half 1 evaluates its terms under half 0's MFMAs
template <int RT>
__host__ __device__ constexpr int cov_reg_split() { return RT / 2; }
template <int RT>
__host__ __device__ constexpr size_t cov_reg_lds() {
  // kernel terms [4 line tiles][RT * 4][64], exchanged half sums [4][RT * 4][64], exchanged variances [RT][16]
  return ((size_t)4 * RT * 4 * 64 * 2 + (size_t)RT * 16) * sizeof(double);
}

template <int DM, int RT>
__global__ __launch_bounds__(PR_WAVES * WAVE) __attribute__((amdgpu_waves_per_eu(2))) void posterior_cov_reg_kernel(
    const Plan* __restrict__ P, const double* __restrict__ xnew, int B, int dst, int order) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  typedef double v2d __attribute__((ext_vector_type(2)));
  const int N = P->N;
  const int nbx = (N + 63) / 64, nby = (B + 16 * RT - 1) / (16 * RT);
  int bx, by, oi;
  if (!block_order(blockIdx.x, nbx, nby, P->m, order, bx, by, oi)) return;
  unsigned long long* st = kst_slot(dst, P, 1);
  KST_BEGIN(st);
  const dkg_output& o = P->o[oi];
  const int d = P->d;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wl = wave & 3, half = wave >> 2;
  constexpr int H0 = cov_reg_split<RT>();  // half 0 finalises (and evaluates the terms of) row tiles h < H0
  const int hlo = half ? H0 : 0, hhi = half ? RT : H0;
  const int RTt = pad16(B) / 16, CT = pad16(N) / 16;
  const int KB = pad16(o.n) / 4, KP = KB / 2, KPs = (KP + 1) / 2;  // posterior_cov_body's halves (PC_KS = 2)
  const int ti0 = RT * by;
  const int tk = 4 * bx + wl;  // this wave's line tile
  typedef const __attribute__((address_space(1))) v2d* gv2d;  // global loads (not flat)
  gv2d ap[RT];  // lane's word-0 fragments of the candidate tiles (dead tiles read a live one)
#pragma unroll
  for (int h = 0; h < RT; ++h)
    ap[h] = reinterpret_cast<gv2d>(reinterpret_cast<uintptr_t>(P->q[oi])) + ((size_t)min(ti0 + h, RTt - 1) * KP) * 64 + lane;
  const gv2d bp =
      reinterpret_cast<gv2d>(reinterpret_cast<uintptr_t>(o.disc_frag)) + ((size_t)min(tk, CT - 1) * KP) * 64 + lane;
  double* kvs = smem + (size_t)wl * RT * 4 * 64;                 // kernel terms of line tile wl
  double* xch = smem + (size_t)4 * RT * 4 * 64 + (size_t)wl * RT * 4 * 64;  // the other half's sums, line tile wl
  double* xvar = smem + (size_t)4 * RT * 4 * 64 * 2;              // half 1's variance sums [RT][16]
  // the kernel terms' inputs first (loads complete in order: the terms then wait for these, not the operands)
  const double* __restrict__ il_p = o.inv_lengthscale;
  double il[DM], xk[DM];
  const int kcol = 16 * tk + (lane & 15);
#pragma unroll
  for (int c = 0; c < DM; ++c) {
    il[c] = il_p[min(c, d - 1)];
    xk[c] = P->disc[(size_t)min(kcol, N - 1) * d + min(c, d - 1)];
  }
  constexpr int HT = RT - H0 > H0 ? RT - H0 : H0;  // row tiles whose terms a wave evaluates (at most)
  double xb[HT][4][DM];
#pragma unroll
  for (int u = 0; u < HT; ++u)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int h = min(hlo + u, RT - 1);
      const int b = 16 * (ti0 + h) + mfma_drow<double>(lane, r);
#pragma unroll
      for (int c = 0; c < DM; ++c) xb[u][r][c] = xnew[(size_t)min(b, B - 1) * d + min(c, d - 1)];
    }
  struct Word {
    v2d a[RT];
    v2d b;
  };
  auto load = [&](Word& w, int j) __attribute__((always_inline)) {
#pragma unroll
    for (int h = 0; h < RT; ++h) w.a[h] = ap[h][(size_t)j * 64];
    w.b = bp[(size_t)j * 64];
  };
  const int j0 = half ? KPs : 0, j1 = half ? KP : KPs;
  Word w0, w1;
  load(w0, min(j0, KP - 1));
  // kernel terms s k(x_b, D_k) of row tiles hlo .. hhi - 1 (scaled_r2_dm's / kernel_profile's arithmetic,
  // contraction-free), parked in LDS for the waves that finalise them
  const double os = o.outputscale;
  uint32_t zero_r2 = 0;  // r^2 == 0 (Plan::dup) of the terms this wave evaluates, bit (h - hlo) * 4 + r
  {
    auto terms = [&](auto kind_c) __attribute__((always_inline)) {
      constexpr int KIND = decltype(kind_c)::value;
      const const_dptr tab = psi_tab();
#pragma unroll
      for (int u = 0; u < HT; ++u)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          double r2 = 0.0;
#pragma unroll
          for (int c = 0; c < DM; ++c) {
            const double t = (xb[u][r][c] - xk[c]) * il[c];
            r2 = fma(t, (c < d) ? t : 0.0, r2);
          }
          const double kv = os * kernel_term_nc<KIND>(r2, tab);  // rounded (stored)
          if (hlo + u < hhi) {  // wave-uniform
            kvs[((hlo + u) * 4 + r) * 64 + lane] = kv;
            zero_r2 |= (r2 == 0.0 ? 1u : 0u) << (u * 4 + r);
          }
        }
    };
    switch (o.kernel) {
      case DKG_MATERN12: terms(std::integral_constant<int, DKG_MATERN12>{}); break;
      case DKG_MATERN32: terms(std::integral_constant<int, DKG_MATERN32>{}); break;
      case DKG_RBF: terms(std::integral_constant<int, DKG_RBF>{}); break;
      default: terms(std::integral_constant<int, DKG_MATERN52>{}); break;
    }
  }
  d4 acc[RT][4];
#pragma unroll
  for (int h = 0; h < RT; ++h)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[h][q] = d4{0.0, 0.0, 0.0, 0.0};
  double qsq[RT];  // every wave forms them (branch-free); line tile 0's waves use them
#pragma unroll
  for (int h = 0; h < RT; ++h) qsq[h] = 0.0;
  KST(st, 2);
  // word at relative index jr of the half: k-blocks 2 jr, 2 jr + 1 -> chains 2 (jr & 1), 2 (jr & 1) + 1
  auto mul = [&](const Word& w, int ch) __attribute__((always_inline)) {
#pragma unroll
    for (int h = 0; h < RT; ++h) acc[h][ch] = mfma_f64(w.a[h].x, w.b.x, acc[h][ch]);
#pragma unroll
    for (int h = 0; h < RT; ++h) acc[h][ch + 1] = mfma_f64(w.a[h].y, w.b.y, acc[h][ch + 1]);
#pragma unroll
    for (int h = 0; h < RT; ++h) {
      qsq[h] = fma(w.a[h].x, w.a[h].x, qsq[h]);
      qsq[h] = fma(w.a[h].y, w.a[h].y, qsq[h]);
    }
  };
  int j = j0;
#pragma unroll 1
  for (; j + 2 <= j1; j += 2) {
    load(w1, j + 1);
    mul(w0, 0);
    load(w0, min(j + 2, KP - 1));
    mul(w1, 2);
  }
  if (j < j1) mul(w0, 0);  // an odd half
  KST(st, 3);
  // the halves meet: each wave hands the sums of the row tiles the other half finalises to it (LDS), and the
  // variances of line tile 0's half 1 to its half 0
  d4 tot[RT];
#pragma unroll
  for (int h = 0; h < RT; ++h) {
    tot[h] = (acc[h][0] + acc[h][1]) + (acc[h][2] + acc[h][3]);
    if (h < hlo || h >= hhi) {  // wave-uniform
#pragma unroll
      for (int r = 0; r < 4; ++r) xch[(h * 4 + r) * 64 + lane] = tot[h][r];
    }
  }
  const bool want_var = tk == 0;
  if (want_var && half) {
#pragma unroll
    for (int h = 0; h < RT; ++h) {
      double q = qsq[h];
      q += __shfl_xor(q, 16);
      q += __shfl_xor(q, 32);
      if (lane < 16) xvar[h * 16 + lane] = q;
    }
  }
  __syncthreads();
  const int rec = cov_rec(P->m);
  int le = lane;
  asm volatile("" : "+v"(le));  // store addresses formed here
  const int k = 16 * tk + (le & 15);
#pragma unroll
  for (int h = 0; h < RT; ++h) {
    if (h < hlo || h >= hhi) continue;  // wave-uniform
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int b = 16 * (ti0 + h) + mfma_drow<double>(le, r);
      const double sum = tot[h][r] + xch[(h * 4 + r) * 64 + le];  // half 0 + half 1 (commutes)
      if (b < B && k < N) {
        const double kt = kvs[(h * 4 + r) * 64 + le];
        P->cov_all[(size_t)b * P->cov_stride + (size_t)k * rec + oi] = kt - sum;
        if (DKG_DUP_MARK && ((zero_r2 >> ((h - hlo) * 4 + r)) & 1)) atomicMin(&P->dup[b], k);  // Plan::dup
      }
    }
  }
  if (want_var && !half) {
#pragma unroll
    for (int h = 0; h < RT; ++h) {
      double q = qsq[h];
      q += __shfl_xor(q, 16);
      q += __shfl_xor(q, 32);
      const int bb = 16 * (ti0 + h) + lane;
      if (lane < 16 && bb < B) P->var[oi][bb] = os - (q + xvar[h * 16 + lane]);
    }
  }
  KST_END(st);
}

// ---------------------------------------------------------------------------
// posterior_cov_rec2_kernel<DM, RT> (fp64, m = 2 outputs: the headline family): posterior_cov_reg_kernel with the
// two outputs of a line in one workgroup, so the block's line records leave as whole 16-byte records.  Block:
// RT candidate tiles x 2 line tiles x both outputs; wave w: line tile w & 1, output (w >> 1) & 1, K half w >> 2.
// The halves meet in LDS as in posterior_cov_reg_kernel, the finalised values are gathered into the block's
// record tile in LDS ([16 RT candidates][32 lines][2 outputs], 512 contiguous bytes per candidate in cov_all),
// and the workgroup writes it with one 16-byte store per lane per two candidates: with one output per workgroup,
// the 8-byte stores of every other record slot (16 per lane and wave) took 37 % of the block's lifetime
// (profiles/r06/cov/covst_reg2_g5.txt).  A 5-batch headline launch is 8 x 32 = 256 blocks of 5 candidate tiles.
template <int RT>
__host__ __device__ constexpr size_t cov_rec2_lds() {
  // terms [4 (line tile, output)][RT * 4][64], exchanged half sums [4][RT * 4][64], the record tile
  // [16 RT][32][2], exchanged variances [2 outputs][RT][16]
  return ((size_t)4 * RT * 4 * 64 * 2 + (size_t)16 * RT * 32 * 2 + (size_t)2 * RT * 16) * sizeof(double);
}

template <int DM, int RT>
__global__ __launch_bounds__(PR_WAVES * WAVE) __attribute__((amdgpu_waves_per_eu(2))) void posterior_cov_rec2_kernel(
    const Plan* __restrict__ P, const double* __restrict__ xnew, int B, int dst, int order) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  typedef double v2d __attribute__((ext_vector_type(2)));
  const int N = P->N;
  const int nbx = (N + 31) / 32, nby = (B + 16 * RT - 1) / (16 * RT);
  int bx, by, one;
  if (!block_order(blockIdx.x, nbx, nby, 1, order, bx, by, one)) return;
  unsigned long long* st = kst_slot(dst, P, 1);
  KST_BEGIN(st);
  const int d = P->d;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lt = wave & 1, oi = (wave >> 1) & 1, half = wave >> 2;
  const int slot = wave & 3;  // (line tile, output) of the wave
  const dkg_output& o = P->o[oi];
  constexpr int H0 = cov_reg_split<RT>();  // half 0 finalises (and evaluates the terms of) row tiles h < H0
  const int hlo = half ? H0 : 0, hhi = half ? RT : H0;
  const int RTt = pad16(B) / 16, CT = pad16(N) / 16;
  const int KB = pad16(o.n) / 4, KP = KB / 2, KPs = (KP + 1) / 2;  // posterior_cov_body's halves (PC_KS = 2)
  const int ti0 = RT * by;
  const int tk = 2 * bx + lt;  // this wave's line tile
  typedef const __attribute__((address_space(1))) v2d* gv2d;  // global loads (not flat)
  gv2d ap[RT];
#pragma unroll
  for (int h = 0; h < RT; ++h)
    ap[h] = reinterpret_cast<gv2d>(reinterpret_cast<uintptr_t>(P->q[oi])) + ((size_t)min(ti0 + h, RTt - 1) * KP) * 64 + lane;
  const gv2d bp =
      reinterpret_cast<gv2d>(reinterpret_cast<uintptr_t>(o.disc_frag)) + ((size_t)min(tk, CT - 1) * KP) * 64 + lane;
  double* kvs = smem + (size_t)slot * RT * 4 * 64;
  double* xch = smem + (size_t)4 * RT * 4 * 64 + (size_t)slot * RT * 4 * 64;
  double* rtile = smem + (size_t)4 * RT * 4 * 64 * 2;  // [16 RT][32][2]
  double* xvar = rtile + (size_t)16 * RT * 32 * 2;     // [2][RT][16]
  const double* __restrict__ il_p = o.inv_lengthscale;
  double il[DM], xk[DM];
  const int kcol = 16 * tk + (lane & 15);
#pragma unroll
  for (int c = 0; c < DM; ++c) {
    il[c] = il_p[min(c, d - 1)];
    xk[c] = P->disc[(size_t)min(kcol, N - 1) * d + min(c, d - 1)];
  }
  constexpr int HT = RT - H0 > H0 ? RT - H0 : H0;
  struct Word {
    v2d a[RT];
    v2d b;
  };
  auto load = [&](Word& w, int j) __attribute__((always_inline)) {
#pragma unroll
    for (int h = 0; h < RT; ++h) w.a[h] = ap[h][(size_t)j * 64];
    w.b = bp[(size_t)j * 64];
  };
  const int j0 = half ? KPs : 0, j1 = half ? KP : KPs;
  Word w0, w1;
  load(w0, min(j0, KP - 1));
  const double os = o.outputscale;
  uint32_t zero_r2 = 0;
  // The kernel terms s k(x_b, D_k) of row tiles hlo .. hhi - 1 (scaled_r2_dm's / kernel_profile's arithmetic,
  // contraction-free), parked in LDS for the epilogue.  Half 1's waves evaluate theirs before their contraction,
  // half 0's after it: the two waves of a SIMD (one per half) then overlap one's VALU terms with the other's MFMAs
  // at both ends instead of both running VALU first.
  auto terms_of = [&]() {
    double xb[HT][4][DM];
#pragma unroll
    for (int u = 0; u < HT; ++u)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int h = min(hlo + u, RT - 1);
        const int b = 16 * (ti0 + h) + mfma_drow<double>(lane, r);
#pragma unroll
        for (int c = 0; c < DM; ++c) xb[u][r][c] = xnew[(size_t)min(b, B - 1) * d + min(c, d - 1)];
      }
    auto terms = [&](auto kind_c) __attribute__((always_inline)) {
      constexpr int KIND = decltype(kind_c)::value;
      const const_dptr tab = psi_tab();
#pragma unroll
      for (int u = 0; u < HT; ++u)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          double r2 = 0.0;
#pragma unroll
          for (int c = 0; c < DM; ++c) {
            const double t = (xb[u][r][c] - xk[c]) * il[c];
            r2 = fma(t, (c < d) ? t : 0.0, r2);
          }
          const double kv = os * kernel_term_nc<KIND>(r2, tab);  // rounded (stored)
          if (hlo + u < hhi) {  // wave-uniform
            kvs[((hlo + u) * 4 + r) * 64 + lane] = kv;
            zero_r2 |= (r2 == 0.0 ? 1u : 0u) << (u * 4 + r);
          }
        }
    };
    switch (o.kernel) {
      case DKG_MATERN12: terms(std::integral_constant<int, DKG_MATERN12>{}); break;
      case DKG_MATERN32: terms(std::integral_constant<int, DKG_MATERN32>{}); break;
      case DKG_RBF: terms(std::integral_constant<int, DKG_RBF>{}); break;
      default: terms(std::integral_constant<int, DKG_MATERN52>{}); break;
    }
  };
  d4 acc[RT][4];
#pragma unroll
  for (int h = 0; h < RT; ++h)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[h][q] = d4{0.0, 0.0, 0.0, 0.0};
  double qsq[RT];
#pragma unroll
  for (int h = 0; h < RT; ++h) qsq[h] = 0.0;
  auto mul = [&](const Word& w, int ch) __attribute__((always_inline)) {
#pragma unroll
    for (int h = 0; h < RT; ++h) acc[h][ch] = mfma_f64(w.a[h].x, w.b.x, acc[h][ch]);
#pragma unroll
    for (int h = 0; h < RT; ++h) acc[h][ch + 1] = mfma_f64(w.a[h].y, w.b.y, acc[h][ch + 1]);
#pragma unroll
    for (int h = 0; h < RT; ++h) {
      qsq[h] = fma(w.a[h].x, w.a[h].x, qsq[h]);
      qsq[h] = fma(w.a[h].y, w.a[h].y, qsq[h]);
    }
  };
  d4 tot[RT];  // the half's sums (c0 + c1) + (c2 + c3): formed right after the contraction, so the chains are dead
  if (half) terms_of();  // wave-uniform
  KST(st, 2);
  {
    int j = j0;
#pragma unroll 1
    for (; j + 2 <= j1; j += 2) {
      load(w1, j + 1);
      mul(w0, 0);
      load(w0, min(j + 2, KP - 1));
      mul(w1, 2);
    }
    if (j < j1) mul(w0, 0);
  }
#pragma unroll
  for (int h = 0; h < RT; ++h) tot[h] = (acc[h][0] + acc[h][1]) + (acc[h][2] + acc[h][3]);
  if (!half) terms_of();
  KST(st, 3);
#pragma unroll
  for (int h = 0; h < RT; ++h) {
    if (h < hlo || h >= hhi) {  // wave-uniform: the other half finalises this row tile
#pragma unroll
      for (int r = 0; r < 4; ++r) xch[(h * 4 + r) * 64 + lane] = tot[h][r];
    }
  }
  const bool want_var = tk == 0;
  if (want_var && half) {
#pragma unroll
    for (int h = 0; h < RT; ++h) {
      double q = qsq[h];
      q += __shfl_xor(q, 16);
      q += __shfl_xor(q, 32);
      if (lane < 16) xvar[(oi * RT + h) * 16 + lane] = q;
    }
  }
  __syncthreads();
  // finalise: s k - (half 0 + half 1) into the record tile (candidate row 16 h + drow, line 16 lt + (l & 15))
#pragma unroll
  for (int h = 0; h < RT; ++h) {
    if (h < hlo || h >= hhi) continue;  // wave-uniform
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rl = 16 * h + mfma_drow<double>(lane, r);
      const double sum = tot[h][r] + xch[(h * 4 + r) * 64 + lane];  // half 0 + half 1 (commutes)
      rtile[((size_t)rl * 32 + 16 * lt + (lane & 15)) * 2 + oi] = kvs[(h * 4 + r) * 64 + lane] - sum;
      if (DKG_DUP_MARK && ((zero_r2 >> ((h - hlo) * 4 + r)) & 1)) {
        const int b = 16 * (ti0 + h) + mfma_drow<double>(lane, r);
        if (b < B && kcol < N) atomicMin(&P->dup[b], kcol);  // Plan::dup
      }
    }
  }
  if (want_var && !half) {
#pragma unroll
    for (int h = 0; h < RT; ++h) {
      double q = qsq[h];
      q += __shfl_xor(q, 16);
      q += __shfl_xor(q, 32);
      const int bb = 16 * (ti0 + h) + lane;
      if (lane < 16 && bb < B) P->var[oi][bb] = os - (q + xvar[(oi * RT + h) * 16 + lane]);
    }
  }
  __syncthreads();
  // the record tile out: lane l of a store instruction writes record (l & 31) of candidate row 2 i + (l >> 5)
  const int k0 = 32 * bx;
  const int kl = lane & 31;
  const bool kin = k0 + kl < N;
  typedef __attribute__((address_space(1))) v2d* gv2dw;
  const v2d* rt2 = reinterpret_cast<const v2d*>(rtile);
  for (int i = wave; i < 8 * RT; i += PR_WAVES) {
    const int rl = 2 * i + (lane >> 5);
    const int b = 16 * ti0 + rl;
    if (b < B && kin) {
      gv2dw dstp = reinterpret_cast<gv2dw>(reinterpret_cast<uintptr_t>(P->cov_all + (size_t)b * P->cov_stride)) + k0 + kl;
      *dstp = rt2[(size_t)rl * 32 + kl];
    }
  }
  KST_END(st);
}

// ---------------------------------------------------------------------------
// posterior_cov_blk_kernel (fp64): the covariance rows of launches over many candidates (forward batches in one
// launch, the stress shape) in 64 x 32 blocks -- 4 candidate tiles x 2 line tiles of one output -- with
// posterior_cov_kernel's arithmetic element for element (the two K halves, four k-block chains each,
// (c0 + c1) + (c2 + c3), half 0 + half 1; the variance sums per half, xor-16 / xor-32, half 0 + half 1), so the
// block shape stays a speed matter.  Wave w owns candidate tile w of the block and both line tiles: 8 chains and
// 8 kernel terms per lane, ~150 VGPRs, three workgroups per CU.  posterior_cov_big_kernel's 64 x 64 blocks
// (234 VGPRs, two per CU) gave a 5-batch headline launch 320 workgroups for 256 CUs: the CUs holding two set the
// stage (28 us against 19 us alone, profiles/r06/cov/covst_b1_g5.txt); 640 of these fit the device at once.
// The operand panels arrive by glds16 (hidden from hipcc: no compiler drain of the DMAs in flight) in chunks of
// PK_WC words, PK_NSTG buffers deep, and are read with plain LDS loads whose waits hipcc places (the inline-asm
// reads of posterior_cov_big_kernel left the allocator free to copy their registers early); the
// kernel terms are evaluated into registers while the first chunks land.
constexpr int PK_RT = 4;  // candidate tiles per block (one per wave)
constexpr int PK_CT = 2;  // line tiles per block
#ifndef DKG_PK_WC
#define DKG_PK_WC 2
#endif
constexpr int PK_WC = DKG_PK_WC;  // words (two k-blocks each) per chunk; even, so the chains restart in step
#ifndef DKG_PK_NSTG
#define DKG_PK_NSTG 3
#endif
constexpr int PK_NSTG = DKG_PK_NSTG;
constexpr int PK_STAGE = (PK_RT + PK_CT) * PK_WC * 64;  // 16-byte words per stage buffer
constexpr size_t PK_LDS = PK_NSTG * (size_t)PK_STAGE * 16;

template <int DM>
__global__ __launch_bounds__(PB_WAVES * WAVE) __attribute__((amdgpu_waves_per_eu(3))) void posterior_cov_blk_kernel(
    const Plan* __restrict__ P, const double* __restrict__ xnew, int B, int dst, int order) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  typedef double v2d __attribute__((ext_vector_type(2)));
  v2d* stg = reinterpret_cast<v2d*>(smem);
  const int N = P->N;
  const int nbx = (N + 16 * PK_CT - 1) / (16 * PK_CT), nby = (B + 16 * PK_RT - 1) / (16 * PK_RT);
  int bx, by, oi;
  if (!block_order(blockIdx.x, nbx, nby, P->m, order, bx, by, oi)) return;
  unsigned long long* st = kst_slot(dst, P, 1);
  KST_BEGIN(st);
  const dkg_output& o = P->o[oi];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int RT = pad16(B) / 16, CT = pad16(N) / 16;
  const int KB = pad16(o.n) / 4, KP = KB / 2, KPs = (KP + 1) / 2;  // posterior_cov_body's halves (PC_KS = 2)
  const int ti0 = PK_RT * by, tk0 = PK_CT * bx;
  const int ti = ti0 + wave;  // this wave's candidate tile
  const double* qx = P->q[oi];
  const double* qd = o.disc_frag;
  const int nc0 = (KPs + PK_WC - 1) / PK_WC, nc = nc0 + (KP - KPs + PK_WC - 1) / PK_WC;
  auto chunk_start = [&](int c) { return c < nc0 ? c * PK_WC : KPs + (c - nc0) * PK_WC; };
  auto chunk_words = [&](int c) { return c < nc0 ? min(PK_WC, KPs - c * PK_WC) : min(PK_WC, KP - chunk_start(c)); };
  constexpr int PIECES = (PK_RT + PK_CT) * PK_WC / PB_WAVES;
  static_assert((PK_RT + PK_CT) * PK_WC % PB_WAVES == 0 && (PIECES == 3 || PIECES == 6), "DMA pieces per wave");
  const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>(stg);
  auto stage = [&](int c) {  // chunk c's panels into buffer c % PK_NSTG; words past its end repeat a live word
    const int j0 = chunk_start(c), nw = chunk_words(c);
    const uint32_t buf = lds0 + (uint32_t)((c % PK_NSTG) * PK_STAGE) * 16u;
#pragma unroll
    for (int q = 0; q < PIECES; ++q) {
      const int piece = wave + PB_WAVES * q;
      const int t = piece / PK_WC, w = min(piece % PK_WC, nw - 1);
      const double* src = t < PK_RT ? qx : qd;
      const int tile = t < PK_RT ? min(ti0 + t, RT - 1) : min(tk0 + t - PK_RT, CT - 1);
      glds16(src + (((size_t)tile * KP + j0 + w) * 64 + lane) * 2, buf + (uint32_t)piece * 1024u);
    }
  };
#pragma unroll
  for (int c = 0; c < PK_NSTG - 1; ++c)
    if (c < nc) stage(c);
  // the kernel terms s k(x_b, D_k) of the wave's 8 elements per lane (big_block_terms' arithmetic), in registers
  const double os = o.outputscale;
  double kv[2][4];
  uint32_t zero_r2 = 0;  // r^2 == 0 (Plan::dup), bit g * 4 + r
  {
    const int d = P->d;
    const int kind = o.kernel;
    const double* __restrict__ il_p = o.inv_lengthscale;
    const double* __restrict__ disc = P->disc;
    double il[DM], xkv[2][DM];
#pragma unroll
    for (int c = 0; c < DM; ++c) il[c] = il_p[min(c, d - 1)];
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const int k = 16 * (tk0 + g) + (lane & 15);
#pragma unroll
      for (int c = 0; c < DM; ++c) xkv[g][c] = disc[(size_t)min(k, N - 1) * d + min(c, d - 1)];
    }
    auto terms = [&](auto kind_c) __attribute__((always_inline)) {
      constexpr int KIND = decltype(kind_c)::value;
      const const_dptr tab = psi_tab();
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int b = 16 * ti + mfma_drow<double>(lane, r);
        double xb[DM];
#pragma unroll
        for (int c = 0; c < DM; ++c) xb[c] = xnew[(size_t)min(b, B - 1) * d + min(c, d - 1)];
#pragma unroll
        for (int g = 0; g < 2; ++g) {
          double r2 = 0.0;
#pragma unroll
          for (int c = 0; c < DM; ++c) {
            const double t = (xb[c] - xkv[g][c]) * il[c];
            r2 = fma(t, (c < d) ? t : 0.0, r2);
          }
          kv[g][r] = os * kernel_term_nc<KIND>(r2, tab);
          asm("" : "+v"(kv[g][r]));  // rounded here, never fused into the epilogue's subtraction (posterior_cov_body)
          zero_r2 |= (r2 == 0.0 ? 1u : 0u) << (g * 4 + r);
        }
      }
    };
    switch (kind) {
      case DKG_MATERN12: terms(std::integral_constant<int, DKG_MATERN12>{}); break;
      case DKG_MATERN32: terms(std::integral_constant<int, DKG_MATERN32>{}); break;
      case DKG_RBF: terms(std::integral_constant<int, DKG_RBF>{}); break;
      default: terms(std::integral_constant<int, DKG_MATERN52>{}); break;
    }
  }
  const bool want_var = bx == 0;  // the block's line tiles include tile 0: the wave's candidates' variances
  d4 acc[2][4], sum0[2];
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    sum0[g] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[g][q] = d4{0.0, 0.0, 0.0, 0.0};
  }
  double qsq = 0.0, qh0 = 0.0;
  KST(st, 2);
  for (int c = 0; c < nc; ++c) {
    static_assert(PK_NSTG >= 2 && PK_NSTG <= 3, "vmcnt cases");
    const int later = min(nc - 1 - c, PK_NSTG - 2);  // chunks issued after c (wave-uniform)
    if (later >= 1) {
      if constexpr (PIECES == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_barrier" ::: "memory");  // (no workgroup fence: it would wait for every DMA in flight)
    if (c + PK_NSTG - 1 < nc) stage(c + PK_NSTG - 1);
    if (c == nc0) {  // half 0 done: its sums, and the chains restart for half 1
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        sum0[g] = (acc[g][0] + acc[g][1]) + (acc[g][2] + acc[g][3]);
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[g][q] = d4{0.0, 0.0, 0.0, 0.0};
      }
      if (want_var) {
        double q = qsq;
        q += __shfl_xor(q, 16);
        q += __shfl_xor(q, 32);
        qh0 = q;
        qsq = 0.0;
      }
    }
    const v2d* bufw = stg + (size_t)(c % PK_NSTG) * PK_STAGE + lane;
    const int nw = chunk_words(c);  // wave-uniform
    // word w of the chunk: k-blocks 2 j, 2 j + 1 of the half (j = its word from the half's start, j = w mod 2):
    // chains 2 (w & 1) and 2 (w & 1) + 1
    auto word = [&](int w) __attribute__((always_inline)) {
      const v2d a = bufw[(wave * PK_WC + w) * 64];
      const v2d b0 = bufw[(PK_RT * PK_WC + w) * 64];
      const v2d b1 = bufw[((PK_RT + 1) * PK_WC + w) * 64];
      const int ch = 2 * (w & 1);
      acc[0][ch] = mfma_f64(a.x, b0.x, acc[0][ch]);
      acc[1][ch] = mfma_f64(a.x, b1.x, acc[1][ch]);
      acc[0][ch + 1] = mfma_f64(a.y, b0.y, acc[0][ch + 1]);
      acc[1][ch + 1] = mfma_f64(a.y, b1.y, acc[1][ch + 1]);
      if (want_var) {
        qsq = fma(a.x, a.x, qsq);
        qsq = fma(a.y, a.y, qsq);
      }
    };
    if (nw == PK_WC) {  // a whole chunk: straight-line code, hipcc interleaves the reads with the MFMAs
#pragma unroll
      for (int w = 0; w < PK_WC; ++w) word(w);
    } else {
#pragma unroll
      for (int w = 0; w < PK_WC; ++w)
        if (w < nw) word(w);
    }
  }
  KST(st, 3);
  const int rec = cov_rec(P->m);
  int le = lane;
  asm volatile("" : "+v"(le));  // store addresses formed here, not hoisted across the loop
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const d4 tot = sum0[g] + ((acc[g][0] + acc[g][1]) + (acc[g][2] + acc[g][3]));  // half 0 + half 1
    const int k = 16 * (tk0 + g) + (le & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int b = 16 * ti + mfma_drow<double>(le, r);
      if (b < B && k < N) {
        P->cov_all[(size_t)b * P->cov_stride + (size_t)k * rec + oi] = kv[g][r] - tot[r];
        if (DKG_DUP_MARK && ((zero_r2 >> (g * 4 + r)) & 1)) atomicMin(&P->dup[b], k);  // Plan::dup
      }
    }
  }
  if (want_var) {
    double q = qsq;
    q += __shfl_xor(q, 16);
    q += __shfl_xor(q, 32);
    const int bb = 16 * ti + lane;
    if (lane < 16 && bb < B) P->var[oi][bb] = os - (qh0 + q);
  }
  KST_END(st);
}

// ---------------------------------------------------------------------------
// posterior_cov_big32_kernel (DKG_PLAN_F32, BASELINE configs[4]): posterior_cov_big_kernel's 64 x 64 blocks on
// v_mfma_f32_16x16x4_f32.  Same block, wave and staging geometry (4 waves, each a 2 x 2 group of 16 x 16 tiles;
// the operand panels of a block staged once by LDS-DMA; the kernel terms evaluated while the first chunks land
// and parked in LDS), fp32 operands quad-packed (Plan::q32 / disc32: four k-blocks per 16-byte word).  An fp32
// MFMA issues in 32 cycles against the fp64 one's 64, and a 16-byte word carries four k-blocks instead of two,
// so a word feeds 16 MFMAs per wave at the fp64 kernel's LDS bytes per MFMA cycle: half the words, half the
// time.  No bit-replay constraint (the fp32 plan has no other big-block path to agree with): one fp32
// accumulator per tile and chunk (an f32 MFMA's dependent latency, 40 cycles, is covered by the other three
// tiles' MFMAs), added into fp64 sums at the next chunk's start, so only 8-term partial sums round in fp32
// (one fp32 chain over n = 1024 terms had 3x the slope error of posterior_cov_body<float>'s eight chains).
// The panels arrive by glds16 (hidden from hipcc) and are read with plain LDS loads.  Kernel terms,
// subtraction and variances in fp64, as posterior_cov_body<float>.
constexpr int PB32_WC = 2;  // 16-byte words (four k-blocks each) per staged chunk
#ifndef DKG_PB32_NSTG
#define DKG_PB32_NSTG 3
#endif
constexpr int PB32_NSTG = DKG_PB32_NSTG;
constexpr int PB32_STAGE = (PB_RT + PB_CT) * PB32_WC * 64;  // 16-byte words per stage buffer
constexpr size_t PB32_LDS = PB32_NSTG * (size_t)PB32_STAGE * 16 + (size_t)PB_WAVES * 16 * 64 * 8;

template <int DM>
__global__ __launch_bounds__(PB_WAVES * WAVE) __attribute__((amdgpu_waves_per_eu(2))) void posterior_cov_big32_kernel(
    const Plan* __restrict__ P, const double* __restrict__ xnew, int B, int dst, int order) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  typedef float v4f __attribute__((ext_vector_type(4)));
  v4f* stg = reinterpret_cast<v4f*>(smem);  // 16-byte words
  const int N = P->N;
  const int nbx = (N + 16 * PB_CT - 1) / (16 * PB_CT), nby = (B + 16 * PB_RT - 1) / (16 * PB_RT);
  int bx, by, oi;
  if (!block_order(blockIdx.x, nbx, nby, P->m, order, bx, by, oi)) return;
  unsigned long long* st = kst_slot(dst, P, 1);
  KST_BEGIN(st);
  const dkg_output& o = P->o[oi];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int rp = wave & 1, cp = wave >> 1;  // the wave's tiles: rows 2 rp, 2 rp + 1; columns 2 cp, 2 cp + 1
  const int RT = pad16(B) / 16, CT = pad16(N) / 16;
  const int KB = pad16(o.n) / 4, KP = KB / 4;  // quad words
  const int ti0 = PB_RT * by, tk0 = PB_CT * bx;
  const float* qx = P->q32[oi];
  const float* qd = P->disc32[oi];
  const int nc = (KP + PB32_WC - 1) / PB32_WC;
  constexpr int PIECES = (PB_RT + PB_CT) * PB32_WC / PB_WAVES;
  static_assert((PB_RT + PB_CT) * PB32_WC % PB_WAVES == 0 && PIECES == 4, "four DMA pieces per wave per chunk");
  const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>(stg);
  auto stage = [&](int c) {  // chunk c's panels into buffer c % PB32_NSTG (glds16: counted by vmcnt below)
    const int j0 = c * PB32_WC, nw = min(PB32_WC, KP - j0);
    const uint32_t buf = lds0 + (uint32_t)((c % PB32_NSTG) * PB32_STAGE) * 16u;
#pragma unroll
    for (int q = 0; q < PIECES; ++q) {
      const int piece = wave + PB_WAVES * q;
      const int t = piece / PB32_WC, w = min(piece % PB32_WC, nw - 1);
      const float* src = t < PB_RT ? qx : qd;
      const int tile = t < PB_RT ? min(ti0 + t, RT - 1) : min(tk0 + t - PB_RT, CT - 1);
      glds16(src + (((size_t)tile * KP + j0 + w) * 64 + lane) * 4, buf + (uint32_t)piece * 1024u);
    }
  };
  const bool want_var = bx == 0 && cp == 0;  // the wave's column tiles include tile 0: its row tiles' variances
  // fp32 MFMA partial sums of one chunk (8 k-blocks), added into fp64 sums at the next chunk's start (the
  // results have long landed by then): the contraction accumulates in fp64 but for the 8-term chunk sums
  f4 acc[2][2];
  d4 sum[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      acc[h][g] = f4{0.f, 0.f, 0.f, 0.f};
      sum[h][g] = d4{0.0, 0.0, 0.0, 0.0};
    }
  double qsq[2] = {0.0, 0.0};
#pragma unroll
  for (int c = 0; c < PB32_NSTG - 1; ++c)
    if (c < nc) stage(c);
  const double os = o.outputscale;
  double* kvs = reinterpret_cast<double*>(stg + (size_t)PB32_NSTG * PB32_STAGE) + (size_t)wave * 16 * 64;
  const uint32_t zero_r2 = big_block_terms<DM, float>(P, o, xnew, B, ti0 + 2 * rp, tk0 + 2 * cp, lane, kvs);
  KST(st, 2);
  for (int c = 0; c < nc; ++c) {
    // chunk c landed (this wave's pieces), then every wave's; the later chunks' DMAs stay in flight
    static_assert(PB32_NSTG >= 2 && PB32_NSTG <= 3, "vmcnt cases");
    const int later = min(nc - 1 - c, PB32_NSTG - 2);  // chunks issued after c (wave-uniform)
    if (later >= 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_barrier" ::: "memory");  // (no workgroup fence: it would wait for every DMA in flight)
    if (c + PB32_NSTG - 1 < nc) stage(c + PB32_NSTG - 1);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int g = 0; g < 2; ++g) {
#pragma unroll
        for (int r = 0; r < 4; ++r) sum[h][g][r] += (double)acc[h][g][r];
        acc[h][g] = f4{0.f, 0.f, 0.f, 0.f};
      }
    const v4f* bufw = stg + (size_t)(c % PB32_NSTG) * PB32_STAGE + lane;
    const int nw = min(PB32_WC, KP - c * PB32_WC);  // wave-uniform
    v4f fa0[PB32_WC], fa1[PB32_WC], fb0[PB32_WC], fb1[PB32_WC];  // every word read up front (slots past nw repeat a live word)
#pragma unroll
    for (int w = 0; w < PB32_WC; ++w) {
      fa0[w] = bufw[((2 * rp) * PB32_WC + w) * 64];
      fa1[w] = bufw[((2 * rp + 1) * PB32_WC + w) * 64];
      fb0[w] = bufw[((PB_RT + 2 * cp) * PB32_WC + w) * 64];
      fb1[w] = bufw[((PB_RT + 2 * cp + 1) * PB32_WC + w) * 64];
    }
#pragma unroll
    for (int w = 0; w < PB32_WC; ++w) {
      if (w < nw) {  // (nw < PB32_WC only for an odd word count: the last chunk)
        const v4f a0 = fa0[w], a1 = fa1[w], b0 = fb0[w], b1 = fb1[w];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          acc[0][0] = mfma_f32(a0[q], b0[q], acc[0][0]);
          acc[0][1] = mfma_f32(a0[q], b1[q], acc[0][1]);
          acc[1][0] = mfma_f32(a1[q], b0[q], acc[1][0]);
          acc[1][1] = mfma_f32(a1[q], b1[q], acc[1][1]);
        }
        if (want_var) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            qsq[0] = fma((double)a0[q], (double)a0[q], qsq[0]);
            qsq[1] = fma((double)a1[q], (double)a1[q], qsq[1]);
          }
        }
      }
    }
  }
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int r = 0; r < 4; ++r) sum[h][g][r] += (double)acc[h][g][r];
  KST(st, 3);
  const int rec = cov_rec(P->m);
  int le = lane;
  asm volatile("" : "+v"(le));  // store addresses formed here (posterior_cov_big_kernel)
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int k = 16 * (tk0 + 2 * cp + g) + (le & 15);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int b = 16 * (ti0 + 2 * rp + h) + mfma_drow<float>(le, r);
        const int e = (g * 2 + h) * 4 + r;
        if (b < B && k < N) {
          P->cov_all[(size_t)b * P->cov_stride + (size_t)k * rec + oi] = kvs[e * 64 + le] - sum[h][g][r];
          if (DKG_DUP_MARK && ((zero_r2 >> e) & 1)) atomicMin(&P->dup[b], k);  // Plan::dup
        }
      }
  }
  if (want_var) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      double q = qsq[h];
      q += __shfl_xor(q, 16);
      q += __shfl_xor(q, 32);
      const int bb = 16 * (ti0 + 2 * rp + h) + lane;
      if (lane < 16 && bb < B) P->var[oi][bb] = os - q;
    }
  }
  KST_END(st);
}

// ---------------------------------------------------------------------------
// cross_big_kernel (fp64 forward, launches with the K(x, X) fill, cross_kfill_launch): Q_X = K(x, X) R for
// 64 x 32 blocks (4 candidate tiles x 2 column tiles of Q, one output) with cross_root_impl's arithmetic
// element for element, so the two give the same bits and the choice is a speed matter only.  cross_root_impl
// sums column tile tj of Q over the k range of its pair (tj, T - 1 - tj) split in 8 wave chunks of
// cw = ceil(kbW / 16) words (kbW = 4 (max(tj, T - 1 - tj) + 1) k-blocks), each chunk as two k-block-parity
// chains of MFMAs (R^T as the A operand, K as the B operand) added, the chunks summed in order from 0; the
// tile's k range ends at 4 (tj + 1) (R upper triangular).  Here wave w keeps those chains and running sums for
// column tile w % 2 against candidate tiles 2 (w / 2) and 2 (w / 2) + 1, flushing the chains at the tile's chunk
// ends.  Operands staged through LDS by LDS-DMA as in posterior_cov_big_kernel: K is read once per 32 columns
// instead of once per column pair, R once per 64 candidates instead of 16 (the stress cross stage's L2
// fetches).  Blocks of 32 columns: the longest (k = n) takes 128 words x 4 MFMAs per wave at n = 1024, so the
// triangle's longest blocks are not the whole stage; they are dispatched first, and the candidate blocks of one
// column block and output sit side by side on one XCD (xcd_group), sharing its R panel.
#ifndef DKG_XB_WAVES
#define DKG_XB_WAVES 4
#endif
constexpr int XB_WAVES = DKG_XB_WAVES;  // 4; 2 (32 x 32 blocks, twice the workgroups) was slower: stress cross
                                        // 43.7 -> 48.6 us, headline x 10 21.2 -> 24.4 us
constexpr int XB_TT = 2;  // column tiles of Q (row tiles of R^T) per block
constexpr int XB_RT = XB_WAVES == 2 ? 2 : 4;  // candidate tiles per block
constexpr int XB_WC = 4;  // words per staged chunk (one barrier per 16 MFMAs per wave)
constexpr int XB_STAGE = (XB_TT + XB_RT) * XB_WC * 64;  // 16-byte words per stage buffer
#ifndef DKG_XB_NSTG
#define DKG_XB_NSTG 3
#endif
constexpr int XB_NSTG = DKG_XB_NSTG;  // stage buffers: chunks in flight during the current one's MFMAs
constexpr size_t XB_LDS = XB_NSTG * (size_t)XB_STAGE * 16;

__host__ __device__ inline int cross_big_blocks(int max_np, int B, int m) {
  const int nbj = (max_np / 16 + XB_TT - 1) / XB_TT, nbi = (pad16(B) / 16 + XB_RT - 1) / XB_RT;
  return xcd_group_size(nbj * m, nbi);
}

// One block of cross_big_kernel (dkg_kernels.hip: the launch also holds the means' workgroups), L its index.
__device__ __forceinline__ void cross_big_body(const Plan* __restrict__ P, int B, int L, double* smem) {
  double2* stg = reinterpret_cast<double2*>(smem);
  const int m = P->m;
  const int RT = pad16(B) / 16, nbi = (RT + XB_RT - 1) / XB_RT;
  const int nbj = (P->max_np / 16 + XB_TT - 1) / XB_TT;
  int blk, bi;
  if (!xcd_group(L, nbj * m, nbi, blk, bi)) return;
  const int bj = nbj - 1 - blk / m, oi = blk % m;
  const dkg_output& o = P->o[oi];
  const int np = pad16(o.n), T = np / 16, KB = np / 4, KP = KB / 2;
  const int tj0 = XB_TT * bj, ti0 = XB_RT * bi;
  if (tj0 >= T) return;  // an output with fewer training points than the widest
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int rp = wave % XB_TT, cp = wave / XB_TT;  // column tile tj0 + rp; candidate tiles ti0 + 2 cp, + 1
  const double* rt = o.root_frag;
  const double* kx = P->kx[oi];
  const int W = 2 * min(tj0 + XB_TT, T);  // words the block reads: its last live column tile's k range
  const int nc = (W + XB_WC - 1) / XB_WC;
  constexpr int XB_PIECES = (XB_TT + XB_RT) * XB_WC / XB_WAVES;
  static_assert((XB_TT + XB_RT) * XB_WC % XB_WAVES == 0 && (XB_PIECES == 6 || XB_PIECES == 8), "DMA pieces per wave");
  auto stage = [&](int c) {
    const int j0 = c * XB_WC, nw = min(XB_WC, W - j0);
    double2* buf = stg + (size_t)(c % XB_NSTG) * XB_STAGE;
#pragma unroll
    for (int q = 0; q < XB_PIECES; ++q) {
      const int piece = wave + XB_WAVES * q;
      const int t = piece / XB_WC, w = min(piece % XB_WC, nw - 1);
      const double* src = t < XB_TT ? rt : kx;
      const int tile = t < XB_TT ? min(tj0 + t, T - 1) : min(ti0 + t - XB_TT, RT - 1);
      __builtin_amdgcn_global_load_lds(
          reinterpret_cast<const void*>(src + (((size_t)tile * KP + j0 + w) * 64 + lane) * 2),
          reinterpret_cast<__attribute__((address_space(3))) void*>(reinterpret_cast<uintptr_t>(buf + piece * 64)),
          16, 0, 0);
    }
  };
  // the wave's column tile: live, k extent in words, chunk width in words (cross_root_impl's pair split)
  const int tj = tj0 + rp;
  const bool live = tj < T;
  const int E = 2 * (tj + 1);
  const int CW = (2 * (max(tj, T - 1 - tj) + 1) + CR_WAVES - 1) / CR_WAVES;  // kbW / 2 words over 8 chunks
  typedef double v2d __attribute__((ext_vector_type(2)));
  const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>(stg);
  const uint32_t addrA = lds0 + (uint32_t)((rp * XB_WC) * 64 + lane) * 16;
  const uint32_t addrB = lds0 + (uint32_t)(((XB_TT + 2 * cp) * XB_WC) * 64 + lane) * 16;
  d4 ch[2][2], sum[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    sum[h] = d4{0.0, 0.0, 0.0, 0.0};
    ch[h][0] = ch[h][1] = d4{0.0, 0.0, 0.0, 0.0};
  }
  int seg_left = CW;  // words left in the current chunk of cross_root_impl's split
#pragma unroll
  for (int c = 0; c < XB_NSTG - 1; ++c)
    if (c < nc) stage(c);
  for (int c = 0; c < nc; ++c) {
    // chunk c landed: the chunks issued after it (at most XB_NSTG - 2, XB_PIECES pieces each) may stay in flight
    static_assert(XB_NSTG >= 2 && XB_NSTG <= 4, "vmcnt cases");
    switch (min(nc - 1 - c, XB_NSTG - 2) * XB_PIECES) {  // wave-uniform
      case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
      case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
      case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
      case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
      default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
    asm volatile("s_barrier" ::: "memory");  // (posterior_cov_big_kernel: no workgroup fence, no vmcnt(0))
    if (c + XB_NSTG - 1 < nc) stage(c + XB_NSTG - 1);
    const int j0 = c * XB_WC;
    if (!(live && j0 < E)) continue;  // wave-uniform: this tile's k range is done (the stores come last)
    const uint32_t so = (uint32_t)(c % XB_NSTG) * (uint32_t)(XB_STAGE * 16);
    const uint32_t aA = addrA + so, aB = addrB + so;
    const int nw = min(XB_WC, E - j0);  // words of this tile in the chunk (even, wave-uniform)
    // word j: the R^T fragment of the wave's column tile and the K fragments of its two candidate tiles, then
    // k-blocks 2 j (chain 0) and 2 j + 1 (chain 1); the chains join the sums at the tile's chunk ends and at its
    // extent.  Two words per iteration in register sets X and Y, each set's reads issued before the other
    // set's MFMAs (LDS reads complete in order: lgkmcnt(3) = the older set has landed); a rolled loop, so the
    // flush branch's paths keep the chains in the same registers (unrolled over the chunk, the merges copied
    // MFMA results between words and waited for them every word).
    auto mfmas = [&](const v2d& a, const v2d& b0, const v2d& b1, int j) __attribute__((always_inline)) {
      ch[0][0] = mfma_f64(a.x, b0.x, ch[0][0]);
      ch[1][0] = mfma_f64(a.x, b1.x, ch[1][0]);
      ch[0][1] = mfma_f64(a.y, b0.y, ch[0][1]);
      ch[1][1] = mfma_f64(a.y, b1.y, ch[1][1]);
      if (--seg_left == 0 || j + 1 == E) {  // wave-uniform
        seg_left = CW;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          sum[h] += ch[h][0] + ch[h][1];
          ch[h][0] = ch[h][1] = d4{0.0, 0.0, 0.0, 0.0};
        }
      }
    };
    v2d xa, xb0, xb1, ya, yb0, yb1;
    asm volatile("ds_read_b128 %0, %3\n\tds_read_b128 %1, %4\n\tds_read_b128 %2, %4 offset:%5"
                 : "=&v"(xa), "=&v"(xb0), "=&v"(xb1)
                 : "v"(aA), "v"(aB), "i"(XB_WC * 1024)
                 : "memory");
#pragma unroll 1
    for (int w = 0; w < nw; w += 2) {  // nw even
      const uint32_t o = (uint32_t)(w + 1) * 1024u;
      // set Y's rewrite follows set Y's MFMAs of the previous pair by only set X's rewrite: eight wait states
      // first, so at least 16 issue cycles separate an MFMA from a rewrite of its operands on every path
      // (tools/asm_audit.py checks the compiled kernel; the MFMA pipe keeps Y's queued MFMAs running meanwhile)
      asm volatile("s_nop 7\n\tds_read_b128 %0, %3\n\tds_read_b128 %1, %4\n\tds_read_b128 %2, %4 offset:%5"
                   : "=&v"(ya), "=&v"(yb0), "=&v"(yb1)
                   : "v"(aA + o), "v"(aB + o), "i"(XB_WC * 1024)
                   : "memory");
      asm volatile("s_waitcnt lgkmcnt(3)" : "+v"(xa), "+v"(xb0), "+v"(xb1));
      mfmas(xa, xb0, xb1, j0 + w);
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(ya), "+v"(yb0), "+v"(yb1));
      mfmas(ya, yb0, yb1, j0 + w + 1);
      // set X is rewritten only after set Y's MFMAs have issued: the MFMA pipe is in order, so X's MFMAs have
      // read their operands (a rewrite right after X's own MFMAs changed results).  The rewrite is inline asm
      // with no data dependence on Y's MFMAs (memory-free builtins the scheduler may move across asm, and the
      // hazard recognizer does not see into asm): a scheduling barrier holds the order.
      __builtin_amdgcn_sched_barrier(0);
      if (w + 2 < nw) {
        const uint32_t o2 = (uint32_t)(w + 2) * 1024u;
        asm volatile("ds_read_b128 %0, %3\n\tds_read_b128 %1, %4\n\tds_read_b128 %2, %4 offset:%5"
                     : "=&v"(xa), "=&v"(xb0), "=&v"(xb1)
                     : "v"(aA + o2), "v"(aB + o2), "i"(XB_WC * 1024)
                     : "memory");
      }
      __builtin_amdgcn_sched_barrier(0);  // (the next iteration's set-Y rewrite stays after these)
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (!live) return;
  // D = R^T K^T: lane l, register r holds Q[16 ti + (l & 15)][16 tj + dr], dr = (l >> 4) + 4 r (cross_root_impl)
  double* qout = P->q[oi];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int ti = ti0 + 2 * cp + h;
    if (ti >= RT) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int dr = mfma_drow<double>(lane, r);
      qout[frag_index(ti, 4 * tj + (dr >> 2), (lane & 15) | ((dr & 3) << 4), KB)] = sum[h][r];
    }
  }
}

// ---------------------------------------------------------------------------
// cross_big32 (DKG_PLAN_F32 with the K(x, X) fill): cross_big_body's 64 x 32 blocks on v_mfma_f32_16x16x4_f32,
// R^T and K(x, X) quad-packed in fp32 (Plan::root32, Plan::kx32 written by the fill), Q_X written quad-packed
// (Plan::q32, the covariance stage's A operand).  Column tile tj needs the words j < tj + 1 (k-blocks
// < 4 (tj + 1): R upper triangular).  No bit-replay constraint: per candidate tile two fp32 chains (k-block
// parity: an f32 MFMA's dependent latency is 40 cycles against the 32-cycle issue of the one MFMA between),
// added into fp64 sums at every chunk's start (16-term fp32 partial sums, as the split-K chunks of
// cross_root_impl<float>); XB32_WC words per chunk (32 MFMAs per wave between barriers).  Panels by glds16,
// read with plain LDS loads (posterior_cov_big32_kernel).
constexpr int XB32_WC = 4;
constexpr int XB32_NSTG = 3;
constexpr int XB32_STAGE = (XB_TT + XB_RT) * XB32_WC * 64;  // 16-byte words per stage buffer
constexpr size_t XB32_LDS = XB32_NSTG * (size_t)XB32_STAGE * 16;

__device__ __forceinline__ void cross_big32_body(const Plan* __restrict__ P, int B, int L, double* smem) {
  static_assert(XB_WAVES == 4 && XB_RT == 4, "the fp32 blocks keep the fp64 blocks' 4-wave geometry");
  typedef float v4f __attribute__((ext_vector_type(4)));
  v4f* stg = reinterpret_cast<v4f*>(smem);
  const int m = P->m;
  const int RT = pad16(B) / 16, nbi = (RT + XB_RT - 1) / XB_RT;
  const int nbj = (P->max_np / 16 + XB_TT - 1) / XB_TT;
  int blk, bi;
  if (!xcd_group(L, nbj * m, nbi, blk, bi)) return;
  const int bj = nbj - 1 - blk / m, oi = blk % m;
  const dkg_output& o = P->o[oi];
  const int np = pad16(o.n), T = np / 16, KB = np / 4, KP = KB / 4;
  const int tj0 = XB_TT * bj, ti0 = XB_RT * bi;
  if (tj0 >= T) return;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int rp = wave % XB_TT, cp = wave / XB_TT;  // column tile tj0 + rp; candidate tiles ti0 + 2 cp, + 1
  const float* rt = P->root32[oi];
  const float* kx = P->kx32[oi];
  const int W = min(tj0 + XB_TT, T);  // quad words the block reads: its last live column tile's k range
  const int nc = (W + XB32_WC - 1) / XB32_WC;
  constexpr int PIECES = (XB_TT + XB_RT) * XB32_WC / XB_WAVES;
  static_assert(PIECES == 6, "six DMA pieces per wave per chunk");
  const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>(stg);
  auto stage = [&](int c) {
    const int j0 = c * XB32_WC, nw = min(XB32_WC, W - j0);
    const uint32_t buf = lds0 + (uint32_t)((c % XB32_NSTG) * XB32_STAGE) * 16u;
#pragma unroll
    for (int q = 0; q < PIECES; ++q) {
      const int piece = wave + XB_WAVES * q;
      const int t = piece / XB32_WC, w = min(piece % XB32_WC, nw - 1);
      const float* src = t < XB_TT ? rt : kx;
      const int tile = t < XB_TT ? min(tj0 + t, T - 1) : min(ti0 + t - XB_TT, RT - 1);
      glds16(src + (((size_t)tile * KP + j0 + w) * 64 + lane) * 4, buf + (uint32_t)piece * 1024u);
    }
  };
  const int tj = tj0 + rp;
  const bool live = tj < T;
  const int E = tj + 1;  // the tile's quad words
  f4 ch[2][2];
  d4 sum[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    ch[h][0] = ch[h][1] = f4{0.f, 0.f, 0.f, 0.f};
    sum[h] = d4{0.0, 0.0, 0.0, 0.0};
  }
  auto flush = [&]() {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int r = 0; r < 4; ++r) sum[h][r] += (double)ch[h][0][r] + (double)ch[h][1][r];
      ch[h][0] = ch[h][1] = f4{0.f, 0.f, 0.f, 0.f};
    }
  };
#pragma unroll
  for (int c = 0; c < XB32_NSTG - 1; ++c)
    if (c < nc) stage(c);
  for (int c = 0; c < nc; ++c) {
    if (min(nc - 1 - c, XB32_NSTG - 2) >= 1) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // wave-uniform
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_barrier" ::: "memory");
    if (c + XB32_NSTG - 1 < nc) stage(c + XB32_NSTG - 1);
    const int j0 = c * XB32_WC;
    if (!(live && j0 < E)) continue;  // wave-uniform: this tile's k range is done
    flush();  // the previous chunk's chains (landed long ago) into the fp64 sums
    const v4f* bufw = stg + (size_t)(c % XB32_NSTG) * XB32_STAGE + lane;
    const int nw = min(XB32_WC, E - j0);  // wave-uniform, 1 .. XB32_WC
    // every word of the chunk read up front (the stage fills all XB32_WC slots, repeating a live word past the
    // block's range, so the reads past nw are defined), the MFMAs of the tile's words only
    v4f a[XB32_WC], b0[XB32_WC], b1[XB32_WC];
#pragma unroll
    for (int w = 0; w < XB32_WC; ++w) {
      a[w] = bufw[(rp * XB32_WC + w) * 64];
      b0[w] = bufw[((XB_TT + 2 * cp) * XB32_WC + w) * 64];
      b1[w] = bufw[((XB_TT + 2 * cp + 1) * XB32_WC + w) * 64];
    }
    // words past the tile's range take a zero R^T operand (branch-free: the waits stay counted per word)
#pragma unroll
    for (int w = 0; w < XB32_WC; ++w) {
      const bool lw = w < nw;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float aq = lw ? a[w][q] : 0.f;
        ch[0][q & 1] = mfma_f32(aq, b0[w][q], ch[0][q & 1]);
        ch[1][q & 1] = mfma_f32(aq, b1[w][q], ch[1][q & 1]);
      }
    }
  }
  if (!live) return;
  flush();
  // D = R^T K^T in the f32 D map: lane l, register r holds Q[16 ti + (l & 15)][16 tj + 4 (l >> 4) + r]
  float* qout = P->q32[oi];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int ti = ti0 + 2 * cp + h;
    if (ti >= RT) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int dr = mfma_drow<float>(lane, r);
      qout[frag32_index(ti, 4 * tj + (dr >> 2), (lane & 15) | ((dr & 3) << 4), KB)] = (float)sum[h][r];
    }
  }
}

// (DKG_PC_WPE 4 holds it to 128 VGPRs, so two blocks share a CU, but spills 20 bytes a lane: one forward's stage
// 7.9 -> 8.7 us (profiles/r06/cov/blk_h_pcw2.txt against blk_h_blk.txt); the default lets it take 130.)
#ifndef DKG_PC_WPE
#define DKG_PC_WPE 2
#endif
template <int DM, class T = double>
__global__ __launch_bounds__(PC_WAVES * WAVE) __attribute__((amdgpu_waves_per_eu(DKG_PC_WPE))) void posterior_cov_kernel(const Plan* __restrict__ P,
                                                                         const double* __restrict__ xnew, int B,
                                                                         int dst) {
  __shared__ __attribute__((aligned(16))) double part[(PC_KS - 1) * 2 * PC_RB * 4 * 64];  // K-split 1.. partial tiles
  __shared__ double qpart[(PC_KS - 1) * 2 * PC_RB * 16];
  unsigned long long* st = kst_slot(dst, P, 1);
  if (DKG_ABLATIONS && (__builtin_amdgcn_readfirstlane(P->debug_cov) & 1)) return;  // ablation: empty covariance stage
  // 1-D grid, the outputs of one 32 x 32 block side by side on one XCD (xcd_group)
  const int nbx = max(1, (P->N + 31) / 32), nby = (B + 16 * PC_RB - 1) / (16 * PC_RB);
  int blk, oi;
  if (!xcd_group(blockIdx.x, nbx * nby, P->m, blk, oi)) return;
  posterior_cov_body<DM, T>(P, xnew, B, blk % nbx, blk / nbx, oi, part, qpart, st);
}

}  // namespace dkg
