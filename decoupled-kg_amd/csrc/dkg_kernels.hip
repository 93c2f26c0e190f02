// HIP kernels of the Discrete-KG hot path for gfx950 (MI355X, CDNA4).
//
// Pipeline per forward (DESIGN.md "Kernels"):
//   cross_root_kernel   Q = K(x, X) R  (fp64 MFMA, R upper triangular), mean = c + K(x,X) alpha
//   posterior_cov_kernel cov[b][k] = s k(x_b, D_k) - Q_b . Q_D[k]   (fp64 MFMA GEMM, split-K)
//   envelope_kernel     lines a_k + b_k z per (candidate, scalarisation), upper
//                       envelope, closed-form Gaussian expectation, mean over S
#include "dkg_common.h"
#include "dkg_kernels.h"

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
// K(x, X) tile is evaluated once into LDS in B-operand order and the k range
// is split over the 8 waves (split-K), partials reduced in LDS in fixed order.
constexpr int CR_WAVES = 8;

__global__ __launch_bounds__(CR_WAVES * WAVE) void cross_root_kernel(CrossArgs args) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int ti = blockIdx.x;
  const int p = blockIdx.y;
  const int oi = blockIdx.z;
  const dkg_output& o = args.outs.o[oi];
  const int d = args.d;
  const int rows = args.rows;
  const int n = o.n;
  const int np = pad16(n);
  const int T = np / 16;
  const int KB = np / 4;
  const int P = (T + 1) / 2;
  if (p >= P) return;
  const int tA = p, tB = T - 1 - p;       // tA <= tB
  const int kbA = 4 * (tA + 1), kbB = 4 * (tB + 1);  // k-block extents (kbB >= kbA)

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  double* kb_lds = smem;                                   // [kbB][64]
  double* part = smem + (size_t)KB * 64;                   // [CR_WAVES][8][64]
  double* mred = part + CR_WAVES * 8 * 64;                 // [CR_WAVES][16]

  // ---- fill K(x_row, X_col) for col < 4*kbB, in B-operand order.
  const int row = ti * 16 + (lane & 15);
  const bool rv = row < rows;
  double xr[DKG_MAX_DIM];
#pragma unroll
  for (int k = 0; k < DKG_MAX_DIM; ++k) xr[k] = (rv && k < d) ? args.x[(size_t)row * d + k] : 0.0;
  const bool want_mean = (args.mean[oi] != nullptr) && (p == 0);  // p == 0 covers every column
  double mpart = 0.0;
  for (int e = tid; e < kbB * 64; e += CR_WAVES * WAVE) {
    const int col = 4 * (e >> 6) + (lane >> 4);
    double v = 0.0;
    if (rv && col < n) {
      v = o.outputscale *
          kernel_profile(o.kernel, scaled_r2_reg(xr, o.train_x + (size_t)col * d, o.inv_lengthscale, d));
      if (want_mean) mpart = fma(v, o.alpha[col], mpart);
    }
    kb_lds[e] = v;
  }
  __syncthreads();

  // ---- split-K MFMA over the pair.
  const double* rfA = o.root_frag + (size_t)tA * KB * 64 + lane;
  const double* rfB = o.root_frag + (size_t)tB * KB * 64 + lane;
  const int chunk = (kbB + CR_WAVES - 1) / CR_WAVES;
  const int k0 = wave * chunk;
  const int k1 = min(kbB, k0 + chunk);
  d4 accA = {0.0, 0.0, 0.0, 0.0};
  d4 accB = {0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
  for (int kb = k0; kb < k1; ++kb) {
    const double bop = kb_lds[kb * 64 + lane];
    accB = mfma_f64(rfB[(size_t)kb * 64], bop, accB);
    if (kb < kbA && tA != tB) accA = mfma_f64(rfA[(size_t)kb * 64], bop, accA);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    part[(wave * 8 + r) * 64 + lane] = accA[r];
    part[(wave * 8 + 4 + r) * 64 + lane] = accB[r];
  }
  // mean partials: lanes l, l^16, l^32, l^48 share a row.
  if (want_mean) {
    mpart += __shfl_xor(mpart, 16);
    mpart += __shfl_xor(mpart, 32);
    if (lane < 16) mred[wave * 16 + lane] = mpart;
  }
  __syncthreads();

  // ---- reduce partials in fixed wave order; wave w finalises (tile, reg) = w.
  {
    const int tsel = wave >> 2;  // 0 -> tA, 1 -> tB
    const int r = wave & 3;
    const bool active = (tsel == 1) || (tA != tB);
    if (active) {
      double s = 0.0;
      for (int w = 0; w < CR_WAVES; ++w) s += part[(w * 8 + tsel * 4 + r) * 64 + lane];
      const int tj = tsel ? tB : tA;
      // D = R^T K^T: lane holds Q[16ti + (l&15)][16tj + 4r + (l>>4)] = q_frag[ti][4tj + r][l]
      args.q[oi][((size_t)ti * KB + 4 * tj + r) * 64 + lane] = s;
    }
  }
  if (want_mean && tid < 16) {
    double s = 0.0;
    for (int w = 0; w < CR_WAVES; ++w) s += mred[w * 16 + tid];
    const int rr = ti * 16 + tid;
    args.mean[oi][rr] = (rr < rows) ? o.mean_constant + s : 0.0;
  }
  if (args.tickets != nullptr && ti == 0 && p == 0 && oi == 0) {
    for (int i = tid; i < args.n_tickets; i += blockDim.x) args.tickets[i] = 0;
  }
}

size_t cross_root_lds_bytes(int np) { return ((size_t)(np / 4) * 64 + CR_WAVES * 8 * 64 + CR_WAVES * 16) * 8; }

// ---------------------------------------------------------------------------
// posterior_cov_kernel: cov[b][k] = s k(x_b, D_k) - sum_l Q[b][l] Q_D[k][l]
// One workgroup per 16x16 output tile (ti candidates x tk points) per output;
// the 4 waves split the n_pad/4 k-blocks, operands stream straight from the
// fragment-packed arrays (one coalesced 512-byte load per operand per MFMA),
// partials are reduced in LDS in fixed wave order.
constexpr int PC_WAVES = 4;

__global__ __launch_bounds__(PC_WAVES * WAVE) void posterior_cov_kernel(CovArgs args) {
  __shared__ __attribute__((aligned(16))) double part[PC_WAVES * 4 * 64];
  const int tk = blockIdx.x;
  const int ti = blockIdx.y;
  const int oi = blockIdx.z;
  const dkg_output& o = args.outs.o[oi];
  const int N = args.N;
  if (tk * 16 >= N) return;
  const int np = pad16(o.n);
  const int KB = np / 4;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;

  const int chunk = (KB + PC_WAVES - 1) / PC_WAVES;
  const int k0 = wave * chunk;
  const int k1 = min(KB, k0 + chunk);
  const double* qa = args.q[oi] + (size_t)ti * KB * 64 + lane;
  const double* qd = o.disc_frag + (size_t)tk * KB * 64 + lane;
  d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll 8
  for (int kb = k0; kb < k1; ++kb) acc = mfma_f64(qa[(size_t)kb * 64], qd[(size_t)kb * 64], acc);
#pragma unroll
  for (int r = 0; r < 4; ++r) part[(wave * 4 + r) * 64 + lane] = acc[r];
  __syncthreads();

  // wave w finalises register r = w: row b = 16ti + (l>>4) + 4w, col k = 16tk + (l&15)
  const int r = wave;
  double s = 0.0;
#pragma unroll
  for (int w = 0; w < PC_WAVES; ++w) s += part[(w * 4 + r) * 64 + lane];
  const int b = ti * 16 + (lane >> 4) + 4 * r;
  const int k = tk * 16 + (lane & 15);
  if (b < args.B && k < N) {
    const int d = args.d;
    const double kv = o.outputscale * kernel_profile(o.kernel, scaled_r2(args.xnew + (size_t)b * d,
                                                                          args.disc + (size_t)k * d,
                                                                          o.inv_lengthscale, d));
    args.cov[oi][(size_t)b * N + k] = kv - s;
  }
}

// ---------------------------------------------------------------------------
// envelope_kernel: one wave per (candidate b, scalarisation j).
//
// Lines k = 0..N (k = 0 is the candidate itself, discretekg.py:182-183):
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
// The hull: extremes L (min b), R (max b), T by wave reductions; lines above
// the chords L-T / T-R survive into an LDS list; gift-wrapping from L over the
// survivors (argmin of the next intersection, the reference's walk :382-401).
constexpr int ENV_CAP = 128;  // survivor list per wave (overflow -> scan all lines)

struct Key3 {
  double c, b, a;
};

template <int MAXL>
__device__ __forceinline__ double envelope_kg(const double (&la)[MAXL], const double (&lb)[MAXL], int nl, int lane,
                                              double* sb, double* sa, int* nhull) {
  // ---- extremes: T = argmax a; L = min b (tie max a); R = max b (tie max a); max |b|
  double aT = -INFINITY, bT = 0.0;
  double bL = INFINITY, aL = -INFINITY;
  double bR = -INFINITY, aR = -INFINITY;
  double babs = 0.0;
#pragma unroll
  for (int t = 0; t < MAXL; ++t) {
    if (lane + 64 * t < nl) {
      const double a = la[t], bb = lb[t];
      if (a > aT) { aT = a; bT = bb; }
      if (bb < bL || (bb == bL && a > aL)) { bL = bb; aL = a; }
      if (bb > bR || (bb == bR && a > aR)) { bR = bb; aR = a; }
      babs = fmax(babs, fabs(bb));
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const double oaT = __shfl_xor(aT, off), obT = __shfl_xor(bT, off);
    // tie on a: keep the smaller b so every lane agrees (deterministic)
    if (oaT > aT || (oaT == aT && obT < bT)) { aT = oaT; bT = obT; }
    const double obL = __shfl_xor(bL, off), oaL = __shfl_xor(aL, off);
    if (obL < bL || (obL == bL && oaL > aL)) { bL = obL; aL = oaL; }
    const double obR = __shfl_xor(bR, off), oaR = __shfl_xor(aR, off);
    if (obR > bR || (obR == bR && oaR > aR)) { bR = obR; aR = oaR; }
    babs = fmax(babs, __shfl_xor(babs, off));
  }

  double kgj = 0.0;
  int hull = 1;
  // short-circuit of discretekg.py:363-367 (all slopes ~ 0), and the
  // single-slope case: one hull vertex, E = max a, KG = 0.
  if (babs >= 1e-9 && bL < bR) {
    // ---- survivors strictly above the chords L-T and T-R
    int cnt = 0;
#pragma unroll
    for (int t = 0; t < MAXL; ++t) {
      bool s = false;
      const double a = la[t], bb = lb[t];
      if (lane + 64 * t < nl) {
        if (bb < bT) s = (bT > bL) && ((a - aL) * (bT - bL) - (aT - aL) * (bb - bL) > 0.0);
        else if (bb > bT) s = (bR > bT) && ((a - aT) * (bR - bT) - (aR - aT) * (bb - bT) > 0.0);
      }
      const uint64_t mask = __ballot(s);
      if (s) {
        const int pos = cnt + lanes_below(mask);
        if (pos < ENV_CAP) { sb[pos] = bb; sa[pos] = a; }
      }
      cnt += __popcll(mask);
    }
    const bool overflow = cnt + 2 > ENV_CAP;
    if (!overflow && lane == 0) {
      sb[cnt] = bT; sa[cnt] = aT;
      sb[cnt + 1] = bR; sa[cnt + 1] = aR;
    }
    const int ncand = cnt + 2;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // ---- gift wrap from L to R
    double bc = bL, ac = aL;
    for (int guard = 0; guard <= nl && bc < bR; ++guard) {
      Key3 best = {INFINITY, -INFINITY, -INFINITY};
      auto consider = [&](double bb, double a) {
        if (bb > bc) {
          const double c = (ac - a) / (bb - bc);
          if (c < best.c || (c == best.c && bb > best.b)) best = {c, bb, a};
        }
      };
      if (!overflow) {
        for (int e = lane; e < ncand; e += 64) consider(sb[e], sa[e]);
      } else {
#pragma unroll
        for (int t = 0; t < MAXL; ++t)
          if (lane + 64 * t < nl) consider(lb[t], la[t]);
      }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        const double oc = __shfl_xor(best.c, off), ob = __shfl_xor(best.b, off), oa = __shfl_xor(best.a, off);
        if (oc < best.c || (oc == best.c && ob > best.b)) best = {oc, ob, oa};
      }
      if (!(best.b > bc)) break;  // nothing further right (also NaN guard)
      const double db = best.b - bc;
      kgj += db * ((best.b <= bT) ? psi(-best.c) : psi(best.c));
      bc = best.b;
      ac = best.a;
      ++hull;
    }
  }
  if (nhull != nullptr) *nhull = hull;
  return kgj;
}

template <int MAXL>
__global__ __launch_bounds__(512) void envelope_kernel(EnvArgs args) {
  __shared__ double sv[DKG_MAX_OUTPUTS];   // noiseless posterior variance at x_b per output
  __shared__ double smx[DKG_MAX_OUTPUTS];  // posterior mean at x_b per output (model space)
  __shared__ double wsum[16];              // per-wave partial KG sums
  extern __shared__ __attribute__((aligned(16))) double sbuf[];  // [waves][2][ENV_CAP]

  const int b = blockIdx.x;
  const int g = blockIdx.y;
  const int SW = blockDim.x >> 6;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int m = args.m;
  const int N = args.N;
  const int S = args.S;
  const int B = args.B;

  // ---- per-candidate posterior variance v_i = s_i - |Q_i[b]|^2 and mean
  for (int oi = wave; oi < m; oi += SW) {
    const dkg_output& o = args.outs.o[oi];
    const int KB = pad16(o.n) / 4;
    const double* q = args.q[oi] + (size_t)(b >> 4) * KB * 64 + (b & 15);
    double acc = 0.0;
    for (int e = lane; e < KB * 4; e += 64) {
      const double v = q[(size_t)(e >> 2) * 64 + 16 * (e & 3)];
      acc = fma(v, v, acc);
    }
    acc = wave_sum(acc);
    if (lane == 0) {
      sv[oi] = o.outputscale - acc;
      smx[oi] = args.mux[oi][b];
    }
  }
  __syncthreads();

  double* sb = sbuf + (size_t)wave * 2 * ENV_CAP;
  double* sa = sb + ENV_CAP;
  double wave_acc = 0.0;
  const int waves_total = SW * gridDim.y;

  for (int j = g * SW + wave; j < S; j += waves_total) {
    // ---- lines in registers: a = a_off + sum_i wa_i mu_i, b = sum_i wb_i cov_i
    const bool full = args.target < 0;
    double a_off = 0.0, den = 0.0;
    for (int i = 0; i < m; ++i) {
      const dkg_output& o = args.outs.o[i];
      const double w = args.weights[(size_t)j * m + i];
      a_off = fma(w, o.y_mean, a_off);
      if (full) den = fma(w * w, o.y_std * o.y_std * (sv[i] + o.noise), den);
    }
    const double inv_den = full ? 1.0 / sqrt(den) : 0.0;
    double la[MAXL], lb[MAXL];
#pragma unroll
    for (int t = 0; t < MAXL; ++t) {
      la[t] = (lane + 64 * t <= N) ? a_off : -INFINITY;
      lb[t] = 0.0;
    }
#pragma unroll 1
    for (int i = 0; i < m; ++i) {
      const dkg_output& o = args.outs.o[i];
      const double w = args.weights[(size_t)j * m + i];
      const double sd2 = o.y_std * o.y_std;
      const double wa = w * o.y_std;
      double wb = 0.0;
      if (full) wb = w * w * sd2 * inv_den;
      else if (i == args.target) wb = w * sd2 / sqrt(sd2 * (sv[i] + o.noise));
      const double* mu = o.disc_mean - 1;
      const double* cv = args.cov[i] + (size_t)b * N - 1;
      const double mu0 = smx[i], cv0 = sv[i];
#pragma unroll
      for (int t = 0; t < MAXL; ++t) {
        const int k = lane + 64 * t;
        if (k <= N) {
          la[t] = fma(wa, (k == 0) ? mu0 : mu[k], la[t]);
          if (wb != 0.0) lb[t] = fma(wb, (k == 0) ? cv0 : cv[k], lb[t]);
        }
      }
    }

    const double kgj = envelope_kg<MAXL>(la, lb, N + 1, lane, sb, sa, nullptr);
    if (args.pairs_out != nullptr && lane == 0) args.pairs_out[(size_t)b * S + j] = kgj;
    wave_acc += kgj;
  }

  // ---- deterministic mean over S: per-wave sums -> per-WG sum -> last WG sums the WG partials
  if (lane == 0) wsum[wave] = wave_acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int w = 0; w < SW; ++w) s += wsum[w];
    if (gridDim.y == 1) {
      args.kg[b] = s / (double)S;
    } else {
      args.wg_part[(size_t)b * gridDim.y + g] = s;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int prev = atomicAdd(&args.tickets[b], 1);
      if (prev == (int)gridDim.y - 1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        double tot = 0.0;
        for (int q = 0; q < (int)gridDim.y; ++q)
          tot += __hip_atomic_load(&args.wg_part[(size_t)b * gridDim.y + q], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        args.kg[b] = tot / (double)S;
      }
    }
  }
  (void)B;
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
    const int k = lane + 64 * t;
    la[t] = (k < L) ? a[(size_t)p * L + k] : -INFINITY;
    lb[t] = (k < L) ? b[(size_t)p * L + k] : 0.0;
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

hipError_t launch_cross_root(const CrossArgs& a, int m, int max_np, hipStream_t s) {
  const int T = max_np / 16;
  dim3 grid(pad16(a.rows) / 16, (T + 1) / 2, m);
  hipLaunchKernelGGL(cross_root_kernel, grid, dim3(CR_WAVES * WAVE), cross_root_lds_bytes(max_np), s, a);
  return hipGetLastError();
}

hipError_t launch_posterior_cov(const CovArgs& a, int m, hipStream_t s) {
  dim3 grid(pad16(a.N) / 16, pad16(a.B) / 16, m);
  hipLaunchKernelGGL(posterior_cov_kernel, grid, dim3(PC_WAVES * WAVE), 0, s, a);
  return hipGetLastError();
}

void envelope_geometry(int B, int S, int* waves_per_wg, int* split) {
  // Aim for >= 512 workgroups (2 per CU) while keeping up to 8 scalarisation
  // waves of one candidate together.
  int sw = std::max(1, std::min(8, S));
  while (sw > 1 && (long)B * ((S + sw - 1) / sw) < 512) sw /= 2;
  *waves_per_wg = sw;
  *split = (S + sw - 1) / sw;
}

hipError_t launch_envelope(const EnvArgs& a, int sw, int split, hipStream_t s) {
  dim3 grid(a.B, split);
  dim3 block(sw * WAVE);
  const size_t lds = (size_t)sw * 2 * ENV_CAP * sizeof(double);
  const int lines = a.N + 1;
  if (lines <= 64 * 2) hipLaunchKernelGGL(envelope_kernel<2>, grid, block, lds, s, a);
  else if (lines <= 64 * 4) hipLaunchKernelGGL(envelope_kernel<4>, grid, block, lds, s, a);
  else if (lines <= 64 * 8) hipLaunchKernelGGL(envelope_kernel<8>, grid, block, lds, s, a);
  else if (lines <= 64 * 17) hipLaunchKernelGGL(envelope_kernel<17>, grid, block, lds, s, a);
  else if (lines <= 64 * 33) hipLaunchKernelGGL(envelope_kernel<33>, grid, block, lds, s, a);
  else return hipErrorInvalidValue;
  return hipGetLastError();
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

hipError_t launch_debug_mfma(const double* a, const double* b, double* c, hipStream_t s) {
  hipLaunchKernelGGL(debug_mfma_kernel, dim3(1), dim3(64), 0, s, a, b, c);
  return hipGetLastError();
}

}  // namespace dkg
