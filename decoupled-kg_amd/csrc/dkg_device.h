// Device-side envelope stage of the Discrete-KG forward and gradient (gfx950):
// the wave-level upper-envelope machinery and the envelope_kernel template.
// Included by dkg_kernels.hip (lines_kg_kernel) and by the per-output-bucket
// translation units dkg_env_m<M>.hip that instantiate envelope_kernel.
#pragma once

#include <type_traits>

#include "dkg_common.h"
#include "dkg_kernels.h"
#include "dkg_walk.h"

namespace dkg {

// Per-workgroup phase stamps (Plan.debug_stamp, buffer Plan.kstamps [3][KST_WG][8]):
// slot 0 = s_memrealtime at start (100 MHz), 1..6 = s_memtime at phase
// boundaries, 7 = s_memrealtime at end.  `dst` is a kernel argument, so
// production launches pay no dependent load for it.
__device__ __forceinline__ unsigned long long* kst_slot(int dst, const Plan* P, int kid) {
  if (dst != 1) return nullptr;
  const int wg = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
  return (threadIdx.x == 0 && wg < KST_WG) ? P->kstamps + ((size_t)kid * KST_WG + wg) * 8 : nullptr;
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
constexpr int ENV_CAP = 128;
#ifndef DKG_ENV_REFINE
#define DKG_ENV_REFINE 1
#endif
#ifndef DKG_REFINE_OVERFLOW  // a list past ENV_CAP filtered against the chain of its entries
#define DKG_REFINE_OVERFLOW 1
#endif
constexpr int HCAP = 128;  // GRAD: queued envelope lines per wave before their gradient terms are flushed
constexpr int STREAM_CHUNK = 16;  // register slots per streamed chunk (1024 lines)
// Staged forward: the intercepts from the plan's per-scalarisation cache (Plan::icpt) instead of the staged
// mu_D records.  Off by default: the cache rows cost each wave 17 global loads per pair, and the envelope
// was slower with them (profiles/r04/ab: 10.6 -> 11.0 us alone, 11.5 -> 9.9 M KG-evals/s with 4 streams).
#ifndef DKG_ICP
#define DKG_ICP 0
#endif
// The staged forward takes T (max a, tie: min b) from the plan's per-scalarisation top intercept when that
// decides it (TopHint), instead of two wave reductions.
#ifndef DKG_TOP_HINT
#define DKG_TOP_HINT 1
#endif
// Streaming forward with LDS-staged chunks (M = 2..4): the extremes and filter passes read the line
// records from LDS, STAGED_SLOTS * 64 lines per chunk, double-buffered and shared by the workgroup's pairs.
constexpr int STAGED_SLOTS = 8;
__host__ __device__ constexpr bool stream_staged(int M) { return M >= 2 && M <= 4; }
// Doubles of one staged chunk array: the records of the chunk's STAGED_SLOTS * 64 lines, transposed into
// rec / 2 planes of 16-byte component pairs (plane-major), so a lane's 16-byte reads are consecutive
// across the wave (no LDS bank conflict); four arrays: (mu, cov) x 2 buffers.
__host__ __device__ constexpr int staged_chunk_len(int rec) { return STAGED_SLOTS * 64 * rec; }
// Streaming forward (no LDS staging): the survivor list holds up to
// LIST_CAP_STREAM entries per wave; a list that does not fit the hull stage
// (ENV_CAP - 3) is cut down by quickhull rounds (refine_list) instead of the
// gift wrap over all streamed lines.  VCAP: known hull vertices per wave.
constexpr int LIST_CAP_STREAM = 512;
constexpr int VCAP = 64;
__host__ __device__ constexpr int list_cap(bool refine) { return refine ? LIST_CAP_STREAM : ENV_CAP; }
// LDS doubles per wave for the refinement's vertex arrays (vb, va, vn)
constexpr int VREG = 3 * VCAP;

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
  // (raw v_min/v_max: the padding lines' NaN intercepts drop out, see
  // envelope_kernel; the tie passes select a quiet NaN for non-ties)
  double bmin = INFINITY, bmax = -INFINITY, amax = -INFINITY;
#pragma unroll
  for (int t = 0; t < MAXL; ++t) {
    bmin = fmin_raw(bmin, lb[t]);
    bmax = fmax_raw(bmax, lb[t]);
    amax = fmax_raw(amax, la[t]);
  }
  DKG_BUTTERFLY_ROW({
    bmin = fmin_raw(bmin, partner_f64<S_>(bmin));
    bmax = fmax_raw(bmax, partner_f64<S_>(bmax));
    amax = fmax_raw(amax, partner_f64<S_>(amax));
  })
  bmin = combine_rows(bmin, [](double a, double b) { return fmin(a, b); });
  bmax = combine_rows(bmax, [](double a, double b) { return fmax(a, b); });
  amax = combine_rows(amax, [](double a, double b) { return fmax(a, b); });
  // short-circuit of discretekg.py:363-367 (all |b| < 1e-9), and the
  // single-slope case (one hull vertex, E = max a): KG = 0.
  if (!uniform(fmax(fabs(bmin), fabs(bmax)) >= 1e-9 && bmin < bmax)) {
    f.status = 1;
    return f;
  }
  double aL = -INFINITY, aR = -INFINITY, bT = INFINITY;
#pragma unroll
  for (int t = 0; t < MAXL; ++t) {
    aL = fmax_raw(aL, keep_or_qnan(lb[t] == bmin, la[t]));
    aR = fmax_raw(aR, keep_or_qnan(lb[t] == bmax, la[t]));
    bT = fmin_raw(bT, keep_or_qnan(la[t] == amax, lb[t]));
  }
  DKG_BUTTERFLY_ROW({
    aL = fmax_raw(aL, partner_f64<S_>(aL));
    aR = fmax_raw(aR, partner_f64<S_>(aR));
    bT = fmin_raw(bT, partner_f64<S_>(bT));
  })
  aL = combine_rows(aL, [](double a, double b) { return fmax(a, b); });
  aR = combine_rows(aR, [](double a, double b) { return fmax(a, b); });
  bT = combine_rows(bT, [](double a, double b) { return fmin(a, b); });
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
    bool s = fma(a, db1, -bb * da1) > k1 || fma(a, db2, -bb * da2) > k2;
    // IDX: also every exact copy of L and R and every line attaining max a, so
    // the list carries their indices (lowest index among duplicates) and the
    // max-a count without another pass over the lines
    if constexpr (IDX) s = s || a == aT || (bb == bL && a == aL) || (bb == bR && a == aR);
    const uint64_t mk = ballot(s);
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
  // IDX (list overflow only): the line indices of L, T, R and the count of max-a lines are
  // resolved lazily by the caller (rarely needed; keeps register pressure low)
  f.kL = f.kT = f.kR = -1;
  f.cntT = -1;
  return f;
}

// ---------------------------------------------------------------------------
// Forward envelope of one set of lines (one (candidate, scalarisation) pair,
// or one set of dkg_lines_kg / dkg_epigraph): extremes, the margin chord
// filter into the wave's LDS list (slope, intercept, line index), and the
// reference's walk over that list (dkg_walk.h), redone over all lines when
// the list overflows or a breakpoint leaves WALK_XGUARD.

struct FwdEnv {
  double bL, aL, bR, aR, bT, aT;
  int cnt;     // list entries (may exceed the capacity: overflow)
  int status;  // 0: list ready, 1: KG = 0 (short-circuit or one slope), 2: overflow
};

// Wave-uniform max (MAXV) or min of val[t] over the register lines with
// key[t] == k exactly (-inf / +inf if none): a per-lane fold of compare +
// select + min/max, all on the VALU (a scalar branch per slot on the compare
// mask costs more: tools/ubench/env_phases.hip), then the wave reduction.
// Keys are never NaN-equal, so the padding lines (NaN intercept and slope)
// never hit.
template <int MAXL, bool MAXV>
__device__ __forceinline__ double tie_fold(const double (&key)[MAXL], double k, const double (&val)[MAXL]) {
  double v = MAXV ? -INFINITY : INFINITY;
#pragma unroll
  for (int t = 0; t < MAXL; ++t)
    v = MAXV ? fmax_raw(v, keep_or_qnan(key[t] == k, val[t])) : fmin_raw(v, keep_or_qnan(key[t] == k, val[t]));
  DKG_BUTTERFLY_ROW({ v = MAXV ? fmax_raw(v, partner_f64<S_>(v)) : fmin_raw(v, partner_f64<S_>(v)); })
  return MAXV ? combine_rows(v, [](double a, double b) { return fmax(a, b); })
              : combine_rows(v, [](double a, double b) { return fmin(a, b); });
}

// The chord ends' intercepts aL (max a at b = bL) and aR (max a at b = bR),
// both folds interleaved; needed only once the flat test has failed.
template <int MAXL>
__device__ __forceinline__ void env_ends(const double (&la)[MAXL], const double (&lb)[MAXL], FwdEnv& f) {
  double aL = -INFINITY, aR = -INFINITY;
#pragma unroll
  for (int t = 0; t < MAXL; ++t) {
    aL = fmax_raw(aL, keep_or_qnan(lb[t] == f.bL, la[t]));
    aR = fmax_raw(aR, keep_or_qnan(lb[t] == f.bR, la[t]));
  }
  DKG_BUTTERFLY_ROW({
    aL = fmax_raw(aL, partner_f64<S_>(aL));
    aR = fmax_raw(aR, partner_f64<S_>(aR));
  })
  f.aL = combine_rows(aL, [](double a, double b) { return fmax(a, b); });
  f.aR = combine_rows(aR, [](double a, double b) { return fmax(a, b); });
}

// Extremes with their exact ties over register lines: L = min b (tie: max a),
// R = max b (tie: max a), T = max a (tie: min b).  Padding slots hold lines
// with a NaN intercept, which drop out of every raw min / max (IEEE maxNum)
// and fail every comparison.  status 1: every |b| < 1e-9 (discretekg.py:363-367)
// or a single slope (the walk stops at its first line): KG = 0, one line.
// aL and aR are left to env_ends (after the flat test).
template <int MAXL>
__device__ __forceinline__ FwdEnv env_extremes(const double (&la)[MAXL], const double (&lb)[MAXL]) {
  FwdEnv f;
  double bmin = INFINITY, bmax = -INFINITY, amax = -INFINITY;
#pragma unroll
  for (int t = 0; t < MAXL; ++t) {
    bmin = fmin_raw(bmin, lb[t]);
    bmax = fmax_raw(bmax, lb[t]);
    amax = fmax_raw(amax, la[t]);
  }
  DKG_BUTTERFLY_ROW({
    bmin = fmin_raw(bmin, partner_f64<S_>(bmin));
    bmax = fmax_raw(bmax, partner_f64<S_>(bmax));
    amax = fmax_raw(amax, partner_f64<S_>(amax));
  })
  bmin = combine_rows(bmin, [](double a, double b) { return fmin(a, b); });
  bmax = combine_rows(bmax, [](double a, double b) { return fmax(a, b); });
  amax = combine_rows(amax, [](double a, double b) { return fmax(a, b); });
  f.bL = bmin; f.bR = bmax; f.aT = amax;
  f.cnt = 0;
  if (!uniform(fmax(fabs(bmin), fabs(bmax)) >= 1e-9 && bmin < bmax)) {
    f.status = 1;
    return f;
  }
  // T's slope here (the flat test needs it); the chord ends' intercepts by env_ends
  f.bT = tie_fold<MAXL, false>(la, amax, lb);
  f.aL = f.aR = -INFINITY;
  f.status = 0;
  return f;
}

// The flat-first order (envelope forward): T's intercept and slope alone, then
// the flat test; the slope range and the short-circuit test (env_span) only for
// the pairs it does not settle.  A flat pair's KG is 0 whichever test decides it.
template <int MAXL>
__device__ __forceinline__ void env_top(const double (&la)[MAXL], const double (&lb)[MAXL], FwdEnv& f) {
  double amax = -INFINITY;
#pragma unroll
  for (int t = 0; t < MAXL; ++t) amax = fmax_raw(amax, la[t]);
  DKG_BUTTERFLY_ROW({ amax = fmax_raw(amax, partner_f64<S_>(amax)); })
  f.aT = combine_rows(amax, [](double a, double b) { return fmax(a, b); });
  f.bT = tie_fold<MAXL, false>(la, f.aT, lb);
  f.aL = f.aR = -INFINITY;
  f.cnt = 0;
  f.status = 0;
}

// env_extremes' slope range and status after env_top.
template <int MAXL>
__device__ __forceinline__ void env_span(const double (&lb)[MAXL], FwdEnv& f) {
  double bmin = INFINITY, bmax = -INFINITY;
#pragma unroll
  for (int t = 0; t < MAXL; ++t) {
    bmin = fmin_raw(bmin, lb[t]);
    bmax = fmax_raw(bmax, lb[t]);
  }
  DKG_BUTTERFLY_ROW({
    bmin = fmin_raw(bmin, partner_f64<S_>(bmin));
    bmax = fmax_raw(bmax, partner_f64<S_>(bmax));
  })
  f.bL = combine_rows(bmin, [](double a, double b) { return fmin(a, b); });
  f.bR = combine_rows(bmax, [](double a, double b) { return fmax(a, b); });
  f.status = uniform(fmax(fabs(f.bL), fabs(f.bR)) >= 1e-9 && f.bL < f.bR) ? 0 : 1;
}

// Flat envelope: line T (max a, then min b) lies strictly above every other
// line, exact copies of T aside, on the whole of [-ENV_FLAT_Z, ENV_FLAT_Z].
// Then every envelope breakpoint has |c| > ENV_FLAT_Z > 40, every edge term
// (b_Q - b_P) psi(+-c) is psi_edge's exact 0, and KG_w = 0: the value the
// walk would return, bit for bit, without the filter and the walk.  Per line
// the test is fma(Z, |b - bT|, a - aT) <= 2^-40 (a - aT): its three roundings
// (at most 3u (|a - aT| + Z |b - bT|) <= 6.001u |a - aT| once it passes) stay
// far inside the 2^-40 |a - aT| it demands, so a passing line other than a
// copy of T is strictly below T on the interval.  A copy of T gives 0 (passes);
// a line with a = aT and b != bT gives Z |b - bT| > 0 (fails).  NaN padding
// lines drop out of the maximum.
constexpr double ENV_FLAT_Z = 48.0;
constexpr double ENV_FLAT_REL = 9.094947017729282e-13;  // 2^-40

template <int MAXL>
__device__ __forceinline__ bool env_flat(const double (&la)[MAXL], const double (&lb)[MAXL], const FwdEnv& f) {
  double worst = -INFINITY;
#pragma unroll
  for (int t = 0; t < MAXL; ++t) {
    const double da = la[t] - f.aT;
    const double v = fma(ENV_FLAT_Z, fabs(lb[t] - f.bT), da);
    worst = fmax_raw(worst, fma(-ENV_FLAT_REL, da, v));
  }
  return ballot(worst > 0.0) == 0;
}

// The margin chord filter (EnvChords) over register lines into the list
// (capacity CAP entries; the count goes on past it).
template <int MAXL, int CAP, class Chords = EnvChords>
__device__ __forceinline__ int env_compact(const double (&la)[MAXL], const double (&lb)[MAXL], const Chords& ch,
                                           int lane, double* sb, double* sa, int* si, int cnt0 = 0) {
  // the keep masks of a group of four slots first (independent compares, no
  // branch between them), then the group's writes (rarely any)
  int cnt = cnt0;
#pragma unroll
  for (int t0 = 0; t0 < MAXL; t0 += 4) {
    uint64_t mk[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) mk[u] = (t0 + u < MAXL) ? env_keep_mask(ch, la[t0 + u], lb[t0 + u]) : 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int t = t0 + u;
      if (t < MAXL && mk[u] != 0) {  // wave-uniform, rarely taken
        if ((mk[u] >> lane) & 1) {
          const int pos = cnt + lanes_below(mk[u]);
          if (pos < CAP) {
            sb[pos] = lb[t];
            sa[pos] = la[t];
            si[pos] = lane + 64 * t;
          }
        }
        cnt += __popcll(mk[u]);
      }
    }
  }
  return cnt;
}

// Lists longer than ENV_REFINE_MIN after the L-T-R filter are filtered again against a longer chain: one
// quickhull round over the register lines puts V1 (the line farthest above the chord L-T) and V2 (farthest
// above T-R) into the chain L, V1, T, V2, R, and a line is kept iff it lies within the EnvChords margin of
// one of the four chords' extensions.  Any chain of lines of the set with increasing slopes lies below the
// upper hull H over its slope range (H is concave), so a line failing every chord is at least the margin
// below H there -- the argument of the L-T-R filter, and WALK_XGUARD's guard holds unchanged; rounding in the
// choice of V1 / V2 only changes which lines of the set form the chain.  The successor table of the walk costs
// ~ entries^2 / 64 divisions per lane (a 17-entry list: 6-7 K cycles in table<32> against 2-3 K for <= 8), and a
// list past ENV_CAP took the walk over all lines (25-37 K cycles, headline_nd).
constexpr int ENV_REFINE_MIN = 16;

struct EnvChain {
  double s[4], k[4];  // chord c: keep a line iff fma(-s_c, b, a) >= k_c (k_c = +inf: no chord)
};

__device__ __forceinline__ void chain_chord(double bP, double aP, double bQ, double aQ, double Wb, double rel,
                                            double& s, double& k) {
  const double db = bQ - bP;
  s = (db > 0.0) ? (aQ - aP) / db : 0.0;
  const double tau = rel * (fmax(fabs(aP), fabs(aQ)) + fabs(s) * (fmax(fabs(bP), fabs(bQ)) + Wb) + Wb);
  k = (db > 0.0) ? fma(-s, bP, aP) - tau : INFINITY;
}

// Heights above the chords L-T (u1) and T-R (u2), scaled by the chord's db > 0 (the same argmax); -inf off
// the chord's slope range (NaN padding lines too).
struct ChainHeights {
  double bL, aL, bT, aT, bR, aR, db1, da1, db2, da2;
  __device__ __forceinline__ explicit ChainHeights(const FwdEnv& f)
      : bL(f.bL), aL(f.aL), bT(f.bT), aT(f.aT), bR(f.bR), aR(f.aR), db1(f.bT - f.bL), da1(f.aT - f.aL),
        db2(f.bR - f.bT), da2(f.aR - f.aT) {}
  __device__ __forceinline__ double u1(double b, double a) const {
    return (b > bL && b < bT) ? fma(a - aL, db1, -(b - bL) * da1) : -INFINITY;
  }
  __device__ __forceinline__ double u2(double b, double a) const {
    return (b > bT && b < bR) ? fma(a - aT, db2, -(b - bT) * da2) : -INFINITY;
  }
};

// The chords of the chain L, V1, T, V2, R (a chord with no line above it stays whole), wave-uniform in SGPRs.
__device__ __forceinline__ EnvChain chain_of(const FwdEnv& f, bool v1, double b1v, double a1v, bool v2, double b2v,
                                             double a2v, double rel = WALK_MARGIN) {
  const double Wb = f.bR - f.bL;
  if (!v1) { b1v = f.bT; a1v = f.aT; }
  if (!v2) { b2v = f.bR; a2v = f.aR; }
  EnvChain c;
  chain_chord(f.bL, f.aL, b1v, a1v, Wb, rel, c.s[0], c.k[0]);  // L - V1 (L - T without V1)
  chain_chord(b1v, a1v, f.bT, f.aT, Wb, rel, c.s[1], c.k[1]);  // V1 - T (none without V1: db = 0)
  chain_chord(f.bT, f.aT, b2v, a2v, Wb, rel, c.s[2], c.k[2]);  // T - V2 (T - R without V2)
  chain_chord(b2v, a2v, f.bR, f.aR, Wb, rel, c.s[3], c.k[3]);  // V2 - R (none without V2)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    c.s[i] = sgpr_f64(c.s[i]);
    c.k[i] = sgpr_f64(c.k[i]);
  }
  return c;
}

// Half of a chain's chords: the lines with slope <= bT (upper: > bT) tested against two chords.
struct HalfChords {
  EnvChords ch;
  double bT;
  bool upper;
};

__device__ __forceinline__ uint64_t env_keep_mask(const HalfChords& c, double a, double b) {
  return env_keep_mask(c.ch, a, b) & (c.upper ? ballot(b > c.bT) : ballot(b <= c.bT));
}

__device__ __forceinline__ bool chain_keep1(const EnvChain& c, double b, double a) {
  return fma(-c.s[0], b, a) >= c.k[0] || fma(-c.s[1], b, a) >= c.k[1] || fma(-c.s[2], b, a) >= c.k[2] ||
         fma(-c.s[3], b, a) >= c.k[3];
}

// The list (cnt entries, ENV_REFINE_MIN < cnt <= ENV_CAP, line-index order) filtered against the chain
// L, V1, T, V2, R built from its own entries (every upper-hull line of the set is in it), compacted in place in
// the same order.  Two entries per lane at most: a few registers, one reduction round.  Returns the new count.
__device__ __forceinline__ int env_refine_list(int cnt, int lane, double* sb, double* sa, int* si, const FwdEnv& f,
                                               EnvChain* chain_only = nullptr, double rel = WALK_MARGIN) {
  const ChainHeights H(f);
  double eb[2], ea[2];
  int ek[2];
  bool ev[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int e = lane + 64 * q;
    ev[q] = e < cnt;
    const int ee = min(e, cnt - 1);
    eb[q] = ev[q] ? sb[ee] : __builtin_nan("");
    ea[q] = ev[q] ? sa[ee] : __builtin_nan("");
    ek[q] = si[ee];
  }
  double m1 = fmax(H.u1(eb[0], ea[0]), H.u1(eb[1], ea[1]));
  double m2 = fmax(H.u2(eb[0], ea[0]), H.u2(eb[1], ea[1]));
  DKG_BUTTERFLY_ROW({
    m1 = fmax(m1, partner_f64<S_>(m1));
    m2 = fmax(m2, partner_f64<S_>(m2));
  })
  m1 = combine_rows(m1, [](double p, double q) { return fmax(p, q); });
  m2 = combine_rows(m2, [](double p, double q) { return fmax(p, q); });
  // the first entry (list order) attaining each maximum
  double b1v = 0.0, a1v = 0.0, b2v = 0.0, a2v = 0.0;
  const bool v1 = m1 > 0.0, v2 = m2 > 0.0;
  if (v1) {
    const uint64_t k0 = ballot(H.u1(eb[0], ea[0]) == m1), k1 = ballot(H.u1(eb[1], ea[1]) == m1);
    const int q = k0 ? 0 : 1, w = __builtin_ctzll(k0 ? k0 : k1);
    b1v = readlane_f64(q ? eb[1] : eb[0], w);
    a1v = readlane_f64(q ? ea[1] : ea[0], w);
  }
  if (v2) {
    const uint64_t k0 = ballot(H.u2(eb[0], ea[0]) == m2), k1 = ballot(H.u2(eb[1], ea[1]) == m2);
    const int q = k0 ? 0 : 1, w = __builtin_ctzll(k0 ? k0 : k1);
    b2v = readlane_f64(q ? eb[1] : eb[0], w);
    a2v = readlane_f64(q ? ea[1] : ea[0], w);
  }
  const EnvChain c = chain_of(f, v1, b1v, a1v, v2, b2v, a2v, rel);
  if (chain_only != nullptr) {  // an overflowing list: the chain only (the caller filters the lines)
    *chain_only = c;
    return cnt;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // every entry read before the list is rewritten
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  int n = 0;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const bool keep = ev[q] && chain_keep1(c, eb[q], ea[q]);
    const uint64_t mk = ballot(keep);
    if (keep) {
      const int pos = n + lanes_below(mk);
      sb[pos] = eb[q];
      sa[pos] = ea[q];
      si[pos] = ek[q];
    }
    n += __popcll(mk);
  }
  return n;
}

// Short-circuit index (dkg_epigraph): the first line attaining max a
// (torch.max over the intercepts, discretekg.py:366).
template <int MAXL>
__device__ __forceinline__ int first_max_index(const double (&la)[MAXL], int nl, int lane, double amax) {
  int k = KEY_NONE;
#pragma unroll
  for (int t = MAXL - 1; t >= 0; --t) k = (lane + 64 * t < nl && la[t] == amax) ? lane + 64 * t : k;
  return wave_min_i32(k);
}

// KG_w (and the envelope size) of register-held lines: build(la, lb) fills the
// lines (line k in lane k % 64, slot k / 64; k >= nl: NaN intercepts); it runs
// again only for a second filter or the walk over all lines, so no register
// line is live across the list walk.  force_walk: test hook (every set takes
// the walk over all lines).  pst (debug, DKG_DEBUG_STAMPS=2): phase stamps.
// T (max a, tie: min b) known before the lines are in registers (the staged forward's plan keeps each
// scalarisation's largest intercept over k >= 1: Plan::itop): valid when it is decided without a tie
// (line 0 strictly above every other line, or one line k >= 1 strictly above the rest, line 0 included).
struct TopHint {
  bool valid;
  double aT, bT;
};

template <int MAXL, class Build, class Build0 = int>
__device__ __forceinline__ EdgeSum env_pair_regs_edges(Build&& build, int nl, int lane, double* sb, double* sa, int* si,
                                                bool force_walk, int* nhull, const WalkOut* out = nullptr,
                                                unsigned long long* pst = nullptr, bool flat_ok = false,
                                                const Build0* build0 = nullptr,
                                                TopHint hint = TopHint{false, 0.0, 0.0}) {
  FwdEnv f;
  if (pst) pst[0] = __builtin_amdgcn_s_memtime();
  {
    double la[MAXL], lb[MAXL];
    if constexpr (std::is_same_v<Build0, int>) {
      build(la, lb);
    } else {
      (*build0)(la, lb);  // the first build (e.g. from registers loaded ahead)
    }
    if (pst) pst[1] = __builtin_amdgcn_s_memtime();
    if (flat_ok && hint.valid) {
      f.aT = hint.aT;  // what env_top finds, without its two wave reductions
      f.bT = hint.bT;
      f.aL = f.aR = -INFINITY;
      f.cnt = 0;
      f.status = 0;
    } else if (flat_ok) {
      env_top<MAXL>(la, lb, f);
    }
    if (flat_ok) {
      if (pst) pst[2] = __builtin_amdgcn_s_memtime();
      if (env_flat<MAXL>(la, lb, f)) {
        *nhull = 0;  // not walked: KG_w = 0 exactly (env_flat)
        if (pst) {
          pst[3] = __builtin_amdgcn_s_memtime();
          pst[6] = 0;
          pst[7] = 1ull << 34;
        }
        return EdgeSum{0.0, 0.0, 0.0, false};
      }
      env_span<MAXL>(lb, f);
    } else {
      f = env_extremes<MAXL>(la, lb);
      if (pst) pst[2] = __builtin_amdgcn_s_memtime();
    }
    if (f.status == 1) {
      if (out && out->cap > 0) {
        const int k = first_max_index<MAXL>(la, nl, lane, f.aT);
        if (lane == 0) out->idx[0] = k;
      }
      *nhull = 1;
      return EdgeSum{0.0, 0.0, 0.0, false};
    }
    env_ends<MAXL>(la, lb, f);
    f.cnt = env_compact<MAXL, ENV_CAP>(la, lb, env_chords(f.bL, f.aL, f.bT, f.aT, f.bR, f.aR), lane, sb, sa, si);
    if (pst) {
      pst[3] = __builtin_amdgcn_s_memtime();
      pst[6] = (unsigned long long)f.cnt;
    }
  }
  // opaque copies of the chain ends: no term of the first filter's chords is kept live for the later filters
  asm volatile("" : "+v"(f.bL), "+v"(f.aL), "+v"(f.bT), "+v"(f.aT), "+v"(f.bR), "+v"(f.aR));
  if (DKG_ENV_REFINE && f.cnt > ENV_REFINE_MIN && !force_walk) {  // wave-uniform: the chain L, V1, T, V2, R
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (f.cnt <= ENV_CAP) {
      f.cnt = env_refine_list(f.cnt, lane, sb, sa, si, f);
    } else if (DKG_REFINE_OVERFLOW) {
      // the chain of the entries the list holds (lines of the set), then the lines filtered against it in
      // two halves: slopes <= bT against the chords L-V1, V1-T, the rest against T-V2, V2-R (the largest
      // height of a line above the chain is at the breakpoint its slope brackets), each half in line order
      EnvChain c;
      env_refine_list(ENV_CAP, lane, sb, sa, si, f, &c);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      double la[MAXL], lb[MAXL];
      build(la, lb);
      const double bT = sgpr_f64(f.bT);
      int n = env_compact<MAXL, ENV_CAP>(la, lb, HalfChords{{c.s[0], c.k[0], c.s[1], c.k[1]}, bT, false}, lane, sb,
                                         sa, si);
      n = env_compact<MAXL, ENV_CAP>(la, lb, HalfChords{{c.s[2], c.k[2], c.s[3], c.k[3]}, bT, true}, lane, sb, sa,
                                     si, n);
      f.cnt = n;
    }
    if (pst) pst[6] |= (unsigned long long)min(f.cnt, 0xffff) << 16;
  }
  if (!force_walk) {
    // up to three list walks: at WALK_MARGIN; after an overflow at the tight margin; after a
    // breakpoint beyond the guard at the margin that covers it
    double rel = WALK_MARGIN;
    for (int level = 0; level < 3; ++level) {
      double next = 0.0;
      if (f.cnt <= ENV_CAP) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        double cmax;
        int h;
        const EdgeSum kg = walk_small(f.cnt, lane, sb, sa, si, f.bL, f.aL, f.bT, &h, &cmax, out);
        if (pst) pst[4] = __builtin_amdgcn_s_memtime();
        if (uniform(cmax <= rel * WALK_POW2_50)) {
          *nhull = h;
          if (pst) pst[7] = (unsigned long long)h | ((unsigned long long)(level > 0) << 33);
          return kg;
        }
        next = WALK_REFILTER * cmax / WALK_POW2_50;  // a breakpoint beyond the guard
        if (!uniform(next < WALK_REL_MAX)) break;
      } else {
        if (!(rel > WALK_MARGIN_TIGHT)) break;     // overflow at the tight margin
        next = WALK_MARGIN_TIGHT;
      }
      rel = next;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      double la[MAXL], lb[MAXL];
      build(la, lb);
      f.cnt = env_compact<MAXL, ENV_CAP>(la, lb, env_chords(f.bL, f.aL, f.bT, f.aT, f.bR, f.aR, rel), lane, sb, sa,
                                         si);
    }
  }
  double la[MAXL], lb[MAXL];
  build(la, lb);
  const EdgeSum kgw = walk_regs<MAXL>(la, lb, nl, lane, f.bL, f.aL, f.bT, nhull, out);
  if (pst) {
    pst[5] = __builtin_amdgcn_s_memtime();
    pst[7] = (unsigned long long)(*nhull) | (1ull << 32);
  }
  return kgw;
}

// KG_w of register-held lines (env_pair_regs_edges), with the single psi evaluation of its edge terms.
template <int MAXL, class Build, class Build0 = int>
__device__ __forceinline__ double env_pair_regs(Build&& build, int nl, int lane, double* sb, double* sa, int* si,
                                                bool force_walk, int* nhull, const WalkOut* out = nullptr,
                                                unsigned long long* pst = nullptr, bool flat_ok = false,
                                                const Build0* build0 = nullptr,
                                                TopHint hint = TopHint{false, 0.0, 0.0}) {
  return finish_edges(
      env_pair_regs_edges<MAXL>(build, nl, lane, sb, sa, si, force_walk, nhull, out, pst, flat_ok, build0, hint));
}

// ---------------------------------------------------------------------------
// Vertex visitors for the gradient: the envelope lines in increasing slope,
// each with its breakpoints (cL, cR) (-inf / +inf at the ends), passed to
// visit(k, b, a, cL, cR); the return value is KG_w as in the forward.

// Gradient hull over the candidate list of an IDX filter (every entry's line
// index known, exact copies of L / R and all max-a lines included).  The
// chain from L is followed serially (one v_readlane per vertex); everything
// else is vertex-parallel, one hull vertex per lane: breakpoints cL / cR,
// dE/da = Phi(cR) - Phi(cL), dE/db = phi(cL) - phi(cR), the KG edge terms and
// the queue of envelope lines k >= 1 (index, dE/db) for the gradient flush.
struct HullGrad {
  double kg;     // KG_w (same edge sum as envelope_hull)
  double sumDb;  // sum over hull lines of dE/db * b
  double Pw0, Dw0;  // line 0 (the candidate itself) if on the hull, else 0
  int nq;        // queued lines k >= 1 (hk / hD)
  int cntT;      // lines attaining max a
};

__device__ __forceinline__ HullGrad envelope_hull_grad(const EnvFilter& f, int lane, const double* sb,
                                                       const double* sa, const int* si, double* scl, int* hk,
                                                       double* hD, int N) {
  HullGrad r;
  const int nc = f.cnt;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  double lb_[2], la_[2];
  int li_[2];
  bool ok[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int e = min(c * 64 + lane, nc - 1);
    ok[c] = c * 64 + lane < nc;
    lb_[c] = sb[e];
    la_[c] = sa[e];
    li_[c] = si[e];
  }
  // chain start: the lowest-index copy of L; and the max-a count
  int kst = 1 << 30, cntT = 0;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    if (ok[c] && lb_[c] == f.bL && la_[c] == f.aL) kst = min(kst, li_[c]);
    cntT += __popcll(ballot(ok[c] && la_[c] == f.aT));
  }
  kst = wave_min_i32(kst);
  int start;
  {
    const uint64_t m0 = ballot(ok[0] && li_[0] == kst), m1 = ballot(ok[1] && li_[1] == kst);
    start = m0 ? __builtin_ctzll(m0) : 64 + __builtin_ctzll(m1);
  }
  // right neighbour of every entry (as envelope_hull)
  int nxt[2] = {-1, -1};
  double cn[2] = {0.0, 0.0}, cd[2] = {1.0, 1.0}, cb[2] = {0.0, 0.0};
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
    nxt[c] = rj; cn[c] = rn; cd[c] = rd; cb[c] = rb;
  }
  // follow the chain from the start: its members are the envelope lines
  uint64_t on0 = 0, on1 = 0;
  for (int cur = start, guard = 0; cur >= 0 && guard < nc; ++guard) {
    if (cur < 64) on0 |= 1ull << cur; else on1 |= 1ull << (cur - 64);
    cur = (cur < 64) ? __builtin_amdgcn_readlane(nxt[0], cur) : __builtin_amdgcn_readlane(nxt[1], cur - 64);
  }
  // left breakpoints: every hull vertex hands its right breakpoint to its successor
  double cR[2];
  bool on[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    on[c] = (((c == 0) ? on0 : on1) >> lane) & 1;
    cR[c] = (nxt[c] >= 0) ? cn[c] / cd[c] : INFINITY;
  }
  if (lane == 0) scl[start] = -INFINITY;
#pragma unroll
  for (int c = 0; c < 2; ++c)
    if (on[c] && nxt[c] >= 0) scl[nxt[c]] = cR[c];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  double kg = 0.0, sdb = 0.0, pw0 = 0.0, dw0 = 0.0;
  int nq = 0;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    if (c * 64 >= nc) break;
    double Dw = 0.0;
    if (on[c]) {
      const double cl = scl[c * 64 + lane], cr = cR[c];
      if (nxt[c] >= 0) kg += (cb[c] - lb_[c]) * psi((cb[c] <= f.bT) ? -cr : cr);
      const double Pw = norm_cdf(cr) - norm_cdf(cl);
      Dw = norm_pdf(cl) - norm_pdf(cr);
      sdb = fma(Dw, lb_[c], sdb);
      if (li_[c] == 0) { pw0 = Pw; dw0 = Dw; }
    }
    const bool q = on[c] && li_[c] >= 1 && li_[c] <= N;
    const uint64_t mq = ballot(q);
    if (q) {
      const int pos = nq + lanes_below(mq);
      hk[pos] = li_[c];
      hD[pos] = Dw;
    }
    nq += __popcll(mq);
  }
  r.kg = wave_sum(kg);
  r.sumDb = wave_sum(sdb);
  r.Pw0 = wave_sum(pw0);  // at most one lane holds line 0
  r.Dw0 = wave_sum(dw0);
  r.nq = nq;
  r.cntT = cntT;
  return r;
}

// ---------------------------------------------------------------------------
// Streaming variants for line sets larger than registers and LDS staging hold
// (N + 1 > 64 * 33, or the staging exceeds LDS): every pass rebuilds the
// lines chunk by chunk (64 * MAXL lines each) through build(c, la, lb);
// line k = c * 64 * MAXL + lane + 64 t.
template <int MAXL, bool IDX, int CAP = ENV_CAP, class Build>
__device__ __forceinline__ EnvFilter envelope_filter_stream(int nch, int lane, double* sb, double* sa, int* si,
                                                            Build&& build) {
  EnvFilter f;
  // One pass for the extremes with their exact ties (lexicographic: L = min b
  // then max a, R = max b then max a, T = max a then min b): the streamed
  // lines cost loads, so this trades select work for a whole pass over them.
  double bmin = INFINITY, aLx = -INFINITY, bmax = -INFINITY, aRx = -INFINITY, amax = -INFINITY, bTx = INFINITY;
  for (int c = 0; c < nch; ++c) {
    double la[MAXL], lb[MAXL];
    build(c, la, lb);
#pragma unroll
    for (int t = 0; t < MAXL; ++t) {
      const double a = la[t], b = lb[t];
      const bool l = b < bmin || (b == bmin && a > aLx);
      bmin = l ? b : bmin;
      aLx = l ? a : aLx;
      const bool r = b > bmax || (b == bmax && a > aRx);
      bmax = r ? b : bmax;
      aRx = r ? a : aRx;
      const bool tt = a > amax || (a == amax && b < bTx);
      amax = tt ? a : amax;
      bTx = tt ? b : bTx;
    }
  }
  DKG_BUTTERFLY({
    const double ob = partner_f64<S_>(bmin), oa = partner_f64<S_>(aLx);
    const bool l = ob < bmin || (ob == bmin && oa > aLx);
    bmin = l ? ob : bmin;
    aLx = l ? oa : aLx;
    const double ob2 = partner_f64<S_>(bmax), oa2 = partner_f64<S_>(aRx);
    const bool r = ob2 > bmax || (ob2 == bmax && oa2 > aRx);
    bmax = r ? ob2 : bmax;
    aRx = r ? oa2 : aRx;
    const double oa3 = partner_f64<S_>(amax), ob3 = partner_f64<S_>(bTx);
    const bool tt = oa3 > amax || (oa3 == amax && ob3 < bTx);
    amax = tt ? oa3 : amax;
    bTx = tt ? ob3 : bTx;
  })
  if (!uniform(fmax(fabs(bmin), fabs(bmax)) >= 1e-9 && bmin < bmax)) {
    f.status = 1;
    return f;
  }
  const double aL = aLx, aR = aRx, bT = bTx;
  const double bL = bmin, bR = bmax, aT = amax;
  f.bL = bL; f.aL = aL; f.bR = bR; f.aR = aR; f.bT = bT; f.aT = aT;
  const double db1 = bT - bL, da1 = aT - aL, k1 = aL * db1 - bL * da1;
  const double db2 = bR - bT, da2 = aR - aT, k2 = aT * db2 - bT * da2;
  int cnt = 0;
  for (int c = 0; c < nch; ++c) {
    double la[MAXL], lb[MAXL];
    build(c, la, lb);
#pragma unroll
    for (int t = 0; t < MAXL; ++t) {
      const double a = la[t], bb = lb[t];
      bool s = fma(a, db1, -bb * da1) > k1 || fma(a, db2, -bb * da2) > k2;
      if constexpr (IDX) s = s || a == aT || (bb == bL && a == aL) || (bb == bR && a == aR);
      const uint64_t mk = ballot(s);
      if (mk != 0) {
        if (s) {
          const int pos = cnt + lanes_below(mk);
          if (pos < CAP) {
            sb[pos] = bb;
            sa[pos] = a;
            if constexpr (IDX) si[pos] = c * 64 * MAXL + lane + 64 * t;
          }
        }
        cnt += __popcll(mk);
      }
    }
  }
  f.cnt = cnt;
  f.status = (cnt + 3 > ENV_CAP) ? 2 : 0;
  f.kL = f.kT = f.kR = -1;
  f.cntT = -1;
  return f;
}

// Gift wrap over streamed lines (list overflow), index carried; visit may be a no-op.
template <int MAXL, class Build, class Visit>
__device__ __forceinline__ double envelope_walk_stream(int nch, int nl, int lane, const EnvFilter& f, Build&& build,
                                                       Visit&& visit, int kL) {
  double bc = f.bL, ac = f.aL, kg = 0.0, cL = -INFINITY;
  int kc = kL;
  for (int guard = 0; guard <= nl; ++guard) {
    if (!uniform(bc < f.bR)) break;
    double bn = INFINITY, bd = 1.0, bbest = -INFINITY, abest = -INFINITY;
    int kbest = 1 << 30;
    for (int c = 0; c < nch; ++c) {
      double la[MAXL], lb[MAXL];
      build(c, la, lb);
#pragma unroll
      for (int t = 0; t < MAXL; ++t) {
        const double bb = lb[t], a = la[t];
        const int k = c * 64 * MAXL + lane + 64 * t;
        if (k < nl && bb > bc) {
          const double num = ac - a, den = bb - bc;
          const double lhs = num * bd, rhs = bn * den;
          if (bbest == -INFINITY || lhs < rhs || (lhs == rhs && (bb > bbest || (bb == bbest && a > abest)))) {
            bn = num; bd = den; bbest = bb; abest = a; kbest = k;
          }
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

// Streaming quickhull round(s) for survivor lists longer than the LDS list
// holds (cnt > LIST_CAP_STREAM): per chord of the known vertices V (L, T, R to
// start), one pass over the streamed lines finds the farthest line strictly
// above it (an upper-hull vertex, as in refine_list); a second pass re-filters
// the lines against the doubled chord set into the list.  Up to two rounds
// (3 -> 5 -> 9 vertices), then refine_list continues on the list.  Returns
// the hull-stage list length, or -1 (the caller walks).
template <int MAXL, int NV, class Build>
__device__ __forceinline__ int chord_of(double b, const double (&vb_)[NV], int nv) {
  int c = 0;
#pragma unroll
  for (int i = 1; i < NV - 1; ++i) c += (i < nv - 1 && b > vb_[i]) ? 1 : 0;
  return c;
}

template <int NV>
__device__ __forceinline__ double chord_h_reg(double b, double a, const double (&vb_)[NV], const double (&va_)[NV],
                                              int c) {
  double b0 = vb_[0], a0 = va_[0], b1 = vb_[1], a1 = va_[1];
#pragma unroll
  for (int i = 1; i < NV - 1; ++i) {
    const bool s = c == i;
    b0 = s ? vb_[i] : b0;
    a0 = s ? va_[i] : a0;
    b1 = s ? vb_[i + 1] : b1;
    a1 = s ? va_[i + 1] : a1;
  }
  return (a - a0) * (b1 - b0) - (b - b0) * (a1 - a0);
}

// Margin form of the chord test (EnvChords): h >= -tau for the chord c the
// line's slope falls in; a degenerate chord keeps only exact copies of its end.
template <int NV>
__device__ __forceinline__ bool chord_keep_reg(double b, double a, const double (&vb_)[NV], const double (&va_)[NV],
                                               int c, double Wb) {
  double b0 = vb_[0], a0 = va_[0], b1 = vb_[1], a1 = va_[1];
#pragma unroll
  for (int i = 1; i < NV - 1; ++i) {
    const bool s = c == i;
    b0 = s ? vb_[i] : b0;
    a0 = s ? va_[i] : a0;
    b1 = s ? vb_[i + 1] : b1;
    a1 = s ? va_[i + 1] : a1;
  }
  const double db = b1 - b0, da = a1 - a0;
  if (!(db > 0.0)) return b == b0 && a == a0;
  const double tau = WALK_MARGIN * (fmax(fabs(a0), fabs(a1)) * db + fmax(fabs(b0), fabs(b1)) * fabs(da) + Wb * db);
  return (a - a0) * db - (b - b0) * da >= -tau;
}

// Quickhull extension of a vertex chain (vb, va in LDS, nv <= NV vertices in increasing slope; lane 0 writes):
// for every chord the line farthest above it (scaled height > 0; ties -> lowest line index) over the lines
// build(ch, la, lb) gives for ch < nch, inserted after the chord's left end.  Returns the vertices found
// (0: no line above any chord); nv and tpos (T's position) are updated.
template <int MAXL, int NV, class Build>
__device__ __forceinline__ int qh_extend(int nch, int nl, int lane, double* vb, double* va, int& nv, int& tpos,
                                         Build&& build) {
  constexpr int NC = NV - 1;
  double vb_[NV], va_[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    vb_[i] = vb[min(i, nv - 1)];
    va_[i] = va[min(i, nv - 1)];
  }
  // pass A: farthest line above each chord (ties -> lowest line index)
  double bh[NC], bb[NC], ba[NC];
  int bk[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) { bh[c] = 0.0; bb[c] = 0.0; ba[c] = 0.0; bk[c] = 1 << 30; }
  for (int ch = 0; ch < nch; ++ch) {
    double la[MAXL], lb[MAXL];
    build(ch, la, lb);
#pragma unroll
    for (int t = 0; t < MAXL; ++t) {
      const int k = ch * 64 * MAXL + lane + 64 * t;
      const int c = chord_of<MAXL, NV, Build>(lb[t], vb_, nv);
      const double h = chord_h_reg<NV>(lb[t], la[t], vb_, va_, c);
      const bool live = k < nl;
#pragma unroll
      for (int cc = 0; cc < NC; ++cc) {
        const bool take = live && c == cc && h > bh[cc];
        bh[cc] = take ? h : bh[cc];
        bb[cc] = take ? lb[t] : bb[cc];
        ba[cc] = take ? la[t] : ba[cc];
        bk[cc] = take ? k : bk[cc];
      }
    }
  }
  uint64_t hasnew = 0;
  int found = 0;
#pragma unroll
  for (int cc = 0; cc < NC; ++cc) {
    if (cc >= nv - 1) break;
    double h = bh[cc], b = bb[cc], a = ba[cc];
    int k = bk[cc];
    DKG_BUTTERFLY({
      const double oh = partner_f64<S_>(h), ob = partner_f64<S_>(b), oa = partner_f64<S_>(a);
      const int ok = __shfl_xor(k, S_ == 0 ? 1 : S_ == 1 ? 2 : S_ == 2 ? 4 : S_ == 3 ? 8 : S_ == 4 ? 16 : 32);
      const bool take = oh > h || (oh == h && ok < k);
      h = take ? oh : h;
      b = take ? ob : b;
      a = take ? oa : a;
      k = take ? ok : k;
    })
    if (uniform(h > 0.0)) {
      hasnew |= 1ull << cc;
      ++found;
      bb[cc] = b;
      ba[cc] = a;
    }
  }
  if (found == 0) return 0;
  // insert the new vertices (lane 0, from the back, as refine_list)
  if (lane == 0) {
    for (int i = nv - 1; i >= 0; --i) {
      const int w = i + __popcll(hasnew & ((1ull << i) - 1));
      const double b0 = vb[i], a0 = va[i];
#pragma unroll
      for (int cc = 0; cc < NC; ++cc)
        if (cc == i && ((hasnew >> cc) & 1)) {
          vb[w + 1] = bb[cc];
          va[w + 1] = ba[cc];
        }
      vb[w] = b0;
      va[w] = a0;
    }
  }
  tpos += __popcll(hasnew & ((1ull << tpos) - 1));
  nv += found;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return found;
}

// One streaming round with NV = nv vertices (compile-time bound) read from LDS:
// new vertices inserted into vb/va (lane 0, qh_extend), survivors of the 2(nv-1)
// chords written to the list (capacity LIST_CAP_STREAM).  Returns the survivor count
// (may exceed the capacity), or -1 if no line is above any chord.
template <int MAXL, int NV, class Build>
__device__ __forceinline__ int stream_round(int nch, int nl, int lane, double* sb, double* sa, int* si, double* vb,
                                            double* va, int& nv, int& tpos, Build&& build) {
  if (qh_extend<MAXL, NV>(nch, nl, lane, vb, va, nv, tpos, build) == 0) return -1;
  // pass B: survivors of the new chords into the list
  constexpr int NV2 = 2 * NV - 1;
  const double Wb = vb[nv - 1] - vb[0];
  double wb_[NV2], wa_[NV2];
#pragma unroll
  for (int i = 0; i < NV2; ++i) {
    wb_[i] = vb[min(i, nv - 1)];
    wa_[i] = va[min(i, nv - 1)];
  }
  int cnt = 0;
  for (int ch = 0; ch < nch; ++ch) {
    double la[MAXL], lb[MAXL];
    build(ch, la, lb);
#pragma unroll
    for (int t = 0; t < MAXL; ++t) {
      const int k = ch * 64 * MAXL + lane + 64 * t;
      const int c = chord_of<MAXL, NV2, Build>(lb[t], wb_, nv);
      const bool keep = k < nl && chord_keep_reg<NV2>(lb[t], la[t], wb_, wa_, c, Wb);
      const uint64_t mk = ballot(keep);
      if (mk != 0) {
        if (keep) {
          const int pos = cnt + lanes_below(mk);
          if (pos < LIST_CAP_STREAM) {
            sb[pos] = lb[t];
            sa[pos] = la[t];
            si[pos] = k;
          }
        }
        cnt += __popcll(mk);
      }
    }
  }
  return cnt;
}

template <int MAXL, class Build>
__device__ __forceinline__ int refine_stream(const FwdEnv& f, int nch, int nl, int lane, double* sb, double* sa,
                                             int* si, double* vreg, Build&& build) {
  double* vb = vreg;
  double* va = vreg + VCAP;
  if (lane == 0) {
    vb[0] = f.bL; va[0] = f.aL;
    vb[1] = f.bT; va[1] = f.aT;
    vb[2] = f.bR; va[2] = f.aR;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  int nv = 3, tpos = 1;
  int cnt = stream_round<MAXL, 3>(nch, nl, lane, sb, sa, si, vb, va, nv, tpos, build);
  if (cnt > LIST_CAP_STREAM) cnt = stream_round<MAXL, 5>(nch, nl, lane, sb, sa, si, vb, va, nv, tpos, build);
  return (cnt < 0 || cnt > LIST_CAP_STREAM) ? -1 : cnt;
}

// Streaming forward (line sets too large for registers / LDS staging): the
// extremes in one lexicographic pass over the streamed lines, the margin
// filter into the wave's long list (LIST_CAP_STREAM entries), streamed
// quickhull rounds when that overflows, then the walk over the list.
// Per-lane running extremes of streamed lines (L = min b, tie max a; R = max b, tie max a; T = max a,
// tie min b), folded chunk by chunk and reduced over the wave once (env_extremes_stream).
struct ExtAcc {
  double bmin = INFINITY, aLx = -INFINITY, bmax = -INFINITY, aRx = -INFINITY, amax = -INFINITY, bTx = INFINITY;
};

template <int MAXL>
__device__ __forceinline__ void ext_fold(const double (&la)[MAXL], const double (&lb)[MAXL], int base, int nl, int lane,
                                         ExtAcc& e) {
#pragma unroll
  for (int t = 0; t < MAXL; ++t) {
    // bitwise, not short-circuit, logic: lane masks and selects, no branch per slot
    const bool live = base + lane + 64 * t < nl;
    const double a = la[t], b = lb[t];
    const bool l = live & ((b < e.bmin) | ((b == e.bmin) & (a > e.aLx)));
    e.bmin = l ? b : e.bmin;
    e.aLx = l ? a : e.aLx;
    const bool r = live & ((b > e.bmax) | ((b == e.bmax) & (a > e.aRx)));
    e.bmax = r ? b : e.bmax;
    e.aRx = r ? a : e.aRx;
    const bool tt = live & ((a > e.amax) | ((a == e.amax) & (b < e.bTx)));
    e.amax = tt ? a : e.amax;
    e.bTx = tt ? b : e.bTx;
  }
}

__device__ __forceinline__ FwdEnv ext_reduce(ExtAcc e) {
  DKG_BUTTERFLY({
    const double ob = partner_f64<S_>(e.bmin), oa = partner_f64<S_>(e.aLx);
    const bool l = ob < e.bmin || (ob == e.bmin && oa > e.aLx);
    e.bmin = l ? ob : e.bmin;
    e.aLx = l ? oa : e.aLx;
    const double ob2 = partner_f64<S_>(e.bmax), oa2 = partner_f64<S_>(e.aRx);
    const bool r = ob2 > e.bmax || (ob2 == e.bmax && oa2 > e.aRx);
    e.bmax = r ? ob2 : e.bmax;
    e.aRx = r ? oa2 : e.aRx;
    const double oa3 = partner_f64<S_>(e.amax), ob3 = partner_f64<S_>(e.bTx);
    const bool tt = oa3 > e.amax || (oa3 == e.amax && ob3 < e.bTx);
    e.amax = tt ? oa3 : e.amax;
    e.bTx = tt ? ob3 : e.bTx;
  })
  FwdEnv f;
  f.bL = e.bmin; f.aL = e.aLx; f.bR = e.bmax; f.aR = e.aRx; f.aT = e.amax; f.bT = e.bTx;
  f.cnt = 0;
  f.status = uniform(fmax(fabs(e.bmin), fabs(e.bmax)) >= 1e-9 && e.bmin < e.bmax) ? 0 : 1;
  return f;
}

template <int MAXL, class Build>
__device__ __forceinline__ FwdEnv env_extremes_stream(int nch, int nl, int lane, Build&& build) {
  ExtAcc e;
  for (int c = 0; c < nch; ++c) {
    double la[MAXL], lb[MAXL];
    build(c, la, lb);
    ext_fold<MAXL>(la, lb, c * 64 * MAXL, nl, lane, e);
  }
  return ext_reduce(e);
}

// The chord filter of one streamed chunk (lines base + lane + 64 t) into the wave's long list
// (LIST_CAP_STREAM entries; cnt counts on past it).
template <int MAXL>
__device__ __forceinline__ void stream_keep(const double (&la)[MAXL], const double (&lb)[MAXL], int base, int nl,
                                            const EnvChords& ch, int lane, double* sb, double* sa, int* si,
                                            int& cnt) {
#pragma unroll
  for (int t = 0; t < MAXL; ++t) {
    const int k = base + lane + 64 * t;
    // env_keep with bitwise logic: lane masks, no branch per slot
    const bool s = (k < nl) & ((fma(-ch.s1, lb[t], la[t]) >= ch.k1) | (fma(-ch.s2, lb[t], la[t]) >= ch.k2));
    const uint64_t mk = ballot(s);
    if (mk != 0) {
      if (s) {
        const int pos = cnt + lanes_below(mk);
        if (pos < LIST_CAP_STREAM) {
          sb[pos] = lb[t];
          sa[pos] = la[t];
          si[pos] = k;
        }
      }
      cnt += __popcll(mk);
    }
  }
}

// ---------------------------------------------------------------------------
// Staged streaming forward, one pass (DKG_STG_SAMPLE): the survivor list is filtered against a chain of
// lines of the set (the quickhull vertices of a strided sample of the pair's lines) instead of the chords
// L-T / T-R of the exact extremes, which took a pass of their own.
//
// Why it is exact.  For a chain P_0 .. P_n of lines of the set with increasing slopes, the chord of P_c, P_c+1
// is below the upper hull H of the whole set over [b_c, b_c+1] (H is concave and above every line), so
// min_c ext_c(b) <= H(b) for every b in [b_0, b_n].  A line (a, b) is kept iff b < b_0, or b > b_n, or it is
// within the margin tau_c of some chord's extension: fma(-s_c, b, a) >= K_c = fma(-s_c, b_c, a_c) - tau_c
// (EnvChords' test and margin, W an upper bound of the set's slope range).  A line that fails every test lies
// at least tau_c below H at its slope, so below the envelope by at least rel W everywhere: the guard argument
// of DESIGN.md 4.3 holds for the walk over the list as for the two-chord list.  Every line of H (L, T, R
// with their tie rules included) passes, so the list's own extremes are the set's.
#ifndef DKG_STG_SAMPLE
#define DKG_STG_SAMPLE 1
#endif
#ifndef DKG_SH_ROUNDS
#define DKG_SH_ROUNDS 1
#endif
constexpr int SH_ROUNDS = DKG_SH_ROUNDS;  // quickhull rounds on the sample: 3 -> 5 (-> 9) vertices; one measured faster
constexpr int SH_NC = SH_ROUNDS > 1 ? 8 : 4;     // chords of the chain

template <int NC>
struct ChainChords {
  double s[NC], k[NC];
  double blo, bhi;
};

// Keep tests of the chain (vb, va: nv lines of the set, increasing slope, in LDS) with the EnvChords margin;
// W bounds the set's slope range.  Chords past the chain, or of zero width, keep nothing.
template <int NC>
__device__ __forceinline__ ChainChords<NC> chain_chords(const double* vb, const double* va, int nv, double W) {
  ChainChords<NC> c;
  c.blo = vb[0];
  c.bhi = vb[nv - 1];
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int i0 = min(i, nv - 1), i1 = min(i + 1, nv - 1);
    const double b0 = vb[i0], a0 = va[i0], b1 = vb[i1], a1 = va[i1];
    const double db = b1 - b0;
    const double s = (i + 1 < nv && db > 0.0) ? (a1 - a0) / db : 0.0;
    const double tau = WALK_MARGIN * (fmax(fabs(a0), fabs(a1)) + fabs(s) * (fmax(fabs(b0), fabs(b1)) + W) + W);
    c.s[i] = s;
    c.k[i] = (i + 1 < nv && db > 0.0) ? fma(-s, b0, a0) - tau : INFINITY;
  }
  return c;
}

// The chain filter of one staged chunk (lines base + lane + 64 t) into the wave's long list (LIST_CAP_STREAM
// entries; cnt counts on past it).
template <int MAXL, int NC>
__device__ __forceinline__ void chain_keep(const double (&la)[MAXL], const double (&lb)[MAXL], int base, int nl,
                                           const ChainChords<NC>& c, int lane, double* sb, double* sa, int* si,
                                           int& cnt) {
  // the keep masks of a group of four slots first (independent tests, no branch between them), then the
  // group's writes (rarely any)
#pragma unroll
  for (int t0 = 0; t0 < MAXL; t0 += 4) {
    uint64_t mk[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int t = t0 + u;
      if (t < MAXL) {
        const double a = la[t], b = lb[t];
        bool s = (b < c.blo) | (b > c.bhi);
#pragma unroll
        for (int i = 0; i < NC; ++i) s = s | (fma(-c.s[i], b, a) >= c.k[i]);
        mk[u] = ballot(s & (base + lane + 64 * t < nl));
      } else {
        mk[u] = 0;
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int t = t0 + u;
      if (t < MAXL && mk[u] != 0) {  // wave-uniform, rarely taken
        if ((mk[u] >> lane) & 1) {
          const int pos = cnt + lanes_below(mk[u]);
          if (pos < LIST_CAP_STREAM) {
            sb[pos] = lb[t];
            sa[pos] = la[t];
            si[pos] = base + lane + 64 * t;
          }
        }
        cnt += __popcll(mk[u]);
      }
    }
  }
}

// L, T, R (with the tie rules of ext_fold) and the short-circuit status of the cnt lines of a survivor list.
__device__ __forceinline__ FwdEnv list_extremes(int cnt, int lane, const double* sb, const double* sa) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  ExtAcc e;
  for (int q = 0; 64 * q < cnt; ++q) {
    const int i = lane + 64 * q;
    const bool live = i < cnt;
    const int ii = live ? i : 0;
    const double a = sa[ii], b = sb[ii];
    const bool l = live & ((b < e.bmin) | ((b == e.bmin) & (a > e.aLx)));
    e.bmin = l ? b : e.bmin;
    e.aLx = l ? a : e.aLx;
    const bool r = live & ((b > e.bmax) | ((b == e.bmax) & (a > e.aRx)));
    e.bmax = r ? b : e.bmax;
    e.aRx = r ? a : e.aRx;
    const bool tt = live & ((a > e.amax) | ((a == e.amax) & (b < e.bTx)));
    e.amax = tt ? a : e.amax;
    e.bTx = tt ? b : e.bTx;
  }
  return ext_reduce(e);
}

// After the extremes and the filter pass (cnt survivors in the list): quickhull rounds if the list
// overflowed, the list walk, and the walk over all streamed lines when neither settles the pair.
template <int MAXL, class Build>
__device__ __forceinline__ EdgeSum env_pair_stream_tail(const FwdEnv& f, int cnt, int nch, int nl, int lane,
                                                        double* sb, double* sa, int* si, double* vreg,
                                                        bool force_walk, int* nhull, Build&& build) {
  if (cnt > LIST_CAP_STREAM && !force_walk) cnt = refine_stream<MAXL>(f, nch, nl, lane, sb, sa, si, vreg, build);
  if (cnt >= 0 && cnt <= LIST_CAP_STREAM && !force_walk) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    double cmax;
    EdgeSum kg;
    int h;
    if (cnt <= 128) kg = walk_small(cnt, lane, sb, sa, si, f.bL, f.aL, f.bT, &h, &cmax);
    else if (cnt <= 256) kg = walk_list<4>(cnt, lane, sb, sa, si, f.bL, f.aL, f.bT, &h, &cmax);
    else kg = walk_list<8>(cnt, lane, sb, sa, si, f.bL, f.aL, f.bT, &h, &cmax);
    if (uniform(cmax <= WALK_XGUARD)) {
      *nhull = h;
      return kg;
    }
  }
  return walk_stream<MAXL>(nch, nl, lane, f.bL, f.aL, f.bT, nhull, build);
}

template <int MAXL, class Build>
__device__ __forceinline__ EdgeSum env_pair_stream_edges(int nch, int nl, int lane, double* sb, double* sa, int* si,
                                                  double* vreg, bool force_walk, int* nhull, Build&& build) {
  const FwdEnv f = env_extremes_stream<MAXL>(nch, nl, lane, build);
  if (f.status == 1) {
    *nhull = 1;
    return EdgeSum{0.0, 0.0, 0.0, false};
  }
  const EnvChords ch = env_chords(f.bL, f.aL, f.bT, f.aT, f.bR, f.aR);
  int cnt = 0;
  for (int c = 0; c < nch; ++c) {
    double la[MAXL], lb[MAXL];
    build(c, la, lb);
    stream_keep<MAXL>(la, lb, c * 64 * MAXL, nl, ch, lane, sb, sa, si, cnt);
  }
  return env_pair_stream_tail<MAXL>(f, cnt, nch, nl, lane, sb, sa, si, vreg, force_walk, nhull, build);
}

template <int MAXL, class Build>
__device__ __forceinline__ double env_pair_stream(int nch, int nl, int lane, double* sb, double* sa, int* si,
                                                  double* vreg, bool force_walk, int* nhull, Build&& build) {
  return finish_edges(env_pair_stream_edges<MAXL>(nch, nl, lane, sb, sa, si, vreg, force_walk, nhull, build));
}

// Line coefficients of one (candidate, scalarisation) pair (discretekg.py:
// 182-223 full, :300-321 decoupled), wave-uniform: a_k = a_off + sum_i wa_i
// mu_i(z_k), b_k = sum_i wb_i cov_i(x_b, z_k); den = the scalarised noisy
// variance under the square root.  Outputs i >= m carry zero weights.  One
// definition for envelope_kernel and lines_export_kernel, so the exported
// lines are the envelope's lines bit for bit.
template <int M>
__device__ __forceinline__ void pair_coefs(const double* wrow, int m, bool full, int target, const double (&ysd)[M],
                                           const double (&ymu)[M], const double (&nz)[M], const double (&sv)[M],
                                           double (&w)[M], double (&wa)[M], double (&wb)[M], double& a_off,
                                           double& den) {
  a_off = 0.0;
  den = 0.0;
#pragma unroll
  for (int i = 0; i < M; ++i) {
    w[i] = (i < m) ? wrow[i] : 0.0;
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
}

// Padded length (doubles) of one LDS-staged line array: whole 1 KiB DMA pieces.
__host__ __device__ inline int stage_len(int N) { return ((N + 127) / 128) * 128; }


// Doubles in front of a staged record array: line 0 (the candidate, built from
// registers) reads record -1 there.
constexpr int STAGE_FRONT = 8;

// Stride (doubles) of one staged record array [N][rec]: room for the DMA
// pieces and for every register slot (line k reads record k - 1; records N ..
// 64 * slots - 2 hold the padding lines), plus the front pad.
__host__ __device__ inline int stage_stride(int N, int rec) {
  const int slots = 64 * env_slots(N + 1) * rec;
  return (stage_len(N * rec) > slots ? stage_len(N * rec) : slots) + STAGE_FRONT;
}

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

// Waves per SIMD the register allocation targets.  The forward up to 17
// slots fits 4 (<= 128 VGPRs: two envelope workgroups, or an envelope and a
// covariance workgroup, share a CU) without a spill: one pair per wave
// (nothing carried across pairs), the workgroup-uniform pair coefficients in
// SGPRs, and psi's exp / rational coefficients read as scalar operands
// (dkg_common.h psi) instead of libm's constants materialised in VGPRs.
// Measured steps: 2 waves/SIMD (220 VGPRs) 8.2 M KG-evals/s; 3 (168) 9.07 M;
// a loop of claimed pairs per wave needed 194 VGPRs at 2 and was slower
// (profiles/r02/r02y).
#ifndef DKG_ENV_FWD_WPE
#define DKG_ENV_FWD_WPE 4
#endif
__host__ __device__ constexpr int env_waves_per_eu(int maxl, int m, bool grad, bool stream) {
  return (grad || stream || maxl > 17) ? 2 : (m >= 8 && maxl > 8) ? 3 : DKG_ENV_FWD_WPE;  // m = 8: 3 spill-free
}


// GRAD: also dKG/dx_b (envelope theorem; include/dkg.h dkg_plan_forward_grad),
// accumulated into dkg[b x d]; the extra LDS follows the survivor lists.
// STREAM: no LDS staging of the line data; every pass rebuilds the lines
// chunk by chunk (64 * MAXL lines) from global memory (large N).
// HO (fused one-launch forward, dkg_fused.h): the covariance rows, variances and means are handed
// off by the workgroups of this launch: mu_D, the weights and the per-output scalars are staged
// first, then the wait on the candidate's row block (Handoff cnt2), then its rows; the last
// envelope workgroup to finish re-zeroes the launch's counters.
// The line data (mu_all, cov_all), the candidate posteriors (var_all, mux_all)
// and the weights arrive as arguments, so the first DMA issues after a
// single kernel-argument load instead of a pointer chase through the plan.
template <int MAXL, int M, bool GRAD, bool STREAM, bool HO = false>
__device__ __forceinline__ void envelope_body(const Plan* __restrict__ P, int B, double* __restrict__ kg,
                                              double* __restrict__ pairs_out, int dst,
                                              const double* __restrict__ xnew, double* __restrict__ dkg,
                                              const double* __restrict__ mu_all, const double* __restrict__ cov_all,
                                              const double* __restrict__ var_all,
                                              const double* __restrict__ mux_all, const double* __restrict__ wts,
                                              const int* __restrict__ dupv, long long cov_stride, int bpad, int b,
                                              int g, int G, double* smem, unsigned long long* st,
                                              const Handoff* ho = nullptr, double* __restrict__ hout = nullptr) {
  static_assert(!HO || (!GRAD && !STREAM), "the fused forward stages its lines (no gradient, no streaming)");
  // per output i: y_std, y_mean, noise, outputscale, noiseless variance at x_b, mean at x_b (model space),
  // and line 0's inputs: the mean and slope component it is built from (x_b's own, or, when x_b coincides
  // with a discretisation point (Plan::dup), that line's record: line 0 is then its exact copy)
  constexpr int NPP = 8;
  __shared__ double s_pp[DKG_MAX_OUTPUTS * NPP];
  __shared__ int s_kind[DKG_MAX_OUTPUTS];  // GRAD: covariance family per output
  const int SW = blockDim.x >> 6;
  const int lane_k = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int m = P->m;  // <= M
  const int N = P->N;
  const int NL = N + 1;
  const int S = P->S;
  const int target = P->target;
  const bool full = target < 0;
  static_assert(STREAM || MAXL == 2 || MAXL == 8 || MAXL == 17 || MAXL == 33, "slot bucket");
  KST_BEGIN(st);

  // The DMA sources first, in one scalar-load batch: the LDS-DMA intrinsics
  // count as memory writes, so anything read from P after them is re-read.
  const double* mu_src[M];
  const double* cv_src[M];
#pragma unroll
  for (int i = 0; i < M; ++i) {
    mu_src[i] = mu_all;
    cv_src[i] = cov_all + (size_t)b * cov_stride;  // records of candidate b
  }

  // LDS: [pad][mu_i over D] per output, [pad][cov_i over D] per output (line
  // k >= 1 reads index k - 1; the pad makes the lane-0 / slot-0 read legal),
  // the weights, then the per-wave survivor lists.
  constexpr int MP = cov_rec(M);  // doubles per line record
  const int SLp = STREAM ? 0 : stage_stride(N, MP);
  constexpr int LC = list_cap(STREAM && !GRAD);  // survivor-list capacity per wave
  // (the staged forward without mu_D records: its covariance records start where they would)
  constexpr bool ICP = DKG_ICP && !GRAD && !STREAM && !HO;  // intercepts from the plan's cache (Plan::icpt)
  constexpr bool MU_STAGED = !ICP;
  double* lmu = smem + STAGE_FRONT;
  double* lcv = lmu + ((STREAM || MU_STAGED) ? SLp : 0);
  double* lw = lcv + SLp;
  double* skg = lw + ((S * m + 1) & ~1);  // KG_j of the group's pairs (summed in j order)
  double* sbuf = skg + ((S + 1) & ~1);
  // GRAD regions: per-wave index lists, per-wave Q_D accumulators u_i[c], the
  // candidate's q_i and J_i rows, gv / gm / per-wave gradient scratch, x_b.
  const int d = P->d;
  const int NP = P->max_np;
  const int NPS = stage_len(NP);  // GRAD: LDS row stride of the candidate's q_i / J_i rows
  const double* disc = GRAD ? P->disc : nullptr;
  // test hook (DKG_PLAN_FORCE_WALK): every pair takes the list-overflow path
  const bool force_walk = __builtin_amdgcn_readfirstlane(P->debug_env) & 1;
  int* sidx = nullptr;
  double *qrow = nullptr, *jrow = nullptr, *sgv = nullptr, *sgm = nullptr, *sgw = nullptr, *sx = nullptr;
  double *sil = nullptr, *shD = nullptr, *suw = nullptr, *sscl = nullptr;
  int* shk = nullptr;
  if constexpr (GRAD) {
    double* gb = sbuf + (size_t)SW * 2 * LC;
    sidx = reinterpret_cast<int*>(gb);
    qrow = gb + (SW * ENV_CAP + 1) / 2;
    jrow = qrow + (size_t)M * NPS;                   // rows of stride NPS: whole DMA pieces
    sgv = jrow + (size_t)M * d * NPS;               // [M][16]  d v_i / dx
    sgm = sgv + M * DKG_MAX_DIM;                     // [M][16]  d mu_i / dx
    sgw = sgm + M * DKG_MAX_DIM;                     // [SW][64] per wave: gacc | ga0 | gvv | gtot
    sx = sgw + SW * 64;                              // [16]     x_b
    sil = sx + DKG_MAX_DIM;                          // [M][16]  1 / lengthscale per output
    shD = sil + M * DKG_MAX_DIM;                     // [SW][HCAP] per wave: pending hull lines' dE/db
    suw = shD + SW * HCAP;                           // [SW][NP]   per wave: u_i = sum_h coef_h Q_D,i[k_h]
    sscl = suw + (size_t)SW * NP;                    // [SW][ENV_CAP] per wave: left breakpoints of hull vertices
    shk = reinterpret_cast<int*>(sscl + SW * ENV_CAP);  // [SW][HCAP] pending hull lines' indices
  }

  // ---- one round of memory traffic: DMA the line data, plain loads for the rest
  // per-output scalars and the candidate's own posterior (variance from the
  // covariance stage, mean from the cross stage): lane i of wave 0 loads output i
  double pp[NPP] = {1.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  double g_gm[M], g_il[M], g_x = 0.0;  // GRAD: staged to LDS after the wait
  if (threadIdx.x < m) {
    const dkg_output* o = &P->o[threadIdx.x];
    pp[0] = o->y_std;
    pp[1] = o->y_mean;
    pp[2] = o->noise;
    pp[3] = o->outputscale;
    if constexpr (!HO) {
      pp[4] = var_all[(size_t)threadIdx.x * bpad + b];
      pp[5] = mux_all[(size_t)threadIdx.x * bpad + b];
      pp[6] = pp[5];
      pp[7] = pp[4];
    }
    if constexpr (GRAD) s_kind[threadIdx.x] = o->kernel;
  }
  const double* wsrc = wts;
  if constexpr (!STREAM) {
    // (the staged forward reads its intercepts from the plan's cache instead: no mu_D records in LDS)
    if constexpr (MU_STAGED) dma_to_lds(mu_src[0], lmu, N * MP, wave, SW, lane_k);
    if constexpr (!HO) dma_to_lds(cv_src[0], lcv, N * MP, wave, SW, lane_k);
  }
  if constexpr (GRAD) {
    // the candidate's q_i and J_i rows (row-major in the workspace) by LDS-DMA with the line data, so
    // they cost no extra memory round trip; entries npi .. NP-1 are zeroed after the wait
#pragma unroll
    for (int i = 0; i < M; ++i) {
      if (i < m) {
        const int npi = pad16(P->o[i].n);
        const size_t mat = (size_t)P->bpad * npi;
        dma_to_lds(P->qxrm[i] + (size_t)b * npi, qrow + (size_t)i * NPS, npi, wave, SW, lane_k);
        for (int dd = 0; dd < d; ++dd)
          dma_to_lds(P->jq[i] + dd * mat + (size_t)b * npi, jrow + ((size_t)i * d + dd) * NPS, npi, wave, SW, lane_k);
      }
    }
  }
  for (int e = threadIdx.x; e < S * m; e += blockDim.x) lw[e] = wsrc[e];
  // candidate b's coincidence mark (the covariance stage's; loaded with the first batch, used after the wait)
  int dupk = DUP_NONE;
  if constexpr (!HO) dupk = dupv[b];
  // this wave's scalarisation's top intercept over k >= 1 (TopHint), read with the first batch
  double hA1 = 0.0;
  int hk1 = 0, hc1 = 0;
  constexpr bool HINT = DKG_TOP_HINT && !GRAD && !STREAM && !HO;
  if constexpr (HINT) {
    if (P->itop != nullptr) {
      const int jh = min(g * SW + wave, S - 1);
      hA1 = P->itop[jh];
      hk1 = P->itopk[2 * jh];
      hc1 = P->itopk[2 * jh + 1];
    }
  }
  if (threadIdx.x < m) {
#pragma unroll
    for (int q = 0; q < (HO ? 4 : NPP); ++q) s_pp[threadIdx.x * NPP + q] = pp[q];
  }
  if constexpr (HO) {
    // the candidate's row block of covariance rows (and, transitively, its cross stage's means) is out
    handoff_wait(ho->cnt2 + (size_t)(b / ho->rb_rows) * HANDOFF_STRIDE, 1, ho->quota2, ho->err, 2);
    if (threadIdx.x < m) {
      s_pp[threadIdx.x * NPP + 4] = s_pp[threadIdx.x * NPP + 7] = var_all[(size_t)threadIdx.x * bpad + b];
      s_pp[threadIdx.x * NPP + 5] = s_pp[threadIdx.x * NPP + 6] = mux_all[(size_t)threadIdx.x * bpad + b];
    }
    dupk = dupv[b];
    dma_to_lds(cv_src[0], lcv, N * MP, wave, SW, lane_k);
  }
  if constexpr (GRAD) {
    // d mu_i/dx, 1/lengthscale and x_b into registers: per-output pointers by scalar loads (lgkmcnt,
    // not queued behind the DMAs on vmcnt), the values stored to LDS after the staging wait
#pragma unroll
    for (int i = 0; i < M; ++i) {
      g_gm[i] = 0.0;
      g_il[i] = 0.0;
      if (i < m && threadIdx.x < d) {
        g_gm[i] = P->gmu[i][(size_t)threadIdx.x * P->bpad + b];
        g_il[i] = P->o[i].inv_lengthscale[threadIdx.x];
      }
    }
    if (threadIdx.x < d) g_x = xnew[(size_t)b * d + threadIdx.x];
  }
  // Padding lines k = N+1 .. 64*MAXL-1 (records N .. 64*MAXL-2) come out of
  // the branch-free line build as (a = NaN, b = NaN): mu = cov = NaN makes
  // both NaN whatever the weights.  NaN drops out of every fmin/fmax (maxNum)
  // and fails every comparison, so the padding lines are never an extreme, a
  // tie, a survivor or counted, and the register lines need no per-slot
  // padding selects.  Doubles the DMA does not touch (>= stage_len(N * MP))
  // are written while it is in flight; the ones it over-writes with its last
  // piece (N * MP .. stage_len(N * MP) - 1) after it has landed.
  const int SLd = STREAM ? 0 : stage_len(N * MP);
  const int pad_end = (64 * MAXL - 1) * MP;
  auto pad_lines = [&](int lo, int hi) {  // doubles lo .. hi-1 of both record arrays
    for (int e = lo + (int)threadIdx.x; e < hi; e += blockDim.x) {
      if constexpr (MU_STAGED) lmu[e] = __builtin_nan("");
      lcv[e] = __builtin_nan("");
    }
  };
  if constexpr (!STREAM) pad_lines(max(N * MP, SLd), pad_end);
  // pairs j0 .. j1-1 of the candidate, one per wave (gridDim.y = ceil(S / SW), envelope_geometry)
  const int j0 = g * SW, j1 = min(S, j0 + SW);
  // Staged forward with the plan's intercept cache (Plan::icpt): this wave's intercepts a_k (slot t of lane
  // l: line l + 64 t) straight into registers, in flight with the staging DMA; only the covariance records
  // are built from LDS.
  gdptr icp = nullptr;  // this wave's row of the cache (wave-uniform)
  double ila[ICP ? MAXL : 1];
  if constexpr (ICP) {
    // always set for a staged plan (dkg_abi.hip build_plan)
    icp = uniform_gptr(P->icpt + (size_t)min(j0 + wave, S - 1) * P->icpt_stride);
    if (j0 + wave < j1) {
#pragma unroll
      for (int t = 0; t < MAXL; ++t) ila[t] = icp[lane_k + 64 * t];
    }
  }
  if (!GRAD) KST(st, 2);  // GRAD stamps: 2 preamble done, 3 filter, 4 hull, 5 gradient flush (first pair)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if constexpr (!STREAM) {
    if (SLd > N * MP) {  // uniform
      pad_lines(N * MP, min(SLd, pad_end));
      __syncthreads();
    }
  }
  dupk = __builtin_amdgcn_readfirstlane(dupk);
  if (dupk != DUP_NONE) {  // rare (workgroup-uniform): line 0 from record dupk, the same bits as line dupk + 1
    if (threadIdx.x < m) {
      s_pp[threadIdx.x * NPP + 6] = mu_all[(size_t)dupk * MP + threadIdx.x];
      s_pp[threadIdx.x * NPP + 7] = cov_all[(size_t)b * cov_stride + (size_t)dupk * MP + threadIdx.x];
    }
    __syncthreads();
  }
  if constexpr (GRAD) {
    if (threadIdx.x < d) {
      sx[threadIdx.x] = g_x;
#pragma unroll
      for (int i = 0; i < M; ++i) {
        if (i < m) {
          sgm[i * DKG_MAX_DIM + threadIdx.x] = g_gm[i];
          sil[i * DKG_MAX_DIM + threadIdx.x] = g_il[i];
        }
      }
    }
    // rows of outputs with fewer (padded) training points than the widest: zero the tail the DMA filled
    bool tail = false;
#pragma unroll
    for (int i = 0; i < M; ++i) {
      if (i < m) {
        const int npi = pad16(P->o[i].n);
        if (npi < NP) {
          tail = true;
          for (int c = npi + (int)threadIdx.x; c < NP; c += blockDim.x) {
            qrow[(size_t)i * NPS + c] = 0.0;
            for (int dd = 0; dd < d; ++dd) jrow[((size_t)i * d + dd) * NPS + c] = 0.0;
          }
        }
      }
    }
    if (tail) __syncthreads();  // uniform
  }
  if (!GRAD) KST(st, 3);

  double* sb = sbuf + (size_t)wave * 2 * LC;
  double* sa = sb + LC;
  // streaming forward: the quickhull refinement's vertex arrays after the lists
  // staged streaming forward: the chunk buffers take the vertex arrays' place (the refinement runs
  // after the staged passes, so it reuses their room)
  constexpr bool STG = STREAM && !GRAD && stream_staged(M);
  constexpr int CBL = STG ? staged_chunk_len(cov_rec(M)) : 0;
  const int vreg_room = STG ? max(SW * VREG, 4 * CBL) : ((STREAM && !GRAD) ? SW * VREG : 0);
  double* cbuf = sbuf + (size_t)SW * 2 * LC;
  double* vreg = cbuf + (size_t)wave * VREG;
  // forward: the list's line indices after the vertex arrays (GRAD: sidx)
  int* sif = reinterpret_cast<int*>(sbuf + (size_t)SW * 2 * LC + vreg_room) +
             (size_t)wave * LC;
  int* si = nullptr;
  double* gw = nullptr;
  if constexpr (GRAD) {
    si = sidx + (size_t)wave * ENV_CAP;
    gw = sgw + wave * 64;
    // d v_i / dx = -2 J_i^T q_i (model space), one (output, coordinate) per wave
    for (int pidx = wave; pidx < m * d; pidx += SW) {
      const int i = pidx / d, dd = pidx % d;
      double acc = 0.0;
      for (int c = lane_k; c < NP; c += 64) acc = fma(jrow[((size_t)i * d + dd) * NPS + c], qrow[(size_t)i * NPS + c], acc);
      acc = wave_sum(acc);
      if (lane_k == 0) sgv[i * DKG_MAX_DIM + dd] = -2.0 * acc;
    }
    gw[lane_k] = 0.0;
    __syncthreads();
    KST(st, 2);
  }
  // One pair per wave, written as a one-shot block: nothing pair-invariant (psi's coefficients, lane
  // addresses) is hoisted out of a loop and kept live in registers.
  // sv / mx0: the candidate's noiseless variance and mean (the slopes' normaliser, the gradient);
  // l0v / l0m: what line 0 is built from (the same unless x_b coincides with a discretisation point)
  double sv[M], mx0[M], ysd[M], ymu[M], nz[M], os[M], l0m[M], l0v[M];
#pragma unroll
  for (int i = 0; i < M; ++i) {
    const bool live = i < m;
    // workgroup-uniform: kept in SGPRs across the pair loop
    ysd[i] = sgpr_f64(live ? s_pp[i * NPP + 0] : 1.0);
    ymu[i] = sgpr_f64(live ? s_pp[i * NPP + 1] : 0.0);
    nz[i] = sgpr_f64(live ? s_pp[i * NPP + 2] : 0.0);
    os[i] = sgpr_f64(live ? s_pp[i * NPP + 3] : 0.0);
    sv[i] = sgpr_f64(live ? s_pp[i * NPP + 4] : 0.0);
    mx0[i] = sgpr_f64(live ? s_pp[i * NPP + 5] : 0.0);
    l0m[i] = sgpr_f64(live ? s_pp[i * NPP + 6] : 0.0);
    l0v[i] = sgpr_f64(live ? s_pp[i * NPP + 7] : 0.0);
  }

  // ---- staged streaming forward: the extremes pass and the filter pass of every pair of the workgroup
  // over LDS-staged chunks of the line records (chunk q: lines q*SCH .. q*SCH + SCH - 1, records k - 1),
  // the next chunk's DMA in flight while the current one is read; the survivor lists then go to the
  // per-pair tail (refinement, walks) below.  Waves without a pair stage with the others.
  FwdEnv sf;
  int scnt = 0;
  if constexpr (STG) {
    constexpr int CS = STAGED_SLOTS, SCH = 64 * CS;
    const int lane = lane_k;
    const bool has = j0 + wave < j1;
    const int jj = has ? j0 + wave : j0;
    double w[M], wa[M], wb[M];
    double a_off, den;
    pair_coefs<M>(lw + jj * m, m, full, target, ysd, ymu, nz, sv, w, wa, wb, a_off, den);
#pragma unroll
    for (int i = 0; i < M; ++i) {
      wa[i] = sgpr_f64(wa[i]);
      wb[i] = sgpr_f64(wb[i]);
    }
    a_off = sgpr_f64(a_off);
    double bb0 = 0.0, a0 = a_off, wbt = 0.0;
#pragma unroll
    for (int i = 0; i < M; ++i) {
      bb0 = fma(wb[i], l0v[i], bb0);
      a0 = fma(wa[i], l0m[i], a0);
      wbt = (i == target) ? wb[i] : wbt;
    }
    const int nq = (NL + SCH - 1) / SCH;
    const double* cvb = cov_all + (size_t)b * cov_stride;
    // chunk q's records into buffer q & 1 by a transposing DMA: position p of plane q2 holds component
    // pair q2 of record q*SCH - 1 + p (line q*SCH + p; clamped into 0 .. N-1, the clamped positions are
    // line 0, built from registers, and padding lines); one instruction = 64 positions of one plane
    auto stage = [&](int q) {
      constexpr int NP2 = MP / 2, GR = SCH / 64, NI = NP2 * GR;
      double* bm = cbuf + (size_t)(q & 1) * 2 * CBL;
      for (int ii = wave; ii < 2 * NI; ii += SW) {
        const int arr = ii / NI, rem = ii % NI, q2 = rem / GR, gi = rem % GR;
        const double* src = arr ? cvb : mu_all;
        const int rec = min(max(q * SCH - 1 + gi * 64 + lane_k, 0), N - 1);
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + (size_t)rec * MP + 2 * q2),
                                         reinterpret_cast<__attribute__((address_space(3))) void*>(
                                             reinterpret_cast<uintptr_t>(bm + (size_t)arr * CBL +
                                                                         ((size_t)q2 * SCH + gi * 64) * 2)),
                                         16, 0, 0);
      }
    };
    // build_chunk's lines (same arithmetic, same order) from the staged records of chunk q
    auto build_staged = [&](int q, double (&la)[CS], double (&lb)[CS]) {
      const double* bm = cbuf + (size_t)(q & 1) * 2 * CBL;
      const double* mur = bm + lane * 2;        // plane q2, slot t: + (q2 * SCH + 64 t) * 2
      const double* cvr = bm + CBL + lane * 2;
      const int kbase = q * SCH;
      // 16-byte reads, consecutive across the wave; components i >= m carry zero weights over zero
      // padding, so the sums are build_chunk's.  The full / target choice outside the slot loop: one LDS
      // read stream, no wait per slot.
      auto adot = [&](const double* r, const double (&c)[M], double acc) __attribute__((always_inline)) {
#pragma unroll
        for (int q2 = 0; 2 * q2 < M; ++q2) {
          const double2 u = *reinterpret_cast<const double2*>(r + (size_t)q2 * SCH * 2);
          acc = fma(c[2 * q2], u.x, acc);
          if (2 * q2 + 1 < M) acc = fma(c[2 * q2 + 1], u.y, acc);
        }
        return acc;
      };
      const int tg = full ? 0 : target;
      const double* cvt = cvr + (size_t)(tg >> 1) * SCH * 2 + (tg & 1);  // target path
      if (full) {
#pragma unroll
        for (int t = 0; t < CS; ++t) {
          la[t] = adot(mur + 128 * t, wa, a_off);
          lb[t] = adot(cvr + 128 * t, wb, 0.0);
        }
      } else {
#pragma unroll
        for (int t = 0; t < CS; ++t) {
          la[t] = adot(mur + 128 * t, wa, a_off);
          lb[t] = fma(wbt, cvt[128 * t], 0.0);
        }
      }
#pragma unroll
      for (int t = 0; t < CS; ++t) {
        if (kbase + 64 * t + 63 > N) {  // wave-uniform: padding lines in this slot
          const bool pad = kbase + lane + 64 * t > N;
          la[t] = pad ? -INFINITY : la[t];
          lb[t] = pad ? bb0 : lb[t];
        }
      }
      if (q == 0) {
        la[0] = (lane == 0) ? a0 : la[0];
        lb[0] = (lane == 0) ? bb0 : lb[0];
      }
    };
#if DKG_STG_SAMPLE
    // pass 0: the pair's sample hull.  Every stride-th line (line j * stride in slot j of a staged chunk laid
    // out as chunk 0) staged in buffer 0 by one strided DMA, then per wave the sample's extremes and
    // SH_ROUNDS quickhull rounds in registers; the vertex chain (lines of the set) goes to buffer 1.
    const int stride = (NL + SCH - 1) / SCH;
    {
      constexpr int NP2 = MP / 2, GR = SCH / 64, NI = NP2 * GR;
      for (int ii = wave; ii < 2 * NI; ii += SW) {
        const int arr = ii / NI, rem = ii % NI, q2 = rem / GR, gi = rem % GR;
        const double* src = arr ? cvb : mu_all;
        const int rec = min(max((gi * 64 + lane_k) * stride - 1, 0), N - 1);
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + (size_t)rec * MP + 2 * q2),
                                         reinterpret_cast<__attribute__((address_space(3))) void*>(
                                             reinterpret_cast<uintptr_t>(cbuf + (size_t)arr * CBL +
                                                                         ((size_t)q2 * SCH + gi * 64) * 2)),
                                         16, 0, 0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    ChainChords<SH_NC> cc;
    bool chain_ok = false;
    // test hook (DKG_PLAN_NO_CHAIN): no chain, every pair takes the overflow path
    if (has && !(__builtin_amdgcn_readfirstlane(P->debug_env) & 8)) {
      double la[CS], lb[CS];
      build_staged(0, la, lb);  // sample line j in slot j (q = 0: line 0 from registers; j * stride > N: a copy
                                // of line N, still a line of the set)
      ExtAcc es;
      ext_fold<CS>(la, lb, 0, SCH, lane, es);
      const FwdEnv fs = ext_reduce(es);
      double* vb = cbuf + 2 * (size_t)CBL + (size_t)wave * VREG;
      double* va = vb + VCAP;
      if (fs.status == 0) {
        if (lane == 0) {
          vb[0] = fs.bL; va[0] = fs.aL;
          vb[1] = fs.bT; va[1] = fs.aT;
          vb[2] = fs.bR; va[2] = fs.aR;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        int nv = 3, tpos = 1;
        auto sample = [&](int, double (&xa)[CS], double (&xb)[CS]) {
#pragma unroll
          for (int t = 0; t < CS; ++t) { xa[t] = la[t]; xb[t] = lb[t]; }
        };
        if (qh_extend<CS, 3>(1, SCH, lane, vb, va, nv, tpos, sample) > 0 && SH_ROUNDS > 1)
          qh_extend<CS, 5>(1, SCH, lane, vb, va, nv, tpos, sample);
        // the set's slope range is at most 2 sum_i |wb_i| sqrt(v_i(x) s_i) (Cauchy-Schwarz on the posterior
        // covariance, the posterior variance at z below the prior s_i), with room for the rounding of cov
        double bm = 0.0;
#pragma unroll
        for (int i = 0; i < M; ++i)
          bm = fma(fabs(wb[i]), sqrt(fmax(sv[i], 0.0) * fmax(os[i], 0.0)) + 1e-8 * fabs(os[i]), bm);
        cc = chain_chords<SH_NC>(vb, va, nv, 2.0 * bm * (1.0 + 1e-6));
        chain_ok = true;
      }
    }
    __syncthreads();  // every wave has its chain in registers: the buffers take the staged chunks
#ifdef DKG_STG_STAMPS
    if (st) st[4] = __builtin_amdgcn_s_memtime();  // pass 0 done
#endif
    // the staged pass: the chain filter into the survivor list
    stage(0);
    for (int q = 0; q < nq; ++q) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (q + 1 < nq) stage(q + 1);
      if (chain_ok) {
        double la[CS], lb[CS];
        build_staged(q, la, lb);
        chain_keep<CS, SH_NC>(la, lb, q * SCH, NL, cc, lane, sb, sa, sif, scnt);
      }
    }
    __syncthreads();  // the chunk buffers are the refinement's vertex arrays from here
#ifdef DKG_STG_STAMPS
    if (st) st[5] = __builtin_amdgcn_s_memtime();  // staged pass done
#endif
    // no chain (the sample has a single slope): the per-pair tail takes the extremes and the filter from the
    // streamed lines (overflow path)
    if (!chain_ok) scnt = LIST_CAP_STREAM + 1;
    sf.status = 0;
#else
    // pass 1: extremes
    ExtAcc e;
#ifdef DKG_STG_STAMPS
    unsigned long long twait = 0, tw0 = 0;
#define STG_W0 tw0 = __builtin_amdgcn_s_memtime();
#define STG_W1 twait += __builtin_amdgcn_s_memtime() - tw0;
#else
#define STG_W0
#define STG_W1
#endif
    stage(0);
    for (int q = 0; q < nq; ++q) {
      STG_W0
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();  // chunk q landed; every wave is done with the other buffer
      STG_W1
      if (q + 1 < nq) stage(q + 1);
      if (has) {
        double la[CS], lb[CS];
        build_staged(q, la, lb);
        ext_fold<CS>(la, lb, q * SCH, NL, lane, e);
      }
    }
    sf = ext_reduce(e);
    // pass 2: the chord filter into the survivor list
    const bool live = has && sf.status == 0;
    const EnvChords ch = env_chords(sf.bL, sf.aL, sf.bT, sf.aT, sf.bR, sf.aR);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // every wave is done with the last chunk of pass 1
    stage(0);
    for (int q = 0; q < nq; ++q) {
      STG_W0
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      STG_W1
      if (q + 1 < nq) stage(q + 1);
      if (live) {
        double la[CS], lb[CS];
        build_staged(q, la, lb);
        stream_keep<CS>(la, lb, q * SCH, NL, ch, lane, sb, sa, sif, scnt);
      }
    }
    __syncthreads();  // the chunk buffers are the refinement's vertex arrays from here
#ifdef DKG_STG_STAMPS
    if (st) st[4] = twait;  // raw: wait cycles of wave 0 over both passes
    if (st) st[5] = __builtin_amdgcn_s_memtime();
#endif
#endif  // DKG_STG_SAMPLE
  }
#undef STG_W0
#undef STG_W1

  if (const int j = j0 + wave; j < j1) {
    const int lane = lane_k;
    // ---- line coefficients (wave uniform; shared with lines_export_kernel)
    double w[M], wa[M], wb[M];
    double a_off, den;
    pair_coefs<M>(lw + j * m, m, full, target, ysd, ymu, nz, sv, w, wa, wb, a_off, den);
#pragma unroll
    for (int i = 0; i < M; ++i) {  // wave-uniform: SGPRs, not VGPRs, while the lines are live
      w[i] = sgpr_f64(w[i]);
      wa[i] = sgpr_f64(wa[i]);
      wb[i] = sgpr_f64(wb[i]);
    }
    a_off = sgpr_f64(a_off);
    den = sgpr_f64(den);
    // ---- lines: slot t of lane l is line k = l + 64 t (k = 0: the candidate).
    // Branch-free bodies (one LDS read stream per array, no per-slot waits):
    // unused output slots read output 0 with a zero weight.  Rebuilt from the
    // staged LDS data when the survivor list overflows, so the register copy
    // is dead once the filter has run.
    double bb0 = 0.0;  // line 0's slope (the padding lines reuse it)
#pragma unroll
    for (int i = 0; i < M; ++i) bb0 = fma(wb[i], l0v[i], bb0);
    // STREAM: chunk c of the lines straight from global memory
    auto build_chunk = [&](int c, double (&la)[MAXL], double (&lb)[MAXL]) {
      const int kbase = c * 64 * MAXL;
      const size_t rowoff = (size_t)b * cov_stride;  // candidate b's records
      const int nmax = max(N, 1) - 1;
#pragma unroll
      for (int t = 0; t < MAXL; ++t) {
        const int k = kbase + lane + 64 * t;
        const int idx = min(max(k - 1, 0), nmax);
        double a = a_off, bb = 0.0;
#pragma unroll
        for (int i = 0; i < M; ++i) {
          if (i < m) {
            a = fma(wa[i], mu_all[(size_t)idx * MP + i], a);
            if (full || i == target) bb = fma(wb[i], cov_all[rowoff + (size_t)idx * MP + i], bb);
          }
        }
        la[t] = a;
        lb[t] = bb;
        if (kbase + 64 * t + 63 > N) {  // wave-uniform: padding lines in this slot
          const bool pad = k > N;
          la[t] = pad ? -INFINITY : la[t];
          lb[t] = pad ? bb0 : lb[t];
        }
      }
      if (c == 0) {
        double a = a_off;  // line 0: the candidate itself (discretekg.py:182-183)
#pragma unroll
        for (int i = 0; i < M; ++i) a = fma(wa[i], l0m[i], a);
        la[0] = (lane == 0) ? a : la[0];
        lb[0] = (lane == 0) ? bb0 : lb[0];
      }
    };
    const int nch = (NL + 64 * MAXL - 1) / (64 * MAXL);
    auto build_lines = [&](double (&la)[MAXL], double (&lb)[MAXL]) {
      // line k = lane + 64 t reads record k - 1; outputs in output order (the FMA order of the
      // reference's weighted sums), two per 16-byte read; components >= m are zero with zero weight
      const double* mur = lmu + (lane - 1) * MP;
      const double* cvr = lcv + (lane - 1) * MP;
      // sum_i c[i] r_i over record r (weights c)
      auto rec_dot = [&](const double* r, const double (&c)[M], double acc) __attribute__((always_inline)) {
        if constexpr (MP == 1) {
          acc = fma(c[0], r[0], acc);
        } else {
#pragma unroll
          for (int q = 0; 2 * q < M; ++q) {
            const double2 u = *reinterpret_cast<const double2*>(r + 2 * q);
            acc = fma(c[2 * q], u.x, acc);
            if (2 * q + 1 < M) acc = fma(c[2 * q + 1], u.y, acc);
          }
        }
        return acc;
      };
      if (full) {
#pragma unroll
        for (int t = 0; t < MAXL; ++t) {
          la[t] = rec_dot(mur + 64 * MP * t, wa, a_off);
          lb[t] = rec_dot(cvr + 64 * MP * t, wb, 0.0);
        }
      } else {
        const double* cvt = cvr + target;
        double wbt = 0.0;
#pragma unroll
        for (int i = 0; i < M; ++i) wbt = (i == target) ? wb[i] : wbt;
#pragma unroll
        for (int t = 0; t < MAXL; ++t) {
          la[t] = rec_dot(mur + 64 * MP * t, wa, a_off);
          lb[t] = wbt * cvt[64 * MP * t];
        }
      }
      {
        double a = a_off, bb = 0.0;  // line 0: the candidate itself (discretekg.py:182-183)
#pragma unroll
        for (int i = 0; i < M; ++i) {
          a = fma(wa[i], l0m[i], a);
          bb = fma(wb[i], l0v[i], bb);
        }
        la[0] = (lane == 0) ? a : la[0];
        lb[0] = (lane == 0) ? bb : lb[0];
      }
      // padding lines beyond N: (NaN, NaN) from the padded staging (see above)
    };

    double kgj;
    int hn = 1;  // upper-envelope lines of this pair (recorded with kg_pairs)
    if constexpr (GRAD) {
      EnvFilter f;
      if constexpr (STREAM) {
        f = envelope_filter_stream<MAXL, true>(nch, lane, sb, sa, si, build_chunk);
      } else {
        double la[MAXL], lb[MAXL];
        build_lines(la, lb);
        // Flat envelope (env_flat, as in the forward): every breakpoint beyond +-48, so every phi / psi
        // term is exactly 0 and every Phi exactly 0 or 1: KG_w = 0 and the pair's gradient terms cancel to
        // exactly 0 (line 0 off the top: no da_0 term; line 0 = T: Phi(cR) - Phi(cL) = 1 against the
        // [line 0 attains max a] / cnt term with cnt = 1).  Only an exact copy of line 0 at the top (cnt > 1,
        // a subgradient share) needs the full path.
        bool flat = false;
        if (!force_walk) {
          FwdEnv fe;
          env_top<MAXL>(la, lb, fe);
          if (env_flat<MAXL>(la, lb, fe)) {
            const double a0l = readlane_f64(la[0], 0);
            int ct = 0;
#pragma unroll
            for (int t = 0; t < MAXL; ++t) ct += __popcll(ballot(la[t] == fe.aT));
            flat = !(a0l == fe.aT) || ct == 1;
          }
        }
        if (flat)
          f.status = 3;
        else
          f = envelope_filter<MAXL, true>(la, lb, lane, sb, sa, si);
      }
      if (force_walk && f.status == 0) f.status = 2;
      if (j == j0 + wave) KST(st, 3);
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
      // Envelope lines k >= 1 are queued (index, dE/db) in the wave's list and
      // their gradient terms evaluated together by flush(): the kernel
      // derivative one line per lane, and J_i^T Q_D,i[k] as one dot per
      // (output, coordinate) against u_i = sum_h coef_h Q_D,i[k_h], so the
      // gathers of all queued rows are independent and the wave sums are paid
      // once per flush instead of once per line.
      int* hk = shk + wave * HCAP;
      double* scl = sscl + wave * ENV_CAP;
      double* hD = shD + wave * HCAP;
      double* uw = suw + (size_t)wave * NP;
      int nh = 0;
      auto flush = [&]() __attribute__((always_inline)) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // kernel-derivative terms: lane h handles queued line h
        {
          const bool act = lane < nh;
          const int k = act ? hk[lane] : 1;
          const double Dw = act ? hD[lane] : 0.0;
          const double* z = disc + (size_t)(k - 1) * d;
          double hc[M];
#pragma unroll
          for (int i = 0; i < M; ++i) {
            hc[i] = 0.0;
            if (i < m && wb[i] != 0.0) {
              double r2 = 0.0;
              for (int dd = 0; dd < d; ++dd) {
                const double t = (sx[dd] - z[dd]) * sil[i * DKG_MAX_DIM + dd];
                r2 = fma(t, t, r2);
              }
              hc[i] = Dw * wb[i] * os[i] * kernel_dprofile(__builtin_amdgcn_readfirstlane(s_kind[i]), r2);
            }
          }
          for (int dd = 0; dd < d; ++dd) {
            const double t = sx[dd] - z[dd];
            double v = 0.0;
#pragma unroll
            for (int i = 0; i < M; ++i) {
              const double il = sil[((i < m) ? i : 0) * DKG_MAX_DIM + dd];
              v = fma(hc[i] * t, il * il, v);
            }
            v = wave_sum(v);
            if (lane == 0) gw[dd] += v;
          }
        }
        // - sum_h coef_h J_i^T Q_D,i[k_h - 1]
        if (uniform(NP <= 256)) {
          // every output's rows of every queued line in flight together; the
          // dots J_i^T u_i come straight from the registers
          double u[M][4];
          const double* qd[M];
          int npo[M];
#pragma unroll
          for (int i = 0; i < M; ++i) {
            qd[i] = P->qdrm[(i < m) ? i : 0];
            npo[i] = pad16(P->o[(i < m) ? i : 0].n);
#pragma unroll
            for (int q = 0; q < 4; ++q) u[i][q] = 0.0;
          }
#pragma unroll 4
          for (int h = 0; h < nh; ++h) {
            const int r = hk[h] - 1;
            const double dw = hD[h];
#pragma unroll
            for (int i = 0; i < M; ++i) {
              if (i < m) {
                const double* row = qd[i] + (size_t)r * npo[i];
#pragma unroll
                for (int q = 0; q < 4; ++q) u[i][q] = fma(dw, row[min(lane + 64 * q, npo[i] - 1)], u[i][q]);
              }
            }
          }
#pragma unroll
          for (int i = 0; i < M; ++i) {
            if (i < m && wb[i] != 0.0) {
              for (int dd = 0; dd < d; ++dd) {
                const double* jr = jrow + ((size_t)i * d + dd) * NPS;
                double acc = 0.0;
#pragma unroll
                for (int q = 0; q < 4; ++q)
                  if (lane + 64 * q < npo[i]) acc = fma(jr[lane + 64 * q], u[i][q], acc);
                acc = wave_sum(acc);
                if (lane == 0) gw[dd] -= acc * wb[i];
              }
            }
          }
        } else {
#pragma unroll
        for (int i = 0; i < M; ++i) {
          if (i < m && wb[i] != 0.0) {
            const double* qd = P->qdrm[i];
            const int npi = pad16(P->o[i].n);
            for (int c0 = 0; c0 < npi; c0 += 4 * 64) {
              // 4 column chunks of every queued row in flight together
              double u[4] = {0.0, 0.0, 0.0, 0.0};
              const int c = c0 + lane;
              for (int h = 0; h < nh; ++h) {
                const double* row = qd + (size_t)(hk[h] - 1) * npi;
                const double dw = hD[h];
#pragma unroll
                for (int q = 0; q < 4; ++q) u[q] = fma(dw, row[min(c + 64 * q, npi - 1)], u[q]);
              }
#pragma unroll
              for (int q = 0; q < 4; ++q)
                if (c + 64 * q < npi) uw[c + 64 * q] = u[q] * wb[i];
            }
            for (int dd = 0; dd < d; ++dd) {
              const double* jr = jrow + ((size_t)i * d + dd) * NPS;
              double acc = 0.0;
              for (int c = lane; c < npi; c += 64) acc = fma(jr[c], uw[c], acc);
              acc = wave_sum(acc);
              if (lane == 0) gw[dd] -= acc;
            }
          }
        }
        }
        nh = 0;
      };
      // one envelope line: d/dx of its slope (and of line 0's intercept), weighted
      // by dE/db = phi(cL) - phi(cR) and dE/da = Phi(cR) - Phi(cL)
      auto visit = [&](int k, double bP, double aP, double cL, double cR) __attribute__((always_inline)) {
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
          if (lane == 0) {
            hk[nh] = k;
            hD[nh] = Dw;
          }
          if (++nh == HCAP) flush();
        }
      };
      // line indices of L, T, R (lowest among exact duplicates) and the number
      // of lines attaining max a: one pass over the rebuilt lines, after the
      // filter has released its registers
      if (f.status == 2) {
        int kL = 1 << 30, kT = 1 << 30, kR = 1 << 30, ct = 0;
        auto scan = [&](const double (&la)[MAXL], const double (&lb)[MAXL], int base) {
#pragma unroll
          for (int t = MAXL - 1; t >= 0; --t) {
            const int k = base + lane + 64 * t;
            kL = (lb[t] == f.bL && la[t] == f.aL) ? k : kL;
            kT = (la[t] == f.aT && lb[t] == f.bT) ? k : kT;
            kR = (lb[t] == f.bR && la[t] == f.aR) ? k : kR;
            ct += __popcll(ballot(la[t] == f.aT));
          }
        };
        if constexpr (STREAM) {
          for (int c = nch - 1; c >= 0; --c) {
            double la[MAXL], lb[MAXL];
            build_chunk(c, la, lb);
            scan(la, lb, c * 64 * MAXL);
          }
        } else {
          double la[MAXL], lb[MAXL];
          build_lines(la, lb);
          scan(la, lb, 0);
        }
        DKG_BUTTERFLY({
          const int st = S_ == 0 ? 1 : S_ == 1 ? 2 : S_ == 2 ? 4 : S_ == 3 ? 8 : S_ == 4 ? 16 : 32;
          kL = min(kL, __shfl_xor(kL, st));
          kT = min(kT, __shfl_xor(kT, st));
          kR = min(kR, __shfl_xor(kR, st));
        })
        f.kL = __builtin_amdgcn_readfirstlane(kL);
        f.kT = __builtin_amdgcn_readfirstlane(kT);
        f.kR = __builtin_amdgcn_readfirstlane(kR);
        f.cntT = ct;
      }
      if (f.status == 1 || f.status == 3) {  // short-circuit, flat envelope: KG_w = 0, no gradient terms
        kgj = 0.0;
      } else {
        if (f.status == 0) {
          const HullGrad hg = envelope_hull_grad(f, lane, sb, sa, si, scl, hk, hD, N);
          kgj = hg.kg;
          sumDb = hg.sumDb;
          nh = hg.nq;
          f.cntT = hg.cntT;
          if (lane == 0) {  // line 0 (the candidate): d b_0 and d a_0 terms
            for (int dd = 0; dd < d; ++dd) {
              double gvs = 0.0;
#pragma unroll
              for (int i = 0; i < M; ++i)
                if (i < m) gvs = fma(wb[i], sgv[i * DKG_MAX_DIM + dd], gvs);
              gw[dd] += hg.Dw0 * gvs + hg.Pw0 * gw[16 + dd];
            }
          }
        } else if constexpr (STREAM) {
          kgj = envelope_walk_stream<MAXL>(nch, NL, lane, f, build_chunk, visit, f.kL);
        } else {
          // list overflow: gift wrap, rebuilding the staged lines every step so
          // no register lines stay live across the visits
          auto rebuild = [&](int, double (&la)[MAXL], double (&lb)[MAXL]) { build_lines(la, lb); };
          kgj = envelope_walk_stream<MAXL>(1, NL, lane, f, rebuild, visit, f.kL);
        }
        if (j == j0 + wave) KST(st, 4);
        if (nh > 0) flush();
        if (j == j0 + wave) KST(st, 5);
        // - sum_e Dw_e b_e * dV/(2V), - [line 0 attains max a] da_0/dx
        double a0 = a_off;
#pragma unroll
        for (int i = 0; i < M; ++i) a0 = fma(wa[i], l0m[i], a0);
        const double tfac = (a0 == f.aT) ? 1.0 / (double)f.cntT : 0.0;
        if (lane == 0)
          for (int dd = 0; dd < d; ++dd) gw[48 + dd] += gw[dd] - sumDb * gw[32 + dd] - tfac * gw[16 + dd];
      }
      if (lane == 0)
        for (int dd = 0; dd < d; ++dd) gw[dd] = 0.0;
    } else if constexpr (STG) {
#if DKG_STG_SAMPLE
      // L, T, R and the short-circuit test from the list (it holds every upper-hull line of the set), or,
      // after an overflow, from the streamed lines
      sf = (scnt <= LIST_CAP_STREAM) ? list_extremes(scnt, lane, sb, sa) : env_extremes_stream<MAXL>(nch, NL, lane,
                                                                                                     build_chunk);
#ifdef DKG_STG_STAMPS
      if (lane == 0) P->hull_pairs[(size_t)b * S + j] = scnt;  // diagnostics build: the list length per pair
#endif
#endif
      if (sf.status == 1) {
        kgj = 0.0;
        hn = 1;
      } else {
        kgj = finish_edges(env_pair_stream_tail<MAXL>(sf, scnt, nch, NL, lane, sb, sa, sif, vreg, force_walk, &hn,
                                                      build_chunk));
      }
    } else if constexpr (STREAM) {
      kgj = env_pair_stream<MAXL>(nch, NL, lane, sb, sa, sif, vreg, force_walk, &hn, build_chunk);
    } else {
      // wave-uniform (every lane writes the same stamps): a pointer that stays in SGPRs
      unsigned long long* pst = (dst == 2 && (size_t)b * S + j < 2 * KST_WG)
                                    ? P->kstamps + ((size_t)b * S + j) * 8 : nullptr;
      // pairs_out also records the envelope size: every pair is walked then
      const bool flat_ok = pairs_out == nullptr && !force_walk;
      // T without a wave reduction when the plan's top intercept decides it (TopHint): the intercepts of lines
      // k >= 1 do not depend on the candidate, so the plan keeps each scalarisation's largest (Plan::itop)
      TopHint hint{false, 0.0, 0.0};
      if (HINT && flat_ok && P->itop != nullptr) {
        double a0 = a_off, b0 = 0.0;
#pragma unroll
        for (int i = 0; i < M; ++i) {
          a0 = fma(wa[i], l0m[i], a0);
          b0 = fma(wb[i], l0v[i], b0);
        }
        const double A1 = hA1;
        const int k1 = hk1, c1 = hc1;
        if (a0 > A1) {
          hint = TopHint{true, a0, b0};
        } else if (a0 < A1 && c1 == 1) {
          // line k1's slope, as the build computes it (record k1 - 1)
          const double* r = lcv + (size_t)(k1 - 1) * MP;
          double bk = 0.0;
          if (full) {
            if constexpr (MP == 1) {
              bk = fma(wb[0], r[0], bk);
            } else {
#pragma unroll
              for (int q = 0; 2 * q < M; ++q) {
                const double2 u = *reinterpret_cast<const double2*>(r + 2 * q);
                bk = fma(wb[2 * q], u.x, bk);
                if (2 * q + 1 < M) bk = fma(wb[2 * q + 1], u.y, bk);
              }
            }
          } else {
            double wbt = 0.0;
#pragma unroll
            for (int i = 0; i < M; ++i) wbt = (i == target) ? wb[i] : wbt;
            bk = wbt * r[target];
          }
          hint = TopHint{true, A1, bk};
        }
      }
      if constexpr (ICP) {
        // intercepts from the plan (first build: the registers loaded ahead; a rebuild: global memory)
        auto slopes = [&](double (&lb)[MAXL]) {
          const double* cvr = lcv + (lane - 1) * MP;
          if (full) {
#pragma unroll
            for (int t = 0; t < MAXL; ++t) {
              double acc = 0.0;  // build_lines' rec_dot of the covariance record
              if constexpr (MP == 1) {
                acc = fma(wb[0], cvr[64 * MP * t], acc);
              } else {
#pragma unroll
                for (int q = 0; 2 * q < M; ++q) {
                  const double2 u = *reinterpret_cast<const double2*>(cvr + 64 * MP * t + 2 * q);
                  acc = fma(wb[2 * q], u.x, acc);
                  if (2 * q + 1 < M) acc = fma(wb[2 * q + 1], u.y, acc);
                }
              }
              lb[t] = acc;
            }
          } else {
            double wbt = 0.0;
#pragma unroll
            for (int i = 0; i < M; ++i) wbt = (i == target) ? wb[i] : wbt;
#pragma unroll
            for (int t = 0; t < MAXL; ++t) lb[t] = wbt * cvr[64 * MP * t + target];
          }
          double a = a_off, bb = 0.0;  // line 0: the candidate itself (discretekg.py:182-183)
#pragma unroll
          for (int i = 0; i < M; ++i) {
            a = fma(wa[i], l0m[i], a);
            bb = fma(wb[i], l0v[i], bb);
          }
          lb[0] = (lane == 0) ? bb : lb[0];
          return a;
        };
        auto first = [&](double (&la)[MAXL], double (&lb)[MAXL]) {
          const double a0 = slopes(lb);
#pragma unroll
          for (int t = 0; t < MAXL; ++t) la[t] = ila[t];
          la[0] = (lane == 0) ? a0 : la[0];
        };
        auto again = [&](double (&la)[MAXL], double (&lb)[MAXL]) {
          const double a0 = slopes(lb);
#pragma unroll
          for (int t = 0; t < MAXL; ++t) la[t] = icp[lane + 64 * t];
          la[0] = (lane == 0) ? a0 : la[0];
        };
        kgj = env_pair_regs<MAXL>(again, NL, lane, sb, sa, sif, force_walk, &hn, nullptr, pst, flat_ok, &first, hint);
      } else {
        // the lines are rebuilt from the staged LDS data if the list walk cannot finish,
        // so no register line is live across it
        auto rebuild = [&](double (&la)[MAXL], double (&lb)[MAXL]) { build_lines(la, lb); };
        kgj = env_pair_regs<MAXL>(rebuild, NL, lane, sb, sa, sif, force_walk, &hn, nullptr, pst, flat_ok,
                                  static_cast<const int*>(nullptr), hint);
      }
    }
    if (pairs_out != nullptr && lane == 0) {
      pairs_out[(size_t)b * S + j] = kgj;
#ifdef DKG_STG_STAMPS
      if constexpr (!GRAD && !STG) P->hull_pairs[(size_t)b * S + j] = hn;  // STG: the list length, above
#else
      if constexpr (!GRAD) P->hull_pairs[(size_t)b * S + j] = hn;
#endif
    }
    if (lane == 0) skg[j - j0] = kgj;
  }

  // ---- mean over S: per-wave sums -> per-WG sum (fixed order) -> across WGs
#ifndef DKG_STG_STAMPS
  if (!GRAD) KST(st, 4);
#endif
  __syncthreads();
#ifndef DKG_STG_STAMPS
  if (!GRAD) KST(st, 5);
#endif
  // The candidate's KG, whatever the launch geometry (waves per workgroup, workgroups per candidate:
  // envelope_geometry), is  sum_g G_g / S  over the groups g of 8 consecutive pairs, G_g the group's pair
  // values summed in pair order, the groups folded in order; dKG/dx likewise.  So a narrow small-batch launch,
  // the fused launch and the wide launch give the same bits:
  //  * a workgroup of 8 waves holds a whole group and sums it from LDS; narrower workgroups (small batches)
  //    leave their pair values in the plan (write-through stores, drained), count themselves into the
  //    group's ticket, and the group's last arriver sums the 8 values in order (write-through loads: no
  //    fence, cdna_hip_programming.md Guideline 16, every handed-off byte sc1);
  //  * one group: the group's sum / S is the result; two groups: each adds its G_g / S onto the zeroed kg[b]
  //    with one atomic (two addends onto 0 commute: the same bits in either order, and no workgroup waits);
  //    more groups, or a pinned host copy to write: the group sums meet in the same ticket form, in order.
  // The tickets and kg / dkg are zeroed by the cross stage of the launch sequence.
  {
    const int ng = (S + 7) >> 3;                 // groups of 8 pairs (a workgroup never spans two)
    const int grp = j0 >> 3;
    const int gpairs = min(8, S - 8 * grp);      // pairs in this workgroup's group
    const int gwgs = (gpairs + SW - 1) / SW;     // workgroups sharing it (1 unless the launch is narrow)
    const size_t prow = (size_t)b * (S + ng);    // wg_part row of candidate b: S pair values, ng group terms
    int* tk = P->tickets + (size_t)b * (ng + 1); // [ng] group tickets, [ng] the candidate's
    __shared__ int s_last;
    const int dg = GRAD ? d : 0;
    // ---- level 1: G_g (thread 0) and, GRAD, its gradient (threads 1 .. d, one coordinate each)
    double gsum = 0.0;
    const int gi = (int)threadIdx.x - 1;  // GRAD coordinate of this thread (threads 1 .. d)
    if (gwgs == 1) {
      if (threadIdx.x == 0)
        for (int q = 0; q < j1 - j0; ++q) gsum += skg[q];
      if (GRAD && gi >= 0 && gi < dg)
        for (int q = 0; q < j1 - j0; ++q) gsum += sgw[q * 64 + 48 + gi];
    } else {
      if (threadIdx.x == 0)
        for (int q = 0; q < j1 - j0; ++q) __hip_atomic_store(&P->wg_part[prow + j0 + q], skg[q], __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_AGENT);
      if (GRAD && gi >= 0 && gi < dg)
        for (int q = 0; q < j1 - j0; ++q)
          __hip_atomic_store(&P->wg_gpart[(prow + j0 + q) * dg + gi], sgw[q * 64 + 48 + gi], __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its write-through stores
      __syncthreads();
      if (threadIdx.x == 0)
        s_last = __hip_atomic_fetch_add(&tk[grp], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gwgs - 1;
      __syncthreads();
      if (s_last) {
        if (threadIdx.x == 0)
          for (int q = 8 * grp; q < 8 * grp + gpairs; ++q)
            gsum += __hip_atomic_load(&P->wg_part[prow + q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (GRAD && gi >= 0 && gi < dg)
          for (int q = 8 * grp; q < 8 * grp + gpairs; ++q)
            gsum += __hip_atomic_load(&P->wg_gpart[(prow + q) * dg + gi], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    const bool holds = (gwgs == 1 || s_last) && (threadIdx.x == 0 || (GRAD && gi >= 0 && gi < dg));
    const double term = gsum / (double)S;
    // where this thread's result goes: kg[b] (thread 0) or dkg[b][gi]; the host copy at the same offsets
    double* dst_dev = threadIdx.x == 0 ? &kg[b] : (GRAD ? &dkg[(size_t)b * d + max(gi, 0)] : &kg[b]);
    const size_t hoff = threadIdx.x == 0 ? (size_t)b : (size_t)B + (size_t)b * d + max(gi, 0);
    // ---- level 2
    const bool fold = ng > 2 || (hout != nullptr && ng > 1);
    if (ng == 1) {
      if (holds) {
        *dst_dev = term;
        if (hout != nullptr) hout[hoff] = term;
      }
    } else if (!fold) {
      if (holds) atomicAdd(dst_dev, term);
    } else if (gwgs == 1 || s_last) {  // workgroup-uniform
      if (holds)
        __hip_atomic_store(threadIdx.x == 0 ? &P->wg_part[prow + S + grp] : &P->wg_gpart[(prow + S + grp) * dg + gi],
                           term, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0)
        s_last = __hip_atomic_fetch_add(&tk[ng], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ng - 1;
      __syncthreads();
      if (s_last && holds) {
        double tot = 0.0;
        for (int q = 0; q < ng; ++q)
          tot += __hip_atomic_load(threadIdx.x == 0 ? &P->wg_part[prow + S + q] : &P->wg_gpart[(prow + S + q) * dg + gi],
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *dst_dev = tot;
        if (hout != nullptr) hout[hoff] = tot;
      }
    }
  }
  if constexpr (HO) {
    // launch done when every envelope workgroup has counted itself: the last re-zeroes the counters
    // for the next launch on this plan (stream-ordered after this one)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned long long prev =
          __hip_atomic_fetch_add(ho->done, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (prev + 1 == ho->quota_done) {
        for (int i = 0; i < P->m * ho->rt; ++i)
          __hip_atomic_store(ho->cnt1 + (size_t)i * HANDOFF_STRIDE, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (int i = 0; i < ho->nrb; ++i)
          __hip_atomic_store(ho->cnt2 + (size_t)i * HANDOFF_STRIDE, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ho->done, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  if (st) __syncthreads();  // workgroup-uniform: the end stamp covers every wave
  KST_END(st);
}

template <int MAXL, int M, bool GRAD, bool STREAM>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(env_waves_per_eu(MAXL, M, GRAD, STREAM)))) void envelope_kernel(const Plan* __restrict__ P, int B, double* __restrict__ kg,
                                                       double* __restrict__ pairs_out, int dst,
                                                       const double* __restrict__ xnew, double* __restrict__ dkg,
                                                       const double* __restrict__ mu_all,
                                                       const double* __restrict__ cov_all,
                                                       const double* __restrict__ var_all,
                                                       const double* __restrict__ mux_all,
                                                       const double* __restrict__ wts,
                                                       const int* __restrict__ dupv, long long cov_stride,
                                                       int bpad, double* __restrict__ hout, int split) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  if (DKG_ABLATIONS && (__builtin_amdgcn_readfirstlane(P->debug_env) & 2)) return;  // ablation: empty envelope stage
  // 1-D grid: the `split` workgroups of one candidate side by side on one XCD (xcd_group), so its line
  // records come from HBM once and from that XCD's L2 for the others
  int b, g;
  if (!xcd_group(blockIdx.x, B, split, b, g)) return;
  envelope_body<MAXL, M, GRAD, STREAM>(P, B, kg, pairs_out, dst, xnew, dkg, mu_all, cov_all, var_all, mux_all, wts,
                                       dupv, cov_stride, bpad, b, g, split, smem, kst_slot(dst, P, 2), nullptr, hout);
}

// The lines of every (candidate, scalarisation) pair of the plan's last
// cross / covariance stages, as the envelope builds them (dkg_plan_lines):
// a_out / b_out [B][S][N + 1], line 0 the candidate itself.  Grid (B, S).
template <int M>
__global__ __launch_bounds__(256) void lines_export_kernel(const Plan* __restrict__ P, double* __restrict__ a_out,
                                                            double* __restrict__ b_out) {
  const int b = blockIdx.x, j = blockIdx.y;
  const int m = P->m, N = P->N, S = P->S, target = P->target, bpad = P->bpad;
  const bool full = target < 0;
  double sv[M], mx0[M], ysd[M], ymu[M], nz[M];
  const int dk = P->dup[b];  // line 0 from that record when x_b coincides with a discretisation point
#pragma unroll
  for (int i = 0; i < M; ++i) {
    const bool live = i < m;
    ysd[i] = live ? P->o[i].y_std : 1.0;
    ymu[i] = live ? P->o[i].y_mean : 0.0;
    nz[i] = live ? P->o[i].noise : 0.0;
    sv[i] = live ? P->var_all[(size_t)i * bpad + b] : 0.0;
    mx0[i] = live ? P->mux_all[(size_t)i * bpad + b] : 0.0;
  }
  double w[M], wa[M], wb[M];
  double a_off, den;
  pair_coefs<M>(P->weights + (size_t)j * m, m, full, target, ysd, ymu, nz, sv, w, wa, wb, a_off, den);
  (void)den;
  double* ao = a_out + ((size_t)b * S + j) * (N + 1);
  double* bo = b_out + ((size_t)b * S + j) * (N + 1);
  for (int k = threadIdx.x; k <= N; k += blockDim.x) {
    double a = a_off, bb = 0.0;
    if (k == 0 && dk == DUP_NONE) {
#pragma unroll
      for (int i = 0; i < M; ++i) {
        a = fma(wa[i], mx0[i], a);
        bb = fma(wb[i], sv[i], bb);
      }
    } else {
      const int r = (k == 0) ? dk : k - 1;  // the record line k is built from (line 0: the coincident one)
#pragma unroll
      for (int i = 0; i < M; ++i) {
        if (i < m) {
          a = fma(wa[i], P->mu_all[(size_t)r * cov_rec(M) + i], a);
          if (full) bb = fma(wb[i], P->cov_all[(size_t)b * P->cov_stride + (size_t)r * cov_rec(M) + i], bb);
        }
      }
      if (!full) {
        double wbt = 0.0;
#pragma unroll
        for (int i = 0; i < M; ++i) wbt = (i == target) ? wb[i] : wbt;
        bb = wbt * P->cov_all[(size_t)b * P->cov_stride + (size_t)r * cov_rec(M) + target];
      }
    }
    ao[k] = a;
    bo[k] = bb;
  }
}

struct EnvLaunch {
  const Plan* host;
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
  double* hout;        // GRAD: pinned host [kg | dkg] (dkg_plan_forward_grad_hostx), nullable
};

template <int MAXL, int M, bool GRAD, bool STREAM>
hipError_t launch_env_t(const EnvLaunch& a) {
  raise_lds_limit((const void*)envelope_kernel<MAXL, M, GRAD, STREAM>, a.lds);
  const Plan& h = *a.host;
  hipLaunchKernelGGL((envelope_kernel<MAXL, M, GRAD, STREAM>), a.grid, a.block, a.lds, a.s, a.dev, a.B, a.kg, a.pairs,
                     a.dst, a.xnew, a.dkg, h.mu_all, h.cov_all, h.var_all, h.mux_all, h.weights, h.dup,
                     (long long)h.cov_stride, h.bpad, a.hout, h.split);
  return hipGetLastError();
}


// One output bucket M: picks the line-slot instantiation (MAXL) or the
// streaming kernel.  Defined in dkg_env_m<M>.hip (one translation unit per
// bucket, compiled in parallel).
template <int M, bool GRAD>
hipError_t launch_env_bucket(int lines, bool stream, const EnvLaunch& a) {
  if (stream) return launch_env_t<STREAM_CHUNK, M, GRAD, true>(a);
  if (lines <= 64 * 2) return launch_env_t<2, M, GRAD, false>(a);
  if (lines <= 64 * 8) return launch_env_t<8, M, GRAD, false>(a);
  if (lines <= 64 * 17) return launch_env_t<17, M, GRAD, false>(a);
  if (lines <= 64 * 33) return launch_env_t<33, M, GRAD, false>(a);
  return hipErrorInvalidValue;
}

// Per-bucket launchers (dkg_env_m<M>.hip).
hipError_t launch_env_m1(bool grad, int lines, bool stream, const EnvLaunch& a);
hipError_t launch_env_m2(bool grad, int lines, bool stream, const EnvLaunch& a);
hipError_t launch_env_m3(bool grad, int lines, bool stream, const EnvLaunch& a);
hipError_t launch_env_m4(bool grad, int lines, bool stream, const EnvLaunch& a);
hipError_t launch_env_m8(bool grad, int lines, bool stream, const EnvLaunch& a);

}  // namespace dkg
