// The reference's epigraph walk, exactly (calculate_epigraph_indices,
// discretekg.py:341-412), as wave-level device code for gfx950.
//
// The reference sorts the lines by slope ascending, then intercept descending
// (:370-374), starts from the first line and repeatedly jumps to the later
// line with a different slope whose intersection
//     x = -(a_cur - a_j) / (b_cur - b_j)                           (:388-396)
// comes first; torch.argmin takes the first index among equal x, i.e. the
// smallest slope, then the largest intercept, then (sorts taken stable) the
// smallest line index.  Here a step is an argmin over the candidate lines of
// the key (x, b, -a, k), with x computed by the same IEEE operations: the
// numerator a_cur - a_j and the denominator b_j - b_cur are the reference's
// operands up to sign (exact), and the division is correctly rounded, so x is
// bit-identical to the reference's and the walk visits the same lines in the
// same order — concurrent lines at a breakpoint included (a zero-length
// envelope segment in exact arithmetic, kept by the reference's argmin-first
// rule).
//
// The walk runs over a candidate list rather than all N+1 lines: the lines on
// or above the chords L-T and T-R less a margin (EnvChords).  A line below a
// chord by more than the margin is below the upper hull by at least as much;
// it can win a rounded argmin step only where the step's intersection exceeds
// WALK_XGUARD in magnitude (derivation in DESIGN.md 4.3), so a walk whose
// breakpoints all stay within WALK_XGUARD is the reference's walk over all
// lines.  A walk that leaves it is redone over all lines (walk_regs /
// walk_stream), as is a list that overflows.
#pragma once

#include "dkg_common.h"

namespace dkg {

constexpr int KEY_NONE = 0x7fffffff;
// Relative chord margin 2^-20 (EnvChords) and the breakpoint bound under which
// the list walk is provably the full walk: 2^30 < 2^33 / 6.
constexpr double WALK_MARGIN = 9.5367431640625e-07;    // 2^-20
constexpr double WALK_XGUARD = 1073741824.0;           // 2^30
// The guard for a relative margin rel is rel * 2^50 (the same derivation:
// rel (1 - 3u) / (6u) > rel * 2^50 with u = 2^-53).  A list walk whose largest
// breakpoint leaves the first guard is redone over a list filtered with the
// margin WALK_REFILTER * (that breakpoint) * 2^-50, whose guard is then
// WALK_REFILTER times the breakpoint; the walk over all lines runs only when
// that margin would reach WALK_REL_MAX (the filter would keep most lines).
constexpr double WALK_POW2_50 = 1125899906842624.0;    // 2^50
constexpr double WALK_REFILTER = 16.0;
constexpr double WALK_REL_MAX = 0.00390625;            // 2^-8
// A list that overflows at WALK_MARGIN is filtered again at the tight margin
// 2^-30 (guard 2^20) before the walk over all lines is considered.
constexpr double WALK_MARGIN_TIGHT = 9.313225746154785e-10;  // 2^-30

// psi(c) = E[(Z - c)_+] with the far tail cut to its fp64 value (0 beyond
// c = 40: exp(-800) underflows), so an infinite breakpoint gives 0, not NaN.
__device__ __forceinline__ double psi_edge(double c) { return c > 40.0 ? 0.0 : psi(c); }

// Walk order of candidate successors: intersection, then the reference's sort
// order (slope ascending, intercept descending, index ascending).
__device__ __forceinline__ bool walk_less(double x1, double b1, double a1, int k1, double x2, double b2, double a2,
                                          int k2) {
  return x1 < x2 || (x1 == x2 && (b1 < b2 || (b1 == b2 && (a1 > a2 || (a1 == a2 && k1 < k2)))));
}

struct WalkPick {
  double x, b, a;
  int k;
};

// Wave argmin of the walk key; lanes without a candidate hold
// (+inf, +inf, -inf, KEY_NONE), which every candidate beats.  The common case
// is one lane at the minimal x; ties fall through to the sort keys.
__device__ __forceinline__ WalkPick wave_walk_min(double x, double b, double a, int k) {
  double xm = x;
  DKG_BUTTERFLY_ROW({ xm = fmin_raw(xm, partner_f64<S_>(xm)); })
  xm = combine_rows(xm, [](double p, double q) { return fmin(p, q); });
  const uint64_t tie = ballot(x == xm);
  WalkPick r;
  r.x = xm;
  if (__popcll(tie) == 1) {
    const int w = __builtin_ctzll(tie);
    r.b = readlane_f64(b, w);
    r.a = readlane_f64(a, w);
    r.k = __builtin_amdgcn_readlane(k, w);
    return r;
  }
  const bool t0 = x == xm;
  double bm = t0 ? b : INFINITY;
  DKG_BUTTERFLY_ROW({ bm = fmin_raw(bm, partner_f64<S_>(bm)); })
  bm = combine_rows(bm, [](double p, double q) { return fmin(p, q); });
  const bool t1 = t0 && b == bm;
  double am = t1 ? a : -INFINITY;
  DKG_BUTTERFLY_ROW({ am = fmax_raw(am, partner_f64<S_>(am)); })
  am = combine_rows(am, [](double p, double q) { return fmax(p, q); });
  const bool t2 = t1 && a == am;
  r.b = bm;
  r.a = am;
  r.k = wave_min_i32(t2 ? k : KEY_NONE);
  return r;
}

// Optional per-pair epigraph output (dkg_epigraph): indices [cap] (left to
// right) and intersections [cap - 1]; entries beyond cap are counted, not written.
struct WalkOut {
  long long* idx;
  double* x;
  int cap;
};

// After the accepted walk of h lines: indices h .. cap-1 = -1 and intersections h-1 .. cap-2 = NaN (a list
// walk rejected for a breakpoint beyond its guard, and redone, may have written past the final count).
__device__ __forceinline__ void pad_walk_out(const WalkOut& out, int h, int lane) {
  for (int e = h + lane; e < out.cap; e += 64) out.idx[e] = -1;
  for (int e = (h > 0 ? h - 1 : 0) + lane; e < out.cap - 1; e += 64) out.x[e] = __builtin_nan("");
}

// The KG edge terms a walk leaves for the single psi evaluation of its caller
// (finish_edges): `kg` is the part already summed (walks of more than 64
// steps flush every 64), and each lane with `on` holds one pending edge
// (b_Q - b_P, +-c).  One psi site per kernel: its exp / erfc coefficients
// are materialised once, not per walk variant.
struct EdgeSum {
  double kg, ec, ed;
  bool on;
};

__device__ __forceinline__ double finish_edges(const EdgeSum& e) {
  // every pending edge beyond psi_edge's cut: its term is exactly 0 (skip exp / erfc)
  if (ballot(e.on && e.ec <= 40.0) == 0) return e.kg;
  return e.kg + wave_sum(e.on ? e.ed * psi_edge(e.ec) : 0.0);
}

// Per-step bookkeeping shared by the walks: the KG edge terms
// (b_Q - b_P) psi(+-c) (minus sign for edges ending at or left of T), one
// edge per lane, flushed by a wave sum every 64 steps; the largest |c|; and
// the optional epigraph output.
struct WalkAcc {
  double ec = 0.0, ed = 0.0, kg = 0.0, cmax = 0.0;
  int h = 0;  // steps taken (envelope lines - 1)

  __device__ __forceinline__ void start(int k0, int lane, const WalkOut* out) {
    if (out && lane == 0 && out->cap > 0) out->idx[0] = k0;
  }
  __device__ __forceinline__ void step(const WalkPick& p, double bc, double bT, int lane, const WalkOut* out) {
    if (lane == (h & 63)) {
      ec = (p.b <= bT) ? -p.x : p.x;
      ed = p.b - bc;
    }
    cmax = fmax(cmax, fabs(p.x));
    if (out && lane == 0 && h + 1 < out->cap) {
      out->idx[h + 1] = p.k;
      out->x[h] = p.x;
    }
    ++h;
    if ((h & 63) == 0) {
      kg += wave_sum(ed * psi_edge(ec));
      ec = 0.0;
      ed = 0.0;
    }
  }
  __device__ __forceinline__ EdgeSum pending(int lane) const { return {kg, ec, ed, lane < (h & 63)}; }
};

// Chords L-T and T-R of the candidate filter with the margin: a line (a, b)
// is kept iff fma(-s, b, a) >= K for either chord, s = da / db its slope in
// the (b, a) plane and K = fma(-s, b0, a0) - tau with
// tau = rel (max|a_end| + |s| (max|b_end| + Wb) + Wb), Wb = b_R - b_L: the
// margin is at least rel Wb in intercept units, and the rounding of the test
// itself (a few ulps of |a| + |s b|, and of s db against da) is far inside it.
// Exact copies of the chord ends evaluate to at least K, so L, T, R and their
// duplicates are always kept.  A degenerate chord (db = 0) keeps nothing.
struct EnvChords {
  double s1, k1, s2, k2;
};

__device__ __forceinline__ EnvChords env_chords(double bL, double aL, double bT, double aT, double bR, double aR,
                                                double rel = WALK_MARGIN) {
  EnvChords c;
  const double Wb = bR - bL;
  const double db1 = bT - bL, db2 = bR - bT;
  c.s1 = (db1 > 0.0) ? (aT - aL) / db1 : 0.0;
  c.s2 = (db2 > 0.0) ? (aR - aT) / db2 : 0.0;
  const double t1 = rel * (fmax(fabs(aL), fabs(aT)) + fabs(c.s1) * (fmax(fabs(bL), fabs(bT)) + Wb) + Wb);
  const double t2 = rel * (fmax(fabs(aT), fabs(aR)) + fabs(c.s2) * (fmax(fabs(bT), fabs(bR)) + Wb) + Wb);
  c.k1 = (db1 > 0.0) ? fma(-c.s1, bL, aL) - t1 : INFINITY;
  c.k2 = (db2 > 0.0) ? fma(-c.s2, bT, aT) - t2 : INFINITY;
  return c;
}

__device__ __forceinline__ bool env_keep(const EnvChords& c, double a, double b) {
  return fma(-c.s1, b, a) >= c.k1 || fma(-c.s2, b, a) >= c.k2;
}

// The wave's keep mask: the two compares' lane masks OR-ed (no VGPR round trip).
__device__ __forceinline__ uint64_t env_keep_mask(const EnvChords& c, double a, double b) {
  return ballot(fma(-c.s1, b, a) >= c.k1) | ballot(fma(-c.s2, b, a) >= c.k2);
}

// Exact walk over the candidate list (sb, sa, si; nc <= 64 PL entries) from
// the lowest-index copy of L = (bL, aL).  Returns the edge terms (EdgeSum: KG_w after finish_edges, the cancellation-free edge
// sum); *nhull = envelope lines; *cmax = largest |breakpoint| (the caller
// checks it against WALK_XGUARD).
template <int PL>
__device__ __forceinline__ EdgeSum walk_list(int nc, int lane, const double* sb, const double* sa, const int* si,
                                            double bL, double aL, double bT, int* nhull, double* cmax,
                                            const WalkOut* out = nullptr) {
  double eb[PL], ea[PL];
  int ek[PL];
#pragma unroll
  for (int q = 0; q < PL; ++q) {
    const int e = lane + 64 * q;
    const int ee = min(e, max(nc - 1, 0));
    const bool v = e < nc;
    eb[q] = v ? sb[ee] : -INFINITY;  // never a successor, never the start
    ea[q] = sa[ee];
    ek[q] = v ? si[ee] : KEY_NONE;
  }
  int ks = KEY_NONE;
#pragma unroll
  for (int q = 0; q < PL; ++q) ks = (eb[q] == bL && ea[q] == aL) ? min(ks, ek[q]) : ks;
  ks = wave_min_i32(ks);
  WalkAcc acc;
  acc.start(ks, lane, out);
  double bc = bL, ac = aL;
  for (int guard = 0; guard < nc; ++guard) {
    double xb = INFINITY, bb = INFINITY, ab = -INFINITY;
    int kb = KEY_NONE;
#pragma unroll
    for (int q = 0; q < PL; ++q) {
      if (eb[q] > bc) {
        const double x = (ac - ea[q]) / (eb[q] - bc);
        if (walk_less(x, eb[q], ea[q], ek[q], xb, bb, ab, kb)) {
          xb = x; bb = eb[q]; ab = ea[q]; kb = ek[q];
        }
      }
    }
    if (ballot(kb != KEY_NONE) == 0) break;
    const WalkPick p = wave_walk_min(xb, bb, ab, kb);
    acc.step(p, bc, bT, lane, out);
    bc = p.b;
    ac = p.a;
  }
  *nhull = acc.h + 1;
  *cmax = acc.cmax;
  return acc.pending(lane);
}

// Exact walk over a short candidate list (nc <= R <= 32 entries) by a
// successor table: row i (lanes G i .. G i + G - 1, G = 64 / R) evaluates the
// walk step from entry i over its share j = g + G q (q < R / G) of the list,
// keeps the lane's best under the walk key, and a DPP minimum over the row's
// lanes gives the row's best intersection.  Every entry's successor is so
// known at once; the walk is then a chase of row winners by scalar mask
// operations and one v_readlane per step (the reference's sequence of argmin
// steps, :382-401, each step's argmin being exactly the row's).  A row whose
// minimum is attained by several lanes (concurrent lines, duplicates) is
// resolved by the full key over those lanes (wave_walk_min).  The KG edge
// terms are left on the winning lanes (EdgeSum, evaluated by finish_edges);
// *cmax = 0 when every breakpoint is within WALK_XGUARD, else the largest
// |breakpoint|.
template <int R>
__device__ __forceinline__ EdgeSum walk_table(int nc, int lane, const double* sb, const double* sa, const int* si,
                                             double bL, double aL, double bT, int* nhull, double* cmax,
                                             const WalkOut* out = nullptr) {
  constexpr int G = 64 / R, JL = R / G;
  // the row / column split of the lane index inside this instantiation (an opaque copy of the lane:
  // not hoisted and shared across the table sizes, which would keep their addresses live)
  int ln = lane;
  asm volatile("" : "+v"(ln));
  const int i = ln / G, g = ln % G;
  const int ii = min(i, nc - 1);
  const double bi = sb[ii], ai = sa[ii];
  // the lane's share in chunks of up to four entries, each chunk's loads first (one LDS round trip per
  // chunk, few registers)
  constexpr int CH = JL < 4 ? JL : 4;
  double xb = INFINITY, bb = INFINITY, ab = -INFINITY;
  int kb = KEY_NONE, jb = -1;
  // only the chunks that hold list entries (a 17-entry list in the 32-row table: 3 of 4 chunks)
  const int jl = min(JL, (nc + G - 1) / G);
#pragma unroll 1
  for (int q0 = 0; q0 < jl; q0 += CH) {
    double ebj[CH], eaj[CH];
    int ekj[CH];
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      int jj = min(g + G * (q0 + u), nc - 1);
      ebj[u] = sb[jj];
      eaj[u] = sa[jj];
      ekj[u] = si[jj];
    }
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const int j = g + G * (q0 + u);
      const double bj = ebj[u], aj = eaj[u];
      const int kj = ekj[u];
      const double x = (ai - aj) / (bj - bi);
      if (j < nc && bj > bi && walk_less(x, bj, aj, kj, xb, bb, ab, kb)) {
        xb = x; bb = bj; ab = aj; kb = kj; jb = j;
      }
    }
  }
  double xm = xb;
  if constexpr (G >= 2) xm = fmin_raw(xm, dpp_f64<0xB1>(xm));
  if constexpr (G >= 4) xm = fmin_raw(xm, dpp_f64<0x4E>(xm));
  if constexpr (G >= 8) xm = fmin_raw(xm, dpp_f64<0x141>(xm));
  const uint64_t hits = ballot(i < nc && jb >= 0 && xb == xm);
  // start: the first list position holding L (the list is in line-index order)
  const uint64_t lead = ballot(g == 0 && i < nc && bi == bL && ai == aL);
  int cur = (int)__builtin_ctzll(lead) / G;
  if (out && lane == 0 && out->cap > 0) out->idx[0] = si[cur];
  uint64_t win = 0;
  int h = 0;
  constexpr uint64_t ROW = (G == 64) ? ~0ull : ((1ull << G) - 1);
  for (int guard = 0; guard < nc; ++guard) {
    const uint64_t rm = hits & (ROW << (cur * G));
    if (rm == 0) break;
    int w = (int)__builtin_ctzll(rm);
    if (__popcll(rm) > 1) {  // several lanes at the row minimum: the full key decides
      const bool sel = (rm >> lane) & 1;
      const WalkPick p = wave_walk_min(sel ? xb : INFINITY, sel ? bb : INFINITY, sel ? ab : -INFINITY,
                                       sel ? kb : KEY_NONE);
      w = (int)__builtin_ctzll(ballot(sel && kb == p.k));
    }
    win |= 1ull << w;
    if (out && h + 1 < out->cap) {
      const int kw = __builtin_amdgcn_readlane(kb, w);
      const double xw = readlane_f64(xb, w);
      if (lane == 0) {
        out->idx[h + 1] = kw;
        out->x[h] = xw;
      }
    }
    cur = __builtin_amdgcn_readlane(jb, w);
    ++h;
  }
  const bool won = (win >> lane) & 1;
  *nhull = h + 1;
  *cmax = (ballot(won && !(fabs(xb) <= WALK_XGUARD)) != 0) ? wave_max(won ? fabs(xb) : 0.0) : 0.0;
  return {0.0, (bb <= bT) ? -xb : xb, bb - bi, won};
}

// Walk over the candidate list: the successor table up to 32 entries, the
// step-by-step argmin walk beyond (PL list entries per lane).
__device__ __forceinline__ EdgeSum walk_small(int nc, int lane, const double* sb, const double* sa, const int* si,
                                             double bL, double aL, double bT, int* nhull, double* cmax,
                                             const WalkOut* out = nullptr) {
  if (nc <= 8) return walk_table<8>(nc, lane, sb, sa, si, bL, aL, bT, nhull, cmax, out);
  if (nc <= 16) return walk_table<16>(nc, lane, sb, sa, si, bL, aL, bT, nhull, cmax, out);
  if (nc <= 32) return walk_table<32>(nc, lane, sb, sa, si, bL, aL, bT, nhull, cmax, out);
  if (nc <= 64) return walk_list<1>(nc, lane, sb, sa, si, bL, aL, bT, nhull, cmax, out);
  return walk_list<2>(nc, lane, sb, sa, si, bL, aL, bT, nhull, cmax, out);
}

// Exact walk over all register lines (line k = lane + 64 t, k < nl).
template <int MAXL>
__device__ __forceinline__ EdgeSum walk_regs(const double (&la)[MAXL], const double (&lb)[MAXL], int nl, int lane,
                                            double bL, double aL, double bT, int* nhull,
                                            const WalkOut* out = nullptr) {
  int ks = KEY_NONE;
#pragma unroll
  for (int t = MAXL - 1; t >= 0; --t) ks = (lane + 64 * t < nl && lb[t] == bL && la[t] == aL) ? lane + 64 * t : ks;
  ks = wave_min_i32(ks);
  WalkAcc acc;
  acc.start(ks, lane, out);
  double bc = bL, ac = aL;
  for (int guard = 0; guard < nl; ++guard) {
    double xb = INFINITY, bb = INFINITY, ab = -INFINITY;
    int kb = KEY_NONE;
#pragma unroll
    for (int t = 0; t < MAXL; ++t) {
      const int k = lane + 64 * t;
      if (k < nl && lb[t] > bc) {
        const double x = (ac - la[t]) / (lb[t] - bc);
        if (walk_less(x, lb[t], la[t], k, xb, bb, ab, kb)) {
          xb = x; bb = lb[t]; ab = la[t]; kb = k;
        }
      }
    }
    if (ballot(kb != KEY_NONE) == 0) break;
    const WalkPick p = wave_walk_min(xb, bb, ab, kb);
    acc.step(p, bc, bT, lane, out);
    bc = p.b;
    ac = p.a;
  }
  *nhull = acc.h + 1;
  return acc.pending(lane);
}

// Exact walk over streamed lines: build(c, la, lb) rebuilds chunk c (line
// k = c * 64 * MAXL + lane + 64 t) every step.
template <int MAXL, class Build>
__device__ __forceinline__ EdgeSum walk_stream(int nch, int nl, int lane, double bL, double aL, double bT, int* nhull,
                                              Build&& build, const WalkOut* out = nullptr) {
  int ks = KEY_NONE;
  for (int c = nch - 1; c >= 0; --c) {
    double la[MAXL], lb[MAXL];
    build(c, la, lb);
#pragma unroll
    for (int t = MAXL - 1; t >= 0; --t) {
      const int k = c * 64 * MAXL + lane + 64 * t;
      ks = (k < nl && lb[t] == bL && la[t] == aL) ? k : ks;
    }
  }
  ks = wave_min_i32(ks);
  WalkAcc acc;
  acc.start(ks, lane, out);
  double bc = bL, ac = aL;
  for (int guard = 0; guard < nl; ++guard) {
    double xb = INFINITY, bb = INFINITY, ab = -INFINITY;
    int kb = KEY_NONE;
    for (int c = 0; c < nch; ++c) {
      double la[MAXL], lb[MAXL];
      build(c, la, lb);
#pragma unroll
      for (int t = 0; t < MAXL; ++t) {
        const int k = c * 64 * MAXL + lane + 64 * t;
        if (k < nl && lb[t] > bc) {
          const double x = (ac - la[t]) / (lb[t] - bc);
          if (walk_less(x, lb[t], la[t], k, xb, bb, ab, kb)) {
            xb = x; bb = lb[t]; ab = la[t]; kb = k;
          }
        }
      }
    }
    if (ballot(kb != KEY_NONE) == 0) break;
    const WalkPick p = wave_walk_min(xb, bb, ab, kb);
    acc.step(p, bc, bT, lane, out);
    bc = p.b;
    ac = p.a;
  }
  *nhull = acc.h + 1;
  return acc.pending(lane);
}

}  // namespace dkg
