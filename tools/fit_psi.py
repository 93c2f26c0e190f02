"""Rational approximations of psi(x) = E[(Z - x)_+] = phi(x) g(x), x >= 0 (dkg_common.h psi).

g(x) = 1 - x Q(x) / phi(x) (one minus x times the Mills ratio) is smooth and decays like 1/x^2:
  x in [0, 4]:   g = PA(v) / QA(v),        v = x / 4,                    degree 8 / 8
  x in [4, 40]:  g = s PB(u) / QB(u),      s = 1 / x^2, u = (s - 1/1600) / (1/16 - 1/1600), degree 6 / 6
Linearized rational least squares (iteratively reweighted, QA(0) = QB(0) = 1) at 60 digits with
mpmath, coefficients rounded to double; prints them as C arrays and the worst relative error of
the double-precision Horner evaluation on 3000 points per range (each about 5e-16).
Run: python tools/fit_psi.py  (about a minute)
"""
import mpmath as mp

mp.mp.dps = 60
SQ2PI = mp.sqrt(2 * mp.pi)


def gfun(x):
    x = mp.mpf(x)
    return 1 - x * (mp.erfc(x / mp.sqrt(2)) / 2) / (mp.exp(-x * x / 2) / SQ2PI)


def ratfit(f, a, b, n, m, npts, iters=8):
    xs = [a + (b - a) * (1 - mp.cos(mp.pi * (k + 0.5) / npts)) / 2 for k in range(npts)]
    vs = [(x - a) / (b - a) for x in xs]
    fs = [f(x) for x in xs]
    w = [mp.mpf(1)] * npts
    for _ in range(iters):
        A = mp.matrix(npts, n + 1 + m)
        rhs = mp.matrix(npts, 1)
        for i in range(npts):
            W = w[i] / abs(fs[i])
            for j in range(n + 1):
                A[i, j] = W * vs[i] ** j
            for j in range(1, m + 1):
                A[i, n + j] = -W * fs[i] * vs[i] ** j
            rhs[i] = W * fs[i]
        sol = mp.qr_solve(A, rhs)[0]
        p = [sol[j] for j in range(n + 1)]
        q = [mp.mpf(1)] + [sol[n + j] for j in range(1, m + 1)]
        w = [1 / abs(mp.polyval(q[::-1], v)) for v in vs]
    pd, qd = [float(c) for c in p], [float(c) for c in q]
    worst = 0
    for k in range(3000):
        x = a + (b - a) * mp.mpf(k) / 2999
        v = float((x - a) / (b - a))
        P = 0.0
        for c in reversed(pd):
            P = P * v + c
        Qv = 0.0
        for c in reversed(qd):
            Qv = Qv * v + c
        worst = max(worst, abs(mp.mpf(P / Qv) / f(x) - 1))
    return pd, qd, float(worst)


def carr(name, c):
    return f"constexpr double {name}[{len(c)}] = {{" + ", ".join(repr(v) for v in c) + "};"


if __name__ == "__main__":
    pa, qa, ea = ratfit(gfun, mp.mpf(0), mp.mpf(4), 8, 8, 200)
    pb, qb, eb = ratfit(lambda s: gfun(1 / mp.sqrt(s)) / s, mp.mpf(1) / 1600, mp.mpf(1) / 16, 6, 6, 150)
    print(f"// range A [0, 4]: worst relative error {ea:.2e}; range B [4, 40]: {eb:.2e}")
    for name, c in (("PSI_PA", pa), ("PSI_QA", qa), ("PSI_PB", pb), ("PSI_QB", qb)):
        print(carr(name, c))
