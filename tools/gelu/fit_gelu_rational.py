"""Fit the round-6 GELU core: t(x) = tanh(u(x)), u = sqrt(2/pi) (x + 0.044715 x^3) (the reference's
jax.nn.gelu(approximate=True), gnn_layers.py:354/386/412), as ONE rational in x,

    t(x) ~= x P(x^2) / Q(x^2),  Q(0) = 1,  |x| clamped to X,

minimax in relative error on [0, X] (LP on a dense grid in s = x^2 / X^2), then the coefficients
rounded to float32 (Q's first, then P refitted against the rounded Q, then rounded). The XLA form
evaluates u first and a [13/6] rational in u (22 issue slots per packed pair); this one skips u and
needs degree (5, 4) in x^2: 19 slots. Prints the float32 coefficients as C literals.

    python tools/gelu/fit_gelu_rational.py [--m 5] [--n 4] [--X 5.05]
"""
import argparse

import numpy as np
from scipy.optimize import linprog

K0 = np.sqrt(2.0 / np.pi)
K1 = 0.044715


def f(x):
    return np.tanh(K0 * (x + K1 * x ** 3))


P0 = float(np.float32(K0))  # x P(x^2) ~ sqrt(2/pi) x near 0: P(0) pinned to float32(sqrt(2/pi))


def lp(x, t, s, m, n, e, q_fixed=None):
    # unknowns: P's coefficients 1..m (P(0) = P0 fixed), Q's 1..n (Q(0) = 1) or none of Q (q_fixed)
    Sp = np.stack([s ** k for k in range(1, m + 1)], 1) * (x / t)[:, None]
    c0 = P0 * (x / t)
    if q_fixed is None:
        Sq = np.stack([s ** k for k in range(1, n + 1)], 1)
        A1 = np.hstack([Sp, -(1 + e) * Sq])
        A2 = np.hstack([-Sp, (1 - e) * Sq])
        B1 = np.full(len(x), 1 + e) - c0
        B2 = np.full(len(x), -(1 - e)) + c0
        nv = m + n
    else:
        Q = np.polyval(q_fixed[::-1], s)
        A1, A2 = Sp, -Sp
        B1, B2 = (1 + e) * Q - c0, -(1 - e) * Q + c0
        nv = m
    r = linprog(np.zeros(nv), A_ub=np.vstack([A1, A2]), b_ub=np.concatenate([B1, B2]), bounds=[(None, None)] * nv,
                method="highs", options={"primal_feasibility_tolerance": 1e-10, "dual_feasibility_tolerance": 1e-10})
    return r.x if r.status == 0 else None


def minimax(x, t, s, m, n, q_fixed=None):
    lo, hi, best = 1e-11, 1e-3, None
    for _ in range(28):
        mid = np.sqrt(lo * hi)
        r = lp(x, t, s, m, n, mid, q_fixed)
        if r is not None:
            hi, best = mid, r
        else:
            lo = mid
    return hi, best


def fma32(a, b, c):
    return np.float32(np.float64(a) * np.float64(b) + np.float64(c))


def eval32(x, P, Q):
    """t(x) in the kernels' float32 sequence (Horner fmas, x*p, IEEE quotient)."""
    x = np.float32(x)
    s = (x * x).astype(np.float32)
    q = fma32(s, np.float32(Q[-1]), np.float32(Q[-2]))
    for c in Q[-3::-1]:
        q = fma32(s, q, np.float32(c))
    p = fma32(s, np.float32(P[-1]), np.float32(P[-2]))
    for c in P[-3::-1]:
        p = fma32(s, p, np.float32(c))
    p = (x * p).astype(np.float32)
    return (p.astype(np.float64) / q.astype(np.float64)).astype(np.float32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=5)
    ap.add_argument("--n", type=int, default=4)
    ap.add_argument("--X", type=float, default=5.05)
    a = ap.parse_args()
    X = a.X
    x = np.linspace(1e-4, X, 3000)
    t = f(x)
    s = (x / X) ** 2
    e, sol = minimax(x, t, s, a.m, a.n)
    P = np.concatenate([[P0], sol[:a.m]]) / X ** (2 * np.arange(a.m + 1))
    Q = np.concatenate([[1.0], sol[a.m:]]) / X ** (2 * np.arange(a.n + 1))
    Q32 = Q.astype(np.float32).astype(np.float64)
    # refit P against the rounded Q (linear in P), in the scaled variable
    e2, solp = minimax(x, t, s, a.m, a.n, q_fixed=Q32 * X ** (2 * np.arange(a.n + 1)))
    P32 = (np.concatenate([[P0], solp]) / X ** (2 * np.arange(a.m + 1))).astype(np.float32).astype(np.float64)
    xx = np.linspace(0, X, 400001)[1:]
    got = eval32(xx, P32, Q32).astype(np.float64)
    rel = np.abs(got / f(xx) - 1)
    print(f"(m, n) = ({a.m}, {a.n}), X = {X}: minimax rel err {e:.3e} (exact coefficients), {e2:.3e} (P refit on "
          f"float32 Q); float32 evaluation on a 4e5 grid: max rel err {rel.max():.3e}; 1 - f(X) = {1 - f(X):.3e}")
    print("P (x^0 .. x^2m of x P(x^2)):", ", ".join(f"{v:.9e}f" for v in np.float32(P32)))
    # the clamp: the first float32 x from X/2 up whose float32 t(x) is exactly 1.0f (as XLA's
    # 7.99881172 is for its rational), so |x| beyond it gives 2g = 2x or 0 exactly
    lo = np.float32(X / 2).view(np.uint32)
    grid = np.arange(lo, np.float32(X + 1).view(np.uint32), dtype=np.uint32).view(np.float32)
    tv = eval32(grid, P32, Q32)
    hit = np.nonzero(tv >= np.float32(1.0))[0]
    if len(hit):
        X = float(grid[hit[0]])
        print(f"float32 t(x) first reaches 1.0f at x = {X!r}; max t below it {float(tv[:hit[0]].max())!r}")
    else:
        print("float32 t(x) never reaches 1.0f below X + 1")
    print("Q (x^0 .. x^2n):", ", ".join(f"{v:.9e}f" for v in np.float32(Q32)))
    print("clamp X =", repr(float(np.float32(X))))
    return X


if __name__ == "__main__":
    main()
