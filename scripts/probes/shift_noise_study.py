"""FD noise of the walks' diagonal shift in the high-norm regime (CPU study; oracle restatement
with its exponential swapped).

The C3 problem (d = 9, four error sources) at N_t = 1 ... 256 (max step |A|_1 = 84 ... 0.33) is
evaluated by oracle.grape_oracle with its exp! replaced by
  ref      an extended-precision (longdouble) Taylor exponential rounded to double (the yardstick),
  julia    Julia's exp! (the oracle's own, Pade 13 above |A|_1 = 5.4),
  noshift  Taylor 30 of A / 2^s, s = ceil(log2(|A|_1 / 3.2)), s squarings (the walks at high norm),
  shift    the same of A - i mu I (mu the midpoint of the diagonal's imaginary parts, on a 1/16 grid
           so that the eps-variants of a step share it) times e^{i mu},
  lowonly  shift only when |A - i mu I|_1 <= 0.25 (the walks' rule since round 4; here on the whole
           9 x 9 matrix, the walks decide per sector),
and the max errors of F_dx, F_d2err and F_d2err_dx against `ref` are printed (4 seeds per N_t).
Usage: python scripts/probes/shift_noise_study.py [N_t ...]   (default 1 2 4 8 16 32 64 256)"""
import sys
from math import ceil, factorial, log2

import numpy as np

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from oracle import grape_oracle as O  # noqa: E402
from tests import problems as P  # noqa: E402


def ref_exp(A):
    A = np.asarray(A, complex).astype(np.clongdouble)
    n = float(np.max(np.sum(np.abs(A), axis=0)))
    s = max(0, int(ceil(log2(n / 0.05)))) if n > 0.05 else 0
    X = A / (2 ** s)
    E = np.eye(A.shape[0], dtype=np.clongdouble)
    T = E.copy()
    for k in range(1, 30):
        T = T @ X / k
        E = E + T
    for _ in range(s):
        E = E @ E
    return E.astype(np.complex128)


def taylor_ps(A, m):
    d = A.shape[0]
    eye = np.eye(d, dtype=complex)
    A2 = A @ A
    A3 = A2 @ A
    c = [1.0 / factorial(k) for k in range(m + 1)]
    X = c[m - 3] * eye + c[m - 2] * A + c[m - 1] * A2 + c[m] * A3
    for st in range((m - 3) // 3 - 1, -1, -1):
        X = A3 @ X + (c[3 * st] * eye + c[3 * st + 1] * A + c[3 * st + 2] * A2)
    return X


def walk(A, mode, m=30, theta=3.2):
    A = np.asarray(A, complex)
    im = np.imag(np.diag(A))
    mu = np.round(0.5 * (im.min() + im.max()) * 16) / 16
    As = A - 1j * mu * np.eye(A.shape[0])
    if mode == "noshift" or (mode == "lowonly" and np.max(np.sum(np.abs(As), axis=0)) > 0.25):
        mu, As = 0.0, A
    n = np.max(np.sum(np.abs(As), axis=0))
    s = 0 if n <= theta else int(ceil(log2(n / theta)))
    E = taylor_ps(As / 2 ** s, m)
    for _ in range(s):
        E = E @ E
    return E * np.exp(1j * mu)


def main(nts):
    julia = O.julia_exp
    for nt in nts:
        fo = P.full9_problem(nt, nerr=4, device=False)
        acc, norm = {}, 0.0
        for seed in range(900, 904):
            x = P.random_x(nt, seed)
            norm = max(norm, P.max_step_norm(P.full9_problem(nt, nerr=4), x[None]))
            O.julia_exp = lambda A, stats=None: ref_exp(A)
            r = O.calculate_fidelity_and_derivatives(fo, x)
            for k in ("julia", "noshift", "shift", "lowonly"):
                O.julia_exp = julia if k == "julia" else (lambda A, stats=None, k=k: walk(A, k))
                v = O.calculate_fidelity_and_derivatives(fo, x)
                e = [np.max(np.abs(np.asarray(v[1]) - r[1])), np.max(np.abs(np.asarray(v[2]) - r[2])),
                     np.max(np.abs(np.asarray(v[3])[:nt] - np.asarray(r[3])[:nt]))]
                acc[k] = np.maximum(acc.get(k, 0.0), e)
            O.julia_exp = julia
        print(f"N_t={nt:4d} |A|_1={norm:5.1f} " + "  ".join(
            f"{k}: F_dx {v[0]:.1e} F_d2err {v[1]:.1e} F_d2err_dx {v[2]:.1e}" for k, v in acc.items()), flush=True)


if __name__ == "__main__":
    main([int(a) for a in sys.argv[1:]] or [1, 2, 4, 8, 16, 32, 64, 256])
