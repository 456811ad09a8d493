"""Accuracy of the chunk walks' exponential in the high-norm regime (CPU study, numpy + longdouble).

For random 4 x 4 skew-Hermitian A at |A|_1 = 0.3 ... 80 and perturbation directions B, C: the max
error against an extended-precision (longdouble, 64-bit mantissa) evaluation of the SAME formulas of
  E = exp(A),  D1 = (exp(A + eps B) - exp(A)) / eps  (eps = 1e-8, UnitaryCalculations.jl:51-52),
  D2 = (exp(A + eps2 B + eps2 C) + exp(A) - exp(A + eps2 C) - exp(A + eps2 B)) / eps2^2  (:77-83),
for Julia's exp! (oracle.grape_oracle.julia_exp: Pade 13 from |A|_1 > 5.4) and for Taylor(m) by
Paterson-Stockmeyer in A^3 of the diagonal-shifted A / 2^s, s = ceil(log2(|A|_1 / theta)), squared
s times (the walks' algorithm, csrc/grape_walk.hpp).  Round 3's walks: m = 12, theta = 0.25
("walk12@0.25"); round 4: m = 30, theta = 3.2 ("t30@3.2").  Output of a run (seed 1, 20 draws per
norm) is in DESIGN.md 4.2.  Usage: python scripts/probes/highnorm_study.py"""
import sys, numpy as np
sys.path.insert(0, '/root/repo')
from oracle.grape_oracle import julia_exp
from math import factorial, ceil, log2

def ref_exp(A):  # longdouble reference
    A = A.astype(np.clongdouble)
    n = np.max(np.sum(np.abs(A), axis=0))
    s = max(0, int(ceil(log2(float(n) / 0.05)))) if n > 0.05 else 0
    X = A / (2 ** s)
    E = np.eye(A.shape[0], dtype=np.clongdouble); T = E.copy()
    for k in range(1, 30):
        T = T @ X / k; E = E + T
    for _ in range(s): E = E @ E
    return E

def taylor_ps(A, m):  # Paterson-Stockmeyer in A^3 like the walks (degree m = 3 nst + 3), double
    d = A.shape[0]; I = np.eye(d, dtype=complex)
    A2 = A @ A; A3 = A2 @ A
    nst = (m - 3) // 3
    c = [1.0 / factorial(k) for k in range(m + 1)]
    X = c[m - 3] * I + c[m - 2] * A + c[m - 1] * A2 + c[m] * A3
    for st in range(nst - 1, -1, -1):
        X = A3 @ X + (c[3 * st] * I + c[3 * st + 1] * A + c[3 * st + 2] * A2)
    return X

def walk_exp(A, m=12, theta=0.25, shift=True):
    d = A.shape[0]
    mu = 0.0
    if shift:
        im = np.imag(np.diag(A)); mu = 0.5 * (im.min() + im.max())
        A = A - 1j * mu * np.eye(d)
    n = np.max(np.sum(np.abs(A), axis=0))
    s = 0 if n <= theta else int(ceil(log2(n / theta)))
    E = taylor_ps(A / 2 ** s, m)
    for _ in range(s): E = E @ E
    return E * np.exp(1j * mu)

def skew(rng, d):
    G = rng.normal(size=(d, d)) + 1j * rng.normal(size=(d, d))
    H = (G + G.conj().T) / 2
    return -1j * H

rng = np.random.default_rng(1)
d = 4
methods = {"julia": julia_exp,
           "walk12@0.25": lambda A: walk_exp(A, 12, 0.25),
           "t18@1.0": lambda A: walk_exp(A, 18, 1.0),
           "t24@2.0": lambda A: walk_exp(A, 24, 2.0),
           "t30@3.2": lambda A: walk_exp(A, 30, 3.2),
           "t36@4.5": lambda A: walk_exp(A, 36, 4.5)}
eps, eps2 = 1e-8, 1e-4
for norm in [0.3, 1.0, 3.0, 10.0, 30.0, 80.0]:
    errs = {k: [0, 0, 0] for k in methods}
    for trial in range(20):
        A = skew(rng, d); A *= norm / np.max(np.sum(np.abs(A), axis=0))
        B = skew(rng, d) * 0.3; C = skew(rng, d) * 0.3
        Er, Ebr = ref_exp(A), ref_exp(A + eps * B)
        D1r = (Ebr - Er) / eps
        Ec, Ecb = ref_exp(A + eps2 * C), ref_exp(A + eps2 * B + eps2 * C)
        Eb2 = ref_exp(A + eps2 * B)
        D2r = (Ecb + Er - Ec - Eb2) / eps2 ** 2
        for k, f in methods.items():
            E, Eb = f(A), f(A + eps * B)
            D1 = (Eb - E) / eps
            D2 = (f(A + eps2 * B + eps2 * C) + E - f(A + eps2 * C) - f(A + eps2 * B)) / eps2 ** 2
            e0 = float(np.max(np.abs(E - Er)))
            e1 = float(np.max(np.abs(D1 - D1r)) / np.max(np.abs(D1r)))
            e2 = float(np.max(np.abs(D2 - D2r)) / np.max(np.abs(D2r)))
            errs[k] = [max(errs[k][0], e0), max(errs[k][1], e1), max(errs[k][2], e2)]
    print(f"|A|_1={norm:5.1f} " + "  ".join(f"{k}: E {v[0]:.1e} D1 {v[1]:.1e} D2 {v[2]:.1e}" for k, v in errs.items()))
