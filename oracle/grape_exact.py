"""Extended-precision restatement of the reference's fidelity gradient: the value the reference's
forward differences would return without rounding in the exponentials, the chain and the traces.

TEST INFRASTRUCTURE ONLY (like grape_oracle.py): used by tests/ and scripts/probes/ as a second
checker, never by robustgrape_amd/.

The reference (FidelityCalculations.jl:19-119 over UnitaryCalculations.jl:20-155) computes, with
eps = 1e-8 (Types.jl:38) and the controls and Hamiltonians in double precision,
  E_k = exp(-i dt H0(k, x_k, x_add)),  C_k = E_k C_{k-1}                     (UnitaryCalculations.jl:45-47)
  U_dx[p, k] = U C_k^-1 (exp(-i dt H0(k, x_k + eps e_p, x_add)) - E_k) / eps C_{k-1}   (:48-56, :114-118)
  U0_dx_add[q] = (U0(x_add + eps e_q) - U0(x_add)) / eps                       (FidelityCalculations.jl:32-40)
  F, F_dx, F_dx_add                                                          (:47-76)
in double arithmetic, so every implementation's F_dx carries its own u / eps rounding noise (its
exponential's rounding and the rounding of the Hamiltonian's trig, amplified by 1 / eps).  Here the
SAME inputs -- the controls and the perturbed control fl(x + eps) as the reference forms it, the
operators and the target in double -- go through the Hamiltonian's coefficients (operator bases;
closures stay double), exponentials (Taylor 40 with scaling and squaring), products and traces in
numpy longdouble (64-bit mantissa: the result's own noise is ~1e-19 2^s / 1e-8 = 1e-11 2^s of |F_dx|
with s the squarings of the largest step); an
operator-basis target likewise.  What is left is the forward difference itself, O(eps) truncation
included: the quantity
the reference means to return, against which the noise of the oracle, the C++ port and the device
paths can each be read off (scripts/probes/fd_exact_probe.py, tests/test_gpu_gauge.py).

Scope: no error sources (F, F_dx, F_dx_add), H0 free of x_add (the target part of F_dx_add only).
"""
from __future__ import annotations

import math

import numpy as np

LD = np.clongdouble
# the whole point is a wider mantissa than double's 52 bits: on a platform whose longdouble is double
# the "exact" tiers would silently compare double with double
assert np.finfo(np.longdouble).nmant >= 63, "grape_exact needs an x87 80-bit (or wider) np.longdouble"


def squarings(norm1):
    """Squarings exp_ld takes at |A|_1 = norm1 (its noise grows like 2^s: about 1e-19 * 2^s relative)."""
    return max(0, int(math.ceil(math.log2(norm1)))) if norm1 > 1.0 else 0


def exp_ld(A):
    """exp of a longdouble complex matrix: Taylor 40 of A / 2^s with |A / 2^s|_1 <= 1 (remainder below
    1 / 41! = 3e-50), s squarings."""
    n = float(np.max(np.sum(np.abs(A), axis=0)))
    s = squarings(n)
    X = A / LD(2 ** s)
    E = np.eye(A.shape[0], dtype=LD)
    T = E.copy()
    for k in range(1, 41):
        T = T @ X / LD(k)
        E = E + T
    for _ in range(s):
        E = E @ E
    return E


def _h0_ld(H0, k, xk, xa):
    """H0(k, x_k, x_add) in longdouble: an operator basis (objects with .terms: op, var, index, func,
    a, b, scale -- the grape_term fields) has its coefficients evaluated in longdouble from the double
    controls, so the two propagators of a forward difference differ only through the exact change of
    the control; any other closure is evaluated in double as the reference does."""
    terms = getattr(H0, "terms", None)
    if terms is None:
        return np.asarray(H0(k, xk.copy(), xa.copy()), dtype=np.complex128).astype(LD)
    H = np.zeros(terms[0].op.shape, dtype=LD)
    for t in terms:  # var: 0 one, 1 x, 2 x_add, 3 step; func: 0 one, 1 linear, 2 cos, 3 sin, 4 cis
        v = {0: np.longdouble(1), 1: np.longdouble(xk[t.index]) if t.var == 1 else 0,
             2: np.longdouble(xa[t.index]) if t.var == 2 else 0, 3: np.longdouble(k)}[t.var]
        arg = np.longdouble(t.a) * v + np.longdouble(t.b)
        f = {0: LD(1), 1: LD(arg), 2: LD(np.cos(arg)), 3: LD(np.sin(arg)),
             4: LD(np.cos(arg)) + LD(1j) * LD(np.sin(arg))}[t.func]
        H = H + LD(complex(t.scale)) * f * np.asarray(t.op, dtype=np.complex128).astype(LD)
    return H


def _target_ld(target, xa):
    """target_unitary(x_add) in longdouble for an operator basis (as _h0_ld), else in double."""
    terms = getattr(target, "terms", None)
    if terms is None:
        return np.asarray(target(xa.copy()), dtype=np.complex128).astype(LD)
    return _h0_ld(target, 1, np.zeros(0), xa)


def _reads_xadd(H, na, err=False):
    """True when the Hamiltonian (an operator basis: a term with var == 2; a closure: a probe at two
    x_add values) depends on x_add -- outside this evaluator's scope (it takes U_dx_add = 0)."""
    if na == 0:
        return False
    terms = getattr(H, "terms", None)
    if terms is not None:
        return any(t.var == 2 for t in terms)
    rng = np.random.default_rng(7)
    x = rng.uniform(-1.0, 1.0, size=8)
    xa = rng.uniform(-1.0, 1.0, size=na)
    args = (lambda a: (1, x.copy(), a.copy(), 0.01)) if err else (lambda a: (1, x.copy(), a.copy()))
    try:
        h0 = np.asarray(H(*args(xa)))
        h1 = np.asarray(H(*args(xa + 0.37)))
    except (IndexError, TypeError, ValueError):
        return False  # a closure that cannot be probed this way: left to the caller
    return not np.array_equal(h0, h1)


def _check_scope(up):
    na = up.nb_additional_param
    if _reads_xadd(up.H0, na):
        raise ValueError("grape_exact covers H0 independent of x_add (it takes U_dx_add = 0)")
    for src in up.error_sources:
        if _reads_xadd(src.Herror, na, err=True):
            raise ValueError("grape_exact covers Herror independent of x_add (it takes U_derr_dx_add = 0)")


def fidelity_and_gradient(fp, x, nparam=1):
    """(F, F_dx_tot) of calculate_fidelity_and_derivatives(fp, x), evaluated in longdouble."""
    up = fp.unitary_problem
    _check_scope(up)
    if len(up.error_sources):
        raise ValueError("grape_exact covers problems without error sources")
    nt, d, na = up.ntimes, up.ndim, up.nb_additional_param
    eps = up.eps
    dt = up.t0 / nt
    x = np.asarray(x, dtype=np.float64)
    xm = x[:len(x) - na].reshape(nt, nparam)
    xa = x[len(x) - na:].copy()
    Es, dEs = [], []
    for k in range(nt):
        E = exp_ld(LD(-1j * dt) * _h0_ld(up.H0, k + 1, xm[k], xa))
        Es.append(E)
        row = []
        for p in range(nparam):
            xp = xm[k].copy()
            xp[p] = xp[p] + eps  # fl(x + eps): the perturbed control the reference forms
            row.append((exp_ld(LD(-1j * dt) * _h0_ld(up.H0, k + 1, xp, xa)) - E) / LD(eps))
        dEs.append(row)
    C = [np.eye(d, dtype=LD)]
    for E in Es:
        C.append(E @ C[-1])
    U = C[-1]
    P0 = np.asarray(fp.projector, dtype=np.complex128)
    P = P0.copy()
    P[P != 0] = 1
    Dn = float(np.real(np.trace(P0)))
    P0, P = P0.astype(LD), P.astype(LD)
    DD = Dn * (Dn + 1)
    ct = lambda A: A.conj().T  # noqa: E731
    tr_mod = lambda A: np.trace(P0 @ A)  # noqa: E731
    U0 = _target_ld(fp.target_unitary, xa)
    F = (np.real(tr_mod(P @ ct(U0) @ U @ P @ ct(U) @ U0)) + abs(tr_mod(P @ ct(U0) @ U)) ** 2) / DD
    tau_c = np.conj(tr_mod(P @ ct(U0) @ U))
    Fdx = np.zeros(len(x))
    for k in range(nt):
        for p in range(nparam):
            Ud = U @ ct(C[k + 1]) @ dEs[k][p] @ C[k]  # C_k^-1 = C_k^dag (exact to 1e-19 here)
            Fdx[k * nparam + p] = float(np.real(tr_mod(P @ ct(U0) @ Ud @ P @ ct(U) @ U0
                                                       + P @ ct(U0) @ U @ P @ ct(Ud) @ U0))
                                        + 2 * np.real(tau_c * tr_mod(P @ ct(U0) @ Ud))) / DD
    for q in range(na):  # FidelityCalculations.jl:32-40, 67-76 with U_dx_add = 0 (H0 free of x_add)
        xq = xa.copy()
        xq[q] = xq[q] + eps
        U0q = _target_ld(fp.target_unitary, xq)
        U0d = (U0q - U0) / LD(eps)
        Fdx[nt * nparam + q] = float(np.real(tr_mod(P @ ct(U0d) @ U @ P @ ct(U) @ U0
                                                    + P @ ct(U0) @ U @ P @ ct(U) @ U0d))
                                     + 2 * np.real(tau_c * tr_mod(P @ ct(U0d) @ U))) / DD
    return float(F), Fdx


def _herr_ld(src, k, xk, xa, err):
    """Herror_e(k, x_k, x_add, err) in longdouble (an operator-basis error is err * sum of terms)."""
    H = src.Herror
    if getattr(H, "terms", None) is None:
        return np.asarray(H(k, xk.copy(), xa.copy(), err), dtype=np.complex128).astype(LD)
    return LD(err) * _h0_ld(H, k, xk, xa)


def fidelity_and_derivatives(fp, x, nparam=1):
    """(F, F_dx_tot, F_d2err, F_d2err_dx_tot) of calculate_fidelity_and_derivatives(fp, x) with error
    sources (UnitaryCalculations.jl:44-151, FidelityCalculations.jl:19-119), evaluated in longdouble:
    the eps differences of the error propagators (:66-73) and the eps2 mixed stencils (:75-97, left to
    right as the reference writes them), the cumulative sums (:112-113) and the assembly (:114-151).
    Scope: H0 and Herror free of x_add (then U_dx_add and U_derr_dx_add are exactly zero in the
    reference too; the target's difference remains in F_dx_add and F_d2err_dx_add)."""
    up = fp.unitary_problem
    _check_scope(up)
    nt, d, na, ne = up.ntimes, up.ndim, up.nb_additional_param, len(up.error_sources)
    eps, eps2 = up.eps, up.eps2
    dt = up.t0 / nt
    x = np.asarray(x, dtype=np.float64)
    xm = x[:len(x) - na].reshape(nt, nparam)
    xa = x[len(x) - na:].copy()
    cdt = LD(-1j * dt)
    ct = lambda A: A.conj().T  # noqa: E731
    C = np.eye(d, dtype=LD)
    Vdx = np.zeros((nparam, nt, d, d), dtype=LD)
    Verr = np.zeros((ne, nt, d, d), dtype=LD)
    Vmix = np.zeros((nparam, ne, nt, d, d), dtype=LD)
    for k in range(nt):
        xk = xm[k].copy()
        H0k = _h0_ld(up.H0, k + 1, xk, xa)
        E = exp_ld(cdt * H0k)
        Cold, C = C, E @ C
        Ci = ct(C)  # the unitary chain's inverse (exact here to 1e-19)
        Edx2 = []
        for p in range(nparam):
            xp = xk.copy()
            xp[p] = xp[p] + eps
            Vdx[p, k] = Ci @ ((exp_ld(cdt * _h0_ld(up.H0, k + 1, xp, xa)) - E) / LD(eps)) @ Cold
            xp[p] = xk[p] + eps2
            Edx2.append(exp_ld(cdt * _h0_ld(up.H0, k + 1, xp, xa)))
        for e, src in enumerate(up.error_sources):
            E1 = exp_ld(cdt * (_herr_ld(src, k + 1, xk, xa, eps) + H0k))
            Verr[e, k] = Ci @ ((E1 - E) / LD(eps)) @ Cold
            E2 = exp_ld(cdt * (_herr_ld(src, k + 1, xk, xa, eps2) + H0k))
            for p in range(nparam):
                xp = xk.copy()
                xp[p] = xp[p] + eps2
                Em = exp_ld(cdt * (_herr_ld(src, k + 1, xp, xa, eps2) + _h0_ld(up.H0, k + 1, xp, xa)))
                Vmix[p, e, k] = Ci @ (((Em + E) - E2 - Edx2[p]) / LD(eps2 * eps2)) @ Cold
    U = C
    P0 = np.asarray(fp.projector, dtype=np.complex128)
    P = P0.copy()
    P[P != 0] = 1
    Dn = float(np.real(np.trace(P0)))
    P0, P = P0.astype(LD), P.astype(LD)
    DD = Dn * (Dn + 1)
    tr_mod = lambda A: np.trace(P0 @ A)  # noqa: E731
    U0 = _target_ld(fp.target_unitary, xa)
    U0d = []
    for q in range(na):
        xq = xa.copy()
        xq[q] = xq[q] + eps
        U0d.append((_target_ld(fp.target_unitary, xq) - U0) / LD(eps))
    F = (np.real(tr_mod(P @ ct(U0) @ U @ P @ ct(U) @ U0)) + abs(tr_mod(P @ ct(U0) @ U)) ** 2) / DD
    tau_c = np.conj(tr_mod(P @ ct(U0) @ U))
    Fdx = np.zeros(nt * nparam + na)
    for k in range(nt):
        for p in range(nparam):
            Ud = U @ Vdx[p, k]
            Fdx[k * nparam + p] = float((np.real(tr_mod(P @ ct(U0) @ Ud @ P @ ct(U) @ U0
                                                         + P @ ct(U0) @ U @ P @ ct(Ud) @ U0))
                                         + 2 * np.real(tau_c * tr_mod(P @ ct(U0) @ Ud))) / DD)
    for q in range(na):
        Fdx[nt * nparam + q] = float((np.real(tr_mod(P @ ct(U0d[q]) @ U @ P @ ct(U) @ U0
                                                     + P @ ct(U0) @ U @ P @ ct(U) @ U0d[q]))
                                      + 2 * np.real(tau_c * tr_mod(P @ ct(U0d[q]) @ U))) / DD)
    Fd2 = np.zeros(ne)
    Fd2dx = np.zeros((nt * nparam + na, ne))
    for e in range(ne):
        S = np.cumsum(Verr[e], axis=0)                      # S[k] = sum_{j <= k}
        R = np.flip(np.cumsum(np.flip(Verr[e], 0), axis=0), 0)  # R[k] = sum_{j >= k}
        Ue = U @ S[-1]
        Fd2[e] = float(2 * (np.real(tr_mod(P @ ct(U0) @ Ue @ P @ ct(Ue) @ U0 - P @ ct(Ue) @ Ue))
                            + abs(tr_mod(P @ ct(U0) @ Ue)) ** 2
                            - Dn * np.real(tr_mod(P @ ct(Ue) @ Ue))) / DD)
        te_c = np.conj(tr_mod(P @ ct(U0) @ Ue))
        for k in range(nt):
            for p in range(nparam):
                acc = Vmix[p, e, k].copy()
                if k >= 1:
                    acc = acc + Vdx[p, k] @ S[k - 1]
                if k <= nt - 2:
                    acc = acc + R[k + 1] @ Vdx[p, k]
                Y = U @ acc
                Fd2dx[k * nparam + p, e] = float(2 * (
                    np.real(tr_mod(P @ ct(U0) @ Y @ P @ ct(Ue) @ U0 + P @ ct(U0) @ Ue @ P @ ct(Y) @ U0
                                   - P @ ct(Y) @ Ue - P @ ct(Ue) @ Y))
                    + 2 * np.real(te_c * tr_mod(P @ ct(U0) @ Y))
                    - Dn * np.real(tr_mod(P @ ct(Y) @ Ue + P @ ct(Ue) @ Y))) / DD)
        for q in range(na):  # U_derr_dx_add = 0 (H0, Herror free of x_add): the target's part only
            Fd2dx[nt * nparam + q, e] = float(2 * (
                np.real(tr_mod(P @ ct(U0d[q]) @ Ue @ P @ ct(Ue) @ U0 + P @ ct(U0) @ Ue @ P @ ct(Ue) @ U0d[q]))
                + 2 * np.real(te_c * tr_mod(P @ ct(U0d[q]) @ Ue))) / DD)
    return float(F), Fdx, Fd2, Fd2dx


def sensitivities_and_xadd(fp, x, nparam=1):
    """(F, F_d2err, F_d2err_dx[n_main:]) evaluated in longdouble -- the x_add rows of the mixed gradient
    without the mixed stencils: with H0 and Herror free of x_add, U_derr_dx_add = 0 and those rows are
    the target's difference against U_derr (FidelityCalculations.jl:96-113), so only the nominal and the
    eps error propagators are needed (UnitaryCalculations.jl:45-47, 66-73; 1 + ne exponentials per step
    instead of fidelity_and_derivatives' 1 + 2 np + ne (2 + np)).  The same expressions as
    fidelity_and_derivatives, so the values are its own."""
    up = fp.unitary_problem
    _check_scope(up)
    nt, d, na, ne = up.ntimes, up.ndim, up.nb_additional_param, len(up.error_sources)
    eps = up.eps
    dt = up.t0 / nt
    x = np.asarray(x, dtype=np.float64)
    xm = x[:len(x) - na].reshape(nt, nparam)
    xa = x[len(x) - na:].copy()
    cdt = LD(-1j * dt)
    ct = lambda A: A.conj().T  # noqa: E731
    C = np.eye(d, dtype=LD)
    Ssum = np.zeros((ne, d, d), dtype=LD)
    for k in range(nt):
        xk = xm[k].copy()
        H0k = _h0_ld(up.H0, k + 1, xk, xa)
        E = exp_ld(cdt * H0k)
        Cold, C = C, E @ C
        Ci = ct(C)
        for e, src in enumerate(up.error_sources):
            E1 = exp_ld(cdt * (_herr_ld(src, k + 1, xk, xa, eps) + H0k))
            Ssum[e] = Ssum[e] + Ci @ ((E1 - E) / LD(eps)) @ Cold
    U = C
    P0 = np.asarray(fp.projector, dtype=np.complex128)
    P = P0.copy()
    P[P != 0] = 1
    Dn = float(np.real(np.trace(P0)))
    P0, P = P0.astype(LD), P.astype(LD)
    DD = Dn * (Dn + 1)
    tr_mod = lambda A: np.trace(P0 @ A)  # noqa: E731
    U0 = _target_ld(fp.target_unitary, xa)
    U0d = []
    for q in range(na):
        xq = xa.copy()
        xq[q] = xq[q] + eps
        U0d.append((_target_ld(fp.target_unitary, xq) - U0) / LD(eps))
    F = (np.real(tr_mod(P @ ct(U0) @ U @ P @ ct(U) @ U0)) + abs(tr_mod(P @ ct(U0) @ U)) ** 2) / DD
    Fd2 = np.zeros(ne)
    add = np.zeros((na, ne))
    for e in range(ne):
        Ue = U @ Ssum[e]
        Fd2[e] = float(2 * (np.real(tr_mod(P @ ct(U0) @ Ue @ P @ ct(Ue) @ U0 - P @ ct(Ue) @ Ue))
                            + abs(tr_mod(P @ ct(U0) @ Ue)) ** 2
                            - Dn * np.real(tr_mod(P @ ct(Ue) @ Ue))) / DD)
        te_c = np.conj(tr_mod(P @ ct(U0) @ Ue))
        for q in range(na):
            add[q, e] = float(2 * (
                np.real(tr_mod(P @ ct(U0d[q]) @ Ue @ P @ ct(Ue) @ U0 + P @ ct(U0) @ Ue @ P @ ct(Ue) @ U0d[q]))
                + 2 * np.real(te_c * tr_mod(P @ ct(U0d[q]) @ Ue))) / DD)
    return float(F), Fd2, add
