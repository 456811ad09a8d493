"""CPU oracle: numpy restatement of RobustGRAPE.jl's hot path.

TEST INFRASTRUCTURE ONLY.  Nothing under ``robustgrape_amd/`` imports this
module; only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg use it, and only as the checker.

What it restates (citations are into the read-only reference tree):

* ``calculate_unitary_and_derivatives``  -- src/UnitaryCalculations.jl:20-155,
  op for op: the nominal propagator (:45), the forward chain and the LU
  ``inv`` of it (:46-47), the eps forward differences and the eps2
  exponentials that only the mixed stencils consume (:48-64), the error
  differences and mixed stencils (:66-98), the permutes (:102-104) and the
  assembly loops with cumsum / reverse cumsum (:106-154).
* ``calculate_fidelity_and_derivatives`` -- src/FidelityCalculations.jl:19-119.
* ``calculate_interaction_error_operators`` -- src/UnitaryCalculations.jl:180-204,
  ``calculate_expectation_values`` -- src/FidelityCalculations.jl:368-390,
  ``calculate_fidelity_response`` -- :246-280, ``calculate_fidelity_response_fft``
  -- :306-343 (used by the "next" rows of SURVEY.md section 8f).
* ``regularization_cost`` / ``regularization_cost_phase`` -- src/Regularization.jl:26-115,
  and the optimiser's cost assembly ``calculate_common!`` -- src/FidelityCalculations.jl:172-196.
* Julia's ``LinearAlgebra.exp!`` (third-party: Julia stdlib, the only Julia
  the reference pins is 1.9 in .github/workflows/docs.yml:17; not present in
  /root/reference).  Restated from its published algorithm: ``isdiag`` early
  exit, LAPACK ``zgebal('B')`` (permute + scale, LAPACK <= 3.11 semantics as
  bundled with Julia 1.9's OpenBLAS), Higham-2005 Pade degree by 1-norm
  thresholds 0.015/0.25/0.95/2.1 (m = 3/5/7/9) else m = 13 with
  s = ceil(log2(|A|_1/5.4)) squarings, the even/odd U, V build in Julia's
  accumulation order, ``gesv(V-U, V+U)``, squaring, balancing undone.
* ``inv`` = LAPACK getrf + getri (Julia ``inv`` on a dense matrix).

Parity pinning: the reference's Julia toolchain is absent from this container
(nothing was refused, ``julia`` is simply not installed),
so no reference-produced golden vector exists.  This oracle is pinned by the
reference's own known-answer and identity tests (test/runtests.jl:48-165,
:292-354, :418-529, :531-619) re-run with numpy seeds in
tests/test_oracle_reference_identities.py.  Bit-level parity with Julia's
OpenBLAS rounding is not claimed (it is not reproducible without Julia).

Conventions: matrices are numpy 2-D complex128 arrays indexed [row, col];
``x`` is laid out like the reference: x[p + k*nparam] is control p at step k
(0-based), the last ``nb_additional_param`` entries are x_add.  Closures
H0(nt, x, x_add) and Herror(nt, x, x_add, err) receive a 1-based ``nt`` like
the reference (Types.jl:25).
"""
from __future__ import annotations

import math

import numpy as np
import scipy.linalg.lapack as lapack

# ---------------------------------------------------------------------------
# Julia stdlib pieces
# ---------------------------------------------------------------------------

_SFMIN1 = np.finfo(np.float64).tiny / np.finfo(np.float64).eps  # dlamch('S')/dlamch('P')
_SFMAX1 = 1.0 / _SFMIN1
_SFMIN2 = _SFMIN1 * 2.0
_SFMAX2 = 1.0 / _SFMIN2


def zgebal_b(A):
    """LAPACK zgebal with JOB='B' (LAPACK 3.10 algorithm: permute then scale).

    Returns (A_balanced, ilo, ihi, scale) with 1-based ilo/ihi and the SCALE
    array as LAPACK stores it (permutation targets as 1-based indices for
    j < ilo and j > ihi, scaling factors in between).
    """
    A = np.array(A, dtype=np.complex128, copy=True)
    n = A.shape[0]
    scale = np.ones(n)
    if n == 0:
        return A, 1, 0, scale
    k, l = 1, n  # 1-based active window [k, l]

    def swap(j, m):
        # SCALE(M) = J; swap columns J,M over rows 1..L and rows J,M over cols K..N
        scale[m - 1] = j
        if j != m:
            A[: l, [j - 1, m - 1]] = A[: l, [m - 1, j - 1]]
            A[[j - 1, m - 1], k - 1:] = A[[m - 1, j - 1], k - 1:]

    # Search for rows isolating an eigenvalue and push them down.
    while True:
        found = False
        for j in range(l, 0, -1):
            row_zero = True
            for i in range(1, l + 1):
                if i == j:
                    continue
                if A[j - 1, i - 1] != 0:
                    row_zero = False
                    break
            if row_zero:
                swap(j, l)
                found = True
                break
        if not found:
            break
        if l == 1:
            return A, k, l, scale
        l -= 1
    # Search for columns isolating an eigenvalue and push them left.
    while True:
        found = False
        for j in range(k, l + 1):
            col_zero = True
            for i in range(k, l + 1):
                if i == j:
                    continue
                if A[i - 1, j - 1] != 0:
                    col_zero = False
                    break
            if col_zero:
                swap(j, k)
                found = True
                break
        if not found:
            break
        k += 1
    for i in range(k, l + 1):
        scale[i - 1] = 1.0
    # Iterative norm reduction on rows/cols k..l.
    sclfac, factor = 2.0, 0.95
    noconv = True
    while noconv:
        noconv = False
        for i in range(k, l + 1):
            c = float(np.linalg.norm(A[k - 1:l, i - 1]))
            r = float(np.linalg.norm(A[i - 1, k - 1:l]))
            ca = float(np.max(np.abs(A[:l, i - 1])))
            ra = float(np.max(np.abs(A[i - 1, k - 1:])))
            if c == 0.0 or r == 0.0:
                continue
            g = r / sclfac
            f = 1.0
            s = c + r
            while not (c >= g or max(f, c, ca) >= _SFMAX2 or min(r, g, ra) <= _SFMIN2):
                f *= sclfac
                c *= sclfac
                ca *= sclfac
                r /= sclfac
                g /= sclfac
                ra /= sclfac
            g = c / sclfac
            while not (g < r or max(r, ra) >= _SFMAX2 or min(f, c, g, ca) <= _SFMIN2):
                f /= sclfac
                c /= sclfac
                g /= sclfac
                ca /= sclfac
                r *= sclfac
                ra *= sclfac
            if (c + r) >= factor * s:
                continue
            if f < 1.0 and scale[i - 1] < 1.0 and f * scale[i - 1] <= _SFMIN1:
                continue
            if f > 1.0 and scale[i - 1] > 1.0 and scale[i - 1] >= _SFMAX1 / f:
                continue
            g = 1.0 / f
            scale[i - 1] *= f
            noconv = True
            A[i - 1, k - 1:] *= g
            A[:l, i - 1] *= f
    return A, k, l, scale


def _rcswap(X, i, j):
    """Julia's rcswap!(i, j, X): swap columns i,j then rows i,j (1-based)."""
    X[:, [i - 1, j - 1]] = X[:, [j - 1, i - 1]]
    X[[i - 1, j - 1], :] = X[[j - 1, i - 1], :]


_PADE = {
    3: [120.0, 60.0, 12.0, 1.0],
    5: [30240.0, 15120.0, 3360.0, 420.0, 30.0, 1.0],
    7: [17297280.0, 8648640.0, 1995840.0, 277200.0, 25200.0, 1512.0, 56.0, 1.0],
    9: [17643225600.0, 8821612800.0, 2075673600.0, 302702400.0, 30270240.0,
        2162160.0, 110880.0, 3960.0, 90.0, 1.0],
}
_PADE13 = [64764752532480000.0, 32382376266240000.0, 7771770303897600.0,
           1187353796428800.0, 129060195264000.0, 10559470521600.0,
           670442572800.0, 33522128640.0, 1323241920.0,
           40840800.0, 960960.0, 16380.0, 182.0, 1.0]


def pade_degree(norm1):
    """(m, s) Julia's exp! picks for a balanced matrix with 1-norm ``norm1``."""
    if norm1 <= 2.1:
        if norm1 > 0.95:
            return 9, 0
        if norm1 > 0.25:
            return 7, 0
        if norm1 > 0.015:
            return 5, 0
        return 3, 0
    s = math.log2(norm1 / 5.4)
    return 13, (math.ceil(s) if s > 0 else 0)


def julia_exp(A, stats=None):
    """Restatement of Julia 1.9 ``LinearAlgebra.exp!`` for ComplexF64 matrices."""
    A = np.array(A, dtype=np.complex128, copy=True)
    n = A.shape[0]
    if np.count_nonzero(A - np.diag(np.diag(A))) == 0:  # isdiag(A)
        return np.diag(np.exp(np.diag(A)))
    A, ilo, ihi, scale = zgebal_b(A)
    nA = float(np.max(np.sum(np.abs(A), axis=0)))  # opnorm(A, 1)
    Inn = np.eye(n, dtype=np.complex128)
    m, si = pade_degree(nA)
    if stats is not None:
        stats[(m, si)] = stats.get((m, si), 0) + 1
    if m <= 9:
        C = _PADE[m]
        A2 = A @ A
        P = Inn.copy()
        U = C[1] * P
        V = C[0] * P
        for kk in range(1, len(C) // 2):
            k2 = 2 * kk
            P = P @ A2
            U = U + C[k2 + 1] * P
            V = V + C[k2] * P
        U = A @ U
        X = V + U
        X = _gesv(V - U, X)
    else:
        if si > 0:
            A = A / float(2 ** si)
        CC = _PADE13
        A2 = A @ A
        A4 = A2 @ A2
        A6 = A2 @ A4
        U = A @ (A6 @ (CC[13] * A6 + CC[11] * A4 + CC[9] * A2)
                 + CC[7] * A6 + CC[5] * A4 + CC[3] * A2 + CC[1] * Inn)
        V = (A6 @ (CC[12] * A6 + CC[10] * A4 + CC[8] * A2)
             + CC[6] * A6 + CC[4] * A4 + CC[2] * A2 + CC[0] * Inn)
        X = V + U
        X = _gesv(V - U, X)
        for _ in range(si):
            X = X @ X
    # Undo the balancing.
    for j in range(ilo, ihi + 1):
        scj = scale[j - 1]
        X[j - 1, :] *= scj
        X[:, j - 1] /= scj
    if ilo > 1:
        for j in range(ilo - 1, 0, -1):
            _rcswap(X, j, int(scale[j - 1]))
    if ihi < n:
        for j in range(ihi + 1, n + 1):
            _rcswap(X, j, int(scale[j - 1]))
    return X


def _gesv(A, B):
    _, _, x, info = lapack.zgesv(np.asfortranarray(A), np.asfortranarray(B))
    if info > 0:
        raise np.linalg.LinAlgError("singular matrix in gesv")
    return x


def julia_inv(A):
    """Julia ``inv`` for a dense square matrix: LAPACK getrf + getri."""
    lu, piv, info = lapack.zgetrf(np.asfortranarray(A))
    if info > 0:
        raise np.linalg.LinAlgError("singular matrix in getrf")
    inv, info = lapack.zgetri(lu, piv)
    return inv


# ---------------------------------------------------------------------------
# src/UnitaryCalculations.jl
# ---------------------------------------------------------------------------

def _unpack(problem, x):
    """UnitaryCalculations.jl:21-26."""
    x = np.asarray(x, dtype=np.float64)
    na = problem.nb_additional_param
    x_main = x[: len(x) - na]
    if len(x_main) % problem.ntimes != 0:
        raise AssertionError("Control parameter size must be a multiple of time steps")
    nparam = len(x_main) // problem.ntimes
    x_main = x_main.reshape(problem.ntimes, nparam).T.copy()  # (nparam, ntimes)
    x_add = x[len(x) - na:].copy()
    return x_main, x_add, nparam


def calculate_unitary_and_derivatives(problem, x, stats=None):
    """Restatement of UnitaryCalculations.jl:20-155 (op for op)."""
    x_main, x_add, nparam = _unpack(problem, x)
    ntimes = problem.ntimes
    na = problem.nb_additional_param
    x_add_copy = x_add.copy()
    ndim = problem.ndim
    nerr = len(problem.error_sources)
    dt = problem.t0 / problem.ntimes
    eps, eps2 = problem.eps, problem.eps2
    inv_eps = 1.0 / eps
    inv_eps2sq = 1.0 / eps2 ** 2
    cdt = -1j * dt
    E = lambda H: julia_exp(cdt * np.asarray(H, dtype=np.complex128), stats)

    cum_evo = np.eye(ndim, dtype=np.complex128)
    old_cum_evo = cum_evo.copy()
    infimU_dx = np.zeros((ndim, ndim, nparam, ntimes), np.complex128)
    infimU_dx_add = np.zeros((ndim, ndim, na, ntimes), np.complex128)
    infimU_derr = np.zeros((ndim, ndim, nerr, ntimes), np.complex128)
    infimU_derr_dx = np.zeros((ndim, ndim, nparam, nerr, ntimes), np.complex128)
    infimU_derr_dx_add = np.zeros((ndim, ndim, na, nerr, ntimes), np.complex128)
    infim_evo_derr_array = np.zeros((ndim, ndim, nerr), np.complex128)
    infim_evo_dx_array = np.zeros((ndim, ndim, nparam), np.complex128)
    infim_evo_dx_add_array = np.zeros((ndim, ndim, na), np.complex128)

    for it in range(ntimes):
        nt = it + 1
        xk = x_main[:, it].copy()
        infim_evo = E(problem.H0(nt, xk.copy(), x_add.copy()))
        cum_evo = infim_evo @ cum_evo
        cum_evo_inv = julia_inv(cum_evo)
        x_main_copy = xk.copy()
        for p in range(nparam):
            x_main_copy[p] += eps
            infim_evo_dx = E(problem.H0(nt, x_main_copy.copy(), x_add.copy()))
            infimU_dx[:, :, p, it] = cum_evo_inv @ (inv_eps * (infim_evo_dx - infim_evo)) @ old_cum_evo
            x_main_copy[p] = xk[p] + eps2
            infim_evo_dx_array[:, :, p] = E(problem.H0(nt, x_main_copy.copy(), x_add.copy()))
            x_main_copy[p] = xk[p]
        for q in range(na):
            x_add_copy[q] += eps
            infim_evo_dx_add = E(problem.H0(nt, xk.copy(), x_add_copy.copy()))
            infimU_dx_add[:, :, q, it] = cum_evo_inv @ (inv_eps * (infim_evo_dx_add - infim_evo)) @ old_cum_evo
            x_add_copy[q] = x_add[q] + eps2
            infim_evo_dx_add_array[:, :, q] = E(problem.H0(nt, xk.copy(), x_add_copy.copy()))
            x_add_copy[q] = x_add[q]
        for e, src in enumerate(problem.error_sources):
            H0k = np.asarray(problem.H0(nt, xk.copy(), x_add.copy()), np.complex128)
            infim_evo_derr = E(np.asarray(src.Herror(nt, xk.copy(), x_add.copy(), eps), np.complex128) + H0k)
            infimU_derr[:, :, e, it] = cum_evo_inv @ (inv_eps * (infim_evo_derr - infim_evo)) @ old_cum_evo
            infim_evo_derr_array[:, :, e] = E(
                np.asarray(src.Herror(nt, xk.copy(), x_add.copy(), eps2), np.complex128) + H0k)
            for p in range(nparam):
                x_main_copy[p] += eps2
                infim_evo_derr_dx = E(
                    np.asarray(src.Herror(nt, x_main_copy.copy(), x_add.copy(), eps2), np.complex128)
                    + np.asarray(problem.H0(nt, x_main_copy.copy(), x_add.copy()), np.complex128))
                infimU_derr_dx[:, :, p, e, it] = cum_evo_inv @ (inv_eps2sq * (
                    infim_evo_derr_dx + infim_evo
                    - infim_evo_derr_array[:, :, e] - infim_evo_dx_array[:, :, p])) @ old_cum_evo
                x_main_copy[p] = xk[p]
            for q in range(na):
                x_add_copy[q] += eps2
                infim_evo_derr_dx_add = E(
                    np.asarray(src.Herror(nt, xk.copy(), x_add_copy.copy(), eps2), np.complex128)
                    + np.asarray(problem.H0(nt, xk.copy(), x_add_copy.copy()), np.complex128))
                infimU_derr_dx_add[:, :, q, e, it] = cum_evo_inv @ (inv_eps2sq * (
                    infim_evo_derr_dx_add + infim_evo
                    - infim_evo_derr_array[:, :, e] - infim_evo_dx_add_array[:, :, q])) @ old_cum_evo
                x_add_copy[q] = x_add[q]
        old_cum_evo = cum_evo.copy()

    # permutedims (:102-104)
    infimU_derr = infimU_derr.transpose(0, 1, 3, 2)            # (d,d,nt,ne)
    infimU_derr_dx = infimU_derr_dx.transpose(0, 1, 2, 4, 3)   # (d,d,np,nt,ne)
    infimU_derr_dx_add = infimU_derr_dx_add.transpose(0, 1, 2, 4, 3)  # (d,d,na,nt,ne)

    U_dx = np.zeros((ndim, ndim, nparam, ntimes), np.complex128)
    U_dx_add = np.zeros((ndim, ndim, na), np.complex128)
    U_derr = np.zeros((ndim, ndim, nerr), np.complex128)
    U_derr_dx = np.zeros((ndim, ndim, nparam, ntimes, nerr), np.complex128)
    U_derr_dx_add = np.zeros((ndim, ndim, na, nerr), np.complex128)

    cums = np.cumsum(infimU_derr, axis=2)
    revcums = np.flip(np.cumsum(np.flip(infimU_derr, axis=2), axis=2), axis=2)
    for it in range(ntimes):
        for p in range(nparam):
            U_dx[:, :, p, it] = cum_evo @ infimU_dx[:, :, p, it]
    for q in range(na):
        U_dx_add[:, :, q] = cum_evo @ np.sum(infimU_dx_add[:, :, q, :], axis=2)
    for e in range(nerr):
        U_derr[:, :, e] = cum_evo @ np.sum(infimU_derr[:, :, :, e], axis=2)
        for it in range(1, ntimes):
            for p in range(nparam):
                U_derr_dx[:, :, p, it, e] += infimU_dx[:, :, p, it] @ cums[:, :, it - 1, e]
        for it in range(ntimes - 1):
            for p in range(nparam):
                U_derr_dx[:, :, p, it, e] += revcums[:, :, it + 1, e] @ infimU_dx[:, :, p, it]
        for it in range(ntimes):
            for p in range(nparam):
                U_derr_dx[:, :, p, it, e] += infimU_derr_dx[:, :, p, it, e]
                U_derr_dx[:, :, p, it, e] = cum_evo @ U_derr_dx[:, :, p, it, e]
        for q in range(na):
            acc = np.zeros((ndim, ndim), np.complex128)
            for it in range(1, ntimes):
                acc += infimU_dx_add[:, :, q, it] @ cums[:, :, it - 1, e]
            for it in range(ntimes - 1):
                acc += revcums[:, :, it + 1, e] @ infimU_dx_add[:, :, q, it]
            for it in range(ntimes):
                acc += infimU_derr_dx_add[:, :, q, it, e]
            U_derr_dx_add[:, :, q, e] = cum_evo @ acc
    return cum_evo, U_dx, U_dx_add, U_derr, U_derr_dx, U_derr_dx_add


def calculate_interaction_error_operators(problem, x):
    """Restatement of UnitaryCalculations.jl:180-204 -> (d, d, ntimes, nerr)."""
    x_main, x_add, nparam = _unpack(problem, x)
    ntimes, ndim = problem.ntimes, problem.ndim
    nerr = len(problem.error_sources)
    dt = problem.t0 / ntimes
    cum_evo = np.eye(ndim, dtype=np.complex128)
    out = np.zeros((ndim, ndim, nerr, ntimes), np.complex128)
    for it in range(ntimes):
        nt = it + 1
        xk = x_main[:, it].copy()
        cum_evo_inv = julia_inv(cum_evo)
        for e, src in enumerate(problem.error_sources):
            Oerr = (1.0 / problem.eps) * np.asarray(src.Herror(nt, xk.copy(), x_add.copy(), problem.eps),
                                                    np.complex128)
            out[:, :, e, it] = cum_evo_inv @ Oerr @ cum_evo
        infim_evo = julia_exp(-1j * dt * np.asarray(problem.H0(nt, xk.copy(), x_add.copy()), np.complex128))
        cum_evo = infim_evo @ cum_evo
    return out.transpose(0, 1, 3, 2)


# ---------------------------------------------------------------------------
# src/FidelityCalculations.jl
# ---------------------------------------------------------------------------

def _projector_parts(fp):
    """FidelityCalculations.jl:47-51: W = P0, P = (P0 != 0), D = tr(P0)."""
    P0 = np.asarray(fp.projector, dtype=np.complex128)
    P = P0.copy()
    P[P != 0] = 1
    D = float(np.real(np.trace(P0)))
    return P0, P, D


def calculate_fidelity_and_derivatives(fp, x, stats=None):
    """Restatement of FidelityCalculations.jl:19-119."""
    up = fp.unitary_problem
    ndim = up.ndim
    U, U_dx, U_dx_add, U_derr, U_derr_dx, U_derr_dx_add = calculate_unitary_and_derivatives(up, x, stats)
    ntimes = up.ntimes
    na = up.nb_additional_param
    nerr = len(up.error_sources)
    x_main, x_add, nparam = _unpack(up, x)

    U0 = np.asarray(fp.target_unitary(x_add.copy()), dtype=np.complex128)
    U0_dx_add = np.zeros((ndim, ndim, na), np.complex128)
    x_add_copy = x_add.copy()
    for q in range(na):
        x_add_copy[q] += up.eps
        U0_temp = np.asarray(fp.target_unitary(x_add_copy.copy()), dtype=np.complex128)
        U0_dx_add[:, :, q] = (1.0 / up.eps) * (U0_temp - U0)
        x_add_copy[q] = x_add[q]
    F_dx = np.zeros((nparam, ntimes))
    F_dx_add = np.zeros(na)
    F_d2err = np.zeros(nerr)
    F_d2err_dx = np.zeros((nparam, ntimes, nerr))
    F_d2err_dx_add = np.zeros((na, nerr))

    P0, P, D = _projector_parts(fp)
    tr_mod = lambda A: np.trace(P0 @ A)
    ct = lambda A: A.conj().T
    DD = D * (D + 1)

    F = (np.real(tr_mod(P @ ct(U0) @ U @ P @ ct(U) @ U0)) + abs(tr_mod(P @ ct(U0) @ U)) ** 2) / DD
    tau_c = np.conj(tr_mod(P @ ct(U0) @ U))
    for it in range(ntimes):
        for p in range(nparam):
            Ud = U_dx[:, :, p, it]
            F_dx[p, it] = (np.real(tr_mod(P @ ct(U0) @ Ud @ P @ ct(U) @ U0
                                          + P @ ct(U0) @ U @ P @ ct(Ud) @ U0))
                           + 2 * np.real(tau_c * tr_mod(P @ ct(U0) @ Ud))) / DD
    for q in range(na):
        Ud = U_dx_add[:, :, q]
        U0d = U0_dx_add[:, :, q]
        F_dx_add[q] = (np.real(tr_mod(P @ ct(U0) @ Ud @ P @ ct(U) @ U0
                                      + P @ ct(U0) @ U @ P @ ct(Ud) @ U0
                                      + P @ ct(U0d) @ U @ P @ ct(U) @ U0
                                      + P @ ct(U0) @ U @ P @ ct(U) @ U0d))
                       + 2 * np.real(tau_c * tr_mod(P @ ct(U0) @ Ud + P @ ct(U0d) @ U))) / DD
    for e in range(nerr):
        Ue = U_derr[:, :, e]
        F_d2err[e] = 2 * (np.real(tr_mod(P @ ct(U0) @ Ue @ P @ ct(Ue) @ U0 - P @ ct(Ue) @ Ue))
                          + abs(tr_mod(P @ ct(U0) @ Ue)) ** 2
                          - D * np.real(tr_mod(P @ ct(Ue) @ Ue))) / DD
        te_c = np.conj(tr_mod(P @ ct(U0) @ Ue))
        for it in range(ntimes):
            for p in range(nparam):
                Y = U_derr_dx[:, :, p, it, e]
                F_d2err_dx[p, it, e] = 2 * (
                    np.real(tr_mod(P @ ct(U0) @ Y @ P @ ct(Ue) @ U0
                                   + P @ ct(U0) @ Ue @ P @ ct(Y) @ U0
                                   - P @ ct(Y) @ Ue
                                   - P @ ct(Ue) @ Y))
                    + 2 * np.real(te_c * tr_mod(P @ ct(U0) @ Y))
                    - D * np.real(tr_mod(P @ ct(Y) @ Ue + P @ ct(Ue) @ Y))) / DD
        for q in range(na):
            Y = U_derr_dx_add[:, :, q, e]
            U0d = U0_dx_add[:, :, q]
            F_d2err_dx_add[q, e] = 2 * (
                np.real(tr_mod(P @ ct(U0d) @ Ue @ P @ ct(Ue) @ U0
                               + P @ ct(U0) @ Y @ P @ ct(Ue) @ U0
                               + P @ ct(U0) @ Ue @ P @ ct(Y) @ U0
                               + P @ ct(U0) @ Ue @ P @ ct(Ue) @ U0d
                               - P @ ct(Y) @ Ue
                               - P @ ct(Ue) @ Y))
                + 2 * np.real(te_c * tr_mod(P @ ct(U0d) @ Ue + P @ ct(U0) @ Y))
                - D * np.real(tr_mod(P @ ct(Y) @ Ue + P @ ct(Ue) @ Y))) / DD

    F_dx_tot = np.concatenate([F_dx.T.reshape(-1), F_dx_add])
    F_d2err_dx_tot = np.concatenate(
        [F_d2err_dx.transpose(1, 0, 2).reshape(nparam * ntimes, nerr), F_d2err_dx_add], axis=0)
    return float(F), F_dx_tot, F_d2err, F_d2err_dx_tot


def calculate_expectation_values(fp, x):
    """Restatement of FidelityCalculations.jl:368-390 -> (ntimes, nerr)."""
    up = fp.unitary_problem
    ops = calculate_interaction_error_operators(up, x)
    ntimes = up.ntimes
    nerr = ops.shape[3]
    cums = np.cumsum(ops, axis=2)
    dt = up.t0 / ntimes
    P0, P, D = _projector_parts(fp)
    out = np.zeros((ntimes, nerr))
    for e in range(nerr):
        for it in range(ntimes):
            out[it, e] = np.real(dt * np.trace(P0 @ cums[:, :, it, e]) / D)
    return out


def calculate_fidelity_response(fp, x, normalized_frequencies):
    """Restatement of FidelityCalculations.jl:246-280 -> (nfreq, nerr)."""
    up = fp.unitary_problem
    ntimes = up.ntimes
    nerr = len(up.error_sources)
    freqs = np.asarray(normalized_frequencies, dtype=np.float64)
    dt = up.t0 / ntimes
    ops = calculate_interaction_error_operators(up, x)
    P0, P, D = _projector_parts(fp)
    tr_mod = lambda A: np.trace(P0 @ A)
    tidx = np.arange(ntimes)
    out = np.zeros((len(freqs), nerr))
    for e in range(nerr):
        for nf, w in enumerate(freqs):
            phases = np.exp(-1j * w * dt * tidx)
            sum_err = np.einsum("ijk,k->ij", ops[:, :, :, e], phases)
            r = 0.0
            for it in range(ntimes):
                k = it + 1
                ph = np.exp(1j * w * dt * k)
                Ok = ops[:, :, it, e]
                r += (1.0 / D * np.real(ph * tr_mod(Ok @ sum_err @ P))
                      - 1.0 / (D * (D + 1)) * np.real(ph * tr_mod(Ok @ P @ sum_err @ P))
                      - 1.0 / (D * (D + 1)) * np.real(ph * tr_mod(Ok @ P) * tr_mod(sum_err @ P)))
            out[nf, e] = dt ** 2 * r
    return out


def calculate_fidelity_response_fft(fp, x, oversampling=1):
    """Restatement of FidelityCalculations.jl:306-343 -> (response, norm_frequencies)."""
    assert oversampling >= 1
    up = fp.unitary_problem
    ntimes, ndim = up.ntimes, up.ndim
    nerr = len(up.error_sources)
    dt = up.t0 / ntimes
    ops = calculate_interaction_error_operators(up, x)
    nfft = ntimes * oversampling
    padded = np.zeros((ndim, ndim, nfft, nerr), np.complex128)
    padded[:, :, :ntimes, :] = ops
    P0, P, D = _projector_parts(fp)
    tr_mod = lambda A: np.trace(P0 @ A)
    out = np.zeros((nfft, nerr))
    for e in range(nerr):
        f = np.fft.fft(padded[:, :, :, e], axis=2)
        fi = nfft * np.fft.ifft(padded[:, :, :, e], axis=2)
        for it in range(nfft):
            out[it, e] = dt ** 2 * (
                1 / D * np.real(tr_mod(fi[:, :, it] @ f[:, :, it] @ P))
                - 1 / (D * (D + 1)) * np.real(tr_mod(fi[:, :, it] @ P @ f[:, :, it] @ P))
                - 1 / (D * (D + 1)) * np.real(tr_mod(fi[:, :, it] @ P) * tr_mod(f[:, :, it] @ P)))
    freqs = (2 * np.pi / (nfft * dt)) * np.arange(nfft)
    return out, freqs


# ---------------------------------------------------------------------------
# src/Regularization.jl and the optimiser's cost (FidelityCalculations.jl:161-218)
# ---------------------------------------------------------------------------

def regularization_cost(x, f=None, df=None):
    """Regularization.jl:26-48 (and :76-81 with a transform f, derivative df):
    (reg1, jac1, reg2, jac2) for one control's time series, written loop by
    loop like the reference (jac2 has explicit end stencils, n >= 4)."""
    x = np.asarray(x, dtype=np.float64)
    if f is not None:
        fx = np.array([f(v) for v in x])
        r1, j1, r2, j2 = regularization_cost(fx)
        dfx = np.array([df(v) for v in x])
        return r1, dfx * j1, r2, dfx * j2
    n = x.shape[0]
    diff_x = np.diff(x)
    diff_diff_x = np.diff(diff_x)
    reg1 = float(np.sum(diff_x ** 2))
    reg2 = float(np.sum(diff_diff_x ** 2))
    jac1 = np.zeros(n)
    jac2 = np.zeros(n)
    jac1[1:n - 1] = -2.0 * diff_diff_x
    jac1[0] += -2.0 * diff_x[0]
    jac1[n - 1] += 2.0 * diff_x[n - 2]
    jac2[0] = 2 * (x[2] - 2 * x[1] + x[0])
    jac2[1] = 2 * (x[3] - 4 * x[2] + 5 * x[1] - 2 * x[0])
    for i in range(2, n - 2):
        jac2[i] = 2 * (x[i + 2] - 4 * x[i + 1] + 6 * x[i] - 4 * x[i - 1] + x[i - 2])
    jac2[n - 2] = 2 * (x[n - 4] - 4 * x[n - 3] + 5 * x[n - 2] - 2 * x[n - 1])
    jac2[n - 1] = 2 * (x[n - 3] - 2 * x[n - 2] + x[n - 1])
    return reg1, jac1, reg2, jac2


def regularization_cost_phase(phis):
    """Regularization.jl:111-115: cos and sin transforms, summed."""
    a = regularization_cost(phis, math.cos, lambda v: -math.sin(v))
    b = regularization_cost(phis, math.sin, math.cos)
    return a[0] + b[0], a[1] + b[1], a[2] + b[2], a[3] + b[3]


def optimization_cost(fp, x, regularization_functions, coeff1, coeff2, error_source_coeff):
    """calculate_common! (FidelityCalculations.jl:172-196): returns the buffer
    [cost, grad...] the optimiser's f / g! read.  nparam > 1 follows the intent
    (each control's regularisation gradient on its own entries); the reference's
    `buffer[2:end-na] += sum(reg_costs_grad, dims=1)[1,:]` (:195) only has matching
    shapes for nparam == 1."""
    up = fp.unitary_problem
    na = up.nb_additional_param
    F, F_dx, F_d2err, F_d2err_dx = calculate_fidelity_and_derivatives(fp, x)
    x_main, _, nparam = _unpack(up, x)
    buf = np.zeros(len(x) + 1)
    buf[0] = 1.0 - F
    buf[1:] = -F_dx
    if len(F_d2err) > 0:
        c = np.asarray(error_source_coeff, dtype=np.float64)
        buf[0] += float(np.sum(c * F_d2err ** 2))
        buf[1:] += 2.0 * np.sum((c * F_d2err)[None, :] * F_d2err_dx, axis=1)
    reg_tot = np.zeros(nparam)
    reg_grad = np.zeros((nparam, up.ntimes))
    for p in range(nparam):
        r1, j1, r2, j2 = regularization_functions[p](x_main[p, :])
        reg_tot[p] = coeff1[p] * r1 + coeff2[p] * r2
        reg_grad[p, :] = coeff1[p] * np.asarray(j1) + coeff2[p] * np.asarray(j2)
    buf[0] += float(np.sum(reg_tot))
    buf[1:len(buf) - na] += reg_grad.T.reshape(-1)
    return buf


# ---------------------------------------------------------------------------
# src/RydbergTools.jl (model builders used by the configs)
# ---------------------------------------------------------------------------
_S2 = math.sqrt(2.0)


def rydberg_hamiltonian_symmetric_blockaded(phi, eps, delta):
    """RydbergTools.jl:31-39."""
    a = np.exp(-1j * phi) * (1 + eps)
    b = np.exp(1j * phi) * (1 + eps)
    H = np.zeros((5, 5), np.complex128)
    H[1, 3] = a / 2
    H[2, 4] = a / _S2
    H[3, 1] = b / 2
    H[3, 3] = delta
    H[4, 2] = b / _S2
    H[4, 4] = delta
    return H


def rydberg_hamiltonian_full_blockaded(phi, eps, delta):
    """RydbergTools.jl:71-81."""
    a = np.exp(-1j * phi) * (1 + eps)
    b = np.exp(1j * phi) * (1 + eps)
    H = np.zeros((7, 7), np.complex128)
    H[1, 4] = a / 2
    H[2, 5] = a / 2
    H[3, 6] = a / _S2
    H[4, 1] = b / 2
    H[4, 4] = delta
    H[5, 2] = b / 2
    H[5, 5] = delta
    H[6, 3] = b / _S2
    H[6, 6] = delta
    return H


def rydberg_hamiltonian_full(phi, O1, O2, d1, d2, B):
    """RydbergTools.jl:118-130."""
    em = np.exp(-1j * phi)
    ep = np.exp(1j * phi)
    H = np.zeros((9, 9), np.complex128)
    H[1, 4] = em * O1 / 2
    H[2, 5] = em * O2 / 2
    H[3, 6] = em * O1 / 2
    H[3, 7] = em * O2 / 2
    H[4, 1] = ep * O1 / 2
    H[4, 4] = d1
    H[5, 2] = ep * O2 / 2
    H[5, 5] = d2
    H[6, 3] = ep * O1 / 2
    H[6, 6] = d1
    H[6, 8] = em * O2 / 2
    H[7, 3] = ep * O2 / 2
    H[7, 7] = d2
    H[7, 8] = em * O1 / 2
    H[8, 6] = ep * O2 / 2
    H[8, 7] = ep * O1 / 2
    H[8, 8] = d1 + d2 + B
    return H


def cz_with_1q_phase_symmetric(theta):
    """RydbergTools.jl:160-162."""
    return np.diag([1.0, np.exp(1j * theta), np.exp(1j * (2 * theta + np.pi)), 0.0, 0.0]).astype(np.complex128)


def cz_with_1q_phase_full(theta, rydberg_dimension=5):
    """RydbergTools.jl:197-203."""
    d = np.zeros(4 + rydberg_dimension, np.complex128)
    d[0] = 1
    d[1:3] = np.exp(1j * theta)
    d[3] = np.exp(1j * (2 * theta + np.pi))
    return np.diag(d)
