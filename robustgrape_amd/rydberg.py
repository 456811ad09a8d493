"""Rydberg two-atom models and CZ targets (src/RydbergTools.jl), in two forms.

* ``rydberg_hamiltonian_*`` / ``cz_with_1q_phase_*`` return the matrices,
  like the reference (closure form, host-evaluated).
* ``*_operator_basis`` return the same models as operator-basis descriptors
  (:mod:`robustgrape_amd.operators`) so the GPU builds H on device:
  a phase-controlled drive is H(phi) = cos(phi) Hc + sin(phi) Hs + Hd, with
  Hc/Hs the real/imaginary patterns of the e^{-i phi} couplings.
"""
from __future__ import annotations

import math

import numpy as np

from .operators import (FN_CIS, FN_COS, FN_ONE, FN_SIN, VAR_ONE, VAR_X, VAR_XADD,
                        OperatorBasisError, OperatorBasisHamiltonian, OperatorBasisTarget, Term)

_S2 = math.sqrt(2.0)

# (row, col, weight) of the upper-triangle e^{-i phi} couplings, 0-based.
_SYM_COUPLINGS = [(1, 3, 0.5, 1), (2, 4, 1.0 / _S2, 1)]                  # RydbergTools.jl:31-39
_FULLBLK_COUPLINGS = [(1, 4, 0.5, 1), (2, 5, 0.5, 1), (3, 6, 1.0 / _S2, 1)]  # :71-81
# d=9 full model (:118-130): last entry says which Rabi frequency (1 or 2) drives it
_FULL_COUPLINGS = [(1, 4, 0.5, 1), (2, 5, 0.5, 2), (3, 6, 0.5, 1), (3, 7, 0.5, 2),
                   (6, 8, 0.5, 2), (7, 8, 0.5, 1)]


def rydberg_hamiltonian_symmetric_blockaded(phi, eps, delta):
    """RydbergTools.jl:31-39 (basis |00>,|01>,|11>,|0r>,|W>)."""
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
    """RydbergTools.jl:71-81 (basis |00>,|01>,|10>,|11>,|0r>,|r0>,|W'>)."""
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
    """RydbergTools.jl:118-130 (basis |00>,|01>,|10>,|11>,|0r>,|r0>,|1r>,|r1>,|rr>)."""
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


def unwrap_phase(phi):
    """RydbergTools.jl:221-232 (plotting helper)."""
    p = np.mod(np.array(phi, dtype=np.float64), 2 * np.pi)
    for i in range(len(p) - 1):
        if p[i + 1] - p[i] > np.pi:
            p[i + 1:] -= 2 * np.pi
        elif p[i + 1] - p[i] < -np.pi:
            p[i + 1:] += 2 * np.pi
    return p


# ---------------------------------------------------------------------------
# operator-basis forms
# ---------------------------------------------------------------------------

def _phase_pair(ndim, couplings, scale_of):
    """Hc, Hs with H_coupling(phi) = cos(phi) Hc + sin(phi) Hs."""
    Hc = np.zeros((ndim, ndim), np.complex128)
    Hs = np.zeros((ndim, ndim), np.complex128)
    for r, c, w, which in couplings:
        s = w * scale_of(which)
        if s == 0.0:
            continue
        Hc[r, c] += s
        Hc[c, r] += s
        Hs[r, c] += -1j * s   # e^{-i phi} above the diagonal
        Hs[c, r] += 1j * s    # e^{+i phi} below
    return Hc, Hs


def _drive_terms(Hc, Hs, param=0):
    return [Term(op=Hc, var=VAR_X, index=param, func=FN_COS),
            Term(op=Hs, var=VAR_X, index=param, func=FN_SIN)]


def rydberg_symmetric_blockaded_operator_basis(eps=0.0, delta=0.0, param=0):
    """H0(nt, x, x_add) = rydberg_hamiltonian_symmetric_blockaded(x[param], eps, delta)."""
    Hc, Hs = _phase_pair(5, _SYM_COUPLINGS, lambda _: 1.0 + eps)
    terms = _drive_terms(Hc, Hs, param)
    if delta != 0.0:
        terms.append(Term(op=np.diag([0, 0, 0, delta, delta]).astype(np.complex128)))
    return OperatorBasisHamiltonian(terms)


def rydberg_full_blockaded_operator_basis(eps=0.0, delta=0.0, param=0):
    """H0 = rydberg_hamiltonian_full_blockaded(x[param], eps, delta)."""
    Hc, Hs = _phase_pair(7, _FULLBLK_COUPLINGS, lambda _: 1.0 + eps)
    terms = _drive_terms(Hc, Hs, param)
    if delta != 0.0:
        terms.append(Term(op=np.diag([0, 0, 0, 0, delta, delta, delta]).astype(np.complex128)))
    return OperatorBasisHamiltonian(terms)


def rydberg_full_operator_basis(O1=1.0, O2=1.0, d1=0.0, d2=0.0, B=10.0, param=0):
    """H0 = rydberg_hamiltonian_full(x[param], O1, O2, d1, d2, B)."""
    Hc, Hs = _phase_pair(9, _FULL_COUPLINGS, lambda w: O1 if w == 1 else O2)
    terms = _drive_terms(Hc, Hs, param)
    Hd = np.diag([0, 0, 0, 0, d1, d2, d1, d2, d1 + d2 + B]).astype(np.complex128)
    if np.any(Hd != 0):
        terms.append(Term(op=Hd))
    return OperatorBasisHamiltonian(terms)


def symmetric_amplitude_error(param=0):
    """Herror = H(phi, err, 0) - H(phi, 0, 0) for the d=5 model (runtests.jl:59)."""
    Hc, Hs = _phase_pair(5, _SYM_COUPLINGS, lambda _: 1.0)
    return OperatorBasisError(_drive_terms(Hc, Hs, param))


def symmetric_frequency_error():
    """Herror = H(phi, 0, err) - H(phi, 0, 0) for the d=5 model (runtests.jl:498)."""
    return OperatorBasisError([Term(op=np.diag([0, 0, 0, 1, 1]).astype(np.complex128))])


def full_blockaded_amplitude_error(param=0):
    Hc, Hs = _phase_pair(7, _FULLBLK_COUPLINGS, lambda _: 1.0)
    return OperatorBasisError(_drive_terms(Hc, Hs, param))


def full_blockaded_frequency_error():
    return OperatorBasisError([Term(op=np.diag([0, 0, 0, 0, 1, 1, 1]).astype(np.complex128))])


def full_rabi_error(which, param=0):
    """d=9: Omega_which -> Omega_which + err."""
    Hc, Hs = _phase_pair(9, _FULL_COUPLINGS, lambda w: 1.0 if w == which else 0.0)
    return OperatorBasisError(_drive_terms(Hc, Hs, param))


def full_detuning_error(which):
    """d=9: delta_which -> err."""
    d = np.zeros(9)
    for i in ((4, 6, 8) if which == 1 else (5, 7, 8)):
        d[i] = 1.0
    return OperatorBasisError([Term(op=np.diag(d).astype(np.complex128))])


def cz_symmetric_target(index=0):
    """target_unitary(x_add) = cz_with_1q_phase_symmetric(x_add[index])."""
    e = lambda k: np.diag([1.0 if i == k else 0.0 for i in range(5)]).astype(np.complex128)
    return OperatorBasisTarget([
        Term(op=e(0)),
        Term(op=e(1), var=VAR_XADD, index=index, func=FN_CIS),
        Term(op=e(2), var=VAR_XADD, index=index, func=FN_CIS, a=2.0, b=math.pi),
    ])


def cz_full_target(index=0, rydberg_dimension=5):
    """target_unitary(x_add) = cz_with_1q_phase_full(x_add[index]; rydberg_dimension)."""
    n = 4 + rydberg_dimension
    def diag(ks):
        return np.diag([1.0 if i in ks else 0.0 for i in range(n)]).astype(np.complex128)
    return OperatorBasisTarget([
        Term(op=diag((0,))),
        Term(op=diag((1, 2)), var=VAR_XADD, index=index, func=FN_CIS),
        Term(op=diag((3,)), var=VAR_XADD, index=index, func=FN_CIS, a=2.0, b=math.pi),
    ])
