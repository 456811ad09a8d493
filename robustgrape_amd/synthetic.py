"""the synthetic dense-GEMM problem (d = 64, N_t = 1024).

    H(x_k) = H_d + x_{1,k} H_1 + x_{2,k} H_2

each H = (G + G^dagger)/2 from a complex Ginibre matrix G (seeds 64, 65, 66),
normalised to |H|_1 = 1; dt = 0.5 (t0 = 0.5 N_t); controls x ~ U[-1, 1)
(seed 67); np = 2, na = 0, no error sources; target = the Q factor of a
Ginibre matrix (seed 68); projector W = diag(1 x 16, 0 x 48).  |A|_1 =
dt |H|_1 <= 1.5, so the Pade degree m in {5, 7, 9} is data dependent.

The reference has no d = 64 problem (its tests stop at d = 7); this one exists
to exercise the dense (MFMA) engine.  ``dense_problem`` also builds smaller
members of the family (any d, N_t, projector rank) for the parity tests.
"""
from __future__ import annotations

import numpy as np

from .operators import (FN_LINEAR, VAR_X, OperatorBasisHamiltonian, OperatorBasisTarget, Term)
from .types import FidelityRobustGRAPEProblem, UnitaryRobustGRAPEProblem

C5_DIM, C5_NTIMES, C5_DT, C5_RANK = 64, 1024, 0.5, 16


def _ginibre(d, seed):
    rng = np.random.default_rng(seed)
    return rng.normal(size=(d, d)) + 1j * rng.normal(size=(d, d))


def _hermitian(d, seed):
    G = _ginibre(d, seed)
    H = (G + G.conj().T) / 2
    return H / np.abs(H).sum(axis=0).max()


def dense_operators(d, seeds=(64, 65, 66)):
    return [_hermitian(d, s) for s in seeds]


def dense_target(d, seed=68):
    Q, R = np.linalg.qr(_ginibre(d, seed))
    return Q


def dense_problem(d=C5_DIM, ntimes=C5_NTIMES, dt=C5_DT, rank=C5_RANK, scale=1.0):
    """The C5 family: np = 2 linear controls on Hermitian Ginibre operators.
    ``scale`` multiplies every operator (|A|_1 up to 1.5 scale: selects the Pade degrees)."""
    Hd, H1, H2 = [scale * h for h in dense_operators(d)]
    H0 = OperatorBasisHamiltonian([Term(Hd), Term(H1, var=VAR_X, index=0, func=FN_LINEAR),
                                   Term(H2, var=VAR_X, index=1, func=FN_LINEAR)])
    up = UnitaryRobustGRAPEProblem(t0=dt * ntimes, ntimes=ntimes, ndim=d, H0=H0, nb_additional_param=0)
    W = np.diag([1.0] * min(rank, d) + [0.0] * max(0, d - rank))
    return FidelityRobustGRAPEProblem(up, W, OperatorBasisTarget([Term(dense_target(d))]))


def dense_x(ntimes=C5_NTIMES, seed=67, nparam=2):
    """x ~ U[-1, 1), x[p + k*nparam] = control p at step k."""
    return np.random.default_rng(seed).uniform(-1.0, 1.0, size=ntimes * nparam)


def dense_error_problem(d=C5_DIM, ntimes=C5_NTIMES, dt=C5_DT, rank=C5_RANK, scale=1.0, nerr=2, phase=False):
    """C5 with error sources (the dense engine's error path): error 0 is an amplitude error on
    control 1 (Herror = err x_1 H_1, the reference idiom H(1 + err) - H), error 1 a static
    Hermitian Ginibre perturbation (seed 69).  phase=True adds one additional parameter, a
    phase theta on the first column of the target (target = Q (I - e0 e0^T) + Q e0 e0^T cis(theta)),
    so that F_dx_add and the target part of F_d2err_dx_add are exercised too."""
    from .operators import FN_CIS, VAR_XADD, OperatorBasisError
    from .types import ErrorSource
    fp = dense_problem(d, ntimes, dt, rank, scale)
    Hd, H1, H2 = [scale * h for h in dense_operators(d)]
    Hs = scale * _hermitian(d, 69)
    errs = [ErrorSource(OperatorBasisError([Term(H1, var=VAR_X, index=0, func=FN_LINEAR)])),
            ErrorSource(OperatorBasisError([Term(Hs)]))][:nerr]
    up = fp.unitary_problem.replace(error_sources=errs, nb_additional_param=1 if phase else 0)
    target = fp.target_unitary
    if phase:
        Q = dense_target(d)
        P0 = np.zeros((d, d), complex)
        P0[0, 0] = 1.0
        target = OperatorBasisTarget([Term(Q @ (np.eye(d) - P0)), Term(Q @ P0, var=VAR_XADD, index=0, func=FN_CIS)])
    return fp.replace(unitary_problem=up, target_unitary=target)
