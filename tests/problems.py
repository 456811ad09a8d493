"""Problem builders shared by the tests: the reference's test/example problems
(test/runtests.jl, examples/*.jl) and the SURVEY.md section 8d configs, each in
closure form (reference idiom, host-evaluated) and operator-basis form (device)."""
from __future__ import annotations

import math

import numpy as np

from robustgrape_amd import rydberg as R
from robustgrape_amd.types import ErrorSource, FidelityRobustGRAPEProblem, UnitaryRobustGRAPEProblem

T0_TEST = 2 * math.pi * 1.22     # runtests.jl:53
T0_TO = 7.613                    # examples/time_optimal_cz.jl:14
W_SYM = np.diag([1.0, 2.0, 1.0, 0.0, 0.0])   # runtests.jl:73
W_FULLBLK = np.diag([1.0, 1.0, 1.0, 1.0, 0.0, 0.0, 0.0])  # runtests.jl:492
W_FULL9 = np.diag([1.0, 1.0, 1.0, 1.0, 0.0, 0.0, 0.0, 0.0, 0.0])


def sym_problem(ntimes, t0=T0_TEST, errors=(), device=True):
    """d=5 symmetric blockaded CZ (runtests.jl:57-75); errors subset of {'amp','freq'}."""
    if device:
        H0 = R.rydberg_symmetric_blockaded_operator_basis()
        errs = [ErrorSource(R.symmetric_amplitude_error() if e == "amp" else R.symmetric_frequency_error())
                for e in errors]
        target = R.cz_symmetric_target()
    else:
        H0 = lambda t, p, xa: R.rydberg_hamiltonian_symmetric_blockaded(p[0], 0, 0)
        amp = lambda t, p, xa, e: (R.rydberg_hamiltonian_symmetric_blockaded(p[0], e, 0)
                                   - R.rydberg_hamiltonian_symmetric_blockaded(p[0], 0, 0))
        frq = lambda t, p, xa, e: (R.rydberg_hamiltonian_symmetric_blockaded(p[0], 0, e)
                                   - R.rydberg_hamiltonian_symmetric_blockaded(p[0], 0, 0))
        errs = [ErrorSource(amp if e == "amp" else frq) for e in errors]
        target = lambda xa: R.cz_with_1q_phase_symmetric(xa[0])
    up = UnitaryRobustGRAPEProblem(t0=t0, ntimes=ntimes, ndim=5, H0=H0, nb_additional_param=1,
                                   error_sources=errs)
    return FidelityRobustGRAPEProblem(up, W_SYM, target)


def fullblk_problem(ntimes, t0=T0_TO, errors=(), device=True):
    """d=7 full blockaded CZ (runtests.jl:474-494)."""
    if device:
        H0 = R.rydberg_full_blockaded_operator_basis()
        errs = [ErrorSource(R.full_blockaded_amplitude_error() if e == "amp"
                            else R.full_blockaded_frequency_error()) for e in errors]
        target = R.cz_full_target(rydberg_dimension=3)
    else:
        H0 = lambda t, p, xa: R.rydberg_hamiltonian_full_blockaded(p[0], 0, 0)
        amp = lambda t, p, xa, e: (R.rydberg_hamiltonian_full_blockaded(p[0], e, 0)
                                   - R.rydberg_hamiltonian_full_blockaded(p[0], 0, 0))
        frq = lambda t, p, xa, e: (R.rydberg_hamiltonian_full_blockaded(p[0], 0, e)
                                   - R.rydberg_hamiltonian_full_blockaded(p[0], 0, 0))
        errs = [ErrorSource(amp if e == "amp" else frq) for e in errors]
        target = lambda xa: R.cz_with_1q_phase_full(xa[0], rydberg_dimension=3)
    up = UnitaryRobustGRAPEProblem(t0=t0, ntimes=ntimes, ndim=7, H0=H0, nb_additional_param=1,
                                   error_sources=errs)
    return FidelityRobustGRAPEProblem(up, W_FULLBLK, target)


# sector layouts of the d = 9 Rydberg model (GrapePlan.sectors()): with equal Rabi frequencies and
# detunings the atom-swap symmetry splits the 4-level block (include/grape.h GRAPE_OPT_NO_SYMMETRY,
# csrc/grape_symmetry.hpp) -- one 3-level sector + two 2-level ones; single-atom error sources
# (C3) break the symmetry and keep the permutation sectors.
FULL9_SYM = ((3, 1), (2, 2))
FULL9_PERM = ((4, 1), (2, 2))


def full9_problem(ntimes=512, t0=T0_TO, nerr=0, device=True, B=10.0):
    """SURVEY.md 8d C2 (nerr=0) / C3 (nerr=4): d=9 rydberg_hamiltonian_full, Omega=1, B=10."""
    kinds = [("rabi", 1), ("rabi", 2), ("det", 1), ("det", 2)][:nerr]
    if device:
        H0 = R.rydberg_full_operator_basis(1.0, 1.0, 0.0, 0.0, B)
        errs = [ErrorSource(R.full_rabi_error(w) if k == "rabi" else R.full_detuning_error(w))
                for k, w in kinds]
        target = R.cz_full_target()
    else:
        H0 = lambda t, p, xa: R.rydberg_hamiltonian_full(p[0], 1, 1, 0, 0, B)

        def mk(k, w):
            def herr(t, p, xa, e):
                args = [1.0, 1.0, 0.0, 0.0]
                if k == "rabi":
                    args[w - 1] = 1.0 + e
                else:
                    args[1 + w] = e
                return R.rydberg_hamiltonian_full(p[0], *args, B) - R.rydberg_hamiltonian_full(p[0], 1, 1, 0, 0, B)
            return herr
        errs = [ErrorSource(mk(k, w)) for k, w in kinds]
        target = lambda xa: R.cz_with_1q_phase_full(xa[0])
    up = UnitaryRobustGRAPEProblem(t0=t0, ntimes=ntimes, ndim=9, H0=H0, nb_additional_param=1,
                                   error_sources=errs)
    return FidelityRobustGRAPEProblem(up, W_FULL9, target)


def evered_pulse(ntimes=1000):
    """runtests.jl:127-138: the Evered et al. time-optimal CZ pulse."""
    t0 = 2 * math.pi * 1.22
    A, w0, p0, d0 = 0.7701624, 0.97525275, -0.97449603, -0.04319765
    theta = 2.0802725844516097
    ts = np.linspace(0, t0, ntimes)
    phis = A * np.cos(w0 * ts - p0) + d0 * ts
    return np.concatenate([phis, [theta]])


def max_step_norm(fp, X, nparam=1):
    """max over rows of X and steps k of |dt H0(k, x_k, x_add)|_1: the exponentials' regime.
    Up to 0.25 every implementation here and the reference evaluate exp without squaring (Taylor
    12 / Pade 5); above it the engines differ in algorithm (the chunk walks: Taylor 30 of A / 2^s
    at |A / 2^s|_1 <= 3.2; the row groups and Julia: Pade 7 / 9 / 13, squaring from 5.4)."""
    up = fp.unitary_problem
    dt = up.t0 / up.ntimes
    X = np.atleast_2d(np.asarray(X, np.float64))
    na = up.nb_additional_param
    best = 0.0
    for x in X:
        xm = x[:len(x) - na].reshape(up.ntimes, nparam)
        xa = x[len(x) - na:]
        for k in range(up.ntimes):
            H = np.asarray(up.H0(k + 1, xm[k], xa))
            best = max(best, dt * np.abs(H).sum(axis=0).max())
    return best


def short_steps(fp, X, nparam=1):
    """True when every step of every row is in the no-squaring range (the T2s tier applies)."""
    return max_step_norm(fp, X, nparam) <= 0.25


# Julia's exp! squares from |A|_1 > 5.4 (Pade 13's theta): up to there no tolerance scaling
JULIA_THETA13 = 5.4


def fd_tier(fp, X, nparam=1):
    """(relative, absolute) tolerance of eps-FD quantities (F_dx) for these rows: the short-step
    T2s tier (1e-7 max|ref| + 1e-9) when no step needs more than Taylor 12 / Pade 5, else the T2
    tier (1e-6 max|ref| + 1e-7), scaled by max(1, max_k |dt H_k|_1 / 5.4) beyond Julia's Pade-13
    threshold: there the reference squares s = ceil(log2(|A|_1 / 5.4)) times and its own rounding
    -- the u / eps noise of (E' - E) / eps -- grows like 2^s in any implementation (measured:
    profiles/r04/highnorm_study.txt, Julia's D1 error against an extended-precision evaluation is
    1.6e-7 at |A|_1 = 3, 2e-6 at 30, 5e-6 at 80; the walks' Taylor 30 matches it at every norm)."""
    n = max_step_norm(fp, X, nparam)
    if n <= 0.25:
        return 1e-7, 1e-9
    f = max(1.0, n / JULIA_THETA13)
    return 1e-6 * f, 1e-7 * f


def fd_factor(fp, X, nparam=1):
    """The step-norm factor of the FD tiers (fd_tier's rule): 1 up to Julia's Pade-13
    threshold |dt H_k|_1 = 5.4, max_k |dt H_k|_1 / 5.4 beyond it (the reference squares there and its
    u / eps noise grows like 2^s).  Used for the tiers fd_tier does not return (T2 of uncontracted
    tensors and sensitivities, T3 of the mixed stencils)."""
    return max(1.0, max_step_norm(fp, X, nparam) / JULIA_THETA13)


def tensor_factor(fp, X, nparam=1):
    """The step-norm factor for UNCONTRACTED finite-difference tensors (U_dx, U_derr, U_derr_dx of
    calculate_unitary_and_derivatives): max(1, max_k |dt H_k|_1) beyond the no-squaring range, like
    T0.  An entry of (E' - E) / eps carries the exponential's own rounding, ~u |A|_1 per entry, over
    eps; the traces of the fidelity path average it (fd_factor's 5.4 rule), a single tensor entry
    does not."""
    n = max_step_norm(fp, X, nparam)
    return 1.0 if n <= 0.25 else max(1.0, n)


def random_x(ntimes, seed, nparam=1, small=False):
    """x_main = 2pi*U (runtests.jl:335) or 2pi*0.001*U (examples/time_optimal_cz.jl:32); theta = 2pi*U."""
    rng = np.random.default_rng(seed)
    scale = 2 * math.pi * (0.001 if small else 1.0)
    return np.concatenate([scale * rng.uniform(size=ntimes * nparam), [2 * math.pi * rng.uniform()]])


def xadd_err_problem(d, ntimes, nerr=2, device=True):
    """Error sources together with an H0 that reads x_add (UnitaryCalculations.jl:57-64, 87-95,
    140-151): the d=5 symmetric (runtests.jl:57-75) or d=9 full Rydberg
    problem with a second additional parameter x_add[1], a global detuning on a diagonal
    occupation operator, and an error source whose strength is modulated by cos(x_add[1]).
    x_add[0] stays the target's single-qubit phase.  device=False: the same physics as plain
    closures (the reference's idiom), which the table path and the oracle evaluate."""
    from robustgrape_amd.operators import (FN_COS, FN_LINEAR, VAR_XADD, OperatorBasisError,
                                           OperatorBasisHamiltonian, Term)
    base = sym_problem(ntimes, errors=("amp", "freq")[:nerr]) if d == 5 else full9_problem(ntimes, nerr=nerr)
    up = base.unitary_problem
    Nr = np.diag(np.linspace(0.0, 1.0, d)).astype(np.complex128)
    H0 = OperatorBasisHamiltonian(list(up.H0.terms) + [Term(Nr, var=VAR_XADD, index=1, func=FN_LINEAR, scale=0.5)])
    errs = []
    for e, es in enumerate(up.error_sources):
        terms = list(es.Herror.terms)
        if e == 0:
            terms.append(Term(Nr, var=VAR_XADD, index=1, func=FN_COS, scale=0.3))
        errs.append(ErrorSource(OperatorBasisError(terms)))
    target = base.target_unitary
    if not device:
        Hdev, tdev, edev = H0, target, errs
        H0 = lambda t, x, xa: Hdev(t, x, xa)  # noqa: E731
        target = lambda xa: tdev(xa)  # noqa: E731
        errs = [ErrorSource(lambda t, x, xa, e, es=es: es.Herror(t, x, xa, e)) for es in edev]
    up2 = UnitaryRobustGRAPEProblem(t0=up.t0, ntimes=ntimes, ndim=d, H0=H0, nb_additional_param=2,
                                    error_sources=errs)
    return FidelityRobustGRAPEProblem(up2, base.projector, target)


def xadd_x(ntimes, seed):
    """Control vector of xadd_err_problem: x_main = 2pi U, theta = 2pi U, detuning U[-0.5, 0.5)."""
    rng = np.random.default_rng(seed)
    return np.concatenate([2 * math.pi * rng.uniform(size=ntimes), [2 * math.pi * rng.uniform(), rng.uniform(-0.5, 0.5)]])


def with_decay(fp, gamma=0.4, levels=(4,), device=True):
    """fp with a non-Hermitian H0: -i gamma/2 on each of `levels` (a Rydberg-decay term, the
    reference accepts any H0: UnitaryCalculations.jl:45-47 exponentiates and LU-inverts it).
    Device form: one more OperatorBasisHamiltonian term; oracle form: a wrapped closure."""
    up = fp.unitary_problem
    G = np.zeros((up.ndim, up.ndim), np.complex128)
    for l in levels:
        G[l, l] = 1.0
    if device:
        from robustgrape_amd.operators import OperatorBasisHamiltonian, Term
        H0 = OperatorBasisHamiltonian(list(up.H0.terms) + [Term(G, scale=-0.5j * gamma)])
    else:
        h = up.H0
        H0 = lambda t, p, xa: np.asarray(h(t, p, xa), np.complex128) - 0.5j * gamma * G  # noqa: E731
    return fp.replace(unitary_problem=up.replace(H0=H0))


def as_closures(fp):
    """The same problem with plain-function H0 / Herror / target (the reference's idiom,
    Types.jl:13,25,55): the engine then takes the host-table (closure) path."""
    from robustgrape_amd.types import ErrorSource as ES
    up = fp.unitary_problem
    h, tgt = up.H0, fp.target_unitary
    wrap_err = lambda f: (lambda t, p, xa, e: f(t, p, xa, e))  # noqa: E731
    errs = [ES(wrap_err(es.Herror)) for es in up.error_sources]
    up2 = up.replace(H0=lambda t, p, xa: h(t, p, xa), error_sources=errs)
    return fp.replace(unitary_problem=up2, target_unitary=lambda xa: tgt(xa))
