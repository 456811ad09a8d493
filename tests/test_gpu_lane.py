"""Lane-matrix exponential (robustgrape_amd/csrc/grape_lane.hpp k_expm_lane): for d <= 3 one lane
owns one whole propagator (generator and exponential; every stored variant: the nominal one and,
with error sources, the FD and error variants) instead of a row group of d lanes.  The
arithmetic is the row-group kernel's operation for operation, so the two paths must agree
BITWISE (GRAPE_OPT_NO_LANE selects the row groups), and both must match the oracle
(UnitaryCalculations.jl:45-90, FidelityCalculations.jl:56-113).

Covered: the Rydberg sector class S = 2 (d = 9 -> 4 + 2 x 2, d = 5 -> 2 x 2, d = 7 -> 3 x 2; the
S = 4 class keeps the row groups), whole-matrix problems at d = 2, 3 (and d = 4, row groups),
error sources (C3's 4 sources on d = 9 sectors, amplitude + frequency on d = 5: every output,
F_d2err and F_d2err_dx included, bitwise), chunk starts (N_t = 1, 3), parked high-norm steps
(Pade 7/9/13 items handed to k_expm_high), x_add-dependent H0.  Sector problems without error
sources take k_expm_chain_lane (propagators and chunk chains per lane; k_scan starts from the
chunk totals): the chunk-start cases and the parked steps (whose chunks k_scan rechains from E)
exercise it bitwise against k_scan's own Phase A.  Both runs turn the chunk walks off
(GRAPE_OPT_NO_WALK): the walks serve the no-error sector classes by default and are tested in
tests/test_gpu_walk.py."""
import numpy as np
import pytest

from tests import problems as P

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _run(fp, X, monkeypatch, lane, nparam=1):
    from robustgrape_amd.engine import GrapePlan
    from robustgrape_amd.operators import OPT_NO_LANE, OPT_NO_WALK
    opts = OPT_NO_WALK | (0 if lane else OPT_NO_LANE)
    pl = GrapePlan(fp, nparam=nparam, device=0, max_batch=max(len(X), 65), options=opts)  # > 64: stream path
    try:
        return pl.fidelity_grad(np.concatenate([X] * (65 // len(X) + 1))[:65])
    finally:
        pl.close()


def _bitwise(fp, X, monkeypatch, nparam=1):
    a = _run(fp, X, monkeypatch, True, nparam)
    b = _run(fp, X, monkeypatch, False, nparam)
    for x, y in zip(a, b):  # F, F_dx (and the empty error outputs)
        assert np.array_equal(np.asarray(x), np.asarray(y)), np.max(np.abs(np.asarray(x) - np.asarray(y)))
    return a[0], a[1]


def _dense_problem(d, nt, seed):
    """A d-level problem with two drive terms (no block structure: whole-matrix lane path)."""
    from robustgrape_amd.operators import (FN_COS, FN_SIN, VAR_X, OperatorBasisHamiltonian,
                                           OperatorBasisTarget, Term)
    from robustgrape_amd.types import FidelityRobustGRAPEProblem, UnitaryRobustGRAPEProblem
    rng = np.random.default_rng(seed)
    M = rng.normal(size=(d, d)) + 1j * rng.normal(size=(d, d))
    Hx = (M + M.conj().T) / 2
    Hz = np.diag(rng.normal(size=d)).astype(np.complex128)
    Hy = 1j * (np.triu(np.ones((d, d)), 1) - np.tril(np.ones((d, d)), -1)).astype(np.complex128)
    H0 = OperatorBasisHamiltonian([Term(Hz), Term(Hx, var=VAR_X, index=0, func=FN_COS),
                                   Term(Hy, var=VAR_X, index=0, func=FN_SIN, scale=0.5)])
    up = UnitaryRobustGRAPEProblem(t0=2.0, ntimes=nt, ndim=d, H0=H0, nb_additional_param=0)
    U0 = np.linalg.qr(rng.normal(size=(d, d)) + 1j * rng.normal(size=(d, d)))[0]
    W = np.diag([1.0] * (d - 1) + [0.0])
    return FidelityRobustGRAPEProblem(up, W, OperatorBasisTarget([Term(U0)]))


@pytest.mark.parametrize("name,fp,nt", [
    ("full9", lambda: P.full9_problem(40), 40),
    ("full9-chunk-starts", lambda: P.full9_problem(3), 3),
    ("full9-one-step", lambda: P.full9_problem(1), 1),
    ("sym5", lambda: P.sym_problem(24), 24),
    ("fullblk7", lambda: P.fullblk_problem(24), 24),
    ("full9-parked", lambda: P.full9_problem(6, t0=40.0), 6),
    ("full9-C3-errors", lambda: P.full9_problem(24, nerr=4), 24),
    ("sym5-amp-freq", lambda: P.sym_problem(20, errors=("amp", "freq")), 20),
])
def test_lane_bitwise_and_oracle(name, fp, nt, monkeypatch):
    from oracle import grape_oracle as O
    f = fp()
    X = np.stack([P.random_x(nt, 900 + s) for s in range(5)])
    F, g = _bitwise(f, X, monkeypatch)
    F0, g0 = O.calculate_fidelity_and_derivatives(f, X[3])[:2]
    ef, eg, sc = abs(F[3] - F0), np.max(np.abs(g[3] - g0)), np.max(np.abs(g0))
    print(f"{name}: |F-F_oracle| {ef:.2e}  max|F_dx-oracle| {eg:.2e} (scale {sc:.2e})")
    assert ef <= 1e-12
    assert eg <= 1e-6 * sc + 1e-7


@pytest.mark.parametrize("d", [2, 3, 4])
def test_lane_whole_matrix_dims(d, monkeypatch):
    from oracle import grape_oracle as O
    nt = 16
    f = _dense_problem(d, nt, 40 + d)
    rng = np.random.default_rng(d)
    X = rng.uniform(-2, 2, size=(4, nt))
    F, g = _bitwise(f, X, monkeypatch)
    F0, g0 = O.calculate_fidelity_and_derivatives(f, X[1])[:2]
    print(f"d={d}: |F-F_oracle| {abs(F[1] - F0):.2e}  max|F_dx-oracle| {np.max(np.abs(g[1] - g0)):.2e}")
    assert abs(F[1] - F0) <= 1e-12
    assert np.max(np.abs(g[1] - g0)) <= 1e-6 * np.max(np.abs(g0)) + 1e-7


def test_lane_xadd_dependent_h0(monkeypatch):
    """x_add read by H0 (the S = 2 sectors of the d = 5 problem take the lane propagators)."""
    f = P.xadd_err_problem(5, 12, nerr=0)
    X = np.stack([P.xadd_x(12, 30 + s) for s in range(3)])
    _bitwise(f, X, monkeypatch)
