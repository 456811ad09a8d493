"""Every compiled dimension of the small-d engine (GRAPE_DIMS: d = 2..12) against the
oracle, with and without error sources, on random Hermitian operator bases with the
Rydberg-style cos/sin phase control plus a linear amplitude control (np = 2) and a
cis target phase (x_add).  The oracle evaluates the same operators through plain
closures, the reference's idiom (src/Types.jl:10,25,50)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
T1 = 1e-12
T2, T2_ABS = 1e-6, 1e-7
T3, T3_ABS, T3_XADD_ABS = 1e-5, 1e-7, 1e-5


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def random_problem(d, ntimes, nerr, device, seed=0):
    from robustgrape_amd.operators import (FN_CIS, FN_COS, FN_LINEAR, FN_SIN, VAR_X, VAR_XADD,
                                           OperatorBasisError, OperatorBasisHamiltonian,
                                           OperatorBasisTarget, Term)
    from robustgrape_amd.types import ErrorSource, FidelityRobustGRAPEProblem, UnitaryRobustGRAPEProblem
    rng = np.random.default_rng(seed + 97 * d)

    def herm():
        G = rng.normal(size=(d, d)) + 1j * rng.normal(size=(d, d))
        H = (G + G.conj().T) / 2
        return H / np.abs(H).sum(axis=0).max()
    Hd, Hc, Hs, Ha = herm(), herm(), herm(), herm()
    H0 = OperatorBasisHamiltonian([Term(Hd), Term(Hc, var=VAR_X, index=0, func=FN_COS),
                                   Term(Hs, var=VAR_X, index=0, func=FN_SIN),
                                   Term(Ha, var=VAR_X, index=1, func=FN_LINEAR)])
    errs = [ErrorSource(OperatorBasisError([Term(herm())])) for _ in range(nerr)]
    P1 = np.zeros((d, d), complex)
    P1[1, 1] = 1.0
    tgt = OperatorBasisTarget([Term(np.eye(d, dtype=complex) - P1), Term(P1, var=VAR_XADD, index=0, func=FN_CIS)])
    if not device:  # the same problem as plain closures
        Hdev, tdev, edev = H0, tgt, errs
        H0 = lambda t, x, xa: Hdev(t, x, xa)  # noqa: E731
        tgt = lambda xa: tdev(xa)  # noqa: E731
        errs = [ErrorSource(lambda t, x, xa, e, es=es: es.Herror(t, x, xa, e)) for es in edev]
    up = UnitaryRobustGRAPEProblem(t0=2.0 * ntimes / 16, ntimes=ntimes, ndim=d, H0=H0, nb_additional_param=1,
                                   error_sources=errs)
    half = max(1, d // 2)
    W = np.diag([1.0] * half + [0.0] * (d - half))
    return FidelityRobustGRAPEProblem(up, W, tgt)


@pytest.mark.parametrize("d", list(range(2, 13)))
@pytest.mark.parametrize("nerr,nt", [(0, 21), (2, 9)])
def test_every_small_dimension_matches_live_oracle(d, nerr, nt):
    from oracle import grape_oracle as O
    from robustgrape_amd import calculate_fidelity_and_derivatives
    rng = np.random.default_rng(d * 10 + nerr)
    x = np.concatenate([rng.uniform(-1, 1, size=2 * nt), [rng.uniform(0, 2 * np.pi)]])
    F0, g0, d20, d2dx0 = O.calculate_fidelity_and_derivatives(random_problem(d, nt, nerr, False), x)
    F, g, d2, d2dx = calculate_fidelity_and_derivatives(random_problem(d, nt, nerr, True), x)
    assert abs(F - F0) <= T1, (F, F0)
    assert np.max(np.abs(g - g0)) <= T2 * np.max(np.abs(g0)) + T2_ABS
    if nerr:
        nmain = len(x) - 1
        assert np.max(np.abs(d2 - d20)) <= T3 * np.max(np.abs(d20)) + T3_ABS
        assert np.max(np.abs(d2dx[:nmain] - d2dx0[:nmain])) <= T3 * np.max(np.abs(d2dx0[:nmain])) + T3_ABS
        from tests.xadd_pin import check_xadd, exact_rows
        check_xadd(f"dims_d{d}_nt{nt}", d2dx, d2dx0, nmain, exact_rows(random_problem(d, nt, nerr, True), x, 2))
