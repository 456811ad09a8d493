"""Closure problems above 12 levels (the reference takes closures at any d,
Types.jl:13,35,55): the host tabulates H at every call site (robustgrape_amd/tables.py), the
dense engine exponentiates the tables (grape_dense.hip launch_table_variants) and the general
path assembles the derivatives and the fidelity terms (grape_unitary.hip), one evaluation at a
time.  Against the oracle on the same closures; tiers as tests/test_gpu_dense.py, the FD tiers
scaled by max(1, max_k |dt H_k|_1) (tests/problems.py fd_tier)."""
import numpy as np
import pytest

from tests import problems as P

pytestmark = pytest.mark.gpu
T1 = 1e-12
T2, T2_ABS = 1e-6, 1e-7
T3, T3_ABS = 1e-5, 1e-7


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _fp(d, nt, nerr, phase=False):
    from robustgrape_amd import synthetic as S
    fp = S.dense_error_problem(d=d, ntimes=nt, dt=0.5, rank=min(8, d), nerr=nerr, phase=phase) if nerr or phase \
        else S.dense_problem(d=d, ntimes=nt, dt=0.5, rank=min(8, d))
    return P.as_closures(fp)


def _x(fp, seed):
    up = fp.unitary_problem
    rng = np.random.default_rng(seed)
    return np.concatenate([rng.uniform(-1.0, 1.0, size=2 * up.ntimes), rng.uniform(0, 2 * np.pi, size=up.nb_additional_param)])


@pytest.mark.parametrize("d,nt,nerr,phase", [(16, 12, 0, False), (16, 9, 2, False), (24, 6, 1, True), (13, 5, 0, True)])
def test_closures_above_12_levels_match_oracle(d, nt, nerr, phase):
    from oracle import grape_oracle as O
    from robustgrape_amd.engine import GrapePlan
    fp = _fp(d, nt, nerr, phase)
    X = np.stack([_x(fp, 900 + s) for s in range(2)])
    plan = GrapePlan(fp, nparam=2, max_batch=2)
    try:
        F, Fdx, Fd2, Fd2dx = plan.fidelity_grad(X)
    finally:
        plan.close()
    for b in range(len(X)):
        ref = O.calculate_fidelity_and_derivatives(fp, X[b])
        t2, t2a = P.fd_tier(fp, X[b], nparam=2)
        fac = P.fd_factor(fp, X[b], nparam=2)
        assert abs(F[b] - ref[0]) <= T1, (F[b], ref[0])
        checks = [(Fdx[b], ref[1], t2, t2a)]
        if nerr:
            checks += [(Fd2[b], ref[2], T2 * fac, T2_ABS), (Fd2dx[b], ref[3], T3 * fac, T3_ABS)]
        for n, (a, r, t, ta) in enumerate(checks):
            err, scale = np.max(np.abs(a - r)), np.max(np.abs(r))
            print(f"d{d} nt{nt} ne{nerr} b{b} term{n}: {err:.2e}/{scale:.2e}")
            assert err <= t * scale + ta, (n, err, scale)


def test_closure_unitary_derivatives_above_12_levels():
    from oracle import grape_oracle as O
    from robustgrape_amd import calculate_unitary_and_derivatives
    fp = _fp(16, 7, 2)
    x = _x(fp, 77)
    ref = O.calculate_unitary_and_derivatives(fp.unitary_problem, x)
    got = calculate_unitary_and_derivatives(fp.unitary_problem, x)
    fac = P.tensor_factor(fp, x, nparam=2)  # uncontracted tensors (tests/problems.py)
    assert np.max(np.abs(got[0] - ref[0])) <= T1 * fac
    for n, (t, ta) in ((1, (T2, T2_ABS)), (3, (T2, T2_ABS)), (4, (T3, T3_ABS))):
        a, b = np.asarray(got[n]), np.asarray(ref[n])
        assert a.shape == b.shape
        assert np.max(np.abs(a - b)) <= t * fac * np.max(np.abs(b)) + ta, (n, np.max(np.abs(a - b)))


def test_non_hermitian_closures_above_12_levels_are_refused():
    from robustgrape_amd.engine import GrapePlan
    fp = _fp(16, 4, 0)
    up = fp.unitary_problem
    h = up.H0
    G = np.zeros((16, 16), complex)
    G[3, 3] = 1.0
    bad = fp.replace(unitary_problem=up.replace(H0=lambda t, p, xa: np.asarray(h(t, p, xa)) - 0.2j * G))
    plan = GrapePlan(bad, nparam=2, max_batch=1)
    try:
        with pytest.raises(ValueError, match="Hermitian"):
            plan.fidelity_grad(_x(bad, 5)[None, :])
    finally:
        plan.close()
