"""General (non-Hermitian) H0 on the GPU against the oracle: a -i Gamma/2 Rydberg-decay term
makes the propagators non-unitary, so the chain is inverted by LU as the reference does
(UnitaryCalculations.jl:47, inv(cum_evo); grape_unitary.hip k_u_inverse) and the fidelity path
runs from the materialised derivatives (FidelityCalculations.jl:19-119; k_u_fid_head /
k_u_fid_contract).  Operator-basis plans select the path at creation, closure plans when the
host sees a non-Hermitian H0 table (GrapePlan.general_h0_for).

Tiers as tests/test_gpu_parity.py: F at T1 = 1e-12; F_dx at tests/problems.py fd_tier (the
short-step T2s tier 1e-7 max|ref| + 1e-9 when every |dt H|_1 <= 0.25, else the long-step T2 tier
scaled by the step norm: Julia's Pade 7/9/13 and the device's exponentials then differ in
algorithm, not only in rounding); with error sources the oracle's
closure idiom Herror = H(eps) - H(0) carries u/eps rounding (tests/test_gpu_analysis.py), so
F_d2err at T2 (1e-6) and F_d2err_dx at T3 (1e-5 max|ref| + 1e-7)."""
import numpy as np
import pytest

from tests import problems as P

pytestmark = pytest.mark.gpu
T1 = 1e-12
T2S, T2S_ABS = 1e-7, 1e-9
T2, T2_ABS = 1e-6, 1e-7
T3, T3_ABS = 1e-5, 1e-7


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _mk(kind, nt, errs, dev, gamma=0.4):
    if kind == "sym":
        fp = P.sym_problem(nt, errors=errs, device=dev)
        return P.with_decay(fp, gamma, (3, 4), dev)
    if kind == "fullblk":
        return P.with_decay(P.fullblk_problem(nt, errors=errs, device=dev), gamma, (5, 6), dev)
    return P.with_decay(P.full9_problem(nt, nerr=errs, device=dev), gamma, (3, 5, 7), dev)


def _check(got, ref, label, ne, tier=(T2S, T2S_ABS)):
    """tier: the F_dx tier (tests/problems.py fd_tier: T2s on short steps, else the scaled T2)."""
    errs = {"F": float(np.max(np.abs(np.asarray(got[0]) - ref[0])))}
    assert errs["F"] <= T1, (label, errs)
    for n, (t, ta) in enumerate([tier, (T2, T2_ABS), (T3, T3_ABS)], start=1):
        if n > 1 and ne == 0:
            break
        a, b = np.asarray(got[n]), np.asarray(ref[n])
        err, scale = float(np.max(np.abs(a - b))), float(np.max(np.abs(b)))
        errs[("F_dx", "F_d2err", "F_d2err_dx")[n - 1]] = f"{err:.2e}/{scale:.2e}"
        assert err <= t * scale + ta, (label, n, err, scale)
    print(label, errs)


CASES = [("sym", 7, ()), ("sym", 40, ("amp", "freq")), ("fullblk", 13, ("amp",)), ("full9", 24, 0),
         ("full9", 16, 2), ("sym", 1, ())]


@pytest.mark.parametrize("kind,nt,errs", CASES)
def test_decay_h0_matches_oracle(kind, nt, errs):
    from oracle import grape_oracle as O
    from robustgrape_amd import calculate_fidelity_and_derivatives
    x = P.random_x(nt, 300 + nt)
    ref = O.calculate_fidelity_and_derivatives(_mk(kind, nt, errs, False), x)
    got = calculate_fidelity_and_derivatives(_mk(kind, nt, errs, True), x)
    assert ref[0] < 1.0 - 1e-6  # the decay is visible: the propagators are not unitary
    ne = len(errs) if isinstance(errs, tuple) else errs
    _check(got, ref, f"general_{kind}_nt{nt}_ne{ne}", ne, P.fd_tier(_mk(kind, nt, errs, False), x))


def test_decay_h0_closures_take_the_general_path():
    """The same physics as plain closures (host tables): the plan moves to the general path."""
    from oracle import grape_oracle as O
    from robustgrape_amd.engine import GrapePlan
    from robustgrape_amd.operators import OPT_GENERAL_H0
    nt = 20
    X = np.stack([P.random_x(nt, 400 + s) for s in range(3)])
    fp = _mk("sym", nt, ("amp",), False)
    plan = GrapePlan(fp, nparam=1, max_batch=2)
    try:
        F, Fdx, Fd2, Fd2dx = plan.fidelity_grad(X)
        assert plan.options & OPT_GENERAL_H0
    finally:
        plan.close()
    for b in range(len(X)):
        ref = O.calculate_fidelity_and_derivatives(fp, X[b])
        _check((F[b], Fdx[b], Fd2[b], Fd2dx[b]), ref, f"general_tables_{b}", 1, P.fd_tier(fp, X[b]))


def test_decay_h0_batches_are_single_calls():
    """A batch is the single evaluations, bit for bit; ragged chunks of the plan."""
    from robustgrape_amd.engine import GrapePlan
    nt = 12
    fp = _mk("full9", nt, 0, True)
    X = np.stack([P.random_x(nt, 500 + s) for s in range(5)])
    plan = GrapePlan(fp, nparam=1, max_batch=2)
    try:
        F, Fdx, _, _ = plan.fidelity_grad(X)
        for b in (0, 3, 4):
            Fs, gs, _, _ = plan.fidelity_grad(X[b:b + 1])
            assert Fs[0] == F[b] and np.array_equal(gs[0], Fdx[b])
    finally:
        plan.close()


def test_general_path_on_a_hermitian_problem_matches_the_fused_path():
    """GRAPE_OPT_GENERAL_H0 forced on a Hermitian H0: LU inverse + materialised derivatives
    against the fused kernels (C_k^dagger), same inputs."""
    from robustgrape_amd.engine import GrapePlan
    from robustgrape_amd.operators import OPT_GENERAL_H0
    nt = 30
    fp = P.sym_problem(nt, errors=("amp", "freq"))
    X = np.stack([P.random_x(nt, 600 + s) for s in range(3)])
    outs = []
    for opts in (0, OPT_GENERAL_H0):
        plan = GrapePlan(fp, nparam=1, max_batch=4, options=opts)
        try:
            outs.append(plan.fidelity_grad(X))
        finally:
            plan.close()
    for b in range(len(X)):
        _check(tuple(o[b] for o in outs[1]), tuple(o[b] for o in outs[0]), f"general_vs_fused_{b}", 2,
               P.fd_tier(fp, X[b]))


@pytest.mark.parametrize("kind,nt,errs", [("sym", 9, ("amp", "freq")), ("full9", 11, 2)])
def test_decay_unitary_derivatives_and_interaction_operators(kind, nt, errs):
    """calculate_unitary_and_derivatives (UnitaryCalculations.jl:20-155) and the interaction
    operators (:180-204, inv(cum_evo)) for a non-Hermitian H0."""
    from oracle import grape_oracle as O
    from robustgrape_amd import calculate_interaction_error_operators, calculate_unitary_and_derivatives
    x = P.random_x(nt, 700 + nt)
    upo, upd = _mk(kind, nt, errs, False).unitary_problem, _mk(kind, nt, errs, True).unitary_problem
    ref = O.calculate_unitary_and_derivatives(upo, x)
    got = calculate_unitary_and_derivatives(upd, x)
    assert np.max(np.abs(got[0] - ref[0])) <= T1
    assert abs(abs(np.linalg.det(ref[0])) - 1.0) > 1e-3  # not unitary
    # uncontracted FD tensors: tests/problems.py tensor_factor (as tests/test_gpu_parity.py
    # _assert_unitary): an entry of (E' - E) / eps carries the exponential's rounding over eps
    fac = P.tensor_factor(_mk(kind, nt, errs, False), x)
    for n, (tol, atol) in ((1, (T2 * fac, T2_ABS)), (2, (T2 * fac, T2_ABS)), (3, (T2 * fac, T2_ABS)),
                           (4, (T3 * fac, T3_ABS)), (5, (T3 * fac, T3_ABS))):
        a, b = np.asarray(got[n]), np.asarray(ref[n])
        assert a.shape == b.shape, (n, a.shape, b.shape)
        if b.size:
            assert np.max(np.abs(a - b)) <= tol * np.max(np.abs(b)) + atol, (n, np.max(np.abs(a - b)))
    Oref = O.calculate_interaction_error_operators(upo, x)
    Og = calculate_interaction_error_operators(upd, x)
    assert np.max(np.abs(Og - Oref)) <= 1e-7 * np.max(np.abs(Oref))
