"""Error sources together with an H0 (and an error generator) that read x_add.

The reference takes the x_add finite differences at every step for any H0
(src/UnitaryCalculations.jl:57-64), the mixed x_add stencils with each error
(:87-95), sums them into U_dx_add / U_derr_dx_add (:119-121, :140-151) and contracts
them with the target's x_add derivative (src/FidelityCalculations.jl:67-76, 99-113).
Checked through both device paths -- the operator basis (fused kernels) and the
closure fallback (host tables) -- against the live oracle, the committed golden
(tests/golden/xadd_err.npz) and, for the materialised tensors and the analysis
entry points, the oracle's calculate_unitary_and_derivatives /
calculate_interaction_error_operators on the same closures."""
import os

import numpy as np
import pytest

from tests import problems as P

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
T1 = 1e-12
# eps-FD tier: these problems take long steps (dt = t0 / N_t up to ~7.6, Pade 9/13 with
# squarings, each doubling the u/eps rounding of a difference): measured 3e-7 relative at
# d = 9, N_t = 7; the short-step C2/C4 goldens use the tighter 1e-7 (test_gpu_parity.py)
T2, T2_ABS = 1e-6, 1e-8
T2_XADD = 1e-6                # x_add rows (sums over N_t steps)
T3, T3_ABS = 1e-5, 1e-7       # eps2 mixed stencils


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _check(out, ref, label="", t2=T2):
    F, g, e, ed = out
    F0, g0, e0, ed0 = ref
    errs = {"F": abs(F - F0), "F_dx": np.max(np.abs(g - g0)) / np.max(np.abs(g0)),
            "F_d2err": np.max(np.abs(e - e0)) / np.max(np.abs(e0)),
            "F_d2err_dx": np.max(np.abs(ed - ed0)) / np.max(np.abs(ed0)),
            "F_d2err_dx_add": np.max(np.abs(ed[-2:] - ed0[-2:])) / np.max(np.abs(ed0[-2:]))}
    print(label, {k: f"{v:.2e}" for k, v in errs.items()})
    assert abs(F - F0) <= T1
    assert np.max(np.abs(g[:-2] - g0[:-2])) <= t2 * np.max(np.abs(g0)) + T2_ABS
    # F_dx_add sums one eps-difference per step (U_dx_add = U sum_k V^dxa_k): its u/eps
    # rounding noise grows with N_t, not with the gradient's size
    nt = (len(g) - 2)
    assert np.max(np.abs(g[-2:] - g0[-2:])) <= T2_XADD * np.max(np.abs(g0[-2:])) + T2_ABS * nt
    assert np.max(np.abs(e - e0)) <= t2 * np.max(np.abs(e0)) + T2_ABS
    assert np.max(np.abs(ed - ed0)) <= T3 * np.max(np.abs(ed0)) + T3_ABS
    # the x_add rows are really exercised and really checked
    assert np.min(np.abs(ed0[-2:])) > 1e-4 and np.min(np.abs(g0[-2:])) > 1e-4
    assert np.max(np.abs(ed[-2:] - ed0[-2:])) <= T3 * np.max(np.abs(ed0[-2:])) + T3_ABS


@pytest.mark.parametrize("device", [True, False], ids=["operator-basis", "closures"])
@pytest.mark.parametrize("d,ntimes", [(5, 1), (5, 13), (9, 7), (9, 64)])
def test_xadd_dependent_h0_with_errors_matches_live_oracle(device, d, ntimes):
    from oracle import grape_oracle as O
    from robustgrape_amd import calculate_fidelity_and_derivatives, get_plan
    x = P.xadd_x(ntimes, 40 + ntimes)
    ref = O.calculate_fidelity_and_derivatives(P.xadd_err_problem(d, ntimes, device=False), x)
    fp = P.xadd_err_problem(d, ntimes, device=device)
    out = calculate_fidelity_and_derivatives(fp, x)
    _check(out, ref, f"d={d} Nt={ntimes} {'ob' if device else 'tables'}")
    assert get_plan(fp, 1, 0, 1).tables == (not device)


@pytest.mark.parametrize("device", [True, False], ids=["operator-basis", "closures"])
def test_xadd_dependent_h0_with_errors_matches_golden(device):
    g = dict(np.load(os.path.join(GOLDEN, "xadd_err.npz"), allow_pickle=False))
    from robustgrape_amd import calculate_fidelity_and_derivatives
    fp = P.xadd_err_problem(int(g["d"]), int(g["ntimes"]), device=device)
    out = calculate_fidelity_and_derivatives(fp, g["x"])
    _check(out, (float(g["F"]), g["F_dx"], g["F_d2err"], g["F_d2err_dx"]), "golden")


def test_xadd_with_errors_batch_is_bitwise_the_single_calls():
    from robustgrape_amd import calculate_fidelity_and_derivatives
    fp = P.xadd_err_problem(9, 20)
    X = np.stack([P.xadd_x(20, s) for s in range(6)])
    F, Fdx, d2, d2dx = calculate_fidelity_and_derivatives(fp, X)
    for b in (0, 3, 5):
        Fs, gs, es, eds = calculate_fidelity_and_derivatives(fp, X[b])
        assert Fs == F[b] and np.array_equal(gs, Fdx[b]) and np.array_equal(es, d2[b])
        assert np.array_equal(eds, d2dx[b])


@pytest.mark.parametrize("device", [True, False], ids=["operator-basis", "closures"])
@pytest.mark.parametrize("d", [5, 9])
def test_unitary_derivatives_xadd_with_errors(device, d):
    """calculate_unitary_and_derivatives (UnitaryCalculations.jl:20-155) for both problem forms,
    U_dx_add and U_derr_dx_add included (f4: closures through grape_unitary_derivs_tables)."""
    from oracle import grape_oracle as O
    from robustgrape_amd import calculate_unitary_and_derivatives
    nt = 9
    x = P.xadd_x(nt, 77)
    ref = O.calculate_unitary_and_derivatives(P.xadd_err_problem(d, nt, device=False).unitary_problem, x)
    out = calculate_unitary_and_derivatives(P.xadd_err_problem(d, nt, device=device).unitary_problem, x)
    names = ["U", "U_dx", "U_dx_add", "U_derr", "U_derr_dx", "U_derr_dx_add"]
    tol = [T1, T2, T2_XADD, T2, T3, T3]
    for name, a, r, t in zip(names, out, ref, tol):
        assert a.shape == r.shape, name
        err = np.max(np.abs(a - r))
        print(name, f"{err:.2e}", f"{np.max(np.abs(r)):.2e}")
        assert err <= t * max(1.0, np.max(np.abs(r))), name


def test_closure_analysis_entry_points_match_oracle():
    """calculate_interaction_error_operators / calculate_expectation_values / the fidelity
    response for a closure problem (f2/f3/f4: the _tables entry points)."""
    from oracle import grape_oracle as O
    from robustgrape_amd import analysis as A
    nt = 16
    fc = P.xadd_err_problem(5, nt, device=False)
    x = P.xadd_x(nt, 5)
    Oref = O.calculate_interaction_error_operators(fc.unitary_problem, x)
    Odev = A.calculate_interaction_error_operators(fc.unitary_problem, x)
    assert Odev.shape == Oref.shape
    assert np.max(np.abs(Odev - Oref)) <= T2 * np.max(np.abs(Oref)) + T2_ABS
    ev0 = O.calculate_expectation_values(fc, x)
    ev = A.calculate_expectation_values(fc, x)
    assert np.max(np.abs(ev - ev0)) <= T2 * np.max(np.abs(ev0)) + T2_ABS
    w = np.linspace(0.0, 2.0, 7)
    r0 = O.calculate_fidelity_response(fc, x, w)
    r = A.calculate_fidelity_response(fc, x, w)
    assert np.max(np.abs(r - r0)) <= T2 * np.max(np.abs(r0)) + T2_ABS
    # the same physics through the operator basis gives the same operators
    Oob = A.calculate_interaction_error_operators(P.xadd_err_problem(5, nt).unitary_problem, x)
    assert np.max(np.abs(Oob - Odev)) <= T2 * np.max(np.abs(Oref)) + T2_ABS


@pytest.mark.parametrize("device", [True, False], ids=["operator-basis", "closures"])
def test_non_hermitian_error_generator_matches_oracle(device):
    """A decay-rate error source Herror = -i (e/2) |r><r| (non-Hermitian): its propagators only
    enter through differences transported by the unitary nominal chain, so the device serves it;
    against the oracle (which balances with zgebal and inverts with getrf/getri, as Julia)."""
    from oracle import grape_oracle as O
    from robustgrape_amd import calculate_fidelity_and_derivatives
    from robustgrape_amd.operators import OperatorBasisError, Term
    from robustgrape_amd.types import ErrorSource
    nt = 24
    decay = np.diag([0, 0, 0, 0, 1.0]).astype(complex)
    base = P.sym_problem(nt, errors=("amp",))
    ob = ErrorSource(OperatorBasisError([Term(decay, scale=-0.5j)]))
    cl = ErrorSource(lambda t, x, xa, e: -0.5j * e * decay)
    fo = base.replace(unitary_problem=base.unitary_problem.replace(
        error_sources=list(base.unitary_problem.error_sources) + [ob]))
    fc0 = P.sym_problem(nt, errors=("amp",), device=False)
    fc = fc0.replace(unitary_problem=fc0.unitary_problem.replace(
        error_sources=list(fc0.unitary_problem.error_sources) + [cl]))
    x = P.random_x(nt, 3)
    ref = O.calculate_fidelity_and_derivatives(fc, x)
    F, g, e, ed = calculate_fidelity_and_derivatives(fo if device else fc, x)
    assert abs(F - ref[0]) <= T1
    assert np.max(np.abs(g - ref[1])) <= T2 * np.max(np.abs(ref[1])) + T2_ABS
    assert np.max(np.abs(e - ref[2])) <= T2 * np.max(np.abs(ref[2])) + T2_ABS
    assert np.max(np.abs(ed[:-1] - ref[3][:-1])) <= T3 * np.max(np.abs(ref[3][:-1])) + T3_ABS
    assert abs(ref[2][1]) > 1e-3  # the decay sensitivity is really exercised
