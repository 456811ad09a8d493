"""Closure fallback (GRAPE_DESC_HOST_TABLES / grape_fidelity_grad_tables) on the GPU.

Problems whose H0 / target are plain closures -- the reference's own idiom
(src/Types.jl:10,50) -- are evaluated through host tables of every closure call
site (UnitaryCalculations.jl:45,51,59; FidelityCalculations.jl:32-40); the device
runs the exponentials, the scan and the contractions.  Checked against the golden
fixtures and the live oracle on the same closures, and against the operator-basis
path on the same physics."""
import os

import numpy as np
import pytest

from tests import problems as P

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
T1 = 1e-12
T2, T2_ABS = 1e-6, 1e-7


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _assert_fid(F, Fdx, ref_F, ref_Fdx):
    assert abs(F - ref_F) <= T1, (F, ref_F)
    err = np.max(np.abs(Fdx - ref_Fdx))
    assert err <= T2 * np.max(np.abs(ref_Fdx)) + T2_ABS, (err, np.max(np.abs(ref_Fdx)))


@pytest.mark.parametrize("name,builder", [
    ("c1", lambda: P.sym_problem(500, t0=P.T0_TO, device=False)),
    ("c2", lambda: P.full9_problem(512, device=False)),
])
def test_closure_problem_matches_golden(name, builder):
    from robustgrape_amd import calculate_fidelity_and_derivatives, get_plan
    g = dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))
    fp = builder()
    F, Fdx, d2, d2dx = calculate_fidelity_and_derivatives(fp, g["x"])
    _assert_fid(F, Fdx, float(g["F"]), g["F_dx"])
    assert d2.shape == (0,) and d2dx.shape == (len(g["x"]), 0)
    assert get_plan(fp, 1, 0, 1).tables  # it really took the table path


@pytest.mark.parametrize("d,ntimes", [(5, 1), (5, 9), (7, 3), (9, 13), (9, 57)])
def test_closure_problem_matches_live_oracle(d, ntimes):
    from oracle import grape_oracle as O
    from robustgrape_amd import calculate_fidelity_and_derivatives
    mk = {5: P.sym_problem, 7: P.fullblk_problem, 9: P.full9_problem}[d]
    fp = mk(ntimes, device=False)
    x = P.random_x(ntimes, 300 + ntimes)
    F0, g0, _, _ = O.calculate_fidelity_and_derivatives(fp, x)
    F, g, _, _ = calculate_fidelity_and_derivatives(fp, x)
    _assert_fid(F, g, F0, g0)


def _xadd_problem(d, ntimes, nparam, seed=5):
    """A closure H0 that DOES read x_add (exercises the dxa variants and the x_add
    reduction) and a general (non-operator-basis) target closure."""
    from robustgrape_amd.types import FidelityRobustGRAPEProblem, UnitaryRobustGRAPEProblem
    rng = np.random.default_rng(seed + d)

    def herm():
        G = rng.normal(size=(d, d)) + 1j * rng.normal(size=(d, d))
        H = (G + G.conj().T) / 2
        return H / np.abs(H).sum(axis=0).max()
    Hd, Hs = herm(), [herm() for _ in range(nparam)]
    Ha, Hb = herm(), herm()
    Q, _ = np.linalg.qr(rng.normal(size=(d, d)) + 1j * rng.normal(size=(d, d)))

    def H0(nt, x, xa):
        H = Hd + (0.3 + 0.01 * nt) * np.cos(xa[0]) * Ha + xa[1] ** 2 * Hb
        for p in range(nparam):
            H = H + np.sin(x[p] + 0.1 * p) * Hs[p]
        return H

    def target(xa):
        return Q @ np.diag(np.exp(1j * xa[0] * np.arange(d))) * np.exp(1j * xa[1])
    up = UnitaryRobustGRAPEProblem(t0=1.5, ntimes=ntimes, ndim=d, H0=H0, nb_additional_param=2)
    W = np.diag(np.linspace(1.0, 0.0, d))
    return FidelityRobustGRAPEProblem(up, W, target)


@pytest.mark.parametrize("d,ntimes,nparam", [(3, 17, 1), (6, 40, 2), (9, 25, 3), (12, 11, 2)])
def test_xadd_dependent_closure_matches_live_oracle(d, ntimes, nparam):
    from oracle import grape_oracle as O
    from robustgrape_amd import calculate_fidelity_and_derivatives
    fp = _xadd_problem(d, ntimes, nparam)
    rng = np.random.default_rng(d)
    x = np.concatenate([rng.uniform(-1, 1, size=nparam * ntimes), [0.7, 0.4]])
    F0, g0, _, _ = O.calculate_fidelity_and_derivatives(fp, x)
    F, g, _, _ = calculate_fidelity_and_derivatives(fp, x)
    _assert_fid(F, g, F0, g0)
    assert np.max(np.abs(g[-2:])) > 1e-3  # the x_add gradient is really exercised


def test_closure_batch_equals_single_and_equals_operator_basis_path():
    """Batched closure evaluations are bitwise the single ones, and the closure path agrees
    with the operator-basis path on the same physics to the FD tier."""
    from robustgrape_amd import calculate_fidelity_and_derivatives
    fp_c, fp_o = P.full9_problem(64, device=False), P.full9_problem(64)
    X = np.stack([P.random_x(64, s) for s in range(5)])
    F, Fdx, _, _ = calculate_fidelity_and_derivatives(fp_c, X)
    Fo, Fdxo, _, _ = calculate_fidelity_and_derivatives(fp_o, X)
    for b in range(5):
        Fs, gs, _, _ = calculate_fidelity_and_derivatives(fp_c, X[b])
        assert Fs == F[b] and np.array_equal(gs, Fdx[b])
        _assert_fid(F[b], Fdx[b], Fo[b], Fdxo[b])


# ---------------------------------------------------------------- error sources through the tables
T3, T3_ABS, T3_XADD_ABS = 1e-5, 1e-7, 1e-5


def _assert_err(nx_add, d2, d2dx, ref_d2, ref_d2dx, fp=None, x=None, test="tables_err"):
    nmain = d2dx.shape[0] - nx_add
    assert np.max(np.abs(d2 - ref_d2)) <= T3 * np.max(np.abs(ref_d2)) + T3_ABS, (d2, ref_d2)
    err = np.max(np.abs(d2dx[:nmain] - ref_d2dx[:nmain]))
    assert err <= T3 * np.max(np.abs(ref_d2dx[:nmain])) + T3_ABS, err
    if nx_add:
        # the x_add rows against their exact value (tests/xadd_pin.py); the table path tabulates the
        # reference's x_add stencil itself, so it carries a residue of the checker's kind
        from tests.xadd_pin import check_xadd, exact_rows
        ex = exact_rows(fp, x) if fp is not None else None
        if ex is not None:
            check_xadd(test, d2dx, ref_d2dx, nmain, ex, stencil=True)
        else:
            assert np.max(np.abs(d2dx[nmain:] - ref_d2dx[nmain:])) <= T3_XADD_ABS


@pytest.mark.parametrize("name,builder", [
    ("c1err", lambda: P.sym_problem(500, t0=P.T0_TO, errors=("amp", "freq"), device=False)),
    ("d7err", lambda: P.fullblk_problem(500, errors=("amp", "freq"), device=False)),
    ("c3n64", lambda: P.full9_problem(64, nerr=4, device=False)),
])
def test_closure_error_sources_match_golden(name, builder):
    """The reference's own idiom Herror = H(eps) - H(0) as closures (runtests.jl:57-75, 474-494)."""
    from robustgrape_amd import calculate_fidelity_and_derivatives
    g = dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))
    fp = builder()
    F, Fdx, d2, d2dx = calculate_fidelity_and_derivatives(fp, g["x"])
    _assert_fid(F, Fdx, float(g["F"]), g["F_dx"])
    _assert_err(1, d2, d2dx, g["F_d2err"], g["F_d2err_dx"], fp, g["x"], "tables_golden_" + name)


@pytest.mark.parametrize("d,ntimes,errors", [(5, 1, ("amp",)), (5, 11, ("amp", "freq")), (7, 6, ("freq",))])
def test_closure_error_sources_match_live_oracle(d, ntimes, errors):
    from oracle import grape_oracle as O
    from robustgrape_amd import calculate_fidelity_and_derivatives
    mk = {5: P.sym_problem, 7: P.fullblk_problem}[d]
    fp = mk(ntimes, errors=errors, device=False)
    x = P.random_x(ntimes, 500 + ntimes)
    F0, g0, e0, ed0 = O.calculate_fidelity_and_derivatives(fp, x)
    F, g, e, ed = calculate_fidelity_and_derivatives(fp, x)
    _assert_fid(F, g, F0, g0)
    _assert_err(1, e, ed, e0, ed0, fp, x, f"tables_live_d{d}_nt{ntimes}")


def test_closure_error_sources_with_xadd_dependent_h0():
    """Formerly refused (round 1): an x_add-dependent closure H0 with an error source now takes
    every x_add call site of the reference (UnitaryCalculations.jl:57-64, 87-95)."""
    from oracle import grape_oracle as O
    from robustgrape_amd import calculate_fidelity_and_derivatives
    from robustgrape_amd.types import ErrorSource
    fp = _xadd_problem(4, 5, 1)
    up = fp.unitary_problem
    Hz = np.diag(np.arange(4.0))
    fp = fp.replace(unitary_problem=up.replace(error_sources=[ErrorSource(lambda t, x, xa, e: e * np.cos(xa[1]) * Hz)]))
    x = np.concatenate([np.linspace(-0.5, 0.5, 5), [0.3, 0.2]])
    F0, g0, e0, ed0 = O.calculate_fidelity_and_derivatives(fp, x)
    F, g, e, ed = calculate_fidelity_and_derivatives(fp, x)
    _assert_fid(F, g, F0, g0)
    _assert_err(0, e, ed, e0, ed0)
    assert np.max(np.abs(ed0[-2:])) > 1e-3


@pytest.mark.parametrize("d", list(range(2, 13)))
def test_every_dimension_with_errors_through_tables(d):
    """The operator-basis random problems of test_gpu_dims (two controls, cis target, two
    error sources) handed over as plain closures: the table path against the live oracle."""
    from oracle import grape_oracle as O
    from robustgrape_amd import calculate_fidelity_and_derivatives, get_plan
    from tests.test_gpu_dims import random_problem
    nt = 7
    fp = random_problem(d, nt, 2, False)
    rng = np.random.default_rng(d + 77)
    x = np.concatenate([rng.uniform(-1, 1, size=2 * nt), [rng.uniform(0, 2 * np.pi)]])
    F0, g0, e0, ed0 = O.calculate_fidelity_and_derivatives(fp, x)
    F, g, e, ed = calculate_fidelity_and_derivatives(fp, x)
    _assert_fid(F, g, F0, g0)
    _assert_err(1, e, ed, e0, ed0)
    assert get_plan(fp, 2, 0, 1).tables


def test_table_plan_chunks_batches_and_refuses_the_operator_entry_points():
    """nbatch > max_batch runs in chunks (bitwise equal to single calls); a table plan
    refuses the operator-basis entry point grape_fidelity_grad loudly."""
    from robustgrape_amd import GrapePlan, calculate_fidelity_and_derivatives
    from robustgrape_amd._capi import GrapeError
    fp = P.sym_problem(20, errors=("amp",), device=False)
    X = np.stack([P.random_x(20, s) for s in range(7)])
    plan = GrapePlan(fp, 1, max_batch=3)
    F, Fdx, d2, d2dx = plan.fidelity_grad(X)
    for b in (0, 4, 6):
        Fs, gs, es, eds = calculate_fidelity_and_derivatives(fp, X[b])
        assert Fs == F[b] and np.array_equal(gs, Fdx[b]) and np.array_equal(es, d2[b])
        assert np.array_equal(eds, d2dx[b])
    from robustgrape_amd import _capi
    F1, G1 = np.empty(1), np.empty((1, 21))
    with pytest.raises(GrapeError):
        _capi.check(_capi.lib().grape_fidelity_grad(plan.handle, 1, _capi.dptr(X[:1].copy()), _capi.dptr(F1),
                                                    _capi.dptr(G1), None, None))
    plan.close()


@pytest.mark.parametrize("nerr", [0, 1])
def test_closure_without_additional_parameters(nerr):
    """nb_additional_param = 0 (no x_add, one target slot) with and without an error source."""
    from oracle import grape_oracle as O
    from robustgrape_amd import calculate_fidelity_and_derivatives
    from robustgrape_amd.types import ErrorSource, FidelityRobustGRAPEProblem, UnitaryRobustGRAPEProblem
    d, nt = 4, 12
    rng = np.random.default_rng(11)

    def herm():
        G = rng.normal(size=(d, d)) + 1j * rng.normal(size=(d, d))
        return (G + G.conj().T) / 4
    Hd, H1, H2, He = herm(), herm(), herm(), herm()
    Q, _ = np.linalg.qr(rng.normal(size=(d, d)) + 1j * rng.normal(size=(d, d)))
    errs = [ErrorSource(lambda t, x, xa, e: e * np.cos(x[0]) * He)] if nerr else []
    up = UnitaryRobustGRAPEProblem(t0=2.0, ntimes=nt, ndim=d, nb_additional_param=0, error_sources=errs,
                                   H0=lambda t, x, xa: Hd + x[0] * H1 + np.sin(x[1]) * H2)
    fp = FidelityRobustGRAPEProblem(up, np.diag([1.0, 1.0, 0.5, 0.0]), lambda xa: Q)
    x = rng.uniform(-1, 1, size=2 * nt)
    F0, g0, e0, ed0 = O.calculate_fidelity_and_derivatives(fp, x)
    F, g, e, ed = calculate_fidelity_and_derivatives(fp, x)
    _assert_fid(F, g, F0, g0)
    if nerr:
        _assert_err(0, e, ed, e0, ed0)
