"""GPU parity: the HIP path (through the C ABI) against the oracle and the golden fixtures.

Tolerance tiers (FD noise analysis there):
  T0  propagators E_k              <= 1e-13 relative (max-abs / max|E|, x max(1, |A|_1) for m = 13)
  T1  U, F                         <= 1e-12 absolute
  T2  eps-FD quantities (F_dx)     <= 1e-6 * max|ref| + 1e-7
  T2s the same on the short-step SURVEY configs (C1, C2, C4: dt |H|_1 <= 0.17, Taylor/Pade
      degree <= 12 without squarings), where two implementations differ by ~4e-9 of max|F_dx|:
      <= 1e-7 * max|ref| + 1e-9
Every assertion records its achieved error (tests/parity_log.py -> gpurun_out/parity_errors_*.json).
"""
import os

import numpy as np
import pytest

from tests import problems as P

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
T1 = 1e-12
T2, T2_ABS = 1e-6, 1e-7      # + absolute floor ~10 u/eps: FD noise of a gradient entry near an optimum


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from robustgrape_amd import _capi
    assert _capi.lib().grape_device_count() > 0


def _golden(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


T2S, T2S_ABS = 1e-7, 1e-9


def _assert_fid(F, Fdx, ref_F, ref_Fdx, tight=False, test=""):
    """tight: True (T2s), False (T2) or a (relative, absolute) pair (tests/problems.py fd_tier)."""
    from tests.parity_log import record
    if isinstance(tight, tuple):
        t2, t2a = tight
    else:
        t2, t2a = (T2S, T2S_ABS) if tight else (T2, T2_ABS)
    record(test, "F", abs(F - ref_F), 1.0, T1)
    assert abs(F - ref_F) <= T1, (F, ref_F)
    err, scale = np.max(np.abs(Fdx - ref_Fdx)), np.max(np.abs(ref_Fdx))
    record(test, "F_dx", err, scale, t2 * scale + t2a)
    assert err <= t2 * scale + t2a, (err, scale)


def test_expm_batch_matches_oracle_every_pade_degree():
    from robustgrape_amd import _capi
    g = _golden("expm")
    n = len(g["m"])
    groups = {}
    for i in range(n):
        groups.setdefault(g[f"A{i}"].shape[0], []).append(i)
    for d, idx in groups.items():
        A = np.stack([np.asfortranarray(g[f"A{i}"]) for i in idx])
        Acm = np.ascontiguousarray(A.transpose(0, 2, 1))  # column-major storage per matrix
        E = np.empty_like(Acm)
        stats = (_capi.ctypes.c_int * 5)()
        _capi.check(_capi.lib().grape_expm_batch(0, d, len(idx), _capi.dptr(Acm), _capi.dptr(E), stats))
        E = E.transpose(0, 2, 1)
        for j, i in enumerate(idx):
            ref = g[f"E{i}"]
            norm = np.abs(g[f"A{i}"]).sum(axis=0).max()
            rel = np.max(np.abs(E[j] - ref)) / np.max(np.abs(ref))
            assert rel <= 1e-13 * max(1.0, norm), (d, i, g["m"][i], rel)
        hist = {3: 0, 5: 1, 7: 2, 9: 3, 13: 4}
        expect = [0] * 5
        for i in idx:
            expect[hist[int(g["m"][i])]] += 1
        assert list(stats) == expect


@pytest.mark.parametrize("name,builder", [
    ("c1", lambda: P.sym_problem(500, t0=P.T0_TO)),
    ("c2", lambda: P.full9_problem(512)),
])
def test_fidelity_gradient_matches_golden(name, builder):
    from robustgrape_amd import calculate_fidelity_and_derivatives
    g = _golden(name)
    F, Fdx, d2, d2dx = calculate_fidelity_and_derivatives(builder(), g["x"])
    _assert_fid(F, Fdx, float(g["F"]), g["F_dx"], tight=True, test="golden_" + name)
    assert d2.shape == (0,) and d2dx.shape == (len(g["x"]), 0)


def test_restart_batch_matches_golden():
    """C4 sample: four restarts evaluated in one batched device pass."""
    from robustgrape_amd import calculate_fidelity_and_derivatives
    g = _golden("c4")
    F, Fdx, _, _ = calculate_fidelity_and_derivatives(P.full9_problem(512), g["x"])
    for b in range(len(F)):
        _assert_fid(F[b], Fdx[b], g["F"][b], g["F_dx"][b], tight=True, test=f"golden_c4_{b}")


@pytest.mark.parametrize("d,ntimes", [(5, 1), (5, 2), (5, 7), (7, 3), (9, 1), (9, 13), (9, 57), (5, 130)])
def test_small_problems_match_live_oracle(d, ntimes):
    """Edge sizes (single step, chunk remainders, d = 5/7/9) against the oracle computed here."""
    from oracle import grape_oracle as O
    from robustgrape_amd import calculate_fidelity_and_derivatives
    mk = {5: lambda dev: P.sym_problem(ntimes, device=dev), 7: lambda dev: P.fullblk_problem(ntimes, device=dev),
          9: lambda dev: P.full9_problem(ntimes, device=dev)}[d]
    x = P.random_x(ntimes, 100 + ntimes)
    F0, g0, _, _ = O.calculate_fidelity_and_derivatives(mk(False), x)
    F, g, _, _ = calculate_fidelity_and_derivatives(mk(True), x)
    _assert_fid(F, g, F0, g0, test=f"live_d{d}_nt{ntimes}")


def test_batch_equals_single_and_ragged_batches():
    """Deterministic kernels: a batch element is bitwise the single evaluation; odd batch sizes."""
    from robustgrape_amd import calculate_fidelity_and_derivatives
    fp = P.full9_problem(64)
    X = np.stack([P.random_x(64, s) for s in range(11)])
    F, Fdx, _, _ = calculate_fidelity_and_derivatives(fp, X)
    for b in (0, 5, 10):
        Fs, gs, _, _ = calculate_fidelity_and_derivatives(fp, X[b])
        assert Fs == F[b] and np.array_equal(gs, Fdx[b])


def test_known_answer_and_fd_identity_on_gpu():
    """runtests.jl:115-165 (F > 0.9999) and :292-354 (FD of F vs F_dx) on the device path."""
    from robustgrape_amd import calculate_fidelity_and_derivatives
    fp = P.sym_problem(1000)
    F = calculate_fidelity_and_derivatives(fp, P.evered_pulse(1000))[0]
    assert F > 0.9999 and abs(F - 0.999996184760959) < 1e-12
    fp = P.sym_problem(50)
    rng = np.random.default_rng(7)
    for idx in (3, 17, 49, 50):
        xs = 2 * np.pi * rng.uniform(size=51)
        F0, g0, _, _ = calculate_fidelity_and_derivatives(fp, xs)
        xs[idx] += fp.unitary_problem.eps
        F1 = calculate_fidelity_and_derivatives(fp, xs)[0]
        np.testing.assert_allclose((F1 - F0) / fp.unitary_problem.eps, g0[idx], rtol=1e-3, atol=1e-3)


def test_errors_are_loud():
    from robustgrape_amd import calculate_fidelity_and_derivatives
    with pytest.raises(AssertionError):
        calculate_fidelity_and_derivatives(P.full9_problem(64), np.zeros(64 + 2))
    from robustgrape_amd._capi import GrapeError
    from robustgrape_amd.types import FidelityRobustGRAPEProblem, UnitaryRobustGRAPEProblem
    d = 65  # closures run up to GRAPE_MAX_DENSE_DIM levels; above it GRAPE_ERR_UNSUPPORTED
    up = UnitaryRobustGRAPEProblem(t0=1.0, ntimes=4, ndim=d, H0=lambda t, x, xa: np.eye(d) * x[0],
                                   nb_additional_param=0)
    with pytest.raises(GrapeError):
        calculate_fidelity_and_derivatives(FidelityRobustGRAPEProblem(up, np.eye(d), lambda xa: np.eye(d)),
                                           np.zeros(4))


# ---------------------------------------------------------------- error sources (C3)
T3, T3_ABS, T3_XADD_ABS = 1e-5, 1e-7, 1e-5


def _err_scale(fp, x):
    """Step-norm factor of the FD tiers: tests/problems.py fd_factor (1 up to |dt H_k|_1 = 5.4, where
    Julia's exp! starts squaring; |dt H_k|_1 / 5.4 beyond)."""
    return P.fd_factor(fp, x)


def _assert_err(fp, d2, d2dx, ref_d2, ref_d2dx, test="", x=None, exact=None):
    """F_d2err / F_d2err_dx at T3 (scaled by fd_factor).  exact: (F, F_dx, F_d2err, F_d2err_dx) of
    oracle/grape_exact.py for these inputs -- then the device must be no farther from the exact
    forward differences than the checker (the reference's own algorithm) is, plus the tier, and
    within the tier plus twice that distance of the checker (its noise and the device's own)."""
    from tests.parity_log import record
    f = 1.0 if x is None else _err_scale(fp, x)
    t3, t3a = T3 * f, T3_ABS * f
    nmain = d2dx.shape[0] - fp.unitary_problem.nb_additional_param
    n0 = n1 = 0.0
    if exact is not None:
        n0 = float(np.max(np.abs(ref_d2 - exact[2])))
        n1 = float(np.max(np.abs(ref_d2dx[:nmain] - exact[3][:nmain])))
        x0, s0x = float(np.max(np.abs(d2 - exact[2]))), float(np.max(np.abs(exact[2])))
        record(test + "_vs_exact", "F_d2err", x0, s0x, t3 * s0x + t3a + n0)
        assert x0 <= t3 * s0x + t3a + n0, ("F_d2err vs exact", x0, n0)
        x1, s1x = float(np.max(np.abs(d2dx[:nmain] - exact[3][:nmain]))), float(np.max(np.abs(exact[3][:nmain])))
        record(test + "_vs_exact", "F_d2err_dx", x1, s1x, t3 * s1x + t3a + n1)
        assert x1 <= t3 * s1x + t3a + n1, ("F_d2err_dx vs exact", x1, n1)
    e0, s0 = np.max(np.abs(d2 - ref_d2)), np.max(np.abs(ref_d2))
    record(test, "F_d2err", e0, s0, t3 * s0 + t3a + 2 * n0)
    assert e0 <= t3 * s0 + t3a + 2 * n0, (d2, ref_d2)
    err, scale = np.max(np.abs(d2dx[:nmain] - ref_d2dx[:nmain])), np.max(np.abs(ref_d2dx[:nmain]))
    record(test, "F_d2err_dx", err, scale, t3 * scale + t3a + 2 * n1)
    assert err <= t3 * scale + t3a + 2 * n1, err
    if d2dx.shape[0] > nmain:
        # the x_add rows against their exact value (tests/xadd_pin.py: the reference's own rows there carry
        # the ((a + b) - a - b) / eps2^2 residue of a stencil over a parameter H does not read)
        from tests.xadd_pin import check_xadd, exact_rows
        ex_add = exact[3][nmain:] if exact is not None else (exact_rows(fp, x) if x is not None else None)
        if ex_add is not None:
            check_xadd(test or "err", d2dx, ref_d2dx, nmain, ex_add, rel=t3, ab=t3a)
        else:  # H0 / Herror read x_add: no exact evaluator; the absolute bound of the stencil residue
            ea = np.max(np.abs(d2dx[nmain:] - ref_d2dx[nmain:]))
            record(test, "F_d2err_dx_add", ea, np.max(np.abs(ref_d2dx[nmain:])), T3_XADD_ABS)
            assert ea <= T3_XADD_ABS


@pytest.mark.parametrize("name,builder", [
    ("c1err", lambda: P.sym_problem(500, t0=P.T0_TO, errors=("amp", "freq"))),
    ("d7err", lambda: P.fullblk_problem(500, errors=("amp", "freq"))),
    ("c3n64", lambda: P.full9_problem(64, nerr=4)),
    ("c3", lambda: P.full9_problem(512, nerr=4)),
])
def test_error_sensitivities_match_golden(name, builder):
    from robustgrape_amd import calculate_fidelity_and_derivatives
    g = _golden(name)
    fp = builder()
    F, Fdx, d2, d2dx = calculate_fidelity_and_derivatives(fp, g["x"])
    # C3 steps: T2s while no step needs squaring (N_t = 512), else the step-norm-scaled T2 tier
    # (N_t = 64: |dt H|_1 ~ 1.3; tests/problems.py fd_tier)
    tight = P.fd_tier(fp, g["x"]) if name.startswith("c3") else False
    _assert_fid(F, Fdx, float(g["F"]), g["F_dx"], tight=tight, test="golden_" + name)
    _assert_err(fp, d2, d2dx, g["F_d2err"], g["F_d2err_dx"], test="golden_" + name, x=g["x"])


@pytest.mark.parametrize("d,ntimes,errors", [(5, 1, ("amp",)), (5, 9, ("amp", "freq")), (7, 20, ("freq",)),
                                            (9, 3, 2), (9, 61, 4)])
def test_error_path_small_problems_match_live_oracle(d, ntimes, errors):
    from oracle import grape_oracle as O
    from robustgrape_amd import calculate_fidelity_and_derivatives
    if d == 5:
        mk = lambda dev: P.sym_problem(ntimes, errors=errors, device=dev)
    elif d == 7:
        mk = lambda dev: P.fullblk_problem(ntimes, errors=errors, device=dev)
    else:
        mk = lambda dev: P.full9_problem(ntimes, nerr=errors, device=dev)
    x = P.random_x(ntimes, 200 + ntimes)
    from oracle import grape_exact as E
    F0, g0, d20, d2dx0 = O.calculate_fidelity_and_derivatives(mk(False), x)
    fp = mk(True)
    F, g, d2, d2dx = calculate_fidelity_and_derivatives(fp, x)
    _assert_fid(F, g, F0, g0)
    _assert_err(fp, d2, d2dx, d20, d2dx0, test=f"live_err_d{d}_nt{ntimes}", x=x,
                exact=E.fidelity_and_derivatives(fp, x))


def test_error_sensitivity_gradient_identity_on_gpu():
    """runtests.jl:48-113 on the device path: (F_d2err(x + 1e-4 e_i) - F_d2err(x))/1e-4 vs F_d2err_dx[i]."""
    from robustgrape_amd import calculate_fidelity_and_derivatives
    fp = P.sym_problem(200, errors=("amp",))
    rng = np.random.default_rng(42)
    for idx in (int(rng.integers(200)), 200):
        xs = 2 * np.pi * rng.uniform(size=201)
        _, _, d0, d0dx = calculate_fidelity_and_derivatives(fp, xs)
        xs[idx] += 1e-4
        _, _, d1, _ = calculate_fidelity_and_derivatives(fp, xs)
        np.testing.assert_allclose((d1[0] - d0[0]) / 1e-4, d0dx[idx, 0], rtol=1e-3, atol=1e-5)


def test_error_batch_matches_single():
    from robustgrape_amd import calculate_fidelity_and_derivatives
    fp = P.full9_problem(40, nerr=4)
    X = np.stack([P.random_x(40, s) for s in range(5)])
    F, Fdx, d2, d2dx = calculate_fidelity_and_derivatives(fp, X)
    for b in (0, 4):
        Fs, gs, d2s, d2dxs = calculate_fidelity_and_derivatives(fp, X[b])
        assert Fs == F[b] and np.array_equal(gs, Fdx[b])
        assert np.array_equal(d2s, d2[b]) and np.array_equal(d2dxs, d2dx[b])


@pytest.mark.parametrize("waves", [1, 4, 8, 16])
def test_scan_widths_match_golden(waves):
    """Every k_scan / k_err_scan width (the plan picks 1 or 4 waves for large batches, 16 for the
    latency-bound chunk walks): C2 golden and the C3 (4 error sources) golden through a plan
    forced to each width (16 applies to the walk classes without error sources; C3 keeps its
    batch-size choice)."""
    from robustgrape_amd.engine import GrapePlan
    g = _golden("c2")
    plan = GrapePlan(P.full9_problem(512), nparam=1, max_batch=8, scan_waves=waves)
    F, Fdx, _, _ = plan.fidelity_grad(g["x"][None, :])
    plan.close()
    _assert_fid(F[0], Fdx[0], float(g["F"]), g["F_dx"])
    g = _golden("c3n64")
    fp = P.full9_problem(64, nerr=4)
    plan = GrapePlan(fp, nparam=1, max_batch=8, scan_waves=waves)
    F, Fdx, d2, d2dx = plan.fidelity_grad(g["x"][None, :])
    plan.close()
    _assert_fid(F[0], Fdx[0], float(g["F"]), g["F_dx"])
    _assert_err(fp, d2[0], d2dx[0], g["F_d2err"], g["F_d2err_dx"], x=g["x"])


def test_large_batch_plan_matches_single():
    """A 600-restart launch (narrow scan, several waves of workgroups per CU) against single evaluations."""
    from robustgrape_amd.engine import GrapePlan
    fp = P.full9_problem(512)
    X = np.stack([P.random_x(512, s) for s in range(600)])
    big = GrapePlan(fp, nparam=1, max_batch=600)
    F, Fdx, _, _ = big.fidelity_grad(X)
    big.close()
    one = GrapePlan(fp, nparam=1, max_batch=1)
    for b in (0, 299, 599):
        Fs, gs, _, _ = one.fidelity_grad(X[b][None, :])
        assert abs(Fs[0] - F[b]) <= T1 and np.max(np.abs(gs[0] - Fdx[b])) <= T2 * np.max(np.abs(gs[0])) + T2_ABS
    one.close()


# ---------------------------------------------------------------- materialised derivatives
def _assert_unitary(got, ref, fac=1.0):
    """T1 for U; T2 for eps quantities (U_dx, U_dx_add, U_derr); T3 for the eps2 mixed ones.
    fac = tests/problems.py tensor_factor scales the FD tiers: an uncontracted (E' - E)/eps carries
    the exponential's rounding (T0: 1e-13 x max(1, |A|_1), squarings for Pade 13) over eps."""
    names = ("U", "U_dx", "U_dx_add", "U_derr", "U_derr_dx", "U_derr_dx_add")
    for name, g, r in zip(names, got, ref):
        assert g.shape == r.shape, (name, g.shape, r.shape)
        if r.size == 0:
            continue
        err = np.max(np.abs(g - r))
        scale = np.max(np.abs(r))
        if name == "U":
            tol = T1 * fac
        elif name in ("U_derr_dx", "U_derr_dx_add"):
            tol = T3 * fac * scale + (T3_XADD_ABS if name == "U_derr_dx_add" else T3_ABS)
        else:
            tol = T2 * fac * scale + T2_ABS
        assert err <= tol, (name, err, scale)


def test_unitary_derivatives_match_golden():
    """grape_unitary_derivs vs the committed fixture (d = 5, N_t = 8, two error sources)."""
    from robustgrape_amd import calculate_unitary_and_derivatives
    g = _golden("unitary_small")
    up = P.sym_problem(8, errors=("amp", "freq")).unitary_problem
    got = calculate_unitary_and_derivatives(up, g["x"])
    _assert_unitary(got, [g[k] for k in ("U", "U_dx", "U_dx_add", "U_derr", "U_derr_dx", "U_derr_dx_add")])


@pytest.mark.parametrize("d,ntimes,nerr", [(9, 1, 0), (9, 40, 0), (9, 23, 4), (7, 30, 2), (5, 3, 1)])
def test_unitary_derivatives_match_live_oracle(d, ntimes, nerr):
    from oracle import grape_oracle as O
    from robustgrape_amd import calculate_unitary_and_derivatives
    errs = {0: (), 1: ("amp",), 2: ("amp", "freq")}
    if d == 9:
        mk = lambda dev: P.full9_problem(ntimes, nerr=nerr, device=dev)
    elif d == 7:
        mk = lambda dev: P.fullblk_problem(ntimes, errors=errs[nerr], device=dev)
    else:
        mk = lambda dev: P.sym_problem(ntimes, errors=errs[nerr], device=dev)
    x = P.random_x(ntimes, 500 + ntimes)
    up = mk(False).unitary_problem
    ref = O.calculate_unitary_and_derivatives(up, x)
    got = calculate_unitary_and_derivatives(mk(True).unitary_problem, x)
    _assert_unitary(got, ref, P.tensor_factor(mk(False), x))


def test_unitary_derivatives_consistent_with_fidelity_gradient():
    """F_dx from the fused kernels equals the reference's trace formula applied to the
    materialised U_dx (FidelityCalculations.jl:56-65)."""
    from robustgrape_amd import calculate_fidelity_and_derivatives, calculate_unitary_and_derivatives
    fp = P.full9_problem(32)
    x = P.random_x(32, 9)
    F, Fdx, _, _ = calculate_fidelity_and_derivatives(fp, x)
    U, Udx = calculate_unitary_and_derivatives(fp.unitary_problem, x)[:2]
    U0 = fp.target_unitary(x[-1:])
    W = np.diag(P.W_FULL9).astype(complex)
    Pm = (W != 0).astype(float)
    D = W.sum().real
    trm = lambda A: np.sum(W * np.diag(A))
    tau_c = np.conj(trm((Pm[:, None] * U0.conj().T) @ U))
    for k in (0, 13, 31):
        Ud = Udx[:, :, 0, k]
        A1 = (Pm[:, None] * U0.conj().T) @ Ud @ (Pm[:, None] * U.conj().T) @ U0
        A2 = (Pm[:, None] * U0.conj().T) @ U @ (Pm[:, None] * Ud.conj().T) @ U0
        ref = (np.real(trm(A1 + A2)) + 2 * np.real(tau_c * trm((Pm[:, None] * U0.conj().T) @ Ud))) / (D * (D + 1))
        assert abs(ref - Fdx[k]) <= T2 * np.max(np.abs(Fdx)) + T2_ABS
