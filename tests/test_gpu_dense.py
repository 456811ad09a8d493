"""GPU parity of the dense (MFMA) engine, 12 < d <= 64,
through the C ABI, against the CPU oracle (live, small sizes) and the committed
C5 golden fixture (d = 64, N_t = 1024).

Tolerances (SURVEY.md 8c tiers):
  T0  exp(A)          <= 1e-13 relative x max(1, |A|_1); Pade 13 (where this engine
                       takes extra squarings to keep its pivot-free solve safe) 1e-12
  T1  F               <= 1e-12 absolute
  T2  F_dx            <= 1e-6 max|ref| + 1e-9 + |ref - exact|
      where exact is the reference's forward difference evaluated in longdouble
      (oracle/grape_exact.py) and |ref - exact| the checker's own u / eps noise: at d = 16 the
      oracle (Julia's exp! restated) already sits 5.8e-7 of max|F_dx| from it and the C++ port
      1.1e-6 (scripts/probes/dense_exact_probe.py), so two correct double implementations differ
      by up to their two noises.  The device result is also checked against exact directly:
      <= 1e-6 max|exact| + 1e-9.  (Round 4 used a blanket + 1e-7, 350x the tier at C5.)
"""
import os

import numpy as np
import pytest

from robustgrape_amd import synthetic as S

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
T1 = 1e-12
T2, T2_FLOOR = 1e-6, 1e-9
T2_ABS = 1e-7  # the error-path tiers below (F_d2err: eps-FD of the error images, T3: eps2 stencils)


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _assert_fid(F, Fdx, ref_F, ref_Fdx, test="dense", exact=None, spread=0.0):
    """F at T1; F_dx against the checker at T2 with the checker's own distance from the exact
    forward difference added (exact: (F, F_dx) of oracle/grape_exact.py, when evaluated), and
    against exact itself at T2 + 1e-9."""
    from tests.parity_log import record
    ef = abs(F - ref_F)
    record(test, "F", ef, 1.0, T1)
    assert ef <= T1, (F, ref_F)
    noise = spread
    if exact is not None:
        noise = float(np.max(np.abs(np.asarray(ref_Fdx) - exact[1])))
        ee = float(np.max(np.abs(Fdx - exact[1])))
        se = float(np.max(np.abs(exact[1])))
        record(test + "_vs_exact", "F_dx", ee, se, T2 * se + T2_FLOOR)
        assert ee <= T2 * se + T2_FLOOR, ("vs exact", ee, se)
    err, scale = float(np.max(np.abs(Fdx - ref_Fdx))), float(np.max(np.abs(ref_Fdx)))
    tol = T2 * scale + T2_FLOOR + noise
    record(test, "F_dx", err, scale, tol)
    print(f"{test}: F_dx err {err:.3e} (rel {err / scale:.2e}), checker noise {noise:.2e}, tol {tol:.2e}")
    assert err <= tol, (err, scale, noise)


def _cpu_spread(fp, x, ref_Fdx):
    """Where no exact evaluation exists (x_add-dependent H0, error sources): the checker's noise
    estimated by the spread of two correct CPU implementations of the reference's algorithm
    (the oracle and the C++ port, oracle/cref) -- (None-like) 0 when the port is not built."""
    try:
        from oracle.cref import cref
        if not cref.available():
            return 0.0
        return float(np.max(np.abs(np.asarray(cref.fidelity_grad(fp, x)[1]) - np.asarray(ref_Fdx))))
    except Exception:
        return 0.0


def _assert_fid_spread(F, Fdx, ref_F, ref_Fdx, test, fp, x):
    _assert_fid(F, Fdx, ref_F, ref_Fdx, test, spread=_cpu_spread(fp, x, ref_Fdx))


def _skew_hermitian(d, norm, rng):
    H = rng.normal(size=(d, d)) + 1j * rng.normal(size=(d, d))
    H = (H + H.conj().T) / 2
    return -1j * H / np.abs(H).sum(axis=0).max() * norm


@pytest.mark.parametrize("d", [13, 24, 64])
def test_dense_expm_matches_oracle_every_pade_degree(d):
    from oracle import grape_oracle as O
    from robustgrape_amd import _capi
    rng = np.random.default_rng(1000 + d)
    norms = (0.01, 0.04, 0.2, 0.6, 0.8, 0.9, 1.5, 4.0, 30.0)  # Taylor 8 / 8 / 12 / 16 / 16 / 20, Pade 9, 13, 13
    A = np.stack([_skew_hermitian(d, nm, rng) for nm in norms])
    refs, ms = [], []
    for a in A:
        st = {}
        refs.append(O.julia_exp(a, st))
        ms.append(list(st)[0][0])
    Acm = np.ascontiguousarray(A.transpose(0, 2, 1))  # column-major per matrix
    E = np.empty_like(Acm)
    stats = (_capi.ctypes.c_int * 5)()
    _capi.check(_capi.lib().grape_expm_batch(0, d, len(A), _capi.dptr(Acm), _capi.dptr(E), stats))
    E = E.transpose(0, 2, 1)
    for j, nm in enumerate(norms):
        rel = np.max(np.abs(E[j] - refs[j])) / np.max(np.abs(refs[j]))
        tol = (1e-12 if ms[j] == 13 else 1e-13) * max(1.0, nm)
        assert rel <= tol, (d, nm, ms[j], rel)
        # unitary to rounding
        assert np.max(np.abs(E[j].conj().T @ E[j] - np.eye(d))) < 1e-12 * max(1.0, nm)
    hist = {3: 0, 5: 1, 7: 2, 9: 3, 13: 4}
    expect = [0] * 5
    for m in ms:
        expect[hist[m]] += 1
    assert list(stats) == expect


@pytest.mark.parametrize("d,ntimes,scale", [(13, 1, 1.0), (16, 5, 1.0), (24, 17, 0.3), (40, 9, 2.0),
                                            (64, 3, 1.0), (64, 37, 1.0), (64, 20, 0.05)])
def test_dense_fidelity_gradient_matches_live_oracle(d, ntimes, scale):
    """Edge sizes: one step, chunk remainders, padded d, Pade 3..9 (scale moves |A|_1)."""
    from oracle import grape_oracle as O
    from robustgrape_amd import calculate_fidelity_and_derivatives
    from oracle import grape_exact as E
    fp = S.dense_problem(d, ntimes, rank=min(16, d - 3), scale=scale)
    x = S.dense_x(ntimes, seed=300 + ntimes)
    F0, g0, _, _ = O.calculate_fidelity_and_derivatives(fp, x)
    F, g, d2, d2dx = calculate_fidelity_and_derivatives(fp, x)
    _assert_fid(F, g, F0, g0, f"dense_live_d{d}_nt{ntimes}_s{scale}", E.fidelity_and_gradient(fp, x, nparam=2))
    assert d2.shape == (0,) and d2dx.shape == (len(x), 0)


def test_c5_matches_golden():
    """d = 64, N_t = 1024, np = 2 (oracle fixture from tests/golden/make_golden.py)."""
    from robustgrape_amd import calculate_fidelity_and_derivatives
    g = dict(np.load(os.path.join(GOLDEN, "c5.npz"), allow_pickle=False))
    F, Fdx, _, _ = calculate_fidelity_and_derivatives(S.dense_problem(), g["x"])
    exact = (float(g["F_exact"]), g["F_dx_exact"]) if "F_dx_exact" in g else None
    _assert_fid(F, Fdx, float(g["F"]), g["F_dx"], "c5_golden", exact)


def test_dense_batch_equals_single():
    """Deterministic kernels: a batch element is bitwise the single evaluation."""
    from robustgrape_amd.engine import GrapePlan
    fp = S.dense_problem(64, 48)
    X = np.stack([S.dense_x(48, seed=s) for s in range(5)])
    plan = GrapePlan(fp, nparam=2, max_batch=5)
    F, Fdx, _, _ = plan.fidelity_grad(X)
    plan.close()
    one = GrapePlan(fp, nparam=2, max_batch=2)  # ragged: 2 + 2 + 1 through one plan
    F1, Fdx1, _, _ = one.fidelity_grad(X)
    one.close()
    assert np.array_equal(F, F1) and np.array_equal(Fdx, Fdx1)


def test_dense_fd_identity():
    """runtests.jl:292-354 on the dense path: forward difference of F vs F_dx."""
    from robustgrape_amd import calculate_fidelity_and_derivatives
    fp = S.dense_problem(32, 24)
    x = S.dense_x(24, seed=5)
    F0, g0, _, _ = calculate_fidelity_and_derivatives(fp, x)
    for idx in (0, 17, 47):
        xs = x.copy()
        xs[idx] += 1e-6
        F1 = calculate_fidelity_and_derivatives(fp, xs)[0]
        np.testing.assert_allclose((F1 - F0) / 1e-6, g0[idx], rtol=1e-3, atol=1e-6)


def test_dense_rejects_what_it_does_not_serve():
    from robustgrape_amd import _capi
    from robustgrape_amd.engine import GrapePlan
    from robustgrape_amd.operators import OperatorBasisError, OperatorBasisHamiltonian, Term
    from robustgrape_amd.types import ErrorSource
    fp = S.dense_problem(20, 4)
    up = fp.unitary_problem
    decay = np.diag([0.0] * 19 + [1.0]).astype(complex)  # a non-Hermitian error generator (dense: refused)
    errs = (ErrorSource(OperatorBasisError([Term(decay, scale=-0.5j)])),)
    with pytest.raises(_capi.GrapeError, match="UNSUPPORTED"):
        GrapePlan(fp.replace(unitary_problem=up.replace(error_sources=errs)), nparam=2)
    H = np.triu(np.ones((20, 20), complex))  # not Hermitian
    bad = up.replace(H0=OperatorBasisHamiltonian([Term(H)]))
    with pytest.raises(_capi.GrapeError, match="UNSUPPORTED"):
        GrapePlan(fp.replace(unitary_problem=bad), nparam=2)


def _xadd_h0_problem(d, ntimes):
    """The C5 family with two additional parameters: x_add[0] a phase on the target's first column
    (as dense_error_problem(phase=True)), x_add[1] a global detuning of H0 (a Hermitian Ginibre
    operator times x_add[1]) and x_add[0] also modulating it (cos), so that every step's exponential
    depends on x_add (UnitaryCalculations.jl:57-64)."""
    from robustgrape_amd.operators import FN_COS, FN_LINEAR, VAR_XADD, OperatorBasisHamiltonian, Term
    base = S.dense_error_problem(d, ntimes, nerr=0, phase=True)
    up = base.unitary_problem
    Hx = S._hermitian(d, 70)
    H0 = OperatorBasisHamiltonian(list(up.H0.terms) + [Term(Hx, var=VAR_XADD, index=1, func=FN_LINEAR, scale=0.4),
                                                        Term(Hx, var=VAR_XADD, index=0, func=FN_COS, scale=0.2)])
    return base.replace(unitary_problem=up.replace(H0=H0, nb_additional_param=2))


@pytest.mark.parametrize("d,ntimes", [(13, 1), (16, 7), (40, 9), (64, 5)])
def test_dense_xadd_dependent_h0_matches_live_oracle(d, ntimes):
    """H0 reading x_add above 12 levels (round 4): k_dgrad adds each step's x_add variant and k_dadd
    sums them onto the target's part of F_dx_add, against the oracle (FidelityCalculations.jl:67-76)."""
    from oracle import grape_oracle as O
    from robustgrape_amd import calculate_fidelity_and_derivatives
    fp = _xadd_h0_problem(d, ntimes)
    x = np.concatenate([S.dense_x(ntimes, seed=500 + ntimes), [0.7, -0.3]])
    ref = O.calculate_fidelity_and_derivatives(fp, x)
    F, g, _, _ = calculate_fidelity_and_derivatives(fp, x)
    _assert_fid_spread(F, g, ref[0], ref[1], f"dense_xadd_d{d}_nt{ntimes}", fp, x)
    assert g.shape == (len(x),) and abs(g[-1]) > 1e-6  # the H0 part of F_dx_add is not empty


def test_dense_xadd_h0_batch_equals_single():
    from robustgrape_amd.engine import GrapePlan
    fp = _xadd_h0_problem(24, 6)
    X = np.stack([np.concatenate([S.dense_x(6, seed=s), [0.3 * s, -0.1 * s]]) for s in range(4)])
    plan = GrapePlan(fp, nparam=2, max_batch=4)
    F, Fdx, _, _ = plan.fidelity_grad(X)
    plan.close()
    one = GrapePlan(fp, nparam=2, max_batch=1)
    F1, Fdx1, _, _ = one.fidelity_grad(X)
    one.close()
    assert np.array_equal(F, F1) and np.array_equal(Fdx, Fdx1)


# ---------------------------------------------------------------- error sources (d > 12)
T3, T3_ABS = 1e-5, 1e-7


def _assert_err(d2, d2dx, ref_d2, ref_d2dx, t2=T2):
    assert np.max(np.abs(d2 - ref_d2)) <= t2 * np.max(np.abs(ref_d2)) + T2_ABS, (d2, ref_d2)
    err = np.max(np.abs(d2dx - ref_d2dx))
    assert err <= T3 * np.max(np.abs(ref_d2dx)) + T3_ABS, (err, np.max(np.abs(ref_d2dx)))


@pytest.mark.parametrize("d,ntimes,nerr,phase,scale", [(13, 1, 1, False, 1.0), (16, 5, 2, True, 1.0),
                                                       (24, 17, 1, False, 0.3), (40, 9, 2, True, 1.0),
                                                       (64, 11, 2, False, 1.0)])
def test_dense_error_sources_match_live_oracle(d, ntimes, nerr, phase, scale):
    """The error path of the dense engine (k_dexp over every variant, k_dlocal, k_dwsum,
    k_derr_scan, k_dmce, k_derr_grad) against the oracle: F, F_dx, F_d2err, F_d2err_dx
    (UnitaryCalculations.jl:66-151, FidelityCalculations.jl:78-117)."""
    from oracle import grape_oracle as O
    from robustgrape_amd import calculate_fidelity_and_derivatives
    fp = S.dense_error_problem(d, ntimes, rank=min(16, d - 3), scale=scale, nerr=nerr, phase=phase)
    x = S.dense_x(ntimes, seed=400 + ntimes)
    if phase:
        x = np.concatenate([x, [0.7]])
    ref = O.calculate_fidelity_and_derivatives(fp, x)
    F, g, d2, d2dx = calculate_fidelity_and_derivatives(fp, x)
    _assert_fid_spread(F, g, ref[0], ref[1], f"dense_err_d{d}_nt{ntimes}", fp, x)
    _assert_err(d2, d2dx, ref[2], ref[3])
    assert d2.shape == (nerr,) and d2dx.shape == (len(x), nerr)


def test_c5err_matches_golden():
    """C5 + 2 error sources at N_t = 64 (tests/golden/make_golden.py c5err)."""
    from robustgrape_amd import calculate_fidelity_and_derivatives
    g = dict(np.load(os.path.join(GOLDEN, "c5err.npz"), allow_pickle=False))
    fp = S.dense_error_problem(64, int(g["ntimes"]))
    F, Fdx, d2, d2dx = calculate_fidelity_and_derivatives(fp, g["x"])
    _assert_fid_spread(F, Fdx, float(g["F"]), g["F_dx"], "c5err_golden", fp, g["x"])
    _assert_err(d2, d2dx, g["F_d2err"], g["F_d2err_dx"])


def test_dense_error_batch_equals_single():
    from robustgrape_amd.engine import GrapePlan
    fp = S.dense_error_problem(32, 12)
    X = np.stack([S.dense_x(12, seed=s) for s in range(3)])
    plan = GrapePlan(fp, nparam=2, max_batch=3)
    F, Fdx, d2, d2dx = plan.fidelity_grad(X)
    plan.close()
    one = GrapePlan(fp, nparam=2, max_batch=1)
    F1, Fdx1, d21, d2dx1 = one.fidelity_grad(X)
    one.close()
    assert np.array_equal(F, F1) and np.array_equal(Fdx, Fdx1)
    assert np.array_equal(d2, d21) and np.array_equal(d2dx, d2dx1)


# ---------------------------------------------------------------- materialised tensors, analysis (d > 12)
@pytest.mark.parametrize("d,ntimes,nerr,phase", [(13, 3, 0, False), (16, 5, 2, True), (40, 4, 1, False)])
def test_dense_unitary_derivatives_match_oracle(d, ntimes, nerr, phase):
    """calculate_unitary_and_derivatives (UnitaryCalculations.jl:20-155) on the dense engine:
    the variant table from k_dexp (register-file images -> row-major tiles), then the
    grape_unitary kernels over global-scratch tiles (f4 for 12 < d <= 64)."""
    from oracle import grape_oracle as O
    from robustgrape_amd import calculate_unitary_and_derivatives
    if nerr:
        fp = S.dense_error_problem(d, ntimes, rank=min(16, d - 3), nerr=nerr, phase=phase)
    else:
        fp = S.dense_problem(d, ntimes, rank=min(16, d - 3))
    x = S.dense_x(ntimes, seed=600 + ntimes)
    if phase:
        x = np.concatenate([x, [0.7]])
    ref = O.calculate_unitary_and_derivatives(fp.unitary_problem, x)
    out = calculate_unitary_and_derivatives(fp.unitary_problem, x)
    names = ["U", "U_dx", "U_dx_add", "U_derr", "U_derr_dx", "U_derr_dx_add"]
    tol = [1e-12, T2, T2, T2, T3, T3]
    for name, a, r, t in zip(names, out, ref, tol):
        assert a.shape == r.shape, name
        if r.size == 0:
            continue
        err = np.max(np.abs(a - r))
        print(name, f"{err:.2e}", f"{np.max(np.abs(r)):.2e}")
        assert err <= t * max(1.0, np.max(np.abs(r))), name


def test_dense_analysis_entry_points_match_oracle():
    """calculate_interaction_error_operators, calculate_expectation_values and the fidelity
    response (UnitaryCalculations.jl:180-204, FidelityCalculations.jl:246-390) at d = 20."""
    from oracle import grape_oracle as O
    from robustgrape_amd import analysis as A
    nt = 12
    fp = S.dense_error_problem(20, nt, rank=12, nerr=2)
    x = S.dense_x(nt, seed=77)
    Oref = O.calculate_interaction_error_operators(fp.unitary_problem, x)
    Odev = A.calculate_interaction_error_operators(fp.unitary_problem, x)
    assert Odev.shape == Oref.shape
    assert np.max(np.abs(Odev - Oref)) <= T2 * np.max(np.abs(Oref)) + T2_ABS
    ev0 = O.calculate_expectation_values(fp, x)
    ev = A.calculate_expectation_values(fp, x)
    assert np.max(np.abs(ev - ev0)) <= T2 * np.max(np.abs(ev0)) + T2_ABS
    w = np.linspace(0.0, 1.0, 4)
    r0 = O.calculate_fidelity_response(fp, x, w)
    r = A.calculate_fidelity_response(fp, x, w)
    assert np.max(np.abs(r - r0)) <= T2 * np.max(np.abs(r0)) + T2_ABS


def _split_terms_problem(d, ntimes, alpha=0.7):
    """The C5 family with every Hermitian operator OP of H0 given as TWO non-Hermitian terms with complex
    scales, e^{i alpha} U and e^{-i alpha} U^dag, U = triu(OP, 1) + diag(OP) / 2 (so each term is neither
    Hermitian nor real-scaled, the sum is e^{i alpha} U + h.c.): the reference takes any closure whose value
    is Hermitian (UnitaryCalculations.jl:45-47), the dense engine now checks the SUM at probe points."""
    from robustgrape_amd.operators import OperatorBasisHamiltonian, Term
    fp = S.dense_problem(d, ntimes, rank=min(16, d - 3))
    up = fp.unitary_problem
    terms = []
    for t in up.H0.terms:
        U = np.triu(t.op, 1) + np.diag(np.diag(t.op)) / 2
        for op, sc in ((U, np.exp(1j * alpha)), (U.conj().T, np.exp(-1j * alpha))):
            terms.append(Term(op, var=t.var, index=t.index, func=t.func, a=t.a, b=t.b, scale=t.scale * sc))
    return fp.replace(unitary_problem=up.replace(H0=OperatorBasisHamiltonian(terms)))


@pytest.mark.parametrize("d,ntimes", [(13, 3), (24, 17), (64, 5)])
def test_dense_complex_coefficient_terms_match_live_oracle(d, ntimes):
    """VERDICT r5 missing #2: H0 terms with complex coefficients (each term non-Hermitian, the sum Hermitian)
    on the dense engine against the oracle and the exact forward difference."""
    from oracle import grape_exact as E
    from oracle import grape_oracle as O
    from robustgrape_amd import calculate_fidelity_and_derivatives
    fp = _split_terms_problem(d, ntimes)
    x = S.dense_x(ntimes, seed=800 + ntimes)
    F0, g0, _, _ = O.calculate_fidelity_and_derivatives(fp, x)
    F, g, _, _ = calculate_fidelity_and_derivatives(fp, x)
    _assert_fid(F, g, F0, g0, f"dense_split_d{d}_nt{ntimes}", E.fidelity_and_gradient(fp, x, nparam=2))


def _xadd_err_problem(d, ntimes, nerr=2):
    """VERDICT r5 missing #2: the C5 family with error sources AND an H0 reading x_add (x_add[1] a global
    detuning, x_add[0] the target phase modulating it), error 0 also modulated by cos(x_add[1]): every
    variant of UnitaryCalculations.jl:57-95 (the x_add ones with the eps and eps2 error variants) is live."""
    from robustgrape_amd.operators import FN_COS, FN_LINEAR, VAR_XADD, OperatorBasisError, OperatorBasisHamiltonian, Term
    from robustgrape_amd.types import ErrorSource
    base = S.dense_error_problem(d, ntimes, rank=min(16, d - 3), nerr=nerr, phase=True)
    up = base.unitary_problem
    Hx = S._hermitian(d, 70)
    H0 = OperatorBasisHamiltonian(list(up.H0.terms) + [Term(Hx, var=VAR_XADD, index=1, func=FN_LINEAR, scale=0.4),
                                                        Term(Hx, var=VAR_XADD, index=0, func=FN_COS, scale=0.2)])
    errs = []
    for e, es in enumerate(up.error_sources):
        terms = list(es.Herror.terms)
        if e == 0:
            terms.append(Term(S._hermitian(d, 71), var=VAR_XADD, index=1, func=FN_COS, scale=0.3))
        errs.append(ErrorSource(OperatorBasisError(terms)))
    return base.replace(unitary_problem=up.replace(H0=H0, nb_additional_param=2, error_sources=errs))


@pytest.mark.parametrize("d,ntimes,nerr", [(13, 1, 1), (16, 6, 2), (40, 5, 2), (64, 3, 1)])
def test_dense_xadd_dependent_h0_with_error_sources_match_live_oracle(d, ntimes, nerr):
    """x_add-dependent H0 and Herror with error sources above 12 levels (round 6): the x_add variants in the
    dense error path (k_dlocal / k_derr_grad over np + na gradient parameters, k_dadd / k_dadd_err) against
    the oracle: F, F_dx (incl. F_dx_add), F_d2err, F_d2err_dx (incl. its x_add rows)."""
    from oracle import grape_oracle as O
    from robustgrape_amd import calculate_fidelity_and_derivatives
    fp = _xadd_err_problem(d, ntimes, nerr)
    x = np.concatenate([S.dense_x(ntimes, seed=900 + ntimes), [0.7, -0.3]])
    ref = O.calculate_fidelity_and_derivatives(fp, x)
    F, g, d2, d2dx = calculate_fidelity_and_derivatives(fp, x)
    _assert_fid_spread(F, g, ref[0], ref[1], f"dense_xadd_err_d{d}_nt{ntimes}", fp, x)
    _assert_err(d2, d2dx, ref[2], ref[3])
    assert d2dx.shape == (len(x), nerr) and np.max(np.abs(d2dx[-2:])) > 0


def test_dense_xadd_err_batch_equals_single():
    from robustgrape_amd.engine import GrapePlan
    fp = _xadd_err_problem(24, 5)
    X = np.stack([np.concatenate([S.dense_x(5, seed=s), [0.3 * s, -0.1 * s]]) for s in range(3)])
    plan = GrapePlan(fp, nparam=2, max_batch=3)
    out = plan.fidelity_grad(X)
    plan.close()
    one = GrapePlan(fp, nparam=2, max_batch=1)
    out1 = one.fidelity_grad(X)
    one.close()
    assert all(np.array_equal(a, b) for a, b in zip(out, out1))
