"""The image walk: error sources through the chunk walks (robustgrape_amd/csrc/grape_walk.hpp
k_walk_img / k_img_fdx).

With error sources the sector classes of <= 4 levels form the local-frame images of every
finite difference of a step -- Z1 = Y((E(x+eps) - E)/eps), W_e = Y((E(err eps) - E)/eps),
Z2_e = Y(mixed eps2 stencil), Y(dX) = Q_k^dag dX Q_{k-1} (UnitaryCalculations.jl:48-95) -- in the
lane that walks the chunk, instead of storing every variant propagator (k_expm) and Q (k_scan)
and reading them back (k_err_local).  The error scans / F_d2err_dx walks then run unchanged.

Checked against the oracle (grape_oracle.calculate_fidelity_and_derivatives: F, F_dx, F_d2err,
F_d2err_dx) and against the round-2 stored-intermediate kernels (GRAPE_OPT_NO_WALK), on the
d = 9 / 7 / 5 Rydberg problems with their error sources, one-step and chunk-start sizes,
bench-size plans, and high-norm steps inside long chunks (the walks' scaling-and-squaring path)."""
import numpy as np
import pytest

from tests import problems as P
from tests.xadd_pin import exact_rows

pytestmark = pytest.mark.gpu
T1 = 1e-12
T2S, T2S_ABS = 1e-7, 1e-9
T3, T3_ABS, T3_XADD_ABS = 1e-5, 1e-7, 1e-5


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _plan(fp, max_batch, options=0, nparam=1):
    from robustgrape_amd.engine import GrapePlan
    return GrapePlan(fp, nparam=nparam, device=0, max_batch=max_batch, options=options)


def _run(fp, X, options=0, nparam=1, expect_walk=None):
    pl = _plan(fp, len(X), options, nparam)
    try:
        pl.set_profiling(True)
        out = pl.fidelity_grad(X)
        kt = pl.kernel_times()
        sec = pl.sectors()
    finally:
        pl.close()
    if expect_walk is not None:  # the image walk ran (or not) for this plan
        assert (kt["k_walk_fwd"][1] > 0) == expect_walk, kt
        assert (kt["k_expm"][1] > 0) == (not expect_walk), kt
    return out, sec


def _check_all(test, out, b, ref, tier2, nmain, xadd_exact=None):
    """out / ref: (F, F_dx, F_d2err, F_d2err_dx) batches / single-row tuples; xadd_exact: the exact x_add
    rows of F_d2err_dx (tests/xadd_pin.py), when the problem's H0 and Herror do not read x_add."""
    from tests.parity_log import record
    F, Fdx, d2, d2dx = (o[b] for o in out)
    F0, g0, r2, r2dx = ref
    t2, t2a = tier2
    ef = abs(float(F) - float(F0))
    record(test, "F", ef, 1.0, T1)
    assert ef <= T1, (test, F, F0)
    err, sc = float(np.max(np.abs(Fdx - g0))), float(np.max(np.abs(g0)))
    record(test, "F_dx", err, sc, t2 * sc + t2a)
    assert err <= t2 * sc + t2a, (test, "F_dx", err, sc)
    # eps-FD sensitivities: the T2 tier of the step norm, at least T3's (tests/test_gpu_parity.py)
    e0, s0 = float(np.max(np.abs(d2 - r2))), float(np.max(np.abs(r2)))
    tol = max(T3, t2) * s0 + max(T3_ABS, t2a)
    record(test, "F_d2err", e0, s0, tol)
    assert e0 <= tol, (test, "F_d2err", e0, s0)
    ed, sd = float(np.max(np.abs(d2dx[:nmain] - r2dx[:nmain]))), float(np.max(np.abs(r2dx[:nmain])))
    told = max(T3, t2) * sd + max(T3_ABS, t2a)
    record(test, "F_d2err_dx", ed, sd, told)
    assert ed <= told, (test, "F_d2err_dx", ed, sd)
    # x_add rows: against their exact value at T3 (of the step-norm tier) of its scale, and against the
    # checker within that plus the checker's own distance from exact (tests/xadd_pin.py)
    ea = float(np.max(np.abs(d2dx[nmain:] - r2dx[nmain:])))
    if xadd_exact is not None:
        from tests.xadd_pin import check_xadd
        check_xadd(test, d2dx, r2dx, nmain, xadd_exact, rel=max(T3, t2), ab=max(T3_ABS, t2a))
    else:
        tola = T3_XADD_ABS
        record(test, "F_d2err_dx_add", ea, float(np.max(np.abs(r2dx[nmain:]))), tola)
        assert ea <= tola, (test, "F_d2err_dx_add", ea)
    print(f"{test}: |dF| {ef:.1e} F_dx {err / sc:.1e} F_d2err {e0 / max(s0, 1e-300):.1e} "
          f"F_d2err_dx {ed / max(sd, 1e-300):.1e} add {ea:.1e}")


CASES = [
    ("c3", lambda d: P.full9_problem(40, nerr=4, device=d), ((4, 1), (2, 2))),
    ("c3-one-step", lambda d: P.full9_problem(1, nerr=4, device=d), ((4, 1), (2, 2))),
    ("c3-nt256", lambda d: P.full9_problem(256, nerr=4, device=d), ((4, 1), (2, 2))),  # 0.327: unscaled T2 / T3
    ("c3-chunk-starts", lambda d: P.full9_problem(3, nerr=4, device=d), ((4, 1), (2, 2))),
    ("full9-2err", lambda d: P.full9_problem(33, nerr=2, device=d), ((4, 1), (2, 2))),
    ("sym5-amp-freq", lambda d: P.sym_problem(24, errors=("amp", "freq"), device=d), ((2, 2),)),
    ("fullblk7-amp-freq", lambda d: P.fullblk_problem(24, errors=("amp", "freq"), device=d), ((2, 3),)),
]


@pytest.mark.parametrize("name,mk,layout", CASES)
def test_image_walk_matches_oracle_and_stored_path(name, mk, layout):
    from oracle import grape_oracle as O
    from robustgrape_amd.operators import OPT_NO_WALK
    f, fo = mk(True), mk(False)
    nt = f.unitary_problem.ntimes
    X = np.stack([P.random_x(nt, 900 + s) for s in range(5)])
    out, sec = _run(f, X, expect_walk=True)
    ref, _ = _run(f, X, OPT_NO_WALK, expect_walk=False)
    assert sec == layout
    for b in range(len(X)):
        tier = P.fd_tier(f, X[b])
        _check_all(f"imgwalk_vs_stored_{name}_{b}", out, b, tuple(r[b] for r in ref), tier, nt, exact_rows(f, X[b]))
    for b in (0, 4):
        tier = P.fd_tier(f, X[b])
        _check_all(f"imgwalk_vs_oracle_{name}_{b}", out, b, O.calculate_fidelity_and_derivatives(fo, X[b]), tier, nt,
                   exact_rows(f, X[b]))


def test_image_walk_bench_size_against_oracle():
    """C3 at N_t = 512 in a 2 048-evaluation pass (16 chunks of 32 steps at S = 4, 32 of 16 at S = 2):
    rows scattered through the batch against the oracle."""
    from oracle import grape_oracle as O
    BIG = 2048
    f, fo = P.full9_problem(512, nerr=4), P.full9_problem(512, nerr=4, device=False)
    X = np.stack([P.random_x(512, 7000 + s, small=(s % 2 == 1)) for s in range(BIG)])
    out, _ = _run(f, X, expect_walk=True)
    for b in (0, 777, BIG - 1):
        _check_all(f"imgwalk_big_{b}", out, b, O.calculate_fidelity_and_derivatives(fo, X[b]), P.fd_tier(f, X[b]), 512,
                   exact_rows(f, X[b]))
    assert all(np.all(np.isfinite(o)) for o in out)


def test_image_walk_high_norm_steps():
    """High-norm steps (|dt H|_1 ~ 30: the walks' scaling and squaring; Julia's Pade 13) inside
    32-step chunks, with four error sources: against the oracle at the step-norm-scaled tier."""
    from oracle import grape_oracle as O
    nt = 96
    f, fo = P.full9_problem(nt, nerr=4, B=2000.0), P.full9_problem(nt, nerr=4, device=False, B=2000.0)
    X = np.stack([P.random_x(nt, 40 + s) for s in range(300)])
    out, _ = _run(f, X, expect_walk=True)
    for b in (0, 299):
        tier = P.fd_tier(f, X[b])
        assert tier[0] > 1e-7  # the squaring path is exercised
        _check_all(f"imgwalk_hot_{b}", out, b, O.calculate_fidelity_and_derivatives(fo, X[b]), tier, nt,
                   exact_rows(f, X[b]))


def test_image_walk_single_calls_are_the_batch():
    """Graph-replayed single evaluations through the image walk are bitwise the batch's rows."""
    fp = P.full9_problem(64, nerr=4)
    X = np.stack([P.random_x(64, 60 + s) for s in range(40)])
    pl = _plan(fp, 64)
    try:
        ref = pl.fidelity_grad(X)
        for b in (0, 39):
            one = pl.fidelity_grad(X[b:b + 1])
            for o, r in zip(one, ref):
                assert np.array_equal(o[0], r[b])
    finally:
        pl.close()


def test_image_walk_several_gradient_parameters():
    """An x_add-dependent H0 and error generator (tests/problems.py xadd_err_problem: nvg = 3 gradient
    parameters per step -- the control and both x_add entries) now runs the image walk (round 3 kept
    the stored-intermediate kernels for nvg > 1): against the committed golden (d = 5, N_t = 40,
    tests/golden/xadd_err.npz), and against the stored-variant path (GRAPE_OPT_NO_WALK) and the live
    oracle at d = 9 (sectors of 4 and 2 levels), with test_gpu_xadd_err.py's tiers."""
    import os
    from oracle import grape_oracle as O
    from robustgrape_amd.operators import OPT_NO_WALK
    from tests.test_gpu_xadd_err import _check
    g = dict(np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "xadd_err.npz"),
                     allow_pickle=False))
    fp = P.xadd_err_problem(int(g["d"]), int(g["ntimes"]))
    out, _ = _run(fp, g["x"][None, :], expect_walk=True)
    _check(tuple(o[0] for o in out), (float(g["F"]), g["F_dx"], g["F_d2err"], g["F_d2err_dx"]), "imgwalk xadd golden")
    nt = 24
    f9 = P.xadd_err_problem(9, nt)
    X = np.stack([P.xadd_x(nt, 70 + s) for s in range(3)])
    out, sec = _run(f9, X, expect_walk=True)
    ref, _ = _run(f9, X, OPT_NO_WALK, expect_walk=False)
    assert sec == ((4, 1), (2, 2))
    for b in range(len(X)):
        _check(tuple(o[b] for o in out), tuple(r[b] for r in ref), f"imgwalk xadd d=9 vs stored {b}")
    _check(tuple(o[1] for o in out), O.calculate_fidelity_and_derivatives(P.xadd_err_problem(9, nt, device=False), X[1]),
           "imgwalk xadd d=9 vs oracle")


def test_image_walk_not_for_non_hermitian_error_generator():
    """A decay-rate error source (-i e/2 |r><r|) makes the error variants non-unitary: the image
    walk's exponential is the skew-Hermitian one, so the plan keeps the stored-variant kernels
    (which the oracle test in tests/test_gpu_xadd_err.py checks)."""
    from robustgrape_amd.operators import OperatorBasisError, Term
    from robustgrape_amd.types import ErrorSource
    decay = np.diag([0, 0, 0, 0, 1.0]).astype(complex)
    base = P.sym_problem(12, errors=("amp",))
    fo = base.replace(unitary_problem=base.unitary_problem.replace(
        error_sources=list(base.unitary_problem.error_sources) + [ErrorSource(OperatorBasisError([Term(decay, scale=-0.5j)]))]))
    X = np.stack([P.random_x(12, s) for s in range(2)])
    _run(fo, X, expect_walk=False)


def _symmetric_error_problem(nt, device=True):
    """C2's model with error sources that act on BOTH atoms alike -- a common Rabi-amplitude error
    (Omega1 = Omega2 -> 1 + err) and a common detuning (delta1 = delta2 = err) -- so the atom-swap
    symmetry survives and the plan keeps the symmetry-adapted sectors (the rotated error
    operators, the rotated PA / PB of the sector error head and the 3-level image walk's
    F_d2err / F_d2err_dx had no test; C3's single-atom errors break the symmetry)."""
    from robustgrape_amd import rydberg as R
    from robustgrape_amd.operators import OperatorBasisError, Term
    from robustgrape_amd.types import ErrorSource, FidelityRobustGRAPEProblem, UnitaryRobustGRAPEProblem
    B = 10.0
    if device:
        H0 = R.rydberg_full_operator_basis(1.0, 1.0, 0.0, 0.0, B)
        # one operator pair for both atoms (each basis operator must keep the symmetry: the commutant
        # is taken over the operators, grape_symmetry.hpp)
        rabi = OperatorBasisError(R._drive_terms(*R._phase_pair(9, R._FULL_COUPLINGS, lambda w: 1.0)))
        dd = np.zeros(9)
        for i in (4, 6, 8):
            dd[i] += 1.0
        for i in (5, 7, 8):
            dd[i] += 1.0
        det = OperatorBasisError([Term(op=np.diag(dd).astype(np.complex128))])
        errs, target = [ErrorSource(rabi), ErrorSource(det)], R.cz_full_target()
    else:
        H0 = lambda t, p, xa: R.rydberg_hamiltonian_full(p[0], 1, 1, 0, 0, B)  # noqa: E731
        rabi = lambda t, p, xa, e: (R.rydberg_hamiltonian_full(p[0], 1 + e, 1 + e, 0, 0, B)  # noqa: E731
                                    - R.rydberg_hamiltonian_full(p[0], 1, 1, 0, 0, B))
        det = lambda t, p, xa, e: (R.rydberg_hamiltonian_full(p[0], 1, 1, e, e, B)  # noqa: E731
                                   - R.rydberg_hamiltonian_full(p[0], 1, 1, 0, 0, B))
        errs, target = [ErrorSource(rabi), ErrorSource(det)], (lambda xa: R.cz_with_1q_phase_full(xa[0]))
    up = UnitaryRobustGRAPEProblem(t0=P.T0_TO, ntimes=nt, ndim=9, H0=H0, nb_additional_param=1, error_sources=errs)
    return FidelityRobustGRAPEProblem(up, P.W_FULL9, target)


@pytest.mark.parametrize("nt", [1, 40, 160])
def test_symmetric_error_sources_keep_the_rotated_sectors(nt):
    """Errors that keep the atom-swap symmetry: the symmetry-adapted sectors (3 + 2 + 2) with the
    image walk, against the permutation sectors (GRAPE_OPT_NO_SYMMETRY) and the oracle: F, F_dx,
    F_d2err, F_d2err_dx (FidelityCalculations.jl:78-117 in the rotated frame)."""
    from oracle import grape_oracle as O
    from robustgrape_amd.operators import OPT_NO_SYMMETRY
    fp, fo = _symmetric_error_problem(nt), _symmetric_error_problem(nt, device=False)
    X = np.stack([P.random_x(nt, 4100 + s, small=(s == 1)) for s in range(3)])
    out, sec = _run(fp, X, expect_walk=True)
    # the 3-level symmetric sector (the common detuning also puts the dark level into a sector of
    # its own, so the 2-level class holds three)
    assert sec[0] == (3, 1), sec
    perm, sec_p = _run(fp, X, OPT_NO_SYMMETRY, expect_walk=True)
    assert sec_p[0] == (4, 1), sec_p
    nmain = nt
    for b in range(len(X)):
        tier = P.fd_tier(fp, X[b])
        ref_perm = tuple(o[b] for o in perm)
        _check_all(f"symerr_vs_perm_nt{nt}_{b}", out, b, ref_perm, tier, nmain, exact_rows(fp, X[b]))
    for b in (0, 1):
        ref = O.calculate_fidelity_and_derivatives(fo, X[b])
        _check_all(f"symerr_vs_oracle_nt{nt}_{b}", out, b, ref, P.fd_tier(fp, X[b]), nmain, exact_rows(fp, X[b]))
